// RPC error codes (same numeric values as the reference's
// src/brpc/errno.proto:20-56 so that error_code on the wire interoperates).
#pragma once

namespace mrpc {

enum Errno {
    ENOSERVICE = 1001,
    ENOMETHOD = 1002,
    EREQUEST = 1003,
    ERPCAUTH = 1004,
    ETOOMANYFAILS = 1005,
    EPCHANFINISH = 1006,
    EBACKUPREQUEST = 1007,
    ERPCTIMEDOUT = 1008,
    EFAILEDSOCKET = 1009,
    EHTTP = 1010,
    EOVERCROWDED = 1011,
    ERTMPPUBLISHABLE = 1012,
    ERTMPCREATESTREAM = 1013,
    EEOF = 1014,
    EUNUSED = 1015,
    ESSL = 1016,
    EH2RUNOUTSTREAMS = 1017,
    EREJECT = 1018,
    EINTERNAL = 2001,
    ERESPONSE = 2002,
    ELOGOFF = 2003,
    ELIMIT = 2004,
    ECLOSE = 2005,
    EITP = 2006,
    ERDMA = 3001,
    ERDMAMEM = 3002,
    // MI355X-native additions
    EGPU = 3101,      // HIP runtime / kernel error
    EXGMI = 3102,     // xGMI transport error (IPC mapping, ring overflow)
};

// Registers the texts with base ErrorText(); called by GlobalInitialize.
void RegisterRpcErrnoTexts();

}  // namespace mrpc
