#include "rpc/protocol.h"

#include <cerrno>
#include <mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "base/pool.h"
#include "base/util.h"
#include "rpc/compress.h"
#include "rpc/errno.h"
#include "rpc/retry_policy.h"
#include "rpc/serialized_request.h"

DEFINE_uint64(max_body_size, 64 * 1024 * 1024, "Maximum size of a single message body in all protocols");
MRPC_VALIDATE_FLAG(max_body_size, ::mrpc::PassValidator);

namespace mrpc {

const char* ParseErrorToString(ParseError e) {
    switch (e) {
    case PARSE_OK: return "ok";
    case PARSE_ERROR_TRY_OTHERS: return "try other protocols";
    case PARSE_ERROR_NOT_ENOUGH_DATA: return "not enough data";
    case PARSE_ERROR_TOO_BIG_DATA: return "message too big";
    case PARSE_ERROR_NO_RESOURCE: return "no resource";
    case PARSE_ERROR_ABSOLUTELY_WRONG: return "absolutely wrong message";
    }
    return "unknown";
}

MostCommonMessage* MostCommonMessage::Get() {
    MostCommonMessage* m = get_object<MostCommonMessage>();
    m->_process = nullptr;
    m->_arg = nullptr;
    m->_received_us = 0;
    m->_base_real_us = 0;
    return m;
}

void MostCommonMessage::Destroy() {
    meta.clear();
    payload.clear();
    _socket.reset();
    return_object(this);
}

namespace {
struct ProtocolEntry {
    bool valid = false;
    Protocol p;
};
ProtocolEntry g_protocols[MAX_PROTOCOL_SIZE];
std::mutex g_protocol_mu;
}  // namespace

int RegisterProtocol(ProtocolType type, const Protocol& p) {
    const int idx = (int)type;
    if (idx < 0 || idx >= MAX_PROTOCOL_SIZE) return -1;
    std::lock_guard<std::mutex> g(g_protocol_mu);
    if (g_protocols[idx].valid) return -1;
    g_protocols[idx].p = p;
    g_protocols[idx].valid = true;
    return 0;
}

const Protocol* FindProtocol(ProtocolType type) {
    const int idx = (int)type;
    if (idx < 0 || idx >= MAX_PROTOCOL_SIZE) return nullptr;
    return g_protocols[idx].valid ? &g_protocols[idx].p : nullptr;
}

void ListProtocols(std::vector<std::pair<ProtocolType, Protocol>>* out) {
    out->clear();
    for (int i = 0; i < MAX_PROTOCOL_SIZE; ++i) {
        if (g_protocols[i].valid) out->emplace_back((ProtocolType)i, g_protocols[i].p);
    }
}

ProtocolType StringToProtocolType(const std::string& name0, bool print_log) {
    std::string name = to_lower(name0);
    size_t colon = name.find(':');
    if (colon != std::string::npos) name = name.substr(0, colon);  // "h2:grpc" -> h2
    for (int i = 0; i < MAX_PROTOCOL_SIZE; ++i) {
        if (g_protocols[i].valid && g_protocols[i].p.name && name == g_protocols[i].p.name) return (ProtocolType)i;
    }
    if (name == "grpc") return PROTOCOL_H2;
    if (print_log) LOG(ERROR) << "Unknown protocol `" << name0 << "'";
    return PROTOCOL_UNKNOWN;
}

const char* ProtocolTypeToString(ProtocolType t) {
    const Protocol* p = FindProtocol(t);
    return p && p->name ? p->name : "unknown";
}

bool ParsePbFromBuf(pb::Message* msg, const Buf& buf) {
    if (buf.size() > FLAGS_max_body_size) return false;
    return msg->ParseFromBuf(buf);
}

bool ParsePbFromString(pb::Message* msg, const std::string& s) {
    if (s.size() > FLAGS_max_body_size) return false;
    return msg->ParseFromString(s);
}

bool SerializeAsCompressedData(const pb::Message& msg, Buf* buf, CompressType type) {
    if (const SerializedRequest* sr = dynamic_cast<const SerializedRequest*>(&msg)) {
        buf->append(sr->serialized_data());  // already encoded with `type`
        return true;
    }
    if (type == COMPRESS_TYPE_NONE) return msg.SerializeToBuf(buf);
    if (type == COMPRESS_TYPE_SNAPPY && TrySnappyPackOffload(msg, buf)) return true;
    Buf raw;
    if (!msg.SerializeToBuf(&raw)) return false;
    return CompressBuf(type, raw, buf);
}

bool ParseFromCompressedData(const Buf& data, pb::Message* msg, CompressType type) {
    if (type == COMPRESS_TYPE_NONE) return ParsePbFromBuf(msg, data);
    if (data.size() <= FLAGS_max_body_size) {
        const int rc = TryPbParseOffload(data, type, msg);
        if (rc != 0) return rc > 0;
    }
    Buf raw;
    if (!DecompressBuf(type, data, &raw)) return false;
    return ParsePbFromBuf(msg, raw);
}

// ------------------------------------------------------------- retry policy
namespace {
class DefaultRetryPolicyImpl : public RetryPolicy {
public:
    bool DoRetry(const Controller* cntl) const override;
};
}  // namespace

}  // namespace mrpc

#include "rpc/controller.h"

namespace mrpc {
namespace {
bool DefaultRetryPolicyImpl::DoRetry(const Controller* cntl) const {
    const int ec = cntl->ErrorCode();
    return ec == EFAILEDSOCKET || ec == EEOF || ec == EHOSTDOWN || ec == ELOGOFF || ec == ETIMEDOUT || ec == ELIMIT ||
           ec == ENOENT || ec == EPIPE || ec == ECONNREFUSED || ec == ECONNRESET || ec == ENODATA ||
           ec == EOVERCROWDED || ec == EH2RUNOUTSTREAMS;
}
}  // namespace

const RetryPolicy* DefaultRetryPolicy() {
    static DefaultRetryPolicyImpl p;
    return &p;
}

void RegisterRpcErrnoTexts() {
    RegisterErrorText(ENOSERVICE, "No such service");
    RegisterErrorText(ENOMETHOD, "No such method");
    RegisterErrorText(EREQUEST, "Bad request");
    RegisterErrorText(ERPCAUTH, "Authentication failed");
    RegisterErrorText(ETOOMANYFAILS, "Too many sub channels failed");
    RegisterErrorText(EPCHANFINISH, "ParallelChannel finished");
    RegisterErrorText(EBACKUPREQUEST, "Sending backup request");
    RegisterErrorText(ERPCTIMEDOUT, "RPC call is timed out");
    RegisterErrorText(EFAILEDSOCKET, "Broken socket");
    RegisterErrorText(EHTTP, "Bad http call");
    RegisterErrorText(EOVERCROWDED, "The server is overcrowded");
    RegisterErrorText(EEOF, "Got EOF");
    RegisterErrorText(EUNUSED, "The socket was not needed");
    RegisterErrorText(ESSL, "SSL related operation failed");
    RegisterErrorText(EH2RUNOUTSTREAMS, "The H2 socket was run out of streams");
    RegisterErrorText(EREJECT, "The request is rejected");
    RegisterErrorText(EINTERNAL, "General internal error");
    RegisterErrorText(ERESPONSE, "Bad response");
    RegisterErrorText(ELOGOFF, "Server is stopping");
    RegisterErrorText(ELIMIT, "Reached server's max_concurrency");
    RegisterErrorText(ECLOSE, "Close socket initiatively");
    RegisterErrorText(EITP, "Bad Itp response");
    RegisterErrorText(ERDMA, "RDMA verbs error");
    RegisterErrorText(ERDMAMEM, "Memory not registered for RDMA");
    RegisterErrorText(EGPU, "HIP runtime or kernel error");
    RegisterErrorText(EXGMI, "xGMI transport error");
}

}  // namespace mrpc
