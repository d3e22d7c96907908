// Protocol plug-in interface (role of src/brpc/protocol.h:77-195): every wire
// format registers parse / serialize / pack / process functions. A server
// port speaks all registered protocols (InputMessenger sniffs per socket).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "base/buf.h"
#include "base/endpoint.h"
#include "mrpc/proto/options.pb.h"
#include "net/socket.h"
#include "pb/message.h"

namespace mrpc {

class Controller;
class Authenticator;
class InputMessageBase;
class Server;

enum ParseError {
    PARSE_OK = 0,
    PARSE_ERROR_TRY_OTHERS,
    PARSE_ERROR_NOT_ENOUGH_DATA,
    PARSE_ERROR_TOO_BIG_DATA,
    PARSE_ERROR_NO_RESOURCE,
    PARSE_ERROR_ABSOLUTELY_WRONG,
};
const char* ParseErrorToString(ParseError e);

class ParseResult {
public:
    explicit ParseResult(ParseError e) : _err(e), _msg(nullptr) {}
    explicit ParseResult(InputMessageBase* m) : _err(PARSE_OK), _msg(m) {}
    bool is_ok() const { return _err == PARSE_OK; }
    ParseError error() const { return _err; }
    InputMessageBase* message() const { return _msg; }
private:
    ParseError _err;
    InputMessageBase* _msg;
};
inline ParseResult MakeParseError(ParseError e) { return ParseResult(e); }
inline ParseResult MakeMessage(InputMessageBase* m) { return ParseResult(m); }

// Base of all parsed messages.
class InputMessageBase {
public:
    virtual ~InputMessageBase() {}
    virtual void Destroy() { delete this; }
    Socket* socket() const { return _socket.get(); }
    SocketUniquePtr& socket_ptr() { return _socket; }
    const void* arg() const { return _arg; }
    int64_t received_us() const { return _received_us; }
    int64_t base_real_us() const { return _base_real_us; }

    SocketUniquePtr _socket;
    void (*_process)(InputMessageBase*) = nullptr;
    const void* _arg = nullptr;  // Server* for requests
    int64_t _received_us = 0;
    int64_t _base_real_us = 0;
};

// A message that owns meta+payload Bufs; used by most binary protocols.
class MostCommonMessage : public InputMessageBase {
public:
    Buf meta;
    Buf payload;
    static MostCommonMessage* Get();
    void Destroy() override;
};

struct Protocol {
    ParseResult (*parse)(Buf* source, Socket* socket, bool read_eof, const void* arg) = nullptr;
    // Serialize request message into buf (may compress). Set cntl failure on error.
    void (*serialize_request)(Buf* request_buf, Controller* cntl, const pb::Message* request) = nullptr;
    // Build the on-wire packet (headers + meta + body + attachment).
    void (*pack_request)(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor* method,
                         Controller* controller, const Buf& request_buf, const Authenticator* auth) = nullptr;
    void (*process_request)(InputMessageBase* msg) = nullptr;
    void (*process_response)(InputMessageBase* msg) = nullptr;
    bool (*verify)(const InputMessageBase* msg) = nullptr;
    bool (*parse_server_address)(EndPoint* out, const char* addr) = nullptr;
    const std::string& (*get_method_name)(const pb::MethodDescriptor* method, const Controller* cntl) = nullptr;
    int supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    const char* name = nullptr;
    bool support_client() const { return serialize_request && pack_request && process_response; }
    bool support_server() const { return process_request; }
};

const int MAX_PROTOCOL_SIZE = 128;
int RegisterProtocol(ProtocolType type, const Protocol& p);
const Protocol* FindProtocol(ProtocolType type);
void ListProtocols(std::vector<std::pair<ProtocolType, Protocol>>* out);
ProtocolType StringToProtocolType(const std::string& name, bool print_log = true);
const char* ProtocolTypeToString(ProtocolType t);

// Protobuf glue enforcing max_body_size (reference protocol.h:205-216).
bool ParsePbFromBuf(pb::Message* msg, const Buf& buf);
bool ParsePbFromString(pb::Message* msg, const std::string& s);
bool SerializeAsCompressedData(const pb::Message& msg, Buf* buf, CompressType type);
bool ParseFromCompressedData(const Buf& data, pb::Message* msg, CompressType type);

// Called once per process: registers protocols, compressors, naming
// services, load balancers, concurrency limiters.
void GlobalInitializeOrDie();

}  // namespace mrpc
