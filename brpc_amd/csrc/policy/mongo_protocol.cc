// Mongo server protocol (role of the reference's src/brpc/policy/mongo_protocol.cpp):
//   | message_length i32 | request_id i32 | response_to i32 | op_code i32 | body |   (little endian)
// Only servers with ServerOptions.mongo_service_adaptor accept it; the
// op_code doubles as the magic number. Each message becomes a call of
// mrpc.policy.MongoService.default_method; the reply is an OP_REPLY built
// from MongoResponse (or the adaptor's error reply on failure).
#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "mrpc/proto/mongo.pb.h"
#include "policy/policies.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/mongo.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/usercode_backup_pool.h"

DECLARE_uint64(max_body_size);

namespace mrpc {
namespace policy {

namespace {
bool is_mongo_opcode(int32_t op) {
    switch (op) {
    case OPREPLY: case DBMSG: case DB_UPDATE: case DB_INSERT: case DB_QUERY: case DB_GETMORE:
    case DB_DELETE: case DB_KILLCURSORS: case DB_COMMAND: case DB_COMMANDREPLY: return true;
    default: return false;
    }
}

// Socket-attached holder of the adaptor's per-connection context.
class MongoParsingContext : public ParsingContext {
public:
    static const int kTag = 0x4d4f4e47;  // "MONG"
    int protocol_tag() const override { return kTag; }
    std::shared_ptr<MongoContext> ctx;
};

class MongoInputMessage : public InputMessageBase {
public:
    mongo_head_t head;
    Buf body;
    std::shared_ptr<MongoContext> ctx;
};

struct MongoCall {
    Controller cntl;
    MongoRequest req;
    MongoResponse res;
    Server* server = nullptr;
    MethodStatus* status = nullptr;
    int64_t received_us = 0;
    bool added_concurrency = false;
};

void SendMongoResponse(MongoCall* c) {
    std::unique_ptr<MongoCall> guard(c);
    ConcurrencyRemover remover(c->status, &c->cntl, c->received_us, c->added_concurrency ? c->server : nullptr);
    SocketUniquePtr sock;
    if (Socket::Address(c->cntl._server_socket_id, &sock) != 0) return;
    if (c->cntl.IsCloseConnection()) {
        sock->SetFailed(ECLOSE, "close connection by mongo service");
        return;
    }
    Buf out;
    if (c->cntl.Failed()) {
        c->server->options().mongo_service_adaptor->SerializeError(c->res.header().response_to(), &out);
    } else if (c->res.has_message()) {
        const MongoHeader& h = c->res.header();
        mongo_head_t head;
        head.request_id = h.request_id();
        head.response_to = h.response_to();
        head.op_code = h.op_code() ? h.op_code() : OPREPLY;
        const int32_t flags = c->res.response_flags();
        const int64_t cursor = c->res.cursor_id();
        const int32_t from = c->res.starting_from();
        const int32_t nret = c->res.number_returned();
        head.message_length = (int32_t)(sizeof(head) + 20 + c->res.message().size());
        out.append(&head, sizeof(head));
        out.append(&flags, 4);
        out.append(&cursor, 8);
        out.append(&from, 4);
        out.append(&nret, 4);
        out.append(c->res.message());
    }
    if (!out.empty()) {
        WriteOptions wopt;
        wopt.ignore_eovercrowded = true;
        if (sock->Write(&out, &wopt) != 0) {
            LOG_EVERY_SECOND(WARNING) << "Fail to write into " << sock->description();
        }
    }
}
}  // namespace

ParseResult ParseMongoMessage(Buf* source, Socket* socket, bool, const void* arg) {
    const Server* server = static_cast<const Server*>(arg);
    if (!server || !server->options().mongo_service_adaptor) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    ParsingContext* pc = socket->parsing_context();
    if (pc && pc->protocol_tag() != MongoParsingContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    mongo_head_t head;
    if (source->copy_to(&head, sizeof(head)) < sizeof(head)) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    if (!is_mongo_opcode(head.op_code)) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    if (head.message_length < (int32_t)sizeof(head)) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    if ((uint64_t)head.message_length > FLAGS_max_body_size) return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    if (source->size() < (size_t)head.message_length) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    MongoParsingContext* mpc = static_cast<MongoParsingContext*>(pc);
    if (!mpc) {
        mpc = new MongoParsingContext;
        mpc->ctx.reset(server->options().mongo_service_adaptor->CreateSocketContext());
        if (!socket->InstallParsingContext(mpc)) {
            delete mpc;
            mpc = static_cast<MongoParsingContext*>(socket->parsing_context());
            if (!mpc || mpc->protocol_tag() != MongoParsingContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        }
    }
    MongoInputMessage* m = new MongoInputMessage;
    m->head = head;
    m->ctx = mpc->ctx;
    source->pop_front(sizeof(head));
    source->cutn(&m->body, (size_t)head.message_length - sizeof(head));
    return MakeMessage(m);
}

void ProcessMongoRequest(InputMessageBase* base) {
    std::unique_ptr<MongoInputMessage> m(static_cast<MongoInputMessage*>(base));
    Socket* socket = m->socket();
    Server* server = const_cast<Server*>(static_cast<const Server*>(m->arg()));
    MongoCall* c = new MongoCall;
    c->server = server;
    c->received_us = m->received_us();
    Controller* cntl = &c->cntl;
    cntl->_server = server;
    cntl->_server_socket_id = socket->id();
    cntl->_remote_side = socket->remote_side();
    cntl->_local_side = socket->local_side();
    cntl->_received_us = m->received_us();
    cntl->_begin_us = m->received_us();
    cntl->_protocol_type = PROTOCOL_MONGO;
    cntl->_mongo_session_data = m->ctx;
    c->res.mutable_header()->set_response_to(m->head.request_id);
    const Server::MethodProperty* mp =
        server->FindMethodPropertyByFullName(MongoService::descriptor()->full_name, "default_method");
    do {
        if (!server->IsRunning()) {
            cntl->SetFailed(ELOGOFF, "Server is stopping");
            break;
        }
        if (!server->AddConcurrency(cntl)) {
            cntl->SetFailed(ELIMIT, "Reached server's max_concurrency=%d", server->max_concurrency());
            break;
        }
        c->added_concurrency = true;
        if (!mp) {
            cntl->SetFailed(ENOMETHOD, "Fail to find MongoService.default_method");
            break;
        }
        int rejected = 0;
        if (!mp->status->OnRequested(&rejected, cntl)) {
            mp->status->OnResponded(ELIMIT, 0);
            cntl->SetFailed(ELIMIT, "Rejected by the concurrency limiter, concurrency=%d", rejected);
            break;
        }
        c->status = mp->status.get();
        cntl->set_log_id((uint64_t)(uint32_t)m->head.request_id);
        MongoHeader* h = c->req.mutable_header();
        h->set_message_length(m->head.message_length);
        h->set_request_id(m->head.request_id);
        h->set_response_to(m->head.response_to);
        h->set_op_code((MongoOp)m->head.op_code);
        c->req.set_message(m->body.to_string());
    } while (false);
    m.reset();
    if (cntl->Failed()) {
        SendMongoResponse(c);
        return;
    }
    CallServiceMethod(mp->service, mp->method, cntl, &c->req, &c->res, NewCallback([c] { SendMongoResponse(c); }));
}

void RegisterMongoProtocol() {
    Protocol p;
    p.parse = ParseMongoMessage;
    p.process_request = ProcessMongoRequest;
    p.supported_connection_type = CONNECTION_TYPE_POOLED;
    p.name = "mongo";
    RegisterProtocol(PROTOCOL_MONGO, p);
}

}  // namespace policy
}  // namespace mrpc
