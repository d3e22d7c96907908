// RESP wire protocol (role of the reference's
// src/brpc/policy/redis_protocol.cpp): client pipelining through the socket's
// pipelined-info queue; server commands run in order inside parse().
#include <cstring>
#include <memory>

#include "base/logging.h"
#include "base/util.h"
#include "fiber/call_id.h"
#include "net/input_messenger.h"
#include "policy/policies.h"
#include "redis/redis.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/server.h"

namespace mrpc {
namespace policy {

namespace {

class RedisClientContext : public ParsingContext {
public:
    static const int kTag = 0x52454443;  // "REDC"
    int protocol_tag() const override { return kTag; }
    RedisResponse partial;   // replies of the current pipelined entry
    PipelinedInfo pi;
    bool has_pi = false;
};

class RedisServerContext : public ParsingContext {
public:
    static const int kTag = 0x52454453;  // "REDS"
    int protocol_tag() const override { return kTag; }
    RedisCommandHandler* transaction = nullptr;  // inside MULTI
    std::vector<std::vector<std::string>> queued;
};

class RedisResponseMessage : public InputMessageBase {
public:
    RedisResponse response;
    PipelinedInfo pi;
};

bool is_client_socket(Socket* s) { return s->user() == get_client_side_messenger(); }

// A command as an array of bulk strings (inline commands also accepted).
int parse_command(Buf* in, std::vector<std::string>* args) {
    RedisReply r;
    char first;
    if (in->copy_to(&first, 1) != 1) return 0;
    if (first != '*') {
        // inline command: "PING\r\n"
        std::string line;
        char buf[512];
        const size_t n = in->copy_to(buf, std::min(in->size(), sizeof(buf)));
        const char* nl = (const char*)memchr(buf, '\n', n);
        if (!nl) return n == sizeof(buf) ? -1 : 0;
        line.assign(buf, nl - buf);
        in->pop_front(nl - buf + 1);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        *args = split_string(line, ' ');
        return args->empty() ? -1 : 1;
    }
    const int rc = r.ConsumePartial(in);
    if (rc <= 0) return rc;
    if (!r.is_array() || r.size() == 0) return -1;
    args->clear();
    for (size_t i = 0; i < r.size(); ++i) {
        if (!r[i].is_string()) return -1;
        args->push_back(r[i].data());
    }
    return 1;
}

void run_command(Server* server, RedisServerContext* ctx, std::vector<std::string>& args, RedisReply* out) {
    RedisService* svc = server->options().redis_service;
    const std::string name = to_lower(args[0]);
    args[0] = name;
    if (ctx->transaction) {
        if (name == "exec") {
            RedisCommandHandler* th = ctx->transaction;
            ctx->transaction = nullptr;
            out->SetArray(ctx->queued.size());
            for (size_t i = 0; i < ctx->queued.size(); ++i) th->Run(ctx->queued[i], &(*out)[i], true);
            ctx->queued.clear();
            delete th;
            return;
        }
        if (name == "discard") {
            delete ctx->transaction;
            ctx->transaction = nullptr;
            ctx->queued.clear();
            out->SetStatus("OK");
            return;
        }
        ctx->queued.push_back(args);
        out->SetStatus("QUEUED");
        return;
    }
    RedisCommandHandler* h = svc->FindCommandHandler(name);
    if (!h) {
        out->SetError("ERR unknown command '" + name + "'");
        return;
    }
    if (name == "multi") {
        RedisCommandHandler* th = h->NewTransactionHandler();
        if (!th) {
            out->SetError("ERR MULTI is not supported");
            return;
        }
        ctx->transaction = th;
        out->SetStatus("OK");
        return;
    }
    h->Run(args, out, true);
}

}  // namespace

ParseResult ParseRedisMessage(Buf* source, Socket* socket, bool read_eof, const void* arg) {
    if (source->empty()) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    ParsingContext* pc = socket->parsing_context();
    if (is_client_socket(socket)) {
        RedisClientContext* ctx = nullptr;
        if (pc) {
            if (pc->protocol_tag() != RedisClientContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
            ctx = static_cast<RedisClientContext*>(pc);
        } else {
            // only claim the socket if a redis call is waiting on it
            PipelinedInfo peek;
            if (!socket->PeekPipelinedInfo(&peek) || peek.protocol != PROTOCOL_REDIS) {
                return MakeParseError(PARSE_ERROR_TRY_OTHERS);
            }
            char c;
            source->copy_to(&c, 1);
            if (c == '\0' || !strchr("+-:$*", c)) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
            ctx = new RedisClientContext;
            if (!socket->InstallParsingContext(ctx)) {
                delete ctx;
                return MakeParseError(PARSE_ERROR_TRY_OTHERS);
            }
        }
        if (!ctx->has_pi) {
            if (!socket->PopPipelinedInfo(&ctx->pi)) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
            ctx->has_pi = true;
            ctx->partial.Clear();
        }
        const int rc = ctx->partial.ConsumePartial(source, ctx->pi.count);
        if (rc < 0) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
        if (rc == 0) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
        RedisResponseMessage* msg = new RedisResponseMessage;
        std::swap(msg->response, ctx->partial);
        msg->pi = ctx->pi;
        ctx->has_pi = false;
        return MakeMessage(msg);
    }
    // server side
    const Server* server = static_cast<const Server*>(arg);
    if (!server || !server->options().redis_service) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    RedisServerContext* ctx = nullptr;
    if (pc) {
        if (pc->protocol_tag() != RedisServerContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ctx = static_cast<RedisServerContext*>(pc);
    } else {
        char c;
        source->copy_to(&c, 1);
        if (c != '*') return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ctx = new RedisServerContext;
        if (!socket->InstallParsingContext(ctx)) {
            delete ctx;
            return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        }
    }
    // execute every complete command now, in order; one write per batch
    Buf out;
    for (;;) {
        std::vector<std::string> args;
        const int rc = parse_command(source, &args);
        if (rc < 0) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
        if (rc == 0) break;
        RedisReply reply;
        run_command(const_cast<Server*>(server), ctx, args, &reply);
        reply.SerializeTo(&out);
    }
    if (!out.empty()) socket->Write(&out);
    return MakeMessage(nullptr);  // consumed inside parse
}

void SerializeRedisRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const RedisRequest* rr = dynamic_cast<const RedisRequest*>(request);
    if (!rr) {
        cntl->SetFailed(EREQUEST, "request must be a RedisRequest");
        return;
    }
    if (rr->command_size() == 0 || !rr->SerializeTo(buf)) {
        cntl->SetFailed(EREQUEST, "RedisRequest has no valid command");
        return;
    }
    cntl->_pipelined_count = rr->command_size();
}

void PackRedisRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor*, Controller* cntl,
                      const Buf& request_buf, const Authenticator*) {
    (void)correlation_id;
    packet->append(request_buf);
    if (cntl->_pipelined_count <= 0) cntl->_pipelined_count = 1;
}

void ProcessRedisResponse(InputMessageBase* msg_base) {
    std::unique_ptr<RedisResponseMessage> msg(static_cast<RedisResponseMessage*>(msg_base));
    const fiber::CallId cid = msg->pi.id_wait;
    Controller* cntl = nullptr;
    if (fiber::call_id_lock(cid, (void**)&cntl) != 0) return;
    if (cid != cntl->current_id() && cid != cntl->_unfinished_call.id) {
        fiber::call_id_unlock(cid);
        return;
    }
    int saved_error = 0;
    RedisResponse* res = dynamic_cast<RedisResponse*>(cntl->_response);
    if (res) {
        std::swap(*res, msg->response);
    } else if (cntl->_response) {
        saved_error = ERESPONSE;
        cntl->SetFailed(ERESPONSE, "response must be a RedisResponse");
    }
    msg.reset();
    cntl->OnVersionedRPCReturned(cid, saved_error);
}

void RegisterRedisProtocol() {
    Protocol p;
    p.parse = ParseRedisMessage;
    p.serialize_request = SerializeRedisRequest;
    p.pack_request = PackRedisRequest;
    p.process_request = [](InputMessageBase* m) { m->Destroy(); };  // never produced
    p.process_response = ProcessRedisResponse;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "redis";
    RegisterProtocol(PROTOCOL_REDIS, p);
}

}  // namespace policy
}  // namespace mrpc
