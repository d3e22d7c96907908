// RESP wire protocol (role of the reference's
// src/brpc/policy/redis_protocol.cpp): client pipelining through the socket's
// pipelined-info queue; server commands run in order inside parse().
#include <cstring>
#include <memory>

#include "base/logging.h"
#include "base/util.h"
#include "fiber/call_id.h"
#include "net/input_messenger.h"
#include "policy/authenticators.h"
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
    ~RedisServerContext() override { delete transaction; }
    // commands go here while a handler's transaction is open (it returned
    // CONTINUE) until the transaction handler returns OK
    RedisCommandHandler* transaction = nullptr;
    // replies deferred by handlers that returned BATCHED, owed in the next
    // OK reply (an array of batched + 1 replies)
    int batched = 0;
    // incremental command parser: a command's arguments are consumed from
    // the socket buffer as each one completes, and the state survives
    // across reads (a large SET spanning many reads is parsed once, not
    // re-parsed from its first byte on every read)
    int64_t want_args = -1;   // -1: expecting "*<n>"
    int64_t bulk_len = -1;    // -1: expecting "$<len>" of the next argument
    std::vector<std::string> args;
};

class RedisResponseMessage : public InputMessageBase {
public:
    RedisResponse response;
    PipelinedInfo pi;
};

bool is_client_socket(Socket* s) { return s->user() == get_client_side_messenger(); }

// One CRLF-terminated line from the front of `in`: 1 (consumed into
// *line), 0 (incomplete), -1 (no CRLF within a sane header length).
int read_line(Buf* in, std::string* line, size_t max_len) {
    char small[128];
    std::string big;
    const size_t window = std::min(in->size(), max_len);
    char* buf = small;
    if (window > sizeof(small)) {  // long inline commands: scan a heap window
        big.resize(window);
        buf = &big[0];
    }
    const size_t n = in->copy_to(buf, window);
    const char* nl = static_cast<const char*>(memchr(buf, '\n', n));
    if (!nl) return n >= max_len ? -1 : 0;
    const size_t len = (size_t)(nl - buf);
    line->assign(buf, len && buf[len - 1] == '\r' ? len - 1 : len);
    in->pop_front(len + 1);
    return 1;
}

bool parse_int(const std::string& s, size_t from, int64_t* out) {
    if (from >= s.size()) return false;
    int64_t v = 0;
    for (size_t i = from; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '9' || v > (int64_t(1) << 40)) return false;
        v = v * 10 + (s[i] - '0');
    }
    *out = v;
    return true;
}

const int64_t kMaxArgs = 1 << 20;
const size_t kMaxInline = 64 << 10;  // redis' PROTO_INLINE_MAX_SIZE
const int64_t kMaxBulk = int64_t(512) << 20;  // redis' proto-max-bulk-len

// Next complete command (array of bulk strings, or an inline command):
// 1 (in *args), 0 (need more bytes; progress kept in ctx), -1 (malformed).
int parse_command(RedisServerContext* ctx, Buf* in, std::vector<std::string>* args) {
    if (ctx->want_args < 0) {
        char first;
        if (in->copy_to(&first, 1) != 1) return 0;
        std::string line;
        if (first != '*') {
            // inline command: "PING\r\n", up to redis' 64 KiB inline limit
            const int rc = read_line(in, &line, kMaxInline);
            if (rc <= 0) return rc;
            *args = split_string(line, ' ');
            return args->empty() ? -1 : 1;
        }
        const int rc = read_line(in, &line, 32);
        if (rc <= 0) return rc;
        int64_t n = 0;
        if (!parse_int(line, 1, &n) || n <= 0 || n > kMaxArgs) return -1;
        ctx->want_args = n;
        ctx->bulk_len = -1;
        ctx->args.clear();
        ctx->args.reserve((size_t)std::min<int64_t>(n, 64));
    }
    while ((int64_t)ctx->args.size() < ctx->want_args) {
        if (ctx->bulk_len < 0) {
            std::string line;
            const int rc = read_line(in, &line, 32);
            if (rc <= 0) return rc;
            int64_t len = 0;
            if (line.empty() || line[0] != '$' || !parse_int(line, 1, &len) || len > kMaxBulk) return -1;
            ctx->bulk_len = len;
        }
        // O(1) until the whole argument is there
        if (in->size() < (size_t)ctx->bulk_len + 2) return 0;
        std::string a((size_t)ctx->bulk_len, '\0');
        if (ctx->bulk_len) in->copy_to(&a[0], (size_t)ctx->bulk_len);
        char crlf[2];
        in->pop_front((size_t)ctx->bulk_len);
        in->copy_to(crlf, 2);
        if (crlf[0] != '\r' || crlf[1] != '\n') return -1;
        in->pop_front(2);
        ctx->args.push_back(std::move(a));
        ctx->bulk_len = -1;
    }
    args->swap(ctx->args);
    ctx->args.clear();
    ctx->want_args = -1;
    return 1;
}

// One command under the handler protocol of the reference
// (src/brpc/policy/redis_protocol.cpp:79-131, redis.h RedisCommandHandler):
//  * OK: the reply goes out now; after BATCHED commands it is an array with
//    one reply per batched command plus this one, sent element by element;
//  * CONTINUE: the reply goes out and the handler's transaction handler
//    takes the connection's next commands until it returns OK (MULTI/EXEC);
//  * BATCHED: the reply is owed; flush_batched tells the handler whether
//    this is the last command of what arrived, i.e. whether to settle now.
// Returns -1 on a protocol violation by the handler (the connection fails).
int run_command(Server* server, RedisServerContext* ctx, std::vector<std::string>& args, bool flush_batched,
                Buf* out_buf) {
    RedisService* svc = server->options().redis_service;
    args[0] = to_lower(args[0]);
    RedisReply out;
    RedisCommandHandler::Result r = RedisCommandHandler::OK;
    if (ctx->transaction) {
        r = ctx->transaction->Run(args, &out, flush_batched);
        if (r == RedisCommandHandler::OK) {
            delete ctx->transaction;
            ctx->transaction = nullptr;
        } else if (r == RedisCommandHandler::BATCHED) {
            LOG(ERROR) << "a redis transaction handler returned BATCHED";
            return -1;
        }
    } else {
        RedisCommandHandler* h = svc->FindCommandHandler(args[0]);
        if (!h) {
            out.SetError("ERR unknown command '" + args[0] + "'");
        } else {
            r = h->Run(args, &out, flush_batched);
            if (r == RedisCommandHandler::CONTINUE) {
                if (ctx->batched) {
                    LOG(ERROR) << "a redis handler returned CONTINUE inside a batch";
                    return -1;
                }
                ctx->transaction = h->NewTransactionHandler();
                if (!ctx->transaction) {
                    out.SetError("ERR '" + args[0] + "' opened a transaction its handler cannot run");
                    r = RedisCommandHandler::OK;
                }
            } else if (r == RedisCommandHandler::BATCHED) {
                ++ctx->batched;
            }
        }
    }
    if (r == RedisCommandHandler::BATCHED) return 0;  // owed
    if (r == RedisCommandHandler::OK && ctx->batched) {
        if (!out.is_array() || (int)out.size() != ctx->batched + 1) {
            LOG(ERROR) << "a redis handler settled " << ctx->batched << " batched commands with "
                       << (out.is_array() ? (int)out.size() : -1) << " replies";
            return -1;
        }
        for (size_t i = 0; i < out.size(); ++i) out[i].SerializeTo(out_buf);
        ctx->batched = 0;
        return 0;
    }
    out.SerializeTo(out_buf);
    return 0;
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
        if (ctx->pi.auth_replies > 0) {
            // replies to AUTH/SELECT sent in front of this request: each
            // must be +OK (reference: redis_protocol.cpp:220-243)
            const int rc = ctx->partial.ConsumePartial(source, ctx->pi.auth_replies);
            if (rc < 0) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
            if (rc == 0) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
            for (int i = 0; i < ctx->partial.reply_size(); ++i) {
                const RedisReply& r = ctx->partial.reply(i);
                if (r.type() != REDIS_REPLY_STATUS || r.data() != "OK") {
                    LOG(ERROR) << "redis authentication failed: " << r.ToString();
                    return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
                }
            }
            ctx->partial.Clear();
            ctx->pi.auth_replies = 0;
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
    // execute every complete command now, in order; one write per batch.
    // A command is run once the next one was parsed (or none is left), so
    // the last command of what arrived runs with flush_batched.
    Buf out;
    int rc;
    std::vector<std::string> cur, next;
    bool have = false, broken = false;
    for (;;) {
        rc = parse_command(ctx, source, &next);
        if (rc <= 0) break;
        if (have && run_command(const_cast<Server*>(server), ctx, cur, false, &out) != 0) {
            broken = true;
            break;
        }
        cur.swap(next);
        next.clear();
        have = true;
    }
    if (have && !broken && run_command(const_cast<Server*>(server), ctx, cur, true, &out) != 0) broken = true;
    // a handler that broke the protocol drops the connection without the
    // replies gathered so far (reference redis_protocol.cpp:177-185); a
    // malformed command still gets the replies of the commands before it
    if (broken) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    if (!out.empty()) socket->Write(&out);
    if (rc < 0) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    // every complete command ran inside parse; what is left is the start
    // of the next one: read more (reference: redis_protocol.cpp:167-194)
    return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
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
                      const Buf& request_buf, const Authenticator* auth) {
    (void)correlation_id;
    if (auth) {  // first request of the connection: AUTH / SELECT in front
        std::string cred;
        if (auth->GenerateCredential(&cred) != 0) {
            cntl->SetFailed(ERPCAUTH, "fail to generate redis credential");
            return;
        }
        packet->append(cred);
        const RedisAuthenticator* ra = dynamic_cast<const RedisAuthenticator*>(auth);
        cntl->_auth_replies = ra ? ra->auth_replies() : 1;
    }
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
