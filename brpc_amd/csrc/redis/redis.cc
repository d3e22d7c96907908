#include "redis/redis.h"

#include <cctype>
#include <cerrno>

#include <cstdarg>
#include <cstring>
#include <mutex>

#include "base/util.h"

namespace mrpc {

const pb::Descriptor* OpaqueDescriptor(const char* full_name) {
    static std::mutex mu;
    static std::map<std::string, pb::Descriptor*>* all = new std::map<std::string, pb::Descriptor*>;
    std::lock_guard<std::mutex> g(mu);
    pb::Descriptor*& d = (*all)[full_name];
    if (!d) {
        d = new pb::Descriptor;
        d->full_name = full_name;
        const char* dot = strrchr(full_name, '.');
        d->name = dot ? dot + 1 : full_name;
        d->BuildIndex();
    }
    return d;
}

const char* RedisReplyTypeToString(RedisReplyType t) {
    switch (t) {
    case REDIS_REPLY_STRING: return "string";
    case REDIS_REPLY_ARRAY: return "array";
    case REDIS_REPLY_INTEGER: return "integer";
    case REDIS_REPLY_NIL: return "nil";
    case REDIS_REPLY_STATUS: return "status";
    case REDIS_REPLY_ERROR: return "error";
    }
    return "unknown";
}

// ------------------------------------------------------------------ reply
void RedisReply::SerializeTo(Buf* out) const {
    switch (_type) {
    case REDIS_REPLY_STATUS: out->append("+" + _str + "\r\n"); break;
    case REDIS_REPLY_ERROR: out->append("-" + _str + "\r\n"); break;
    case REDIS_REPLY_INTEGER: out->append(":" + std::to_string(_integer) + "\r\n"); break;
    case REDIS_REPLY_NIL: out->append("$-1\r\n"); break;
    case REDIS_REPLY_STRING:
        out->append("$" + std::to_string(_str.size()) + "\r\n");
        out->append(_str);
        out->append("\r\n");
        break;
    case REDIS_REPLY_ARRAY:
        out->append("*" + std::to_string(_array.size()) + "\r\n");
        for (const RedisReply& r : _array) r.SerializeTo(out);
        break;
    }
}

namespace {
// Reads a CRLF-terminated line starting at `pos`. Returns the index after
// the CRLF, 0 if incomplete, -1 if too long.
int64_t read_line(const Buf& in, size_t pos, std::string* line) {
    line->clear();
    const size_t kMax = 64 * 1024;
    char buf[256];
    size_t off = pos;
    while (off < in.size()) {
        const size_t n = in.copy_to(buf, std::min(sizeof(buf), in.size() - off), off);
        for (size_t i = 0; i < n; ++i) {
            if (buf[i] == '\n') {
                line->append(buf, i);
                if (!line->empty() && line->back() == '\r') line->pop_back();
                return (int64_t)(off + i + 1);
            }
        }
        line->append(buf, n);
        off += n;
        if (line->size() > kMax) return -1;
    }
    return 0;
}

// RESP integers: an optional '-' and digits, nothing else.
bool parse_int(const std::string& s, long long* out) {
    if (s.empty() || s.size() > 20) return false;
    char* end = nullptr;
    errno = 0;
    *out = strtoll(s.c_str(), &end, 10);
    return errno == 0 && end && *end == '\0' && (isdigit((unsigned char)s.back()));
}

// Parses one reply at `pos`; returns the end offset, 0 incomplete, -1 bad.
int64_t parse_at(const Buf& in, size_t pos, RedisReply* r, int depth) {
    if (depth > 64) return -1;
    std::string line;
    const int64_t e = read_line(in, pos, &line);
    if (e <= 0) return e;
    if (line.empty()) return -1;
    const char t = line[0];
    const std::string rest = line.substr(1);
    switch (t) {
    case '+': r->SetStatus(rest); return e;
    case '-': r->SetError(rest); return e;
    case ':': {
        long long v;
        if (!parse_int(rest, &v)) return -1;
        r->SetInteger(v);
        return e;
    }
    case '$': {
        long long n;
        if (!parse_int(rest, &n) || n < -1) return -1;
        if (n == -1) {
            r->SetNil();
            return e;
        }
        if ((size_t)e + n + 2 > in.size()) return 0;
        std::string s;
        in.copy_to(&s, (size_t)n, (size_t)e);
        r->SetString(s);
        return e + n + 2;
    }
    case '*': {
        long long n;
        if (!parse_int(rest, &n) || n < -1) return -1;
        if (n == -1) {
            r->SetNil();
            return e;
        }
        if (n > 1024 * 1024) return -1;
        r->SetArray((size_t)n);
        int64_t p = e;
        for (long long i = 0; i < n; ++i) {
            p = parse_at(in, (size_t)p, &(*r)[(size_t)i], depth + 1);
            if (p <= 0) return p;
        }
        return p;
    }
    default: return -1;
    }
}
}  // namespace

int RedisReply::ConsumePartial(Buf* in) {
    const int64_t e = parse_at(*in, 0, this, 0);
    if (e <= 0) return (int)e;
    in->pop_front((size_t)e);
    return 1;
}

std::string RedisReply::ToString() const {
    switch (_type) {
    case REDIS_REPLY_STRING:
    case REDIS_REPLY_STATUS: return _str;
    case REDIS_REPLY_ERROR: return "(error) " + _str;
    case REDIS_REPLY_INTEGER: return "(integer) " + std::to_string(_integer);
    case REDIS_REPLY_NIL: return "(nil)";
    case REDIS_REPLY_ARRAY: {
        std::string s = "[";
        for (size_t i = 0; i < _array.size(); ++i) s += (i ? ", " : "") + _array[i].ToString();
        return s + "]";
    }
    }
    return "";
}

// ------------------------------------------------------------------ request
const pb::Descriptor* RedisRequest::GetDescriptor() const { return OpaqueDescriptor("mrpc.RedisRequest"); }
const pb::Descriptor* RedisResponse::GetDescriptor() const { return OpaqueDescriptor("mrpc.RedisResponse"); }

void RedisRequest::Clear() {
    _buf.clear();
    _ncommand = 0;
    _has_error = false;
}

bool RedisRequest::AddCommandByComponents(const std::vector<std::string>& args) {
    if (args.empty()) {
        _has_error = true;
        return false;
    }
    _buf.append("*" + std::to_string(args.size()) + "\r\n");
    for (const std::string& a : args) {
        _buf.append("$" + std::to_string(a.size()) + "\r\n");
        _buf.append(a);
        _buf.append("\r\n");
    }
    ++_ncommand;
    return true;
}

bool RedisRequest::AddCommand(const char* fmt, ...) {
    // Split the format into components the way redis-cli does (reference:
    // src/brpc/redis_command.cpp, RedisCommandFormatV): spaces separate
    // components; a '...' or "..." string is one component (spaces kept,
    // possibly empty) and also ends the component before it, so
    // "get ''key" is {get, "", key}. Inside quotes a backslash escapes only
    // the quote character itself ('\'' -> ', "\"" -> "); any other
    // backslash stays. Each %s / %d / %u / %lld / %b consumes an argument
    // and becomes part of the current component, so %s values may hold
    // spaces or quotes.
    std::vector<std::string> comps;
    std::string cur;
    bool in_comp = false;
    char quote = 0;
    va_list ap;
    va_start(ap, fmt);
    auto fail = [&] {
        va_end(ap);
        _has_error = true;
        return false;
    };
    for (const char* p = fmt; *p; ++p) {
        if (quote) {
            if (*p == '\\' && p[1] == quote) {
                cur.push_back(quote);
                ++p;
                continue;
            }
            if (*p == quote) {  // the quoted component ends here
                comps.push_back(cur);
                cur.clear();
                quote = 0;
                in_comp = false;
                continue;
            }
        } else if (*p == ' ') {
            if (in_comp) comps.push_back(cur);
            cur.clear();
            in_comp = false;
            continue;
        } else if (*p == '\'' || *p == '"') {
            if (in_comp) comps.push_back(cur);
            cur.clear();
            in_comp = false;
            quote = *p;
            continue;
        }
        in_comp = true;
        if (*p != '%') {
            cur.push_back(*p);
            continue;
        }
        ++p;
        if (*p == 's') {
            cur.append(va_arg(ap, const char*));
        } else if (*p == 'd') {
            cur.append(std::to_string(va_arg(ap, int)));
        } else if (*p == 'u') {
            cur.append(std::to_string(va_arg(ap, unsigned)));
        } else if (*p == 'l' && p[1] == 'l' && p[2] == 'd') {
            cur.append(std::to_string(va_arg(ap, long long)));
            p += 2;
        } else if (*p == 'b') {  // binary: pointer + size_t
            const char* d = va_arg(ap, const char*);
            const size_t n = va_arg(ap, size_t);
            cur.append(d, n);
        } else if (*p == '%') {
            cur.push_back('%');
        } else {
            return fail();
        }
    }
    if (quote) return fail();  // unterminated quote
    va_end(ap);
    if (in_comp) comps.push_back(cur);
    return AddCommandByComponents(comps);
}

bool RedisRequest::SerializeTo(Buf* out) const {
    if (_has_error) return false;
    out->append(_buf);
    return true;
}

std::string RedisRequest::ToString() const { return _buf.to_string(); }

int RedisResponse::ConsumePartial(Buf* in, int count) {
    while ((int)_replies.size() < count) {
        RedisReply r;
        const int rc = r.ConsumePartial(in);
        if (rc <= 0) return rc;
        _replies.push_back(std::move(r));
    }
    return 1;
}

// ------------------------------------------------------------------ service
bool RedisService::AddCommandHandler(const std::string& name, RedisCommandHandler* handler) {
    const std::string n = to_lower(name);
    if (_handlers.count(n)) return false;
    _handlers[n] = handler;
    return true;
}

RedisCommandHandler* RedisService::FindCommandHandler(const std::string& name) const {
    auto it = _handlers.find(to_lower(name));
    return it == _handlers.end() ? nullptr : it->second;
}

}  // namespace mrpc
