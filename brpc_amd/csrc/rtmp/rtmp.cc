#include "rtmp/rtmp.h"

#include <cmath>

#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/sync.h"
#include "net/input_messenger.h"
#include "net/socket.h"
#include "net/socket_map.h"
#include "policy/policies.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rtmp/handshake.h"

DECLARE_uint64(max_body_size);

namespace mrpc {

using rtmp::AMFValue;

namespace rtmp_detail {

static const size_t kHandshakeSize = 1536;
static const uint32_t kDefaultChunkSize = 128;
static const uint32_t kCommandCsid = 3;
static const uint32_t kAudioCsid = 4;
static const uint32_t kDataCsid = 5;
static const uint32_t kVideoCsid = 6;
static const uint32_t kControlCsid = 2;

std::atomic<int64_t> g_complex_handshakes{0}, g_unsigned_c2{0};

static void be24(std::string* o, uint32_t v) {
    o->push_back((char)(v >> 16));
    o->push_back((char)(v >> 8));
    o->push_back((char)v);
}
static void be32(std::string* o, uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) o->push_back((char)(v >> s));
}
static uint32_t rd24(const uint8_t* p) { return ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2]; }
static uint32_t rd32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

struct ChunkState {
    uint32_t timestamp = 0;  // absolute timestamp of the current message
    uint32_t ts_delta = 0;
    uint32_t length = 0;
    uint8_t type = 0;
    uint32_t stream_id = 0;
    bool extended = false;
    Buf partial;             // bytes of the message being assembled
    bool has_header = false;
};

// One RTMP connection (either side). Lives in the socket's parsing context
// and is shared with streams/clients that send on it.
class Connection : public std::enable_shared_from_this<Connection> {
public:
    enum State { HS_WAIT_C0C1, HS_WAIT_C2, HS_WAIT_S0S1S2, ESTABLISHED };
    typedef std::function<void(const std::vector<AMFValue>& args, bool ok)> TxCallback;

    Connection(bool server, SocketId sid) : _server(server), _sid(sid) {
        _state = server ? HS_WAIT_C0C1 : HS_WAIT_S0S1S2;
    }

    bool is_server() const { return _server; }
    SocketId socket_id() const { return _sid; }
    EndPoint remote_side() const {
        SocketUniquePtr s;
        return Socket::Address(_sid, &s) == 0 ? s->remote_side() : EndPoint();
    }

    int Write(Buf* data) {
        SocketUniquePtr s;
        if (Socket::Address(_sid, &s) != 0) {
            errno = EFAILEDSOCKET;
            return -1;
        }
        WriteOptions wo;
        wo.ignore_eovercrowded = true;
        return s->Write(data, &wo);
    }

    // Chunks one message with the negotiated outgoing chunk size.
    int SendMessage(uint32_t csid, uint8_t type, uint32_t ts, uint32_t stream_id, const Buf& body) {
        std::lock_guard<fiber::Mutex> g(_write_mu);
        Buf out;
        std::string h;
        auto basic = [&](uint8_t fmt) {
            if (csid < 64) {
                h.push_back((char)((fmt << 6) | csid));
            } else if (csid < 320) {
                h.push_back((char)(fmt << 6));
                h.push_back((char)(csid - 64));
            } else {
                h.push_back((char)((fmt << 6) | 1));
                h.push_back((char)((csid - 64) & 0xff));
                h.push_back((char)((csid - 64) >> 8));
            }
        };
        const bool ext = ts >= 0xffffff;
        basic(0);
        be24(&h, ext ? 0xffffff : ts);
        be24(&h, (uint32_t)body.size());
        h.push_back((char)type);
        h.append((const char*)&stream_id, 4);  // message stream id is little endian
        if (ext) be32(&h, ts);
        out.append(h);
        Buf rest = body;
        for (bool first = true; first || !rest.empty(); first = false) {
            if (!first) {
                h.clear();
                basic(3);
                if (ext) be32(&h, ts);
                out.append(h);
            }
            rest.cutn(&out, _out_chunk_size);
        }
        return Write(&out);
    }

    int SendControl(uint8_t type, const std::string& payload) {
        return SendMessage(kControlCsid, type, 0, 0, Buf(payload));
    }

    int SendCommand(uint32_t stream_id, const std::vector<AMFValue>& values) {
        std::string body;
        for (const AMFValue& v : values) rtmp::WriteAMF(&body, v);
        return SendMessage(kCommandCsid, RTMP_COMMAND_AMF0, 0, stream_id, Buf(body));
    }

    // Client: a command expecting _result/_error with its transaction id.
    int Call(const std::string& name, uint32_t stream_id, std::vector<AMFValue> args, TxCallback cb) {
        double tx;
        {
            std::lock_guard<std::mutex> g(_mu);
            tx = ++_next_tx;
            _pending_tx[tx] = std::move(cb);
        }
        std::vector<AMFValue> v;
        v.push_back(AMFValue::String(name));
        v.push_back(AMFValue::Number(tx));
        for (AMFValue& a : args) v.push_back(std::move(a));
        return SendCommand(stream_id, v);
    }

    void AddStream(uint32_t id, RtmpStreamBase* s, bool owned) {
        std::lock_guard<std::mutex> g(_mu);
        _streams[id] = StreamEntry{s, owned};
    }
    RtmpStreamBase* FindStream(uint32_t id) {
        std::lock_guard<std::mutex> g(_mu);
        auto it = _streams.find(id);
        return it == _streams.end() ? nullptr : it->second.s;
    }
    // Detach and stop; deletes owned (server) streams.
    void RemoveStream(uint32_t id) {
        StreamEntry e{nullptr, false};
        {
            std::lock_guard<std::mutex> g(_mu);
            auto it = _streams.find(id);
            if (it == _streams.end()) return;
            e = it->second;
            _streams.erase(it);
        }
        e.s->CallOnStop();
        if (e.owned) delete e.s;
    }
    void StopAll() {
        std::map<uint32_t, StreamEntry> all;
        std::map<double, TxCallback> txs;
        std::map<uint32_t, StatusFn> listeners;
        {
            std::lock_guard<std::mutex> g(_mu);
            all.swap(_streams);
            txs.swap(_pending_tx);
            listeners.swap(_status_listeners);
            _closed = true;
        }
        for (auto& kv : all) {
            kv.second.s->CallOnStop();
            if (kv.second.owned) delete kv.second.s;
        }
        for (auto& kv : txs) kv.second(std::vector<AMFValue>(), false);
        for (auto& kv : listeners) kv.second(std::vector<AMFValue>());
    }
    bool closed() {
        std::lock_guard<std::mutex> g(_mu);
        return _closed;
    }

    // Parse: consumes handshake bytes and complete messages, dispatching
    // each in order. Returns false on a protocol error.
    bool Consume(Buf* source, Socket* sock, const Server* server) {
        const size_t before = source->size();
        const bool ok = ConsumeImpl(source, sock, server);
        if (ok) OnBytesReceived(before - source->size());
        return ok;
    }

    // client-side hooks
    typedef std::function<void(const std::vector<AMFValue>& args)> StatusFn;
    std::function<void()> on_handshake_done;
    // onStatus of a stream (empty args: the connection closed)
    void SetStatusListener(uint32_t stream_id, StatusFn fn) {
        std::lock_guard<std::mutex> g(_mu);
        if (fn) {
            _status_listeners[stream_id] = std::move(fn);
        } else {
            _status_listeners.erase(stream_id);
        }
    }
    void set_out_chunk_size(uint32_t n) {
        std::lock_guard<fiber::Mutex> g(_write_mu);
        _out_chunk_size = n;
    }
    RtmpConnectRequest connect_req;
    // handshake: set by the client when it offered a complex C1
    std::string c1_digest;
    bool complex_handshake = false;  // both sides signed the handshake
    int64_t acks_sent = 0, pings_answered = 0;
    std::function<void()> on_pong;  // guarded by _mu
    void SetPongCallback(std::function<void()> fn) {
        std::lock_guard<std::mutex> g(_mu);
        on_pong = std::move(fn);
    }

private:
    struct StreamEntry {
        RtmpStreamBase* s;
        bool owned;
    };
    bool ConsumeImpl(Buf* source, Socket* sock, const Server* server);
    bool OnMessage(uint8_t type, uint32_t ts, uint32_t stream_id, Buf& body, const Server* server);
    // Acknowledgement (type 3) after every `peer window` bytes received.
    void OnBytesReceived(size_t n) {
        if (!n || _state != ESTABLISHED) return;
        _bytes_in += n;
        if (_peer_window && _bytes_in - _last_ack_at >= _peer_window) {
            _last_ack_at = _bytes_in;
            std::string p;
            be32(&p, (uint32_t)_bytes_in);  // sequence number wraps at 2^32
            SendControl(RTMP_ACK, p);
            ++acks_sent;
        }
    }
    bool OnCommand(uint32_t stream_id, const std::vector<AMFValue>& v, const Server* server);

public:
    // onStatus of a stream (transaction 0, null command object, info).
    void ReplyStatus(uint32_t stream_id, const char* level, const char* code, const std::string& desc);
    // `_error` (transaction 0) of a stream command: level error + code.
    void ReplyError(uint32_t stream_id, const char* code, const std::string& desc);

private:

    const bool _server;
    const SocketId _sid;
    State _state;
    std::string _s1_digest;  // server: digest of the S1 we sent
    uint64_t _bytes_in = 0, _last_ack_at = 0;
    uint32_t _peer_window = 0;  // from the peer's Window Acknowledgement Size
    uint32_t _in_chunk_size = kDefaultChunkSize;
    uint32_t _out_chunk_size = kDefaultChunkSize;
    std::map<uint32_t, ChunkState> _chunks;
    fiber::Mutex _write_mu;  // fiber-aware: held across Socket::Write
    std::mutex _mu;
    std::map<uint32_t, StreamEntry> _streams;
    std::map<double, TxCallback> _pending_tx;
    std::map<uint32_t, StatusFn> _status_listeners;
    double _next_tx = 1;
    uint32_t _next_stream_id = 1;
    bool _closed = false;
};

bool Connection::ConsumeImpl(Buf* source, Socket* sock, const Server* server) {
    for (;;) {
        if (_state == HS_WAIT_C0C1) {
            if (source->size() < 1 + kHandshakeSize) return true;
            std::string c0c1;
            source->cutn(&c0c1, 1 + kHandshakeSize);
            if (c0c1[0] != 3) return false;
            const std::string c1 = c0c1.substr(1);
            std::string s(1, (char)3);
            std::string c1_digest;
            rtmp::HandshakeSchema schema = rtmp::kSchemaInvalid;
            if (rtmp::OffersComplexHandshake(c1)) schema = rtmp::ValidateComplexC1(c1, &c1_digest);
            if (schema != rtmp::kSchemaInvalid) {
                // complex: S1 with our digest in the client's schema, S2 keyed by its digest
                std::string s1, s2;
                rtmp::MakeComplexS1(schema, &s1);
                rtmp::ValidateComplexS1(s1, &_s1_digest);
                rtmp::MakeComplexS2(c1_digest, &s2);
                s += s1;
                s += s2;
                complex_handshake = true;
                g_complex_handshakes.fetch_add(1, std::memory_order_relaxed);
            } else {
                // simple: S1 (time, zero, random) + S2 (echo of C1)
                be32(&s, (uint32_t)(monotonic_us() / 1000));
                be32(&s, 0);
                for (size_t i = 8; i < kHandshakeSize; ++i) s.push_back((char)fast_rand());
                s.append(c1);
            }
            Buf out(s);
            if (Write(&out) != 0) return false;
            _state = HS_WAIT_C2;
            continue;
        }
        if (_state == HS_WAIT_C2) {
            if (source->size() < kHandshakeSize) return true;
            if (complex_handshake) {
                std::string c2;
                source->cutn(&c2, kHandshakeSize);
                // some encoders echo S1 instead of signing it: accept, but count
                if (!rtmp::ValidateComplexC2(c2, _s1_digest)) g_unsigned_c2.fetch_add(1, std::memory_order_relaxed);
            } else {
                source->pop_front(kHandshakeSize);
            }
            _state = ESTABLISHED;
            continue;
        }
        if (_state == HS_WAIT_S0S1S2) {
            if (source->size() < 1 + 2 * kHandshakeSize) return true;
            std::string s0s1s2;
            source->cutn(&s0s1s2, 1 + 2 * kHandshakeSize);
            if (s0s1s2[0] != 3) return false;
            const std::string s1 = s0s1s2.substr(1, kHandshakeSize), s2 = s0s1s2.substr(1 + kHandshakeSize);
            std::string s1_digest, c2;
            if (!c1_digest.empty() && rtmp::OffersComplexHandshake(s1) &&
                rtmp::ValidateComplexS1(s1, &s1_digest) != rtmp::kSchemaInvalid) {
                // the server signed S1 and S2 (our C1 digest): answer with a signed C2
                complex_handshake = rtmp::ValidateComplexS2(s2, c1_digest);
                if (!complex_handshake) return false;  // a server that signs S1 must sign S2
                rtmp::MakeComplexC2(s1_digest, &c2);
            } else {
                c2 = s1;  // simple: echo S1
            }
            Buf c2buf(c2);
            if (Write(&c2buf) != 0) return false;
            _state = ESTABLISHED;
            if (on_handshake_done) on_handshake_done();
            continue;
        }
        // ---- one chunk
        uint8_t hb[3];
        const size_t have = source->copy_to(hb, 3);
        if (have < 1) return true;
        const uint8_t fmt = hb[0] >> 6;
        uint32_t csid = hb[0] & 0x3f;
        size_t basic = 1;
        if (csid == 0) {
            if (have < 2) return true;
            csid = 64 + hb[1];
            basic = 2;
        } else if (csid == 1) {
            if (have < 3) return true;
            csid = 64 + hb[1] + ((uint32_t)hb[2] << 8);
            basic = 3;
        }
        static const size_t kMsgHeader[4] = {11, 7, 3, 0};
        ChunkState& cs = _chunks[csid];
        size_t hlen = basic + kMsgHeader[fmt];
        uint8_t h[18];
        if (source->size() < hlen) return true;
        source->copy_to(h, hlen);
        const uint8_t* m = h + basic;
        uint32_t ts_field = 0;
        bool ext = cs.extended;
        if (fmt <= 2) {
            ts_field = rd24(m);
            ext = ts_field == 0xffffff;
        }
        if (ext) {
            if (source->size() < hlen + 4) return true;
            uint8_t e[4];
            source->copy_to(e, 4, hlen);
            ts_field = rd32(e);
            hlen += 4;
        }
        if (fmt == 3 && !cs.has_header) return false;
        // Size of this chunk's payload
        uint32_t msg_len = cs.length;
        if (fmt <= 1) msg_len = rd24(m + 3);
        const size_t already = (fmt == 3) ? cs.partial.size() : 0;
        if (msg_len > FLAGS_max_body_size) return false;
        const size_t chunk = std::min<size_t>(_in_chunk_size, msg_len - already);
        if (source->size() < hlen + chunk) return true;
        // Commit the header.
        if (fmt == 0) {
            cs.timestamp = ts_field;
            cs.ts_delta = 0;
            cs.length = msg_len;
            cs.type = m[6];
            memcpy(&cs.stream_id, m + 7, 4);
        } else if (fmt == 1) {
            cs.ts_delta = ts_field;
            cs.timestamp += ts_field;
            cs.length = msg_len;
            cs.type = m[6];
        } else if (fmt == 2) {
            cs.ts_delta = ts_field;
            cs.timestamp += ts_field;
        } else if (already == 0) {
            cs.timestamp += cs.ts_delta;  // fmt3 starting a new message
        }
        if (fmt <= 2) cs.partial.clear();
        cs.extended = ext;
        cs.has_header = true;
        source->pop_front(hlen);
        source->cutn(&cs.partial, chunk);
        if (cs.partial.size() < cs.length) continue;
        Buf body;
        body.swap(cs.partial);
        if (!OnMessage(cs.type, cs.timestamp, cs.stream_id, body, server)) return false;
    }
}

void Connection::ReplyStatus(uint32_t stream_id, const char* level, const char* code, const std::string& desc) {
    AMFValue info = AMFValue::Object();
    info.Set("level", AMFValue::String(level));
    info.Set("code", AMFValue::String(code));
    info.Set("description", AMFValue::String(desc));
    SendCommand(stream_id, {AMFValue::String("onStatus"), AMFValue::Number(0), AMFValue::Null(), info});
}

bool Connection::OnMessage(uint8_t type, uint32_t ts, uint32_t stream_id, Buf& body, const Server* server) {
    switch (type) {
    case RTMP_SET_CHUNK_SIZE: {
        uint8_t b[4];
        if (body.copy_to(b, 4) < 4) return false;
        const uint32_t sz = rd32(b) & 0x7fffffff;
        if (sz < 1) return false;
        _in_chunk_size = sz;
        return true;
    }
    case RTMP_ABORT: {
        uint8_t b[4];
        if (body.copy_to(b, 4) == 4) _chunks.erase(rd32(b));
        return true;
    }
    case RTMP_WINDOW_ACK_SIZE: {
        uint8_t b[4];
        if (body.copy_to(b, 4) == 4) _peer_window = rd32(b);
        return true;
    }
    case RTMP_USER_CONTROL: {
        uint8_t b[10];
        const size_t nb = body.copy_to(b, 10);
        const int event = nb >= 2 ? ((b[0] << 8) | b[1]) : -1;
        if (event == 3 && nb >= 10 && _server) {  // SetBufferLength{stream id, ms}
            RtmpStreamBase* st = FindStream(rd32(b + 2));
            if (st) static_cast<RtmpServerStream*>(st)->OnSetBufferLength(rd32(b + 6));
            return true;
        }
        if (event == 2) return true;  // StreamDry: nothing to do on our side
        if (body.copy_to(b, 6) == 6 && ((b[0] << 8) | b[1]) == 7) {  // PingResponse to our Ping()
            std::function<void()> fn;
            {
                std::lock_guard<std::mutex> g(_mu);
                fn.swap(on_pong);
            }
            if (fn) fn();
            return true;
        }
        if (body.copy_to(b, 6) == 6 && ((b[0] << 8) | b[1]) == 6) {  // PingRequest -> PingResponse
            std::string p;
            p.push_back(0);
            p.push_back(7);
            p.append((const char*)b + 2, 4);
            SendControl(RTMP_USER_CONTROL, p);
            ++pings_answered;
        }
        return true;
    }
    case RTMP_ACK:
    case RTMP_SET_PEER_BANDWIDTH: return true;
    case RTMP_COMMAND_AMF3:
    case RTMP_DATA_AMF3: {
        // AMF3 messages of encoders carry a 0 format byte and AMF0 values
        uint8_t f = 1;
        if (body.copy_to(&f, 1) != 1 || f != 0) return true;  // true AMF3 payloads are ignored
        body.pop_front(1);
        return OnMessage(type == RTMP_COMMAND_AMF3 ? RTMP_COMMAND_AMF0 : RTMP_DATA_AMF0, ts, stream_id, body, server);
    }
    case RTMP_COMMAND_AMF0: {
        const std::string s = body.to_string();
        std::vector<AMFValue> v;
        if (!rtmp::ReadAMFList(s.data(), s.size(), &v) || v.empty() || v[0].type() != rtmp::AMF_STRING) return false;
        return OnCommand(stream_id, v, server);
    }
    case RTMP_DATA_AMF0: {
        RtmpStreamBase* st = FindStream(stream_id);
        if (!st) return true;
        const std::string s = body.to_string();
        std::vector<AMFValue> v;
        if (!rtmp::ReadAMFList(s.data(), s.size(), &v) || v.empty()) return true;
        size_t i = 0;
        std::string name = v[0].type() == rtmp::AMF_STRING ? v[0].str() : "";
        if (name == "@setDataFrame" && v.size() > 1) {
            i = 1;
            name = v[1].str();
        }
        st->CallOnFirstMessage();
        if (name == "onCuePoint") {
            RtmpCuePoint cp;
            cp.timestamp = ts;
            if (i + 1 < v.size()) cp.data = v[i + 1];
            st->OnCuePoint(&cp);
            return true;
        }
        RtmpMetaData md;
        md.timestamp = ts;
        if (i + 1 < v.size()) md.data = v[i + 1];
        st->OnMetaData(&md, name);
        return true;
    }
    case RTMP_AUDIO: {
        RtmpStreamBase* st = FindStream(stream_id);
        if (!st || body.empty()) return true;
        char h;
        body.cut1(&h);
        st->CallOnFirstMessage();
        RtmpAudioMessage a;
        a.timestamp = ts;
        a.codec = (uint8_t)h >> 4;
        a.rate = ((uint8_t)h >> 2) & 3;
        a.bits = ((uint8_t)h >> 1) & 1;
        a.type = (uint8_t)h & 1;
        a.data.swap(body);
        st->OnAudioMessage(&a);
        return true;
    }
    case RTMP_VIDEO: {
        RtmpStreamBase* st = FindStream(stream_id);
        if (!st || body.empty()) return true;
        char h;
        body.cut1(&h);
        st->CallOnFirstMessage();
        RtmpVideoMessage vm;
        vm.timestamp = ts;
        vm.frame_type = (uint8_t)h >> 4;
        vm.codec = (uint8_t)h & 0xf;
        vm.data.swap(body);
        st->OnVideoMessage(&vm);
        return true;
    }
    default: return true;  // unknown messages are ignored
    }
}

bool Connection::OnCommand(uint32_t stream_id, const std::vector<AMFValue>& v, const Server* server) {
    const std::string& name = v[0].str();
    const double tx = v.size() > 1 ? v[1].number() : 0;
    if (name == "_error" && tx == 0 && stream_id != 0) {
        // a stream command's failure (seek / pause): reported like onStatus
        StatusFn fn;
        {
            std::lock_guard<std::mutex> g(_mu);
            auto it = _status_listeners.find(stream_id);
            if (it != _status_listeners.end()) fn = it->second;
        }
        if (fn) fn(v);
        return true;
    }
    if (name == "_result" || name == "_error") {
        TxCallback cb;
        {
            std::lock_guard<std::mutex> g(_mu);
            auto it = _pending_tx.find(tx);
            if (it == _pending_tx.end()) return true;
            cb = std::move(it->second);
            _pending_tx.erase(it);
        }
        cb(v, name == "_result");
        return true;
    }
    if (name == "onStatus") {
        StatusFn fn;
        {
            std::lock_guard<std::mutex> g(_mu);
            auto it = _status_listeners.find(stream_id);
            if (it != _status_listeners.end()) fn = it->second;
        }
        if (fn) fn(v);
        return true;
    }
    if (!_server) return true;
    RtmpService* svc = server ? server->options().rtmp_service : nullptr;
    if (!svc) return false;
    if (name == "connect") {
        if (v.size() > 2 && v[2].type() == rtmp::AMF_OBJECT) {
            if (const AMFValue* a = v[2].Find("app")) connect_req.app = a->str();
            if (const AMFValue* a = v[2].Find("tcUrl")) connect_req.tcUrl = a->str();
            if (const AMFValue* a = v[2].Find("flashVer")) connect_req.flashVer = a->str();
        }
        std::string p;
        be32(&p, 2500000);
        SendControl(RTMP_WINDOW_ACK_SIZE, p);
        p.clear();
        be32(&p, 2500000);
        p.push_back(2);  // dynamic
        SendControl(RTMP_SET_PEER_BANDWIDTH, p);
        p.clear();
        be32(&p, 60000);
        SendControl(RTMP_SET_CHUNK_SIZE, p);
        _out_chunk_size = 60000;
        AMFValue props = AMFValue::Object();
        props.Set("fmsVer", AMFValue::String("FMS/3,0,1,123"));
        props.Set("capabilities", AMFValue::Number(31));
        AMFValue info = AMFValue::Object();
        info.Set("level", AMFValue::String("status"));
        info.Set("code", AMFValue::String("NetConnection.Connect.Success"));
        info.Set("description", AMFValue::String("Connection succeeded."));
        info.Set("objectEncoding", AMFValue::Number(0));
        SendCommand(0, {AMFValue::String("_result"), AMFValue::Number(tx), props, info});
        return true;
    }
    if (name == "createStream") {
        RtmpServerStream* st = svc->NewStream(connect_req);
        if (!st) {
            SendCommand(0, {AMFValue::String("_error"), AMFValue::Number(tx), AMFValue::Null(), AMFValue::Null()});
            return true;
        }
        uint32_t id;
        {
            std::lock_guard<std::mutex> g(_mu);
            id = _next_stream_id++;
        }
        st->_conn = shared_from_this();
        st->_stream_id = id;
        AddStream(id, st, true);
        SendCommand(0, {AMFValue::String("_result"), AMFValue::Number(tx), AMFValue::Null(), AMFValue::Number(id)});
        return true;
    }
    if (name == "deleteStream" || name == "closeStream") {
        uint32_t id = stream_id;
        if (name == "deleteStream" && v.size() > 3) id = (uint32_t)v[3].number();
        RemoveStream(id);
        return true;
    }
    RtmpServerStream* st = static_cast<RtmpServerStream*>(FindStream(stream_id));
    if (name == "publish") {
        if (!st) return true;
        std::string err;
        const std::string sname = v.size() > 3 ? v[3].str() : "";
        const std::string type = v.size() > 4 ? v[4].str() : "live";
        st->OnPublish(sname, type, &err);
        if (err.empty()) {
            ReplyStatus(stream_id, "status", "NetStream.Publish.Start", "Start publishing " + sname);
        } else {
            ReplyStatus(stream_id, "error", "NetStream.Publish.BadName", err);
        }
        return true;
    }
    if (name == "play") {
        if (!st) return true;
        RtmpPlayOptions po;
        po.stream_name = v.size() > 3 ? v[3].str() : "";
        if (v.size() > 4 && v[4].type() == rtmp::AMF_NUMBER) po.start = v[4].number();
        if (v.size() > 5 && v[5].type() == rtmp::AMF_NUMBER) po.duration = v[5].number();
        if (v.size() > 6 && v[6].type() == rtmp::AMF_BOOLEAN) po.reset = v[6].boolean();
        std::string err;
        st->OnPlay(po, &err);
        if (err.empty()) {
            std::string p;
            p.push_back(0);
            p.push_back(0);  // StreamBegin
            be32(&p, stream_id);
            SendControl(RTMP_USER_CONTROL, p);
            ReplyStatus(stream_id, "status", "NetStream.Play.Start", "Start playing " + po.stream_name);
        } else {
            ReplyStatus(stream_id, "error", "NetStream.Play.StreamNotFound", err);
        }
        return true;
    }
    if (name == "play2") {
        if (!st || v.size() < 4 || v[3].type() != rtmp::AMF_OBJECT) return true;
        RtmpPlay2Options o;
        const AMFValue& obj = v[3];
        if (const AMFValue* a = obj.Find("len")) o.len = a->number();
        if (const AMFValue* a = obj.Find("offset")) o.offset = a->number();
        if (const AMFValue* a = obj.Find("oldStreamName")) o.old_stream_name = a->str();
        if (const AMFValue* a = obj.Find("start")) o.start = a->number();
        if (const AMFValue* a = obj.Find("streamName")) o.stream_name = a->str();
        if (const AMFValue* a = obj.Find("transition")) o.transition = a->str();
        st->OnPlay2(o);
        return true;
    }
    if (name == "seek") {
        if (!st || v.size() < 4 || v[3].type() != rtmp::AMF_NUMBER) return true;
        if (st->OnSeek(v[3].number()) == 0) {
            ReplyStatus(stream_id, "status", "NetStream.Seek.Notify", "Seek successfully.");
        } else {
            ReplyError(stream_id, "NetStream.Seek.Notify", "Fail to seek");
        }
        return true;
    }
    if (name == "pause") {
        if (!st || v.size() < 5 || v[3].type() != rtmp::AMF_BOOLEAN) return true;
        const bool pause = v[3].boolean();
        const double ms = v[4].type() == rtmp::AMF_NUMBER ? v[4].number() : 0;
        const char* code = pause ? "NetStream.Pause.Notify" : "NetStream.Unpause.Notify";
        if (st->_paused == pause) {  // pausing a paused stream (or the reverse)
            ReplyError(stream_id, code, pause ? "Stream is already paused" : "Stream is not paused");
            return true;
        }
        if (st->OnPause(pause, ms) != 0) {
            ReplyError(stream_id, code, pause ? "Fail to pause" : "Fail to unpause");
            return true;
        }
        st->_paused = pause;
        ReplyStatus(stream_id, "status", code, pause ? "Paused stream." : "Unpaused stream.");
        std::string p;
        p.push_back(0);
        p.push_back(pause ? 1 : 0);  // StreamEOF / StreamBegin
        be32(&p, stream_id);
        SendControl(RTMP_USER_CONTROL, p);
        return true;
    }
    return true;  // other commands (releaseStream, FCPublish, getStreamLength...) are accepted silently
}

void Connection::ReplyError(uint32_t stream_id, const char* code, const std::string& desc) {
    AMFValue info = AMFValue::Object();
    info.Set("level", AMFValue::String("error"));
    info.Set("code", AMFValue::String(code));
    info.Set("description", AMFValue::String(desc));
    SendCommand(stream_id, {AMFValue::String("_error"), AMFValue::Number(0), AMFValue::Null(), info});
}

// Socket-attached holder.
class RtmpContext : public ParsingContext {
public:
    static const int kTag = 0x52544d50;  // "RTMP"
    int protocol_tag() const override { return kTag; }
    std::shared_ptr<Connection> conn;
    ~RtmpContext() override {
        if (conn) conn->StopAll();
    }
};

}  // namespace rtmp_detail

using rtmp_detail::Connection;
using rtmp_detail::RtmpContext;

// ------------------------------------------------------------ protocol

namespace policy {

ParseResult ParseRtmpMessage(Buf* source, Socket* socket, bool read_eof, const void* arg) {
    ParsingContext* pc = socket->parsing_context();
    RtmpContext* ctx = nullptr;
    if (pc) {
        if (pc->protocol_tag() != RtmpContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ctx = static_cast<RtmpContext*>(pc);
    } else {
        const Server* server = static_cast<const Server*>(arg);
        if (!server || !server->options().rtmp_service) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        char c0;
        if (source->copy_to(&c0, 1) < 1) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
        if (c0 != 3) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        if (source->size() < 1 + rtmp_detail::kHandshakeSize) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
        ctx = new RtmpContext;
        ctx->conn = std::make_shared<Connection>(true, socket->id());
        if (!socket->InstallParsingContext(ctx)) {
            delete ctx;
            return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        }
    }
    if (!ctx->conn->Consume(source, socket, static_cast<const Server*>(arg))) {
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    if (read_eof) ctx->conn->StopAll();
    return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);  // everything was dispatched in order
}

void ProcessRtmpMessage(InputMessageBase* msg) { msg->Destroy(); }  // never produced

void RegisterRtmpProtocol() {
    Protocol p;
    p.parse = ParseRtmpMessage;
    p.process_request = ProcessRtmpMessage;
    p.process_response = ProcessRtmpMessage;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE;
    p.name = "rtmp";
    RegisterProtocol(PROTOCOL_RTMP, p);
}

}  // namespace policy

// ------------------------------------------------------------ streams

RtmpStreamBase::~RtmpStreamBase() {}

EndPoint RtmpStreamBase::remote_side() const { return _conn ? _conn->remote_side() : EndPoint(); }

void RtmpStreamBase::CallOnStop() {
    bool expected = false;
    if (_stopped.compare_exchange_strong(expected, true)) OnStop();
}

int RtmpStreamBase::SendMessage(uint8_t type, uint32_t ts, const Buf& body) {
    if (!_conn || is_stopped()) {
        errno = EINVAL;
        return -1;
    }
    const uint32_t csid = type == RTMP_AUDIO ? rtmp_detail::kAudioCsid
                          : type == RTMP_VIDEO ? rtmp_detail::kVideoCsid
                                               : rtmp_detail::kDataCsid;
    return _conn->SendMessage(csid, type, ts, _stream_id, body);
}

int RtmpStreamBase::SendMetaData(const RtmpMetaData& md, const std::string& name) {
    std::string s;
    rtmp::WriteAMF(&s, AMFValue::String(name));
    rtmp::WriteAMF(&s, md.data);
    return SendMessage(RTMP_DATA_AMF0, md.timestamp, Buf(s));
}

int RtmpStreamBase::SendAudioMessage(const RtmpAudioMessage& msg) {
    Buf b;
    b.push_back((char)((msg.codec << 4) | ((msg.rate & 3) << 2) | ((msg.bits & 1) << 1) | (msg.type & 1)));
    b.append(msg.data);
    return SendMessage(RTMP_AUDIO, msg.timestamp, b);
}

int RtmpStreamBase::SendVideoMessage(const RtmpVideoMessage& msg) {
    Buf b;
    b.push_back((char)((msg.frame_type << 4) | (msg.codec & 0xf)));
    b.append(msg.data);
    return SendMessage(RTMP_VIDEO, msg.timestamp, b);
}

int RtmpStreamBase::SendCuePoint(const RtmpCuePoint& cp) {
    std::string s;
    rtmp::WriteAMF(&s, AMFValue::String("onCuePoint"));
    rtmp::WriteAMF(&s, cp.data);
    return SendMessage(RTMP_DATA_AMF0, cp.timestamp, Buf(s));
}

int RtmpStreamBase::SendAACMessage(const RtmpAACMessage& msg) {
    RtmpAudioMessage a;
    msg.ToAudioMessage(&a);
    return SendAudioMessage(a);
}

int RtmpStreamBase::SendAVCMessage(const RtmpAVCMessage& msg) {
    RtmpVideoMessage v;
    msg.ToVideoMessage(&v);
    return SendVideoMessage(v);
}

int RtmpStreamBase::SendUserMessage(void*) {
    LOG(ERROR) << "SendUserMessage is not implemented by this stream class";
    errno = ENOTSUP;
    return -1;
}

int RtmpStreamBase::SendStopMessage(const std::string&) {
    errno = ENOTSUP;
    return -1;
}

// ------------------------------------------------------------ server stream

void RtmpServerStream::OnPlay2(const RtmpPlay2Options& opt) {
    LOG(WARNING) << remote_side() << '[' << stream_id() << "] ignored play2{streamName=" << opt.stream_name
                 << " oldStreamName=" << opt.old_stream_name << " transition=" << opt.transition << '}';
}

int RtmpServerStream::OnSeek(double offset_ms) {
    LOG(WARNING) << remote_side() << '[' << stream_id() << "] ignored seek(" << offset_ms << ")";
    return -1;
}

int RtmpServerStream::OnPause(bool pause, double offset_ms) {
    LOG(WARNING) << remote_side() << '[' << stream_id() << "] ignored " << (pause ? "pause" : "unpause")
                 << "(offset_ms=" << offset_ms << ")";
    return -1;
}

int RtmpServerStream::SendStopMessage(const std::string& error_description) {
    std::shared_ptr<Connection> conn = _conn;
    if (!conn || conn->closed()) {
        errno = EINVAL;
        return -1;
    }
    // players (flash, ffplay, OBS) close the stream on StreamNotFound
    conn->ReplyStatus(_stream_id, "error", "NetStream.Play.StreamNotFound", error_description);
    return 0;
}

int RtmpServerStream::SendStreamDry() {
    std::shared_ptr<Connection> conn = _conn;
    if (!conn || conn->closed()) {
        errno = EINVAL;
        return -1;
    }
    std::string p;
    p.push_back(0);
    p.push_back(2);  // StreamDry
    rtmp_detail::be32(&p, _stream_id);
    return conn->SendControl(RTMP_USER_CONTROL, p);
}

// ------------------------------------------------------------ client

namespace {
// Blocks the caller (fiber or pthread) until signaled or timed out.
struct Waiter {
    fiber::CountdownEvent ev{1};
    bool ok = false;
    std::vector<AMFValue> args;
    bool Wait(int timeout_ms) {
        timespec ts = realtime_after_us((int64_t)timeout_ms * 1000);
        return ev.timed_wait(&ts) == 0;
    }
};
}  // namespace

RtmpClient::RtmpClient() {}
RtmpClient::~RtmpClient() {
    if (_conn) {
        SocketUniquePtr s;
        if (Socket::Address(_conn->socket_id(), &s) == 0) s->SetFailed(ECLOSE, "RtmpClient destroyed");
    }
}

int RtmpClient::Init(const char* server_addr_and_port, const RtmpClientOptions& options) {
    GlobalInitializeOrDie();
    _options = options;
    EndPoint ep;
    if (str2endpoint(server_addr_and_port, &ep) != 0 && hostname2endpoint(server_addr_and_port, &ep) != 0) {
        LOG(ERROR) << "Invalid rtmp server " << server_addr_and_port;
        return -1;
    }
    SocketOptions so;
    so.remote_side = ep;
    so.connect_lazily = true;
    SocketId sid;
    if (get_client_side_messenger()->Create(so, &sid) != 0) return -1;
    SocketUniquePtr sock;
    if (Socket::Address(sid, &sock) != 0) return -1;
    std::shared_ptr<Connection> conn = std::make_shared<Connection>(false, sid);
    RtmpContext* ctx = new RtmpContext;
    ctx->conn = conn;
    sock->reset_parsing_context(ctx);
    std::shared_ptr<Waiter> hs = std::make_shared<Waiter>();
    conn->on_handshake_done = [hs] { hs->ev.signal(); };
    // C0 + C1
    std::string c(1, (char)3);
    if (_options.complex_handshake) {
        std::string c1;
        rtmp::MakeComplexC1(rtmp::kSchema1, &c1);
        rtmp::ValidateComplexC1(c1, &conn->c1_digest);
        c += c1;
    } else {
        rtmp_detail::be32(&c, (uint32_t)(monotonic_us() / 1000));
        rtmp_detail::be32(&c, 0);
        for (size_t i = 8; i < rtmp_detail::kHandshakeSize; ++i) c.push_back((char)fast_rand());
    }
    Buf out(c);
    if (conn->Write(&out) != 0 || !hs->Wait(_options.timeout_ms)) {
        sock->SetFailed(ETIMEDOUT, "rtmp handshake failed");
        return -1;
    }
    std::string p;
    rtmp_detail::be32(&p, _options.chunk_size);
    conn->SendControl(RTMP_SET_CHUNK_SIZE, p);
    conn->set_out_chunk_size(_options.chunk_size);  // applies from the next message on
    AMFValue cmd = AMFValue::Object();
    cmd.Set("app", AMFValue::String(_options.app));
    cmd.Set("flashVer", AMFValue::String(_options.flashVer));
    cmd.Set("tcUrl", AMFValue::String(_options.tcUrl.empty() ? "rtmp://" + std::string(server_addr_and_port) + "/" +
                                                                    _options.app
                                                              : _options.tcUrl));
    cmd.Set("fpad", AMFValue::Bool(false));
    cmd.Set("capabilities", AMFValue::Number(15));
    cmd.Set("audioCodecs", AMFValue::Number(3191));
    cmd.Set("videoCodecs", AMFValue::Number(252));
    cmd.Set("videoFunction", AMFValue::Number(1));
    std::shared_ptr<Waiter> w = std::make_shared<Waiter>();
    conn->Call("connect", 0, {cmd}, [w](const std::vector<AMFValue>& args, bool ok) {
        w->ok = ok;
        w->args = args;
        w->ev.signal();
    });
    if (!w->Wait(_options.timeout_ms) || !w->ok) {
        sock->SetFailed(ECONNREFUSED, "rtmp connect rejected");
        return -1;
    }
    _conn = conn;
    _url_prefix = "rtmp://" + std::string(server_addr_and_port) + "/" + _options.app;
    return 0;
}

uint64_t RtmpClient::socket_id() const { return _conn ? (uint64_t)_conn->socket_id() : 0; }

RtmpClientStream::~RtmpClientStream() { Destroy(); }

int RtmpClientStream::Init(RtmpClient* client, const RtmpClientStreamOptions& options) {
    std::shared_ptr<Connection> conn = client ? client->connection() : nullptr;
    if (!conn || conn->closed()) return -1;
    const int timeout = client->options().timeout_ms;
    std::shared_ptr<Waiter> w = std::make_shared<Waiter>();
    conn->Call("createStream", 0, {AMFValue::Null()}, [w](const std::vector<AMFValue>& args, bool ok) {
        w->ok = ok;
        w->args = args;
        w->ev.signal();
    });
    if (!w->Wait(timeout) || !w->ok || w->args.size() < 4) return -1;
    _stream_id = (uint32_t)w->args[3].number();
    _conn = conn;
    conn->AddStream(_stream_id, this, false);
    // onStatus of this stream completes play/publish; later ones go to
    // OnStatus() while the stream is alive (the sink is cut in Destroy())
    std::shared_ptr<Waiter> st = std::make_shared<Waiter>();
    _sink = std::make_shared<StatusSink>();
    _sink->stream = this;
    std::shared_ptr<StatusSink> sink = _sink;
    conn->SetStatusListener(_stream_id, [st, sink](const std::vector<AMFValue>& args) {
        const AMFValue* info = args.size() > 3 && args[3].type() == rtmp::AMF_OBJECT ? &args[3] : nullptr;
        const AMFValue* code = info ? info->Find("code") : nullptr;
        if (st->ev.count() > 0) {
            st->ok = code && (code->str() == "NetStream.Play.Start" || code->str() == "NetStream.Publish.Start");
            st->ev.signal();
            return;
        }
        const AMFValue* level = info ? info->Find("level") : nullptr;
        const AMFValue* desc = info ? info->Find("description") : nullptr;
        std::lock_guard<std::mutex> g(sink->mu);
        if (!sink->stream) return;
        sink->stream->SetLastStatus(code ? code->str() : "");
        sink->stream->OnStatus(level ? level->str() : "", code ? code->str() : "", desc ? desc->str() : "");
    });
    _name = options.publish_name.empty() ? options.play_name : options.publish_name;
    _url_prefix = client->url_prefix();
    std::vector<AMFValue> cmd;
    if (!options.publish_name.empty()) {
        cmd = {AMFValue::String("publish"), AMFValue::Number(0), AMFValue::Null(),
               AMFValue::String(options.publish_name), AMFValue::String(options.publish_type)};
    } else {
        cmd = {AMFValue::String("play"), AMFValue::Number(0), AMFValue::Null(), AMFValue::String(options.play_name),
               AMFValue::Number(-2)};
    }
    conn->SendCommand(_stream_id, cmd);
    if (options.publish_name.empty() && options.buffer_length_ms >= 0) {
        std::string p;
        p.push_back(0);
        p.push_back(3);  // SetBufferLength{stream id, ms}
        rtmp_detail::be32(&p, _stream_id);
        rtmp_detail::be32(&p, (uint32_t)options.buffer_length_ms);
        conn->SendControl(RTMP_USER_CONTROL, p);
    }
    if (!st->Wait(timeout) || !st->ok) {
        conn->RemoveStream(_stream_id);
        _conn.reset();
        return -1;
    }
    return 0;
}

int RtmpClientStream::Play2(const RtmpPlay2Options& opt) {
    std::shared_ptr<Connection> conn = _conn;
    if (!conn || conn->closed()) {
        errno = EINVAL;
        return -1;
    }
    AMFValue o = AMFValue::Object();
    if (!std::isnan(opt.len)) o.Set("len", AMFValue::Number(opt.len));
    if (!std::isnan(opt.offset)) o.Set("offset", AMFValue::Number(opt.offset));
    if (!opt.old_stream_name.empty()) o.Set("oldStreamName", AMFValue::String(opt.old_stream_name));
    if (!std::isnan(opt.start)) o.Set("start", AMFValue::Number(opt.start));
    if (!opt.stream_name.empty()) o.Set("streamName", AMFValue::String(opt.stream_name));
    if (!opt.transition.empty()) o.Set("transition", AMFValue::String(opt.transition));
    return conn->SendCommand(_stream_id, {AMFValue::String("play2"), AMFValue::Number(0), AMFValue::Null(), o});
}

int RtmpClientStream::Seek(double offset_ms) {
    std::shared_ptr<Connection> conn = _conn;
    if (!conn || conn->closed()) {
        errno = EINVAL;
        return -1;
    }
    return conn->SendCommand(_stream_id,
                             {AMFValue::String("seek"), AMFValue::Number(0), AMFValue::Null(), AMFValue::Number(offset_ms)});
}

int RtmpClientStream::Pause(bool pause, double offset_ms) {
    std::shared_ptr<Connection> conn = _conn;
    if (!conn || conn->closed()) {
        errno = EINVAL;
        return -1;
    }
    return conn->SendCommand(_stream_id, {AMFValue::String("pause"), AMFValue::Number(0), AMFValue::Null(),
                                          AMFValue::Bool(pause), AMFValue::Number(offset_ms)});
}

void RtmpClientStream::SetLastStatus(const std::string& code) {
    std::lock_guard<std::mutex> g(_status_mu);
    _last_status = code;
}

std::string RtmpClientStream::last_status() const {
    std::lock_guard<std::mutex> g(_status_mu);
    return _last_status;
}

std::string RtmpClientStream::rtmp_url() const { return _url_prefix + "/" + _name; }

void RtmpClientStream::Destroy() {
    if (_sink) {  // no OnStatus() after this returns
        std::lock_guard<std::mutex> g(_sink->mu);
        _sink->stream = nullptr;
    }
    std::shared_ptr<Connection> conn = _conn;
    if (!conn) return;
    if (!conn->closed()) {
        conn->SendCommand(0, {AMFValue::String("deleteStream"), AMFValue::Number(0), AMFValue::Null(),
                              AMFValue::Number(_stream_id)});
        conn->SetStatusListener(_stream_id, nullptr);
        conn->RemoveStream(_stream_id);
    }
    CallOnStop();
    _conn.reset();
}

// ------------------------------------------------------------ FLV

FlvWriter::FlvWriter(Buf* out) : _out(out) {}

int FlvWriter::WriteTag(uint8_t type, uint32_t ts, const Buf& body) {
    if (!_wrote_header) {
        static const char hdr[13] = {'F', 'L', 'V', 1, 5, 0, 0, 0, 9, 0, 0, 0, 0};  // audio+video, PreviousTagSize0
        _out->append(hdr, sizeof(hdr));
        _wrote_header = true;
    }
    std::string t;
    t.push_back((char)type);
    rtmp_detail::be24(&t, (uint32_t)body.size());
    rtmp_detail::be24(&t, ts & 0xffffff);
    t.push_back((char)(ts >> 24));
    rtmp_detail::be24(&t, 0);  // stream id
    _out->append(t);
    _out->append(body);
    std::string prev;
    rtmp_detail::be32(&prev, (uint32_t)(11 + body.size()));
    _out->append(prev);
    return 0;
}

int FlvWriter::Write(const RtmpVideoMessage& msg) {
    Buf b;
    b.push_back((char)((msg.frame_type << 4) | (msg.codec & 0xf)));
    b.append(msg.data);
    return WriteTag(RTMP_VIDEO, msg.timestamp, b);
}

int FlvWriter::Write(const RtmpAudioMessage& msg) {
    Buf b;
    b.push_back((char)((msg.codec << 4) | ((msg.rate & 3) << 2) | ((msg.bits & 1) << 1) | (msg.type & 1)));
    b.append(msg.data);
    return WriteTag(RTMP_AUDIO, msg.timestamp, b);
}

int FlvWriter::Write(const RtmpMetaData& md, const std::string& name) {
    std::string s;
    rtmp::WriteAMF(&s, AMFValue::String(name));
    rtmp::WriteAMF(&s, md.data);
    return WriteTag(RTMP_DATA_AMF0, md.timestamp, Buf(s));
}

FlvReader::FlvReader(Buf* in) : _in(in) {}

int FlvReader::PeekMessageType(uint8_t* type) {
    if (!_read_header) {
        char h[13];
        if (_in->copy_to(h, 13) < 13) return EAGAIN;
        if (memcmp(h, "FLV", 3) != 0) return EINVAL;
        _in->pop_front(13);
        _read_header = true;
    }
    char t;
    if (_in->copy_to(&t, 1) < 1) return EAGAIN;
    *type = (uint8_t)t;
    return 0;
}

int FlvReader::ReadTag(uint8_t want, uint32_t* ts, Buf* body) {
    uint8_t type;
    int rc = PeekMessageType(&type);
    if (rc) return rc;
    if (type != want) return EINVAL;
    uint8_t h[11];
    if (_in->copy_to(h, 11) < 11) return EAGAIN;
    const uint32_t size = rtmp_detail::rd24(h + 1);
    if (_in->size() < 11 + size + 4) return EAGAIN;
    *ts = rtmp_detail::rd24(h + 4) | ((uint32_t)h[7] << 24);
    _in->pop_front(11);
    _in->cutn(body, size);
    _in->pop_front(4);
    return 0;
}

int FlvReader::Read(RtmpVideoMessage* msg) {
    Buf b;
    int rc = ReadTag(RTMP_VIDEO, &msg->timestamp, &b);
    if (rc) return rc;
    char h = 0;
    b.cut1(&h);
    msg->frame_type = (uint8_t)h >> 4;
    msg->codec = (uint8_t)h & 0xf;
    msg->data.swap(b);
    return 0;
}

int FlvReader::Read(RtmpAudioMessage* msg) {
    Buf b;
    int rc = ReadTag(RTMP_AUDIO, &msg->timestamp, &b);
    if (rc) return rc;
    char h = 0;
    b.cut1(&h);
    msg->codec = (uint8_t)h >> 4;
    msg->rate = ((uint8_t)h >> 2) & 3;
    msg->bits = ((uint8_t)h >> 1) & 1;
    msg->type = (uint8_t)h & 1;
    msg->data.swap(b);
    return 0;
}

int FlvReader::Read(RtmpMetaData* md, std::string* name) {
    Buf b;
    int rc = ReadTag(RTMP_DATA_AMF0, &md->timestamp, &b);
    if (rc) return rc;
    const std::string s = b.to_string();
    std::vector<AMFValue> v;
    if (!rtmp::ReadAMFList(s.data(), s.size(), &v) || v.size() < 2) return EINVAL;
    *name = v[0].str();
    md->data = v[1];
    return 0;
}

}  // namespace mrpc

namespace mrpc {
bool RtmpClient::complex_handshake_done() const { return _conn && _conn->complex_handshake; }
int64_t RtmpClient::acks_sent() const { return _conn ? _conn->acks_sent : 0; }

int64_t RtmpClient::Ping(int timeout_ms) {
    if (!_conn) return -1;
    struct Pong {
        fiber::CountdownEvent ev{1};
    };
    std::shared_ptr<Pong> w = std::make_shared<Pong>();
    _conn->SetPongCallback([w] { w->ev.signal(); });
    const int64_t t0 = monotonic_us();
    std::string p;
    p.push_back(0);
    p.push_back(6);  // PingRequest
    rtmp_detail::be32(&p, (uint32_t)(t0 / 1000));
    if (_conn->SendControl(RTMP_USER_CONTROL, p) != 0) return -1;
    timespec ts = realtime_after_us((int64_t)timeout_ms * 1000);
    if (w->ev.timed_wait(&ts) != 0) {
        _conn->SetPongCallback(nullptr);
        return -1;
    }
    return monotonic_us() - t0;
}
namespace rtmp {
int64_t ComplexHandshakesServed() { return rtmp_detail::g_complex_handshakes.load(std::memory_order_relaxed); }
int64_t UnsignedC2Count() { return rtmp_detail::g_unsigned_c2.load(std::memory_order_relaxed); }
}  // namespace rtmp
}  // namespace mrpc
