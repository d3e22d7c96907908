#include "rpc/stream.h"

#include <cerrno>
#include <memory>
#include <mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "base/pool.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/butex.h"
#include "fiber/execution_queue.h"
#include "policy/device_payload.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/stream_internal.h"

DECLARE_uint64(max_body_size);

namespace mrpc {

namespace {

struct StreamObj;
// One received DATA frame. HBM chunks are NOT pulled by the reading fiber:
// the frame's descriptors ride along and the consumer pulls every chunk of
// its batch with one launch, in order, so the socket keeps being read while
// the GPU moves the bytes.
struct StreamChunk {
    Buf payload;                           // inline part (everything for host chunks)
    std::shared_ptr<StreamFrameMeta> dmeta;  // device descriptors, or null
    SocketUniquePtr sock;                  // the connection the chunks were lent on
};
typedef fiber::ExecutionQueue<StreamChunk> RecvQueue;

struct StreamObj {
    std::mutex mu;
    uint32_t version = 1;
    bool in_use = false;
    StreamOptions opt;
    StreamId id = 0;
    int64_t remote_id = 0;
    SocketId host = INVALID_SOCKET_ID;
    bool connected = false;
    bool closed = false;        // local close or failure
    bool on_closed_called = false;
    bool remote_need_feedback = false;
    // writer
    int64_t produced = 0;
    int64_t remote_consumed = 0;
    int64_t cur_buf_size = 0;
    std::atomic<int>* writable = nullptr;
    std::vector<Buf> pending;
    // reader
    std::shared_ptr<RecvQueue> queue;
    int64_t local_consumed = 0;
    int64_t last_feedback = 0;
    int64_t last_recv_us = 0;
    fiber::TimerId idle_timer = 0;
};

inline uint32_t sid_slot(StreamId id) { return (uint32_t)(id >> 32); }
inline uint32_t sid_ver(StreamId id) { return (uint32_t)id; }

// Returns the object locked if the id is valid.
StreamObj* lock_stream(StreamId id, std::unique_lock<std::mutex>* lk) {
    if (id == INVALID_STREAM_ID) return nullptr;
    StreamObj* s = address_resource<StreamObj>(sid_slot(id));
    if (!s) return nullptr;
    std::unique_lock<std::mutex> g(s->mu);
    if (!s->in_use || s->version != sid_ver(id)) return nullptr;
    *lk = std::move(g);
    return s;
}

int send_frame(SocketId host, int64_t dest_stream, int64_t src_stream, FrameType type, const Buf* payload,
               int64_t consumed = -1) {
    SocketUniquePtr sock;
    if (Socket::Address(host, &sock) != 0) return EFAILEDSOCKET;
    StreamFrameMeta fm;
    fm.set_stream_id(dest_stream);
    fm.set_source_stream_id(src_stream);
    fm.set_frame_type(type);
    if (consumed >= 0) fm.mutable_feedback()->set_consumed_size(consumed);
    // HBM chunks: lent over the connection's xGMI transport and described
    // in the frame meta (staged through host memory when the connection has
    // no device transport); only host bytes go inline
    Buf host_part;
    if (payload && !payload->all_host_accessible()) {
        std::string err;
        if (policy::LendDeviceBlocks(sock.get(), *payload, DeviceLendOptions(), &host_part, fm.mutable_device_payload(), &err) != 0) {
            LOG_EVERY_SECOND(WARNING) << "stream " << src_stream << ": " << err;
            return EINVAL;
        }
        payload = &host_part;
    }
    const uint32_t meta_size = (uint32_t)fm.ByteSizeLong();
    const uint32_t payload_size = payload ? (uint32_t)payload->size() : 0;
    Buf frame;
    char* p = frame.append_contiguous(12 + meta_size);
    memcpy(p, "STRM", 4);
    pack_be32(p + 4, meta_size + payload_size);
    pack_be32(p + 8, meta_size);
    fm.SerializeWithCachedSizesToArray((uint8_t*)p + 12);
    if (payload) frame.append(*payload);
    WriteOptions wopt;
    wopt.ignore_eovercrowded = (type != FRAME_TYPE_DATA);
    if (sock->Write(&frame, &wopt) != 0) {
        const int e = errno;
        // the frame never left: take the lends back
        if (fm.device_payload_size()) policy::CancelDeviceBlocks(fm.device_payload());
        return e;
    }
    return 0;
}

void release_stream(StreamObj* s) {
    // caller holds s->mu
    s->in_use = false;
    ++s->version;
    if (s->version == 0) s->version = 1;
    s->queue.reset();
    s->pending.clear();
    if (s->idle_timer) {
        fiber::timer_del(s->idle_timer);
        s->idle_timer = 0;
    }
    fiber::butex_wake_all(s->writable);
    return_resource<StreamObj>(sid_slot(s->id));
}

int consume(void* meta, RecvQueue::Iterator& it);

StreamId new_stream(const StreamOptions* opt) {
    uint32_t slot;
    StreamObj* s = get_resource<StreamObj>(&slot);
    if (!s) return INVALID_STREAM_ID;
    std::lock_guard<std::mutex> g(s->mu);
    if (!s->writable) s->writable = fiber::butex_create();
    s->in_use = true;
    s->opt = opt ? *opt : StreamOptions();
    s->id = ((uint64_t)slot << 32) | s->version;
    s->remote_id = 0;
    s->host = INVALID_SOCKET_ID;
    s->connected = s->closed = s->on_closed_called = false;
    s->remote_need_feedback = false;
    s->produced = s->remote_consumed = 0;
    s->cur_buf_size = s->opt.max_buf_size > 0 ? std::max(s->opt.min_buf_size, (int64_t)1) : 0;
    s->pending.clear();
    s->local_consumed = s->last_feedback = 0;
    s->last_recv_us = monotonic_us();
    RecvQueue::Options qopt;
    qopt.max_batch = s->opt.messages_in_batch ? s->opt.messages_in_batch : 128;
    s->queue = RecvQueue::Create(consume, (void*)(uintptr_t)s->id, qopt);
    return s->id;
}

void schedule_idle_check(StreamId id);

void* idle_check_fiber(void* arg) {
    const StreamId id = (StreamId)(uintptr_t)arg;
    StreamInputHandler* h = nullptr;
    bool fire = false;
    {
        std::unique_lock<std::mutex> lk;
        StreamObj* s = lock_stream(id, &lk);
        if (!s || s->closed) return nullptr;
        s->idle_timer = 0;
        if (monotonic_us() - s->last_recv_us >= s->opt.idle_timeout_ms * 1000) {
            fire = true;
            h = s->opt.handler;
            s->last_recv_us = monotonic_us();
        }
    }
    if (fire && h) h->on_idle_timeout(id);
    schedule_idle_check(id);
    return nullptr;
}

void idle_timer_cb(void* arg) {
    fiber::fiber_t th;
    fiber::start_background(&th, nullptr, idle_check_fiber, arg);
}

void schedule_idle_check(StreamId id) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(id, &lk);
    if (!s || s->closed || s->opt.idle_timeout_ms <= 0) return;
    fiber::timer_add_us(&s->idle_timer, s->opt.idle_timeout_ms * 1000, idle_timer_cb, (void*)(uintptr_t)id);
}

void mark_connected(StreamObj* s, SocketId host, int64_t remote_id, bool remote_need_feedback) {
    // caller holds s->mu
    s->host = host;
    s->remote_id = remote_id;
    s->remote_need_feedback = remote_need_feedback;
    s->connected = true;
    std::vector<Buf> pending;
    pending.swap(s->pending);
    for (Buf& b : pending) send_frame(host, remote_id, (int64_t)s->id, FRAME_TYPE_DATA, &b);
    const StreamId id = s->id;
    SocketUniquePtr sock;
    if (Socket::Address(host, &sock) == 0) {
        sock->AddFailureCallback([id] {
            std::unique_lock<std::mutex> lk;
            StreamObj* x = lock_stream(id, &lk);
            if (!x || x->closed) return;
            x->closed = true;
            auto q = x->queue;
            fiber::butex_wake_all(x->writable);
            lk.unlock();
            if (q) q->stop();
        });
    }
}

int consume(void* meta, RecvQueue::Iterator& it) {
    const StreamId id = (StreamId)(uintptr_t)meta;
    StreamInputHandler* handler = nullptr;
    {
        std::unique_lock<std::mutex> lk;
        StreamObj* s = lock_stream(id, &lk);
        if (!s) return 0;
        handler = s->opt.handler;
    }
    if (it.is_queue_stopped()) {
        for (; it; ++it) {  // chunks nobody will read: give the lends back
            if (it->dmeta) policy::ReleaseDeviceBlocks(it->sock.get(), it->dmeta->device_payload());
        }
        bool call = false;
        {
            std::unique_lock<std::mutex> lk;
            StreamObj* s = lock_stream(id, &lk);
            if (s && !s->on_closed_called) {
                s->on_closed_called = true;
                call = true;
            }
        }
        if (call && handler) handler->on_closed(id);
        std::unique_lock<std::mutex> lk;
        StreamObj* s = lock_stream(id, &lk);
        if (s) release_stream(s);
        return 0;
    }
    std::vector<Buf*> msgs;
    std::vector<std::pair<const policy::DevicePayloads*, Buf*>> pulls;
    Socket* pull_sock = nullptr;
    int64_t bytes = 0;
    for (; it; ++it) {
        StreamChunk& c = *it;
        if (c.dmeta) {
            if (pull_sock && pull_sock != c.sock.get()) {
                // (never happens: one stream, one host connection)
                std::string err;
                if (policy::PullDeviceBlocksBatch(pull_sock, pulls, &err) != 0) {
                    LOG_EVERY_SECOND(ERROR) << "stream " << id << " lost device chunks: " << err;
                }
                pulls.clear();
            }
            pull_sock = c.sock.get();
            pulls.emplace_back(&c.dmeta->device_payload(), &c.payload);
        }
        msgs.push_back(&c.payload);
    }
    if (!pulls.empty()) {
        std::string err;
        if (policy::PullDeviceBlocksBatch(pull_sock, pulls, &err) != 0) {
            LOG_EVERY_SECOND(ERROR) << "stream " << id << " lost device chunks: " << err;
            for (auto& p : pulls) p.second->clear();
        }
    }
    for (Buf* m : msgs) bytes += (int64_t)m->size();
    if (handler && !msgs.empty()) handler->on_received_messages(id, msgs.data(), msgs.size());
    SocketId host = INVALID_SOCKET_ID;
    int64_t remote = 0, consumed = -1;
    {
        std::unique_lock<std::mutex> lk;
        StreamObj* s = lock_stream(id, &lk);
        if (!s) return 0;
        s->local_consumed += bytes;
        // The writer's window is unknown here, so report after every batch
        // (batches already coalesce up to messages_in_batch messages).
        if (s->remote_need_feedback && s->connected && s->local_consumed > s->last_feedback) {
            s->last_feedback = s->local_consumed;
            host = s->host;
            remote = s->remote_id;
            consumed = s->local_consumed;
        }
    }
    if (consumed >= 0) send_frame(host, remote, (int64_t)id, FRAME_TYPE_FEEDBACK, nullptr, consumed);
    return 0;
}

struct StreamFrameMessage : public InputMessageBase {
    StreamFrameMeta meta;
    Buf payload;
};

void ProcessStreamFrame(InputMessageBase* base);

ParseResult ParseStreamingMessage(Buf* source, Socket* socket, bool, const void*) {
    char header[12];
    const size_t n = source->copy_to(header, sizeof(header));
    if (n >= 4) {
        if (memcmp(header, "STRM", 4) != 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    } else {
        if (memcmp(header, "STRM", n) != 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    }
    if (n < sizeof(header)) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    const uint32_t body_size = unpack_be32(header + 4);
    const uint32_t meta_size = unpack_be32(header + 8);
    if (body_size > FLAGS_max_body_size) return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    if (source->size() < sizeof(header) + body_size) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    if (meta_size > body_size) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    source->pop_front(sizeof(header));
    Buf meta_buf;
    source->cutn(&meta_buf, meta_size);
    StreamFrameMessage* msg = new StreamFrameMessage;
    if (!msg->meta.ParseFromBuf(meta_buf)) {
        delete msg;
        source->pop_front(body_size - meta_size);
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    source->cutn(&msg->payload, body_size - meta_size);
    // Frames of a stream must be handled in arrival order, so they are
    // processed right here in the reading fiber instead of being dispatched
    // to new fibers like RPC messages (nullptr => consumed by the parser).
    socket->AddRef();
    msg->_socket.reset(socket);
    ProcessStreamFrame(msg);
    return MakeMessage(nullptr);
}

void ProcessStreamFrame(InputMessageBase* base) {
    std::unique_ptr<StreamFrameMessage> msg(static_cast<StreamFrameMessage*>(base));
    const StreamFrameMeta& fm = msg->meta;
    const StreamId id = (StreamId)fm.stream_id();
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(id, &lk);
    if (!s) {
        policy::ReleaseDeviceBlocks(msg->socket(), fm.device_payload());
        if (fm.frame_type() == FRAME_TYPE_DATA && fm.source_stream_id()) {
            send_frame(msg->socket()->id(), fm.source_stream_id(), (int64_t)id, FRAME_TYPE_RST, nullptr);
        }
        return;
    }
    switch (fm.frame_type()) {
    case FRAME_TYPE_DATA: {
        s->last_recv_us = monotonic_us();
        if (!s->connected && fm.source_stream_id()) {
            // data may race ahead of the RPC response on the server side
            mark_connected(s, msg->socket()->id(), fm.source_stream_id(), s->remote_need_feedback);
        }
        auto q = s->queue;
        lk.unlock();
        StreamChunk c;
        c.payload = std::move(msg->payload);
        if (fm.device_payload_size() > 0) {
            c.dmeta = std::make_shared<StreamFrameMeta>();
            c.dmeta->mutable_device_payload()->raw().swap(msg->meta.mutable_device_payload()->raw());
            msg->socket()->AddRef();
            c.sock.reset(msg->socket());
        }
        std::shared_ptr<StreamFrameMeta> dmeta = c.dmeta;  // survives a failed execute
        if (!q || q->execute(std::move(c)) != 0) {
            if (dmeta) policy::ReleaseDeviceBlocks(msg->socket(), dmeta->device_payload());
        }
        break;
    }
    case FRAME_TYPE_FEEDBACK: {
        const int64_t c = fm.feedback().consumed_size();
        if (c > s->remote_consumed) s->remote_consumed = c;
        // grow the window towards max_buf_size when the reader keeps up
        if (s->cur_buf_size < s->opt.max_buf_size) s->cur_buf_size = std::min(s->cur_buf_size * 2, s->opt.max_buf_size);
        s->writable->fetch_add(1, std::memory_order_release);
        lk.unlock();
        fiber::butex_wake_all(s->writable);
        break;
    }
    case FRAME_TYPE_CLOSE:
    case FRAME_TYPE_RST: {
        s->closed = true;
        auto q = s->queue;
        fiber::butex_wake_all(s->writable);
        lk.unlock();
        if (q) q->stop();
        break;
    }
    default: break;
    }
}

}  // namespace

void FillStreamSettings(StreamId sid, StreamSettings* settings) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(sid, &lk);
    if (!s) return;
    settings->set_stream_id((int64_t)sid);
    settings->set_need_feedback(s->opt.max_buf_size > 0);
    settings->set_writable(true);
}

void OnRequestStreamSettings(Controller* cntl, Socket* host, const StreamSettings& st) {
    // remember the client's stream; StreamAccept connects to it
    cntl->_request_stream = (StreamId)st.stream_id();
    cntl->_server_socket_id = host->id();
    cntl->_stream_creator = std::make_shared<bool>(st.need_feedback());
}

void OnServerStreamCreated(StreamId sid, SocketId host) {
    (void)sid;
    (void)host;  // connected already in StreamAccept
}

void OnResponseStreamSettings(Controller* cntl, Socket* host, const StreamSettings& st) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(cntl->_request_stream, &lk);
    if (!s) return;
    if (!s->connected) mark_connected(s, host->id(), st.stream_id(), st.need_feedback());
}

void OnRequestStreamCallEnded(StreamId sid) {
    {
        std::unique_lock<std::mutex> lk;
        StreamObj* s = lock_stream(sid, &lk);
        if (!s || s->connected || s->closed) return;
    }
    // the call ended (failed, or the server never accepted the stream): a
    // stream no peer will ever connect to is closed, so its writer and its
    // handler's on_closed learn now instead of never
    StreamClose(sid);
}

int StreamCreate(StreamId* request_stream, Controller& cntl, const StreamOptions* options) {
    if (cntl._request_stream != INVALID_STREAM_ID) {
        LOG(ERROR) << "Can't create more than one stream on a controller";
        return -1;
    }
    StreamId sid = new_stream(options);
    if (sid == INVALID_STREAM_ID) return -1;
    cntl._request_stream = sid;
    *request_stream = sid;
    schedule_idle_check(sid);
    return 0;
}

int StreamAccept(StreamId* response_stream, Controller& cntl, const StreamOptions* options) {
    if (cntl._request_stream == INVALID_STREAM_ID) {
        LOG(ERROR) << "The request has no stream to accept";
        return -1;
    }
    if (cntl._response_stream != INVALID_STREAM_ID) return -1;
    StreamId sid = new_stream(options);
    if (sid == INVALID_STREAM_ID) return -1;
    {
        std::unique_lock<std::mutex> lk;
        StreamObj* s = lock_stream(sid, &lk);
        const bool need_fb = cntl._stream_creator ? *std::static_pointer_cast<bool>(cntl._stream_creator) : true;
        mark_connected(s, cntl._server_socket_id, (int64_t)cntl._request_stream, need_fb);
    }
    cntl._response_stream = sid;
    *response_stream = sid;
    schedule_idle_check(sid);
    return 0;
}

int StreamWrite(StreamId id, const Buf& message, const StreamWriteOptions*) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(id, &lk);
    if (!s || s->closed) return EINVAL;
    if (s->cur_buf_size > 0 && s->produced - s->remote_consumed >= s->cur_buf_size && s->remote_need_feedback) return EAGAIN;
    s->produced += (int64_t)message.size();
    if (!s->connected) {
        s->pending.push_back(message);
        return 0;
    }
    const SocketId host = s->host;
    const int64_t remote = s->remote_id;
    lk.unlock();
    Buf payload = message;
    // device-resident chunks are lent over xGMI inside send_frame
    const int rc = send_frame(host, remote, (int64_t)id, FRAME_TYPE_DATA, &payload);
    return rc == 0 ? 0 : EINVAL;
}

int StreamWait(StreamId id, const timespec* due) {
    for (;;) {
        int expected;
        {
            std::unique_lock<std::mutex> lk;
            StreamObj* s = lock_stream(id, &lk);
            if (!s || s->closed) return EINVAL;
            if (s->cur_buf_size <= 0 || !s->remote_need_feedback || s->produced - s->remote_consumed < s->cur_buf_size) return 0;
            expected = s->writable->load(std::memory_order_acquire);
            std::atomic<int>* w = s->writable;
            lk.unlock();
            if (fiber::butex_wait(w, expected, due) < 0 && errno == ETIMEDOUT) return ETIMEDOUT;
        }
    }
}

void StreamWait(StreamId id, const timespec* due, void (*on_writable)(StreamId, void*, int), void* arg) {
    timespec d;
    const bool has_due = due != nullptr;
    if (due) d = *due;
    fiber::start([=] {
        int rc = StreamWait(id, has_due ? &d : nullptr);
        on_writable(id, arg, rc);
    });
}

int StreamClose(StreamId id) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(id, &lk);
    if (!s) return EINVAL;
    if (s->closed) return 0;
    s->closed = true;
    const bool connected = s->connected;
    const SocketId host = s->host;
    const int64_t remote = s->remote_id;
    auto q = s->queue;
    fiber::butex_wake_all(s->writable);
    lk.unlock();
    if (connected) send_frame(host, remote, (int64_t)id, FRAME_TYPE_CLOSE, nullptr);
    if (q) q->stop();
    return 0;
}

int64_t StreamUnconsumedBytes(StreamId id) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(id, &lk);
    return s ? s->produced - s->remote_consumed : -1;
}

bool StreamIsConnected(StreamId id) {
    std::unique_lock<std::mutex> lk;
    StreamObj* s = lock_stream(id, &lk);
    return s && s->connected;
}

void RegisterStreamingProtocol() {
    Protocol p;
    p.parse = ParseStreamingMessage;
    p.process_request = ProcessStreamFrame;
    p.process_response = ProcessStreamFrame;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE;
    p.name = "streaming_rpc";
    RegisterProtocol(PROTOCOL_STREAMING_RPC, p);
}

}  // namespace mrpc
