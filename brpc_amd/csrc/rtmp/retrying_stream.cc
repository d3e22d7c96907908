// RtmpRetryingClientStream (rtmp/rtmp.h): a sub RtmpClientStream per
// connection attempt; callbacks are forwarded to the owner, a stop that the
// owner did not ask for starts a retry fiber.
#include <atomic>
#include <cerrno>
#include <memory>
#include <mutex>
#include <vector>

#include "base/logging.h"
#include "base/time.h"
#include "fiber/fiber.h"
#include "rtmp/rtmp.h"

namespace mrpc {

namespace {
class SubStream;
}

struct RtmpRetryingClientStream::Impl : public std::enable_shared_from_this<RtmpRetryingClientStream::Impl> {
    RtmpRetryingClientStream* owner = nullptr;
    std::unique_ptr<RtmpSubStreamCreator> creator;
    RtmpRetryingClientStreamOptions options;
    std::mutex mu;
    std::shared_ptr<RtmpClient> client;
    std::unique_ptr<SubStream> current;
    std::vector<std::unique_ptr<SubStream>> retired;  // stopped sub streams (freed off their callbacks)
    std::vector<std::shared_ptr<RtmpClient>> retired_clients;
    std::atomic<bool> destroyed{false};
    bool retrying = false;
    bool started_once = false;
    std::atomic<int64_t> reconnects{0};

    int Start();
    void SubStopped(SubStream* s);
    void RetryLoop();
    void Collect();
};

namespace {

class SubStream : public RtmpClientStream {
public:
    explicit SubStream(std::weak_ptr<RtmpRetryingClientStream::Impl> i) : _impl(std::move(i)) {}
    // detach from the connection before this class's part is destroyed: a
    // status or stop callback racing with ~RtmpClientStream would otherwise
    // dispatch through a half-destroyed object
    ~SubStream() override { Destroy(); }
    std::atomic<bool> by_owner{false};

    void OnMetaData(RtmpMetaData* md, const std::string& name) override {
        if (auto i = live()) i->owner->OnMetaData(md, name);
    }
    void OnAudioMessage(RtmpAudioMessage* m) override {
        if (auto i = live()) i->owner->OnAudioMessage(m);
    }
    void OnVideoMessage(RtmpVideoMessage* m) override {
        if (auto i = live()) i->owner->OnVideoMessage(m);
    }
    void OnCuePoint(RtmpCuePoint* cp) override {
        if (auto i = live()) i->owner->OnCuePoint(cp);
    }
    void OnStop() override {
        if (by_owner.load(std::memory_order_acquire)) return;
        if (auto i = live()) i->SubStopped(this);
    }

private:
    std::shared_ptr<RtmpRetryingClientStream::Impl> live() {
        std::shared_ptr<RtmpRetryingClientStream::Impl> i = _impl.lock();
        return i && !i->destroyed.load(std::memory_order_acquire) ? i : nullptr;
    }
    std::weak_ptr<RtmpRetryingClientStream::Impl> _impl;
};

}  // namespace

int RtmpRetryingClientStream::Impl::Start() {
    std::shared_ptr<RtmpClient> c = creator->NewClient();
    if (!c || !c->initialized()) return -1;
    std::unique_ptr<SubStream> s(new SubStream(shared_from_this()));
    if (s->Init(c.get(), options) != 0) {
        s->by_owner.store(true);
        return -1;
    }
    {
        std::lock_guard<std::mutex> g(mu);
        if (!destroyed.load()) {
            owner->_stream_id = s->stream_id();
            if (current) retired.push_back(std::move(current));
            if (client) retired_clients.push_back(std::move(client));
            current = std::move(s);
            client = std::move(c);
            if (started_once) reconnects.fetch_add(1, std::memory_order_relaxed);
            started_once = true;
        }
    }
    if (s) {  // destroyed meanwhile
        s->by_owner.store(true);
        s->Destroy();
        return -1;
    }
    owner->OnSubStreamStarted();
    return 0;
}

void RtmpRetryingClientStream::Impl::SubStopped(SubStream* s) {
    std::lock_guard<std::mutex> g(mu);
    if (destroyed.load() || s != current.get()) return;
    // keep the object: we are inside its OnStop
    retired.push_back(std::move(current));
    if (client) retired_clients.push_back(std::move(client));
    if (retrying) return;
    retrying = true;
    std::shared_ptr<Impl> self = shared_from_this();
    fiber::start([self] { self->RetryLoop(); });
}

void RtmpRetryingClientStream::Impl::RetryLoop() {
    const int64_t since = monotonic_us();
    for (int attempt = 0; !destroyed.load(); ++attempt) {
        if (attempt >= options.fast_retry_count) {
            // sleep in slices so Destroy() is not held up
            const int64_t wake = monotonic_us() + (int64_t)options.retry_interval_ms * 1000;
            while (!destroyed.load() && monotonic_us() < wake) fiber::usleep(10000);
        }
        if (destroyed.load()) break;
        if (options.max_retry_duration_ms >= 0 &&
            monotonic_us() - since > (int64_t)options.max_retry_duration_ms * 1000) {
            LOG(WARNING) << "rtmp retrying stream gave up after " << attempt << " attempts";
            owner->CallOnStop();  // Destroy() waits for `retrying` to drop
            std::lock_guard<std::mutex> g(mu);
            retrying = false;
            return;
        }
        Collect();
        if (Start() == 0) break;
    }
    std::lock_guard<std::mutex> g(mu);
    retrying = false;
}

void RtmpRetryingClientStream::Impl::Collect() {
    std::vector<std::unique_ptr<SubStream>> subs;
    std::vector<std::shared_ptr<RtmpClient>> clients;
    {
        std::lock_guard<std::mutex> g(mu);
        subs.swap(retired);
        clients.swap(retired_clients);
    }
    for (auto& s : subs) {
        s->by_owner.store(true);
        s->Destroy();  // deleteStream if still open; no callback runs once it returns
    }
    subs.clear();
    clients.clear();
}

RtmpRetryingClientStream::RtmpRetryingClientStream() : _impl(std::make_shared<Impl>()) { _impl->owner = this; }

RtmpRetryingClientStream::~RtmpRetryingClientStream() { Destroy(); }

int RtmpRetryingClientStream::Init(RtmpSubStreamCreator* creator, const RtmpRetryingClientStreamOptions& options) {
    _impl->creator.reset(creator);
    _impl->options = options;
    if (!creator) return -1;
    if (_impl->Start() == 0) return 0;
    {
        std::lock_guard<std::mutex> g(_impl->mu);
        if (_impl->retrying) return -1;
        _impl->retrying = true;
    }
    std::shared_ptr<Impl> self = _impl;
    fiber::start([self] { self->RetryLoop(); });
    return -1;
}

void RtmpRetryingClientStream::Destroy() {
    if (_impl->destroyed.exchange(true)) return;
    std::unique_ptr<SubStream> cur;
    {
        std::lock_guard<std::mutex> g(_impl->mu);
        cur = std::move(_impl->current);
    }
    if (cur) {
        cur->by_owner.store(true);
        cur->Destroy();
    }
    // wait for a retry fiber to notice (it never touches the owner after
    // observing `destroyed`)
    for (int i = 0; i < 1000; ++i) {
        {
            std::lock_guard<std::mutex> g(_impl->mu);
            if (!_impl->retrying) break;
        }
        fiber::usleep(1000);
    }
    _impl->Collect();
    {
        std::lock_guard<std::mutex> g(_impl->mu);
        _impl->client.reset();
    }
    CallOnStop();
}

int64_t RtmpRetryingClientStream::reconnects() const { return _impl->reconnects.load(); }

bool RtmpRetryingClientStream::connected() const {
    std::lock_guard<std::mutex> g(_impl->mu);
    return _impl->current && !_impl->current->is_stopped();
}

int RtmpRetryingClientStream::SendMessage(uint8_t type, uint32_t timestamp, const Buf& body) {
    std::lock_guard<std::mutex> g(_impl->mu);
    if (!_impl->current || _impl->current->is_stopped()) {
        errno = EAGAIN;
        return -1;
    }
    return _impl->current->RtmpStreamBase::SendMessage(type, timestamp, body);
}

}  // namespace mrpc
