// ExecutionQueue: MPSC task queue consumed in batches by one fiber at a time
// (role of bthread/execution_queue.h:159-206). Producers never block; the
// first producer on an idle queue starts the consumer fiber. High-priority
// tasks run before normal ones. After stop(), the consumer is invoked once
// more with iterator.is_queue_stopped() == true, then join() returns.
// Used by Streaming RPC receivers (batched on_received_messages) and by the
// GPU transfer engine.
#pragma once

#include <cerrno>
#include <memory>
#include <mutex>
#include <vector>

#include "fiber/fiber.h"
#include "fiber/sync.h"

namespace mrpc {
namespace fiber {

template <typename T>
class ExecutionQueue : public std::enable_shared_from_this<ExecutionQueue<T>> {
public:
    class Iterator {
    public:
        explicit operator bool() const { return _i < _v->size(); }
        T& operator*() { return (*_v)[_i]; }
        T* operator->() { return &(*_v)[_i]; }
        Iterator& operator++() { ++_i; return *this; }
        bool is_queue_stopped() const { return _stopped; }
        size_t size() const { return _v->size(); }
    private:
        friend class ExecutionQueue;
        Iterator(std::vector<T>* v, bool stopped) : _v(v), _i(0), _stopped(stopped) {}
        std::vector<T>* _v;
        size_t _i;
        bool _stopped;
    };
    typedef int (*ExecuteFn)(void* meta, Iterator& iter);
    struct Options {
        Attr attr;
        size_t max_batch = 128;
        Options() : attr(ATTR_NORMAL) {}
    };

    static std::shared_ptr<ExecutionQueue> Create(ExecuteFn fn, void* meta, const Options& opt = Options()) {
        return std::shared_ptr<ExecutionQueue>(new ExecutionQueue(fn, meta, opt));
    }
    ~ExecutionQueue() {}

    int execute(const T& t, bool high_priority = false) { return execute_impl(T(t), high_priority); }
    int execute(T&& t, bool high_priority = false) { return execute_impl(std::move(t), high_priority); }

    void stop() {
        bool start_consumer = false;
        {
            std::lock_guard<std::mutex> g(_mu);
            if (_stopped) return;
            _stopped = true;
            if (!_running) {
                _running = true;
                start_consumer = true;
            }
        }
        if (start_consumer) launch();
    }
    int join() {
        _done.wait();
        return 0;
    }
    bool stopped() const {
        std::lock_guard<std::mutex> g(_mu);
        return _stopped;
    }
    size_t pending() const {
        std::lock_guard<std::mutex> g(_mu);
        return _high.size() + _normal.size();
    }

private:
    ExecutionQueue(ExecuteFn fn, void* meta, const Options& opt)
        : _fn(fn), _meta(meta), _opt(opt), _running(false), _stopped(false), _stopped_delivered(false), _done(1) {}

    int execute_impl(T&& t, bool high) {
        bool start_consumer = false;
        {
            std::lock_guard<std::mutex> g(_mu);
            if (_stopped) return EINVAL;
            (high ? _high : _normal).push_back(std::move(t));
            if (!_running) {
                _running = true;
                start_consumer = true;
            }
        }
        if (start_consumer) launch();
        return 0;
    }

    void launch() {
        auto self = this->shared_from_this();
        auto* holder = new std::shared_ptr<ExecutionQueue>(self);
        if (start_background(nullptr, &_opt.attr, &ExecutionQueue::consumer, holder) != 0) {
            consumer(holder);
        }
    }

    static void* consumer(void* arg) {
        auto* holder = static_cast<std::shared_ptr<ExecutionQueue>*>(arg);
        ExecutionQueue* q = holder->get();
        std::vector<T> batch;
        for (;;) {
            bool deliver_stop = false;
            {
                std::lock_guard<std::mutex> g(q->_mu);
                batch.clear();
                size_t take = 0;
                while (!q->_high.empty() && take < q->_opt.max_batch) {
                    batch.push_back(std::move(q->_high.front()));
                    q->_high.erase(q->_high.begin());
                    ++take;
                }
                if (take < q->_opt.max_batch && !q->_normal.empty()) {
                    size_t n = std::min(q->_normal.size(), q->_opt.max_batch - take);
                    for (size_t i = 0; i < n; ++i) batch.push_back(std::move(q->_normal[i]));
                    q->_normal.erase(q->_normal.begin(), q->_normal.begin() + n);
                }
                if (batch.empty()) {
                    if (q->_stopped && !q->_stopped_delivered) {
                        q->_stopped_delivered = true;
                        deliver_stop = true;
                    } else {
                        q->_running = false;
                        break;
                    }
                }
            }
            Iterator it(&batch, deliver_stop);
            q->_fn(q->_meta, it);
            if (deliver_stop) {
                std::lock_guard<std::mutex> g(q->_mu);
                q->_running = false;
                q->_done.signal();
                break;
            }
        }
        delete holder;
        return nullptr;
    }

    ExecuteFn _fn;
    void* _meta;
    Options _opt;
    mutable std::mutex _mu;
    std::vector<T> _high;
    std::vector<T> _normal;
    bool _running;
    bool _stopped;
    bool _stopped_delivered;
    CountdownEvent _done;
};

}  // namespace fiber
}  // namespace mrpc
