// ExecutionQueue: MPSC task queue consumed in batches by one fiber at a time
// (role of bthread/execution_queue.h:159-206). Producers never block; the
// first producer on an idle queue starts the consumer fiber. High-priority
// tasks run before normal ones. After stop(), the consumer is invoked once
// more with iterator.is_queue_stopped() == true, then join() returns.
// execute() can hand back a TaskHandle; cancel(handle) removes the task if
// the consumer has not taken it yet (execution_queue_cancel, reference
// bthread/execution_queue.h:206: 0 cancelled, 1 already running or done).
// Used by Streaming RPC receivers (batched on_received_messages) and by the
// GPU transfer engine.
#pragma once

#include <algorithm>
#include <cerrno>
#include <deque>
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
    // Names a task for cancel(); default-constructed handles name nothing.
    struct TaskHandle {
        uint64_t seq = 0;
        bool high = false;
        std::weak_ptr<ExecutionQueue> queue;
    };
    struct Options {
        Attr attr;
        size_t max_batch = 128;
        Options() : attr(ATTR_NORMAL) {}
    };

    static std::shared_ptr<ExecutionQueue> Create(ExecuteFn fn, void* meta, const Options& opt = Options()) {
        return std::shared_ptr<ExecutionQueue>(new ExecutionQueue(fn, meta, opt));
    }
    ~ExecutionQueue() {}

    int execute(const T& t, bool high_priority = false, TaskHandle* handle = nullptr) {
        return execute_impl(T(t), high_priority, handle);
    }
    int execute(T&& t, bool high_priority = false, TaskHandle* handle = nullptr) {
        return execute_impl(std::move(t), high_priority, handle);
    }
    // 0: the task was removed before the consumer took it; 1: it is running
    // or ran already; -1: the handle names no task of this queue.
    int cancel(const TaskHandle& h) {
        std::shared_ptr<ExecutionQueue> q = h.queue.lock();
        if (q.get() != this || h.seq == 0) return -1;
        std::lock_guard<std::mutex> g(_mu);
        std::deque<Node>& d = h.high ? _high : _normal;
        auto it = std::lower_bound(d.begin(), d.end(), h.seq,
                                   [](const Node& n, uint64_t seq) { return n.seq < seq; });
        if (it == d.end() || it->seq != h.seq) return 1;
        d.erase(it);
        return 0;
    }

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

    struct Node {
        T task;
        uint64_t seq;
    };

    int execute_impl(T&& t, bool high, TaskHandle* handle) {
        bool start_consumer = false;
        {
            std::lock_guard<std::mutex> g(_mu);
            if (_stopped) return EINVAL;
            const uint64_t seq = ++_next_seq;
            (high ? _high : _normal).push_back(Node{std::move(t), seq});
            if (handle) {
                handle->seq = seq;
                handle->high = high;
                handle->queue = this->shared_from_this();
            }
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
                    batch.push_back(std::move(q->_high.front().task));
                    q->_high.pop_front();
                    ++take;
                }
                while (take < q->_opt.max_batch && !q->_normal.empty()) {
                    batch.push_back(std::move(q->_normal.front().task));
                    q->_normal.pop_front();
                    ++take;
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
    std::deque<Node> _high;
    std::deque<Node> _normal;
    uint64_t _next_seq = 0;
    bool _running;
    bool _stopped;
    bool _stopped_delivered;
    CountdownEvent _done;
};

}  // namespace fiber
}  // namespace mrpc
