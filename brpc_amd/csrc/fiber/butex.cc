#include "fiber/butex.h"

#include <cerrno>
#include <climits>

#include "base/containers.h"
#include "base/logging.h"
#include "base/pool.h"
#include "base/time.h"
#include "fiber/internal.h"
#include "fiber/timer.h"

namespace mrpc {
namespace fiber {

namespace {

class SpinLock {
public:
    void lock() {
        while (_f.exchange(true, std::memory_order_acquire)) {
            int spins = 0;
            while (_f.load(std::memory_order_relaxed)) {
                if (++spins < 64) cpu_relax();
                else sched_yield();
            }
        }
    }
    void unlock() { _f.store(false, std::memory_order_release); }
private:
    std::atomic<bool> _f{false};
};

enum WaiterState { WAITER_READY = 0, WAITER_TIMEDOUT, WAITER_UNMATCHED, WAITER_INTERRUPTED };

}  // namespace

struct Butex;

struct ButexWaiter : public LinkNode {
    fiber_t tid = 0;  // 0 for pthread waiters
    std::atomic<Butex*> container{nullptr};
};

struct FiberWaiter : public ButexWaiter {
    TaskMeta* meta = nullptr;
    TimerThread::TaskId sleep_id = 0;
    int state = WAITER_READY;
    int expected = 0;
    Butex* initial = nullptr;
    const timespec* abstime = nullptr;
};

struct PthreadWaiter : public ButexWaiter {
    std::atomic<int> sig{0};
};

struct MRPC_CACHELINE_ALIGNED Butex {
    std::atomic<int> value{0};
    LinkNode waiters;
    SpinLock lock;
};

static_assert(offsetof(Butex, value) == 0, "value must be first");

static inline Butex* to_butex(std::atomic<int>* v) { return reinterpret_cast<Butex*>(v); }

std::atomic<int>* butex_create() {
    Butex* b = get_object<Butex>();
    b->value.store(0, std::memory_order_relaxed);
    return &b->value;
}

void butex_destroy(std::atomic<int>* v) {
    if (!v) return;
    return_object<Butex>(to_butex(v));
}

static void wakeup_pthread(PthreadWaiter* pw) {
    pw->sig.store(1, std::memory_order_release);
    futex_wake_private(&pw->sig, 1);
}

static void run_fiber_waiter(FiberWaiter* w, bool nosignal) { ready_to_run_general(w->tid, nosignal); }

int butex_wake(std::atomic<int>* v, bool nosignal) {
    Butex* b = to_butex(v);
    ButexWaiter* front = nullptr;
    b->lock.lock();
    if (b->waiters.empty()) {
        b->lock.unlock();
        return 0;
    }
    front = static_cast<ButexWaiter*>(b->waiters.next);
    front->remove();
    front->container.store(nullptr, std::memory_order_relaxed);
    b->lock.unlock();
    if (front->tid == 0) {
        wakeup_pthread(static_cast<PthreadWaiter*>(front));
    } else {
        run_fiber_waiter(static_cast<FiberWaiter*>(front), nosignal);
    }
    return 1;
}

static int wake_list(LinkNode* head, bool nosignal) {
    int n = 0;
    // most wake-ups release a handful of fibers: no heap allocation for those
    ButexWaiter* inline_fibers[16];
    std::vector<ButexWaiter*> more;
    size_t nf = 0;
    while (!head->empty()) {
        ButexWaiter* w = static_cast<ButexWaiter*>(head->next);
        w->remove();
        ++n;
        if (w->tid == 0) {
            wakeup_pthread(static_cast<PthreadWaiter*>(w));
        } else if (nf < 16) {
            inline_fibers[nf++] = w;
        } else {
            more.push_back(w);
        }
    }
    const size_t total = nf + more.size();
    if (total) {
        TaskGroup* g = tls_group();
        for (size_t i = 0; i < total; ++i) {
            ButexWaiter* w = i < nf ? inline_fibers[i] : more[i - nf];
            const bool last = (i + 1 == total);
            if (g) {
                g->ready_to_run(w->tid, nosignal || !last);
            } else {
                ready_to_run_general(w->tid, nosignal || !last);
            }
        }
        if (!g && !nosignal && total > 1) flush();  // several fibers: wake more than one worker
    }
    return n;
}

int butex_wake_all(std::atomic<int>* v, bool nosignal) {
    Butex* b = to_butex(v);
    LinkNode tmp;
    b->lock.lock();
    if (b->waiters.empty()) {
        b->lock.unlock();
        return 0;
    }
    // move all waiters to tmp
    while (!b->waiters.empty()) {
        ButexWaiter* w = static_cast<ButexWaiter*>(b->waiters.next);
        w->remove();
        w->container.store(nullptr, std::memory_order_relaxed);
        w->insert_before(&tmp);
    }
    b->lock.unlock();
    return wake_list(&tmp, nosignal);
}

int butex_wake_except(std::atomic<int>* v, fiber_t excluded) {
    Butex* b = to_butex(v);
    LinkNode tmp;
    b->lock.lock();
    if (b->waiters.empty()) {
        b->lock.unlock();
        return 0;
    }
    LinkNode* n = b->waiters.next;
    while (n != &b->waiters) {
        ButexWaiter* w = static_cast<ButexWaiter*>(n);
        n = n->next;
        if (w->tid != 0 && w->tid == excluded) continue;
        w->remove();
        w->container.store(nullptr, std::memory_order_relaxed);
        w->insert_before(&tmp);
    }
    b->lock.unlock();
    return wake_list(&tmp, false);
}

int butex_requeue(std::atomic<int>* v1, std::atomic<int>* v2) {
    Butex* b = to_butex(v1);
    Butex* m = to_butex(v2);
    ButexWaiter* front = nullptr;
    {
        // lock ordering by address to avoid deadlocks
        Butex* first = b < m ? b : m;
        Butex* second = b < m ? m : b;
        first->lock.lock();
        if (second != first) second->lock.lock();
        if (!b->waiters.empty()) {
            front = static_cast<ButexWaiter*>(b->waiters.next);
            front->remove();
            front->container.store(nullptr, std::memory_order_relaxed);
            while (!b->waiters.empty()) {
                ButexWaiter* w = static_cast<ButexWaiter*>(b->waiters.next);
                w->remove();
                w->insert_before(&m->waiters);
                w->container.store(m, std::memory_order_relaxed);
            }
        }
        if (second != first) second->lock.unlock();
        first->lock.unlock();
    }
    if (!front) return 0;
    if (front->tid == 0) {
        wakeup_pthread(static_cast<PthreadWaiter*>(front));
    } else {
        run_fiber_waiter(static_cast<FiberWaiter*>(front), false);
    }
    return 1;
}

// Remove w from whichever butex holds it; returns true if it was removed by us.
static bool erase_from_butex(ButexWaiter* w, bool wakeup, int state) {
    bool erased = false;
    Butex* b;
    while ((b = w->container.load(std::memory_order_acquire)) != nullptr) {
        b->lock.lock();
        if (b == w->container.load(std::memory_order_relaxed)) {
            w->remove();
            w->container.store(nullptr, std::memory_order_relaxed);
            if (w->tid) static_cast<FiberWaiter*>(w)->state = state;
            erased = true;
            b->lock.unlock();
            break;
        }
        b->lock.unlock();
    }
    if (erased && wakeup) {
        if (w->tid) {
            ready_to_run_general(w->tid);
        } else {
            wakeup_pthread(static_cast<PthreadWaiter*>(w));
        }
    }
    return erased;
}

static void erase_from_butex_and_wakeup(void* arg) {
    erase_from_butex(static_cast<ButexWaiter*>(arg), true, WAITER_TIMEDOUT);
}

bool erase_from_butex_because_of_interruption(ButexWaiter* w) {
    return erase_from_butex(w, true, WAITER_INTERRUPTED);
}

// Runs as a "remained" callback after the waiting fiber switched out.
static void wait_for_butex(void* arg) {
    FiberWaiter* const bw = static_cast<FiberWaiter*>(arg);
    Butex* const b = bw->initial;
    {
        b->lock.lock();
        if (b->value.load(std::memory_order_relaxed) != bw->expected) {
            bw->state = WAITER_UNMATCHED;
        } else if (bw->state == WAITER_READY && !bw->meta->interrupted) {
            bw->insert_before(&b->waiters);
            bw->container.store(b, std::memory_order_relaxed);
            if (bw->abstime) {
                // Scheduled under the waiter lock so a waker cannot resume
                // the fiber before sleep_id is published.
                bw->sleep_id = get_global_timer_thread()->schedule(erase_from_butex_and_wakeup, bw, *bw->abstime);
                if (!bw->sleep_id) {
                    bw->remove();
                    bw->container.store(nullptr, std::memory_order_relaxed);
                    bw->state = WAITER_TIMEDOUT;
                    b->lock.unlock();
                    tls_group()->ready_to_run(bw->tid);
                    return;
                }
            }
            b->lock.unlock();
            return;
        }
        b->lock.unlock();
    }
    // Not queued: run the fiber again.
    tls_group()->ready_to_run(bw->tid);
}

static int wait_pthread(PthreadWaiter& pw, const timespec* abstime) {
    for (;;) {
        if (pw.sig.load(std::memory_order_acquire) != 0) return 0;
        timespec rel;
        const timespec* prel = nullptr;
        if (abstime) {
            int64_t left_us = (abstime->tv_sec * 1000000LL + abstime->tv_nsec / 1000) - realtime_us();
            if (left_us <= 0) {
                if (erase_from_butex(&pw, false, WAITER_TIMEDOUT)) {
                    errno = ETIMEDOUT;
                    return -1;
                }
                // being woken concurrently; wait for the signal
                while (pw.sig.load(std::memory_order_acquire) == 0) sched_yield();
                return 0;
            }
            rel = ns_to_timespec(left_us * 1000);
            prel = &rel;
        }
        futex_wait_private(&pw.sig, 0, prel);
    }
}

static int butex_wait_from_pthread(TaskGroup* g, Butex* b, int expected, const timespec* abstime) {
    TaskMeta* task = g ? g->current_task() : nullptr;
    PthreadWaiter pw;
    pw.tid = 0;
    int rc;
    b->lock.lock();
    if (b->value.load(std::memory_order_relaxed) != expected) {
        b->lock.unlock();
        errno = EWOULDBLOCK;
        return -1;
    }
    pw.insert_before(&b->waiters);
    pw.container.store(b, std::memory_order_relaxed);
    b->lock.unlock();
    if (task) task->current_waiter.store(&pw, std::memory_order_release);
    rc = wait_pthread(pw, abstime);
    if (task) {
        while (task->current_waiter.exchange(nullptr, std::memory_order_acquire) == nullptr) sched_yield();
        if (task->interrupted) {
            task->interrupted = false;
            if (rc == 0) {
                errno = EINTR;
                return -1;
            }
        }
    }
    return rc;
}

int butex_wait(std::atomic<int>* v, int expected, const timespec* abstime) {
    Butex* b = to_butex(v);
    if (b->value.load(std::memory_order_relaxed) != expected) {
        errno = EWOULDBLOCK;
        std::atomic_thread_fence(std::memory_order_acquire);
        return -1;
    }
    TaskGroup* g = tls_group();
    if (g == nullptr || g->is_current_main_task()) return butex_wait_from_pthread(g, b, expected, abstime);
    if (abstime) {
        int64_t deadline = abstime->tv_sec * 1000000LL + abstime->tv_nsec / 1000;
        if (deadline <= realtime_us() + 2) {
            errno = ETIMEDOUT;
            return -1;
        }
    }
    FiberWaiter bw;
    bw.tid = g->current_tid();
    bw.meta = g->current_task();
    bw.expected = expected;
    bw.initial = b;
    bw.abstime = abstime;
    bw.state = WAITER_READY;
    bw.meta->current_waiter.store(&bw, std::memory_order_release);
    g->set_remained(wait_for_butex, &bw);
    TaskGroup::sched(&g);

    // The timer callback may still be running and touching bw; wait for it.
    if (bw.sleep_id) {
        while (get_global_timer_thread()->unschedule(bw.sleep_id) == -1) cpu_relax();
    }
    // interrupt() may be using bw: spin until it gives the pointer back.
    while (bw.meta->current_waiter.exchange(nullptr, std::memory_order_acquire) == nullptr) cpu_relax();
    bool interrupted = false;
    if (bw.meta->interrupted) {
        bw.meta->interrupted = false;
        interrupted = true;
    }
    if (bw.state == WAITER_TIMEDOUT) {
        errno = ETIMEDOUT;
        return -1;
    }
    if (bw.state == WAITER_UNMATCHED) {
        errno = EWOULDBLOCK;
        return -1;
    }
    if (interrupted || bw.state == WAITER_INTERRUPTED) {
        errno = bw.meta->stop ? ESTOP : EINTR;
        return -1;
    }
    return 0;
}

}  // namespace fiber
}  // namespace mrpc
