// Fiber scheduler implementation. See internal.h for the design notes.
#if defined(__SANITIZE_ADDRESS__)
#include <pthread.h>
#include <sanitizer/asan_interface.h>
#include <sanitizer/common_interface_defs.h>
#endif
#if defined(__SANITIZE_THREAD__)
#include <sanitizer/tsan_interface.h>
#endif
#include <dirent.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <functional>
#include <map>

#include "base/flags.h"
#include "base/logging.h"
#include "base/pool.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/butex.h"
#include "fiber/context.h"

#include "fiber/internal.h"
#include "fiber/interrupt_pthread.h"
#include "fiber/key_internal.h"
#include "fiber/timer.h"

// ThreadSanitizer must be told which logical thread (fiber) runs on a stack,
// or it attributes the accesses of every fiber a worker runs to the worker
// and reports nonsense: each fiber context gets a TSan fiber,
// the worker's main context keeps the thread's own, and every stack switch
// is announced with __tsan_switch_to_fiber right before the jump.
#if defined(__SANITIZE_THREAD__)
#define MRPC_TSAN_NEW_CONTEXT(m) ((m)->tsan_fiber = __tsan_create_fiber(0))
#define MRPC_TSAN_MAIN_CONTEXT(m) ((m)->tsan_fiber = __tsan_get_current_fiber())
#define MRPC_TSAN_SWITCH(next) __tsan_switch_to_fiber((next)->tsan_fiber, 0)
#define MRPC_TSAN_DESTROY(m)                   \
    do {                                       \
        if ((m)->tsan_fiber && !(m)->is_main) { \
            __tsan_destroy_fiber((m)->tsan_fiber); \
        }                                      \
        (m)->tsan_fiber = nullptr;             \
    } while (0)
#else
#define MRPC_TSAN_NEW_CONTEXT(m) (void)0
#define MRPC_TSAN_MAIN_CONTEXT(m) (void)0
#define MRPC_TSAN_SWITCH(next) (void)0
#define MRPC_TSAN_DESTROY(m) (void)0
#endif

DEFINE_int32(fiber_concurrency, 8, "Number of fiber worker pthreads");
DEFINE_int32(fiber_min_concurrency, 0, "Initial number of workers; grows lazily up to fiber_concurrency if > 0");
DEFINE_int32(stack_size_small, 32768, "size of small fiber stacks");
DEFINE_int32(stack_size_normal, 1048576, "size of normal fiber stacks");
DEFINE_int32(stack_size_large, 8388608, "size of large fiber stacks");
DEFINE_int32(guard_page_size, 4096, "size of guard page at the bottom of fiber stacks");
DEFINE_int32(task_group_runqueue_capacity, 4096, "capacity of each worker's run queue");
DEFINE_int32(cpu_l3_domain, -1,
             "confine the whole process (all threads) to the CPUs sharing the k-th L3 cache of the "
             "affinity mask (-1: leave the mask alone); one process per GPU passes a rank-derived k");
DEFINE_int32(fiber_worker_cpu_offset, -1,
             "pin worker i to the (offset + i)-th CPU of the process affinity mask (-1: no pinning); "
             "one process per GPU passes local_rank * cpus_per_rank");
// Off by default: on the MI355X box (16-CPU quota) idle spinning cost more
// throughput than it saved latency (profiles/bench_r1_spin_ab.txt).
DEFINE_bool(fiber_signal_parked_only, true,
            "a ready fiber enters the kernel (FUTEX_WAKE) only when a worker is parked; false: every signal "
            "wakes unconditionally, one syscall per parking lot tried");
DEFINE_int32(fiber_idle_spin_us, 0,
             "an idle worker polls for new fibers this long before sleeping on its parking lot "
             "(trades CPU for futex-wakeup latency on the RPC round trip; 0 disables)");
DEFINE_int32(fiber_max_spinning_workers, 2, "at most this many idle workers spin at once");
DEFINE_bool(fiber_signal_skip_when_spinning, true,
            "with -fiber_idle_spin_us > 0, a ready fiber wakes no parked worker while another worker spins");
DEFINE_int32(fiber_worker_nap_us, 0,
             "an idle worker that ran a fiber within -fiber_worker_nap_window_ms sleeps on its parking lot with "
             "this timeout (us) and re-polls, so its core stays in shallow idle states (warm caches, us wakeups) "
             "instead of the deep state a long sleep lets the governor pick (0 disables)");
DEFINE_int32(fiber_nap_workers, 2, "at most this many idle workers nap at once (the rest sleep for good)");
DEFINE_int32(fiber_worker_nap_window_ms, 1000, "how long after its last fiber a worker keeps napping");

namespace mrpc {
namespace fiber {

const Attr ATTR_NORMAL(STACK_NORMAL, 0);
const Attr ATTR_SMALL(STACK_SMALL, 0);
const Attr ATTR_PTHREAD(STACK_PTHREAD, 0);

// ------------------------------------------------------------------ stacks
struct Stack {
    void* base = nullptr;   // lowest usable address
    size_t size = 0;        // usable size
    StackType type = STACK_UNKNOWN;
    size_t guard = 0;
};

namespace {
struct StackPool {
    std::mutex mu;
    std::vector<Stack*> free;
};
// never destroyed: workers still return stacks while static destructors run at exit
StackPool* const g_stack_pools = new StackPool[5];
std::atomic<int64_t> g_nstack{0};

size_t stack_size_of(StackType t) {
    switch (t) {
    case STACK_SMALL: return (size_t)FLAGS_stack_size_small;
    case STACK_LARGE: return (size_t)FLAGS_stack_size_large;
    default: return (size_t)FLAGS_stack_size_normal;
    }
}

// Per-worker stack cache: a fiber that ends on a worker leaves its stack
// there for the next fiber that worker starts (no lock, warm cache lines);
// overflow goes to the global pools.
const size_t kTlsStackCacheSize = 32;
struct TlsStackCache {
    std::vector<Stack*> v[5];
};
thread_local TlsStackCache tls_stack_cache;

Stack* get_stack(StackType t) {
    if (t == STACK_PTHREAD || t == STACK_UNKNOWN) t = STACK_NORMAL;
    auto& local = tls_stack_cache.v[t];
    if (!local.empty()) {
        Stack* s = local.back();
        local.pop_back();
        return s;
    }
    {
        StackPool& p = g_stack_pools[t];
        std::lock_guard<std::mutex> g(p.mu);
        if (!p.free.empty()) {
            Stack* s = p.free.back();
            p.free.pop_back();
            return s;
        }
    }
    const size_t page = 4096;
    size_t sz = (stack_size_of(t) + page - 1) & ~(page - 1);
    size_t guard = FLAGS_guard_page_size > 0 ? (((size_t)FLAGS_guard_page_size + page - 1) & ~(page - 1)) : 0;
    void* mem = mmap(nullptr, sz + guard, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (mem == MAP_FAILED) {
        PLOG(ERROR) << "mmap fiber stack";
        return nullptr;
    }
    if (guard && mprotect(mem, guard, PROT_NONE) != 0) {
        PLOG(WARNING) << "mprotect guard page";
    }
    Stack* s = new Stack;
    s->base = (char*)mem + guard;
    s->size = sz;
    s->type = t;
    s->guard = guard;
    g_nstack.fetch_add(1, std::memory_order_relaxed);
    return s;
}

void return_stack(Stack* s) {
    auto& local = tls_stack_cache.v[s->type];
    if (local.size() < kTlsStackCacheSize) {
        local.push_back(s);
        return;
    }
    StackPool& p = g_stack_pools[s->type];
    std::lock_guard<std::mutex> g(p.mu);
    if (p.free.size() < 1024) {
        p.free.push_back(s);
        return;
    }
    munmap((char*)s->base - s->guard, s->size + s->guard);
    g_nstack.fetch_sub(1, std::memory_order_relaxed);
    delete s;
}

thread_local TaskGroup* tls_task_group = nullptr;
std::atomic<TaskControl*> g_task_control{nullptr};
std::mutex g_task_control_mu;
}  // namespace

__attribute__((noinline)) TaskGroup* tls_group() {
    TaskGroup* g = tls_task_group;
    asm volatile("" ::: "memory");
    return g;
}

__attribute__((noinline)) static void set_tls_group(TaskGroup* g) {
    tls_task_group = g;
    asm volatile("" ::: "memory");
}

TaskMeta* address_meta(fiber_t tid) { return address_resource<TaskMeta>(tid_slot(tid)); }

TaskControl* get_task_control() { return g_task_control.load(std::memory_order_acquire); }

TaskControl* get_or_new_task_control() {
    TaskControl* c = g_task_control.load(std::memory_order_acquire);
    if (c) return c;
    std::lock_guard<std::mutex> g(g_task_control_mu);
    c = g_task_control.load(std::memory_order_acquire);
    if (c) return c;
    get_global_timer_thread();
    c = new TaskControl;
    int n = FLAGS_fiber_concurrency;
    if (FLAGS_fiber_min_concurrency > 0 && FLAGS_fiber_min_concurrency < n) n = FLAGS_fiber_min_concurrency;
    if (c->init(n) != 0) {
        LOG(FATAL) << "Fail to init fiber TaskControl";
    }
    g_task_control.store(c, std::memory_order_release);
    return c;
}

// ------------------------------------------------------------------ TaskGroup
TaskGroup::TaskGroup(TaskControl* c) : _control(c), _cur_meta(nullptr), _main_meta(nullptr), _main_tid(0) {
    _steal_seed = fast_rand();
    _steal_offset = 0;
}

TaskGroup::~TaskGroup() {}

int TaskGroup::init(size_t rq_cap) {
    size_t cap = 1;
    while (cap < rq_cap) cap <<= 1;
    _rq.init(cap);
    uint32_t slot;
    TaskMeta* m = get_resource<TaskMeta>(&slot);
    if (!m) return -1;
    if (!m->version_butex) {
        m->version_butex = butex_create();
        m->version_butex->store(1, std::memory_order_relaxed);
    }
    m->is_main = true;
    m->stop.store(false, std::memory_order_relaxed);
    m->interrupted.store(false, std::memory_order_relaxed);
    m->fn = nullptr;
    m->arg = nullptr;
    m->stack = nullptr;
    m->attr = ATTR_PTHREAD;
    m->tid = make_tid((uint32_t)m->version_butex->load(std::memory_order_relaxed), slot);
    MRPC_TSAN_MAIN_CONTEXT(m);
    _main_meta = m;
    _main_tid = m->tid;
    _cur_meta = m;
    return 0;
}

void TaskGroup::run_remained() {
    while (_last_fn) {
        void (*fn)(void*) = _last_fn;
        void* arg = _last_arg;
        _last_fn = nullptr;
        fn(arg);
    }
}

static void ready_to_run_in_worker(void* arg) {
    TaskGroup* g = tls_group();
    g->ready_to_run((fiber_t)(uintptr_t)arg);
}

static void ready_to_run_in_worker_nosignal(void* arg) {
    TaskGroup* g = tls_group();
    g->ready_to_run((fiber_t)(uintptr_t)arg, true);
}

void TaskGroup::sched_to(TaskGroup** pg, fiber_t next_tid) {
    TaskMeta* m = address_meta(next_tid);
    sched_to(pg, m);
}

void TaskGroup::sched_to(TaskGroup** pg, TaskMeta* next) { sched_to_impl(pg, next, false); }

// AddressSanitizer must be told about stack switches, otherwise shadow left
// by a fiber on a pooled stack (or by the worker's own stack) reads as
// overflow / use-after-scope once another context runs there.
#if defined(__SANITIZE_ADDRESS__)
static void asan_target_stack(const TaskMeta* next, const void** bottom, size_t* size) {
    if (next->stack) {
        *bottom = next->stack->base;
        *size = next->stack->size;
        return;
    }
    static thread_local const void* t_bottom = nullptr;
    static thread_local size_t t_size = 0;
    if (!t_bottom) {
        pthread_attr_t attr;
        void* addr = nullptr;
        if (pthread_getattr_np(pthread_self(), &attr) == 0) {
            pthread_attr_getstack(&attr, &addr, &t_size);
            pthread_attr_destroy(&attr);
        }
        t_bottom = addr;
    }
    *bottom = t_bottom;
    *size = t_size;
}
#define MRPC_ASAN_START_SWITCH(fake, next)                 \
    do {                                                  \
        const void* _b;                                   \
        size_t _s;                                        \
        asan_target_stack(next, &_b, &_s);                \
        __sanitizer_start_switch_fiber(fake, _b, _s);     \
    } while (0)
#define MRPC_ASAN_FINISH_SWITCH(fake) __sanitizer_finish_switch_fiber(fake, nullptr, nullptr)
#else
#define MRPC_ASAN_START_SWITCH(fake, next) (void)0
#define MRPC_ASAN_FINISH_SWITCH(fake) (void)0
#endif

void TaskGroup::sched_to_impl(TaskGroup** pg, TaskMeta* next, bool handover) {
    TaskGroup* g = *pg;
    TaskMeta* cur = g->_cur_meta;
    if (!handover && next->stack == nullptr && !next->is_main) {
        Stack* s = get_stack(next->attr.stack_type);
        if (!s) {
            LOG(FATAL) << "Out of fiber stacks";
        }
        next->stack = s;
#if defined(__SANITIZE_ADDRESS__)
        // a pooled stack still carries the redzones of the fiber that died on it
        __asan_unpoison_memory_region(s->base, s->size);
#endif
        next->sp = make_context(s->base, s->size, TaskGroup::task_runner);
        MRPC_TSAN_NEW_CONTEXT(next);
    }
    if (next != cur) {
        g->_nswitch.store(g->_nswitch.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
        g->_cur_meta = next;
        cur->running_on.store(0, std::memory_order_relaxed);
        next->running_on.store(pthread_self(), std::memory_order_release);
        if (!handover) {
            void* fake_stack = nullptr;
            (void)fake_stack;
            MRPC_ASAN_START_SWITCH(&fake_stack, next);
            MRPC_TSAN_SWITCH(next);
            mrpc_fiber_jump(&cur->sp, next->sp, nullptr);
            MRPC_ASAN_FINISH_SWITCH(fake_stack);
            g = tls_group();
            *pg = g;
        }
        // else: the ending fiber handed its stack to `next`; we keep running
        // on it and task_runner's loop invokes next->fn directly.
    }
    g->run_remained();
}

void TaskGroup::task_runner(void*) {
    MRPC_ASAN_FINISH_SWITCH(nullptr);  // first entry of a fresh context
    TaskGroup* g = tls_group();
    g->run_remained();
    do {
        TaskMeta* m = g->_cur_meta;
        m->start_ns = monotonic_coarse_ns();  // only the /fibers age (ms)
        if (!m->stop) {
            m->fn(m->arg);
        }
        g = tls_group();
        // fiber-local storage
        if (m->local_storage) {
            return_keytable(m->attr.keytable_pool, m->local_storage);
            m->local_storage = nullptr;
        }
        {
            std::lock_guard<std::mutex> lk(m->version_lock);
            int v = m->version_butex->load(std::memory_order_relaxed);
            m->version_butex->store(v + 1 == 0 ? 1 : v + 1, std::memory_order_release);
        }
        butex_wake_except(m->version_butex, 0);
        g->_control->nfibers.fetch_sub(1, std::memory_order_relaxed);
        g->set_remained([](void* arg) {
            TaskMeta* dead = (TaskMeta*)arg;
            MRPC_TSAN_DESTROY(dead);
            if (dead->stack) {
                return_stack(dead->stack);
                dead->stack = nullptr;
            }
            return_resource<TaskMeta>(tid_slot(dead->tid));
        }, m);
        ending_sched(&g);
    } while (g->_cur_meta != g->_main_meta);
    // Should never reach: the main task never runs on a fiber stack.
    LOG(FATAL) << "task_runner fell through";
}

void TaskGroup::ending_sched(TaskGroup** pg) {
    TaskGroup* g = *pg;
    fiber_t next_tid = 0;
    if (!g->_rq.pop(&next_tid) && !g->steal_task(&next_tid)) next_tid = g->_main_tid;
    TaskMeta* cur = g->_cur_meta;
    TaskMeta* next = address_meta(next_tid);
    if (next->stack == nullptr && !next->is_main && cur->stack &&
        (next->attr.stack_type == cur->stack->type ||
         (next->attr.stack_type == STACK_PTHREAD && cur->stack->type == STACK_NORMAL) ||
         (next->attr.stack_type == STACK_UNKNOWN && cur->stack->type == STACK_NORMAL))) {
        // Hand our stack to the fresh fiber: no context switch needed (it
        // also inherits the TSan fiber of the stack it runs on).
        next->stack = cur->stack;
        cur->stack = nullptr;
#if defined(__SANITIZE_THREAD__)
        next->tsan_fiber = cur->tsan_fiber;
        cur->tsan_fiber = nullptr;
#endif
        sched_to_impl(pg, next, true);
        return;
    }
    sched_to_impl(pg, next, false);
}

void TaskGroup::sched(TaskGroup** pg) {
    TaskGroup* g = *pg;
    fiber_t next_tid = 0;
    if (!g->_rq.pop(&next_tid) && !g->steal_task(&next_tid)) next_tid = g->_main_tid;
    sched_to(pg, next_tid);
}

void TaskGroup::yield(TaskGroup** pg) {
    TaskGroup* g = *pg;
    g->set_remained(ready_to_run_in_worker, (void*)(uintptr_t)g->current_tid());
    sched(pg);
}

struct SleepArgs {
    uint64_t timeout_us;
    fiber_t tid;
    TaskMeta* meta;
    TaskGroup* group;
    uint64_t gen;  // the sleep's generation (TaskMeta::sleep_gen when armed)
};

static void ready_to_run_from_timer(void* arg) { ready_to_run_general((fiber_t)(uintptr_t)arg); }

static void add_sleep_event(void* arg) {
    // `arg` lives on the sleeping fiber's stack: once the timer is armed the
    // fiber may wake on another worker and return from usleep(), so copy
    // everything out before scheduling and never touch `arg` afterwards.
    const SleepArgs e = *(const SleepArgs*)arg;
    TimerThread::TaskId id =
        get_global_timer_thread()->schedule_after_us(ready_to_run_from_timer, (void*)(uintptr_t)e.tid, e.timeout_us);
    if (!id) {
        tls_group()->ready_to_run(e.tid);
        return;
    }
    // Publish the timer id so interrupt() can cancel the sleep (TaskMeta is
    // pooled memory, valid even if the fiber already woke). If this worker
    // was delayed until the fiber woke, returned and maybe slept again, the
    // generation no longer matches and the stale id is dropped.
    {
        std::lock_guard<std::mutex> g(e.meta->sleep_mu);
        if (e.meta->sleep_gen != e.gen) return;
        e.meta->current_sleep.store(id, std::memory_order_seq_cst);
    }
    // interrupt() sets `interrupted` and then takes current_sleep; we publish
    // current_sleep and then look at `interrupted` (both seq_cst): one of the
    // two sees the other, so an interrupt that raced with this publish still
    // ends the sleep (whoever takes the id wakes the fiber)
    if (e.meta->interrupted.load(std::memory_order_seq_cst)) {
        const uint64_t taken = e.meta->current_sleep.exchange(0, std::memory_order_acq_rel);
        if (taken && get_global_timer_thread()->unschedule(taken) == 0) tls_group()->ready_to_run(e.tid);
    }
}

int TaskGroup::usleep(TaskGroup** pg, uint64_t us) {
    if (us == 0) {
        yield(pg);
        return 0;
    }
    TaskGroup* g = *pg;
    TaskMeta* m = g->_cur_meta;
    if (m->interrupted.load(std::memory_order_acquire)) {  // interrupted before it slept
        m->interrupted.store(false, std::memory_order_relaxed);
        errno = m->stop ? ESTOP : EINTR;
        return -1;
    }
    uint64_t gen;
    {
        std::lock_guard<std::mutex> lk(m->sleep_mu);
        gen = ++m->sleep_gen;
        m->current_sleep.store(0, std::memory_order_relaxed);
    }
    SleepArgs e{us, g->current_tid(), m, g, gen};
    g->set_remained(add_sleep_event, &e);
    sched(pg);
    // This sleep is over: retire its generation (a publish still in flight
    // is dropped) and take the id. The timer may still be running (it just
    // woke us); spin until it ends.
    uint64_t id;
    {
        std::lock_guard<std::mutex> lk(m->sleep_mu);
        ++m->sleep_gen;
        id = m->current_sleep.exchange(0, std::memory_order_acquire);
    }
    if (id) {
        // -1: the timer callback that woke us is still returning; it is a
        // few instructions from done, but never burn a whole time slice
        for (int spin = 0; get_global_timer_thread()->unschedule(id) == -1; ++spin) {
            if (spin < 64) cpu_relax();
            else sched_yield();
        }
    }
    if (m->interrupted) {
        m->interrupted = false;
        errno = m->stop ? ESTOP : EINTR;
        return -1;
    }
    return 0;
}

int TaskGroup::interrupt(fiber_t tid, TaskControl* c) {
    TaskMeta* m = address_meta(tid);
    if (!m) return EINVAL;
    {
        std::lock_guard<std::mutex> lk(m->version_lock);
        if ((uint32_t)m->version_butex->load(std::memory_order_relaxed) != tid_version(tid)) return EINVAL;
        m->interrupted.store(true, std::memory_order_seq_cst);
    }
    ButexWaiter* w = m->current_waiter.exchange(nullptr, std::memory_order_acquire);
    if (w) {
        erase_from_butex_because_of_interruption(w);
        m->current_waiter.store(w, std::memory_order_release);
        return 0;
    }
    uint64_t sleep_id = m->current_sleep.exchange(0, std::memory_order_seq_cst);
    if (sleep_id) {
        if (get_global_timer_thread()->unschedule(sleep_id) == 0) ready_to_run_general(tid);
        return 0;
    }
    // neither parked nor sleeping: running on a worker, maybe blocked in a
    // system call the runtime cannot see — SIGURG makes that call return
    // EINTR (interrupt_pthread.h); the fiber sees `interrupted` afterwards
    const pthread_t th = m->running_on.load(std::memory_order_acquire);
    if (th && !pthread_equal(th, pthread_self()) && !m->is_main) interrupt_pthread(th);
    (void)c;
    return 0;
}

void TaskGroup::ready_to_run(fiber_t tid, bool nosignal) {
    if (!_rq.push(tid)) {
        // Run queue full: spill into our remote queue (unbounded).
        std::lock_guard<std::mutex> lk(_remote_mu);
        _remote_rq.push_back(tid);
        _remote_size.fetch_add(1, std::memory_order_release);
    }
    if (nosignal) {
        ++_num_nosignal;
    } else {
        const int n = _num_nosignal + 1;
        _num_nosignal = 0;
        _control->signal_task(n);
    }
}

void TaskGroup::flush_nosignal_tasks() {
    const int n = _num_nosignal;
    if (n) {
        _num_nosignal = 0;
        _control->signal_task(n);
    }
}

void TaskGroup::ready_to_run_remote(fiber_t tid, bool nosignal) {
    int n = 0;
    {
        std::lock_guard<std::mutex> lk(_remote_mu);
        _remote_rq.push_back(tid);
        _remote_size.fetch_add(1, std::memory_order_release);
        if (nosignal) {
            ++_remote_num_nosignal;
        } else {
            n = _remote_num_nosignal + 1;
            _remote_num_nosignal = 0;
        }
    }
    if (n) _control->signal_task(n);
}

void TaskGroup::flush_nosignal_tasks_remote() {
    int n;
    {
        std::lock_guard<std::mutex> lk(_remote_mu);
        n = _remote_num_nosignal;
        _remote_num_nosignal = 0;
    }
    if (n) _control->signal_task(n);
}

bool TaskGroup::steal_task(fiber_t* tid) {
    if (_remote_size.load(std::memory_order_acquire) > 0) {
        std::lock_guard<std::mutex> lk(_remote_mu);
        if (!_remote_rq.empty()) {
            *tid = _remote_rq.front();
            _remote_rq.pop_front();
            _remote_size.fetch_sub(1, std::memory_order_relaxed);
            return true;
        }
    }
    _last_pl_state = _pl->get_state();
    return _control->steal_task(tid, &_steal_seed, _steal_offset);
}

static std::atomic<int> g_spinning_workers{0};
static std::atomic<int> g_napping_workers{0};

// Polls for work for up to -fiber_idle_spin_us. Waking a parked worker
// costs a futex round trip plus the kernel's wakeup latency (tens of µs on
// a loaded host, ~100 µs in a VM) on every RPC hop; a short spin turns most
// of those hops into a cache-line poll. Bounded by
// -fiber_max_spinning_workers so idle spinning never eats the CPU quota.
bool TaskGroup::spin_for_task(fiber_t* tid) {
    const int budget_us = FLAGS_fiber_idle_spin_us;
    if (budget_us <= 0) return false;
    if (g_spinning_workers.fetch_add(1, std::memory_order_seq_cst) >= FLAGS_fiber_max_spinning_workers) {
        g_spinning_workers.fetch_sub(1, std::memory_order_seq_cst);
        return false;
    }
    const int64_t deadline = monotonic_ns() + (int64_t)budget_us * 1000;
    bool got = false;
    int i = 0;
    while (!got) {
        for (int k = 0; k < 16; ++k) cpu_relax();
        if (_rq.pop(tid) || steal_task(tid)) {
            got = true;
            break;
        }
        if (_last_pl_state.stopped()) break;
        if ((++i & 7) == 0 && monotonic_ns() >= deadline) break;
    }
    g_spinning_workers.fetch_sub(1, std::memory_order_seq_cst);
    return got;
}

bool TaskGroup::wait_task(fiber_t* tid) {
    if (_rq.pop(tid)) {
        _last_task_ns = 0;
        return true;
    }
    for (;;) {
        if (steal_task(tid)) {
            _last_task_ns = 0;
            return true;
        }
        if (_last_pl_state.stopped()) return false;
        if (spin_for_task(tid)) {
            _last_task_ns = 0;
            return true;
        }
        int64_t t0 = monotonic_ns();
        if (_last_task_ns == 0) _last_task_ns = t0;  // idle since now
        const int nap_us = FLAGS_fiber_worker_nap_us;
        bool nap = false;
        if (nap_us > 0 && t0 - _last_task_ns < (int64_t)FLAGS_fiber_worker_nap_window_ms * 1000000) {
            nap = g_napping_workers.fetch_add(1, std::memory_order_relaxed) < FLAGS_fiber_nap_workers;
            if (!nap) g_napping_workers.fetch_sub(1, std::memory_order_relaxed);
        }
        if (nap) {
            // Nap: a short timed sleep keeps this core out of the deep idle
            // state (its caches stay warm, it answers a signal in a few us);
            // on the timeout it polls again (benchmarks/latency_trace.py).
            _pl->wait_for(_last_pl_state, (int64_t)nap_us * 1000);
            g_napping_workers.fetch_sub(1, std::memory_order_relaxed);
        } else {
            _pl->wait(_last_pl_state);
        }
        _idle_ns.fetch_add(monotonic_ns() - t0, std::memory_order_relaxed);
    }
}

void TaskGroup::run_main_task() {
    TaskGroup* g = this;
    fiber_t tid;
    while (g->wait_task(&tid)) {
        TaskGroup::sched_to(&g, tid);
        // Back on the main stack; drain local work before parking.
    }
}

template <bool REMOTE>
int TaskGroup::start_background(fiber_t* th, const Attr* attr, FiberFn fn, void* arg) {
    uint32_t slot;
    TaskMeta* m = get_resource<TaskMeta>(&slot);
    if (!m) return ENOMEM;
    if (!m->version_butex) {
        m->version_butex = butex_create();
        m->version_butex->store(1, std::memory_order_relaxed);
    }
    m->current_waiter.store(nullptr, std::memory_order_relaxed);
    m->current_sleep.store(0, std::memory_order_relaxed);
    m->stop.store(false, std::memory_order_relaxed);
    m->interrupted.store(false, std::memory_order_relaxed);
    m->is_main = false;
    m->fn = fn;
    m->arg = arg;
    m->stack = nullptr;
    m->attr = attr ? *attr : ATTR_NORMAL;
    m->local_storage = nullptr;
    m->span = nullptr;
    if ((m->attr.flags & ATTR_INHERIT_SPAN)) {
        TaskGroup* cg = tls_group();
        if (cg) m->span = cg->current_task()->span;
    }
    m->tid = make_tid((uint32_t)m->version_butex->load(std::memory_order_relaxed), slot);
    if (m->attr.keytable_pool) m->local_storage = borrow_keytable(m->attr.keytable_pool);
    *th = m->tid;
    _control->nfibers.fetch_add(1, std::memory_order_relaxed);
    const bool nosignal = (m->attr.flags & ATTR_NOSIGNAL);
    if (REMOTE) {
        ready_to_run_remote(m->tid, nosignal);
    } else {
        ready_to_run(m->tid, nosignal);
    }
    return 0;
}

template int TaskGroup::start_background<true>(fiber_t*, const Attr*, FiberFn, void*);
template int TaskGroup::start_background<false>(fiber_t*, const Attr*, FiberFn, void*);

int TaskGroup::start_foreground(TaskGroup** pg, fiber_t* th, const Attr* attr, FiberFn fn, void* arg) {
    TaskGroup* g = *pg;
    // Create then immediately switch to it; the creator is re-queued by a
    // remained callback so that idle workers can steal it.
    fiber_t tid;
    Attr a = attr ? *attr : ATTR_NORMAL;
    const bool nosignal = a.flags & ATTR_NOSIGNAL;
    a.flags |= ATTR_NOSIGNAL;  // don't signal for the new task: we run it now
    uint32_t slot;
    TaskMeta* m = get_resource<TaskMeta>(&slot);
    if (!m) return ENOMEM;
    if (!m->version_butex) {
        m->version_butex = butex_create();
        m->version_butex->store(1, std::memory_order_relaxed);
    }
    m->current_waiter.store(nullptr, std::memory_order_relaxed);
    m->current_sleep.store(0, std::memory_order_relaxed);
    m->stop.store(false, std::memory_order_relaxed);
    m->interrupted.store(false, std::memory_order_relaxed);
    m->is_main = false;
    m->fn = fn;
    m->arg = arg;
    m->stack = nullptr;
    m->attr = attr ? *attr : ATTR_NORMAL;
    m->local_storage = nullptr;
    m->span = (m->attr.flags & ATTR_INHERIT_SPAN) ? g->current_task()->span : nullptr;
    m->tid = make_tid((uint32_t)m->version_butex->load(std::memory_order_relaxed), slot);
    if (m->attr.keytable_pool) m->local_storage = borrow_keytable(m->attr.keytable_pool);
    tid = m->tid;
    if (th) *th = tid;
    g->_control->nfibers.fetch_add(1, std::memory_order_relaxed);
    if (g->is_current_main_task()) {
        // The main task cannot be re-queued; just put the new fiber first.
        g->ready_to_run(tid, nosignal);
        return 0;
    }
    g->set_remained(nosignal ? ready_to_run_in_worker_nosignal : ready_to_run_in_worker,
                    (void*)(uintptr_t)g->current_tid());
    sched_to(pg, m);
    return 0;
}

// ------------------------------------------------------------------ TaskControl
TaskControl::TaskControl() {
    memset(_groups, 0, sizeof(_groups));
    start_ns = monotonic_ns();
}

namespace {

int read_cpu_int(int cpu, const char* what, int dflt) {
    char path[160];
    snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/%s", cpu, what);
    FILE* f = fopen(path, "r");
    int x = dflt;
    if (f) {
        if (fscanf(f, "%d", &x) != 1) x = dflt;
        fclose(f);
    }
    return x;
}

// Orders `cpus` so that the first SMT thread of every physical core comes
// first, then the second threads, ...
std::vector<int> order_by_core(const std::vector<int>& cpus) {
    std::map<std::pair<int, int>, std::vector<int>> by_core;  // (package, core) -> cpus
    for (int cpu : cpus) {
        by_core[{read_cpu_int(cpu, "topology/physical_package_id", 0), read_cpu_int(cpu, "topology/core_id", cpu)}]
            .push_back(cpu);
    }
    std::vector<int> v;
    for (size_t round = 0;; ++round) {
        bool any = false;
        for (auto& kv : by_core) {
            if (round < kv.second.size()) {
                v.push_back(kv.second[round]);
                any = true;
            }
        }
        if (!any) break;
    }
    return v;
}

std::vector<int> allowed_cpus() {
    std::vector<int> v;
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return v;
    for (int cpu = 0; cpu < CPU_SETSIZE; ++cpu) {
        if (CPU_ISSET(cpu, &allowed)) v.push_back(cpu);
    }
    return v;
}

// The k-th group (mod count) of allowed CPUs sharing an L3 cache, ordered by
// core. The machines this runs on expose hundreds of CPUs to a container
// whose CPU-time quota is a small fraction of them: left alone, the
// scheduler scatters the runtime's threads over many L3 domains (and both
// sockets), and every cross-domain cache-line transfer on the request path
// shows up as latency and as large step-to-step throughput swings.
std::vector<int> l3_domain_cpus(int k) {
    std::map<int, std::vector<int>> groups;  // lowest cpu sharing the L3 -> cpus
    for (int cpu : allowed_cpus()) {
        char path[160];
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
        FILE* f = fopen(path, "r");
        int first = cpu;
        if (f) {
            if (fscanf(f, "%d", &first) != 1) first = cpu;
            fclose(f);
        }
        groups[first].push_back(cpu);
    }
    if (groups.empty()) return {};
    auto it = groups.begin();
    std::advance(it, (size_t)k % groups.size());
    return order_by_core(it->second);
}

// Confines every existing thread (the embedding interpreter, HIP's helpers,
// our workers) and, through the calling thread's mask, every thread created
// from now on to `cpus`; with -fiber_worker_cpu_offset, worker i goes back
// to its own core of the new set.
void confine_process(const std::vector<int>& cpus) {
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus) CPU_SET(c, &set);
    const std::vector<int> order = order_by_core(cpus);
    if (DIR* d = opendir("/proc/self/task")) {
        while (dirent* e = readdir(d)) {
            const int tid = atoi(e->d_name);
            if (tid <= 0) continue;
            int worker = -1;
            if (FLAGS_fiber_worker_cpu_offset >= 0 && !order.empty()) {
                char path[64], name[32] = {0};
                snprintf(path, sizeof(path), "/proc/self/task/%d/comm", tid);
                if (FILE* f = fopen(path, "r")) {
                    if (fscanf(f, "mrpc_worker%d", &worker) != 1) worker = -1;
                    fclose(f);
                }
                (void)name;
            }
            if (worker >= 0) {
                cpu_set_t one;
                CPU_ZERO(&one);
                CPU_SET(order[(size_t)(FLAGS_fiber_worker_cpu_offset + worker) % order.size()], &one);
                sched_setaffinity(tid, sizeof(one), &one);
            } else {
                sched_setaffinity(tid, sizeof(set), &set);
            }
        }
        closedir(d);
    }
    sched_setaffinity(0, sizeof(set), &set);
}

void apply_process_affinity() {
    if (FLAGS_cpu_l3_domain < 0) return;
    const std::vector<int> cpus = l3_domain_cpus(FLAGS_cpu_l3_domain);
    if (cpus.empty()) return;
    confine_process(cpus);
    LOG(INFO) << "fiber runtime confined to L3 domain " << FLAGS_cpu_l3_domain << " (" << cpus.size() << " CPUs from "
              << cpus.front() << ")";
}

}  // namespace

// CPUs of the (possibly confined) affinity mask, physical cores first, for
// pinning workers created later (concurrency growth); RebindL3Domain
// replaces it with the new domain's order.
static std::mutex g_cpu_order_mu;
static std::vector<int>* g_cpu_order = nullptr;

static std::vector<int> cpu_order_by_core() {
    std::lock_guard<std::mutex> g(g_cpu_order_mu);
    if (!g_cpu_order) g_cpu_order = new std::vector<int>(order_by_core(allowed_cpus()));
    return *g_cpu_order;
}

static void set_cpu_order(const std::vector<int>& cpus) {
    std::lock_guard<std::mutex> g(g_cpu_order_mu);
    if (!g_cpu_order) g_cpu_order = new std::vector<int>;
    *g_cpu_order = order_by_core(cpus);
}

int RebindL3Domain(int k) {
    // the domains are indexed over the process's allowed CPUs, which the
    // first confinement narrowed to one domain: index the host's CPUs
    // (the cgroup's cpuset) instead
    cpu_set_t all;
    CPU_ZERO(&all);
    if (FILE* f = fopen("/sys/fs/cgroup/cpuset.cpus.effective", "r")) {
        char buf[4096];
        if (fgets(buf, sizeof(buf), f)) {
            char* save = nullptr;
            for (char* tok = strtok_r(buf, ",\n", &save); tok; tok = strtok_r(nullptr, ",\n", &save)) {
                int a = 0, b = 0;
                const int n = sscanf(tok, "%d-%d", &a, &b);
                if (n == 1) b = a;
                for (int c = a; n >= 1 && c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, &all);
            }
        }
        fclose(f);
    }
    if (CPU_COUNT(&all) == 0) {
        for (int c = 0; c < std::min<int>(CPU_SETSIZE, (int)sysconf(_SC_NPROCESSORS_CONF)); ++c) CPU_SET(c, &all);
    }
    if (sched_setaffinity(0, sizeof(all), &all) != 0) return -1;
    const std::vector<int> cpus = l3_domain_cpus(k);
    if (cpus.empty()) return -1;
    set_cpu_order(cpus);
    confine_process(cpus);
    FLAGS_cpu_l3_domain = k;
    LOG(INFO) << "fiber runtime re-confined to L3 domain " << k << " (" << cpus.size() << " CPUs from "
              << cpus.front() << ")";
    return 0;
}

void* TaskControl::worker_thread(void* arg) {
    TaskControl* c = (TaskControl*)arg;
    TaskGroup* g = new TaskGroup(c);
    size_t cap = FLAGS_task_group_runqueue_capacity > 0 ? (size_t)FLAGS_task_group_runqueue_capacity : 4096;
    if (g->init(cap) != 0) {
        LOG(ERROR) << "fail to init TaskGroup";
        delete g;
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(c->_mu);
        int idx = c->_ngroup.load(std::memory_order_relaxed);
        g->_index = idx;
        g->_pl = &c->_pl[idx % kParkingLots];
        g->_last_pl_state = g->_pl->get_state();
        c->_groups[idx] = g;
        c->_ngroup.store(idx + 1, std::memory_order_release);
    }
    char name[32];
    snprintf(name, sizeof(name), "mrpc_worker%d", g->_index);
    pthread_setname_np(pthread_self(), name);
    if (FLAGS_fiber_worker_cpu_offset >= 0) {
        // a worker that never migrates keeps its run queue, stacks and the
        // sockets it serves hot in one core's caches; physical cores are
        // handed out before their SMT siblings
        const std::vector<int> order = cpu_order_by_core();
        if (!order.empty()) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(order[(size_t)(FLAGS_fiber_worker_cpu_offset + g->_index) % order.size()], &one);
            pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
        }
    }
    set_tls_group(g);
    g->run_main_task();
    set_tls_group(nullptr);
    return nullptr;
}

int TaskControl::init(int concurrency) {
    apply_process_affinity();
    if (concurrency <= 0) concurrency = 1;
    if (concurrency > kMaxConcurrency) concurrency = kMaxConcurrency;
    return add_workers(concurrency) > 0 ? 0 : -1;
}

int TaskControl::add_workers(int n) {
    std::unique_lock<std::mutex> lk(_mu);
    int added = 0;
    for (int i = 0; i < n && (int)_workers.size() < kMaxConcurrency; ++i) {
        pthread_t th;
        pthread_attr_t attr;
        pthread_attr_init(&attr);
        pthread_attr_setstacksize(&attr, 8 << 20);
        if (pthread_create(&th, &attr, worker_thread, this) != 0) {
            pthread_attr_destroy(&attr);
            break;
        }
        pthread_attr_destroy(&attr);
        _workers.push_back(th);
        ++added;
    }
    _concurrency.fetch_add(added, std::memory_order_release);
    lk.unlock();
    // Wait until all groups registered so steal/choose see them.
    const int target = _concurrency.load(std::memory_order_acquire);
    while (_ngroup.load(std::memory_order_acquire) < target) sched_yield();
    return added;
}

TaskGroup* TaskControl::choose_one_group() {
    const int n = _ngroup.load(std::memory_order_acquire);
    if (n <= 0) return nullptr;
    return _groups[fast_rand_less_than((uint64_t)n)];
}

bool TaskControl::steal_task(fiber_t* tid, uint64_t* seed, size_t offset) {
    const size_t ngroup = (size_t)_ngroup.load(std::memory_order_acquire);
    if (ngroup == 0) return false;
    size_t s = (size_t)(*seed);
    bool stolen = false;
    for (size_t i = 0; i < ngroup; ++i, s += (offset ? offset : 1)) {
        TaskGroup* g = _groups[s % ngroup];
        if (!g) continue;
        if (g->_rq.steal(tid)) {
            stolen = true;
            break;
        }
        if (g->_remote_size.load(std::memory_order_acquire) > 0) {
            std::lock_guard<std::mutex> lk(g->_remote_mu);
            if (!g->_remote_rq.empty()) {
                *tid = g->_remote_rq.front();
                g->_remote_rq.pop_front();
                g->_remote_size.fetch_sub(1, std::memory_order_relaxed);
                stolen = true;
                break;
            }
        }
    }
    *seed = s + 1;
    if (stolen) nsteal.fetch_add(1, std::memory_order_relaxed);
    return stolen;
}

void TaskControl::signal_task(int num_task) {
    if (num_task <= 0) return;
    if (num_task > 2) num_task = 2;
    // A spinning worker will take the task: no FUTEX_WAKE. Without this
    // every start_background() while any worker is parked paid a wake
    // syscall (~1.5-2 us here, build/bin/mrpc_microbench fiber_create vs
    // fiber_create_nosignal) and the woken worker parked again after one
    // short fiber. Dekker pair, both sides seq_cst: bump every lot, then
    // read the spinner count; a spinner drops out of the count, then parks
    // on a snapshot taken before its last failed steal. Either we see it
    // spinning (then the bump precedes its futex compare, which fails), or
    // it had left the count and we wake as usual.
    if (FLAGS_fiber_idle_spin_us > 0 && FLAGS_fiber_signal_skip_when_spinning) {
        for (int i = 0; i < kParkingLots; ++i) _pl[i].bump();
        if (g_spinning_workers.load(std::memory_order_seq_cst) > 0) return;
    }
    int start = (int)(fast_rand_less_than(kParkingLots));
    for (int i = 0; i < kParkingLots && num_task > 0; ++i) {
        num_task -= _pl[(start + i) % kParkingLots].signal(1);
    }
    if (num_task > 0 && FLAGS_fiber_min_concurrency > 0 &&
        _concurrency.load(std::memory_order_relaxed) < FLAGS_fiber_concurrency) {
        std::unique_lock<std::mutex> lk(_mu, std::try_to_lock);
        if (lk.owns_lock() && _concurrency.load(std::memory_order_relaxed) < FLAGS_fiber_concurrency) {
            lk.unlock();
            add_workers(1);
        }
    }
}

void TaskControl::stop_and_join() {
    {
        std::lock_guard<std::mutex> lk(_mu);
        if (_stop) return;
        _stop = true;
    }
    for (int i = 0; i < kParkingLots; ++i) _pl[i].stop();
    // workers blocked in a system call of user code: EINTR, so they reach
    // the stop check (reference task_control.cpp:244-247)
    for (pthread_t t : _workers) interrupt_pthread(t);
    for (pthread_t t : _workers) pthread_join(t, nullptr);
}

int64_t TaskControl::total_switch() const {
    int64_t s = 0;
    const int n = _ngroup.load(std::memory_order_acquire);
    for (int i = 0; i < n; ++i) {
        if (_groups[i]) s += _groups[i]->nswitch();
    }
    return s;
}

int64_t TaskControl::total_idle_ns() const {
    int64_t s = 0;
    const int n = _ngroup.load(std::memory_order_acquire);
    for (int i = 0; i < n; ++i) {
        if (_groups[i]) s += _groups[i]->idle_ns();
    }
    return s;
}

void ready_to_run_general(fiber_t tid, bool nosignal) {
    TaskGroup* g = tls_group();
    if (g) {
        g->ready_to_run(tid, nosignal);
        return;
    }
    TaskControl* c = get_or_new_task_control();
    c->choose_one_group()->ready_to_run_remote(tid, nosignal);
}

// ------------------------------------------------------------------ public API
int init_runtime() {
    get_or_new_task_control();
    return 0;
}

static int start_from_non_worker(fiber_t* tid, const Attr* attr, FiberFn fn, void* arg) {
    TaskControl* c = get_or_new_task_control();
    TaskGroup* g = c->choose_one_group();
    if (!g) return EAGAIN;
    return g->start_background<true>(tid, attr, fn, arg);
}

int start_urgent(fiber_t* tid, const Attr* attr, FiberFn fn, void* arg) {
    fiber_t dummy;
    if (!tid) tid = &dummy;
    TaskGroup* g = tls_group();
    if (g) return TaskGroup::start_foreground(&g, tid, attr, fn, arg);
    return start_from_non_worker(tid, attr, fn, arg);
}

int start_background(fiber_t* tid, const Attr* attr, FiberFn fn, void* arg) {
    fiber_t dummy;
    if (!tid) tid = &dummy;
    TaskGroup* g = tls_group();
    if (g) return g->start_background<false>(tid, attr, fn, arg);
    return start_from_non_worker(tid, attr, fn, arg);
}

static void* run_std_function(void* arg) {
    std::function<void()>* f = (std::function<void()>*)arg;
    (*f)();
    delete f;
    return nullptr;
}

int start(std::function<void()> fn, bool urgent, const Attr* attr, fiber_t* tid) {
    auto* f = new std::function<void()>(std::move(fn));
    int rc = urgent ? start_urgent(tid, attr, run_std_function, f) : start_background(tid, attr, run_std_function, f);
    if (rc != 0) delete f;
    return rc;
}

void flush() {
    TaskGroup* g = tls_group();
    if (g) {
        g->flush_nosignal_tasks();
        return;
    }
    TaskControl* c = get_task_control();
    if (!c) return;
    // Non-worker threads queue into random groups; flush them all.
    c->signal_task(2);
}

int join(fiber_t tid, void** ret) {
    if (ret) *ret = nullptr;
    if (tid == INVALID_FIBER) return EINVAL;
    TaskMeta* m = address_meta(tid);
    if (!m || !m->version_butex) return EINVAL;
    TaskGroup* g = tls_group();
    if (g && g->current_tid() == tid) return EINVAL;
    const int expected = (int)tid_version(tid);
    while (m->version_butex->load(std::memory_order_acquire) == expected) {
        if (butex_wait(m->version_butex, expected, nullptr) < 0 && errno != EWOULDBLOCK && errno != EINTR) {
            return errno;
        }
    }
    return 0;
}

bool exists(fiber_t tid) {
    TaskMeta* m = address_meta(tid);
    return m && m->version_butex && (uint32_t)m->version_butex->load(std::memory_order_acquire) == tid_version(tid);
}

int stop(fiber_t tid) {
    TaskMeta* m = address_meta(tid);
    if (!m) return EINVAL;
    {
        std::lock_guard<std::mutex> lk(m->version_lock);
        if ((uint32_t)m->version_butex->load(std::memory_order_relaxed) != tid_version(tid)) return EINVAL;
        m->stop = true;
    }
    return TaskGroup::interrupt(tid, get_task_control());
}

bool stopped(fiber_t tid) {
    TaskMeta* m = address_meta(tid);
    if (!m) return true;
    std::lock_guard<std::mutex> lk(m->version_lock);
    if ((uint32_t)m->version_butex->load(std::memory_order_relaxed) != tid_version(tid)) return true;
    return m->stop;
}

int interrupt(fiber_t tid) { return TaskGroup::interrupt(tid, get_task_control()); }

int yield() {
    TaskGroup* g = tls_group();
    if (g && !g->is_current_main_task()) {
        TaskGroup::yield(&g);
        return 0;
    }
    return sched_yield();
}

int usleep(uint64_t us) {
    TaskGroup* g = tls_group();
    if (g && !g->is_current_main_task()) return TaskGroup::usleep(&g, us);
    return ::usleep((useconds_t)us);
}

fiber_t self() {
    TaskGroup* g = tls_group();
    if (!g || g->is_current_main_task()) return INVALID_FIBER;
    return g->current_tid();
}

bool in_fiber() {
    TaskGroup* g = tls_group();
    return g && !g->is_current_main_task();
}

int worker_index() {
    TaskGroup* g = tls_group();
    return g ? g->index() : -1;
}

int set_concurrency(int n) {
    if (n <= 0 || n > TaskControl::kMaxConcurrency) return EINVAL;
    TaskControl* c = get_task_control();
    if (!c) {
        FLAGS_fiber_concurrency = n;
        return 0;
    }
    int cur = c->concurrency();
    if (n < cur) return EPERM;
    FLAGS_fiber_concurrency = n;
    if (n > cur) c->add_workers(n - cur);
    return 0;
}

int get_concurrency() {
    TaskControl* c = get_task_control();
    return c ? c->concurrency() : FLAGS_fiber_concurrency;
}

static std::atomic<bool> g_about_to_quit{false};
void about_to_quit() { g_about_to_quit.store(true); }

// Best-effort listing for debuggers (/fibers, gdb helper): it reads the
// metadata of fibers that keep running, so the values are a racy snapshot
// by design and ThreadSanitizer is told not to instrument the reads.
__attribute__((no_sanitize("thread"))) static void describe_one(const TaskMeta* m, int64_t now, std::string* out) {
    char line[160];
    snprintf(line, sizeof(line), "tid=%llu fn=%p arg=%p sp=%p stack=%p age_ms=%lld\n", (unsigned long long)m->tid,
             (void*)m->fn, m->arg, m->sp, (void*)m->stack, (long long)((now - m->start_ns) / 1000000));
    *out += line;
}

__attribute__((no_sanitize("thread"))) static bool is_listed(const TaskMeta* m) {
    return m->version_butex && !m->is_main && m->fn &&
           (uint32_t)m->version_butex->load(std::memory_order_acquire) == tid_version(m->tid);
}

std::string DescribeFibers(size_t max_lines) {
    std::string out;
    size_t n = 0;
    const int64_t now = monotonic_ns();
    ResourcePool<TaskMeta>::singleton()->for_each([&](uint32_t, TaskMeta* m) {
        if (n >= max_lines || !is_listed(m)) return;
        ++n;
        describe_one(m, now, &out);
    });
    return out;
}

int64_t fiber_count() {
    TaskControl* c = get_task_control();
    return c ? c->nfibers.load(std::memory_order_relaxed) : 0;
}
int64_t switch_count() {
    TaskControl* c = get_task_control();
    return c ? c->total_switch() : 0;
}
int64_t steal_count() {
    TaskControl* c = get_task_control();
    return c ? c->nsteal.load(std::memory_order_relaxed) : 0;
}
double worker_usage() {
    // Average busy workers since the previous call (process-wide sampler).
    static std::mutex mu;
    static int64_t last_idle = 0, last_t = 0;
    TaskControl* c = get_task_control();
    if (!c) return 0;
    std::lock_guard<std::mutex> lk(mu);
    int64_t now = monotonic_ns();
    int64_t idle = c->total_idle_ns();
    if (last_t == 0) {
        last_t = c->start_ns;
    }
    int64_t dt = now - last_t;
    double usage = dt > 0 ? c->concurrency() - (double)(idle - last_idle) / (double)dt : 0;
    last_idle = idle;
    last_t = now;
    return usage < 0 ? 0 : usage;
}

// ------------------------------------------------------------------ timers
int timer_add(TimerId* id, const timespec& abstime, void (*fn)(void*), void* arg) {
    TimerThread::TaskId t = get_global_timer_thread()->schedule(fn, arg, abstime);
    if (!t) return ESTOP;
    if (id) *id = t;
    return 0;
}

int timer_add_us(TimerId* id, int64_t delay_us, void (*fn)(void*), void* arg) {
    TimerThread::TaskId t = get_global_timer_thread()->schedule_after_us(fn, arg, delay_us);
    if (!t) return ESTOP;
    if (id) *id = t;
    return 0;
}

int timer_del(TimerId id) {
    int rc = get_global_timer_thread()->unschedule(id);
    if (rc == -2) return -1;
    return rc == 0 ? 0 : 1;
}

}  // namespace fiber
}  // namespace mrpc

// For debuggers (tools/gdb_fiber_stack.py): `call mrpc_fiber_dump()` returns
// the live fibers with their saved stack pointers, which the gdb commands
// turn back into frames (see fiber/context.cc for the saved layout).
extern "C" const char* mrpc_fiber_dump() {
    static std::string* s = new std::string;
    *s = mrpc::fiber::DescribeFibers(100000);
    return s->c_str();
}
