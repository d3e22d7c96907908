#include "rpc/usercode_backup_pool.h"

#include <pthread.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

#include "base/logging.h"
#include "fiber/fiber.h"
#include "var/var.h"

DEFINE_bool(usercode_in_pthread, false,
            "user callbacks may block their pthread: keep some workers free by moving excess to backup pthreads");
DEFINE_int32(usercode_backup_threads, 5, "pthreads running user code that does not fit in place");
DEFINE_int32(max_pending_in_each_backup_thread, 10, "queued user code per backup thread before ELIMIT");

namespace mrpc {

namespace {
struct UserCode {
    void (*fn)(void*);
    void* arg;
};

struct BackupPool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<UserCode> queue;
    std::atomic<bool> too_many{false};
    var::Adder<int64_t> count;
    std::unique_ptr<var::PerSecond<var::Adder<int64_t>>> per_second;

    BackupPool() {
        count.expose("rpc_usercode_backup_count");
        per_second.reset(new var::PerSecond<var::Adder<int64_t>>("rpc_usercode_backup_second", &count));
        for (int i = 0; i < FLAGS_usercode_backup_threads; ++i) {
            std::thread([this] { Loop(); }).detach();  // like fiber workers, never quit
        }
    }
    void Loop() {
        pthread_setname_np(pthread_self(), "mrpc_usercode");
        for (;;) {
            UserCode uc;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [this] { return !queue.empty(); });
                uc = queue.front();
                queue.pop_front();
                if (too_many.load(std::memory_order_relaxed) && (int)queue.size() <= FLAGS_usercode_backup_threads) {
                    too_many.store(false, std::memory_order_relaxed);
                }
            }
            uc.fn(uc.arg);
            count << 1;
        }
    }
};

std::atomic<int> g_inplace{0};
BackupPool* g_pool = nullptr;
std::once_flag g_pool_once;

BackupPool* pool() {
    std::call_once(g_pool_once, [] { g_pool = new BackupPool; });
    return g_pool;
}
}  // namespace

bool BeginRunningUserCode() {
    const int limit = std::max(1, fiber::get_concurrency() - FLAGS_usercode_backup_threads);
    const int n = g_inplace.fetch_add(1, std::memory_order_relaxed) + 1;
    return n <= limit;
}

void EndRunningUserCodeInPlace() { g_inplace.fetch_sub(1, std::memory_order_relaxed); }

void EndRunningUserCodeInPool(void (*fn)(void*), void* arg) {
    BackupPool* p = pool();
    g_inplace.fetch_sub(1, std::memory_order_relaxed);
    {
        std::lock_guard<std::mutex> g(p->mu);
        p->queue.push_back(UserCode{fn, arg});
        if ((int64_t)p->queue.size() >
            (int64_t)FLAGS_usercode_backup_threads * FLAGS_max_pending_in_each_backup_thread) {
            p->too_many.store(true, std::memory_order_relaxed);
        }
    }
    p->cv.notify_one();
}

bool TooManyUserCode() { return g_pool && g_pool->too_many.load(std::memory_order_relaxed); }

void RunUserCode(void (*fn)(void*), void* arg) {
    if (!FLAGS_usercode_in_pthread) {
        fn(arg);
        return;
    }
    if (BeginRunningUserCode()) {
        fn(arg);
        EndRunningUserCodeInPlace();
    } else {
        EndRunningUserCodeInPool(fn, arg);
    }
}

int64_t UserCodeInPlaceCount() { return g_inplace.load(std::memory_order_relaxed); }

int64_t UserCodeQueueSize() {
    if (!g_pool) return 0;
    std::lock_guard<std::mutex> g(g_pool->mu);
    return (int64_t)g_pool->queue.size();
}

}  // namespace mrpc
