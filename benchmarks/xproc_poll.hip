// The bench's completion pattern, without the framework: launcher threads
// issue copy kernels round-robin on S streams and record an event; ONE
// poller thread watches every pending event with hipEventQuery. Each copy
// kernel's last workgroup also stores a per-op sequence number into pinned
// host memory (system scope), so for every op we know when the kernel was
// really done (the word) and when hipEventQuery first said so.
//
//   build/bin/xproc_poll NPROC [threads] [streams] [iters] [bytes] [ipc] [arena_mb] [bigargs] [mrpc]
//
// mrpc=1: the copies are the framework's own launches (gpu::LaunchBatchedCopy
// with a DoneWord, libmrpc.so) instead of this file's kernel.
// arena_mb > 0: sources are carved from ONE hipMalloc of that size per
// process (the framework's IPC arena), and ipc imports the peer's whole
// arena. bigargs=1: the kernel also takes a 1.6 KB by-value argument (the
// size of the framework's inline segment table).
// ipc=1: process r's kernels read the source buffers of process (r+1) % NPROC
// (exported with hipIpcGetMemHandle, opened with hipIpcOpenMemHandle), the
// bench's cross-process pull.
// NPROC processes are forked before any HIP call. Each prints: ops,
// launch->word p50/p99, launch->event p50/p99 (us).
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "gpu/kernels.h"

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            _exit(2);                                                                          \
        }                                                                                      \
    } while (0)

struct BigArgs {
    unsigned long long pad[200];
};

__global__ void copy_done_big(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16, unsigned* counter,
                              unsigned long long* word, unsigned long long seq, BigArgs big) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
    if (big.pad[blockIdx.x % 200] == 12345) dst[0] = src[1];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned prev = atomicAdd(counter, 1u);
        if (prev == gridDim.x - 1) {
            *counter = 0;
            __threadfence_system();
            __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ void copy_done(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16, unsigned* counter,
                          unsigned long long* word, unsigned long long seq) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned prev = atomicAdd(counter, 1u);
        if (prev == gridDim.x - 1) {
            *counter = 0;
            __threadfence_system();
            __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Op {
    hipEvent_t ev;
    double t_launch = 0, t_word = 0, t_event = 0;
    std::atomic<int> done{0};
    int slot = 0;
    unsigned long long seq = 0;
};

// shared (MAP_SHARED, set up before fork) mailbox for the IPC handles
struct Mailbox {
    std::atomic<int> published;
    std::atomic<int> opened;
    hipIpcMemHandle_t h[16][16];
};
static Mailbox* g_box = nullptr;

static void run(int threads, int nstreams, int iters, size_t bytes, int rank, int nproc, bool ipc, size_t arena_mb,
                bool bigargs, bool mrpc) {
    std::vector<hipStream_t> streams(nstreams);
    for (auto& s : streams) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int nslots = threads;
    unsigned long long* words = nullptr;
    CHECK(hipHostMalloc((void**)&words, sizeof(unsigned long long) * 4 * nslots, hipHostMallocCoherent | hipHostMallocMapped));
    memset(words, 0, sizeof(unsigned long long) * 4 * nslots);  // [word, stamps...] per slot
    unsigned* counters = nullptr;
    CHECK(hipMalloc((void**)&counters, sizeof(unsigned) * nslots));
    CHECK(hipMemset(counters, 0, sizeof(unsigned) * nslots));
    std::vector<void*> src(threads), dst(threads);
    char* arena = nullptr;
    if (arena_mb) CHECK(hipMalloc((void**)&arena, arena_mb << 20));
    for (int t = 0; t < threads; ++t) {
        if (arena) src[t] = arena + (size_t)t * (8u << 20);
        else CHECK(hipMalloc(&src[t], bytes));
        CHECK(hipMalloc(&dst[t], bytes));
    }
    CHECK(hipDeviceSynchronize());
    if (ipc && arena) {
        CHECK(hipIpcGetMemHandle(&g_box->h[rank][0], arena));
        g_box->published.fetch_add(1);
        while (g_box->published.load() < nproc) std::this_thread::yield();
        void* peer_arena = nullptr;
        CHECK(hipIpcOpenMemHandle(&peer_arena, g_box->h[(rank + 1) % nproc][0], hipIpcMemLazyEnablePeerAccess));
        for (int t = 0; t < threads; ++t) src[t] = static_cast<char*>(peer_arena) + (size_t)t * (8u << 20);
        g_box->opened.fetch_add(1);
        while (g_box->opened.load() < nproc) std::this_thread::yield();
    } else if (ipc) {
        for (int t = 0; t < threads; ++t) CHECK(hipIpcGetMemHandle(&g_box->h[rank][t], src[t]));
        g_box->published.fetch_add(1);
        while (g_box->published.load() < nproc) std::this_thread::yield();
        const int peer = (rank + 1) % nproc;
        for (int t = 0; t < threads; ++t) CHECK(hipIpcOpenMemHandle(&src[t], g_box->h[peer][t], hipIpcMemLazyEnablePeerAccess));
        g_box->opened.fetch_add(1);
        while (g_box->opened.load() < nproc) std::this_thread::yield();
    }
    std::mutex mu;
    std::vector<Op*> pending;
    std::atomic<bool> stop{false};
    std::thread poller([&] {
        std::vector<Op*> act;
        while (!stop.load()) {
            {
                std::lock_guard<std::mutex> g(mu);
                act.insert(act.end(), pending.begin(), pending.end());
                pending.clear();
            }
            size_t keep = 0;
            for (Op* o : act) {
                if (!o->t_word && __atomic_load_n(&words[4 * o->slot], __ATOMIC_ACQUIRE) == o->seq) o->t_word = now_us();
                const hipError_t r = hipEventQuery(o->ev);
                if (r == hipErrorNotReady) {
                    act[keep++] = o;
                    continue;
                }
                o->t_event = now_us();
                if (!o->t_word) o->t_word = o->t_event;
                o->done.store(1, std::memory_order_release);
            }
            act.resize(keep);
        }
    });
    std::vector<double> lw, le;
    std::mutex rmu;
    std::vector<std::thread> ths;
    const double t0 = now_us();
    for (int t = 0; t < threads; ++t) {
        ths.emplace_back([&, t] {
            Op o;
            CHECK(hipEventCreateWithFlags(&o.ev, hipEventDisableTiming));
            o.slot = t;
            const size_t n16 = bytes / 16;
            const int blocks = (int)std::min<size_t>(1024, (n16 + 255) / 256);
            std::vector<double> w, e;
            for (int i = 0; i < iters; ++i) {
                o.seq = ((unsigned long long)rank << 48) | ((unsigned long long)t << 32) | (unsigned)(i + 1);
                o.t_word = o.t_event = 0;
                o.done.store(0);
                hipStream_t s = streams[(t + i) % nstreams];
                o.t_launch = now_us();
                if (mrpc) {
                    mrpc::gpu::Segment seg{src[t], dst[t], bytes};
                    mrpc::gpu::DoneWord dw;
                    dw.counter = counters + t;
                    dw.word = reinterpret_cast<uint64_t*>(words + 4 * t);
                    dw.seq = o.seq;
                    if (mrpc::gpu::LaunchBatchedCopy(&seg, 1, s, &dw) != 0) _exit(5);
                } else if (bigargs) {
                    BigArgs big;
                    memset(&big, 0, sizeof(big));
                    hipLaunchKernelGGL(copy_done_big, dim3(blocks), dim3(256), 0, s, (const uint4*)src[t], (uint4*)dst[t],
                                       n16, counters + t, words + 4 * t, o.seq, big);
                } else {
                    hipLaunchKernelGGL(copy_done, dim3(blocks), dim3(256), 0, s, (const uint4*)src[t], (uint4*)dst[t],
                                       n16, counters + t, words + 4 * t, o.seq);
                }
                CHECK(hipEventRecord(o.ev, s));
                {
                    std::lock_guard<std::mutex> g(mu);
                    pending.push_back(&o);
                }
                while (!o.done.load(std::memory_order_acquire)) std::this_thread::yield();
                if (i >= 20) {
                    w.push_back(o.t_word - o.t_launch);
                    e.push_back(o.t_event - o.t_launch);
                }
            }
            std::lock_guard<std::mutex> g(rmu);
            lw.insert(lw.end(), w.begin(), w.end());
            le.insert(le.end(), e.begin(), e.end());
        });
    }
    for (auto& th : ths) th.join();
    const double dt = now_us() - t0;
    stop.store(true);
    poller.join();
    std::sort(lw.begin(), lw.end());
    std::sort(le.begin(), le.end());
    printf("rank %d: threads=%d streams=%d ops=%zu %.0f ops/s | launch->word p50=%.1f p99=%.1f | "
           "launch->event p50=%.1f p99=%.1f us\n",
           rank, threads, nstreams, le.size(), le.size() / dt * 1e6, lw[lw.size() / 2], lw[lw.size() * 99 / 100],
           le[le.size() / 2], le[le.size() * 99 / 100]);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int nproc = argc > 1 ? atoi(argv[1]) : 1;
    const int threads = argc > 2 ? atoi(argv[2]) : 8;
    const int nstreams = argc > 3 ? atoi(argv[3]) : 4;
    const int iters = argc > 4 ? atoi(argv[4]) : 2000;
    const size_t bytes = argc > 5 ? (size_t)atoll(argv[5]) : 65536;
    const bool ipc = argc > 6 && atoi(argv[6]) != 0;
    const size_t arena_mb = argc > 7 ? (size_t)atoll(argv[7]) : 0;
    const bool bigargs = argc > 8 && atoi(argv[8]) != 0;
    const bool mrpc = argc > 9 && atoi(argv[9]) != 0;
    if (nproc > 16 || threads > 16) return 1;
    g_box = static_cast<Mailbox*>(mmap(nullptr, sizeof(Mailbox), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
    if (g_box == MAP_FAILED) return 1;
    std::vector<pid_t> kids;
    for (int r = 1; r < nproc; ++r) {
        const pid_t p = fork();
        if (p == 0) {
            run(threads, nstreams, iters, bytes, r, nproc, ipc, arena_mb, bigargs, mrpc);
            _exit(0);
        }
        kids.push_back(p);
    }
    run(threads, nstreams, iters, bytes, 0, nproc, ipc, arena_mb, bigargs, mrpc);
    int bad = 0;
    for (pid_t p : kids) {
        int st = 0;
        waitpid(p, &st, 0);
        bad |= !WIFEXITED(st) || WEXITSTATUS(st) != 0;
    }
    return bad ? 4 : 0;
}
