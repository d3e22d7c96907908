// Launch-to-completion latency of a small copy kernel, alone and with a
// second process on the same GPU (the cross-process device
// path spends ~590 us per pull between hipEventRecord and the poller seeing
// the event, against 13 us in one process).
//
//   hipcc --offload-arch=gfx950 -O2 benchmarks/xproc_latency.hip -o build/bin/xproc_latency
//   build/bin/xproc_latency MODE [iters] [bytes]
//
// MODE:
//   solo      one process
//   pair      two processes, both running the loop at once
//   idle      two processes; the second only holds a context and a stream
//   ipc       the first reads a buffer the second exported (hipIpcGetMemHandle);
//             the second idles
//   ipc_busy  as ipc, and the second runs the loop on its own buffers
//
// The processes are forked BEFORE any HIP call; each prints one line:
// role, mode, p50 / p99 / mean microseconds from launch to hipEventQuery
// success (polled without sleeping).
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            _exit(2);                                                                          \
        }                                                                                      \
    } while (0)

__global__ void copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void loop(const char* role, const char* mode, const void* src, void* dst, size_t bytes, int iters) {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::vector<double> lat;
    lat.reserve(iters);
    const size_t n16 = bytes / 16;
    const int blocks = (int)std::min<size_t>(1024, (n16 + 255) / 256);
    for (int i = 0; i < iters + 50; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16);
        CHECK(hipEventRecord(ev, s));
        hipError_t r;
        while ((r = hipEventQuery(ev)) == hipErrorNotReady) {
        }
        CHECK(r);
        if (i >= 50) lat.push_back(now_us() - t0);
    }
    std::sort(lat.begin(), lat.end());
    double sum = 0;
    for (double v : lat) sum += v;
    printf("%-8s %-9s bytes=%zu iters=%d p50=%.1f p99=%.1f mean=%.1f max=%.1f us\n", role, mode, bytes, iters,
           lat[lat.size() / 2], lat[lat.size() * 99 / 100], sum / lat.size(), lat.back());
    fflush(stdout);
    hipEventDestroy(ev);
    hipStreamDestroy(s);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s solo|pair|idle|ipc|ipc_busy [iters] [bytes]\n", argv[0]);
        return 1;
    }
    const char* mode = argv[1];
    const int iters = argc > 2 ? atoi(argv[2]) : 2000;
    const size_t bytes = argc > 3 ? (size_t)atoll(argv[3]) : 65536;
    const bool two = strcmp(mode, "solo") != 0;
    const bool ipc = strncmp(mode, "ipc", 3) == 0;
    const bool peer_busy = !strcmp(mode, "pair") || !strcmp(mode, "ipc_busy");
    int to_first[2], to_second[2];  // handle / "ready" to the first; "done" to the second
    if (pipe(to_first) != 0 || pipe(to_second) != 0) return 1;
    pid_t child = -1;
    if (two) child = fork();
    if (two && child == 0) {
        // second process
        void *a = nullptr, *b = nullptr;
        CHECK(hipMalloc(&a, bytes));
        CHECK(hipMalloc(&b, bytes));
        CHECK(hipMemset(a, 1, bytes));
        hipStream_t s;
        CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipIpcMemHandle_t h;
        memset(&h, 0, sizeof(h));
        if (ipc) CHECK(hipIpcGetMemHandle(&h, a));
        CHECK(hipDeviceSynchronize());
        if (write(to_first[1], &h, sizeof(h)) != (ssize_t)sizeof(h)) _exit(3);
        if (peer_busy) loop("second", mode, a, b, bytes, iters * 2);
        char c;
        if (read(to_second[0], &c, 1) != 1) _exit(3);
        hipStreamDestroy(s);
        _exit(0);
    }
    hipIpcMemHandle_t h;
    if (two && read(to_first[0], &h, sizeof(h)) != (ssize_t)sizeof(h)) return 3;
    void *src = nullptr, *dst = nullptr;
    CHECK(hipMalloc(&dst, bytes));
    if (ipc) {
        CHECK(hipIpcOpenMemHandle(&src, h, hipIpcMemLazyEnablePeerAccess));
    } else {
        CHECK(hipMalloc(&src, bytes));
        CHECK(hipMemset(src, 1, bytes));
    }
    CHECK(hipDeviceSynchronize());
    loop("first", mode, src, dst, bytes, iters);
    if (ipc) CHECK(hipIpcCloseMemHandle(src));
    if (two) {
        char c = 1;
        if (write(to_second[1], &c, 1) != 1) return 3;
        int st = 0;
        waitpid(child, &st, 0);
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
            fprintf(stderr, "second process failed (%d)\n", st);
            return 4;
        }
    }
    return 0;
}
