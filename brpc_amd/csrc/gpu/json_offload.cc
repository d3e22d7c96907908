// Device half of json2pb for large bodies (the reference parses
// every http+json body on the CPU, src/json2pb/json_to_pb.cpp): the body is
// copied into a pinned buffer, LaunchJsonIndex (gpu/json_kernels.hip) reads
// it there and writes every structural position straight into pinned
// memory, and json::ParseWithIndex walks the positions: one launch and one
// fiber-friendly wait per body. (-json_index_direct_host=false keeps the
// older staging through HBM: a copy kernel in, the index, a second wait for
// the count, a copy of count * 4 bytes back.)
#include "gpu/json_offload.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstring>

#include "base/flags.h"
#include "base/time.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"
#include "gpu/snappy_offload.h"
#include "json/json2pb.h"
#include "rpc/span.h"
#include "var/var.h"

DEFINE_int32(gpu_pb2json_min_elems, 4096,
             "repeated integer/bool fields with at least this many elements are printed by the device in pb2json "
             "(pb_run_encode_kernel, decimal format) and integer arrays of at least as many elements are parsed by "
             "json_int_array_kernel in json2pb, while the GPU JSON path is enabled");
DEFINE_int32(json_index_min_density, 8,
             "structural characters per KiB (sampled in three windows) a JSON body needs before the GPU index is "
             "used; sparser bodies (long strings) parse faster on the host; 0: always offload");
DEFINE_bool(json_index_direct_host, true,
            "the JSON index kernel reads the pinned body and writes positions to pinned memory directly");

namespace mrpc {
namespace gpu {

namespace {

int g_device = -1;
std::atomic<int64_t> g_bodies{0}, g_bytes{0}, g_failures{0};
std::atomic<int64_t> g_sparse{0};

struct Hbm {
    void* p = nullptr;
    size_t n = 0;
    int dev = -1;
    Hbm(size_t bytes, int d) : p(HbmAlloc(bytes, d)), n(bytes), dev(d) {}
    ~Hbm() {
        if (p) HbmFree(p, n, dev);
    }
};

struct Pinned {
    void* p = nullptr;
    size_t n = 0;
    explicit Pinned(size_t bytes) : p(PinnedAlloc(bytes)), n(bytes) {}
    ~Pinned() {
        if (p) PinnedFree(p, n);
    }
};

// Structural characters per KiB in three 1 KiB windows (start, middle,
// end). A body that is mostly one long string (the http_json_64KB leg)
// has almost none: the host parser crosses it with memchr faster than a
// device round trip returns its index, so such bodies are not offloaded.
bool structurally_sparse(const char* data, size_t n) {
    const int need = FLAGS_json_index_min_density;
    if (need <= 0 || n < 3 * 1024) return false;
    int hits = 0;
    for (size_t w : {(size_t)0, n / 2 - 512, n - 1024}) {
        for (size_t i = w; i < w + 1024; ++i) {
            const char c = data[i];
            hits += c == '"' || c == ',' || c == ':' || c == '{' || c == '[';
        }
    }
    return hits < 3 * need;
}

bool offload(const char* data, size_t n, std::vector<uint32_t>* index) {
    if (g_device < 0) return false;
    if (structurally_sparse(data, n)) {
        g_sparse.fetch_add(1, std::memory_order_relaxed);
        return false;
    }
    Span* span = IsRpczEnabled() ? Span::tls_parent() : nullptr;
    const int64_t t0 = span ? monotonic_us() : 0;
    const int rc = JsonIndex(data, n, index, g_device);
    if (rc != 0) {
        g_failures.fetch_add(1, std::memory_order_relaxed);
        return false;  // malformed or no device: the CPU parser reports it
    }
    g_bodies.fetch_add(1, std::memory_order_relaxed);
    g_bytes.fetch_add((int64_t)n, std::memory_order_relaxed);
    if (span) {
        span->AnnotateDevice(string_printf("json index %zu B -> %zu positions dev%d", n, index->size(), g_device),
                             (float)(monotonic_us() - t0) / 1000.0f);
    }
    return true;
}

}  // namespace

int JsonIndex(const char* data, size_t n, std::vector<uint32_t>* out, int device) {
    out->clear();
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFull || device < 0) return -1;
    if (FLAGS_json_index_direct_host) {
        Pinned body(n), pos(n * sizeof(uint32_t)), meta(16);  // every byte could be a position
        Hbm scratch(JsonIndexScratchBytes(n), device);
        if (!body.p || !pos.p || !meta.p || !scratch.p) return -1;
        memcpy(body.p, data, n);
        uint64_t* count = static_cast<uint64_t*>(meta.p);
        int* err = reinterpret_cast<int*>(count + 1);
        int prev = 0;
        hipGetDevice(&prev);
        if (prev != device) hipSetDevice(device);
        hipStream_t s = PoolStream(device);
        int rc = s ? LaunchJsonIndex(static_cast<const uint8_t*>(body.p), n, static_cast<uint32_t*>(pos.p), n, count,
                                     err, scratch.p, s)
                   : -1;
        const int wrc = s ? SyncStream(s) : -1;  // never free buffers a launched kernel may still use
        if (prev != device) hipSetDevice(prev);
        if (rc != 0 || wrc != 0 || *err != 0 || *count > n) return -1;
        const uint32_t* p = static_cast<const uint32_t*>(pos.p);
        out->assign(p, p + *count);
        return 0;
    }
    // every byte could be a position; the count decides what comes back
    Hbm in(n, device), pos(n * sizeof(uint32_t), device), scratch(JsonIndexScratchBytes(n), device);
    Pinned bounce(n), meta(16);
    if (!in.p || !pos.p || !scratch.p || !bounce.p || !meta.p) return -1;
    memcpy(bounce.p, data, n);
    uint64_t* count = static_cast<uint64_t*>(meta.p);
    int* err = reinterpret_cast<int*>(count + 1);
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    hipStream_t s = PoolStream(device);
    int rc = -1;
    if (s) {
        Segment seg{bounce.p, in.p, n};
        rc = LaunchBatchedCopy(&seg, 1, s);
        if (rc == 0) {
            rc = LaunchJsonIndex(static_cast<const uint8_t*>(in.p), n, static_cast<uint32_t*>(pos.p), n, count, err,
                                 scratch.p, s);
        }
        const int wrc = SyncStream(s);  // never free buffers a launched kernel may still use
        if (rc == 0) rc = wrc;
        if (rc == 0 && *err != 0) rc = -1;
        if (rc == 0 && *count > 0) {
            const size_t bytes = (size_t)*count * sizeof(uint32_t);
            Pinned back(bytes);
            if (!back.p) {
                rc = -1;
            } else {
                Segment seg2{pos.p, back.p, bytes};
                rc = LaunchBatchedCopy(&seg2, 1, s);
                const int w2 = SyncStream(s);
                if (rc == 0) rc = w2;
                if (rc == 0) {
                    const uint32_t* p = static_cast<const uint32_t*>(back.p);
                    out->assign(p, p + *count);
                }
            }
        }
    }
    if (prev != device) hipSetDevice(prev);
    return rc == 0 ? 0 : -1;
}

namespace {

std::atomic<int64_t> g_arrays{0}, g_array_elems{0}, g_array_failures{0};

// pb2json number arrays: pb_run_encode_kernel prints the
// field's values in the codec batch (gpu/snappy_offload.h
// EncodeRunOnDevice), the host only sizes them and wraps the brackets.
bool array_offload(const void* values, size_t n, uint32_t kind, std::string* text) {
    const int dev = g_device;
    if (dev < 0) return false;
    if (EncodeRunOnDevice(values, n, kind, PB_RUN_DECIMAL, text, dev) != 0) {
        g_array_failures.fetch_add(1, std::memory_order_relaxed);
        return false;
    }
    g_arrays.fetch_add(1, std::memory_order_relaxed);
    g_array_elems.fetch_add((int64_t)n, std::memory_order_relaxed);
    return true;
}

std::atomic<int64_t> g_int_arrays{0}, g_int_array_fallbacks{0};

struct PinnedTmp {
    void* p = nullptr;
    size_t n = 0;
    explicit PinnedTmp(size_t bytes) : p(PinnedAlloc(bytes)), n(bytes) {}
    ~PinnedTmp() {
        if (p) PinnedFree(p, n);
    }
};

// json2pb integer arrays (SURVEY K6 parse half): the array's text and its
// separators go to pinned memory, json_int_array_kernel parses one element
// per lane, one fiber-friendly wait.
bool int_array_offload(const char* base, const uint32_t* seps, size_t nseps, std::vector<int64_t>* out) {
    const int dev = g_device;
    if (dev < 0 || nseps < 2) return false;
    const uint32_t lo = seps[0], hi = seps[nseps - 1];
    const size_t n = nseps - 1;
    PinnedTmp text(hi - lo + 1), sep(nseps * sizeof(uint32_t)), vals(n * sizeof(int64_t) + 64);
    if (!text.p || !sep.p || !vals.p) return false;
    memcpy(text.p, base + lo, hi - lo + 1);
    uint32_t* sp = static_cast<uint32_t*>(sep.p);
    for (size_t i = 0; i < nseps; ++i) sp[i] = seps[i] - lo;
    int32_t* bad = reinterpret_cast<int32_t*>(static_cast<char*>(vals.p) + n * sizeof(int64_t));
    *bad = 0;
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
    hipStream_t s = PoolStream(dev);
    int rc = s ? LaunchJsonIntArray(static_cast<const char*>(text.p), sp, (uint32_t)n,
                                    static_cast<int64_t*>(vals.p), bad, s)
               : -1;
    const int wrc = s ? SyncStream(s) : -1;  // buffers stay until the kernel is done
    if (prev != dev) hipSetDevice(prev);
    if (rc != 0 || wrc != 0 || *bad != 0) {
        g_int_array_fallbacks.fetch_add(1, std::memory_order_relaxed);
        return false;
    }
    const int64_t* v = static_cast<const int64_t*>(vals.p);
    out->assign(v, v + n);
    g_int_arrays.fetch_add(1, std::memory_order_relaxed);
    return true;
}

}  // namespace

int EnableGpuJsonIndex(int device, size_t min_bytes, std::string* error) {
    if (Init(device, error) != 0 || InitHbmPool(device, error) != 0) return -1;
    g_device = device;
    json2pb::SetJsonIndexOffload(offload, min_bytes);
    json2pb::SetPb2JsonArrayOffload(array_offload, (size_t)std::max(1, FLAGS_gpu_pb2json_min_elems));
    json::SetIntArrayOffload(int_array_offload, (size_t)std::max(1, FLAGS_gpu_pb2json_min_elems));
    static var::PassiveStatus<int64_t> v5("gpu_json_int_arrays", [] { return g_int_arrays.load(); });
    static var::PassiveStatus<int64_t> v4("gpu_pb2json_arrays", [] { return g_arrays.load(); });
    static var::PassiveStatus<int64_t> v1("gpu_json_indexed_bodies", [] { return g_bodies.load(); });
    static var::PassiveStatus<int64_t> v2("gpu_json_indexed_bytes", [] { return g_bytes.load(); });
    static var::PassiveStatus<int64_t> v3("gpu_json_index_failures", [] { return g_failures.load(); });
    return 0;
}

void DisableGpuJsonIndex() {
    json2pb::SetJsonIndexOffload(nullptr, (size_t)-1);
    json2pb::SetPb2JsonArrayOffload(nullptr, (size_t)-1);
    json::SetIntArrayOffload(nullptr, (size_t)-1);
}

GpuJsonStats GetGpuJsonStats() {
    GpuJsonStats s;
    s.indexed_bodies = g_bodies.load();
    s.indexed_bytes = g_bytes.load();
    s.failures = g_failures.load();
    s.pb2json_arrays = g_arrays.load();
    s.pb2json_elems = g_array_elems.load();
    s.pb2json_failures = g_array_failures.load();
    s.int_arrays = g_int_arrays.load();
    s.int_array_fallbacks = g_int_array_fallbacks.load();
    s.sparse_skips = g_sparse.load();
    return s;
}

}  // namespace gpu
}  // namespace mrpc
