// Bindings of the device kernels for torch tensors. Python passes raw
// device pointers (tensor.data_ptr()) and the HIP stream handle
// (torch.cuda.current_stream().cuda_stream) so the native module never
// links libtorch; the ops run stream-ordered with torch's own work.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <hip/hip_runtime_api.h>

#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"
#include "gpu/copy_engine.h"
#include "gpu/device_codec.h"
#include "policy/device_payload.h"
#include "gpu/gpu.h"
#include "gpu/kernels.h"

namespace py = pybind11;
using namespace mrpc;

static hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + " failed: " + hipGetErrorString(hipGetLastError()));
}

namespace {
struct ParkedWaiters {
    std::vector<fiber::fiber_t> tids;
    std::vector<int64_t> waited_us;
    std::vector<int> rcs;
    int device = 0;
    uint64_t us = 0;
};
struct ParkArg {
    ParkedWaiters* p;
    size_t i;
};
void* park_on_kernel(void* arg) {
    ParkArg* a = static_cast<ParkArg*>(arg);
    ParkedWaiters* p = a->p;
    const size_t i = a->i;
    delete a;
    hipSetDevice(p->device);
    hipStream_t s = gpu::PoolStream(p->device);
    hipEvent_t ev = gpu::AcquireEvent();
    const int64_t t0 = monotonic_us();
    int rc = -1;
    if (s && ev && gpu::LaunchSleepKernel(p->us, s) == 0 && hipEventRecord(ev, s) == hipSuccess) {
        rc = gpu::WaitEvent(ev);  // parks this fiber, never the worker
    }
    p->waited_us[i] = monotonic_us() - t0;
    p->rcs[i] = rc;
    if (ev) gpu::ReleaseEvent(ev);
    return nullptr;
}
}  // namespace

namespace {
// Device buffer owned for the duration of one benchmark call.
struct DevBuf {
    void* p = nullptr;
    explicit DevBuf(size_t n) {
        if (hipMalloc(&p, n ? n : 1) != hipSuccess) p = nullptr;
    }
    ~DevBuf() {
        if (p) hipFree(p);
    }
    template <typename T>
    T* as() const { return static_cast<T*>(p); }
};

}  // namespace

void bind_gpu_ops(py::module_& g) {
    // n fibers each launch a kernel that runs `us` microseconds and wait for
    // its event; returns a handle for park_join (tests of the fiber-aware
    // GPU wait: RPCs must keep flowing on the same workers meanwhile)
    g.def("park_start", [](int n, uint64_t us, int device) {
        ParkedWaiters* p = new ParkedWaiters;
        p->device = device;
        p->us = us;
        p->tids.resize(n);
        p->waited_us.assign(n, 0);
        p->rcs.assign(n, -1);
        for (int i = 0; i < n; ++i) {
            if (fiber::start_background(&p->tids[i], &fiber::ATTR_NORMAL, park_on_kernel, new ParkArg{p, (size_t)i}) != 0) {
                throw std::runtime_error("fiber start failed");
            }
        }
        return reinterpret_cast<uintptr_t>(p);
    }, py::arg("n"), py::arg("us"), py::arg("device") = 0);
    g.def("park_join", [](uintptr_t h) {
        ParkedWaiters* p = reinterpret_cast<ParkedWaiters*>(h);
        {
            py::gil_scoped_release nogil;
            for (fiber::fiber_t t : p->tids) fiber::join(t, nullptr);
        }
        py::list waited, rcs;
        for (int64_t w : p->waited_us) waited.append(w);
        for (int r : p->rcs) rcs.append(r);
        delete p;
        return py::make_tuple(waited, rcs);
    });
    g.def("crc32c_lds_launch", [](const std::vector<uintptr_t>& ptrs, const std::vector<uint64_t>& lens, uintptr_t out,
                              uintptr_t stream) {
        if (ptrs.size() != lens.size()) throw std::invalid_argument("ptrs/lens size mismatch");
        std::vector<gpu::Segment> segs(ptrs.size());
        for (size_t i = 0; i < ptrs.size(); ++i) segs[i] = gpu::Segment{(const void*)ptrs[i], nullptr, lens[i]};
        check(gpu::LaunchCrc32c(segs.data(), (int)segs.size(), (uint32_t*)out, as_stream(stream)), "crc32c");
    }, py::arg("ptrs"), py::arg("lens"), py::arg("out"), py::arg("stream") = 0);
    g.def("crc32c_scratch_bytes", &gpu::Crc32cScratchBytes);
    g.def("crc32c_segments_launch", [](uintptr_t starts, uintptr_t lens, int64_t nseg, uint64_t total_bytes,
                                       uint64_t max_seg_len, uintptr_t out, uintptr_t scratch, uintptr_t stream) {
        check(gpu::LaunchCrc32cSegments((const uint64_t*)starts, (const uint64_t*)lens, nseg, total_bytes, max_seg_len,
                                        (uint32_t*)out, (void*)scratch, as_stream(stream)),
              "crc32c_segments");
    });
    g.def("crc32c_sync", [](uintptr_t ptr, uint64_t len, int device) {
        uint32_t out = 0;
        const void* p = (const void*)ptr;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::Crc32cDevice(&p, &len, 1, &out, device);
        }
        check(rc, "crc32c_sync");
        return out;
    }, py::arg("ptr"), py::arg("len"), py::arg("device") = -1);
    g.def("batched_copy_launch", [](const std::vector<uintptr_t>& srcs, const std::vector<uintptr_t>& dsts,
                                    const std::vector<uint64_t>& lens, uintptr_t stream) {
        if (srcs.size() != lens.size() || dsts.size() != lens.size()) throw std::invalid_argument("size mismatch");
        std::vector<gpu::Segment> segs(lens.size());
        for (size_t i = 0; i < lens.size(); ++i) segs[i] = gpu::Segment{(const void*)srcs[i], (void*)dsts[i], lens[i]};
        check(gpu::LaunchBatchedCopy(segs.data(), (int)segs.size(), as_stream(stream)), "batched_copy");
    }, py::arg("srcs"), py::arg("dsts"), py::arg("lens"), py::arg("stream") = 0);
    // The copy engine itself (gpu/copy_engine.h): blocks until the batch it
    // joined completed; with_crc returns one CRC32C per segment (or, with
    // fold, one for the concatenation). A 0 dst only checksums.
    g.def("engine_copy", [](const std::vector<uintptr_t>& srcs, const std::vector<uintptr_t>& dsts,
                            const std::vector<uint64_t>& lens, int device, bool with_crc, bool fold) {
        if (srcs.size() != lens.size() || dsts.size() != lens.size()) throw std::invalid_argument("size mismatch");
        std::vector<gpu::Segment> segs(lens.size());
        for (size_t i = 0; i < lens.size(); ++i) segs[i] = gpu::Segment{(const void*)srcs[i], (void*)dsts[i], lens[i]};
        std::vector<uint32_t> crcs(with_crc ? segs.size() : 0);
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::BatchedCopy(segs.data(), (int)segs.size(), device, with_crc ? crcs.data() : nullptr, fold);
        }
        check(rc, "engine_copy");
        if (fold && !crcs.empty()) crcs.resize(1);
        return crcs;
    }, py::arg("srcs"), py::arg("dsts"), py::arg("lens"), py::arg("device") = 0, py::arg("with_crc") = false,
       py::arg("fold") = false);
    // Device-payload codec (gpu/device_codec.h), for numerics tests: encode
    // `len` bytes at src into blocks at dst (layout of -device_payload_block_kb)
    // -> (block_ulen, stride, [clen...]); decode such a table back -> per-job
    // code (0 ok, 1 bad table, 2 malformed block) and the field table when scanned.
    g.def("device_snappy_layout", [](uint64_t len) {
        const gpu::DeviceSnappyLayout l = gpu::DeviceSnappyLayoutFor(len);
        return py::make_tuple(l.block_ulen, l.stride, l.nblocks);
    });
    g.def("device_snappy_encode", [](uintptr_t src, uint64_t len, uintptr_t dst, int device) {
        const gpu::DeviceSnappyLayout l = gpu::DeviceSnappyLayoutFor(len);
        std::vector<uint32_t> clen(l.nblocks);
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::DeviceSnappyEncode((const void*)src, len, (void*)dst, l, clen.data(), device);
        }
        check(rc, "device_snappy_encode");
        return clen;
    });
    g.def("device_snappy_decode", [](uintptr_t region, uint64_t region_len, uint32_t block_ulen, uint32_t stride,
                                     const std::vector<uint32_t>& clen, uintptr_t dst, uint64_t len, bool scan,
                                     int device) {
        gpu::DeviceSnappyBlocks j;
        j.region = (const char*)region;
        j.region_len = region_len;
        j.lay.block_ulen = block_ulen;
        j.lay.stride = stride;
        j.lay.nblocks = (uint32_t)clen.size();
        j.clen = clen.data();
        j.dst = (void*)dst;
        j.len = len;
        j.scan = scan;
        int err = 0, rc;
        DevicePayloadIndex idx;
        {
            py::gil_scoped_release nogil;
            rc = gpu::DeviceSnappyDecode(&j, 1, &err, &idx, device);
        }
        check(rc, "device_snappy_decode");
        return py::make_tuple(err, idx.nfields, idx.fields);
    });
    // Packed numeric fields already in HBM -> device arrays (one codec
    // request for all runs): [(count, code)] per run, code 0 ok, 1 malformed
    // or truncated, 2 refused.
    g.def("device_decode_packed", [](const std::vector<uintptr_t>& srcs, const std::vector<uint64_t>& lens,
                                     const std::vector<uint32_t>& kinds, const std::vector<uintptr_t>& dsts,
                                     int device) {
        if (srcs.size() != lens.size() || kinds.size() != lens.size() || dsts.size() != lens.size())
            throw std::invalid_argument("size mismatch");
        std::vector<gpu::DevicePackedRun> runs(lens.size());
        for (size_t i = 0; i < lens.size(); ++i) {
            runs[i].src = (const void*)srcs[i];
            runs[i].len = lens[i];
            runs[i].kind = kinds[i];
            runs[i].dst = (void*)dsts[i];
        }
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::DeviceDecodePackedRuns(runs.data(), (int)runs.size(), device);
        }
        check(rc, "device_decode_packed");
        py::list out;
        for (const gpu::DevicePackedRun& r : runs) out.append(py::make_tuple(r.count, r.err));
        return out;
    }, py::arg("srcs"), py::arg("lens"), py::arg("kinds"), py::arg("dsts"), py::arg("device") = 0);
    g.def("device_payload_field", [](int nfields, const std::vector<uint64_t>& fields, uint32_t number) -> py::object {
        DevicePayloadIndex idx;
        idx.nfields = nfields;
        idx.fields = fields;
        uint64_t off = 0, len = 0;
        if (!gpu::DevicePayloadField(idx, number, &off, &len)) return py::none();
        return py::make_tuple(off, len);
    });
    g.def("resident_stats", [] {
        const gpu::ResidentStats s = gpu::GetResidentStats();
        py::dict d;
        d["launches"] = s.launches;
        d["batches"] = s.batches;
        d["ring_full_waits"] = s.ring_full_waits;
        return d;
    });
    g.def("batched_copy_crc32c_launch", [](const std::vector<uintptr_t>& srcs, const std::vector<uintptr_t>& dsts,
                                           const std::vector<uint64_t>& lens, uintptr_t out, uintptr_t stream,
                                           bool mfma) {
        if (srcs.size() != lens.size() || dsts.size() != lens.size()) throw std::invalid_argument("size mismatch");
        std::vector<gpu::Segment> segs(lens.size());
        for (size_t i = 0; i < lens.size(); ++i) segs[i] = gpu::Segment{(const void*)srcs[i], (void*)dsts[i], lens[i]};
        check(gpu::LaunchBatchedCopyCrc32c(segs.data(), (int)segs.size(), (uint32_t*)out, as_stream(stream), mfma),
              "batched_copy_crc32c");
    }, py::arg("srcs"), py::arg("dsts"), py::arg("lens"), py::arg("out"), py::arg("stream") = 0,
       py::arg("mfma") = true);
    g.def("pb_scan_launch", [](uintptr_t buf, uint64_t buf_len, uintptr_t offsets, int64_t n, uint32_t max_fields,
                               uintptr_t fields, uintptr_t nfields, uintptr_t stream) {
        check(gpu::LaunchPbScan((const uint8_t*)buf, buf_len, (const int64_t*)offsets, n, max_fields,
                                (uint64_t*)fields, (int32_t*)nfields, as_stream(stream)),
              "pb_scan");
    });
    g.def("snappy_max_block", [] { return gpu::kSnappyMaxBlock; });
    // jobs: device array of {src, dst, src_len, dst_cap} (4 x u64 per job)
    g.def("snappy_decompress_launch", [](uintptr_t jobs, int n, uint32_t max_ulen, uintptr_t out_len, uintptr_t err,
                                         uintptr_t stream) {
        check(gpu::LaunchSnappyDecompress((const gpu::SnappyJob*)jobs, n, max_ulen, (uint32_t*)out_len, (int*)err,
                                          as_stream(stream)),
              "snappy_decompress");
    });
    // streams: {src, dst, src_len|dst_cap<<32, first|max_pieces<<32}; pieces: 24 B each (device)
    g.def("snappy_max_pieces", [](uint64_t ulen, uint32_t limit) { return gpu::SnappyMaxPieces(ulen, limit); });
    g.def("snappy_piece_bytes", [] { return sizeof(gpu::SnappyPiece); });
    g.def("snappy_split_launch", [](uintptr_t streams, int n, uint32_t limit, uintptr_t pieces, uintptr_t err,
                                    uintptr_t stream) {
        check(gpu::LaunchSnappySplit((const gpu::SnappyStream*)streams, n, limit, (gpu::SnappyPiece*)pieces, (int*)err,
                                     as_stream(stream)),
              "snappy_split");
    });
    g.def("snappy_decompress_pieces_launch", [](uintptr_t pieces, int n, uint32_t lo, uint32_t hi, uintptr_t err,
                                                uintptr_t stream) {
        check(gpu::LaunchSnappyDecompressPieces((const gpu::SnappyPiece*)pieces, n, lo, hi, (int*)err,
                                                as_stream(stream)),
              "snappy_decompress_pieces");
    });
    g.def("snappy_decompress_pieces_serial_launch", [](uintptr_t pieces, int n, uint32_t lo, uint32_t hi,
                                                       uintptr_t err, uintptr_t stream) {
        check(gpu::LaunchSnappyDecompressPiecesSerial((const gpu::SnappyPiece*)pieces, n, lo, hi, (int*)err,
                                                      as_stream(stream)),
              "snappy_decompress_pieces_serial");
    });
    g.def("snappy_compress_stamped_launch", [](uintptr_t jobs, int n, uint32_t max_ulen, uintptr_t scratch,
                                                  uintptr_t out_len, uintptr_t err, uintptr_t stamps, uintptr_t stream) {
        check(gpu::LaunchSnappyCompressStamped((const gpu::SnappyJob*)jobs, n, max_ulen, (void*)scratch,
                                               (uint32_t*)out_len, (int*)err, (uint64_t*)stamps, as_stream(stream)),
              "snappy_compress_stamped");
    });
    g.def("snappy_decompress_pieces_stamped_launch", [](uintptr_t pieces, int n, uint32_t lo, uint32_t hi,
                                                        uintptr_t err, uintptr_t stamps, uintptr_t stream) {
        check(gpu::LaunchSnappyDecompressPiecesStamped((const gpu::SnappyPiece*)pieces, n, lo, hi, (int*)err,
                                                       (uint64_t*)stamps, as_stream(stream)),
              "snappy_decompress_pieces_stamped");
    });
    g.def("snappy_compress_scratch_per_block", [] { return gpu::SnappyCompressScratchPerBlock(); });
    g.def("snappy_max_compressed_length", [](uint64_t n) { return gpu::SnappyMaxCompressedLength(n); });
    g.def("snappy_compress_launch", [](uintptr_t jobs, int n, uint32_t max_ulen, uintptr_t scratch, uintptr_t out_len,
                                       uintptr_t err, uintptr_t stream) {
        check(gpu::LaunchSnappyCompress((const gpu::SnappyJob*)jobs, n, max_ulen, (void*)scratch, (uint32_t*)out_len,
                                        (int*)err, as_stream(stream)),
              "snappy_compress");
    });
    g.def("varint_scratch_bytes", &gpu::VarintScratchBytes);
    g.def("varint_decode_launch", [](uintptr_t in, uint64_t n, uintptr_t out, uint64_t max_out, bool zigzag,
                                     uintptr_t count, uintptr_t err, uintptr_t scratch, uintptr_t stream) {
        check(gpu::LaunchVarintDecode((const uint8_t*)in, n, (uint64_t*)out, max_out, zigzag, (uint64_t*)count,
                                      (int*)err, (void*)scratch, as_stream(stream)),
              "varint_decode");
    });
    g.def("varint_encode_launch", [](uintptr_t in, uint64_t n, bool zigzag, uintptr_t out, uintptr_t nbytes,
                                     uintptr_t scratch, uintptr_t stream) {
        check(gpu::LaunchVarintEncode((const uint64_t*)in, n, zigzag, (uint8_t*)out, (uint64_t*)nbytes,
                                      (void*)scratch, as_stream(stream)),
              "varint_encode");
    });
    g.def("json_index_scratch_bytes", &gpu::JsonIndexScratchBytes);
    g.def("json_index_launch", [](uintptr_t in, uint64_t n, uintptr_t out, uint64_t max_out, uintptr_t count,
                                  uintptr_t err, uintptr_t scratch, uintptr_t stream) {
        check(gpu::LaunchJsonIndex((const uint8_t*)in, n, (uint32_t*)out, max_out, (uint64_t*)count, (int*)err,
                                   (void*)scratch, as_stream(stream)),
              "json_index");
    });
}
