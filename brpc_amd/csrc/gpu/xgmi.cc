#include "gpu/xgmi.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "gpu/copy_engine.h"
#include "gpu/device_codec.h"
#include "gpu/device_handler.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"
#include "mrpc/proto/options.pb.h"
#include "mrpc/proto/rpc_meta.pb.h"
#include "net/socket.h"
#include "policy/device_payload.h"
#include "rpc/periodic_task.h"
#include "var/var.h"

DEFINE_int32(xgmi_slots, 65536, "release-table slots per process (max payload blocks lent at once)");
DEFINE_int32(xgmi_reap_interval_ms, 5, "reap released lends this often while any are outstanding");
DEFINE_int32(xgmi_reap_scan_mb, 256,
             "scan every outstanding lend for releases once they hold this many MiB (out-of-order releases "
             "of large payloads otherwise pin arena blocks until the 100 ms scan)");
DEFINE_int32(device_payload_compress_min_bytes, 16384,
             "device blocks of at least this many bytes are snappy-encoded on the device when the sender asked "
             "for device payload compression (Controller::set_device_payload_compress_type)");
DEFINE_int32(xgmi_dead_peer_reap_ms, 2000,
             "lent blocks whose connection failed are reclaimed after this long (the peer may still be pulling)");

namespace mrpc {
namespace gpu {

namespace {

const uint64_t kShmMagic = 0x58474d4952454c32ull;  // "XGMIREL2"

struct ShmTable {
    uint64_t magic;
    uint32_t nslots;
    uint32_t pad;
    std::atomic<uint64_t> released[1];  // nslots entries: seq of the released lend
};

size_t shm_bytes(uint32_t nslots) { return sizeof(ShmTable) + sizeof(uint64_t) * (nslots - 1); }

std::string boot_id() {
    static std::string id = [] {
        std::ifstream f("/proc/sys/kernel/random/boot_id");
        std::string s;
        std::getline(f, s);
        char host[256] = {0};
        gethostname(host, sizeof(host) - 1);
        return s + "@" + host;
    }();
    return id;
}

std::atomic<int64_t> g_sent_bytes{0}, g_recv_bytes{0}, g_sent_payloads{0}, g_recv_payloads{0}, g_busy{0},
    g_crc_fail{0}, g_copied_in{0}, g_released_unconsumed{0}, g_cross_bytes{0}, g_cross_payloads{0},
    g_peer_fail{0}, g_peer_access{0}, g_attach_fail{0}, g_peer_maps{0}, g_comp_sent{0}, g_comp_recv{0},
    g_comp_raw{0}, g_comp_fail{0}, g_comp_skipped{0};

// ------------------------------------------------------------------ lending
// The process-wide table of blocks lent to peers. A slot holds a Buf that
// references the lent bytes until the borrower writes the slot's seq into
// released[slot] (shared memory) — or the connection is gone for good.
class Lender {
public:
    int init(int device, std::string* err) {
        _device = device;
        _nslots = (uint32_t)std::max(1024, FLAGS_xgmi_slots);
        _shm_name = "/mrpc_xgmi_" + std::to_string(getpid()) + "_" + std::to_string(device);
        const int fd = shm_open(_shm_name.c_str(), O_CREAT | O_RDWR, 0600);
        if (fd < 0) {
            if (err) *err = "shm_open failed";
            return -1;
        }
        const size_t bytes = shm_bytes(_nslots);
        if (ftruncate(fd, (off_t)bytes) != 0) {
            close(fd);
            if (err) *err = "ftruncate failed";
            return -1;
        }
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED) {
            if (err) *err = "mmap failed";
            return -1;
        }
        _table = static_cast<ShmTable*>(m);
        _table->magic = kShmMagic;
        _table->nslots = _nslots;
        for (uint32_t i = 0; i < _nslots; ++i) _table->released[i].store(0, std::memory_order_relaxed);
        _slots.resize(_nslots);
        _free.reserve(_nslots);
        for (uint32_t i = _nslots; i > 0; --i) _free.push_back(i - 1);
        atexit([] { Lender::unlink_all(); });
        registry().push_back(_shm_name);
        return 0;
    }

    // Lend `hold` (one reference to the bytes) to the peer behind `sock_id`.
    bool lend(Buf&& hold, SocketId sock_id, uint32_t* slot, uint64_t* seq) {
        std::vector<Buf> dead;
        bool ok = false;
        {
            std::lock_guard<std::mutex> g(_mu);
            reap_locked(&dead, false);
            if (_free.empty()) reap_locked(&dead, true);
            if (!_free.empty()) {
                const uint32_t s = _free.back();
                _free.pop_back();
                Slot& e = _slots[s];
                e.hold = std::move(hold);
                e.seq = ++_next_seq;
                e.sock = sock_id;
                e.since_us = monotonic_us();
                e.bytes = e.hold.size();
                _held_bytes += e.bytes;
                _outstanding.push_back(s);
                *slot = s;
                *seq = e.seq;
                ok = true;
            }
        }
        return ok;  // `dead` drops its references outside the lock
    }

    // Sender-side give-back of a lend that never left this process.
    void cancel(uint32_t slot, uint64_t seq) {
        if (slot < _nslots) _table->released[slot].store(seq, std::memory_order_release);
    }

    void reap(bool full) {
        std::vector<Buf> dead;
        std::lock_guard<std::mutex> g(_mu);
        reap_locked(&dead, full);
    }

    int64_t outstanding() {
        std::lock_guard<std::mutex> g(_mu);
        return (int64_t)_outstanding.size();
    }

    ShmTable* table() const { return _table; }
    uint32_t nslots() const { return _nslots; }
    const std::string& shm_name() const { return _shm_name; }
    int device() const { return _device; }

private:
    struct Slot {
        Buf hold;
        uint64_t seq = 0;
        SocketId sock = 0;
        int64_t since_us = 0;
        size_t bytes = 0;
    };

    bool released(uint32_t s) const {
        return _table->released[s].load(std::memory_order_acquire) == _slots[s].seq;
    }
    void free_slot(uint32_t s, std::vector<Buf>* dead) {
        dead->emplace_back(std::move(_slots[s].hold));
        _slots[s].hold.clear();
        _held_bytes -= _slots[s].bytes;
        _slots[s].bytes = 0;
        _free.push_back(s);
    }
    // Cheap pass: pop released slots from the front (borrowers release in
    // roughly FIFO order). Full pass (slots exhausted, the outstanding list
    // or the bytes it holds grew large, or every 100 ms while something is
    // stuck at the front): compact the list, also reclaiming lends of
    // connections that failed more than xgmi_dead_peer_reap_ms ago. The
    // byte trigger matters for large payloads: sixteen 16 MiB lends
    // released out of order must not pin the arena for 100 ms.
    void reap_locked(std::vector<Buf>* dead, bool full) {
        while (!_outstanding.empty() && released(_outstanding.front())) {
            free_slot(_outstanding.front(), dead);
            _outstanding.pop_front();
        }
        if (_outstanding.empty()) return;
        const int64_t now = monotonic_us();
        if (!full && _outstanding.size() < _next_full_scan && _held_bytes < _next_scan_bytes &&
            now - _last_full_us < 100000)
            return;
        _last_full_us = now;
        std::deque<uint32_t> keep;
        for (uint32_t s : _outstanding) {
            bool drop = released(s);
            if (!drop && now - _slots[s].since_us > (int64_t)FLAGS_xgmi_dead_peer_reap_ms * 1000) {
                SocketUniquePtr p;
                drop = Socket::Address(_slots[s].sock, &p) != 0;
            }
            if (drop) free_slot(s, dead);
            else keep.push_back(s);
        }
        _outstanding.swap(keep);
        _next_full_scan = std::max<size_t>(1024, _outstanding.size() * 2);
        _next_scan_bytes = std::max<size_t>((size_t)FLAGS_xgmi_reap_scan_mb << 20, _held_bytes * 2);
    }

    static std::vector<std::string>& registry() {
        static std::vector<std::string>* v = new std::vector<std::string>;
        return *v;
    }
    static void unlink_all() {
        for (const std::string& n : registry()) shm_unlink(n.c_str());
    }

    int _device = -1;
    uint32_t _nslots = 0;
    std::string _shm_name;
    ShmTable* _table = nullptr;
    std::mutex _mu;
    std::vector<Slot> _slots;
    std::vector<uint32_t> _free;
    std::deque<uint32_t> _outstanding;
    uint64_t _next_seq = 0;
    size_t _next_full_scan = 1024;
    size_t _held_bytes = 0;  // bytes of the outstanding lends
    size_t _next_scan_bytes = (size_t)256 << 20;
    int64_t _last_full_us = 0;
};

std::mutex g_mu;
Lender* g_lender = nullptr;  // the enabled device's lender
int g_device = -1;

// ------------------------------------------------------------------ peers
struct PeerMap {
    char* base = nullptr;
    size_t size = 0;
    ShmTable* table = nullptr;
    uint32_t nslots = 0;  // slots covered by the mapping (from the hello)
    size_t table_bytes = 0;
    bool local = false;
    int device = -1;  // the peer's GPU (== ours: HBM-local pulls; else xGMI)
};

// Peer arenas are mapped once per (pid, device) and shared by sockets.
std::mutex g_peer_mu;
std::map<std::pair<int, int>, std::shared_ptr<PeerMap>> g_peers;

std::shared_ptr<PeerMap> map_peer(const policy::XgmiHello& h, std::string* err) {
    const auto key = std::make_pair(h.pid(), h.device());
    std::lock_guard<std::mutex> g(g_peer_mu);
    auto it = g_peers.find(key);
    if (it != g_peers.end()) return it->second;
    auto pm = std::make_shared<PeerMap>();
    pm->device = h.device();
    if (h.pid() == getpid()) {
        const ArenaDesc a = GetArena(g_device);
        if (!g_lender || h.device() != g_device || !a.base) {
            if (err) *err = "local arena mismatch";
            return nullptr;
        }
        pm->base = a.base;
        pm->size = a.size;
        pm->table = g_lender->table();
        pm->nslots = g_lender->nslots();
        pm->local = true;
    } else {
        hipIpcMemHandle_t handle;
        if (h.ipc_handle().size() != sizeof(handle) || h.nslots() == 0 || h.arena_size() <= 0) {
            if (err) *err = "bad xgmi hello";
            return nullptr;
        }
        memcpy(&handle, h.ipc_handle().data(), sizeof(handle));
        void* p = nullptr;
        int prev = 0;
        hipGetDevice(&prev);
        hipSetDevice(g_device);
        // a peer on another GPU of this node: the pull kernel reads its HBM
        // directly over xGMI, which needs peer access from our device
        if (h.device() != g_device && h.device() >= 0 && h.device() < DeviceCount()) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, g_device, h.device()) == hipSuccess && can) {
                const hipError_t pe = hipDeviceEnablePeerAccess(h.device(), 0);
                if (pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled) {
                    g_peer_access.fetch_add(1, std::memory_order_relaxed);
                }
                if (pe != hipSuccess) (void)hipGetLastError();  // already enabled is fine
            } else {
                LOG(WARNING) << "xgmi: device " << g_device << " cannot access peer device " << h.device()
                             << "; the pull goes through the IPC mapping alone";
            }
        }
        const hipError_t r = hipIpcOpenMemHandle(&p, handle, hipIpcMemLazyEnablePeerAccess);
        hipSetDevice(prev);
        if (r != hipSuccess) {
            if (err) *err = std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(r);
            return nullptr;
        }
        const int fd = shm_open(h.shm_name().c_str(), O_RDWR, 0600);
        if (fd < 0) {
            hipIpcCloseMemHandle(p);
            if (err) *err = "peer release table " + h.shm_name() + " not found";
            return nullptr;
        }
        const size_t bytes = shm_bytes(h.nslots());
        struct stat st;
        if (fstat(fd, &st) != 0 || (size_t)st.st_size < bytes) {
            close(fd);
            hipIpcCloseMemHandle(p);
            if (err) *err = "peer release table is smaller than announced";
            return nullptr;
        }
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED || static_cast<ShmTable*>(m)->magic != kShmMagic ||
            static_cast<ShmTable*>(m)->nslots != h.nslots()) {
            if (m != MAP_FAILED) munmap(m, bytes);
            hipIpcCloseMemHandle(p);
            if (err) *err = "bad peer release table";
            return nullptr;
        }
        pm->base = static_cast<char*>(p);
        pm->size = (size_t)h.arena_size();
        pm->table = static_cast<ShmTable*>(m);
        pm->nslots = h.nslots();
        pm->table_bytes = bytes;
    }
    g_peers[key] = pm;
    g_peer_maps.fetch_add(1, std::memory_order_relaxed);
    return pm;
}

class XgmiEndpoint : public Transport {
public:
    explicit XgmiEndpoint(std::shared_ptr<PeerMap> p) : peer(std::move(p)) {}
    const char* name() const override { return "xgmi"; }
    std::shared_ptr<PeerMap> peer;
};

PeerMap* peer_of(Socket* sock, std::shared_ptr<Transport>* keep) {
    *keep = sock ? sock->transport() : nullptr;
    XgmiEndpoint* ep = dynamic_cast<XgmiEndpoint*>(keep->get());
    return ep ? ep->peer.get() : nullptr;
}

// Adaptive skip (per connection, hashed): after kSkipAfter incompressible
// payloads in a row a connection lends raw without encoding, probing again
// every kProbeEvery payloads — a stream of random or already-compressed
// tensors stops paying for an encode it throws away.
constexpr int kSkipAfter = 4, kProbeEvery = 32;
std::atomic<int32_t> g_incompressible[1024];
std::atomic<int32_t>& streak_of(Socket* sock) { return g_incompressible[(sock->id() * 0x9E3779B97F4A7C15ull) >> 54]; }

// Encode the payload on the device into a fresh lendable block and lend
// that (gpu/device_codec.h). 0: lent; 1: not worth it or not possible (the
// caller lends the raw bytes); <0: error.
int lend_compressed(Socket* sock, const char* src, uint32_t len, const DeviceLendOptions& opt,
                    policy::DevicePayload* d) {
    const DeviceSnappyLayout lay = DeviceSnappyLayoutFor(len);
    Buf hold;
    void* p = AppendNewDeviceBlock(&hold, lay.region(), g_device);
    const int64_t aoff = p ? ArenaOffset(p, g_device) : -1;
    if (aoff < 0) return 1;
    std::vector<uint32_t> clen(lay.nblocks);
    if (DeviceSnappyEncode(src, len, p, lay, clen.data(), g_device) != 0) {
        g_comp_fail.fetch_add(1, std::memory_order_relaxed);
        return 1;
    }
    uint64_t total = 0;
    for (uint32_t c : clen) total += c;
    if (total * 8 > (uint64_t)len * 7) {
        // incompressible (random bytes, already-compressed data): decoding
        // would cost the receiver more than the bytes it saves
        g_comp_raw.fetch_add(1, std::memory_order_relaxed);
        streak_of(sock).fetch_add(1, std::memory_order_relaxed);
        return 1;
    }
    streak_of(sock).store(0, std::memory_order_relaxed);
    if (opt.verify) {
        // the receiver checks the DECODED bytes: checksum the source
        Segment seg{src, nullptr, len};
        uint32_t crc = 0;
        if (BatchedCopy(&seg, 1, g_device, &crc) != 0) return -1;
        d->set_crc32c(crc);
        d->set_has_crc(true);
    }
    uint32_t slot = 0;
    uint64_t seq = 0;
    if (!g_lender->lend(std::move(hold), sock->id(), &slot, &seq)) {
        g_busy.fetch_add(1, std::memory_order_relaxed);
        d->clear_has_crc();
        return 1;
    }
    d->set_ring_offset(aoff);
    d->set_length((int64_t)len);
    d->set_lent_length((int64_t)lay.region());
    d->set_compress_type(COMPRESS_TYPE_SNAPPY);
    d->set_block_stride(lay.stride);
    d->set_block_ulen(lay.block_ulen);
    for (uint32_t c : clen) d->add_block_clen(c);
    d->set_pb_scan(opt.scan);
    d->set_src_device(g_device);
    d->set_slot(slot);
    d->set_seq(seq);
    g_sent_bytes.fetch_add((int64_t)total, std::memory_order_relaxed);
    g_sent_payloads.fetch_add(1, std::memory_order_relaxed);
    g_comp_sent.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

// ------------------------------------------------------------------ hooks
int xgmi_send(Socket* sock, BufBlock* block, uint32_t offset, uint32_t len, const DeviceLendOptions& opt,
              policy::DevicePayload* d) {
    Lender* l = g_lender;
    if (!l) return -1;
    if (block->device != g_device) return 1;  // another GPU's block: stage it
    const char* src = block->data + offset;
    if (opt.compress == COMPRESS_TYPE_SNAPPY && len >= (uint32_t)std::max(1, FLAGS_device_payload_compress_min_bytes)) {
        const int32_t streak = streak_of(sock).load(std::memory_order_relaxed);
        if (streak < kSkipAfter || streak % kProbeEvery == 0) {
            const int rc = lend_compressed(sock, src, len, opt, d);
            if (rc <= 0) return rc;
        } else {
            streak_of(sock).fetch_add(1, std::memory_order_relaxed);
            g_comp_skipped.fetch_add(1, std::memory_order_relaxed);
        }
    }
    int64_t aoff = ArenaOffset(src, g_device);
    Buf hold;
    if (aoff < 0) {
        // not arena memory (a tensor, a user hipMalloc): one copy into a
        // lendable block, then lend that
        void* p = AppendNewDeviceBlock(&hold, len, g_device);
        aoff = p ? ArenaOffset(p, g_device) : -1;
        if (aoff < 0) {
            g_busy.fetch_add(1, std::memory_order_relaxed);
            return 1;
        }
        // the copy-in folds the checksum while the bytes pass through
        // registers: one pass over HBM instead of two
        Segment seg{src, p, len};
        uint32_t crc = 0;
        if (BatchedCopy(&seg, 1, g_device, opt.verify ? &crc : nullptr) != 0) return -1;
        g_copied_in.fetch_add(1, std::memory_order_relaxed);
        src = static_cast<const char*>(p);
        if (opt.verify) {
            d->set_crc32c(crc);
            d->set_has_crc(true);
        }
    } else {
        hold.append_block(block, offset, len);
        if (opt.verify) {
            // checksum-only segment (null dst) through the copy engine, so
            // concurrent senders' checksums share one launch and one event
            Segment seg{src, nullptr, len};
            uint32_t crc = 0;
            if (BatchedCopy(&seg, 1, g_device, &crc) != 0) return -1;
            d->set_crc32c(crc);
            d->set_has_crc(true);
        }
    }
    uint32_t slot = 0;
    uint64_t seq = 0;
    if (!l->lend(std::move(hold), sock->id(), &slot, &seq)) {
        g_busy.fetch_add(1, std::memory_order_relaxed);
        return 1;  // every slot is out: the caller stages this block inline
    }
    d->set_ring_offset(aoff);
    d->set_length((int64_t)len);
    d->set_pb_scan(opt.scan);
    d->set_src_device(g_device);
    d->set_slot(slot);
    d->set_seq(seq);
    g_sent_bytes.fetch_add((int64_t)len, std::memory_order_relaxed);
    g_sent_payloads.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

void release_in(PeerMap* pm, const policy::DevicePayload& d) {
    if (pm && d.slot() < pm->nslots) pm->table->released[d.slot()].store(d.seq(), std::memory_order_release);
}

int xgmi_recv(Socket* sock, const policy::DevicePayload* const* descs, int n, Buf* outs,
              DevicePayloadIndex* index) {
    std::shared_ptr<Transport> keep;
    PeerMap* pm = peer_of(sock, &keep);
    if (!pm) {
        for (int i = 0; i < n; ++i) outs[i].clear();
        return -1;
    }
    // raw payloads are pulled by one batched copy; device-compressed ones are
    // decoded straight out of the lent region by one codec request
    std::vector<Segment> segs;
    std::vector<int> seg_of;  // payload of each segment
    std::vector<DeviceSnappyBlocks> jobs;
    std::vector<int> job_of;
    segs.reserve(n);
    int rc = 0;
    for (int i = 0; i < n && rc == 0; ++i) {
        const policy::DevicePayload& d = *descs[i];
        const bool comp = d.compress_type() != 0;
        const int64_t off = d.ring_offset(), len = d.length(), region = comp ? d.lent_length() : len;
        if (off < 0 || len < 0 || region < 0 || (uint64_t)off > pm->size || (uint64_t)region > pm->size - (uint64_t)off ||
            d.slot() >= pm->nslots || (comp && (d.compress_type() != COMPRESS_TYPE_SNAPPY || len == 0))) {
            rc = -1;
            break;
        }
        if (len == 0) continue;
        void* dst = AppendNewDeviceBlock(&outs[i], (size_t)len, g_device);
        if (!dst) {
            rc = -1;
            break;
        }
        if (comp) {
            DeviceSnappyBlocks j;
            j.region = pm->base + off;
            j.region_len = (uint64_t)region;
            j.lay.block_ulen = d.block_ulen();
            j.lay.stride = d.block_stride();
            j.lay.nblocks = (uint32_t)d.block_clen_size();
            j.clen = d.block_clen().data();
            j.dst = dst;
            j.len = (uint64_t)len;
            j.scan = d.pb_scan() && index;
            jobs.push_back(j);
            job_of.push_back(i);
        } else {
            segs.push_back(Segment{pm->base + off, dst, (uint64_t)len});
            seg_of.push_back(i);
        }
    }
    // one pull for every raw payload; when the sender asked for verification
    // the pull kernel folds CRC32C while the bytes pass through registers
    bool want_crc = false;
    for (int i : seg_of) want_crc |= descs[i]->has_crc();
    std::vector<uint32_t> crcs(want_crc ? segs.size() : 0);
    if (rc == 0 && !segs.empty())
        rc = BatchedCopy(segs.data(), (int)segs.size(), g_device, want_crc ? crcs.data() : nullptr);
    std::vector<int> jerr(jobs.size(), 0);
    std::vector<DevicePayloadIndex> jidx(jobs.size());
    if (rc == 0 && !jobs.empty()) {
        rc = DeviceSnappyDecode(jobs.data(), (int)jobs.size(), jerr.data(), jidx.data(), g_device);
        for (int e : jerr) rc |= e ? -1 : 0;
    }
    // the bytes are ours now (or never will be): give every region back
    for (int i = 0; i < n; ++i) release_in(pm, *descs[i]);
    auto fail = [&] {
        for (int k = 0; k < n; ++k) outs[k].clear();
        if (pm->device != g_device) g_peer_fail.fetch_add(1, std::memory_order_relaxed);
        return -1;
    };
    if (rc != 0) return fail();
    for (size_t k = 0; k < seg_of.size(); ++k) {
        const policy::DevicePayload& d = *descs[seg_of[k]];
        if (d.has_crc() && crcs[k] != d.crc32c()) {
            g_crc_fail.fetch_add(1, std::memory_order_relaxed);
            return fail();
        }
    }
    // decoded payloads are verified on their output (the sender checksummed
    // its source): checksum-only segments, one engine call for all of them
    std::vector<Segment> vsegs;
    std::vector<int> vof;
    for (size_t k = 0; k < jobs.size(); ++k) {
        if (!descs[job_of[k]]->has_crc()) continue;
        vsegs.push_back(Segment{jobs[k].dst, nullptr, jobs[k].len});
        vof.push_back(job_of[k]);
    }
    if (!vsegs.empty()) {
        std::vector<uint32_t> v(vsegs.size());
        if (BatchedCopy(vsegs.data(), (int)vsegs.size(), g_device, v.data()) != 0) return fail();
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] != descs[vof[k]]->crc32c()) {
                g_crc_fail.fetch_add(1, std::memory_order_relaxed);
                return fail();
            }
        }
    }
    if (index) {
        // raw payloads that asked for an index are scanned where they landed
        std::vector<const void*> bufs;
        std::vector<uint64_t> lens;
        std::vector<int> of;
        for (size_t k = 0; k < seg_of.size(); ++k) {
            if (!descs[seg_of[k]]->pb_scan()) continue;
            bufs.push_back(segs[k].dst);
            lens.push_back(segs[k].len);
            of.push_back(seg_of[k]);
        }
        if (!bufs.empty()) {
            std::vector<DevicePayloadIndex> got(bufs.size());
            if (DevicePbScan(bufs.data(), lens.data(), (int)bufs.size(), got.data(), g_device) != 0) return fail();
            for (size_t k = 0; k < of.size(); ++k) index[of[k]] = std::move(got[k]);
        }
        for (size_t k = 0; k < jobs.size(); ++k) {
            if (jobs[k].scan) index[job_of[k]] = std::move(jidx[k]);
        }
    }
    for (int i = 0; i < n; ++i) {
        const policy::DevicePayload& d = *descs[i];
        int64_t moved = d.length();
        if (d.compress_type()) {
            moved = 0;
            for (uint32_t c : d.block_clen()) moved += c;
        }
        g_recv_bytes.fetch_add(moved, std::memory_order_relaxed);
        if (pm->device != g_device) g_cross_bytes.fetch_add(d.length(), std::memory_order_relaxed);
        if (d.compress_type()) g_comp_recv.fetch_add(1, std::memory_order_relaxed);
    }
    g_recv_payloads.fetch_add(n, std::memory_order_relaxed);
    if (pm->device != g_device) g_cross_payloads.fetch_add(n, std::memory_order_relaxed);
    return 0;
}

void xgmi_release(Socket* sock, const policy::DevicePayload& d) {
    std::shared_ptr<Transport> keep;
    PeerMap* pm = peer_of(sock, &keep);
    if (!pm) return;
    release_in(pm, d);
    g_released_unconsumed.fetch_add(1, std::memory_order_relaxed);
}

void xgmi_cancel(const policy::DevicePayload& d) {
    if (g_lender) g_lender->cancel(d.slot(), d.seq());
}

}  // namespace

namespace {
// Reaps the lender every -xgmi_reap_interval_ms while it holds lends, so
// blocks whose borrowers already released them go back to the arena even
// when this process stops lending (otherwise they wait for the next lend).
class LenderReaper : public PeriodicTask {
public:
    bool OnTriggeringTask(timespec* next) override {
        if (g_lender && g_lender->outstanding() > 0) g_lender->reap(true);
        *next = realtime_after_us((int64_t)std::max(1, FLAGS_xgmi_reap_interval_ms) * 1000);
        return true;
    }
    void OnDestroyingTask() override { delete this; }
};
}  // namespace

int EnableXgmiTransport(int device, std::string* error) {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_lender) return g_lender->device() == device || device < 0 ? 0 : -1;
    if (device < 0) device = CurrentDevice();
    if (Init(device, error) != 0 || InitHbmPool(device, error) != 0) return -1;
    Lender* l = new Lender;
    if (l->init(device, error) != 0) {
        delete l;
        return -1;
    }
    UsePinnedBlocks();
    SetStageToHostHook(StageToPinnedHost);
    g_device = device;
    g_lender = l;
    SetHbmReclaimHook(ReapLentBlocks);
    PeriodicTaskManager::StartTaskAt(new LenderReaper, realtime_after_us(10000));
    DeviceTransportHooks h;
    h.send = xgmi_send;
    h.recv = xgmi_recv;
    h.release = xgmi_release;
    h.cancel = xgmi_cancel;
    SetDeviceTransportHooks(h);
    static var::PassiveStatus<int64_t> v1("xgmi_sent_bytes", [] { return g_sent_bytes.load(); });
    static var::PassiveStatus<int64_t> v2("xgmi_recv_bytes", [] { return g_recv_bytes.load(); });
    static var::PassiveStatus<int64_t> v3("xgmi_busy_fallbacks", [] { return g_busy.load(); });
    static var::PassiveStatus<int64_t> v4("xgmi_lent_outstanding",
                                          [] { return g_lender ? g_lender->outstanding() : 0; });
    static var::PassiveStatus<int64_t> v5("xgmi_copy_launches", [] { return GetCopyEngineStats().launches; });
    return 0;
}

bool XgmiEnabled() { return g_lender != nullptr; }
int XgmiDevice() { return g_device; }

bool FillXgmiHello(policy::XgmiHello* h) {
    if (!g_lender) return false;
    const ArenaDesc a = GetArena(g_device);
    if (!a.base) return false;
    h->set_ipc_handle(a.ipc_handle);
    h->set_device(g_device);
    h->set_arena_size((int64_t)a.size);
    h->set_pid(getpid());
    h->set_shm_name(g_lender->shm_name());
    h->set_nslots(g_lender->nslots());
    h->set_host_id(boot_id());
    return true;
}

int AttachXgmiPeer(Socket* sock, const policy::XgmiHello& hello, std::string* error) {
    if (!g_lender) {
        if (error) *error = "xgmi transport is not enabled in this process";
        return -1;
    }
    if (hello.host_id() != boot_id()) {
        if (error) *error = "peer is on another node";
        return -1;
    }
    if (sock->transport()) return 0;
    std::shared_ptr<PeerMap> pm = map_peer(hello, error);
    if (!pm) {
        // counted fallback: the connection stays on TCP, device payloads
        // are staged through pinned memory
        g_attach_fail.fetch_add(1, std::memory_order_relaxed);
        return -1;
    }
    sock->set_transport(std::make_shared<XgmiEndpoint>(pm));
    return 0;
}

void ReapLentBlocks() {
    if (g_lender) g_lender->reap(true);
}



XgmiStats GetXgmiStats() {
    XgmiStats s;
    s.sent_bytes = g_sent_bytes.load();
    s.recv_bytes = g_recv_bytes.load();
    s.sent_payloads = g_sent_payloads.load();
    s.recv_payloads = g_recv_payloads.load();
    s.ring_full_fallbacks = g_busy.load();
    s.crc_failures = g_crc_fail.load();
    s.lent_outstanding = g_lender ? g_lender->outstanding() : 0;
    s.copied_into_arena = g_copied_in.load();
    s.released_unconsumed = g_released_unconsumed.load();
    s.cross_device_payloads = g_cross_payloads.load();
    s.cross_device_bytes = g_cross_bytes.load();
    s.cross_device_pull_failures = g_peer_fail.load();
    s.peer_access_enabled = g_peer_access.load();
    s.attach_failures = g_attach_fail.load();
    s.peer_maps = g_peer_maps.load();
    s.compressed_sent = g_comp_sent.load();
    s.compressed_recv = g_comp_recv.load();
    s.compress_skipped_raw = g_comp_raw.load();
    s.compress_failures = g_comp_fail.load();
    s.compress_skipped_adaptive = g_comp_skipped.load();
    return s;
}

}  // namespace gpu
}  // namespace mrpc
