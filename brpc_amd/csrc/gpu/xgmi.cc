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
#include "gpu/gpu.h"
#include "gpu/kernels.h"
#include "mrpc/proto/rpc_meta.pb.h"
#include "net/socket.h"
#include "policy/device_payload.h"
#include "var/var.h"

DEFINE_int32(xgmi_arena_mb, 256, "HBM arena per device for outgoing device payloads (MiB)");
DEFINE_int32(xgmi_slots, 65536, "release-table slots per arena (max in-flight payload regions)");

namespace mrpc {
namespace gpu {

namespace {

const uint64_t kShmMagic = 0x58474d4952454c31ull;  // "XGMIREL1"

struct ShmTable {
    uint64_t magic;
    uint32_t nslots;
    uint32_t pad;
    std::atomic<uint64_t> released[1];  // nslots entries: seq of the released region
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

std::atomic<int64_t> g_sent_bytes{0}, g_recv_bytes{0}, g_sent_payloads{0}, g_recv_payloads{0}, g_ring_full{0},
    g_crc_fail{0};

// ------------------------------------------------------------------ arena
class Arena {
public:
    int init(int device, std::string* err) {
        _device = device;
        _size = (size_t)FLAGS_xgmi_arena_mb << 20;
        _base = static_cast<char*>(Malloc(_size, device, err));
        if (!_base) return -1;
        int prev = 0;
        hipGetDevice(&prev);
        hipSetDevice(device);
        const hipError_t r = hipIpcGetMemHandle(&_handle, _base);
        hipSetDevice(prev);
        if (r != hipSuccess) {
            if (err) *err = std::string("hipIpcGetMemHandle: ") + hipGetErrorString(r);
            return -1;
        }
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
        static std::once_flag unlink_once;
        std::call_once(unlink_once, [] { atexit([] { Arena::unlink_all(); }); });
        registry().push_back(_shm_name);
        return 0;
    }

    // Reserve `len` bytes; returns false when the ring is full.
    bool alloc(size_t len, uint64_t* off, uint32_t* slot, uint64_t* seq) {
        const size_t need = (len + 255) & ~(size_t)255;
        std::lock_guard<std::mutex> g(_mu);
        while (!_q.empty() && _table->released[_q.front().slot].load(std::memory_order_acquire) == _q.front().seq) {
            _q.pop_front();
        }
        if (_q.size() >= _nslots || need > _size) return false;
        size_t at;
        if (_q.empty()) {
            at = 0;  // everything released: restart at the bottom
        } else {
            const size_t tail = _q.front().off;  // oldest live region
            if (_head > tail) {
                // live = [tail, head); free = [head, size) + [0, tail)
                if (_size - _head >= need) at = _head;
                else if (tail > need) at = 0;  // wrap; keep head != tail
                else return false;
            } else {
                // wrapped: live = [tail, size) + [0, head); free = [head, tail)
                if (tail - _head > need) at = _head;
                else return false;
            }
        }
        _head = at + need;
        Region r{at, need, _next_slot, ++_next_seq};
        _next_slot = (_next_slot + 1) % _nslots;
        _q.push_back(r);
        *off = at;
        *slot = r.slot;
        *seq = r.seq;
        return true;
    }

    char* base() const { return _base; }
    size_t size() const { return _size; }
    int device() const { return _device; }
    ShmTable* table() const { return _table; }
    void fill(policy::XgmiHello* h) const {
        h->set_ipc_handle(std::string(reinterpret_cast<const char*>(&_handle), sizeof(_handle)));
        h->set_device(_device);
        h->set_arena_size((int64_t)_size);
        h->set_pid(getpid());
        h->set_shm_name(_shm_name);
        h->set_nslots(_nslots);
        h->set_host_id(boot_id());
    }
    static void unlink_all() {
        for (const std::string& n : registry()) shm_unlink(n.c_str());
    }

private:
    static std::vector<std::string>& registry() {
        static std::vector<std::string>* v = new std::vector<std::string>;
        return *v;
    }
    struct Region {
        size_t off, len;
        uint32_t slot;
        uint64_t seq;
    };
    int _device = -1;
    char* _base = nullptr;
    size_t _size = 0;
    hipIpcMemHandle_t _handle;
    uint32_t _nslots = 0;
    std::string _shm_name;
    ShmTable* _table = nullptr;
    std::mutex _mu;
    std::deque<Region> _q;
    size_t _head = 0;
    uint32_t _next_slot = 0;
    uint64_t _next_seq = 0;
};

std::mutex g_mu;
Arena* g_arena = nullptr;  // the enabled device's arena
int g_device = -1;

// ------------------------------------------------------------------ peers
struct PeerMap {
    char* base = nullptr;
    size_t size = 0;
    ShmTable* table = nullptr;
    size_t table_bytes = 0;
    bool local = false;
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
    if (h.pid() == getpid()) {
        if (!g_arena || h.device() != g_arena->device()) {
            if (err) *err = "local arena mismatch";
            return nullptr;
        }
        pm->base = g_arena->base();
        pm->size = g_arena->size();
        pm->table = g_arena->table();
        pm->local = true;
    } else {
        hipIpcMemHandle_t handle;
        if (h.ipc_handle().size() != sizeof(handle)) {
            if (err) *err = "bad ipc handle size";
            return nullptr;
        }
        memcpy(&handle, h.ipc_handle().data(), sizeof(handle));
        void* p = nullptr;
        int prev = 0;
        hipGetDevice(&prev);
        hipSetDevice(g_device);
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
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED || static_cast<ShmTable*>(m)->magic != kShmMagic) {
            hipIpcCloseMemHandle(p);
            if (err) *err = "bad peer release table";
            return nullptr;
        }
        pm->base = static_cast<char*>(p);
        pm->size = (size_t)h.arena_size();
        pm->table = static_cast<ShmTable*>(m);
        pm->table_bytes = bytes;
    }
    g_peers[key] = pm;
    return pm;
}

class XgmiEndpoint : public Transport {
public:
    explicit XgmiEndpoint(std::shared_ptr<PeerMap> p) : peer(std::move(p)) {}
    const char* name() const override { return "xgmi"; }
    std::shared_ptr<PeerMap> peer;
};

// ------------------------------------------------------------------ hooks
int xgmi_send(Socket* sock, const void* dev_ptr, size_t len, int device, bool with_crc, policy::DevicePayload* d) {
    Arena* a = g_arena;
    if (!a) return -1;
    uint64_t off = 0, seq = 0;
    uint32_t slot = 0;
    if (!a->alloc(len, &off, &slot, &seq)) {
        g_ring_full.fetch_add(1, std::memory_order_relaxed);
        return 1;  // ring full: the caller stages this block through host memory
    }
    // a region that never reaches the peer must still be released, or the
    // FIFO ring would stall behind it forever
    auto give_back = [&] { a->table()->released[slot].store(seq, std::memory_order_release); };
    hipStream_t s = PoolStream(a->device());
    if (!s || hipMemcpyAsync(a->base() + off, dev_ptr, len, hipMemcpyDeviceToDevice, s) != hipSuccess ||
        SyncStream(s) != 0) {
        give_back();
        return -1;
    }
    if (with_crc) {
        const void* p = a->base() + off;
        uint64_t l = len;
        uint32_t crc = 0;
        if (Crc32cDevice(&p, &l, 1, &crc, a->device()) != 0) {
            give_back();
            return -1;
        }
        d->set_crc32c(crc);
        d->set_has_crc(true);
    }
    d->set_ring_offset((int64_t)off);
    d->set_length((int64_t)len);
    d->set_src_device(device);
    d->set_slot(slot);
    d->set_seq(seq);
    g_sent_bytes.fetch_add((int64_t)len, std::memory_order_relaxed);
    g_sent_payloads.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

void pool_deleter(void* p, void*) { PoolFree(p); }

int xgmi_recv(Socket* sock, const policy::DevicePayload& d, Buf* out) {
    std::shared_ptr<Transport> t = sock->transport();
    XgmiEndpoint* ep = dynamic_cast<XgmiEndpoint*>(t.get());
    if (!ep || !ep->peer) return -1;
    PeerMap* pm = ep->peer.get();
    const size_t len = (size_t)d.length();
    if (d.ring_offset() < 0 || (size_t)d.ring_offset() + len > pm->size || d.slot() >= pm->table->nslots) return -1;
    void* dst = PoolAlloc(len, g_device);
    if (!dst) return -1;
    hipStream_t s = PoolStream(g_device);
    if (!s || hipMemcpyAsync(dst, pm->base + d.ring_offset(), len, hipMemcpyDeviceToDevice, s) != hipSuccess ||
        SyncStream(s) != 0) {
        PoolFree(dst);
        return -1;
    }
    // the bytes are ours now: give the region back to the sender
    pm->table->released[d.slot()].store(d.seq(), std::memory_order_release);
    if (d.has_crc()) {
        const void* p = dst;
        uint64_t l = len;
        uint32_t crc = 0;
        if (Crc32cDevice(&p, &l, 1, &crc, g_device) != 0 || crc != d.crc32c()) {
            g_crc_fail.fetch_add(1, std::memory_order_relaxed);
            PoolFree(dst);
            return -1;
        }
    }
    out->append_user_data(dst, len, pool_deleter, nullptr, MemKind::DEVICE, g_device);
    g_recv_bytes.fetch_add((int64_t)len, std::memory_order_relaxed);
    g_recv_payloads.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

// ------------------------------------------------------------------ pool
struct PoolState {
    std::mutex mu;
    std::map<size_t, std::vector<void*>> free;  // size class -> blocks
    std::map<void*, std::pair<size_t, int>> live;  // ptr -> (class, device)
};
PoolState& pool() {
    static PoolState* p = new PoolState;
    return *p;
}

size_t size_class(size_t n) {
    size_t c = 4096;
    while (c < n) c <<= 1;
    return c;
}

}  // namespace

void* PoolAlloc(size_t n, int device) {
    const size_t c = size_class(n);
    PoolState& ps = pool();
    {
        std::lock_guard<std::mutex> g(ps.mu);
        auto& v = ps.free[c * 64 + (size_t)device];  // classes are multiples of 4096: room for the device
        if (!v.empty()) {
            void* p = v.back();
            v.pop_back();
            ps.live[p] = {c, device};
            return p;
        }
    }
    void* p = Malloc(c, device);
    if (!p) return nullptr;
    std::lock_guard<std::mutex> g(ps.mu);
    ps.live[p] = {c, device};
    return p;
}

void PoolFree(void* p) {
    if (!p) return;
    PoolState& ps = pool();
    std::lock_guard<std::mutex> g(ps.mu);
    auto it = ps.live.find(p);
    if (it == ps.live.end()) return;
    ps.free[it->second.first * 64 + (size_t)it->second.second].push_back(p);
    ps.live.erase(it);
}

int EnableXgmiTransport(int device, std::string* error) {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_arena) return g_arena->device() == device || device < 0 ? 0 : -1;
    if (device < 0) device = CurrentDevice();
    if (Init(device, error) != 0) return -1;
    Arena* a = new Arena;
    if (a->init(device, error) != 0) {
        delete a;
        return -1;
    }
    g_device = device;
    g_arena = a;
    DeviceTransportHooks h;
    h.send = xgmi_send;
    h.recv = xgmi_recv;
    SetDeviceTransportHooks(h);
    static var::PassiveStatus<int64_t> v1("xgmi_sent_bytes", [] { return g_sent_bytes.load(); });
    static var::PassiveStatus<int64_t> v2("xgmi_recv_bytes", [] { return g_recv_bytes.load(); });
    static var::PassiveStatus<int64_t> v3("xgmi_ring_full_fallbacks", [] { return g_ring_full.load(); });
    return 0;
}

bool XgmiEnabled() { return g_arena != nullptr; }

bool FillXgmiHello(policy::XgmiHello* hello) {
    if (!g_arena) return false;
    g_arena->fill(hello);
    return true;
}

int AttachXgmiPeer(Socket* sock, const policy::XgmiHello& hello, std::string* error) {
    if (!g_arena) {
        if (error) *error = "xgmi transport is not enabled in this process";
        return -1;
    }
    if (hello.host_id() != boot_id()) {
        if (error) *error = "peer is on another node";
        return -1;
    }
    if (sock->transport()) return 0;
    std::shared_ptr<PeerMap> pm = map_peer(hello, error);
    if (!pm) return -1;
    sock->set_transport(std::make_shared<XgmiEndpoint>(pm));
    return 0;
}

XgmiStats GetXgmiStats() {
    XgmiStats s;
    s.sent_bytes = g_sent_bytes.load();
    s.recv_bytes = g_recv_bytes.load();
    s.sent_payloads = g_sent_payloads.load();
    s.recv_payloads = g_recv_payloads.load();
    s.ring_full_fallbacks = g_ring_full.load();
    s.crc_failures = g_crc_fail.load();
    return s;
}

}  // namespace gpu
}  // namespace mrpc
