// Verbs providers behind rdma::Provider.
//
//  * soft    — an in-process reliable-connected fabric: queue pairs find
//              their peer by QP number, a SEND is matched with the oldest
//              posted RECV of the peer (held back, like RNR retry, until
//              one is posted), data is gathered from the SGEs into the
//              receive buffer, and completions (with immediate data) land
//              in the CQs, whose notification fd is an eventfd armed the
//              way ibv_req_notify_cq is. Memory must be registered: every
//              SGE is checked against its MR, and DEVICE MRs are read
//              through the Buf device-copy hook (hipMemcpy D2H), the way a
//              GPUDirect HCA reads HBM.
//  * ibverbs — libibverbs loaded with dlopen (the reference's
//              rdma_helper.cpp:49-74 pattern), RC QPs over the first active
//              port, ibv_reg_dmabuf_mr for HBM. Always compiled, against the
//              in-tree ABI declaration rdma/verbs_abi.h; exercised in the
//              unit tests through a stub verbs library implementing that
//              ABI (tests/fake_ibverbs.cc). No HCA exists on this pool, so
//              real-hardware behaviour stays unverified.
#include <sys/eventfd.h>
#include <unistd.h>

#include <cstring>
#include <map>
#include <random>

#include "base/logging.h"
#include "rdma/rdma.h"

namespace mrpc {
namespace rdma {

namespace {

class SoftQp;

struct SoftMr {
    uintptr_t base;
    size_t len;
    bool device;
    int gpu;
};

struct SoftFabric {
    std::mutex mu;
    std::map<uint32_t, SoftQp*> qps;
    uint32_t next_qpn = 0x100;
    std::map<uint32_t, SoftMr> mrs;          // lkey -> region
    std::map<uintptr_t, uint32_t> by_base;   // base -> lkey
    uint32_t next_lkey = 1;
    uint64_t gid_hi = 0xfe80000000000000ull;
    uint64_t gid_lo;
    SoftFabric() {
        std::random_device rd;
        gid_lo = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)getpid();
    }
};

SoftFabric& fabric() {
    static SoftFabric* f = new SoftFabric;
    return *f;
}

class SoftCq : public CompletionQueue {
public:
    explicit SoftCq(int depth) : _depth(depth) { _efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC); }
    ~SoftCq() override {
        if (_efd >= 0) ::close(_efd);
    }
    int Poll(WorkCompletion* wc, int n) override {
        std::lock_guard<std::mutex> g(_mu);
        int k = 0;
        while (k < n && !_q.empty()) {
            wc[k++] = _q.front();
            _q.pop_front();
        }
        return k;
    }
    int Arm() override {
        std::lock_guard<std::mutex> g(_mu);
        _armed = true;
        return 0;
    }
    int notify_fd() const override { return _efd; }
    void AckEvent() override {
        uint64_t v;
        while (::read(_efd, &v, sizeof(v)) == (ssize_t)sizeof(v)) {
        }
    }
    void Push(const WorkCompletion& wc) {
        std::lock_guard<std::mutex> g(_mu);
        if ((int)_q.size() >= _depth) {
            LOG(ERROR) << "soft rdma: CQ overrun (depth " << _depth << ")";
        }
        _q.push_back(wc);
        if (_armed) {
            _armed = false;
            uint64_t one = 1;
            ssize_t r = ::write(_efd, &one, sizeof(one));
            (void)r;
        }
    }
    bool ok() const { return _efd >= 0; }

private:
    std::mutex _mu;
    std::deque<WorkCompletion> _q;
    int _efd = -1;
    int _depth;
    bool _armed = false;
};

struct PendingSend {
    SoftQp* src;
    uint64_t wr_id;
    std::vector<Sge> sge;
    bool with_imm;
    uint32_t imm;
    bool signaled;
};

class SoftQp : public QueuePair {
public:
    SoftQp(SoftCq* cq, int sq, int rq) : _cq(cq), _sq_depth(sq), _rq_depth(rq) {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        _addr.gid_hi = f.gid_hi;
        _addr.gid_lo = f.gid_lo;
        _addr.qpn = f.next_qpn++;
        f.qps[_addr.qpn] = this;
    }
    ~SoftQp() override {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        f.qps.erase(_addr.qpn);
        for (auto& kv : f.qps) {
            auto& pq = kv.second->_pending_in;
            for (auto it = pq.begin(); it != pq.end();) it = it->src == this ? pq.erase(it) : it + 1;
        }
    }
    QpAddress local() const override { return _addr; }
    int Connect(const QpAddress& remote) override {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        if (remote.gid_hi != f.gid_hi || remote.gid_lo != f.gid_lo) {
            errno = EHOSTUNREACH;  // the soft fabric spans one process
            return -1;
        }
        if (f.qps.find(remote.qpn) == f.qps.end()) {
            errno = ENOENT;
            return -1;
        }
        _peer = remote.qpn;
        return 0;
    }
    int PostSend(uint64_t wr_id, const Sge* sge, int nsge, bool with_imm, uint32_t imm, bool signaled) override {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        auto it = f.qps.find(_peer);
        if (_peer == 0 || it == f.qps.end()) {
            errno = ENOTCONN;
            return -1;
        }
        for (int i = 0; i < nsge; ++i) {
            if (!CheckMrLocked(f, sge[i])) {
                errno = EFAULT;
                return -1;
            }
        }
        SoftQp* peer = it->second;
        peer->_pending_in.push_back(PendingSend{this, wr_id, std::vector<Sge>(sge, sge + nsge), with_imm, imm, signaled});
        peer->DeliverLocked(f);
        return 0;
    }
    int PostRecv(uint64_t wr_id, const Sge& sge) override {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        if (!CheckMrLocked(f, sge) || (int)_rq.size() >= _rq_depth) {
            errno = EINVAL;
            return -1;
        }
        _rq.push_back(std::make_pair(wr_id, sge));
        DeliverLocked(f);
        return 0;
    }

private:
    static bool CheckMrLocked(SoftFabric& f, const Sge& s) {
        if (s.length == 0) return true;
        auto it = f.mrs.find(s.lkey);
        return it != f.mrs.end() && s.addr >= it->second.base && s.addr + s.length <= it->second.base + it->second.len;
    }
    void DeliverLocked(SoftFabric& f) {
        while (!_pending_in.empty() && !_rq.empty()) {
            PendingSend ps = std::move(_pending_in.front());
            _pending_in.pop_front();
            const uint64_t rwr = _rq.front().first;
            const Sge dst = _rq.front().second;
            _rq.pop_front();
            size_t total = 0;
            for (const Sge& s : ps.sge) total += s.length;
            WorkCompletion rwc, swc;
            rwc.wr_id = rwr;
            rwc.opcode = WC_RECV;
            swc.wr_id = ps.wr_id;
            swc.opcode = WC_SEND;
            if (total > dst.length) {
                rwc.status = swc.status = 1;  // IBV_WC_LOC_LEN_ERR
            } else {
                char* out = reinterpret_cast<char*>(dst.addr);
                for (const Sge& s : ps.sge) {
                    if (s.length == 0) continue;
                    const SoftMr& mr = f.mrs[s.lkey];
                    if (mr.device) {
                        DeviceCopyFn cp = GetDeviceCopyHook();
                        if (!cp || cp(out, reinterpret_cast<const void*>(s.addr), s.length, MemKind::DEVICE, mr.gpu) != 0) {
                            rwc.status = swc.status = 2;  // remote access error
                            break;
                        }
                    } else {
                        memcpy(out, reinterpret_cast<const void*>(s.addr), s.length);
                    }
                    out += s.length;
                }
                rwc.byte_len = (uint32_t)total;
                rwc.has_imm = ps.with_imm;
                rwc.imm = ps.imm;
            }
            _cq->Push(rwc);
            if (ps.signaled || swc.status != 0) ps.src->_cq->Push(swc);
        }
    }

    SoftCq* _cq;
    int _sq_depth, _rq_depth;
    QpAddress _addr;
    uint32_t _peer = 0;
    std::deque<std::pair<uint64_t, Sge>> _rq;
    std::deque<PendingSend> _pending_in;
};

class SoftProvider : public Provider {
public:
    const char* name() const override { return "soft"; }
    std::string device_name() const override { return "soft-rc0 (in-process)"; }
    int max_sge() const override { return 16; }
    int RegisterMemory(void* p, size_t n, bool device, int gpu, uint32_t* lkey) override {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        const uint32_t k = f.next_lkey++;
        f.mrs[k] = SoftMr{reinterpret_cast<uintptr_t>(p), n, device, gpu};
        f.by_base[reinterpret_cast<uintptr_t>(p)] = k;
        *lkey = k;
        return 0;
    }
    void DeregisterMemory(void* p) override {
        SoftFabric& f = fabric();
        std::lock_guard<std::mutex> g(f.mu);
        auto it = f.by_base.find(reinterpret_cast<uintptr_t>(p));
        if (it == f.by_base.end()) return;
        f.mrs.erase(it->second);
        f.by_base.erase(it);
    }
    std::unique_ptr<CompletionQueue> CreateCq(int depth) override {
        std::unique_ptr<SoftCq> cq(new SoftCq(depth));
        if (!cq->ok()) return nullptr;
        return std::unique_ptr<CompletionQueue>(cq.release());
    }
    std::unique_ptr<QueuePair> CreateQp(CompletionQueue* cq, int sq_depth, int rq_depth) override {
        return std::unique_ptr<QueuePair>(new SoftQp(static_cast<SoftCq*>(cq), sq_depth, rq_depth));
    }
};

}  // namespace

std::unique_ptr<Provider> CreateSoftProvider() { return std::unique_ptr<Provider>(new SoftProvider); }

}  // namespace rdma
}  // namespace mrpc

// ------------------------------------------------------------------ ibverbs
// Compiled against the in-tree ABI declaration (rdma/verbs_abi.h), library
// loaded at run time with dlopen (-rdma_verbs_library), so hosts without
// an HCA or rdma-core simply report the provider unavailable.
#include <arpa/inet.h>
#include <dlfcn.h>
#include <fcntl.h>

#include "base/flags.h"
#include "rdma/verbs_abi.h"

DEFINE_string(rdma_verbs_library, "libibverbs.so.1", "verbs library dlopen()ed by the ibverbs RDMA provider");

namespace mrpc {
namespace rdma {
namespace {

using namespace verbs;

struct IbvApi {
    void* handle = nullptr;
    std::string loaded_from;
    ibv_get_device_list_fn get_device_list = nullptr;
    ibv_free_device_list_fn free_device_list = nullptr;
    ibv_get_device_name_fn get_device_name = nullptr;
    ibv_open_device_fn open_device = nullptr;
    ibv_close_device_fn close_device = nullptr;
    ibv_alloc_pd_fn alloc_pd = nullptr;
    ibv_dealloc_pd_fn dealloc_pd = nullptr;
    ibv_reg_mr_fn reg_mr = nullptr;
    ibv_reg_dmabuf_mr_fn reg_dmabuf_mr = nullptr;
    ibv_dereg_mr_fn dereg_mr = nullptr;
    ibv_create_comp_channel_fn create_comp_channel = nullptr;
    ibv_destroy_comp_channel_fn destroy_comp_channel = nullptr;
    ibv_create_cq_fn create_cq = nullptr;
    ibv_destroy_cq_fn destroy_cq = nullptr;
    ibv_get_cq_event_fn get_cq_event = nullptr;
    ibv_ack_cq_events_fn ack_cq_events = nullptr;
    ibv_create_qp_fn create_qp = nullptr;
    ibv_destroy_qp_fn destroy_qp = nullptr;
    ibv_modify_qp_fn modify_qp = nullptr;
    ibv_query_port_fn query_port = nullptr;
    ibv_query_gid_fn query_gid = nullptr;

    // The symbols are resolved once per library path; a failed load is
    // retried with the next Open (the flag may have changed).
    bool Load(std::string* why) {
        std::lock_guard<std::mutex> g(mu);
        const std::string lib = FLAGS_rdma_verbs_library;
        if (handle && lib == loaded_from) return true;
        void* h = dlopen(lib.c_str(), RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            *why = lib + " not loadable";
            return false;
        }
#define MRPC_IBV_SYM(f)                                                         \
    f = reinterpret_cast<decltype(f)>(dlsym(h, "ibv_" #f));                     \
    if (!f) {                                                                   \
        *why = "missing ibv_" #f " in " + lib;                                  \
        return false;                                                           \
    }
        MRPC_IBV_SYM(get_device_list) MRPC_IBV_SYM(free_device_list) MRPC_IBV_SYM(get_device_name)
        MRPC_IBV_SYM(open_device) MRPC_IBV_SYM(close_device) MRPC_IBV_SYM(alloc_pd) MRPC_IBV_SYM(dealloc_pd)
        MRPC_IBV_SYM(reg_mr) MRPC_IBV_SYM(dereg_mr) MRPC_IBV_SYM(create_comp_channel)
        MRPC_IBV_SYM(destroy_comp_channel) MRPC_IBV_SYM(create_cq) MRPC_IBV_SYM(destroy_cq)
        MRPC_IBV_SYM(get_cq_event) MRPC_IBV_SYM(ack_cq_events) MRPC_IBV_SYM(create_qp) MRPC_IBV_SYM(destroy_qp)
        MRPC_IBV_SYM(modify_qp) MRPC_IBV_SYM(query_port) MRPC_IBV_SYM(query_gid)
#undef MRPC_IBV_SYM
        // optional: rdma-core >= 34 (GPUDirect through dmabuf)
        reg_dmabuf_mr = reinterpret_cast<ibv_reg_dmabuf_mr_fn>(dlsym(h, "ibv_reg_dmabuf_mr"));
        handle = h;  // never dlclose()d: contexts may outlive a provider
        loaded_from = lib;
        return true;
    }
    std::mutex mu;
};

IbvApi& api() {
    static IbvApi* a = new IbvApi;
    return *a;
}

class IbvCq : public CompletionQueue {
public:
    IbvCq(ibv_context* ctx, int depth) {
        _ch = api().create_comp_channel(ctx);
        if (!_ch) return;
        // the endpoint waits on the fd with the fiber poller and then
        // drains events: the channel must not block
        const int fl = fcntl(_ch->fd, F_GETFL);
        if (fl < 0 || fcntl(_ch->fd, F_SETFL, fl | O_NONBLOCK) < 0) return;
        _cq = api().create_cq(ctx, depth, nullptr, _ch, 0);
    }
    ~IbvCq() override {
        if (_cq) {
            if (_unacked) api().ack_cq_events(_cq, _unacked);
            api().destroy_cq(_cq);
        }
        if (_ch) api().destroy_comp_channel(_ch);
    }
    bool ok() const { return _cq != nullptr; }
    int Poll(WorkCompletion* out, int n) override {
        ibv_wc wc[32];
        const int k = _cq->context->ops.poll_cq(_cq, std::min(n, 32), wc);
        for (int i = 0; i < k; ++i) {
            out[i].wr_id = wc[i].wr_id;
            out[i].opcode = (wc[i].opcode & IBV_WC_RECV) ? WC_RECV : WC_SEND;
            out[i].status = wc[i].status;
            out[i].byte_len = wc[i].byte_len;
            out[i].has_imm = (wc[i].wc_flags & IBV_WC_WITH_IMM) != 0;
            out[i].imm = out[i].has_imm ? ntohl(wc[i].imm_data) : 0;
        }
        return k;
    }
    int Arm() override { return _cq->context->ops.req_notify_cq(_cq, 0); }
    int notify_fd() const override { return _ch->fd; }
    void AckEvent() override {
        // the channel fd is non-blocking, so this drains what is pending; acks are batched (ibv_ack_cq_events
        // takes a mutex in the library)
        ibv_cq* cq;
        void* ctx;
        while (api().get_cq_event(_ch, &cq, &ctx) == 0) {
            if (++_unacked >= 64) {
                api().ack_cq_events(_cq, _unacked);
                _unacked = 0;
            }
        }
    }
    ibv_cq* cq() const { return _cq; }

private:
    ibv_comp_channel* _ch = nullptr;
    ibv_cq* _cq = nullptr;
    unsigned _unacked = 0;
};

class IbvQp : public QueuePair {
public:
    IbvQp(ibv_pd* pd, IbvCq* cq, int sq, int rq, int max_sge, int port, const ibv_port_attr& pa, const ibv_gid& gid,
          int gid_index)
        : _port(port), _gid_index(gid_index), _max_sge(max_sge), _mtu(pa.active_mtu) {
        ibv_qp_init_attr a;
        memset(&a, 0, sizeof(a));
        a.send_cq = cq->cq();
        a.recv_cq = cq->cq();
        a.cap.max_send_wr = sq;
        a.cap.max_recv_wr = rq;
        a.cap.max_send_sge = max_sge;
        a.cap.max_recv_sge = 1;
        a.qp_type = IBV_QPT_RC;
        _qp = api().create_qp(pd, &a);
        memcpy(&_addr.gid_hi, gid.raw, 8);
        memcpy(&_addr.gid_lo, gid.raw + 8, 8);
        _addr.lid = pa.lid;
        if (_qp) _addr.qpn = _qp->qp_num;
    }
    ~IbvQp() override {
        if (_qp) api().destroy_qp(_qp);
    }
    bool ok() const { return _qp != nullptr; }
    QpAddress local() const override { return _addr; }
    int Prepare() override {
        if (_inited) return 0;
        ibv_qp_attr a;
        memset(&a, 0, sizeof(a));
        a.qp_state = IBV_QPS_INIT;
        a.port_num = _port;
        a.pkey_index = 0;
        a.qp_access_flags = IBV_ACCESS_LOCAL_WRITE;
        if (api().modify_qp(_qp, &a, IBV_QP_STATE | IBV_QP_PKEY_INDEX | IBV_QP_PORT | IBV_QP_ACCESS_FLAGS)) return -1;
        _inited = true;
        return 0;
    }
    // (RESET -> INIT via Prepare) -> RTR -> RTS (RC, reliable: retries and
    // infinite RNR retry — the credit window keeps receivers from running dry).
    int Connect(const QpAddress& r) override {
        if (Prepare() != 0) return -1;
        ibv_qp_attr a;
        memset(&a, 0, sizeof(a));
        a.qp_state = IBV_QPS_RTR;
        a.path_mtu = _mtu;
        a.dest_qp_num = r.qpn;
        a.rq_psn = 0;
        a.max_dest_rd_atomic = 1;
        a.min_rnr_timer = 12;
        a.ah_attr.is_global = 1;
        memcpy(a.ah_attr.grh.dgid.raw, &r.gid_hi, 8);
        memcpy(a.ah_attr.grh.dgid.raw + 8, &r.gid_lo, 8);
        a.ah_attr.grh.sgid_index = _gid_index;
        a.ah_attr.grh.hop_limit = 64;
        a.ah_attr.dlid = r.lid;
        a.ah_attr.port_num = _port;
        if (api().modify_qp(_qp, &a, IBV_QP_STATE | IBV_QP_AV | IBV_QP_PATH_MTU | IBV_QP_DEST_QPN | IBV_QP_RQ_PSN |
                                        IBV_QP_MAX_DEST_RD_ATOMIC | IBV_QP_MIN_RNR_TIMER)) {
            return -1;
        }
        memset(&a, 0, sizeof(a));
        a.qp_state = IBV_QPS_RTS;
        a.timeout = 14;
        a.retry_cnt = 7;
        a.rnr_retry = 7;
        a.sq_psn = 0;
        a.max_rd_atomic = 1;
        return api().modify_qp(_qp, &a, IBV_QP_STATE | IBV_QP_TIMEOUT | IBV_QP_RETRY_CNT | IBV_QP_RNR_RETRY |
                                             IBV_QP_SQ_PSN | IBV_QP_MAX_QP_RD_ATOMIC);
    }
    int PostSend(uint64_t wr_id, const Sge* sge, int nsge, bool with_imm, uint32_t imm, bool signaled) override {
        if (nsge > _max_sge || nsge > 16) return EINVAL;
        ibv_sge s[16];
        for (int i = 0; i < nsge; ++i) {
            s[i].addr = sge[i].addr;
            s[i].length = sge[i].length;
            s[i].lkey = sge[i].lkey;
        }
        ibv_send_wr wr, *bad = nullptr;
        memset(&wr, 0, sizeof(wr));
        wr.wr_id = wr_id;
        wr.sg_list = s;
        wr.num_sge = nsge;
        wr.opcode = with_imm ? IBV_WR_SEND_WITH_IMM : IBV_WR_SEND;
        wr.imm_data = htonl(imm);
        wr.send_flags = signaled ? IBV_SEND_SIGNALED : 0;
        return _qp->context->ops.post_send(_qp, &wr, &bad);
    }
    int PostRecv(uint64_t wr_id, const Sge& sge) override {
        ibv_sge s;
        s.addr = sge.addr;
        s.length = sge.length;
        s.lkey = sge.lkey;
        ibv_recv_wr wr, *bad = nullptr;
        memset(&wr, 0, sizeof(wr));
        wr.wr_id = wr_id;
        wr.sg_list = &s;
        wr.num_sge = 1;
        return _qp->context->ops.post_recv(_qp, &wr, &bad);
    }

private:
    ibv_qp* _qp = nullptr;
    bool _inited = false;
    int _port, _gid_index, _max_sge;
    ibv_mtu _mtu;
    QpAddress _addr;
};

class IbvProvider : public Provider {
public:
    ~IbvProvider() override {
        for (auto& kv : _mrs) api().dereg_mr(kv.second);
        if (_pd) api().dealloc_pd(_pd);
        if (_ctx) api().close_device(_ctx);
    }
    bool Open(std::string* why) {
        if (!api().Load(why)) return false;
        int n = 0;
        ibv_device** list = api().get_device_list(&n);
        if (!list || n == 0) {
            *why = "no RDMA device";
            if (list) api().free_device_list(list);
            return false;
        }
        for (int i = 0; i < n && !_ctx; ++i) {
            ibv_context* ctx = api().open_device(list[i]);
            if (!ctx) continue;
            for (int port = 1; port <= 2; ++port) {
                ibv_port_attr pa;
                memset(&pa, 0, sizeof(pa));
                if (api().query_port(ctx, (uint8_t)port, &pa) == 0 && pa.state == IBV_PORT_ACTIVE) {
                    _ctx = ctx;
                    _port = port;
                    _pa = pa;
                    _name = api().get_device_name(list[i]);
                    break;
                }
            }
            if (!_ctx) api().close_device(ctx);
        }
        api().free_device_list(list);
        if (!_ctx) {
            *why = "no active RDMA port";
            return false;
        }
        if (api().query_gid(_ctx, (uint8_t)_port, _gid_index, &_gid) != 0) {
            *why = "ibv_query_gid failed";
            return false;
        }
        _pd = api().alloc_pd(_ctx);
        if (!_pd) *why = "ibv_alloc_pd failed";
        return _pd != nullptr;
    }
    const char* name() const override { return "ibverbs"; }
    std::string device_name() const override { return _name; }
    int max_sge() const override { return 16; }
    int RegisterMemory(void* p, size_t n, bool device, int gpu, uint32_t* lkey) override {
        ibv_mr* mr = nullptr;
        const int access = IBV_ACCESS_LOCAL_WRITE;
        if (device) {
            // GPUDirect: HBM exported as a dmabuf by the HIP runtime
            DmabufExportFn exp = GetDmabufExportHook();
            int fd = -1;
            uint64_t off = 0;
            if (!api().reg_dmabuf_mr || !exp || exp(p, n, gpu, &fd, &off) != 0) return -1;
            mr = api().reg_dmabuf_mr(_pd, off, n, (uint64_t)(uintptr_t)p, fd, access);
        } else {
            mr = api().reg_mr(_pd, p, n, access);
        }
        if (!mr) return -1;
        std::lock_guard<std::mutex> g(_mu);
        _mrs[p] = mr;
        *lkey = mr->lkey;
        return 0;
    }
    void DeregisterMemory(void* p) override {
        std::lock_guard<std::mutex> g(_mu);
        auto it = _mrs.find(p);
        if (it == _mrs.end()) return;
        api().dereg_mr(it->second);
        _mrs.erase(it);
    }
    std::unique_ptr<CompletionQueue> CreateCq(int depth) override {
        std::unique_ptr<IbvCq> cq(new IbvCq(_ctx, depth));
        if (!cq->ok()) return nullptr;
        return std::unique_ptr<CompletionQueue>(cq.release());
    }
    std::unique_ptr<QueuePair> CreateQp(CompletionQueue* cq, int sq, int rq) override {
        std::unique_ptr<IbvQp> qp(
            new IbvQp(_pd, static_cast<IbvCq*>(cq), sq, rq, max_sge(), _port, _pa, _gid, _gid_index));
        if (!qp->ok()) return nullptr;
        return std::unique_ptr<QueuePair>(qp.release());
    }

private:
    ibv_context* _ctx = nullptr;
    ibv_pd* _pd = nullptr;
    int _port = 1;
    int _gid_index = 0;
    ibv_port_attr _pa;
    ibv_gid _gid;
    std::string _name;
    std::mutex _mu;
    std::map<void*, ibv_mr*> _mrs;
};

}  // namespace

bool IbverbsCompiledIn() { return true; }
std::unique_ptr<Provider> CreateIbverbsProvider(std::string* why) {
    std::unique_ptr<IbvProvider> p(new IbvProvider);
    if (!p->Open(why)) return nullptr;
    return std::unique_ptr<Provider>(p.release());
}

}  // namespace rdma
}  // namespace mrpc
