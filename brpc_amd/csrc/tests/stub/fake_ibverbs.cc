// Stub verbs library (libfake_ibverbs.so) implementing the libibverbs ABI
// subset declared in rdma/verbs_abi.h, for the ibverbs-provider unit tests
// (tests/rdma_unittest.cc RdmaVerbs.*): the provider dlopen()s it through
// -rdma_verbs_library exactly as it would libibverbs.so.1.
//
// One device ("fake_mlx5_0", port 1 ACTIVE, RoCE-style GID) and an
// in-process reliable-connected fabric. The library checks what a real HCA
// would refuse: QP state machine and the attribute masks of every
// transition, the destination GID/LID of RTR, posting on a QP that is not
// RTS (send) / RESET (recv), lkeys that do not cover an SGE, more SGEs than
// the QP's capability, receive buffers too small for the message, and the
// channel/notify protocol (an event only after req_notify_cq, consumed by
// ibv_get_cq_event, acknowledged with ibv_ack_cq_events before destroy).
// SENDs with no posted RECV are held (RNR retry) until one is posted.
#include <errno.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <vector>

#include "rdma/verbs_abi.h"

using namespace mrpc::rdma::verbs;

namespace {

const uint16_t kLid = 7;
const uint64_t kGidPrefix = 0x80feull;  // fe80:: (little-endian store of the first 8 bytes)

struct FakeDevice {
    int dummy;
};
FakeDevice g_dev;

struct FakeCq;
struct FakeChannel {
    ibv_comp_channel base;
    std::deque<FakeCq*> fired;
};

struct FakeCq {
    ibv_cq base;
    std::deque<ibv_wc> q;
    int depth;
    bool armed = false;
    unsigned events = 0, acked = 0;
    int overruns = 0;
};

struct FakeQp;
struct PendingSend {
    FakeQp* src;
    ibv_send_wr wr;
    std::vector<ibv_sge> sge;
};

struct FakeQp {
    ibv_qp base;
    ibv_qp_cap cap;
    uint32_t dest_qpn = 0;
    std::deque<std::pair<uint64_t, ibv_sge>> recvs;
    std::deque<PendingSend> held;  // RNR: waiting for a RECV at this QP
};

struct Region {
    uintptr_t addr;
    size_t len;
    bool dmabuf;
};

struct Fabric {
    std::recursive_mutex mu;
    std::map<uint32_t, FakeQp*> qps;
    std::map<uint32_t, Region> mrs;  // lkey -> region
    uint32_t next_qpn = 0x40, next_key = 0x1000, next_handle = 1;
    int open_contexts = 0, live_pds = 0, live_cqs = 0, live_qps = 0, live_channels = 0;
    long sends = 0, recvs = 0, bytes = 0, rnr_holds = 0, errors = 0, dmabuf_regs = 0, events = 0;
};
Fabric& fab() {
    static Fabric* f = new Fabric;
    return *f;
}

void push_wc(FakeCq* cq, const ibv_wc& wc) {
    if ((int)cq->q.size() >= cq->depth) ++cq->overruns;
    cq->q.push_back(wc);
    if (cq->armed && cq->base.channel) {
        cq->armed = false;
        auto* ch = reinterpret_cast<FakeChannel*>(cq->base.channel);
        ch->fired.push_back(cq);
        ++cq->events;
        ++fab().events;
        uint64_t one = 1;
        ssize_t r = write(ch->base.fd, &one, sizeof(one));
        (void)r;
    }
}

bool covered(const ibv_sge& s) {
    auto it = fab().mrs.find(s.lkey);
    if (it == fab().mrs.end()) return false;
    return s.addr >= it->second.addr && s.addr + s.length <= it->second.addr + it->second.len;
}

ibv_wc make_wc(uint64_t wr_id, int status, ibv_wc_opcode op, uint32_t len, uint32_t qpn) {
    ibv_wc wc;
    memset(&wc, 0, sizeof(wc));
    wc.wr_id = wr_id;
    wc.status = (ibv_wc_status)status;
    wc.opcode = op;
    wc.byte_len = len;
    wc.qp_num = qpn;
    return wc;
}

// Deliver one SEND into the oldest RECV of `dst` (caller checked there is one).
void deliver(FakeQp* dst, PendingSend& ps) {
    auto r = dst->recvs.front();
    dst->recvs.pop_front();
    size_t total = 0;
    for (auto& s : ps.sge) total += s.length;
    auto* rcq = reinterpret_cast<FakeCq*>(dst->base.recv_cq);
    auto* scq = reinterpret_cast<FakeCq*>(ps.src->base.send_cq);
    if (total > r.second.length) {
        ++fab().errors;
        push_wc(rcq, make_wc(r.first, 1 /*LOC_LEN_ERR*/, IBV_WC_RECV, 0, dst->base.qp_num));
        push_wc(scq, make_wc(ps.wr.wr_id, 9 /*REM_INV_REQ_ERR*/, IBV_WC_SEND, 0, ps.src->base.qp_num));
        return;
    }
    char* out = reinterpret_cast<char*>(r.second.addr);
    for (auto& s : ps.sge) {
        memcpy(out, reinterpret_cast<const void*>(s.addr), s.length);
        out += s.length;
    }
    ibv_wc wc = make_wc(r.first, IBV_WC_SUCCESS, IBV_WC_RECV, (uint32_t)total, dst->base.qp_num);
    wc.src_qp = ps.src->base.qp_num;
    if (ps.wr.opcode == IBV_WR_SEND_WITH_IMM) {
        wc.wc_flags |= IBV_WC_WITH_IMM;
        wc.imm_data = ps.wr.imm_data;
    }
    push_wc(rcq, wc);
    ++fab().recvs;
    fab().bytes += (long)total;
    if (ps.wr.send_flags & IBV_SEND_SIGNALED) {
        push_wc(scq, make_wc(ps.wr.wr_id, IBV_WC_SUCCESS, IBV_WC_SEND, (uint32_t)total, ps.src->base.qp_num));
    }
}

int fake_poll_cq(ibv_cq* cq, int n, ibv_wc* wc) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    auto* c = reinterpret_cast<FakeCq*>(cq);
    int k = 0;
    while (k < n && !c->q.empty()) {
        wc[k++] = c->q.front();
        c->q.pop_front();
    }
    return k;
}

int fake_req_notify_cq(ibv_cq* cq, int) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    reinterpret_cast<FakeCq*>(cq)->armed = true;
    return 0;
}

int fake_post_send(ibv_qp* qp, ibv_send_wr* wr, ibv_send_wr** bad) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    auto* q = reinterpret_cast<FakeQp*>(qp);
    for (; wr; wr = wr->next) {
        if (q->base.state != IBV_QPS_RTS || (wr->opcode != IBV_WR_SEND && wr->opcode != IBV_WR_SEND_WITH_IMM) ||
            wr->num_sge < 0 || (uint32_t)wr->num_sge > q->cap.max_send_sge) {
            ++fab().errors;
            *bad = wr;
            return EINVAL;
        }
        PendingSend ps{q, *wr, {}};
        for (int i = 0; i < wr->num_sge; ++i) {
            if (!covered(wr->sg_list[i])) {
                ++fab().errors;
                *bad = wr;
                return EINVAL;  // a real HCA completes with LOC_PROT_ERR; fail loudly here
            }
            ps.sge.push_back(wr->sg_list[i]);
        }
        ps.wr.sg_list = nullptr;
        ps.wr.next = nullptr;
        ++fab().sends;
        auto it = fab().qps.find(q->dest_qpn);
        if (it == fab().qps.end()) {
            ++fab().errors;
            push_wc(reinterpret_cast<FakeCq*>(q->base.send_cq),
                    make_wc(wr->wr_id, 12 /*RETRY_EXC_ERR*/, IBV_WC_SEND, 0, q->base.qp_num));
            continue;
        }
        FakeQp* dst = it->second;
        if (dst->recvs.empty() || !dst->held.empty()) {
            ++fab().rnr_holds;
            dst->held.push_back(std::move(ps));
        } else {
            deliver(dst, ps);
        }
    }
    return 0;
}

int fake_post_recv(ibv_qp* qp, ibv_recv_wr* wr, ibv_recv_wr** bad) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    auto* q = reinterpret_cast<FakeQp*>(qp);
    for (; wr; wr = wr->next) {
        if (q->base.state == IBV_QPS_RESET || q->base.state == IBV_QPS_ERR || wr->num_sge != 1 ||
            !covered(wr->sg_list[0]) || q->recvs.size() >= q->cap.max_recv_wr) {
            ++fab().errors;
            *bad = wr;
            return EINVAL;
        }
        q->recvs.emplace_back(wr->wr_id, wr->sg_list[0]);
        while (!q->held.empty() && !q->recvs.empty()) {
            PendingSend ps = std::move(q->held.front());
            q->held.pop_front();
            deliver(q, ps);
        }
    }
    return 0;
}

int fake_post_srq_recv(ibv_srq*, ibv_recv_wr*, ibv_recv_wr**) { return ENOSYS; }

}  // namespace

extern "C" {

__attribute__((visibility("default"))) ibv_device** ibv_get_device_list(int* n) {
    ibv_device** l = new ibv_device*[2];
    l[0] = reinterpret_cast<ibv_device*>(&g_dev);
    l[1] = nullptr;
    if (n) *n = 1;
    return l;
}
__attribute__((visibility("default"))) void ibv_free_device_list(ibv_device** l) { delete[] l; }
__attribute__((visibility("default"))) const char* ibv_get_device_name(ibv_device*) { return "fake_mlx5_0"; }

__attribute__((visibility("default"))) ibv_context* ibv_open_device(ibv_device* d) {
    if (d != reinterpret_cast<ibv_device*>(&g_dev)) return nullptr;
    ibv_context* c = new ibv_context;
    memset(c, 0, sizeof(*c));
    c->device = d;
    c->ops.poll_cq = fake_poll_cq;
    c->ops.req_notify_cq = fake_req_notify_cq;
    c->ops.post_send = fake_post_send;
    c->ops.post_recv = fake_post_recv;
    c->ops.post_srq_recv = fake_post_srq_recv;
    c->cmd_fd = c->async_fd = -1;
    c->num_comp_vectors = 1;
    pthread_mutex_init(&c->mutex, nullptr);
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    ++fab().open_contexts;
    return c;
}
__attribute__((visibility("default"))) int ibv_close_device(ibv_context* c) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    --fab().open_contexts;
    delete c;
    return 0;
}

__attribute__((visibility("default"))) int ibv_query_port(ibv_context*, uint8_t port, ibv_port_attr* a) {
    if (port != 1) return EINVAL;
    // write only the legacy (pre-extension) part, as the exported
    // IBVERBS_1.1 symbol of the real library does
    memset(a, 0, offsetof(ibv_port_attr, port_cap_flags2));
    a->state = IBV_PORT_ACTIVE;
    a->max_mtu = IBV_MTU_4096;
    a->active_mtu = IBV_MTU_4096;
    a->gid_tbl_len = 1;
    a->lid = kLid;
    a->link_layer = 2;  // Ethernet (RoCE)
    return 0;
}

__attribute__((visibility("default"))) int ibv_query_gid(ibv_context*, uint8_t port, int index, ibv_gid* gid) {
    if (port != 1 || index != 0) return EINVAL;
    memset(gid, 0, sizeof(*gid));
    memcpy(gid->raw, &kGidPrefix, 8);
    const uint64_t id = 0x0202c9fffe000001ull;
    memcpy(gid->raw + 8, &id, 8);
    return 0;
}

__attribute__((visibility("default"))) ibv_pd* ibv_alloc_pd(ibv_context* c) {
    ibv_pd* pd = new ibv_pd;
    pd->context = c;
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    pd->handle = fab().next_handle++;
    ++fab().live_pds;
    return pd;
}
__attribute__((visibility("default"))) int ibv_dealloc_pd(ibv_pd* pd) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    --fab().live_pds;
    delete pd;
    return 0;
}

static ibv_mr* new_mr(ibv_pd* pd, uintptr_t addr, size_t len, bool dmabuf) {
    ibv_mr* mr = new ibv_mr;
    memset(mr, 0, sizeof(*mr));
    mr->context = pd->context;
    mr->pd = pd;
    mr->addr = reinterpret_cast<void*>(addr);
    mr->length = len;
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    mr->handle = fab().next_handle++;
    mr->lkey = mr->rkey = fab().next_key++;
    fab().mrs[mr->lkey] = Region{addr, len, dmabuf};
    return mr;
}

__attribute__((visibility("default"))) ibv_mr* ibv_reg_mr(ibv_pd* pd, void* addr, size_t len, int access) {
    if (!pd || !addr || !len || !(access & IBV_ACCESS_LOCAL_WRITE)) {
        errno = EINVAL;
        return nullptr;
    }
    return new_mr(pd, reinterpret_cast<uintptr_t>(addr), len, false);
}

// dmabuf registration: the stub reads the range at `iova` directly, which
// the tests back with host memory (their export hook hands out a memfd).
__attribute__((visibility("default"))) ibv_mr* ibv_reg_dmabuf_mr(ibv_pd* pd, uint64_t offset, size_t len,
                                                                 uint64_t iova, int fd, int access) {
    if (!pd || fd < 0 || !len || !(access & IBV_ACCESS_LOCAL_WRITE)) {
        errno = EINVAL;
        return nullptr;
    }
    (void)offset;
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    ++fab().dmabuf_regs;
    return new_mr(pd, (uintptr_t)iova, len, true);
}

__attribute__((visibility("default"))) int ibv_dereg_mr(ibv_mr* mr) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    fab().mrs.erase(mr->lkey);
    delete mr;
    return 0;
}

__attribute__((visibility("default"))) ibv_comp_channel* ibv_create_comp_channel(ibv_context* c) {
    auto* ch = new FakeChannel;
    ch->base.context = c;
    ch->base.fd = eventfd(0, EFD_CLOEXEC);  // blocking, like the real channel fd
    ch->base.refcnt = 0;
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    ++fab().live_channels;
    return &ch->base;
}
__attribute__((visibility("default"))) int ibv_destroy_comp_channel(ibv_comp_channel* c) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    if (c->refcnt) return EBUSY;
    close(c->fd);
    delete reinterpret_cast<FakeChannel*>(c);
    --fab().live_channels;
    return 0;
}

__attribute__((visibility("default"))) ibv_cq* ibv_create_cq(ibv_context* c, int cqe, void* ctx, ibv_comp_channel* ch,
                                                             int) {
    auto* cq = new FakeCq;
    memset(&cq->base, 0, sizeof(cq->base));
    cq->base.context = c;
    cq->base.channel = ch;
    cq->base.cq_context = ctx;
    cq->base.cqe = cqe;
    cq->depth = cqe;
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    cq->base.handle = fab().next_handle++;
    if (ch) ++ch->refcnt;
    ++fab().live_cqs;
    return &cq->base;
}
__attribute__((visibility("default"))) int ibv_destroy_cq(ibv_cq* cq) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    auto* c = reinterpret_cast<FakeCq*>(cq);
    if (c->acked != c->events) return EBUSY;  // the real library blocks here forever
    if (cq->channel) {
        --cq->channel->refcnt;
        auto& f = reinterpret_cast<FakeChannel*>(cq->channel)->fired;
        for (auto it = f.begin(); it != f.end();) it = (*it == c) ? f.erase(it) : std::next(it);
    }
    delete c;
    --fab().live_cqs;
    return 0;
}

__attribute__((visibility("default"))) int ibv_get_cq_event(ibv_comp_channel* ch, ibv_cq** cq, void** ctx) {
    uint64_t v;
    auto* c = reinterpret_cast<FakeChannel*>(ch);
    {
        std::lock_guard<std::recursive_mutex> g(fab().mu);
        if (!c->fired.empty()) {
            FakeCq* f = c->fired.front();
            c->fired.pop_front();
            if (c->fired.empty()) {
                ssize_t r = read(ch->fd, &v, sizeof(v));  // clears readiness (non-blocking when set)
                (void)r;
            }
            *cq = &f->base;
            *ctx = f->base.cq_context;
            return 0;
        }
    }
    // nothing fired: a blocking fd would wait here, a non-blocking one fails
    if (read(ch->fd, &v, sizeof(v)) < 0) return -1;
    return -1;
}

__attribute__((visibility("default"))) void ibv_ack_cq_events(ibv_cq* cq, unsigned int n) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    reinterpret_cast<FakeCq*>(cq)->acked += n;
}

__attribute__((visibility("default"))) ibv_qp* ibv_create_qp(ibv_pd* pd, ibv_qp_init_attr* a) {
    if (a->qp_type != IBV_QPT_RC || !a->send_cq || !a->recv_cq || a->cap.max_send_sge > 30 ||
        a->cap.max_recv_sge > 30 || a->cap.max_send_wr == 0 || a->cap.max_recv_wr == 0) {
        errno = EINVAL;
        return nullptr;
    }
    auto* q = new FakeQp;
    memset(&q->base, 0, sizeof(q->base));
    q->base.context = pd->context;
    q->base.qp_context = a->qp_context;
    q->base.pd = pd;
    q->base.send_cq = a->send_cq;
    q->base.recv_cq = a->recv_cq;
    q->base.state = IBV_QPS_RESET;
    q->base.qp_type = IBV_QPT_RC;
    q->cap = a->cap;
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    q->base.handle = fab().next_handle++;
    q->base.qp_num = fab().next_qpn++;
    fab().qps[q->base.qp_num] = q;
    ++fab().live_qps;
    return &q->base;
}

__attribute__((visibility("default"))) int ibv_destroy_qp(ibv_qp* qp) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    fab().qps.erase(qp->qp_num);
    delete reinterpret_cast<FakeQp*>(qp);
    --fab().live_qps;
    return 0;
}

__attribute__((visibility("default"))) int ibv_modify_qp(ibv_qp* qp, ibv_qp_attr* a, int mask) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    auto* q = reinterpret_cast<FakeQp*>(qp);
    if (!(mask & IBV_QP_STATE)) return EINVAL;
    auto need = [&](int m) { return (mask & m) == m; };
    const ibv_qp_state from = qp->state, to = a->qp_state;
    bool ok = false;
    if (to == IBV_QPS_ERR || to == IBV_QPS_RESET) {
        ok = true;
    } else if (from == IBV_QPS_RESET && to == IBV_QPS_INIT) {
        ok = need(IBV_QP_PKEY_INDEX | IBV_QP_PORT | IBV_QP_ACCESS_FLAGS) && a->port_num == 1;
    } else if (from == IBV_QPS_INIT && to == IBV_QPS_RTR) {
        uint64_t prefix;
        memcpy(&prefix, a->ah_attr.grh.dgid.raw, 8);
        ok = need(IBV_QP_AV | IBV_QP_PATH_MTU | IBV_QP_DEST_QPN | IBV_QP_RQ_PSN | IBV_QP_MAX_DEST_RD_ATOMIC |
                  IBV_QP_MIN_RNR_TIMER) &&
             a->path_mtu >= IBV_MTU_256 && a->path_mtu <= IBV_MTU_4096 && a->ah_attr.port_num == 1 &&
             a->ah_attr.is_global && prefix == kGidPrefix && a->ah_attr.dlid == kLid && a->dest_qp_num != 0;
        if (ok) q->dest_qpn = a->dest_qp_num;
    } else if (from == IBV_QPS_RTR && to == IBV_QPS_RTS) {
        ok = need(IBV_QP_TIMEOUT | IBV_QP_RETRY_CNT | IBV_QP_RNR_RETRY | IBV_QP_SQ_PSN | IBV_QP_MAX_QP_RD_ATOMIC) &&
             a->retry_cnt <= 7 && a->rnr_retry <= 7;
    }
    if (!ok) {
        ++fab().errors;
        return EINVAL;
    }
    qp->state = to;
    return 0;
}

// Test introspection (not part of the verbs ABI).
struct FakeIbvStats {
    long sends, recvs, bytes, rnr_holds, errors, dmabuf_regs, events;
    int open_contexts, live_pds, live_cqs, live_qps, live_channels, live_mrs;
};
__attribute__((visibility("default"))) void fake_ibv_stats(FakeIbvStats* s) {
    std::lock_guard<std::recursive_mutex> g(fab().mu);
    Fabric& f = fab();
    *s = FakeIbvStats{f.sends,         f.recvs,    f.bytes,    f.rnr_holds, f.errors,        f.dmabuf_regs,
                      f.events,        f.open_contexts, f.live_pds, f.live_cqs, f.live_qps, f.live_channels,
                      (int)f.mrs.size()};
}

}  // extern "C"
