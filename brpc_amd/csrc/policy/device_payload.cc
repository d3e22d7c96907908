#include "policy/device_payload.h"

#include <atomic>

#include <algorithm>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "gpu/rccl_plane.h"
#include "mrpc/proto/rpc_meta.pb.h"
#include "net/socket.h"
#include "rpc/controller.h"
#include "rpc/errno.h"

DEFINE_int64(rccl_min_bytes, int64_t(1) << 40,
             "attachment payloads of at least this many bytes to a rank of the job's RCCL plane move by "
             "ncclSend/ncclRecv (gpu/rccl_plane.h) instead of xGMI lending (reloadable; default: never)");

namespace mrpc {

namespace {
DeviceTransportHooks g_hooks;
int (*g_stage_hook)(const Buf& in, Buf* out) = nullptr;
}

void SetStageToHostHook(int (*fn)(const Buf& in, Buf* out)) { g_stage_hook = fn; }

void SetDeviceTransportHooks(const DeviceTransportHooks& h) { g_hooks = h; }

bool HasDeviceTransport(Socket* sock) {
    return sock && g_hooks.send && sock->transport() != nullptr;
}

std::atomic<int64_t> g_staged_payloads{0}, g_staged_bytes{0};

void GetStagedStats(int64_t* payloads, int64_t* bytes) {
    *payloads = g_staged_payloads.load(std::memory_order_relaxed);
    *bytes = g_staged_bytes.load(std::memory_order_relaxed);
}

void StageDeviceBufToHost(const Buf& in, Buf* out) {
    // device bytes that travel inline on the connection instead (no device
    // transport to the peer, or the transport refused them)
    g_staged_payloads.fetch_add(1, std::memory_order_relaxed);
    g_staged_bytes.fetch_add((int64_t)in.size(), std::memory_order_relaxed);
    // batched path: every device block in one launch into pinned memory
    if (g_stage_hook) {
        Buf staged;
        if (g_stage_hook(in, &staged) == 0) {
            out->append(std::move(staged));
            return;
        }
    }
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        if (IsHostAccessible(r.block->kind)) {
            out->append_block(r.block, r.offset, r.length);
        } else {
            char* p = out->append_contiguous(r.length);
            Buf tmp;
            tmp.append_block(r.block, r.offset, r.length);
            tmp.copy_to(p, r.length);  // device copy hook (hipMemcpy D2H)
        }
    }
}

namespace policy {

// One descriptor the receiver will not pull: a lent block goes back to the
// sender's release table, an RCCL payload is dropped from the plane's stash.
static void ReleaseOne(Socket* sock, const DevicePayload& d) {
    if (d.has_rccl_seq()) {
        gpu::rccl::Discard(d.rccl_src(), d.rccl_seq(), (size_t)std::max<int64_t>(0, d.length()));
        return;
    }
    if (g_hooks.release && sock) g_hooks.release(sock, d);
}

// One descriptor the sender made for a message that is never sent.
static void CancelOne(const DevicePayload& d) {
    if (d.has_rccl_seq()) {
        gpu::rccl::Cancelled(d.rccl_dst(), d.rccl_seq());
        return;
    }
    if (g_hooks.cancel) g_hooks.cancel(d);
}

namespace {

// Queue one payload on the RCCL plane and describe it. Host-memory planes
// (the CPU stub) take a run of host blocks, gathered when it spans several.
bool plane_send(int peer, const Buf& piece, int64_t pos, DevicePayloads* descs) {
    const size_t len = piece.size();
    Buf hold;
    const char* p = nullptr;
    if (piece.backing_block_num() == 1) {
        const BlockRef& r = piece.ref_at(0);
        p = r.block->data + r.offset;
        hold = piece;
    } else {
        char* dst = hold.append_contiguous(len);  // host planes only
        if (!dst) return false;
        piece.copy_to(dst, len);
        p = dst;
        if (hold.backing_block_num() != 1) return false;
    }
    const int64_t seq = gpu::rccl::Send(peer, p, len, std::move(hold));
    if (seq < 0) return false;
    DevicePayload* d = descs->Add();
    d->set_position(pos);
    d->set_length((int64_t)len);
    d->set_rccl_seq((uint64_t)seq);
    d->set_rccl_src(gpu::rccl::Rank());
    d->set_rccl_dst(peer);
    return true;
}

}  // namespace

int LendDeviceBlocks(Socket* sock, const Buf& in, const DeviceLendOptions& opt, Buf* host_out,
                     DevicePayloads* descs, std::string* err) {
    // the RCCL plane takes large payloads to a rank of our plane (never the
    // verified ones: the integrity check rides on the lending pull)
    const int prank = (!opt.verify && sock && in.size() >= (size_t)FLAGS_rccl_min_bytes) ? sock->plane_rank() : -1;
    const bool plane = prank >= 0 && gpu::rccl::Active();
    const bool host_plane = plane && gpu::rccl::HostMemory();
    if (in.all_host_accessible() && !host_plane) {
        host_out->append(in);
        return 0;
    }
    const bool direct = HasDeviceTransport(sock);
    const int lent_before = descs->size();
    size_t pos = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        if (host_plane && IsHostAccessible(r.block->kind)) {
            // the run of host blocks starting here
            size_t j = i, run = 0;
            while (j < in.backing_block_num() && IsHostAccessible(in.ref_at(j).block->kind)) run += in.ref_at(j++).length;
            if (run >= (size_t)FLAGS_rccl_min_bytes) {
                Buf piece;
                for (size_t k = i; k < j; ++k) piece.append_block(in.ref_at(k).block, in.ref_at(k).offset, in.ref_at(k).length);
                if (plane_send(prank, piece, (int64_t)pos, descs)) {
                    pos += run;
                    i = j - 1;
                    continue;
                }
            }
        }
        if (plane && !host_plane && r.length >= (uint64_t)FLAGS_rccl_min_bytes && gpu::rccl::AcceptsBlock(r.block)) {
            Buf piece;
            piece.append_block(r.block, r.offset, r.length);
            if (plane_send(prank, piece, (int64_t)pos, descs)) {
                pos += r.length;
                continue;
            }
        }
        if (IsHostAccessible(r.block->kind) || !direct) {
            if (IsHostAccessible(r.block->kind)) {
                host_out->append_block(r.block, r.offset, r.length);
            } else {
                Buf one;
                one.append_block(r.block, r.offset, r.length);
                StageDeviceBufToHost(one, host_out);
            }
        } else {
            DevicePayload* d = descs->Add();
            d->set_position((int64_t)pos);
            const int rc = g_hooks.send(sock, r.block, r.offset, r.length, opt, d);
            if (rc > 0) {  // transport busy: stage this block inline
                descs->RemoveLast();
                Buf one;
                one.append_block(r.block, r.offset, r.length);
                StageDeviceBufToHost(one, host_out);
            } else if (rc != 0) {
                descs->RemoveLast();
                // blocks lent for this message so far will never be pulled
                for (int k = lent_before; k < descs->size(); ++k) CancelOne(descs->Get(k));
                while (descs->size() > lent_before) descs->RemoveLast();
                if (err) *err = "fail to send " + std::to_string(r.length) + " device bytes over " + sock->description();
                return -1;
            }
        }
        pos += r.length;
    }
    return 0;
}

int PullDeviceBlocksBatch(Socket* sock, const std::vector<std::pair<const DevicePayloads*, Buf*>>& items,
                          std::string* err, std::vector<DevicePayloadIndex>* indexes) {
    if (indexes) indexes->assign(items.size(), DevicePayloadIndex());
    size_t total = 0;
    for (const auto& it : items) total += (size_t)it.first->size();
    if (total == 0) return 0;
    auto release_all = [&] {
        for (const auto& it : items) ReleaseDeviceBlocks(sock, *it.first);
    };
    // per item: descriptors sorted by position, validated against the
    // inline (host) part before anything is pulled, so a bad meta never
    // leaves half-consumed slots
    std::vector<std::vector<const DevicePayload*>> sorted(items.size());
    std::vector<const DevicePayload*> flat;
    flat.reserve(total);
    for (size_t k = 0; k < items.size(); ++k) {
        const DevicePayloads& d = *items[k].first;
        std::vector<const DevicePayload*>& v = sorted[k];
        for (int i = 0; i < d.size(); ++i) v.push_back(&d.Get(i));
        std::sort(v.begin(), v.end(),
                  [](const DevicePayload* a, const DevicePayload* b) { return a->position() < b->position(); });
        int64_t cursor = 0, host_left = (int64_t)items[k].second->size();
        for (const DevicePayload* x : v) {
            const int64_t nhost = x->position() - cursor;
            if (nhost < 0 || nhost > host_left || x->length() < 0) {
                release_all();
                if (err) *err = "bad device payload position";
                return -1;
            }
            host_left -= nhost;
            cursor += nhost + x->length();
        }
        flat.insert(flat.end(), v.begin(), v.end());
    }
    // one transport call (one batched pull) for every lent payload of every
    // item; payloads that travel over the RCCL plane are claimed after it
    std::vector<Buf> pulled(flat.size());
    std::vector<const DevicePayload*> lent;
    std::vector<size_t> lent_at, plane_at;
    for (size_t i = 0; i < flat.size(); ++i) {
        if (flat[i]->has_rccl_seq()) plane_at.push_back(i);
        else {
            lent.push_back(flat[i]);
            lent_at.push_back(i);
        }
    }
    auto discard_plane = [&] {
        for (size_t i : plane_at) ReleaseOne(sock, *flat[i]);
    };
    bool bad_plane = false;
    for (size_t i : plane_at) {
        const DevicePayload& d = *flat[i];
        bad_plane |= d.rccl_dst() != gpu::rccl::Rank() || d.rccl_src() != sock->plane_rank() || d.length() <= 0;
    }
    if (bad_plane) {
        release_all();
        if (err) *err = "bad RCCL plane payload descriptor";
        return -1;
    }
    if (!lent.empty()) {
        if (!g_hooks.recv) {
            release_all();
            if (err) *err = "received device payload but no device transport is registered";
            return -1;
        }
        std::vector<Buf> got(lent.size());
        bool any_scan = false;
        for (const DevicePayload* x : lent) any_scan |= x->pb_scan();
        std::vector<DevicePayloadIndex> idx(indexes && any_scan ? lent.size() : 0);
        if (g_hooks.recv(sock, lent.data(), (int)lent.size(), got.data(), idx.empty() ? nullptr : idx.data()) != 0) {
            // the hook released every lent slot whatever happened
            discard_plane();
            if (err) *err = "fail to receive " + std::to_string(lent.size()) + " device payload(s)";
            return -1;
        }
        for (size_t k = 0; k < lent.size(); ++k) pulled[lent_at[k]] = std::move(got[k]);
        if (!idx.empty()) {
            // flat index -> item: the first scanned payload of each item
            for (size_t k = 0, at = 0, item = 0; k < lent.size(); ++k) {
                while (item + 1 < items.size() && lent_at[k] >= at + sorted[item].size()) at += sorted[item++].size();
                if (lent[k]->pb_scan() && (*indexes)[item].nfields < 0 && idx[k].nfields >= 0)
                    (*indexes)[item] = std::move(idx[k]);
            }
        }
    }
    if (!plane_at.empty()) {
        std::vector<int> src;
        std::vector<uint64_t> seq;
        std::vector<size_t> len;
        for (size_t i : plane_at) {
            src.push_back(flat[i]->rccl_src());
            seq.push_back(flat[i]->rccl_seq());
            len.push_back((size_t)flat[i]->length());
        }
        std::vector<Buf> got(plane_at.size());
        if (gpu::rccl::Recv((int)plane_at.size(), src.data(), seq.data(), len.data(), got.data()) != 0) {
            if (err) *err = "fail to receive " + std::to_string(plane_at.size()) + " RCCL plane payload(s)";
            return -1;
        }
        for (size_t k = 0; k < plane_at.size(); ++k) pulled[plane_at[k]] = std::move(got[k]);
    }
    size_t at = 0;
    for (size_t k = 0; k < items.size(); ++k) {
        Buf* attachment = items[k].second;
        Buf host;
        host.swap(*attachment);
        int64_t cursor = 0;
        for (const DevicePayload* x : sorted[k]) {
            const int64_t nhost = x->position() - cursor;
            host.cutn(attachment, (size_t)nhost);
            attachment->append(std::move(pulled[at++]));
            cursor += nhost + x->length();
        }
        attachment->append(std::move(host));
    }
    return 0;
}

int PullDeviceBlocks(Socket* sock, const DevicePayloads& descs, Buf* attachment, std::string* err,
                     DevicePayloadIndex* index) {
    if (descs.size() == 0) return 0;
    if (!index) return PullDeviceBlocksBatch(sock, {{&descs, attachment}}, err);
    std::vector<DevicePayloadIndex> idx;
    const int rc = PullDeviceBlocksBatch(sock, {{&descs, attachment}}, err, &idx);
    if (rc == 0 && !idx.empty()) *index = std::move(idx[0]);
    return rc;
}

void ReleaseDeviceBlocks(Socket* sock, const DevicePayloads& descs) {
    for (int i = 0; i < descs.size(); ++i) ReleaseOne(sock, descs.Get(i));
}

bool SplitDevicePayload(Controller* cntl, bool request, const Buf& attachment, Buf* host_out, RpcMeta* meta,
                        Socket* sock) {
    if (!sock) sock = cntl->_pack_socket;
    std::string err;
    DeviceLendOptions opt;
    opt.verify = cntl->verify_device_payload();
    opt.compress = (int)cntl->device_payload_compress_type();
    opt.scan = cntl->device_payload_scan();
    if (LendDeviceBlocks(sock, attachment, opt, host_out, meta->mutable_device_payload(), &err) != 0) {
        cntl->SetFailed(EXGMI, "%s", err.c_str());
        return false;
    }
    if (request) {
        if (meta->device_payload_size() > 0) {
            if (!cntl->_packed_payloads) cntl->_packed_payloads.reset(new PackedPayloads);
            DevicePayloads& d = cntl->_packed_payloads->descs;
            d.Clear();
            for (const DevicePayload& x : meta->device_payload()) d.Add()->CopyFrom(x);
        } else if (cntl->_packed_payloads) {
            cntl->_packed_payloads->descs.Clear();
        }
    }
    return true;
}

bool MergeDevicePayload(Controller* cntl, Socket* sock, const RpcMeta& meta, bool request, Buf* attachment) {
    (void)request;
    std::string err;
    bool scanned = false;
    CompressType got = COMPRESS_TYPE_NONE;
    for (const DevicePayload& x : meta.device_payload()) {
        scanned |= x.pb_scan();
        if (x.compress_type()) got = (CompressType)x.compress_type();
    }
    cntl->_device_payload_index.nfields = -1;
    cntl->_device_payload_index.fields.clear();
    cntl->_received_device_compress = got;
    if (PullDeviceBlocks(sock, meta.device_payload(), attachment, &err,
                         scanned ? &cntl->_device_payload_index : nullptr) != 0) {
        cntl->SetFailed(EXGMI, "%s", err.c_str());
        return false;
    }
    return true;
}

void ReleaseDevicePayload(Socket* sock, const RpcMeta& meta) { ReleaseDeviceBlocks(sock, meta.device_payload()); }

void CancelDeviceBlocks(const DevicePayloads& descs) {
    for (int i = 0; i < descs.size(); ++i) CancelOne(descs.Get(i));
}

void CancelDevicePayload(const RpcMeta& meta) { CancelDeviceBlocks(meta.device_payload()); }

}  // namespace policy
}  // namespace mrpc
