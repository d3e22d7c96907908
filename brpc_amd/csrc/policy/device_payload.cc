#include "policy/device_payload.h"

#include <algorithm>
#include <vector>

#include "base/logging.h"
#include "mrpc/proto/rpc_meta.pb.h"
#include "net/socket.h"
#include "rpc/controller.h"
#include "rpc/errno.h"

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

void StageDeviceBufToHost(const Buf& in, Buf* out) {
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

int LendDeviceBlocks(Socket* sock, const Buf& in, bool verify, Buf* host_out, DevicePayloads* descs,
                     std::string* err) {
    if (in.all_host_accessible()) {
        host_out->append(in);
        return 0;
    }
    const bool direct = HasDeviceTransport(sock);
    const int lent_before = descs->size();
    size_t pos = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
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
            const int rc = g_hooks.send(sock, r.block, r.offset, r.length, verify, d);
            if (rc > 0) {  // transport busy: stage this block inline
                descs->RemoveLast();
                Buf one;
                one.append_block(r.block, r.offset, r.length);
                StageDeviceBufToHost(one, host_out);
            } else if (rc != 0) {
                descs->RemoveLast();
                // blocks lent for this message so far will never be pulled
                for (int k = lent_before; k < descs->size(); ++k) {
                    if (g_hooks.cancel) g_hooks.cancel(descs->Get(k));
                }
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
                          std::string* err) {
    size_t total = 0;
    for (const auto& it : items) total += (size_t)it.first->size();
    if (total == 0) return 0;
    auto release_all = [&] {
        for (const auto& it : items) ReleaseDeviceBlocks(sock, *it.first);
    };
    if (!g_hooks.recv) {
        release_all();
        if (err) *err = "received device payload but no device transport is registered";
        return -1;
    }
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
    // one transport call (one batched pull) for every payload of every item
    std::vector<Buf> pulled(flat.size());
    if (g_hooks.recv(sock, flat.data(), (int)flat.size(), pulled.data()) != 0) {
        // the hook released every slot whatever happened
        if (err) *err = "fail to receive " + std::to_string(flat.size()) + " device payload(s)";
        return -1;
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

int PullDeviceBlocks(Socket* sock, const DevicePayloads& descs, Buf* attachment, std::string* err) {
    if (descs.size() == 0) return 0;
    return PullDeviceBlocksBatch(sock, {{&descs, attachment}}, err);
}

void ReleaseDeviceBlocks(Socket* sock, const DevicePayloads& descs) {
    if (!g_hooks.release || !sock) return;
    for (int i = 0; i < descs.size(); ++i) g_hooks.release(sock, descs.Get(i));
}

bool SplitDevicePayload(Controller* cntl, bool request, const Buf& attachment, Buf* host_out, RpcMeta* meta,
                        Socket* sock) {
    (void)request;
    if (!sock) sock = cntl->_pack_socket;
    std::string err;
    if (LendDeviceBlocks(sock, attachment, cntl->verify_device_payload(), host_out, meta->mutable_device_payload(),
                         &err) != 0) {
        cntl->SetFailed(EXGMI, "%s", err.c_str());
        return false;
    }
    return true;
}

bool MergeDevicePayload(Controller* cntl, Socket* sock, const RpcMeta& meta, bool request, Buf* attachment) {
    (void)request;
    std::string err;
    if (PullDeviceBlocks(sock, meta.device_payload(), attachment, &err) != 0) {
        cntl->SetFailed(EXGMI, "%s", err.c_str());
        return false;
    }
    return true;
}

void ReleaseDevicePayload(Socket* sock, const RpcMeta& meta) { ReleaseDeviceBlocks(sock, meta.device_payload()); }

void CancelDeviceBlocks(const DevicePayloads& descs) {
    if (!g_hooks.cancel) return;
    for (int i = 0; i < descs.size(); ++i) g_hooks.cancel(descs.Get(i));
}

void CancelDevicePayload(const RpcMeta& meta) { CancelDeviceBlocks(meta.device_payload()); }

}  // namespace policy
}  // namespace mrpc
