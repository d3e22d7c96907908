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
}

void SetDeviceTransportHooks(const DeviceTransportHooks& h) { g_hooks = h; }

bool HasDeviceTransport(Socket* sock) {
    return sock && g_hooks.send && sock->transport() != nullptr;
}

void StageDeviceBufToHost(const Buf& in, Buf* out) {
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

bool SplitDevicePayload(Controller* cntl, bool request, const Buf& attachment, Buf* host_out, RpcMeta* meta,
                        Socket* sock) {
    (void)request;
    if (attachment.all_host_accessible()) {
        host_out->append(attachment);
        return true;
    }
    if (!sock) sock = cntl->_pack_socket;
    const bool direct = HasDeviceTransport(sock);
    const int lent_before = meta->device_payload_size();
    size_t pos = 0;
    for (size_t i = 0; i < attachment.backing_block_num(); ++i) {
        const BlockRef& r = attachment.ref_at(i);
        if (IsHostAccessible(r.block->kind) || !direct) {
            if (IsHostAccessible(r.block->kind)) {
                host_out->append_block(r.block, r.offset, r.length);
            } else {
                Buf one;
                one.append_block(r.block, r.offset, r.length);
                StageDeviceBufToHost(one, host_out);
            }
        } else {
            DevicePayload* d = meta->add_device_payload();
            d->set_position((int64_t)pos);
            const int rc = g_hooks.send(sock, r.block, r.offset, r.length, cntl->verify_device_payload(), d);
            if (rc > 0) {  // transport busy: stage this block inline
                meta->mutable_device_payload()->RemoveLast();
                Buf one;
                one.append_block(r.block, r.offset, r.length);
                StageDeviceBufToHost(one, host_out);
            } else if (rc != 0) {
                meta->mutable_device_payload()->RemoveLast();
                // blocks lent for this message so far will never be pulled
                for (int k = lent_before; k < meta->device_payload_size(); ++k) {
                    if (g_hooks.cancel) g_hooks.cancel(meta->device_payload(k));
                }
                meta->mutable_device_payload()->Clear();
                cntl->SetFailed(EXGMI, "fail to send %u device bytes over %s", r.length, sock->description().c_str());
                return false;
            }
        }
        pos += r.length;
    }
    return true;
}

bool MergeDevicePayload(Controller* cntl, Socket* sock, const RpcMeta& meta, bool request, Buf* attachment) {
    (void)request;
    if (!g_hooks.recv) {
        cntl->SetFailed(EXGMI, "received device payload but no device transport is registered");
        return false;
    }
    const int n = meta.device_payload_size();
    std::vector<const DevicePayload*> descs;
    descs.reserve(n);
    for (int i = 0; i < n; ++i) descs.push_back(&meta.device_payload(i));
    std::sort(descs.begin(), descs.end(),
              [](const DevicePayload* a, const DevicePayload* b) { return a->position() < b->position(); });
    // positions must be consistent with the inline (host) part before any
    // payload is pulled, so a bad meta never leaves half-consumed slots
    int64_t cursor = 0, host_left = (int64_t)attachment->size();
    for (const DevicePayload* d : descs) {
        const int64_t nhost = d->position() - cursor;
        if (nhost < 0 || nhost > host_left || d->length() < 0) {
            ReleaseDevicePayload(sock, meta);
            cntl->SetFailed(ERESPONSE, "bad device payload position");
            return false;
        }
        host_left -= nhost;
        cursor += nhost + d->length();
    }
    std::vector<Buf> pulled(descs.size());
    if (g_hooks.recv(sock, descs.data(), (int)descs.size(), pulled.data()) != 0) {
        // the hook released every slot whatever happened
        cntl->SetFailed(EXGMI, "fail to receive %d device payload(s)", n);
        return false;
    }
    Buf host;
    host.swap(*attachment);
    cursor = 0;
    for (size_t i = 0; i < descs.size(); ++i) {
        const int64_t nhost = descs[i]->position() - cursor;
        host.cutn(attachment, (size_t)nhost);
        attachment->append(std::move(pulled[i]));
        cursor += nhost + descs[i]->length();
    }
    attachment->append(std::move(host));
    return true;
}

void ReleaseDevicePayload(Socket* sock, const RpcMeta& meta) {
    if (!g_hooks.release || !sock) return;
    for (int i = 0; i < meta.device_payload_size(); ++i) g_hooks.release(sock, meta.device_payload(i));
}

void CancelDevicePayload(const RpcMeta& meta) {
    if (!g_hooks.cancel) return;
    for (int i = 0; i < meta.device_payload_size(); ++i) g_hooks.cancel(meta.device_payload(i));
}

}  // namespace policy
}  // namespace mrpc
