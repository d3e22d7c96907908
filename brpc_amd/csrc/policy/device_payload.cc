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
            const int rc = g_hooks.send(sock, r.block->data + r.offset, r.length, r.block->device,
                                        cntl->verify_device_payload(), d);
            if (rc > 0) {  // transport busy (ring full): stage this block inline
                meta->mutable_device_payload()->RemoveLast();
                Buf one;
                one.append_block(r.block, r.offset, r.length);
                StageDeviceBufToHost(one, host_out);
            } else if (rc != 0) {
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
    std::vector<const DevicePayload*> descs;
    for (int i = 0; i < meta.device_payload_size(); ++i) descs.push_back(&meta.device_payload(i));
    std::sort(descs.begin(), descs.end(),
              [](const DevicePayload* a, const DevicePayload* b) { return a->position() < b->position(); });
    Buf host;
    host.swap(*attachment);
    int64_t cursor = 0;
    for (const DevicePayload* d : descs) {
        const int64_t nhost = d->position() - cursor;
        if (nhost < 0 || (size_t)nhost > host.size()) {
            cntl->SetFailed(ERESPONSE, "bad device payload position");
            return false;
        }
        host.cutn(attachment, (size_t)nhost);
        cursor += nhost;
        if (g_hooks.recv(sock, *d, attachment) != 0) {
            cntl->SetFailed(EXGMI, "fail to receive device payload of %lld bytes", (long long)d->length());
            return false;
        }
        cursor += d->length();
    }
    attachment->append(std::move(host));
    return true;
}

}  // namespace policy
}  // namespace mrpc
