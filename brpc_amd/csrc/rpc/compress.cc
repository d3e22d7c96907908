#include "rpc/compress.h"

#include <zlib.h>

#include <atomic>
#include <mutex>

#include "base/logging.h"
#include "base/snappy.h"
#include "pb/message.h"

namespace mrpc {

namespace {
CompressHandler g_handlers[16];
std::atomic<SnappyOffload> g_snappy_offload{nullptr};
size_t g_snappy_offload_min = (size_t)-1;

bool snappy_compress(const Buf& in, Buf* out) {
    SnappyOffload off = g_snappy_offload.load(std::memory_order_acquire);
    if (off && in.size() >= g_snappy_offload_min && off(in, out, true)) return true;
    std::string src = in.to_string();
    std::string dst;
    if (!snappy::Compress(src.data(), src.size(), &dst)) return false;
    out->append(dst);
    return true;
}

// Uncompressed length from the stream's varint header (0 if malformed).
size_t snappy_ulen(const Buf& in) {
    unsigned char h[5];
    const size_t n = in.copy_to(h, sizeof(h));
    size_t v = 0;
    for (size_t i = 0; i < n; ++i) {
        v |= (size_t)(h[i] & 0x7f) << (7 * i);
        if (!(h[i] & 0x80)) return v;
    }
    return 0;
}

bool snappy_decompress(const Buf& in, Buf* out) {
    SnappyOffload off = g_snappy_offload.load(std::memory_order_acquire);
    // offload by the work (the uncompressed size), not the wire size
    if (off && snappy_ulen(in) >= g_snappy_offload_min && off(in, out, false)) return true;
    std::string src = in.to_string();
    std::string dst;
    if (!snappy::Uncompress(src.data(), src.size(), &dst)) return false;
    out->append(dst);
    return true;
}

bool zlib_like_compress(const Buf& in, Buf* out, bool gzip) {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, gzip ? 31 : 15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    char outbuf[16384];
    const size_t nblk = in.backing_block_num();
    for (size_t i = 0; i <= nblk; ++i) {
        const bool last = (i == nblk);
        if (!last) {
            zs.next_in = (Bytef*)in.block_data(i);
            zs.avail_in = (uInt)in.block_len(i);
        } else {
            zs.next_in = nullptr;
            zs.avail_in = 0;
        }
        do {
            zs.next_out = (Bytef*)outbuf;
            zs.avail_out = sizeof(outbuf);
            int rc = deflate(&zs, last ? Z_FINISH : Z_NO_FLUSH);
            if (rc == Z_STREAM_ERROR) {
                deflateEnd(&zs);
                return false;
            }
            out->append(outbuf, sizeof(outbuf) - zs.avail_out);
        } while (zs.avail_out == 0);
    }
    deflateEnd(&zs);
    return true;
}

bool zlib_like_decompress(const Buf& in, Buf* out, bool gzip) {
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, gzip ? 31 : 15) != Z_OK) return false;
    char outbuf[16384];
    int rc = Z_OK;
    const size_t nblk = in.backing_block_num();
    for (size_t i = 0; i < nblk && rc != Z_STREAM_END; ++i) {
        zs.next_in = (Bytef*)in.block_data(i);
        zs.avail_in = (uInt)in.block_len(i);
        do {
            zs.next_out = (Bytef*)outbuf;
            zs.avail_out = sizeof(outbuf);
            rc = inflate(&zs, Z_NO_FLUSH);
            if (rc != Z_OK && rc != Z_STREAM_END) {
                inflateEnd(&zs);
                return false;
            }
            out->append(outbuf, sizeof(outbuf) - zs.avail_out);
        } while (zs.avail_out == 0 && rc != Z_STREAM_END);
    }
    inflateEnd(&zs);
    return rc == Z_STREAM_END;
}

bool gzip_compress(const Buf& in, Buf* out) { return zlib_like_compress(in, out, true); }
bool gzip_decompress(const Buf& in, Buf* out) { return zlib_like_decompress(in, out, true); }
bool zlib_compress(const Buf& in, Buf* out) { return zlib_like_compress(in, out, false); }
bool zlib_decompress(const Buf& in, Buf* out) { return zlib_like_decompress(in, out, false); }
}  // namespace

int RegisterCompressHandler(CompressType type, const CompressHandler& h) {
    if ((int)type <= 0 || (int)type >= 16) return -1;
    if (g_handlers[type].Compress) return -1;
    g_handlers[type] = h;
    return 0;
}

const CompressHandler* FindCompressHandler(CompressType type) {
    if ((int)type <= 0 || (int)type >= 16) return nullptr;
    RegisterBuiltinCompressHandlers();  // usable before any server or channel exists
    return g_handlers[type].Compress ? &g_handlers[type] : nullptr;
}

const char* CompressTypeToCStr(CompressType type) {
    if (type == COMPRESS_TYPE_NONE) return "none";
    const CompressHandler* h = FindCompressHandler(type);
    return h ? h->name : "unknown";
}

void RegisterBuiltinCompressHandlers() {
    static std::once_flag once;
    std::call_once(once, [] {
        CompressHandler sh;
        sh.Compress = snappy_compress;
        sh.Decompress = snappy_decompress;
        sh.name = "snappy";
        RegisterCompressHandler(COMPRESS_TYPE_SNAPPY, sh);
        CompressHandler gh;
        gh.Compress = gzip_compress;
        gh.Decompress = gzip_decompress;
        gh.name = "gzip";
        RegisterCompressHandler(COMPRESS_TYPE_GZIP, gh);
        CompressHandler zh;
        zh.Compress = zlib_compress;
        zh.Decompress = zlib_decompress;
        zh.name = "zlib";
        RegisterCompressHandler(COMPRESS_TYPE_ZLIB, zh);
    });
}

bool CompressBuf(CompressType type, const Buf& in, Buf* out) {
    if (type == COMPRESS_TYPE_NONE) {
        out->append(in);
        return true;
    }
    const CompressHandler* h = FindCompressHandler(type);
    return h && h->Compress(in, out);
}

bool DecompressBuf(CompressType type, const Buf& in, Buf* out) {
    if (type == COMPRESS_TYPE_NONE) {
        out->append(in);
        return true;
    }
    const CompressHandler* h = FindCompressHandler(type);
    return h && h->Decompress(in, out);
}

namespace {
std::atomic<PbParseOffload> g_pb_offload{nullptr};
size_t g_pb_offload_min = (size_t)-1;
}  // namespace

void SetPbParseOffload(PbParseOffload fn, size_t min_bytes) {
    g_pb_offload_min = min_bytes;
    g_pb_offload.store(fn, std::memory_order_release);
}

int TryPbParseOffload(const Buf& compressed, CompressType type, pb::Message* msg) {
    PbParseOffload off = g_pb_offload.load(std::memory_order_acquire);
    if (!off || type != COMPRESS_TYPE_SNAPPY || snappy_ulen(compressed) < g_pb_offload_min) return 0;
    return off(compressed, type, msg);
}

namespace {
std::atomic<SnappyPackOffload> g_pack_offload{nullptr};
size_t g_pack_offload_min = (size_t)-1;
}  // namespace

void SetSnappyPackOffload(SnappyPackOffload fn, size_t min_bytes) {
    g_pack_offload_min = min_bytes;
    g_pack_offload.store(fn, std::memory_order_release);
}

bool TrySnappyPackOffload(const pb::Message& msg, Buf* out) {
    SnappyPackOffload off = g_pack_offload.load(std::memory_order_acquire);
    if (!off) return false;
    const size_t n = msg.ByteSizeLong();  // caches the sizes the serializer uses
    return n >= g_pack_offload_min && off(msg, n, out);
}

void SetSnappyOffload(SnappyOffload fn, size_t min_bytes) {
    g_snappy_offload_min = min_bytes;
    g_snappy_offload.store(fn, std::memory_order_release);
}

}  // namespace mrpc
