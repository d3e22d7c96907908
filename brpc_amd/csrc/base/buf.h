// Buf: non-contiguous, ref-counted, zero-copy byte rope.
//
// Capability parity with butil::IOBuf (reference src/butil/iobuf.h:61-110,
// iobuf.cpp:163-164,321-334,921,1574): a queue of BlockRef{offset,length,block}
// over ref-counted blocks, pluggable block memory (the RDMA/GPU hook), a
// per-thread append block, user-owned memory attachment, scatter/gather
// writev(<=256 iov)/readv(<=64 iov) with sockets.
//
// MI355X-first differences:
//  * every block carries a MemKind tag (HOST / PINNED / DEVICE(HBM) / PEER
//    (xGMI-mapped HBM of another GPU)). Host parsers only ever touch
//    host-accessible blocks; copies out of device blocks go through a
//    registered device-copy hook (hipMemcpy D2H) instead of memcpy.
//  * the default block allocator can be swapped to pinned host memory
//    (hipHostMalloc) so that socket payloads are DMA-able into HBM.
//  * payloads >= 64 KB get one dedicated block instead of 8 KB chunks, which
//    keeps large bodies as few large regions (one hipMemcpyAsync / one xGMI
//    transfer each).
#pragma once

#include <sys/uio.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "base/macros.h"

namespace mrpc {

enum class MemKind : uint8_t { HOST = 0, PINNED = 1, DEVICE = 2, PEER = 3 };
const char* MemKindName(MemKind k);
inline bool IsHostAccessible(MemKind k) { return k == MemKind::HOST || k == MemKind::PINNED; }

struct BufBlock;

// Hook for block memory (the analog of butil::iobuf::blockmem_allocate).
struct BlockMemAllocator {
    void* (*alloc)(size_t bytes);
    void (*dealloc)(void* p, size_t bytes);
    MemKind kind;
};
// Set the allocator used for default-size blocks. Must be called before any
// block is allocated or after all blocks have been freed.
void SetBlockMemAllocator(const BlockMemAllocator& a);
const BlockMemAllocator& GetBlockMemAllocator();

// Copy hook used when a Buf needs host bytes of a non-host block.
// (dst_host, src_device, n) -> 0 on success.
using DeviceCopyFn = int (*)(void* dst, const void* src, size_t n, MemKind src_kind, int device);
void SetDeviceCopyHook(DeviceCopyFn fn);
DeviceCopyFn GetDeviceCopyHook();

struct BufBlock {
    std::atomic<int32_t> nshared;
    uint16_t flags;
    MemKind kind;
    int8_t device;     // device ordinal for DEVICE/PEER blocks, -1 for host
    uint32_t size;     // bytes written so far (append cursor)
    uint32_t cap;      // capacity of data
    char* data;
    void (*deleter)(void* data, void* arg);  // for user blocks
    void* deleter_arg;
    uint64_t meta;     // user meta (e.g. xGMI slot / registration key)

    enum : uint16_t { F_INLINE_DATA = 1, F_USER_DATA = 2, F_LARGE = 4 };
    bool full() const { return size >= cap; }
    uint32_t left() const { return cap - size; }
    void inc_ref() { nshared.fetch_add(1, std::memory_order_relaxed); }
    void dec_ref();
};

struct BlockRef {
    uint32_t offset;
    uint32_t length;
    BufBlock* block;
};

class BufPortal;

class Buf {
public:
    static const size_t DEFAULT_BLOCK_SIZE = 8192;
    static const size_t LARGE_BLOCK_THRESHOLD = 65536;
    static const int MAX_WRITEV_IOV = 256;

    Buf();
    Buf(const Buf& rhs);
    Buf(Buf&& rhs) noexcept;
    Buf& operator=(const Buf& rhs);
    Buf& operator=(Buf&& rhs) noexcept;
    ~Buf();
    explicit Buf(const std::string& s) : Buf() { append(s); }

    void swap(Buf& other) noexcept;
    void clear();
    size_t size() const { return _nbytes; }
    size_t length() const { return _nbytes; }
    bool empty() const { return _nbytes == 0; }

    // ---- append ----
    int append(const void* data, size_t n);
    int append(const std::string& s) { return append(s.data(), s.size()); }
    int append(const char* s) { return append(s, strlen(s)); }
    void append(const Buf& other);
    void append(Buf&& other);
    int push_back(char c) { return append(&c, 1); }
    // Reserve `n` contiguous writable bytes at the tail. The returned pointer
    // is valid until the next mutation; bytes are part of the buffer already.
    char* append_contiguous(size_t n);
    // Attach memory owned by the user; deleter(data, arg) is called when the
    // last reference goes away. Zero copy.
    int append_user_data(void* data, size_t n, void (*deleter)(void*, void*), void* arg = nullptr,
                         MemKind kind = MemKind::HOST, int device = -1, uint64_t meta = 0);
    // Append a whole block (takes one new reference).
    void append_block(BufBlock* b, uint32_t offset, uint32_t length);

    // ---- cut / pop ----
    size_t cutn(Buf* out, size_t n);
    size_t cutn(void* out, size_t n);
    size_t cutn(std::string* out, size_t n);
    bool cut1(char* c);
    size_t pop_front(size_t n);
    size_t pop_back(size_t n);
    // Cut until (and excluding) delimiter; delim is removed. Returns -1 if not found.
    int cut_until(Buf* out, const char* delim);

    // ---- read ----
    size_t copy_to(void* out, size_t n, size_t pos = 0) const;
    size_t copy_to(std::string* out, size_t n = (size_t)-1, size_t pos = 0) const;
    std::string to_string() const;
    // Returns pointer to n contiguous bytes at the front, copying into aux if
    // they span blocks. NULL if fewer than n bytes.
    const void* fetch(void* aux, size_t n) const;
    const char* fetch1() const;
    bool equals(const std::string& s) const;

    // ---- blocks ----
    size_t backing_block_num() const { return _end - _begin; }
    const BlockRef& ref_at(size_t i) const { return _refs[_begin + i]; }
    // Pointer and length of the i-th backing region.
    const char* block_data(size_t i) const { const BlockRef& r = ref_at(i); return r.block->data + r.offset; }
    size_t block_len(size_t i) const { return ref_at(i).length; }
    bool all_host_accessible() const;

    // ---- fd io ----
    // writev at most MAX_WRITEV_IOV regions; consumed bytes are popped.
    ssize_t cut_into_fd(int fd, size_t size_hint = 1024 * 1024);
    // writev the front of several Bufs in one syscall.
    static ssize_t cut_multiple_into_fd(int fd, Buf* const* pieces, size_t count);
    // Fill iovecs for the first bytes (<= max_iov); returns count.
    int fill_iov(struct iovec* iov, int max_iov, size_t max_bytes, size_t* nbytes) const;

    // stats
    static int64_t block_count();
    static int64_t block_memory();
    static int64_t new_bigview_count();

private:
    friend class BufPortal;
    void push_ref(const BlockRef& r);   // takes ownership of one reference
    void push_ref_merge(const BlockRef& r);
    void pop_front_ref();
    void reserve_refs(uint32_t n);

    BlockRef* _refs;
    uint32_t _begin;
    uint32_t _end;
    uint32_t _cap;
    size_t _nbytes;
    BlockRef _inline[2];
};

// A Buf that can read from fds into its own blocks (analog of IOPortal).
class BufPortal : public Buf {
public:
    BufPortal() : _pending(nullptr) {}
    BufPortal(const BufPortal&) = delete;  // owns refs of its pending and spare blocks
    BufPortal& operator=(const BufPortal&) = delete;
    ~BufPortal();
    // readv up to max_count bytes. Returns bytes read (0 = EOF), -1 on error.
    ssize_t append_from_fd(int fd, size_t max_count);
    void return_cached_blocks();
private:
    BufBlock* _pending;  // the partially-filled block the next read continues
    // Blocks a read sized for but did not fill, kept for the next read (as
    // IOPortal keeps its block chain): a read of max_count bytes takes up to
    // 64 blocks, and freeing the unused ones every call cost page faults and
    // heap trims in the kernel (32 KiB echo: ~290 us of system time per RPC)
    std::vector<BufBlock*> _spare;
};

// Block level helpers
BufBlock* NewBlock(size_t min_cap = 0);  // nshared = 1
BufBlock* NewUserBlock(void* data, size_t n, void (*deleter)(void*, void*), void* arg, MemKind kind, int device,
                       uint64_t meta);

// Zero-copy sequential writer into a Buf (analog of IOBufAppender).
class BufAppender {
public:
    explicit BufAppender(Buf* b) : _buf(b) {}
    int append(const void* d, size_t n) { return _buf->append(d, n); }
    int push_back(char c) { return _buf->push_back(c); }
    Buf* buf() { return _buf; }
private:
    Buf* _buf;
};

// Sequential byte iterator over a Buf (analog of IOBufBytesIterator).
class BufBytesIterator {
public:
    explicit BufBytesIterator(const Buf& b) : _buf(b), _idx(0), _off(0), _left(b.size()) { settle(); }
    bool done() const { return _left == 0; }
    char operator*() const { return _cur[_off]; }
    size_t bytes_left() const { return _left; }
    BufBytesIterator& operator++() {
        ++_off;
        --_left;
        if (_off >= _len) { ++_idx; _off = 0; settle(); }
        return *this;
    }
    size_t copy_and_forward(void* out, size_t n);
    size_t forward(size_t n);
private:
    void settle() {
        while (_idx < _buf.backing_block_num() && _buf.block_len(_idx) == 0) ++_idx;
        if (_idx < _buf.backing_block_num()) { _cur = _buf.block_data(_idx); _len = _buf.block_len(_idx); }
        else { _cur = nullptr; _len = 0; }
    }
    const Buf& _buf;
    size_t _idx;
    size_t _off;
    size_t _left;
    const char* _cur = nullptr;
    size_t _len = 0;
};

}  // namespace mrpc
