#include "base/buf.h"

#include <errno.h>
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>

#include "base/logging.h"

namespace mrpc {

const char* MemKindName(MemKind k) {
    switch (k) {
    case MemKind::HOST: return "host";
    case MemKind::PINNED: return "pinned";
    case MemKind::DEVICE: return "device";
    case MemKind::PEER: return "peer";
    }
    return "?";
}

namespace {

std::atomic<int64_t> g_nblock{0};
std::atomic<int64_t> g_blockmem{0};
std::atomic<int64_t> g_nbigview{0};

void* default_alloc(size_t n) { return malloc(n); }
void default_dealloc(void* p, size_t) { free(p); }

BlockMemAllocator g_alloc = {default_alloc, default_dealloc, MemKind::HOST};
DeviceCopyFn g_devcopy = nullptr;

const size_t kHeader = (sizeof(BufBlock) + 15) & ~(size_t)15;
const size_t kMaxTLSCache = 8;

struct TLSBlocks {
    BufBlock* share = nullptr;
    BufBlock* cache[kMaxTLSCache];
    size_t ncache = 0;
    bool alive = true;
    ~TLSBlocks();
};
thread_local TLSBlocks tls_blocks;

void free_block_memory(BufBlock* b) {
    if (b->flags & BufBlock::F_USER_DATA) {
        if (b->deleter) b->deleter(b->data, b->deleter_arg);
        g_nblock.fetch_sub(1, std::memory_order_relaxed);
        delete b;
        return;
    }
    size_t total = kHeader + b->cap;
    auto dealloc = reinterpret_cast<void (*)(void*, size_t)>(b->deleter_arg);
    g_nblock.fetch_sub(1, std::memory_order_relaxed);
    g_blockmem.fetch_sub((int64_t)total, std::memory_order_relaxed);
    dealloc(b, total);
}

TLSBlocks::~TLSBlocks() {
    alive = false;
    if (share) {
        share->dec_ref();
        share = nullptr;
    }
    for (size_t i = 0; i < ncache; ++i) free_block_memory(cache[i]);
    ncache = 0;
}

BufBlock* create_inline_block(size_t total) {
    void* mem = g_alloc.alloc(total);
    if (!mem) return nullptr;
    BufBlock* b = new (mem) BufBlock;
    b->nshared.store(1, std::memory_order_relaxed);
    b->flags = BufBlock::F_INLINE_DATA;
    b->kind = g_alloc.kind;
    b->device = -1;
    b->size = 0;
    b->cap = (uint32_t)(total - kHeader);
    b->data = (char*)mem + kHeader;
    b->deleter = nullptr;
    b->deleter_arg = reinterpret_cast<void*>(g_alloc.dealloc);
    b->meta = 0;
    g_nblock.fetch_add(1, std::memory_order_relaxed);
    g_blockmem.fetch_add((int64_t)total, std::memory_order_relaxed);
    return b;
}

BufBlock* acquire_default_block() {
    TLSBlocks& t = tls_blocks;
    if (t.alive && t.ncache > 0) {
        BufBlock* b = t.cache[--t.ncache];
        b->nshared.store(1, std::memory_order_relaxed);
        b->size = 0;
        b->meta = 0;
        return b;
    }
    return create_inline_block(Buf::DEFAULT_BLOCK_SIZE);
}

inline BufBlock* share_tls_block() {
    TLSBlocks& t = tls_blocks;
    BufBlock* b = t.share;
    if (MRPC_LIKELY(b && !b->full())) return b;
    if (b) b->dec_ref();
    b = acquire_default_block();
    t.share = t.alive ? b : nullptr;
    if (!t.alive) {
        // thread is exiting: hand the block out without caching it.
        return b;
    }
    return b;
}

}  // namespace

void SetBlockMemAllocator(const BlockMemAllocator& a) {
    CHECK(IsHostAccessible(a.kind)) << "default Buf blocks must be host accessible";
    // Drop this thread's cached blocks which were allocated by the old allocator.
    TLSBlocks& t = tls_blocks;
    if (t.share) { t.share->dec_ref(); t.share = nullptr; }
    for (size_t i = 0; i < t.ncache; ++i) free_block_memory(t.cache[i]);
    t.ncache = 0;
    g_alloc = a;
}
const BlockMemAllocator& GetBlockMemAllocator() { return g_alloc; }
void SetDeviceCopyHook(DeviceCopyFn fn) { g_devcopy = fn; }
DeviceCopyFn GetDeviceCopyHook() { return g_devcopy; }

void BufBlock::dec_ref() {
    if (nshared.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
    if ((flags & F_INLINE_DATA) && !(flags & F_LARGE) && cap + kHeader == Buf::DEFAULT_BLOCK_SIZE &&
        reinterpret_cast<void*>(g_alloc.dealloc) == deleter_arg) {
        TLSBlocks& t = tls_blocks;
        if (t.alive && t.ncache < kMaxTLSCache) {
            t.cache[t.ncache++] = this;
            return;
        }
    }
    free_block_memory(this);
}

BufBlock* NewBlock(size_t min_cap) {
    if (min_cap <= Buf::DEFAULT_BLOCK_SIZE - kHeader) return acquire_default_block();
    size_t total = (kHeader + min_cap + 4095) & ~(size_t)4095;
    BufBlock* b = create_inline_block(total);
    if (b) b->flags |= BufBlock::F_LARGE;
    return b;
}

BufBlock* NewUserBlock(void* data, size_t n, void (*deleter)(void*, void*), void* arg, MemKind kind, int device,
                       uint64_t meta) {
    BufBlock* b = new BufBlock;
    b->nshared.store(1, std::memory_order_relaxed);
    b->flags = BufBlock::F_USER_DATA;
    b->kind = kind;
    b->device = (int8_t)device;
    b->size = (uint32_t)n;
    b->cap = (uint32_t)n;
    b->data = (char*)data;
    b->deleter = deleter;
    b->deleter_arg = arg;
    b->meta = meta;
    g_nblock.fetch_add(1, std::memory_order_relaxed);
    return b;
}

int64_t Buf::block_count() { return g_nblock.load(std::memory_order_relaxed); }
int64_t Buf::block_memory() { return g_blockmem.load(std::memory_order_relaxed); }
int64_t Buf::new_bigview_count() { return g_nbigview.load(std::memory_order_relaxed); }

// ---------------------------------------------------------------- Buf

Buf::Buf() : _refs(_inline), _begin(0), _end(0), _cap(2), _nbytes(0) {}

Buf::Buf(const Buf& rhs) : Buf() { append(rhs); }

Buf::Buf(Buf&& rhs) noexcept : Buf() { swap(rhs); }

Buf& Buf::operator=(const Buf& rhs) {
    if (this != &rhs) {
        clear();
        append(rhs);
    }
    return *this;
}

Buf& Buf::operator=(Buf&& rhs) noexcept {
    if (this != &rhs) {
        clear();
        swap(rhs);
    }
    return *this;
}

Buf::~Buf() {
    clear();
    if (_refs != _inline) free(_refs);
}

void Buf::swap(Buf& o) noexcept {
    const bool a_inline = (_refs == _inline);
    const bool b_inline = (o._refs == o._inline);
    std::swap(_inline[0], o._inline[0]);
    std::swap(_inline[1], o._inline[1]);
    std::swap(_refs, o._refs);
    std::swap(_begin, o._begin);
    std::swap(_end, o._end);
    std::swap(_cap, o._cap);
    std::swap(_nbytes, o._nbytes);
    if (a_inline) o._refs = o._inline;
    if (b_inline) _refs = _inline;
}

void Buf::clear() {
    for (uint32_t i = _begin; i < _end; ++i) _refs[i].block->dec_ref();
    _begin = _end = 0;
    _nbytes = 0;
}

void Buf::reserve_refs(uint32_t n) {
    if (_end + n <= _cap) return;
    uint32_t used = _end - _begin;
    if (_begin > 0 && used + n <= _cap) {
        memmove(_refs, _refs + _begin, used * sizeof(BlockRef));
        _begin = 0;
        _end = used;
        return;
    }
    uint32_t ncap = _cap * 2;
    while (ncap < used + n) ncap *= 2;
    BlockRef* nr = (BlockRef*)malloc(ncap * sizeof(BlockRef));
    CHECK(nr);
    memcpy(nr, _refs + _begin, used * sizeof(BlockRef));
    if (_refs != _inline) free(_refs);
    else g_nbigview.fetch_add(1, std::memory_order_relaxed);
    _refs = nr;
    _cap = ncap;
    _begin = 0;
    _end = used;
}

void Buf::push_ref(const BlockRef& r) {
    if (r.length == 0) {
        r.block->dec_ref();
        return;
    }
    reserve_refs(1);
    _refs[_end++] = r;
    _nbytes += r.length;
}

void Buf::push_ref_merge(const BlockRef& r) {
    if (r.length == 0) {
        r.block->dec_ref();
        return;
    }
    if (_end > _begin) {
        BlockRef& last = _refs[_end - 1];
        if (last.block == r.block && last.offset + last.length == r.offset) {
            last.length += r.length;
            _nbytes += r.length;
            r.block->dec_ref();
            return;
        }
    }
    reserve_refs(1);
    _refs[_end++] = r;
    _nbytes += r.length;
}

void Buf::pop_front_ref() {
    BlockRef& r = _refs[_begin];
    _nbytes -= r.length;
    r.block->dec_ref();
    if (++_begin == _end) _begin = _end = 0;
}

int Buf::append(const void* data, size_t n) {
    const char* p = (const char*)data;
    while (n > 0) {
        if (n >= LARGE_BLOCK_THRESHOLD) {
            BufBlock* b = NewBlock(n);
            if (!b) return -1;
            memcpy(b->data, p, n);
            b->size = (uint32_t)n;
            push_ref(BlockRef{0, (uint32_t)n, b});
            return 0;
        }
        BufBlock* b = share_tls_block();
        if (!b) return -1;
        size_t c = std::min<size_t>(n, b->left());
        memcpy(b->data + b->size, p, c);
        b->inc_ref();
        BlockRef r{b->size, (uint32_t)c, b};
        b->size += (uint32_t)c;
        push_ref_merge(r);
        p += c;
        n -= c;
    }
    return 0;
}

char* Buf::append_contiguous(size_t n) {
    if (n == 0) return nullptr;
    BufBlock* b = share_tls_block();
    if (b && n > b->left()) {
        if (n <= DEFAULT_BLOCK_SIZE - kHeader) {
            // start a fresh shared block
            tls_blocks.share = nullptr;
            b->dec_ref();
            b = share_tls_block();
        } else {
            BufBlock* big = NewBlock(n);
            if (!big) return nullptr;
            big->size = (uint32_t)n;
            push_ref(BlockRef{0, (uint32_t)n, big});
            return big->data;
        }
    }
    if (!b) return nullptr;
    char* out = b->data + b->size;
    b->inc_ref();
    BlockRef r{b->size, (uint32_t)n, b};
    b->size += (uint32_t)n;
    push_ref_merge(r);
    return out;
}

void Buf::append(const Buf& other) {
    if (&other == this) {
        Buf copy(other);
        append(std::move(copy));
        return;
    }
    reserve_refs(other._end - other._begin);
    for (uint32_t i = other._begin; i < other._end; ++i) {
        const BlockRef& r = other._refs[i];
        r.block->inc_ref();
        push_ref_merge(r);
    }
}

void Buf::append(Buf&& other) {
    if (_nbytes == 0) {
        clear();
        swap(other);
        return;
    }
    reserve_refs(other._end - other._begin);
    for (uint32_t i = other._begin; i < other._end; ++i) push_ref_merge(other._refs[i]);
    other._begin = other._end = 0;
    other._nbytes = 0;
}

int Buf::append_user_data(void* data, size_t n, void (*deleter)(void*, void*), void* arg, MemKind kind, int device,
                          uint64_t meta) {
    if (n > 0xFFFFFFFFu) return -1;
    BufBlock* b = NewUserBlock(data, n, deleter, arg, kind, device, meta);
    push_ref(BlockRef{0, (uint32_t)n, b});
    return 0;
}

void Buf::append_block(BufBlock* b, uint32_t offset, uint32_t length) {
    b->inc_ref();
    push_ref_merge(BlockRef{offset, length, b});
}

size_t Buf::cutn(Buf* out, size_t n) {
    n = std::min(n, _nbytes);
    size_t left = n;
    while (left > 0) {
        BlockRef& r = _refs[_begin];
        if (r.length <= left) {
            left -= r.length;
            _nbytes -= r.length;
            out->push_ref_merge(r);  // transfers the reference
            if (++_begin == _end) _begin = _end = 0;
        } else {
            r.block->inc_ref();
            out->push_ref_merge(BlockRef{r.offset, (uint32_t)left, r.block});
            r.offset += (uint32_t)left;
            r.length -= (uint32_t)left;
            _nbytes -= left;
            left = 0;
        }
    }
    return n;
}

size_t Buf::cutn(void* out, size_t n) {
    n = copy_to(out, n);
    pop_front(n);
    return n;
}

size_t Buf::cutn(std::string* out, size_t n) {
    n = std::min(n, _nbytes);
    size_t old = out->size();
    out->resize(old + n);
    return cutn(&(*out)[old], n);
}

bool Buf::cut1(char* c) {
    if (_nbytes == 0) return false;
    BlockRef& r = _refs[_begin];
    if (IsHostAccessible(r.block->kind)) {
        *c = r.block->data[r.offset];
        if (r.length == 1) {
            pop_front_ref();
        } else {
            ++r.offset;
            --r.length;
            --_nbytes;
        }
        return true;
    }
    return cutn(c, 1) == 1;
}

size_t Buf::pop_front(size_t n) {
    n = std::min(n, _nbytes);
    size_t left = n;
    while (left > 0) {
        BlockRef& r = _refs[_begin];
        if (r.length <= left) {
            left -= r.length;
            pop_front_ref();
        } else {
            r.offset += (uint32_t)left;
            r.length -= (uint32_t)left;
            _nbytes -= left;
            left = 0;
        }
    }
    return n;
}

size_t Buf::pop_back(size_t n) {
    n = std::min(n, _nbytes);
    size_t left = n;
    while (left > 0) {
        BlockRef& r = _refs[_end - 1];
        if (r.length <= left) {
            left -= r.length;
            _nbytes -= r.length;
            r.block->dec_ref();
            if (--_end == _begin) _begin = _end = 0;
        } else {
            r.length -= (uint32_t)left;
            _nbytes -= left;
            left = 0;
        }
    }
    return n;
}

static void copy_region(void* dst, const BufBlock* b, size_t off, size_t n) {
    if (IsHostAccessible(b->kind)) {
        memcpy(dst, b->data + off, n);
    } else {
        CHECK(g_devcopy) << "copy from " << MemKindName(b->kind) << " block without a device copy hook";
        CHECK_EQ(0, g_devcopy(dst, b->data + off, n, b->kind, b->device));
    }
}

size_t Buf::copy_to(void* out, size_t n, size_t pos) const {
    if (pos >= _nbytes) return 0;
    n = std::min(n, _nbytes - pos);
    char* o = (char*)out;
    size_t left = n;
    for (uint32_t i = _begin; i < _end && left > 0; ++i) {
        const BlockRef& r = _refs[i];
        if (pos >= r.length) {
            pos -= r.length;
            continue;
        }
        size_t c = std::min<size_t>(left, r.length - pos);
        copy_region(o, r.block, r.offset + pos, c);
        o += c;
        left -= c;
        pos = 0;
    }
    return n;
}

size_t Buf::copy_to(std::string* out, size_t n, size_t pos) const {
    if (pos >= _nbytes) {
        out->clear();
        return 0;
    }
    n = std::min(n, _nbytes - pos);
    out->resize(n);
    return copy_to(&(*out)[0], n, pos);
}

std::string Buf::to_string() const {
    std::string s;
    copy_to(&s);
    return s;
}

const void* Buf::fetch(void* aux, size_t n) const {
    if (n > _nbytes) return nullptr;
    if (n == 0) return aux;
    const BlockRef& r = _refs[_begin];
    if (r.length >= n && IsHostAccessible(r.block->kind)) return r.block->data + r.offset;
    copy_to(aux, n);
    return aux;
}

const char* Buf::fetch1() const {
    if (_nbytes == 0) return nullptr;
    const BlockRef& r = _refs[_begin];
    if (!IsHostAccessible(r.block->kind)) return nullptr;
    return r.block->data + r.offset;
}

bool Buf::equals(const std::string& s) const {
    if (s.size() != _nbytes) return false;
    size_t pos = 0;
    for (uint32_t i = _begin; i < _end; ++i) {
        const BlockRef& r = _refs[i];
        if (!IsHostAccessible(r.block->kind)) return to_string() == s;
        if (memcmp(r.block->data + r.offset, s.data() + pos, r.length) != 0) return false;
        pos += r.length;
    }
    return true;
}

bool Buf::all_host_accessible() const {
    for (uint32_t i = _begin; i < _end; ++i) {
        if (!IsHostAccessible(_refs[i].block->kind)) return false;
    }
    return true;
}

int Buf::cut_until(Buf* out, const char* delim) {
    const size_t dl = strlen(delim);
    if (dl == 0 || _nbytes < dl) return -1;
    // linear scan with a small sliding window
    size_t pos = 0;
    size_t matched = 0;
    for (uint32_t i = _begin; i < _end; ++i) {
        const BlockRef& r = _refs[i];
        if (!IsHostAccessible(r.block->kind)) return -1;
        const char* d = r.block->data + r.offset;
        for (uint32_t j = 0; j < r.length; ++j) {
            char c = d[j];
            if (c == delim[matched]) {
                if (++matched == dl) {
                    size_t end = pos + j + 1;  // bytes including delim
                    cutn(out, end - dl);
                    pop_front(dl);
                    return 0;
                }
            } else if (matched) {
                // restart (delimiters we use have no self-overlap except
                // repeated chars; handle that by re-checking c)
                matched = (c == delim[0]) ? 1 : 0;
            }
        }
        pos += r.length;
    }
    return -1;
}

int Buf::fill_iov(struct iovec* iov, int max_iov, size_t max_bytes, size_t* nbytes) const {
    int n = 0;
    size_t total = 0;
    for (uint32_t i = _begin; i < _end && n < max_iov && total < max_bytes; ++i) {
        const BlockRef& r = _refs[i];
        CHECK(IsHostAccessible(r.block->kind)) << "cannot write " << MemKindName(r.block->kind) << " block to fd";
        iov[n].iov_base = r.block->data + r.offset;
        iov[n].iov_len = r.length;
        total += r.length;
        ++n;
    }
    if (nbytes) *nbytes = total;
    return n;
}

ssize_t Buf::cut_into_fd(int fd, size_t size_hint) {
    if (_nbytes == 0) return 0;
    struct iovec iov[MAX_WRITEV_IOV];
    int n = fill_iov(iov, MAX_WRITEV_IOV, size_hint, nullptr);
    ssize_t nw = ::writev(fd, iov, n);
    if (nw > 0) pop_front((size_t)nw);
    return nw;
}

ssize_t Buf::cut_multiple_into_fd(int fd, Buf* const* pieces, size_t count) {
    struct iovec iov[MAX_WRITEV_IOV];
    int n = 0;
    for (size_t i = 0; i < count && n < MAX_WRITEV_IOV; ++i) {
        n += pieces[i]->fill_iov(iov + n, MAX_WRITEV_IOV - n, (size_t)-1, nullptr);
    }
    if (n == 0) return 0;
    ssize_t nw = ::writev(fd, iov, n);
    if (nw > 0) {
        size_t left = (size_t)nw;
        for (size_t i = 0; i < count && left > 0; ++i) left -= pieces[i]->pop_front(left);
    }
    return nw;
}

// ---------------------------------------------------------------- BufPortal

BufPortal::~BufPortal() { return_cached_blocks(); }

void BufPortal::return_cached_blocks() {
    if (_pending) {
        _pending->dec_ref();
        _pending = nullptr;
    }
    for (BufBlock* b : _spare) b->dec_ref();
    _spare.clear();
}

ssize_t BufPortal::append_from_fd(int fd, size_t max_count) {
    const int kMaxIov = 64;
    struct iovec iov[kMaxIov];
    BufBlock* blocks[kMaxIov];
    int nb = 0;
    size_t space = 0;
    // at most max_count bytes per call (the last region is cut short), as
    // IOPortal::append_from_file_descriptor: callers bound one read with it
    if (_pending && !_pending->full()) {
        blocks[nb] = _pending;
        iov[nb].iov_base = _pending->data + _pending->size;
        iov[nb].iov_len = std::min<size_t>(_pending->left(), max_count);
        space += iov[nb].iov_len;
        ++nb;
    } else if (_pending) {
        _pending->dec_ref();
        _pending = nullptr;
    }
    while (space < max_count && nb < kMaxIov) {
        BufBlock* b = nullptr;
        if (!_spare.empty()) {
            b = _spare.back();
            _spare.pop_back();
        } else {
            b = acquire_default_block();
        }
        if (!b) break;
        blocks[nb] = b;  // we own one ref
        iov[nb].iov_base = b->data;
        iov[nb].iov_len = std::min<size_t>(b->cap, max_count - space);
        space += iov[nb].iov_len;
        ++nb;
    }
    ssize_t nr = ::readv(fd, iov, nb);
    size_t left = nr > 0 ? (size_t)nr : 0;
    BufBlock* new_pending = nullptr;
    for (int i = 0; i < nb; ++i) {
        BufBlock* b = blocks[i];
        if (left > 0) {
            size_t c = std::min<size_t>(left, b->left());
            b->inc_ref();
            BlockRef r{b->size, (uint32_t)c, b};
            b->size += (uint32_t)c;
            push_ref_merge(r);
            left -= c;
        }
        // Each block here carries one portal-owned ref. Keep the first
        // non-full block as the next pending block, release the others.
        if (!new_pending && !b->full()) {
            new_pending = b;
        } else if (b->size == 0 && b->cap + kHeader == Buf::DEFAULT_BLOCK_SIZE && (size_t)kMaxIov > _spare.size()) {
            _spare.push_back(b);  // untouched: the portal's ref moves to the spare list
        } else {
            b->dec_ref();
        }
    }
    _pending = new_pending;
    return nr;
}

// ---------------------------------------------------------------- iterator

size_t BufBytesIterator::copy_and_forward(void* out, size_t n) {
    char* o = (char*)out;
    size_t done = 0;
    while (done < n && _left > 0) {
        size_t c = std::min(n - done, _len - _off);
        memcpy(o + done, _cur + _off, c);
        done += c;
        _off += c;
        _left -= c;
        if (_off >= _len) { ++_idx; _off = 0; settle(); }
    }
    return done;
}

size_t BufBytesIterator::forward(size_t n) {
    size_t done = 0;
    while (done < n && _left > 0) {
        size_t c = std::min(n - done, _len - _off);
        done += c;
        _off += c;
        _left -= c;
        if (_off >= _len) { ++_idx; _off = 0; settle(); }
    }
    return done;
}

}  // namespace mrpc
