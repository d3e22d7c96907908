// Typed slab pools with O(1) id->address.
//
// ResourcePool<T> plays the role of butil::ResourcePool
// (reference src/butil/resource_pool.h:96-129, resource_pool_inl.h:225-306):
// objects are never freed, each has a stable 32-bit slot id, free slots are
// recycled through per-thread free lists with a global overflow. Versioned
// 64-bit ids (SocketId, fiber_t, CallId) are built on top by storing a
// version next to the object. ObjectPool<T> is a plain thread-cached
// free-list allocator (butil::ObjectPool).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <new>
#include <vector>

#include "base/macros.h"
#include "base/tsan.h"

namespace mrpc {

// The per-thread free lists hand an object from the fiber that returned it
// to the next fiber that takes it on the same worker with no atomic in
// between (program order of the worker orders them); TSan tracks fibers as
// separate threads, so put()/get() carry explicit release/acquire marks.
template <typename T>
class ResourcePool {
public:
    static constexpr uint32_t kBlockShift = 8;
    static constexpr uint32_t kBlockItems = 1u << kBlockShift;
    static constexpr uint32_t kMaxBlocks = 1u << 16;  // 16M objects
    static constexpr size_t kLocalMax = 128;
    static constexpr uint32_t kInvalid = 0xFFFFFFFFu;

    static ResourcePool* singleton() {
        static ResourcePool* p = new ResourcePool;
        return p;
    }

    T* get(uint32_t* id) {
        Local& l = local();
        if (!l.free_ids.empty() || refill_from_global(l)) {
            uint32_t i = l.free_ids.back();
            l.free_ids.pop_back();
            *id = i;
            T* t = address(i);
            MRPC_TSAN_ACQUIRE(t);
            return t;
        }
        if (l.cur_block == kInvalid || l.cur_index >= kBlockItems) {
            uint32_t b = _nblock.fetch_add(1, std::memory_order_relaxed);
            if (b >= kMaxBlocks) return nullptr;
            Block* blk = new Block;
            _blocks[b].store(blk, std::memory_order_release);
            l.cur_block = b;
            l.cur_index = 0;
        }
        uint32_t i = (l.cur_block << kBlockShift) | l.cur_index++;
        *id = i;
        return address(i);
    }

    void put(uint32_t id) {
        MRPC_TSAN_RELEASE(address(id));
        Local& l = local();
        if (l.free_ids.size() >= kLocalMax) {
            std::lock_guard<std::mutex> g(_mu);
            for (size_t k = kLocalMax / 2; k < l.free_ids.size(); ++k) _global_free.push_back(l.free_ids[k]);
            l.free_ids.resize(kLocalMax / 2);
        }
        l.free_ids.push_back(id);
    }

    T* address(uint32_t id) const {
        uint32_t b = id >> kBlockShift;
        if (MRPC_UNLIKELY(b >= kMaxBlocks)) return nullptr;
        Block* blk = _blocks[b].load(std::memory_order_acquire);
        if (MRPC_UNLIKELY(!blk)) return nullptr;
        return &blk->items[id & (kBlockItems - 1)];
    }

    size_t capacity() const { return (size_t)_nblock.load(std::memory_order_relaxed) * kBlockItems; }

    // Walk all constructed objects (for /sockets, /fibers listings).
    template <typename Fn>
    void for_each(Fn fn) const {
        uint32_t nb = std::min<uint32_t>(_nblock.load(std::memory_order_acquire), kMaxBlocks);
        for (uint32_t b = 0; b < nb; ++b) {
            Block* blk = _blocks[b].load(std::memory_order_acquire);
            if (!blk) continue;
            for (uint32_t i = 0; i < kBlockItems; ++i) fn((b << kBlockShift) | i, &blk->items[i]);
        }
    }

private:
    struct Block {
        T items[kBlockItems];
    };
    struct Local {
        std::vector<uint32_t> free_ids;
        uint32_t cur_block = kInvalid;
        uint32_t cur_index = 0;
    };
    static Local& local() {
        static thread_local Local l;
        return l;
    }
    bool refill_from_global(Local& l) {
        std::lock_guard<std::mutex> g(_mu);
        if (_global_free.empty()) return false;
        size_t n = std::min<size_t>(_global_free.size(), kLocalMax / 2);
        for (size_t k = 0; k < n; ++k) {
            l.free_ids.push_back(_global_free.back());
            _global_free.pop_back();
        }
        return true;
    }
    ResourcePool() : _nblock(0) {
        _blocks = new std::atomic<Block*>[kMaxBlocks];
        for (uint32_t i = 0; i < kMaxBlocks; ++i) _blocks[i].store(nullptr, std::memory_order_relaxed);
    }
    std::atomic<Block*>* _blocks;
    std::atomic<uint32_t> _nblock;
    std::mutex _mu;
    std::vector<uint32_t> _global_free;
};

template <typename T>
inline T* get_resource(uint32_t* id) { return ResourcePool<T>::singleton()->get(id); }
template <typename T>
inline void return_resource(uint32_t id) { ResourcePool<T>::singleton()->put(id); }
template <typename T>
inline T* address_resource(uint32_t id) { return ResourcePool<T>::singleton()->address(id); }

// Thread-cached free-list pool. get() returns a constructed object (new T on
// miss); put() keeps the object alive for reuse, so callers reset state.
template <typename T>
class ObjectPool {
public:
    static constexpr size_t kLocalMax = 64;
    static ObjectPool* singleton() {
        static ObjectPool* p = new ObjectPool;
        return p;
    }
    // Objects move between a thread's cache and the global list kBatch at
    // a time: a thread that only gets (a socket's reader cutting messages)
    // and threads that only put (the workers that ran them) would otherwise
    // take the global mutex once per object each (~1% of the 32 B echo's
    // host samples in MostCommonMessage::Get alone).
    static constexpr size_t kBatch = kLocalMax / 2;
    T* get() {
        Local& l = local();
        if (l.items.empty()) {
            std::lock_guard<std::mutex> g(_mu);
            const size_t n = std::min(kBatch, _global.size());
            l.items.insert(l.items.end(), _global.end() - n, _global.end());
            _global.resize(_global.size() - n);
        }
        if (!l.items.empty()) {
            T* t = l.items.back();
            l.items.pop_back();
            MRPC_TSAN_ACQUIRE(t);
            return t;
        }
        return new T;
    }
    void put(T* t) {
        MRPC_TSAN_RELEASE(t);
        Local& l = local();
        if (l.items.size() >= kLocalMax) {
            std::lock_guard<std::mutex> g(_mu);
            _global.insert(_global.end(), l.items.end() - kBatch, l.items.end());
            l.items.resize(l.items.size() - kBatch);
        }
        l.items.push_back(t);
    }
private:
    struct Local {
        std::vector<T*> items;
        ~Local() {
            ObjectPool* p = ObjectPool::singleton();
            std::lock_guard<std::mutex> g(p->_mu);
            for (T* t : items) p->_global.push_back(t);
        }
    };
    static Local& local() {
        static thread_local Local l;
        return l;
    }
    std::mutex _mu;
    std::vector<T*> _global;
};

template <typename T>
inline T* get_object() { return ObjectPool<T>::singleton()->get(); }
template <typename T>
inline void return_object(T* t) { ObjectPool<T>::singleton()->put(t); }

}  // namespace mrpc
