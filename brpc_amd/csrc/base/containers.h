// Containers: FlatMap (open-addressing hash map, role of
// butil/containers/flat_map.h:131), CaseIgnoredFlatMap, BoundedQueue
// (bounded_queue.h), DoublyBufferedData (doubly_buffered_data.h:56-170:
// read-mostly data with near lock-free reads; used by every load balancer),
// and an intrusive doubly linked list.
#pragma once

#include <unordered_map>

#include <list>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "base/macros.h"

namespace mrpc {

// Open addressing + linear probing + backward-shift deletion. Keys/values
// stored inline; no tombstones so lookups stay short under churn.
template <typename K, typename V, typename Hash = std::hash<K>, typename Eq = std::equal_to<K>>
class FlatMap {
public:
    struct Slot {
        bool used = false;
        std::pair<K, V> kv;
    };
    class iterator {
    public:
        iterator(Slot* s, Slot* e) : _s(s), _e(e) { skip(); }
        std::pair<K, V>& operator*() const { return _s->kv; }
        std::pair<K, V>* operator->() const { return &_s->kv; }
        iterator& operator++() { ++_s; skip(); return *this; }
        bool operator!=(const iterator& o) const { return _s != o._s; }
        bool operator==(const iterator& o) const { return _s == o._s; }
    private:
        void skip() { while (_s != _e && !_s->used) ++_s; }
        Slot* _s;
        Slot* _e;
    };

    explicit FlatMap(size_t initial = 16, int load_factor_percent = 70)
        : _size(0), _lf(load_factor_percent) { rehash(initial); }

    size_t size() const { return _size; }
    bool empty() const { return _size == 0; }
    size_t bucket_count() const { return _slots.size(); }

    V* seek(const K& k) {
        size_t i = find_index(k);
        return i == npos ? nullptr : &_slots[i].kv.second;
    }
    const V* seek(const K& k) const { return const_cast<FlatMap*>(this)->seek(k); }
    bool contains(const K& k) const { return seek(k) != nullptr; }

    V* insert(const K& k, const V& v) {
        V& slot = (*this)[k];
        slot = v;
        return &slot;
    }
    V& operator[](const K& k) {
        size_t i = find_index(k);
        if (i != npos) return _slots[i].kv.second;
        if ((_size + 1) * 100 > _slots.size() * (size_t)_lf) rehash(_slots.size() * 2);
        size_t mask = _slots.size() - 1;
        size_t j = _hash(k) & mask;
        while (_slots[j].used) j = (j + 1) & mask;
        _slots[j].used = true;
        _slots[j].kv.first = k;
        _slots[j].kv.second = V();
        ++_size;
        return _slots[j].kv.second;
    }
    size_t erase(const K& k) {
        size_t i = find_index(k);
        if (i == npos) return 0;
        size_t mask = _slots.size() - 1;
        _slots[i].used = false;
        --_size;
        // backward shift
        size_t j = i;
        for (;;) {
            j = (j + 1) & mask;
            if (!_slots[j].used) break;
            size_t home = _hash(_slots[j].kv.first) & mask;
            // is home cyclically in (i, j]? if not, move j to i
            bool in_range = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
            if (!in_range) {
                _slots[i].used = true;
                _slots[i].kv = std::move(_slots[j].kv);
                _slots[j].used = false;
                i = j;
            }
        }
        return 1;
    }
    void clear() {
        for (auto& s : _slots) {
            if (s.used) { s.used = false; s.kv = std::pair<K, V>(); }
        }
        _size = 0;
    }
    iterator begin() { return iterator(_slots.data(), _slots.data() + _slots.size()); }
    iterator end() { return iterator(_slots.data() + _slots.size(), _slots.data() + _slots.size()); }
    // read-only walk (the reference's const iteration)
    template <typename Fn>
    void for_each(Fn fn) const {
        for (const Slot& s : _slots) {
            if (s.used) fn(s.kv.first, s.kv.second);
        }
    }
    void swap(FlatMap& o) {
        _slots.swap(o._slots);
        std::swap(_size, o._size);
        std::swap(_lf, o._lf);
    }

private:
    static const size_t npos = (size_t)-1;
    size_t find_index(const K& k) const {
        size_t mask = _slots.size() - 1;
        size_t j = _hash(k) & mask;
        while (_slots[j].used) {
            if (_eq(_slots[j].kv.first, k)) return j;
            j = (j + 1) & mask;
        }
        return npos;
    }
    void rehash(size_t n) {
        size_t cap = 8;
        while (cap < n) cap <<= 1;
        std::vector<Slot> old;
        old.swap(_slots);
        _slots.resize(cap);
        _size = 0;
        for (auto& s : old) {
            if (s.used) (*this)[s.kv.first] = std::move(s.kv.second);
        }
    }
    std::vector<Slot> _slots;
    size_t _size;
    int _lf;
    Hash _hash;
    Eq _eq;
};

struct CaseIgnoredHash {
    size_t operator()(const std::string& s) const {
        size_t h = 1469598103934665603ull;
        for (char c : s) h = (h ^ (size_t)tolower((unsigned char)c)) * 1099511628211ull;
        return h;
    }
};
struct CaseIgnoredEqual {
    bool operator()(const std::string& a, const std::string& b) const {
        if (a.size() != b.size()) return false;
        for (size_t i = 0; i < a.size(); ++i) {
            if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
        }
        return true;
    }
};
template <typename V>
using CaseIgnoredFlatMap = FlatMap<std::string, V, CaseIgnoredHash, CaseIgnoredEqual>;

// Fixed-capacity ring queue (not thread safe).
template <typename T>
class BoundedQueue {
public:
    explicit BoundedQueue(size_t cap) : _buf(cap), _start(0), _count(0) {}
    bool push(const T& t) {
        if (_count == _buf.size()) return false;
        _buf[(_start + _count) % _buf.size()] = t;
        ++_count;
        return true;
    }
    bool pop(T* out) {
        if (_count == 0) return false;
        *out = std::move(_buf[_start]);
        _start = (_start + 1) % _buf.size();
        --_count;
        return true;
    }
    bool full() const { return _count == _buf.size(); }
    bool empty() const { return _count == 0; }
    size_t size() const { return _count; }
    size_t capacity() const { return _buf.size(); }
private:
    std::vector<T> _buf;
    size_t _start;
    size_t _count;
};

// Read-mostly data. Readers lock only their own thread's mutex (uncontended
// except during Modify); Modify applies fn to the background copy, flips,
// waits for readers of the old foreground by taking each reader's mutex, then
// applies fn to the other copy.
template <typename T>
class DoublyBufferedData {
    struct Wrapper {
        std::mutex mu;
        DoublyBufferedData* owner = nullptr;
    };

public:
    class ScopedPtr {
    public:
        ScopedPtr() : _data(nullptr), _w(nullptr) {}
        ~ScopedPtr() { if (_w) _w->mu.unlock(); }
        const T* get() const { return _data; }
        const T& operator*() const { return *_data; }
        const T* operator->() const { return _data; }
    private:
        friend class DoublyBufferedData;
        const T* _data;
        Wrapper* _w;
    };

    DoublyBufferedData() : _index(0) {}
    ~DoublyBufferedData() {
        std::lock_guard<std::mutex> g(_wrappers_mu);
        for (auto& w : _wrappers) w->owner = nullptr;
    }

    int Read(ScopedPtr* ptr) {
        Wrapper* w = local_wrapper();
        w->mu.lock();
        ptr->_data = &_data[_index.load(std::memory_order_acquire)];
        ptr->_w = w;
        return 0;
    }

    template <typename Fn>
    size_t Modify(Fn&& fn) {
        std::lock_guard<std::mutex> g(_modify_mu);
        int bg = !_index.load(std::memory_order_relaxed);
        size_t r = fn(_data[bg]);
        if (!r) return 0;
        _index.store(bg, std::memory_order_release);
        {
            std::lock_guard<std::mutex> g2(_wrappers_mu);
            for (auto& w : _wrappers) {
                w->mu.lock();
                w->mu.unlock();
            }
        }
        size_t r2 = fn(_data[!bg]);
        (void)r2;
        return r;
    }

private:
    Wrapper* local_wrapper() {
        // One wrapper per (thread, instance). A thread-local map keyed by
        // instance pointer keeps this generic without a static per-T slot.
        struct TLS {
            std::vector<std::pair<DoublyBufferedData*, std::shared_ptr<Wrapper>>> v;
        };
        static thread_local TLS tls;
        for (auto& p : tls.v) {
            if (p.first == this && p.second->owner == this) return p.second.get();
        }
        auto w = std::make_shared<Wrapper>();
        w->owner = this;
        {
            std::lock_guard<std::mutex> g(_wrappers_mu);
            _wrappers.push_back(w);
        }
        // drop stale entries of destroyed instances
        tls.v.erase(std::remove_if(tls.v.begin(), tls.v.end(),
                                   [](const std::pair<DoublyBufferedData*, std::shared_ptr<Wrapper>>& p) {
                                       return p.second->owner == nullptr;
                                   }),
                    tls.v.end());
        tls.v.emplace_back(this, w);
        return w.get();
    }
    T _data[2]{};  // value-initialized: scalar T starts at zero in both copies
    std::atomic<int> _index;
    std::mutex _modify_mu;
    std::mutex _wrappers_mu;
    std::vector<std::shared_ptr<Wrapper>> _wrappers;
};

// Intrusive doubly-linked list node.
struct LinkNode {
    LinkNode* prev;
    LinkNode* next;
    LinkNode() : prev(this), next(this) {}
    bool empty() const { return next == this; }
    void insert_before(LinkNode* n) {  // insert this before n
        next = n;
        prev = n->prev;
        n->prev->next = this;
        n->prev = this;
    }
    void remove() {
        prev->next = next;
        next->prev = prev;
        prev = next = this;
    }
};

// Most-recently-used cache with a fixed capacity: Put/Get move the entry
// to the front, inserting past capacity evicts the least recently used
// (reference butil/containers/mru_cache.h). Not thread-safe.
template <typename K, typename V, typename Hash = std::hash<K>>
class MRUCache {
public:
    explicit MRUCache(size_t capacity) : _cap(capacity ? capacity : 1) {}
    // Insert or overwrite; returns true if an old entry was evicted.
    bool Put(const K& k, V v, K* evicted_key = nullptr) {
        auto it = _index.find(k);
        if (it != _index.end()) {
            it->second->second = std::move(v);
            _order.splice(_order.begin(), _order, it->second);
            return false;
        }
        _order.emplace_front(k, std::move(v));
        _index[k] = _order.begin();
        if (_order.size() <= _cap) return false;
        if (evicted_key) *evicted_key = _order.back().first;
        _index.erase(_order.back().first);
        _order.pop_back();
        return true;
    }
    // Pointer to the value (refreshes recency), nullptr if absent.
    V* Get(const K& k) {
        auto it = _index.find(k);
        if (it == _index.end()) return nullptr;
        _order.splice(_order.begin(), _order, it->second);
        return &it->second->second;
    }
    // Lookup without touching recency.
    const V* Peek(const K& k) const {
        auto it = _index.find(k);
        return it == _index.end() ? nullptr : &it->second->second;
    }
    bool Erase(const K& k) {
        auto it = _index.find(k);
        if (it == _index.end()) return false;
        _order.erase(it->second);
        _index.erase(it);
        return true;
    }
    size_t size() const { return _order.size(); }
    size_t capacity() const { return _cap; }
    void clear() {
        _order.clear();
        _index.clear();
    }
    // Iterate from most to least recently used.
    template <typename Fn>
    void for_each(Fn fn) const {
        for (const auto& kv : _order) fn(kv.first, kv.second);
    }

private:
    size_t _cap;
    std::list<std::pair<K, V>> _order;
    std::unordered_map<K, typename std::list<std::pair<K, V>>::iterator, Hash> _index;
};

}  // namespace mrpc
