// Fiber-local storage (role of bthread/key.cpp:407-462): versioned keys,
// per-fiber KeyTables, pthread fallback tables, and KeyTablePools that let
// servers reuse fiber-local data across requests.
#include <cerrno>
#include <mutex>
#include <vector>

#include "base/logging.h"
#include "fiber/internal.h"
#include "fiber/key_internal.h"

namespace mrpc {
namespace fiber {

namespace {
const uint32_t kMaxKeys = 4096;

struct KeyInfo {
    uint32_t version = 1;
    bool used = false;
    void (*dtor)(void*, const void*) = nullptr;
    const void* dtor_arg = nullptr;
};

struct KeyRegistry {
    std::mutex mu;
    KeyInfo infos[kMaxKeys];
    std::vector<uint32_t> free_idx;
    uint32_t next = 0;
};
KeyRegistry& registry() {
    static KeyRegistry* r = new KeyRegistry;
    return *r;
}

inline uint32_t key_index(FiberKey k) { return (uint32_t)(k >> 32); }
inline uint32_t key_version(FiberKey k) { return (uint32_t)k; }

void dtor_adaptor(void* data, const void* arg) {
    void (*d)(void*) = (void (*)(void*))arg;
    if (d) d(data);
}
}  // namespace

struct KeyTable {
    struct Entry {
        uint32_t version = 0;
        void* data = nullptr;
    };
    std::vector<Entry> entries;
    KeyTable* next = nullptr;

    void* get(FiberKey k) {
        uint32_t i = key_index(k);
        if (i >= entries.size()) return nullptr;
        return entries[i].version == key_version(k) ? entries[i].data : nullptr;
    }
    void set(FiberKey k, void* d) {
        uint32_t i = key_index(k);
        if (i >= entries.size()) entries.resize(i + 1);
        entries[i].version = key_version(k);
        entries[i].data = d;
    }
    void destroy_all() {
        KeyRegistry& r = registry();
        // Destructors may set new keys; iterate a few rounds like pthreads.
        for (int round = 0; round < 4; ++round) {
            bool any = false;
            for (uint32_t i = 0; i < entries.size(); ++i) {
                void* d = entries[i].data;
                if (!d) continue;
                uint32_t ver = entries[i].version;
                entries[i].data = nullptr;
                void (*dtor)(void*, const void*) = nullptr;
                const void* arg = nullptr;
                {
                    std::lock_guard<std::mutex> g(r.mu);
                    if (r.infos[i].used && r.infos[i].version == ver) {
                        dtor = r.infos[i].dtor;
                        arg = r.infos[i].dtor_arg;
                    }
                }
                if (dtor) {
                    dtor(d, arg);
                    any = true;
                }
            }
            if (!any) break;
        }
    }
};

struct KeyTablePool {
    std::mutex mu;
    KeyTable* head = nullptr;
    size_t size = 0;
    bool destroyed = false;
};

int key_create2(FiberKey*key, void (*dtor)(void*, const void*), const void* dtor_arg) {
    KeyRegistry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    uint32_t idx;
    if (!r.free_idx.empty()) {
        idx = r.free_idx.back();
        r.free_idx.pop_back();
    } else {
        if (r.next >= kMaxKeys) return EAGAIN;
        idx = r.next++;
    }
    KeyInfo& ki = r.infos[idx];
    __atomic_store_n(&ki.used, true, __ATOMIC_RELEASE);  // read lock-free by setspecific
    ki.dtor = dtor;
    ki.dtor_arg = dtor_arg;
    *key = ((uint64_t)idx << 32) | ki.version;
    return 0;
}

int key_create(FiberKey*key, void (*dtor)(void*)) {
    return key_create2(key, dtor ? dtor_adaptor : nullptr, (const void*)dtor);
}

int key_delete(FiberKey key) {
    KeyRegistry& r = registry();
    std::lock_guard<std::mutex> g(r.mu);
    uint32_t idx = key_index(key);
    if (idx >= kMaxKeys || !r.infos[idx].used || r.infos[idx].version != key_version(key)) return EINVAL;
    __atomic_store_n(&r.infos[idx].used, false, __ATOMIC_RELEASE);
    r.infos[idx].dtor = nullptr;
    uint32_t v = r.infos[idx].version + 1;
    if (v == 0) v = 1;
    __atomic_store_n(&r.infos[idx].version, v, __ATOMIC_RELEASE);
    r.free_idx.push_back(idx);
    return 0;
}

static thread_local KeyTable* tls_pthread_table = nullptr;
struct PthreadTableCleaner {
    ~PthreadTableCleaner() {
        if (tls_pthread_table) {
            tls_pthread_table->destroy_all();
            delete tls_pthread_table;
            tls_pthread_table = nullptr;
        }
    }
};
static thread_local PthreadTableCleaner tls_cleaner;

static KeyTable** current_table_slot() {
    TaskGroup* g = tls_group();
    if (g && !g->is_current_main_task()) return &g->current_task()->local_storage;
    (void)tls_cleaner;
    return &tls_pthread_table;
}

int setspecific(FiberKey key, void* data) {
    // a key that was never created, or was deleted (its slot's version moved
    // on), is refused like the reference's bthread_setspecific (EINVAL)
    {
        KeyRegistry& r = registry();
        const uint32_t idx = key_index(key);
        if (idx >= kMaxKeys || !__atomic_load_n(&r.infos[idx].used, __ATOMIC_ACQUIRE) ||
            __atomic_load_n(&r.infos[idx].version, __ATOMIC_ACQUIRE) != key_version(key)) {
            return EINVAL;
        }
    }
    KeyTable** slot = current_table_slot();
    if (!*slot) {
        TaskGroup* g = tls_group();
        KeyTablePool* pool = (g && !g->is_current_main_task()) ? g->current_task()->attr.keytable_pool : nullptr;
        *slot = pool ? borrow_keytable(pool) : nullptr;
        if (!*slot) *slot = new KeyTable;
    }
    (*slot)->set(key, data);
    return 0;
}

void* getspecific(FiberKey key) {
    KeyTable** slot = current_table_slot();
    if (!*slot) {
        TaskGroup* g = tls_group();
        if (g && !g->is_current_main_task() && g->current_task()->attr.keytable_pool) {
            *slot = borrow_keytable(g->current_task()->attr.keytable_pool);
        }
        if (!*slot) return nullptr;
    }
    return (*slot)->get(key);
}

KeyTable* borrow_keytable(KeyTablePool* pool) {
    if (!pool) return nullptr;
    std::lock_guard<std::mutex> g(pool->mu);
    KeyTable* kt = pool->head;
    if (kt) {
        pool->head = kt->next;
        kt->next = nullptr;
        --pool->size;
    }
    return kt;
}

void return_keytable(KeyTablePool* pool, KeyTable* kt) {
    if (!kt) return;
    if (pool) {
        std::lock_guard<std::mutex> g(pool->mu);
        if (!pool->destroyed) {
            kt->next = pool->head;
            pool->head = kt;
            ++pool->size;
            return;
        }
    }
    kt->destroy_all();
    delete kt;
}

KeyTablePool* keytable_pool_create() { return new KeyTablePool; }

void keytable_pool_destroy(KeyTablePool* p) {
    if (!p) return;
    KeyTable* head;
    {
        std::lock_guard<std::mutex> g(p->mu);
        p->destroyed = true;
        head = p->head;
        p->head = nullptr;
        p->size = 0;
    }
    while (head) {
        KeyTable* n = head->next;
        head->destroy_all();
        delete head;
        head = n;
    }
    // The pool object itself is leaked intentionally: fibers still running
    // may return tables to it (they will see destroyed=true).
}

size_t keytable_pool_size(KeyTablePool* p) {
    std::lock_guard<std::mutex> g(p->mu);
    return p->size;
}

}  // namespace fiber
}  // namespace mrpc
