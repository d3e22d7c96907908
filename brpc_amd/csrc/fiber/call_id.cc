#include "fiber/call_id.h"

#include <cerrno>
#include <deque>
#include <mutex>

#include "base/logging.h"
#include "base/pool.h"
#include "fiber/butex.h"

namespace mrpc {
namespace fiber {

namespace {
struct PendingError {
    CallId id;
    int code;
    std::string text;
};

// butex values relative to the current range:
//   first_ver                 unlocked
//   locked_ver                locked
//   locked_ver + 1            locked and contended
//   locked_ver + 2            locked, about to be destroyed (lock -> EPERM)
//   locked_ver + 3 (end_ver)  destroyed; becomes first_ver of the next use
struct IdSlot {
    std::mutex mu;
    uint32_t first_ver = 1;
    uint32_t locked_ver = 1;
    void* data = nullptr;
    CallIdOnError on_error = nullptr;
    std::atomic<int>* butex = nullptr;
    std::atomic<int>* join_butex = nullptr;
    std::deque<PendingError> pending;

    bool has_version(uint32_t v) const { return v >= first_ver && v < locked_ver; }
    uint32_t contended_ver() const { return locked_ver + 1; }
    uint32_t unlockable_ver() const { return locked_ver + 2; }
    uint32_t end_ver() const { return locked_ver + 3; }
};

inline uint32_t id_slot(CallId id) { return (uint32_t)(id.value >> 32); }
inline uint32_t id_ver(CallId id) { return (uint32_t)id.value; }
inline CallId make_id(uint32_t slot, uint32_t ver) { return CallId{((uint64_t)slot << 32) | ver}; }

IdSlot* get_slot(CallId id) { return address_resource<IdSlot>(id_slot(id)); }

int default_on_error(CallId id, void*, int, const std::string&) { return call_id_unlock_and_destroy(id); }
}  // namespace

int call_id_create_ranged(CallId* id, void* data, CallIdOnError on_error, int range) {
    if (range < 1 || range > 1024) return EINVAL;
    uint32_t slot;
    IdSlot* s = get_resource<IdSlot>(&slot);
    if (!s) return ENOMEM;
    std::lock_guard<std::mutex> g(s->mu);
    if (!s->butex) {
        s->butex = butex_create();
        s->join_butex = butex_create();
    }
    // first_ver is already past every version ever handed out for this slot.
    if (s->first_ver == 0) s->first_ver = 1;
    s->locked_ver = s->first_ver + (uint32_t)range;
    s->data = data;
    s->on_error = on_error ? on_error : default_on_error;
    s->pending.clear();
    s->butex->store((int)s->first_ver, std::memory_order_release);
    s->join_butex->store((int)s->first_ver, std::memory_order_release);
    *id = make_id(slot, s->first_ver);
    return 0;
}

int call_id_create(CallId* id, void* data, CallIdOnError on_error) {
    return call_id_create_ranged(id, data, on_error, 1);
}

static int lock_impl(CallId id, void** pdata, int range, bool try_only) {
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    std::unique_lock<std::mutex> g(s->mu);
    bool waited = false;
    for (;;) {
        if (!s->has_version(ver)) return EINVAL;
        const uint32_t v = (uint32_t)s->butex->load(std::memory_order_relaxed);
        if (v == s->first_ver) {
            if (range > 0 && s->first_ver + (uint32_t)range > s->locked_ver) s->locked_ver = s->first_ver + (uint32_t)range;
            s->butex->store((int)(waited ? s->contended_ver() : s->locked_ver), std::memory_order_relaxed);
            if (pdata) *pdata = s->data;
            return 0;
        }
        if (v == s->unlockable_ver()) return EPERM;
        if (try_only) return EBUSY;
        const int expected = (int)s->contended_ver();
        s->butex->store(expected, std::memory_order_relaxed);
        g.unlock();
        butex_wait(s->butex, expected, nullptr);
        waited = true;
        g.lock();
    }
}

int call_id_lock(CallId id, void** pdata) { return lock_impl(id, pdata, 0, false); }
int call_id_trylock(CallId id, void** pdata) { return lock_impl(id, pdata, 0, true); }

int call_id_lock_and_reset_range(CallId id, void** pdata, int range) {
    if (range < 1 || range > 1024) return EINVAL;
    return lock_impl(id, pdata, range, false);
}

int call_id_unlock(CallId id) {
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    std::unique_lock<std::mutex> g(s->mu);
    if (!s->has_version(ver)) return EINVAL;
    const uint32_t v = (uint32_t)s->butex->load(std::memory_order_relaxed);
    if (v == s->first_ver) {
        LOG(ERROR) << "call_id_unlock on an unlocked id";
        return EPERM;
    }
    if (!s->pending.empty()) {
        // Hand the lock over to the queued error handler.
        PendingError pe = std::move(s->pending.front());
        s->pending.pop_front();
        void* data = s->data;
        CallIdOnError fn = s->on_error;
        g.unlock();
        fn(pe.id, data, pe.code, pe.text);
        return 0;
    }
    const bool contended = (v == s->contended_ver() || v == s->unlockable_ver());
    s->butex->store((int)s->first_ver, std::memory_order_release);
    g.unlock();
    if (contended) butex_wake_all(s->butex);
    return 0;
}

int call_id_unlock_and_destroy(CallId id) {
    uint32_t slot = id_slot(id);
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    std::unique_lock<std::mutex> g(s->mu);
    if (!s->has_version(ver)) return EINVAL;
    const uint32_t v = (uint32_t)s->butex->load(std::memory_order_relaxed);
    if (v == s->first_ver) {
        LOG(ERROR) << "call_id_unlock_and_destroy on an unlocked id";
        return EPERM;
    }
    const uint32_t next = s->end_ver();
    s->first_ver = next;
    s->locked_ver = next;
    s->pending.clear();
    s->butex->store((int)next, std::memory_order_release);
    s->join_butex->store((int)next, std::memory_order_release);
    g.unlock();
    butex_wake_all(s->butex);
    butex_wake_all(s->join_butex);
    return_resource<IdSlot>(slot);
    return 0;
}

int call_id_about_to_destroy(CallId id) {
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    std::unique_lock<std::mutex> g(s->mu);
    if (!s->has_version(ver)) return EINVAL;
    const uint32_t v = (uint32_t)s->butex->load(std::memory_order_relaxed);
    if (v == s->first_ver) return EPERM;
    const bool contended = (v == s->contended_ver());
    s->butex->store((int)s->unlockable_ver(), std::memory_order_release);
    g.unlock();
    if (contended) butex_wake_all(s->butex);
    return 0;
}

int call_id_cancel(CallId id) {
    uint32_t slot = id_slot(id);
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    std::unique_lock<std::mutex> g(s->mu);
    if (!s->has_version(ver)) return EINVAL;
    if ((uint32_t)s->butex->load(std::memory_order_relaxed) != s->first_ver) return EPERM;
    const uint32_t next = s->end_ver();
    s->first_ver = next;
    s->locked_ver = next;
    s->butex->store((int)next, std::memory_order_release);
    s->join_butex->store((int)next, std::memory_order_release);
    g.unlock();
    butex_wake_all(s->join_butex);
    return_resource<IdSlot>(slot);
    return 0;
}

int call_id_error(CallId id, int error_code, const std::string& error_text) {
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    std::unique_lock<std::mutex> g(s->mu);
    if (!s->has_version(ver)) return EINVAL;
    const uint32_t v = (uint32_t)s->butex->load(std::memory_order_relaxed);
    if (v == s->first_ver) {
        s->butex->store((int)s->locked_ver, std::memory_order_relaxed);
        void* data = s->data;
        CallIdOnError fn = s->on_error;
        g.unlock();
        fn(id, data, error_code, error_text);
        return 0;
    }
    if (v == s->unlockable_ver()) return EPERM;
    s->pending.push_back(PendingError{id, error_code, error_text});
    return 0;
}

int call_id_join(CallId id) {
    IdSlot* s = get_slot(id);
    if (!s) return EINVAL;
    const uint32_t ver = id_ver(id);
    for (;;) {
        int expected;
        {
            std::lock_guard<std::mutex> g(s->mu);
            if (!s->has_version(ver)) return 0;
            expected = s->join_butex->load(std::memory_order_relaxed);
        }
        butex_wait(s->join_butex, expected, nullptr);
    }
}

bool call_id_exists(CallId id) {
    IdSlot* s = get_slot(id);
    if (!s) return false;
    std::lock_guard<std::mutex> g(s->mu);
    return s->has_version(id_ver(id));
}

}  // namespace fiber
}  // namespace mrpc
