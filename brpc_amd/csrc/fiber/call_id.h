// CallId: 64-bit versioned lockable identifier with a range of versions.
// This is the RPC correlation-id mechanism (role of bthread_id, reference
// src/bthread/id.cpp:101-608; controller.cpp:996-1003 uses one version per
// retry/backup attempt). Capabilities: lock/unlock, error() that runs the
// on_error handler under the lock (or queues it while locked), join (wait for
// destruction), about_to_destroy, lock_and_reset_range.
#pragma once

#include <cstdint>
#include <string>

namespace mrpc {
namespace fiber {

struct CallId {
    uint64_t value;
    bool operator==(const CallId& o) const { return value == o.value; }
    bool operator!=(const CallId& o) const { return value != o.value; }
};
const CallId INVALID_CALL_ID = {0};

// on_error(id, data, error_code, error_text) is called with the id LOCKED; it
// must unlock or unlock_and_destroy the id.
typedef int (*CallIdOnError)(CallId id, void* data, int error_code, const std::string& error_text);

int call_id_create(CallId* id, void* data, CallIdOnError on_error);
int call_id_create_ranged(CallId* id, void* data, CallIdOnError on_error, int range);
// Returns 0 and *data; EINVAL if the id (version) is invalid/destroyed;
// EPERM if about_to_destroy was called.
int call_id_lock(CallId id, void** pdata);
int call_id_trylock(CallId id, void** pdata);
int call_id_lock_and_reset_range(CallId id, void** pdata, int range);
int call_id_unlock(CallId id);
int call_id_unlock_and_destroy(CallId id);
int call_id_about_to_destroy(CallId id);
int call_id_cancel(CallId id);  // destroy an id that was never locked
int call_id_error(CallId id, int error_code, const std::string& error_text = std::string());
int call_id_join(CallId id);
// Version arithmetic helpers: ids of successive versions in a range.
inline CallId call_id_with_version(CallId base, int nth) { return CallId{base.value + (uint64_t)nth}; }
inline uint32_t call_id_version(CallId id) { return (uint32_t)id.value; }
bool call_id_exists(CallId id);

}  // namespace fiber
}  // namespace mrpc
