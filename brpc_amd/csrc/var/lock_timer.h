// Lock contention as a metric (role of the reference's
// bvar/utils/lock_timer.h: MutexWithRecorder / MutexWithLatencyRecorder and
// LockTimer). Every acquisition records how long the caller waited for the
// lock, in microseconds, into an IntRecorder (average wait) or a
// LatencyRecorder (percentiles, max, acquisitions per second).
//
//   var::MutexWithLatencyRecorder<std::mutex> mu("my_table_lock");
//   { std::lock_guard<decltype(mu)> g(mu); ... }   // works with std guards
#pragma once

#include <mutex>
#include <string>

#include "base/time.h"
#include "var/percentile.h"
#include "var/recorder.h"

namespace mrpc {
namespace var {

template <typename Mutex, typename Recorder>
class MutexWithRecorderBase {
public:
    MutexWithRecorderBase() {}
    // Exposes the recorder as `name` (a LatencyRecorder exposes the family
    // name_latency, name_max_latency, name_qps, ...).
    explicit MutexWithRecorderBase(const std::string& name) { _recorder.expose(name); }
    void lock() {
        const int64_t t0 = monotonic_us();
        _mu.lock();
        _recorder << (monotonic_us() - t0);
    }
    bool try_lock() {
        // an uncontended acquisition costs nothing to record
        if (!_mu.try_lock()) return false;
        _recorder << 0;
        return true;
    }
    void unlock() { _mu.unlock(); }
    Mutex& native() { return _mu; }
    Recorder& recorder() { return _recorder; }
    const Recorder& recorder() const { return _recorder; }

private:
    Mutex _mu;
    Recorder _recorder;
};

template <typename Mutex = std::mutex>
using MutexWithRecorder = MutexWithRecorderBase<Mutex, IntRecorder>;
template <typename Mutex = std::mutex>
using MutexWithLatencyRecorder = MutexWithRecorderBase<Mutex, LatencyRecorder>;

// Times the acquisition of any lockable into a recorder supplied by the
// caller (for locks that cannot be wrapped): `LockTimer<std::mutex, IntRecorder>
// t(mu, rec);` locks, records the wait and unlocks at scope end.
template <typename Mutex, typename Recorder>
class LockTimer {
public:
    LockTimer(Mutex& mu, Recorder& rec) : _mu(mu) {
        const int64_t t0 = monotonic_us();
        _mu.lock();
        rec << (monotonic_us() - t0);
    }
    ~LockTimer() { _mu.unlock(); }
    LockTimer(const LockTimer&) = delete;
    LockTimer& operator=(const LockTimer&) = delete;

private:
    Mutex& _mu;
};

}  // namespace var
}  // namespace mrpc
