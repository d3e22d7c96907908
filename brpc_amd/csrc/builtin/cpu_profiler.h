// Sampling CPU profiler behind /hotspots/cpu and /pprof/profile (the
// reference links gperftools for this: src/brpc/builtin/hotspots_service.cpp,
// pprof_service.cpp). SIGPROF from ITIMER_PROF samples the interrupted
// thread's stack (backtrace()) into a preallocated ring; the result is
// rendered as folded stacks (flame-graph input) or as a gperftools legacy
// binary profile that `pprof` reads.
#pragma once

#include <cstdint>
#include <string>

namespace mrpc {
namespace profiler {

// Profile the whole process for `seconds` (blocking the caller; use from a
// fiber). Returns false if another profile is running.
bool ProfileCpu(double seconds, int frequency_hz, std::string* folded, std::string* pprof_binary,
                int64_t* nsamples);
bool IsCpuProfilerRunning();
// addr -> "symbol+off" (demangled) for /pprof/symbol
std::string Symbolize(uintptr_t addr);

}  // namespace profiler
}  // namespace mrpc
