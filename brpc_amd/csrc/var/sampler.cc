#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "base/time.h"
#include "var/window.h"

namespace mrpc {
namespace var {

namespace {
struct SamplerCollector {
    std::mutex mu;  // held while sampling: unschedule() waits on it
    std::vector<Sampler*> samplers;
    bool started = false;
    void ensure_started() {
        if (started) return;
        started = true;
        std::thread([this] {
            pthread_setname_np(pthread_self(), "mrpc_sampler");
            int64_t next = monotonic_us() + 1000000;
            for (;;) {
                int64_t now = monotonic_us();
                if (now < next) ::usleep((useconds_t)(next - now));
                next += 1000000;
                std::lock_guard<std::mutex> g(mu);
                for (Sampler* s : samplers) s->take_sample();
            }
        }).detach();
    }
};
SamplerCollector& collector() {
    static SamplerCollector* c = new SamplerCollector;
    return *c;
}
}  // namespace

void Sampler::schedule() {
    SamplerCollector& c = collector();
    std::lock_guard<std::mutex> g(c.mu);
    c.samplers.push_back(this);
    c.ensure_started();
}

void Sampler::unschedule() {
    SamplerCollector& c = collector();
    std::lock_guard<std::mutex> g(c.mu);
    c.samplers.erase(std::remove(c.samplers.begin(), c.samplers.end(), this), c.samplers.end());
}

}  // namespace var
}  // namespace mrpc
