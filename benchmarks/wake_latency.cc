// Wake-up latency of an idle thread on this host: a sender writes an eventfd
// every --gap_us and a receiver waiting in epoll measures how long the wake
// took (send timestamp -> receiver running). Modes of waiting:
//   block   epoll_wait(-1): the kernel idles the core (deep C-states possible)
//   nap:N   epoll_pwait2 with an N us timeout in a loop: the core wakes every
//           N us, so the idle governor only picks shallow states
//   spin    epoll_wait(0) in a loop (a burning core)
// Prints p50/p90/p99/p999 per mode and the receiver's CPU use.
//
//   g++ -O2 -pthread benchmarks/wake_latency.cc -o build/bin/wake_latency
//   build/bin/wake_latency --gap_us 10000 --samples 600
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/resource.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static int64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

static double thread_cpu_s() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct Result {
    std::vector<int64_t> lat_ns;
    double cpu_s = 0, wall_s = 0;
};

static Result run(const std::string& mode, int gap_us, int samples) {
    const int efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    const int ep = epoll_create1(EPOLL_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLET;
    ev.data.fd = efd;
    epoll_ctl(ep, EPOLL_CTL_ADD, efd, &ev);
    std::atomic<int64_t> sent_at{0};
    std::atomic<bool> stop{false};
    Result r;
    r.lat_ns.reserve(samples);
    const int nap_us = mode.rfind("nap:", 0) == 0 ? atoi(mode.c_str() + 4) : 0;
    std::thread rx([&] {
        const double c0 = thread_cpu_s();
        const int64_t w0 = now_ns();
        epoll_event e[4];
        while (!stop.load(std::memory_order_relaxed)) {
            int n;
            if (mode == "spin") {
                n = epoll_wait(ep, e, 4, 0);
            } else if (nap_us > 0) {
                timespec ts{0, (long)nap_us * 1000};
                n = epoll_pwait2(ep, e, 4, &ts, nullptr);
            } else {
                n = epoll_wait(ep, e, 4, 100);
            }
            if (n <= 0) continue;
            const int64_t t = now_ns();
            uint64_t v;
            while (read(efd, &v, sizeof(v)) > 0) {
            }
            const int64_t s = sent_at.load(std::memory_order_acquire);
            if (s) r.lat_ns.push_back(t - s);
        }
        r.cpu_s = thread_cpu_s() - c0;
        r.wall_s = (now_ns() - w0) * 1e-9;
    });
    usleep(20000);
    for (int i = 0; i < samples; ++i) {
        usleep(gap_us);
        sent_at.store(now_ns(), std::memory_order_release);
        const uint64_t one = 1;
        if (write(efd, &one, sizeof(one)) != sizeof(one)) perror("write");
    }
    usleep(20000);
    stop = true;
    const uint64_t one = 1;
    if (write(efd, &one, sizeof(one)) < 0) perror("write");
    rx.join();
    close(ep);
    close(efd);
    return r;
}

int main(int argc, char** argv) {
    int gap_us = 10000, samples = 500;
    std::vector<std::string> modes = {"block", "nap:20", "nap:50", "nap:200", "spin"};
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--gap_us")) gap_us = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--samples")) samples = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--modes")) {
            modes.clear();
            std::string s = argv[i + 1];
            size_t p = 0;
            while (p <= s.size()) {
                size_t q = s.find(',', p);
                if (q == std::string::npos) q = s.size();
                modes.push_back(s.substr(p, q - p));
                p = q + 1;
            }
        }
    }
    for (const std::string& m : modes) {
        Result r = run(m, gap_us, samples);
        std::vector<int64_t>& v = r.lat_ns;
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        auto pct = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * v.size()))] / 1000.0; };
        printf("mode=%-8s gap_us=%d n=%zu p50=%.1f p90=%.1f p99=%.1f p999=%.1f max=%.1f us  rx_cpu=%.1f%%\n",
               m.c_str(), gap_us, v.size(), pct(0.5), pct(0.9), pct(0.99), pct(0.999), v.back() / 1000.0,
               100.0 * r.cpu_s / std::max(1e-9, r.wall_s));
        fflush(stdout);
    }
    return 0;
}
