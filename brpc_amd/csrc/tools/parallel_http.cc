// parallel_http: fetch many http urls concurrently (role of the reference's
// tools/parallel_http). Urls come from -url_file (one per line) or -url
// (repeated -count times); -thread_num fibers share the list; each result
// prints as "<status> <bytes> <ms> <url>" and a summary follows.
#include <atomic>
#include <cstdio>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "http/http_client.h"

DEFINE_string(url_file, "", "file with one url per line");
DEFINE_string(url, "", "a single url (with -count)");
DEFINE_int32(count, 1, "times to fetch -url");
DEFINE_int32(thread_num, 32, "concurrent fetching fibers");
DEFINE_int32(timeout_ms, 3000, "timeout of each fetch");
DEFINE_bool(quiet, false, "print only the summary");

using namespace mrpc;

int main(int argc, char** argv) {
    ParseCommandLineFlags(&argc, &argv);
    std::vector<std::string> urls;
    if (!FLAGS_url_file.empty()) {
        std::ifstream f(FLAGS_url_file);
        std::string line;
        while (std::getline(f, line)) {
            while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
            if (!line.empty() && line[0] != '#') urls.push_back(line);
        }
    }
    for (int i = 0; !FLAGS_url.empty() && i < FLAGS_count; ++i) urls.push_back(FLAGS_url);
    if (urls.empty()) {
        fprintf(stderr, "usage: parallel_http -url_file=FILE | -url=URL [-count=N] [-thread_num=N]\n");
        return 1;
    }
    fiber::init_runtime();
    std::atomic<size_t> next{0};
    std::atomic<int64_t> ok{0}, failed{0}, bytes{0};
    std::mutex out_mu;
    const int64_t t0 = monotonic_us();
    const int n = std::max(1, std::min<int>(FLAGS_thread_num, (int)urls.size()));
    fiber::CountdownEvent all(n);
    for (int t = 0; t < n; ++t) {
        fiber::start([&] {
            for (size_t i; (i = next.fetch_add(1)) < urls.size();) {
                HttpSimpleResponse resp;
                const int64_t s = monotonic_us();
                const int rc = HttpFetch("GET", urls[i], "", &resp, FLAGS_timeout_ms);
                const double ms = (monotonic_us() - s) / 1000.0;
                (rc == 0 ? ok : failed).fetch_add(1);
                bytes.fetch_add((int64_t)resp.body.size());
                if (!FLAGS_quiet) {
                    std::lock_guard<std::mutex> g(out_mu);
                    printf("%d %zu %.2f %s\n", resp.status, resp.body.size(), ms, urls[i].c_str());
                }
            }
            all.signal();
        });
    }
    all.wait();
    const double sec = (monotonic_us() - t0) / 1e6;
    printf("fetched %zu urls in %.3fs: ok=%lld failed=%lld bytes=%lld (%.1f urls/s)\n", urls.size(), sec,
           (long long)ok.load(), (long long)failed.load(), (long long)bytes.load(), urls.size() / std::max(sec, 1e-9));
    return failed.load() ? 2 : 0;
}
