// Memcache client (reference example/memcache_c++): batches of binary-
// protocol operations pipelined on one connection by the "memcache"
// channel protocol — SET a batch of keys, GET them back, counters, ADD
// conflicts, DELETE — then -thread_num threads hammer GETs for a while.
// The reference needs a real memcached; this demo starts a small one
// in-process (binary protocol, a connection per thread) when -server is
// empty.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "base/time.h"
#include "examples/common.h"
#include "redis/memcache.h"

DEFINE_string(server, "", "memcached ip:port (empty: start the in-process one)");
DEFINE_int32(batch, 100, "operations per pipelined request (>= 3: the checks append to key_1 and delete key_2)");
DEFINE_int32(thread_num, 4, "threads of the load phase");
DEFINE_double(duration_s, 0.5, "seconds of the load phase");

namespace {

// Minimal memcached speaking the binary protocol (enough for the demo).
class MiniMemcached {
public:
    MiniMemcached() {
        _lfd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        socklen_t len = sizeof(a);
        if (bind(_lfd, (sockaddr*)&a, sizeof(a)) != 0 || listen(_lfd, 64) != 0 ||
            getsockname(_lfd, (sockaddr*)&a, &len) != 0) {
            LOG(FATAL) << "mini memcached: cannot listen";
        }
        _port = ntohs(a.sin_port);
        _acceptor = std::thread([this] { accept_loop(); });
    }
    ~MiniMemcached() {
        shutdown(_lfd, SHUT_RDWR);
        close(_lfd);
        _acceptor.join();
        {
            std::lock_guard<std::mutex> g(_mu);
            for (int fd : _fds) shutdown(fd, SHUT_RDWR);  // clients may keep connections open
        }
        for (auto& t : _conns) t.join();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(_port); }

private:
    struct Item {
        std::string value;
        uint32_t flags = 0;
        uint64_t cas = 0;
    };
    static uint64_t be(const char* p, int n) {
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 8) | (uint8_t)p[i];
        return v;
    }
    static void put_be(std::string* s, uint64_t v, int n) {
        for (int i = n - 1; i >= 0; --i) s->push_back((char)(v >> (8 * i)));
    }
    static bool read_full(int fd, char* p, size_t n) {
        while (n) {
            const ssize_t r = read(fd, p, n);
            if (r <= 0) return false;
            p += r;
            n -= (size_t)r;
        }
        return true;
    }
    static void respond(std::string* out, uint8_t op, uint16_t status, const std::string& ext, const std::string& val,
                        uint64_t cas, uint32_t opaque) {
        out->push_back((char)0x81);
        out->push_back((char)op);
        put_be(out, 0, 2);
        out->push_back((char)ext.size());
        out->push_back(0);
        put_be(out, status, 2);
        put_be(out, ext.size() + val.size(), 4);
        put_be(out, opaque, 4);
        put_be(out, cas, 8);
        *out += ext + val;
    }
    void accept_loop() {
        for (;;) {
            const int fd = accept(_lfd, nullptr, nullptr);
            if (fd < 0) return;
            // one write per response: without NODELAY, Nagle holds every
            // response after the first of a pipelined batch until the
            // client's delayed ACK (~30 ms per batch of 10 GETs)
            const int one = 1;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
            {
                std::lock_guard<std::mutex> g(_mu);
                _fds.push_back(fd);
            }
            _conns.emplace_back([this, fd] { serve(fd); });
        }
    }
    void serve(int fd) {
        char h[24];
        while (read_full(fd, h, 24)) {
            const uint8_t op = (uint8_t)h[1];
            const size_t klen = be(h + 2, 2), elen = (uint8_t)h[4], blen = be(h + 8, 4);
            const uint32_t opaque = (uint32_t)be(h + 12, 4);
            const uint64_t req_cas = be(h + 16, 8);
            std::string body(blen, '\0');
            if (blen && !read_full(fd, &body[0], blen)) break;
            const std::string ext = body.substr(0, elen), key = body.substr(elen, klen), val = body.substr(elen + klen);
            std::string out;
            std::lock_guard<std::mutex> g(_mu);
            auto it = _kv.find(key);
            switch (op) {
            case 0x00:  // GET
                if (it == _kv.end()) {
                    respond(&out, op, 0x01, "", "Not found", 0, opaque);
                } else {
                    std::string fl;
                    put_be(&fl, it->second.flags, 4);
                    respond(&out, op, 0, fl, it->second.value, it->second.cas, opaque);
                }
                break;
            case 0x01: case 0x02: case 0x03: {  // SET ADD REPLACE
                const bool exists = it != _kv.end();
                if ((op == 0x02 && exists) || (op == 0x03 && !exists) ||
                    (req_cas && (!exists || it->second.cas != req_cas))) {
                    respond(&out, op, exists ? 0x02 : 0x01, "", "", 0, opaque);
                    break;
                }
                Item& item = _kv[key];
                item.value = val;
                item.flags = (uint32_t)be(ext.data(), 4);
                item.cas = ++_cas;
                respond(&out, op, 0, "", "", item.cas, opaque);
                break;
            }
            case 0x0e: case 0x0f:  // APPEND PREPEND
                if (it == _kv.end()) {
                    respond(&out, op, 0x05, "", "", 0, opaque);
                } else {
                    it->second.value = op == 0x0e ? it->second.value + val : val + it->second.value;
                    it->second.cas = ++_cas;
                    respond(&out, op, 0, "", "", it->second.cas, opaque);
                }
                break;
            case 0x04:  // DELETE
                respond(&out, op, _kv.erase(key) ? 0 : 0x01, "", "", 0, opaque);
                break;
            case 0x05: case 0x06: {  // INCR DECR
                const uint64_t delta = be(ext.data(), 8), init = be(ext.data() + 8, 8);
                uint64_t v = init;
                if (it != _kv.end()) {
                    const uint64_t cur = strtoull(it->second.value.c_str(), nullptr, 10);
                    v = op == 0x05 ? cur + delta : (cur > delta ? cur - delta : 0);
                }
                Item& item = _kv[key];
                item.value = std::to_string(v);
                item.cas = ++_cas;
                std::string num;
                put_be(&num, v, 8);
                respond(&out, op, 0, "", num, item.cas, opaque);
                break;
            }
            case 0x0b:  // VERSION
                respond(&out, op, 0, "", "1.6-mini", 0, opaque);
                break;
            default:
                respond(&out, op, 0x81, "", "Unknown command", 0, opaque);
            }
            if (write(fd, out.data(), out.size()) != (ssize_t)out.size()) break;
        }
        std::lock_guard<std::mutex> g(_mu);
        _fds.erase(std::find(_fds.begin(), _fds.end(), fd));
        close(fd);
    }
    int _lfd = -1, _port = 0;
    std::thread _acceptor;
    std::vector<std::thread> _conns;
    std::vector<int> _fds;
    std::mutex _mu;
    std::map<std::string, Item> _kv;
    uint64_t _cas = 0;
};

}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    std::unique_ptr<MiniMemcached> local;
    std::string addr = FLAGS_server;
    if (addr.empty()) {
        local.reset(new MiniMemcached);
        addr = local->addr();
    }
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "memcache";
    opt.timeout_ms = 2000;
    if (ch.Init(addr.c_str(), &opt) != 0) return 1;
    bool ok = true;
    {  // one pipelined request: VERSION + a batch of SETs
        mrpc::MemcacheRequest req;
        mrpc::MemcacheResponse res;
        mrpc::Controller cntl;
        req.Version();
        for (int i = 0; i < FLAGS_batch; ++i) req.Set("key_" + std::to_string(i), "value_" + std::to_string(i), 0xf00 + i, 0, 0);
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        std::string version;
        ok = !cntl.Failed() && res.PopVersion(&version);
        for (int i = 0; i < FLAGS_batch && ok; ++i) {
            uint64_t cas = 0;
            ok = res.PopSet(&cas) && cas != 0;
        }
        printf("version %s, %d keys set in one round trip (%lld us)\n", version.c_str(), FLAGS_batch,
               (long long)cntl.latency_us());
    }
    {  // GET them back, a counter, an ADD conflict and a DELETE, pipelined
        mrpc::MemcacheRequest req;
        mrpc::MemcacheResponse res;
        mrpc::Controller cntl;
        for (int i = 0; i < FLAGS_batch; ++i) req.Get("key_" + std::to_string(i));
        req.Increment("hits", 5, 100, 0);
        req.Increment("hits", 5, 100, 0);
        req.Add("key_0", "again", 0, 0, 0);
        req.Append("key_1", "+tail", 0, 0, 0);
        req.Get("key_1");
        req.Delete("key_2");
        req.Get("key_2");
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ok = ok && !cntl.Failed();
        for (int i = 0; i < FLAGS_batch && ok; ++i) {
            std::string v;
            uint32_t flags = 0;
            uint64_t cas = 0;
            ok = res.PopGet(&v, &flags, &cas) && v == "value_" + std::to_string(i) && flags == (uint32_t)(0xf00 + i);
        }
        uint64_t h1 = 0, h2 = 0, cas = 0;
        ok = ok && res.PopIncrement(&h1, &cas) && res.PopIncrement(&h2, &cas) && h1 == 100 && h2 == 105;
        ok = ok && !res.PopAdd(&cas);  // key exists
        std::string v;
        uint32_t flags;
        ok = ok && res.PopAppend(&cas) && res.PopGet(&v, &flags, &cas) && v == "value_1+tail";
        ok = ok && res.PopDelete() && !res.PopGet(&v, &flags, &cas);
        printf("batch of %d GETs + counters/add/append/delete: %s\n", FLAGS_batch + 7, ok ? "as expected" : "MISMATCH");
    }
    // load phase: threads issue pipelined GET batches of 10
    std::atomic<bool> stop{false};
    std::atomic<int64_t> ops{0}, errors{0};
    std::vector<std::thread> th;
    for (int t = 0; t < FLAGS_thread_num; ++t) {
        th.emplace_back([&, t] {
            int i = t;
            while (!stop.load(std::memory_order_relaxed)) {
                mrpc::MemcacheRequest req;
                mrpc::MemcacheResponse res;
                mrpc::Controller cntl;
                for (int k = 0; k < 10; ++k) req.Get("key_" + std::to_string((i + k) % FLAGS_batch));
                ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
                if (cntl.Failed()) ++errors;
                else ops += 10;
                i += 10;
            }
        });
    }
    mrpc::fiber::usleep((uint64_t)(FLAGS_duration_s * 1e6));
    stop = true;
    for (auto& t : th) t.join();
    printf("load: %lld GETs/s over %d threads, %lld failed calls\n", (long long)(ops / FLAGS_duration_s),
           FLAGS_thread_num, (long long)errors.load());
    return demo::Check(ok && errors.load() == 0 && ops.load() > 0, "memcache binary protocol pipelining");
}
