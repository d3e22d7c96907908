#include "rpc/rpc_dump.h"

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <memory>
#include <mutex>

#include "base/logging.h"
#include "base/recordio.h"
#include "base/time.h"
#include "base/util.h"

DEFINE_bool(rpc_dump, false, "sample requests into -rpc_dump_dir for rpc_replay");
DEFINE_string(rpc_dump_dir, "./rpc_data/rpc_dump", "directory of rpc_dump files");
DEFINE_int32(rpc_dump_max_files, 32, "keep at most this many dump files in -rpc_dump_dir");
DEFINE_int32(rpc_dump_max_requests_in_one_file, 1000, "start a new dump file after this many requests");
DEFINE_int32(rpc_dump_max_samples_per_second, 1000, "speed limit of the sampler");

namespace mrpc {

namespace {
var::CollectorSpeedLimit* dump_limit() {
    static var::CollectorSpeedLimit* sl = new var::CollectorSpeedLimit(FLAGS_rpc_dump_max_samples_per_second);
    return sl;
}

// Owned by the collector thread only (dump_and_destroy runs there).
struct DumpFiles {
    std::mutex mu;
    std::string dir;
    std::unique_ptr<RecordWriter> writer;
    int in_current = 0;
    int seq = 0;

    static int mkdirs(const std::string& d) {
        // create every prefix ending before a '/' and the full path
        for (size_t pos = 1; pos <= d.size(); ++pos) {
            if (pos < d.size() && d[pos] != '/') continue;
            const std::string cur = d.substr(0, pos);
            if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
        }
        return 0;
    }

    void remove_old() {
        std::vector<std::string> files = ListRpcDumpFiles(dir);
        while ((int)files.size() > FLAGS_rpc_dump_max_files) {
            unlink((dir + "/" + files.front()).c_str());
            files.erase(files.begin());
        }
    }

    RecordWriter* get() {
        if (dir != FLAGS_rpc_dump_dir) {
            writer.reset();
            dir = FLAGS_rpc_dump_dir;
        }
        if (writer && in_current < FLAGS_rpc_dump_max_requests_in_one_file) return writer.get();
        writer.reset();
        if (mkdirs(dir) != 0) {
            LOG_ONCE(ERROR) << "rpc_dump: cannot create " << dir;
            return nullptr;
        }
        // names sort by creation time: requests.<unix_us>.<seq>
        const std::string name = string_printf("requests.%016lld.%04d", (long long)realtime_us(), seq++ % 10000);
        writer.reset(new RecordWriter(dir + "/" + name));
        in_current = 0;
        if (!writer->ok()) {
            writer.reset();
            return nullptr;
        }
        remove_old();
        return writer.get();
    }
};

DumpFiles& files() {
    static DumpFiles* f = new DumpFiles;
    return *f;
}
}  // namespace

var::CollectorSpeedLimit* SampledRequest::speed_limit() { return dump_limit(); }

void SampledRequest::dump_and_destroy(size_t) {
    std::unique_ptr<SampledRequest> self(this);
    DumpFiles& f = files();
    std::lock_guard<std::mutex> g(f.mu);
    RecordWriter* w = f.get();
    if (!w) return;
    Record r;
    meta.SerializeToBuf(r.MutableMeta("meta"));
    *r.MutablePayload() = request;
    if (w->Write(r) == 0) {
        ++f.in_current;
        w->Flush();
    }
}

SampledRequest* AskToBeSampled() {
    if (!FLAGS_rpc_dump) return nullptr;
    var::CollectorSpeedLimit* sl = dump_limit();
    sl->max_per_second.store(FLAGS_rpc_dump_max_samples_per_second, std::memory_order_relaxed);
    if (!var::is_collectable(sl)) return nullptr;
    return new SampledRequest;
}

std::vector<std::string> ListRpcDumpFiles(const std::string& dir) {
    std::vector<std::string> out;
    DIR* d = opendir(dir.c_str());
    if (!d) return out;
    while (dirent* e = readdir(d)) {
        if (starts_with(e->d_name, "requests.")) out.push_back(e->d_name);
    }
    closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}

void FlushRpcDump() {
    // The collector grabs every 100 ms; wait for a couple of rounds.
    const int64_t target = var::collector_dumped_count();
    (void)target;
    usleep(250000);
    DumpFiles& f = files();
    std::lock_guard<std::mutex> g(f.mu);
    if (f.writer) f.writer->Flush();
}

}  // namespace mrpc
