#include "rpc/span_db.h"

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "base/buf.h"
#include "base/flags.h"
#include "base/logging.h"
#include "base/recordio.h"
#include "base/time.h"
#include "base/util.h"
#include "mrpc/proto/rpcz.pb.h"

DEFINE_string(rpcz_database_dir, "./rpc_data/rpcz", "directory of the rpcz span files");
DEFINE_int32(rpcz_keep_span_seconds, 3600, "spans older than this are deleted from disk");
DEFINE_int32(rpcz_file_span_seconds, 300, "a new span file is started every so many seconds");
DEFINE_bool(rpcz_keep_span_db, false, "reload the span files of a previous run instead of wiping them");
DEFINE_int32(rpcz_max_queued_spans, 65536, "spans waiting for the writer thread beyond this are dropped");

namespace mrpc {
namespace span_db {

namespace {

struct Loc {
    uint32_t file;
    uint64_t offset;
    int64_t end_us;
};

struct FileInfo {
    uint32_t id;
    std::string path;
    int64_t first_us;
};

class Db {
public:
    static Db& get() {
        static Db* d = new Db;
        return *d;
    }

    bool submit(SpanRecord* s) {
        std::unique_lock<std::mutex> g(_qmu);
        start_locked();
        if ((int)_queue.size() >= FLAGS_rpcz_max_queued_spans) {
            ++_dropped;
            g.unlock();
            delete s;
            return false;
        }
        _queue.push_back(s);
        _qcv.notify_one();
        return true;
    }

    void flush() {
        std::unique_lock<std::mutex> g(_qmu);
        if (!_started) return;
        const uint64_t target = _enqueued_seq + _queue.size();
        _flush_cv.wait_until(g, std::chrono::system_clock::now() + std::chrono::seconds(5),
                             [&] { return _done_seq >= target; });
    }

    std::vector<std::string> find_trace(uint64_t trace, size_t max) {
        ensure_started();
        std::vector<Loc> locs;
        {
            std::lock_guard<std::mutex> g(_imu);
            auto it = _by_trace.find(trace);
            if (it != _by_trace.end()) locs = it->second;
        }
        return read(locs, max);
    }

    std::vector<std::string> list_before(int64_t before_us, size_t max) {
        ensure_started();
        std::vector<Loc> locs;
        {
            std::lock_guard<std::mutex> g(_imu);
            if (before_us <= 0) before_us = INT64_MAX;
            // the time index is append-ordered (end time, roughly sorted):
            // walk back from the newest record
            for (auto it = _by_time.rbegin(); it != _by_time.rend() && locs.size() < max; ++it) {
                if (it->end_us <= before_us) locs.push_back(*it);
            }
        }
        return read(locs, max);
    }

    Stats stats() {
        ensure_started();
        Stats s;
        std::lock_guard<std::mutex> g(_imu);
        s.written = _written;
        s.dropped = _dropped;
        s.indexed = (int64_t)_by_time.size();
        s.files = (int64_t)_files.size();
        s.bytes = _bytes;
        s.reloaded = _reloaded;
        s.dir = FLAGS_rpcz_database_dir;
        return s;
    }

private:
    // First use (a span or a query): open the directory — wiping or
    // reloading the previous run's files — before anything is indexed.
    void start_locked() {
        if (_started) return;
        _started = true;
        open_dir();
        std::thread([this] { run(); }).detach();
    }

    void ensure_started() {
        std::lock_guard<std::mutex> g(_qmu);
        start_locked();
    }

    static int mkdirs(const std::string& dir) {
        std::string cur;
        for (const std::string& part : split_string(dir, '/')) {
            cur += (cur.empty() && dir[0] == '/' ? "/" : cur.empty() ? "" : "/") + part;
            if (part.empty()) continue;
            mkdir(cur.c_str(), 0755);
        }
        struct stat st;
        return stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode) ? 0 : -1;
    }

    // Previous run's files: reload (keep_span_db) or delete.
    void open_dir() {
        _dir = FLAGS_rpcz_database_dir;
        if (mkdirs(_dir) != 0) {
            LOG(ERROR) << "rpcz: cannot create " << _dir;
            return;
        }
        std::vector<std::string> names;
        if (DIR* d = opendir(_dir.c_str())) {
            while (dirent* e = readdir(d)) {
                const std::string n = e->d_name;
                if (n.size() > 5 && n.compare(0, 5, "spans") == 0) names.push_back(n);
            }
            closedir(d);
        }
        std::sort(names.begin(), names.end());
        for (const std::string& n : names) {
            const std::string path = _dir + "/" + n;
            if (!FLAGS_rpcz_keep_span_db) {
                unlink(path.c_str());
                continue;
            }
            const uint32_t id = (uint32_t)strtoul(n.c_str() + 6, nullptr, 10);
            FileInfo fi{id, path, 0};
            RecordReader rr(path);
            Record rec;
            while (rr.ok() && rr.ReadNext(&rec)) {
                SpanRecord sr;
                if (sr.ParseFromBuf(rec.Payload())) {
                    index_locked_free(sr, Loc{id, rr.last_offset(), end_time(sr, 0)});
                    if (!fi.first_us) fi.first_us = sr.received_real_us() ? sr.received_real_us() : end_time(sr, 0);
                    std::lock_guard<std::mutex> g(_imu);
                    ++_reloaded;
                }
            }
            std::lock_guard<std::mutex> g(_imu);
            _files.push_back(fi);
            _next_file = std::max(_next_file, id + 1);
        }
    }

    // Server spans end when the response is sent, client spans when it arrives.
    static int64_t end_time(const SpanRecord& sr, int64_t dflt) {
        const int64_t t = sr.type() == 0 ? sr.sent_real_us() : sr.received_real_us();
        return t ? t : dflt;
    }

    void index_locked_free(const SpanRecord& sr, const Loc& loc) {
        std::lock_guard<std::mutex> g(_imu);
        _by_trace[sr.trace_id()].push_back(loc);
        _by_time.push_back(loc);
    }

    void rotate_if_needed(int64_t now_us) {
        if (_writer && now_us - _file_start_us < (int64_t)FLAGS_rpcz_file_span_seconds * 1000000) return;
        const uint32_t id = _next_file++;
        char name[64];
        snprintf(name, sizeof(name), "spans.%010u", id);
        FileInfo fi{id, _dir + "/" + name, now_us};
        _writer.reset(new RecordWriter(fi.path));
        _file_start_us = now_us;
        std::lock_guard<std::mutex> g(_imu);
        _files.push_back(fi);
        _cur_file = id;
    }

    // Delete files (and their index entries) older than the retention.
    void expire(int64_t now_us) {
        const int64_t cutoff = now_us - (int64_t)FLAGS_rpcz_keep_span_seconds * 1000000;
        std::lock_guard<std::mutex> g(_imu);
        while (_files.size() > 1 && _files[1].first_us && _files[1].first_us < cutoff) {
            const uint32_t dead = _files.front().id;
            unlink(_files.front().path.c_str());
            _files.erase(_files.begin());
            _by_time.erase(std::remove_if(_by_time.begin(), _by_time.end(), [&](const Loc& l) { return l.file == dead; }),
                           _by_time.end());
            for (auto it = _by_trace.begin(); it != _by_trace.end();) {
                auto& v = it->second;
                v.erase(std::remove_if(v.begin(), v.end(), [&](const Loc& l) { return l.file == dead; }), v.end());
                it = v.empty() ? _by_trace.erase(it) : std::next(it);
            }
        }
    }

    void run() {
        for (;;) {
            std::deque<SpanRecord*> batch;
            {
                std::unique_lock<std::mutex> g(_qmu);
                // system_clock deadlines: steady-clock waits go through
                // pthread_cond_clockwait, which the toolchain's TSan runtime
                // does not intercept (it then sees _qmu held for good and
                // reports every later lock as a double lock); a clock step
                // only stretches or shortens one poll
                _qcv.wait_until(g, std::chrono::system_clock::now() + std::chrono::seconds(1),
                                [&] { return !_queue.empty(); });
                batch.swap(_queue);
                _enqueued_seq += batch.size();
            }
            const int64_t now = realtime_us();
            for (SpanRecord* s : batch) {
                rotate_if_needed(now);
                const SpanRecord& sr = *s;
                Record rec;
                Buf payload;
                sr.SerializeToBuf(&payload);
                *rec.MutablePayload() = payload;
                const uint64_t at = _writer->offset();
                if (_writer->Write(rec) == 0) {
                    index_locked_free(sr, Loc{_cur_file, at, end_time(sr, now)});
                    std::lock_guard<std::mutex> g(_imu);
                    ++_written;
                    _bytes += (int64_t)(_writer->offset() - at);
                }
                delete s;
            }
            if (_writer) _writer->Flush();
            expire(now);
            std::lock_guard<std::mutex> g(_qmu);
            _done_seq += batch.size();
            _flush_cv.notify_all();
        }
    }

    std::vector<std::string> read(const std::vector<Loc>& locs, size_t max) {
        std::vector<std::string> out;
        std::map<uint32_t, std::string> paths;
        {
            std::lock_guard<std::mutex> g(_imu);
            for (const FileInfo& f : _files) paths[f.id] = f.path;
        }
        std::map<uint32_t, std::unique_ptr<RecordReader>> readers;
        for (const Loc& l : locs) {
            if (out.size() >= max) break;
            auto p = paths.find(l.file);
            if (p == paths.end()) continue;
            auto& r = readers[l.file];
            if (!r) r.reset(new RecordReader(p->second));
            Record rec;
            SpanRecord sr;
            if (r->ok() && r->SeekTo(l.offset) && r->ReadNext(&rec) && sr.ParseFromBuf(rec.Payload())) {
                out.push_back(DescribeRecord(sr));
            }
        }
        return out;
    }

    std::mutex _qmu;
    std::condition_variable _qcv, _flush_cv;
    std::deque<SpanRecord*> _queue;
    bool _started = false;
    uint64_t _enqueued_seq = 0, _done_seq = 0;

    std::mutex _imu;  // indexes, files, counters
    std::unordered_map<uint64_t, std::vector<Loc>> _by_trace;
    std::vector<Loc> _by_time;
    std::vector<FileInfo> _files;
    int64_t _written = 0, _dropped = 0, _bytes = 0, _reloaded = 0;

    std::string _dir;
    std::unique_ptr<RecordWriter> _writer;
    uint32_t _next_file = 0, _cur_file = 0;
    int64_t _file_start_us = 0;
};

}  // namespace

bool Submit(SpanRecord* r) { return Db::get().submit(r); }
std::vector<std::string> FindTrace(uint64_t trace_id, size_t max) { return Db::get().find_trace(trace_id, max); }
std::vector<std::string> ListBefore(int64_t before_us, size_t max) { return Db::get().list_before(before_us, max); }
void Flush() { Db::get().flush(); }
Stats GetStats() { return Db::get().stats(); }

std::string DescribeRecord(const SpanRecord& r, int indent) {
    const std::string pad(indent, ' ');
    std::string out = pad + string_printf("%s trace=%016llx span=%016llx parent=%016llx %s %s err=%d req=%lld res=%lld",
                                          r.type() == 0 ? "S" : "C", (unsigned long long)r.trace_id(),
                                          (unsigned long long)r.span_id(), (unsigned long long)r.parent_span_id(),
                                          r.full_method_name().c_str(), r.remote().c_str(), r.error_code(),
                                          (long long)r.request_size(), (long long)r.response_size());
    if (r.type() == 0) {
        const int64_t b = r.received_real_us();
        string_appendf(&out, " received=%lld parse=+%lld callback=+%lld send=+%lld sent=+%lld", (long long)b,
                       (long long)(r.start_parse_real_us() - b), (long long)(r.start_callback_real_us() - b),
                       (long long)(r.start_send_real_us() - b), (long long)(r.sent_real_us() - b));
    } else {
        string_appendf(&out, " latency=%lldus", (long long)(r.received_real_us() - r.start_send_real_us()));
    }
    for (int i = 0; i < r.annotations_size(); ++i) {
        string_appendf(&out, "\n%s    %lld %s", pad.c_str(), (long long)r.annotations(i).realtime_us(),
                       r.annotations(i).text().c_str());
    }
    for (int i = 0; i < r.client_spans_size(); ++i) out += "\n" + DescribeRecord(r.client_spans(i), indent + 2);
    return out;
}

}  // namespace span_db
}  // namespace mrpc
