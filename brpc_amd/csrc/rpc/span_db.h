// Persistent rpcz span store (role of the reference's leveldb-backed span
// database, src/brpc/span.cpp:306-560: spans indexed by id and by time,
// browsed at /rpcz, optionally kept across restarts with
// -rpcz_keep_span_db).
//
// Submitted spans are queued and written by one background thread as
// checksummed recordio records (base/recordio.h) into files rotated every
// rpcz_file_span_seconds; files older than rpcz_keep_span_seconds are
// deleted. Two in-memory indexes point at (file, offset): trace id -> spans
// and a time-ordered list, so /rpcz?trace_id= and /rpcz?time= read only the
// records they show. Nothing on the RPC path touches the disk.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mrpc {

class SpanRecord;

namespace span_db {

// Queue a finished span's record (takes ownership). Returns false if the
// queue is full (record dropped).
bool Submit(SpanRecord* r);
// Spans of one trace, oldest first.
std::vector<std::string> FindTrace(uint64_t trace_id, size_t max);
// Spans that ended at or before `before_us` (realtime; 0 = now), newest first.
std::vector<std::string> ListBefore(int64_t before_us, size_t max);
// Wait until queued spans are on disk (tests, shutdown).
void Flush();

struct Stats {
    int64_t written = 0, dropped = 0, indexed = 0, files = 0, bytes = 0, reloaded = 0;
    std::string dir;
};
Stats GetStats();

// Describe a stored span (the /rpcz text form).
std::string DescribeRecord(const SpanRecord& r, int indent = 0);

}  // namespace span_db
}  // namespace mrpc
