// Self-delimiting record files (role of the reference's src/butil/recordio.h,
// used by rpc_dump / rpc_replay). Each record:
//   "MRIO" | body_size u32 LE | crc32c(body) u32 LE | body
//   body = nmeta varint | { name_len varint | name | data_len varint | data }* | payload
// The reader verifies the checksum and, on a corrupted or truncated record,
// resynchronizes at the next "MRIO" so one bad record does not lose the file.
#pragma once

#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "base/buf.h"

namespace mrpc {

class Record {
public:
    size_t MetaCount() const { return _metas.size(); }
    const std::pair<std::string, Buf>& MetaAt(size_t i) const { return _metas[i]; }
    const Buf* Meta(const std::string& name) const;
    // Adds the meta if absent (nullptr if present and null_on_found).
    Buf* MutableMeta(const std::string& name, bool null_on_found = false);
    bool RemoveMeta(const std::string& name);
    const Buf& Payload() const { return _payload; }
    Buf* MutablePayload() { return &_payload; }
    void Clear();
    size_t ByteSize() const;

private:
    friend class RecordWriter;
    friend class RecordReader;
    std::vector<std::pair<std::string, Buf>> _metas;
    Buf _payload;
};

class RecordWriter {
public:
    // Appends to `path` (created if missing).
    explicit RecordWriter(const std::string& path);
    ~RecordWriter();
    bool ok() const { return _f != nullptr; }
    int Write(const Record& r);  // 0 on success
    int Flush();
    // Byte offset the next record will be written at (RecordReader::SeekTo).
    uint64_t offset() const;
    size_t written_bytes() const { return _bytes; }

private:
    FILE* _f = nullptr;
    size_t _bytes = 0;
};

class RecordReader {
public:
    explicit RecordReader(const std::string& path);
    ~RecordReader();
    bool ok() const { return _f != nullptr; }
    // false at end of file (last_error()==0) or on I/O error.
    bool ReadNext(Record* out);
    // Position the reader at a record boundary returned by
    // RecordWriter::offset() (random access for indexed stores).
    bool SeekTo(uint64_t offset);
    // File offset of the record ReadNext last returned.
    uint64_t last_offset() const { return _last_offset; }
    int last_error() const { return _err; }
    size_t skipped_bytes() const { return _skipped; }  // bytes dropped while resyncing

private:
    bool fill(size_t n);
    FILE* _f = nullptr;
    std::string _buf;
    size_t _pos = 0;
    uint64_t _base = 0;  // file offset of _buf[0]
    uint64_t _last_offset = 0;
    bool _eof = false;
    int _err = 0;
    size_t _skipped = 0;
};

}  // namespace mrpc
