#include "base/recordio.h"

#include <cerrno>
#include <cstring>

#include "base/crc32c.h"

namespace mrpc {

static const char kMagic[4] = {'M', 'R', 'I', 'O'};
static const size_t kHead = 12;
static const uint32_t kMaxBody = 512u << 20;

static void put_varint(std::string* s, uint64_t v) {
    while (v >= 0x80) {
        s->push_back((char)(v | 0x80));
        v >>= 7;
    }
    s->push_back((char)v);
}

static bool get_varint(const char*& p, const char* end, uint64_t* v) {
    uint64_t r = 0;
    for (int shift = 0; shift < 64 && p < end; shift += 7) {
        const uint8_t b = (uint8_t)*p++;
        r |= (uint64_t)(b & 0x7f) << shift;
        if (!(b & 0x80)) {
            *v = r;
            return true;
        }
    }
    return false;
}

const Buf* Record::Meta(const std::string& name) const {
    for (auto& m : _metas) {
        if (m.first == name) return &m.second;
    }
    return nullptr;
}

Buf* Record::MutableMeta(const std::string& name, bool null_on_found) {
    for (auto& m : _metas) {
        if (m.first == name) return null_on_found ? nullptr : &m.second;
    }
    _metas.emplace_back(name, Buf());
    return &_metas.back().second;
}

bool Record::RemoveMeta(const std::string& name) {
    for (size_t i = 0; i < _metas.size(); ++i) {
        if (_metas[i].first == name) {
            _metas.erase(_metas.begin() + i);
            return true;
        }
    }
    return false;
}

void Record::Clear() {
    _metas.clear();
    _payload.clear();
}

size_t Record::ByteSize() const {
    size_t n = kHead + 10 + _payload.size();
    for (auto& m : _metas) n += 20 + m.first.size() + m.second.size();
    return n;
}

RecordWriter::RecordWriter(const std::string& path) {
    _f = fopen(path.c_str(), "ab");
    if (_f) fseek(_f, 0, SEEK_END);  // offset() is meaningful before the first write
}

uint64_t RecordWriter::offset() const {
    if (!_f) return 0;
    const long off = ftell(_f);
    return off < 0 ? 0 : (uint64_t)off;
}

bool RecordReader::SeekTo(uint64_t offset) {
    if (!_f || fseek(_f, (long)offset, SEEK_SET) != 0) return false;
    _buf.clear();
    _pos = 0;
    _base = offset;
    _eof = false;
    _err = 0;
    return true;
}
RecordWriter::~RecordWriter() {
    if (_f) fclose(_f);
}

int RecordWriter::Write(const Record& r) {
    if (!_f) return EINVAL;
    std::string body;
    put_varint(&body, r._metas.size());
    for (auto& m : r._metas) {
        put_varint(&body, m.first.size());
        body.append(m.first);
        put_varint(&body, m.second.size());
        body.append(m.second.to_string());
    }
    body.append(r._payload.to_string());
    if (body.size() > kMaxBody) return E2BIG;
    char head[kHead];
    memcpy(head, kMagic, 4);
    const uint32_t size = (uint32_t)body.size();
    const uint32_t crc = crc32c::Value(body.data(), body.size());
    memcpy(head + 4, &size, 4);
    memcpy(head + 8, &crc, 4);
    if (fwrite(head, 1, kHead, _f) != kHead || fwrite(body.data(), 1, body.size(), _f) != body.size()) return errno;
    _bytes += kHead + body.size();
    return 0;
}

int RecordWriter::Flush() { return _f && fflush(_f) == 0 ? 0 : errno; }

RecordReader::RecordReader(const std::string& path) { _f = fopen(path.c_str(), "rb"); }
RecordReader::~RecordReader() {
    if (_f) fclose(_f);
}

bool RecordReader::fill(size_t n) {
    if (_pos > (1u << 20)) {
        _buf.erase(0, _pos);
        _base += _pos;
        _pos = 0;
    }
    while (_buf.size() - _pos < n && !_eof) {
        char tmp[65536];
        const size_t r = fread(tmp, 1, sizeof(tmp), _f);
        if (r == 0) {
            _eof = true;
            if (ferror(_f)) _err = EIO;
            break;
        }
        _buf.append(tmp, r);
    }
    return _buf.size() - _pos >= n;
}

bool RecordReader::ReadNext(Record* out) {
    if (!_f) return false;
    for (;;) {
        if (!fill(kHead)) {
            _skipped += _buf.size() - _pos;
            return false;
        }
        const char* h = _buf.data() + _pos;
        if (memcmp(h, kMagic, 4) != 0) {
            ++_pos;  // resync byte by byte
            ++_skipped;
            continue;
        }
        uint32_t size, crc;
        memcpy(&size, h + 4, 4);
        memcpy(&crc, h + 8, 4);
        if (size > kMaxBody || !fill(kHead + size)) {
            ++_pos;
            ++_skipped;
            if (size <= kMaxBody && _eof) {
                _skipped += _buf.size() - _pos;
                _pos = _buf.size();
                return false;  // truncated tail
            }
            continue;
        }
        const char* body = _buf.data() + _pos + kHead;
        if (crc32c::Value(body, size) != crc) {
            ++_pos;
            ++_skipped;
            continue;
        }
        out->Clear();
        const char* p = body;
        const char* end = body + size;
        uint64_t nmeta = 0;
        bool good = get_varint(p, end, &nmeta);
        for (uint64_t i = 0; good && i < nmeta; ++i) {
            uint64_t nl = 0, dl = 0;
            good = get_varint(p, end, &nl) && (uint64_t)(end - p) >= nl;
            if (!good) break;
            std::string name(p, nl);
            p += nl;
            good = get_varint(p, end, &dl) && (uint64_t)(end - p) >= dl;
            if (!good) break;
            out->MutableMeta(name)->append(p, dl);
            p += dl;
        }
        if (!good) {
            ++_pos;
            ++_skipped;
            continue;
        }
        out->_payload.append(p, (size_t)(end - p));
        _last_offset = _base + _pos;
        _pos += kHead + size;
        return true;
    }
}

}  // namespace mrpc
