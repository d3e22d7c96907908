// HPACK header compression for HTTP/2 (RFC 7541; role of the reference's
// src/brpc/details/hpack.cpp): static + dynamic tables, prefix integers,
// string literals with the canonical Huffman code.
#pragma once

#include <cstdint>
#include <deque>
#include <string>
#include <utility>
#include <vector>

#include "base/buf.h"

namespace mrpc {

struct HPackHeader {
    std::string name;
    std::string value;
};

// NOT_INDEXED_RAW: a literal that is neither indexed nor Huffman-coded
// (per-message binary metadata, base64: Huffman saves ~1/4 of its bytes for
// an encode and a bit-by-bit decode on every message)
enum class HPackIndexPolicy { INCREMENTAL, NOT_INDEXED, NEVER_INDEXED, NOT_INDEXED_RAW };

class HPackTable {
public:
    explicit HPackTable(size_t max_size = 4096) : _max_size(max_size) {}
    // 1-based index over static (1..61) then dynamic entries
    const HPackHeader* Get(size_t index) const;
    void Add(const std::string& name, const std::string& value);
    void SetMaxSize(size_t n);
    size_t max_size() const { return _max_size; }
    size_t size() const { return _size; }
    // Search: returns index of (name,value) match in *full or name-only in
    // *name_only (0 when none).
    void Find(const std::string& name, const std::string& value, size_t* full, size_t* name_only) const;
    size_t dynamic_count() const { return _entries.size(); }

private:
    void evict();
    std::deque<HPackHeader> _entries;  // front = most recent
    size_t _size = 0;
    size_t _max_size;
};

class HPackEncoder {
public:
    explicit HPackEncoder(size_t table_size = 4096) : _table(table_size) {}
    void Encode(Buf* out, const HPackHeader& h, HPackIndexPolicy policy = HPackIndexPolicy::INCREMENTAL);
    // peer's SETTINGS_HEADER_TABLE_SIZE: emitted as a size update next time
    void ResizeTable(size_t n);

private:
    HPackTable _table;
    bool _pending_resize = false;
    size_t _resize_to = 0;
};

class HPackDecoder {
public:
    explicit HPackDecoder(size_t max_table_size = 4096) : _table(max_table_size), _limit(max_table_size) {}
    // Decodes a complete header block. Returns false on a malformed block.
    bool Decode(const std::string& block, std::vector<HPackHeader>* out);

private:
    HPackTable _table;
    size_t _limit;
};

namespace hpack {
void EncodeInteger(std::string* out, uint8_t first_byte_flags, int prefix_bits, uint64_t value);
// Returns bytes consumed or 0 on error.
size_t DecodeInteger(const uint8_t* p, size_t n, int prefix_bits, uint64_t* value);
void HuffmanEncode(std::string* out, const std::string& in);
size_t HuffmanEncodedLength(const std::string& in);
bool HuffmanDecode(const uint8_t* p, size_t n, std::string* out);
}  // namespace hpack

}  // namespace mrpc
