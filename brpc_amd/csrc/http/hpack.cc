#include "http/hpack.h"

#include <cstring>
#include <mutex>

namespace mrpc {

namespace {

struct HuffCode {
    uint32_t code;
    int len;
};

const HuffCode kHuff[257] = {
#include "http/hpack_huffman_table.inc"
};

const HPackHeader kStatic[61] = {
    {":authority", ""},
    {":method", "GET"},
    {":method", "POST"},
    {":path", "/"},
    {":path", "/index.html"},
    {":scheme", "http"},
    {":scheme", "https"},
    {":status", "200"},
    {":status", "204"},
    {":status", "206"},
    {":status", "304"},
    {":status", "400"},
    {":status", "404"},
    {":status", "500"},
    {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"},
    {"accept-language", ""},
    {"accept-ranges", ""},
    {"accept", ""},
    {"access-control-allow-origin", ""},
    {"age", ""},
    {"allow", ""},
    {"authorization", ""},
    {"cache-control", ""},
    {"content-disposition", ""},
    {"content-encoding", ""},
    {"content-language", ""},
    {"content-length", ""},
    {"content-location", ""},
    {"content-range", ""},
    {"content-type", ""},
    {"cookie", ""},
    {"date", ""},
    {"etag", ""},
    {"expect", ""},
    {"expires", ""},
    {"from", ""},
    {"host", ""},
    {"if-match", ""},
    {"if-modified-since", ""},
    {"if-none-match", ""},
    {"if-range", ""},
    {"if-unmodified-since", ""},
    {"last-modified", ""},
    {"link", ""},
    {"location", ""},
    {"max-forwards", ""},
    {"proxy-authenticate", ""},
    {"proxy-authorization", ""},
    {"range", ""},
    {"referer", ""},
    {"refresh", ""},
    {"retry-after", ""},
    {"server", ""},
    {"set-cookie", ""},
    {"strict-transport-security", ""},
    {"transfer-encoding", ""},
    {"user-agent", ""},
    {"vary", ""},
    {"via", ""},
    {"www-authenticate", ""},
};

// Binary decode tree built from the canonical code: node children are
// indices into g_tree; leaves hold symbol+1 in `sym` (0 = internal).
struct Node {
    int child[2] = {0, 0};
    int sym = 0;
};
std::vector<Node>* g_tree = nullptr;

void build_tree() {
    static std::once_flag once;
    std::call_once(once, [] {
        g_tree = new std::vector<Node>(1);
        for (int s = 0; s < 257; ++s) {
            int cur = 0;
            for (int b = kHuff[s].len - 1; b >= 0; --b) {
                const int bit = (kHuff[s].code >> b) & 1;
                if ((*g_tree)[cur].child[bit] == 0) {
                    (*g_tree)[cur].child[bit] = (int)g_tree->size();
                    g_tree->emplace_back();
                }
                cur = (*g_tree)[cur].child[bit];
            }
            (*g_tree)[cur].sym = s + 1;
        }
    });
}

inline size_t entry_size(const HPackHeader& h) { return 32 + h.name.size() + h.value.size(); }

}  // namespace

// ------------------------------------------------------------------ table
const HPackHeader* HPackTable::Get(size_t index) const {
    if (index == 0) return nullptr;
    if (index <= 61) return &kStatic[index - 1];
    const size_t d = index - 62;
    return d < _entries.size() ? &_entries[d] : nullptr;
}

void HPackTable::evict() {
    while (_size > _max_size && !_entries.empty()) {
        _size -= entry_size(_entries.back());
        _entries.pop_back();
    }
}

void HPackTable::Add(const std::string& name, const std::string& value) {
    HPackHeader h{name, value};
    const size_t sz = entry_size(h);
    if (sz > _max_size) {  // an entry larger than the table empties it
        _entries.clear();
        _size = 0;
        return;
    }
    _entries.push_front(std::move(h));
    _size += sz;
    evict();
}

void HPackTable::SetMaxSize(size_t n) {
    _max_size = n;
    evict();
}

void HPackTable::Find(const std::string& name, const std::string& value, size_t* full, size_t* name_only) const {
    *full = 0;
    *name_only = 0;
    for (size_t i = 0; i < 61; ++i) {
        if (kStatic[i].name == name) {
            if (kStatic[i].value == value) {
                *full = i + 1;
                return;
            }
            if (!*name_only) *name_only = i + 1;
        }
    }
    for (size_t i = 0; i < _entries.size(); ++i) {
        if (_entries[i].name == name) {
            if (_entries[i].value == value) {
                *full = 62 + i;
                return;
            }
            if (!*name_only) *name_only = 62 + i;
        }
    }
}

// ------------------------------------------------------------------ primitives
namespace hpack {

void EncodeInteger(std::string* out, uint8_t flags, int prefix_bits, uint64_t v) {
    const uint64_t max_prefix = (1u << prefix_bits) - 1;
    if (v < max_prefix) {
        out->push_back((char)(flags | v));
        return;
    }
    out->push_back((char)(flags | max_prefix));
    v -= max_prefix;
    while (v >= 128) {
        out->push_back((char)((v & 0x7f) | 0x80));
        v >>= 7;
    }
    out->push_back((char)v);
}

size_t DecodeInteger(const uint8_t* p, size_t n, int prefix_bits, uint64_t* value) {
    if (n == 0) return 0;
    const uint64_t max_prefix = (1u << prefix_bits) - 1;
    uint64_t v = p[0] & max_prefix;
    if (v < max_prefix) {
        *value = v;
        return 1;
    }
    int shift = 0;
    for (size_t i = 1; i < n; ++i) {
        if (shift > 56) return 0;
        v += (uint64_t)(p[i] & 0x7f) << shift;
        shift += 7;
        if (!(p[i] & 0x80)) {
            *value = v;
            return i + 1;
        }
    }
    return 0;
}

size_t HuffmanEncodedLength(const std::string& in) {
    uint64_t bits = 0;
    for (unsigned char c : in) bits += kHuff[c].len;
    return (size_t)((bits + 7) / 8);
}

void HuffmanEncode(std::string* out, const std::string& in) {
    uint64_t acc = 0;
    int nbits = 0;
    for (unsigned char c : in) {
        acc = (acc << kHuff[c].len) | kHuff[c].code;
        nbits += kHuff[c].len;
        while (nbits >= 8) {
            nbits -= 8;
            out->push_back((char)(acc >> nbits));
        }
        acc &= (1ull << nbits) - 1;
    }
    if (nbits > 0) {  // pad with the EOS prefix (all ones)
        out->push_back((char)((acc << (8 - nbits)) | ((1u << (8 - nbits)) - 1)));
    }
}

bool HuffmanDecode(const uint8_t* p, size_t n, std::string* out) {
    build_tree();
    const std::vector<Node>& t = *g_tree;
    int cur = 0;
    int depth = 0;      // bits consumed since the last symbol
    bool all_ones = true;
    for (size_t i = 0; i < n; ++i) {
        for (int b = 7; b >= 0; --b) {
            const int bit = (p[i] >> b) & 1;
            cur = t[cur].child[bit];
            if (cur == 0) return false;
            ++depth;
            all_ones = all_ones && bit;
            if (t[cur].sym) {
                if (t[cur].sym == 257) return false;  // EOS inside a string
                out->push_back((char)(t[cur].sym - 1));
                cur = 0;
                depth = 0;
                all_ones = true;
            }
        }
    }
    // padding must be < 8 bits of the EOS prefix
    return depth < 8 && all_ones;
}

}  // namespace hpack

// ------------------------------------------------------------------ encoder
static void encode_string(std::string* out, const std::string& s, bool huffman = true) {
    const size_t hl = huffman ? hpack::HuffmanEncodedLength(s) : s.size();
    if (hl < s.size()) {
        hpack::EncodeInteger(out, 0x80, 7, hl);
        hpack::HuffmanEncode(out, s);
    } else {
        hpack::EncodeInteger(out, 0x00, 7, s.size());
        out->append(s);
    }
}

void HPackEncoder::ResizeTable(size_t n) {
    _pending_resize = true;
    _resize_to = std::min<size_t>(n, 4096);
}

void HPackEncoder::Encode(Buf* out, const HPackHeader& h, HPackIndexPolicy policy) {
    std::string s;
    if (_pending_resize) {
        hpack::EncodeInteger(&s, 0x20, 5, _resize_to);
        _table.SetMaxSize(_resize_to);
        _pending_resize = false;
    }
    size_t full = 0, name_only = 0;
    if (policy != HPackIndexPolicy::NEVER_INDEXED) _table.Find(h.name, h.value, &full, &name_only);
    if (full) {
        hpack::EncodeInteger(&s, 0x80, 7, full);
    } else if (policy == HPackIndexPolicy::INCREMENTAL) {
        hpack::EncodeInteger(&s, 0x40, 6, name_only);
        if (!name_only) encode_string(&s, h.name);
        encode_string(&s, h.value);
        _table.Add(h.name, h.value);
    } else {
        hpack::EncodeInteger(&s, policy == HPackIndexPolicy::NEVER_INDEXED ? 0x10 : 0x00, 4, name_only);
        if (!name_only) encode_string(&s, h.name);
        encode_string(&s, h.value, policy != HPackIndexPolicy::NOT_INDEXED_RAW);
    }
    out->append(s);
}

// ------------------------------------------------------------------ decoder
static bool decode_string(const uint8_t* p, size_t n, size_t* pos, std::string* out) {
    if (*pos >= n) return false;
    const bool huff = p[*pos] & 0x80;
    uint64_t len = 0;
    const size_t c = hpack::DecodeInteger(p + *pos, n - *pos, 7, &len);
    if (!c || len > n - *pos - c) return false;
    *pos += c;
    out->clear();
    if (huff) {
        if (!hpack::HuffmanDecode(p + *pos, (size_t)len, out)) return false;
    } else {
        out->assign(reinterpret_cast<const char*>(p + *pos), (size_t)len);
    }
    *pos += (size_t)len;
    return true;
}

bool HPackDecoder::Decode(const std::string& block, std::vector<HPackHeader>* out) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(block.data());
    const size_t n = block.size();
    size_t pos = 0;
    while (pos < n) {
        const uint8_t b = p[pos];
        uint64_t idx = 0;
        if (b & 0x80) {  // indexed
            const size_t c = hpack::DecodeInteger(p + pos, n - pos, 7, &idx);
            if (!c) return false;
            pos += c;
            const HPackHeader* h = _table.Get((size_t)idx);
            if (!h) return false;
            out->push_back(*h);
        } else if ((b & 0xe0) == 0x20) {  // dynamic table size update
            const size_t c = hpack::DecodeInteger(p + pos, n - pos, 5, &idx);
            if (!c || idx > _limit) return false;
            pos += c;
            _table.SetMaxSize((size_t)idx);
        } else {
            const bool incremental = (b & 0xc0) == 0x40;
            const int prefix = incremental ? 6 : 4;
            const size_t c = hpack::DecodeInteger(p + pos, n - pos, prefix, &idx);
            if (!c) return false;
            pos += c;
            HPackHeader h;
            if (idx) {
                const HPackHeader* nh = _table.Get((size_t)idx);
                if (!nh) return false;
                h.name = nh->name;
            } else if (!decode_string(p, n, &pos, &h.name)) {
                return false;
            }
            if (!decode_string(p, n, &pos, &h.value)) return false;
            if (incremental) _table.Add(h.name, h.value);
            out->push_back(std::move(h));
        }
    }
    return true;
}

}  // namespace mrpc
