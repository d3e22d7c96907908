#include "rtmp/media.h"

#include <cstring>

#include "rtmp/rtmp.h"

namespace mrpc {

namespace {

const uint32_t kAacRates[13] = {96000, 88200, 64000, 48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000, 7350};

// MSB-first bit reader over RBSP bytes with exp-Golomb codes.
class BitReader {
public:
    BitReader(const uint8_t* p, size_t n) : _p(p), _n(n) {}
    bool ok() const { return !_overrun; }
    uint32_t bits(int k) {
        uint32_t v = 0;
        for (int i = 0; i < k; ++i) v = (v << 1) | bit();
        return v;
    }
    uint32_t bit() {
        if (_pos >= _n * 8) {
            _overrun = true;
            return 0;
        }
        const uint32_t b = (_p[_pos >> 3] >> (7 - (_pos & 7))) & 1;
        ++_pos;
        return b;
    }
    uint32_t ue() {
        int zeros = 0;
        while (bit() == 0) {
            if (_overrun || ++zeros > 31) {
                _overrun = true;
                return 0;
            }
        }
        if (zeros == 0) return 0;
        return ((1u << zeros) - 1) + bits(zeros);
    }
    int32_t se() {
        const uint32_t k = ue();
        return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
    }

private:
    const uint8_t* _p;
    size_t _n;
    size_t _pos = 0;
    bool _overrun = false;
};

void skip_scaling_list(BitReader* br, int size) {
    int last = 8, next = 8;
    for (int j = 0; j < size; ++j) {
        if (next != 0) {
            const int32_t delta = br->se();
            next = (last + delta + 256) % 256;
        }
        last = next == 0 ? last : next;
    }
}

void put_u16(std::string* s, size_t v) {
    s->push_back((char)((v >> 8) & 0xff));
    s->push_back((char)(v & 0xff));
}

}  // namespace

// ------------------------------------------------------------------ AAC

uint8_t AacSampleRateIndex(uint32_t rate) {
    for (uint8_t i = 0; i < 13; ++i)
        if (kAacRates[i] == rate) return i;
    return 15;
}

uint32_t AacSampleRate(uint8_t index) { return index < 13 ? kAacRates[index] : 0; }

int RtmpAACMessage::Create(const RtmpAudioMessage& msg) {
    if (msg.codec != 10 || msg.data.empty()) return -1;
    timestamp = msg.timestamp;
    rate = msg.rate;
    bits = msg.bits;
    type = msg.type;
    uint8_t pt = 0;
    msg.data.copy_to(&pt, 1);
    if (pt > AAC_PACKET_RAW) return -1;
    packet_type = (AACPacketType)pt;
    data.clear();
    Buf rest = msg.data;
    rest.pop_front(1);
    data.append(std::move(rest));
    return 0;
}

void RtmpAACMessage::ToAudioMessage(RtmpAudioMessage* msg) const {
    msg->timestamp = timestamp;
    msg->codec = 10;
    msg->rate = rate;
    msg->bits = bits;
    msg->type = type;
    msg->data.clear();
    msg->data.push_back((char)packet_type);
    msg->data.append(data);
}

int AudioSpecificConfig::Create(const Buf& d) {
    const std::string s = d.to_string();
    return Create(s.data(), s.size());
}

int AudioSpecificConfig::Create(const void* data, size_t n) {
    BitReader br(static_cast<const uint8_t*>(data), n);
    uint32_t obj = br.bits(5);
    if (obj == 31) obj = 32 + br.bits(6);
    const uint32_t idx = br.bits(4);
    uint32_t rate = idx == 15 ? br.bits(24) : AacSampleRate((uint8_t)idx);
    const uint32_t ch = br.bits(4);
    if (!br.ok() || obj == 0 || obj > 255 || rate == 0 || ch > 7) return -1;
    aac_object = (uint8_t)obj;
    sample_rate_index = (uint8_t)idx;
    sample_rate = rate;
    channels = (uint8_t)ch;
    return 0;
}

std::string AudioSpecificConfig::Serialize() const {
    // object(5 or 5+6) | index(4) [| rate(24)] | channels(4) | 3 zero bits (GASpecificConfig)
    uint64_t acc = 0;
    int nbits = 0;
    auto put = [&](uint64_t v, int k) {
        acc = (acc << k) | (v & ((1ull << k) - 1));
        nbits += k;
    };
    if (aac_object >= 31) {
        put(31, 5);
        put(aac_object - 32, 6);
    } else {
        put(aac_object, 5);
    }
    const uint8_t idx = sample_rate_index == 15 || AacSampleRate(sample_rate_index) != sample_rate
                            ? AacSampleRateIndex(sample_rate)
                            : sample_rate_index;
    put(idx, 4);
    if (idx == 15) put(sample_rate, 24);
    put(channels, 4);
    put(0, 3);
    const int pad = (8 - nbits % 8) % 8;
    put(0, pad);
    std::string out;
    for (int i = nbits - 8; i >= 0; i -= 8) out.push_back((char)((acc >> i) & 0xff));
    return out;
}

int AudioSpecificConfig::MakeAdtsHeader(size_t payload_len, uint8_t out[7]) const {
    const size_t frame = payload_len + 7;
    const uint8_t idx = AacSampleRateIndex(sample_rate);
    if (frame > 0x1fff || idx == 15 || aac_object < 1 || aac_object > 4 || channels > 7) return -1;
    const uint8_t profile = aac_object - 1;
    out[0] = 0xff;
    out[1] = 0xf1;  // sync, MPEG-4, layer 0, no CRC
    out[2] = (uint8_t)((profile << 6) | (idx << 2) | ((channels >> 2) & 1));
    out[3] = (uint8_t)(((channels & 3) << 6) | ((frame >> 11) & 3));
    out[4] = (uint8_t)((frame >> 3) & 0xff);
    out[5] = (uint8_t)(((frame & 7) << 5) | 0x1f);  // buffer fullness 0x7ff (VBR)
    out[6] = 0xfc;                                   // ... and one raw data block
    return 0;
}

// ------------------------------------------------------------------ AVC

int RtmpAVCMessage::Create(const RtmpVideoMessage& msg) {
    if (msg.codec != 7 || msg.data.size() < 4) return -1;
    uint8_t h[4];
    msg.data.copy_to(h, 4);
    if (h[0] > AVC_PACKET_END_OF_SEQUENCE) return -1;
    timestamp = msg.timestamp;
    frame_type = msg.frame_type;
    packet_type = (AVCPacketType)h[0];
    int32_t ct = (int32_t)((h[1] << 16) | (h[2] << 8) | h[3]);
    if (ct & 0x800000) ct -= 0x1000000;  // sign-extend SI24
    composition_time = ct;
    data.clear();
    Buf rest = msg.data;
    rest.pop_front(4);
    data.append(std::move(rest));
    return 0;
}

void RtmpAVCMessage::ToVideoMessage(RtmpVideoMessage* msg) const {
    msg->timestamp = timestamp;
    msg->frame_type = frame_type;
    msg->codec = 7;
    msg->data.clear();
    const uint32_t ct = (uint32_t)composition_time & 0xffffff;
    const char h[4] = {(char)packet_type, (char)(ct >> 16), (char)(ct >> 8), (char)ct};
    msg->data.append(h, 4);
    msg->data.append(data);
}

std::string AvcUnescapeRbsp(const void* data, size_t n) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    std::string out;
    out.reserve(n);
    int zeros = 0;
    for (size_t i = 0; i < n; ++i) {
        if (zeros >= 2 && p[i] == 3) {
            zeros = 0;
            continue;
        }
        zeros = p[i] == 0 ? zeros + 1 : 0;
        out.push_back((char)p[i]);
    }
    return out;
}

int AvcSps::Parse(const std::string& nalu) {
    if (nalu.size() < 4 || (nalu[0] & 0x1f) != AVC_NALU_SPS) return -1;
    const std::string rbsp = AvcUnescapeRbsp(nalu.data() + 1, nalu.size() - 1);
    BitReader br(reinterpret_cast<const uint8_t*>(rbsp.data()), rbsp.size());
    profile_idc = (uint8_t)br.bits(8);
    constraint_flags = (uint8_t)br.bits(8);
    level_idc = (uint8_t)br.bits(8);
    sps_id = br.ue();
    if (sps_id > 31) return -1;
    chroma_format_idc = 1;
    bool separate_planes = false;
    switch (profile_idc) {
    case 100: case 110: case 122: case 244: case 44: case 83: case 86: case 118: case 128: case 138: case 139:
    case 134: case 135: {
        chroma_format_idc = br.ue();
        if (chroma_format_idc > 3) return -1;
        if (chroma_format_idc == 3) separate_planes = br.bit();
        bit_depth_luma = br.ue() + 8;
        bit_depth_chroma = br.ue() + 8;
        br.bit();  // qpprime_y_zero_transform_bypass_flag
        if (br.bit()) {  // seq_scaling_matrix_present_flag
            const int lists = chroma_format_idc != 3 ? 8 : 12;
            for (int i = 0; i < lists; ++i)
                if (br.bit()) skip_scaling_list(&br, i < 6 ? 16 : 64);
        }
        break;
    }
    default: break;
    }
    log2_max_frame_num = br.ue() + 4;
    pic_order_cnt_type = br.ue();
    if (pic_order_cnt_type == 0) {
        br.ue();  // log2_max_pic_order_cnt_lsb_minus4
    } else if (pic_order_cnt_type == 1) {
        br.bit();  // delta_pic_order_always_zero_flag
        br.se();   // offset_for_non_ref_pic
        br.se();   // offset_for_top_to_bottom_field
        const uint32_t cycle = br.ue();
        if (cycle > 255) return -1;
        for (uint32_t i = 0; i < cycle; ++i) br.se();
    } else if (pic_order_cnt_type != 2) {
        return -1;
    }
    max_num_ref_frames = br.ue();
    br.bit();  // gaps_in_frame_num_value_allowed_flag
    const uint32_t w_mbs = br.ue() + 1;
    const uint32_t h_units = br.ue() + 1;
    frame_mbs_only = br.bit();
    if (!frame_mbs_only) br.bit();  // mb_adaptive_frame_field_flag
    br.bit();                       // direct_8x8_inference_flag
    uint32_t cl = 0, cr = 0, ct = 0, cb = 0;
    if (br.bit()) {
        cl = br.ue();
        cr = br.ue();
        ct = br.ue();
        cb = br.ue();
    }
    if (!br.ok() || w_mbs > 1024 || h_units > 1024) return -1;
    const uint32_t fm = frame_mbs_only ? 1 : 2;
    uint32_t cux = 1, cuy = fm;
    const uint32_t chroma = separate_planes ? 0 : chroma_format_idc;
    if (chroma == 1) {
        cux = 2;
        cuy = 2 * fm;
    } else if (chroma == 2) {
        cux = 2;
        cuy = fm;
    }
    const int64_t w = (int64_t)w_mbs * 16 - (int64_t)cux * (cl + cr);
    const int64_t h = (int64_t)h_units * 16 * fm - (int64_t)cuy * (ct + cb);
    if (w <= 0 || h <= 0) return -1;
    width = (int)w;
    height = (int)h;
    return 0;
}

int AVCDecoderConfigurationRecord::Create(const Buf& d) {
    const std::string s = d.to_string();
    return Create(s.data(), s.size());
}

int AVCDecoderConfigurationRecord::Create(const void* data, size_t n) {
    const uint8_t* p = static_cast<const uint8_t*>(data);
    if (n < 7 || p[0] != 1) return -1;
    avc_profile = p[1];
    profile_compatibility = p[2];
    avc_level = p[3];
    length_size_minus1 = p[4] & 3;
    if (length_size_minus1 == 2) return -1;  // 3-byte lengths are not allowed
    sps_list.clear();
    pps_list.clear();
    size_t at = 5;
    auto read_sets = [&](size_t count, std::vector<std::string>* out) {
        for (size_t i = 0; i < count; ++i) {
            if (at + 2 > n) return false;
            const size_t len = ((size_t)p[at] << 8) | p[at + 1];
            at += 2;
            if (len == 0 || at + len > n) return false;
            out->emplace_back(reinterpret_cast<const char*>(p + at), len);
            at += len;
        }
        return true;
    };
    if (!read_sets(p[at++] & 0x1f, &sps_list)) return -1;
    if (at >= n || !read_sets(p[at++], &pps_list)) return -1;
    width = height = 0;
    AvcSps sps;
    if (!sps_list.empty() && sps.Parse(sps_list[0]) == 0) {
        width = sps.width;
        height = sps.height;
    }
    return 0;
}

std::string AVCDecoderConfigurationRecord::Serialize() const {
    std::string s;
    s.push_back(1);
    s.push_back((char)avc_profile);
    s.push_back((char)profile_compatibility);
    s.push_back((char)avc_level);
    s.push_back((char)(0xfc | (length_size_minus1 & 3)));
    s.push_back((char)(0xe0 | (sps_list.size() & 0x1f)));
    for (const std::string& x : sps_list) {
        put_u16(&s, x.size());
        s += x;
    }
    s.push_back((char)(pps_list.size() & 0xff));
    for (const std::string& x : pps_list) {
        put_u16(&s, x.size());
        s += x;
    }
    return s;
}

AVCNaluIterator::AVCNaluIterator(const Buf* data, int length_size, AVCNaluFormat* format)
    : _bytes(data ? data->to_string() : std::string()), _length_size(length_size), _format(format) {}

bool AVCNaluIterator::Next(std::string* nalu, AVCNaluType* type) {
    if (_error || _pos >= _bytes.size()) return false;
    if (*_format == AVC_NALU_FORMAT_UNKNOWN) {
        const char* b = _bytes.data() + _pos;
        const size_t left = _bytes.size() - _pos;
        const bool sc3 = left >= 3 && b[0] == 0 && b[1] == 0 && b[2] == 1;
        const bool sc4 = left >= 4 && b[0] == 0 && b[1] == 0 && b[2] == 0 && b[3] == 1;
        *_format = sc3 || sc4 ? AVC_NALU_FORMAT_ANNEXB : AVC_NALU_FORMAT_IBMF;
    }
    const bool ok = *_format == AVC_NALU_FORMAT_ANNEXB ? NextAnnexB(nalu) : NextIbmf(nalu);
    if (ok && type) *type = (AVCNaluType)((*nalu)[0] & 0x1f);
    return ok;
}

bool AVCNaluIterator::NextIbmf(std::string* nalu) {
    if (_length_size != 1 && _length_size != 2 && _length_size != 4) {
        _error = true;
        return false;
    }
    if (_pos + (size_t)_length_size > _bytes.size()) {
        _error = true;
        return false;
    }
    size_t len = 0;
    for (int i = 0; i < _length_size; ++i) len = (len << 8) | (uint8_t)_bytes[_pos + i];
    _pos += _length_size;
    if (len == 0 || _pos + len > _bytes.size()) {
        _error = true;
        return false;
    }
    nalu->assign(_bytes, _pos, len);
    _pos += len;
    return true;
}

bool AVCNaluIterator::NextAnnexB(std::string* nalu) {
    const size_t n = _bytes.size();
    const char* b = _bytes.data();
    // skip the start code (and zero padding before it)
    size_t i = _pos;
    while (i < n && b[i] == 0) ++i;
    if (i >= n || b[i] != 1 || i - _pos < 2) {
        _error = i < n;  // trailing zeros are fine, anything else is not
        _pos = n;
        return false;
    }
    const size_t start = i + 1;
    size_t end = n;
    for (size_t k = start; k + 2 < n; ++k) {
        if (b[k] == 0 && b[k + 1] == 0 && (b[k + 2] == 1 || (b[k + 2] == 0 && k + 3 < n && b[k + 3] == 1))) {
            end = k;
            break;
        }
    }
    size_t stop = end;
    while (stop > start && b[stop - 1] == 0) --stop;  // trailing_zero_8bits
    _pos = end;
    if (stop == start) {
        _error = true;
        return false;
    }
    nalu->assign(b + start, stop - start);
    return true;
}

}  // namespace mrpc
