#include "rtmp/ts.h"

#include <cstring>

namespace mrpc {

namespace {

const size_t kTsPacket = 188;

int cc_index(uint16_t pid) {
    switch (pid) {
    case TS_PID_PAT: return 0;
    case TS_PID_PMT: return 1;
    case TS_PID_VIDEO: return 2;
    default: return 3;
    }
}

// 33-bit timestamp in the PES 5-byte layout with a 4-bit prefix.
void put_ts(uint8_t* p, uint8_t prefix, int64_t t) {
    const uint64_t v = (uint64_t)t & 0x1FFFFFFFFull;
    p[0] = (uint8_t)((prefix << 4) | (((v >> 30) & 0x07) << 1) | 1);
    p[1] = (uint8_t)(v >> 22);
    p[2] = (uint8_t)((((v >> 15) & 0x7F) << 1) | 1);
    p[3] = (uint8_t)(v >> 7);
    p[4] = (uint8_t)(((v & 0x7F) << 1) | 1);
}

uint32_t be(const std::string& s, size_t pos, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 8) | (uint8_t)s[pos + i];
    return v;
}

}  // namespace

// AVCDecoderConfigurationRecord (ISO 14496-15 5.2.4.1).
bool AvcConfig::Parse(const std::string& r) {
    if (r.size() < 7 || (uint8_t)r[0] != 1) return false;
    profile = (uint8_t)r[1];
    level = (uint8_t)r[3];
    nalu_length_size = ((uint8_t)r[4] & 3) + 1;
    sps.clear();
    pps.clear();
    size_t p = 5;
    const int nsps = (uint8_t)r[p++] & 0x1f;
    for (int i = 0; i < nsps; ++i) {
        if (p + 2 > r.size()) return false;
        const size_t len = be(r, p, 2);
        p += 2;
        if (p + len > r.size()) return false;
        sps.push_back(r.substr(p, len));
        p += len;
    }
    if (p >= r.size()) return false;
    const int npps = (uint8_t)r[p++];
    for (int i = 0; i < npps; ++i) {
        if (p + 2 > r.size()) return false;
        const size_t len = be(r, p, 2);
        p += 2;
        if (p + len > r.size()) return false;
        pps.push_back(r.substr(p, len));
        p += len;
    }
    return !sps.empty() && !pps.empty();
}

// AudioSpecificConfig (ISO 14496-3 1.6.2.1), the 2-byte common form.
bool AacConfig::Parse(const std::string& a) {
    if (a.size() < 2) return false;
    const uint8_t b0 = (uint8_t)a[0], b1 = (uint8_t)a[1];
    object_type = b0 >> 3;
    sample_rate_index = ((b0 & 7) << 1) | (b1 >> 7);
    channels = (b1 >> 3) & 0x0f;
    return object_type > 0 && object_type < 31 && sample_rate_index < 13 && channels > 0 && channels < 8;
}

uint32_t TsWriter::Crc32(const uint8_t* p, size_t n) {
    uint32_t crc = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) {
        crc ^= (uint32_t)p[i] << 24;
        for (int k = 0; k < 8; ++k) crc = (crc & 0x80000000u) ? (crc << 1) ^ 0x04C11DB7u : crc << 1;
    }
    return crc;
}

TsWriter::TsWriter(Buf* out) : _out(out) {}

uint8_t TsWriter::NextCc(uint16_t pid) {
    uint8_t& c = _cc[cc_index(pid)];
    const uint8_t v = c;
    c = (uint8_t)((c + 1) & 0x0f);
    return v;
}

void TsWriter::WritePsi(uint16_t pid, const std::vector<uint8_t>& section) {
    uint8_t pkt[kTsPacket];
    memset(pkt, 0xFF, sizeof(pkt));
    pkt[0] = 0x47;
    pkt[1] = (uint8_t)(0x40 | (pid >> 8));  // payload_unit_start
    pkt[2] = (uint8_t)pid;
    pkt[3] = (uint8_t)(0x10 | NextCc(pid));  // payload only
    pkt[4] = 0;                               // pointer_field
    memcpy(pkt + 5, section.data(), section.size());
    _out->append(pkt, sizeof(pkt));
}

void TsWriter::WritePatPmt() {
    // PAT: program 1 -> PMT PID.
    std::vector<uint8_t> pat = {0x00, 0xB0, 0, 0x00, 0x01, 0xC1, 0x00, 0x00, 0x00, 0x01,
                                (uint8_t)(0xE0 | (TS_PID_PMT >> 8)), (uint8_t)TS_PID_PMT};
    pat[2] = (uint8_t)(pat.size() - 3 + 4);  // section_length incl. CRC
    uint32_t crc = Crc32(pat.data(), pat.size());
    for (int i = 3; i >= 0; --i) pat.push_back((uint8_t)(crc >> (8 * i)));
    WritePsi(TS_PID_PAT, pat);
    // PMT: H.264 and/or AAC elementary streams; PCR rides on video if any.
    const uint16_t pcr_pid = _has_video ? TS_PID_VIDEO : TS_PID_AUDIO;
    std::vector<uint8_t> pmt = {0x02, 0xB0, 0, 0x00, 0x01, 0xC1, 0x00, 0x00,
                                (uint8_t)(0xE0 | (pcr_pid >> 8)), (uint8_t)pcr_pid, 0xF0, 0x00};
    if (_has_video) {
        const uint8_t es[] = {TS_STREAM_H264, (uint8_t)(0xE0 | (TS_PID_VIDEO >> 8)), (uint8_t)TS_PID_VIDEO, 0xF0, 0x00};
        pmt.insert(pmt.end(), es, es + 5);
    }
    if (_has_audio) {
        const uint8_t es[] = {TS_STREAM_AAC, (uint8_t)(0xE0 | (TS_PID_AUDIO >> 8)), (uint8_t)TS_PID_AUDIO, 0xF0, 0x00};
        pmt.insert(pmt.end(), es, es + 5);
    }
    pmt[2] = (uint8_t)(pmt.size() - 3 + 4);
    crc = Crc32(pmt.data(), pmt.size());
    for (int i = 3; i >= 0; --i) pmt.push_back((uint8_t)(crc >> (8 * i)));
    WritePsi(TS_PID_PMT, pmt);
    _wrote_pat_pmt = true;
}

void TsWriter::WritePes(uint16_t pid, uint8_t stream_id, const std::string& es, int64_t pts, int64_t dts,
                        bool keyframe, bool with_pcr) {
    // PES header
    uint8_t hdr[19];
    const bool has_dts = dts != pts;
    const uint8_t hlen = has_dts ? 10 : 5;
    hdr[0] = 0x00;
    hdr[1] = 0x00;
    hdr[2] = 0x01;
    hdr[3] = stream_id;
    const size_t pes_len = 3 + hlen + es.size();
    const uint16_t field = (stream_id == 0xE0 && pes_len > 0xFFFF) ? 0 : (uint16_t)pes_len;  // 0: unbounded video
    hdr[4] = (uint8_t)(field >> 8);
    hdr[5] = (uint8_t)field;
    hdr[6] = 0x84;  // '10', data_alignment_indicator
    hdr[7] = has_dts ? 0xC0 : 0x80;
    hdr[8] = hlen;
    put_ts(hdr + 9, has_dts ? 3 : 2, pts);
    if (has_dts) put_ts(hdr + 14, 1, dts);
    std::string pes(reinterpret_cast<const char*>(hdr), 9 + hlen);
    pes += es;

    size_t off = 0;
    bool first = true;
    while (off < pes.size()) {
        uint8_t pkt[kTsPacket];
        pkt[0] = 0x47;
        pkt[1] = (uint8_t)((first ? 0x40 : 0) | (pid >> 8));
        pkt[2] = (uint8_t)pid;
        // adaptation field: PCR / random access on the first packet, stuffing
        // on the last one
        uint8_t af[kTsPacket];
        size_t aflen = 0;  // bytes after the length byte
        bool need_af = false;
        if (first && (with_pcr || keyframe)) {
            need_af = true;
            af[0] = (uint8_t)((keyframe ? 0x40 : 0) | (with_pcr ? 0x10 : 0));
            aflen = 1;
            if (with_pcr) {
                const uint64_t base = (uint64_t)dts & 0x1FFFFFFFFull;
                af[1] = (uint8_t)(base >> 25);
                af[2] = (uint8_t)(base >> 17);
                af[3] = (uint8_t)(base >> 9);
                af[4] = (uint8_t)(base >> 1);
                af[5] = (uint8_t)(((base & 1) << 7) | 0x7E);  // 6 reserved bits, ext msb 0
                af[6] = 0;
                aflen = 7;
            }
        }
        size_t room = kTsPacket - 4 - (need_af ? 1 + aflen : 0);
        const size_t left = pes.size() - off;
        if (left < room) {
            // stuff the adaptation field so the payload ends the packet
            size_t stuff = room - left;
            if (!need_af) {
                need_af = true;
                --stuff;  // the length byte itself
                if (stuff > 0) {
                    af[0] = 0x00;
                    aflen = 1;
                    --stuff;
                }
            }
            memset(af + aflen, 0xFF, stuff);
            aflen += stuff;
            room = left;
        }
        pkt[3] = (uint8_t)((need_af ? 0x30 : 0x10) | NextCc(pid));
        size_t p = 4;
        if (need_af) {
            pkt[p++] = (uint8_t)aflen;
            memcpy(pkt + p, af, aflen);
            p += aflen;
        }
        memcpy(pkt + p, pes.data() + off, room);
        off += room;
        _out->append(pkt, sizeof(pkt));
        first = false;
    }
}

int TsWriter::Write(const RtmpVideoMessage& msg) {
    if (msg.codec != 7) {
        _error = "only AVC video can be muxed into TS";
        return -1;
    }
    const std::string d = msg.data.to_string();
    if (d.size() < 4) {
        _error = "short AVC packet";
        return -1;
    }
    const uint8_t type = (uint8_t)d[0];
    int32_t cts = (int32_t)be(d, 1, 3);
    if (cts & 0x800000) cts -= 0x1000000;  // SI24
    if (type == 0) {
        if (!_avc.Parse(d.substr(4))) {
            _error = "bad AVCDecoderConfigurationRecord";
            return -1;
        }
        _avc_ready = true;
        if (!_has_video) {
            _has_video = true;
            _wrote_pat_pmt = false;
        }
        return 0;
    }
    if (type != 1) return 0;  // end of sequence
    if (!_avc_ready) {
        _error = "AVC frame before the sequence header";
        return -1;
    }
    // AVCC -> Annex B: AUD, then SPS/PPS before an IDR, then every NALU.
    static const char kStart[4] = {0, 0, 0, 1};
    std::string es;
    bool has_aud = false, has_idr = false;
    std::vector<std::pair<size_t, size_t>> nalus;
    for (size_t p = 4; p < d.size();) {
        if (p + (size_t)_avc.nalu_length_size > d.size()) {
            _error = "truncated NALU length";
            return -1;
        }
        const size_t len = be(d, p, _avc.nalu_length_size);
        p += (size_t)_avc.nalu_length_size;
        if (p + len > d.size()) {
            _error = "truncated NALU";
            return -1;
        }
        if (len > 0) {
            const int nt = (uint8_t)d[p] & 0x1f;
            has_aud |= nt == 9;
            has_idr |= nt == 5;
            nalus.emplace_back(p, len);
        }
        p += len;
    }
    if (!has_aud) es.append("\x00\x00\x00\x01\x09\xf0", 6);
    if (has_idr) {
        for (const std::string& s : _avc.sps) es.append(kStart, 4).append(s);
        for (const std::string& s : _avc.pps) es.append(kStart, 4).append(s);
    }
    for (auto& n : nalus) es.append(kStart, 4).append(d, n.first, n.second);
    if (!_wrote_pat_pmt) WritePatPmt();
    const int64_t dts = (int64_t)msg.timestamp * 90;
    const int64_t pts = dts + (int64_t)cts * 90;
    WritePes(TS_PID_VIDEO, 0xE0, es, pts, dts, has_idr || msg.frame_type == 1, true);
    return 0;
}

int TsWriter::Write(const RtmpAudioMessage& msg) {
    if (msg.codec != 10) {
        _error = "only AAC audio can be muxed into TS";
        return -1;
    }
    const std::string d = msg.data.to_string();
    if (d.size() < 2) {
        _error = "short AAC packet";
        return -1;
    }
    if ((uint8_t)d[0] == 0) {
        if (!_aac.Parse(d.substr(1))) {
            _error = "bad AudioSpecificConfig";
            return -1;
        }
        _aac_ready = true;
        if (!_has_audio) {
            _has_audio = true;
            _wrote_pat_pmt = false;
        }
        return 0;
    }
    if (!_aac_ready) {
        _error = "AAC frame before the sequence header";
        return -1;
    }
    const size_t raw = d.size() - 1;
    const size_t flen = raw + 7;
    if (flen > 0x1FFF) {
        _error = "AAC frame too large for ADTS";
        return -1;
    }
    uint8_t adts[7];
    const int profile = (_aac.object_type - 1) & 3;
    adts[0] = 0xFF;
    adts[1] = 0xF1;  // MPEG-4, layer 0, no CRC
    adts[2] = (uint8_t)((profile << 6) | (_aac.sample_rate_index << 2) | ((_aac.channels >> 2) & 1));
    adts[3] = (uint8_t)(((_aac.channels & 3) << 6) | (flen >> 11));
    adts[4] = (uint8_t)(flen >> 3);
    adts[5] = (uint8_t)(((flen & 7) << 5) | 0x1F);  // buffer fullness 0x7FF
    adts[6] = 0xFC;
    std::string es(reinterpret_cast<const char*>(adts), 7);
    es.append(d, 1, raw);
    if (!_wrote_pat_pmt) WritePatPmt();
    const int64_t pts = (int64_t)msg.timestamp * 90;
    WritePes(TS_PID_AUDIO, 0xC0, es, pts, pts, false, !_has_video);
    return 0;
}

}  // namespace mrpc
