// MPEG-TS muxer tests: the output is parsed back packet by packet (sync
// bytes, continuity counters per PID, PSI CRCs), PES packets are reassembled
// and their PTS/DTS, Annex-B NALUs (AUD, SPS/PPS before IDR) and ADTS
// headers are checked against the RTMP input. The reference ships no TS
// test or fixture, so parity is pinned to ISO 13818-1 layout only.
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "rtmp/ts.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

struct Pes {
    uint16_t pid;
    int64_t pts = -1, dts = -1;
    std::string es;
    bool random_access = false;
    bool has_pcr = false;
    int64_t pcr_base = -1;
};

int64_t get_ts(const uint8_t* p) {
    return ((int64_t)((p[0] >> 1) & 7) << 30) | ((int64_t)p[1] << 22) | ((int64_t)(p[2] >> 1) << 15) |
           ((int64_t)p[3] << 7) | (p[4] >> 1);
}

struct Demux {
    std::map<uint16_t, int> last_cc;
    std::map<uint16_t, std::string> psi;  // first section per PID
    std::vector<Pes> pes;
    std::map<uint16_t, size_t> open;  // pid -> index in pes
    std::map<uint16_t, std::string> raw;
    int errors = 0;
    void Feed(const std::string& ts) {
        if (ts.size() % 188) ++errors;
        for (size_t off = 0; off + 188 <= ts.size(); off += 188) {
            const uint8_t* p = reinterpret_cast<const uint8_t*>(ts.data()) + off;
            if (p[0] != 0x47) ++errors;
            const bool pusi = p[1] & 0x40;
            const uint16_t pid = (uint16_t)(((p[1] & 0x1f) << 8) | p[2]);
            const int afc = (p[3] >> 4) & 3;
            const int cc = p[3] & 0x0f;
            if (last_cc.count(pid) && ((last_cc[pid] + 1) & 0x0f) != cc) ++errors;
            last_cc[pid] = cc;
            size_t i = 4;
            bool ra = false, pcr = false;
            int64_t pcr_base = -1;
            if (afc & 2) {
                const size_t alen = p[4];
                if (alen > 0) {
                    ra = p[5] & 0x40;
                    pcr = p[5] & 0x10;
                    if (pcr) pcr_base = ((int64_t)p[6] << 25) | (p[7] << 17) | (p[8] << 9) | (p[9] << 1) | (p[10] >> 7);
                }
                i = 5 + alen;
            }
            if (!(afc & 1)) continue;
            std::string payload(reinterpret_cast<const char*>(p) + i, 188 - i);
            if (pid == 0 || pid == TS_PID_PMT) {
                if (pusi && !psi.count(pid)) psi[pid] = payload.substr(1);
                continue;
            }
            if (pusi) {
                Pes x;
                x.pid = pid;
                x.random_access = ra;
                x.has_pcr = pcr;
                x.pcr_base = pcr_base;
                open[pid] = pes.size();
                pes.push_back(x);
                raw[pid].clear();
            }
            if (!open.count(pid)) {
                ++errors;
                continue;
            }
            raw[pid] += payload;
        }
    }
};

// Collect PES packets by re-muxing one message at a time.
Pes OnePes(TsWriter&, Buf* out, Demux* d) {
    std::string s = out->to_string();
    out->clear();
    d->Feed(s);
    Pes x = d->pes.back();
    const std::string& r = d->raw[x.pid];
    const uint8_t* p = reinterpret_cast<const uint8_t*>(r.data());
    if (r.size() < 9 || p[0] != 0 || p[1] != 0 || p[2] != 1) {
        ++d->errors;
        return x;
    }
    const int flags = p[7] >> 6;
    const int hlen = p[8];
    if (flags & 2) x.pts = get_ts(p + 9);
    x.dts = (flags & 1) ? get_ts(p + 14) : x.pts;
    const size_t pes_len = ((size_t)p[4] << 8) | p[5];
    x.es = r.substr(9 + hlen);
    if (pes_len && pes_len != r.size() - 6) ++d->errors;
    return x;
}

RtmpVideoMessage AvcSeqHeader(const std::string& sps, const std::string& pps) {
    std::string rec;
    rec += (char)1;
    rec += sps[1];
    rec += sps[2];
    rec += sps[3];
    rec += (char)0xFF;  // 4-byte NALU lengths
    rec += (char)0xE1;
    rec += (char)(sps.size() >> 8);
    rec += (char)sps.size();
    rec += sps;
    rec += (char)1;
    rec += (char)(pps.size() >> 8);
    rec += (char)pps.size();
    rec += pps;
    RtmpVideoMessage m;
    m.frame_type = 1;
    std::string d("\x00\x00\x00\x00", 4);
    d += rec;
    m.data.append(d);
    return m;
}

RtmpVideoMessage AvcFrame(uint32_t ts, int cts, bool key, const std::vector<std::string>& nalus) {
    RtmpVideoMessage m;
    m.timestamp = ts;
    m.frame_type = key ? 1 : 2;
    std::string d;
    d += (char)1;
    d += (char)(cts >> 16);
    d += (char)(cts >> 8);
    d += (char)cts;
    for (const std::string& n : nalus) {
        const uint32_t l = (uint32_t)n.size();
        d += (char)(l >> 24);
        d += (char)(l >> 16);
        d += (char)(l >> 8);
        d += (char)l;
        d += n;
    }
    m.data.append(d);
    return m;
}

}  // namespace

TEST(Ts, crc32_mpeg2_check_value) {
    // CRC-32/MPEG-2 check value over "123456789"
    EXPECT_EQ(TsWriter::Crc32(reinterpret_cast<const uint8_t*>("123456789"), 9), 0x0376E6E7u);
}

TEST(Ts, avc_and_aac_round_trip) {
    Buf out;
    TsWriter w(&out);
    Demux d;
    const std::string sps("\x67\x64\x00\x1f\xac\xd9\x40\x50", 8), pps("\x68\xeb\xe3\xcb", 4);
    ASSERT_EQ(w.Write(AvcSeqHeader(sps, pps)), 0);
    RtmpAudioMessage ash;
    ash.data.append(std::string("\x00\x12\x10", 3));  // AAC LC, 44.1 kHz, stereo
    ASSERT_EQ(w.Write(ash), 0);
    EXPECT_EQ(out.size(), 0u);  // sequence headers produce no packets

    std::string idr(5000, '\x11');
    idr[0] = 0x65;
    ASSERT_EQ(w.Write(AvcFrame(1000, 40, true, {idr})), 0);
    // PAT + PMT first
    std::string first = out.to_string();
    d.Feed(first.substr(0, 376));
    ASSERT_TRUE(d.psi.count(0) && d.psi.count(TS_PID_PMT));
    for (uint16_t pid : {(uint16_t)0, (uint16_t)TS_PID_PMT}) {
        const std::string& s = d.psi[pid];
        const size_t slen = (((uint8_t)s[1] & 0x0f) << 8) | (uint8_t)s[2];
        EXPECT_EQ(TsWriter::Crc32(reinterpret_cast<const uint8_t*>(s.data()), 3 + slen), 0u);
    }
    const std::string& pmt = d.psi[TS_PID_PMT];
    EXPECT_EQ((uint8_t)pmt[0], 0x02);
    EXPECT_EQ((((uint8_t)pmt[8] & 0x1f) << 8) | (uint8_t)pmt[9], (int)TS_PID_VIDEO);  // PCR PID
    EXPECT_EQ((uint8_t)pmt[12], TS_STREAM_H264);
    EXPECT_EQ((uint8_t)pmt[17], TS_STREAM_AAC);
    out.clear();
    out.append(first.substr(376));
    Pes v = OnePes(w, &out, &d);
    EXPECT_EQ(v.pid, (uint16_t)TS_PID_VIDEO);
    EXPECT_EQ(v.dts, 90000);
    EXPECT_EQ(v.pts, 90000 + 40 * 90);
    EXPECT_TRUE(v.random_access);
    EXPECT_TRUE(v.has_pcr);
    EXPECT_EQ(v.pcr_base, 90000);
    const std::string sc("\x00\x00\x00\x01", 4);
    const std::string want = sc + std::string("\x09\xf0", 2) + sc + sps + sc + pps + sc + idr;
    EXPECT_EQ(v.es.size(), want.size());
    EXPECT_TRUE(v.es == want);

    // inter frame: AUD + NALUs, no SPS/PPS, no random access, DTS == PTS
    std::string p1(300, '\x22'), p2(77, '\x33');
    p1[0] = 0x41;
    p2[0] = 0x41;
    ASSERT_EQ(w.Write(AvcFrame(1040, 0, false, {p1, p2})), 0);
    Pes v2 = OnePes(w, &out, &d);
    EXPECT_FALSE(v2.random_access);
    EXPECT_EQ(v2.pts, 1040 * 90);
    EXPECT_EQ(v2.dts, v2.pts);
    EXPECT_TRUE(v2.es == sc + std::string("\x09\xf0", 2) + sc + p1 + sc + p2);

    // AAC frame: ADTS header + raw data
    RtmpAudioMessage a;
    a.timestamp = 1023;
    std::string raw(371, '\x5a');
    a.data.append(std::string("\x01", 1) + raw);
    ASSERT_EQ(w.Write(a), 0);
    Pes au = OnePes(w, &out, &d);
    EXPECT_EQ(au.pid, (uint16_t)TS_PID_AUDIO);
    EXPECT_EQ(au.pts, 1023 * 90);
    ASSERT_EQ(au.es.size(), raw.size() + 7);
    const uint8_t* h = reinterpret_cast<const uint8_t*>(au.es.data());
    EXPECT_EQ(h[0], 0xFF);
    EXPECT_EQ(h[1] & 0xF6, 0xF0);
    EXPECT_EQ(h[2] >> 6, 1);             // profile = AAC LC - 1
    EXPECT_EQ((h[2] >> 2) & 0x0f, 4);    // 44.1 kHz
    EXPECT_EQ(((h[2] & 1) << 2) | (h[3] >> 6), 2);  // stereo
    const size_t flen = ((size_t)(h[3] & 3) << 11) | ((size_t)h[4] << 3) | (h[5] >> 5);
    EXPECT_EQ(flen, raw.size() + 7);
    EXPECT_TRUE(au.es.substr(7) == raw);
    EXPECT_FALSE(au.has_pcr);  // PCR rides on video

    // many frames of varied sizes: packet stream stays consistent
    for (int i = 0; i < 50; ++i) {
        std::string n((size_t)(i * 97 + 1), (char)i);
        n[0] = (i % 10 == 0) ? 0x65 : 0x41;
        ASSERT_EQ(w.Write(AvcFrame(1080 + i * 40, 0, i % 10 == 0, {n})), 0);
        RtmpAudioMessage am;
        am.timestamp = 1080 + i * 23;
        am.data.append(std::string("\x01", 1) + std::string((size_t)(i * 13 + 1), 'a'));
        ASSERT_EQ(w.Write(am), 0);
    }
    d.Feed(out.to_string());
    EXPECT_EQ(d.errors, 0);

    // PAT/PMT again at a segment boundary, continuity counters keep going
    w.add_pat_pmt_on_next_write();
    out.clear();
    ASSERT_EQ(w.Write(AvcFrame(5000, 0, true, {idr})), 0);
    const std::string seg = out.to_string();
    EXPECT_EQ((uint8_t)seg[1] & 0x1f, 0);
    EXPECT_EQ((uint8_t)seg[2], 0);
    d.Feed(seg);
    EXPECT_EQ(d.errors, 0);
}

TEST(Ts, rejects_bad_input) {
    Buf out;
    TsWriter w(&out);
    RtmpVideoMessage v;
    v.codec = 2;  // Sorenson H.263
    v.data.append("xxxxxx");
    EXPECT_NE(w.Write(v), 0);
    EXPECT_NE(w.Write(AvcFrame(0, 0, true, {std::string("\x65", 1)})), 0);  // before the sequence header
    RtmpAudioMessage a;
    a.codec = 2;  // MP3
    a.data.append("xx");
    EXPECT_NE(w.Write(a), 0);
    AvcConfig c;
    EXPECT_FALSE(c.Parse(std::string("\x02\x00", 2)));
    AacConfig ac;
    EXPECT_FALSE(ac.Parse(std::string("\xff\xff", 2)));
    EXPECT_EQ(out.size(), 0u);
}
