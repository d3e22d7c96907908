// MPEG-2 transport stream muxer for RTMP media: turns the AVC/H.264 video
// and AAC audio messages of an RTMP stream into 188-byte TS packets (PAT,
// PMT, PES with PTS/DTS, PCR, continuity counters), the format HLS segments
// use. Capability parity with the reference's TsWriter (src/brpc/ts.h:1225,
// ts.cpp:1068-1477): sequence headers are remembered, AVCC NALUs become
// Annex-B with an access-unit delimiter and SPS/PPS before every IDR, raw AAC
// frames get ADTS headers built from the AudioSpecificConfig.
// Written from ISO/IEC 13818-1 (TS/PES), 14496-10 Annex B and 14496-3 (ADTS).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "base/buf.h"
#include "rtmp/rtmp.h"

namespace mrpc {

enum TsPid : uint16_t { TS_PID_PAT = 0x0000, TS_PID_PMT = 0x1000, TS_PID_VIDEO = 0x0100, TS_PID_AUDIO = 0x0101 };
enum TsStreamType : uint8_t { TS_STREAM_AAC = 0x0f, TS_STREAM_H264 = 0x1b };

// Parsed AVCDecoderConfigurationRecord (the AVC sequence header).
struct AvcConfig {
    int nalu_length_size = 4;
    std::vector<std::string> sps, pps;
    int profile = 0, level = 0;
    bool Parse(const std::string& rec);
};

// Parsed AudioSpecificConfig (the AAC sequence header).
struct AacConfig {
    int object_type = 2;  // AAC LC
    int sample_rate_index = 4;  // 44100
    int channels = 2;
    bool Parse(const std::string& asc);
};

class TsWriter {
public:
    explicit TsWriter(Buf* out);
    // 0 on success; sequence headers are consumed without output.
    int Write(const RtmpVideoMessage& msg);
    int Write(const RtmpAudioMessage& msg);
    // Re-emit PAT/PMT before the next frame (e.g. at a segment boundary).
    void add_pat_pmt_on_next_write() { _wrote_pat_pmt = false; }
    int64_t discontinuity_counter() const { return _discontinuity; }
    std::string last_error() const { return _error; }

    // MPEG-2 CRC32 of PSI sections (poly 0x04C11DB7, MSB first).
    static uint32_t Crc32(const uint8_t* p, size_t n);

private:
    void WritePatPmt();
    void WritePsi(uint16_t pid, const std::vector<uint8_t>& section);
    void WritePes(uint16_t pid, uint8_t stream_id, const std::string& es, int64_t pts, int64_t dts, bool keyframe,
                  bool with_pcr);
    uint8_t NextCc(uint16_t pid);

    Buf* _out;
    bool _wrote_pat_pmt = false;
    bool _has_video = false, _has_audio = false;
    AvcConfig _avc;
    AacConfig _aac;
    bool _avc_ready = false, _aac_ready = false;
    uint8_t _cc[4] = {0, 0, 0, 0};  // PAT, PMT, video, audio
    int64_t _discontinuity = 0;
    std::string _error;
};

}  // namespace mrpc
