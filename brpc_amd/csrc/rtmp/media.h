// RTMP media payloads: AAC and AVC/H.264 inside RTMP audio/video messages
// (the reference's RtmpAACMessage / AudioSpecificConfig / RtmpAVCMessage /
// AVCDecoderConfigurationRecord / AVCNaluIterator / RtmpCuePoint,
// src/brpc/rtmp.h:107-384). Written from the FLV spec (AUDIODATA/VIDEODATA
// tag headers), ISO/IEC 14496-3 (AudioSpecificConfig, ADTS) and 14496-10
// (SPS syntax, Annex B byte streams) and 14496-15 (avcC).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "base/buf.h"
#include "rtmp/amf.h"

namespace mrpc {

struct RtmpAudioMessage;
struct RtmpVideoMessage;

// ---------------------------------------------------------------- AAC
enum AACPacketType : uint8_t { AAC_PACKET_SEQUENCE_HEADER = 0, AAC_PACKET_RAW = 1 };

struct RtmpAACMessage {
    uint32_t timestamp = 0;
    uint8_t rate = 3;   // FLV SoundRate: always 3 (44 kHz) for AAC
    uint8_t bits = 1;   // 16 bit
    uint8_t type = 1;   // stereo
    AACPacketType packet_type = AAC_PACKET_RAW;
    Buf data;           // AudioSpecificConfig (sequence header) or one raw frame

    // From an audio message whose codec is AAC (10); -1 otherwise.
    int Create(const RtmpAudioMessage& msg);
    void ToAudioMessage(RtmpAudioMessage* msg) const;
};

struct AudioSpecificConfig {
    uint8_t aac_object = 2;          // 1 main, 2 LC, 3 SSR, 5 SBR, ...
    uint8_t sample_rate_index = 4;   // 15 = explicit sample_rate
    uint32_t sample_rate = 44100;
    uint8_t channels = 2;            // channelConfiguration

    // Parse the sequence header payload; -1 when malformed.
    int Create(const Buf& data);
    int Create(const void* data, size_t n);
    // Serialize (2 bytes for the indexed rates, 5 with an explicit rate).
    std::string Serialize() const;
    // 7-byte ADTS header (no CRC) for a raw frame of `payload_len` bytes;
    // -1 when the config cannot be expressed in ADTS.
    int MakeAdtsHeader(size_t payload_len, uint8_t out[7]) const;
};

// Index into the ISO sampling-frequency table, or 15 when not listed.
uint8_t AacSampleRateIndex(uint32_t rate);
uint32_t AacSampleRate(uint8_t index);  // 0 for 13..15

// ---------------------------------------------------------------- AVC
enum AVCPacketType : uint8_t { AVC_PACKET_SEQUENCE_HEADER = 0, AVC_PACKET_NALU = 1, AVC_PACKET_END_OF_SEQUENCE = 2 };

enum AVCNaluType : uint8_t {
    AVC_NALU_NONIDR = 1,
    AVC_NALU_IDR = 5,
    AVC_NALU_SEI = 6,
    AVC_NALU_SPS = 7,
    AVC_NALU_PPS = 8,
    AVC_NALU_ACCESS_UNIT_DELIMITER = 9,
};

struct RtmpAVCMessage {
    uint32_t timestamp = 0;
    uint8_t frame_type = 1;          // 1 key frame, 2 inter frame
    AVCPacketType packet_type = AVC_PACKET_NALU;
    int32_t composition_time = 0;    // SI24, milliseconds (pts - dts)
    Buf data;                        // avcC record or length-prefixed NALUs

    // From a video message whose codec is AVC (7); -1 otherwise.
    int Create(const RtmpVideoMessage& msg);
    void ToVideoMessage(RtmpVideoMessage* msg) const;
};

struct AVCDecoderConfigurationRecord {
    uint8_t avc_profile = 0;
    uint8_t profile_compatibility = 0;
    uint8_t avc_level = 0;
    uint8_t length_size_minus1 = 3;
    std::vector<std::string> sps_list, pps_list;
    // From the first SPS (0 when it could not be parsed).
    int width = 0, height = 0;

    int Create(const Buf& data);
    int Create(const void* data, size_t n);
    std::string Serialize() const;
};

// Parsed fields of a sequence parameter set NALU (with its 1-byte header).
struct AvcSps {
    uint8_t profile_idc = 0, constraint_flags = 0, level_idc = 0;
    uint32_t sps_id = 0, chroma_format_idc = 1;
    uint32_t bit_depth_luma = 8, bit_depth_chroma = 8;
    uint32_t log2_max_frame_num = 4, pic_order_cnt_type = 0, max_num_ref_frames = 0;
    bool frame_mbs_only = true;
    int width = 0, height = 0;
    // -1 when truncated or out of range.
    int Parse(const std::string& nalu);
};

// Strip emulation-prevention bytes (00 00 03 -> 00 00) of a NALU payload.
std::string AvcUnescapeRbsp(const void* data, size_t n);

enum AVCNaluFormat { AVC_NALU_FORMAT_UNKNOWN = 0, AVC_NALU_FORMAT_ANNEXB = 1, AVC_NALU_FORMAT_IBMF = 2 };

// Walks the NALUs of one AVC packet: length-prefixed ("IBMF"/avcC framing,
// `length_size` bytes big endian) or Annex B start codes. The format is
// detected on the first call when *format is UNKNOWN and written back.
class AVCNaluIterator {
public:
    AVCNaluIterator(const Buf* data, int length_size, AVCNaluFormat* format);
    // Next NALU (with its header byte); false at the end or on a framing
    // error (error() tells them apart).
    bool Next(std::string* nalu, AVCNaluType* type = nullptr);
    bool error() const { return _error; }

private:
    bool NextAnnexB(std::string* nalu);
    bool NextIbmf(std::string* nalu);
    std::string _bytes;
    size_t _pos = 0;
    int _length_size;
    AVCNaluFormat* _format;
    bool _error = false;
};

// ---------------------------------------------------------------- cue points
struct RtmpCuePoint {
    uint32_t timestamp = 0;
    rtmp::AMFValue data = rtmp::AMFValue::Object();  // name, time, type, parameters
};

}  // namespace mrpc
