// RTMP: media streaming over one TCP connection (role of the reference's
// src/brpc/rtmp.h, policy/rtmp_protocol.cpp and rtmp.cpp).
//
// Server: set ServerOptions.rtmp_service; every createStream asks the
// service for a RtmpServerStream that receives play/publish and media
// callbacks. Client: RtmpClient owns a connection (handshake + connect),
// RtmpClientStreams multiplex on it (createStream + play/publish).
//
// Wire: simple or digest ("complex", rtmp/handshake.h) handshake, chunk streams with
// format 0-3 headers, extended timestamps and negotiated chunk sizes, AMF0
// commands (connect/createStream/play/publish/deleteStream/onStatus),
// audio/video/data messages. Incoming messages of a connection are
// dispatched in order on the connection's read fiber.
//
// FlvWriter/FlvReader convert between RTMP messages and FLV tags.
//
// Servers also acknowledge received bytes per the peer's window
// (Acknowledgement after every window-ack-size bytes), answer user-control
// pings, and accept AMF3-wrapped commands/data (types 17/15).
#pragma once

#include <atomic>
#include <cstdint>
#include <limits>
#include <memory>
#include <mutex>
#include <string>

#include "base/buf.h"
#include "base/endpoint.h"
#include "rtmp/amf.h"
#include "rtmp/media.h"

namespace mrpc {

namespace rtmp_detail {
class Connection;
}

enum RtmpMessageType : uint8_t {
    RTMP_SET_CHUNK_SIZE = 1,
    RTMP_ABORT = 2,
    RTMP_ACK = 3,
    RTMP_USER_CONTROL = 4,
    RTMP_WINDOW_ACK_SIZE = 5,
    RTMP_SET_PEER_BANDWIDTH = 6,
    RTMP_AUDIO = 8,
    RTMP_VIDEO = 9,
    RTMP_DATA_AMF3 = 15,
    RTMP_COMMAND_AMF3 = 17,
    RTMP_DATA_AMF0 = 18,
    RTMP_COMMAND_AMF0 = 20,
};

struct RtmpAudioMessage {
    uint32_t timestamp = 0;
    uint8_t codec = 10;  // 10 = AAC
    uint8_t rate = 3;    // 44 kHz
    uint8_t bits = 1;    // 16 bit
    uint8_t type = 1;    // stereo
    Buf data;            // payload after the 1-byte audio header
};

struct RtmpVideoMessage {
    uint32_t timestamp = 0;
    uint8_t frame_type = 1;  // 1 key frame, 2 inter frame
    uint8_t codec = 7;       // 7 = AVC
    Buf data;                // payload after the 1-byte video header
};

struct RtmpMetaData {
    uint32_t timestamp = 0;
    rtmp::AMFValue data = rtmp::AMFValue::EcmaArray();
};

class RtmpStreamBase {
public:
    virtual ~RtmpStreamBase();
    // Media callbacks, called in order on the connection's read fiber.
    virtual void OnMetaData(RtmpMetaData* md, const std::string& name) {}
    virtual void OnAudioMessage(RtmpAudioMessage* msg) {}
    virtual void OnVideoMessage(RtmpVideoMessage* msg) {}
    // Data messages named "onCuePoint".
    virtual void OnCuePoint(RtmpCuePoint* cp) {}
    // Called once, before the first media/metadata/cue-point callback.
    virtual void OnFirstMessage() {}
    // The stream ended (deleteStream, connection closed, Destroy()).
    virtual void OnStop() {}

    int SendMetaData(const RtmpMetaData& md, const std::string& name = "onMetaData");
    int SendAudioMessage(const RtmpAudioMessage& msg);
    int SendVideoMessage(const RtmpVideoMessage& msg);
    int SendCuePoint(const RtmpCuePoint& cp);
    int SendAACMessage(const RtmpAACMessage& msg);
    int SendAVCMessage(const RtmpAVCMessage& msg);
    // A message of the application's own kind (reference rtmp.h:564): the
    // stream class that has one overrides this; the base fails (ENOTSUP).
    // `msg` stays owned by the caller.
    virtual int SendUserMessage(void* msg);
    // Ask the peer to stop; what is sent depends on the stream kind (a
    // server stream sends NetStream.Play.StreamNotFound). 0 when sent.
    virtual int SendStopMessage(const std::string& error_description);

    uint32_t stream_id() const { return _stream_id; }
    bool is_stopped() const { return _stopped.load(std::memory_order_acquire); }
    EndPoint remote_side() const;

    // ---- internal
    virtual int SendMessage(uint8_t type, uint32_t timestamp, const Buf& body);
    void CallOnStop();
    void CallOnFirstMessage() {
        if (!_has_data_ever) {
            _has_data_ever = true;
            OnFirstMessage();
        }
    }
    std::shared_ptr<rtmp_detail::Connection> _conn;
    uint32_t _stream_id = 0;
    std::atomic<bool> _stopped{false};
    bool _has_data_ever = false;  // touched only on the connection's read fiber
};

struct RtmpPlayOptions {
    std::string stream_name;
    double start = -2;
    double duration = -1;
    bool reset = true;
};

// play2 (switch bitrate / stream, reference rtmp.proto RtmpPlay2Options):
// NaN numbers and empty strings are left out of the AMF object.
struct RtmpPlay2Options {
    double len = std::numeric_limits<double>::quiet_NaN();
    double offset = std::numeric_limits<double>::quiet_NaN();
    std::string old_stream_name;
    double start = std::numeric_limits<double>::quiet_NaN();
    std::string stream_name;
    std::string transition;  // "switch", "swap", ...
};

struct RtmpConnectRequest {
    std::string app;
    std::string tcUrl;
    std::string flashVer;
};

class RtmpServerStream : public RtmpStreamBase {
public:
    // Accept by leaving *error empty, reject by setting it.
    virtual void OnPlay(const RtmpPlayOptions& opt, std::string* error) {}
    virtual void OnPublish(const std::string& name, const std::string& type, std::string* error) {}
    // play2 from the client (no reply is sent). The default logs and ignores.
    virtual void OnPlay2(const RtmpPlay2Options& opt);
    // seek / pause: 0 accepts (the client gets NetStream.Seek.Notify,
    // NetStream.Pause.Notify + StreamEOF or NetStream.Unpause.Notify +
    // StreamBegin), -1 rejects (_error). The defaults reject.
    virtual int OnSeek(double offset_ms);
    virtual int OnPause(bool pause, double offset_ms);
    // The client's buffer length (user control SetBufferLength).
    virtual void OnSetBufferLength(uint32_t buffer_length_ms) {}
    // NetStream.Play.StreamNotFound (level error) with the description.
    int SendStopMessage(const std::string& error_description) override;
    // User control StreamDry: no more data for now.
    int SendStreamDry();
    bool paused() const { return _paused; }

    bool _paused = false;  // read fiber only
};

class RtmpService {
public:
    virtual ~RtmpService() {}
    // A new stream of a connected client; the framework owns the result and
    // deletes it after OnStop().
    virtual RtmpServerStream* NewStream(const RtmpConnectRequest& req) = 0;
};

struct RtmpClientOptions {
    std::string app = "live";
    std::string tcUrl;
    std::string flashVer = "MRPC 1.0";
    int timeout_ms = 1000;          // connect / createStream / play / publish
    uint32_t chunk_size = 60000;    // announced with SetChunkSize
    uint32_t window_ack_size = 2500000;
    // Offer the digest ("complex") handshake; servers that do not sign
    // their S1 fall back to the simple one.
    bool complex_handshake = false;
};

class RtmpClient {
public:
    RtmpClient();
    ~RtmpClient();
    // Connects, handshakes and sends `connect`; 0 when the server accepted.
    int Init(const char* server_addr_and_port, const RtmpClientOptions& options);
    bool initialized() const { return (bool)_conn; }
    const RtmpClientOptions& options() const { return _options; }
    std::shared_ptr<rtmp_detail::Connection> connection() const { return _conn; }
    // Both sides signed the handshake (complex_handshake offered and accepted).
    bool complex_handshake_done() const;
    // User-control PingRequest; the round trip in microseconds, -1 on timeout.
    int64_t Ping(int timeout_ms = 1000);
    // Acknowledgements this connection sent for the server's window.
    int64_t acks_sent() const;
    // The connection's socket (0 before Init); failing it drops every stream.
    uint64_t socket_id() const;
    // "rtmp://HOST:PORT/APP"
    const std::string& url_prefix() const { return _url_prefix; }

private:
    RtmpClientOptions _options;
    std::string _url_prefix;
    std::shared_ptr<rtmp_detail::Connection> _conn;
};

struct RtmpClientStreamOptions {
    std::string play_name;      // set one of play_name / publish_name
    std::string publish_name;
    std::string publish_type = "live";
    // Announced with SetBufferLength after play (-1: not sent).
    int buffer_length_ms = 1000;
};

class RtmpClientStream : public RtmpStreamBase {
public:
    ~RtmpClientStream() override;
    // createStream + play/publish; returns 0 once the server accepted.
    int Init(RtmpClient* client, const RtmpClientStreamOptions& options);
    // deleteStream and detach (OnStop is called). Idempotent.
    void Destroy();
    // Change bitrate / stream of a playing stream (no reply expected).
    int Play2(const RtmpPlay2Options& opt);
    // Seek to offset_ms in the media / playlist; pause (true) or resume.
    // 0 when the command was sent; the server's verdict arrives as
    // onStatus (see last_status()).
    int Seek(double offset_ms);
    int Pause(bool pause, double offset_ms);
    // Called for every onStatus / _error of this stream after it started.
    virtual void OnStatus(const std::string& level, const std::string& code, const std::string& description) {}
    // code of the last onStatus / _error seen for this stream ("" if none)
    std::string last_status() const;
    // "rtmp://HOST:PORT/APP/STREAM"
    std::string rtmp_url() const;

    // ---- internal
    void SetLastStatus(const std::string& code);
    struct StatusSink {
        std::mutex mu;
        RtmpClientStream* stream = nullptr;
    };
    std::shared_ptr<StatusSink> _sink;
    std::string _url_prefix;
    std::string _name;
    mutable std::mutex _status_mu;
    std::string _last_status;
};

// A client stream that outlives its connection (the reference's
// RtmpRetryingClientStream, src/brpc/rtmp.h:880-1050): when the sub stream
// stops for any reason other than Destroy(), a new client is obtained from
// the creator and the play/publish is re-issued, first `fast_retry_count`
// times immediately, then every `retry_interval_ms`, until
// `max_retry_duration_ms` of failing (-1: forever). Media sent while no sub
// stream is up fails with EAGAIN; callbacks of every sub stream arrive on
// this object.
struct RtmpRetryingClientStreamOptions : public RtmpClientStreamOptions {
    int retry_interval_ms = 1000;
    int max_retry_duration_ms = -1;
    int fast_retry_count = 2;
};

class RtmpSubStreamCreator {
public:
    virtual ~RtmpSubStreamCreator() {}
    // A connected client for the next sub stream (nullptr: try later).
    virtual std::shared_ptr<RtmpClient> NewClient() = 0;
};

class RtmpRetryingClientStream : public RtmpStreamBase {
public:
    RtmpRetryingClientStream();
    ~RtmpRetryingClientStream() override;
    // Takes ownership of `creator`. 0 when the first sub stream is up;
    // otherwise retries continue in the background and -1 is returned.
    int Init(RtmpSubStreamCreator* creator, const RtmpRetryingClientStreamOptions& options);
    void Destroy();
    // Sub streams started after the first one.
    int64_t reconnects() const;
    bool connected() const;
    // Called after every successful (re)start of the sub stream.
    virtual void OnSubStreamStarted() {}

    int SendMessage(uint8_t type, uint32_t timestamp, const Buf& body) override;

    struct Impl;

private:
    std::shared_ptr<Impl> _impl;
};

// FLV container <-> RTMP messages.
class FlvWriter {
public:
    explicit FlvWriter(Buf* out);  // writes the FLV header on the first tag
    int Write(const RtmpVideoMessage& msg);
    int Write(const RtmpAudioMessage& msg);
    int Write(const RtmpMetaData& md, const std::string& name = "onMetaData");

private:
    int WriteTag(uint8_t type, uint32_t ts, const Buf& body);
    Buf* _out;
    bool _wrote_header = false;
};

class FlvReader {
public:
    explicit FlvReader(Buf* in);
    // 0 and the type of the next tag (8/9/18); EAGAIN when incomplete.
    int PeekMessageType(uint8_t* type);
    int Read(RtmpVideoMessage* msg);
    int Read(RtmpAudioMessage* msg);
    int Read(RtmpMetaData* md, std::string* name);

private:
    int ReadTag(uint8_t want, uint32_t* ts, Buf* body);
    Buf* _in;
    bool _read_header = false;
};

namespace rtmp {
// Server-side handshake counters (tests, /vars): complex handshakes served,
// and clients whose C2 was not signed.
int64_t ComplexHandshakesServed();
int64_t UnsignedC2Count();
}  // namespace rtmp

}  // namespace mrpc
