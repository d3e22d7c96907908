// RTMP (spirit of the reference's test/brpc_rtmp_unittest.cpp): AMF0 round
// trips, FLV writer/reader, and a live relay over loopback — one client
// publishes metadata/audio/video, two players receive them in order.
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "base/time.h"
#include "net/socket.h"
#include "rpc/server.h"
#include "rtmp/handshake.h"
#include "rtmp/rtmp.h"
#include "tests/test.h"

using namespace mrpc;
using rtmp::AMFValue;

TEST(Rtmp, amf0_round_trip) {
    AMFValue o = AMFValue::Object();
    o.Set("app", AMFValue::String("live"));
    o.Set("n", AMFValue::Number(3.5));
    o.Set("ok", AMFValue::Bool(true));
    o.Set("nil", AMFValue::Null());
    AMFValue arr = AMFValue::StrictArray();
    arr.items().push_back(AMFValue::Number(1));
    arr.items().push_back(AMFValue::String(std::string(70000, 'L')));  // long string
    o.Set("arr", arr);
    AMFValue ecma = AMFValue::EcmaArray();
    ecma.Set("width", AMFValue::Number(1920));
    o.Set("meta", ecma);
    std::string s;
    rtmp::WriteAMF(&s, AMFValue::String("connect"));
    rtmp::WriteAMF(&s, AMFValue::Number(1));
    rtmp::WriteAMF(&s, o);
    std::vector<AMFValue> v;
    ASSERT_TRUE(rtmp::ReadAMFList(s.data(), s.size(), &v));
    ASSERT_EQ(v.size(), 3u);
    EXPECT_EQ(v[0].str(), "connect");
    EXPECT_EQ(v[1].number(), 1.0);
    EXPECT_EQ(v[2].Find("app")->str(), "live");
    EXPECT_EQ(v[2].Find("n")->number(), 3.5);
    EXPECT_TRUE(v[2].Find("ok")->boolean());
    EXPECT_TRUE(v[2].Find("nil")->is_null());
    EXPECT_EQ(v[2].Find("arr")->items()[1].str().size(), 70000u);
    EXPECT_EQ(v[2].Find("meta")->Find("width")->number(), 1920.0);
    EXPECT_FALSE(rtmp::ReadAMFList(s.data(), s.size() - 3, &v));  // truncated
}

TEST(Rtmp, flv_writer_reader) {
    Buf flv;
    FlvWriter w(&flv);
    RtmpMetaData md;
    md.data.Set("duration", AMFValue::Number(12));
    ASSERT_EQ(w.Write(md), 0);
    for (int i = 0; i < 5; ++i) {
        RtmpVideoMessage vm;
        vm.timestamp = (uint32_t)(i * 40);
        vm.frame_type = i == 0 ? 1 : 2;
        vm.data.append("frame" + std::to_string(i));
        ASSERT_EQ(w.Write(vm), 0);
        RtmpAudioMessage am;
        am.timestamp = (uint32_t)(i * 40 + 1);
        am.data.append("aac" + std::to_string(i));
        ASSERT_EQ(w.Write(am), 0);
    }
    FlvReader r(&flv);
    uint8_t t;
    ASSERT_EQ(r.PeekMessageType(&t), 0);
    ASSERT_EQ((int)t, (int)RTMP_DATA_AMF0);
    RtmpMetaData md2;
    std::string name;
    ASSERT_EQ(r.Read(&md2, &name), 0);
    EXPECT_EQ(name, "onMetaData");
    EXPECT_EQ(md2.data.Find("duration")->number(), 12.0);
    for (int i = 0; i < 5; ++i) {
        RtmpVideoMessage vm;
        ASSERT_EQ(r.Read(&vm), 0);
        EXPECT_EQ(vm.timestamp, (uint32_t)(i * 40));
        EXPECT_EQ(vm.data.to_string(), "frame" + std::to_string(i));
        RtmpAudioMessage am;
        ASSERT_EQ(r.Read(&am), 0);
        EXPECT_EQ(am.data.to_string(), "aac" + std::to_string(i));
    }
    EXPECT_EQ(r.PeekMessageType(&t), EAGAIN);
}

namespace {
// Live relay: publishers' messages are forwarded to the players of the
// same stream name.
class RelayService;
class RelayStream : public RtmpServerStream {
public:
    explicit RelayStream(RelayService* s) : _svc(s) {}
    void OnPlay(const RtmpPlayOptions& opt, std::string* error) override;
    void OnPublish(const std::string& name, const std::string& type, std::string* error) override;
    void OnMetaData(RtmpMetaData* md, const std::string& name) override;
    void OnAudioMessage(RtmpAudioMessage* msg) override;
    void OnVideoMessage(RtmpVideoMessage* msg) override;
    void OnStop() override;

private:
    RelayService* _svc;
    std::string _name;
};

class RelayService : public RtmpService {
public:
    RtmpServerStream* NewStream(const RtmpConnectRequest& req) override {
        app = req.app;
        return new RelayStream(this);
    }
    std::mutex mu;
    std::map<std::string, std::set<RelayStream*>> players;
    std::atomic<int> stopped{0};
    std::string app;
    template <typename F>
    void ForEachPlayer(const std::string& name, F f) {
        std::lock_guard<std::mutex> g(mu);
        for (RelayStream* p : players[name]) f(p);
    }
};

void RelayStream::OnPlay(const RtmpPlayOptions& opt, std::string* error) {
    if (opt.stream_name == "missing") {
        *error = "no such stream";
        return;
    }
    _name = opt.stream_name;
    std::lock_guard<std::mutex> g(_svc->mu);
    _svc->players[_name].insert(this);
}
void RelayStream::OnPublish(const std::string& name, const std::string&, std::string*) { _name = name; }
void RelayStream::OnMetaData(RtmpMetaData* md, const std::string& name) {
    _svc->ForEachPlayer(_name, [&](RelayStream* p) { p->SendMetaData(*md, name); });
}
void RelayStream::OnAudioMessage(RtmpAudioMessage* msg) {
    _svc->ForEachPlayer(_name, [&](RelayStream* p) { p->SendAudioMessage(*msg); });
}
void RelayStream::OnVideoMessage(RtmpVideoMessage* msg) {
    _svc->ForEachPlayer(_name, [&](RelayStream* p) { p->SendVideoMessage(*msg); });
}
void RelayStream::OnStop() {
    _svc->stopped.fetch_add(1);
    std::lock_guard<std::mutex> g(_svc->mu);
    _svc->players[_name].erase(this);
}

class Player : public RtmpClientStream {
public:
    std::mutex mu;
    std::vector<std::string> got;
    std::atomic<int> n{0};
    void OnMetaData(RtmpMetaData* md, const std::string& name) override {
        std::lock_guard<std::mutex> g(mu);
        got.push_back("meta:" + name + ":" + std::to_string((int)md->data.Find("fps")->number()));
        n.fetch_add(1);
    }
    void OnVideoMessage(RtmpVideoMessage* m) override {
        std::lock_guard<std::mutex> g(mu);
        got.push_back("v" + std::to_string(m->timestamp) + ":" + m->data.to_string().substr(0, 8) + ":" +
                      std::to_string(m->data.size()));
        n.fetch_add(1);
    }
    void OnAudioMessage(RtmpAudioMessage* m) override {
        std::lock_guard<std::mutex> g(mu);
        got.push_back("a" + std::to_string(m->timestamp) + ":" + m->data.to_string());
        n.fetch_add(1);
    }
};
}  // namespace

TEST(Rtmp, live_relay_publish_and_play) {
    RelayService svc;
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    o.rtmp_service = &svc;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());

    RtmpClient client;
    RtmpClientOptions copt;
    copt.app = "relay";
    copt.timeout_ms = 3000;
    ASSERT_EQ(client.Init(addr.c_str(), copt), 0);
    Player p1, p2;
    RtmpClientStreamOptions po;
    po.play_name = "cam1";
    ASSERT_EQ(p1.Init(&client, po), 0);
    EXPECT_EQ(svc.app, "relay");  // the connect request reaches NewStream
    ASSERT_EQ(p2.Init(&client, po), 0);
    Player bad;
    RtmpClientStreamOptions bo;
    bo.play_name = "missing";
    EXPECT_NE(bad.Init(&client, bo), 0);

    RtmpClient pub_client;
    ASSERT_EQ(pub_client.Init(addr.c_str(), copt), 0);
    RtmpClientStream publisher;
    RtmpClientStreamOptions pubo;
    pubo.publish_name = "cam1";
    ASSERT_EQ(publisher.Init(&pub_client, pubo), 0);

    RtmpMetaData md;
    md.data.Set("fps", AMFValue::Number(25));
    ASSERT_EQ(publisher.SendMetaData(md), 0);
    const int N = 20;
    for (int i = 0; i < N; ++i) {
        RtmpVideoMessage vm;
        vm.timestamp = (uint32_t)(i * 40);
        // big frames exercise chunking (chunk size 60000) and fmt-3 continuations
        vm.data.append("frame" + std::to_string(100 + i) + std::string(i == 3 ? 200000 : 500, 'x'));
        ASSERT_EQ(publisher.SendVideoMessage(vm), 0);
        RtmpAudioMessage am;
        am.timestamp = (uint32_t)(i * 40 + 20);
        am.data.append("pcm" + std::to_string(i));
        ASSERT_EQ(publisher.SendAudioMessage(am), 0);
    }
    const int64_t deadline = monotonic_us() + 5000000;
    while ((p1.n.load() < 2 * N + 1 || p2.n.load() < 2 * N + 1) && monotonic_us() < deadline) usleep(2000);
    ASSERT_EQ(p1.n.load(), 2 * N + 1);
    ASSERT_EQ(p2.n.load(), 2 * N + 1);
    {
        std::lock_guard<std::mutex> g(p1.mu);
        EXPECT_EQ(p1.got[0], "meta:onMetaData:25");
        EXPECT_EQ(p1.got[1], "v0:frame100:508");
        EXPECT_EQ(p1.got[2], "a20:pcm0");
        EXPECT_EQ(p1.got[7], "v120:frame103:200008");  // reassembled across chunks
        EXPECT_EQ(p1.got[2 * N], "a" + std::to_string((N - 1) * 40 + 20) + ":pcm" + std::to_string(N - 1));
    }
    publisher.Destroy();
    p1.Destroy();
    p2.Destroy();
    const int64_t d2 = monotonic_us() + 3000000;
    while (svc.stopped.load() < 3 && monotonic_us() < d2) usleep(2000);
    EXPECT_GE(svc.stopped.load(), 3);
}

TEST(Rtmp, complex_handshake_digests) {
    for (rtmp::HandshakeSchema schema : {rtmp::kSchema0, rtmp::kSchema1}) {
        std::string c1, s1, d1, ds, s2, c2;
        rtmp::MakeComplexC1(schema, &c1);
        ASSERT_EQ(c1.size(), rtmp::kRtmpHandshakeSize);
        EXPECT_TRUE(rtmp::OffersComplexHandshake(c1));
        EXPECT_EQ(rtmp::ValidateComplexC1(c1, &d1), schema);
        EXPECT_EQ(d1.size(), 32u);
        EXPECT_EQ(rtmp::ValidateComplexS1(c1, nullptr), rtmp::kSchemaInvalid);  // player key != server key
        std::string bad = c1;
        bad[100] ^= 1;
        EXPECT_EQ(rtmp::ValidateComplexC1(bad, nullptr), rtmp::kSchemaInvalid);
        rtmp::MakeComplexS1(schema, &s1);
        EXPECT_EQ(rtmp::ValidateComplexS1(s1, &ds), schema);
        rtmp::MakeComplexS2(d1, &s2);
        EXPECT_TRUE(rtmp::ValidateComplexS2(s2, d1));
        EXPECT_FALSE(rtmp::ValidateComplexS2(s2, ds));  // bound to the client's digest
        rtmp::MakeComplexC2(ds, &c2);
        EXPECT_TRUE(rtmp::ValidateComplexC2(c2, ds));
        EXPECT_FALSE(rtmp::ValidateComplexC2(c2, d1));
    }
    std::string simple(rtmp::kRtmpHandshakeSize, '\0');
    EXPECT_FALSE(rtmp::OffersComplexHandshake(simple));
}

TEST(Rtmp, complex_handshake_ping_and_acks) {
    RelayService svc;
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    o.rtmp_service = &svc;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    const int64_t served0 = rtmp::ComplexHandshakesServed();
    RtmpClientOptions copt;
    copt.app = "relay";
    copt.timeout_ms = 3000;
    copt.complex_handshake = true;
    RtmpClient client;
    ASSERT_EQ(client.Init(addr.c_str(), copt), 0);
    EXPECT_TRUE(client.complex_handshake_done());
    EXPECT_EQ(rtmp::ComplexHandshakesServed(), served0 + 1);
    EXPECT_EQ(rtmp::UnsignedC2Count(), 0);
    RtmpClient simple;  // simple clients keep working on the same server
    copt.complex_handshake = false;
    ASSERT_EQ(simple.Init(addr.c_str(), copt), 0);
    EXPECT_FALSE(simple.complex_handshake_done());
    // user-control ping answered by the server
    const int64_t rtt = client.Ping(2000);
    EXPECT_GE(rtt, 0);
    // a player that receives more than the server's window acknowledges it
    Player player;
    RtmpClientStreamOptions po;
    po.play_name = "big";
    ASSERT_EQ(player.Init(&client, po), 0);
    RtmpClientStream pub;
    RtmpClientStreamOptions pubo;
    pubo.publish_name = "big";
    ASSERT_EQ(pub.Init(&simple, pubo), 0);
    const int N = 30;
    for (int i = 0; i < N; ++i) {
        RtmpVideoMessage vm;
        vm.timestamp = (uint32_t)(i * 40);
        vm.data.append(std::string(200000, (char)('a' + i % 26)));  // 6 MB in total
        ASSERT_EQ(pub.SendVideoMessage(vm), 0);
    }
    const int64_t deadline = monotonic_us() + 5000000;
    while (player.n.load() < N && monotonic_us() < deadline) usleep(2000);
    EXPECT_EQ(player.n.load(), N);
    EXPECT_GE(client.acks_sent(), 1);  // 6 MB over a 2.5 MB window
    pub.Destroy();
    player.Destroy();
}

// ------------------------------------------------------------ media payloads

namespace {
// MSB-first bit writer with exp-Golomb codes (builds SPS test vectors)
struct BitWriter {
    std::string out;
    uint32_t acc = 0;
    int n = 0;
    void bit(uint32_t b) {
        acc = (acc << 1) | (b & 1);
        if (++n == 8) {
            out.push_back((char)acc);
            acc = 0;
            n = 0;
        }
    }
    void bits(uint32_t v, int k) {
        for (int i = k - 1; i >= 0; --i) bit((v >> i) & 1);
    }
    void ue(uint32_t v) {
        const uint32_t x = v + 1;
        int len = 0;
        while ((x >> len) > 1) ++len;
        bits(0, len);
        bits(x, len + 1);
    }
    void se(int32_t v) { ue(v > 0 ? 2 * v - 1 : -2 * v); }
    std::string finish() {  // rbsp_stop_one_bit + alignment
        bit(1);
        while (n) bit(0);
        return out;
    }
};

// A high-profile SPS for w x h (crop to the exact size) in escaped form.
std::string make_sps(int w, int h, bool high) {
    BitWriter bw;
    bw.bits(high ? 100 : 66, 8);  // profile_idc
    bw.bits(0, 8);
    bw.bits(40, 8);  // level 4.0
    bw.ue(0);        // sps id
    if (high) {
        bw.ue(1);   // 4:2:0
        bw.ue(0);   // bit depth luma - 8
        bw.ue(0);   // chroma
        bw.bit(0);  // qpprime
        bw.bit(1);  // scaling matrix present
        for (int i = 0; i < 8; ++i) {
            bw.bit(i == 0 ? 1 : 0);
            if (i == 0)
                for (int j = 0; j < 16; ++j) bw.se(j == 0 ? 8 : 0);  // one flat delta list
        }
    }
    bw.ue(0);  // log2_max_frame_num - 4
    bw.ue(0);  // poc type 0
    bw.ue(2);  // log2_max_poc_lsb - 4
    bw.ue(4);  // max_num_ref_frames
    bw.bit(0);
    const int wm = (w + 15) / 16, hm = (h + 15) / 16;
    bw.ue(wm - 1);
    bw.ue(hm - 1);
    bw.bit(1);  // frame_mbs_only
    bw.bit(1);  // direct_8x8
    const int cr = wm * 16 - w, cb = hm * 16 - h;
    bw.bit(cr || cb ? 1 : 0);
    if (cr || cb) {
        bw.ue(0);
        bw.ue(cr / 2);
        bw.ue(0);
        bw.ue(cb / 2);
    }
    bw.bit(0);  // vui
    const std::string rbsp = bw.finish();
    // escape 00 00 0x (x <= 3) -> 00 00 03 0x
    std::string nalu(1, (char)0x67);
    int zeros = 0;
    for (char c : rbsp) {
        if (zeros >= 2 && (uint8_t)c <= 3) {
            nalu.push_back(3);
            zeros = 0;
        }
        zeros = c == 0 ? zeros + 1 : 0;
        nalu.push_back(c);
    }
    return nalu;
}
}  // namespace

TEST(RtmpMedia, aac_config_and_adts) {
    AudioSpecificConfig asc;
    const uint8_t lc_44k_stereo[2] = {0x12, 0x10};  // object 2, index 4, 2 channels
    ASSERT_EQ(asc.Create(lc_44k_stereo, 2), 0);
    EXPECT_EQ((int)asc.aac_object, 2);
    EXPECT_EQ(asc.sample_rate, 44100u);
    EXPECT_EQ((int)asc.channels, 2);
    EXPECT_EQ(asc.Serialize(), std::string("\x12\x10", 2));
    uint8_t h[7];
    ASSERT_EQ(asc.MakeAdtsHeader(100, h), 0);
    EXPECT_EQ((int)h[0], 0xff);
    EXPECT_EQ((int)h[1], 0xf1);
    EXPECT_EQ((int)(h[2] >> 6), 1);          // profile = object - 1
    EXPECT_EQ((int)((h[2] >> 2) & 0xf), 4);  // 44.1 kHz
    const int frame = ((h[3] & 3) << 11) | (h[4] << 3) | (h[5] >> 5);
    EXPECT_EQ(frame, 107);
    // explicit sampling rate (index 15) round trips through 24 bits
    AudioSpecificConfig odd;
    odd.aac_object = 2;
    odd.sample_rate = 12345;
    odd.sample_rate_index = 15;
    odd.channels = 1;
    const std::string s = odd.Serialize();
    AudioSpecificConfig back;
    ASSERT_EQ(back.Create(s.data(), s.size()), 0);
    EXPECT_EQ(back.sample_rate, 12345u);
    EXPECT_EQ((int)back.channels, 1);
    EXPECT_NE(back.MakeAdtsHeader(10, h), 0);  // ADTS cannot carry an explicit rate
    EXPECT_NE(asc.Create(lc_44k_stereo, 1), 0);  // truncated

    RtmpAACMessage aac;
    aac.timestamp = 33;
    aac.packet_type = AAC_PACKET_SEQUENCE_HEADER;
    aac.data.append(asc.Serialize());
    RtmpAudioMessage am;
    aac.ToAudioMessage(&am);
    EXPECT_EQ((int)am.codec, 10);
    RtmpAACMessage aac2;
    ASSERT_EQ(aac2.Create(am), 0);
    EXPECT_EQ((int)aac2.packet_type, (int)AAC_PACKET_SEQUENCE_HEADER);
    EXPECT_EQ(aac2.data.to_string(), asc.Serialize());
    am.codec = 2;  // MP3
    EXPECT_NE(aac2.Create(am), 0);
}

TEST(RtmpMedia, sps_dimensions) {
    struct Case {
        int w, h;
        bool high;
    } cases[] = {{1920, 1080, true}, {1280, 720, false}, {640, 360, true}, {176, 144, false}};
    for (const Case& c : cases) {
        AvcSps sps;
        ASSERT_EQ(sps.Parse(make_sps(c.w, c.h, c.high)), 0);
        EXPECT_EQ(sps.width, c.w);
        EXPECT_EQ(sps.height, c.h);
        EXPECT_EQ((int)sps.profile_idc, c.high ? 100 : 66);
        EXPECT_EQ((int)sps.max_num_ref_frames, 4);
    }
    AvcSps bad;
    EXPECT_NE(bad.Parse(std::string("\x67\x64", 2)), 0);     // truncated
    EXPECT_NE(bad.Parse(std::string("\x68\x64\x00\x28", 4)), 0);  // a PPS
    EXPECT_EQ(AvcUnescapeRbsp("\x00\x00\x03\x01\x00\x00\x03", 7), std::string("\x00\x00\x01\x00\x00", 5));
}

TEST(RtmpMedia, avc_config_record_and_nalus) {
    AVCDecoderConfigurationRecord rec;
    rec.avc_profile = 100;
    rec.avc_level = 40;
    rec.length_size_minus1 = 3;
    rec.sps_list.push_back(make_sps(1920, 1080, true));
    rec.pps_list.push_back(std::string("\x68\xee\x3c\x80", 4));
    const std::string bytes = rec.Serialize();
    AVCDecoderConfigurationRecord back;
    ASSERT_EQ(back.Create(bytes.data(), bytes.size()), 0);
    EXPECT_EQ(back.width, 1920);
    EXPECT_EQ(back.height, 1080);
    ASSERT_EQ(back.sps_list.size(), 1u);
    ASSERT_EQ(back.pps_list.size(), 1u);
    EXPECT_EQ(back.pps_list[0], rec.pps_list[0]);
    EXPECT_EQ(back.Serialize(), bytes);
    EXPECT_NE(back.Create(bytes.data(), bytes.size() - 2), 0);  // PPS cut short

    // the record rides in an AVC sequence-header message; composition time is SI24
    RtmpAVCMessage m;
    m.timestamp = 1000;
    m.frame_type = 1;
    m.packet_type = AVC_PACKET_NALU;
    m.composition_time = -40;
    const std::string idr("\x65\x88\x84\x00\x33", 5), sei("\x06\x05\x01\xff", 4);
    auto put32 = [](Buf* b, uint32_t v) {
        const char x[4] = {(char)(v >> 24), (char)(v >> 16), (char)(v >> 8), (char)v};
        b->append(x, 4);
    };
    put32(&m.data, (uint32_t)sei.size());
    m.data.append(sei);
    put32(&m.data, (uint32_t)idr.size());
    m.data.append(idr);
    RtmpVideoMessage vm;
    m.ToVideoMessage(&vm);
    RtmpAVCMessage m2;
    ASSERT_EQ(m2.Create(vm), 0);
    EXPECT_EQ(m2.composition_time, -40);
    EXPECT_EQ((int)m2.packet_type, (int)AVC_PACKET_NALU);

    AVCNaluFormat fmt = AVC_NALU_FORMAT_UNKNOWN;
    AVCNaluIterator it(&m2.data, back.length_size_minus1 + 1, &fmt);
    std::string nalu;
    AVCNaluType t;
    ASSERT_TRUE(it.Next(&nalu, &t));
    EXPECT_EQ((int)fmt, (int)AVC_NALU_FORMAT_IBMF);
    EXPECT_EQ((int)t, (int)AVC_NALU_SEI);
    ASSERT_TRUE(it.Next(&nalu, &t));
    EXPECT_EQ((int)t, (int)AVC_NALU_IDR);
    EXPECT_EQ(nalu, idr);
    EXPECT_FALSE(it.Next(&nalu));
    EXPECT_FALSE(it.error());

    // Annex B: 4- and 3-byte start codes, trailing zero bytes
    Buf annexb;
    annexb.append(std::string("\x00\x00\x00\x01", 4) + rec.sps_list[0] + std::string("\x00\x00\x01", 3) +
                  rec.pps_list[0] + std::string("\x00\x00\x00\x01", 4) + idr + std::string("\x00\x00", 2));
    AVCNaluFormat f2 = AVC_NALU_FORMAT_UNKNOWN;
    AVCNaluIterator it2(&annexb, 4, &f2);
    std::vector<int> types;
    while (it2.Next(&nalu, &t)) types.push_back((int)t);
    EXPECT_EQ((int)f2, (int)AVC_NALU_FORMAT_ANNEXB);
    EXPECT_FALSE(it2.error());
    ASSERT_EQ(types.size(), 3u);
    EXPECT_EQ(types[0], (int)AVC_NALU_SPS);
    EXPECT_EQ(types[1], (int)AVC_NALU_PPS);
    EXPECT_EQ(types[2], (int)AVC_NALU_IDR);
    EXPECT_EQ(nalu, idr);

    // a length prefix running past the packet is a framing error
    Buf broken;
    put32(&broken, 100);
    broken.append("\x65\x01", 2);
    AVCNaluFormat f3 = AVC_NALU_FORMAT_IBMF;
    AVCNaluIterator it3(&broken, 4, &f3);
    EXPECT_FALSE(it3.Next(&nalu));
    EXPECT_TRUE(it3.error());
}

namespace {
class CueSink : public RtmpServerStream {
public:
    explicit CueSink(std::atomic<int>* n, std::string* last) : _n(n), _last(last) {}
    void OnCuePoint(RtmpCuePoint* cp) override {
        const AMFValue* name = cp->data.Find("name");
        *_last = (name ? name->str() : "") + "@" + std::to_string(cp->timestamp);
        _n->fetch_add(1);
    }
    void OnVideoMessage(RtmpVideoMessage* m) override {
        RtmpAVCMessage avc;
        if (avc.Create(*m) == 0 && avc.composition_time == 80) _n->fetch_add(100);
    }

private:
    std::atomic<int>* _n;
    std::string* _last;
};

class CueService : public RtmpService {
public:
    std::atomic<int> n{0}, streams{0};
    std::string last;
    RtmpServerStream* NewStream(const RtmpConnectRequest&) override {
        streams.fetch_add(1);
        return new CueSink(&n, &last);
    }
};

class FixedCreator : public RtmpSubStreamCreator {
public:
    explicit FixedCreator(std::string addr) : _addr(std::move(addr)) {}
    std::shared_ptr<RtmpClient> NewClient() override {
        auto c = std::make_shared<RtmpClient>();
        RtmpClientOptions o;
        o.timeout_ms = 2000;
        if (c->Init(_addr.c_str(), o) != 0) return nullptr;
        std::lock_guard<std::mutex> g(mu);
        last = c;
        return c;
    }
    std::mutex mu;
    std::shared_ptr<RtmpClient> last;

private:
    std::string _addr;
};
}  // namespace

TEST(RtmpMedia, cue_points_and_retrying_publisher) {
    CueService svc;
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    o.rtmp_service = &svc;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());

    FixedCreator* creator = new FixedCreator(addr);
    RtmpRetryingClientStream pub;
    RtmpRetryingClientStreamOptions ro;
    ro.publish_name = "cues";
    ro.retry_interval_ms = 50;
    ro.fast_retry_count = 1;
    ASSERT_EQ(pub.Init(creator, ro), 0);
    EXPECT_TRUE(pub.connected());
    RtmpCuePoint cp;
    cp.timestamp = 777;
    cp.data.Set("name", AMFValue::String("ad-break"));
    cp.data.Set("time", AMFValue::Number(7.77));
    ASSERT_EQ(pub.SendCuePoint(cp), 0);
    RtmpAVCMessage avc;
    avc.composition_time = 80;
    avc.data.append("\x00\x00\x00\x01\x65", 5);
    ASSERT_EQ(pub.SendAVCMessage(avc), 0);
    int64_t deadline = monotonic_us() + 3000000;
    while (svc.n.load() < 101 && monotonic_us() < deadline) usleep(2000);
    EXPECT_EQ(svc.n.load(), 101);
    EXPECT_EQ(svc.last, "ad-break@777");

    // kill the publisher's connection: the stream comes back on a new one
    {
        std::lock_guard<std::mutex> g(creator->mu);
        SocketUniquePtr s;
        ASSERT_EQ(Socket::Address(creator->last->socket_id(), &s), 0);
        s->SetFailed(ECONNRESET, "test kills the publisher connection");
    }
    deadline = monotonic_us() + 5000000;
    while (pub.reconnects() < 1 && monotonic_us() < deadline) usleep(5000);
    ASSERT_EQ(pub.reconnects(), 1);
    deadline = monotonic_us() + 2000000;
    while (!pub.connected() && monotonic_us() < deadline) usleep(2000);
    cp.timestamp = 888;
    ASSERT_EQ(pub.SendCuePoint(cp), 0);
    deadline = monotonic_us() + 3000000;
    while (svc.n.load() < 102 && monotonic_us() < deadline) usleep(2000);
    EXPECT_EQ(svc.n.load(), 102);
    EXPECT_EQ(svc.last, "ad-break@888");
    EXPECT_GE(svc.streams.load(), 2);
    pub.Destroy();
    EXPECT_FALSE(pub.connected());
    EXPECT_NE(pub.SendCuePoint(cp), 0);
}

namespace {
// A VOD-like server stream: seeks within [0, 60000] ms, pauses, records
// play2 / buffer length; the client sees every verdict as onStatus/_error.
class VodStream : public RtmpServerStream {
public:
    std::mutex mu;
    std::vector<std::string> log;
    void OnPlay(const RtmpPlayOptions& opt, std::string* error) override { add("play:" + opt.stream_name); }
    void OnPlay2(const RtmpPlay2Options& o) override {
        add("play2:" + o.stream_name + ":" + o.old_stream_name + ":" + o.transition + ":" +
            std::to_string((int)o.offset) + (std::isnan(o.len) ? ":nolen" : ":len"));
    }
    int OnSeek(double ms) override {
        add("seek:" + std::to_string((int)ms));
        return ms >= 0 && ms <= 60000 ? 0 : -1;
    }
    int OnPause(bool pause, double ms) override {
        add(std::string(pause ? "pause:" : "unpause:") + std::to_string((int)ms));
        return 0;
    }
    void OnSetBufferLength(uint32_t ms) override { add("buffer:" + std::to_string(ms)); }
    void add(const std::string& s) {
        std::lock_guard<std::mutex> g(mu);
        log.push_back(s);
    }
    size_t size() {
        std::lock_guard<std::mutex> g(mu);
        return log.size();
    }
};
class VodService : public RtmpService {
public:
    std::atomic<VodStream*> last{nullptr};
    RtmpServerStream* NewStream(const RtmpConnectRequest&) override {
        VodStream* s = new VodStream;
        last.store(s);
        return s;
    }
};
class VodPlayer : public RtmpClientStream {
public:
    std::mutex mu;
    std::vector<std::string> statuses;
    std::atomic<int> first{0}, media{0};
    void OnStatus(const std::string& level, const std::string& code, const std::string& desc) override {
        std::lock_guard<std::mutex> g(mu);
        statuses.push_back(level + ":" + code + ":" + desc);
    }
    void OnFirstMessage() override {
        EXPECT_EQ(media.load(), 0);  // before any media callback
        first.fetch_add(1);
    }
    void OnVideoMessage(RtmpVideoMessage*) override { media.fetch_add(1); }
    size_t nstatus() {
        std::lock_guard<std::mutex> g(mu);
        return statuses.size();
    }
};
template <typename F>
bool wait_until(F f, int ms = 3000) {
    const int64_t deadline = monotonic_us() + (int64_t)ms * 1000;
    while (!f() && monotonic_us() < deadline) usleep(1000);
    return f();
}
}  // namespace

// Reference: rtmp.h:814-819 (Play2/Seek/Pause), :1096-1112 (OnPlay2/OnSeek/
// OnPause/OnSetBufferLength, SendStopMessage, SendStreamDry), :564-568.
TEST(Rtmp, play2_seek_pause_and_stop) {
    VodService svc;
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    o.rtmp_service = &svc;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    RtmpClient client;
    RtmpClientOptions copt;
    copt.app = "vod";
    copt.timeout_ms = 3000;
    ASSERT_EQ(client.Init(addr.c_str(), copt), 0);
    VodPlayer player;
    RtmpClientStreamOptions po;
    po.play_name = "movie";
    po.buffer_length_ms = 2500;
    ASSERT_EQ(player.Init(&client, po), 0);
    EXPECT_EQ(player.rtmp_url(), "rtmp://" + addr + "/vod/movie");
    VodStream* vs = svc.last.load();
    ASSERT_TRUE(vs != nullptr);
    ASSERT_TRUE(wait_until([&] { return vs->size() >= 2; }));

    RtmpPlay2Options p2;
    p2.stream_name = "movie_720p";
    p2.old_stream_name = "movie";
    p2.transition = "switch";
    p2.offset = 1500;
    ASSERT_EQ(player.Play2(p2), 0);
    ASSERT_EQ(player.Seek(30000), 0);
    ASSERT_TRUE(wait_until([&] { return player.nstatus() >= 1; }));
    EXPECT_EQ(player.last_status(), "NetStream.Seek.Notify");
    ASSERT_EQ(player.Seek(90000), 0);  // out of range: rejected with _error
    ASSERT_TRUE(wait_until([&] { return player.nstatus() >= 2; }));
    ASSERT_EQ(player.Pause(true, 31000), 0);
    ASSERT_TRUE(wait_until([&] { return player.nstatus() >= 3; }));
    EXPECT_TRUE(vs->paused());
    ASSERT_EQ(player.Pause(true, 31000), 0);  // already paused: _error, OnPause not called
    ASSERT_TRUE(wait_until([&] { return player.nstatus() >= 4; }));
    ASSERT_EQ(player.Pause(false, 31000), 0);
    ASSERT_TRUE(wait_until([&] { return player.nstatus() >= 5; }));
    EXPECT_FALSE(vs->paused());
    {
        std::lock_guard<std::mutex> g(player.mu);
        EXPECT_EQ(player.statuses[0], "status:NetStream.Seek.Notify:Seek successfully.");
        EXPECT_EQ(player.statuses[1], "error:NetStream.Seek.Notify:Fail to seek");
        EXPECT_EQ(player.statuses[2], "status:NetStream.Pause.Notify:Paused stream.");
        EXPECT_EQ(player.statuses[3], "error:NetStream.Pause.Notify:Stream is already paused");
        EXPECT_EQ(player.statuses[4], "status:NetStream.Unpause.Notify:Unpaused stream.");
    }
    {
        std::lock_guard<std::mutex> g(vs->mu);
        const std::vector<std::string> want = {"play:movie",  "buffer:2500", "play2:movie_720p:movie:switch:1500:nolen",
                                               "seek:30000",  "seek:90000",  "pause:31000",
                                               "unpause:31000"};
        std::string got_all, want_all;
        for (const std::string& x : vs->log) got_all += x + ";";
        for (const std::string& x : want) want_all += x + ";";
        EXPECT_EQ(got_all, want_all);
    }
    // media: OnFirstMessage once, before the first callback
    RtmpVideoMessage vm;
    vm.data.append("frame");
    ASSERT_EQ(vs->SendVideoMessage(vm), 0);
    ASSERT_EQ(vs->SendVideoMessage(vm), 0);
    ASSERT_TRUE(wait_until([&] { return player.media.load() == 2; }));
    EXPECT_EQ(player.first.load(), 1);
    // StreamDry is accepted silently; SendStopMessage reaches the player
    EXPECT_EQ(vs->SendStreamDry(), 0);
    EXPECT_EQ(vs->SendStopMessage("gone away"), 0);
    ASSERT_TRUE(wait_until([&] { return player.nstatus() >= 6; }));
    EXPECT_EQ(player.last_status(), "NetStream.Play.StreamNotFound");
    // the base stream class has no user message and no stop message
    int dummy = 0;
    EXPECT_EQ(player.SendUserMessage(&dummy), -1);
    EXPECT_EQ(errno, ENOTSUP);
    EXPECT_EQ(player.SendStopMessage("x"), -1);
    player.Destroy();
    EXPECT_EQ(player.Seek(1), -1);  // not attached any more
}
