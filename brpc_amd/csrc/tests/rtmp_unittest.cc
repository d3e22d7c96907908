// RTMP (spirit of the reference's test/brpc_rtmp_unittest.cpp): AMF0 round
// trips, FLV writer/reader, and a live relay over loopback — one client
// publishes metadata/audio/video, two players receive them in order.
#include <unistd.h>

#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "base/time.h"
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
