// RDMA transport tests (spirit of the reference's test/brpc_rdma_unittest.cpp):
// the hello codec and malformed hellos, the soft verbs provider on its own
// (SEND_WITH_IMM, RNR hold-back, length errors, unregistered memory), then
// baidu_std echo over RDMA end to end — small calls, multi-MiB attachments
// that exhaust and refill the credit window, concurrent callers, 64 KiB
// receive blocks, unregistered user memory (bounce copy) vs registered user
// memory (zero copy), plain TCP clients on an RDMA port, and an RDMA client
// against a server without RDMA.
#include <dlfcn.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "mrpc/proto/echo.pb.h"
#include "net/socket.h"
#include "rdma/rdma.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

DECLARE_string(rdma_provider);
DECLARE_string(rdma_recv_block_type);

using namespace mrpc;

namespace {

void InitSoft() {
    FLAGS_rdma_provider = "auto";  // no HCA here: falls back to soft
    std::string err;
    int rc = rdma::GlobalRdmaInitialize(&err);
    if (rc != 0) fprintf(stderr, "rdma init: %s\n", err.c_str());
}

struct RdmaServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    explicit RdmaServer(bool rdma = true) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.use_rdma = rdma;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
    int RdmaConnections() {
        std::vector<SocketId> conns;
        server.acceptor()->ListConnections(&conns);
        int n = 0;
        for (SocketId id : conns) {
            SocketUniquePtr p;
            if (Socket::Address(id, &p) == 0 && p->is_rdma()) ++n;
        }
        return n;
    }
};

std::string Pattern(size_t n, int seed) {
    std::string s(n, '\0');
    for (size_t i = 0; i < n; ++i) s[i] = (char)(i * 131 + seed * 7 + (i >> 9));
    return s;
}

bool EchoOnce(example::EchoService_Stub& stub, const std::string& msg, const Buf& att, std::string* why = nullptr) {
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(msg);
    cntl.request_attachment() = att;
    stub.Echo(&cntl, &req, &res, nullptr);
    if (cntl.Failed()) {
        if (why) *why = cntl.ErrorText();
        return false;
    }
    if (res.message() != msg) {
        if (why) *why = "message mismatch";
        return false;
    }
    if (cntl.response_attachment().to_string() != att.to_string()) {
        if (why) *why = "attachment mismatch";
        return false;
    }
    return true;
}

}  // namespace

TEST(Rdma, hello_codec) {
    rdma::Hello h;
    h.sq_size = 128;
    h.rq_size = 64;
    h.flags = 1;
    h.block_size = 8128;
    h.addr.gid_hi = 0xfe80000000000000ull;
    h.addr.gid_lo = 0x0123456789abcdefull;
    h.addr.qpn = 0x11223;
    h.addr.lid = 7;
    char buf[rdma::Hello::kSize];
    h.Serialize(buf);
    EXPECT_EQ(memcmp(buf, "RDMA", 4), 0);
    rdma::Hello g;
    ASSERT_TRUE(g.Parse(buf));
    EXPECT_EQ(g.sq_size, 128);
    EXPECT_EQ(g.rq_size, 64);
    EXPECT_EQ(g.flags, 1);
    EXPECT_EQ(g.block_size, 8128u);
    EXPECT_EQ(g.addr.gid_lo, h.addr.gid_lo);
    EXPECT_EQ(g.addr.qpn, 0x11223u);
    EXPECT_EQ(g.addr.lid, 7);
    char bad[rdma::Hello::kSize];
    memcpy(bad, buf, sizeof(bad));
    bad[0] = 'X';
    EXPECT_FALSE(g.Parse(bad));  // magic
    memcpy(bad, buf, sizeof(bad));
    bad[5] = 9;
    EXPECT_FALSE(g.Parse(bad));  // version
    memcpy(bad, buf, sizeof(bad));
    bad[8] = 0;
    bad[9] = 2;
    EXPECT_FALSE(g.Parse(bad));  // rq too small for the ACK reserve
}

TEST(Rdma, soft_provider_send_recv_imm_and_rnr) {
    std::unique_ptr<rdma::Provider> pr = rdma::CreateSoftProvider();
    std::vector<char> a(1 << 16), b(1 << 16);
    uint32_t la = 0, lb = 0;
    ASSERT_EQ(pr->RegisterMemory(a.data(), a.size(), false, -1, &la), 0);
    ASSERT_EQ(pr->RegisterMemory(b.data(), b.size(), false, -1, &lb), 0);
    auto cq1 = pr->CreateCq(64);
    auto cq2 = pr->CreateCq(64);
    auto q1 = pr->CreateQp(cq1.get(), 16, 16);
    auto q2 = pr->CreateQp(cq2.get(), 16, 16);
    ASSERT_EQ(q1->Connect(q2->local()), 0);
    ASSERT_EQ(q2->Connect(q1->local()), 0);
    rdma::QpAddress bogus = q2->local();
    bogus.gid_lo ^= 1;
    EXPECT_EQ(q1->Connect(bogus), -1);  // another "host"
    ASSERT_EQ(q1->Connect(q2->local()), 0);
    // send before any receive is posted: held back like RNR retry
    memcpy(a.data(), "hello rdma", 10);
    rdma::Sge s1{(uint64_t)(uintptr_t)a.data(), 5, la};
    rdma::Sge s2{(uint64_t)(uintptr_t)(a.data() + 5), 5, la};
    rdma::Sge sg[2] = {s1, s2};
    ASSERT_EQ(q1->PostSend(42, sg, 2, true, 17, true), 0);
    rdma::WorkCompletion wc[4];
    EXPECT_EQ(cq1->Poll(wc, 4), 0);
    EXPECT_EQ(cq2->Poll(wc, 4), 0);
    // arming makes the notify fd readable on the next completion
    ASSERT_EQ(cq2->Arm(), 0);
    rdma::Sge r{(uint64_t)(uintptr_t)b.data(), 4096, lb};
    ASSERT_EQ(q2->PostRecv(7, r), 0);
    char v[8];
    EXPECT_EQ(::read(cq2->notify_fd(), v, 8), 8);
    ASSERT_EQ(cq2->Poll(wc, 4), 1);
    EXPECT_EQ(wc[0].wr_id, 7u);
    EXPECT_EQ(wc[0].opcode, (int)rdma::WC_RECV);
    EXPECT_EQ(wc[0].byte_len, 10u);
    EXPECT_TRUE(wc[0].has_imm);
    EXPECT_EQ(wc[0].imm, 17u);
    EXPECT_EQ(memcmp(b.data(), "hello rdma", 10), 0);
    ASSERT_EQ(cq1->Poll(wc, 4), 1);
    EXPECT_EQ(wc[0].wr_id, 42u);
    EXPECT_EQ(wc[0].opcode, (int)rdma::WC_SEND);
    // unsignaled sends produce no send completion
    ASSERT_EQ(q2->PostRecv(8, r), 0);
    ASSERT_EQ(q1->PostSend(43, sg, 1, false, 0, false), 0);
    ASSERT_EQ(cq2->Poll(wc, 4), 1);
    EXPECT_FALSE(wc[0].has_imm);
    EXPECT_EQ(cq1->Poll(wc, 4), 0);
    // message longer than the receive buffer: error completions both sides
    rdma::Sge small{(uint64_t)(uintptr_t)b.data(), 4, lb};
    ASSERT_EQ(q2->PostRecv(9, small), 0);
    ASSERT_EQ(q1->PostSend(44, sg, 2, false, 0, false), 0);
    ASSERT_EQ(cq2->Poll(wc, 4), 1);
    EXPECT_NE(wc[0].status, 0);
    ASSERT_EQ(cq1->Poll(wc, 4), 1);
    EXPECT_NE(wc[0].status, 0);
    // unregistered memory is refused
    char stack_buf[16];
    rdma::Sge unreg{(uint64_t)(uintptr_t)stack_buf, 16, la};
    EXPECT_EQ(q1->PostSend(45, &unreg, 1, false, 0, true), -1);
    q1.reset();
    q2.reset();
    pr->DeregisterMemory(a.data());
    pr->DeregisterMemory(b.data());
}

TEST(Rdma, echo_small_and_pool_swap) {
    InitSoft();
    ASSERT_TRUE(rdma::RdmaAvailable());
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 5000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < 300; ++i) {
        std::string why;
        Buf att;
        if (i % 3 == 0) att.append(Pattern(100 + i, i));
        ASSERT_TRUE(EchoOnce(stub, "rdma-" + std::to_string(i), att, &why));
    }
    EXPECT_EQ(s.RdmaConnections(), 1);
    // the client socket moved onto verbs as well
    SocketUniquePtr cs;
    ASSERT_EQ(Socket::Address(ch.server_id(), &cs), 0);
    EXPECT_TRUE(cs->is_rdma());
    ASSERT_TRUE(cs->rdma_endpoint() != nullptr);
    rdma::EndpointStats st = cs->rdma_endpoint()->stats();
    EXPECT_GE(st.sent_msgs, 300);
    EXPECT_GE(st.recv_msgs, 300);
    rdma::PoolStats ps = rdma::GetPoolStats();
    EXPECT_GE(ps.regions, 1);
    EXPECT_GT(ps.blocks_8k, 0);
    EXPECT_TRUE(rdma::DescribeRdma().find("provider: soft") != std::string::npos);
    EXPECT_TRUE(cs->description().find("rdma{") != std::string::npos);
}

TEST(Rdma, large_attachments_exhaust_and_refill_window) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 10000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    // 3 MiB = ~390 receive blocks of 8 KiB: three times the 128-deep ring
    for (int i = 0; i < 6; ++i) {
        Buf att;
        att.append(Pattern((3 << 20) + i * 977, i));
        std::string why;
        ASSERT_TRUE(EchoOnce(stub, "big", att, &why));
    }
    SocketUniquePtr cs;
    ASSERT_EQ(Socket::Address(ch.server_id(), &cs), 0);
    rdma::EndpointStats st = cs->rdma_endpoint()->stats();
    EXPECT_GT(st.window_full, 0);  // the writer really waited for credits
    EXPECT_GT(st.sent_bytes, 6ll * (3 << 20));
}

TEST(Rdma, concurrent_callers) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 10000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    std::atomic<int> ok{0}, bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t) {
        th.emplace_back([&, t] {
            example::EchoService_Stub stub(&ch);
            for (int i = 0; i < 40; ++i) {
                Buf att;
                att.append(Pattern((size_t)(i % 4) * 20000 + 64, t * 100 + i));
                std::string why;
                if (EchoOnce(stub, "c" + std::to_string(t) + "-" + std::to_string(i), att, &why)) {
                    ++ok;
                } else {
                    fprintf(stderr, "call failed: %s\n", why.c_str());
                    ++bad;
                }
            }
        });
    }
    for (auto& x : th) x.join();
    EXPECT_EQ(ok.load(), 320);
    EXPECT_EQ(bad.load(), 0);
}

TEST(Rdma, large_receive_blocks) {
    InitSoft();
    const std::string saved = FLAGS_rdma_recv_block_type;
    FLAGS_rdma_recv_block_type = "large";  // 64 KiB receive blocks on both sides
    {
        RdmaServer s;
        ASSERT_GT(s.port, 0);
        Channel ch;
        ChannelOptions opt;
        opt.use_rdma = true;
        opt.timeout_ms = 10000;
        opt.connection_group = "large-blocks";
        ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
        example::EchoService_Stub stub(&ch);
        for (int i = 0; i < 5; ++i) {
            Buf att;
            att.append(Pattern(1 << 20, i));
            std::string why;
            ASSERT_TRUE(EchoOnce(stub, "L", att, &why));
        }
        SocketUniquePtr cs;
        ASSERT_EQ(Socket::Address(ch.server_id(), &cs), 0);
        rdma::EndpointStats st = cs->rdma_endpoint()->stats();
        // ~1 MiB per call in ~64 KiB messages, not 8 KiB ones
        EXPECT_LT(st.sent_msgs, 5 * 40);
        EXPECT_GT(rdma::GetPoolStats().blocks_64k, 0);
    }
    FLAGS_rdma_recv_block_type = saved;
}

TEST(Rdma, user_memory_bounce_vs_registered) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 5000;
    opt.connection_group = "user-mem";
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    ASSERT_TRUE(EchoOnce(stub, "warm", Buf()));
    SocketUniquePtr cs;
    ASSERT_EQ(Socket::Address(ch.server_id(), &cs), 0);
    rdma::Endpoint* ep = cs->rdma_endpoint();
    ASSERT_TRUE(ep != nullptr);
    const size_t n = 6000;
    char* unreg = static_cast<char*>(malloc(n));
    std::string pat = Pattern(n, 3);
    memcpy(unreg, pat.data(), n);
    const int64_t b0 = ep->stats().bounce_copies;
    {
        Buf att;
        att.append_user_data(unreg, n, [](void* d, void*) { free(d); });
        ASSERT_TRUE(EchoOnce(stub, "unreg", att));
    }
    const int64_t b1 = ep->stats().bounce_copies;
    EXPECT_GT(b1, b0);  // copied into a registered block
    static char reg_mem[1 << 16];
    memcpy(reg_mem, pat.data(), n);
    ASSERT_EQ(rdma::RegisterMemoryForRdma(reg_mem, sizeof(reg_mem)), 0);
    uint32_t lkey;
    EXPECT_TRUE(rdma::LookupLkey(reg_mem + 100, 1000, &lkey));
    EXPECT_FALSE(rdma::LookupLkey(reg_mem + sizeof(reg_mem) - 10, 100, &lkey));
    {
        Buf att;
        att.append_user_data(reg_mem, n, [](void*, void*) {});
        ASSERT_TRUE(EchoOnce(stub, "reg", att));
    }
    // request went out zero-copy (the response came back into pool blocks)
    EXPECT_EQ(ep->stats().bounce_copies, b1);
    rdma::DeregisterMemoryForRdma(reg_mem);
    EXPECT_FALSE(rdma::LookupLkey(reg_mem + 100, 1000, &lkey));
}

TEST(Rdma, tcp_client_on_rdma_port_and_rdma_client_on_tcp_server) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    {
        Channel ch;  // plain TCP client, same port
        ChannelOptions opt;
        opt.timeout_ms = 5000;
        ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
        example::EchoService_Stub stub(&ch);
        Buf att;
        att.append(Pattern(50000, 1));
        ASSERT_TRUE(EchoOnce(stub, "tcp", att));
        EXPECT_EQ(s.RdmaConnections(), 0);
    }
    RdmaServer plain(false);
    ASSERT_GT(plain.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 2000;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(plain.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    std::string why;
    EXPECT_FALSE(EchoOnce(stub, "x", Buf(), &why));
}

TEST(Rdma, server_stop_fails_rdma_calls_cleanly) {
    InitSoft();
    std::unique_ptr<RdmaServer> s(new RdmaServer);
    ASSERT_GT(s->port, 0);
    const std::string addr = s->addr();
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 2000;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(addr.c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    ASSERT_TRUE(EchoOnce(stub, "before", Buf()));
    s->server.Stop(0);
    s->server.Join();
    s.reset();
    usleep(200000);
    std::string why;
    EXPECT_FALSE(EchoOnce(stub, "after", Buf(), &why));
}

// ------------------------------------------------------------------------
// The ibverbs provider, compiled against rdma/verbs_abi.h and driven through
// a stub verbs library (tests/stub/fake_ibverbs.cc) that it dlopen()s
// exactly as it would libibverbs.so.1. Own suite: it selects the provider
// process-wide.

DECLARE_string(rdma_verbs_library);

namespace {

struct FakeIbvStats {
    long sends, recvs, bytes, rnr_holds, errors, dmabuf_regs, events;
    int open_contexts, live_pds, live_cqs, live_qps, live_channels, live_mrs;
};

std::string StubPath() {
    char self[4096];
    const ssize_t n = readlink("/proc/self/exe", self, sizeof(self) - 1);
    if (n <= 0) return "";
    self[n] = 0;
    std::string dir(self);
    dir = dir.substr(0, dir.rfind('/'));
    return dir + "/../lib/libfake_ibverbs.so";
}

FakeIbvStats StubStats() {
    FakeIbvStats s;
    memset(&s, 0, sizeof(s));
    void* h = dlopen(StubPath().c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!h) return s;
    auto fn = reinterpret_cast<void (*)(FakeIbvStats*)>(dlsym(h, "fake_ibv_stats"));
    if (fn) fn(&s);
    dlclose(h);
    return s;
}

int FakeDmabufExport(void* p, size_t n, int gpu, int* fd, uint64_t* off) {
    (void)p;
    (void)n;
    (void)gpu;
    *fd = memfd_create("fake_dmabuf", MFD_CLOEXEC);
    *off = 0;
    return *fd >= 0 ? 0 : -1;
}

}  // namespace

TEST(RdmaVerbs, missing_library_reports_why) {
    FLAGS_rdma_verbs_library = "/nonexistent/libibverbs.so.1";
    std::string why;
    EXPECT_TRUE(rdma::IbverbsCompiledIn());
    EXPECT_TRUE(rdma::CreateIbverbsProvider(&why) == nullptr);
    EXPECT_TRUE(why.find("not loadable") != std::string::npos);
}

TEST(RdmaVerbs, provider_queue_pairs_over_stub_library) {
    FLAGS_rdma_verbs_library = StubPath();
    std::string why;
    std::unique_ptr<rdma::Provider> pr = rdma::CreateIbverbsProvider(&why);
    ASSERT_TRUE(pr != nullptr);
    EXPECT_EQ(std::string(pr->name()), "ibverbs");
    EXPECT_EQ(pr->device_name(), "fake_mlx5_0");
    const FakeIbvStats s0 = StubStats();
    EXPECT_EQ(s0.open_contexts, 1);
    EXPECT_EQ(s0.live_pds, 1);
    {
        std::vector<char> a(1 << 16), b(1 << 16);
        uint32_t la = 0, lb = 0;
        ASSERT_EQ(pr->RegisterMemory(a.data(), a.size(), false, -1, &la), 0);
        ASSERT_EQ(pr->RegisterMemory(b.data(), b.size(), false, -1, &lb), 0);
        EXPECT_NE(la, lb);
        auto cq1 = pr->CreateCq(64);
        auto cq2 = pr->CreateCq(64);
        ASSERT_TRUE(cq1 && cq2);
        auto q1 = pr->CreateQp(cq1.get(), 16, 16);
        auto q2 = pr->CreateQp(cq2.get(), 16, 16);
        ASSERT_TRUE(q1 && q2);
        EXPECT_NE(q1->local().qpn, q2->local().qpn);
        EXPECT_EQ(q1->local().lid, 7);
        // sending before the RESET->INIT->RTR->RTS walk is refused
        memcpy(a.data(), "hello verbs", 11);
        rdma::Sge sg[2] = {{(uint64_t)(uintptr_t)a.data(), 5, la}, {(uint64_t)(uintptr_t)(a.data() + 5), 6, la}};
        EXPECT_NE(q1->PostSend(1, sg, 2, false, 0, true), 0);
        ASSERT_EQ(q1->Connect(q2->local()), 0);
        ASSERT_EQ(q2->Connect(q1->local()), 0);
        // held until a receive is posted (RNR), then delivered with imm
        ASSERT_EQ(q1->PostSend(42, sg, 2, true, 0xabcdef, true), 0);
        rdma::WorkCompletion wc[4];
        EXPECT_EQ(cq2->Poll(wc, 4), 0);
        ASSERT_EQ(cq2->Arm(), 0);
        rdma::Sge r{(uint64_t)(uintptr_t)b.data(), 4096, lb};
        ASSERT_EQ(q2->PostRecv(7, r), 0);
        // notification through the (non-blocking) completion channel
        pollfd pfd{cq2->notify_fd(), POLLIN, 0};
        EXPECT_EQ(poll(&pfd, 1, 1000), 1);
        cq2->AckEvent();
        ASSERT_EQ(cq2->Poll(wc, 4), 1);
        EXPECT_EQ(wc[0].wr_id, 7u);
        EXPECT_EQ(wc[0].opcode, (int)rdma::WC_RECV);
        EXPECT_EQ(wc[0].status, 0);
        EXPECT_EQ(wc[0].byte_len, 11u);
        EXPECT_TRUE(wc[0].has_imm);
        EXPECT_EQ(wc[0].imm, 0xabcdefu);  // network byte order round trip
        EXPECT_EQ(memcmp(b.data(), "hello verbs", 11), 0);
        ASSERT_EQ(cq1->Poll(wc, 4), 1);
        EXPECT_EQ(wc[0].wr_id, 42u);
        EXPECT_EQ(wc[0].opcode, (int)rdma::WC_SEND);
        // an SGE outside every registered region
        char stack_buf[16];
        rdma::Sge unreg{(uint64_t)(uintptr_t)stack_buf, 16, la};
        EXPECT_NE(q1->PostSend(45, &unreg, 1, false, 0, true), 0);
        // more SGEs than the QP was created for
        std::vector<rdma::Sge> many(17, sg[0]);
        EXPECT_NE(q1->PostSend(46, many.data(), 17, false, 0, true), 0);
        // receive buffer too small: error completions on both sides
        rdma::Sge small{(uint64_t)(uintptr_t)b.data(), 4, lb};
        ASSERT_EQ(q2->PostRecv(9, small), 0);
        ASSERT_EQ(q1->PostSend(47, sg, 2, false, 0, true), 0);
        ASSERT_EQ(cq2->Poll(wc, 4), 1);
        EXPECT_NE(wc[0].status, 0);
        ASSERT_EQ(cq1->Poll(wc, 4), 1);
        EXPECT_NE(wc[0].status, 0);
        // GPUDirect registration goes through the dmabuf export hook
        rdma::DmabufExportFn prev = rdma::GetDmabufExportHook();
        rdma::SetDmabufExportHook(FakeDmabufExport);
        std::vector<char> hbm_stand_in(1 << 16);
        uint32_t ld = 0;
        EXPECT_EQ(pr->RegisterMemory(hbm_stand_in.data(), hbm_stand_in.size(), true, 0, &ld), 0);
        EXPECT_EQ(StubStats().dmabuf_regs, s0.dmabuf_regs + 1);
        pr->DeregisterMemory(hbm_stand_in.data());
        rdma::SetDmabufExportHook(prev);
        pr->DeregisterMemory(a.data());
        pr->DeregisterMemory(b.data());
        const FakeIbvStats s1 = StubStats();
        EXPECT_EQ(s1.live_qps, 2);
        EXPECT_EQ(s1.live_cqs, 2);
        EXPECT_EQ(s1.live_mrs, 0);
    }
    // QPs, CQs (after acking their events) and channels are all destroyed
    const FakeIbvStats s2 = StubStats();
    EXPECT_EQ(s2.live_qps, 0);
    EXPECT_EQ(s2.live_cqs, 0);
    EXPECT_EQ(s2.live_channels, 0);
    pr.reset();
    const FakeIbvStats s3 = StubStats();
    EXPECT_EQ(s3.open_contexts, 0);
    EXPECT_EQ(s3.live_pds, 0);
}

TEST(RdmaVerbs, echo_over_ibverbs_provider) {
    FLAGS_rdma_verbs_library = StubPath();
    FLAGS_rdma_provider = "ibverbs";
    std::string err;
    ASSERT_EQ(rdma::GlobalRdmaInitialize(&err), 0);
    EXPECT_TRUE(rdma::DescribeRdma().find("provider: ibverbs") != std::string::npos);
    EXPECT_TRUE(rdma::DescribeRdma().find("fake_mlx5_0") != std::string::npos);
    const FakeIbvStats s0 = StubStats();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.use_rdma = true;
    opt.timeout_ms = 10000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < 200; ++i) {
        std::string why;
        Buf att;
        if (i % 4 == 0) att.append(Pattern(100 + 37 * i, i));
        ASSERT_TRUE(EchoOnce(stub, "verbs-" + std::to_string(i), att, &why));
    }
    // multi-MiB attachments: many blocks per message, the credit window
    // runs dry and refills through the stub's RNR hold-back
    for (int i = 0; i < 4; ++i) {
        std::string why;
        Buf att;
        att.append(Pattern((3 << 20) + i * 4099, i));
        ASSERT_TRUE(EchoOnce(stub, "big", att, &why));
    }
    EXPECT_EQ(s.RdmaConnections(), 1);
    const FakeIbvStats s1 = StubStats();
    EXPECT_GT(s1.sends - s0.sends, 400);
    EXPECT_EQ(s1.sends - s0.sends, s1.recvs - s0.recvs);  // every SEND landed
    EXPECT_GT(s1.bytes - s0.bytes, 2 * 4 * (3 << 20));
    EXPECT_EQ(s1.errors, s0.errors);
    EXPECT_GT(s1.events, s0.events);  // completion channel drove the pollers
}
