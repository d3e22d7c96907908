// TLS over the socket layer (spirit of the reference's test/brpc_ssl_unittest.cpp):
// a self-signed certificate is generated in-process, then baidu_std and
// http calls run over TLS, plaintext clients share the TLS port, and large
// attachments exercise partial-write crediting of encrypted records.
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>
#include <openssl/x509.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <string>
#include <vector>

#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

bool MakeSelfSignedCert(const std::string& cert_path, const std::string& key_path) {
    EVP_PKEY* pkey = EVP_RSA_gen(2048);
    if (!pkey) return false;
    X509* x = X509_new();
    ASN1_INTEGER_set(X509_get_serialNumber(x), 1);
    X509_gmtime_adj(X509_getm_notBefore(x), 0);
    X509_gmtime_adj(X509_getm_notAfter(x), 3600);
    X509_set_pubkey(x, pkey);
    X509_NAME* name = X509_get_subject_name(x);
    X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, (const unsigned char*)"localhost", -1, -1, 0);
    X509_set_issuer_name(x, name);
    bool ok = X509_sign(x, pkey, EVP_sha256()) > 0;
    FILE* f = fopen(cert_path.c_str(), "w");
    ok = ok && f && PEM_write_X509(f, x);
    if (f) fclose(f);
    f = fopen(key_path.c_str(), "w");
    ok = ok && f && PEM_write_PrivateKey(f, pkey, nullptr, nullptr, 0, nullptr, nullptr);
    if (f) fclose(f);
    X509_free(x);
    EVP_PKEY_free(pkey);
    return ok;
}

struct TlsServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    TlsServer() {
        const std::string cert = "/tmp/mrpc_test_cert_" + std::to_string(getpid()) + ".pem";
        const std::string key = "/tmp/mrpc_test_key_" + std::to_string(getpid()) + ".pem";
        if (!MakeSelfSignedCert(cert, key)) return;
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.ssl_cert_file = cert;
        o.ssl_key_file = key;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

void EchoCalls(const std::string& addr, bool ssl, const std::string& protocol, int n, size_t attach) {
    Channel ch;
    ChannelOptions opt;
    opt.use_ssl = ssl;
    opt.protocol = protocol;
    opt.timeout_ms = 5000;
    opt.ssl_sni = "localhost";
    ASSERT_EQ(ch.Init(addr.c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    std::string big(attach, '\0');
    for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 31 + 7);
    for (int i = 0; i < n; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("tls-" + std::to_string(i));
        if (attach && protocol == "baidu_std") cntl.request_attachment().append(big);
        stub.Echo(&cntl, &req, &res, nullptr);
        if (cntl.Failed()) fprintf(stderr, "call %d failed: %s\n", i, cntl.ErrorText().c_str());
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.message(), req.message());
        if (attach && protocol == "baidu_std") EXPECT_TRUE(cntl.response_attachment().equals(big));
    }
}

}  // namespace

TEST(Ssl, baidu_std_over_tls) {
    TlsServer s;
    ASSERT_GT(s.port, 0);
    EchoCalls(s.addr(), true, "baidu_std", 50, 0);
    // the accepted connection really negotiated TLS (keep a channel open)
    Channel ch;
    ChannelOptions opt;
    opt.use_ssl = true;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    std::vector<SocketId> conns;
    s.server.acceptor()->ListConnections(&conns);
    int tls = 0;
    for (SocketId id : conns) {
        SocketUniquePtr p;
        if (Socket::Address(id, &p) == 0 && p->is_ssl()) {
            ++tls;
            std::shared_ptr<SslSession> ss = p->ssl_session();
            EXPECT_TRUE(ss && ss->handshake_done());
            EXPECT_TRUE(ss->version().find("TLS") == 0);
        }
    }
    EXPECT_GE(tls, 1);
}

TEST(Ssl, large_attachments_partial_writes) {
    TlsServer s;
    ASSERT_GT(s.port, 0);
    EchoCalls(s.addr(), true, "baidu_std", 8, 3 << 20);
}

TEST(Ssl, plaintext_and_tls_share_the_port) {
    TlsServer s;
    ASSERT_GT(s.port, 0);
    EchoCalls(s.addr(), false, "baidu_std", 10, 1000);
    EchoCalls(s.addr(), true, "baidu_std", 10, 1000);
    EchoCalls(s.addr(), false, "baidu_std", 10, 0);
}

TEST(Ssl, http_over_tls_and_concurrency) {
    TlsServer s;
    ASSERT_GT(s.port, 0);
    EchoCalls(s.addr(), true, "http", 10, 0);
    // many concurrent async calls on one TLS connection
    Channel ch;
    ChannelOptions opt;
    opt.use_ssl = true;
    opt.timeout_ms = 5000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    const int N = 200;
    std::vector<std::unique_ptr<Controller>> cntls(N);
    std::vector<example::EchoRequest> reqs(N);
    std::vector<example::EchoResponse> ress(N);
    for (int i = 0; i < N; ++i) {
        cntls[i].reset(new Controller);
        reqs[i].set_message(std::string(100 + i * 97, 'a' + i % 26));
        stub.Echo(cntls[i].get(), &reqs[i], &ress[i], NewCallback([] {}));
    }
    for (int i = 0; i < N; ++i) {
        cntls[i]->Join();
        ASSERT_FALSE(cntls[i]->Failed());
        EXPECT_EQ(ress[i].message(), reqs[i].message());
    }
}
