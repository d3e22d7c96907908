// TLS over the socket layer (spirit of the reference's test/brpc_ssl_unittest.cpp):
// a self-signed certificate is generated in-process, then baidu_std and
// http calls run over TLS, plaintext clients share the TLS port, and large
// attachments exercise partial-write crediting of encrypted records.
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>
#include <openssl/ssl.h>
#include <arpa/inet.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <string>
#include <vector>

#include "mrpc/proto/echo.pb.h"
#include "base/endpoint.h"
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

// ---------------------------------------------------------------- SNI
namespace {

// A self-signed certificate for `cn` (and DNS SAN `san` when given), as
// PEM text.
bool MakeCertPem(const std::string& cn, const std::string& san, std::string* cert, std::string* key) {
    EVP_PKEY* pkey = EVP_RSA_gen(2048);
    if (!pkey) return false;
    X509* x = X509_new();
    ASN1_INTEGER_set(X509_get_serialNumber(x), (long)std::hash<std::string>()(cn) & 0x7fffffff);
    X509_gmtime_adj(X509_getm_notBefore(x), 0);
    X509_gmtime_adj(X509_getm_notAfter(x), 3600);
    X509_set_pubkey(x, pkey);
    X509_NAME* name = X509_get_subject_name(x);
    X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, (const unsigned char*)cn.c_str(), -1, -1, 0);
    X509_set_issuer_name(x, name);
    if (!san.empty()) {
        X509V3_CTX v3;
        X509V3_set_ctx_nodb(&v3);
        X509V3_set_ctx(&v3, x, x, nullptr, nullptr, 0);
        X509_EXTENSION* ext = X509V3_EXT_conf_nid(nullptr, &v3, NID_subject_alt_name, ("DNS:" + san).c_str());
        if (ext) {
            X509_add_ext(x, ext, -1);
            X509_EXTENSION_free(ext);
        }
    }
    bool ok = X509_sign(x, pkey, EVP_sha256()) > 0;
    BIO* b = BIO_new(BIO_s_mem());
    ok = ok && PEM_write_bio_X509(b, x);
    char* p = nullptr;
    long n = BIO_get_mem_data(b, &p);
    cert->assign(p, (size_t)n);
    BIO_free(b);
    b = BIO_new(BIO_s_mem());
    ok = ok && PEM_write_bio_PrivateKey(b, pkey, nullptr, nullptr, 0, nullptr, nullptr);
    n = BIO_get_mem_data(b, &p);
    key->assign(p, (size_t)n);
    BIO_free(b);
    X509_free(x);
    EVP_PKEY_free(pkey);
    return ok;
}

// Handshake with `sni` (empty: none) and return the CN of the certificate
// the server presented; "" when the handshake failed.
std::string PresentedCn(int port, const std::string& sni) {
    SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
    SSL_CTX_set_verify(ctx, SSL_VERIFY_NONE, nullptr);
    int fd = tcp_connect(EndPoint(htonl(INADDR_LOOPBACK), port), 2000);
    std::string cn;
    if (fd >= 0) {
        timeval tv{2, 0};
        setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        SSL* ssl = SSL_new(ctx);
        SSL_set_fd(ssl, fd);
        if (!sni.empty()) SSL_set_tlsext_host_name(ssl, sni.c_str());
        if (SSL_connect(ssl) == 1) {
            X509* peer = SSL_get1_peer_certificate(ssl);
            char buf[256];
            if (peer && X509_NAME_get_text_by_NID(X509_get_subject_name(peer), NID_commonName, buf, sizeof(buf)) > 0) {
                cn = buf;
            }
            if (peer) X509_free(peer);
        }
        SSL_free(ssl);
        close(fd);
    }
    SSL_CTX_free(ctx);
    return cn;
}

}  // namespace

// reference: src/brpc/server.h:450-465 (AddCertificate / RemoveCertificate /
// ResetCertificates), src/brpc/ssl_options.h:30-42,97-110 (CertInfo,
// sni_filters with a leading wildcard, strict_sni)
TEST(Ssl, sni_certificate_maps_and_runtime_changes) {
    std::string dc, dk, ac, ak, wc, wk;
    ASSERT_TRUE(MakeCertPem("default.test", "", &dc, &dk));
    ASSERT_TRUE(MakeCertPem("alpha.test", "beta.test", &ac, &ak));
    ASSERT_TRUE(MakeCertPem("wild.test", "", &wc, &wk));
    const std::string cert_file = "/tmp/mrpc_sni_cert_" + std::to_string(getpid()) + ".pem";
    const std::string key_file = "/tmp/mrpc_sni_key_" + std::to_string(getpid()) + ".pem";
    {
        FILE* f = fopen(cert_file.c_str(), "w");
        fwrite(dc.data(), 1, dc.size(), f);
        fclose(f);
        f = fopen(key_file.c_str(), "w");
        fwrite(dk.data(), 1, dk.size(), f);
        fclose(f);
    }
    Server server;
    EchoServiceImpl echo;
    server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.ssl_cert_file = cert_file;  // default certificate from files
    o.ssl_key_file = key_file;
    CertInfo alpha{ac, ak, {}};   // an SNI certificate as PEM text
    o.ssl_certs.push_back(alpha);
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const int port = server.listen_port();
    EXPECT_EQ(PresentedCn(port, "alpha.test"), "alpha.test");
    EXPECT_EQ(PresentedCn(port, "BETA.test"), "alpha.test");  // SAN, case-insensitive
    EXPECT_EQ(PresentedCn(port, "default.test"), "default.test");
    EXPECT_EQ(PresentedCn(port, "unknown.test"), "default.test");  // not strict: default
    EXPECT_EQ(PresentedCn(port, ""), "default.test");
    // a wildcard filter added while running
    CertInfo wild{wc, wk, {"*.wild.test"}};
    ASSERT_EQ(server.AddCertificate(wild), 0);
    EXPECT_EQ(PresentedCn(port, "a.wild.test"), "wild.test");
    EXPECT_EQ(PresentedCn(port, "wild.test"), "wild.test");      // its CN
    EXPECT_EQ(PresentedCn(port, "a.b.wild.test"), "default.test");  // one label only
    // RPCs keep working over TLS after the change
    EchoCalls("127.0.0.1:" + std::to_string(port), true, "baidu_std", 5, 100);
    ASSERT_EQ(server.RemoveCertificate(alpha), 0);
    EXPECT_EQ(PresentedCn(port, "alpha.test"), "default.test");
    EXPECT_NE(server.RemoveCertificate(alpha), 0);  // not there any more
    ASSERT_EQ(server.ResetCertificates({alpha}), 0);  // replaces every SNI certificate
    EXPECT_EQ(PresentedCn(port, "alpha.test"), "alpha.test");
    EXPECT_EQ(PresentedCn(port, "a.wild.test"), "default.test");
    CertInfo broken{"-----BEGIN CERTIFICATE-----\nnot a cert\n-----END CERTIFICATE-----\n", ak, {}};
    EXPECT_NE(server.AddCertificate(broken), 0);
    server.Stop(0);
    server.Join();

    // strict_sni: no name, or a name no certificate serves, is refused
    Server strict;
    EchoServiceImpl echo2;
    strict.AddService(&echo2, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so = o;
    so.ssl_strict_sni = true;
    ASSERT_EQ(strict.Start("127.0.0.1:0", &so), 0);
    const int sport = strict.listen_port();
    EXPECT_EQ(PresentedCn(sport, "alpha.test"), "alpha.test");
    EXPECT_EQ(PresentedCn(sport, "default.test"), "default.test");
    EXPECT_EQ(PresentedCn(sport, "unknown.test"), "");
    EXPECT_EQ(PresentedCn(sport, ""), "");
    strict.Stop(0);
    strict.Join();
    unlink(cert_file.c_str());
    unlink(key_file.c_str());
}
