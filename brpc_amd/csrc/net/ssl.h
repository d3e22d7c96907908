// TLS for sockets (role of the reference's src/brpc/details/ssl_helper.cpp,
// ssl_options.h and the SSL state machine in socket.cpp:1852-2035).
//
// The TLS engine runs over memory BIOs so it fits the edge-triggered,
// wait-free socket design unchanged: DoRead feeds raw bytes in and gets
// plaintext out; writes encrypt plaintext into a per-session ciphertext
// queue. A write request is only credited once the ciphertext of its bytes
// reached the kernel, so KeepWrite / partial-write accounting stays exact.
// Servers detect TLS per connection from the first byte (0x16 = handshake
// record), so one port serves TLS and plaintext clients alike.
#pragma once

#include <atomic>

#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "base/buf.h"

typedef struct ssl_ctx_st SSL_CTX;
typedef struct ssl_st SSL;
typedef struct bio_st BIO;

namespace mrpc {

// A certificate and its key (reference: src/brpc/ssl_options.h:30-42).
// Each is a PEM file path, or the PEM text itself ("-----BEGIN ...").
// The certificate serves its CN and DNS subject-alt-names plus
// sni_filters; a wildcard may only lead a name ("*.example.com").
struct CertInfo {
    std::string certificate;
    std::string private_key;
    std::vector<std::string> sni_filters;
};

struct ServerSslOptions {
    std::string cert_file;      // PEM certificate chain (default certificate)
    std::string key_file;       // PEM private key
    CertInfo default_cert;      // alternative to cert_file/key_file (files or PEM text)
    std::vector<CertInfo> certs;  // more certificates, chosen by the client's SNI name
    std::string ciphers;        // OpenSSL cipher list (empty: default)
    std::string alpns;          // comma separated, e.g. "h2,http/1.1"
    // Refuse handshakes without an SNI name, or whose name no certificate
    // (the default one included) serves; otherwise the default certificate
    // answers them.
    bool strict_sni = false;
};

struct ChannelSslOptions {
    std::string sni_name;
    std::string ciphers;
    std::string ca_file;        // verify the server when set
    bool verify = false;
};

class SslContext {
public:
    ~SslContext();
    static std::shared_ptr<SslContext> NewServer(const ServerSslOptions& opt, std::string* err);
    // Server contexts: certificates chosen by SNI, changeable while the
    // server runs (handshakes in progress keep the certificate they chose).
    // The default certificate is fixed. 0 on success.
    int AddCertificate(const CertInfo& cert, std::string* err);
    int RemoveCertificate(const CertInfo& cert);
    int ResetCertificates(const std::vector<CertInfo>& certs, std::string* err);
    // The hostnames a certificate serves (CN, DNS SANs, then sni_filters).
    static bool CertificateNames(const CertInfo& cert, std::vector<std::string>* names, std::string* err);
    struct SniMap;
    static std::shared_ptr<SslContext> NewClient(const ChannelSslOptions& opt, std::string* err);
    // Shared no-verification client context (Channel use_ssl).
    static std::shared_ptr<SslContext> DefaultClient();
    SSL_CTX* ctx() const { return _ctx; }
    bool is_server() const { return _server; }

private:
    friend int sni_callback(SSL*, int*, void*);
    SSL_CTX* _ctx = nullptr;
    bool _server = false;
    // SNI: per-certificate contexts by hostname, published as one immutable
    // map (std::atomic_load in the handshake, rebuilt under _cert_mu)
    ServerSslOptions _opt;
    std::mutex _cert_mu;
    std::vector<std::pair<CertInfo, std::shared_ptr<SslContext>>> _certs;
    std::vector<std::string> _default_names;
    std::shared_ptr<const SniMap> _sni;
    void publish_locked();
};

class SslSession {
public:
    SslSession(const std::shared_ptr<SslContext>& ctx, bool server, const std::string& sni);
    ~SslSession();
    bool ok() const { return _ssl != nullptr; }
    // read by the writer (KeepWrite) while the reader completes the handshake
    bool handshake_done() const { return _handshake_done.load(std::memory_order_acquire); }

    // Read path: raw ciphertext in, plaintext appended to *out. Returns the
    // plaintext bytes produced, or -1 on a TLS error (errno EPROTO).
    // *handshake_completed is set when this call finished the handshake
    // (writers blocked on it should be woken).
    ssize_t Feed(const Buf& raw, Buf* out, bool* handshake_completed);
    bool peer_closed() const { return _peer_closed; }
    // Write path over fd: credits plaintext of data_list whose ciphertext
    // has been written; returns credited bytes or -1 with errno EAGAIN
    // (socket buffer full) or EINPROGRESS (waiting for the handshake).
    ssize_t Write(int fd, Buf** data_list, size_t n);
    // Flushes pending ciphertext (handshake records); true if empty after.
    bool Flush(int fd);
    bool has_pending_output();
    std::string cipher() const;
    std::string version() const;

private:
    void drain_wbio_locked();
    ssize_t flush_locked(int fd);  // credits plaintext, returns credited bytes
    std::shared_ptr<SslContext> _ctxref;
    SSL* _ssl = nullptr;
    BIO* _rbio = nullptr;
    BIO* _wbio = nullptr;
    std::mutex _mu;
    std::atomic<bool> _handshake_done{false};
    Buf _cipher_out;                            // ciphertext not yet written
    std::deque<std::pair<size_t, size_t>> _records;  // (cipher bytes, plain bytes) per SSL_write
    size_t _uncredited_plain = 0;               // encrypted plaintext not yet credited
    size_t _credited_pending = 0;               // ciphertext bytes of the front record already written
    size_t _claimable = 0;                      // plaintext credited by reader-side flushes
    bool _peer_closed = false;
};

// Is this a TLS ClientHello start? (1 yes, 0 no, -1 need more bytes)
int LooksLikeTls(const char* p, size_t n);

}  // namespace mrpc
