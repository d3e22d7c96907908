#include "net/ssl.h"

#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <cerrno>
#include <mutex>
#include <unordered_map>

#include "base/logging.h"
#include "base/util.h"

namespace mrpc {

static void init_openssl_once() {
    static std::once_flag once;
    std::call_once(once, [] {
        OPENSSL_init_ssl(OPENSSL_INIT_LOAD_SSL_STRINGS | OPENSSL_INIT_LOAD_CRYPTO_STRINGS, nullptr);
    });
}

static std::string last_ssl_error() {
    char buf[256];
    const unsigned long e = ERR_get_error();
    if (!e) return "unknown TLS error";
    ERR_error_string_n(e, buf, sizeof(buf));
    return buf;
}

int LooksLikeTls(const char* p, size_t n) {
    if (n < 1) return -1;
    // TLS record: content type 22 (handshake), then version major 3
    if ((uint8_t)p[0] != 0x16) return 0;
    if (n < 2) return -1;
    return (uint8_t)p[1] == 0x03 ? 1 : 0;
}

SslContext::~SslContext() {
    if (_ctx) SSL_CTX_free(_ctx);
}

static int alpn_select_cb(SSL*, const unsigned char** out, unsigned char* outlen, const unsigned char* in,
                          unsigned int inlen, void* arg) {
    const std::string* wire = static_cast<const std::string*>(arg);
    if (SSL_select_next_proto((unsigned char**)out, outlen, (const unsigned char*)wire->data(), (unsigned)wire->size(),
                              in, inlen) == OPENSSL_NPN_NEGOTIATED) {
        return SSL_TLSEXT_ERR_OK;
    }
    return SSL_TLSEXT_ERR_NOACK;
}

namespace {

bool is_pem_text(const std::string& s) { return s.compare(0, 10, "-----BEGIN") == 0; }

// certificate chain + key into ctx, from files or PEM text
bool load_cert(SSL_CTX* ctx, const std::string& cert, const std::string& key, std::string* err) {
    bool ok;
    if (is_pem_text(cert)) {
        BIO* b = BIO_new_mem_buf(cert.data(), (int)cert.size());
        X509* x = b ? PEM_read_bio_X509(b, nullptr, nullptr, nullptr) : nullptr;
        ok = x && SSL_CTX_use_certificate(ctx, x) == 1;
        if (x) X509_free(x);
        while (ok) {  // the rest of the chain
            X509* ca = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
            if (!ca) {
                ERR_clear_error();
                break;
            }
            if (SSL_CTX_add_extra_chain_cert(ctx, ca) != 1) {  // takes ownership on success
                X509_free(ca);
                ok = false;
            }
        }
        if (b) BIO_free(b);
    } else {
        ok = SSL_CTX_use_certificate_chain_file(ctx, cert.c_str()) == 1;
    }
    if (ok) {
        if (is_pem_text(key)) {
            BIO* b = BIO_new_mem_buf(key.data(), (int)key.size());
            EVP_PKEY* k = b ? PEM_read_bio_PrivateKey(b, nullptr, nullptr, nullptr) : nullptr;
            ok = k && SSL_CTX_use_PrivateKey(ctx, k) == 1;
            if (k) EVP_PKEY_free(k);
            if (b) BIO_free(b);
        } else {
            ok = SSL_CTX_use_PrivateKey_file(ctx, key.c_str(), SSL_FILETYPE_PEM) == 1;
        }
    }
    ok = ok && SSL_CTX_check_private_key(ctx) == 1;
    if (!ok) {
        *err = "certificate/key " + (is_pem_text(cert) ? std::string("(PEM text)") : cert) + "/" +
               (is_pem_text(key) ? std::string("(PEM text)") : key) + ": " + last_ssl_error();
    }
    return ok;
}

X509* read_x509(const std::string& cert) {
    BIO* b = is_pem_text(cert) ? BIO_new_mem_buf(cert.data(), (int)cert.size()) : BIO_new_file(cert.c_str(), "r");
    if (!b) return nullptr;
    X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
    BIO_free(b);
    return x;
}

std::string lower(std::string s) {
    for (char& c : s) c = (char)tolower((unsigned char)c);
    return s;
}

}  // namespace

bool SslContext::CertificateNames(const CertInfo& cert, std::vector<std::string>* names, std::string* err) {
    X509* x = read_x509(cert.certificate);
    if (!x) {
        *err = "cannot read certificate: " + last_ssl_error();
        return false;
    }
    char cn[256];
    if (X509_NAME_get_text_by_NID(X509_get_subject_name(x), NID_commonName, cn, sizeof(cn)) > 0) {
        names->push_back(lower(cn));
    }
    GENERAL_NAMES* sans = static_cast<GENERAL_NAMES*>(X509_get_ext_d2i(x, NID_subject_alt_name, nullptr, nullptr));
    for (int i = 0; sans && i < sk_GENERAL_NAME_num(sans); ++i) {
        const GENERAL_NAME* g = sk_GENERAL_NAME_value(sans, i);
        if (g->type != GEN_DNS) continue;
        const unsigned char* d = ASN1_STRING_get0_data(g->d.dNSName);
        names->push_back(lower(std::string((const char*)d, (size_t)ASN1_STRING_length(g->d.dNSName))));
    }
    if (sans) GENERAL_NAMES_free(sans);
    X509_free(x);
    for (const std::string& f : cert.sni_filters) names->push_back(lower(f));
    return true;
}

// hostname -> context; "*.example.com" is stored under "example.com" in
// `wildcard` and matches exactly one more leading label
struct SslContext::SniMap {
    std::unordered_map<std::string, std::shared_ptr<SslContext>> exact, wildcard;
    std::shared_ptr<SslContext> find(const std::string& host) const {
        auto it = exact.find(host);
        if (it != exact.end()) return it->second;
        const size_t dot = host.find('.');
        if (dot != std::string::npos) {
            auto w = wildcard.find(host.substr(dot + 1));
            if (w != wildcard.end()) return w->second;
        }
        return nullptr;
    }
};

int sni_callback(SSL* ssl, int* alert, void* arg) {
    SslContext* self = static_cast<SslContext*>(arg);
    const char* name = SSL_get_servername(ssl, TLSEXT_NAMETYPE_host_name);
    const bool strict = self->_opt.strict_sni;
    if (!name || !*name) {
        if (!strict) return SSL_TLSEXT_ERR_OK;  // the default certificate
        *alert = SSL_AD_UNRECOGNIZED_NAME;
        return SSL_TLSEXT_ERR_ALERT_FATAL;
    }
    std::shared_ptr<const SslContext::SniMap> m = std::atomic_load(&self->_sni);
    std::shared_ptr<SslContext> c = m ? m->find(lower(name)) : nullptr;
    if (c) {
        // the SSL holds its own reference to the chosen SSL_CTX
        if (c.get() != self) SSL_set_SSL_CTX(ssl, c->ctx());
        return SSL_TLSEXT_ERR_OK;
    }
    if (!strict) return SSL_TLSEXT_ERR_OK;
    *alert = SSL_AD_UNRECOGNIZED_NAME;
    return SSL_TLSEXT_ERR_ALERT_FATAL;
}

namespace {

// A server SSL_CTX with the options every certificate shares.
SSL_CTX* new_server_ctx(const ServerSslOptions& opt, const std::string& cert, const std::string& key,
                        std::string* err) {
    SSL_CTX* ctx = SSL_CTX_new(TLS_server_method());
    if (!ctx) {
        *err = last_ssl_error();
        return nullptr;
    }
    SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
    SSL_CTX_set_mode(ctx, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    if (!load_cert(ctx, cert, key, err)) {
        SSL_CTX_free(ctx);
        return nullptr;
    }
    if (!opt.ciphers.empty() && SSL_CTX_set_cipher_list(ctx, opt.ciphers.c_str()) != 1) {
        *err = "ciphers: " + last_ssl_error();
        SSL_CTX_free(ctx);
        return nullptr;
    }
    if (!opt.alpns.empty()) {
        // wire format: length-prefixed protocol names; kept alive with the ctx
        static std::mutex mu;
        static std::vector<std::unique_ptr<std::string>> keep;
        std::unique_ptr<std::string> wire(new std::string);
        for (const std::string& p : split_string(opt.alpns, ',')) {
            wire->push_back((char)p.size());
            wire->append(p);
        }
        SSL_CTX_set_alpn_select_cb(ctx, alpn_select_cb, wire.get());
        std::lock_guard<std::mutex> g(mu);
        keep.push_back(std::move(wire));
    }
    return ctx;
}

}  // namespace

std::shared_ptr<SslContext> SslContext::NewServer(const ServerSslOptions& opt, std::string* err) {
    init_openssl_once();
    std::shared_ptr<SslContext> c(new SslContext);
    c->_server = true;
    c->_opt = opt;
    if (c->_opt.default_cert.certificate.empty()) {
        c->_opt.default_cert.certificate = opt.cert_file;
        c->_opt.default_cert.private_key = opt.key_file;
    }
    const CertInfo& dc = c->_opt.default_cert;
    c->_ctx = new_server_ctx(opt, dc.certificate, dc.private_key, err);
    if (!c->_ctx) return nullptr;
    if (!CertificateNames(dc, &c->_default_names, err)) return nullptr;
    SSL_CTX_set_tlsext_servername_callback(c->_ctx, sni_callback);
    SSL_CTX_set_tlsext_servername_arg(c->_ctx, c.get());
    std::lock_guard<std::mutex> g(c->_cert_mu);
    for (const CertInfo& ci : opt.certs) {
        std::shared_ptr<SslContext> x(new SslContext);
        x->_server = true;
        x->_ctx = new_server_ctx(opt, ci.certificate, ci.private_key, err);
        if (!x->_ctx) return nullptr;
        c->_certs.emplace_back(ci, x);
    }
    c->publish_locked();
    return c;
}

void SslContext::publish_locked() {
    std::shared_ptr<SniMap> m = std::make_shared<SniMap>();
    auto add = [&m](const std::string& name, const std::shared_ptr<SslContext>& ctx) {
        if (name.compare(0, 2, "*.") == 0) m->wildcard.emplace(name.substr(2), ctx);
        else if (!name.empty()) m->exact.emplace(name, ctx);
    };
    // later certificates win over earlier ones for the same name (emplace
    // keeps the first: walk newest first); the default one serves its own
    // names unless another certificate claims them
    for (auto it = _certs.rbegin(); it != _certs.rend(); ++it) {
        std::vector<std::string> names;
        std::string err;
        if (CertificateNames(it->first, &names, &err)) {
            for (const std::string& n : names) add(n, it->second);
        }
    }
    // the default context is not owned by a shared_ptr here: a non-owning
    // alias marks "stay on the default" for the callback
    std::shared_ptr<SslContext> self(std::shared_ptr<SslContext>(), this);
    for (const std::string& n : _default_names) add(n, self);
    std::atomic_store(&_sni, std::shared_ptr<const SniMap>(std::move(m)));
}

int SslContext::AddCertificate(const CertInfo& cert, std::string* err) {
    if (!_server) return -1;
    std::vector<std::string> names;
    if (!CertificateNames(cert, &names, err)) return -1;
    std::shared_ptr<SslContext> x(new SslContext);
    x->_server = true;
    x->_ctx = new_server_ctx(_opt, cert.certificate, cert.private_key, err);
    if (!x->_ctx) return -1;
    std::lock_guard<std::mutex> g(_cert_mu);
    for (auto& e : _certs) {
        if (e.first.certificate == cert.certificate) {  // replace (new key or filters)
            e = {cert, x};
            publish_locked();
            return 0;
        }
    }
    _certs.emplace_back(cert, x);
    publish_locked();
    return 0;
}

int SslContext::RemoveCertificate(const CertInfo& cert) {
    std::lock_guard<std::mutex> g(_cert_mu);
    for (size_t i = 0; i < _certs.size(); ++i) {
        if (_certs[i].first.certificate == cert.certificate) {
            _certs.erase(_certs.begin() + (long)i);
            publish_locked();
            return 0;
        }
    }
    return -1;
}

int SslContext::ResetCertificates(const std::vector<CertInfo>& certs, std::string* err) {
    std::vector<std::pair<CertInfo, std::shared_ptr<SslContext>>> fresh;
    for (const CertInfo& ci : certs) {
        std::shared_ptr<SslContext> x(new SslContext);
        x->_server = true;
        x->_ctx = new_server_ctx(_opt, ci.certificate, ci.private_key, err);
        if (!x->_ctx) return -1;
        fresh.emplace_back(ci, x);
    }
    std::lock_guard<std::mutex> g(_cert_mu);
    _certs.swap(fresh);
    publish_locked();
    return 0;
}

std::shared_ptr<SslContext> SslContext::NewClient(const ChannelSslOptions& opt, std::string* err) {
    init_openssl_once();
    std::shared_ptr<SslContext> c(new SslContext);
    c->_ctx = SSL_CTX_new(TLS_client_method());
    if (!c->_ctx) {
        *err = last_ssl_error();
        return nullptr;
    }
    SSL_CTX_set_min_proto_version(c->_ctx, TLS1_2_VERSION);
    SSL_CTX_set_mode(c->_ctx, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    if (!opt.ciphers.empty() && SSL_CTX_set_cipher_list(c->_ctx, opt.ciphers.c_str()) != 1) {
        *err = "ciphers: " + last_ssl_error();
        return nullptr;
    }
    if (opt.verify) {
        SSL_CTX_set_verify(c->_ctx, SSL_VERIFY_PEER, nullptr);
        if (!opt.ca_file.empty() ? SSL_CTX_load_verify_locations(c->_ctx, opt.ca_file.c_str(), nullptr) != 1
                                 : SSL_CTX_set_default_verify_paths(c->_ctx) != 1) {
            *err = "ca: " + last_ssl_error();
            return nullptr;
        }
    } else {
        SSL_CTX_set_verify(c->_ctx, SSL_VERIFY_NONE, nullptr);
    }
    return c;
}

std::shared_ptr<SslContext> SslContext::DefaultClient() {
    static std::shared_ptr<SslContext> c = [] {
        std::string err;
        std::shared_ptr<SslContext> x = NewClient(ChannelSslOptions(), &err);
        if (!x) LOG(ERROR) << "Fail to create the default TLS client context: " << err;
        return x;
    }();
    return c;
}

SslSession::SslSession(const std::shared_ptr<SslContext>& ctx, bool server, const std::string& sni) : _ctxref(ctx) {
    if (!ctx || !ctx->ctx()) return;
    _ssl = SSL_new(ctx->ctx());
    if (!_ssl) return;
    _rbio = BIO_new(BIO_s_mem());
    _wbio = BIO_new(BIO_s_mem());
    BIO_set_mem_eof_return(_rbio, -1);
    SSL_set_bio(_ssl, _rbio, _wbio);  // _ssl owns both BIOs
    if (server) {
        SSL_set_accept_state(_ssl);
    } else {
        SSL_set_connect_state(_ssl);
        if (!sni.empty()) SSL_set_tlsext_host_name(_ssl, sni.c_str());
        // Produce the ClientHello right away.
        SSL_do_handshake(_ssl);
        drain_wbio_locked();
    }
}

SslSession::~SslSession() {
    if (_ssl) SSL_free(_ssl);
}

void SslSession::drain_wbio_locked() {
    char tmp[16384];
    size_t total = 0;
    for (;;) {
        const int r = BIO_read(_wbio, tmp, sizeof(tmp));
        if (r <= 0) break;
        _cipher_out.append(tmp, (size_t)r);
        total += (size_t)r;
    }
    if (total) _records.emplace_back(total, 0);
}

ssize_t SslSession::flush_locked(int fd) {
    ssize_t credited = 0;
    while (!_cipher_out.empty()) {
        const ssize_t nw = _cipher_out.cut_into_fd(fd);
        if (nw < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            return -1;
        }
        size_t w = (size_t)nw;
        while (w > 0 && !_records.empty()) {
            std::pair<size_t, size_t>& r = _records.front();
            const size_t remain = r.first - _credited_pending;
            if (w >= remain) {
                w -= remain;
                credited += (ssize_t)r.second;
                _uncredited_plain -= r.second;
                _records.pop_front();
                _credited_pending = 0;
            } else {
                _credited_pending += w;
                w = 0;
            }
        }
    }
    return credited;
}

static void pop_plain(Buf** list, size_t n, size_t k) {
    for (size_t i = 0; i < n && k; ++i) {
        const size_t take = std::min(k, list[i]->size());
        list[i]->pop_front(take);
        k -= take;
    }
}

ssize_t SslSession::Write(int fd, Buf** list, size_t n) {
    if (!_ssl) {
        errno = EPROTO;
        return -1;
    }
    std::lock_guard<std::mutex> g(_mu);
    ssize_t credited = flush_locked(fd);
    if (credited < 0) return -1;
    credited += (ssize_t)_claimable;
    _claimable = 0;
    if (_cipher_out.empty()) {
        // Everything encrypted so far is on the wire: encrypt more plaintext,
        // skipping what this call is about to credit.
        size_t skip = (size_t)credited;
        size_t budget = 1 << 20;
        bool stop = false;
        for (size_t i = 0; i < n && budget && !stop; ++i) {
            const Buf* b = list[i];
            for (size_t k = 0; k < b->backing_block_num() && budget && !stop; ++k) {
                const char* p = b->block_data(k);
                size_t len = b->block_len(k);
                if (skip >= len) {
                    skip -= len;
                    continue;
                }
                p += skip;
                len -= skip;
                skip = 0;
                while (len && budget) {
                    const int chunk = (int)std::min<size_t>(std::min<size_t>(len, 16384), budget);
                    const int r = SSL_write(_ssl, p, chunk);
                    if (r <= 0) {
                        const int e = SSL_get_error(_ssl, r);
                        drain_wbio_locked();
                        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) {
                            stop = true;  // handshake still in progress
                            break;
                        }
                        LOG(WARNING) << "SSL_write: " << last_ssl_error();
                        errno = EPROTO;
                        return -1;
                    }
                    size_t before = _cipher_out.size();
                    char tmp[16384 + 512];
                    for (;;) {
                        const int c = BIO_read(_wbio, tmp, sizeof(tmp));
                        if (c <= 0) break;
                        _cipher_out.append(tmp, (size_t)c);
                    }
                    _records.emplace_back(_cipher_out.size() - before, (size_t)r);
                    _uncredited_plain += (size_t)r;
                    p += r;
                    len -= (size_t)r;
                    budget -= (size_t)std::min<size_t>(budget, (size_t)r);
                }
            }
        }
        const ssize_t more = flush_locked(fd);
        if (more < 0) return -1;
        credited += more;
    }
    if (credited == 0) {
        errno = (!_handshake_done && _cipher_out.empty()) ? EINPROGRESS : EAGAIN;
        return -1;
    }
    pop_plain(list, n, (size_t)credited);
    return credited;
}

bool SslSession::Flush(int fd) {
    std::lock_guard<std::mutex> g(_mu);
    const ssize_t c = flush_locked(fd);
    if (c > 0) _claimable += (size_t)c;  // credited plaintext the writer will claim
    return _cipher_out.empty();
}

bool SslSession::has_pending_output() {
    std::lock_guard<std::mutex> g(_mu);
    return !_cipher_out.empty();
}

ssize_t SslSession::Feed(const Buf& raw, Buf* out, bool* handshake_completed) {
    *handshake_completed = false;
    if (!_ssl) {
        errno = EPROTO;
        return -1;
    }
    std::lock_guard<std::mutex> g(_mu);
    for (size_t k = 0; k < raw.backing_block_num(); ++k) {
        if (BIO_write(_rbio, raw.block_data(k), (int)raw.block_len(k)) != (int)raw.block_len(k)) {
            errno = ENOMEM;
            return -1;
        }
    }
    if (!_handshake_done) {
        const int r = SSL_do_handshake(_ssl);
        if (r == 1) {
            _handshake_done.store(true, std::memory_order_release);
            *handshake_completed = true;
        } else {
            const int e = SSL_get_error(_ssl, r);
            if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE) {
                LOG(WARNING) << "TLS handshake failed: " << last_ssl_error();
                drain_wbio_locked();  // alert
                errno = EPROTO;
                return -1;
            }
        }
    }
    ssize_t produced = 0;
    if (_handshake_done) {
        char tmp[16384];
        for (;;) {
            const int r = SSL_read(_ssl, tmp, sizeof(tmp));
            if (r > 0) {
                out->append(tmp, (size_t)r);
                produced += r;
                continue;
            }
            const int e = SSL_get_error(_ssl, r);
            if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
            if (e == SSL_ERROR_ZERO_RETURN) {
                _peer_closed = true;
                break;
            }
            LOG(WARNING) << "SSL_read: " << last_ssl_error();
            errno = EPROTO;
            return -1;
        }
    }
    drain_wbio_locked();
    return produced;
}

std::string SslSession::cipher() const { return _ssl ? SSL_get_cipher_name(_ssl) : ""; }
std::string SslSession::version() const { return _ssl ? SSL_get_version(_ssl) : ""; }

}  // namespace mrpc
