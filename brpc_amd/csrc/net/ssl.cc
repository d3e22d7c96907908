#include "net/ssl.h"

#include <openssl/err.h>
#include <openssl/ssl.h>

#include <cerrno>
#include <mutex>

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

std::shared_ptr<SslContext> SslContext::NewServer(const ServerSslOptions& opt, std::string* err) {
    init_openssl_once();
    std::shared_ptr<SslContext> c(new SslContext);
    c->_server = true;
    c->_ctx = SSL_CTX_new(TLS_server_method());
    if (!c->_ctx) {
        *err = last_ssl_error();
        return nullptr;
    }
    SSL_CTX_set_min_proto_version(c->_ctx, TLS1_2_VERSION);
    SSL_CTX_set_mode(c->_ctx, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    if (SSL_CTX_use_certificate_chain_file(c->_ctx, opt.cert_file.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(c->_ctx, opt.key_file.c_str(), SSL_FILETYPE_PEM) != 1 ||
        SSL_CTX_check_private_key(c->_ctx) != 1) {
        *err = "certificate/key " + opt.cert_file + "/" + opt.key_file + ": " + last_ssl_error();
        return nullptr;
    }
    if (!opt.ciphers.empty() && SSL_CTX_set_cipher_list(c->_ctx, opt.ciphers.c_str()) != 1) {
        *err = "ciphers: " + last_ssl_error();
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
        SSL_CTX_set_alpn_select_cb(c->_ctx, alpn_select_cb, wire.get());
        std::lock_guard<std::mutex> g(mu);
        keep.push_back(std::move(wire));
    }
    return c;
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
