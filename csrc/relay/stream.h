// Byte streams for the native data plane: a plain non-blocking TCP socket or
// a TLS session (OpenSSL) over one.  The pumps in relay_core.h move every
// body byte through this interface, so https origins and https S3 endpoints
// take the same GIL-free path as plain http (reference: the HTTP plug-in
// registers "https", internal/downloader/http/http.go:25-33; the uploader
// speaks TLS when S3_ENDPOINT is https, internal/uploader/uploader.go:31-33).
//
// Ownership: the Python control plane owns the socket fd.  A Stream never
// closes it; a TlsStream owns only its SSL object.  One thread drives a
// stream at a time (the event loop for heads, then a pump for the body).
//
// Cancellation: Stream::abort() is a sticky flag every pump loop checks
// (including waits on a download Flow), so Python can stop a pump without
// closing the fd under it, then wait for the pump to return.
//
// Also here: a throwaway PKI generator (EC P-256 CA + leaf with SANs) for
// the TLS fakes and tests — no `cryptography` package or openssl CLI needed.
#pragma once

#include <arpa/inet.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace tritondl_relay {

using Clock = std::chrono::steady_clock;
inline double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

inline std::string errno_str(const char* what) { return std::string(what) + ": " + std::strerror(errno); }

// 1 = ready, 0 = not yet (slice elapsed), -1 = error/hangup with no data
inline int wait_fd(int fd, short ev, int ms) {
  struct pollfd p {};
  p.fd = fd;
  p.events = ev;
  const int r = ::poll(&p, 1, ms);
  if (r < 0) return errno == EINTR ? 0 : -1;
  if (r == 0) return 0;
  if (p.revents & (ev | POLLHUP)) return 1;  // hangup: let recv/send report EOF / EPIPE
  return (p.revents & (POLLERR | POLLNVAL)) ? -1 : 1;
}

constexpr ssize_t IO_AGAIN = -1;  // would block: wait for *want (POLLIN / POLLOUT)
constexpr ssize_t IO_ERR = -2;    // hard error: *err set

class Stream {
 public:
  virtual ~Stream() = default;
  virtual int fd() const = 0;
  // > 0 bytes read, 0 = orderly end of stream, IO_AGAIN, IO_ERR
  virtual ssize_t recv_nb(char* p, size_t n, short* want, std::string* err) = 0;
  // > 0 bytes taken from the front of iov, IO_AGAIN, IO_ERR.  After IO_AGAIN
  // the caller must retry with the same (unconsumed) iov — a TLS record
  // already half on the wire is resumed, not re-encrypted.
  virtual ssize_t send_nb(const struct iovec* iov, int cnt, short* want, std::string* err) = 0;
  // true for a bare socket: the zero-copy kernel paths (splice, sendfile) apply
  virtual bool plain() const { return false; }
  // Push out bytes a stream buffered internally (TLS ciphertext): true when
  // nothing is pending; false with *want = POLLOUT (retry) or *err set.
  virtual bool flush_nb(short* want, std::string* err) {
    (void)want;
    (void)err;
    return true;
  }

  void abort() { aborted_.store(true); }
  bool aborted() const { return aborted_.load(std::memory_order_relaxed); }
  const std::atomic<bool>* abort_flag() const { return &aborted_; }

 protected:
  std::atomic<bool> aborted_{false};
};

class PlainStream : public Stream {
 public:
  explicit PlainStream(int fd) : fd_(fd) {}
  int fd() const override { return fd_; }
  bool plain() const override { return true; }
  ssize_t recv_nb(char* p, size_t n, short* want, std::string* err) override {
    for (;;) {
      const ssize_t r = ::recv(fd_, p, n, MSG_DONTWAIT);
      if (r >= 0) return r;
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        *want = POLLIN;
        return IO_AGAIN;
      }
      *err = errno_str("recv");
      return IO_ERR;
    }
  }
  ssize_t send_nb(const struct iovec* iov, int cnt, short* want, std::string* err) override {
    struct msghdr mh {};
    mh.msg_iov = const_cast<struct iovec*>(iov);
    mh.msg_iovlen = static_cast<size_t>(cnt);
    for (;;) {
      const ssize_t w = ::sendmsg(fd_, &mh, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (w >= 0) return w;
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        *want = POLLOUT;
        return IO_AGAIN;
      }
      *err = errno_str("send");
      return IO_ERR;
    }
  }

 private:
  int fd_;
};

// ---------------------------------------------------------------------------
// TLS

inline std::string ssl_errors(const std::string& what) {
  std::string s = what;
  char buf[256];
  bool first = true;
  for (unsigned long e; (e = ERR_get_error()) != 0;) {
    ERR_error_string_n(e, buf, sizeof buf);
    s += first ? ": " : "; ";
    s += buf;
    first = false;
  }
  return s;
}

inline bool is_ip_literal(const std::string& h) {
  unsigned char b[16];
  return ::inet_pton(AF_INET, h.c_str(), b) == 1 || ::inet_pton(AF_INET6, h.c_str(), b) == 1;
}

class TlsContext {
 public:
  // Client: trust `ca_pem` (PEM text, may hold several certs) and/or
  // `ca_file`, else the system store (honours SSL_CERT_FILE / SSL_CERT_DIR).
  static std::shared_ptr<TlsContext> client(const std::string& ca_pem, const std::string& ca_file, bool verify) {
    auto c = std::shared_ptr<TlsContext>(new TlsContext(false));
    c->verify_ = verify;
    if (verify) {
      SSL_CTX_set_verify(c->ctx_, SSL_VERIFY_PEER, nullptr);
      if (!ca_pem.empty()) c->add_ca_pem(ca_pem);
      if (!ca_file.empty() && SSL_CTX_load_verify_locations(c->ctx_, ca_file.c_str(), nullptr) != 1)
        throw std::runtime_error(ssl_errors("load CA file " + ca_file));
      if (ca_pem.empty() && ca_file.empty() && SSL_CTX_set_default_verify_paths(c->ctx_) != 1)
        throw std::runtime_error(ssl_errors("load system CA store"));
    } else {
      SSL_CTX_set_verify(c->ctx_, SSL_VERIFY_NONE, nullptr);
    }
    // resumption: keep the newest session (TLS 1.3 ticket) per host:port
    SSL_CTX_set_session_cache_mode(c->ctx_, SSL_SESS_CACHE_CLIENT | SSL_SESS_CACHE_NO_INTERNAL_STORE);
    SSL_CTX_sess_set_new_cb(c->ctx_, &TlsContext::on_new_session);
    return c;
  }
  // Server: leaf certificate first, then any chain certificates, all PEM.
  static std::shared_ptr<TlsContext> server(const std::string& cert_pem, const std::string& key_pem) {
    auto c = std::shared_ptr<TlsContext>(new TlsContext(true));
    BIO* b = BIO_new_mem_buf(cert_pem.data(), static_cast<int>(cert_pem.size()));
    X509* leaf = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
    if (!leaf || SSL_CTX_use_certificate(c->ctx_, leaf) != 1) {
      X509_free(leaf);
      BIO_free(b);
      throw std::runtime_error(ssl_errors("load server certificate"));
    }
    X509_free(leaf);
    for (X509* x; (x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr)) != nullptr;) {
      SSL_CTX_add1_chain_cert(c->ctx_, x);
      X509_free(x);
    }
    ERR_clear_error();  // the chain loop ends on a "no start line" error
    BIO_free(b);
    b = BIO_new_mem_buf(key_pem.data(), static_cast<int>(key_pem.size()));
    EVP_PKEY* k = PEM_read_bio_PrivateKey(b, nullptr, nullptr, nullptr);
    BIO_free(b);
    if (!k || SSL_CTX_use_PrivateKey(c->ctx_, k) != 1 || SSL_CTX_check_private_key(c->ctx_) != 1) {
      EVP_PKEY_free(k);
      throw std::runtime_error(ssl_errors("load server key"));
    }
    EVP_PKEY_free(k);
    return c;
  }
  ~TlsContext() {
    for (auto& kv : sessions_) SSL_SESSION_free(kv.second);
    SSL_CTX_free(ctx_);
  }
  TlsContext(const TlsContext&) = delete;
  TlsContext& operator=(const TlsContext&) = delete;

  static constexpr size_t kMaxSessions = 512;  // resumption tickets kept (one per host:port)

  SSL_CTX* ctx() const { return ctx_; }
  bool is_server() const { return server_; }
  bool verify() const { return verify_; }
  size_t cached_sessions() const {
    std::lock_guard<std::mutex> l(mu_);
    return sessions_.size();
  }

  // a new reference to the cached session for `key`, or nullptr
  SSL_SESSION* take_session(const std::string& key) {
    std::lock_guard<std::mutex> l(mu_);
    auto it = sessions_.find(key);
    if (it == sessions_.end()) return nullptr;
    if (!SSL_SESSION_is_resumable(it->second)) {
      SSL_SESSION_free(it->second);
      sessions_.erase(it);
      return nullptr;
    }
    SSL_SESSION_up_ref(it->second);
    return it->second;
  }
  void forget_session(const std::string& key) {
    std::lock_guard<std::mutex> l(mu_);
    auto it = sessions_.find(key);
    if (it != sessions_.end()) {
      SSL_SESSION_free(it->second);
      sessions_.erase(it);
    }
  }

  static int ex_index() {
    static const int i = SSL_get_ex_new_index(0, nullptr, nullptr, nullptr, nullptr);
    return i;
  }

 private:
  explicit TlsContext(bool server) : server_(server) {
    ctx_ = SSL_CTX_new(server ? TLS_server_method() : TLS_client_method());
    if (!ctx_) throw std::runtime_error(ssl_errors("SSL_CTX_new"));
    SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
    // retry-safe non-blocking writes from staging buffers that may move
    SSL_CTX_set_mode(ctx_, SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    // close-delimited bodies end with a bare TCP FIN on many servers; the HTTP
    // layer checks Content-Length, so a missing close_notify is not an error
    SSL_CTX_set_options(ctx_, SSL_OP_IGNORE_UNEXPECTED_EOF | SSL_OP_NO_COMPRESSION);
    // AES-128-GCM first: the cheapest AEAD with AES-NI/VAES on the host CPUs
    SSL_CTX_set_ciphersuites(ctx_, "TLS_AES_128_GCM_SHA256:TLS_AES_256_GCM_SHA384:TLS_CHACHA20_POLY1305_SHA256");
    SSL_CTX_set_cipher_list(ctx_, "ECDHE+AESGCM:ECDHE+CHACHA20:!aNULL:!MD5");
    // read several records per recv(2) on bulk bodies
    SSL_CTX_set_read_ahead(ctx_, 1);
    SSL_CTX_set_default_read_buffer_len(ctx_, 256 << 10);
  }
  void add_ca_pem(const std::string& pem) {
    BIO* b = BIO_new_mem_buf(pem.data(), static_cast<int>(pem.size()));
    X509_STORE* st = SSL_CTX_get_cert_store(ctx_);
    int n = 0;
    for (X509* x; (x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr)) != nullptr; ++n) {
      X509_STORE_add_cert(st, x);
      X509_free(x);
    }
    ERR_clear_error();
    BIO_free(b);
    if (n == 0) throw std::runtime_error("no certificate in CA PEM");
  }
  static int on_new_session(SSL* ssl, SSL_SESSION* sess);

  SSL_CTX* ctx_ = nullptr;
  bool server_ = false;
  bool verify_ = true;
  mutable std::mutex mu_;
  std::map<std::string, SSL_SESSION*> sessions_;
  friend class TlsStream;
};

// Write-side BIO: records are appended to the owning stream's out_ buffer
// (no copy beyond the encryption output itself); flush_nb() sends from it.
class TlsStream;
namespace detail {
BIO_METHOD* out_bio_method();
}

class TlsStream : public Stream {
 public:
  // `host`: server name for SNI + certificate verification (client side);
  // `session_key`: resumption cache key (typically "host:port").
  TlsStream(std::shared_ptr<TlsContext> ctx, int fd, const std::string& host, const std::string& session_key)
      : ctx_(std::move(ctx)), fd_(fd), key_(session_key) {
    ssl_ = SSL_new(ctx_->ctx());
    if (!ssl_) throw std::runtime_error(ssl_errors("SSL_new"));
    SSL_set_ex_data(ssl_, TlsContext::ex_index(), this);
    // Reads come straight from the socket (with read-ahead); records are
    // written into a memory BIO and sent in large batches (flush_nb): one
    // send(2) per ~256 KiB of ciphertext instead of one per 16 KiB record.
    BIO* rbio = BIO_new_socket(fd, BIO_NOCLOSE);
    wbio_ = BIO_new(detail::out_bio_method());
    if (!rbio || !wbio_) {
      BIO_free(rbio);
      BIO_free(wbio_);
      SSL_free(ssl_);
      throw std::runtime_error(ssl_errors("BIO_new"));
    }
    BIO_set_data(wbio_, this);
    BIO_set_init(wbio_, 1);
    SSL_set_bio(ssl_, rbio, wbio_);  // ssl_ owns both
    if (ctx_->is_server()) {
      SSL_set_accept_state(ssl_);
    } else {
      SSL_set_connect_state(ssl_);
      if (!host.empty()) {
        const bool ip = is_ip_literal(host);
        if (!ip) SSL_set_tlsext_host_name(ssl_, host.c_str());
        if (ctx_->verify()) {
          X509_VERIFY_PARAM* p = SSL_get0_param(ssl_);
          X509_VERIFY_PARAM_set_hostflags(p, X509_CHECK_FLAG_NO_PARTIAL_WILDCARDS);
          const int ok = ip ? X509_VERIFY_PARAM_set1_ip_asc(p, host.c_str())
                            : X509_VERIFY_PARAM_set1_host(p, host.c_str(), 0);
          if (ok != 1) {
            SSL_free(ssl_);
            throw std::runtime_error(ssl_errors("set verify host " + host));
          }
        }
      }
      if (!key_.empty()) {
        if (SSL_SESSION* s = ctx_->take_session(key_)) {
          SSL_set_session(ssl_, s);
          SSL_SESSION_free(s);
        }
      }
    }
  }
  ~TlsStream() override { SSL_free(ssl_); }
  TlsStream(const TlsStream&) = delete;
  TlsStream& operator=(const TlsStream&) = delete;

  int fd() const override { return fd_; }
  const std::string& session_key() const { return key_; }

  // One non-blocking handshake step: 0 = done, POLLIN / POLLOUT = wait for
  // that, -1 = failed (*err says why, incl. the certificate verdict).
  int handshake_step(std::string* err) {
    short fw = POLLOUT;
    if (!flush_nb(&fw, err)) return err->empty() ? POLLOUT : -1;  // earlier flight still leaving
    ERR_clear_error();
    const int r = SSL_do_handshake(ssl_);
    const int e = r == 1 ? SSL_ERROR_NONE : SSL_get_error(ssl_, r);
    if (!flush_nb(&fw, err)) return err->empty() ? POLLOUT : -1;  // this flight: send before waiting
    if (r == 1) return 0;
    if (e == SSL_ERROR_WANT_READ) return POLLIN;
    if (e == SSL_ERROR_WANT_WRITE) return POLLOUT;
    std::string msg = ssl_errors("tls handshake");
    const long v = SSL_get_verify_result(ssl_);
    if (v != X509_V_OK) msg += std::string(" (certificate verify: ") + X509_verify_cert_error_string(v) + ")";
    if (e == SSL_ERROR_SYSCALL && errno) msg += " (" + errno_str("socket") + ")";
    if (e == SSL_ERROR_SYSCALL && !errno && msg == "tls handshake") msg += ": peer closed the connection";
    if (!ctx_->is_server() && !key_.empty()) ctx_->forget_session(key_);
    *err = msg;
    return -1;
  }
  // Blocking handshake with poll (GIL released by the binding).
  std::string handshake(double timeout_s) {
    const auto t0 = Clock::now();
    for (;;) {
      std::string err;
      const int w = handshake_step(&err);
      if (w == 0) return "";
      if (w < 0) return err;
      if (aborted()) return "cancelled";
      if (since(t0) > timeout_s) return "tls handshake timeout";
      if (wait_fd(fd_, static_cast<short>(w), 50) < 0) return "socket error during tls handshake";
    }
  }

  ssize_t recv_nb(char* p, size_t n, short* want, std::string* err) override {
    ERR_clear_error();
    size_t got = 0;
    const int ok = SSL_read_ex(ssl_, p, n, &got);
    const int e = ok == 1 ? SSL_ERROR_NONE : SSL_get_error(ssl_, 0);
    if (out_pending()) {  // reading can produce records to send (key update, alerts)
      short w = POLLOUT;
      std::string ferr;
      flush_nb(&w, &ferr);
    }
    if (ok == 1) return static_cast<ssize_t>(got);
    return fail(e, "tls recv", want, err);
  }

  size_t out_pending() const { return out_.size() - out_off_; }
  void out_append(const char* p, size_t n) {
    if (out_off_ && out_off_ == out_.size()) {
      out_.clear();
      out_off_ = 0;
    }
    out_.insert(out_.end(), p, p + n);
  }

  bool flush_nb(short* want, std::string* err) override {
    for (;;) {
      const size_t n = out_pending();
      if (n == 0) {
        out_.clear();
        out_off_ = 0;
        return true;
      }
      const ssize_t w = ::send(fd_, out_.data() + out_off_, n, MSG_NOSIGNAL | MSG_DONTWAIT);
      if (w > 0) {
        out_off_ += static_cast<size_t>(w);
        continue;
      }
      if (w < 0 && errno == EINTR) continue;
      if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
        *want = POLLOUT;
        return false;
      }
      *err = errno_str("tls send");
      return false;
    }
  }

  ssize_t send_nb(const struct iovec* iov, int cnt, short* want, std::string* err) override {
    // OpenSSL has no writev: a large leading buffer goes out directly, small
    // pieces (aws-chunk headers, CRLFs) are gathered into a staging buffer.
    // Both choices depend only on the iov, so a retry after IO_AGAIN repeats
    // exactly the same write, as SSL_write requires.
    const char* src;
    size_t len;
    if (cnt == 1 || iov[0].iov_len >= kDirect) {
      src = static_cast<const char*>(iov[0].iov_base);
      len = std::min(iov[0].iov_len, kMaxWrite);
    } else {
      stage_.clear();
      for (int i = 0; i < cnt && stage_.size() < kStage; ++i) {
        const size_t take = std::min(iov[i].iov_len, kStage - stage_.size());
        const char* b = static_cast<const char*>(iov[i].iov_base);
        stage_.insert(stage_.end(), b, b + take);
      }
      src = stage_.data();
      len = stage_.size();
    }
    if (len == 0) return 0;
    // bounded ciphertext backlog: flush what is pending before encrypting more
    if (out_pending() >= kBacklog && !flush_nb(want, err)) {
      if (!err->empty()) return IO_ERR;
      if (out_pending() >= kBacklog) return IO_AGAIN;
    }
    ERR_clear_error();
    size_t w = 0;
    if (SSL_write_ex(ssl_, src, len, &w) != 1) return fail(SSL_get_error(ssl_, 0), "tls send", want, err);
    short fw = POLLOUT;
    if (!flush_nb(&fw, err) && !err->empty()) return IO_ERR;  // a backlog left here goes out on the next call
    return static_cast<ssize_t>(w);
  }

  // Decrypted bytes already buffered (readable without touching the socket).
  size_t pending() const { return static_cast<size_t>(SSL_pending(ssl_)); }

  // Pooled-connection liveness: processes stray records (session tickets,
  // close_notify) without consuming application data.  true = idle and open.
  bool alive() {
    char c;
    ERR_clear_error();
    size_t got = 0;
    if (SSL_peek_ex(ssl_, &c, 1, &got) == 1) return false;  // unexpected bytes: not reusable
    const int e = SSL_get_error(ssl_, 0);
    ERR_clear_error();
    return e == SSL_ERROR_WANT_READ;
  }

  // Best-effort close_notify (non-blocking, one attempt).
  void shutdown_notify() {
    ERR_clear_error();
    SSL_shutdown(ssl_);
    ERR_clear_error();
    short w = POLLOUT;
    std::string err;
    flush_nb(&w, &err);
  }

  // ALPN (RFC 7301), client side, before the handshake: protocols in order of preference.
  void set_alpn(const std::vector<std::string>& protos) {
    std::string wire;
    for (const std::string& p : protos) {
      if (p.empty() || p.size() > 255) throw std::invalid_argument("bad ALPN protocol name");
      wire += char(p.size());
      wire += p;
    }
    if (SSL_set_alpn_protos(ssl_, reinterpret_cast<const unsigned char*>(wire.data()),
                            static_cast<unsigned>(wire.size())) != 0)
      throw std::runtime_error(ssl_errors("SSL_set_alpn_protos"));
  }
  // The protocol the server picked ("" = none).
  std::string alpn() const {
    const unsigned char* p = nullptr;
    unsigned n = 0;
    SSL_get0_alpn_selected(ssl_, &p, &n);
    return p ? std::string(reinterpret_cast<const char*>(p), n) : std::string();
  }

  std::string version() const { return SSL_get_version(ssl_); }
  std::string cipher() const {
    const SSL_CIPHER* c = SSL_get_current_cipher(ssl_);
    return c ? SSL_CIPHER_get_name(c) : "";
  }
  bool resumed() const { return SSL_session_reused(ssl_) == 1; }
  SSL* ssl() const { return ssl_; }
  TlsContext* context() const { return ctx_.get(); }

 private:
  ssize_t fail(int e, const char* what, short* want, std::string* err) {
    switch (e) {
      case SSL_ERROR_ZERO_RETURN:
        return 0;
      case SSL_ERROR_WANT_READ:
        *want = POLLIN;
        return IO_AGAIN;
      case SSL_ERROR_WANT_WRITE:
        *want = POLLOUT;
        return IO_AGAIN;
      case SSL_ERROR_SYSCALL:
        if (errno == 0) return 0;  // EOF without close_notify (tolerated, see context options)
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
          *want = POLLIN | POLLOUT;
          return IO_AGAIN;
        }
        *err = errno_str(what);
        return IO_ERR;
      default:
        *err = ssl_errors(what);
        return IO_ERR;
    }
  }

  static constexpr size_t kDirect = 16 << 10;
  static constexpr size_t kMaxWrite = 256 << 10;  // plaintext per SSL_write: ~16 records, one flush
  static constexpr size_t kStage = 256 << 10;
  static constexpr size_t kBacklog = 1 << 20;     // unsent ciphertext held before the writer must wait
  std::shared_ptr<TlsContext> ctx_;
  SSL* ssl_ = nullptr;
  BIO* wbio_ = nullptr;                           // owned by ssl_
  std::vector<char> out_;                         // ciphertext not yet sent: [out_off_, size)
  size_t out_off_ = 0;
  int fd_;
  std::string key_;
  std::vector<char> stage_;
};

namespace detail {
inline int out_bio_write(BIO* b, const char* p, int n) {
  if (n <= 0) return 0;
  static_cast<TlsStream*>(BIO_get_data(b))->out_append(p, static_cast<size_t>(n));
  return n;
}
inline long out_bio_ctrl(BIO* b, int cmd, long num, void* ptr) {
  (void)num;
  (void)ptr;
  switch (cmd) {
    case BIO_CTRL_FLUSH:
      return 1;  // flushed for real by TlsStream::flush_nb
    case BIO_CTRL_WPENDING:
    case BIO_CTRL_PENDING:
      return static_cast<long>(static_cast<TlsStream*>(BIO_get_data(b))->out_pending());
    default:
      return 0;
  }
}
inline BIO_METHOD* out_bio_method() {
  static BIO_METHOD* m = [] {
    BIO_METHOD* x = BIO_meth_new(BIO_get_new_index() | BIO_TYPE_SOURCE_SINK, "tritondl tls out");
    BIO_meth_set_write(x, out_bio_write);
    BIO_meth_set_ctrl(x, out_bio_ctrl);
    return x;
  }();
  return m;
}
}  // namespace detail

inline int TlsContext::on_new_session(SSL* ssl, SSL_SESSION* sess) {
  auto* st = static_cast<TlsStream*>(SSL_get_ex_data(ssl, ex_index()));
  if (!st || st->session_key().empty()) return 0;
  TlsContext* c = st->context();
  std::lock_guard<std::mutex> l(c->mu_);
  auto it = c->sessions_.find(st->session_key());
  if (it != c->sessions_.end()) {
    SSL_SESSION_free(it->second);
  } else if (c->sessions_.size() >= TlsContext::kMaxSessions) {
    // a worker that meets thousands of origins keeps tickets for a bounded few
    auto victim = c->sessions_.begin();
    SSL_SESSION_free(victim->second);
    c->sessions_.erase(victim);
  }
  c->sessions_[st->session_key()] = sess;
  return 1;  // we keep the reference
}

// ---------------------------------------------------------------------------
// Test PKI: self-signed EC P-256 CA + one leaf for `hosts` (DNS names and/or
// IP literals as subjectAltName).  Returns {ca_pem, leaf_cert_pem, leaf_key_pem}.

struct TestPki {
  std::string ca_pem, cert_pem, key_pem;
};

namespace detail {
inline std::string pem_of(X509* x) {
  BIO* b = BIO_new(BIO_s_mem());
  PEM_write_bio_X509(b, x);
  char* p = nullptr;
  const long n = BIO_get_mem_data(b, &p);
  std::string s(p, static_cast<size_t>(n));
  BIO_free(b);
  return s;
}
inline std::string pem_of(EVP_PKEY* k) {
  BIO* b = BIO_new(BIO_s_mem());
  PEM_write_bio_PrivateKey(b, k, nullptr, nullptr, 0, nullptr, nullptr);
  char* p = nullptr;
  const long n = BIO_get_mem_data(b, &p);
  std::string s(p, static_cast<size_t>(n));
  BIO_free(b);
  return s;
}
inline void add_ext(X509* issuer, X509* subj, int nid, const std::string& value) {
  X509V3_CTX c;
  X509V3_set_ctx_nodb(&c);
  X509V3_set_ctx(&c, issuer, subj, nullptr, nullptr, 0);
  X509_EXTENSION* e = X509V3_EXT_conf_nid(nullptr, &c, nid, value.c_str());
  if (!e) throw std::runtime_error(ssl_errors("x509 extension " + value));
  X509_add_ext(subj, e, -1);
  X509_EXTENSION_free(e);
}
inline X509* new_cert(EVP_PKEY* key, const std::string& cn, long serial, long days) {
  X509* x = X509_new();
  X509_set_version(x, 2);
  ASN1_INTEGER_set(X509_get_serialNumber(x), serial);
  X509_gmtime_adj(X509_getm_notBefore(x), -3600);
  X509_gmtime_adj(X509_getm_notAfter(x), days * 86400L);
  X509_set_pubkey(x, key);
  X509_NAME* n = X509_get_subject_name(x);
  X509_NAME_add_entry_by_txt(n, "O", MBSTRING_ASC, reinterpret_cast<const unsigned char*>("tritondl test"), -1, -1, 0);
  X509_NAME_add_entry_by_txt(n, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>(cn.c_str()), -1, -1, 0);
  return x;
}
}  // namespace detail

inline TestPki make_test_pki(const std::vector<std::string>& hosts, long days = 30) {
  using namespace detail;
  if (hosts.empty()) throw std::runtime_error("make_test_pki: no hosts");
  EVP_PKEY* ca_key = EVP_EC_gen("P-256");
  EVP_PKEY* leaf_key = EVP_EC_gen("P-256");
  if (!ca_key || !leaf_key) throw std::runtime_error(ssl_errors("EC key generation"));
  X509* ca = new_cert(ca_key, "tritondl test CA", 1, days);
  X509_set_issuer_name(ca, X509_get_subject_name(ca));
  add_ext(ca, ca, NID_basic_constraints, "critical,CA:TRUE");
  add_ext(ca, ca, NID_key_usage, "critical,keyCertSign,cRLSign");
  add_ext(ca, ca, NID_subject_key_identifier, "hash");
  X509_sign(ca, ca_key, EVP_sha256());
  X509* leaf = new_cert(leaf_key, hosts[0], 2, days);
  X509_set_issuer_name(leaf, X509_get_subject_name(ca));
  std::string san;
  for (const auto& h : hosts) san += (san.empty() ? "" : ",") + std::string(is_ip_literal(h) ? "IP:" : "DNS:") + h;
  add_ext(ca, leaf, NID_subject_alt_name, san);
  add_ext(ca, leaf, NID_basic_constraints, "critical,CA:FALSE");
  add_ext(ca, leaf, NID_key_usage, "critical,digitalSignature");
  add_ext(ca, leaf, NID_ext_key_usage, "serverAuth");
  add_ext(ca, leaf, NID_authority_key_identifier, "keyid");
  if (X509_sign(leaf, ca_key, EVP_sha256()) <= 0) throw std::runtime_error(ssl_errors("sign leaf"));
  TestPki out{pem_of(ca), pem_of(leaf), pem_of(leaf_key)};
  X509_free(leaf);
  X509_free(ca);
  EVP_PKEY_free(leaf_key);
  EVP_PKEY_free(ca_key);
  return out;
}

}  // namespace tritondl_relay
