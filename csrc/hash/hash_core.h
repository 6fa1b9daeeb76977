// Host hashing core (OpenSSL EVP; no Python) — shared by the pybind11 module
// hash_host.cpp and the sanitizer self-test csrc/tests/native_selftest.cpp.
//
// Everything here is thread-safe and allocation-bounded by its inputs.
#pragma once

#include <openssl/evp.h>
#include <openssl/hmac.h>
// The low-level SHA256_* API is deprecated in OpenSSL 3 but still exported; the
// HMAC chain below needs plain copyable SHA-256 states (EVP contexts allocate on
// every copy, and one-shot HMAC() re-fetches the MAC implementation per call).
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/sha.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <pthread.h>
#include <utility>
#include <vector>

#include "sha1_mb.h"
#include "sha256_mb.h"
#include "sha_ni.h"

namespace tritondl_hash {

// OpenSSL 3: sha256_md() & co. are legacy handles, and every
// EVP_DigestInit_ex with one re-fetches the provider implementation through a
// locked store — with many small digests on many threads (16 KiB merkle
// leaves, 64 KiB aws-chunks) that lock serialised the workers (v2 verify ran
// at 1/3 of SHA-256 speed on 16 threads).  Fetch each algorithm once.
inline const EVP_MD* fetched_md(const char* name, const EVP_MD* legacy) {
  const EVP_MD* m = EVP_MD_fetch(nullptr, name, nullptr);  // leaked on purpose: process lifetime
  return m ? m : legacy;
}
inline const EVP_MD* sha256_md() {
  static const EVP_MD* m = fetched_md("SHA256", EVP_sha256());
  return m;
}
inline const EVP_MD* sha1_md() {
  static const EVP_MD* m = fetched_md("SHA1", EVP_sha1());
  return m;
}
inline const EVP_MD* md5_md() {
  static const EVP_MD* m = fetched_md("MD5", EVP_md5());
  return m;
}

inline const EVP_MD* md_for(const std::string& kind) {
  if (kind == "sha1") return sha1_md();
  if (kind == "sha256") return sha256_md();
  if (kind == "md5") return md5_md();
  throw std::invalid_argument("unknown hash kind: " + kind);
}

struct MdCtx {
  EVP_MD_CTX* ctx;
  explicit MdCtx(const EVP_MD* md) : ctx(EVP_MD_CTX_new()) {
    if (!ctx || EVP_DigestInit_ex(ctx, md, nullptr) != 1) throw std::runtime_error("EVP init failed");
  }
  ~MdCtx() { EVP_MD_CTX_free(ctx); }
  MdCtx(const MdCtx&) = delete;
  MdCtx& operator=(const MdCtx&) = delete;
  void update(const void* p, size_t n) {
    if (n && EVP_DigestUpdate(ctx, p, n) != 1) throw std::runtime_error("EVP update failed");
  }
  std::string final() {
    unsigned char out[EVP_MAX_MD_SIZE];
    unsigned int len = 0;
    if (EVP_DigestFinal_ex(ctx, out, &len) != 1) throw std::runtime_error("EVP final failed");
    return std::string(reinterpret_cast<char*>(out), len);
  }
};

inline std::string one_shot(const EVP_MD* md, const void* p, size_t n) {
  MdCtx c(md);
  c.update(p, n);
  return c.final();
}

// SHA-256 of one / two buffers into raw 32-byte digests: SHA-NI (two
// messages in lockstep, sha_ni.h) when the CPU has it, else OpenSSL.
inline void sha256_raw(const void* p, size_t n, unsigned char out[32]) {
  if (sha2x::cpu_has_sha_ni()) {
    sha2x::sha256_x1(p, n, out);
    return;
  }
  unsigned int len = 32;
  EVP_Digest(n ? p : "", n, out, &len, sha256_md(), nullptr);
}
inline void sha256_pair(const void* a, size_t na, const void* b, size_t nb, unsigned char oa[32],
                        unsigned char ob[32]) {
  if (sha2x::cpu_has_sha_ni()) {
    sha2x::sha256_x2(a, na, b, nb, oa, ob);
    return;
  }
  sha256_raw(a, na, oa);
  sha256_raw(b, nb, ob);
}

// SHA-256 of n messages into out[32*i]: every run of 16 equal-length
// messages goes through the 16-lane AVX-512 kernel (sha256_mb.h, ~1.45x
// SHA-NI pairs per core on the Zen 5 host), the rest in SHA-NI pairs.
inline void sha256_batch(const void* const* p, const size_t* len, size_t n, unsigned char* out) {
  size_t i = 0;
  if (n >= 16 && sha16::cpu_has_avx512()) {
    while (i + 16 <= n) {
      bool same = true;
      for (size_t j = 1; j < 16 && same; ++j) same = len[i + j] == len[i];
      if (!same) break;
      sha16::sha256_x16(p + i, len[i], out + 32 * i);
      i += 16;
    }
  }
  for (; i + 1 < n; i += 2) sha256_pair(p[i], len[i], p[i + 1], len[i + 1], out + 32 * i, out + 32 * (i + 1));
  if (i < n) sha256_raw(p[i], len[i], out + 32 * i);
}
// Chunks per hashing claim that keep the widest kernel fed.
inline size_t sha256_claim() { return sha16::cpu_has_avx512() ? 16 : 2; }

// Raw digest with an EVP algorithm; SHA-1 / SHA-256 take the SHA-NI path.
inline void md_raw(const EVP_MD* md, const void* p, size_t n, unsigned char* out) {
  if (sha2x::cpu_has_sha_ni()) {
    if (md == sha256_md()) return sha2x::sha256_x1(p, n, out);
    if (md == sha1_md()) return sha2x::sha1_x1(p, n, out);
  }
  unsigned int len = 0;
  EVP_Digest(n ? p : "", n, out, &len, md, nullptr);
}
// Two messages: in lockstep on SHA-NI (SHA-1 / SHA-256), else one by one.
inline void md_pair(const EVP_MD* md, const void* a, size_t na, const void* b, size_t nb, unsigned char* oa,
                    unsigned char* ob) {
  if (sha2x::cpu_has_sha_ni()) {
    if (md == sha256_md()) return sha2x::sha256_x2(a, na, b, nb, oa, ob);
    if (md == sha1_md()) return sha2x::sha1_x2(a, na, b, nb, oa, ob);
  }
  md_raw(md, a, na, oa);
  md_raw(md, b, nb, ob);
}

// Digests of n messages into out + i*digest_size: runs of 16 equal-length
// messages take the 16-lane AVX-512 kernels (SHA-1 and SHA-256), the rest
// SHA-NI pairs; other algorithms one by one.
inline void md_batch(const EVP_MD* md, const void* const* p, const size_t* len, size_t n, unsigned char* out) {
  if (md == sha256_md()) return sha256_batch(p, len, n, out);
  const size_t dl = static_cast<size_t>(EVP_MD_size(md));
  size_t i = 0;
  if (md == sha1_md() && n >= 16 && sha16::cpu_has_avx512()) {
    while (i + 16 <= n) {
      bool same = true;
      for (size_t j = 1; j < 16 && same; ++j) same = len[i + j] == len[i];
      if (!same) break;
      sha16::sha1_x16(p + i, len[i], out + dl * i);
      i += 16;
    }
  }
  for (; i + 1 < n; i += 2) md_pair(md, p[i], len[i], p[i + 1], len[i + 1], out + dl * i, out + dl * (i + 1));
  if (i < n) md_raw(md, p[i], len[i], out + dl * i);
}
// Messages per claim that keep the widest kernel for `md` fed.
inline size_t md_claim(const EVP_MD* md) {
  return (md == sha1_md() || md == sha256_md()) && sha16::cpu_has_avx512() ? 16 : 2;
}

inline std::string hex_raw(const unsigned char* d, size_t n) {
  static const char* hx = "0123456789abcdef";
  std::string out(n * 2, '0');
  for (size_t i = 0; i < n; ++i) {
    out[2 * i] = hx[d[i] >> 4];
    out[2 * i + 1] = hx[d[i] & 15];
  }
  return out;
}

inline std::string hex(const std::string& d) {
  static const char* hx = "0123456789abcdef";
  std::string out;
  out.reserve(d.size() * 2);
  for (unsigned char ch : d) {
    out.push_back(hx[ch >> 4]);
    out.push_back(hx[ch & 15]);
  }
  return out;
}

inline std::string hmac256(const std::string& key, const std::string& msg) {
  unsigned char out[32];
  unsigned int len = 32;
  if (!HMAC(EVP_sha256(), key.data(), static_cast<int>(key.size()),
            reinterpret_cast<const unsigned char*>(msg.data()), msg.size(), out, &len))
    throw std::runtime_error("HMAC failed");
  return std::string(reinterpret_cast<char*>(out), len);
}

// HMAC-SHA256 with the key's inner/outer pad blocks absorbed once: each MAC
// is a struct copy + the message blocks + one outer block (4.2 -> ~0.5 us per
// aws-chunked chunk signature, which is a serial chain on the PUT's critical
// path — 160 links per 10 MiB object).
class HmacSha256 {
 public:
  explicit HmacSha256(const std::string& key) {
    unsigned char k[64] = {0};
    if (key.size() > 64) {
      SHA256(reinterpret_cast<const unsigned char*>(key.data()), key.size(), k);
    } else if (!key.empty()) {
      std::memcpy(k, key.data(), key.size());
    }
    unsigned char ip[64], op[64];
    for (int i = 0; i < 64; ++i) {
      ip[i] = static_cast<unsigned char>(k[i] ^ 0x36);
      op[i] = static_cast<unsigned char>(k[i] ^ 0x5c);
    }
    SHA256_Init(&inner_);
    SHA256_Update(&inner_, ip, 64);
    SHA256_Init(&outer_);
    SHA256_Update(&outer_, op, 64);
  }
  void mac(const void* msg, size_t n, unsigned char out[32]) const {
    SHA256_CTX c = inner_;
    unsigned char ih[32];
    SHA256_Update(&c, msg, n);
    SHA256_Final(ih, &c);
    c = outer_;
    SHA256_Update(&c, ih, 32);
    SHA256_Final(out, &c);
  }

 private:
  SHA256_CTX inner_, outer_;
};

inline void hex_into(const unsigned char* d, size_t n, char* out) {
  static const char* hx = "0123456789abcdef";
  for (size_t i = 0; i < n; ++i) {
    out[2 * i] = hx[d[i] >> 4];
    out[2 * i + 1] = hx[d[i] & 15];
  }
}

// aws-chunked (STREAMING-AWS4-HMAC-SHA256-PAYLOAD) signature chain.  The
// string to sign is kept in one buffer whose previous-signature and
// chunk-hash fields are overwritten in place:
//   "AWS4-HMAC-SHA256-PAYLOAD\n" amzdate "\n" scope "\n" prev "\n" hex(sha256("")) "\n" hex(sha256(chunk))
class SigChain {
 public:
  SigChain(const std::string& signing_key, const std::string& amzdate, const std::string& scope,
           const std::string& seed)
      : mac_(signing_key), head_("AWS4-HMAC-SHA256-PAYLOAD\n" + amzdate + "\n" + scope + "\n") {
    layout(seed);
  }
  // signature (hex) of the next chunk, given the hex SHA-256 of its data
  const std::string& next(const char* chunk_hash_hex) {
    std::memcpy(&buf_[hash_off_], chunk_hash_hex, 64);
    unsigned char sig[32];
    mac_.mac(buf_.data(), buf_.size(), sig);
    char hx[64];
    hex_into(sig, 32, hx);
    if (prev_.size() != 64) {
      layout(std::string(hx, 64));    // a seed of unusual length: every later link is 64 chars
    } else {
      std::memcpy(&prev_[0], hx, 64);
      std::memcpy(&buf_[prev_off_], hx, 64);
    }
    return prev_;
  }
  const std::string& next(const std::string& chunk_hash_hex) {
    if (chunk_hash_hex.size() != 64) throw std::invalid_argument("chunk hash must be 64 hex chars");
    return next(chunk_hash_hex.data());
  }
  const std::string& prev() const { return prev_; }

 private:
  void layout(const std::string& prev) {
    static const char empty[] = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855";
    prev_ = prev;
    buf_ = head_;
    prev_off_ = buf_.size();
    buf_ += prev + "\n" + empty + "\n";
    hash_off_ = buf_.size();
    buf_.append(64, '0');
  }
  HmacSha256 mac_;
  std::string head_, buf_, prev_;
  size_t prev_off_ = 0, hash_off_ = 0;
};

// pread that loops over short reads; returns bytes read (may be < n at EOF)
inline size_t pread_full(int fd, char* dst, size_t n, off_t off) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = ::pread(fd, dst + got, n - got, off + static_cast<off_t>(got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return got;
    }
    if (r == 0) break;
    got += static_cast<size_t>(r);
  }
  return got;
}

// Name the calling thread (<= 15 chars) so per-thread CPU accounting
// (-cpuprofile, top -H, /proc/<pid>/task/*/comm) can tell the pools apart.
inline void name_thread(const char* name) { pthread_setname_np(pthread_self(), name); }

// Process-wide pool of parked worker threads.  A worker ran its hasher pools
// on fresh std::threads per call — per 10 MiB job that was 8 thread creations
// and joins for the PUT's chunk hashers alone — and threads that exited
// within a profiler tick were invisible to per-thread CPU accounting.
// Tasks may block (on a ring slot, on download progress), so the pool never
// queues a task behind a busy worker: it starts another thread instead, and
// keeps at most `max_idle` parked.  Each task names its thread while it runs.
class TaskPool {
 public:
  struct Group {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
    void wait() {
      std::unique_lock<std::mutex> l(mu);
      cv.wait(l, [&] { return left == 0; });
    }
  };

  static TaskPool& get() {
    static TaskPool* p = new TaskPool();  // never destroyed: threads stay parked until exit
    return *p;
  }

  // Run `fn` on `copies` threads at once; the returned group's wait() joins them.
  std::shared_ptr<Group> run(int copies, std::function<void()> fn, const char* name) {
    auto g = std::make_shared<Group>();
    g->left = copies;
    auto shared_fn = std::make_shared<std::function<void()>>(std::move(fn));
    std::lock_guard<std::mutex> l(mu_);
    for (int k = 0; k < copies; ++k) q_.push_back(Task{shared_fn, g, name});
    const size_t want = q_.size();
    while (idle_ < want) {
      ++idle_;  // counted idle until it takes a task
      ++threads_;
      std::thread([this] { loop(); }).detach();
    }
    // one parked thread per task: notify_all woke every parked thread (a
    // dozen once pumps and hashers share the pool) to fight over mu_ for
    // one or two tasks
    for (int k = 0; k < copies; ++k) cv_.notify_one();
    return g;
  }
  size_t threads() const {
    std::lock_guard<std::mutex> l(mu_);
    return threads_;
  }

 private:
  struct Task {
    std::shared_ptr<std::function<void()>> fn;
    std::shared_ptr<Group> g;
    const char* name;
  };
  static constexpr size_t max_idle = 64;

  void loop() {
    const char* named = nullptr;
    std::unique_lock<std::mutex> l(mu_);
    for (;;) {
      cv_.wait(l, [&] { return !q_.empty(); });
      Task t = std::move(q_.front());
      q_.erase(q_.begin());
      --idle_;
      l.unlock();
      if (t.name != named) {  // pthread_setname_np is a write to /proc: only on a change of task kind
        name_thread(t.name);
        named = t.name;
      }
      (*t.fn)();
      {
        std::lock_guard<std::mutex> gl(t.g->mu);
        if (--t.g->left == 0) t.g->cv.notify_all();
      }
      // keeps the task's name while parked: CPU accounting that samples names
      // (-cpuprofile) charges the work just done to that task kind
      t = Task{};
      l.lock();
      if (idle_ >= max_idle) {
        --threads_;
        return;
      }
      ++idle_;
    }
  }

  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Task> q_;
  size_t idle_ = 0, threads_ = 0;
};

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  if (threads <= 1 || n <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  int t = static_cast<int>(std::min<size_t>(static_cast<size_t>(threads), n));
  TaskPool::get().run(t, [&] {
    for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
  }, "tdl-hash")->wait();
}

inline int default_threads() {
  unsigned h = std::thread::hardware_concurrency();
  return h ? static_cast<int>(std::min(h, 32u)) : 4;
}

// Concatenated per-piece digests of a contiguous buffer.
inline std::string piece_hashes(const EVP_MD* md, const char* data, size_t len, size_t piece_len, int threads) {
  if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  const size_t n = (len + piece_len - 1) / piece_len;
  const size_t dl = static_cast<size_t>(EVP_MD_size(md));
  std::string out(n * dl, '\0');
  const size_t g = md_claim(md);  // pieces per task: 16 for the AVX-512 kernels, else a SHA-NI pair
  parallel_for((n + g - 1) / g, threads <= 0 ? default_threads() : threads, [&](size_t k) {
    const size_t i0 = k * g, cnt = std::min(g, n - i0);
    const void* p[16];
    size_t m[16];
    for (size_t j = 0; j < cnt; ++j) {
      const size_t a = (i0 + j) * piece_len;
      p[j] = data + a;
      m[j] = std::min(piece_len, len - a);
    }
    md_batch(md, p, m, cnt, reinterpret_cast<unsigned char*>(&out[i0 * dl]));
  });
  return out;
}

struct FileSpan {
  std::string path;  // empty: a BEP 47 padding file (zeros)
  long long length;
  long long start;  // offset of this file in the torrent's concatenated stream
};

// Verify a torrent's pieces against the concatenated file layout; one byte per
// piece (1 = verified, 0 = mismatch / missing / short data).
inline std::string verify_pieces(const std::vector<std::pair<std::string, long long>>& files, size_t piece_len,
                                 const std::string& expected, int threads, const EVP_MD* md) {
  const size_t dl = static_cast<size_t>(EVP_MD_size(md));
  if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  if (expected.size() % dl) throw std::invalid_argument("expected digest blob has wrong size");
  std::vector<FileSpan> spans;
  long long total = 0;
  for (auto& f : files) {
    if (f.second < 0) throw std::invalid_argument("negative file length");
    spans.push_back({f.first, f.second, total});
    total += f.second;
  }
  const size_t n = expected.size() / dl;
  const size_t need = total > 0 ? (static_cast<size_t>(total) + piece_len - 1) / piece_len : 0;
  if (n != need) throw std::invalid_argument("piece count does not match total length");
  std::string ok(n, '\0');
  std::vector<int> fds(spans.size(), -1);
  for (size_t i = 0; i < spans.size(); ++i)
    if (!spans[i].path.empty()) fds[i] = ::open(spans[i].path.c_str(), O_RDONLY | O_CLOEXEC);
  // read [pstart, pstart + plen) of the layout into dst; false if a file is
  // missing or short
  auto read_at = [&](long long pstart, long long plen, char* dst) -> bool {
    long long filled = 0;
    size_t lo = 0, hi = spans.size();  // last span starting at or before pstart
    while (hi - lo > 1) {
      size_t mid = (lo + hi) / 2;
      if (spans[mid].start <= pstart) lo = mid; else hi = mid;
    }
    for (size_t s = lo; s < spans.size() && filled < plen; ++s) {
      const long long fstart = spans[s].start, flen = spans[s].length;
      const long long a = std::max(pstart + filled, fstart);
      const long long e = std::min(pstart + plen, fstart + flen);
      if (e <= a) continue;
      const size_t want = static_cast<size_t>(e - a);
      if (a == pstart + filled && spans[s].path.empty()) {  // BEP 47 padding file: zeros, not on disk
        std::memset(dst + filled, 0, want);
        filled += static_cast<long long>(want);
        continue;
      }
      if (a != pstart + filled || fds[s] < 0) return false;
      if (pread_full(fds[s], dst + filled, want, static_cast<off_t>(a - fstart)) != want) return false;
      filled += static_cast<long long>(want);
    }
    return filled == plen;
  };
  // piece p into buf (sized to the piece)
  auto load = [&](size_t p, std::vector<char>& buf) -> bool {
    const long long pstart = static_cast<long long>(p) * static_cast<long long>(piece_len);
    const long long plen = std::min<long long>(static_cast<long long>(piece_len), total - pstart);
    buf.resize(static_cast<size_t>(plen));
    return read_at(pstart, plen, buf.data());
  };
  // SHA-1 pieces go 16 at a time through the AVX-512 kernel, streamed: each
  // lane's next 64 KiB is read into a 1 MiB staging area that stays in the
  // core's L2, hashed, and the area reused.  Loading 16 whole pieces first
  // (16 MiB per task) hashed from DRAM and halved host throughput.  The
  // rest, and the torrent's last (short) piece, go in SHA-NI pairs.
  constexpr size_t kStage = 64u << 10;
  const bool wide = md == sha1_md() && sha16::cpu_has_avx512() && piece_len % 64 == 0 &&
                    (piece_len <= kStage || piece_len % kStage == 0);
  const size_t g = wide ? 16 : 2;
  parallel_for((n + g - 1) / g, threads <= 0 ? default_threads() : threads, [&](size_t k) {
    const size_t p0 = k * g, cnt = std::min(g, n - p0);
    if (cnt == 16 && static_cast<long long>((p0 + 16) * piece_len) <= total) {
      const size_t step = std::min(piece_len, kStage);
      std::unique_ptr<char[]> stage(new char[16 * step]);
      const void* lane[16];
      bool lane_ok[16];
      for (size_t j = 0; j < 16; ++j) {
        lane[j] = stage.get() + j * step;
        lane_ok[j] = true;
      }
      sha16::Sha1x16 st;
      sha16::sha1_x16_init(&st);
      for (size_t off = 0; off < piece_len; off += step) {
        for (size_t j = 0; j < 16; ++j)
          if (lane_ok[j] && !read_at(static_cast<long long>((p0 + j) * piece_len + off), static_cast<long long>(step),
                                     stage.get() + j * step))
            lane_ok[j] = false;  // its digest is discarded; the lane keeps hashing whatever is staged
        sha16::sha1_x16_update(&st, lane, step / 64);
      }
      unsigned char d[16 * 20];
      sha16::sha1_x16_finish(&st, lane, piece_len, d);  // piece_len % 64 == 0: no data in the tail
      for (size_t j = 0; j < 16; ++j)
        if (lane_ok[j] && std::memcmp(d + 20 * j, expected.data() + (p0 + j) * dl, dl) == 0) ok[p0 + j] = 1;
      return;
    }
    // whole pieces, two at a time (a SHA-NI pair), so a task never holds
    // more than two pieces in memory
    std::vector<char> bufs[2];
    for (size_t j0 = 0; j0 < cnt; j0 += 2) {
      const void* p[2];
      size_t m[2], idx[2], got = 0;
      for (size_t j = j0; j < std::min(cnt, j0 + 2); ++j) {
        if (!load(p0 + j, bufs[got])) continue;  // missing / short: stays 0
        p[got] = bufs[got].data();
        m[got] = bufs[got].size();
        idx[got] = p0 + j;
        ++got;
      }
      unsigned char d[2 * EVP_MAX_MD_SIZE];
      md_batch(md, p, m, got, d);
      for (size_t j = 0; j < got; ++j)
        if (std::memcmp(d + j * dl, expected.data() + idx[j] * dl, dl) == 0) ok[idx[j]] = 1;
    }
  });
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
  return ok;
}

// aws-chunked (STREAMING-AWS4-HMAC-SHA256-PAYLOAD) signature chain over
// chunk_size chunks of [data, data+len) (+ the final empty chunk when
// include_final).  String to sign per chunk:
//   "AWS4-HMAC-SHA256-PAYLOAD\n" amzdate "\n" scope "\n" prev "\n" hex(sha256("")) "\n" hex(sha256(chunk))
//
// Only the HMAC chain is sequential; the per-chunk SHA-256 — all the bytes —
// is independent per chunk, so it runs as a parallel map first (threads > 1)
// and the cheap ~2 µs/chunk HMAC chain follows (a map + sequential scan).
inline std::vector<std::string> chunk_hashes(const char* data, size_t len, size_t chunk_size, bool include_final,
                                             int threads) {
  const size_t nfull = (len + chunk_size - 1) / chunk_size;
  const size_t n = nfull + ((include_final || len == 0) ? 1 : 0);
  std::vector<std::string> h(n);
  const size_t per_thread = (1u << 20) / chunk_size + 1;  // >= ~1 MiB of hashing per thread
  const int t = threads <= 0 ? default_threads() : threads;
  const int used = static_cast<int>(std::min<size_t>(static_cast<size_t>(t), std::max<size_t>(1, nfull / per_thread)));
  // chunks in groups of 16 (the AVX-512 kernel; SHA-NI pairs without it)
  parallel_for((n + 15) / 16, used, [&](size_t k) {
    unsigned char d[16 * 32];
    const void* p[16];
    size_t m[16];
    const size_t cnt = std::min<size_t>(16, n - 16 * k);
    for (size_t j = 0; j < cnt; ++j) {
      const size_t off = (16 * k + j) * chunk_size;
      m[j] = off < len ? std::min(chunk_size, len - off) : 0;
      p[j] = m[j] ? data + off : "";
    }
    sha256_batch(p, m, cnt, d);
    for (size_t j = 0; j < cnt; ++j) h[16 * k + j] = hex_raw(d + 32 * j, 32);
  });
  return h;
}

inline std::vector<std::string> chunk_signatures(const std::string& key, const std::string& amzdate,
                                                 const std::string& scope, const std::string& seed,
                                                 const char* data, size_t len, size_t chunk_size,
                                                 bool include_final, int threads = 1) {
  if (chunk_size == 0) throw std::invalid_argument("chunk_size must be > 0");
  const std::vector<std::string> h = chunk_hashes(data, len, chunk_size, include_final, threads);
  SigChain chain(key, amzdate, scope, seed);
  std::vector<std::string> sigs;
  sigs.reserve(h.size());
  for (const auto& hc : h) sigs.push_back(chain.next(hc));
  return sigs;
}

inline size_t hexlen(size_t n) {
  size_t l = 1;
  while (n >>= 4) ++l;
  return l;
}

// Exact size of the aws-chunked encoding of len bytes.
inline size_t aws_chunk_encoded_size(size_t len, size_t chunk_size, bool final_chunk) {
  const size_t sig_part = 17 + 64 + 2;  // ";chunk-signature=" + sig + CRLF
  size_t total = 0;
  for (size_t off = 0; off < len; off += chunk_size) {
    const size_t n = std::min(chunk_size, len - off);
    total += hexlen(n) + sig_part + n + 2;
  }
  if (final_chunk) total += 1 + sig_part + 2;
  return total;
}

// Fused aws-chunked encoder into dst (which must hold aws_chunk_encoded_size
// bytes).  Frame offsets are fixed by the chunk sizes, so the parallel map
// both hashes each chunk and copies it into place; the sequential scan then
// chains the signatures and writes each 64-hex slot.  Returns the last one.
inline std::string aws_chunk_encode(const std::string& key, const std::string& amzdate, const std::string& scope,
                                    std::string prev, const char* data, size_t len, size_t chunk_size,
                                    bool final_chunk, char* dst, int threads = 1) {
  if (chunk_size == 0) throw std::invalid_argument("chunk_size must be > 0");
  const size_t nfull = (len + chunk_size - 1) / chunk_size;
  const size_t n = nfull + (final_chunk ? 1 : 0);
  std::vector<size_t> frame(n + 1, 0);  // start of each frame in dst
  for (size_t i = 0; i < n; ++i) {
    const size_t m = i < nfull ? std::min(chunk_size, len - i * chunk_size) : 0;
    frame[i + 1] = frame[i] + hexlen(m) + 17 + 64 + 2 + m + 2;
  }
  std::vector<std::string> h(n);
  const size_t per_thread = (1u << 20) / chunk_size + 1;
  const int t = threads <= 0 ? default_threads() : threads;
  const int used = static_cast<int>(std::min<size_t>(static_cast<size_t>(t), std::max<size_t>(1, nfull / per_thread)));
  auto write_frame = [&](size_t i, const char* p, size_t m) {
    char hx[32];
    const int hl = std::snprintf(hx, sizeof hx, "%zx", m);
    char* w = dst + frame[i];
    std::memcpy(w, hx, static_cast<size_t>(hl));
    w += hl;
    std::memcpy(w, ";chunk-signature=", 17);
    w += 17 + 64;  // signature slot filled by the scan below
    *w++ = '\r';
    *w++ = '\n';
    if (m) std::memcpy(w, p, m);
    w += m;
    *w++ = '\r';
    *w++ = '\n';
  };
  parallel_for((n + 15) / 16, used, [&](size_t k) {  // groups of 16 chunks (sha256_batch)
    const size_t cnt = std::min<size_t>(16, n - 16 * k);
    const void* p[16];
    size_t m[16];
    unsigned char d[16 * 32];
    for (size_t j = 0; j < cnt; ++j) {
      const size_t i = 16 * k + j;
      m[j] = i < nfull ? std::min(chunk_size, len - i * chunk_size) : 0;
      p[j] = m[j] ? data + i * chunk_size : "";
    }
    sha256_batch(p, m, cnt, d);
    for (size_t j = 0; j < cnt; ++j) {
      h[16 * k + j] = hex_raw(d + 32 * j, 32);
      write_frame(16 * k + j, static_cast<const char*>(p[j]), m[j]);
    }
  });
  SigChain chain(key, amzdate, scope, prev);
  for (size_t i = 0; i < n; ++i) {
    prev = chain.next(h[i]);
    const size_t m = i < nfull ? std::min(chunk_size, len - i * chunk_size) : 0;
    std::memcpy(dst + frame[i] + hexlen(m) + 17, prev.data(), 64);
  }
  return prev;
}

// Parse + verify an aws-chunked body in one pass over the raw bytes (the
// server side of aws_chunk_encode): frames are located sequentially (cheap),
// payload SHA-256s run as a parallel map, the signature chain is a serial
// scan compared against the claimed signatures.  On success the decoded
// payload is written to *decoded (if non-null).  Returns "" or an error.
// require_final=false accepts a buffer that ends on a frame boundary without
// the terminating zero-length chunk (a streamed batch; the next batch is
// seeded with this batch's last claimed signature).
inline std::string aws_chunk_decode(const std::string& key, const std::string& amzdate, const std::string& scope,
                                    const std::string& seed, const char* raw, size_t len, int threads,
                                    std::string* decoded, bool require_final = true) {
  struct Frame {
    size_t off, n;
    const char* sig;
  };
  std::vector<Frame> frames;
  size_t pos = 0, total = 0;
  for (;;) {
    if (!require_final && pos == len) break;
    size_t hexend = pos;
    while (hexend < len && hexend - pos < 16 && std::isxdigit(static_cast<unsigned char>(raw[hexend]))) ++hexend;
    if (hexend == pos || hexend + 17 + 64 + 2 > len || std::memcmp(raw + hexend, ";chunk-signature=", 17) != 0)
      return "malformed aws-chunked framing";
    const size_t n = std::strtoull(std::string(raw + pos, hexend - pos).c_str(), nullptr, 16);
    const char* sig = raw + hexend + 17;
    const size_t hdr_end = hexend + 17 + 64;
    if (raw[hdr_end] != '\r' || raw[hdr_end + 1] != '\n') return "malformed chunk header";
    const size_t a = hdr_end + 2;
    if (n > len || a + n + 2 > len) return "truncated chunk";
    if (raw[a + n] != '\r' || raw[a + n + 1] != '\n') return "chunk not terminated";
    frames.push_back({a, n, sig});
    total += n;
    pos = a + n + 2;
    if (n == 0) break;
  }
  if (pos != len) return "trailing bytes after final chunk";
  std::vector<std::string> h(frames.size());
  const int t = threads <= 0 ? default_threads() : threads;
  const int used = static_cast<int>(std::min<size_t>(static_cast<size_t>(t), std::max<size_t>(1, total >> 20)));
  if (decoded) decoded->assign(total, '\0');
  std::vector<size_t> dst_off(frames.size() + 1, 0);
  for (size_t i = 0; i < frames.size(); ++i) dst_off[i + 1] = dst_off[i] + frames[i].n;
  const size_t nf = frames.size();
  parallel_for((nf + 15) / 16, used, [&](size_t k) {  // groups of 16 frames (sha256_batch)
    const size_t i0 = 16 * k, cnt = std::min<size_t>(16, nf - i0);
    const void* p[16];
    size_t m[16];
    unsigned char d[16 * 32];
    for (size_t j = 0; j < cnt; ++j) {
      p[j] = raw + frames[i0 + j].off;
      m[j] = frames[i0 + j].n;
    }
    sha256_batch(p, m, cnt, d);
    for (size_t j = 0; j < cnt; ++j) {
      const Frame& a = frames[i0 + j];
      h[i0 + j] = hex_raw(d + 32 * j, 32);
      if (decoded && a.n) std::memcpy(&(*decoded)[dst_off[i0 + j]], raw + a.off, a.n);
    }
  });
  SigChain chain(key, amzdate, scope, seed);
  for (size_t i = 0; i < frames.size(); ++i) {
    if (std::memcmp(chain.next(h[i]).data(), frames[i].sig, 64) != 0) return "chunk signature mismatch";
  }
  return "";
}


// ---------------------------------------------------------------------------
// BitTorrent v2 (BEP 52) merkle verification.  Piece p covers bytes
// [p*piece_len, p*piece_len + real[p]) of the piece-aligned layout; its leaves
// are SHA-256 of each 16 KiB block (the last one may be short), padded with
// all-zero hashes to width[p] leaves and reduced pairwise with SHA-256.  The
// root must equal expected[32p .. 32p+32).  known[p] == 0 -> ok[p] = 0.
constexpr size_t kMerkleLeaf = 16384;

inline void merkle_reduce(std::vector<unsigned char>& row, size_t width) {
  // row holds `width` 32-byte nodes; reduce in place to row[0..32).  Parent
  // nodes are hashed 16 at a time (sha256_batch: the AVX-512 kernel, or
  // SHA-NI pairs); a group's outputs land in [32k, 32k+512) only after all
  // of its inputs [64k, 64k+1024) were read, and later groups read above that.
  unsigned char h[16 * 32];
  const void* p[16];
  size_t m[16];
  while (width > 1) {
    const size_t half = width / 2;
    for (size_t k = 0; k < half; k += 16) {
      const size_t cnt = std::min<size_t>(16, half - k);
      for (size_t j = 0; j < cnt; ++j) {
        p[j] = row.data() + 64 * (k + j);
        m[j] = 64;
      }
      sha256_batch(p, m, cnt, h);
      std::memcpy(row.data() + 32 * k, h, 32 * cnt);
    }
    width = half;
  }
}

inline bool merkle_piece_ok(const unsigned char* leaves, size_t nleaves, size_t width, const char* expected) {
  if (width == 0 || (width & (width - 1)) || nleaves > width) return false;
  std::vector<unsigned char> row(32 * width, 0);
  std::memcpy(row.data(), leaves, 32 * nleaves);
  merkle_reduce(row, width);
  return std::memcmp(row.data(), expected, 32) == 0;
}

// From precomputed leaf digests of the whole layout (e.g. the HIP kernel at
// 16 KiB "pieces"); leaf_ok[k] == 0 marks a block that could not be read.
inline std::string merkle_check(const std::string& leaves, const std::string& leaf_ok, size_t piece_len,
                                const std::string& expected, const std::vector<long long>& widths,
                                const std::vector<long long>& reals, const std::string& known, int threads) {
  if (piece_len == 0 || piece_len % kMerkleLeaf) throw std::invalid_argument("piece_len must be a multiple of 16 KiB");
  const size_t n = widths.size();
  if (reals.size() != n || known.size() != n || expected.size() != 32 * n)
    throw std::invalid_argument("merkle_check: per-piece arrays disagree in length");
  const size_t nleaf_total = leaves.size() / 32;
  if (leaf_ok.size() != nleaf_total) throw std::invalid_argument("leaf_ok size mismatch");
  const size_t per = piece_len / kMerkleLeaf;
  std::string ok(n, '\0');
  parallel_for(n, threads <= 0 ? default_threads() : threads, [&](size_t p) {
    if (!known[p] || reals[p] < 0) return;
    const size_t nl = (static_cast<size_t>(reals[p]) + kMerkleLeaf - 1) / kMerkleLeaf;
    const size_t first = p * per;
    if (first + nl > nleaf_total) return;
    for (size_t k = 0; k < nl; ++k)
      if (!leaf_ok[first + k]) return;
    ok[p] = merkle_piece_ok(reinterpret_cast<const unsigned char*>(leaves.data()) + 32 * first, nl,
                            static_cast<size_t>(widths[p]), expected.data() + 32 * p);
  });
  return ok;
}

// Straight from files (host path): read each piece, hash its leaves, reduce.
inline std::string merkle_verify(const std::vector<std::pair<std::string, long long>>& files, size_t piece_len,
                                 const std::string& expected, const std::vector<long long>& widths,
                                 const std::vector<long long>& reals, const std::string& known, int threads) {
  if (piece_len == 0 || piece_len % kMerkleLeaf) throw std::invalid_argument("piece_len must be a multiple of 16 KiB");
  const size_t n = widths.size();
  if (reals.size() != n || known.size() != n || expected.size() != 32 * n)
    throw std::invalid_argument("merkle_verify: per-piece arrays disagree in length");
  std::vector<FileSpan> spans;
  long long total = 0;
  for (auto& f : files) {
    if (f.second < 0) throw std::invalid_argument("negative file length");
    spans.push_back({f.first, f.second, total});
    total += f.second;
  }
  std::vector<int> fds(spans.size(), -1);
  for (size_t i = 0; i < spans.size(); ++i)
    if (!spans[i].path.empty()) fds[i] = ::open(spans[i].path.c_str(), O_RDONLY | O_CLOEXEC);
  std::string ok(n, '\0');
  const EVP_MD* md = sha256_md();
  parallel_for(n, threads <= 0 ? default_threads() : threads, [&](size_t p) {
    if (!known[p] || reals[p] < 0 || static_cast<size_t>(reals[p]) > piece_len) return;
    const long long pstart = static_cast<long long>(p) * static_cast<long long>(piece_len);
    const long long plen = reals[p];
    if (pstart + plen > total) return;
    std::vector<char> buf(static_cast<size_t>(plen));
    long long filled = 0;
    for (size_t s = 0; s < spans.size() && filled < plen; ++s) {
      const long long fstart = spans[s].start, flen = spans[s].length;
      const long long a = std::max(pstart + filled, fstart);
      const long long e = std::min(pstart + plen, fstart + flen);
      if (e <= a) continue;
      const size_t want = static_cast<size_t>(e - a);
      if (a != pstart + filled) return;
      if (spans[s].path.empty()) {
        std::memset(buf.data() + filled, 0, want);
      } else if (fds[s] < 0 || pread_full(fds[s], buf.data() + filled, want, static_cast<off_t>(a - fstart)) != want) {
        return;
      }
      filled += static_cast<long long>(want);
    }
    if (filled != plen) return;
    const size_t nl = (static_cast<size_t>(plen) + kMerkleLeaf - 1) / kMerkleLeaf;
    const size_t width = static_cast<size_t>(widths[p]);
    if (width == 0 || (width & (width - 1)) || nl > width) return;
    std::vector<unsigned char> row(32 * width, 0);
    for (size_t k = 0; k < nl; k += 16) {  // leaves 16 at a time (sha256_batch)
      const size_t cnt = std::min<size_t>(16, nl - k);
      const void* lp[16];
      size_t ll[16];
      for (size_t j = 0; j < cnt; ++j) {
        const size_t off = (k + j) * kMerkleLeaf;
        lp[j] = buf.data() + off;
        ll[j] = std::min(kMerkleLeaf, static_cast<size_t>(plen) - off);
      }
      if (md == sha256_md()) {
        sha256_batch(lp, ll, cnt, row.data() + 32 * k);
      } else {
        for (size_t j = 0; j < cnt; ++j) md_raw(md, lp[j], ll[j], row.data() + 32 * (k + j));
      }
    }
    merkle_reduce(row, width);
    ok[p] = std::memcmp(row.data(), expected.data() + 32 * p, 32) == 0;
  });
  for (int fd : fds)
    if (fd >= 0) ::close(fd);
  return ok;
}

// RC4 keystream for BitTorrent Message Stream Encryption (MSE/PE).  MSE
// mandates RC4 (and discarding the first 1024 keystream bytes); OpenSSL 3
// only ships it in the legacy provider, so it lives here.  Byte-serial by
// construction (each output depends on the evolving S-box), ~1 GB/s per core.
class Rc4 {
 public:
  Rc4(const uint8_t* key, size_t n) {
    for (int k = 0; k < 256; ++k) s_[k] = static_cast<uint8_t>(k);
    uint8_t j = 0;
    for (int k = 0; k < 256; ++k) {
      j = static_cast<uint8_t>(j + s_[k] + key[k % n]);
      std::swap(s_[k], s_[j]);
    }
  }
  void crypt(const uint8_t* in, uint8_t* out, size_t n) {
    // Work on a local, word-sized copy of the S-box: `out` is a char pointer
    // and may alias any member, which forced a reload per byte (235 MB/s);
    // a non-escaping local cannot alias it.
    uint32_t S[256];
    for (int k = 0; k < 256; ++k) S[k] = s_[k];
    uint32_t i = i_, j = j_;
    for (size_t k = 0; k < n; ++k) {
      i = (i + 1) & 0xFF;
      uint32_t si = S[i];
      j = (j + si) & 0xFF;
      uint32_t sj = S[j];
      S[i] = sj;
      S[j] = si;
      out[k] = static_cast<uint8_t>(in[k] ^ S[(si + sj) & 0xFF]);
    }
    for (int k = 0; k < 256; ++k) s_[k] = static_cast<uint8_t>(S[k]);
    i_ = static_cast<uint8_t>(i);
    j_ = static_cast<uint8_t>(j);
  }
  void discard(size_t n) {
    std::vector<uint8_t> z(n, 0);
    crypt(z.data(), z.data(), n);
  }

 private:
  uint8_t s_[256];
  uint8_t i_ = 0, j_ = 0;
};

}  // namespace tritondl_hash
