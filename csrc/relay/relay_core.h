// Native data plane for the fetch -> S3 relay (no Python; shared by the
// pybind11 module relay.cpp and the sanitizer self-test).
//
// The Python control plane (asyncio) opens connections, writes/parses HTTP
// heads, signs requests and handles retries; every BYTE of a job moves here,
// in threads that never touch the interpreter:
//
//   recv_body  : origin stream -> file (pwrite at the segment's offset),
//                publishing per-segment progress on a Flow;
//   send_body  : file -> S3 socket as an aws-chunked (SigV4 streaming) or
//                unsigned body, following the Flow so an upload can run
//                while the download is still landing.  Chunk SHA-256s run on a
//                small hasher pool ahead of the sender (the per-chunk HMAC
//                chain is the only serial part); the sender batches many
//                frames per writev.  Unsigned bodies go out with sendfile.
//
// Every pump works on a Stream (stream.h): a bare socket — where the kernel
// zero-copy paths (splice, sendfile) apply — or a TLS session, so https
// bodies stay native too.  Stream::abort() stops any pump promptly.
//
// Reference behaviour replaced: grab's single-stream copy
// (internal/downloader/http/http.go:36-71) and minio-go's PutObject body
// (internal/uploader/uploader.go:89) — here they are one fused pipeline.
#pragma once

#include <fcntl.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/sendfile.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cctype>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../hash/gpu_chunk_api.h"
#include "../hash/hash_core.h"
#include "stream.h"

namespace tritondl_relay {


// Timed condition wait used only as a polling slice.  system_clock-based
// (pthread_cond_timedwait): libstdc++'s steady-clock wait_for goes through
// pthread_cond_clockwait, which ThreadSanitizer does not intercept (false
// "double lock" reports in the sanitizer self-test).
template <class Pred>
inline bool cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& l, int ms, Pred pred) {
  return cv.wait_until(l, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), pred);
}
inline void cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& l, int ms) {
  cv.wait_until(l, std::chrono::system_clock::now() + std::chrono::milliseconds(ms));
}

// ---------------------------------------------------------------------------
// Flow: progress of one download made of contiguous segments
// [start, end) (end < 0: open-ended, length unknown), shared by the receive
// pumps (writers) and any number of readers (upload pump, Python waiters).
class Flow {
 public:
  struct Seg {
    uint64_t start;
    int64_t end;  // exclusive; < 0 = unknown length
    uint64_t done;
    Clock::time_point moved{};  // last advance (stall detection)
  };

  explicit Flow(std::vector<Seg> segs) : segs_(std::move(segs)) {
    const auto now = Clock::now();
    for (Seg& s : segs_) s.moved = now;
  }

  // A reader waiting for bytes gives up with rc 4 ("stalled") once no segment
  // it needs has advanced for this long (0 = never).  An upload that follows
  // the download must not sit idle on its PUT past the store's request
  // timeout (S3 drops a body that sends nothing for ~20 s with 400
  // RequestTimeout); the caller falls back to uploading after the download.
  void set_stall(double s) {
    std::lock_guard<std::mutex> l(mu_);
    stall_s_ = s;
  }
  double stall() const {
    std::lock_guard<std::mutex> l(mu_);
    return stall_s_;
  }

  // Wakes exactly the waiters whose range became covered: the upload's chunk
  // hashers wait for ranges ahead of the receive frontier, and waking all of
  // them on every 256 KiB of progress was a thundering herd of futex
  // wake-ups (4 hashers x ~40 advances per 10 MiB job, most going straight
  // back to sleep).  Each waiter owns its condition variable; the notify
  // happens under the lock, so a waiter that timed out and left cannot be
  // notified after it is gone.
  void advance(size_t seg, uint64_t done) {
    std::lock_guard<std::mutex> l(mu_);
    if (seg >= segs_.size()) return;
    if (done > segs_[seg].done) {
      segs_[seg].done = done;
      segs_[seg].moved = Clock::now();
    }
    for (Waiter* w : waiters_)
      if (!w->woken && covered_locked(w->a, w->b)) {
        w->woken = true;
        w->cv.notify_one();
      }
  }
  // All bytes below `total` are on disk (also resolves open-ended segments).
  void finish(uint64_t total) {
    std::lock_guard<std::mutex> l(mu_);
    finished_ = true;
    total_ = total;
    wake_all_locked();
  }
  void fail(const std::string& why) {
    std::lock_guard<std::mutex> l(mu_);
    if (!failed_) err_ = why;
    failed_ = true;
    wake_all_locked();
  }
  void cancel() {
    cancel_.store(true);
    fail("cancelled");
  }
  bool cancelled() const { return cancel_.load(std::memory_order_relaxed); }

  uint64_t done(size_t seg) const {
    std::lock_guard<std::mutex> l(mu_);
    return seg < segs_.size() ? segs_[seg].done : 0;
  }
  size_t nsegs() const { return segs_.size(); }
  std::string error() const {
    std::lock_guard<std::mutex> l(mu_);
    return err_;
  }
  bool failed() const {
    std::lock_guard<std::mutex> l(mu_);
    return failed_;
  }
  bool finished() const {
    std::lock_guard<std::mutex> l(mu_);
    return finished_;
  }

  // How far the download still is from covering [a, b): each segment fills
  // sequentially from its frontier, segments in parallel, so this is the
  // largest number of bytes any one overlapping segment must still receive
  // (0 = on disk).  Used to schedule multipart uploads in arrival order.
  uint64_t bytes_until_covered(uint64_t a, uint64_t b) const {
    std::lock_guard<std::mutex> l(mu_);
    if (b <= a || finished_) return 0;
    uint64_t worst = 0;
    for (const Seg& s : segs_) {
      const uint64_t s_end = s.end < 0 ? UINT64_MAX : static_cast<uint64_t>(s.end);
      const uint64_t hi = std::min(b, s_end);
      if (hi <= std::max(a, s.start)) continue;
      const uint64_t frontier = s.start + s.done;
      if (hi > frontier) worst = std::max(worst, hi - frontier);
    }
    return worst;
  }

  // Receive frontier (start + done) of every segment still filling; empty
  // once finished.  Lets a scheduler rank only the ranges at a frontier
  // instead of every pending range.
  std::vector<uint64_t> frontiers() const {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<uint64_t> out;
    if (finished_) return out;
    for (const Seg& s : segs_) {
      const uint64_t f = s.start + s.done;
      if (s.end < 0 || f < static_cast<uint64_t>(s.end)) out.push_back(f);
    }
    return out;
  }

  // Start offset of every segment still filling (see frontiers()).
  std::vector<uint64_t> open_starts() const {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<uint64_t> out;
    if (finished_) return out;
    for (const Seg& s : segs_) {
      const uint64_t f = s.start + s.done;
      if (s.end < 0 || f < static_cast<uint64_t>(s.end)) out.push_back(s.start);
    }
    return out;
  }

  // Bytes of [a, b) already on disk (for scheduling uploads of ranges).
  uint64_t covered_bytes(uint64_t a, uint64_t b) const {
    std::lock_guard<std::mutex> l(mu_);
    if (b <= a) return 0;
    if (finished_) return std::min(b, total_) > a ? std::min(b, total_) - a : 0;
    uint64_t got = 0;
    for (const Seg& s : segs_) {
      const uint64_t lo = std::max(a, s.start), hi = std::min(b, s.start + s.done);
      if (hi > lo) got += hi - lo;
    }
    return got;
  }

  // Bytes of [a, b) on disk contiguously from a (stops at the first gap).
  uint64_t covered_prefix(uint64_t a, uint64_t b) const {
    std::lock_guard<std::mutex> l(mu_);
    if (b <= a) return 0;
    if (finished_) return std::min(b, total_) > a ? std::min(b, total_) - a : 0;
    uint64_t need = a;
    for (;;) {
      uint64_t best = need;
      for (const Seg& s : segs_) {
        const uint64_t s_end = s.end < 0 ? UINT64_MAX : static_cast<uint64_t>(s.end);
        if (s.start > need || s_end <= need) continue;
        best = std::max(best, std::min(s.start + s.done, s_end));
      }
      if (best <= need || best >= b) return std::min(best, b) - a;
      need = best;
    }
  }

  // Length of the contiguous prefix on disk.
  uint64_t watermark() const {
    std::lock_guard<std::mutex> l(mu_);
    return watermark_locked();
  }

  // 0 = [a, b) is on disk, 1 = flow failed/cancelled, 2 = timed out,
  // 3 = the download finished short of b, 4 = stalled (see set_stall).
  int wait_covered(uint64_t a, uint64_t b, double timeout_s, const std::atomic<bool>* abort = nullptr) {
    std::unique_lock<std::mutex> l(mu_);
    if (covered_locked(a, b)) return 0;
    const auto entered = Clock::now();
    const auto deadline = entered + std::chrono::duration_cast<Clock::duration>(
                                        std::chrono::duration<double>(std::max(0.0, timeout_s)));
    Waiter me{a, b};
    waiters_.push_back(&me);  // advance() wakes us once this range is covered
    int rc;
    for (;;) {
      if (covered_locked(a, b)) { rc = 0; break; }
      if (failed_) { rc = 1; break; }
      if (finished_) { rc = 3; break; }
      if (abort && abort->load()) { rc = 1; break; }
      const auto now = Clock::now();
      if (now >= deadline) { rc = 2; break; }
      if (stall_s_ > 0 && std::chrono::duration<double>(now - last_move_locked(a, b, entered)).count() >= stall_s_) {
        rc = 4;
        break;
      }
      // short slices so an aborting caller (the upload pump's sender) is seen promptly
      cv_wait_ms(me.cv, l, 20);
    }
    waiters_.erase(std::find(waiters_.begin(), waiters_.end(), &me));
    return rc;
  }

 private:
  struct Waiter {
    uint64_t a, b;
    std::condition_variable cv;
    bool woken = false;
    Waiter(uint64_t a_, uint64_t b_) : a(a_), b(b_) {}
  };
  void wake_all_locked() {
    for (Waiter* w : waiters_) {
      w->woken = true;
      w->cv.notify_one();
    }
  }
  // Latest advance of any unfinished segment that still owes bytes of [a, b)
  // (not before `floor`, the time the wait began).
  Clock::time_point last_move_locked(uint64_t a, uint64_t b, Clock::time_point floor) const {
    Clock::time_point t = floor;
    for (const Seg& s : segs_) {
      const uint64_t s_end = s.end < 0 ? UINT64_MAX : static_cast<uint64_t>(s.end);
      const uint64_t frontier = s.start + s.done;
      if (std::min(b, s_end) <= std::max(a, frontier)) continue;  // owes nothing of [a, b)
      if (s.moved > t) t = s.moved;
    }
    return t;
  }
  uint64_t watermark_locked() const {
    if (finished_) return total_;
    uint64_t w = 0;
    for (const Seg& s : segs_) {
      w = s.start + s.done;
      if (s.end < 0 || w < static_cast<uint64_t>(s.end)) break;
    }
    return w;
  }
  bool covered_locked(uint64_t a, uint64_t b) const {
    if (b <= a) return true;
    if (finished_) return b <= total_;
    uint64_t need = a;  // first byte of [a, b) not yet shown to be on disk
    for (const Seg& s : segs_) {
      const uint64_t s_end = s.end < 0 ? UINT64_MAX : static_cast<uint64_t>(s.end);
      if (s_end <= need || s.start > need) continue;
      const uint64_t have = s.start + s.done;  // [s.start, have) is on disk
      if (have <= need) return false;
      need = std::min(have, s_end);
      if (need >= b) return true;
    }
    return need >= b;
  }

  mutable std::mutex mu_;
  std::vector<Seg> segs_;
  std::vector<Waiter*> waiters_;  // wait_covered() calls blocked on a range (their frames own them)
  bool finished_ = false;
  uint64_t total_ = 0;
  bool failed_ = false;
  double stall_s_ = 0;
  std::string err_;
  std::atomic<bool> cancel_{false};
};

// Why a send pump's wait for source bytes ended (Flow::wait_covered rc 1-4).
inline std::string flow_wait_error(int w, const Flow& flow) {
  return w == 3   ? "source shorter than expected"
         : w == 2 ? "timed out waiting for source bytes"
         : w == 4 ? "source stalled"
                  : "source transfer failed: " + flow.error();
}

// ---------------------------------------------------------------------------
// Buffer cache.  A 10 MiB job touches ~20 MiB of pump buffers; fresh
// allocations of that size come from mmap and fault in page by page on every
// job (thousands of faults), so the pumps borrow buffers that stay mapped.
class BufCache {
 public:
  static BufCache& get() {
    static BufCache* c = new BufCache();  // process lifetime (pumps may run at exit)
    return *c;
  }
  char* take(size_t n, size_t* cap) {
    {
      std::lock_guard<std::mutex> l(mu_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].second >= n && (best == free_.size() || free_[i].second < free_[best].second)) best = i;
      if (best != free_.size()) {
        char* p = free_[best].first;
        *cap = free_[best].second;
        cached_ -= *cap;
        free_.erase(free_.begin() + static_cast<long>(best));
        return p;
      }
    }
    *cap = n;
    return new char[n];
  }
  void give(char* p, size_t cap) {
    std::lock_guard<std::mutex> l(mu_);
    if (cached_ + cap > kMaxCached) {
      delete[] p;
      return;
    }
    free_.emplace_back(p, cap);
    cached_ += cap;
  }

 private:
  static constexpr size_t kMaxCached = size_t(256) << 20;
  std::mutex mu_;
  std::vector<std::pair<char*, size_t>> free_;
  size_t cached_ = 0;
};

// RAII borrowed buffer with vector-like grow (contents kept).
struct Buf {
  char* p = nullptr;
  size_t cap = 0;
  Buf() = default;
  explicit Buf(size_t n) { p = BufCache::get().take(n, &cap); }
  ~Buf() {
    if (p) BufCache::get().give(p, cap);
  }
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  char* data() { return p; }
  const char* data() const { return p; }
  size_t size() const { return cap; }
  void ensure(size_t n, size_t keep) {
    if (n <= cap) return;
    size_t ncap = 0;
    char* q = BufCache::get().take(std::max(n, cap * 2), &ncap);
    if (keep) std::memcpy(q, p, keep);
    if (p) BufCache::get().give(p, cap);
    p = q;
    cap = ncap;
  }
};

// ---------------------------------------------------------------------------
// socket helpers (non-blocking fds owned by the asyncio side; the pumps poll)

// A pump must stop: its stream was aborted or the download it follows was cancelled.
inline bool stopped(const Stream& io, const Flow* flow) { return io.aborted() || (flow && flow->cancelled()); }

inline bool pwrite_full(int fd, const char* p, size_t n, uint64_t off, std::string* err) {
  while (n) {
    const ssize_t w = ::pwrite(fd, p, n, static_cast<off_t>(off));
    if (w < 0) {
      if (errno == EINTR) continue;
      *err = errno_str("pwrite");
      return false;
    }
    p += w;
    n -= static_cast<size_t>(w);
    off += static_cast<uint64_t>(w);
  }
  return true;
}

// Write every iovec (partial writes resumed); waits for writability on EAGAIN.
inline bool writev_all(Stream& io, std::vector<struct iovec>& iov, double idle_timeout, const Flow* flow,
                       std::string* err) {
  size_t k = 0;
  auto last = Clock::now();
  while (k < iov.size()) {
    const int cnt = static_cast<int>(std::min<size_t>(iov.size() - k, IOV_MAX));
    short want = POLLOUT;
    const ssize_t w = io.send_nb(&iov[k], cnt, &want, err);
    if (w == IO_ERR) return false;
    if (w == IO_AGAIN || w == 0) {
      if (stopped(io, flow)) {
        *err = "cancelled";
        return false;
      }
      if (since(last) > idle_timeout) {
        *err = "send timeout";
        return false;
      }
      if (wait_fd(io.fd(), want, 50) < 0) {
        *err = "socket error while sending";
        return false;
      }
      continue;
    }
    last = Clock::now();
    size_t left = static_cast<size_t>(w);
    while (left && k < iov.size()) {
      if (left >= iov[k].iov_len) {
        left -= iov[k].iov_len;
        ++k;
      } else {
        iov[k].iov_base = static_cast<char*>(iov[k].iov_base) + left;
        iov[k].iov_len -= left;
        left = 0;
      }
    }
    while (k < iov.size() && iov[k].iov_len == 0) ++k;
  }
  // a TLS stream may still hold the last records' ciphertext
  for (;;) {
    short want = POLLOUT;
    if (io.flush_nb(&want, err)) return true;
    if (!err->empty()) return false;
    if (stopped(io, flow)) {
      *err = "cancelled";
      return false;
    }
    if (since(last) > idle_timeout) {
      *err = "send timeout";
      return false;
    }
    if (wait_fd(io.fd(), want, 50) < 0) {
      *err = "socket error while sending";
      return false;
    }
    last = Clock::now();
  }
}

inline bool send_all(Stream& io, const char* p, size_t n, double idle_timeout, const Flow* flow, std::string* err) {
  if (!n) return true;
  std::vector<struct iovec> iov{{const_cast<char*>(p), n}};
  return writev_all(io, iov, idle_timeout, flow, err);
}

// One receive with waiting: > 0 bytes, 0 = end of stream, -1 = error/stop (*err set).
inline ssize_t recv_wait(Stream& io, char* p, size_t n, Clock::time_point* last, double idle_timeout,
                         const Flow* flow, std::string* err) {
  for (;;) {
    if (stopped(io, flow)) {
      *err = "cancelled";
      return -1;
    }
    short want = POLLIN;
    const ssize_t r = io.recv_nb(p, n, &want, err);
    if (r >= 0) {
      if (r > 0) *last = Clock::now();
      return r;
    }
    if (r == IO_ERR) return -1;
    if (since(*last) > idle_timeout) {
      *err = "read timeout";
      return -1;
    }
    if (wait_fd(io.fd(), want, 50) < 0) {
      *err = "socket error while receiving";
      return -1;
    }
  }
}

// ---------------------------------------------------------------------------
// recv_body: stream a response body from `sock` into `fd` at file offset
// `off` (fd < 0: receive and drop).  `prefix` = body bytes already read
// together with the head.
// length < 0: until EOF.  Progress: flow->advance(seg, seg_done0 + received).
struct RecvResult {
  uint64_t received = 0;
  bool eof = false;    // peer closed (normal end for length < 0)
  bool ended = false;  // chunked: the last chunk and its trailers were read
  bool extra = false;  // chunked: bytes arrived after the body (connection not reusable)
  std::string err;
};

// Incremental decoder of an HTTP/1.1 chunked body (RFC 9112 §7.1):
//   chunk = hex-size [; ext] CRLF data CRLF ... 0 [; ext] CRLF *(trailer CRLF) CRLF
// decode() works in place: the data bytes of buf[0, n) are moved to the front
// of buf (the framing between them is overwritten; dst <= src always), so one
// pwrite stores what a whole receive buffer carried.
class ChunkedDecoder {
 public:
  // Consumes buf[0, n); returns bytes consumed (< n only once the body ended).
  // *data_n = data bytes now at buf[0, *data_n).  Malformed framing sets *err.
  size_t decode(char* buf, size_t n, size_t* data_n, std::string* err) {
    size_t i = 0, w = 0;
    while (i < n && phase_ != kDone) {
      const char c = buf[i];
      switch (phase_) {
        case kSize: {
          const int v = hexval(c);
          if (v >= 0) {
            if (++digits_ > 15) return fail(err, "chunk size too large", data_n, w);
            size_ = (size_ << 4) | uint64_t(v);
          } else if (digits_ && (c == ';' || c == ' ' || c == '\t')) {
            phase_ = kExt;
          } else if (digits_ && c == '\r') {
            phase_ = kSizeLF;
          } else {
            return fail(err, "malformed chunk size line", data_n, w);
          }
          ++i;
          break;
        }
        case kExt:  // chunk extensions are ignored (bounded)
          if (c == '\r') phase_ = kSizeLF;
          else if (++ext_ > 4096) return fail(err, "chunk extension too long", data_n, w);
          ++i;
          break;
        case kSizeLF:
          if (c != '\n') return fail(err, "malformed chunk size line", data_n, w);
          ++i;
          if (size_ == 0) {
            phase_ = kTrailer;
            line_ = 0;
          } else {
            phase_ = kData;
            left_ = size_;
          }
          break;
        case kData: {
          const size_t m = size_t(std::min<uint64_t>(left_, n - i));
          if (w != i) std::memmove(buf + w, buf + i, m);
          w += m;
          i += m;
          left_ -= m;
          if (left_ == 0) phase_ = kDataCR;
          break;
        }
        case kDataCR:
          if (c != '\r') return fail(err, "chunk data not followed by CRLF", data_n, w);
          phase_ = kDataLF;
          ++i;
          break;
        case kDataLF:
          if (c != '\n') return fail(err, "chunk data not followed by CRLF", data_n, w);
          phase_ = kSize;
          size_ = 0;
          digits_ = 0;
          ext_ = 0;
          ++i;
          break;
        case kTrailer:  // trailer fields (ignored), then the empty line
          if (c == '\r') phase_ = kTrailerLF;
          else ++line_;
          if (++trailer_ > (64u << 10)) return fail(err, "chunked trailer too large", data_n, w);
          ++i;
          break;
        case kTrailerLF:
          if (c != '\n') return fail(err, "malformed chunked trailer", data_n, w);
          ++i;
          if (line_ == 0) phase_ = kDone;
          line_ = 0;
          if (phase_ != kDone) phase_ = kTrailer;
          break;
        case kDone:
          break;
      }
    }
    *data_n = w;
    return i;
  }
  bool done() const { return phase_ == kDone; }

 private:
  enum Phase { kSize, kExt, kSizeLF, kData, kDataCR, kDataLF, kTrailer, kTrailerLF, kDone };
  static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static size_t fail(std::string* err, const char* why, size_t* data_n, size_t w) {
    *err = why;
    *data_n = w;
    return 0;
  }
  Phase phase_ = kSize;
  uint64_t size_ = 0, left_ = 0;
  int digits_ = 0;
  size_t ext_ = 0, line_ = 0, trailer_ = 0;
};

// Zero-user-copy receive: socket -> pipe (page references move) -> file
// (one copy into the page cache).  Returns false when splice is unsupported
// here (then nothing was consumed and the caller falls back to recv+pwrite).
inline bool splice_body(Stream& io, int fd, uint64_t off, uint64_t want, RecvResult& r, Flow* flow, size_t seg,
                        uint64_t seg_done0, double idle_timeout) {
  const int sock = io.fd();
  int p[2];
  if (::pipe2(p, O_CLOEXEC | O_NONBLOCK) != 0) return false;
  ::fcntl(p[1], F_SETPIPE_SZ, 1 << 20);  // best effort; the default is 64 KiB
  auto last = Clock::now();
  size_t in_pipe = 0;
  bool ok = true;
  while (r.received < want && r.err.empty()) {
    if (stopped(io, flow)) {
      r.err = "cancelled";
      break;
    }
    const size_t cap = static_cast<size_t>(std::min<uint64_t>(1u << 20, want - r.received));
    const ssize_t n = ::splice(sock, nullptr, p[1], nullptr, cap, SPLICE_F_MOVE | SPLICE_F_NONBLOCK);
    if (n > 0) {
      in_pipe = static_cast<size_t>(n);
      while (in_pipe) {
        loff_t o = static_cast<loff_t>(off + r.received);
        const ssize_t w = ::splice(p[0], nullptr, fd, &o, in_pipe, SPLICE_F_MOVE);
        if (w < 0) {
          if (errno == EINTR) continue;
          if (r.received == 0 && (errno == EINVAL || errno == ENOSYS)) {
            ok = false;  // filesystem without splice-write support; bytes still sit in the pipe
            break;
          }
          r.err = errno_str("splice to file");
          break;
        }
        in_pipe -= static_cast<size_t>(w);
        r.received += static_cast<uint64_t>(w);
      }
      if (!ok || !r.err.empty()) break;
      if (flow) flow->advance(seg, seg_done0 + r.received);
      last = Clock::now();
      continue;
    }
    if (n == 0) {
      r.eof = true;
      if (want != UINT64_MAX) r.err = "connection closed early";
      break;
    }
    if (errno == EINTR) continue;
    if (errno == EINVAL && r.received == 0) {
      ok = false;  // socket type without splice support
      break;
    }
    if (errno != EAGAIN && errno != EWOULDBLOCK) {
      r.err = errno_str("splice from socket");
      break;
    }
    if (since(last) > idle_timeout) {
      r.err = "read timeout";
      break;
    }
    if (wait_fd(sock, POLLIN, 50) < 0) r.err = "socket error while receiving";
  }
  if (!ok && in_pipe) {
    // the file refused splice: move what sits in the pipe with read + pwrite
    Buf tmp(in_pipe);
    size_t left = in_pipe;
    while (left && r.err.empty()) {
      const ssize_t got = ::read(p[0], tmp.data(), left);
      if (got <= 0) {
        if (got < 0 && errno == EINTR) continue;
        r.err = "pipe drain failed";
        break;
      }
      if (pwrite_full(fd, tmp.data(), static_cast<size_t>(got), off + r.received, &r.err)) {
        r.received += static_cast<uint64_t>(got);
        left -= static_cast<size_t>(got);
      }
    }
    if (flow) flow->advance(seg, seg_done0 + r.received);
  }
  ::close(p[0]);
  ::close(p[1]);
  return ok;  // false: caller continues with recv + pwrite
}

// recv_chunked: the chunked-transfer form of recv_body.  Decoded bytes go to
// the file at off + received; `length` >= 0 caps them (a longer body is an
// error).  Ends at the last chunk, so the connection stays reusable.
inline RecvResult recv_chunked(Stream& io, int fd, uint64_t off, int64_t length, const char* prefix,
                               size_t prefix_len, Flow* flow, size_t seg, uint64_t seg_done0, double idle_timeout) {
  RecvResult r;
  ChunkedDecoder dec;
  Buf buf(256u << 10);
  auto last = Clock::now();
  // one decode + write step over buf[0, have)
  auto step = [&](size_t have) -> bool {
    size_t data_n = 0;
    const size_t used = dec.decode(buf.data(), have, &data_n, &r.err);
    if (!r.err.empty()) return false;
    bool capped = false;
    if (length >= 0 && r.received + data_n >= uint64_t(length)) {
      // the segment ends here (the probe's stream runs on into the next
      // segment's bytes): keep what belongs to it and drop the connection
      capped = r.received + data_n > uint64_t(length) || !dec.done();
      data_n = size_t(uint64_t(length) - r.received);
    }
    if (data_n) {
      if (fd >= 0 && !pwrite_full(fd, buf.data(), data_n, off + r.received, &r.err)) return false;
      r.received += data_n;
      if (flow) flow->advance(seg, seg_done0 + r.received);
    }
    if (capped) {
      r.ended = r.extra = true;
    } else if (dec.done()) {
      r.ended = true;
      r.extra = used < have;
    }
    return true;
  };
  for (size_t p = 0; p < prefix_len && !r.ended;) {
    const size_t m = std::min(prefix_len - p, buf.size());
    std::memcpy(buf.data(), prefix + p, m);
    if (!step(m)) return r;
    p += m;
  }
  while (!r.ended) {
    const ssize_t n = recv_wait(io, buf.data(), buf.size(), &last, idle_timeout, flow, &r.err);
    if (n < 0) return r;
    if (n == 0) {
      r.eof = true;
      r.err = "connection closed inside a chunked body";
      return r;
    }
    if (!step(size_t(n))) return r;
  }
  return r;
}

inline RecvResult recv_body(Stream& io, int fd, uint64_t off, int64_t length, const char* prefix, size_t prefix_len,
                            Flow* flow, size_t seg, uint64_t seg_done0, double idle_timeout,
                            size_t buf_size = 4u << 20, bool use_splice = true, bool chunked = false) {
  RecvResult r;
  if (stopped(io, flow)) {  // before touching the file: a cancelled segment writes nothing
    r.err = "cancelled";
    return r;
  }
  if (chunked) return recv_chunked(io, fd, off, length, prefix, prefix_len, flow, seg, seg_done0, idle_timeout);
  const uint64_t want = length < 0 ? UINT64_MAX : static_cast<uint64_t>(length);
  if (prefix_len) {
    const size_t n = static_cast<size_t>(std::min<uint64_t>(prefix_len, want));
    if (fd >= 0 && !pwrite_full(fd, prefix, n, off, &r.err)) return r;
    r.received = n;
    if (flow) flow->advance(seg, seg_done0 + r.received);
  }
  if (fd >= 0 && use_splice && io.plain() && r.received < want) {
    if (splice_body(io, fd, off, want, r, flow, seg, seg_done0, idle_timeout) || !r.err.empty() || r.eof)
      return r;
  }
  // TLS: decrypt into an L2-sized buffer so pwrite copies cache-hot bytes
  Buf buf(io.plain() ? std::max<size_t>(buf_size, 64 << 10) : (256u << 10));
  // with a follower (the S3 send pump hashes 64 KiB chunks as soon as the
  // flow covers them) publish progress every 256 KiB, so the upload trails the
  // download by a few chunks instead of a whole 1 MiB batch at the end
  const size_t fill = io.plain() && !flow ? (1u << 20) : (256u << 10);
  auto last = Clock::now();
  while (r.received < want) {
    // fill the buffer with whatever is ready (TLS yields one record per read),
    // then one pwrite
    const size_t cap = static_cast<size_t>(std::min<uint64_t>(buf.size(), want - r.received));
    size_t have = 0;
    bool eof = false;
    const ssize_t n = recv_wait(io, buf.data(), cap, &last, idle_timeout, flow, &r.err);
    if (n < 0) return r;
    if (n == 0) {
      eof = true;
    } else {
      have = static_cast<size_t>(n);
      while (have < cap && have < fill) {
        short w = POLLIN;
        std::string e;
        const ssize_t m = io.recv_nb(buf.data() + have, cap - have, &w, &e);
        if (m > 0) {
          have += static_cast<size_t>(m);
          continue;
        }
        if (m == 0) eof = true;
        if (m == IO_ERR) r.err = e;
        break;
      }
    }
    if (have) {
      if (fd >= 0 && !pwrite_full(fd, buf.data(), have, off + r.received, &r.err)) return r;
      r.received += have;
      if (flow) flow->advance(seg, seg_done0 + r.received);
    }
    if (!r.err.empty()) return r;
    if (eof) {
      r.eof = true;
      if (length >= 0 && r.received < want) r.err = "connection closed early";
      return r;
    }
  }
  return r;
}

// ---------------------------------------------------------------------------
// send_body: request head + body of one PUT.
//   mode 0: plain body (sendfile from fd), e.g. UNSIGNED-PAYLOAD
//   mode 1: aws-chunked STREAMING-AWS4-HMAC-SHA256-PAYLOAD, chunk signatures
//           chained from `seed` with signing key `key`.
// Body bytes are [off, off+length) of fd; with a flow, each range is awaited
// before it is read (upload follows the download).
struct SendResult {
  uint64_t sent = 0;     // body payload bytes
  std::string last_sig;  // mode 1: the final chunk's signature
  std::string err;
};

struct ChunkSigner {
  tritondl_hash::SigChain chain;
  std::string empty_hash;
  ChunkSigner(const std::string& k, const std::string& amzdate, const std::string& scope, const std::string& seed)
      : chain(k, amzdate, scope, seed),
        empty_hash(tritondl_hash::hex(tritondl_hash::one_shot(tritondl_hash::sha256_md(), "", 0))) {}
  const std::string& next(const std::string& chunk_hash_hex) { return chain.next(chunk_hash_hex); }
  const std::string& prev() const { return chain.prev(); }
};

// A read-only MAP_SHARED view of [off, off + length) of fd, for encrypting
// straight from the page cache (TLS): no pread copy into a user buffer.  Only
// when the file already spans the range (a mapping read past EOF is SIGBUS);
// otherwise empty and the caller preads.  `populate`: fault the whole range
// in with one call (complete files; a range still being downloaded is
// faulted in as it is read, behind the flow).
struct FileView {
  const char* p = nullptr;  // byte `off` of the file
  void* base = MAP_FAILED;
  size_t len = 0;
  FileView(int fd, uint64_t off, uint64_t length, bool populate) {
    struct stat st;
    if (!length || ::fstat(fd, &st) != 0 || static_cast<uint64_t>(st.st_size) < off + length) return;
    const uint64_t page = static_cast<uint64_t>(::sysconf(_SC_PAGESIZE));
    const uint64_t a = off & ~(page - 1);
    len = static_cast<size_t>(off + length - a);
    base = ::mmap(nullptr, len, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, static_cast<off_t>(a));
    if (base == MAP_FAILED) return;
    ::madvise(base, len, MADV_SEQUENTIAL);
    p = static_cast<const char*>(base) + (off - a);
  }
  ~FileView() {
    if (base != MAP_FAILED) ::munmap(base, len);
  }
  FileView(const FileView&) = delete;
  FileView& operator=(const FileView&) = delete;
};

inline bool tls_send_mapped() {
  static const bool on = [] {
    const char* v = std::getenv("TRITONDL_TLS_SEND_MAP");
    return !(v && (std::string(v) == "0" || std::string(v) == "off"));
  }();
  return on;
}

inline SendResult send_plain(Stream& io, int fd, uint64_t off, uint64_t length, Flow* flow, double idle_timeout) {
  SendResult r;
  // sendfile moves 4 MiB per call; TLS encrypts from user-space bytes: a
  // mapping of the file's page cache (no copy), else an L2-sized buffer so
  // the pread'd bytes are still cache-hot when encrypted
  const uint64_t step = io.plain() ? (4u << 20) : (256u << 10);
  auto last = Clock::now();
  std::unique_ptr<FileView> view;
  if (!io.plain() && tls_send_mapped()) {
    view.reset(new FileView(fd, off, length, flow == nullptr && length <= (256ull << 20)));
    if (!view->p) view.reset();
  }
  Buf buf(io.plain() || view ? 0 : static_cast<size_t>(std::min<uint64_t>(step, std::max<uint64_t>(length, 1))));
  while (r.sent < length) {
    uint64_t n = std::min(step, length - r.sent);
    if (flow) {
      // follow the download closely: wait for a slice (not a whole 4 MiB step, which
      // left up to 4 MiB to send after the last byte landed), then send everything
      // already on disk from here, up to the step
      const uint64_t slice = std::min<uint64_t>(n, 256u << 10);
      const int w = flow->wait_covered(off + r.sent, off + r.sent + slice, idle_timeout, io.abort_flag());
      if (w) {
        r.err = io.aborted() ? "cancelled" : flow_wait_error(w, *flow);
        return r;
      }
      n = std::max(slice, std::min(n, flow->covered_prefix(off + r.sent, off + r.sent + n)));
    }
    if (!io.plain()) {  // TLS: the record layer needs the bytes in user space
      const size_t m = static_cast<size_t>(n);
      if (view) {
        if (!send_all(io, view->p + r.sent, m, idle_timeout, flow, &r.err)) return r;
        r.sent += n;
        continue;
      }
      if (tritondl_hash::pread_full(fd, buf.data(), m, static_cast<off_t>(off + r.sent)) != m) {
        r.err = "source file shorter than expected";
        return r;
      }
      if (!send_all(io, buf.data(), m, idle_timeout, flow, &r.err)) return r;
      r.sent += n;
      continue;
    }
    const int sock = io.fd();
    uint64_t k = 0;
    while (k < n) {
      off_t o = static_cast<off_t>(off + r.sent + k);
      const ssize_t w = ::sendfile(sock, fd, &o, static_cast<size_t>(n - k));
      if (w > 0) {
        k += static_cast<uint64_t>(w);
        last = Clock::now();
        continue;
      }
      if (w == 0) {
        r.sent += k;
        r.err = "source file shorter than expected";
        return r;
      }
      if (errno == EINTR) continue;
      if (errno != EAGAIN && errno != EWOULDBLOCK) {
        r.sent += k;
        r.err = errno_str("sendfile");
        return r;
      }
      if (stopped(io, flow) || since(last) > idle_timeout || wait_fd(sock, POLLOUT, 50) < 0) {
        r.sent += k;
        r.err = stopped(io, flow) ? "cancelled" : "send timeout";
        return r;
      }
    }
    r.sent += n;
  }
  return r;
}

inline SendResult send_chunked(Stream& io, int fd, uint64_t off, uint64_t length, Flow* flow, ChunkSigner& signer,
                               size_t chunk, int threads, double idle_timeout, size_t batch = 64) {
  SendResult r;
  if (chunk == 0) {
    r.err = "chunk size must be > 0";
    return r;
  }
  const size_t n = static_cast<size_t>((length + chunk - 1) / chunk);
  const size_t K = std::max<size_t>(1, std::min<size_t>(n, 2 * batch));  // ring slots
  batch = std::min(batch, K);
  Buf ring(K * chunk);
  std::vector<int64_t> ready(K, -1);       // chunk index held by each slot, once hashed
  std::vector<std::string> hashes(K);
  std::mutex mu;
  std::condition_variable cv_ready, cv_free;
  int64_t sent_chunks = 0;
  std::atomic<bool> abort{false};
  std::string worker_err;
  std::atomic<size_t> next{0};

  auto set_err = [&](const std::string& e) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (worker_err.empty()) worker_err = e;
      abort.store(true);
    }
    cv_ready.notify_all();
    cv_free.notify_all();
  };

  // Each hasher takes two consecutive chunks: SHA-NI hashes them in lockstep
  // (sha_ni.h).  Both ring slots must be free (K >= 2 whenever n >= 2), and
  // the chunk the sender waits for always belongs to a pair whose slots are.
  auto hasher = [&] {
    for (;;) {
      const size_t i = next.fetch_add(2);
      if (i >= n) return;
      const size_t cnt = std::min<size_t>(2, n - i);
      const size_t last = i + cnt - 1;
      {
        std::unique_lock<std::mutex> l(mu);
        cv_free.wait(l, [&] { return abort.load() || static_cast<int64_t>(last) < sent_chunks + static_cast<int64_t>(K); });
        if (abort.load()) return;
      }
      const uint64_t a = off + static_cast<uint64_t>(i) * chunk;
      size_t m[2] = {0, 0};
      for (size_t j = 0; j < cnt; ++j)
        m[j] = static_cast<size_t>(std::min<uint64_t>(chunk, length - static_cast<uint64_t>(i + j) * chunk));
      if (flow) {
        const int w = flow->wait_covered(a, a + m[0] + m[1], idle_timeout, &abort);
        if (w) {
          if (!abort.load())
            set_err(flow_wait_error(w, *flow));
          return;
        }
      }
      char* dst[2];
      for (size_t j = 0; j < cnt; ++j) {
        dst[j] = ring.data() + ((i + j) % K) * chunk;
        if (tritondl_hash::pread_full(fd, dst[j], m[j], static_cast<off_t>(a + j * chunk)) != m[j]) {
          set_err("source file shorter than expected");
          return;
        }
      }
      unsigned char d[2][32];
      if (cnt == 2) {
        tritondl_hash::sha256_pair(dst[0], m[0], dst[1], m[1], d[0], d[1]);
      } else {
        tritondl_hash::sha256_raw(dst[0], m[0], d[0]);
      }
      {
        std::lock_guard<std::mutex> l(mu);
        for (size_t j = 0; j < cnt; ++j) {
          hashes[(i + j) % K] = tritondl_hash::hex_raw(d[j], 32);
          ready[(i + j) % K] = static_cast<int64_t>(i + j);
        }
      }
      cv_ready.notify_all();
    }
  };

  const int nthreads = static_cast<int>(std::max<size_t>(1, std::min<size_t>(threads <= 0 ? 4 : threads, (n + 1) / 2)));
  std::shared_ptr<tritondl_hash::TaskPool::Group> pool;  // parked pool threads, not fresh ones per PUT
  if (n) pool = tritondl_hash::TaskPool::get().run(nthreads, hasher, "tdl-sha256");

  std::vector<std::string> heads;
  std::vector<struct iovec> iov;
  static const char crlf[] = "\r\n";
  size_t i = 0;
  while (i < n && r.err.empty()) {
    std::vector<std::string> hs;
    size_t j = i;
    {
      std::unique_lock<std::mutex> l(mu);
      while (!abort.load() && ready[i % K] != static_cast<int64_t>(i)) {
        if (io.aborted()) {  // the hashers may sit in a flow wait: stop them too
          if (worker_err.empty()) worker_err = "cancelled";
          abort.store(true);
          cv_free.notify_all();
          break;
        }
        cv_wait_ms(cv_ready, l, 20);
      }
      if (abort.load()) {
        r.err = worker_err;
        break;
      }
      while (j < n && j < i + batch && ready[j % K] == static_cast<int64_t>(j)) {
        hs.push_back(hashes[j % K]);
        ++j;
      }
    }
    heads.clear();
    heads.reserve(j - i);
    iov.clear();
    iov.reserve(3 * (j - i));
    for (size_t c = i; c < j; ++c) {
      const size_t m = static_cast<size_t>(std::min<uint64_t>(chunk, length - static_cast<uint64_t>(c) * chunk));
      char hx[32];
      std::snprintf(hx, sizeof hx, "%zx", m);
      heads.push_back(std::string(hx) + ";chunk-signature=" + signer.next(hs[c - i]) + "\r\n");
    }
    for (size_t c = i; c < j; ++c) {
      const size_t m = static_cast<size_t>(std::min<uint64_t>(chunk, length - static_cast<uint64_t>(c) * chunk));
      iov.push_back({const_cast<char*>(heads[c - i].data()), heads[c - i].size()});
      iov.push_back({ring.data() + (c % K) * chunk, m});
      iov.push_back({const_cast<char*>(crlf), 2});
      r.sent += m;
    }
    std::string e;
    if (!writev_all(io, iov, idle_timeout, flow, &e)) {
      r.err = e;
      break;
    }
    {
      std::lock_guard<std::mutex> l(mu);
      sent_chunks = static_cast<int64_t>(j);
    }
    cv_free.notify_all();
    i = j;
  }
  if (!r.err.empty()) {
    abort.store(true);
    cv_free.notify_all();
    cv_ready.notify_all();
  }
  if (r.err.empty()) {
    // the final frame first; the hashers are joined after it (off the critical path)
    const std::string fin = "0;chunk-signature=" + signer.next(signer.empty_hash) + "\r\n\r\n";
    std::string e;
    if (send_all(io, fin.data(), fin.size(), idle_timeout, flow, &e))
      r.last_sig = signer.prev();
    else
      r.err = e;
  }
  if (pool) pool->wait();
  return r;
}

// send() on a plain non-blocking socket until done; MSG_MORE holds a short
// header back so it leaves in the same segment as the payload that follows.
inline bool send_more(Stream& io, const char* p, size_t n, double idle_timeout, const Flow* flow, std::string* err) {
  const int sock = io.fd();
  auto last = Clock::now();
  while (n) {
    const ssize_t w = ::send(sock, p, n, MSG_MORE | MSG_NOSIGNAL);
    if (w > 0) {
      p += w;
      n -= static_cast<size_t>(w);
      last = Clock::now();
      continue;
    }
    if (w < 0 && errno == EINTR) continue;
    if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK) {
      *err = errno_str("send");
      return false;
    }
    if (stopped(io, flow)) {
      *err = "cancelled";
      return false;
    }
    if (since(last) > idle_timeout || wait_fd(sock, POLLOUT, 50) < 0) {
      *err = "send timeout";
      return false;
    }
  }
  return true;
}

// sendfile [o, o + n) of fd to a plain socket (page cache -> socket).
inline bool sendfile_all(Stream& io, int fd, uint64_t o, uint64_t n, double idle_timeout, const Flow* flow,
                         std::string* err) {
  const int sock = io.fd();
  auto last = Clock::now();
  uint64_t k = 0;
  while (k < n) {
    off_t pos = static_cast<off_t>(o + k);
    const ssize_t w = ::sendfile(sock, fd, &pos, static_cast<size_t>(n - k));
    if (w > 0) {
      k += static_cast<uint64_t>(w);
      last = Clock::now();
      continue;
    }
    if (w == 0) {
      *err = "source file shorter than expected";
      return false;
    }
    if (errno == EINTR) continue;
    if (errno != EAGAIN && errno != EWOULDBLOCK) {
      *err = errno_str("sendfile");
      return false;
    }
    if (stopped(io, flow)) {
      *err = "cancelled";
      return false;
    }
    if (since(last) > idle_timeout || wait_fd(sock, POLLOUT, 50) < 0) {
      *err = "send timeout";
      return false;
    }
  }
  return true;
}

// Where a PUT that follows a download hashes in SHA-NI pairs instead of
// 16-wide claims: a 16-chunk claim's digests come ~0.2 ms after its last
// byte lands (one 64 KiB chain per lane), and the sender, which sends in
// order, trails the download by that much.  Pairs over the first `head`
// (default 0) and the last `tail` (default 32) chunks let it start early
// and catch up before the end; wider pair regions measured no better
// (profiles/r03_mb_ab/SUMMARY.md).  TRITONDL_SHA_MB_HEAD /
// TRITONDL_SHA_MB_TAIL override (chunks).
inline size_t zc_env_chunks(const char* name, size_t dflt) {
  const char* v = std::getenv(name);
  return v && *v ? static_cast<size_t>(std::strtoul(v, nullptr, 10)) : dflt;
}
inline size_t zc_head_pairs() {
  static const size_t n = zc_env_chunks("TRITONDL_SHA_MB_HEAD", 0);
  return n;
}
inline size_t zc_tail_pairs() {
  static const size_t n = zc_env_chunks("TRITONDL_SHA_MB_TAIL", 32);
  return n;
}
// Streamed signed PUTs (a Flow): wide hash claims only over bytes already on
// disk, pairs at the receive frontier (TRITONDL_SHA_MB_FOLLOW=0: by position).
inline bool zc_follow() {
  static const bool on = zc_env_chunks("TRITONDL_SHA_MB_FOLLOW", 1) != 0;
  return on;
}
// One timing line per signed PUT on stderr (TRITONDL_ZC_TRACE=1; diagnostics).
inline bool zc_trace() {
  static const bool on = zc_env_chunks("TRITONDL_ZC_TRACE", 0) != 0;
  return on;
}
// Pre-map a streamed signed PUT's file mapping (TRITONDL_ZC_POPULATE=1).
inline bool zc_populate() {
  static const bool on = zc_env_chunks("TRITONDL_ZC_POPULATE", 0) != 0;
  return on;
}
// Signed zero-copy PUT pumps running in this process (parallel multipart parts).
inline std::atomic<int>& zc_active_pumps() {
  static std::atomic<int> n{0};
  return n;
}
// Frames per writev when the file is mapped (TRITONDL_ZC_WRITE_BATCH; 0/1 =
// a header send + a zero-copy sendfile per frame, the default).  Batching
// every ready frame into one writev won 5 % on the 10 MiB job while the
// hashers lagged the download (profiles/r05_batch_ab/); once they followed
// the receive frontier and the final frame went out first it lost 3 %
// (402.4 vs 390.3 jobs/s, 6 alternated runs, profiles/r05_batch_ab3/), and
// on parallel multipart parts its payload copy cost 10 % (r05_gib_ab/).
inline size_t zc_write_batch() {
  static const size_t n = zc_env_chunks("TRITONDL_ZC_WRITE_BATCH", 0);
  return n;
}

// send_chunked_zc: the aws-chunked body over a PLAIN socket with no payload
// copy through user space.  send_chunked reads every chunk into a ring
// (pread: one 10 MiB copy per 10 MiB job) and writev's the ring into the
// socket (a second one).  Here:
//   * chunk SHA-256s are computed straight from a read-only MAP_SHARED mapping
//     of the file (the download's page cache), when the file already spans the
//     range (it is pre-sized when the length is known); otherwise from a
//     per-task pread scratch;
//   * each frame's payload leaves with sendfile (page cache -> socket), and
//     only the ~90-byte chunk header is written from user space, with MSG_MORE
//     so it shares a segment with the payload after it.
// Hashers run ahead of the sender as far as the download allows (a digest is
// 32 bytes, so there is no ring to bound them).  TLS streams keep
// send_chunked: the record layer needs the bytes in user space anyway.
//
// With `gpu` (the HIP module's chunk API, pool mode on a CPU-bound node) each
// hasher task claims `gpu_batch` consecutive chunks and hashes them on the
// GPU in one call (a lane per chunk) instead of pairs on SHA-NI; a batch the
// GPU call fails on is hashed on the CPU.  One kernel per 16 MiB: a lane's
// 64 KiB chain takes ~2.6 ms whatever the lane count, and kernels from
// several streams of one process were measured to serialize (5 x 2 MiB
// batches per 10 MiB job cost ~9 ms per job, one 10 MiB batch ~3 ms).
inline SendResult send_chunked_zc(Stream& io, int fd, uint64_t off, uint64_t length, Flow* flow,
                                  ChunkSigner& signer, size_t chunk, int threads, double idle_timeout,
                                  const TdlGpuChunkApi* gpu = nullptr, size_t gpu_batch = 256) {
  SendResult r;
  if (chunk == 0) {
    r.err = "chunk size must be > 0";
    return r;
  }
  const size_t n = static_cast<size_t>((length + chunk - 1) / chunk);
  std::vector<std::array<unsigned char, 32>> dig(n);
  std::vector<uint8_t> ready(n, 0);
  // TRITONDL_ZC_TRACE=1: per chunk, when its bytes were on disk for its hasher,
  // when its digest was ready, when the sender wrote it (ns since the pump began);
  // one summary line per PUT on stderr
  const bool ztrace = zc_trace();
  const auto t_start = Clock::now();
  std::vector<int64_t> t_cov(ztrace ? n : 0), t_hash(ztrace ? n : 0), t_sent(ztrace ? n : 0);
  std::atomic<size_t> n_wide{0}, n_pair{0};
  auto ns_now = [&] {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t_start).count();
  };
  std::mutex mu;
  std::condition_variable cv_ready;
  std::atomic<bool> abort{false};
  std::string worker_err;
  std::atomic<size_t> next{0};

  // the mapping: only over bytes the file already holds (a read past EOF of a
  // mapping is SIGBUS, a pread past EOF is a short read)
  const char* map = nullptr;
  size_t map_len = 0;
  uint64_t base = 0;
  struct stat st;
  if (length && ::fstat(fd, &st) == 0 && static_cast<uint64_t>(st.st_size) >= off + length) {
    const uint64_t page = static_cast<uint64_t>(::sysconf(_SC_PAGESIZE));
    base = off & ~(page - 1);
    map_len = static_cast<size_t>(off + length - base);
    void* m = ::mmap(nullptr, map_len, PROT_READ, MAP_SHARED, fd, static_cast<off_t>(base));
    if (m != MAP_FAILED) {
      map = static_cast<const char*>(m);
      ::madvise(m, map_len, MADV_SEQUENTIAL);
      // map every page now, in one call, instead of one minor fault per 4 KiB page in
      // the hashers and the sender (MADV_POPULATE_READ, Linux 5.14; ignored before)
      if (zc_populate()) ::madvise(m, map_len, 22 /* MADV_POPULATE_READ */);
    }
  }

  auto set_err = [&](const std::string& e) {
    {
      std::lock_guard<std::mutex> l(mu);
      if (worker_err.empty()) worker_err = e;
      abort.store(true);
    }
    cv_ready.notify_all();
  };
  // the sender sleeps on one chunk at a time: a hasher wakes it only when it
  // just finished that chunk (not on every pair, most of which it is not
  // waiting for yet)
  size_t sender_wants = SIZE_MAX;
  auto publish = [&](size_t i, size_t cnt) {
    std::lock_guard<std::mutex> l(mu);
    for (size_t j = 0; j < cnt; ++j) ready[i + j] = 1;
    if (sender_wants >= i && sender_wants < i + cnt) cv_ready.notify_one();
  };
  // Chunks per claim: 16 for the 16-lane AVX-512 kernel, else an SHA-NI
  // pair.  The last 32 chunks always go in pairs (zc_tail_pairs): a 16-chunk
  // claim cannot start before its last byte lands, so near the end of a
  // download it would leave 1 MiB to hash on one core after the transfer;
  // pairs spread that over the hashers.
  const size_t wide = gpu ? 0 : tritondl_hash::sha256_claim();
  const size_t per = gpu ? std::max<size_t>(1, gpu_batch) : wide;
  const size_t lead = flow ? zc_head_pairs() : 0, trail = zc_tail_pairs();
  const bool follow = flow != nullptr && zc_follow();
  auto claim = [&](size_t* take) {
    if (gpu || wide <= 2) {
      *take = per;
      return next.fetch_add(per);
    }
    size_t i = next.load();
    do {
      bool w = i >= lead && i + wide + trail <= n;
      if (w && follow) {
        // a wide claim waits for all its bytes: take one only where the download
        // has already landed them (a hasher catching up); at the receive frontier
        // pairs keep each chunk's digest right behind its bytes
        const uint64_t a = off + static_cast<uint64_t>(i) * chunk, span = static_cast<uint64_t>(wide) * chunk;
        w = flow->covered_prefix(a, a + span) >= span;
      }
      *take = w ? wide : 2;
    } while (!next.compare_exchange_weak(i, i + *take));
    return i;
  };
  auto hasher = [&] {
    std::vector<char> scratch(map ? 0 : per * chunk);
    for (;;) {
      size_t take = 0;
      const size_t i = claim(&take);
      if (i >= n || abort.load()) return;
      if (gpu) {
        const size_t cnt = std::min(per, n - i);
        const uint64_t a = off + static_cast<uint64_t>(i) * chunk;
        const size_t len = static_cast<size_t>(std::min<uint64_t>(cnt * chunk, off + length - a));
        if (flow) {
          const int w = flow->wait_covered(a, a + len, idle_timeout, &abort);
          if (w) {
            if (!abort.load())
              set_err(flow_wait_error(w, *flow));
            return;
          }
        }
        const char* src = map ? map + (a - base) : scratch.data();
        if (!map && tritondl_hash::pread_full(fd, scratch.data(), len, static_cast<off_t>(a)) != len) {
          set_err("source file shorter than expected");
          return;
        }
        char gerr[256] = {0};
        if (gpu->sha256_chunks(src, len, chunk, dig[i].data(), gerr, sizeof gerr) != 0) {
          for (size_t j = 0; j < cnt; ++j) {  // the GPU failed this batch: SHA-NI instead
            const size_t mj = std::min<size_t>(chunk, len - j * chunk);
            tritondl_hash::sha256_raw(src + j * chunk, mj, dig[i + j].data());
          }
        }
        publish(i, cnt);
        continue;
      }
      const size_t cnt = std::min(take, n - i);
      const uint64_t a = off + static_cast<uint64_t>(i) * chunk;
      size_t m[16] = {0};
      uint64_t span = 0;
      for (size_t j = 0; j < cnt; ++j) {
        m[j] = static_cast<size_t>(std::min<uint64_t>(chunk, length - static_cast<uint64_t>(i + j) * chunk));
        span += m[j];
      }
      if (flow) {
        const int w = flow->wait_covered(a, a + span, idle_timeout, &abort);
        if (w) {
          if (!abort.load())
            set_err(flow_wait_error(w, *flow));
          return;
        }
      }
      if (ztrace) {
        const int64_t t = ns_now();
        for (size_t j = 0; j < cnt; ++j) t_cov[i + j] = t;
        (cnt > 2 ? n_wide : n_pair).fetch_add(1);
      }
      const void* src[16];
      for (size_t j = 0; j < cnt; ++j) {
        if (map) {
          src[j] = map + (a + j * chunk - base);
        } else {
          char* d = scratch.data() + j * chunk;
          if (tritondl_hash::pread_full(fd, d, m[j], static_cast<off_t>(a + j * chunk)) != m[j]) {
            set_err("source file shorter than expected");
            return;
          }
          src[j] = d;
        }
      }
      tritondl_hash::sha256_batch(src, m, cnt, dig[i].data());
      if (ztrace) {
        const int64_t t = ns_now();
        for (size_t j = 0; j < cnt; ++j) t_hash[i + j] = t;
      }
      publish(i, cnt);
    }
  };
  const int nthreads = static_cast<int>(
      std::max<size_t>(1, std::min<size_t>(threads <= 0 ? 4 : threads, (n + per - 1) / per)));
  std::shared_ptr<tritondl_hash::TaskPool::Group> pool;
  if (n) pool = tritondl_hash::TaskPool::get().run(nthreads, hasher, gpu ? "tdl-gpu-sha256" : "tdl-sha256");

  std::string head;
  char hx[32];
  const size_t batch = map ? zc_write_batch() : 0;
  std::vector<std::string> heads;
  std::vector<struct iovec> iov;
  // batching costs a copy of every payload into the socket; it pays for one PUT whose
  // tail is the job's critical path, not for parallel multipart parts that are bound by
  // CPU (1 GiB job: 12.0 vs 10.5 jobs/s with batching; profiles/r05_gib_ab/)
  struct Active {
    Active() { zc_active_pumps().fetch_add(1); }
    ~Active() { zc_active_pumps().fetch_sub(1); }
  } active;
  for (size_t c = 0; c < n && r.err.empty(); ++c) {
    size_t avail = 1;  // chunks from c on whose digests are ready
    {
      std::unique_lock<std::mutex> l(mu);
      sender_wants = c;
      while (!abort.load() && !ready[c]) {
        if (io.aborted()) {  // the hashers may sit in a flow wait: stop them too
          if (worker_err.empty()) worker_err = "cancelled";
          abort.store(true);
          break;
        }
        cv_wait_ms(cv_ready, l, 20);
      }
      sender_wants = SIZE_MAX;
      if (abort.load()) {
        r.err = worker_err;
        break;
      }
      while (batch > 1 && avail < batch && c + avail < n && ready[c + avail]) ++avail;
    }
    if (batch > 1 && zc_active_pumps().load(std::memory_order_relaxed) == 1) {
      // every ready frame in one writev from the mapping: headers and payloads
      // interleaved, one syscall per batch instead of two per 64 KiB frame
      heads.assign(avail, std::string());
      iov.clear();
      uint64_t bytes = 0;
      for (size_t k = 0; k < avail; ++k) {
        const size_t cc = c + k;
        const uint64_t a = off + static_cast<uint64_t>(cc) * chunk;
        const size_t m = static_cast<size_t>(std::min<uint64_t>(chunk, length - static_cast<uint64_t>(cc) * chunk));
        std::snprintf(hx, sizeof hx, "%zx", m);
        std::string& h = heads[k];
        h.assign(cc ? "\r\n" : "");
        h += hx;
        h += ";chunk-signature=";
        h += signer.next(tritondl_hash::hex_raw(dig[cc].data(), 32));
        h += "\r\n";
        iov.push_back({h.data(), h.size()});
        iov.push_back({const_cast<char*>(map + (a - base)), m});
        bytes += m;
      }
      if (!writev_all(io, iov, idle_timeout, flow, &r.err)) break;
      r.sent += bytes;
      if (ztrace) {
        const int64_t t = ns_now();
        for (size_t k = 0; k < avail; ++k) t_sent[c + k] = t;
      }
      c += avail - 1;
      continue;
    }
    const uint64_t a = off + static_cast<uint64_t>(c) * chunk;
    const size_t m = static_cast<size_t>(std::min<uint64_t>(chunk, length - static_cast<uint64_t>(c) * chunk));
    std::snprintf(hx, sizeof hx, "%zx", m);
    head.assign(c ? "\r\n" : "");
    head += hx;
    head += ";chunk-signature=";
    head += signer.next(tritondl_hash::hex_raw(dig[c].data(), 32));
    head += "\r\n";
    if (!send_more(io, head.data(), head.size(), idle_timeout, flow, &r.err)) break;
    if (!sendfile_all(io, fd, a, m, idle_timeout, flow, &r.err)) break;
    r.sent += m;
  }
  if (!r.err.empty()) set_err(r.err);
  if (r.err.empty()) {
    // the final frame goes out before the clean-up: joining the hashers and
    // unmapping the file (a TLB shootdown on every core that touched it) are
    // not on the request's critical path
    const std::string fin = std::string(n ? "\r\n" : "") + "0;chunk-signature=" + signer.next(signer.empty_hash) +
                            "\r\n\r\n";
    if (send_all(io, fin.data(), fin.size(), idle_timeout, flow, &r.err)) r.last_sig = signer.prev();
  }
  if (ztrace && n && r.err.empty()) {
    // the last chunk's bytes landing = the download's end, as its hasher saw it
    int64_t cov_last = 0, hash_last = 0, sent_last = t_sent[n - 1], max_lag = 0;
    for (size_t k = 0; k < n; ++k) {
      cov_last = std::max(cov_last, t_cov[k]);
      hash_last = std::max(hash_last, t_hash[k]);
      max_lag = std::max(max_lag, t_sent[k] - t_cov[k]);
    }
    std::fprintf(stderr,
                 "zc-trace n=%zu wide=%zu pair=%zu cov_last_us=%.1f hash_last_us=%.1f sent_last_us=%.1f "
                 "fin_us=%.1f max_cov_to_sent_us=%.1f\n",
                 n, n_wide.load(), n_pair.load(), cov_last / 1e3, hash_last / 1e3, sent_last / 1e3, ns_now() / 1e3,
                 max_lag / 1e3);
  }
  if (pool) pool->wait();
  if (map) ::munmap(const_cast<char*>(map), map_len);
  return r;
}

// Zero-copy chunked sends for plain sockets (TRITONDL_RELAY_ZC=0: the ring path).
inline bool zc_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("TRITONDL_RELAY_ZC");
    return !(v && (std::strcmp(v, "0") == 0 || std::strcmp(v, "off") == 0 || std::strcmp(v, "false") == 0));
  }();
  return on;
}

inline SendResult send_body(Stream& io, const std::string& head, int fd, uint64_t off, uint64_t length, Flow* flow,
                            int mode, const std::string& key, const std::string& amzdate, const std::string& scope,
                            const std::string& seed, size_t chunk, int threads, double idle_timeout,
                            const TdlGpuChunkApi* gpu = nullptr) {
  SendResult r;
  if (mode == 0) {
    if (!send_all(io, head.data(), head.size(), idle_timeout, flow, &r.err)) return r;
    return send_plain(io, fd, off, length, flow, idle_timeout);
  }
  ChunkSigner signer(key, amzdate, scope, seed);
  if (io.plain() && (zc_enabled() || gpu)) {
    // the request head goes out with MSG_MORE too: it shares the first segment
    if (!send_more(io, head.data(), head.size(), idle_timeout, flow, &r.err)) return r;
    return send_chunked_zc(io, fd, off, length, flow, signer, chunk, threads, idle_timeout, gpu);
  }
  if (!send_all(io, head.data(), head.size(), idle_timeout, flow, &r.err)) return r;
  return send_chunked(io, fd, off, length, flow, signer, chunk, threads, idle_timeout);
}

// ---------------------------------------------------------------------------
// recv_verify_chunked: the SERVER side of send_chunked (the fake S3's PUT
// path).  Receives exactly raw_len body bytes, parses aws-chunked frames and
// verifies every chunk signature.  Windows of ~`window` raw bytes alternate
// between two buffers: while window k is verified (payload SHA-256s as a
// parallel map, then the serial HMAC chain) window k+1 is being received.
struct VerifyResult {
  uint64_t decoded = 0;
  std::string err;
  std::string data;  // decoded payload when keep
  // content fingerprint of the decoded payload, free from the chunk
  // verification: the payload SHA-256s of its 64 KiB leaves, concatenated
  // (32 bytes per leaf).  Only when every frame but the last carries exactly
  // one 64 KiB leaf (the client's chunking); empty otherwise.  Leaf lists of
  // consecutive multipart parts concatenate to the whole object's
  std::string leaf_hashes;
};

constexpr size_t kLeafBytes = 64u << 10;

// leaf_hashes from the frames' payload SHA-256s (raw, 32 bytes each, in
// order; zero-length frames excluded by the caller), if the frames are leaves
inline std::string leaf_hashes_of(std::string hashes, const std::vector<size_t>& sizes) {
  for (size_t i = 0; i + 1 < sizes.size(); ++i)
    if (sizes[i] != kLeafBytes) return std::string();
  if (!sizes.empty() && (sizes.back() == 0 || sizes.back() > kLeafBytes)) return std::string();
  return hashes;
}

struct RawFrame {
  size_t off, n;  // payload offset in its window buffer, payload length
  size_t sig;     // offset of the 64-hex claimed signature
};

// Parse whole frames in [0, have); stops at the first incomplete one.
// Returns the end of the last whole frame; sets *final on the 0-length frame.
inline size_t parse_frames(const char* raw, size_t have, std::vector<RawFrame>* out, bool* final, std::string* err) {
  size_t pos = 0;
  while (pos < have) {
    size_t hexend = pos;
    while (hexend < have && hexend - pos < 16 && std::isxdigit(static_cast<unsigned char>(raw[hexend]))) ++hexend;
    if (hexend == have || hexend + 17 + 64 + 2 > have) {
      if (hexend - pos >= 16 && hexend < have) *err = "malformed aws-chunked framing";
      break;  // header incomplete
    }
    if (hexend == pos || std::memcmp(raw + hexend, ";chunk-signature=", 17) != 0) {
      *err = "malformed aws-chunked framing";
      break;
    }
    const size_t n = std::strtoull(std::string(raw + pos, hexend - pos).c_str(), nullptr, 16);
    const size_t sig = hexend + 17;
    const size_t a = sig + 64 + 2;
    if (raw[sig + 64] != '\r' || raw[sig + 65] != '\n') {
      *err = "malformed chunk header";
      break;
    }
    if (n > (size_t(1) << 40)) {
      *err = "chunk too large";
      break;
    }
    if (a + n + 2 > have) break;  // payload incomplete
    if (raw[a + n] != '\r' || raw[a + n + 1] != '\n') {
      *err = "chunk not terminated";
      break;
    }
    out->push_back({a, n, sig});
    pos = a + n + 2;
    if (n == 0) {
      *final = true;
      break;
    }
  }
  return pos;
}

inline VerifyResult recv_verify_windowed(Stream& io, uint64_t raw_len, const char* prefix, size_t plen,
                                         const std::string& key, const std::string& amzdate, const std::string& scope,
                                         const std::string& seed, bool keep, int threads, double idle_timeout,
                                         size_t window = 4u << 20) {
  VerifyResult r;
  Buf buf[2];
  int cur = 0;
  size_t have = 0;
  uint64_t received = 0;
  ChunkSigner signer(key, amzdate, scope, seed);
  std::thread verifier;
  std::string verr;  // verifier error (read after join)
  bool final_seen = false;
  const int t = threads <= 0 ? 4 : threads;
  std::string leaf_hashes;          // raw payload SHA-256s of the non-empty frames, in order
  std::vector<size_t> leaf_sizes;   // (appended by one verifier thread at a time)

  auto join = [&] {
    if (verifier.joinable()) verifier.join();
  };
  auto ensure = [&](Buf& b, size_t n, size_t keep) { b.ensure(n, keep); };
  const size_t pre = static_cast<size_t>(std::min<uint64_t>(plen, raw_len));
  ensure(buf[cur], std::max(window, pre) + 1, 0);
  std::memcpy(buf[cur].data(), prefix, pre);
  have = pre;
  received = pre;
  auto last = Clock::now();

  while (!final_seen) {
    // fill the current window
    while (have < window && received < raw_len) {
      ensure(buf[cur], have + std::min<uint64_t>(window, raw_len - received), have);
      const size_t cap = static_cast<size_t>(std::min<uint64_t>(buf[cur].size() - have, raw_len - received));
      const ssize_t n = recv_wait(io, buf[cur].data() + have, cap, &last, idle_timeout, nullptr, &r.err);
      if (n > 0) {
        have += static_cast<size_t>(n);
        received += static_cast<uint64_t>(n);
        continue;
      }
      if (n == 0) r.err = "client closed inside the request body";
      break;
    }
    if (!r.err.empty()) break;
    std::vector<RawFrame> frames;
    std::string perr;
    const size_t end = parse_frames(buf[cur].data(), have, &frames, &final_seen, &perr);
    if (!perr.empty()) {
      r.err = perr;
      break;
    }
    if (frames.empty()) {
      if (received >= raw_len) {
        r.err = "truncated chunk";
        break;
      }
      window = std::max(window, have + (1u << 20));  // one frame bigger than the window: grow it
      continue;
    }
    join();
    if (!verr.empty()) {
      r.err = verr;
      break;
    }
    const int nxt = 1 - cur;
    ensure(buf[nxt], std::max(window, have - end) + 1, 0);
    if (have > end) std::memcpy(buf[nxt].data(), buf[cur].data() + end, have - end);
    const size_t leftover = have - end;
    const size_t dbase = r.data.size();
    size_t wtotal = 0;
    for (const RawFrame& f : frames) wtotal += f.n;
    r.decoded += wtotal;
    if (keep) r.data.resize(dbase + wtotal);
    Buf* wb = &buf[cur];
    verifier = std::thread([&, wb, frames = std::move(frames), dbase] {
      tritondl_hash::name_thread("tdl-verify");
      const char* raw = wb->data();
      std::vector<std::string> h(frames.size());
      std::string rawh(32 * frames.size(), '\0');
      std::vector<size_t> doff(frames.size() + 1, 0);
      for (size_t i = 0; i < frames.size(); ++i) doff[i + 1] = doff[i] + frames[i].n;
      const int used = static_cast<int>(std::min<size_t>(static_cast<size_t>(t), std::max<size_t>(1, doff.back() >> 20)));
      const size_t nf = frames.size();
      tritondl_hash::parallel_for((nf + 1) / 2, used, [&](size_t k) {  // frame pairs: SHA-NI lockstep
        const size_t i = 2 * k;
        unsigned char d[2][32];
        const RawFrame& f = frames[i];
        if (i + 1 < nf) {
          const RawFrame& g = frames[i + 1];
          tritondl_hash::sha256_pair(raw + f.off, f.n, raw + g.off, g.n, d[0], d[1]);
          h[i + 1] = tritondl_hash::hex_raw(d[1], 32);
          std::memcpy(&rawh[32 * (i + 1)], d[1], 32);
          if (keep && g.n) std::memcpy(&r.data[dbase + doff[i + 1]], raw + g.off, g.n);
        } else {
          tritondl_hash::sha256_raw(raw + f.off, f.n, d[0]);
        }
        h[i] = tritondl_hash::hex_raw(d[0], 32);
        std::memcpy(&rawh[32 * i], d[0], 32);
        if (keep && f.n) std::memcpy(&r.data[dbase + doff[i]], raw + f.off, f.n);
      });
      for (size_t i = 0; i < frames.size(); ++i) {
        if (std::memcmp(signer.next(h[i]).data(), raw + frames[i].sig, 64) != 0) {
          verr = "chunk signature mismatch";
          return;
        }
        if (frames[i].n) {
          leaf_hashes.append(rawh, 32 * i, 32);
          leaf_sizes.push_back(frames[i].n);
        }
      }
    });
    cur = nxt;
    have = leftover;
  }
  join();
  if (r.err.empty() && !verr.empty()) r.err = verr;
  if (r.err.empty() && (have != 0 || received != raw_len)) r.err = "trailing bytes after final chunk";
  if (r.err.empty()) r.leaf_hashes = leaf_hashes_of(std::move(leaf_hashes), leaf_sizes);
  return r;
}

// Streamed variant for bodies that fit one buffer (every PUT / part our
// client sends): the receiver thread lands bytes contiguously, parses frames
// as soon as they are complete and publishes them; a per-request hasher pool
// hashes published frames in place; the receiver checks the signature chain
// in order as hashes become ready.  The last frame's hash + HMAC is all that
// remains after the last byte arrives.
struct StreamFrame {
  size_t off, n, sig;
  unsigned char h[32];
  std::atomic<uint8_t> ready{0};
};

inline VerifyResult recv_verify_stream(Stream& io, uint64_t raw_len, const char* prefix, size_t plen,
                                       const std::string& key, const std::string& amzdate, const std::string& scope,
                                       const std::string& seed, bool keep, int threads, double idle_timeout) {
  VerifyResult r;
  Buf whole(static_cast<size_t>(raw_len) + 1);
  char* raw = whole.data();
  const size_t pre = static_cast<size_t>(std::min<uint64_t>(plen, raw_len));
  std::memcpy(raw, prefix, pre);
  size_t have = pre, parsed = 0;
  constexpr size_t kB = 1024;                                        // frames per table block
  const size_t max_frames = static_cast<size_t>(raw_len / 86) + 2;  // a frame is >= 86 bytes
  std::vector<std::unique_ptr<StreamFrame[]>> blocks((max_frames + kB - 1) / kB);
  auto frame = [&](size_t j) -> StreamFrame& { return blocks[j / kB][j % kB]; };
  std::mutex mu;
  std::condition_variable cv_pub, cv_ready;
  size_t published = 0;  // guarded by mu
  bool parse_done = false, stop = false;
  bool final_seen = false;

  // Frames are claimed in pairs (SHA-NI lockstep) as they are published, or
  // 16 at a time for the AVX-512 kernel once the hashers have fallen behind
  // (a backlog of >= 32 frames): then throughput is what counts, while
  // hashers keeping up with the receiver stay on pairs, so the last frame's
  // hash still lands right after its bytes.
  size_t claimed = 0;  // guarded by mu
  const size_t wide = tritondl_hash::sha256_claim();
  auto hasher = [&] {
    for (;;) {
      size_t j, cnt;
      {
        std::unique_lock<std::mutex> l(mu);
        cv_pub.wait(l, [&] { return stop || parse_done || published >= claimed + 2; });
        if (stop || published == claimed) return;  // (parse done: nothing left)
        const size_t avail = published - claimed;
        cnt = wide > 2 && avail >= 2 * wide ? wide : std::min<size_t>(2, avail);
        j = claimed;
        claimed += cnt;
      }
      const void* p[16];
      size_t n[16];
      unsigned char d[16 * 32];
      for (size_t k = 0; k < cnt; ++k) {
        const StreamFrame& f = frame(j + k);
        p[k] = raw + f.off;
        n[k] = f.n;
      }
      tritondl_hash::sha256_batch(p, n, cnt, d);
      for (size_t k = 0; k < cnt; ++k) {
        StreamFrame& f = frame(j + k);
        std::memcpy(f.h, d + 32 * k, 32);
        f.ready.store(1, std::memory_order_release);
      }
      {
        std::lock_guard<std::mutex> l(mu);  // pairs with the checker's wait
      }
      cv_ready.notify_one();
    }
  };
  const int nthreads = std::max(1, threads <= 0 ? 4 : threads);
  auto pool = tritondl_hash::TaskPool::get().run(nthreads, hasher, "tdl-s3verify");

  ChunkSigner signer(key, amzdate, scope, seed);
  size_t checked = 0;
  auto check_ready = [&](bool wait_all) -> bool {
    for (;;) {
      size_t pub;
      {
        std::unique_lock<std::mutex> l(mu);
        pub = published;
        if (wait_all && checked < pub && !frame(checked).ready.load(std::memory_order_acquire))
          cv_wait_ms(cv_ready, l, 5, [&] { return frame(checked).ready.load(std::memory_order_acquire) != 0; });
      }
      while (checked < pub && frame(checked).ready.load(std::memory_order_acquire)) {
        StreamFrame& f = frame(checked);
        if (std::memcmp(signer.next(tritondl_hash::hex(std::string(reinterpret_cast<char*>(f.h), 32))).data(),
                        raw + f.sig, 64) != 0)
          return false;
        ++checked;
      }
      if (!wait_all || checked >= pub) return true;
    }
  };

  auto last = Clock::now();
  bool sig_ok = true;
  while (r.err.empty()) {
    // parse every complete frame in [parsed, have)
    std::vector<RawFrame> fr;
    std::string perr;
    bool fin = false;
    const size_t end = parsed + parse_frames(raw + parsed, have - parsed, &fr, &fin, &perr);
    if (!perr.empty()) {
      r.err = perr;
      break;
    }
    if (!fr.empty()) {
      std::lock_guard<std::mutex> l(mu);
      for (const RawFrame& x : fr) {
        const size_t j = published;
        if (j >= max_frames) {
          r.err = "too many chunks";
          break;
        }
        if (!blocks[j / kB]) blocks[j / kB].reset(new StreamFrame[kB]);
        StreamFrame& f = frame(j);
        f.off = parsed + x.off;
        f.n = x.n;
        f.sig = parsed + x.sig;
        r.decoded += x.n;
        ++published;
      }
      parsed = end;
    }
    if (!fr.empty()) cv_pub.notify_all();
    if (!r.err.empty()) break;
    if (fin) {
      final_seen = true;
      break;
    }
    if (!(sig_ok = check_ready(false))) break;
    if (have >= raw_len) {
      r.err = "truncated chunk";
      break;
    }
    const ssize_t n = recv_wait(io, raw + have, static_cast<size_t>(raw_len - have), &last, idle_timeout, nullptr,
                                &r.err);
    if (n > 0) {
      have += static_cast<size_t>(n);
      continue;
    }
    if (n == 0) r.err = "client closed inside the request body";
    break;
  }
  {
    std::lock_guard<std::mutex> l(mu);
    parse_done = true;
    if (!r.err.empty() || !sig_ok) stop = true;
  }
  cv_pub.notify_all();
  if (r.err.empty() && sig_ok) sig_ok = check_ready(true);
  {
    std::lock_guard<std::mutex> l(mu);
    stop = true;
  }
  cv_pub.notify_all();
  pool->wait();
  if (r.err.empty() && !sig_ok) r.err = "chunk signature mismatch";
  if (r.err.empty() && (!final_seen || parsed != raw_len || have != raw_len)) r.err = "trailing bytes after final chunk";
  if (r.err.empty()) {
    std::string hs;
    std::vector<size_t> sizes;
    hs.reserve(32 * published);
    sizes.reserve(published);
    for (size_t j = 0; j < published; ++j) {
      if (!frame(j).n) continue;
      hs.append(reinterpret_cast<const char*>(frame(j).h), 32);
      sizes.push_back(frame(j).n);
    }
    r.leaf_hashes = leaf_hashes_of(std::move(hs), sizes);
  }
  if (r.err.empty() && keep) {
    r.data.resize(static_cast<size_t>(r.decoded));
    size_t o = 0;
    for (size_t j = 0; j < published; ++j) {
      std::memcpy(&r.data[o], raw + frame(j).off, frame(j).n);
      o += frame(j).n;
    }
  }
  return r;
}

// recv_leaf_hashes: the fake S3's side of an UNSIGNED-PAYLOAD PUT with a
// content check — receive exactly `len` body bytes and return the SHA-256 of
// every 64 KiB leaf (VerifyResult.leaf_hashes).  Leaves are hashed by a
// hasher pool as soon as they have landed, 16 at a time for the AVX-512
// kernel when a backlog builds up, so little is left after the last byte.
inline VerifyResult recv_leaf_hashes(Stream& io, uint64_t len, const char* prefix, size_t plen, int threads,
                                     double idle_timeout) {
  VerifyResult r;
  Buf whole(static_cast<size_t>(len) + 1);
  char* raw = whole.data();
  const size_t pre = static_cast<size_t>(std::min<uint64_t>(plen, len));
  std::memcpy(raw, prefix, pre);
  const size_t nleaves = static_cast<size_t>((len + kLeafBytes - 1) / kLeafBytes);
  std::string hashes(32 * nleaves, '\0');
  std::mutex mu;
  std::condition_variable cv;
  size_t landed = 0, claimed = 0;  // leaves fully received / taken by a hasher (guarded by mu)
  bool done = false;
  const size_t wide = tritondl_hash::sha256_claim();
  auto hasher = [&] {
    for (;;) {
      size_t j, cnt;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return done || landed >= claimed + 2; });
        if (landed == claimed) return;  // done, nothing left
        const size_t avail = landed - claimed;
        cnt = wide > 2 && avail >= 2 * wide ? wide : std::min<size_t>(2, avail);
        j = claimed;
        claimed += cnt;
      }
      const void* p[16];
      size_t n[16];
      for (size_t k = 0; k < cnt; ++k) {
        const uint64_t off = static_cast<uint64_t>(j + k) * kLeafBytes;
        p[k] = raw + off;
        n[k] = static_cast<size_t>(std::min<uint64_t>(kLeafBytes, len - off));
      }
      tritondl_hash::sha256_batch(p, n, cnt, reinterpret_cast<unsigned char*>(&hashes[32 * j]));
    }
  };
  const int nthreads = std::max(1, threads <= 0 ? 4 : threads);
  auto pool = tritondl_hash::TaskPool::get().run(nthreads, hasher, "tdl-s3leaf");
  size_t have = pre;
  auto last = Clock::now();
  auto publish = [&] {
    const size_t full = have == len ? nleaves : have / kLeafBytes;
    std::lock_guard<std::mutex> l(mu);
    if (full > landed) {
      landed = full;
      cv.notify_all();
    }
  };
  publish();
  while (have < len) {
    const ssize_t n = recv_wait(io, raw + have, static_cast<size_t>(len - have), &last, idle_timeout, nullptr, &r.err);
    if (n <= 0) {
      if (n == 0) r.err = "client closed inside the request body";
      break;
    }
    have += static_cast<size_t>(n);
    publish();
  }
  {
    std::lock_guard<std::mutex> l(mu);
    done = true;
    if (!r.err.empty()) landed = claimed;  // drop what has not been claimed
  }
  cv.notify_all();
  pool->wait();
  r.decoded = have;
  if (r.err.empty()) r.leaf_hashes = std::move(hashes);
  return r;
}

inline VerifyResult recv_verify_chunked(Stream& io, uint64_t raw_len, const char* prefix, size_t plen,
                                        const std::string& key, const std::string& amzdate, const std::string& scope,
                                        const std::string& seed, bool keep, int threads, double idle_timeout) {
  if (raw_len <= (uint64_t(256) << 20))
    return recv_verify_stream(io, raw_len, prefix, plen, key, amzdate, scope, seed, keep, threads, idle_timeout);
  return recv_verify_windowed(io, raw_len, prefix, plen, key, amzdate, scope, seed, keep, threads, idle_timeout);
}

// Exact on-the-wire size of an aws-chunked body of `len` payload bytes.
inline uint64_t chunked_length(uint64_t len, uint64_t chunk) {
  return tritondl_hash::aws_chunk_encoded_size(static_cast<size_t>(len), static_cast<size_t>(chunk), true);
}

// ---------------------------------------------------------------------------
// CompletionPort: pumps started on the native task pool report back to ONE
// event loop through an eventfd, instead of running inside an interpreter
// executor thread.  An executor hop costs a Python thread wake-up, two GIL
// hand-offs, a future callback and the loop's self-pipe write (~30-70 µs of
// CPU); here the pump thread never touches the interpreter, and the loop's
// reader drains every finished pump per wake-up.  The eventfd is written
// only when the queue goes from empty to non-empty (the reader takes the
// whole queue under the same lock), so a burst of completions costs one
// wake-up.
class CompletionPort {
 public:
  struct Done {
    uint64_t id = 0;
    int kind = 0;  // 1 = recv_body, 2 = send_body
    bool chunked = false;
    RecvResult rr;
    SendResult sr;
  };

  CompletionPort() : efd_(::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC)) {
    if (efd_ < 0) throw std::runtime_error(errno_str("eventfd"));
  }
  ~CompletionPort() { ::close(efd_); }
  CompletionPort(const CompletionPort&) = delete;
  CompletionPort& operator=(const CompletionPort&) = delete;

  int fd() const { return efd_; }
  size_t inflight() const { return inflight_.load(); }

  void started() { inflight_.fetch_add(1); }
  void post(Done&& d) {
    bool was_empty;
    {
      std::lock_guard<std::mutex> l(mu_);
      was_empty = q_.empty();
      q_.push_back(std::move(d));
      inflight_.fetch_sub(1);
    }
    if (was_empty) {
      const uint64_t one = 1;
      ssize_t w;
      do w = ::write(efd_, &one, sizeof one);
      while (w < 0 && errno == EINTR);
    }
  }
  // Everything finished so far (clears the eventfd first, so a post racing
  // with this call re-arms it or lands in this batch).
  std::vector<Done> reap() {
    uint64_t v;
    while (::read(efd_, &v, sizeof v) < 0 && errno == EINTR) {
    }
    std::vector<Done> out;
    std::lock_guard<std::mutex> l(mu_);
    out.swap(q_);
    return out;
  }
  // Blocks until something is queued or timeout_ms passed (tests / the self-test).
  bool wait(int timeout_ms) const {
    pollfd p{efd_, POLLIN, 0};
    return ::poll(&p, 1, timeout_ms) > 0;
  }

 private:
  int efd_;
  std::atomic<size_t> inflight_{0};
  std::mutex mu_;
  std::vector<Done> q_;
};

// Start a pump on the task pool; `done` is posted to `port` when it returns.
// The closure owns everything the pump touches (stream and flow by
// shared_ptr), so the caller may drop its references at once; the file
// descriptors stay the caller's, who must not close them before the
// completion (rawhttp.run_pump awaits it even when cancelled).
template <class Pump>
inline void start_pump(std::shared_ptr<CompletionPort> port, uint64_t id, int kind, bool chunked, Pump pump,
                       const char* name) {
  port->started();
  tritondl_hash::TaskPool::get().run(
      1,
      [port, id, kind, chunked, pump]() mutable {
        CompletionPort::Done d;
        d.id = id;
        d.kind = kind;
        d.chunked = chunked;
        try {
          pump(d);
        } catch (const std::exception& e) {
          (kind == 1 ? d.rr.err : d.sr.err) = std::string("native pump failed: ") + e.what();
        }
        port->post(std::move(d));
      },
      name);
}

}  // namespace tritondl_relay
