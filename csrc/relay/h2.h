// HTTP/2 client session pump (RFC 9113) for the native data plane.
//
// grab's Go transport spoke HTTP/2 to any https origin that offered it
// (reference internal/downloader/http/http.go:18-22).  The worker's HTTP/2
// path (tritondl/fetch/h2.py) keeps the protocol logic in Python: requests,
// HPACK, SETTINGS, GOAWAY, RST_STREAM.  The bytes move here, on one thread
// per connection that owns the TLS session (OpenSSL objects are not safe to
// read and write from two threads):
//
//  * DATA payloads of a stream with a file sink are pwrite()n at the
//    stream's file offset and published on the download's Flow, like
//    recv_body does for an HTTP/1.1 body, so the S3 upload follows them;
//  * window credit is returned from here: a stream's once a quarter of its
//    window is written (never past the bytes its sink will take, so a probe
//    stream that becomes segment 0 does not fetch segment 1's bytes), the
//    connection's once a quarter of its window has arrived;
//  * every other frame goes to Python as an event (an eventfd the event loop
//    watches), and Python's frames (HEADERS, SETTINGS ACK, RST_STREAM, ...)
//    come back through send() to be written in order.
//
// A stream's DATA is buffered here until Python attaches a sink: a file
// (sink_file) or events (sink_events, for small bodies read in Python).
// drop() stops a stream's writes before it returns, so Python may close the
// file right after it.
#pragma once

#include <poll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <atomic>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "relay_core.h"

namespace tritondl_relay {

struct H2Event {
  int type = 0;     // frame type (0..255), or H2Session::kSinkDone / kSinkError / kConnError
  int flags = 0;    // frame flags; kSinkDone: 1 = END_STREAM seen, 0 = the sink's limit was reached
  uint32_t sid = 0;
  std::string payload;  // frame payload, or the error text
  uint64_t n = 0;       // kSinkDone / kSinkError: bytes the sink wrote
};

class H2Session {
 public:
  static constexpr int kSinkDone = 0x100, kSinkError = 0x101, kConnError = 0x102;
  static constexpr uint8_t DATA = 0, HEADERS = 1, RST_STREAM = 3, WINDOW_UPDATE = 8;
  static constexpr uint8_t F_END_STREAM = 0x1, F_PADDED = 0x8;

  H2Session(std::shared_ptr<Stream> io, uint32_t stream_window, uint64_t conn_window, uint32_t max_frame)
      : io_(std::move(io)), stream_window_(stream_window), conn_window_(conn_window), max_frame_(max_frame) {
    efd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    wake_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (efd_ < 0 || wake_ < 0) throw std::runtime_error(errno_str("eventfd"));
  }
  ~H2Session() {
    close();
    ::close(efd_);
    ::close(wake_);
  }
  H2Session(const H2Session&) = delete;
  H2Session& operator=(const H2Session&) = delete;

  int notify_fd() const { return efd_; }
  bool running() const { return th_.joinable() && !dead_.load(); }
  uint64_t bytes_in() const { return bytes_in_.load(); }
  uint64_t bytes_written() const { return bytes_written_.load(); }

  void start() {
    if (!th_.joinable()) th_ = std::thread([this] { run(); });
  }

  // Frames to write, in order (the caller builds them).
  void send(const std::string& frames) {
    {
      std::lock_guard<std::mutex> l(mu_);
      out_q_ += frames;
    }
    poke(wake_);
  }

  // Register a stream before its HEADERS go out: its DATA is buffered until a sink is attached.
  void open_stream(uint32_t sid) {
    std::lock_guard<std::mutex> l(io_mu_);
    St& s = streams_[sid];
    s.window = stream_window_;
  }

  // Write the stream's body at `pos` onward (at most `limit` bytes, < 0 = all),
  // publishing done0 + written on flow segment `seg`.  Buffered bytes go out now.
  void sink_file(uint32_t sid, int fd, uint64_t pos, int64_t limit, std::shared_ptr<Flow> flow, size_t seg,
                 uint64_t done0) {
    std::lock_guard<std::mutex> l(io_mu_);
    auto it = streams_.find(sid);
    if (it == streams_.end()) {
      push_event(H2Event{kSinkError, 0, sid, "stream is closed", 0});
      return;
    }
    St& s = it->second;
    s.mode = kFile;
    s.fd = fd;
    s.pos = pos;
    s.limit = limit;
    s.flow = std::move(flow);
    s.seg = seg;
    s.done0 = done0;
    std::deque<std::string> pend;
    pend.swap(s.pend);
    s.pend_bytes = 0;
    for (const std::string& b : pend) {
      if (!write_file(sid, s, b.data(), b.size())) return;
      if (s.limit >= 0 && s.written >= uint64_t(s.limit)) break;
    }
    if (!flush_file(sid, s)) return;
    if (s.limit >= 0 && s.written >= uint64_t(s.limit)) {
      finish_sink(sid, s, s.ended ? 1 : 0);
    } else if (s.ended) {
      finish_sink(sid, s, 1);
    } else {
      credit_stream(sid, s);
    }
    flush_credit();
  }

  // Deliver the stream's body as DATA events (payload = body bytes; flags carry END_STREAM).
  void sink_events(uint32_t sid) {
    std::lock_guard<std::mutex> l(io_mu_);
    auto it = streams_.find(sid);
    if (it == streams_.end()) return;
    St& s = it->second;
    s.mode = kEvents;
    std::deque<std::string> pend;
    pend.swap(s.pend);
    s.pend_bytes = 0;
    for (size_t i = 0; i < pend.size(); ++i) {
      const bool last = i + 1 == pend.size() && s.ended;
      s.unacked += pend[i].size();
      push_event(H2Event{DATA, last ? F_END_STREAM : 0, sid, std::move(pend[i]), 0});
    }
    if (pend.empty() && s.ended) push_event(H2Event{DATA, F_END_STREAM, sid, std::string(), 0});
    if (s.ended) {
      streams_.erase(it);
    } else {
      credit_stream(sid, s);
    }
    flush_credit();
  }

  // Stop the stream: no write into its sink happens after this returns.
  void drop(uint32_t sid) {
    std::lock_guard<std::mutex> l(io_mu_);
    streams_.erase(sid);
  }

  // Bytes the stream's file sink has written so far (0 once the stream is gone).
  uint64_t written(uint32_t sid) {
    std::lock_guard<std::mutex> l(io_mu_);
    auto it = streams_.find(sid);
    return it == streams_.end() ? 0 : it->second.flushed;
  }

  std::vector<H2Event> take_events() {
    uint64_t v;
    while (::read(efd_, &v, sizeof v) > 0) {
    }
    std::lock_guard<std::mutex> l(mu_);
    std::vector<H2Event> out(std::make_move_iterator(events_.begin()), std::make_move_iterator(events_.end()));
    events_.clear();
    return out;
  }

  // Stop the pump (it writes out what Python queued first, within ~0.2 s) and join it.
  void close() {
    stop_.store(true);
    poke(wake_);
    if (th_.joinable()) th_.join();
  }

 private:
  enum Mode { kBuffer = 0, kFile = 1, kEvents = 2 };
  struct St {
    int mode = kBuffer;
    int fd = -1;
    uint64_t pos = 0;
    int64_t limit = -1;
    std::shared_ptr<Flow> flow;
    size_t seg = 0;
    uint64_t done0 = 0;
    uint64_t written = 0;  // body bytes the sink took (on disk or in wbuf)
    uint64_t flushed = 0;  // ... of which on disk
    std::string wbuf;      // taken, not yet written: small DATA frames become one pwrite
    std::deque<std::string> pend;  // body bytes received before a sink was attached
    uint64_t pend_bytes = 0;
    int64_t window = 0;    // what the server may still send on this stream
    uint64_t unacked = 0;  // consumed (written / delivered / padding) but not yet credited
    bool ended = false;    // END_STREAM seen
  };

  static void poke(int fd) {
    const uint64_t one = 1;
    ssize_t r = ::write(fd, &one, sizeof one);
    (void)r;
  }

  void push_event(H2Event e) {
    bool was_empty;
    {
      std::lock_guard<std::mutex> l(mu_);
      was_empty = events_.empty();
      events_.push_back(std::move(e));
    }
    if (was_empty) poke(efd_);
  }

  static void put_frame_head(std::string& out, uint32_t len, uint8_t type, uint8_t flags, uint32_t sid) {
    const char h[9] = {char(len >> 16), char(len >> 8), char(len), char(type), char(flags),
                       char((sid >> 24) & 0x7f), char(sid >> 16), char(sid >> 8), char(sid)};
    out.append(h, 9);
  }
  void queue_window_update(uint32_t sid, uint32_t inc) {
    put_frame_head(credit_, 4, WINDOW_UPDATE, 0, sid);
    const char p[4] = {char((inc >> 24) & 0x7f), char(inc >> 16), char(inc >> 8), char(inc)};
    credit_.append(p, 4);
  }
  // Credit frames built under io_mu_ go to the out queue in one piece.
  void flush_credit() {
    if (credit_.empty()) return;
    {
      std::lock_guard<std::mutex> l(mu_);
      out_q_ += credit_;
    }
    credit_.clear();
    if (std::this_thread::get_id() != th_.get_id()) poke(wake_);
  }

  // Return a stream's window credit once a quarter of the window is consumed
  // or the window runs low, never past the bytes its sink will still take.
  void credit_stream(uint32_t sid, St& s) {
    if (s.ended || s.unacked == 0) return;
    uint64_t inc = s.unacked;
    if (s.mode == kFile && s.limit >= 0) {
      const int64_t need = s.limit - int64_t(s.written);
      inc = std::min<uint64_t>(inc, uint64_t(std::max<int64_t>(0, need - s.window)));
    }
    inc = std::min<uint64_t>(inc, 0x7fffffffu);
    if (inc && (inc >= stream_window_ / 4 || s.window < int64_t(stream_window_ / 4))) {
      queue_window_update(sid, uint32_t(inc));
      s.unacked -= inc;
      s.window += int64_t(inc);
    }
  }

  void finish_sink(uint32_t sid, St& s, int eof) {
    if (!flush_file(sid, s)) return;
    push_event(H2Event{kSinkDone, eof, sid, std::string(), s.flushed});
    streams_.erase(sid);
  }

  // Take body bytes into the stream's file sink (io_mu_ held): buffered, and
  // written once kFlush bytes are waiting (or at the end of a receive batch),
  // so 16 KiB frames do not cost a pwrite each.  false: a write failed, the
  // stream is gone (`s` dangles) and Python has the error.
  static constexpr size_t kFlush = 256u << 10;
  bool write_file(uint32_t sid, St& s, const char* p, size_t n) {
    size_t take = n;
    if (s.limit >= 0) take = size_t(std::min<uint64_t>(n, uint64_t(s.limit) - s.written));
    if (take >= kFlush && s.wbuf.empty()) {  // a big frame goes straight from the record buffer
      std::string err;
      if (!pwrite_full(s.fd, p, take, s.pos + s.flushed, &err)) {
        push_event(H2Event{kSinkError, 0, sid, err, s.flushed});
        streams_.erase(sid);
        return false;
      }
      s.written += take;
      s.flushed += take;
      s.unacked += take;
      bytes_written_.fetch_add(take, std::memory_order_relaxed);
      if (s.flow) s.flow->advance(s.seg, s.done0 + s.flushed);
    } else if (take) {
      s.wbuf.append(p, take);
      s.written += take;
      if (s.wbuf.size() >= kFlush) return flush_file(sid, s);
    }
    return true;
  }
  bool flush_file(uint32_t sid, St& s) {
    if (s.wbuf.empty()) return true;
    std::string err;
    if (!pwrite_full(s.fd, s.wbuf.data(), s.wbuf.size(), s.pos + s.flushed, &err)) {
      push_event(H2Event{kSinkError, 0, sid, err, s.flushed});
      streams_.erase(sid);
      return false;
    }
    s.flushed += s.wbuf.size();
    bytes_written_.fetch_add(s.wbuf.size(), std::memory_order_relaxed);
    s.unacked += s.wbuf.size();
    s.wbuf.clear();
    if (s.flow) s.flow->advance(s.seg, s.done0 + s.flushed);
    return true;
  }
  // End of a receive batch: what the file sinks took goes to disk (and its credit out).
  void flush_all() {
    std::lock_guard<std::mutex> l(io_mu_);
    std::vector<uint32_t> sids;
    for (auto& kv : streams_)
      if (kv.second.mode == kFile && !kv.second.wbuf.empty()) sids.push_back(kv.first);
    for (uint32_t sid : sids) {
      auto it = streams_.find(sid);
      if (it != streams_.end() && flush_file(sid, it->second)) credit_stream(sid, it->second);
    }
    flush_credit();
  }

  void on_data(uint8_t flags, uint32_t sid, const char* p, size_t len) {
    size_t pad = 0, off = 0;
    if (flags & F_PADDED) {
      if (len < 1 || size_t(uint8_t(p[0])) >= len) throw std::runtime_error("DATA padding longer than the frame");
      pad = uint8_t(p[0]);
      off = 1;
    }
    const char* body = p + off;
    const size_t blen = len - off - pad;
    std::lock_guard<std::mutex> l(io_mu_);
    conn_unacked_ += len;  // the connection's credit covers every flow-controlled byte
    if (conn_unacked_ >= conn_window_ / 4) {
      queue_window_update(0, uint32_t(std::min<uint64_t>(conn_unacked_, 0x7fffffffu)));
      conn_unacked_ = 0;
    }
    auto it = streams_.find(sid);
    if (it != streams_.end()) {
      St& s = it->second;
      s.window -= int64_t(len);
      s.unacked += len - blen;  // padding counts against the window too
      const bool end = flags & F_END_STREAM;
      switch (s.mode) {
        case kBuffer:
          if (blen) {
            s.pend.emplace_back(body, blen);
            s.pend_bytes += blen;
          }
          s.ended = s.ended || end;
          break;
        case kEvents:
          s.unacked += blen;
          push_event(H2Event{DATA, end ? F_END_STREAM : 0, sid, std::string(body, blen), 0});
          s.ended = s.ended || end;
          if (end) {
            streams_.erase(it);
            flush_credit();
            return;
          }
          break;
        case kFile:
          if (!write_file(sid, s, body, blen)) {  // the write failed: the stream is gone
            flush_credit();
            return;
          }
          s.ended = s.ended || end;
          if (s.limit >= 0 && s.written >= uint64_t(s.limit)) {
            finish_sink(sid, s, end ? 1 : 0);
            flush_credit();
            return;
          }
          if (end) {
            finish_sink(sid, s, 1);
            flush_credit();
            return;
          }
          break;
        default:
          break;
      }
      auto jt = streams_.find(sid);
      if (jt != streams_.end()) credit_stream(sid, jt->second);
    }
    flush_credit();
  }

  void on_frame(uint8_t type, uint8_t flags, uint32_t sid, const char* p, size_t len) {
    if (type == DATA) {
      on_data(flags, sid, p, len);
      return;
    }
    if (type == RST_STREAM) {
      std::lock_guard<std::mutex> l(io_mu_);
      auto it = streams_.find(sid);  // writes stop now; Python fails the stream from the event
      if (it != streams_.end()) {
        if (it->second.mode == kFile && flush_file(sid, it->second))
          push_event(H2Event{kSinkError, 0, sid, "reset by the server", it->second.flushed});
        streams_.erase(sid);
      }
    } else if (type == HEADERS && (flags & F_END_STREAM)) {
      // trailers (or a bodiless response) end the stream: a sink ends with what it wrote
      std::lock_guard<std::mutex> l(io_mu_);
      auto it = streams_.find(sid);
      if (it != streams_.end()) {
        it->second.ended = true;
        if (it->second.mode == kFile) {
          finish_sink(sid, it->second, 1);
        } else if (it->second.mode == kEvents) {
          push_event(H2Event{DATA, F_END_STREAM, sid, std::string(), 0});
          streams_.erase(it);
        }
      }
    }
    push_event(H2Event{type, flags, sid, std::string(p, len), 0});
  }

  // Frames in rbuf_[0, rlen_): handle every complete one, keep the rest.
  void parse() {
    size_t p = 0;
    while (rlen_ - p >= 9) {
      const unsigned char* h = reinterpret_cast<const unsigned char*>(rbuf_.data() + p);
      const uint32_t len = (uint32_t(h[0]) << 16) | (uint32_t(h[1]) << 8) | h[2];
      if (len > max_frame_)
        throw std::runtime_error("frame of " + std::to_string(len) + " bytes above the " +
                                 std::to_string(max_frame_) + " allowed");
      if (rlen_ - p < 9 + size_t(len)) break;
      const uint32_t sid = ((uint32_t(h[5]) << 24) | (uint32_t(h[6]) << 16) | (uint32_t(h[7]) << 8) | h[8]) &
                           0x7fffffffu;
      on_frame(h[3], h[4], sid, rbuf_.data() + p + 9, len);
      p += 9 + size_t(len);
    }
    if (p) {
      std::memmove(rbuf_.data(), rbuf_.data() + p, rlen_ - p);
      rlen_ -= p;
    }
  }

  void fail_all(const std::string& why) {
    {
      std::lock_guard<std::mutex> l(io_mu_);
      std::vector<uint32_t> sids;
      for (auto& kv : streams_)
        if (kv.second.mode == kFile) sids.push_back(kv.first);
      for (uint32_t sid : sids) {
        auto it = streams_.find(sid);
        if (it != streams_.end() && flush_file(sid, it->second))
          push_event(H2Event{kSinkError, 0, sid, why, it->second.flushed});
      }
      streams_.clear();
    }
    push_event(H2Event{kConnError, 0, 0, why, 0});
  }

  void run() {
    rbuf_.resize(size_t(max_frame_) + 9 + (256u << 10));
    std::string out;
    size_t out_off = 0;
    std::string why;
    try {
      for (;;) {
        {
          std::lock_guard<std::mutex> l(mu_);
          if (!out_q_.empty()) {
            if (out_off == out.size()) {
              out.clear();
              out_off = 0;
            }
            out += out_q_;
            out_q_.clear();
          }
        }
        short want_out = 0;
        while (out_off < out.size()) {  // write what Python and the credit logic queued
          struct iovec iov{&out[out_off], out.size() - out_off};
          short w = POLLOUT;
          std::string err;
          const ssize_t n = io_->send_nb(&iov, 1, &w, &err);
          if (n == IO_ERR) throw std::runtime_error(err);
          if (n == IO_AGAIN) {
            want_out = w;
            break;
          }
          out_off += size_t(n);
        }
        if (out_off == out.size() && !want_out) {
          short w = POLLOUT;
          std::string err;
          if (!io_->flush_nb(&w, &err)) {
            if (!err.empty()) throw std::runtime_error(err);
            want_out = w;
          }
        }
        if (stop_.load() && out_off == out.size() && !want_out) break;
        short want_in = POLLIN;
        for (;;) {  // read whatever is ready (TLS may hold decrypted records)
          if (rlen_ == rbuf_.size()) rbuf_.resize(rbuf_.size() * 2);
          std::string err;
          short w = POLLIN;
          const ssize_t n = io_->recv_nb(rbuf_.data() + rlen_, rbuf_.size() - rlen_, &w, &err);
          if (n > 0) {
            rlen_ += size_t(n);
            bytes_in_.fetch_add(uint64_t(n), std::memory_order_relaxed);
            parse();
            continue;
          }
          flush_all();  // nothing more to read right now: the sinks' buffers go to disk
          if (n == 0) throw std::runtime_error("connection closed by the server");
          if (n == IO_ERR) throw std::runtime_error(err);
          want_in = w;
          break;
        }
        {
          std::lock_guard<std::mutex> l(mu_);  // credit queued while parsing goes out before we sleep
          if (!out_q_.empty()) continue;
        }
        struct pollfd pf[2] {};
        pf[0].fd = io_->fd();
        pf[0].events = short(want_in | want_out);
        pf[1].fd = wake_;
        pf[1].events = POLLIN;
        const int r = ::poll(pf, 2, stop_.load() ? 20 : 200);
        if (r < 0 && errno != EINTR) throw std::runtime_error(errno_str("poll"));
        if (pf[1].revents & POLLIN) {
          uint64_t v;
          while (::read(wake_, &v, sizeof v) > 0) {
          }
        }
        if (stop_.load() && r == 0) break;  // nothing left to write that the peer will take
        if (pf[0].revents & (POLLERR | POLLNVAL)) throw std::runtime_error("socket error");
      }
      why = "session closed";
    } catch (const std::exception& e) {
      why = e.what();
    }
    dead_.store(true);
    fail_all(why);
  }

  std::shared_ptr<Stream> io_;
  const uint32_t stream_window_;
  const uint64_t conn_window_;
  const uint32_t max_frame_;
  int efd_ = -1, wake_ = -1;
  std::thread th_;
  std::atomic<bool> stop_{false}, dead_{false};
  std::atomic<uint64_t> bytes_in_{0}, bytes_written_{0};

  std::mutex mu_;                     // events_, out_q_
  std::deque<H2Event> events_;
  std::string out_q_;

  std::mutex io_mu_;                  // streams_ and every write into a sink
  std::unordered_map<uint32_t, St> streams_;
  std::string credit_;                // WINDOW_UPDATE frames not yet queued (io_mu_)
  uint64_t conn_unacked_ = 0;         // io_mu_

  std::vector<char> rbuf_;            // pump thread only
  size_t rlen_ = 0;
};

}  // namespace tritondl_relay
