// BitTorrent peer-wire data plane core (no Python): see btwire.cpp for the
// bindings and the design notes.  Header-only so the native self-test
// (csrc/tests/native_selftest.cpp) runs it under ASan/UBSan/TSan — it parses
// bytes straight off untrusted peer connections.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include <cerrno>
#include <unistd.h>

namespace tritondl_btwire {


constexpr uint32_t kBlock = 16384;
constexpr uint8_t kChoke = 0, kUnchoke = 1, kPiece = 7, kRequest = 6, kCancel = 8, kReject = 16;
constexpr uint32_t kMaxMsg = 2 * 1024 * 1024 + 13;
constexpr uint32_t kMaxRequest = 128 * 1024;  // larger REQUESTs are refused (as libtorrent does)

using Clock = std::chrono::steady_clock;

// What Link::feed reports back (see Link::feed).
struct Event {
  enum Kind : uint8_t { kPieceDone, kMsg, kChoked, kUnchoked, kBad } kind;
  uint32_t piece = 0;   // kPieceDone
  uint8_t id = 0;       // kMsg: message id
  std::string data;     // kMsg: payload; kBad: reason
  static Event bad(const char* why) { return Event{kBad, 0, 0, why}; }
};

inline uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline void put_be32(std::string& s, uint32_t v) {
  const char b[4] = {char(v >> 24), char(v >> 16), char(v >> 8), char(v)};
  s.append(b, 4);
}
inline uint64_t key(uint32_t piece, uint32_t block) { return (uint64_t(piece) << 32) | block; }

// Recycled piece buffers: a 1 MiB bytes object per piece would be a fresh
// mmap (256 page faults) plus a copy; a completed piece instead moves its
// buffer into a Piece (buffer protocol, no copy) that hands it back here
// when Python drops the last reference (after verify + write).
struct Pool {
  std::mutex mu;
  std::vector<std::vector<uint8_t>> free;
  size_t cached = 0;                       // bytes held in `free`
  size_t cap_bytes = size_t(256) << 20;    // 16 x 16 MiB pieces, 256 x 1 MiB
  std::vector<uint8_t> get(size_t n) {
    std::vector<uint8_t> v;
    {
      std::lock_guard<std::mutex> g(mu);
      if (!free.empty()) {
        v = std::move(free.back());
        free.pop_back();
        cached -= v.capacity();
      }
    }
    v.resize(n);  // zero-fills only growth; a recycled buffer keeps its bytes
    return v;
  }
  void put(std::vector<uint8_t>&& v) {
    std::lock_guard<std::mutex> g(mu);
    if (cached + v.capacity() <= cap_bytes) {
      cached += v.capacity();
      free.push_back(std::move(v));
    }
  }
};

// A completed piece handed to Python: read-only bytes-like (memoryview(),
// hashlib, os.pwrite accept it), buffer returned to the pool on release.
class Piece {
 public:
  Piece(std::vector<uint8_t>&& d, std::shared_ptr<Pool> pool) : data_(std::move(d)), pool_(std::move(pool)) {}
  ~Piece() {
    if (pool_) pool_->put(std::move(data_));
  }
  Piece(const Piece&) = delete;
  Piece& operator=(const Piece&) = delete;
  const std::vector<uint8_t>& data() const { return data_; }

 private:
  std::vector<uint8_t> data_;
  std::shared_ptr<Pool> pool_;
};

struct PieceBuf {
  std::vector<uint8_t> data;
  std::vector<uint8_t> got;
  std::vector<uint32_t> from;  // per block: id of the link that supplied it (blame on a hash failure)
  uint32_t nblocks = 0, ngot = 0;
  uint64_t nbytes = 0;
};

class PieceStore {
 public:
  PieceStore(uint32_t num_pieces, uint64_t piece_len, uint64_t total_len)
      : n_(num_pieces), plen_(piece_len), total_(total_len) {
    if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
    if (num_pieces == 0 ? total_len != 0
                        : (total_len > uint64_t(num_pieces) * piece_len || total_len <= uint64_t(num_pieces - 1) * piece_len))
      throw std::invalid_argument("total_len does not match num_pieces x piece_len");
  }

  uint64_t piece_size(uint32_t i) const {
    if (i >= n_) throw std::out_of_range("piece index");
    return i + 1 == n_ ? total_ - uint64_t(i) * plen_ : plen_;
  }
  uint32_t blocks(uint32_t i) const { return uint32_t((piece_size(i) + kBlock - 1) / kBlock); }

  // Start buffering piece i (no-op if it already is).  Returns true if new.
  bool begin(uint32_t i) {
    if (pieces_.count(i)) return false;
    PieceBuf& b = pieces_[i];
    b.data = pool_->get(piece_size(i));
    b.nblocks = blocks(i);
    b.got.assign(b.nblocks, 0);
    b.from.assign(b.nblocks, 0);
    return true;
  }
  bool active(uint32_t i) const { return pieces_.count(i) != 0; }
  bool has_block(uint32_t i, uint32_t b) const {
    auto it = pieces_.find(i);
    return it != pieces_.end() && b < it->second.nblocks && it->second.got[b];
  }
  uint32_t received(uint32_t i) const {
    auto it = pieces_.find(i);
    return it == pieces_.end() ? 0 : it->second.ngot;
  }
  // Copy one block in, supplied by link `who`.  Returns 1 if it completed the
  // piece, 0 if stored / duplicate / not wanted, -1 on bad geometry.
  int put(uint32_t i, uint32_t off, const uint8_t* p, size_t n, uint32_t who = 0) {
    auto it = pieces_.find(i);
    if (it == pieces_.end()) return 0;
    PieceBuf& b = it->second;
    if (off % kBlock) return -1;
    const uint32_t bi = off / kBlock;
    if (bi >= b.nblocks) return -1;
    const uint64_t want = std::min<uint64_t>(kBlock, b.data.size() - off);
    if (n != want) return -1;
    if (b.got[bi]) return 0;
    std::memcpy(b.data.data() + off, p, n);
    b.got[bi] = 1;
    b.from[bi] = who;
    b.nbytes += n;
    bytes_ += n;
    return ++b.ngot == b.nblocks ? 1 : 0;
  }
  // Per block of a buffered piece: the id of the link that supplied it (0 =
  // not received).  Call before take(): blame / smart ban on a hash failure.
  std::vector<uint32_t> block_sources(uint32_t i) const {
    auto it = pieces_.find(i);
    if (it == pieces_.end()) return {};
    const PieceBuf& b = it->second;
    std::vector<uint32_t> v(b.nblocks, 0);
    for (uint32_t k = 0; k < b.nblocks; ++k)
      if (b.got[k]) v[k] = b.from[k];
    return v;
  }
  std::unique_ptr<Piece> take(uint32_t i) {
    auto it = pieces_.find(i);
    if (it == pieces_.end()) throw std::out_of_range("piece not buffered");
    auto out = std::make_unique<Piece>(std::move(it->second.data), pool_);
    bytes_ -= it->second.nbytes;
    pieces_.erase(it);
    return out;
  }
  void reset(uint32_t i) {
    auto it = pieces_.find(i);
    if (it == pieces_.end()) return;
    bytes_ -= it->second.nbytes;
    pool_->put(std::move(it->second.data));
    pieces_.erase(it);
  }
  size_t pooled() {
    std::lock_guard<std::mutex> g(pool_->mu);
    return pool_->free.size();
  }
  std::vector<uint32_t> active_pieces() const {
    std::vector<uint32_t> v;
    v.reserve(pieces_.size());
    for (auto& kv : pieces_) v.push_back(kv.first);
    std::sort(v.begin(), v.end());
    return v;
  }
  uint64_t partial_bytes() const { return bytes_; }   // bytes of not-yet-complete buffered pieces
  uint32_t num_pieces() const { return n_; }

 private:
  uint32_t n_;
  uint64_t plen_, total_;
  uint64_t bytes_ = 0;
  std::unordered_map<uint32_t, PieceBuf> pieces_;
  std::shared_ptr<Pool> pool_ = std::make_shared<Pool>();
};

// Read side of a torrent's files, for answering REQUESTs without Python.
// Holds its own dup()s of the storage fds (closing the storage cannot make a
// link read a reused descriptor); close() ends serving before the job's
// files go away.  BEP 47 padding files (fd -1) read as zeros.
class Source {
 public:
  Source(uint32_t num_pieces, uint64_t piece_len, uint64_t total_len)
      : n_(num_pieces), plen_(piece_len), total_(total_len), have_(num_pieces, 0) {
    if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  }
  ~Source() { close(); }
  Source(const Source&) = delete;
  Source& operator=(const Source&) = delete;

  // Files in stream order: [start, start + len) of the torrent's byte stream.
  void add_file(int fd, uint64_t start, uint64_t len) {
    if (!spans_.empty() && start < spans_.back().start) throw std::invalid_argument("files out of order");
    const int own = fd >= 0 ? ::dup(fd) : -1;
    if (fd >= 0 && own < 0) throw std::runtime_error("dup failed");
    spans_.push_back({own, start, len});
  }
  void close() {
    for (auto& s : spans_)
      if (s.fd >= 0) ::close(s.fd);
    spans_.clear();
    closed_ = true;
  }
  void set_have(uint32_t i) {
    if (i < n_) have_[i] = 1;
  }
  void set_have_bits(const uint8_t* bits, size_t n) {
    for (size_t i = 0; i < n && i < n_; ++i) have_[i] = bits[i] ? 1 : 0;
  }
  bool has(uint32_t i) const { return !closed_ && i < n_ && have_[i]; }
  uint32_t num_pieces() const { return n_; }
  uint64_t piece_size(uint32_t i) const { return i + 1 == n_ ? total_ - uint64_t(i) * plen_ : plen_; }
  uint64_t piece_len() const { return plen_; }

  // Copy stream bytes [gofs, gofs + n) into dst; false on a short read.
  bool read(uint64_t gofs, char* dst, size_t n) const {
    if (closed_) return false;
    const uint64_t end = gofs + n;
    auto it = std::upper_bound(spans_.begin(), spans_.end(), gofs,
                               [](uint64_t g, const Span& s) { return g < s.start; });
    if (it != spans_.begin()) --it;
    uint64_t pos = gofs;
    for (; it != spans_.end() && pos < end; ++it) {
      const uint64_t fe = it->start + it->len;
      if (it->len == 0 || fe <= pos) continue;
      if (it->start > pos) return false;  // hole in the layout
      const uint64_t b = std::min(end, fe);
      char* d = dst + (pos - gofs);
      const size_t m = size_t(b - pos);
      if (it->fd < 0) {
        std::memset(d, 0, m);
      } else {
        size_t got = 0;
        while (got < m) {
          const ssize_t r = ::pread(it->fd, d + got, m - got, off_t(pos - it->start + got));
          if (r < 0 && errno == EINTR) continue;
          if (r <= 0) return false;
          got += size_t(r);
        }
      }
      pos = b;
    }
    return pos == end;
  }

 private:
  struct Span {
    int fd;
    uint64_t start, len;
  };
  uint32_t n_;
  uint64_t plen_, total_;
  std::vector<uint8_t> have_;
  std::vector<Span> spans_;
  bool closed_ = false;
};

class Link {
 public:
  Link(std::shared_ptr<PieceStore> store, int pipeline, bool fast, uint32_t id = 0)
      : store_(std::move(store)), pipeline_(std::max(1, pipeline)), refill_(std::max(1, pipeline_ / 4)), fast_(fast),
        id_(id) {}
  uint32_t id() const { return id_; }

  // Parse `n` more bytes of the stream.  Appends to *ev: kPieceDone when a
  // block from this link completed a piece; kMsg (id, payload) for every
  // non-data message; kChoked / kUnchoked after handling them here; kBad
  // (reason) on a protocol violation (the caller drops the peer).  *out gets
  // the requests/cancels to send now.
  void feed(const uint8_t* p, size_t n, std::vector<Event>* ev, std::string* out) {
    reserve(n);
    if (n) std::memcpy(buf_.data() + wpos_, p, n);
    wpos_ += n;
    parse(ev, out);
  }

  // Zero-copy receive: the socket reads straight into the returned span of
  // the link's buffer, then feed_n(nbytes) parses what arrived.  The span
  // stays valid until the next feed / feed_n / recv_buffer call.
  std::pair<uint8_t*, size_t> recv_buffer(size_t want) {
    reserve(std::max<size_t>(want, 4096));
    return {buf_.data() + wpos_, buf_.size() - wpos_};
  }
  void feed_n(size_t n, std::vector<Event>* ev, std::string* out) {
    if (n > buf_.size() - wpos_) throw std::out_of_range("feed_n past the receive buffer");
    wpos_ += n;
    parse(ev, out);
  }

 private:
  // Room for n more bytes after wpos_: drop consumed bytes first (the kept
  // tail is less than one message), grow only if still short.
  void reserve(size_t n) {
    if (rpos_) {
      if (wpos_ > rpos_) std::memmove(buf_.data(), buf_.data() + rpos_, wpos_ - rpos_);
      wpos_ -= rpos_;
      rpos_ = 0;
    }
    if (buf_.size() - wpos_ < n) buf_.resize(wpos_ + n);
  }

  void parse(std::vector<Event>* ev, std::string* out) {
    size_t pos = rpos_;
    const size_t len = wpos_;
    bool bad = false;
    stalled_ = false;
    while (len - pos >= 4) {
      if (source_ && out->size() >= serve_budget_) {
        // enough PIECE replies for one write: leave the rest parsed later
        // (feed_n(0) once the socket drains), so a peer that pipelines
        // thousands of REQUESTs cannot make one read queue unbounded output
        stalled_ = true;
        break;
      }
      const uint32_t ml = be32(&buf_[pos]);
      if (ml > kMaxMsg) {
        ev->push_back(Event::bad("message too large"));
        bad = true;
        break;
      }
      if (len - pos < 4 + size_t(ml)) break;
      const uint8_t* m = &buf_[pos + 4];
      pos += 4 + ml;
      if (ml == 0) continue;  // keep-alive
      const uint8_t id = m[0];
      const uint8_t* pl = m + 1;
      const size_t pn = ml - 1;
      if (id == kPiece) {
        if (pn < 8) {
          ev->push_back(Event::bad("short piece message"));
          bad = true;
          break;
        }
        const uint32_t i = be32(pl), off = be32(pl + 4);
        if (i >= store_->num_pieces()) {
          ev->push_back(Event::bad("piece index out of range"));
          bad = true;
          break;
        }
        if (off % kBlock) {
          ev->push_back(Event::bad("bad block geometry"));
          bad = true;
          break;
        }
        const uint64_t k = key(i, off / kBlock);
        if (!out_req_.erase(k) && !recent_.erase(k)) {
          // never asked of this link (nor recently withdrawn from it): a peer
          // pushing blocks could poison pieces other links are filling, and
          // the hash failure would be blamed on whoever completed the piece
          wasted_ += pn - 8;
          continue;
        }
        const int r = store_->put(i, off, pl + 8, pn - 8, id_);
        if (r < 0) {
          ev->push_back(Event::bad("bad block geometry"));
          bad = true;
          break;
        }
        downloaded_ += pn - 8;
        if (r == 1) ev->push_back(Event{Event::kPieceDone, i, 0, {}});
      } else if (id == kChoke) {
        peer_choking_ = true;
        if (!fast_) lapse_all();  // BEP 3: a choke drops every pending request
        ev->push_back(Event{Event::kChoked, 0, 0, {}});
      } else if (id == kUnchoke) {
        peer_choking_ = false;
        ev->push_back(Event{Event::kUnchoked, 0, 0, {}});
      } else if (id == kReject && pn >= 12) {
        const uint32_t i = be32(pl), off = be32(pl + 4);
        if (out_req_.erase(key(i, off / kBlock))) redo_.push_back(key(i, off / kBlock));
        recent_.erase(key(i, off / kBlock));
      } else if (id == kRequest && source_ && pn >= 12) {
        serve(be32(pl), be32(pl + 4), be32(pl + 8), out);
      } else if (id == kCancel && source_ && pn >= 12) {
        // every REQUEST was answered in the read that carried it: nothing to withdraw
      } else {
        ev->push_back(Event{Event::kMsg, 0, id, std::string(reinterpret_cast<const char*>(pl), pn)});
      }
    }
    rpos_ = pos;
    if (rpos_ == wpos_) rpos_ = wpos_ = 0;
    if (!bad) requests(out);
  }

 public:

  // Requests (and queued cancels) to send now.
  std::string pump() {
    std::string out;
    requests(&out);
    return out;
  }

  void assign(uint32_t i) {
    if (i >= store_->num_pieces()) throw std::out_of_range("piece index");
    store_->begin(i);
    if (std::find(assigned_.begin(), assigned_.end(), i) == assigned_.end()) {
      assigned_.push_back(i);
      cursor_[i] = 0;
    }
  }
  // Another link (or a web seed) completed piece i: forget it, cancel what we asked for.
  void piece_done(uint32_t i) {
    unassign(i, true);
  }
  // Drop piece i without cancelling (e.g. failed verification: Python re-plans it).
  void drop(uint32_t i) { unassign(i, false); }

  // Room for more work: fewer unrequested-but-assigned blocks than the pipeline.
  bool need_work() const {
    size_t pending = redo_.size();
    for (uint32_t i : assigned_) {
      auto it = cursor_.find(i);
      if (it != cursor_.end()) pending += store_->blocks(i) - std::min(store_->blocks(i), it->second);
      if (pending >= size_t(pipeline_)) return false;
    }
    return true;
  }
  std::vector<uint32_t> assigned() const { return assigned_; }
  size_t outstanding() const { return out_req_.size(); }
  double oldest_request_age() const {
    if (out_req_.empty()) return 0.0;
    auto oldest = Clock::time_point::max();
    for (auto& kv : out_req_) oldest = std::min(oldest, kv.second);
    return std::chrono::duration<double>(Clock::now() - oldest).count();
  }
  // Everything this link had asked for goes back to the pool (timeout / snub).
  void lapse_all() {
    for (auto& kv : out_req_) {
      redo_.push_back(kv.first);
      withdrew(kv.first);
    }
    out_req_.clear();
  }
  // Bytes of PIECE messages this link never requested (dropped, not stored).
  uint64_t wasted() const { return wasted_; }
  bool peer_choking() const { return peer_choking_; }
  void set_peer_choking(bool c) { peer_choking_ = c; }
  uint64_t downloaded() const { return downloaded_; }
  size_t buffered() const { return wpos_ - rpos_; }

  // Answer the peer's block REQUESTs from `src` (PIECE, or REJECT on a fast
  // connection for what we cannot serve).  Without a source REQUEST and
  // CANCEL reach Python as kMsg events.
  void set_source(std::shared_ptr<Source> src) { source_ = std::move(src); }
  bool serving() const { return serving_; }
  void set_serving(bool s) { serving_ = s; }   // false: we choke this peer
  uint64_t uploaded() const { return uploaded_; }
  // The last feed stopped at the serve budget with messages left unparsed.
  bool stalled() const { return stalled_; }
  uint64_t serve_errors() const { return serve_errors_; }

 private:
  void unassign(uint32_t i, bool cancel) {
    auto it = std::find(assigned_.begin(), assigned_.end(), i);
    if (it != assigned_.end()) assigned_.erase(it);
    cursor_.erase(i);
    for (auto r = out_req_.begin(); r != out_req_.end();) {
      if (uint32_t(r->first >> 32) == i) {
        if (cancel) cancels_.push_back(r->first);
        withdrew(r->first);
        r = out_req_.erase(r);
      } else {
        ++r;
      }
    }
    redo_.erase(std::remove_if(redo_.begin(), redo_.end(), [&](uint64_t k) { return uint32_t(k >> 32) == i; }),
                redo_.end());
  }

  void serve(uint32_t i, uint32_t off, uint32_t n, std::string* out) {
    bool ok = serving_ && source_->has(i) && n > 0 && n <= kMaxRequest &&
              uint64_t(off) + n <= source_->piece_size(i);
    if (ok) {
      const size_t at = out->size();
      out->resize(at + 13 + n);
      char* h = &(*out)[at];
      const uint32_t ml = 9 + n;
      const char hdr[13] = {char(ml >> 24), char(ml >> 16), char(ml >> 8), char(ml), char(kPiece),
                            char(i >> 24),  char(i >> 16),  char(i >> 8),  char(i),  char(off >> 24),
                            char(off >> 16), char(off >> 8), char(off)};
      std::memcpy(h, hdr, 13);
      ok = source_->read(uint64_t(i) * source_->piece_len() + off, h + 13, n);
      if (ok) {
        uploaded_ += n;
      } else {
        out->resize(at);
        ++serve_errors_;
      }
    }
    if (!ok && fast_) msg3(*out, kReject, i, off, n);
  }

  // A request taken back (lapsed, or cancelled because another link finished
  // the piece): the block may still be in flight, so it stays acceptable.
  // Bounded FIFO, so a peer cannot grow it.
  void withdrew(uint64_t k) {
    if (recent_.insert(k).second) recent_fifo_.push_back(k);
    while (recent_fifo_.size() > kRecent) {
      recent_.erase(recent_fifo_.front());
      recent_fifo_.pop_front();
    }
  }

  void msg3(std::string& out, uint8_t id, uint32_t i, uint32_t off, uint32_t n) {
    put_be32(out, 13);
    out.push_back(char(id));
    put_be32(out, i);
    put_be32(out, off);
    put_be32(out, n);
  }

  void requests(std::string* outp) {
    std::string& out = *outp;
    for (uint64_t k : cancels_) {
      const uint32_t i = uint32_t(k >> 32), b = uint32_t(k);
      msg3(out, kCancel, i, b * kBlock, uint32_t(std::min<uint64_t>(kBlock, store_->piece_size(i) - uint64_t(b) * kBlock)));
    }
    cancels_.clear();
    if (peer_choking_) return;
    // refill in batches (a quarter of the pipeline): one small send per ~4
    // received blocks instead of one per socket read; the pipeline stays >= 3/4 full
    if (out_req_.size() + size_t(refill_) > size_t(pipeline_)) return;
    const auto now = Clock::now();
    auto issue = [&](uint32_t i, uint32_t b) {
      out_req_[key(i, b)] = now;
      msg3(out, kRequest, i, b * kBlock, uint32_t(std::min<uint64_t>(kBlock, store_->piece_size(i) - uint64_t(b) * kBlock)));
    };
    while (out_req_.size() < size_t(pipeline_) && !redo_.empty()) {
      const uint64_t k = redo_.front();
      redo_.pop_front();
      const uint32_t i = uint32_t(k >> 32), b = uint32_t(k);
      if (cursor_.count(i) && !store_->has_block(i, b) && !out_req_.count(k)) issue(i, b);
    }
    for (size_t a = 0; a < assigned_.size() && out_req_.size() < size_t(pipeline_); ++a) {
      const uint32_t i = assigned_[a];
      uint32_t& cur = cursor_[i];
      const uint32_t nb = store_->blocks(i);
      while (cur < nb && out_req_.size() < size_t(pipeline_)) {
        const uint32_t b = cur++;
        if (!store_->has_block(i, b) && !out_req_.count(key(i, b))) issue(i, b);
      }
    }
  }

  std::shared_ptr<PieceStore> store_;
  uint32_t id_ = 0;  // stamped on every block this link stores (PieceStore::contributors)
  std::shared_ptr<Source> source_;
  bool serving_ = true;
  bool stalled_ = false;
  size_t serve_budget_ = size_t(2) << 20;  // PIECE reply bytes per feed call
  uint64_t uploaded_ = 0, serve_errors_ = 0;
  int pipeline_;
  int refill_;   // issue new requests only once this many slots are free
  bool fast_;
  bool peer_choking_ = true;
  std::vector<uint8_t> buf_;                              // received bytes [rpos_, wpos_)
  size_t rpos_ = 0, wpos_ = 0;
  std::vector<uint32_t> assigned_;
  std::unordered_map<uint32_t, uint32_t> cursor_;        // next never-requested block per assigned piece
  std::unordered_map<uint64_t, Clock::time_point> out_req_;
  std::deque<uint64_t> redo_;                             // lapsed / rejected blocks to ask for again
  std::vector<uint64_t> cancels_;
  static constexpr size_t kRecent = 2048;
  std::unordered_set<uint64_t> recent_;                   // withdrawn requests still acceptable
  std::deque<uint64_t> recent_fifo_;                      // their order, for the bound
  uint64_t downloaded_ = 0, wasted_ = 0;
};

}  // namespace tritondl_btwire
