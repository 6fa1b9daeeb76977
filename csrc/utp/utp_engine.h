// uTP (BEP 29) protocol engine — header-only core shared by the pybind11
// module (utp.cpp) and the sanitizer self-test (csrc/tests/native_selftest.cpp).
// See utp.cpp for the design notes.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace tritondl_utp {

enum PktType : uint8_t { ST_DATA = 0, ST_FIN = 1, ST_STATE = 2, ST_RESET = 3, ST_SYN = 4 };
enum ConnState : int { CS_SYN_SENT = 0, CS_CONNECTED = 1, CS_FIN_SENT = 2, CS_CLOSED = 3, CS_RESET = 4 };

constexpr size_t kHeader = 20;
constexpr uint32_t kMss = 1400 - kHeader;        // payload per packet (fits a 1500-byte MTU path)
constexpr int64_t kTargetDelay = 100000;          // LEDBAT target: 100 ms
constexpr double kGain = 1.0;
constexpr uint32_t kMinWindow = 2 * kMss;
constexpr uint32_t kMaxWindow = 4u << 20;
constexpr uint32_t kRecvWindow = 1u << 20;        // advertised receive window
constexpr int64_t kMinRto = 500000;
constexpr int64_t kMaxRto = 60000000;
constexpr int kMaxRetransmits = 8;
constexpr size_t kMaxSendBuffer = 8u << 20;

inline uint16_t seq_diff(uint16_t a, uint16_t b) { return static_cast<uint16_t>(a - b); }
// a < b in sequence space
inline bool seq_lt(uint16_t a, uint16_t b) { return seq_diff(b, a) != 0 && seq_diff(b, a) < 0x8000; }

struct Header {
  uint8_t type, ver, ext;
  uint16_t conn_id;
  uint32_t ts, ts_diff, wnd;
  uint16_t seq, ack;
};

inline void put16(std::string& s, uint16_t v) {
  s.push_back(static_cast<char>(v >> 8));
  s.push_back(static_cast<char>(v & 0xFF));
}
inline void put32(std::string& s, uint32_t v) {
  for (int k = 3; k >= 0; --k) s.push_back(static_cast<char>((v >> (8 * k)) & 0xFF));
}
inline uint16_t get16(const uint8_t* p) { return static_cast<uint16_t>((p[0] << 8) | p[1]); }
inline uint32_t get32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}

// FIFO byte buffer with O(1) amortised pop-front (std::string::erase(0, n)
// per 1380-byte packet was an O(pending) memmove: quadratic at 8 MiB buffers).
struct ByteQueue {
  std::string buf;
  size_t off = 0;
  size_t size() const { return buf.size() - off; }
  bool empty() const { return off == buf.size(); }
  void append(const char* p, size_t n) {
    if (off && off == buf.size()) {
      buf.clear();
      off = 0;
    }
    buf.append(p, n);
  }
  void take_into(std::string& dst, size_t n) {
    n = std::min(n, size());
    dst.append(buf, off, n);
    off += n;
    if (off == buf.size()) {
      buf.clear();
      off = 0;
    } else if (off >= (1u << 20) && off * 2 >= buf.size()) {
      buf.erase(0, off);
      off = 0;
    }
  }
  std::string take(size_t n) {
    std::string r = buf.substr(off, n);
    off += r.size();
    if (off == buf.size()) {
      buf.clear();
      off = 0;
    } else if (off >= (1u << 20) && off * 2 >= buf.size()) {
      buf.erase(0, off);
      off = 0;
    }
    return r;
  }
  void clear() {
    buf.clear();
    off = 0;
  }
};

struct OutPkt {
  uint16_t seq;
  uint8_t type;
  std::shared_ptr<const std::string> pkt;  // header + payload as last sent (shared with the send queue)
  uint32_t psize = 0;                       // payload bytes
  int64_t sent_at = 0;
  int transmissions = 0;
  bool need_resend = false;
  bool fast_resent = false;   // already fast-retransmitted once (SACK / dup-ack)
  bool sacked = false;        // selectively acked: kept until the cumulative ack passes it
};

// One queued datagram: the peer address and packet bytes are shared (refcounted)
// with the connection / retransmission queue, so queueing copies neither.
struct Datagram {
  std::shared_ptr<const std::string> addr;
  std::shared_ptr<const std::string> pkt;
};

struct Conn {
  int id = 0;
  std::string addr;
  std::shared_ptr<const std::string> addr_p;  // same, shared with queued datagrams
  int state = CS_SYN_SENT;
  bool accepted = false;
  uint16_t recv_id = 0, send_id = 0;
  uint16_t seq_nr = 1;   // next seq to send
  uint16_t ack_nr = 0;   // last in-order seq received
  bool got_syn_ack = false;
  // send side
  std::deque<OutPkt> inflight;          // unacked, ordered by seq
  ByteQueue pending;                    // bytes not yet packetized
  uint32_t cur_window = 0;              // bytes in flight
  double max_window = kMinWindow * 4;   // LEDBAT cwnd
  uint32_t peer_wnd = kRecvWindow;
  int64_t rtt = 0, rtt_var = 800000, rto = 1000000;
  int64_t last_timeout_check = 0;
  int dup_acks = 0;
  bool slow_start = true;
  int64_t last_cut = 0;
  uint16_t last_ack_seen = 0;
  // delay measurements
  uint32_t reply_micro = 0;             // their ts -> our receive delta, echoed back
  std::deque<std::pair<int64_t, uint32_t>> base_delay;  // (minute bucket, min delay)
  uint32_t our_delay = 0;
  // receive side
  std::map<uint16_t, std::string> ooo;  // out-of-order payloads keyed by seq
  size_t ooo_bytes = 0;                  // their total: held to the receive window
  std::string inbuf;                    // in-order bytes for the app
  bool fin_received = false;
  uint16_t fin_seq = 0;
  bool fin_acked = false;
  bool need_ack = false;
  bool closing = false;                 // app called close: FIN after pending drains
  int64_t last_recv = 0;
  bool forget = false;                  // app is done with it: free once closed
  bool in_batch = false;                // touched in the current receive batch
  // stats
  uint64_t bytes_sent = 0, bytes_recv = 0, retransmits = 0, timeouts = 0, fast_retransmits = 0;
  uint64_t window_full_drops = 0;       // in-order packets dropped: the app's unread bytes filled the window
};

class Engine {
 public:
  explicit Engine(uint64_t seed) : rng_(seed ? seed : std::random_device{}()) {}

  int connect(const std::string& addr, int64_t now) {
    auto c = std::make_unique<Conn>();
    c->id = next_id_++;
    c->addr = addr;
    c->addr_p = std::make_shared<const std::string>(addr);
    c->recv_id = static_cast<uint16_t>(rng_());
    c->send_id = static_cast<uint16_t>(c->recv_id + 1);
    c->seq_nr = 1;
    c->state = CS_SYN_SENT;
    c->last_recv = now;
    by_addr_[addr][c->recv_id] = c->id;
    Conn& r = *c;
    conns_[c->id] = std::move(c);
    send_control(r, ST_SYN, now, /*consume_seq=*/true);
    return r.id;
  }

  int incoming(const std::string& pkt, const std::string& addr, int64_t now) {
    return incoming(pkt.data(), pkt.size(), addr, now);
  }

  // Zero-copy form (the socket pump hands its receive buffers straight in).
  int incoming(const char* data, size_t size, const std::string& addr, int64_t now) {
    if (size < kHeader) return -1;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(data);
    Header h{static_cast<uint8_t>(p[0] >> 4), static_cast<uint8_t>(p[0] & 0xF), p[1], get16(p + 2), get32(p + 4),
             get32(p + 8), get32(p + 12), get16(p + 16), get16(p + 18)};
    if (h.ver != 1 || h.type > ST_SYN) return -1;
    // parse extensions
    size_t off = kHeader;
    uint8_t ext = h.ext;
    std::string sack;
    while (ext != 0) {
      if (off + 2 > size) return -1;
      uint8_t next = p[off], len = p[off + 1];
      if (off + 2 + len > size) return -1;
      if (ext == 1) sack.assign(data + off + 2, len);
      ext = next;
      off += 2 + len;
    }
    const char* payload = data + off;
    const size_t payload_n = size - off;

    if (h.type == ST_SYN) {
      // new inbound connection (or a retransmitted SYN for one we know)
      uint16_t rid = static_cast<uint16_t>(h.conn_id + 1);
      const int known = find_conn(addr, rid);
      if (known > 0) {
        Conn& c = *conns_[known];
        c.need_ack = true;  // our SYN-ACK was lost: answer again
        flush(c, now);
        return c.id;
      }
      auto c = std::make_unique<Conn>();
      c->id = next_id_++;
      c->addr = addr;
      c->addr_p = std::make_shared<const std::string>(addr);
      c->recv_id = rid;
      c->send_id = h.conn_id;
      c->seq_nr = static_cast<uint16_t>(rng_());
      c->ack_nr = h.seq;
      c->state = CS_CONNECTED;
      c->accepted = true;
      c->got_syn_ack = true;
      c->last_recv = now;
      c->peer_wnd = h.wnd;
      c->reply_micro = static_cast<uint32_t>(now) - h.ts;
      by_addr_[addr][rid] = c->id;
      Conn& r = *c;
      conns_[c->id] = std::move(c);
      accepted_.push_back(r.id);
      send_state(r, now);
      return r.id;
    }
    const int cid = find_conn(addr, h.conn_id);
    if (cid <= 0) {
      if (h.type != ST_RESET) send_reset(addr, h.conn_id, h.seq, now);
      return -1;
    }
    Conn& c = *conns_[cid];
    c.last_recv = now;
    c.reply_micro = static_cast<uint32_t>(now) - h.ts;
    if (h.ts_diff != 0) update_delay(c, h.ts_diff, now);
    c.peer_wnd = h.wnd;

    if (h.type == ST_RESET) {
      c.state = CS_RESET;
      c.inflight.clear();
      c.pending.clear();
      return c.id;
    }
    if (c.state == CS_SYN_SENT) {
      if (h.type != ST_STATE) return c.id;
      c.state = CS_CONNECTED;
      c.got_syn_ack = true;
      c.ack_nr = static_cast<uint16_t>(h.seq - 1);  // their next DATA carries h.seq
    }
    process_ack(c, h.ack, sack, now);
    if (h.type == ST_DATA || h.type == ST_FIN) {
      if (h.type == ST_FIN) {
        c.fin_received = true;
        c.fin_seq = h.seq;
      }
      accept_data(c, h.seq, payload, payload_n, h.type == ST_FIN);
    }
    if (batch_) {
      // defer: one flush (so one cumulative ACK + SACK) per connection per
      // receive batch instead of one ACK per data packet
      if (!c.in_batch) {
        c.in_batch = true;
        touched_.push_back(c.id);
      }
    } else {
      flush(c, now);
    }
    return c.id;
  }

  // Receive batching: between begin_batch() and end_batch(), incoming() only
  // updates state; end_batch() flushes every touched connection once and
  // returns their ids (the app then drains each one's inbuf once).
  void begin_batch() { batch_ = true; }
  std::vector<int> end_batch(int64_t now) {
    batch_ = false;
    std::vector<int> ids;
    ids.swap(touched_);
    for (int id : ids) {
      Conn* c = get(id);
      if (!c) continue;
      c->in_batch = false;
      flush(*c, now);
    }
    return ids;
  }

  size_t write(int id, const std::string& data) {
    Conn* c = get(id);
    if (!c || c->state >= CS_FIN_SENT || c->closing) return 0;
    size_t room = kMaxSendBuffer > c->pending.size() ? kMaxSendBuffer - c->pending.size() : 0;
    size_t n = std::min(room, data.size());
    c->pending.append(data.data(), n);
    return n;
  }

  std::string read(int id) {
    Conn* c = get(id);
    std::string out;
    if (!c) return out;
    // a read that reopens a window we had advertised as (nearly) closed sends a
    // window update at the next flush, so the sender does not wait for a timeout
    if (c->inbuf.size() + 2 * kMss > kRecvWindow) c->need_ack = true;
    out.swap(c->inbuf);
    return out;
  }

  void close(int id, int64_t now) {
    Conn* c = get(id);
    if (!c) return;
    c->closing = true;
    flush(*c, now);
  }

  void abort(int id) {
    Conn* c = get(id);
    if (!c) return;
    if (c->state < CS_CLOSED) send_reset(c->addr, c->send_id, c->ack_nr, 0);
    c->state = CS_RESET;
  }

  void tick(int64_t now) {
    for (auto& kv : conns_) {
      Conn& c = *kv.second;
      if (c.forget && c.state == CS_FIN_SENT && c.fin_acked && c.inflight.empty()) c.state = CS_CLOSED;
      if (c.state >= CS_CLOSED) continue;
      // retransmission timeout on the oldest unacked packet
      if (!c.inflight.empty()) {
        OutPkt& o = c.inflight.front();
        if (now - o.sent_at > c.rto) {
          if (o.transmissions >= kMaxRetransmits) {
            c.state = CS_RESET;
            continue;
          }
          c.timeouts++;
          c.rto = std::min<int64_t>(c.rto * 2, kMaxRto);
          c.max_window = kMinWindow;  // LEDBAT: collapse to min on timeout
          c.slow_start = false;
          for (auto& q : c.inflight) q.need_resend = true;
        }
      } else if (c.state == CS_CONNECTED && now - c.last_recv > 120000000) {
        c.state = CS_RESET;  // idle two minutes with nothing to send: dead peer
        continue;
      }
      flush(c, now);
    }
    // forget dead connections once the app has drained them
    for (auto it = conns_.begin(); it != conns_.end();) {
      Conn& c = *it->second;
      if (c.state >= CS_CLOSED && c.inbuf.empty() && c.forget) {
        erase_conn(c.addr, c.recv_id);
        it = conns_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void forget(int id) {
    Conn* c = get(id);
    if (c) c->forget = true;
  }

  // Copying form (Python API / tests): [(addr, packet)].
  std::vector<std::pair<std::string, std::string>> outgoing() {
    std::vector<std::pair<std::string, std::string>> v;
    v.reserve(out_.size());
    for (auto& d : out_) v.emplace_back(*d.addr, *d.pkt);
    out_.clear();
    return v;
  }

  // Zero-copy form for the socket pump.
  std::vector<Datagram> take_datagrams() {
    std::vector<Datagram> v;
    v.swap(out_);
    return v;
  }

  std::vector<int> accepted() {
    std::vector<int> v;
    v.swap(accepted_);
    return v;
  }

  int state(int id) {
    Conn* c = get(id);
    if (!c) return CS_CLOSED;
    // a FIN_SENT connection whose FIN is acked and peer FIN received is closed
    return c->state;
  }

  bool eof(int id) {
    Conn* c = get(id);
    return !c || c->state == CS_RESET || (c->fin_received && seq_diff(c->ack_nr, c->fin_seq) == 0);
  }

  size_t send_buffered(int id) {
    Conn* c = get(id);
    return c ? c->pending.size() + c->cur_window : 0;
  }

  struct Stats {
    int state = CS_CLOSED;
    int64_t rtt_us = 0, rto_us = 0;
    double cwnd = 0;
    uint32_t inflight = 0, our_delay_us = 0;
    uint64_t bytes_sent = 0, bytes_recv = 0, retransmits = 0, timeouts = 0, fast_retransmits = 0;
    uint64_t window_full_drops = 0;
    uint64_t ooo_bytes = 0;
    std::string addr;
  };

  Stats stats(int id) {
    Stats s;
    Conn* c = get(id);
    if (!c) return s;
    s.state = c->state;
    s.rtt_us = c->rtt;
    s.rto_us = c->rto;
    s.cwnd = c->max_window;
    s.inflight = c->cur_window;
    s.our_delay_us = c->our_delay;
    s.bytes_sent = c->bytes_sent;
    s.bytes_recv = c->bytes_recv;
    s.retransmits = c->retransmits;
    s.timeouts = c->timeouts;
    s.fast_retransmits = c->fast_retransmits;
    s.window_full_drops = c->window_full_drops;
    s.ooo_bytes = c->ooo_bytes;
    s.addr = c->addr;
    return s;
  }

  size_t size() const { return conns_.size(); }

 private:
  int find_conn(const std::string& addr, uint16_t id) const {
    auto a = by_addr_.find(addr);  // no key string is built per packet
    if (a == by_addr_.end()) return -1;
    auto b = a->second.find(id);
    return b == a->second.end() ? -1 : b->second;
  }
  void erase_conn(const std::string& addr, uint16_t id) {
    auto a = by_addr_.find(addr);
    if (a == by_addr_.end()) return;
    a->second.erase(id);
    if (a->second.empty()) by_addr_.erase(a);
  }
  Conn* get(int id) {
    auto it = conns_.find(id);
    return it == conns_.end() ? nullptr : it->second.get();
  }

  std::string header(const Conn& c, uint8_t type, uint16_t seq, int64_t now, const std::string* sack) {
    std::string s;
    s.reserve(kHeader + kMss + 8);
    s.push_back(static_cast<char>((type << 4) | 1));
    s.push_back(static_cast<char>(sack ? 1 : 0));
    put16(s, type == ST_SYN ? c.recv_id : c.send_id);
    put32(s, static_cast<uint32_t>(now));
    put32(s, c.reply_micro);
    uint32_t avail = kRecvWindow > c.inbuf.size() ? kRecvWindow - static_cast<uint32_t>(c.inbuf.size()) : 0;
    put32(s, avail);
    put16(s, seq);
    put16(s, c.ack_nr);
    if (sack) {
      s.push_back(0);  // no further extension
      s.push_back(static_cast<char>(sack->size()));
      s += *sack;
    }
    return s;
  }

  std::string build_sack(const Conn& c) {
    if (c.ooo.empty()) return std::string();
    // bit k = seq ack_nr + 2 + k received
    std::string bits(4, '\0');
    for (auto& kv : c.ooo) {
      uint16_t d = seq_diff(kv.first, static_cast<uint16_t>(c.ack_nr + 2));
      if (d < 32) bits[d >> 3] |= static_cast<char>(1 << (d & 7));
    }
    return bits;
  }

  void send_state(Conn& c, int64_t now) {
    std::string sack = build_sack(c);
    out_.push_back({c.addr_p, std::make_shared<const std::string>(
                                 header(c, ST_STATE, c.seq_nr, now, sack.empty() ? nullptr : &sack))});
    c.need_ack = false;
  }

  void send_control(Conn& c, uint8_t type, int64_t now, bool consume_seq) {
    OutPkt o;
    o.seq = c.seq_nr;
    o.type = type;
    o.sent_at = now;
    o.transmissions = 1;
    o.pkt = std::make_shared<const std::string>(header(c, type, o.seq, now, nullptr));
    out_.push_back({c.addr_p, o.pkt});
    if (consume_seq) {
      c.seq_nr++;
      c.inflight.push_back(std::move(o));
    }
  }

  void send_reset(const std::string& addr, uint16_t conn_id, uint16_t ack, int64_t now) {
    std::string s;
    s.push_back(static_cast<char>((ST_RESET << 4) | 1));
    s.push_back(0);
    put16(s, conn_id);
    put32(s, static_cast<uint32_t>(now));
    put32(s, 0);
    put32(s, 0);
    put16(s, static_cast<uint16_t>(rng_()));
    put16(s, ack);
    out_.push_back({std::make_shared<const std::string>(addr), std::make_shared<const std::string>(std::move(s))});
  }

  void update_delay(Conn& c, uint32_t sample, int64_t now) {
    int64_t minute = now / 60000000;
    if (c.base_delay.empty() || c.base_delay.back().first != minute) {
      c.base_delay.emplace_back(minute, sample);
      while (c.base_delay.size() > 13) c.base_delay.pop_front();  // ~13 minute history
    } else if (static_cast<int32_t>(sample - c.base_delay.back().second) < 0) {
      c.base_delay.back().second = sample;
    }
    uint32_t base = c.base_delay.front().second;
    for (auto& b : c.base_delay)
      if (static_cast<int32_t>(b.second - base) < 0) base = b.second;
    c.our_delay = sample - base;
  }

  void process_ack(Conn& c, uint16_t ack, const std::string& sack, int64_t now) {
    uint32_t acked_bytes = 0;
    int64_t min_rtt_sample = -1;
    // cumulative ack: everything with seq <= ack
    while (!c.inflight.empty() && !seq_lt(ack, c.inflight.front().seq)) {
      OutPkt& o = c.inflight.front();
      if (o.transmissions == 1) {
        int64_t sample = now - o.sent_at;
        if (min_rtt_sample < 0 || sample < min_rtt_sample) min_rtt_sample = sample;
      }
      if (!o.sacked) {
        acked_bytes += static_cast<uint32_t>(o.psize);
        c.cur_window -= std::min<uint32_t>(c.cur_window, static_cast<uint32_t>(o.psize));
      }
      if (o.type == ST_FIN) c.fin_acked = true;
      c.inflight.pop_front();
    }
    // selective acks: mark packets beyond ack+1 as delivered (their bytes leave
    // the window) but keep them until the cumulative ack passes; an unsacked
    // packet with >= 3 sacked packets after it is lost -> fast retransmit once
    if (!sack.empty()) {
      for (auto& o : c.inflight) {
        uint16_t d = seq_diff(o.seq, static_cast<uint16_t>(ack + 2));
        if (!o.sacked && d < sack.size() * 8 && ((static_cast<uint8_t>(sack[d >> 3]) >> (d & 7)) & 1)) {
          o.sacked = true;
          acked_bytes += static_cast<uint32_t>(o.psize);
          c.cur_window -= std::min<uint32_t>(c.cur_window, static_cast<uint32_t>(o.psize));
        }
      }
      int after = 0;
      bool lost = false;
      for (auto it = c.inflight.rbegin(); it != c.inflight.rend(); ++it) {
        if (it->sacked) {
          ++after;
        } else if (after >= 3 && !it->fast_resent && it->type != ST_SYN) {
          it->need_resend = true;
          it->fast_resent = true;
          lost = true;
        }
      }
      if (lost) on_loss(c, now);
    }
    if (ack == c.last_ack_seen && acked_bytes == 0 && !c.inflight.empty()) {
      if (++c.dup_acks >= 3 && !c.inflight.front().fast_resent) {
        c.inflight.front().need_resend = true;
        c.inflight.front().fast_resent = true;
        c.dup_acks = 0;
        on_loss(c, now);
      }
    } else if (acked_bytes) {
      c.dup_acks = 0;
    }
    c.last_ack_seen = ack;
    if (min_rtt_sample >= 0) {
      if (c.rtt == 0) {
        c.rtt = min_rtt_sample;
        c.rtt_var = min_rtt_sample / 2;
      } else {
        int64_t delta = c.rtt - min_rtt_sample;
        c.rtt_var += ((delta < 0 ? -delta : delta) - c.rtt_var) / 4;
        c.rtt += (min_rtt_sample - c.rtt) / 8;
      }
      c.rto = std::clamp<int64_t>(c.rtt + 4 * c.rtt_var, kMinRto, kMaxRto);
    }
    if (acked_bytes && c.slow_start && c.our_delay < kTargetDelay / 2) {
      // slow start (RFC 6817 §2.4.2 allows it) until loss or half the target delay
      c.max_window = std::min<double>(c.max_window + acked_bytes, kMaxWindow);
    } else if (acked_bytes) {
      c.slow_start = false;
      // LEDBAT window update
      double off_target = static_cast<double>(kTargetDelay - static_cast<int64_t>(c.our_delay)) / kTargetDelay;
      double gain = kGain * off_target * acked_bytes * kMss / std::max(c.max_window, 1.0);
      c.max_window = std::clamp(c.max_window + gain, static_cast<double>(kMinWindow), static_cast<double>(kMaxWindow));
    }
  }

  // multiplicative decrease at most once per RTT
  void on_loss(Conn& c, int64_t now) {
    c.fast_retransmits++;
    c.slow_start = false;
    if (now - c.last_cut > std::max<int64_t>(c.rtt, 10000)) {
      c.max_window = std::max<double>(kMinWindow, c.max_window / 2);
      c.last_cut = now;
    }
  }

  void accept_data(Conn& c, uint16_t seq, const char* payload, size_t payload_n, bool fin) {
    uint16_t expect = static_cast<uint16_t>(c.ack_nr + 1);
    if (seq_lt(seq, expect)) {  // duplicate: re-ack
      c.need_ack = true;
      return;
    }
    if (seq != expect) {
      // a peer may send up to 1024 packets ahead, but what it parks here stays
      // within the receive window we advertise (datagrams can be 64 KiB each)
      const size_t n = fin ? 0 : payload_n;
      if (seq_diff(seq, expect) < 1024 && !c.ooo.count(seq) && c.ooo_bytes + n <= kRecvWindow) {
        c.ooo[seq] = std::string(payload, n);
        c.ooo_bytes += n;
      }
      c.need_ack = true;
      return;
    }
    if (!fin) {
      if (c.inbuf.size() + payload_n > kRecvWindow + kMss) {
        // the app stopped reading (it is backed up) and the window we advertised
        // is used up: drop the packet unacked; the sender retries after the window
        // update that the next read() sends.  The bytes held for a paused reader
        // therefore stay bounded by the window.
        c.window_full_drops++;
        return;
      }
      c.inbuf.append(payload, payload_n);
      c.bytes_recv += payload_n;
    }
    c.ack_nr = seq;
    // pull in buffered successors
    for (;;) {
      auto it = c.ooo.find(static_cast<uint16_t>(c.ack_nr + 1));
      if (it == c.ooo.end()) break;
      bool is_fin = c.fin_received && it->first == c.fin_seq;
      if (!is_fin) {
        c.inbuf += it->second;
        c.bytes_recv += it->second.size();
      }
      c.ack_nr = it->first;
      c.ooo_bytes -= it->second.size();
      c.ooo.erase(it);
    }
    c.need_ack = true;
  }

  void flush(Conn& c, int64_t now) {
    if (c.state == CS_RESET || c.state == CS_CLOSED) return;
    // 1) retransmissions (bounded by the window as well)
    for (auto& o : c.inflight) {
      if (!o.need_resend || o.sacked) {
        o.need_resend = false;
        continue;
      }
      o.need_resend = false;
      o.sent_at = now;
      o.transmissions++;
      c.retransmits++;
      // fresh header (timestamps, ack) in front of the same payload
      auto np = std::make_shared<std::string>(header(c, o.type, o.seq, now, nullptr));
      if (o.pkt && o.pkt->size() > kHeader) np->append(*o.pkt, kHeader, std::string::npos);
      o.pkt = np;
      out_.push_back({c.addr_p, o.pkt});
      c.need_ack = false;
    }
    // 2) new data within min(cwnd, peer window)
    if (c.state == CS_CONNECTED) {
      uint32_t win = static_cast<uint32_t>(std::min<double>(c.max_window, c.peer_wnd ? c.peer_wnd : kMss));
      while (!c.pending.empty() && (c.cur_window + std::min<size_t>(kMss, c.pending.size()) <= win ||
                                    c.cur_window == 0)) {
        size_t n = std::min<size_t>(kMss, c.pending.size());
        OutPkt o;
        o.seq = c.seq_nr++;
        o.type = ST_DATA;
        o.psize = static_cast<uint32_t>(n);
        o.sent_at = now;
        o.transmissions = 1;
        auto pk = std::make_shared<std::string>(header(c, ST_DATA, o.seq, now, nullptr));
        c.pending.take_into(*pk, n);  // one copy: send buffer -> packet
        o.pkt = pk;
        out_.push_back({c.addr_p, o.pkt});
        c.cur_window += static_cast<uint32_t>(n);
        c.bytes_sent += n;
        c.inflight.push_back(std::move(o));
        c.need_ack = false;
      }
      if (c.closing && c.pending.empty()) {
        send_control(c, ST_FIN, now, true);
        c.state = CS_FIN_SENT;
      }
    }
    if (c.state == CS_FIN_SENT && c.fin_acked && c.inflight.empty() && c.fin_received) c.state = CS_CLOSED;
    if (c.need_ack) send_state(c, now);
  }

  std::mt19937_64 rng_;
  int next_id_ = 1;
  std::unordered_map<int, std::unique_ptr<Conn>> conns_;
  std::unordered_map<std::string, std::unordered_map<uint16_t, int>> by_addr_;
  std::vector<Datagram> out_;
  std::vector<int> accepted_;
  bool batch_ = false;
  std::vector<int> touched_;
};

}  // namespace tritondl_utp
