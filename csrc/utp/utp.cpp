// uTP — the Micro Transport Protocol (BEP 29) with LEDBAT congestion control.
//
// Native replacement for the transport the reference reaches through
// anacrolix/torrent: cgo libutp (go-libutp) or pure-Go anacrolix/utp
// (SURVEY.md §2.2).  Design: a *sans-IO* engine.  Python owns the single UDP
// socket (asyncio) and the clock; this module owns every protocol decision:
// connection ids, sequence/ack numbers, the reorder buffer, selective ACKs,
// RTT/RTO estimation, LEDBAT window control, retransmission, FIN/RESET.
//
//   Engine.connect(addr, now_us)            -> conn id (SYN queued)
//   Engine.incoming(pkt, addr, now_us)      -> conn id (or -1); may create an
//                                              accepted conn for a SYN
//   Engine.write(cid, bytes) -> n accepted  Engine.read(cid) -> bytes
//   Engine.close(cid)   Engine.tick(now_us)  Engine.outgoing() -> [(addr, pkt)]
//   Engine.state(cid)   Engine.accepted() -> [cid]   Engine.stats(cid)
//
// Thread model: called from one event-loop thread; no locks.  All integer
// sequence arithmetic is modulo 2^16 as the wire format requires.
//
// Pump: optional native socket I/O for the engine.  Python registers the UDP
// fd with its event loop; on readability Pump.recv() drains the socket with
// recvmmsg (64 datagrams per syscall) into the engine inside one receive batch
// (one ACK per connection per batch), and Pump.send() ships every queued
// packet with sendmmsg.  Per-datagram Python callbacks were the uTP
// throughput ceiling (~12k packets/s).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/socket.h>

#include <cerrno>

#include "utp_engine.h"

namespace py = pybind11;
using tritondl_utp::Engine;

namespace {

struct SockAddr {
  sockaddr_storage ss{};
  socklen_t len = 0;
};

bool parse_key(const std::string& key, SockAddr* out) {
  auto colon = key.rfind(':');
  if (colon == std::string::npos) return false;
  std::string host = key.substr(0, colon);
  int port = std::atoi(key.c_str() + colon + 1);
  if (port <= 0 || port > 65535) return false;
  if (!host.empty() && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  auto* v4 = reinterpret_cast<sockaddr_in*>(&out->ss);
  if (inet_pton(AF_INET, host.c_str(), &v4->sin_addr) == 1) {
    v4->sin_family = AF_INET;
    v4->sin_port = htons(static_cast<uint16_t>(port));
    out->len = sizeof(sockaddr_in);
    return true;
  }
  auto* v6 = reinterpret_cast<sockaddr_in6*>(&out->ss);
  if (inet_pton(AF_INET6, host.c_str(), &v6->sin6_addr) == 1) {
    v6->sin6_family = AF_INET6;
    v6->sin6_port = htons(static_cast<uint16_t>(port));
    out->len = sizeof(sockaddr_in6);
    return true;
  }
  return false;
}

std::pair<std::string, int> format_addr(const sockaddr_storage& ss) {
  char buf[INET6_ADDRSTRLEN] = {0};
  if (ss.ss_family == AF_INET) {
    auto* v4 = reinterpret_cast<const sockaddr_in*>(&ss);
    inet_ntop(AF_INET, &v4->sin_addr, buf, sizeof(buf));
    return {buf, ntohs(v4->sin_port)};
  }
  auto* v6 = reinterpret_cast<const sockaddr_in6*>(&ss);
  inet_ntop(AF_INET6, &v6->sin6_addr, buf, sizeof(buf));
  return {buf, ntohs(v6->sin6_port)};
}

class Pump {
 public:
  static constexpr int kBatch = 64;
  static constexpr size_t kBufSize = 2048;

  Pump(Engine& e, int fd) : e_(e), fd_(fd), bufs_(kBatch * kBufSize) {}

  // -> (touched conn ids, [(datagram, (host, port))] that are not uTP)
  py::tuple recv(int64_t now, int max_packets) {
    std::vector<std::pair<std::string, std::pair<std::string, int>>> others;
    int got_total = 0;
    e_.begin_batch();
    while (got_total < max_packets) {
      mmsghdr msgs[kBatch];
      iovec iov[kBatch];
      sockaddr_storage from[kBatch];
      for (int k = 0; k < kBatch; ++k) {
        iov[k] = {bufs_.data() + k * kBufSize, kBufSize};
        std::memset(&msgs[k].msg_hdr, 0, sizeof(msghdr));
        msgs[k].msg_hdr.msg_iov = &iov[k];
        msgs[k].msg_hdr.msg_iovlen = 1;
        msgs[k].msg_hdr.msg_name = &from[k];
        msgs[k].msg_hdr.msg_namelen = sizeof(sockaddr_storage);
      }
      int n = recvmmsg(fd_, msgs, kBatch, MSG_DONTWAIT, nullptr);
      if (n <= 0) break;  // EAGAIN (drained) or a transient error (ICMP unreachable): stop this round
      for (int k = 0; k < n; ++k) {
        const char* d = bufs_.data() + k * kBufSize;
        size_t len = msgs[k].msg_len;
        bool utp = len >= 1 && (static_cast<uint8_t>(d[0]) & 0x0F) == 1 && (static_cast<uint8_t>(d[0]) >> 4) <= 4;
        if (!utp || len < tritondl_utp::kHeader) {
          others.emplace_back(std::string(d, len), format_addr(from[k]));
          continue;
        }
        e_.incoming(d, len, addr_key(from[k]), now);  // zero-copy into the engine
      }
      got_total += n;
      if (n < kBatch) break;
    }
    std::vector<int> touched = e_.end_batch(now);
    py::list py_others;
    for (auto& o : others)
      py_others.append(py::make_tuple(py::bytes(o.first), py::make_tuple(o.second.first, o.second.second)));
    return py::make_tuple(touched, py_others);
  }

  // Ship queued packets; returns how many are still queued (socket full).
  size_t send() {
    for (auto& d : e_.take_datagrams()) q_.push_back(std::move(d));
    while (!q_.empty()) {
      int n = static_cast<int>(std::min<size_t>(kBatch, q_.size()));
      mmsghdr msgs[kBatch];
      iovec iov[kBatch];
      SockAddr to[kBatch];
      int m = 0;
      for (int k = 0; k < n; ++k) {
        auto& dg = q_[k];
        if (!lookup(*dg.addr, &to[m])) continue;  // unparseable address: dropped below
        iov[m] = {const_cast<char*>(dg.pkt->data()), dg.pkt->size()};
        std::memset(&msgs[m].msg_hdr, 0, sizeof(msghdr));
        msgs[m].msg_hdr.msg_iov = &iov[m];
        msgs[m].msg_hdr.msg_iovlen = 1;
        msgs[m].msg_hdr.msg_name = &to[m].ss;
        msgs[m].msg_hdr.msg_namelen = to[m].len;
        ++m;
      }
      if (m == 0) {
        q_.erase(q_.begin(), q_.begin() + n);
        continue;
      }
      int sent = sendmmsg(fd_, msgs, m, MSG_DONTWAIT);
      if (sent < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOBUFS) break;
        sent = 1;  // hard error on the first packet (e.g. unreachable): drop it, keep going
      }
      // advance past `sent` sendable packets, plus any unparseable ones among them
      int consumed = 0, sendable = 0;
      while (consumed < n && sendable < sent) {
        SockAddr tmp;
        if (lookup(*q_[consumed].addr, &tmp)) ++sendable;
        ++consumed;
      }
      q_.erase(q_.begin(), q_.begin() + consumed);
      if (sent < m) break;  // partial: socket buffer full
    }
    return q_.size();
  }

  size_t queued() const { return q_.size(); }

 private:
  bool lookup(const std::string& key, SockAddr* out) {
    auto it = cache_.find(key);
    if (it != cache_.end()) {
      *out = it->second;
      return it->second.len != 0;
    }
    SockAddr a;
    if (!parse_key(key, &a)) a.len = 0;
    if (cache_.size() > 4096) cache_.clear();
    cache_[key] = a;
    *out = a;
    return a.len != 0;
  }

  Engine& e_;
  int fd_;
  std::vector<char> bufs_;
  // "ip:port" engine key of a peer sockaddr, memoised (IPv4: keyed by addr+port)
  const std::string& addr_key(const sockaddr_storage& ss) {
    uint64_t k = 0;
    if (ss.ss_family == AF_INET) {
      auto* v4 = reinterpret_cast<const sockaddr_in*>(&ss);
      k = (static_cast<uint64_t>(v4->sin_addr.s_addr) << 16) | v4->sin_port;
      auto it = keys_.find(k);
      if (it != keys_.end()) return it->second;
    }
    auto a = format_addr(ss);
    std::string key = a.first + ":" + std::to_string(a.second);
    if (ss.ss_family != AF_INET) {
      scratch_ = std::move(key);
      return scratch_;
    }
    if (keys_.size() > 4096) keys_.clear();
    return keys_.emplace(k, std::move(key)).first->second;
  }

  std::deque<tritondl_utp::Datagram> q_;
  std::unordered_map<std::string, SockAddr> cache_;
  std::unordered_map<uint64_t, std::string> keys_;
  std::string scratch_;
};

}  // namespace

PYBIND11_MODULE(_utp, m) {
  m.doc() = "tritondl native uTP (BEP 29) engine: LEDBAT, selective ACK, retransmission (sans-IO)";
  m.attr("SYN_SENT") = static_cast<int>(tritondl_utp::CS_SYN_SENT);
  m.attr("CONNECTED") = static_cast<int>(tritondl_utp::CS_CONNECTED);
  m.attr("FIN_SENT") = static_cast<int>(tritondl_utp::CS_FIN_SENT);
  m.attr("CLOSED") = static_cast<int>(tritondl_utp::CS_CLOSED);
  m.attr("RESET") = static_cast<int>(tritondl_utp::CS_RESET);
  m.attr("MSS") = tritondl_utp::kMss;
  py::class_<Engine>(m, "Engine")
      .def(py::init<uint64_t>(), py::arg("seed") = 0)
      .def("connect", &Engine::connect)
      .def("incoming", [](Engine& e, py::bytes pkt, const std::string& addr, int64_t now) {
        return e.incoming(std::string(pkt), addr, now);
      })
      .def("write", [](Engine& e, int id, py::bytes data) { return e.write(id, std::string(data)); })
      .def("read", [](Engine& e, int id) { return py::bytes(e.read(id)); })
      .def("close", &Engine::close)
      .def("abort", &Engine::abort)
      .def("forget", &Engine::forget)
      .def("tick", &Engine::tick)
      .def("outgoing", [](Engine& e) {
        py::list out;
        for (auto& kv : e.outgoing()) out.append(py::make_tuple(kv.first, py::bytes(kv.second)));
        return out;
      })
      .def("accepted", &Engine::accepted)
      .def("state", &Engine::state)
      .def("eof", &Engine::eof)
      .def("send_buffered", &Engine::send_buffered)
      .def("stats", [](Engine& e, int id) {
        auto s = e.stats(id);
        py::dict d;
        d["state"] = s.state;
        d["rtt_us"] = s.rtt_us;
        d["rto_us"] = s.rto_us;
        d["cwnd"] = s.cwnd;
        d["inflight"] = s.inflight;
        d["our_delay_us"] = s.our_delay_us;
        d["bytes_sent"] = s.bytes_sent;
        d["bytes_recv"] = s.bytes_recv;
        d["retransmits"] = s.retransmits;
        d["timeouts"] = s.timeouts;
        d["fast_retransmits"] = s.fast_retransmits;
        d["window_full_drops"] = s.window_full_drops;
        d["ooo_bytes"] = s.ooo_bytes;
        d["addr"] = s.addr;
        return d;
      })
      .def("begin_batch", &Engine::begin_batch)
      .def("end_batch", &Engine::end_batch)
      .def("__len__", &Engine::size);
  py::class_<Pump>(m, "Pump")
      .def(py::init<Engine&, int>(), py::keep_alive<1, 2>(), py::arg("engine"), py::arg("fd"))
      .def("recv", &Pump::recv, py::arg("now"), py::arg("max_packets") = 4096)
      .def("send", &Pump::send)
      .def("queued", &Pump::queued);
}
