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
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "utp_engine.h"

namespace py = pybind11;
using tritondl_utp::Engine;

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
        d["addr"] = s.addr;
        return d;
      })
      .def("__len__", &Engine::size);
}
