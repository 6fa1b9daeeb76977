// BitTorrent peer-wire data plane (reference: the anacrolix/torrent client the
// reference drives from internal/downloader/torrent/torrent.go:40-106).
//
// The control logic (which piece from which peer, choking, metadata, PEX,
// verification, storage) stays in the Python Torrent; the per-16 KiB-block
// work moves here:
//
//  * PieceStore — per-torrent buffers of the pieces being fetched, with a
//    received-block bitmap.  Blocks from any connection land in the same
//    buffer, so end-game duplicates cost a copy, not a second piece.
//  * Link — one per peer connection.  feed() takes the plaintext bytes the
//    connection read (TCP, uTP or MSE-decrypted alike), splits BitTorrent
//    messages, copies PIECE payloads straight into the store, handles
//    CHOKE / UNCHOKE / REJECT for its own requests, and returns only what
//    Python must see: completed pieces and the non-data messages.  It also
//    keeps up to `pipeline` block REQUESTs outstanding over the pieces Python
//    assigned to it, and emits CANCELs when another link finished a piece.
//
// Everything runs on the caller's (event-loop) thread with the GIL held:
// one native call per socket read instead of ~10 Python operations per block.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "btwire_core.h"

namespace py = pybind11;
using namespace tritondl_btwire;

namespace {

// Events as the tuples Torrent._native_events expects.
py::list to_py(const std::vector<Event>& ev) {
  py::list out;
  for (const Event& e : ev) {
    switch (e.kind) {
      case Event::kPieceDone: out.append(py::make_tuple("piece", e.piece)); break;
      case Event::kMsg: out.append(py::make_tuple("msg", int(e.id), py::bytes(e.data))); break;
      case Event::kChoked: out.append(py::make_tuple("choke")); break;
      case Event::kUnchoked: out.append(py::make_tuple("unchoke")); break;
      case Event::kBad: out.append(py::make_tuple("bad", e.data)); break;
    }
  }
  return out;
}

py::tuple feed_bytes(Link& l, const py::bytes& data) {
  char* p = nullptr;
  Py_ssize_t n = 0;
  PyBytes_AsStringAndSize(data.ptr(), &p, &n);
  std::vector<Event> ev;
  std::string out;
  l.feed(reinterpret_cast<const uint8_t*>(p), size_t(n), &ev, &out);
  return py::make_tuple(to_py(ev), py::bytes(out));
}

py::tuple feed_n(Link& l, size_t n) {
  std::vector<Event> ev;
  std::string out;
  l.feed_n(n, &ev, &out);
  return py::make_tuple(to_py(ev), py::bytes(out));
}

}  // namespace

PYBIND11_MODULE(_btwire, m) {
  m.doc() = "tritondl BitTorrent peer-wire data plane (block assembly + request pipelining)";
  m.attr("BLOCK") = kBlock;
  py::class_<Piece>(m, "Piece", py::buffer_protocol())
      .def_buffer([](Piece& p) {
        return py::buffer_info(const_cast<uint8_t*>(p.data().data()), 1, "B", 1, {py::ssize_t(p.data().size())},
                               {py::ssize_t(1)}, true);
      })
      .def("__len__", [](const Piece& p) { return p.data().size(); })
      .def("tobytes", [](const Piece& p) {
        return py::bytes(reinterpret_cast<const char*>(p.data().data()), p.data().size());
      });
  py::class_<PieceStore, std::shared_ptr<PieceStore>>(m, "PieceStore")
      .def(py::init<uint32_t, uint64_t, uint64_t>(), py::arg("num_pieces"), py::arg("piece_len"),
           py::arg("total_len"))
      .def("begin", &PieceStore::begin)
      .def("active", &PieceStore::active)
      .def("has_block", &PieceStore::has_block)
      .def("received", &PieceStore::received)
      .def("blocks", &PieceStore::blocks)
      .def("piece_size", &PieceStore::piece_size)
      .def("put", [](PieceStore& s, uint32_t i, uint32_t off, const py::bytes& b, uint32_t who) {
        char* p = nullptr;
        Py_ssize_t n = 0;
        PyBytes_AsStringAndSize(b.ptr(), &p, &n);
        return s.put(i, off, reinterpret_cast<const uint8_t*>(p), size_t(n), who);
      }, py::arg("i"), py::arg("off"), py::arg("data"), py::arg("who") = 0)
      .def("block_sources", &PieceStore::block_sources,
           "per block of buffered piece i: id of the link that supplied it (0 = missing); call before take()")
      .def("take", &PieceStore::take)
      .def_property_readonly("pooled", &PieceStore::pooled)
      .def("reset", &PieceStore::reset)
      .def("active_pieces", &PieceStore::active_pieces)
      .def_property_readonly("partial_bytes", &PieceStore::partial_bytes);
  py::class_<Source, std::shared_ptr<Source>>(m, "Source")
      .def(py::init<uint32_t, uint64_t, uint64_t>(), py::arg("num_pieces"), py::arg("piece_len"),
           py::arg("total_len"))
      .def("add_file", &Source::add_file, py::arg("fd"), py::arg("start"), py::arg("length"),
           "Next file of the stream (fd is dup()ed; -1 = padding, reads as zeros).")
      .def("close", &Source::close)
      .def("set_have", &Source::set_have)
      .def("set_have_bits",
           [](Source& s, const py::bytes& b) {
             char* p = nullptr;
             Py_ssize_t n = 0;
             PyBytes_AsStringAndSize(b.ptr(), &p, &n);
             s.set_have_bits(reinterpret_cast<const uint8_t*>(p), size_t(n));
           },
           "One byte per piece, nonzero = have.")
      .def("has", &Source::has)
      .def("read",
           [](const Source& s, uint64_t gofs, size_t n) {
             std::string out(n, '\0');
             if (!s.read(gofs, &out[0], n)) throw std::runtime_error("short read");
             return py::bytes(out);
           });
  py::class_<Link>(m, "Link")
      .def(py::init<std::shared_ptr<PieceStore>, int, bool, uint32_t>(), py::arg("store"), py::arg("pipeline") = 128,
           py::arg("fast") = false, py::arg("id") = 0)
      .def_property_readonly("id", &Link::id)
      .def("feed", &feed_bytes,
           "Parse bytes read from the peer; returns (events, bytes to send).  events: ('piece', i) when a "
           "block from this link completed piece i; ('msg', id, payload) for every non-data message; "
           "('choke',) / ('unchoke',) after handling them here; ('bad', reason) on a protocol violation.")
      .def("recv_buffer",
           [](Link& l, size_t want) {
             auto span = l.recv_buffer(want);
             return py::memoryview::from_memory(span.first, py::ssize_t(span.second), false);
           },
           py::arg("want") = 262144,
           "Writable view of the receive buffer for recv_into (valid until the next feed/feed_n/recv_buffer).")
      .def("feed_n", &feed_n, "Parse the n bytes just written into recv_buffer(); same result as feed().")
      .def("pump", [](Link& l) { return py::bytes(l.pump()); })
      .def("assign", &Link::assign)
      .def("piece_done", &Link::piece_done)
      .def("drop", &Link::drop)
      .def("need_work", &Link::need_work)
      .def("assigned", &Link::assigned)
      .def("lapse_all", &Link::lapse_all)
      .def("oldest_request_age", &Link::oldest_request_age)
      .def_property_readonly("outstanding", &Link::outstanding)
      .def_property("peer_choking", &Link::peer_choking, &Link::set_peer_choking)
      .def_property_readonly("downloaded", &Link::downloaded)
      .def_property_readonly("wasted", &Link::wasted, "bytes of unrequested PIECE messages (dropped)")
      .def("set_source", &Link::set_source)
      .def_property("serving", &Link::serving, &Link::set_serving)
      .def_property_readonly("uploaded", &Link::uploaded)
      .def_property_readonly("stalled", &Link::stalled,
                             "the last feed hit the serve budget; feed_n(0) / feed(b'') parses the rest")
      .def_property_readonly("serve_errors", &Link::serve_errors)
      .def_property_readonly("buffered", &Link::buffered);
}
