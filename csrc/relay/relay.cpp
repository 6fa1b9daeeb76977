// pybind11 bindings for the native fetch -> S3 data plane (relay_core.h).
// Every pump releases the GIL for its whole run; Python awaits it from an
// executor thread while the event loop keeps serving the control plane.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "relay_core.h"

namespace py = pybind11;
using namespace tritondl_relay;

PYBIND11_MODULE(_relay, m) {
  m.doc() = "tritondl native data plane: socket->file receive pump, file->socket aws-chunked/plain send pump";

  py::class_<Flow, std::shared_ptr<Flow>>(m, "Flow")
      .def(py::init([](const std::vector<std::tuple<uint64_t, int64_t, uint64_t>>& segs) {
             std::vector<Flow::Seg> v;
             v.reserve(segs.size());
             for (auto& s : segs) v.push_back({std::get<0>(s), std::get<1>(s), std::get<2>(s)});
             return std::make_shared<Flow>(std::move(v));
           }),
           py::arg("segments"), "segments: [(start, end_or_-1, done), ...]")
      .def("advance", &Flow::advance, py::arg("seg"), py::arg("done"))
      .def("finish", &Flow::finish, py::arg("total"))
      .def("fail", &Flow::fail, py::arg("why"))
      .def("cancel", &Flow::cancel)
      .def("done", &Flow::done, py::arg("seg"))
      .def("watermark", &Flow::watermark)
      .def("covered_bytes", &Flow::covered_bytes, py::arg("start"), py::arg("end"))
      .def("bytes_until_covered", &Flow::bytes_until_covered, py::arg("start"), py::arg("end"))
      .def_property_readonly("cancelled", &Flow::cancelled)
      .def_property_readonly("failed", &Flow::failed)
      .def_property_readonly("finished", &Flow::finished)
      .def_property_readonly("error", &Flow::error)
      .def("wait_covered", [](Flow& f, uint64_t a, uint64_t b, double timeout) {
             py::gil_scoped_release nogil;
             return f.wait_covered(a, b, timeout);
           },
           py::arg("start"), py::arg("end"), py::arg("timeout"),
           "0 = on disk, 1 = failed/cancelled, 2 = timeout, 3 = download ended short");

  m.def("recv_body",
        [](int sock, int fd, uint64_t off, int64_t length, const py::bytes& prefix, std::shared_ptr<Flow> flow,
           size_t seg, uint64_t seg_done0, double idle_timeout, size_t buf_size, bool use_splice) {
          std::string pre = prefix;
          RecvResult r;
          {
            py::gil_scoped_release nogil;
            r = recv_body(sock, fd, off, length, pre.data(), pre.size(), flow.get(), seg, seg_done0, idle_timeout,
                          buf_size, use_splice);
          }
          return py::make_tuple(r.received, r.eof, r.err);
        },
        py::arg("sock"), py::arg("fd"), py::arg("offset"), py::arg("length"), py::arg("prefix"), py::arg("flow"),
        py::arg("seg") = 0, py::arg("seg_done0") = 0, py::arg("idle_timeout") = 120.0,
        py::arg("buf_size") = 4u << 20, py::arg("splice") = true,
        "Stream a body into fd at offset (splice socket->pipe->file when possible, else recv+pwrite); "
        "returns (received, eof, error).");

  m.def("send_body",
        [](int sock, const py::bytes& head, int fd, uint64_t off, uint64_t length, std::shared_ptr<Flow> flow, int mode,
           const py::bytes& key, const std::string& amzdate, const std::string& scope, const std::string& seed,
           size_t chunk, int threads, double idle_timeout) {
          std::string h = head, k = key;
          SendResult r;
          {
            py::gil_scoped_release nogil;
            r = send_body(sock, h, fd, off, length, flow.get(), mode, k, amzdate, scope, seed, chunk, threads,
                          idle_timeout);
          }
          return py::make_tuple(r.sent, r.last_sig, r.err);
        },
        py::arg("sock"), py::arg("head"), py::arg("fd"), py::arg("offset"), py::arg("length"), py::arg("flow"),
        py::arg("mode"), py::arg("signing_key") = py::bytes(), py::arg("amzdate") = "", py::arg("scope") = "",
        py::arg("seed") = "", py::arg("chunk") = 64 << 10, py::arg("threads") = 4, py::arg("idle_timeout") = 300.0,
        "Send head + body (mode 0 plain / 1 aws-chunked); returns (payload_sent, last_signature, error).");

  m.def("recv_verify_chunked",
        [](int sock, uint64_t raw_len, const py::bytes& prefix, const py::bytes& key, const std::string& amzdate,
           const std::string& scope, const std::string& seed, bool keep, int threads, double idle_timeout) {
          std::string pre = prefix, k = key;
          VerifyResult r;
          {
            py::gil_scoped_release nogil;
            r = recv_verify_chunked(sock, raw_len, pre.data(), pre.size(), k, amzdate, scope, seed, keep, threads,
                                    idle_timeout);
          }
          return py::make_tuple(r.decoded, r.err, keep ? py::object(py::bytes(r.data)) : py::object(py::none()));
        },
        py::arg("sock"), py::arg("raw_len"), py::arg("prefix"), py::arg("signing_key"), py::arg("amzdate"),
        py::arg("scope"), py::arg("seed"), py::arg("keep") = false, py::arg("threads") = 4,
        py::arg("idle_timeout") = 300.0,
        "Receive + verify an aws-chunked body; returns (decoded_len, error, data_or_None).");

  m.def("chunked_length", &chunked_length, py::arg("length"), py::arg("chunk") = 64 << 10);
}
