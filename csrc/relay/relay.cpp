// pybind11 bindings for the native fetch -> S3 data plane (relay_core.h,
// stream.h).  A pump runs either inside the call with the GIL released
// (recv_body / send_body, for executor threads and tests) or on the native
// task pool (start_recv_body / start_send_body), reporting to a
// CompletionPort whose eventfd the event loop watches — the worker's path.
// Pumps take a stream: a `Sock` / `TlsConn` object (abortable), or a bare
// socket fd (int).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "h2.h"
#include "relay_core.h"

namespace py = pybind11;
using namespace tritondl_relay;

namespace {

// A pump's view of its `sock` argument: a Stream object, or a temporary plain
// stream over an int fd.
struct StreamArg {
  std::shared_ptr<Stream> keep;
  std::unique_ptr<PlainStream> tmp;
  Stream* s = nullptr;
};

StreamArg as_stream(const py::object& o) {
  StreamArg a;
  if (py::isinstance<Stream>(o)) {
    a.keep = o.cast<std::shared_ptr<Stream>>();
    a.s = a.keep.get();
  } else {
    a.tmp.reset(new PlainStream(o.cast<int>()));
    a.s = a.tmp.get();
  }
  return a;
}

// The same for a pump that outlives the call (start_*): always shared.
std::shared_ptr<Stream> stream_ptr(const py::object& o) {
  if (py::isinstance<Stream>(o)) return o.cast<std::shared_ptr<Stream>>();
  return std::make_shared<PlainStream>(o.cast<int>());
}

const TdlGpuChunkApi* gpu_api(const py::object& gpu) {
  if (gpu.is_none()) return nullptr;
  auto api = static_cast<const TdlGpuChunkApi*>(PyCapsule_GetPointer(gpu.ptr(), TDL_GPU_CHUNK_API_NAME));
  if (!api) throw py::error_already_set();
  if (api->version != 1) throw std::invalid_argument("unsupported GPU chunk API version");
  return api;
}

py::tuple recv_tuple(const RecvResult& r, bool chunked) {
  if (chunked) return py::make_tuple(r.received, r.eof, r.err, r.ended && !r.extra);
  return py::make_tuple(r.received, r.eof, r.err);
}

}  // namespace

PYBIND11_MODULE(_relay, m) {
  m.doc() = "tritondl native data plane: stream->file receive pump, file->stream aws-chunked/plain send pump, "
            "TLS (OpenSSL) streams";

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
      .def("covered_prefix", &Flow::covered_prefix, py::arg("start"), py::arg("end"),
           "bytes of [start, end) on disk contiguously from start")
      .def("bytes_until_covered", &Flow::bytes_until_covered, py::arg("start"), py::arg("end"))
      .def("frontiers", &Flow::frontiers, "receive frontier of every unfinished segment")
      .def("open_starts", &Flow::open_starts, "start offset of every unfinished segment")
      .def_property_readonly("cancelled", &Flow::cancelled)
      .def_property_readonly("failed", &Flow::failed)
      .def_property_readonly("finished", &Flow::finished)
      .def_property_readonly("error", &Flow::error)
      .def_property("stall", &Flow::stall, &Flow::set_stall,
                    "seconds without progress after which readers waiting for bytes give up (0 = never)")
      .def("wait_covered", [](Flow& f, uint64_t a, uint64_t b, double timeout) {
             py::gil_scoped_release nogil;
             return f.wait_covered(a, b, timeout);
           },
           py::arg("start"), py::arg("end"), py::arg("timeout"),
           "0 = on disk, 1 = failed/cancelled, 2 = timeout, 3 = download ended short, 4 = stalled");

  py::class_<Stream, std::shared_ptr<Stream>>(m, "Stream")
      .def("abort", &Stream::abort, "stop any pump running on this stream (sticky; the fd stays open)")
      .def_property_readonly("aborted", &Stream::aborted)
      .def("fileno", &Stream::fd)
      .def_property_readonly("plain", &Stream::plain);

  py::class_<PlainStream, Stream, std::shared_ptr<PlainStream>>(m, "Sock")
      .def(py::init<int>(), py::arg("fd"), "plain stream over a connected non-blocking socket (fd not owned)");

  py::class_<TlsContext, std::shared_ptr<TlsContext>>(m, "TlsContext")
      .def_static("client", &TlsContext::client, py::arg("ca_pem") = "", py::arg("ca_file") = "",
                  py::arg("verify") = true,
                  "client context: trust ca_pem / ca_file, else the system store (SSL_CERT_FILE honoured)")
      .def_static("server", &TlsContext::server, py::arg("cert_pem"), py::arg("key_pem"))
      .def_property_readonly("is_server", &TlsContext::is_server)
      .def_property_readonly("cached_sessions", &TlsContext::cached_sessions);

  py::class_<TlsStream, Stream, std::shared_ptr<TlsStream>>(m, "TlsConn")
      .def(py::init<std::shared_ptr<TlsContext>, int, const std::string&, const std::string&>(), py::arg("ctx"),
           py::arg("fd"), py::arg("server_hostname") = "", py::arg("session_key") = "")
      .def("handshake_step", [](TlsStream& t) {
             std::string err;
             const int w = t.handshake_step(&err);
             if (w < 0) throw std::runtime_error(err);
             return w;
           },
           "one non-blocking handshake step: 0 = done, else the poll events to wait for")
      .def("handshake", [](TlsStream& t, double timeout) {
             std::string err;
             {
               py::gil_scoped_release nogil;
               err = t.handshake(timeout);
             }
             if (!err.empty()) throw std::runtime_error(err);
           },
           py::arg("timeout") = 30.0)
      .def("read_nb", [](TlsStream& t, size_t n) -> py::object {
             std::string buf(n, '\0');
             short want = POLLIN;
             std::string err;
             const ssize_t r = t.recv_nb(&buf[0], n, &want, &err);
             if (r == IO_ERR) throw std::runtime_error(err);
             if (r == IO_AGAIN) return py::int_(want);
             return py::bytes(buf.data(), static_cast<size_t>(r));
           },
           py::arg("n"), "bytes (b'' = end of stream) or the poll events to wait for")
      .def("write_nb", [](TlsStream& t, const py::bytes& data) -> py::tuple {
             std::string d = data;
             if (d.empty()) return py::make_tuple(0, 0);
             struct iovec iov{&d[0], d.size()};
             short want = POLLOUT;
             std::string err;
             const ssize_t r = t.send_nb(&iov, 1, &want, &err);
             if (r == IO_ERR) throw std::runtime_error(err);
             if (r == IO_AGAIN) return py::make_tuple(0, static_cast<int>(want));
             return py::make_tuple(static_cast<int64_t>(r), 0);
           },
           py::arg("data"), "(bytes written, poll events to wait for); retry unwritten bytes unchanged")
      .def("flush_nb", [](TlsStream& t) {
             short want = POLLOUT;
             std::string err;
             if (t.flush_nb(&want, &err)) return 0;
             if (!err.empty()) throw std::runtime_error(err);
             return static_cast<int>(want);
           },
           "send buffered ciphertext: 0 = all out, else the poll events to wait for")
      .def("set_alpn", &TlsStream::set_alpn, py::arg("protocols"), "offer these ALPN protocols (before the handshake)")
      .def_property_readonly("alpn", &TlsStream::alpn, "the ALPN protocol the server selected ('' = none)")
      .def("pending", &TlsStream::pending)
      .def("alive", &TlsStream::alive)
      .def("shutdown_notify", &TlsStream::shutdown_notify)
      .def_property_readonly("version", &TlsStream::version)
      .def_property_readonly("cipher", &TlsStream::cipher)
      .def_property_readonly("resumed", &TlsStream::resumed);

  py::class_<H2Session, std::shared_ptr<H2Session>>(m, "H2Session")
      .def(py::init([](const py::object& sock, uint32_t stream_window, uint64_t conn_window, uint32_t max_frame) {
             return std::make_shared<H2Session>(stream_ptr(sock), stream_window, conn_window, max_frame);
           }),
           py::arg("sock"), py::arg("stream_window"), py::arg("conn_window"), py::arg("max_frame"),
           "HTTP/2 client session pump over a connected stream (TlsConn after an h2 ALPN handshake, or Sock); "
           "the windows and max_frame are what this side advertises")
      .def("start", &H2Session::start, "start the pump thread (it owns the stream from now on)")
      .def("fileno", &H2Session::notify_fd, "eventfd, readable while events wait to be taken")
      .def("send", [](H2Session& h, const py::bytes& frames) { h.send(std::string(frames)); }, py::arg("frames"),
           "queue frames to write, in order")
      .def("open_stream", &H2Session::open_stream, py::arg("sid"),
           "register a stream before its HEADERS are sent (its DATA is buffered until a sink is attached)")
      .def("sink_file", &H2Session::sink_file, py::arg("sid"), py::arg("fd"), py::arg("offset"), py::arg("limit"),
           py::arg("flow"), py::arg("seg") = 0, py::arg("seg_done0") = 0, py::call_guard<py::gil_scoped_release>(),
           "write the stream's body into fd at offset (at most limit bytes, < 0 = all), publishing progress on flow")
      .def("sink_events", &H2Session::sink_events, py::arg("sid"), py::call_guard<py::gil_scoped_release>(),
           "deliver the stream's body as DATA events")
      .def("drop", &H2Session::drop, py::arg("sid"), py::call_guard<py::gil_scoped_release>(),
           "stop the stream; no write into its sink happens after this returns")
      .def("written", &H2Session::written, py::arg("sid"), py::call_guard<py::gil_scoped_release>())
      .def("take_events", [](H2Session& h) {
             std::vector<H2Event> ev = h.take_events();
             py::list out;
             for (H2Event& e : ev)
               out.append(py::make_tuple(e.type, e.flags, e.sid, py::bytes(e.payload), e.n));
             return out;
           },
           "[(type, flags, sid, payload, n), ...]: frames (type < 256), or SINK_DONE (n = bytes written, flags 1 = "
           "END_STREAM), SINK_ERROR (payload = error, n = bytes written) and CONN_ERROR (payload = error)")
      .def("close", &H2Session::close, py::call_guard<py::gil_scoped_release>(),
           "stop the pump after it has written what was queued, and join it")
      .def_property_readonly("running", &H2Session::running)
      .def_property_readonly("bytes_in", &H2Session::bytes_in)
      .def_property_readonly("bytes_written", &H2Session::bytes_written)
      .def_readonly_static("SINK_DONE", &H2Session::kSinkDone)
      .def_readonly_static("SINK_ERROR", &H2Session::kSinkError)
      .def_readonly_static("CONN_ERROR", &H2Session::kConnError);

  m.def("make_test_pki", [](const std::vector<std::string>& hosts, long days) {
          TestPki p = make_test_pki(hosts, days);
          return py::make_tuple(p.ca_pem, p.cert_pem, p.key_pem);
        },
        py::arg("hosts"), py::arg("days") = 30, "throwaway EC P-256 CA + leaf for hosts: (ca_pem, cert_pem, key_pem)");

  m.def("recv_body",
        [](const py::object& sock, int fd, uint64_t off, int64_t length, const py::bytes& prefix,
           std::shared_ptr<Flow> flow, size_t seg, uint64_t seg_done0, double idle_timeout, size_t buf_size,
           bool use_splice, bool chunked) -> py::tuple {
          std::string pre = prefix;
          StreamArg io = as_stream(sock);
          RecvResult r;
          {
            py::gil_scoped_release nogil;
            r = recv_body(*io.s, fd, off, length, pre.data(), pre.size(), flow.get(), seg, seg_done0, idle_timeout,
                          buf_size, use_splice, chunked);
          }
          return recv_tuple(r, chunked);
        },
        py::arg("sock"), py::arg("fd"), py::arg("offset"), py::arg("length"), py::arg("prefix"), py::arg("flow"),
        py::arg("seg") = 0, py::arg("seg_done0") = 0, py::arg("idle_timeout") = 120.0,
        py::arg("buf_size") = 4u << 20, py::arg("splice") = true, py::arg("chunked") = false,
        "Stream a body into fd at offset (plain sockets: splice socket->pipe->file when possible, else "
        "recv+pwrite); returns (received, eof, error).  chunked=True decodes a chunked transfer coding "
        "and returns (received, eof, error, reusable).");

  m.def("send_body",
        [](const py::object& sock, const py::bytes& head, int fd, uint64_t off, uint64_t length,
           std::shared_ptr<Flow> flow, int mode, const py::bytes& key, const std::string& amzdate,
           const std::string& scope, const std::string& seed, size_t chunk, int threads, double idle_timeout,
           const py::object& gpu) {
          std::string h = head, k = key;
          StreamArg io = as_stream(sock);
          const TdlGpuChunkApi* api = gpu_api(gpu);
          SendResult r;
          {
            py::gil_scoped_release nogil;
            r = send_body(*io.s, h, fd, off, length, flow.get(), mode, k, amzdate, scope, seed, chunk, threads,
                          idle_timeout, api);
          }
          return py::make_tuple(r.sent, r.last_sig, r.err);
        },
        py::arg("sock"), py::arg("head"), py::arg("fd"), py::arg("offset"), py::arg("length"), py::arg("flow"),
        py::arg("mode"), py::arg("signing_key") = py::bytes(), py::arg("amzdate") = "", py::arg("scope") = "",
        py::arg("seed") = "", py::arg("chunk") = 64 << 10, py::arg("threads") = 4, py::arg("idle_timeout") = 300.0,
        py::arg("gpu") = py::none(),
        "Send head + body (mode 0 plain / 1 aws-chunked); returns (payload_sent, last_signature, error).  "
        "gpu: _gpu_hash.chunk_api() to hash the aws-chunked chunks on the GPU (plain sockets).");

  py::class_<CompletionPort, std::shared_ptr<CompletionPort>>(m, "CompletionPort")
      .def(py::init<>())
      .def("fileno", &CompletionPort::fd, "eventfd, readable while finished pumps wait to be reaped")
      .def_property_readonly("inflight", &CompletionPort::inflight)
      .def("wait", [](const CompletionPort& p, int timeout_ms) {
             py::gil_scoped_release nogil;
             return p.wait(timeout_ms);
           },
           py::arg("timeout_ms"))
      .def("reap", [](CompletionPort& p) {
             py::list out;
             for (const CompletionPort::Done& d : p.reap())
               out.append(py::make_tuple(d.id, d.kind == 1 ? recv_tuple(d.rr, d.chunked)
                                                           : py::make_tuple(d.sr.sent, d.sr.last_sig, d.sr.err)));
             return out;
           },
           "[(id, result), ...] of every pump finished since the last call; result as recv_body / send_body");

  m.def("start_recv_body",
        [](std::shared_ptr<CompletionPort> port, uint64_t id, const py::object& sock, int fd, uint64_t off,
           int64_t length, const py::bytes& prefix, std::shared_ptr<Flow> flow, size_t seg, uint64_t seg_done0,
           double idle_timeout, size_t buf_size, bool use_splice, bool chunked) {
          std::string pre = prefix;
          std::shared_ptr<Stream> io = stream_ptr(sock);
          start_pump(
              std::move(port), id, 1, chunked,
              [io, pre, fd, off, length, flow, seg, seg_done0, idle_timeout, buf_size, use_splice,
               chunked](CompletionPort::Done& d) {
                d.rr = recv_body(*io, fd, off, length, pre.data(), pre.size(), flow.get(), seg, seg_done0,
                                 idle_timeout, buf_size, use_splice, chunked);
              },
              "tdl-recv");
        },
        py::arg("port"), py::arg("id"), py::arg("sock"), py::arg("fd"), py::arg("offset"), py::arg("length"),
        py::arg("prefix"), py::arg("flow"), py::arg("seg") = 0, py::arg("seg_done0") = 0,
        py::arg("idle_timeout") = 120.0, py::arg("buf_size") = 4u << 20, py::arg("splice") = true,
        py::arg("chunked") = false, "recv_body on the native task pool; the result is reaped from `port`.");

  m.def("start_send_body",
        [](std::shared_ptr<CompletionPort> port, uint64_t id, const py::object& sock, const py::bytes& head, int fd,
           uint64_t off, uint64_t length, std::shared_ptr<Flow> flow, int mode, const py::bytes& key,
           const std::string& amzdate, const std::string& scope, const std::string& seed, size_t chunk, int threads,
           double idle_timeout, const py::object& gpu) {
          std::string h = head, k = key;
          std::shared_ptr<Stream> io = stream_ptr(sock);
          const TdlGpuChunkApi* api = gpu_api(gpu);
          start_pump(
              std::move(port), id, 2, false,
              [io, h, fd, off, length, flow, mode, k, amzdate, scope, seed, chunk, threads, idle_timeout,
               api](CompletionPort::Done& d) {
                d.sr = send_body(*io, h, fd, off, length, flow.get(), mode, k, amzdate, scope, seed, chunk, threads,
                                 idle_timeout, api);
              },
              "tdl-send");
        },
        py::arg("port"), py::arg("id"), py::arg("sock"), py::arg("head"), py::arg("fd"), py::arg("offset"),
        py::arg("length"), py::arg("flow"), py::arg("mode"), py::arg("signing_key") = py::bytes(),
        py::arg("amzdate") = "", py::arg("scope") = "", py::arg("seed") = "", py::arg("chunk") = 64 << 10,
        py::arg("threads") = 4, py::arg("idle_timeout") = 300.0, py::arg("gpu") = py::none(),
        "send_body on the native task pool; the result is reaped from `port`.");

  m.def("recv_verify_chunked",
        [](const py::object& sock, uint64_t raw_len, const py::bytes& prefix, const py::bytes& key,
           const std::string& amzdate, const std::string& scope, const std::string& seed, bool keep, int threads,
           double idle_timeout) {
          std::string pre = prefix, k = key;
          StreamArg io = as_stream(sock);
          VerifyResult r;
          {
            py::gil_scoped_release nogil;
            r = recv_verify_chunked(*io.s, raw_len, pre.data(), pre.size(), k, amzdate, scope, seed, keep, threads,
                                    idle_timeout);
          }
          return py::make_tuple(r.decoded, r.err, keep ? py::object(py::bytes(r.data)) : py::object(py::none()),
                                py::bytes(r.leaf_hashes));
        },
        py::arg("sock"), py::arg("raw_len"), py::arg("prefix"), py::arg("signing_key"), py::arg("amzdate"),
        py::arg("scope"), py::arg("seed"), py::arg("keep") = false, py::arg("threads") = 4,
        py::arg("idle_timeout") = 300.0,
        "Receive + verify an aws-chunked body; returns (decoded_len, error, data_or_None, leaf_hashes): "
        "leaf_hashes = the payload SHA-256s of its 64 KiB leaves, concatenated (b'' unless every frame "
        "but the last is one 64 KiB leaf).");

  m.def("recv_leaf_hashes",
        [](const py::object& sock, uint64_t len, const py::bytes& prefix, int threads, double idle_timeout) {
          std::string pre = prefix;
          StreamArg io = as_stream(sock);
          VerifyResult r;
          {
            py::gil_scoped_release nogil;
            r = recv_leaf_hashes(*io.s, len, pre.data(), pre.size(), threads, idle_timeout);
          }
          return py::make_tuple(r.decoded, r.err, py::bytes(r.leaf_hashes));
        },
        py::arg("sock"), py::arg("length"), py::arg("prefix"), py::arg("threads") = 4,
        py::arg("idle_timeout") = 300.0,
        "Receive exactly `length` body bytes; returns (received, error, leaf_hashes): the SHA-256 of every "
        "64 KiB leaf, concatenated (hashed while the body lands).");
  m.def("chunked_length", &chunked_length, py::arg("length"), py::arg("chunk") = 64 << 10);
  m.def("pool_threads", [] { return tritondl_hash::TaskPool::get().threads(); },
        "threads of this module's native task pool (chunk hashers; parked + busy)");
}
