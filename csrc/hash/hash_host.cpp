// Host-side hashing hot paths for tritondl (C++17, pybind11, OpenSSL EVP).
//
// Replaces the native pieces the reference reaches through its dependencies
// (SURVEY.md §2.2): Go crypto/sha1 for BitTorrent piece verification
// (anacrolix/torrent, reference internal/downloader/torrent/torrent.go:79-106)
// and minio/sha256-simd + MD5 for S3 SigV4 payload hashing
// (internal/uploader/uploader.go:89).  OpenSSL dispatches to SHA-NI / AVX2
// at run time.  Every entry point releases the GIL.
//
//   Hasher(kind)                  streaming md5/sha1/sha256
//   digest(kind, buffer)          one-shot
//   hash_file(path, kinds, off, len, bufsize)   one pass, several digests
//   piece_hashes(kind, buffer, piece_len, threads)   concatenated digests
//   verify_pieces(files, piece_len, expected, threads, kind) -> bytes(0/1)
//   hmac_sha256(key, msg)         SigV4 signing-key derivation
//   chunk_signatures(...)         aws-chunked streaming signature chain
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

const EVP_MD* md_for(const std::string& kind) {
  if (kind == "sha1") return EVP_sha1();
  if (kind == "sha256") return EVP_sha256();
  if (kind == "md5") return EVP_md5();
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

std::string one_shot(const EVP_MD* md, const void* p, size_t n) {
  MdCtx c(md);
  c.update(p, n);
  return c.final();
}

struct BufView {
  const char* ptr;
  size_t len;
};

BufView view_of(const py::buffer& b, py::buffer_info& keep) {
  keep = b.request();
  if (!(keep.ndim == 1 || keep.ndim == 0) && keep.strides.size() && keep.strides.back() != keep.itemsize)
    throw std::invalid_argument("buffer must be C-contiguous");
  return {static_cast<const char*>(keep.ptr), static_cast<size_t>(keep.size * keep.itemsize)};
}

class Hasher {
 public:
  explicit Hasher(const std::string& kind) : kind_(kind), md_(md_for(kind)), c_(new MdCtx(md_)) {}
  void update(const py::buffer& b) {
    py::buffer_info bi;
    BufView v = view_of(b, bi);
    if (v.len >= 65536) {
      py::gil_scoped_release nogil;
      c_->update(v.ptr, v.len);
    } else {
      c_->update(v.ptr, v.len);
    }
  }
  py::bytes digest() {
    // non-destructive: digest a copy of the state
    MdCtx tmp(md_);
    if (EVP_MD_CTX_copy_ex(tmp.ctx, c_->ctx) != 1) throw std::runtime_error("EVP copy failed");
    return py::bytes(tmp.final());
  }
  std::string hexdigest() {
    std::string d = digest();
    static const char* hx = "0123456789abcdef";
    std::string out;
    for (unsigned char ch : d) {
      out.push_back(hx[ch >> 4]);
      out.push_back(hx[ch & 15]);
    }
    return out;
  }
  const std::string& name() const { return kind_; }

 private:
  std::string kind_;
  const EVP_MD* md_;
  std::unique_ptr<MdCtx> c_;
};

// pread that loops over short reads; returns bytes read (may be < n at EOF)
size_t pread_full(int fd, char* dst, size_t n, off_t off) {
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

py::dict hash_file(const std::string& path, const std::vector<std::string>& kinds, long long offset,
                   long long length, size_t bufsize) {
  std::vector<const EVP_MD*> mds;
  for (auto& k : kinds) mds.push_back(md_for(k));
  std::vector<std::string> outs;
  long long total = 0;
  {
    py::gil_scoped_release nogil;
    int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      int err = errno;
      py::gil_scoped_acquire g;
      errno = err;
      PyErr_SetFromErrnoWithFilename(PyExc_OSError, path.c_str());
      throw py::error_already_set();
    }
    std::vector<std::unique_ptr<MdCtx>> ctxs;
    for (auto* md : mds) ctxs.emplace_back(new MdCtx(md));
    std::vector<char> buf(std::max<size_t>(bufsize, 4096));
    off_t off = offset;
    long long remaining = length < 0 ? (1LL << 62) : length;
    while (remaining > 0) {
      size_t want = static_cast<size_t>(std::min<long long>(remaining, buf.size()));
      size_t got = pread_full(fd, buf.data(), want, off);
      if (got == 0) break;
      for (auto& c : ctxs) c->update(buf.data(), got);
      off += got;
      total += got;
      remaining -= got;
      if (got < want) break;
    }
    ::close(fd);
    for (auto& c : ctxs) outs.push_back(c->final());
  }
  py::dict d;
  for (size_t i = 0; i < kinds.size(); ++i) d[py::str(kinds[i])] = py::bytes(outs[i]);
  d["size"] = total;
  return d;
}

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  if (threads <= 1 || n <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> ts;
  int t = std::min<size_t>(threads, n);
  for (int k = 0; k < t; ++k)
    ts.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (auto& th : ts) th.join();
}

int default_threads() {
  unsigned h = std::thread::hardware_concurrency();
  return h ? static_cast<int>(std::min(h, 32u)) : 4;
}

py::bytes piece_hashes(const std::string& kind, const py::buffer& b, size_t piece_len, int threads) {
  if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  const EVP_MD* md = md_for(kind);
  py::buffer_info bi;
  BufView v = view_of(b, bi);
  size_t n = (v.len + piece_len - 1) / piece_len;
  size_t dl = EVP_MD_size(md);
  std::string out(n * dl, '\0');
  if (threads <= 0) threads = default_threads();
  {
    py::gil_scoped_release nogil;
    parallel_for(n, threads, [&](size_t i) {
      size_t off = i * piece_len;
      size_t len = std::min(piece_len, v.len - off);
      std::string d = one_shot(md, v.ptr + off, len);
      std::memcpy(&out[i * dl], d.data(), dl);
    });
  }
  return py::bytes(out);
}

struct FileSpan {
  std::string path;
  long long length;
  long long start;  // offset of this file in the torrent's concatenated stream
};

// Verify a torrent's pieces against the concatenated file layout.
// Returns one byte per piece: 1 = verified, 0 = mismatch / missing data.
py::bytes verify_pieces(const std::vector<std::pair<std::string, long long>>& files, size_t piece_len,
                        const std::string& expected, int threads, const std::string& kind) {
  const EVP_MD* md = md_for(kind);
  size_t dl = EVP_MD_size(md);
  if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  if (expected.size() % dl) throw std::invalid_argument("expected digest blob has wrong size");
  std::vector<FileSpan> spans;
  long long total = 0;
  for (auto& f : files) {
    spans.push_back({f.first, f.second, total});
    total += f.second;
  }
  size_t n = expected.size() / dl;
  size_t need = total > 0 ? (static_cast<size_t>(total) + piece_len - 1) / piece_len : 0;
  if (n != need) throw std::invalid_argument("piece count does not match total length");
  std::string ok(n, '\0');
  if (threads <= 0) threads = default_threads();
  {
    py::gil_scoped_release nogil;
    // one fd per file per thread would be wasteful; open lazily, shared (pread is thread-safe)
    std::vector<int> fds(spans.size(), -1);
    for (size_t i = 0; i < spans.size(); ++i) fds[i] = ::open(spans[i].path.c_str(), O_RDONLY | O_CLOEXEC);
    parallel_for(n, threads, [&](size_t p) {
      long long pstart = static_cast<long long>(p) * piece_len;
      long long plen = std::min<long long>(piece_len, total - pstart);
      std::vector<char> buf(static_cast<size_t>(plen));
      long long filled = 0;
      // first span overlapping pstart (binary search on start)
      size_t lo = 0, hi = spans.size();
      while (hi - lo > 1) {
        size_t mid = (lo + hi) / 2;
        if (spans[mid].start <= pstart) lo = mid; else hi = mid;
      }
      for (size_t s = lo; s < spans.size() && filled < plen; ++s) {
        long long fstart = spans[s].start, flen = spans[s].length;
        long long a = std::max(pstart + filled, fstart);
        long long e = std::min(pstart + plen, fstart + flen);
        if (e <= a) continue;
        if (a != pstart + filled) return;  // hole: cannot happen with contiguous spans
        if (fds[s] < 0) return;
        size_t want = static_cast<size_t>(e - a);
        size_t got = pread_full(fds[s], buf.data() + filled, want, static_cast<off_t>(a - fstart));
        if (got != want) return;
        filled += want;
      }
      if (filled != plen) return;
      std::string d = one_shot(md, buf.data(), buf.size());
      if (std::memcmp(d.data(), expected.data() + p * dl, dl) == 0) ok[p] = 1;
    });
    for (int fd : fds)
      if (fd >= 0) ::close(fd);
  }
  return py::bytes(ok);
}

std::string hmac256(const std::string& key, const std::string& msg) {
  unsigned char out[32];
  unsigned int len = 32;
  if (!HMAC(EVP_sha256(), key.data(), static_cast<int>(key.size()),
            reinterpret_cast<const unsigned char*>(msg.data()), msg.size(), out, &len))
    throw std::runtime_error("HMAC failed");
  return std::string(reinterpret_cast<char*>(out), len);
}

std::string hex(const std::string& d) {
  static const char* hx = "0123456789abcdef";
  std::string out;
  out.reserve(d.size() * 2);
  for (unsigned char ch : d) {
    out.push_back(hx[ch >> 4]);
    out.push_back(hx[ch & 15]);
  }
  return out;
}

// aws-chunked (STREAMING-AWS4-HMAC-SHA256-PAYLOAD) signature chain for a
// whole buffer split into chunk_size chunks (plus the final empty chunk).
// string-to-sign per chunk:
//   "AWS4-HMAC-SHA256-PAYLOAD\n" + amzdate + "\n" + scope + "\n" +
//   prev_sig + "\n" + hex(sha256("")) + "\n" + hex(sha256(chunk))
std::vector<std::string> chunk_signatures(const std::string& signing_key, const std::string& amzdate,
                                          const std::string& scope, const std::string& seed_sig,
                                          const py::buffer& data, size_t chunk_size, bool include_final) {
  py::buffer_info bi;
  BufView v = view_of(data, bi);
  std::vector<std::string> sigs;
  {
    py::gil_scoped_release nogil;
    const std::string empty_hash = hex(one_shot(EVP_sha256(), "", 0));
    std::string prev = seed_sig;
    size_t off = 0;
    while (true) {
      size_t len = std::min(chunk_size, v.len - off);
      std::string h = hex(one_shot(EVP_sha256(), v.ptr + off, len));
      std::string sts = "AWS4-HMAC-SHA256-PAYLOAD\n" + amzdate + "\n" + scope + "\n" + prev + "\n" +
                        empty_hash + "\n" + h;
      prev = hex(hmac256(signing_key, sts));
      sigs.push_back(prev);
      off += len;
      if (len == 0) break;
      if (off >= v.len && !include_final) break;
    }
  }
  return sigs;
}

// Fused aws-chunked encoder: for every chunk, SHA-256 it (while it is hot in
// cache), chain the HMAC signature and copy it behind its
// "<hex>;chunk-signature=<sig>\r\n" header into ONE pre-sized output buffer.
// Replaces a Python loop of slices/concats that cost ~2.5x the hashing.
py::tuple aws_chunk_encode(const std::string& signing_key, const std::string& amzdate, const std::string& scope,
                           const std::string& prev_sig, const py::buffer& data, size_t chunk_size, bool final_chunk) {
  if (chunk_size == 0) throw std::invalid_argument("chunk_size must be > 0");
  py::buffer_info bi;
  BufView v = view_of(data, bi);
  auto hexlen = [](size_t n) {
    size_t l = 1;
    while (n >>= 4) ++l;
    return l;
  };
  const size_t sig_part = 17 + 64 + 2;  // ";chunk-signature=" + sig + CRLF
  size_t total = 0;
  for (size_t off = 0; off < v.len; off += chunk_size) {
    size_t n = std::min(chunk_size, v.len - off);
    total += hexlen(n) + sig_part + n + 2;
  }
  if (final_chunk) total += 1 + sig_part + 2;
  PyObject* out = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(total));
  if (!out) throw py::error_already_set();
  py::bytes result = py::reinterpret_steal<py::bytes>(out);
  char* dst = PyBytes_AS_STRING(out);
  std::string prev = prev_sig;
  {
    py::gil_scoped_release nogil;
    const std::string empty_hash = hex(one_shot(EVP_sha256(), "", 0));
    const std::string head = "AWS4-HMAC-SHA256-PAYLOAD\n" + amzdate + "\n" + scope + "\n";
    size_t w = 0;
    auto emit = [&](const char* p, size_t n) {
      std::string h = hex(one_shot(EVP_sha256(), p, n));
      prev = hex(hmac256(signing_key, head + prev + "\n" + empty_hash + "\n" + h));
      char hx[32];
      int hl = snprintf(hx, sizeof hx, "%zx", n);
      std::memcpy(dst + w, hx, hl);
      w += hl;
      std::memcpy(dst + w, ";chunk-signature=", 17);
      w += 17;
      std::memcpy(dst + w, prev.data(), 64);
      w += 64;
      dst[w++] = '\r';
      dst[w++] = '\n';
      if (n) {
        std::memcpy(dst + w, p, n);
        w += n;
      }
      dst[w++] = '\r';
      dst[w++] = '\n';
    };
    for (size_t off = 0; off < v.len; off += chunk_size) emit(v.ptr + off, std::min(chunk_size, v.len - off));
    if (final_chunk) emit(nullptr, 0);
  }
  return py::make_tuple(result, prev);
}

}  // namespace

PYBIND11_MODULE(_hash_host, m) {
  m.doc() = "tritondl host hashing (OpenSSL EVP, GIL-free, threaded piece verification)";
  py::class_<Hasher>(m, "Hasher")
      .def(py::init<const std::string&>())
      .def("update", &Hasher::update)
      .def("digest", &Hasher::digest)
      .def("hexdigest", &Hasher::hexdigest)
      .def_property_readonly("name", &Hasher::name);
  m.def("digest", [](const std::string& kind, const py::buffer& b) {
    py::buffer_info bi;
    BufView v = view_of(b, bi);
    const EVP_MD* md = md_for(kind);
    std::string d;
    {
      py::gil_scoped_release nogil;
      d = one_shot(md, v.ptr, v.len);
    }
    return py::bytes(d);
  });
  m.def("hash_file", &hash_file, py::arg("path"), py::arg("kinds"), py::arg("offset") = 0,
        py::arg("length") = -1, py::arg("bufsize") = 1 << 20);
  m.def("piece_hashes", &piece_hashes, py::arg("kind"), py::arg("buffer"), py::arg("piece_len"),
        py::arg("threads") = 0);
  m.def("verify_pieces", &verify_pieces, py::arg("files"), py::arg("piece_len"), py::arg("expected"),
        py::arg("threads") = 0, py::arg("kind") = "sha1");
  m.def("hmac_sha256", [](const py::bytes& k, const py::bytes& msg) { return py::bytes(hmac256(k, msg)); });
  m.def("chunk_signatures", &chunk_signatures, py::arg("signing_key"), py::arg("amzdate"), py::arg("scope"),
        py::arg("seed_signature"), py::arg("data"), py::arg("chunk_size"), py::arg("include_final") = true);
  m.def("default_threads", &default_threads);
  m.def("aws_chunk_encode", &aws_chunk_encode, py::arg("signing_key"), py::arg("amzdate"), py::arg("scope"),
        py::arg("prev_signature"), py::arg("data"), py::arg("chunk_size"), py::arg("final") = false);
}
