// Host-side hashing hot paths for tritondl (C++17, pybind11, OpenSSL EVP).
//
// Replaces the native pieces the reference reaches through its dependencies
// (SURVEY.md §2.2): Go crypto/sha1 for BitTorrent piece verification
// (anacrolix/torrent, reference internal/downloader/torrent/torrent.go:79-106)
// and minio/sha256-simd + MD5 for S3 SigV4 payload hashing
// (internal/uploader/uploader.go:89).  OpenSSL dispatches to SHA-NI / AVX2
// at run time.  Every entry point that touches bulk data releases the GIL.
//
//   Hasher(kind)                  streaming md5/sha1/sha256
//   digest(kind, buffer)          one-shot
//   hash_file(path, kinds, off, len, bufsize)   one pass, several digests
//   piece_hashes(kind, buffer, piece_len, threads)   concatenated digests
//   verify_pieces(files, piece_len, expected, threads, kind) -> bytes(0/1)
//   hmac_sha256(key, msg)         SigV4 signing-key derivation
//   chunk_signatures(...)         aws-chunked streaming signature chain
//   aws_chunk_encode(...)         fused aws-chunked framing + signing
// The OpenSSL-level logic lives in hash_core.h (also used by the ASan/UBSan
// self-test, csrc/tests/native_selftest.cpp).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "hash_core.h"

namespace py = pybind11;
using namespace tritondl_hash;

namespace {

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
    MdCtx tmp(md_);  // non-destructive: digest a copy of the state
    if (EVP_MD_CTX_copy_ex(tmp.ctx, c_->ctx) != 1) throw std::runtime_error("EVP copy failed");
    return py::bytes(tmp.final());
  }
  std::string hexdigest() {
    MdCtx tmp(md_);
    if (EVP_MD_CTX_copy_ex(tmp.ctx, c_->ctx) != 1) throw std::runtime_error("EVP copy failed");
    return hex(tmp.final());
  }
  const std::string& name() const { return kind_; }

 private:
  std::string kind_;
  const EVP_MD* md_;
  std::unique_ptr<MdCtx> c_;
};

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
      size_t want = static_cast<size_t>(std::min<long long>(remaining, static_cast<long long>(buf.size())));
      size_t got = pread_full(fd, buf.data(), want, off);
      if (got == 0) break;
      for (auto& c : ctxs) c->update(buf.data(), got);
      off += static_cast<off_t>(got);
      total += static_cast<long long>(got);
      remaining -= static_cast<long long>(got);
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

py::bytes py_piece_hashes(const std::string& kind, const py::buffer& b, size_t piece_len, int threads) {
  const EVP_MD* md = md_for(kind);
  py::buffer_info bi;
  BufView v = view_of(b, bi);
  std::string out;
  {
    py::gil_scoped_release nogil;
    out = piece_hashes(md, v.ptr, v.len, piece_len, threads);
  }
  return py::bytes(out);
}

py::bytes py_verify_pieces(const std::vector<std::pair<std::string, long long>>& files, size_t piece_len,
                           const std::string& expected, int threads, const std::string& kind) {
  const EVP_MD* md = md_for(kind);
  std::string ok;
  {
    py::gil_scoped_release nogil;
    ok = verify_pieces(files, piece_len, expected, threads, md);
  }
  return py::bytes(ok);
}

std::vector<std::string> py_chunk_signatures(const std::string& key, const std::string& amzdate,
                                             const std::string& scope, const std::string& seed,
                                             const py::buffer& data, size_t chunk_size, bool include_final,
                                             int threads) {
  py::buffer_info bi;
  BufView v = view_of(data, bi);
  py::gil_scoped_release nogil;
  return chunk_signatures(key, amzdate, scope, seed, v.ptr, v.len, chunk_size, include_final, threads);
}

py::tuple py_aws_chunk_encode(const std::string& key, const std::string& amzdate, const std::string& scope,
                              const std::string& prev_sig, const py::buffer& data, size_t chunk_size,
                              bool final_chunk, int threads) {
  if (chunk_size == 0) throw std::invalid_argument("chunk_size must be > 0");
  py::buffer_info bi;
  BufView v = view_of(data, bi);
  const size_t total = aws_chunk_encoded_size(v.len, chunk_size, final_chunk);
  PyObject* out = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(total));
  if (!out) throw py::error_already_set();
  py::bytes result = py::reinterpret_steal<py::bytes>(out);
  char* dst = PyBytes_AS_STRING(out);
  std::string last;
  {
    py::gil_scoped_release nogil;
    last = aws_chunk_encode(key, amzdate, scope, prev_sig, v.ptr, v.len, chunk_size, final_chunk, dst, threads);
  }
  return py::make_tuple(result, last);
}

py::tuple py_aws_chunk_decode(const std::string& key, const std::string& amzdate, const std::string& scope,
                              const std::string& seed, const py::buffer& raw, int threads, bool want_data,
                              bool require_final) {
  py::buffer_info bi;
  BufView v = view_of(raw, bi);
  std::string decoded, err;
  {
    py::gil_scoped_release nogil;
    err = aws_chunk_decode(key, amzdate, scope, seed, v.ptr, v.len, threads, want_data ? &decoded : nullptr,
                           require_final);
  }
  if (!err.empty()) return py::make_tuple(false, py::none(), err);
  return py::make_tuple(true, want_data ? py::object(py::bytes(decoded)) : py::object(py::none()), std::string());
}

}  // namespace

PYBIND11_MODULE(_hash_host, m) {
  m.doc() = "tritondl host hashing (OpenSSL EVP, GIL-free, threaded piece verification)";
  m.def(
      "merkle_verify",
      [](const std::vector<std::pair<std::string, long long>>& files, size_t piece_len, const std::string& expected,
         const std::vector<long long>& widths, const std::vector<long long>& reals, const std::string& known,
         int threads) {
        std::string ok;
        {
          py::gil_scoped_release nogil;
          ok = merkle_verify(files, piece_len, expected, widths, reals, known, threads);
        }
        return py::bytes(ok);
      },
      py::arg("files"), py::arg("piece_len"), py::arg("expected"), py::arg("widths"), py::arg("reals"),
      py::arg("known"), py::arg("threads") = 0,
      "BEP 52 per-piece merkle verification straight from the file layout (threaded).");
  m.def(
      "merkle_check",
      [](const std::string& leaves, const std::string& leaf_ok, size_t piece_len, const std::string& expected,
         const std::vector<long long>& widths, const std::vector<long long>& reals, const std::string& known,
         int threads) {
        std::string ok;
        {
          py::gil_scoped_release nogil;
          ok = merkle_check(leaves, leaf_ok, piece_len, expected, widths, reals, known, threads);
        }
        return py::bytes(ok);
      },
      py::arg("leaves"), py::arg("leaf_ok"), py::arg("piece_len"), py::arg("expected"), py::arg("widths"),
      py::arg("reals"), py::arg("known"), py::arg("threads") = 0,
      "BEP 52 verification from precomputed 16 KiB leaf digests (e.g. the HIP kernel's).");
  py::class_<Rc4>(m, "Rc4")
      .def(py::init([](py::bytes key, size_t drop) {
             std::string k = key;
             if (k.empty()) throw std::invalid_argument("RC4 key must not be empty");
             auto* r = new Rc4(reinterpret_cast<const uint8_t*>(k.data()), k.size());
             if (drop) r->discard(drop);
             return r;
           }),
           py::arg("key"), py::arg("drop") = 1024)
      .def("crypt", [](Rc4& r, const py::buffer& b) {
        py::buffer_info bi;
        BufView v = view_of(b, bi);
        std::string out(v.len, '\0');
        {
          py::gil_scoped_release nogil;
          r.crypt(reinterpret_cast<const uint8_t*>(v.ptr), reinterpret_cast<uint8_t*>(out.data()), v.len);
        }
        return py::bytes(out);
      });
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
  m.def("piece_hashes", &py_piece_hashes, py::arg("kind"), py::arg("buffer"), py::arg("piece_len"),
        py::arg("threads") = 0);
  m.def(
      "merkle_root",
      [](const py::buffer& data, size_t width) {
        py::buffer_info bi;
        BufView v = view_of(data, bi);
        const size_t nl = (v.len + kMerkleLeaf - 1) / kMerkleLeaf;
        if (width == 0 || (width & (width - 1)) || nl > width)
          throw std::invalid_argument("width must be a power of two >= the leaf count");
        std::vector<unsigned char> row(32 * width, 0);
        {
          py::gil_scoped_release nogil;
          for (size_t k = 0; k < nl; k += 16) {  // leaves 16 at a time (sha256_batch)
            const size_t cnt = std::min<size_t>(16, nl - k);
            const void* lp[16];
            size_t ll[16];
            for (size_t j = 0; j < cnt; ++j) {
              const size_t off = (k + j) * kMerkleLeaf;
              lp[j] = v.ptr + off;
              ll[j] = std::min(kMerkleLeaf, v.len - off);
            }
            sha256_batch(lp, ll, cnt, row.data() + 32 * k);
          }
          merkle_reduce(row, width);
        }
        return py::bytes(reinterpret_cast<const char*>(row.data()), 32);
      },
      py::arg("data"), py::arg("width"),
      "BEP 52 merkle root of one piece's data: SHA-256 leaves of 16 KiB, zero-padded to `width`, reduced.");
  m.def(
      "verify_buffers",
      [](const std::string& kind, const std::vector<py::buffer>& bufs, const py::bytes& expected, int threads) {
        const EVP_MD* md = md_for(kind);
        const size_t dl = static_cast<size_t>(EVP_MD_size(md));
        const std::string exp = expected;
        if (exp.size() != dl * bufs.size()) throw std::invalid_argument("expected digest blob has wrong size");
        std::vector<py::buffer_info> keep(bufs.size());
        std::vector<BufView> v;
        v.reserve(bufs.size());
        for (size_t i = 0; i < bufs.size(); ++i) v.push_back(view_of(bufs[i], keep[i]));
        std::string ok(bufs.size(), '\0');
        {
          py::gil_scoped_release nogil;
          // groups of 16 buffers for the AVX-512 kernels, else SHA-NI pairs (md_batch)
          const size_t n = v.size(), g = md_claim(md), groups = (n + g - 1) / g;
          parallel_for(groups, static_cast<int>(std::min<size_t>(groups, threads <= 0 ? default_threads() : threads)),
                       [&](size_t k) {
                         const size_t i0 = k * g, cnt = std::min(g, n - i0);
                         const void* p[16];
                         size_t m[16];
                         for (size_t j = 0; j < cnt; ++j) {
                           p[j] = v[i0 + j].ptr;
                           m[j] = v[i0 + j].len;
                         }
                         unsigned char d[16 * EVP_MAX_MD_SIZE];
                         md_batch(md, p, m, cnt, d);
                         for (size_t j = 0; j < cnt; ++j)
                           ok[i0 + j] = std::memcmp(d + j * dl, exp.data() + (i0 + j) * dl, dl) == 0;
                       });
        }
        return py::bytes(ok);
      },
      py::arg("kind"), py::arg("buffers"), py::arg("expected"), py::arg("threads") = 0,
      "Verify in-memory pieces against concatenated digests (pairs on SHA-NI, GIL released); one byte (0/1) each.");
  m.def("verify_pieces", &py_verify_pieces, py::arg("files"), py::arg("piece_len"), py::arg("expected"),
        py::arg("threads") = 0, py::arg("kind") = "sha1");
  m.def("hmac_sha256", [](const py::bytes& k, const py::bytes& msg) { return py::bytes(hmac256(k, msg)); });
  m.def("sha_ni", &sha2x::cpu_has_sha_ni,
        "SHA-1/SHA-256 run on the two-stream SHA-NI path (False: OpenSSL; TRITONDL_SHA_NI=0 forces that)");
  m.def("sha_mb", &sha16::cpu_has_avx512,
        "batches of 16 equal-length SHA-1/SHA-256 messages run on the 16-lane AVX-512 kernels "
        "(TRITONDL_SHA_MB=0 turns them off)");
  m.def("chunk_signatures", &py_chunk_signatures, py::arg("signing_key"), py::arg("amzdate"), py::arg("scope"),
        py::arg("seed_signature"), py::arg("data"), py::arg("chunk_size"), py::arg("include_final") = true,
        py::arg("threads") = 1);
  m.def("aws_chunk_encode", &py_aws_chunk_encode, py::arg("signing_key"), py::arg("amzdate"), py::arg("scope"),
        py::arg("prev_signature"), py::arg("data"), py::arg("chunk_size"), py::arg("final") = false,
        py::arg("threads") = 1);
  m.def("default_threads", &default_threads);
  m.def("pool_threads", [] { return TaskPool::get().threads(); },
        "threads of the process-wide native task pool (parked + busy)");
  m.def("aws_chunk_decode", &py_aws_chunk_decode, py::arg("signing_key"), py::arg("amzdate"), py::arg("scope"),
        py::arg("seed_signature"), py::arg("raw"), py::arg("threads") = 1, py::arg("want_data") = true,
        py::arg("require_final") = true,
        "verify + decode an aws-chunked body -> (ok, decoded|None, error)");
}
