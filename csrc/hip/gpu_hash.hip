// Batched piece hashing on MI355X (gfx950 / CDNA4) — tritondl's GPU offload.
//
// What it accelerates: BitTorrent piece (re)verification — SURVEY.md §2.2 and
// §5.4: anacrolix/torrent re-verifies every piece of a redelivered job's
// existing data against the info-dict SHA-1s before resuming (reference
// internal/downloader/torrent/torrent.go:40-41,79-106 uses that storage).
// Also SHA-256 for BEP-52 style 16 KiB leaves and S3 multipart part checksums.
//
// Execution model (CDNA4-first, not a CUDA translation):
//  * SHA-1/SHA-256 chains are strictly serial inside one message, so the
//    parallel axis is the PIECE: one 64-wide wavefront hashes 64 pieces, one
//    lane per piece, 64-thread workgroups so that small batches still spread
//    one wave per SIMD across the 256 CUs (8 XCDs) instead of stacking.
//  * The kernel is VALU-bound (~700 int ops / 64 B block): rounds are fully
//    unrolled so the 16-word message window lives in VGPRs; rotates lower to
//    v_alignbit_b32, xor3/Ch/Maj to ONE gfx950 v_bitop3_b32 each, byte swaps
//    to v_perm_b32.
//  * Loads are 4 x dwordx4 per 64-byte block per lane, and the NEXT block is
//    prefetched into registers before compressing the current one so HBM
//    latency hides under ~1.5k cycles of ALU work.  Lanes stride by
//    piece_len, so each wave-load touches 64 lines; every line is consumed in
//    full by two consecutive blocks while it is still L2-resident.
//  * Host side: runs whose bytes sit in one fully present, page-cache
//    resident file are DMA'd to HBM straight from the file's page cache: the
//    read-only file mapping is registered with hipHostRegister in 256 MiB
//    blocks (~2-7 ms per GiB, then 57.6 GB/s, the same as from pinned
//    memory; profiles/r03_reg_probe).  Everything else (cold pages, runs
//    straddling files, BEP 47 padding, short files) goes through a ring of
//    pinned staging slots filled by a pread() reader pool.
//  * Hybrid mode (cpu_threads > 0): the whole job is host->HBM bound
//    (~45 GB/s of page-cache copies + PCIe), so the CPU's SHA-NI threads
//    verify pieces from the BACK of the layout while the GPU pipeline claims
//    staging chunks from the FRONT; they meet wherever the two rates put the
//    boundary (no static split to mis-calibrate).  The GPU stops claiming
//    once the CPU could finish the rest faster than one more kernel's
//    per-lane latency, so the last window's kernel overlaps CPU work.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../hash/gpu_chunk_api.h"
#include "../hash/hash_core.h"  // OpenSSL SHA-NI path for the CPU half of hybrid verification

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace py = pybind11;

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw std::runtime_error(std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

// ------------------------------------------------------------------ device

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return __builtin_rotateright32(x, n); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// gfx950 v_bitop3_b32: any 3-input bitwise function in ONE VALU op (truth table
// over S0=0xF0, S1=0xCC, S2=0xAA).  hipcc does not fuse xor chains / Ch / Maj
// into it on its own (measured: 292 v_xor_b32 per SHA-1 block before).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch3(uint32_t x, uint32_t y, uint32_t z) {  // (x&y)|(~x&z)
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0xCA);
}
__device__ __forceinline__ uint32_t maj3(uint32_t x, uint32_t y, uint32_t z) {  // majority
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0xE8);
}

__device__ __forceinline__ void sha1_compress(uint32_t h[5], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      wt = rotl32(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
      w[t & 15] = wt;
    }
    uint32_t f, k;
    if (t < 20) {
      f = ch3(b, c, d);
      k = 0x5A827999u;
    } else if (t < 40) {
      f = xor3(b, c, d);
      k = 0x6ED9EBA1u;
    } else if (t < 60) {
      f = maj3(b, c, d);
      k = 0x8F1BBCDCu;
    } else {
      f = xor3(b, c, d);
      k = 0xCA62C1D6u;
    }
    uint32_t tmp = rotl32(a, 5) + f + e + k + wt;
    e = d;
    d = c;
    c = rotl32(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
}

__device__ __forceinline__ void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      uint32_t s0 = xor3(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    uint32_t ch = ch3(e, f, g);
    uint32_t t1 = hh + S1 + ch + K[t] + wt;
    uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    uint32_t maj = maj3(a, b, c);
    uint32_t t2 = S0 + maj;
    hh = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + t2;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
  h[5] += f;
  h[6] += g;
  h[7] += hh;
}

template <int ALG>
struct Alg;
template <>
struct Alg<1> {
  static constexpr int kWords = 5;
  __device__ static void init(uint32_t* h) {
    h[0] = 0x67452301u; h[1] = 0xEFCDAB89u; h[2] = 0x98BADCFEu; h[3] = 0x10325476u; h[4] = 0xC3D2E1F0u;
  }
  __device__ static void compress(uint32_t* h, uint32_t* w) { sha1_compress(h, w); }
};
template <>
struct Alg<256> {
  static constexpr int kWords = 8;
  __device__ static void init(uint32_t* h) {
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
  }
  __device__ static void compress(uint32_t* h, uint32_t* w) { sha256_compress(h, w); }
};

__device__ __forceinline__ void words_from_uint4(uint32_t w[16], const uint4& q0, const uint4& q1,
                                                 const uint4& q2, const uint4& q3) {
  w[0] = bswap32(q0.x); w[1] = bswap32(q0.y); w[2] = bswap32(q0.z); w[3] = bswap32(q0.w);
  w[4] = bswap32(q1.x); w[5] = bswap32(q1.y); w[6] = bswap32(q1.z); w[7] = bswap32(q1.w);
  w[8] = bswap32(q2.x); w[9] = bswap32(q2.y); w[10] = bswap32(q2.z); w[11] = bswap32(q2.w);
  w[12] = bswap32(q3.x); w[13] = bswap32(q3.y); w[14] = bswap32(q3.z); w[15] = bswap32(q3.w);
}

// One lane = one piece.  VEC requires piece_len % 16 == 0 and a 16-B aligned base.
template <int ALG, bool VEC>
__global__ __launch_bounds__(64) void hash_pieces_kernel(const uint8_t* __restrict__ data, uint64_t total,
                                                         uint64_t piece_len, uint32_t n_pieces,
                                                         uint32_t* __restrict__ out) {
  using A = Alg<ALG>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // blockDim = lanes per wave (16/32/64)
  if (i >= n_pieces) return;
  const uint64_t start = static_cast<uint64_t>(i) * piece_len;
  const uint64_t len = min(piece_len, total - start);
  const uint8_t* p = data + start;
  const uint64_t nfull = len >> 6;
  uint32_t h[A::kWords];
  A::init(h);
  uint32_t w[16];
  if (VEC) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    if (nfull) {
      uint4 c0 = q[0], c1 = q[1], c2 = q[2], c3 = q[3];
      for (uint64_t b = 0; b < nfull; ++b) {
        words_from_uint4(w, c0, c1, c2, c3);
        if (b + 1 < nfull) {  // prefetch next block; consumed next iteration
          const uint4* nq = q + 4 * (b + 1);
          c0 = nq[0]; c1 = nq[1]; c2 = nq[2]; c3 = nq[3];
        }
        A::compress(h, w);
      }
    }
  } else {
    for (uint64_t b = 0; b < nfull; ++b) {
      const uint8_t* blk = p + 64 * b;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        w[j] = (uint32_t(blk[4 * j]) << 24) | (uint32_t(blk[4 * j + 1]) << 16) |
               (uint32_t(blk[4 * j + 2]) << 8) | uint32_t(blk[4 * j + 3]);
      A::compress(h, w);
    }
  }
  // tail + Merkle–Damgård padding (one or two blocks)
  const uint32_t rem = static_cast<uint32_t>(len & 63);
  const uint8_t* tail = p + (nfull << 6);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t pos = 4 * j + k;
      const uint32_t byte = pos < rem ? uint32_t(tail[pos]) : (pos == rem ? 0x80u : 0u);
      word = (word << 8) | byte;
    }
    w[j] = word;
  }
  const uint64_t bits = len << 3;
  if (rem < 56) {
    w[14] = static_cast<uint32_t>(bits >> 32);
    w[15] = static_cast<uint32_t>(bits);
    A::compress(h, w);
  } else {
    A::compress(h, w);
#pragma unroll
    for (int j = 0; j < 14; ++j) w[j] = 0;
    w[14] = static_cast<uint32_t>(bits >> 32);
    w[15] = static_cast<uint32_t>(bits);
    A::compress(h, w);
  }
  uint32_t* o = out + static_cast<uint64_t>(i) * A::kWords;
#pragma unroll
  for (int k = 0; k < A::kWords; ++k) o[k] = bswap32(h[k]);  // digest bytes in memory order
}

// ------------------------------------------------------------------ host

namespace {

int alg_id(const std::string& kind) {
  if (kind == "sha1") return 1;
  if (kind == "sha256") return 256;
  throw std::invalid_argument("gpu hash supports sha1|sha256, got " + kind);
}
int digest_len(int alg) { return alg == 1 ? 20 : 32; }

void launch_hash(int alg, const uint8_t* d_data, uint64_t total, uint64_t piece_len, uint32_t n,
                 uint32_t* d_out, hipStream_t s, int lanes = 64) {
  if (n == 0) return;
  if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
  if ((static_cast<uint64_t>(n) - 1) * piece_len >= total && total > 0)
    throw std::invalid_argument("n_pieces exceeds data length");
  const bool vec = (piece_len % 16 == 0) && (reinterpret_cast<uintptr_t>(d_data) % 16 == 0);
  if (lanes != 16 && lanes != 32 && lanes != 64) throw std::invalid_argument("lanes must be 16, 32 or 64");
  const uint32_t L = static_cast<uint32_t>(lanes);
  dim3 grid((n + L - 1) / L), block(L);
  if (alg == 1) {
    if (vec) hash_pieces_kernel<1, true><<<grid, block, 0, s>>>(d_data, total, piece_len, n, d_out);
    else hash_pieces_kernel<1, false><<<grid, block, 0, s>>>(d_data, total, piece_len, n, d_out);
  } else {
    if (vec) hash_pieces_kernel<256, true><<<grid, block, 0, s>>>(d_data, total, piece_len, n, d_out);
    else hash_pieces_kernel<256, false><<<grid, block, 0, s>>>(d_data, total, piece_len, n, d_out);
  }
  HIP_CHECK(hipGetLastError());
}

size_t pread_full(int fd, uint8_t* dst, size_t n, off_t off) {
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

struct Span {
  int fd;  // kZeroSpan: a BEP 47 padding file (all zeros, never on disk)
  long long start, length;
};
constexpr int kZeroSpan = -2;

// Counts down the units of one staging fill; the first reader exception wins.
struct Latch {
  explicit Latch(size_t n) : left(n) {}
  void done(std::exception_ptr e) {
    std::lock_guard<std::mutex> g(m);
    if (e && !err) err = e;
    if (--left == 0) cv.notify_all();
  }
  void wait_quiet() {
    std::unique_lock<std::mutex> g(m);
    cv.wait(g, [&] { return left == 0; });
  }
  void wait() {
    wait_quiet();
    if (err) std::rethrow_exception(err);
  }
  std::mutex m;
  std::condition_variable cv;
  size_t left;
  std::exception_ptr err;
};

// Persistent pread/memcpy threads.  Fills of several staging slots are queued
// back to back, so readers move straight on to slot k+1 while the DMA engine
// drains slot k (the previous design spawned threads per slot and had every
// reader wait at a per-slot barrier).
class ReaderPool {
 public:
  explicit ReaderPool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] {
      tritondl_hash::name_thread("tdl-gpu-read");
      loop();
    });
  }
  ~ReaderPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
};

// Page cache -> HBM with no CPU copy.  A run of pieces that lies inside one
// file that is fully present and resident in the page cache is copied by the
// DMA engine straight from the file's read-only mapping, registered with
// hipHostRegister in kBlock-sized blocks (256 MiB; a run may span two; each copy
// stays inside one registration).  Blocks are reference-counted by the HBM
// windows whose copies use them and unregistered once those windows are
// hashed, so at most about two windows' worth of page cache is pinned.
// TRITONDL_GPU_DIRECT=0 turns it off (everything through pinned staging).
class DirectSource {
 public:
  explicit DirectSource(const std::vector<Span>& spans) : spans_(spans), maps_(spans.size()) {
    const char* env = std::getenv("TRITONDL_GPU_DIRECT");
    on_ = !(env && (env[0] == '0' || env[0] == 'n' || env[0] == 'o'));
    const long pg = ::sysconf(_SC_PAGESIZE);
    page_ = pg > 0 ? static_cast<size_t>(pg) : 4096;
    const char* mb = std::getenv("TRITONDL_GPU_DIRECT_BLOCK_MB");
    if (mb && std::atol(mb) > 0) kBlock = static_cast<size_t>(std::atol(mb)) << 20;
    const char* keep = std::getenv("TRITONDL_GPU_DIRECT_KEEP");
    keep_ = keep && keep[0] == '1';
  }
  ~DirectSource() { release_all(); }
  DirectSource(const DirectSource&) = delete;
  DirectSource& operator=(const DirectSource&) = delete;

  bool on() const { return on_; }
  size_t bytes() const { return bytes_; }

  // Can layout bytes [off, off+len) go direct?  Registers the blocks they
  // need; false leaves the run to the staging path.
  bool prepare(size_t off, size_t len) {
    if (!on_ || len == 0) return false;
    const int i = span_of(off, len);
    if (i < 0) return false;
    Map& m = mapping(i);
    if (!m.base) return false;
    const size_t fo = off - static_cast<size_t>(spans_[i].start);
    const size_t a = fo / page_ * page_;
    const size_t np = (fo + len - a + page_ - 1) / page_;
    resident_.resize(np);
    if (::mincore(m.base + a, np * page_, resident_.data()) != 0) return false;
    for (unsigned char r : resident_)
      if (!(r & 1)) return false;  // cold pages: parallel preads beat one faulting thread
    for (size_t b = fo / kBlock; b <= (fo + len - 1) / kBlock; ++b) {
      const uint64_t key = (static_cast<uint64_t>(i) << 32) | b;
      if (regs_.count(key)) continue;
      uint8_t* p = m.base + b * kBlock;
      const size_t rl = std::min(kBlock, m.len - b * kBlock);
      if (hipHostRegister(p, rl, hipHostRegisterReadOnly) != hipSuccess) {
        (void)hipGetLastError();
        on_ = false;  // not supported here: stop trying for this call
        return false;
      }
      regs_.emplace(key, Reg{p, 0});
    }
    return true;
  }

  // Enqueue the H2D copies of a prepared run on `s`; `used` collects the
  // blocks the copies read (released by unref once they completed).
  void enqueue(uint8_t* dst, size_t off, size_t len, hipStream_t s, std::vector<uint64_t>& used) {
    const int i = span_of(off, len);
    const Map& m = maps_[i];
    const size_t fo = off - static_cast<size_t>(spans_[i].start);
    for (size_t b = fo / kBlock; b <= (fo + len - 1) / kBlock; ++b) {
      const size_t sa = std::max(fo, b * kBlock), se = std::min(fo + len, (b + 1) * kBlock);
      const uint64_t key = (static_cast<uint64_t>(i) << 32) | b;
      HIP_CHECK(hipMemcpyAsync(dst + (sa - fo), m.base + sa, se - sa, hipMemcpyHostToDevice, s));
      ++regs_.at(key).refs;
      used.push_back(key);
    }
    bytes_ += len;
  }

  // The copies that used these blocks have completed.
  void unref(std::vector<uint64_t>& used) {
    if (keep_) {  // unregister everything at the end of the call instead
      used.clear();
      return;
    }
    for (uint64_t key : used) {
      auto it = regs_.find(key);
      if (it == regs_.end()) continue;
      if (--it->second.refs <= 0) {
        (void)hipHostUnregister(it->second.p);
        regs_.erase(it);
      }
    }
    used.clear();
  }

  // Every copy has completed (or the streams were synchronised after an error).
  void release_all() {
    for (auto& kv : regs_) (void)hipHostUnregister(kv.second.p);
    regs_.clear();
    for (auto& m : maps_)
      if (m.base) ::munmap(m.base, m.len);
    maps_.assign(maps_.size(), Map{});
  }

 private:
  struct Map {
    uint8_t* base = nullptr;
    size_t len = 0;  // mapped bytes (file length rounded up to a page)
    bool tried = false;
  };
  struct Reg {
    uint8_t* p;
    int refs;
  };
  int span_of(size_t off, size_t len) const {
    for (size_t k = 0; k < spans_.size(); ++k) {
      const Span& sp = spans_[k];
      const size_t a = static_cast<size_t>(sp.start), e = a + static_cast<size_t>(sp.length);
      if (off >= a && off < e) return (sp.fd >= 0 && off + len <= e) ? static_cast<int>(k) : -1;
    }
    return -1;
  }
  Map& mapping(int i) {
    Map& m = maps_[i];
    if (m.tried) return m;
    m.tried = true;
    const Span& sp = spans_[i];
    struct stat st {};
    if (sp.length <= 0 || ::fstat(sp.fd, &st) != 0 || st.st_size < sp.length) return m;  // short file: staging
    const size_t len = (static_cast<size_t>(sp.length) + page_ - 1) / page_ * page_;
    void* p = ::mmap(nullptr, len, PROT_READ, MAP_SHARED, sp.fd, 0);
    if (p == MAP_FAILED) return m;
    m.base = static_cast<uint8_t*>(p);
    m.len = len;
    return m;
  }
  size_t kBlock = 256u << 20;  // TRITONDL_GPU_DIRECT_BLOCK_MB; 64-1024 measured alike (profiles/r03_direct_knobs)
  bool keep_ = false;
  const std::vector<Span>& spans_;
  std::vector<Map> maps_;
  std::map<uint64_t, Reg> regs_;
  std::vector<unsigned char> resident_;
  size_t page_ = 4096;
  size_t bytes_ = 0;
  bool on_ = true;
};

// Host pipeline: disk / host memory -> pinned staging (a ring of kStages
// slots filled by the reader pool, up to kStages-1 ahead of the DMA) -> HBM
// window -> ONE kernel over every piece of the window -> digests.
//
// Why windows: the kernel's parallel axis is the piece (one lane each), so a
// 256 MiB batch of 1 MiB pieces is only 256 lanes (4 waves on a 256-CU chip).
// Accumulating the copies into a multi-GB HBM window (MI355X: 288 GB) first
// gives the launch thousands of lanes; two windows alternate so the copies of
// window k+1 (copy stream) overlap the kernel of window k (compute stream),
// and the pinned staging slots are recycled as soon as their H2D completes.
class GpuHasher {
 public:
  GpuHasher(int device, size_t stage_bytes, int reader_threads, size_t window_bytes, size_t max_hbm = 0)
      : device_(device),
        stage_req_(std::max<size_t>(stage_bytes, 1 << 20)),
        readers_(std::max(1, reader_threads)),
        window_req_(window_bytes),
        max_hbm_(max_hbm ? max_hbm : kDefaultMaxHbm),
        pool_(new ReaderPool(std::max(1, reader_threads))) {
    HIP_CHECK(hipSetDevice(device_));
    HIP_CHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&compute_stream_, hipStreamNonBlocking));
    for (auto& st : stage_) HIP_CHECK(hipEventCreateWithFlags(&st.free_ev, hipEventDisableTiming));
    for (auto& w : win_) {
      HIP_CHECK(hipEventCreateWithFlags(&w.copied, hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&w.done, hipEventDisableTiming));
    }
  }
  ~GpuHasher() {
    pool_.reset();
    hipSetDevice(device_);
    hipStreamSynchronize(copy_stream_);
    hipStreamSynchronize(compute_stream_);
    release();
    for (auto& st : stage_) hipEventDestroy(st.free_ev);
    for (auto& w : win_) {
      hipEventDestroy(w.copied);
      hipEventDestroy(w.done);
    }
    hipStreamDestroy(copy_stream_);
    hipStreamDestroy(compute_stream_);
  }

  // Free cached staging / window memory, from Python: waits for a running
  // call (GIL released while waiting; the call's thread re-takes the GIL).
  void release_py() {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(call_mu_);
    hipSetDevice(device_);
    release();
  }

  // The idle reaper: free everything if nothing ran for idle_s seconds and no
  // call is running.  True if memory was freed.
  bool release_if_idle(double idle_s) {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> g(call_mu_, std::try_to_lock);
    if (!g.owns_lock() || held_bytes_locked() == 0) return false;
    const double idle = std::chrono::duration<double>(std::chrono::steady_clock::now() - last_use_).count();
    if (idle < idle_s) return false;
    hipSetDevice(device_);
    release();
    return true;
  }

  // (device bytes, pinned host bytes) held between calls.
  std::pair<size_t, size_t> held_bytes() {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> g(call_mu_);
    size_t dev = 0, host = 0;
    held_split_locked(&dev, &host);
    return {dev, host};
  }
  size_t max_hbm() const { return max_hbm_; }

  // Free cached staging / window memory (caller holds call_mu_ or is the destructor).
  void release() {
    for (auto& st : stage_) {
      if (st.h) hipHostFree(st.h);
      st.h = nullptr;
      st.cap = 0;
      st.used = false;
    }
    for (auto& w : win_) {
      if (w.d) hipFree(w.d);
      if (w.d_out) hipFree(w.d_out);
      if (w.h_out) hipHostFree(w.h_out);
      w.d = nullptr;
      w.d_out = nullptr;
      w.h_out = nullptr;
      w.cap = w.out_cap = 0;
      w.pending = false;
    }
  }

  // Hash a contiguous host buffer into concatenated digests.
  py::bytes hash_buffer(const std::string& kind, const py::buffer& buf, size_t piece_len) {
    const int alg = alg_id(kind);
    py::buffer_info bi = buf.request();
    const uint8_t* src = static_cast<const uint8_t*>(bi.ptr);
    const size_t total = static_cast<size_t>(bi.size * bi.itemsize);
    if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
    const size_t n = (total + piece_len - 1) / piece_len;
    const int dl = digest_len(alg);
    std::string out(n * dl, '\0');
    {
      py::gil_scoped_release nogil;
      CallGuard cg(this);
      run_gpu_only(alg, piece_len, total, n, [&](uint8_t* dst, size_t off, size_t len, char*) {
        std::memcpy(dst, src + off, len);
      }, [&](size_t first, size_t count, const uint8_t* digests, const std::vector<char>&) {
        std::memcpy(&out[first * dl], digests, count * dl);
      });
    }
    return py::bytes(out);
  }

  // Open a layout's files; spans carry stream offsets (kZeroSpan = padding).
  static std::vector<Span> open_spans(const std::vector<std::pair<std::string, long long>>& files, long long& total) {
    std::vector<Span> spans;
    total = 0;
    for (auto& f : files) {
      if (f.second < 0) {
        close_spans(spans);
        throw std::invalid_argument("negative file length");
      }
      spans.push_back({f.first.empty() ? kZeroSpan : ::open(f.first.c_str(), O_RDONLY | O_CLOEXEC), total, f.second});
      total += f.second;
    }
    return spans;
  }
  static void close_spans(std::vector<Span>& spans) {
    for (auto& s : spans)
      if (s.fd >= 0) ::close(s.fd);
    spans.clear();
  }

  // (digests, complete) of every piece of a layout: GPU only, or hybrid with
  // cpu_threads SHA-NI threads working from the other end.
  void layout_digests(int alg, std::vector<Span>& spans, size_t piece_len, size_t total, size_t n, int cpu_threads,
                      std::string& digests, std::string& complete) {
    const int dl = digest_len(alg);
    digests.assign(n * dl, '\0');
    complete.assign(n, '\0');
    py::gil_scoped_release nogil;
    CallGuard cg(this);
    try {
      DirectSource ds(spans);  // unmapped before the spans' fds close
      if (cpu_threads > 0) {
        hybrid_digest(alg, spans, piece_len, total, n, cpu_threads, digests, complete, &ds);
      } else {
        run_gpu_only(alg, piece_len, total, n,
                     [&](uint8_t* dst, size_t off, size_t len, char* comp) { read_unit(spans, dst, off, len, piece_len, comp); },
                     [&](size_t first, size_t count, const uint8_t* d, const std::vector<char>& comp) {
                       std::memcpy(&digests[first * dl], d, count * dl);
                       for (size_t k = 0; k < count; ++k) complete[first + k] = comp[k];
                     },
                     &ds);
        last_gpu_pieces_ = n;
      }
      last_direct_bytes_ = ds.bytes();
    } catch (...) {
      close_spans(spans);
      throw;
    }
    close_spans(spans);
  }

  // Verify a torrent's concatenated file layout against expected digests.
  py::bytes verify_files(const std::vector<std::pair<std::string, long long>>& files, size_t piece_len,
                         const std::string& expected, const std::string& kind, int cpu_threads) {
    const int alg = alg_id(kind);
    const int dl = digest_len(alg);
    if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
    if (expected.size() % dl) throw std::invalid_argument("expected digest blob has wrong size");
    long long total = 0;
    std::vector<Span> spans = open_spans(files, total);
    const size_t n = expected.size() / dl;
    const size_t need = total > 0 ? (static_cast<size_t>(total) + piece_len - 1) / piece_len : 0;
    if (n != need) {
      close_spans(spans);
      throw std::invalid_argument("piece count does not match total length");
    }
    std::string digests, complete;
    layout_digests(alg, spans, piece_len, static_cast<size_t>(total), n, cpu_threads, digests, complete);
    std::string ok(n, '\0');
    for (size_t k = 0; k < n; ++k)
      ok[k] = complete[k] && std::memcmp(digests.data() + k * dl, expected.data() + k * dl, dl) == 0;
    return py::bytes(ok);
  }

  // All piece digests of a file layout plus a per-piece "fully read" mask —
  // used at 16 KiB "pieces" for BitTorrent v2 merkle leaves (host reduces).
  py::tuple digest_files(const std::vector<std::pair<std::string, long long>>& files, size_t piece_len,
                         const std::string& kind, int cpu_threads) {
    const int alg = alg_id(kind);
    if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
    long long total = 0;
    std::vector<Span> spans = open_spans(files, total);
    const size_t n = total > 0 ? (static_cast<size_t>(total) + piece_len - 1) / piece_len : 0;
    std::string digests, complete;
    layout_digests(alg, spans, piece_len, static_cast<size_t>(total), n, cpu_threads, digests, complete);
    return py::make_tuple(py::bytes(digests), py::bytes(complete));
  }

  size_t batch_bytes() const { return stage_req_; }
  size_t last_window_bytes() const { return last_window_; }
  size_t window_bytes_for(size_t total, size_t piece_len) {
    size_t budget = window_req_;
    if (budget == 0) {
      // two windows live at once: each gets half the cap (TRITONDL_GPU_MAX_HBM,
      // default 8 GiB) and at most a third of free HBM, so a co-located ingest
      // worker never takes a big share of a GPU that serves other workloads
      size_t free_b = 0, tot_b = 0;
      if (hipMemGetInfo(&free_b, &tot_b) != hipSuccess) free_b = 8ull << 30;
      budget = std::min<size_t>(free_b / 3, max_hbm_ / 2);
    }
    const size_t aligned = (total + piece_len - 1) / piece_len * piece_len;
    const size_t per = std::max<size_t>(1, budget / piece_len) * piece_len;
    return std::max(piece_len, std::min(aligned, per));
  }

 private:
  static constexpr int kStages = 4;
  static constexpr size_t kDefaultMaxHbm = 8ull << 30;

  // Serialises the public calls with the idle reaper (which frees the
  // staging and windows those calls use) and stamps the last use.
  struct CallGuard {
    GpuHasher* h;
    std::lock_guard<std::mutex> g;
    explicit CallGuard(GpuHasher* x) : h(x), g(x->call_mu_) {}
    ~CallGuard() { h->last_use_ = std::chrono::steady_clock::now(); }
  };
  void held_split_locked(size_t* dev, size_t* host) const {
    for (const auto& st : stage_) *host += st.h ? st.cap : 0;
    for (const auto& w : win_) {
      *dev += (w.d ? w.cap : 0) + (w.d_out ? w.out_cap : 0);
      *host += w.h_out ? w.out_cap : 0;
    }
  }
  size_t held_bytes_locked() const {
    size_t dev = 0, host = 0;
    held_split_locked(&dev, &host);
    return dev + host;
  }
  struct Stage {
    uint8_t* h = nullptr;
    size_t cap = 0;
    hipEvent_t free_ev = nullptr;
    bool used = false;
  };
  struct Window {
    uint8_t* d = nullptr;
    size_t cap = 0;
    uint32_t* d_out = nullptr;
    uint8_t* h_out = nullptr;
    size_t out_cap = 0;
    hipEvent_t copied = nullptr, done = nullptr;
    bool pending = false;
    size_t first = 0, count = 0;
    std::vector<char> complete;
    std::vector<uint64_t> regs;  // DirectSource blocks its copies read
  };

  void ensure_stage(Stage& st, size_t bytes) {
    if (st.cap >= bytes) return;
    if (st.used) HIP_CHECK(hipEventSynchronize(st.free_ev));
    if (st.h) HIP_CHECK(hipHostFree(st.h));
    st.h = nullptr;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&st.h), bytes, hipHostMallocDefault));
    st.cap = bytes;
    st.used = false;
  }

  void ensure_window(Window& w, size_t bytes, size_t out_bytes) {
    if (w.cap < bytes) {
      if (w.d) HIP_CHECK(hipFree(w.d));
      w.d = nullptr;
      HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&w.d), bytes));
      w.cap = bytes;
    }
    if (w.out_cap < out_bytes) {
      if (w.d_out) HIP_CHECK(hipFree(w.d_out));
      if (w.h_out) HIP_CHECK(hipHostFree(w.h_out));
      w.d_out = nullptr;
      w.h_out = nullptr;
      HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&w.d_out), out_bytes));
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&w.h_out), out_bytes, hipHostMallocDefault));
      w.out_cap = out_bytes;
    }
  }

  // Read stream bytes [ga, ge) of the layout into p (single thread); marks
  // complete[k] = 0 for every piece k (relative to the piece at stream offset
  // `base`) that could not be fully read.
  static void read_range(const std::vector<Span>& spans, uint8_t* p, long long ga, long long ge, long long base,
                         size_t piece_len, size_t np, char* complete) {
    auto fail_range = [&](long long a, long long e) {  // stream offsets -> pieces
      if (e <= a) return;
      const size_t k0 = static_cast<size_t>(a - base) / piece_len;
      const size_t k1 = (static_cast<size_t>(e - base) + piece_len - 1) / piece_len;
      for (size_t k = k0; k < std::min(k1, np); ++k) complete[k] = 0;
    };
    long long cur = ga;
    for (const Span& s : spans) {
      if (s.start + s.length <= cur || s.start >= ge) continue;
      const long long ra = std::max(cur, s.start), re = std::min(ge, s.start + s.length);
      const size_t want = static_cast<size_t>(re - ra);
      uint8_t* q = p + (ra - ga);
      size_t got = 0;
      if (s.fd == kZeroSpan) {
        std::memset(q, 0, want);
        got = want;
      } else if (s.fd >= 0) {
        got = pread_full(s.fd, q, want, static_cast<off_t>(ra - s.start));
      }
      if (got != want) {
        std::memset(q + got, 0, want - got);
        fail_range(ra + static_cast<long long>(got), re);
      }
      cur = re;
      if (cur >= ge) break;
    }
    fail_range(cur, ge);  // a gap nobody covers: incomplete
  }

  // One reader unit: stream bytes [off, off+len) (piece-aligned start) into dst.
  static void read_unit(const std::vector<Span>& spans, uint8_t* dst, size_t off, size_t len, size_t piece_len,
                        char* complete) {
    read_range(spans, dst, static_cast<long long>(off), static_cast<long long>(off + len),
               static_cast<long long>(off), piece_len, (len + piece_len - 1) / piece_len, complete);
  }

  // GPU-side timeline of the last call (trace on): H2D copies, kernels, D2H.
  struct TraceRec {
    const char* kind;
    hipEvent_t a, b;
    size_t bytes;
  };
  void trace_begin(hipStream_t s, const char* kind, size_t bytes) {
    if (!trace_) return;
    TraceRec r{kind, nullptr, nullptr, bytes};
    HIP_CHECK(hipEventCreate(&r.a));
    HIP_CHECK(hipEventCreate(&r.b));
    HIP_CHECK(hipEventRecord(r.a, s));
    trace_recs_.push_back(r);
  }
  void trace_end(hipStream_t s) {
    if (trace_) HIP_CHECK(hipEventRecord(trace_recs_.back().b, s));
  }
  void trace_collect() {
    timeline_.clear();
    if (trace_recs_.empty()) return;
    hipEvent_t t0 = trace_recs_.front().a;
    for (auto& r : trace_recs_) {
      float a = 0.f, b = 0.f;
      hipEventElapsedTime(&a, t0, r.a);
      hipEventElapsedTime(&b, t0, r.b);
      timeline_.emplace_back(std::string(r.kind), a, b, r.bytes);
    }
    for (auto& r : trace_recs_) {
      hipEventDestroy(r.a);
      hipEventDestroy(r.b);
    }
    trace_recs_.clear();
  }

  // Pipeline driver.  claim(max) hands out the next contiguous run of pieces
  // [first, first+count) from the front of the layout (count 0 = no more);
  // runs are packed into an HBM window until it is full or claims dry up,
  // then one kernel hashes the window while the next one is being filled.
  // Each claimed run goes to the next staging slot, is split into >= 1 MiB
  // reader units for the pool, and is DMA'd to HBM as soon as its units are
  // done — up to kStages-1 slots are being filled while one is in flight.
  template <class Claim, class Unit, class Harvest>
  void run_windows(int alg, size_t piece_len, size_t total, size_t n, size_t wbytes, Claim&& claim, Unit&& unit,
                   Harvest&& harvest, DirectSource* ds = nullptr) {
    HIP_CHECK(hipSetDevice(device_));
    trace_recs_.clear();
    timeline_.clear();
    if (n == 0) return;
    const int dl = digest_len(alg);
    last_window_ = wbytes;
    const size_t per = std::min(n, std::max<size_t>(1, wbytes / piece_len));      // pieces per window
    const size_t stage_p = std::max<size_t>(1, stage_req_ / piece_len);            // pieces per staging slot
    const size_t stage = stage_p * piece_len;
    for (auto& st : stage_) ensure_stage(st, std::min(stage, per * piece_len));
    const size_t unit_p = std::max<size_t>(1, (1u << 20) / piece_len);             // >= 1 MiB preads
    struct Fill {
      int slot;
      size_t dst, len;
      std::shared_ptr<Latch> latch;
    };
    std::deque<Fill> fills;
    auto push_h2d = [&](Window& w) {  // oldest filled slot -> HBM
      Fill f = fills.front();
      fills.pop_front();
      f.latch->wait();
      progress_.fetch_add(f.len, std::memory_order_relaxed);  // read into pinned staging
      Stage& st = stage_[f.slot];
      trace_begin(copy_stream_, "h2d", f.len);
      HIP_CHECK(hipMemcpyAsync(w.d + f.dst, st.h, f.len, hipMemcpyHostToDevice, copy_stream_));
      trace_end(copy_stream_);
      HIP_CHECK(hipEventRecord(st.free_ev, copy_stream_));
      st.used = true;
    };
    auto drain = [&](Window& w) {
      if (!w.pending) return;
      HIP_CHECK(hipEventSynchronize(w.done));
      harvest(w.first, w.count, w.h_out, w.complete);
      if (ds) ds->unref(w.regs);  // its copies have landed (the kernel waited for them)
      w.pending = false;
    };
    size_t widx = 0, sidx = 0;
    try {
      for (bool more = true; more; ++widx) {
        Window& w = win_[widx % 2];
        drain(w);  // its previous window (widx-2) must be hashed before we overwrite it
        ensure_window(w, per * piece_len, per * dl);
        w.complete.assign(per, 1);
        size_t count = 0, first = 0;
        while (count < per) {
          const auto got = claim(std::min(stage_p, per - count));
          if (got.second == 0) {
            more = false;
            break;
          }
          if (count == 0) first = got.first;
          if (got.first != first + count) throw std::logic_error("non-contiguous GPU claim");
          {
            const size_t off = got.first * piece_len;
            const size_t len = std::min(total - off, got.second * piece_len);
            if (ds && ds->prepare(off, len)) {  // page cache -> HBM, no staging copy
              trace_begin(copy_stream_, "h2d_direct", len);
              ds->enqueue(w.d + count * piece_len, off, len, copy_stream_, w.regs);
              trace_end(copy_stream_);
              progress_.fetch_add(len, std::memory_order_relaxed);
              count += got.second;
              continue;
            }
          }
          if (fills.size() == static_cast<size_t>(kStages)) push_h2d(w);
          const int slot = static_cast<int>(sidx++ % kStages);
          Stage& st = stage_[slot];
          if (st.used) {
            HIP_CHECK(hipEventSynchronize(st.free_ev));  // its previous H2D has landed
            st.used = false;
          }
          const size_t off = got.first * piece_len;
          const size_t len = std::min(total - off, got.second * piece_len);
          const size_t nu = (got.second + unit_p - 1) / unit_p;
          auto latch = std::make_shared<Latch>(nu);
          uint8_t* h = st.h;
          char* comp = w.complete.data() + count;
          for (size_t u = 0; u < nu; ++u) {
            const size_t a = u * unit_p * piece_len, e = std::min(len, a + unit_p * piece_len);
            pool_->submit([&unit, latch, h, comp, off, a, e, u, unit_p] {
              try {
                unit(h + a, off + a, e - a, comp + u * unit_p);
                latch->done(nullptr);
              } catch (...) {
                latch->done(std::current_exception());
              }
            });
          }
          fills.push_back({slot, count * piece_len, len, latch});
          count += got.second;
        }
        while (!fills.empty()) push_h2d(w);
        if (count == 0) break;
        const size_t wlen = std::min(total - first * piece_len, count * piece_len);
        HIP_CHECK(hipEventRecord(w.copied, copy_stream_));
        HIP_CHECK(hipStreamWaitEvent(compute_stream_, w.copied, 0));
        trace_begin(compute_stream_, "kernel", wlen);
        launch_hash(alg, w.d, wlen, piece_len, static_cast<uint32_t>(count), w.d_out, compute_stream_);
        trace_end(compute_stream_);
        trace_begin(compute_stream_, "d2h", count * dl);
        HIP_CHECK(hipMemcpyAsync(w.h_out, w.d_out, count * dl, hipMemcpyDeviceToHost, compute_stream_));
        trace_end(compute_stream_);
        HIP_CHECK(hipEventRecord(w.done, compute_stream_));
        w.first = first;
        w.count = count;
        w.pending = true;
      }
      drain(win_[widx % 2]);
      drain(win_[(widx + 1) % 2]);
    } catch (...) {
      // queued reader units reference this frame: let every one finish first
      for (auto& f : fills) f.latch->wait_quiet();
      hipStreamSynchronize(copy_stream_);
      hipStreamSynchronize(compute_stream_);
      for (auto& st : stage_) st.used = false;
      for (auto& w : win_) {
        w.pending = false;
        if (ds) ds->unref(w.regs);
      }
      for (auto& r : trace_recs_) {
        hipEventDestroy(r.a);
        hipEventDestroy(r.b);
      }
      trace_recs_.clear();
      throw;
    }
    trace_collect();
  }

  // The whole layout front-to-back on the GPU (no CPU share).
  template <class Fill, class Harvest>
  void run_gpu_only(int alg, size_t piece_len, size_t total, size_t n, Fill&& fill, Harvest&& harvest,
                    DirectSource* ds = nullptr) {
    size_t front = 0;
    run_windows(alg, piece_len, total, n, window_bytes_for(total, piece_len),
                [&](size_t mx) {
                  const size_t c = std::min(mx, n - front);
                  const size_t f = front;
                  front += c;
                  return std::make_pair(f, c);
                },
                fill, harvest, ds);
  }

 public:
  // Digest every piece of a file layout with the GPU pipeline claiming from
  // the front and `cpu_threads` SHA-NI threads claiming >= 1 MiB units from
  // the back.  Fills digests (n*dl) and complete (n) for all pieces.
  void hybrid_digest(int alg, const std::vector<Span>& spans, size_t piece_len, size_t total, size_t n,
                     int cpu_threads, std::string& digests, std::string& complete, DirectSource* ds = nullptr) {
    const int dl = digest_len(alg);
    const EVP_MD* md = alg == 1 ? tritondl_hash::sha1_md() : tritondl_hash::sha256_md();
    std::mutex mu;
    size_t front = 0, back = n;
    std::atomic<unsigned long long> cpu_bytes{0};
    const auto t0 = std::chrono::steady_clock::now();
    // one more GPU window costs at least the per-lane latency of one piece
    // (one lane per piece, ~55 MB/s/lane measured) plus set-up
    const double kernel_s = static_cast<double>(piece_len) / 55e6 + 1e-3;
    // page cache -> HBM: ~57 GB/s direct (registered mapping), ~36-45 GB/s through pinned staging
    const double kCopyBps = ds && ds->on() ? 55e9 : 40e9;
    // pieces per CPU claim: >= 16 for the host's 16-lane AVX-512 kernels, else
    // >= 2 for SHA-NI pairs, and about 1 MiB of small pieces.  SHA-1 pieces
    // that are whole 64 KiB multiples stream through the 16-lane kernel: each
    // lane's next 64 KiB is read into a 1 MiB staging area that stays in the
    // core's L2 (the host verifier's loop, hash_core.h verify_pieces), so a
    // claim of 16 x 1 MiB pieces holds 1 MiB, not 16 MiB, and hashes from L2
    // instead of DRAM.  Claims that cannot stream hold at most ~2 MiB.
    constexpr size_t kStage = 64u << 10;
    const size_t wide = piece_len <= (1u << 20) ? tritondl_hash::md_claim(md) : 2;
    const bool stream16 = alg == 1 && wide == 16 && piece_len > kStage && piece_len % kStage == 0 &&
                          tritondl_hash::sha16::cpu_has_avx512();
    size_t unit = std::max<size_t>(wide, (1u << 20) / piece_len);
    if (!stream16 && unit * piece_len > (2u << 20)) unit = std::max<size_t>(2, (2u << 20) / piece_len);
    std::exception_ptr cpu_err;
    auto cpu_worker = [&] {
      try {
        // stream16: the 1 MiB staging area, or two whole pieces for a short
        // claim (the layout's tail); otherwise the whole claim
        std::vector<uint8_t> buf(stream16 ? std::max<size_t>(16 * kStage, 2 * piece_len) : unit * piece_len);
        const size_t cap_pieces = std::max<size_t>(1, buf.size() / piece_len);
        std::vector<char> ok(cap_pieces);
        for (;;) {
          size_t s, e;
          {
            std::lock_guard<std::mutex> g(mu);
            if (back <= front) return;
            e = back;
            s = e - std::min(unit, back - front);
            back = s;
          }
          const long long ga = static_cast<long long>(s * piece_len);
          const long long ge = std::min(static_cast<long long>(total), static_cast<long long>(e * piece_len));
          if (stream16 && e - s == 16 && ge == static_cast<long long>(e * piece_len)) {
            const void* lane[16];
            char lane_ok[16];
            for (size_t j = 0; j < 16; ++j) {
              lane[j] = buf.data() + j * kStage;
              lane_ok[j] = 1;
            }
            tritondl_hash::sha16::Sha1x16 st;
            tritondl_hash::sha16::sha1_x16_init(&st);
            for (size_t off = 0; off < piece_len; off += kStage) {
              for (size_t j = 0; j < 16; ++j) {
                const long long a = static_cast<long long>((s + j) * piece_len + off);
                if (lane_ok[j])  // a failed lane keeps hashing whatever is staged; its digest is discarded
                  read_range(spans, buf.data() + j * kStage, a, a + static_cast<long long>(kStage), a, kStage, 1,
                             &lane_ok[j]);
              }
              tritondl_hash::sha16::sha1_x16_update(&st, lane, kStage / 64);
            }
            unsigned char d[16 * 20];
            tritondl_hash::sha16::sha1_x16_finish(&st, lane, piece_len, d);  // piece_len % 64 == 0: no tail
            std::memcpy(&digests[s * dl], d, 16 * 20);
            for (size_t j = 0; j < 16; ++j) complete[s + j] = lane_ok[j];
            cpu_bytes.fetch_add(static_cast<unsigned long long>(ge - ga), std::memory_order_relaxed);
            progress_.fetch_add(static_cast<unsigned long long>(ge - ga), std::memory_order_relaxed);
            continue;
          }
          // whole pieces, as many at a time as the buffer holds
          for (size_t q = s; q < e; q += cap_pieces) {
            const size_t qe = std::min(e, q + cap_pieces);
            const long long qa = static_cast<long long>(q * piece_len);
            const long long qz = std::min(static_cast<long long>(total), static_cast<long long>(qe * piece_len));
            std::fill(ok.begin(), ok.end(), 1);
            read_range(spans, buf.data(), qa, qz, qa, piece_len, qe - q, ok.data());
            for (size_t p = q; p < qe; p += 16) {  // 16-lane AVX-512 groups, else SHA-NI pairs (md_batch)
              const size_t cnt = std::min<size_t>(16, qe - p);
              const void* src[16];
              size_t len[16];
              for (size_t j = 0; j < cnt; ++j) {
                const size_t po = (p + j - q) * piece_len;
                src[j] = buf.data() + po;
                len[j] = std::min<size_t>(piece_len, static_cast<size_t>(qz - qa) - po);
              }
              tritondl_hash::md_batch(md, src, len, cnt, reinterpret_cast<unsigned char*>(&digests[p * dl]));
              for (size_t j = 0; j < cnt; ++j) complete[p + j] = ok[p + j - q];
            }
          }
          cpu_bytes.fetch_add(static_cast<unsigned long long>(ge - ga), std::memory_order_relaxed);
          progress_.fetch_add(static_cast<unsigned long long>(ge - ga), std::memory_order_relaxed);
        }
      } catch (...) {
        std::lock_guard<std::mutex> g(mu);
        if (!cpu_err) cpu_err = std::current_exception();
        back = front;  // stop everyone
      }
    };
    std::vector<std::thread> ts;
    for (int k = 0; k < cpu_threads; ++k) ts.emplace_back([&] {
      tritondl_hash::name_thread("tdl-hybrid-cpu");
      cpu_worker();
    });
    size_t gpu_pieces = 0;
    try {
      // 1 GiB windows: kernels of earlier windows overlap later copies, so only
      // the last window's latency is exposed — and the claim rule below hands
      // that tail to the CPU threads
      const size_t wb = std::max(piece_len, std::min<size_t>(window_bytes_for(total, piece_len), 1ull << 30));
      run_windows(alg, piece_len, total, n, wb,
                  [&](size_t mx) {
                    std::lock_guard<std::mutex> g(mu);
                    const size_t left = back - front;
                    if (left == 0) return std::make_pair(front, size_t(0));
                    if (cpu_threads > 0) {
                      mx = std::min(mx, std::max<size_t>(unit, left / 2));  // leave the CPU its share near the end
                      // take the chunk only if the GPU would finish it (copy + one
                      // kernel latency) before the CPU threads could finish
                      // everything that is left on their own
                      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                      const double cpu_bps = el > 1e-3 ? cpu_bytes.load() / el : 0.0;
                      const double chunk = static_cast<double>(std::min(mx, left)) * piece_len;
                      if (cpu_bps > 0 && static_cast<double>(left) * piece_len / cpu_bps < chunk / kCopyBps + kernel_s)
                        return std::make_pair(front, size_t(0));
                    }
                    const size_t c = std::min(mx, left);
                    const size_t f = front;
                    front += c;
                    gpu_pieces += c;
                    return std::make_pair(f, c);
                  },
                  [&](uint8_t* dst, size_t off, size_t len, char* comp) { read_unit(spans, dst, off, len, piece_len, comp); },
                  [&](size_t first, size_t count, const uint8_t* d, const std::vector<char>& comp) {
                    std::memcpy(&digests[first * dl], d, count * dl);
                    for (size_t k = 0; k < count; ++k) complete[first + k] = comp[k];
                  },
                  ds);
    } catch (...) {
      {
        std::lock_guard<std::mutex> g(mu);
        back = front;
      }
      for (auto& th : ts) th.join();
      throw;
    }
    for (auto& th : ts) th.join();
    if (cpu_err) std::rethrow_exception(cpu_err);
    last_gpu_pieces_ = gpu_pieces;
  }

  size_t last_gpu_pieces() const { return last_gpu_pieces_; }
  size_t last_direct_bytes() const { return last_direct_bytes_; }
  // Bytes read so far (into staging, mapped for direct DMA, or hashed by the
  // host threads), over the hasher's lifetime: a monotonic counter another
  // thread may read while a call runs (the GPU helper's progress heartbeat).
  unsigned long long progress() const { return progress_.load(std::memory_order_relaxed); }
  bool trace() const { return trace_; }
  void set_trace(bool on) { trace_ = on; }
  std::vector<std::tuple<std::string, float, float, size_t>> last_timeline() const { return timeline_; }

 private:
  size_t last_gpu_pieces_ = 0;
  size_t last_direct_bytes_ = 0;
  int device_;
  size_t stage_req_;
  int readers_;
  size_t window_req_;
  size_t max_hbm_;
  size_t last_window_ = 0;
  std::mutex call_mu_;
  std::atomic<unsigned long long> progress_{0};
  std::chrono::steady_clock::time_point last_use_ = std::chrono::steady_clock::now();
  hipStream_t copy_stream_ = nullptr, compute_stream_ = nullptr;
  Stage stage_[kStages];
  Window win_[2];
  std::unique_ptr<ReaderPool> pool_;
  bool trace_ = false;
  std::vector<TraceRec> trace_recs_;
  std::vector<std::tuple<std::string, float, float, size_t>> timeline_;
};

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------ S3 chunk hashing
// The aws-chunked streaming signature needs the SHA-256 of every 64 KiB chunk
// of an upload; on a CPU-bound node that is half of a worker's CPU.  Each
// calling thread (the relay's parked hasher tasks) owns a stream, a
// blocking-sync event and pinned + device staging that grow to the largest
// batch seen.  One call = copy into pinned staging, H2D, one kernel (a lane
// per chunk), D2H of the digests, then the thread SLEEPS on the event (no
// spin-wait: that would burn the CPU this offload exists to save).
struct ChunkCtx {
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  uint8_t* pin = nullptr;
  uint8_t* dev = nullptr;
  uint32_t* dout = nullptr;
  uint8_t* pout = nullptr;
  size_t cap = 0, ocap = 0;
  ~ChunkCtx() {
    if (pin) (void)hipHostFree(pin);
    if (pout) (void)hipHostFree(pout);
    if (dev) (void)hipFree(dev);
    if (dout) (void)hipFree(dout);
    if (ev) (void)hipEventDestroy(ev);
    if (s) (void)hipStreamDestroy(s);
  }
};

std::atomic<int> g_chunk_device{0};

int sha256_chunks_impl(const void* src, size_t len, size_t chunk, unsigned char* out, char* err, size_t errlen) {
  static thread_local std::unique_ptr<ChunkCtx> tls;
  try {
    if (chunk == 0 || len == 0) throw std::invalid_argument("empty chunk batch");
    const size_t n = (len + chunk - 1) / chunk;
    if (!tls) {
      auto c = std::make_unique<ChunkCtx>();
      HIP_CHECK(hipSetDevice(g_chunk_device.load()));
      HIP_CHECK(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking));
      HIP_CHECK(hipEventCreateWithFlags(&c->ev, hipEventDisableTiming));
      tls = std::move(c);
    }
    ChunkCtx& c = *tls;
    if (c.cap < len) {
      if (c.pin) HIP_CHECK(hipHostFree(c.pin));
      if (c.dev) HIP_CHECK(hipFree(c.dev));
      c.pin = nullptr;
      c.dev = nullptr;
      c.cap = 0;
      const size_t cap = std::max<size_t>(len, 4u << 20);
      HIP_CHECK(hipHostMalloc(&c.pin, cap, hipHostMallocDefault));
      HIP_CHECK(hipMalloc(&c.dev, cap));
      c.cap = cap;
    }
    if (c.ocap < n * 32) {
      if (c.pout) HIP_CHECK(hipHostFree(c.pout));
      if (c.dout) HIP_CHECK(hipFree(c.dout));
      c.pout = nullptr;
      c.dout = nullptr;
      c.ocap = 0;
      const size_t ocap = std::max<size_t>(n * 32, 8192);
      HIP_CHECK(hipHostMalloc(&c.pout, ocap, hipHostMallocDefault));
      HIP_CHECK(hipMalloc(&c.dout, ocap));
      c.ocap = ocap;
    }
    std::memcpy(c.pin, src, len);  // page cache mapping -> pinned (the DMA needs pinned pages)
    HIP_CHECK(hipMemcpyAsync(c.dev, c.pin, len, hipMemcpyHostToDevice, c.s));
    launch_hash(256, c.dev, len, chunk, static_cast<uint32_t>(n), c.dout, c.s, 64);
    HIP_CHECK(hipMemcpyAsync(c.pout, c.dout, n * 32, hipMemcpyDeviceToHost, c.s));
    // Completion: the thread sleeps between event queries.  Both HIP blocking
    // mechanisms cost more CPU than the SHA-NI hashing this replaces
    // (profiles/r03_gpu_sha_ab): hipEventSynchronize, even on a
    // hipEventBlockingSync event, polled (~20 ms of CPU per 10 MiB job over
    // the hasher threads); hipLaunchHostFunc's runtime thread cost ~6.5 ms.
    // The kernel of a 64 KiB-chunk batch runs ~2.6 ms, so 250 us sleeps add
    // little latency and almost no CPU.
    HIP_CHECK(hipEventRecord(c.ev, c.s));
    for (;;) {
      const hipError_t q = hipEventQuery(c.ev);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) HIP_CHECK(q);
      std::this_thread::sleep_for(std::chrono::microseconds(250));
    }
    std::memcpy(out, c.pout, n * 32);
    return 0;
  } catch (const std::exception& e) {
    if (err && errlen) std::snprintf(err, errlen, "%s", e.what());
    return -1;
  }
}

TdlGpuChunkApi g_chunk_api{1, &sha256_chunks_impl};

}  // namespace

PYBIND11_MODULE(_gpu_hash, m) {
  m.doc() = "tritondl HIP (gfx950) batched SHA-1/SHA-256 piece hashing";
  m.def("device_count", &device_count);
  m.def(
      "mem_get_info",
      [](int device) {
        size_t free_b = 0, total_b = 0;
        {
          py::gil_scoped_release nogil;
          HIP_CHECK(hipSetDevice(device));
          HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        }
        return py::make_tuple(free_b, total_b);
      },
      py::arg("device") = 0, "(free, total) HBM bytes of a device (hipMemGetInfo)");
  m.def("chunk_api", [](int device) {
          g_chunk_device.store(device);
          return py::capsule(&g_chunk_api, TDL_GPU_CHUNK_API_NAME);
        },
        py::arg("device") = 0,
        "PyCapsule with the C table the relay's S3 send pump uses to hash aws-chunked chunks on the GPU");
  m.def(
      "sha256_chunks",
      [](const py::buffer& buf, size_t chunk) {
        py::buffer_info bi = buf.request();
        const size_t len = static_cast<size_t>(bi.size * bi.itemsize);
        std::string out(((len + chunk - 1) / chunk) * 32, '\0');
        char err[256] = {0};
        int rc;
        {
          py::gil_scoped_release nogil;
          rc = sha256_chunks_impl(bi.ptr, len, chunk, reinterpret_cast<unsigned char*>(&out[0]), err, sizeof err);
        }
        if (rc) throw std::runtime_error(err);
        return py::bytes(out);
      },
      py::arg("buffer"), py::arg("chunk"), "the chunk_api call from Python (tests): concatenated 32-byte digests");
  m.def(
      "hash_device",
      [](const std::string& kind, uintptr_t data_ptr, uint64_t total, uint64_t piece_len, uintptr_t out_ptr,
         uintptr_t stream, int lanes) {
        const int alg = alg_id(kind);
        if (piece_len == 0) throw std::invalid_argument("piece_len must be > 0");
        const uint64_t n = total ? (total + piece_len - 1) / piece_len : 0;
        if (n > 0xFFFFFFFFull) throw std::invalid_argument("too many pieces");
        launch_hash(alg, reinterpret_cast<const uint8_t*>(data_ptr), total, piece_len, static_cast<uint32_t>(n),
                    reinterpret_cast<uint32_t*>(out_ptr), reinterpret_cast<hipStream_t>(stream), lanes);
        return n;
      },
      py::arg("kind"), py::arg("data_ptr"), py::arg("total"), py::arg("piece_len"), py::arg("out_ptr"),
      py::arg("stream") = 0, py::arg("lanes") = 64,
      "Launch on caller-owned device memory (e.g. torch tensors); out holds n*digest_len bytes.");
  py::class_<GpuHasher>(m, "GpuHasher")
      .def(py::init<int, size_t, int, size_t, size_t>(), py::arg("device") = 0, py::arg("batch_bytes") = 256u << 20,
           py::arg("reader_threads") = 8, py::arg("window_bytes") = 0, py::arg("max_hbm") = 0,
           "batch_bytes: pinned staging chunk (allocated on first use); window_bytes: HBM window per kernel "
           "launch (0 = auto: half of max_hbm, at most a third of free HBM); max_hbm: HBM the two windows "
           "may hold (0 = 8 GiB)")
      .def("hash_buffer", &GpuHasher::hash_buffer, py::arg("kind"), py::arg("buffer"), py::arg("piece_len"))
      .def("verify_files", &GpuHasher::verify_files, py::arg("files"), py::arg("piece_len"), py::arg("expected"),
           py::arg("kind") = "sha1", py::arg("cpu_threads") = 0,
           "one byte (0/1) per piece; cpu_threads > 0: hybrid (SHA-NI threads take pieces from the back)")
      .def("digest_files", &GpuHasher::digest_files, py::arg("files"), py::arg("piece_len"), py::arg("kind") = "sha256",
           py::arg("cpu_threads") = 0, "(digests, fully_read_mask) of every piece of a file layout")
      .def_property("trace", &GpuHasher::trace, &GpuHasher::set_trace,
                    "record a GPU event timeline (H2D / kernel / D2H) of each call")
      .def_property_readonly("last_timeline", &GpuHasher::last_timeline,
                             "[(kind, start_ms, end_ms, bytes)] of the last call, relative to its first op")
      .def_property_readonly("last_gpu_pieces", &GpuHasher::last_gpu_pieces,
                             "pieces the GPU hashed in the last verify/digest call (the rest: CPU threads)")
      .def_property_readonly("last_direct_bytes", &GpuHasher::last_direct_bytes,
                             "bytes of the last verify/digest call DMA'd straight from the page cache")
      .def("release", &GpuHasher::release_py, "free staging + windows now (waits for a running call)")
      .def("release_if_idle", &GpuHasher::release_if_idle, py::arg("idle_s"),
           "free staging + windows if no call ran for idle_s seconds and none is running; True if freed")
      .def_property_readonly("held_bytes", &GpuHasher::held_bytes,
                             "(device, pinned host) bytes held between calls")
      .def_property_readonly("max_hbm", &GpuHasher::max_hbm)
      .def("window_bytes_for", &GpuHasher::window_bytes_for)
      .def_property_readonly("last_window_bytes", &GpuHasher::last_window_bytes)
      .def("progress", &GpuHasher::progress, "bytes read so far (lifetime counter; safe during a call)")
      .def_property_readonly("batch_bytes", &GpuHasher::batch_bytes);
}
