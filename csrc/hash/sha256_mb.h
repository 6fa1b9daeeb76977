// Sixteen-lane SHA-256 with AVX-512 (one message per 32-bit lane of a zmm).
//
// SHA-NI hashes one 64-byte block per ~40 cycles per core on the MI355X
// host (EPYC 9575F, Zen 5), even with two messages in lockstep
// (sha_ni.h): the round instructions are the bottleneck.  Zen 5 executes
// 512-bit integer vector ops at full width, and the SHA-256 round maps onto
// them with few instructions: vprord for the rotations, and vpternlogd for
// Ch, Maj and each three-way XOR of Σ0/Σ1/σ0/σ1.  A round is ~17 vector
// ops for 16 messages at once.  aws-chunked uploads hash hundreds of
// independent 64 KiB chunks per object, so the lanes are always full.
//
// Lanes are filled by loading one 64-byte block from each of the 16
// messages and transposing the 16x16 dword tile in registers (unpack 32/64,
// then two 128-bit shuffles).  That is ~5 ops per lane-block, with no
// gathers.  Every message of a call has the same length; callers hash a
// shorter tail chunk with SHA-NI.
//
// TRITONDL_SHA_MB=0 disables it (the A/B switch); CPUs without AVX-512F/BW
// never take this path.
#pragma once

#include <cpuid.h>
#include <immintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "sha_ni.h"

namespace tritondl_hash {
namespace sha16 {

inline bool cpu_has_avx512() {
  static const bool ok = [] {
    const char* env = std::getenv("TRITONDL_SHA_MB");
    if (env && (env[0] == '0' || env[0] == 'n' || env[0] == 'o')) return false;
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    const bool f = b & (1u << 16), bw = b & (1u << 30);
    if (!(f && bw)) return false;
    // the OS must save the zmm state (XCR0 bits 1,2 and 5-7)
    if (!__get_cpuid(1, &a, &b, &c, &d) || !(c & (1u << 27))) return false;
    unsigned lo, hi;
    __asm__("xgetbv" : "=a"(lo), "=d"(hi) : "c"(0));
    return (lo & 0xe6) == 0xe6;
  }();
  return ok;
}

#define TDL_MB_TARGET __attribute__((target("avx512f,avx512bw")))
#define TDL_MB_INLINE __attribute__((target("avx512f,avx512bw"), always_inline)) inline

TDL_MB_INLINE __m512i xor3(__m512i a, __m512i b, __m512i c) { return _mm512_ternarylogic_epi32(a, b, c, 0x96); }

// 16 rows (one 64-byte block of each lane) -> 16 words W[t] (lane j in element j), big-endian
TDL_MB_INLINE void load_transposed(const uint8_t* const p[16], size_t off, __m512i w[16]) {
  const __m512i bswap = _mm512_set4_epi32(0x0c0d0e0f, 0x08090a0b, 0x04050607, 0x00010203);
  __m512i r[16], t[16];
  for (int j = 0; j < 16; ++j) r[j] = _mm512_loadu_si512(p[j] + off);
  for (int i = 0; i < 16; i += 2) {
    t[i] = _mm512_unpacklo_epi32(r[i], r[i + 1]);
    t[i + 1] = _mm512_unpackhi_epi32(r[i], r[i + 1]);
  }
  // u[q][c]: in 128-bit lane L, rows 4q..4q+3 of dword column 4L+c
  __m512i u[4][4];
  for (int q = 0; q < 4; ++q) {
    const __m512i* T = t + 4 * q;
    u[q][0] = _mm512_unpacklo_epi64(T[0], T[2]);
    u[q][1] = _mm512_unpackhi_epi64(T[0], T[2]);
    u[q][2] = _mm512_unpacklo_epi64(T[1], T[3]);
    u[q][3] = _mm512_unpackhi_epi64(T[1], T[3]);
  }
  for (int c = 0; c < 4; ++c) {
    const __m512i x0 = _mm512_shuffle_i32x4(u[0][c], u[1][c], 0x44);
    const __m512i x1 = _mm512_shuffle_i32x4(u[0][c], u[1][c], 0xee);
    const __m512i x2 = _mm512_shuffle_i32x4(u[2][c], u[3][c], 0x44);
    const __m512i x3 = _mm512_shuffle_i32x4(u[2][c], u[3][c], 0xee);
    w[0 + c] = _mm512_shuffle_epi8(_mm512_shuffle_i32x4(x0, x2, 0x88), bswap);
    w[4 + c] = _mm512_shuffle_epi8(_mm512_shuffle_i32x4(x0, x2, 0xdd), bswap);
    w[8 + c] = _mm512_shuffle_epi8(_mm512_shuffle_i32x4(x1, x3, 0x88), bswap);
    w[12 + c] = _mm512_shuffle_epi8(_mm512_shuffle_i32x4(x1, x3, 0xdd), bswap);
  }
}

// Compress `nblocks` consecutive 64-byte blocks of every lane into s[8].
TDL_MB_TARGET inline void compress(__m512i s[8], const uint8_t* const p[16], size_t nblocks) {
  for (size_t blk = 0; blk < nblocks; ++blk) {
    __m512i w[16];
    load_transposed(p, blk * 64, w);
    __m512i a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
// The round is latency-bound (each op waits on the previous round's e / a),
// so the sums are associated to keep the chains short: h + W + K and
// d + (h + W + K) do not depend on this round's e and are ready early;
// new e = ((d + hwk) + Ch) + Σ1 is three ops deep from e, and new
// a = ((hwk + Ch) + Σ1) + (Σ0 + Maj) four (instead of five for both).
#define TDL_MB_ROUND(t, wt)                                                                              \
  do {                                                                                                   \
    const __m512i hwk = _mm512_add_epi32(h, _mm512_add_epi32(                                            \
                                                wt, _mm512_set1_epi32(static_cast<int>(sha2x::kK[t])))); \
    const __m512i dhwk = _mm512_add_epi32(d, hwk);                                                       \
    const __m512i s1 = xor3(_mm512_ror_epi32(e, 6), _mm512_ror_epi32(e, 11), _mm512_ror_epi32(e, 25));  \
    const __m512i ch = _mm512_ternarylogic_epi32(e, f, g, 0xca);                                         \
    const __m512i s0 = xor3(_mm512_ror_epi32(a, 2), _mm512_ror_epi32(a, 13), _mm512_ror_epi32(a, 22));  \
    const __m512i mj = _mm512_ternarylogic_epi32(a, b, c, 0xe8);                                         \
    const __m512i t1 = _mm512_add_epi32(_mm512_add_epi32(hwk, ch), s1);                                  \
    h = g;                                                                                               \
    g = f;                                                                                               \
    f = e;                                                                                               \
    e = _mm512_add_epi32(_mm512_add_epi32(dhwk, ch), s1);                                                \
    d = c;                                                                                               \
    c = b;                                                                                               \
    b = a;                                                                                               \
    a = _mm512_add_epi32(t1, _mm512_add_epi32(s0, mj));                                                  \
  } while (0)
    // fully unrolled: with a runtime t, w[t & 15] would live in memory
#pragma GCC unroll 16
    for (int t = 0; t < 16; ++t) TDL_MB_ROUND(t, w[t]);
#pragma GCC unroll 48
    for (int t = 16; t < 64; ++t) {
      const __m512i x15 = w[(t - 15) & 15], x2 = w[(t - 2) & 15];
      const __m512i sg0 = xor3(_mm512_ror_epi32(x15, 7), _mm512_ror_epi32(x15, 18), _mm512_srli_epi32(x15, 3));
      const __m512i sg1 = xor3(_mm512_ror_epi32(x2, 17), _mm512_ror_epi32(x2, 19), _mm512_srli_epi32(x2, 10));
      const __m512i wt = _mm512_add_epi32(_mm512_add_epi32(w[t & 15], sg0), _mm512_add_epi32(w[(t - 7) & 15], sg1));
      w[t & 15] = wt;
      TDL_MB_ROUND(t, wt);
    }
#undef TDL_MB_ROUND
    s[0] = _mm512_add_epi32(s[0], a);
    s[1] = _mm512_add_epi32(s[1], b);
    s[2] = _mm512_add_epi32(s[2], c);
    s[3] = _mm512_add_epi32(s[3], d);
    s[4] = _mm512_add_epi32(s[4], e);
    s[5] = _mm512_add_epi32(s[5], f);
    s[6] = _mm512_add_epi32(s[6], g);
    s[7] = _mm512_add_epi32(s[7], h);
  }
}

// SHA-256 of 16 messages of `len` bytes each: out + 32*j = digest of msg[j].
TDL_MB_TARGET inline void sha256_x16(const void* const msg[16], size_t len, unsigned char* out) {
  __m512i s[8];
  for (int i = 0; i < 8; ++i) s[i] = _mm512_set1_epi32(static_cast<int>(sha2x::kH0[i]));
  const uint8_t* p[16];
  for (int j = 0; j < 16; ++j) p[j] = static_cast<const uint8_t*>(msg[j]);
  const size_t full = len / 64;
  compress(s, p, full);
  // tail: the remainder, 0x80, zeros, the bit length (one or two blocks per lane)
  const size_t rem = len % 64;
  const size_t tail_blocks = rem < 56 ? 1 : 2;
  alignas(64) uint8_t tail[16][128];
  const uint64_t bits = static_cast<uint64_t>(len) * 8;
  for (int j = 0; j < 16; ++j) {
    std::memset(tail[j], 0, sizeof tail[j]);
    if (rem) std::memcpy(tail[j], p[j] + full * 64, rem);
    tail[j][rem] = 0x80;
    for (int k = 0; k < 8; ++k) tail[j][tail_blocks * 64 - 1 - k] = static_cast<uint8_t>(bits >> (8 * k));
    p[j] = tail[j];
  }
  compress(s, p, tail_blocks);
  alignas(64) uint32_t st[8][16];
  for (int i = 0; i < 8; ++i) _mm512_store_si512(st[i], s[i]);
  for (int j = 0; j < 16; ++j)
    for (int i = 0; i < 8; ++i) {
      const uint32_t v = st[i][j];
      unsigned char* o = out + 32 * j + 4 * i;
      o[0] = static_cast<unsigned char>(v >> 24);
      o[1] = static_cast<unsigned char>(v >> 16);
      o[2] = static_cast<unsigned char>(v >> 8);
      o[3] = static_cast<unsigned char>(v);
    }
}

#undef TDL_MB_TARGET
#undef TDL_MB_INLINE

}  // namespace sha16
}  // namespace tritondl_hash
