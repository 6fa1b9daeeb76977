// Sixteen-lane SHA-1 with AVX-512 — the BitTorrent v1 piece hash.
//
// It uses the same layout as sha256_mb.h.  Each 32-bit lane of a zmm
// carries one piece, and the message words arrive through the same 16x16
// in-register transpose.  A SHA-1 round is even cheaper in this form than
// a SHA-256 round:
//   * `vprold` does rotl5 and rotl30;
//   * one `vpternlogd` computes Ch, Parity or Maj;
//   * the schedule's four-way XOR is one `vpternlogd` plus one `vpxord`,
//     then a rotate.
// That is ~56 vector ops per lane-block, against ~100 for SHA-256.  SHA-NI
// pairs verify v1 pieces at ~3.4 GB/s per core on the Zen 5 host
// (profiles/r02_sha1_ab/).  Resume verification and live piece checks hash
// many equal-length pieces, so the lanes are full.
//
// Same switch as SHA-256: TRITONDL_SHA_MB=0 disables it.
#pragma once

#include <immintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstring>

#include "sha256_mb.h"

namespace tritondl_hash {
namespace sha16 {

#define TDL_MB1_TARGET __attribute__((target("avx512f,avx512bw")))

TDL_MB1_TARGET inline void sha1_compress(__m512i s[5], const uint8_t* const p[16], size_t nblocks) {
  const __m512i k0 = _mm512_set1_epi32(0x5a827999), k1 = _mm512_set1_epi32(0x6ed9eba1),
                k2 = _mm512_set1_epi32(static_cast<int>(0x8f1bbcdc)), k3 = _mm512_set1_epi32(static_cast<int>(0xca62c1d6));
  for (size_t blk = 0; blk < nblocks; ++blk) {
    __m512i w[16];
    load_transposed(p, blk * 64, w);
    __m512i a = s[0], b = s[1], c = s[2], d = s[3], e = s[4];
#define TDL_MB1_ROUND(wt, fimm, k)                                                                     \
  do {                                                                                                 \
    const __m512i f_ = _mm512_ternarylogic_epi32(b, c, d, fimm);                                        \
    /* rotl5(a) joins last: the new a is two ops deep in a (latency-bound chain) */                    \
    const __m512i tmp_ = _mm512_add_epi32(_mm512_rol_epi32(a, 5),                                     \
                                          _mm512_add_epi32(f_, _mm512_add_epi32(e, _mm512_add_epi32(wt, k)))); \
    e = d;                                                                                             \
    d = c;                                                                                             \
    c = _mm512_rol_epi32(b, 30);                                                                       \
    b = a;                                                                                             \
    a = tmp_;                                                                                          \
  } while (0)
#define TDL_MB1_SCHED(t)                                                                               \
  (w[(t) & 15] = _mm512_rol_epi32(                                                                     \
       _mm512_xor_si512(_mm512_ternarylogic_epi32(w[((t) - 3) & 15], w[((t) - 8) & 15], w[((t) - 14) & 15], 0x96), \
                        w[(t) & 15]),                                                                  \
       1))
    // fully unrolled so every w[] index is a constant (registers, not memory)
#pragma GCC unroll 16
    for (int t = 0; t < 16; ++t) TDL_MB1_ROUND(w[t], 0xca, k0);
#pragma GCC unroll 4
    for (int t = 16; t < 20; ++t) TDL_MB1_ROUND(TDL_MB1_SCHED(t), 0xca, k0);
#pragma GCC unroll 20
    for (int t = 20; t < 40; ++t) TDL_MB1_ROUND(TDL_MB1_SCHED(t), 0x96, k1);
#pragma GCC unroll 20
    for (int t = 40; t < 60; ++t) TDL_MB1_ROUND(TDL_MB1_SCHED(t), 0xe8, k2);
#pragma GCC unroll 20
    for (int t = 60; t < 80; ++t) TDL_MB1_ROUND(TDL_MB1_SCHED(t), 0x96, k3);
#undef TDL_MB1_SCHED
#undef TDL_MB1_ROUND
    s[0] = _mm512_add_epi32(s[0], a);
    s[1] = _mm512_add_epi32(s[1], b);
    s[2] = _mm512_add_epi32(s[2], c);
    s[3] = _mm512_add_epi32(s[3], d);
    s[4] = _mm512_add_epi32(s[4], e);
  }
}

// Incremental form, for messages that do not fit a core's cache at once
// (resume verification streams 16 pieces through a 1 MiB staging area):
// init, any number of update() calls of whole 64-byte blocks, finish() with
// the remaining < 64 bytes of each lane and the total length.
struct Sha1x16 {
  __m512i s[5];
};
TDL_MB1_TARGET inline void sha1_x16_init(Sha1x16* st) {
  static const uint32_t h0[5] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476, 0xc3d2e1f0};
  for (int i = 0; i < 5; ++i) st->s[i] = _mm512_set1_epi32(static_cast<int>(h0[i]));
}
TDL_MB1_TARGET inline void sha1_x16_update(Sha1x16* st, const void* const msg[16], size_t nblocks) {
  const uint8_t* p[16];
  for (int j = 0; j < 16; ++j) p[j] = static_cast<const uint8_t*>(msg[j]);
  sha1_compress(st->s, p, nblocks);
}
TDL_MB1_TARGET inline void sha1_x16_finish(Sha1x16* st, const void* const rest[16], size_t total,
                                           unsigned char* out);

// SHA-1 of 16 messages of `len` bytes each: out + 20*j = digest of msg[j].
TDL_MB1_TARGET inline void sha1_x16(const void* const msg[16], size_t len, unsigned char* out) {
  Sha1x16 st;
  sha1_x16_init(&st);
  const size_t full = len / 64;
  sha1_x16_update(&st, msg, full);
  const void* rest[16];
  for (int j = 0; j < 16; ++j) rest[j] = static_cast<const uint8_t*>(msg[j]) + full * 64;
  sha1_x16_finish(&st, rest, len, out);
}

// rest[j]: the last total % 64 bytes of lane j
TDL_MB1_TARGET inline void sha1_x16_finish(Sha1x16* st, const void* const rest[16], size_t total,
                                           unsigned char* out) {
  const size_t rem = total % 64;
  const size_t tail_blocks = rem < 56 ? 1 : 2;
  alignas(64) uint8_t tail[16][128];
  const uint8_t* p[16];
  const uint64_t bits = static_cast<uint64_t>(total) * 8;
  for (int j = 0; j < 16; ++j) {
    std::memset(tail[j], 0, sizeof tail[j]);
    if (rem) std::memcpy(tail[j], rest[j], rem);
    tail[j][rem] = 0x80;
    for (int k = 0; k < 8; ++k) tail[j][tail_blocks * 64 - 1 - k] = static_cast<uint8_t>(bits >> (8 * k));
    p[j] = tail[j];
  }
  sha1_compress(st->s, p, tail_blocks);
  alignas(64) uint32_t words[5][16];
  for (int i = 0; i < 5; ++i) _mm512_store_si512(words[i], st->s[i]);
  for (int j = 0; j < 16; ++j)
    for (int i = 0; i < 5; ++i) {
      const uint32_t v = words[i][j];
      unsigned char* o = out + 20 * j + 4 * i;
      o[0] = static_cast<unsigned char>(v >> 24);
      o[1] = static_cast<unsigned char>(v >> 16);
      o[2] = static_cast<unsigned char>(v >> 8);
      o[3] = static_cast<unsigned char>(v);
    }
}

#undef TDL_MB1_TARGET

}  // namespace sha16
}  // namespace tritondl_hash
