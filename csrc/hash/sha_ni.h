// Two-stream SHA-256 and SHA-1 with the x86 SHA extensions (SHA-NI).
//
// SHA-256 is a serial chain inside one message, and each sha256rnds2 waits
// on the previous one (3-4 cycles of latency on Zen / Intel cores that can
// issue one every 1-2 cycles).  Hashing TWO independent messages in
// lockstep fills those latency slots.  aws-chunked uploads have exactly
// that shape: every 64 KiB chunk is hashed on its own.  BitTorrent v1
// verification does too (every piece is its own SHA-1).  The result is ~1.6-2x
// the single-stream rate per core (tools/bench_sha.py).  Used by the relay
// send pump, the streamed verifier and the chunk encoders; falls back to
// OpenSSL where the CPU has no SHA-NI.
#pragma once

#include <cpuid.h>
#include <immintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>

namespace tritondl_hash {
namespace sha2x {

alignas(16) static const uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t kH0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

// SHA-NI present (and not disabled with TRITONDL_SHA_NI=0, which selects
// OpenSSL for every digest — the A/B switch).
inline bool cpu_has_sha_ni() {
  static const bool ok = [] {
    const char* env = std::getenv("TRITONDL_SHA_NI");
    if (env && (env[0] == '0' || env[0] == 'n' || env[0] == 'o')) return false;
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
    const bool ssse3 = c & (1u << 9), sse41 = c & (1u << 19);
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return false;
    return ssse3 && sse41 && (b & (1u << 29));
  }();
  return ok;
}

// One lane's working set: the state in the ABEF/CDGH layout sha256rnds2
// uses, and the four message-schedule registers.
struct Lane {
  __m128i s0, s1, m[4];
};

#define TDL_SHA_TARGET __attribute__((target("sha,sse4.1,ssse3"), always_inline))

TDL_SHA_TARGET inline void load_state(Lane& l, const uint32_t st[8]) {
  __m128i t = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st));
  __m128i s1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(st + 4));
  t = _mm_shuffle_epi32(t, 0xB1);          // CDAB
  s1 = _mm_shuffle_epi32(s1, 0x1B);        // EFGH
  l.s0 = _mm_alignr_epi8(t, s1, 8);        // ABEF
  l.s1 = _mm_blend_epi16(s1, t, 0xF0);     // CDGH
}

TDL_SHA_TARGET inline void store_state(const Lane& l, uint32_t st[8]) {
  __m128i t = _mm_shuffle_epi32(l.s0, 0x1B);     // FEBA
  __m128i s1 = _mm_shuffle_epi32(l.s1, 0xB1);    // DCHG
  _mm_storeu_si128(reinterpret_cast<__m128i*>(st), _mm_blend_epi16(t, s1, 0xF0));        // DCBA
  _mm_storeu_si128(reinterpret_cast<__m128i*>(st + 4), _mm_alignr_epi8(s1, t, 8));       // HGFE
}

// Rounds 4g .. 4g+3 of one block for one lane (g is a compile-time constant
// after unrolling, so m[g % 4] etc. stay in registers).
TDL_SHA_TARGET inline void group(Lane& l, int g, const uint8_t* p, __m128i mask) {
  __m128i& cur = l.m[g & 3];
  if (g < 4) cur = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * g)), mask);
  __m128i msg = _mm_add_epi32(cur, _mm_load_si128(reinterpret_cast<const __m128i*>(kK + 4 * g)));
  l.s1 = _mm_sha256rnds2_epu32(l.s1, l.s0, msg);
  if (g >= 3 && g <= 14) {
    __m128i& nxt = l.m[(g + 1) & 3];
    nxt = _mm_add_epi32(nxt, _mm_alignr_epi8(cur, l.m[(g + 3) & 3], 4));
    nxt = _mm_sha256msg2_epu32(nxt, cur);
  }
  msg = _mm_shuffle_epi32(msg, 0x0E);
  l.s0 = _mm_sha256rnds2_epu32(l.s0, l.s1, msg);
  if (g >= 1 && g <= 12) {
    __m128i& prv = l.m[(g + 3) & 3];
    prv = _mm_sha256msg1_epu32(prv, cur);
  }
}

__attribute__((target("sha,sse4.1,ssse3"))) inline void blocks_x1(uint32_t st[8], const uint8_t* p, size_t n) {
  const __m128i mask = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  Lane a;
  load_state(a, st);
  for (; n; --n, p += 64) {
    const __m128i s0 = a.s0, s1 = a.s1;
#pragma GCC unroll 16
    for (int g = 0; g < 16; ++g) group(a, g, p, mask);
    a.s0 = _mm_add_epi32(a.s0, s0);
    a.s1 = _mm_add_epi32(a.s1, s1);
  }
  store_state(a, st);
}

__attribute__((target("sha,sse4.1,ssse3"))) inline void blocks_x2(uint32_t sa[8], uint32_t sb[8], const uint8_t* pa,
                                                                 const uint8_t* pb, size_t n) {
  const __m128i mask = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  Lane a, b;
  load_state(a, sa);
  load_state(b, sb);
  for (; n; --n, pa += 64, pb += 64) {
    const __m128i a0 = a.s0, a1 = a.s1, b0 = b.s0, b1 = b.s1;
#pragma GCC unroll 16
    for (int g = 0; g < 16; ++g) {
      group(a, g, pa, mask);
      group(b, g, pb, mask);
    }
    a.s0 = _mm_add_epi32(a.s0, a0);
    a.s1 = _mm_add_epi32(a.s1, a1);
    b.s0 = _mm_add_epi32(b.s0, b0);
    b.s1 = _mm_add_epi32(b.s1, b1);
  }
  store_state(a, sa);
  store_state(b, sb);
}

#undef TDL_SHA_TARGET

// Padding + length of the last (partial) block(s): 1 or 2 blocks in `tail`.
inline size_t pad_tail(uint8_t tail[128], const uint8_t* rest, size_t nrest, uint64_t total) {
  std::memset(tail, 0, 128);
  if (nrest) std::memcpy(tail, rest, nrest);
  tail[nrest] = 0x80;
  const size_t nb = nrest + 9 <= 64 ? 1 : 2;
  const uint64_t bits = total * 8;
  for (int i = 0; i < 8; ++i) tail[nb * 64 - 1 - i] = uint8_t(bits >> (8 * i));
  return nb;
}

inline void digest_out(const uint32_t st[8], uint8_t out[32]) {
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = uint8_t(st[i] >> 24);
    out[4 * i + 1] = uint8_t(st[i] >> 16);
    out[4 * i + 2] = uint8_t(st[i] >> 8);
    out[4 * i + 3] = uint8_t(st[i]);
  }
}

// SHA-256 of one message (SHA-NI required).
inline void sha256_x1(const void* data, size_t n, uint8_t out[32]) {
  uint32_t st[8];
  std::memcpy(st, kH0, sizeof st);
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const size_t full = n / 64;
  if (full) blocks_x1(st, p, full);
  uint8_t tail[128];
  const size_t nb = pad_tail(tail, p + full * 64, n - full * 64, n);
  blocks_x1(st, tail, nb);
  digest_out(st, out);
}

// SHA-256 of two messages at once (SHA-NI required): the blocks both have
// run in lockstep, the rest of the longer one and both tails single.
inline void sha256_x2(const void* da, size_t na, const void* db, size_t nb, uint8_t oa[32], uint8_t ob[32]) {
  uint32_t sa[8], sb[8];
  std::memcpy(sa, kH0, sizeof sa);
  std::memcpy(sb, kH0, sizeof sb);
  const uint8_t* pa = static_cast<const uint8_t*>(da);
  const uint8_t* pb = static_cast<const uint8_t*>(db);
  const size_t fa = na / 64, fb = nb / 64, both = fa < fb ? fa : fb;
  if (both) blocks_x2(sa, sb, pa, pb, both);
  if (fa > both) blocks_x1(sa, pa + both * 64, fa - both);
  if (fb > both) blocks_x1(sb, pb + both * 64, fb - both);
  uint8_t ta[128], tb[128];
  const size_t ka = pad_tail(ta, pa + fa * 64, na - fa * 64, na);
  const size_t kb = pad_tail(tb, pb + fb * 64, nb - fb * 64, nb);
  if (ka == kb) {
    blocks_x2(sa, sb, ta, tb, ka);
  } else {
    blocks_x1(sa, ta, ka);
    blocks_x1(sb, tb, kb);
  }
  digest_out(sa, oa);
  digest_out(sb, ob);
}

// ------------------------------------------------------------------ SHA-1
// Same scheme for SHA-1 (sha1rnds4 / sha1nexte / sha1msg1 / sha1msg2):
// BitTorrent v1 piece verification on the host (resume, hybrid GPU+CPU).

struct Lane1 {
  __m128i abcd, e[2], m[4];
};

#define TDL_SHA_TARGET __attribute__((target("sha,sse4.1,ssse3"), always_inline))

// Rounds 4g .. 4g+3 (g compile-time after unrolling).  The E register
// alternates between e[0] and e[1] every group.
TDL_SHA_TARGET inline void group1(Lane1& l, int g, const uint8_t* p, __m128i mask) {
  __m128i& cur = l.m[g & 3];
  if (g < 4) cur = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * g)), mask);
  __m128i& ec = l.e[g & 1];
  __m128i& en = l.e[(g + 1) & 1];
  if (g == 0) {
    ec = _mm_add_epi32(ec, cur);
  } else {
    ec = _mm_sha1nexte_epu32(ec, cur);
  }
  en = l.abcd;
  if (g >= 3 && g <= 18) l.m[(g + 1) & 3] = _mm_sha1msg2_epu32(l.m[(g + 1) & 3], cur);
  switch (g / 5) {  // the round function index must be an immediate
    case 0: l.abcd = _mm_sha1rnds4_epu32(l.abcd, ec, 0); break;
    case 1: l.abcd = _mm_sha1rnds4_epu32(l.abcd, ec, 1); break;
    case 2: l.abcd = _mm_sha1rnds4_epu32(l.abcd, ec, 2); break;
    default: l.abcd = _mm_sha1rnds4_epu32(l.abcd, ec, 3); break;
  }
  if (g >= 1 && g <= 16) l.m[(g + 3) & 3] = _mm_sha1msg1_epu32(l.m[(g + 3) & 3], cur);
  if (g >= 2 && g <= 17) l.m[(g + 2) & 3] = _mm_xor_si128(l.m[(g + 2) & 3], cur);
}

__attribute__((target("sha,sse4.1,ssse3"))) inline void sha1_blocks_x1(uint32_t st[5], const uint8_t* p, size_t n) {
  const __m128i mask = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
  Lane1 a;
  a.abcd = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(st)), 0x1B);
  a.e[0] = _mm_set_epi32(int(st[4]), 0, 0, 0);
  for (; n; --n, p += 64) {
    const __m128i abcd0 = a.abcd, e0 = a.e[0];
#pragma GCC unroll 20
    for (int g = 0; g < 20; ++g) group1(a, g, p, mask);
    a.e[0] = _mm_sha1nexte_epu32(a.e[0], e0);
    a.abcd = _mm_add_epi32(a.abcd, abcd0);
  }
  _mm_storeu_si128(reinterpret_cast<__m128i*>(st), _mm_shuffle_epi32(a.abcd, 0x1B));
  st[4] = uint32_t(_mm_extract_epi32(a.e[0], 3));
}

__attribute__((target("sha,sse4.1,ssse3"))) inline void sha1_blocks_x2(uint32_t sa[5], uint32_t sb[5],
                                                                      const uint8_t* pa, const uint8_t* pb,
                                                                      size_t n) {
  const __m128i mask = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
  Lane1 a, b;
  a.abcd = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(sa)), 0x1B);
  a.e[0] = _mm_set_epi32(int(sa[4]), 0, 0, 0);
  b.abcd = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(sb)), 0x1B);
  b.e[0] = _mm_set_epi32(int(sb[4]), 0, 0, 0);
  for (; n; --n, pa += 64, pb += 64) {
    const __m128i a0 = a.abcd, ae = a.e[0], b0 = b.abcd, be = b.e[0];
#pragma GCC unroll 20
    for (int g = 0; g < 20; ++g) {
      group1(a, g, pa, mask);
      group1(b, g, pb, mask);
    }
    a.e[0] = _mm_sha1nexte_epu32(a.e[0], ae);
    a.abcd = _mm_add_epi32(a.abcd, a0);
    b.e[0] = _mm_sha1nexte_epu32(b.e[0], be);
    b.abcd = _mm_add_epi32(b.abcd, b0);
  }
  _mm_storeu_si128(reinterpret_cast<__m128i*>(sa), _mm_shuffle_epi32(a.abcd, 0x1B));
  sa[4] = uint32_t(_mm_extract_epi32(a.e[0], 3));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(sb), _mm_shuffle_epi32(b.abcd, 0x1B));
  sb[4] = uint32_t(_mm_extract_epi32(b.e[0], 3));
}

#undef TDL_SHA_TARGET

static const uint32_t kH1[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};

inline void sha1_out(const uint32_t st[5], uint8_t out[20]) {
  for (int i = 0; i < 5; ++i) {
    out[4 * i] = uint8_t(st[i] >> 24);
    out[4 * i + 1] = uint8_t(st[i] >> 16);
    out[4 * i + 2] = uint8_t(st[i] >> 8);
    out[4 * i + 3] = uint8_t(st[i]);
  }
}

// SHA-1 of one message (SHA-NI required).
inline void sha1_x1(const void* data, size_t n, uint8_t out[20]) {
  uint32_t st[5];
  std::memcpy(st, kH1, sizeof st);
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const size_t full = n / 64;
  if (full) sha1_blocks_x1(st, p, full);
  uint8_t tail[128];
  const size_t nb = pad_tail(tail, p + full * 64, n - full * 64, n);  // same padding as SHA-256
  sha1_blocks_x1(st, tail, nb);
  sha1_out(st, out);
}

// SHA-1 of two messages in lockstep (SHA-NI required).
inline void sha1_x2(const void* da, size_t na, const void* db, size_t nb, uint8_t oa[20], uint8_t ob[20]) {
  uint32_t sa[5], sb[5];
  std::memcpy(sa, kH1, sizeof sa);
  std::memcpy(sb, kH1, sizeof sb);
  const uint8_t* pa = static_cast<const uint8_t*>(da);
  const uint8_t* pb = static_cast<const uint8_t*>(db);
  const size_t fa = na / 64, fb = nb / 64, both = fa < fb ? fa : fb;
  if (both) sha1_blocks_x2(sa, sb, pa, pb, both);
  if (fa > both) sha1_blocks_x1(sa, pa + both * 64, fa - both);
  if (fb > both) sha1_blocks_x1(sb, pb + both * 64, fb - both);
  uint8_t ta[128], tb[128];
  const size_t ka = pad_tail(ta, pa + fa * 64, na - fa * 64, na);
  const size_t kb = pad_tail(tb, pb + fb * 64, nb - fb * 64, nb);
  if (ka == kb) {
    sha1_blocks_x2(sa, sb, ta, tb, ka);
  } else {
    sha1_blocks_x1(sa, ta, ka);
    sha1_blocks_x1(sb, tb, kb);
  }
  sha1_out(sa, oa);
  sha1_out(sb, ob);
}

}  // namespace sha2x
}  // namespace tritondl_hash
