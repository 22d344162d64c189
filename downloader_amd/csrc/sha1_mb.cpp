// 16-lane multi-buffer SHA-1 (AVX-512F): one message per 32-bit lane of a zmm register.
//
// Torrent piece verification hashes many independent, equally long messages (the pieces),
// which is the shape multi-buffer hashing wants: the 80 dependent rounds of one SHA-1 block
// are a serial chain that SHA-NI runs at ~2.5 cycles/byte, while 16 chains side by side keep
// every vector pipe busy. Round functions are single vpternlogd ops (0xCA choose, 0x96
// parity, 0xE8 majority), rotates are vprold. Messages are read 64 bytes per lane per block
// and transposed 16x16 in registers. Lanes whose message is shorter finish early and are
// masked; the caller pads the tail (SHA-1 padding) itself per lane.
#include "native.h"

#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

namespace stager {

namespace {

#define MB_TARGET __attribute__((target("avx512f,avx512bw")))

MB_TARGET inline __m512i rol(__m512i x, int n) {
  switch (n) {  // vprold takes an immediate
    case 1: return _mm512_rol_epi32(x, 1);
    case 5: return _mm512_rol_epi32(x, 5);
    default: return _mm512_rol_epi32(x, 30);
  }
}

// 16x16 dword transpose of rows r[0..15] (row i = lane i's 16 message words) in place.
MB_TARGET inline void transpose16(__m512i r[16]) {
  __m512i t[16];
  for (int i = 0; i < 16; i += 2) {
    t[i] = _mm512_unpacklo_epi32(r[i], r[i + 1]);
    t[i + 1] = _mm512_unpackhi_epi32(r[i], r[i + 1]);
  }
  for (int i = 0; i < 16; i += 4) {
    r[i] = _mm512_unpacklo_epi64(t[i], t[i + 2]);
    r[i + 1] = _mm512_unpackhi_epi64(t[i], t[i + 2]);
    r[i + 2] = _mm512_unpacklo_epi64(t[i + 1], t[i + 3]);
    r[i + 3] = _mm512_unpackhi_epi64(t[i + 1], t[i + 3]);
  }
  // r[4g + k] now holds, per 128-bit lane j, words (4j + ...) of rows 4g..4g+3; shuffle the
  // 128-bit lanes across groups.
  for (int k = 0; k < 4; ++k) {
    __m512i a = r[k], b = r[4 + k], c = r[8 + k], d = r[12 + k];
    __m512i ab_lo = _mm512_shuffle_i32x4(a, b, 0x44), ab_hi = _mm512_shuffle_i32x4(a, b, 0xEE);
    __m512i cd_lo = _mm512_shuffle_i32x4(c, d, 0x44), cd_hi = _mm512_shuffle_i32x4(c, d, 0xEE);
    t[k] = _mm512_shuffle_i32x4(ab_lo, cd_lo, 0x88);
    t[4 + k] = _mm512_shuffle_i32x4(ab_lo, cd_lo, 0xDD);
    t[8 + k] = _mm512_shuffle_i32x4(ab_hi, cd_hi, 0x88);
    t[12 + k] = _mm512_shuffle_i32x4(ab_hi, cd_hi, 0xDD);
  }
  // t[4q + k] = words (4q + k) of all 16 rows: column-major order
  for (int i = 0; i < 16; ++i) r[i] = t[i];
}

}  // namespace

// Compress `nblocks` 64-byte blocks of each lane's message into state[5] (16 lanes each).
// ptr[l] points at lane l's next block; lanes with active bit clear are left unchanged and
// read only ptr[l][0..63] (callers point idle lanes at a dummy block).
MB_TARGET void sha1_mb16_blocks(uint32_t state[5][16], const uint8_t* const ptr[16],
                                size_t nblocks, uint16_t active) {
  const __m512i bswap = _mm512_set_epi8(
      60, 61, 62, 63, 56, 57, 58, 59, 52, 53, 54, 55, 48, 49, 50, 51, 44, 45, 46, 47, 40, 41, 42,
      43, 36, 37, 38, 39, 32, 33, 34, 35, 28, 29, 30, 31, 24, 25, 26, 27, 20, 21, 22, 23, 16, 17,
      18, 19, 12, 13, 14, 15, 8, 9, 10, 11, 4, 5, 6, 7, 0, 1, 2, 3);
  const __mmask16 m = active;
  __m512i A = _mm512_loadu_si512(state[0]), B = _mm512_loadu_si512(state[1]),
          C = _mm512_loadu_si512(state[2]), D = _mm512_loadu_si512(state[3]),
          E = _mm512_loadu_si512(state[4]);
  const __m512i K0 = _mm512_set1_epi32(0x5A827999), K1 = _mm512_set1_epi32(0x6ED9EBA1),
                K2 = _mm512_set1_epi32((int)0x8F1BBCDC), K3 = _mm512_set1_epi32((int)0xCA62C1D6);
  for (size_t blk = 0; blk < nblocks; ++blk) {
    __m512i W[16];
    for (int l = 0; l < 16; ++l)   // idle lanes re-read their (dummy) block: no advance
      W[l] = _mm512_shuffle_epi8(
          _mm512_loadu_si512(ptr[l] + ((active >> l) & 1 ? blk * 64 : 0)), bswap);
    transpose16(W);
    __m512i a = A, b = B, c = C, d = D, e = E;
#define SHA1_ROUND(t, F, K)                                                             \
  {                                                                                     \
    __m512i w;                                                                          \
    if ((t) < 16) {                                                                     \
      w = W[(t)];                                                                       \
    } else {                                                                            \
      w = rol(_mm512_ternarylogic_epi32(W[((t) - 3) & 15], W[((t) - 8) & 15],          \
                                        W[((t) - 14) & 15], 0x96) ^ W[(t) & 15], 1);    \
      W[(t) & 15] = w;                                                                  \
    }                                                                                   \
    __m512i f = _mm512_ternarylogic_epi32(b, c, d, F);                                  \
    __m512i tmp = _mm512_add_epi32(_mm512_add_epi32(rol(a, 5), f),                      \
                                   _mm512_add_epi32(_mm512_add_epi32(e, K), w));        \
    e = d;                                                                              \
    d = c;                                                                              \
    c = rol(b, 30);                                                                     \
    b = a;                                                                              \
    a = tmp;                                                                            \
  }
#pragma GCC unroll 20
    for (int t = 0; t < 20; ++t) SHA1_ROUND(t, 0xCA, K0)
#pragma GCC unroll 20
    for (int t = 20; t < 40; ++t) SHA1_ROUND(t, 0x96, K1)
#pragma GCC unroll 20
    for (int t = 40; t < 60; ++t) SHA1_ROUND(t, 0xE8, K2)
#pragma GCC unroll 20
    for (int t = 60; t < 80; ++t) SHA1_ROUND(t, 0x96, K3)
#undef SHA1_ROUND
    A = _mm512_mask_add_epi32(A, m, A, a);
    B = _mm512_mask_add_epi32(B, m, B, b);
    C = _mm512_mask_add_epi32(C, m, C, c);
    D = _mm512_mask_add_epi32(D, m, D, d);
    E = _mm512_mask_add_epi32(E, m, E, e);
  }
  _mm512_storeu_si512(state[0], A);
  _mm512_storeu_si512(state[1], B);
  _mm512_storeu_si512(state[2], C);
  _mm512_storeu_si512(state[3], D);
  _mm512_storeu_si512(state[4], E);
}

void sha1x16_init(uint32_t st[5][16]) {
  const uint32_t init[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  for (int j = 0; j < 5; ++j)
    for (int l = 0; l < 16; ++l) st[j][l] = init[j];
}

void sha1x16_finish(uint32_t st[5][16], const uint8_t* const tails[16], size_t tail_len,
                    uint64_t total_len, uint16_t active, uint8_t* out) {
  static const uint8_t zero_block[64] = {0};
  const size_t tb = tail_len < 56 ? 1 : 2;
  alignas(64) uint8_t pad[16][128];
  const uint8_t* p[16];
  for (int l = 0; l < 16; ++l) {
    if (!((active >> l) & 1)) {
      p[l] = zero_block;
      continue;
    }
    std::memset(pad[l], 0, tb * 64);
    std::memcpy(pad[l], tails[l], tail_len);
    pad[l][tail_len] = 0x80;
    const uint64_t bits = total_len * 8;
    for (int i = 0; i < 8; ++i) pad[l][tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    p[l] = pad[l];
  }
  sha1_mb16_blocks(st, p, tb, active);
  for (int l = 0; l < 16; ++l) {
    if (!((active >> l) & 1)) continue;
    for (int j = 0; j < 5; ++j) {
      const uint32_t v = st[j][l];
      uint8_t* o = out + 20 * l + 4 * j;
      o[0] = (uint8_t)(v >> 24);
      o[1] = (uint8_t)(v >> 16);
      o[2] = (uint8_t)(v >> 8);
      o[3] = (uint8_t)v;
    }
  }
}

bool sha1_mb_supported() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  return ok;
}

// SHA-1 of n messages msgs[i] (lengths lens[i]) into out (20 bytes each), 16 at a time.
// Lanes of a group run in lockstep over their common block count; each lane's own tail
// (and SHA-1 padding) is finished in a second, short masked pass.
void sha1_mb(const uint8_t* const* msgs, const size_t* lens, size_t n, uint8_t* out) {
  static const uint8_t zero_block[128] = {0};
  for (size_t g = 0; g < n; g += 16) {
    const size_t k = std::min<size_t>(16, n - g);
    uint32_t st[5][16];
    const uint32_t init[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    for (int j = 0; j < 5; ++j)
      for (int l = 0; l < 16; ++l) st[j][l] = init[j];
    // 1) whole blocks every lane of the group has
    size_t common = SIZE_MAX;
    for (size_t l = 0; l < k; ++l) common = std::min(common, lens[g + l] / 64);
    const uint8_t* p[16];
    for (int l = 0; l < 16; ++l) p[l] = (size_t)l < k ? msgs[g + l] : zero_block;
    const uint16_t all = (uint16_t)((1u << k) - 1);
    if (common) sha1_mb16_blocks(st, p, common, all);
    // 2) per lane: remaining whole blocks + padded tail, as up to `rem` masked rounds
    uint8_t tail[16][128 + 64];
    size_t left[16] = {0};   // blocks still to run per lane (whole + 1 or 2 tail blocks)
    const uint8_t* whole[16];
    size_t nwhole[16] = {0};
    for (size_t l = 0; l < k; ++l) {
      const size_t len = lens[g + l];
      const size_t done = common * 64;
      nwhole[l] = len / 64 - common;
      whole[l] = msgs[g + l] + done;
      const size_t r = len % 64;
      const size_t tb = r < 56 ? 1 : 2;
      std::memset(tail[l], 0, tb * 64);
      std::memcpy(tail[l], msgs[g + l] + (len - r), r);
      tail[l][r] = 0x80;
      const uint64_t bits = (uint64_t)len * 8;
      for (int i = 0; i < 8; ++i) tail[l][tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
      left[l] = nwhole[l] + tb;
    }
    for (size_t step = 0;; ++step) {
      uint16_t act = 0;
      for (size_t l = 0; l < k; ++l) {
        if (step < left[l]) {
          act |= (uint16_t)(1u << l);
          p[l] = step < nwhole[l] ? whole[l] + step * 64 : tail[l] + (step - nwhole[l]) * 64;
        } else {
          p[l] = zero_block;
        }
      }
      if (!act) break;
      sha1_mb16_blocks(st, p, 1, act);
    }
    for (size_t l = 0; l < k; ++l)
      for (int j = 0; j < 5; ++j) {
        const uint32_t v = st[j][l];
        uint8_t* o = out + 20 * (g + l) + 4 * j;
        o[0] = (uint8_t)(v >> 24);
        o[1] = (uint8_t)(v >> 16);
        o[2] = (uint8_t)(v >> 8);
        o[3] = (uint8_t)v;
      }
  }
}

}  // namespace stager
