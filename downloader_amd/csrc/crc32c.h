// CRC32C (Castagnoli): AVX-512 VPCLMULQDQ folding for long buffers where the CPU has it, else
// the SSE4.2 crc32 instruction in three interleaved chains.
//
// S3's flexible payload checksum (x-amz-checksum-crc32c) is what the staging path sends per
// PUT / part instead of minio-js' Content-MD5: MD5 runs at ~0.7 GB/s per core,
// one crc32 chain at ~8 bytes / 3 cycles, and three independent chains over adjacent blocks
// keep the crc32 unit busy every cycle (~20-30 GB/s per core). The chains are merged with
// "shift by L zero bytes" operators, which are linear in the CRC state and so reduce to four
// 256-entry tables per block length (built once from the hardware instruction itself).
//
// Shared by the native module (csrc/hashing.cpp, csrc/transfer.cpp) and blobd (the bench's
// S3 sink verifies what the worker sends). Header-only; needs -msse4.2 (x86-64-v3 has it).
#pragma once

#include <immintrin.h>
#include <nmmintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace crc32c_detail {

constexpr size_t kLong = 8192;   // bytes per chain in the long loop
constexpr size_t kShort = 256;   // ... in the short loop

struct ShiftTable {
  uint32_t t[4][256];
};

// Raw (no pre/post inversion) CRC state after `len` zero bytes, starting from `c`.
inline uint32_t zeros_raw(uint32_t c, size_t len) {
  uint64_t s = c;
  size_t i = 0;
  for (; i + 8 <= len; i += 8) s = _mm_crc32_u64(s, 0);
  for (; i < len; ++i) s = _mm_crc32_u8((uint32_t)s, 0);
  return (uint32_t)s;
}

inline void build(ShiftTable& st, size_t len) {
  uint32_t basis[32];
  for (int k = 0; k < 32; ++k) basis[k] = zeros_raw(1u << k, len);
  for (int j = 0; j < 4; ++j)
    for (int b = 0; b < 256; ++b) {
      uint32_t v = 0;
      for (int bit = 0; bit < 8; ++bit)
        if (b & (1 << bit)) v ^= basis[8 * j + bit];
      st.t[j][b] = v;
    }
}

inline const ShiftTable& table(size_t len) {
  static const ShiftTable* lt = [] {
    auto* t = new ShiftTable;
    build(*t, kLong);
    return t;
  }();
  static const ShiftTable* sh = [] {
    auto* t = new ShiftTable;
    build(*t, kShort);
    return t;
  }();
  return len == kLong ? *lt : *sh;
}

inline uint32_t shift(const ShiftTable& st, uint32_t c) {
  return st.t[0][c & 0xff] ^ st.t[1][(c >> 8) & 0xff] ^ st.t[2][(c >> 16) & 0xff] ^ st.t[3][c >> 24];
}

template <size_t L>
inline void three_way(uint64_t& c0, const uint8_t*& p, size_t& n) {
  const ShiftTable& st = table(L);
  while (n >= 3 * L) {
    uint64_t c1 = 0, c2 = 0;
    for (size_t i = 0; i < L; i += 8) {
      uint64_t a, b, d;
      memcpy(&a, p + i, 8);
      memcpy(&b, p + L + i, 8);
      memcpy(&d, p + 2 * L + i, 8);
      c0 = _mm_crc32_u64(c0, a);
      c1 = _mm_crc32_u64(c1, b);
      c2 = _mm_crc32_u64(c2, d);
    }
    c0 = shift(st, (uint32_t)c0) ^ (uint32_t)c1;
    c0 = shift(st, (uint32_t)c0) ^ (uint32_t)c2;
    p += 3 * L;
    n -= 3 * L;
  }
}

// ---- AVX-512 VPCLMULQDQ folding (hosts that have it: Zen 4/5, Ice Lake and later) ------
// Carry-less-multiply folding (Intel, "Fast CRC Computation Using PCLMULQDQ"), four 512-bit
// accumulators = 256 bytes per iteration, then folded down to 128 bits whose raw CRC (two
// crc32 instructions) is the CRC state - no Barrett reduction. Fold constants are
// reflect32(x^(d+32) mod P) << 1 (multiplies the low qword) and reflect32(x^(d-32) mod P) << 1
// (the high qword) for a fold distance of d bits; for P = CRC32C (0x1EDC6F41):
//   d = 2048: 0x0dcb17aa4, 0x0b9e02b86   d = 512: 0x0740eef02, 0x09e4addf8
//   d = 128:  0x0f20c0dfe, 0x14cd00bd6
// (the same generator reproduces zlib-ng's published gzip-CRC32 constants; the result is
// checked against a bitwise reference in tests/test_integrity.py).
#define CRC32C_AVX512 __attribute__((target("avx512f,avx512bw,avx512dq,avx512vl,vpclmulqdq,pclmul,sse4.2")))

CRC32C_AVX512 inline __m512i fold_zmm(__m512i x, __m512i k, __m512i d) {
  return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00),
                                   _mm512_clmulepi64_epi128(x, k, 0x11), d, 0x96);
}

CRC32C_AVX512 inline __m128i fold_xmm(__m128i y, __m128i k, __m128i d) {
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(y, k, 0x00),
                                     _mm_clmulepi64_si128(y, k, 0x11)), d);
}

CRC32C_AVX512 inline uint64_t fold512(uint64_t state, const uint8_t*& p, size_t& n) {
  const __m512i k2048 = _mm512_set_epi64(0x0b9e02b86LL, 0x0dcb17aa4LL, 0x0b9e02b86LL, 0x0dcb17aa4LL,
                                         0x0b9e02b86LL, 0x0dcb17aa4LL, 0x0b9e02b86LL, 0x0dcb17aa4LL);
  const __m512i k512 = _mm512_set_epi64(0x09e4addf8LL, 0x0740eef02LL, 0x09e4addf8LL, 0x0740eef02LL,
                                        0x09e4addf8LL, 0x0740eef02LL, 0x09e4addf8LL, 0x0740eef02LL);
  const __m128i k128 = _mm_set_epi64x(0x14cd00bd6LL, 0x0f20c0dfeLL);
  __m512i x0 = _mm512_loadu_si512((const void*)p);
  __m512i x1 = _mm512_loadu_si512((const void*)(p + 64));
  __m512i x2 = _mm512_loadu_si512((const void*)(p + 128));
  __m512i x3 = _mm512_loadu_si512((const void*)(p + 192));
  x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)(uint32_t)state)));
  p += 256;
  n -= 256;
  while (n >= 256) {
    x0 = fold_zmm(x0, k2048, _mm512_loadu_si512((const void*)p));
    x1 = fold_zmm(x1, k2048, _mm512_loadu_si512((const void*)(p + 64)));
    x2 = fold_zmm(x2, k2048, _mm512_loadu_si512((const void*)(p + 128)));
    x3 = fold_zmm(x3, k2048, _mm512_loadu_si512((const void*)(p + 192)));
    p += 256;
    n -= 256;
  }
  __m512i x = fold_zmm(x0, k512, x1);
  x = fold_zmm(x, k512, x2);
  x = fold_zmm(x, k512, x3);
  __m128i y = _mm512_extracti64x2_epi64(x, 0);
  y = fold_xmm(y, k128, _mm512_extracti64x2_epi64(x, 1));
  y = fold_xmm(y, k128, _mm512_extracti64x2_epi64(x, 2));
  y = fold_xmm(y, k128, _mm512_extracti64x2_epi64(x, 3));
  while (n >= 16) {
    y = fold_xmm(y, k128, _mm_loadu_si128((const __m128i*)p));
    p += 16;
    n -= 16;
  }
  uint64_t c = _mm_crc32_u64(0, (uint64_t)_mm_cvtsi128_si64(y));
  return _mm_crc32_u64(c, (uint64_t)_mm_extract_epi64(y, 1));
}

inline bool have_vpclmul() {
  static const bool ok = __builtin_cpu_supports("vpclmulqdq") &&
                         __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") && __builtin_cpu_supports("avx512dq") &&
                         __builtin_cpu_supports("avx512vl");
  return ok;
}

}  // namespace crc32c_detail

// Standard CRC32C of `n` bytes continuing from `crc` (0 for a fresh stream): the value S3
// expects base64-encoded (big-endian) in x-amz-checksum-crc32c.
inline uint32_t crc32c_update(uint32_t crc, const void* data, size_t n) {
  const uint8_t* p = (const uint8_t*)data;
  uint64_t c = (uint32_t)~crc;
  if (n >= 1024 && crc32c_detail::have_vpclmul()) c = crc32c_detail::fold512(c, p, n);
  while (n && ((uintptr_t)p & 7)) {
    c = _mm_crc32_u8((uint32_t)c, *p++);
    --n;
  }
  crc32c_detail::three_way<crc32c_detail::kLong>(c, p, n);
  crc32c_detail::three_way<crc32c_detail::kShort>(c, p, n);
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  while (n--) c = _mm_crc32_u8((uint32_t)c, *p++);
  return ~(uint32_t)c;
}

// base64 of the big-endian CRC (8 characters), as in x-amz-checksum-crc32c.
inline void crc32c_b64(uint32_t crc, char out[9]) {
  static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  const uint8_t b[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8), (uint8_t)crc};
  out[0] = A[b[0] >> 2];
  out[1] = A[((b[0] & 3) << 4) | (b[1] >> 4)];
  out[2] = A[((b[1] & 15) << 2) | (b[2] >> 6)];
  out[3] = A[b[2] & 63];
  out[4] = A[b[3] >> 2];
  out[5] = A[(b[3] & 3) << 4];
  out[6] = '=';
  out[7] = '=';
  out[8] = 0;
}
