// Batched SHA-1 torrent piece verification on the MI355X (gfx950).
//
// The reference verifies every BitTorrent piece with SHA-1 inside webtorrent
// (simple-sha1 -> Node crypto; reference lib/download.js:64 `client.add`).
// Here a full-torrent verification / recheck can be offloaded to the GPU:
//
//   * SHA-1 is a serial chain over 64-byte blocks inside one piece, so the unit of
//     parallelism is the piece: ONE LANE PER PIECE, 64 pieces per wavefront. Per-lane work is
//     ~616 VALU ops per 64-byte block (80 rounds with v_alignbit rotates, v_bfi for Ch and
//     v_bitop3 for parity/majority, plus the message schedule). Each lane loads block k+1
//     into registers while it hashes block k (sha1_run16): without that every block waited
//     for its own global loads and one wave per SIMD had nothing to hide the wait with.
//     Measured (profiles/archive/r2_kpf, kernel A/B in one process): ~58 MB/s per lane with the
//     prefetch vs ~43 MB/s without (1.37x; ~2,600 cycles per block, 95 % of the 4-cycle
//     VALU issue bound), so throughput is pieces-in-flight x 58 MB/s: ~930 GB/s at 16k
//     pieces (one wave per CU - a quarter of the SIMDs), ~234 GB/s
//     at 4k. Real torrents have 1k-20k pieces, and the host path that feeds the kernel
//     (pread into pinned slots + PCIe Gen5 x16, ~57 GB/s DMA measured) is the bound.
//   * Each lane streams its own piece with 16-byte global loads (4 x dwordx4 per block). The
//     64 lanes of a wave touch 64 different lines per load, but each line is fully consumed
//     by the lane's next load, so the L1/L2 absorb it (no LDS staging needed: the kernel is
//     ALU-bound per lane, not bandwidth-bound).
//   * Grid: 64-lane workgroups (one wave each), so 16k pieces spread over 256 workgroups =
//     every CU; consecutive workgroups land on different XCDs round-robin. No block-to-XCD
//     remapping: lanes share no data (each reads only its own piece once), so there is no
//     L2 reuse for an XCD-aware order to keep local.
//   * The host driver double-buffers pinned staging buffers: reader threads pread() batch
//     i+1 from the page cache while batch i is copied (hipMemcpyAsync) and hashed on its own
//     HIP stream; digests are compared on the device and only one byte per piece returns.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <mutex>
#include <exception>
#include <stdexcept>
#include <string>
#include <pthread.h>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

#include "gpu_part_api.h"
#include "part_dispatch.h"

namespace py = pybind11;

#define HIP_CHECK(x)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + \
                               #x);                                                       \
  } while (0)

namespace {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, 32 - n);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// gfx950 (CDNA4) V_BITOP3_B32: any 3-input bitwise function in one VALU op, selected by an
// 8-bit truth table. Only symmetric tables are used here (operand order cannot matter):
//   0x96 = a ^ b ^ c (SHA-1 parity rounds, message schedule), 0xE8 = majority(a, b, c).
// hipcc does not form these from plain C (no v_xor3 on gfx950 either), so they are emitted
// directly; this removes ~1/6 of the VALU ops per 64-byte block.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

struct Sha1State {
  uint32_t h0, h1, h2, h3, h4;
};

#define SHA1_ROUND(t, F, K)                                              \
  {                                                                      \
    uint32_t tmp = rotl(a, 5) + (F) + e + (K) + w[(t)&15];               \
    e = d;                                                               \
    d = c;                                                               \
    c = rotl(b, 30);                                                     \
    b = a;                                                               \
    a = tmp;                                                             \
  }

// B3 = true: gfx950 v_bitop3 forms; false: plain C (kept for the in-process A/B benchmark).
template <bool B3>
__device__ __forceinline__ uint32_t par3(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (B3) return xor3(a, b, c);
  return a ^ b ^ c;
}
template <bool B3>
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (B3) return maj(a, b, c);
  return (a & b) | (a & c) | (b & c);
}

template <bool B3>
__device__ __forceinline__ void sha1_block(Sha1State& s, uint32_t w[16]) {
  uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    if (t >= 16)
      w[t & 15] = rotl(par3<B3>(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
    if (t < 20) {
      SHA1_ROUND(t, (b & c) | (~b & d), 0x5A827999u);  // -> v_bfi_b32
    } else if (t < 40) {
      SHA1_ROUND(t, par3<B3>(b, c, d), 0x6ED9EBA1u);
    } else if (t < 60) {
      SHA1_ROUND(t, maj3<B3>(b, c, d), 0x8F1BBCDCu);
    } else {
      SHA1_ROUND(t, par3<B3>(b, c, d), 0xCA62C1D6u);
    }
  }
  s.h0 += a;
  s.h1 += b;
  s.h2 += c;
  s.h3 += d;
  s.h4 += e;
}

// ALIGN: 16 -> dwordx4 loads, 4 -> dword loads, 1 -> byte loads.
template <int ALIGN>
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t w[16]) {
  if constexpr (ALIGN == 16) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 v = q[i];
      w[4 * i + 0] = bswap(v.x);
      w[4 * i + 1] = bswap(v.y);
      w[4 * i + 2] = bswap(v.z);
      w[4 * i + 3] = bswap(v.w);
    }
  } else if constexpr (ALIGN == 4) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = bswap(q[i]);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
             ((uint32_t)p[4 * i + 2] << 8) | (uint32_t)p[4 * i + 3];
  }
}

// Raw 64-byte block as four dwordx4 loads, and its conversion to big-endian words: split so
// the loads of block k+1 can be issued before block k is hashed (see sha1_run16).
__device__ __forceinline__ void load_raw16(const uint8_t* p, uint4 v[4]) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = q[i];
}
__device__ __forceinline__ void to_words(const uint4 v[4], uint32_t w[16]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[4 * i + 0] = bswap(v[i].x);
    w[4 * i + 1] = bswap(v[i].y);
    w[4 * i + 2] = bswap(v[i].z);
    w[4 * i + 3] = bswap(v[i].w);
  }
}

// `nblk` whole blocks at p (16-byte aligned) into s. PF: software-prefetch block k+1 into
// registers while block k is hashed. Without it every block waited for its own loads right
// before its first round (s_waitcnt vmcnt(0) at the loop head: ~550 - 900 cycles of an L2 /
// HBM miss on top of ~2,500 cycles of VALU issue), and with one wave per SIMD nothing else
// hides that wait.
template <bool B3, bool PF>
__device__ __forceinline__ void sha1_run16(Sha1State& s, const uint8_t* p, int64_t nblk) {
  uint32_t w[16];
  if constexpr (!PF) {
    for (int64_t blk = 0; blk < nblk; ++blk) {
      load_block<16>(p + (blk << 6), w);
      sha1_block<B3>(s, w);
    }
  } else {
    // Two register buffers with fixed roles (no cur = nxt copy: a move out of a register
    // with a load in flight waits for that load, which is what the prefetch is to avoid).
    // The second load of a pair is clamped to the last block, so it is always in bounds
    // and needs no branch; the duplicate 64 bytes per piece are never hashed.
    if (nblk <= 0) return;
    uint4 a[4], b[4];
    load_raw16(p, a);
    int64_t blk = 0;
    for (; blk + 2 <= nblk; blk += 2) {
      load_raw16(p + ((blk + 1) << 6), b);
      to_words(a, w);
      sha1_block<B3>(s, w);
      const int64_t n2 = blk + 2 < nblk ? blk + 2 : nblk - 1;
      load_raw16(p + (n2 << 6), a);
      to_words(b, w);
      sha1_block<B3>(s, w);
    }
    if (blk < nblk) {
      to_words(a, w);
      sha1_block<B3>(s, w);
    }
  }
}

// SHA-1 of `len` bytes at p (one lane, one piece): whole blocks, then tail + padding.
template <int ALIGN, bool B3, bool PF>
__device__ __forceinline__ void sha1_piece(const uint8_t* p, int64_t len, uint32_t hv[5]) {
  Sha1State s{0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint32_t w[16];
  const int64_t nfull = len >> 6;
  if constexpr (ALIGN == 16) {
    sha1_run16<B3, PF>(s, p, nfull);
  } else {
    for (int64_t blk = 0; blk < nfull; ++blk) {
      load_block<ALIGN>(p + (blk << 6), w);
      sha1_block<B3>(s, w);
    }
  }
  // Tail + padding (one or two blocks), built word by word straight into w[] - no byte
  // array, so the padding logic costs no extra registers or scratch.
  const int rem = (int)(len & 63);
  const uint8_t* tail = p + (nfull << 6);
  const uint64_t bits = (uint64_t)len * 8ull;
  const int nb = rem >= 56 ? 2 : 1;
  for (int b = 0; b < nb; ++b) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int idx = b * 64 + 4 * i + k;
        uint32_t byte = idx < rem ? (uint32_t)tail[idx] : (idx == rem ? 0x80u : 0u);
        v |= byte << (24 - 8 * k);
      }
      w[i] = v;
    }
    if (b == nb - 1) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha1_block<B3>(s, w);
  }
  hv[0] = s.h0;
  hv[1] = s.h1;
  hv[2] = s.h2;
  hv[3] = s.h3;
  hv[4] = s.h4;
}

__device__ __forceinline__ void store_digest(uint8_t* o, const uint32_t hv[5]) {
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    o[4 * k] = (uint8_t)(hv[k] >> 24);
    o[4 * k + 1] = (uint8_t)(hv[k] >> 16);
    o[4 * k + 2] = (uint8_t)(hv[k] >> 8);
    o[4 * k + 3] = (uint8_t)hv[k];
  }
}

// One lane hashes one piece. data holds n_pieces consecutive pieces of piece_len bytes,
// the last one possibly `last_len` bytes. If `expected` is non-null, ok[i] = digest matches,
// otherwise digests are written to `out` (5 words, big-endian byte order as bytes).
template <int ALIGN, bool B3 = true, bool PF = true>
__global__ __launch_bounds__(256) void sha1_pieces(const uint8_t* __restrict__ data,
                                                   int64_t piece_len, int64_t last_len,
                                                   int n_pieces,
                                                   const uint8_t* __restrict__ expected,
                                                   uint8_t* __restrict__ ok,
                                                   uint8_t* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pieces) return;
  const int64_t len = (i == n_pieces - 1) ? last_len : piece_len;
  uint32_t hv[5];
  sha1_piece<ALIGN, B3, PF>(data + (int64_t)i * piece_len, len, hv);
  if (expected) {
    const uint8_t* ex = expected + (int64_t)i * 20;
    bool good = true;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      uint32_t e = ((uint32_t)ex[4 * k] << 24) | ((uint32_t)ex[4 * k + 1] << 16) |
                   ((uint32_t)ex[4 * k + 2] << 8) | (uint32_t)ex[4 * k + 3];
      good = good && (e == hv[k]);
    }
    ok[i] = good ? 1 : 0;
  } else {
    store_digest(out + (int64_t)i * 20, hv);
  }
}

// Batch of relayed parts (PartHasher): lane i hashes lane_len[i] bytes at data + lane_off[i].
// `data` is the base of the hasher's HBM arena (every slot is a window of one allocation), so
// one launch spans the pieces of several slots - every slot that closed while the compute
// streams were busy - and the loads stay global_load_dwordx4: an absolute address per lane
// made them flat loads (a generic pointer), and the kernel 26 % slower (97.8 vs 77.7 ms per
// 4 MiB piece, profiles/r6/parthasher/trace_summary.json).
template <int ALIGN>
__global__ __launch_bounds__(256) void sha1_lanes(const uint8_t* __restrict__ data,
                                                  const int64_t* __restrict__ lane_off,
                                                  const int64_t* __restrict__ lane_len, int n,
                                                  uint8_t* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t hv[5];
  sha1_piece<ALIGN, true, ALIGN == 16>(data + lane_off[i], lane_len[i], hv);
  store_digest(out + (int64_t)i * 20, hv);
}

// ---------------------------------------------------------------------------------------
// Split-wave variant of sha1_lanes: the same batch, every 64 pieces hashed by THREE waves.
//
// One lane of one wave is a serial chain of ~618 VALU ops per 64-byte block, and a wave alone
// on its SIMD issues one wave64 VALU op per ~4 cycles (MI355X_MICROARCH.md, 'vector-instruction
// ISSUE cost'), so a 4 MiB piece takes 65,536 blocks x ~2,650 cycles = 73 ms however idle the
// rest of the device is. In the PartHasher and the swarm that per-piece LATENCY - not the
// device's throughput - is what lands on the end of a job. ~210 of
// those ops per block are the message schedule (W[16..79] = rotl1 of four older words) and the
// byte swaps, which do not depend on the hash state. So a workgroup here is three waves on
// three SIMDs (a workgroup's waves are dealt to SIMDs 0 -> 2 -> 1 -> 3) for the same 64 pieces:
//   * waves 0 and 1, the producers, take the even / odd blocks: in its step a producer swaps
//     its block (dwordx4 loads issued two steps ahead), expands the 80-word schedule and, at
//     the end of the step, writes it to an LDS slot (20 ds_write_b128 per lane: lane l's
//     16-byte group g at ((slot * 20 + g) * 64 + l) - conflict-free); then it idles a step.
//     One producer doing that in every step took ~1,560 cycles per block alone (timed with
//     the rounds taken out: the 20 wide LDS stores of one wave cost ~26 cycles each on top of
//     its ~300 VALU ops) - as long as the rounds, so that pair was no faster than either;
//   * wave 2, the consumer, reads block k + 1's 80 words (20 ds_read_b128) while it runs only
//     the 80 rounds of block k: Ch / parity / majority (v_bitop3), rotl5, rotl30 and two add3
//     (K folds in) - 5 ops per round instead of ~7.7;
//   * one s_barrier per block.
// Lanes of one workgroup may have different lengths: every wave steps through the workgroup's
// longest lane (every wave reaches every barrier), lanes past their own end idle.
constexpr size_t kArenaPad = 256;             // bytes readable past a split launch's data
constexpr int kSplitGroups = 20;              // 80 schedule words = 20 x uint4 per lane per block
// LDS ring: blocks k + 1 (read) and k + 2 (written) of step k, and spare slots. 4 slots = 80 KiB
// (+ 4 bytes) of LDS per workgroup, so at most ONE workgroup fits a CU (160 KiB): the
// PartHasher's two compute streams run launches side by side, and with 60 KiB two of their
// workgroups could land on one CU, their 6 waves on its 4 SIMDs (rocprofv3: 52.7 - 106 ms per
// launch, 68.7 mean, vs 52.8 - 53.4 alone). 256 workgroups = 16,384 lanes still fit at once.
constexpr uint32_t kSplitSlots = 4;
constexpr int kSplitThreads = 192;            // two producer waves + one consumer wave
static_assert(2 * (kSplitSlots * kSplitGroups * 64 * 16 + 4) > 160 * 1024,
              "sha1_lanes_split must not fit twice on one CU");

// The 80-word schedule of one block from its 16 big-endian words.
__device__ __forceinline__ void split_schedule(uint32_t w[16], uint4 g[kSplitGroups]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) g[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
#pragma unroll
  for (int t = 16; t < 80; ++t) {
    w[t & 15] = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
    if ((t & 3) == 3)
      g[t >> 2] = make_uint4(w[(t - 3) & 15], w[(t - 2) & 15], w[(t - 1) & 15], w[t & 15]);
  }
}

// slot points at this lane's column of a ring slot: group q is slot[q * 64]
__device__ __forceinline__ void split_write(const uint4 g[kSplitGroups], uint4* __restrict__ slot) {
#pragma unroll
  for (int q = 0; q < kSplitGroups; ++q) slot[q * 64] = g[q];
}

__device__ __forceinline__ void split_read(const uint4* __restrict__ slot, uint4 g[kSplitGroups]) {
#pragma unroll
  for (int q = 0; q < kSplitGroups; ++q) g[q] = slot[q * 64];
}

__device__ __forceinline__ uint32_t split_word(const uint4 g[kSplitGroups], int t) {
  const uint4 v = g[t >> 2];
  return (t & 3) == 0 ? v.x : (t & 3) == 1 ? v.y : (t & 3) == 2 ? v.z : v.w;
}

#define SHA1_SPLIT_ROUND(F, K)                                            \
  {                                                                       \
    uint32_t tmp = rotl(a, 5) + (F) + (e + (K) + split_word(g, t));       \
    e = d;                                                                \
    d = c;                                                                \
    c = rotl(b, 30);                                                      \
    b = a;                                                                \
    a = tmp;                                                              \
  }

__device__ __forceinline__ void split_rounds(Sha1State& s, const uint4 g[kSplitGroups]) {
  uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    if (t < 20) {
      SHA1_SPLIT_ROUND((b & c) | (~b & d), 0x5A827999u);
    } else if (t < 40) {
      SHA1_SPLIT_ROUND(xor3(b, c, d), 0x6ED9EBA1u);
    } else if (t < 60) {
      SHA1_SPLIT_ROUND(maj(b, c, d), 0x8F1BBCDCu);
    } else {
      SHA1_SPLIT_ROUND(xor3(b, c, d), 0xCA62C1D6u);
    }
  }
  s.h0 += a;
  s.h1 += b;
  s.h2 += c;
  s.h3 += d;
  s.h4 += e;
}

// The last one or two blocks of a lane from the 64 raw bytes at its tail (rem < 64 of them
// belong to the piece): those bytes, 0x80, zero fill, and the bit length in the last block;
// `second` = the all-zero block that follows when rem >= 56.
__device__ __forceinline__ void tail_words(const uint4 v[4], int rem, bool last, bool second,
                                           uint64_t bits, uint32_t w[16]) {
  to_words(v, w);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = rem - 4 * i;                     // piece bytes left at word i
    const uint32_t keep = r >= 4 ? 0xFFFFFFFFu : r <= 0 ? 0u : 0xFFFFFFFFu << (32 - 8 * r);
    const uint32_t pad = (r >= 0 && r < 4) ? 0x80u << (24 - 8 * r) : 0u;
    w[i] = second ? 0u : ((w[i] & keep) | pad);
  }
  if (last) {
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
  }
}

// Workgroup barrier that waits for this wave's LDS traffic only: __syncthreads() also drains
// vmcnt, i.e. a producer's prefetch loads. The wait is the builtin (lgkmcnt(0), vmcnt / expcnt
// left at their maxima: 0xC07F on gfx9) so the compiler's own wait insertion knows every LDS
// access before it is done - inside an asm string it did not, and waited again at the next
// uses. The asm keeps the compiler from moving LDS accesses across the barrier.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  asm volatile("s_barrier" ::: "memory");
}

// Lane i of the batch = (lane_off[i], lane_len[i]) in the arena, 16-byte aligned; 192-thread
// workgroups (grid = ceil(n / 64)). Alternatives timed against this one in one process
// (kernel bench, 4 MiB pieces, 64 / 1,024 lanes; profiles/r6/split/kernel_knobs.jsonl): a
// producer that schedules in one step and writes in the next 60.9 - 61.2 ms, the consumer's
// next-block reads spread through its rounds (one per 4 rounds, pinned by sched_barrier)
// 60.7 - 60.9, both 60.8 - 61.5, the consumer at s_setprio 3 64.7 - 65.1, against 52.8 - 53.4
// here and 73.2 - 73.5 for sha1_lanes<16>. Two blocks per barrier (a ring of three pairs, both
// producers busy every step) came out 1.5 % slower, 58.0 - 58.5 vs 57.0 - 57.7 ms in one
// process (pair_per_barrier.jsonl): the barriers are not where the consumer's time goes.
template <bool DUP>
__global__ __launch_bounds__(192) void sha1_lanes_split_t(const uint8_t* __restrict__ data,
                                                          const int64_t* __restrict__ lane_off,
                                                          const int64_t* __restrict__ lane_len,
                                                          int n, uint8_t* __restrict__ out) {
  __shared__ uint4 ring[kSplitSlots * kSplitGroups * 64];    // 80 KiB: four blocks' schedules
  __shared__ uint32_t longest;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;               // 0, 1: producers (even / odd blocks); 2
  const int i0 = blockIdx.x * 64 + lane;
  const bool live = i0 < n;
  // DUP: a lane past n hashes a live lane's piece again (its digest is not stored), so every
  // lane of every wave is busy. A launch whose waves were partly empty took far longer - 1 /
  // 8 / 16 / 32 live lanes of 64: 86 / 81 / 77 / 59 ms per 4 MiB piece, 80 lanes 74 ms (its
  // second workgroup holds 16), against 57 ms for 48 / 64 and for every one of those counts
  // with DUP (sha1_lanes, whose idle lanes exit: 82 - 88 vs 73 ms; profiles/r6/split/
  // small_launch_dup.jsonl). In the PartHasher a launch is often one part (16 lanes), so its
  // launches took 57 - 104 ms, 71 mean, where the kernel bench said 57.
  const int i = DUP && !live ? blockIdx.x * 64 + lane % (n - (int)blockIdx.x * 64) : i0;
  const bool work = DUP || live;
  const int64_t len = work ? lane_len[i] : 0;
  const uint32_t nfull = (uint32_t)(len >> 6);
  const int rem = (int)(len & 63);
  const int ntail = rem >= 56 ? 2 : 1;
  const uint32_t nblk = work ? nfull + (uint32_t)ntail : 0u;
  if (threadIdx.x == 0) longest = 0;
  __syncthreads();
  if (wave == 0) atomicMax(&longest, nblk);
  __syncthreads();
  const uint32_t M = longest;                      // blocks of the workgroup's longest lane
  // this lane's column of slot j (plain arithmetic on `ring`: an array of slot pointers made
  // them generic pointers - flat_load / flat_store, waited for with vmcnt too)
  auto col = [&](uint32_t j) { return ring + j * (kSplitGroups * 64) + lane; };
  // Two prologue steps, then steps k = 0 .. M - 1, one barrier each. Step k: the consumer
  // hashes block k from registers (read in the step before) while its reads of block k + 1 (slot (k + 1) % 4) are in flight - their latency, and their queueing
  // behind the stores, off its critical path. Producer k % 2 swaps, schedules and writes block
  // k + 2 into slot (k + 2) % 4 (free: block k is in the consumer's registers) - the stores at
  // the end of its step, after the consumer's reads - and idles in the next step.
  if (wave < 2) {
    const uint32_t p = (uint32_t)wave;
    const uint8_t* src = data + (work ? lane_off[i] : 0);
    const uint64_t bits = (uint64_t)len * 8ull;
    const uint32_t last = nblk - 1;
    // every load is unconditional (block index clamped to the tail block, read as 64 raw
    // bytes - the arena has a pad past its end), so the compiler's wait counts stay exact
    auto at = [&](uint32_t b) { return src + ((int64_t)(b < nfull ? b : nfull) << 6); };
    uint4 raw[4], g[kSplitGroups];
    uint32_t w[16];
    auto compute = [&](uint32_t b) {             // raw holds block b: schedule it into g
      if (b < nblk) {
        if (b < nfull) to_words(raw, w);
        else tail_words(raw, rem, b == last, b > nfull, bits, w);
      }
      asm volatile("" ::: "memory");             // the refill below stays behind this use
      load_raw16(at(b + 2), raw);                // this producer's next block, 2 steps ahead
      if (b < nblk) split_schedule(w, g);
    };
    auto write = [&](uint32_t b) {
      if (b < nblk) split_write(g, col(b % kSplitSlots));
    };
    // Roles fixed per wave and whole step pairs inside the loops: `raw` and `g` then stay in
    // the same registers round the back edge - a phi between two register sets made the
    // compiler copy `raw` right after issuing its loads, i.e. wait for them.
    load_raw16(at(p), raw);
    uint32_t k = 0;
    if (p == 0) {
      compute(0);
      write(0);
      lds_barrier();                           // prologue step -2
      lds_barrier();                           // prologue step -1: idle
      for (; k + 2 <= M; k += 2) {
        compute(k + 2);
        write(k + 2);
        lds_barrier();                         // step k
        lds_barrier();                         // step k + 1: idle
      }
      if (k < M) {
        compute(k + 2);
        write(k + 2);
        lds_barrier();
      }
    } else {
      lds_barrier();                           // prologue step -2: idle
      compute(1);
      write(1);
      lds_barrier();                           // prologue step -1
      for (; k + 2 <= M; k += 2) {
        lds_barrier();                         // step k: idle
        compute(k + 3);
        write(k + 3);
        lds_barrier();                         // step k + 1
      }
      if (k < M) lds_barrier();
    }
  } else {
    Sha1State s{0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    uint4 ga[kSplitGroups], gb[kSplitGroups];
    // fixed roles per step of a pair (no register copies): fill one, hash the other
    auto step = [&](uint32_t k, uint4 (&fill)[kSplitGroups], const uint4 (&use)[kSplitGroups]) {
      if (k + 1 < nblk) split_read(col((k + 1) % kSplitSlots), fill);
      if (k < nblk) split_rounds(s, use);
      lds_barrier();
    };
    lds_barrier();                               // prologue step -2
    if (0 < nblk) split_read(col(0), gb);
    lds_barrier();                               // prologue step -1
    uint32_t k = 0;
    for (; k + 2 <= M; k += 2) {
      step(k, ga, gb);
      step(k + 1, gb, ga);
    }
    if (k < M) step(k, ga, gb);
    if (live) {
      const uint32_t hv[5] = {s.h0, s.h1, s.h2, s.h3, s.h4};
      store_digest(out + (int64_t)i * 20, hv);
    }
  }
}

#define sha1_lanes_split sha1_lanes_split_t<true>

// Chunk-streamed variant: lane k owns piece (first + k) of a window - or, with a piece list,
// piece lane_piece[first + k] - and advances it by one CH-byte chunk per launch; the SHA-1
// state lives in `state` between launches. The chunk of lane k sits at data + k * CH. On the
// launch that reaches the end of the piece the lane pads, finalises and writes ok[gi].
// Per-launch latency is CH / lane-rate (~1.6 ms for 64 KiB) instead of piece_len / lane-rate,
// so copies and hashing overlap at a fine grain whatever the piece size.
template <bool B3>
__global__ __launch_bounds__(256) void sha1_chunk(uint32_t* __restrict__ state,
                                                  const uint8_t* __restrict__ data, int64_t CH,
                                                  int n, int64_t piece_len, int64_t last_len,
                                                  int first, int n_total, int64_t chunk_off,
                                                  const uint8_t* __restrict__ expected,
                                                  uint8_t* __restrict__ ok,
                                                  const int* __restrict__ lane_piece) {
  int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int gi = lane_piece ? lane_piece[first + k] : first + k;
  const int64_t len = (gi == n_total - 1) ? last_len : piece_len;
  const int64_t valid = len - chunk_off;          // bytes of this piece at/after this chunk
  if (valid < 0 || (valid == 0 && chunk_off > 0)) return;  // finished in an earlier launch
  uint32_t* st = state + 5 * (int64_t)k;
  Sha1State s;
  if (chunk_off == 0) {
    s = Sha1State{0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  } else {
    s = Sha1State{st[0], st[1], st[2], st[3], st[4]};
  }
  const uint8_t* p = data + (int64_t)k * CH;
  const bool last_chunk = valid <= CH;
  const int64_t here = last_chunk ? valid : CH;
  uint32_t w[16];
  const int64_t nfull = here >> 6;
  sha1_run16<B3, true>(s, p, nfull);
  if (!last_chunk) {
    st[0] = s.h0; st[1] = s.h1; st[2] = s.h2; st[3] = s.h3; st[4] = s.h4;
    return;
  }
  const int rem = (int)(here & 63);
  const uint8_t* tail = p + (nfull << 6);
  const uint64_t bits = (uint64_t)len * 8ull;
  const int nb = rem >= 56 ? 2 : 1;
  for (int b = 0; b < nb; ++b) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t v = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = b * 64 + 4 * i + q;
        uint32_t byte = idx < rem ? (uint32_t)tail[idx] : (idx == rem ? 0x80u : 0u);
        v |= byte << (24 - 8 * q);
      }
      w[i] = v;
    }
    if (b == nb - 1) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha1_block<B3>(s, w);
  }
  const uint32_t hv[5] = {s.h0, s.h1, s.h2, s.h3, s.h4};
  const uint8_t* ex = expected + (int64_t)gi * 20;
  bool good = true;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    uint32_t e = ((uint32_t)ex[4 * q] << 24) | ((uint32_t)ex[4 * q + 1] << 16) |
                 ((uint32_t)ex[4 * q + 2] << 8) | (uint32_t)ex[4 * q + 3];
    good = good && (e == hv[q]);
  }
  ok[gi] = good ? 1 : 0;
}

// Pseudo-random device fill (kernel benches: distinct pieces without a host copy).
__global__ __launch_bounds__(256) void fill_mix(uint4* __restrict__ p, int64_t n16, uint32_t seed) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n16;
       j += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)j * 0x9E3779B1u ^ (uint32_t)(j >> 32) ^ seed;
    uint4 v;
    x ^= x >> 15; x *= 0x2C1B3C6Du; x ^= x >> 12; v.x = x;
    x *= 0x297A2D39u; x ^= x >> 15; v.y = x;
    x *= 0x2C1B3C6Du; x ^= x >> 12; v.z = x;
    x *= 0x297A2D39u; x ^= x >> 15; v.w = x;
    p[j] = v;
  }
}

void launch(hipStream_t st, const uint8_t* d_data, int64_t piece_len, int64_t last_len, int n,
            const uint8_t* d_expected, uint8_t* d_ok, uint8_t* d_out) {
  if (n <= 0) return;
  const int block = 64;  // one wave per workgroup: pieces spread over as many CUs as possible
  const int grid = (n + block - 1) / block;
  if (piece_len % 16 == 0)
    hipLaunchKernelGGL(sha1_pieces<16>, dim3(grid), dim3(block), 0, st, d_data, piece_len,
                       last_len, n, d_expected, d_ok, d_out);
  else if (piece_len % 4 == 0)
    hipLaunchKernelGGL(sha1_pieces<4>, dim3(grid), dim3(block), 0, st, d_data, piece_len,
                       last_len, n, d_expected, d_ok, d_out);
  else
    hipLaunchKernelGGL(sha1_pieces<1>, dim3(grid), dim3(block), 0, st, d_data, piece_len,
                       last_len, n, d_expected, d_ok, d_out);
  HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------
// Storage reader (files concatenated in order), same layout as the host module's Storage.
struct FileSpan {
  std::string path;
  int64_t length, offset;
  int fd;
};

struct Files {
  std::vector<FileSpan> v;
  int64_t total = 0;
  explicit Files(const std::vector<std::pair<std::string, int64_t>>& files) {
    for (auto& f : files) {
      FileSpan s{f.first, f.second, total, -1};
      if (s.length > 0) s.fd = ::open(s.path.c_str(), O_RDONLY | O_CLOEXEC);
      total += f.second;
      v.push_back(s);
    }
  }
  ~Files() {
    for (auto& s : v)
      if (s.fd >= 0) ::close(s.fd);
  }
  bool read(int64_t off, int64_t len, uint8_t* buf) const {
    int64_t done = 0;
    for (auto& e : v) {
      if (done >= len) break;
      int64_t pos = off + done;
      if (e.length == 0 || pos >= e.offset + e.length) continue;
      if (pos < e.offset || e.fd < 0) return false;
      int64_t in_file = pos - e.offset, want = std::min(len - done, e.length - in_file), got = 0;
      while (got < want) {
        ssize_t r = pread(e.fd, buf + done + got, (size_t)(want - got), in_file + got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        got += r;
      }
      done += want;
    }
    return done == len;
  }
};

template <class F>
void parallel_for(size_t n, int threads, F&& fn) {
  threads = std::max(1, std::min<int>(threads, (int)n));
  if (threads == 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  // An exception in a reader (or a thread that cannot be started) reaches the caller instead
  // of std::terminate: the first one is rethrown once every started thread has joined.
  std::atomic<size_t> next{0};
  std::mutex err_mu;
  std::exception_ptr err;
  auto work = [&] {
    try {
      for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
    } catch (...) {
      next.store(n);
      std::lock_guard<std::mutex> g(err_mu);
      if (!err) err = std::current_exception();
    }
  };
  std::vector<std::thread> pool;
  try {
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  } catch (...) {
    // fewer threads than asked: the ones running (and this one) share the work
  }
  work();
  for (auto& th : pool) th.join();
  if (err) std::rethrow_exception(err);
}

// Scoped device memory and events: released on every exit path, a thrown HIP error included
// (hipFree waits for work still using the memory).
template <class T>
struct DevMem {
  T* p = nullptr;
  explicit DevMem(size_t n) {
    if (n) HIP_CHECK(hipMalloc((void**)&p, n * sizeof(T)));
  }
  ~DevMem() {
    if (p) hipFree(p);
  }
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
};
struct DevEvent {
  hipEvent_t e = nullptr;
  explicit DevEvent(unsigned flags = hipEventDisableTiming) {
    HIP_CHECK(hipEventCreateWithFlags(&e, flags));
  }
  ~DevEvent() {
    if (e) hipEventDestroy(e);
  }
  DevEvent(const DevEvent&) = delete;
  DevEvent& operator=(const DevEvent&) = delete;
};

class GpuVerifier {
 public:
  GpuVerifier(int device, int64_t batch_bytes, int reader_threads)
      : device_(device), batch_bytes_(batch_bytes), readers_(reader_threads) {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) throw std::runtime_error("no such HIP device");
    HIP_CHECK(hipSetDevice(device_));
    try {
      for (int s = 0; s < 2; ++s) {
        HIP_CHECK(hipStreamCreateWithFlags(&stream_[s], hipStreamNonBlocking));
        HIP_CHECK(hipHostMalloc((void**)&h_buf_[s], (size_t)batch_bytes_, hipHostMallocDefault));
        HIP_CHECK(hipMalloc((void**)&d_buf_[s], (size_t)batch_bytes_));
        HIP_CHECK(hipEventCreateWithFlags(&done_[s], hipEventDisableTiming));
      }
    } catch (...) {
      release();                       // a failed set-up leaves nothing allocated
      throw;
    }
  }
  ~GpuVerifier() { release(); }

  void release() {
    hipSetDevice(device_);
    for (int s = 0; s < 2; ++s) {
      if (stream_[s]) hipStreamSynchronize(stream_[s]);
      if (h_buf_[s]) hipHostFree(h_buf_[s]);
      if (d_buf_[s]) hipFree(d_buf_[s]);
      if (done_[s]) hipEventDestroy(done_[s]);
      if (stream_[s]) hipStreamDestroy(stream_[s]);
    }
    if (d_meta_) hipFree(d_meta_);
    if (h_meta_) hipHostFree(h_meta_);
    for (int s = 0; s < 2; ++s) stream_[s] = nullptr, h_buf_[s] = d_buf_[s] = nullptr, done_[s] = nullptr;
    d_meta_ = h_meta_ = nullptr;
  }

  // Digests of a contiguous host buffer split into pieces (used by tests and torrent
  // creation). Streams the buffer through the staging slots batch by batch.
  std::string hash_buffer(const uint8_t* p, int64_t n, int64_t piece_len) {
    HIP_CHECK(hipSetDevice(device_));
    int64_t np = n == 0 ? 0 : (n + piece_len - 1) / piece_len;
    std::string out((size_t)np * 20, '\0');
    run_batches(np, piece_len, n, nullptr,
                [&](int64_t first, int64_t cnt, uint8_t* dst) {
                  int64_t off = first * piece_len, len = std::min(cnt * piece_len, n - off);
                  memcpy(dst, p + off, (size_t)len);
                  return true;
                },
                (uint8_t*)out.data(), nullptr);
    return out;
  }

  // Verify pieces stored across files; returns one byte per piece (1 = hash matches).
  std::vector<uint8_t> verify_files(const std::vector<std::pair<std::string, int64_t>>& files,
                                    int64_t piece_len, const std::string& hashes) {
    HIP_CHECK(hipSetDevice(device_));
    Files fs(files);
    int64_t np = fs.total == 0 ? 0 : (fs.total + piece_len - 1) / piece_len;
    if ((int64_t)hashes.size() != np * 20) throw std::invalid_argument("hash list / piece count mismatch");
    std::vector<uint8_t> ok((size_t)np, 0);
    std::vector<uint8_t> readable((size_t)np, 1);
    run_batches(np, piece_len, fs.total, (const uint8_t*)hashes.data(),
                [&](int64_t first, int64_t cnt, uint8_t* dst) {
                  parallel_for((size_t)cnt, readers_, [&](size_t k) {
                    int64_t i = first + (int64_t)k;
                    int64_t off = i * piece_len, len = std::min(piece_len, fs.total - off);
                    if (!fs.read(off, len, dst + (int64_t)k * piece_len)) readable[(size_t)i] = 0;
                  });
                  return true;
                },
                nullptr, ok.data());
    for (int64_t i = 0; i < np; ++i)
      if (!readable[(size_t)i]) ok[(size_t)i] = 0;
    return ok;
  }

  int64_t batch_bytes() const { return batch_bytes_; }

  // Chunk-streamed verification (see sha1_chunk). Pieces are processed in windows of W lanes;
  // each round fills one pinned slot with chunk c of every piece of the window (reader
  // threads, pread from the page cache), copies it on the slot's stream and launches the
  // chunk kernel. Kernels are ordered across the two streams with events (state carries
  // over); the host refills a slot only after its previous copy completed.
  // `which` (optional) restricts the check to those piece indices: the result then holds one
  // byte per listed piece, in list order (incremental verification of downloaded runs).
  std::vector<uint8_t> verify_files_streamed(
      const std::vector<std::pair<std::string, int64_t>>& files, int64_t piece_len,
      const std::string& hashes, int64_t chunk, std::vector<double>* timing,
      const std::vector<int>& which = {}) {
    HIP_CHECK(hipSetDevice(device_));
    Files fs(files);
    const int64_t np = fs.total == 0 ? 0 : (fs.total + piece_len - 1) / piece_len;
    if ((int64_t)hashes.size() != np * 20) throw std::invalid_argument("hash list / piece count mismatch");
    for (int w : which)
      if (w < 0 || (int64_t)w >= np) throw std::invalid_argument("piece index out of range");
    const bool subset = !which.empty();
    const int64_t m = subset ? (int64_t)which.size() : np;   // lanes to run
    auto piece_of = [&](int64_t j) -> int64_t { return subset ? (int64_t)which[(size_t)j] : j; };
    std::vector<uint8_t> ok((size_t)np, 0);
    if (timing) *timing = {0.0, 0.0};
    if (np == 0) return ok;
    const int64_t CH = std::max<int64_t>(64, std::min<int64_t>(chunk, piece_len) & ~(int64_t)63);
    const int64_t W = std::max<int64_t>(1, std::min<int64_t>(m, batch_bytes_ / CH));
    const int64_t last_len = fs.total - (np - 1) * piece_len;
    DevMem<uint8_t> exp_buf((size_t)np * 20), ok_buf((size_t)np);
    DevMem<uint32_t> state_buf((size_t)W * 5);
    DevMem<int> lanes_buf(subset ? (size_t)m : 0);
    uint8_t *d_exp = exp_buf.p, *d_ok = ok_buf.p;
    uint32_t* d_state = state_buf.p;
    int* d_lanes = lanes_buf.p;
    HIP_CHECK(hipMemcpy(d_exp, hashes.data(), (size_t)np * 20, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemset(d_ok, 0, (size_t)np));
    if (subset)
      HIP_CHECK(hipMemcpy(d_lanes, which.data(), (size_t)m * sizeof(int), hipMemcpyHostToDevice));
    std::vector<uint8_t> readable((size_t)np, 1);
    DevEvent copied_ev[2], kdone_ev[2];
    hipEvent_t copied[2] = {copied_ev[0].e, copied_ev[1].e}, kdone[2] = {kdone_ev[0].e, kdone_ev[1].e};
    bool slot_busy[2] = {false, false};
    bool have_prev_kernel = false;
    int prev_slot = 0;
    double t_fill = 0, t_wait = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    int s = 0;
    for (int64_t first = 0; first < m; first += W) {
      const int64_t n = std::min(W, m - first);
      int64_t maxlen = piece_len;
      for (int64_t k = 0; k < n; ++k)
        if (piece_of(first + k) == np - 1) maxlen = std::max(piece_len, last_len);
      const int64_t rounds = (maxlen + CH - 1) / CH;
      for (int64_t c = 0; c < rounds; ++c, s ^= 1) {
        auto t0 = now();
        if (slot_busy[s]) HIP_CHECK(hipEventSynchronize(copied[s]));
        auto t1 = now();
        uint8_t* dst = h_buf_[s];
        const int64_t coff = c * CH;
        parallel_for((size_t)n, readers_, [&](size_t k) {
          const int64_t gi = piece_of(first + (int64_t)k);
          const int64_t len = gi == np - 1 ? last_len : piece_len;
          const int64_t here = std::min<int64_t>(CH, len - coff);
          if (here <= 0) return;
          if (!fs.read(gi * piece_len + coff, here, dst + (int64_t)k * CH)) readable[(size_t)gi] = 0;
        });
        auto t2 = now();
        t_wait += std::chrono::duration<double>(t1 - t0).count();
        t_fill += std::chrono::duration<double>(t2 - t1).count();
        HIP_CHECK(hipMemcpyAsync(d_buf_[s], dst, (size_t)(n * CH), hipMemcpyHostToDevice, stream_[s]));
        HIP_CHECK(hipEventRecord(copied[s], stream_[s]));
        slot_busy[s] = true;
        if (have_prev_kernel) HIP_CHECK(hipStreamWaitEvent(stream_[s], kdone[prev_slot], 0));
        const int block = 64, grid = (int)((n + block - 1) / block);
        hipLaunchKernelGGL((sha1_chunk<true>), dim3(grid), dim3(block), 0, stream_[s], d_state,
                           d_buf_[s], CH, (int)n, piece_len, last_len, (int)first, (int)np, coff,
                           d_exp, d_ok, d_lanes);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(kdone[s], stream_[s]));
        have_prev_kernel = true;
        prev_slot = s;
      }
    }
    HIP_CHECK(hipStreamSynchronize(stream_[0]));
    HIP_CHECK(hipStreamSynchronize(stream_[1]));
    HIP_CHECK(hipMemcpy(ok.data(), d_ok, (size_t)np, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < np; ++i)
      if (!readable[(size_t)i]) ok[(size_t)i] = 0;
    if (timing) *timing = {t_fill, t_wait};
    if (!subset) return ok;
    std::vector<uint8_t> sub((size_t)m);
    for (int64_t j = 0; j < m; ++j) sub[(size_t)j] = ok[(size_t)which[(size_t)j]];
    return sub;
  }

  // Kernel-only A/B of the block-prefetch (both with v_bitop3): ms per launch with and
  // without loading block k+1 while block k is hashed, interleaved in one process.
  std::vector<double> kernel_bench_prefetch(int64_t piece_len, int n_pieces, int iters) {
    HIP_CHECK(hipSetDevice(device_));
    size_t bytes = (size_t)piece_len * (size_t)n_pieces;
    DevMem<uint8_t> data_buf(bytes), out_buf((size_t)n_pieces * 20);
    uint8_t *d = data_buf.p, *dout = out_buf.p;
    HIP_CHECK(hipMemset(d, 0x5a, bytes));
    DevEvent ev0(hipEventDefault), ev1(hipEventDefault);
    hipEvent_t e0 = ev0.e, e1 = ev1.e;
    const int block = 64, grid = (n_pieces + block - 1) / block;
    double t[2] = {0, 0};
    for (int it = 0; it < iters + 1; ++it) {
      for (int v = 0; v < 2; ++v) {
        HIP_CHECK(hipEventRecord(e0, stream_[0]));
        if (v == 0)
          hipLaunchKernelGGL((sha1_pieces<16, true, true>), dim3(grid), dim3(block), 0,
                             stream_[0], d, piece_len, piece_len, n_pieces, nullptr, nullptr,
                             dout);
        else
          hipLaunchKernelGGL((sha1_pieces<16, true, false>), dim3(grid), dim3(block), 0,
                             stream_[0], d, piece_len, piece_len, n_pieces, nullptr, nullptr,
                             dout);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(e1, stream_[0]));
        HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0) t[v] += ms;
      }
    }
    return {t[0] / iters, t[1] / iters};
  }

  // Kernel-only A/B of the PartHasher kernels on one lane table (device-resident, distinct
  // pseudo-random pieces): ms per launch of sha1_lanes_split and sha1_lanes<16>, interleaved,
  // and whether their digests agree. Lane i hashes piece_len - (i * 37) % 131 bytes at
  // i * piece_len, so the lanes of a workgroup end at different blocks and every tail shape
  // (rem < 56: one padding block, >= 56: two) comes up.
  std::vector<double> kernel_bench_split(int64_t piece_len, int n_pieces, int iters,
                                         bool dup) {
    HIP_CHECK(hipSetDevice(device_));
    const size_t bytes = (size_t)piece_len * (size_t)n_pieces;
    DevMem<uint8_t> data_buf(bytes + kArenaPad), out_a((size_t)n_pieces * 20),
        out_b((size_t)n_pieces * 20);
    DevMem<int64_t> tab((size_t)n_pieces * 2);
    std::vector<int64_t> h((size_t)n_pieces * 2);
    for (int i = 0; i < n_pieces; ++i) {
      h[(size_t)i] = (int64_t)i * piece_len;
      h[(size_t)n_pieces + i] = std::max<int64_t>(0, piece_len - (int64_t)((i * 37) % 131));
    }
    HIP_CHECK(hipMemcpy(tab.p, h.data(), h.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_mix, dim3(2048), dim3(256), 0, stream_[0],
                       reinterpret_cast<uint4*>(data_buf.p), (int64_t)(bytes / 16), 0x51u);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemsetAsync(out_a.p, 0, (size_t)n_pieces * 20, stream_[0]));
    HIP_CHECK(hipMemsetAsync(out_b.p, 0xff, (size_t)n_pieces * 20, stream_[0]));
    DevEvent ev0(hipEventDefault), ev1(hipEventDefault);
    hipEvent_t e0 = ev0.e, e1 = ev1.e;
    const int grid = (n_pieces + 63) / 64;
    double t[2] = {0, 0};
    for (int it = 0; it < iters + 1; ++it) {
      for (int v = 0; v < 2; ++v) {
        HIP_CHECK(hipEventRecord(e0, stream_[0]));
        if (v == 0 && dup)
          hipLaunchKernelGGL(sha1_lanes_split_t<true>, dim3(grid), dim3(kSplitThreads), 0,
                             stream_[0], data_buf.p, tab.p, tab.p + n_pieces, n_pieces, out_a.p);
        else if (v == 0)
          hipLaunchKernelGGL(sha1_lanes_split, dim3(grid), dim3(kSplitThreads), 0, stream_[0],
                             data_buf.p, tab.p, tab.p + n_pieces, n_pieces, out_a.p);
        else
          hipLaunchKernelGGL(sha1_lanes<16>, dim3(grid), dim3(64), 0, stream_[0], data_buf.p,
                             tab.p, tab.p + n_pieces, n_pieces, out_b.p);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(e1, stream_[0]));
        HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0) t[v] += ms;
      }
    }
    std::vector<uint8_t> a((size_t)n_pieces * 20), b((size_t)n_pieces * 20);
    HIP_CHECK(hipMemcpy(a.data(), out_a.p, a.size(), hipMemcpyDeviceToHost));
    HIP_CHECK(hipMemcpy(b.data(), out_b.p, b.size(), hipMemcpyDeviceToHost));
    return {t[0] / iters, t[1] / iters, a == b ? 1.0 : 0.0};
  }

  // Two sha1_lanes_split launches at once on the two streams (as the PartHasher's compute
  // streams run them), n0 and n1 lanes, against the first alone: (ms alone, ms stream 0, ms
  // stream 1), means over `iters` rounds. mode 1: stream 1 copies 48 x 64 MiB host -> device
  // (pinned) instead of its launch, as the PartHasher's copy streams do; mode 2: 40 ms of
  // device idleness before each launch.
  std::vector<double> kernel_bench_concurrent(int64_t piece_len, int n0, int n1, int iters,
                                              int mode) {
    HIP_CHECK(hipSetDevice(device_));
    const int n = n0 + n1;
    const size_t bytes = (size_t)piece_len * (size_t)n;
    DevMem<uint8_t> data_buf(bytes + kArenaPad), out((size_t)n * 20);
    DevMem<int64_t> tab((size_t)n * 2);
    std::vector<int64_t> h((size_t)n * 2);
    // launch s's table: offsets then lengths, at tab + (s ? 2 * n0 : 0)
    for (int s = 0, base = 0; s < 2; base += s ? 0 : n0, ++s) {
      const int m = s ? n1 : n0;
      int64_t* t = h.data() + (s ? 2 * n0 : 0);
      for (int i = 0; i < m; ++i) {
        t[i] = ((int64_t)(s ? n0 : 0) + i) * piece_len;
        t[m + i] = piece_len;
      }
    }
    HIP_CHECK(hipMemcpy(tab.p, h.data(), h.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_mix, dim3(2048), dim3(256), 0, stream_[0],
                       reinterpret_cast<uint4*>(data_buf.p), (int64_t)(bytes / 16), 0x77u);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(stream_[0]));
    DevEvent a0(hipEventDefault), a1(hipEventDefault), b0(hipEventDefault), b1(hipEventDefault);
    auto go = [&](int s, hipEvent_t e0, hipEvent_t e1) {
      const int m = s ? n1 : n0;
      const int64_t* t = tab.p + (s ? 2 * n0 : 0);
      HIP_CHECK(hipEventRecord(e0, stream_[s]));
      if (m > 0)
        hipLaunchKernelGGL(sha1_lanes_split, dim3((m + 63) / 64), dim3(kSplitThreads), 0,
                           stream_[s], data_buf.p, t, t + m, m,
                           out.p + (size_t)(s ? n0 : 0) * 20);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipEventRecord(e1, stream_[s]));
    };
    const size_t cp = (size_t)64 << 20;
    uint8_t* hpin = nullptr;
    DevMem<uint8_t> dcp(mode == 1 ? cp : 0);
    if (mode == 1) HIP_CHECK(hipHostMalloc((void**)&hpin, cp, hipHostMallocDefault));
    double t[3] = {0, 0, 0};
    for (int it = 0; it < iters + 1; ++it) {
      if (mode == 2) std::this_thread::sleep_for(std::chrono::milliseconds(40));
      go(0, a0.e, a1.e);
      HIP_CHECK(hipEventSynchronize(a1.e));
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, a0.e, a1.e));
      if (it > 0) t[0] += ms;
      if (mode == 2) std::this_thread::sleep_for(std::chrono::milliseconds(40));
      go(0, a0.e, a1.e);
      if (mode == 1) {
        HIP_CHECK(hipEventRecord(b0.e, stream_[1]));
        for (int c = 0; c < 48; ++c)
          HIP_CHECK(hipMemcpyAsync(dcp.p, hpin, cp, hipMemcpyHostToDevice, stream_[1]));
        HIP_CHECK(hipEventRecord(b1.e, stream_[1]));
      } else {
        go(1, b0.e, b1.e);
      }
      HIP_CHECK(hipEventSynchronize(a1.e));
      HIP_CHECK(hipEventSynchronize(b1.e));
      HIP_CHECK(hipEventElapsedTime(&ms, a0.e, a1.e));
      if (it > 0) t[1] += ms;
      HIP_CHECK(hipEventElapsedTime(&ms, b0.e, b1.e));
      if (it > 0) t[2] += ms;
    }
    if (hpin) hipHostFree(hpin);
    return {t[0] / iters, t[1] / iters, t[2] / iters};
  }

  // Kernel-only timing (device-resident data, hipEvents): ms per launch hashing `n_pieces`
  // pieces of `piece_len` bytes; `bitop3` selects the v_bitop3 or the plain-C round forms
  // so both variants are A/B-timed interleaved in one process.
  std::vector<double> kernel_bench(int64_t piece_len, int n_pieces, int iters) {
    HIP_CHECK(hipSetDevice(device_));
    size_t bytes = (size_t)piece_len * (size_t)n_pieces;
    DevMem<uint8_t> data_buf(bytes), out_buf((size_t)n_pieces * 20);
    uint8_t *d = data_buf.p, *dout = out_buf.p;
    HIP_CHECK(hipMemset(d, 0x5a, bytes));
    DevEvent ev0(hipEventDefault), ev1(hipEventDefault);
    hipEvent_t e0 = ev0.e, e1 = ev1.e;
    const int block = 64, grid = (n_pieces + block - 1) / block;
    double t[2] = {0, 0};
    for (int it = 0; it < iters + 1; ++it) {
      for (int v = 0; v < 2; ++v) {
        HIP_CHECK(hipEventRecord(e0, stream_[0]));
        if (v == 0)
          hipLaunchKernelGGL((sha1_pieces<16, true>), dim3(grid), dim3(block), 0, stream_[0], d,
                             piece_len, piece_len, n_pieces, nullptr, nullptr, dout);
        else
          hipLaunchKernelGGL((sha1_pieces<16, false>), dim3(grid), dim3(block), 0, stream_[0], d,
                             piece_len, piece_len, n_pieces, nullptr, nullptr, dout);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipEventRecord(e1, stream_[0]));
        HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0) t[v] += ms;  // first round is warm-up
      }
    }
    return {t[0] / iters, t[1] / iters};
  }

 private:
  template <class Fill>
  void run_batches(int64_t np, int64_t piece_len, int64_t total, const uint8_t* expected,
                   Fill&& fill, uint8_t* out_digests, uint8_t* out_ok) {
    if (np == 0) return;
    int64_t per = std::max<int64_t>(1, batch_bytes_ / piece_len);
    if (per * piece_len > batch_bytes_) grow(per * piece_len);
    ensure_meta(per);
    struct Pending {
      int64_t first = 0, cnt = 0;
      bool live = false;
    } pend[2];
    auto drain = [&](int s) {
      if (!pend[s].live) return;
      HIP_CHECK(hipStreamSynchronize(stream_[s]));
      uint8_t* hm = h_meta_ + (size_t)s * meta_stride_;
      if (out_digests) memcpy(out_digests + pend[s].first * 20, hm, (size_t)pend[s].cnt * 20);
      if (out_ok) memcpy(out_ok + pend[s].first, hm, (size_t)pend[s].cnt);
      pend[s].live = false;
    };
    int s = 0;
    for (int64_t first = 0; first < np; first += per, s ^= 1) {
      int64_t cnt = std::min(per, np - first);
      drain(s);  // slot s free again (its previous batch has completed)
      fill(first, cnt, h_buf_[s]);
      int64_t off = first * piece_len;
      int64_t bytes = std::min(cnt * piece_len, total - off);
      int64_t last_len = bytes - (cnt - 1) * piece_len;
      uint8_t* dm = d_meta_ + (size_t)s * meta_stride_;
      uint8_t* hm = h_meta_ + (size_t)s * meta_stride_;
      HIP_CHECK(hipMemcpyAsync(d_buf_[s], h_buf_[s], (size_t)bytes, hipMemcpyHostToDevice, stream_[s]));
      const uint8_t* d_exp = nullptr;
      if (expected) {
        uint8_t* de = dm + per;  // expected digests after the ok bytes
        HIP_CHECK(hipMemcpyAsync(de, expected + first * 20, (size_t)cnt * 20, hipMemcpyHostToDevice,
                                 stream_[s]));
        d_exp = de;
        launch(stream_[s], d_buf_[s], piece_len, last_len, (int)cnt, d_exp, dm, nullptr);
        HIP_CHECK(hipMemcpyAsync(hm, dm, (size_t)cnt, hipMemcpyDeviceToHost, stream_[s]));
      } else {
        launch(stream_[s], d_buf_[s], piece_len, last_len, (int)cnt, nullptr, nullptr, dm);
        HIP_CHECK(hipMemcpyAsync(hm, dm, (size_t)cnt * 20, hipMemcpyDeviceToHost, stream_[s]));
      }
      pend[s] = {first, cnt, true};
    }
    drain(0);
    drain(1);
  }

  void grow(int64_t bytes) {
    batch_bytes_ = 0;                  // a failed grow makes the next batch try again
    for (int s = 0; s < 2; ++s) {
      HIP_CHECK(hipStreamSynchronize(stream_[s]));
      HIP_CHECK(hipHostFree(h_buf_[s]));
      h_buf_[s] = nullptr;             // never freed twice if an allocation below throws
      HIP_CHECK(hipFree(d_buf_[s]));
      d_buf_[s] = nullptr;
      HIP_CHECK(hipHostMalloc((void**)&h_buf_[s], (size_t)bytes, hipHostMallocDefault));
      HIP_CHECK(hipMalloc((void**)&d_buf_[s], (size_t)bytes));
    }
    batch_bytes_ = bytes;
  }

  void ensure_meta(int64_t per) {
    size_t need = (size_t)per * 21;  // ok byte + 20-byte expected digest (or 20-byte output)
    if (need <= meta_stride_) return;
    if (d_meta_) HIP_CHECK(hipFree(d_meta_));
    d_meta_ = nullptr;
    if (h_meta_) HIP_CHECK(hipHostFree(h_meta_));
    h_meta_ = nullptr;
    meta_stride_ = 0;                  // set once both allocations are in
    HIP_CHECK(hipMalloc((void**)&d_meta_, need * 2));
    HIP_CHECK(hipHostMalloc((void**)&h_meta_, need * 2, hipHostMallocDefault));
    meta_stride_ = need;
  }

  int device_;
  int64_t batch_bytes_;
  int readers_;
  hipStream_t stream_[2] = {nullptr, nullptr};
  hipEvent_t done_[2] = {nullptr, nullptr};
  uint8_t* h_buf_[2] = {nullptr, nullptr};
  uint8_t* d_buf_[2] = {nullptr, nullptr};
  uint8_t* d_meta_ = nullptr;
  uint8_t* h_meta_ = nullptr;
  size_t meta_stride_ = 0;
};

// ---------------------------------------------------------------------------------------
// PartHasher: piece SHA-1 of parts the hashed relay (csrc/transfer.cpp) has just moved
// webseed -> S3, so the host no longer spends ~40 % of a torrent job's worker CPU on the
// multi-buffer SHA-1 (docs/PERFORMANCE.md). SHA-1 is serial inside a piece, so a piece costs
// piece_len / ~58 MB/s on one lane (72 ms for 4 MiB) whatever else runs: throughput comes
// from many pieces per launch, and the latency is hidden by the stager keeping parts in
// flight. Hence:
//   * the relay submits the finished part (page-locked pooled buffer) and moves on; the
//     dispatcher thread DMAs it into the open device slot at once on a copy stream, and the
//     relay's lease on the buffer ends when that copy completes - not when the hash does;
//   * a slot (up to slot_bytes / max_lanes pieces of any number of parts) is launched as ONE
//     sha1_lanes kernel as soon as a compute stream is idle; while all are busy the open
//     slot keeps filling, so batches grow with the arrival rate (self-balancing: at R bytes/s
//     and T = per-piece kernel time over Q streams, a batch holds ~R*T/Q bytes);
//   * digests return with one D2H per slot; waiters are woken per ticket.
// Copy streams + compute streams fit in GPU_MAX_HW_QUEUES (4) hardware queues: a stream that
// shares its queue serialises behind the other's packets, so a copy stream next to a compute
// stream saw its copy-done markers wait for 77 ms kernels (round 3: 1 copy + 4 compute).
// A HIP error marks the hasher broken: queued and later parts are refused or failed, and the
// relay falls back to the host multi-buffer SHA-1.
// The scheduling state machine (queue, slots, streams, notify) is PartDispatcher in
// part_dispatch.h, shared with the CPU fake device of selftest.cpp; this class is its HIP side.
class HipPartDevice {
 public:
  using Event = hipEvent_t;

  HipPartDevice(int device, int64_t slot_bytes, int slots, int streams, int max_lanes,
                int copy_streams)
      : device_(device), slot_bytes_(slot_bytes), max_lanes_(max_lanes) {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) throw std::runtime_error("no such HIP device");
    if (slots < 2 || slot_bytes < (1 << 20) || max_lanes < 64 || copy_streams < 1 ||
        copy_streams > 4)
      throw std::invalid_argument("PartHasher: bad geometry");
    HIP_CHECK(hipSetDevice(device_));
    try {
      create(slots, streams, copy_streams);
    } catch (...) {
      release();                       // a failed set-up leaves no HBM or streams behind
      throw;
    }
  }
  ~HipPartDevice() { release(); }
  HipPartDevice(const HipPartDevice&) = delete;
  HipPartDevice& operator=(const HipPartDevice&) = delete;

  static bool split_default() {
    const char* e = getenv("STAGER_SHA1_KERNEL");
    return !(e && std::string(e) == "lanes");
  }

  static int hw_queues() {
    const char* e = getenv("GPU_MAX_HW_QUEUES");
    const int n = e ? atoi(e) : 0;
    return n > 0 ? n : 4;            // HIP's default
  }

  // sha1_lanes_split (two waves per 64 pieces) unless STAGER_SHA1_KERNEL=lanes (A/B)
  bool split() const { return split_; }
  int copy_streams() const { return (int)copies_.size(); }
  int compute_streams() const { return (int)streams_.size(); }
  int slots() const { return (int)slots_.size(); }
  void bind_thread() { HIP_CHECK(hipSetDevice(device_)); }
  int64_t* lane_table(int s) { return slots_[(size_t)s].h_lane; }

  Event copy(int s, int64_t off, const uint8_t* host, int64_t len, int cs) {
    hipStream_t st = copies_[(size_t)cs];
    HIP_CHECK(hipMemcpyAsync(slots_[(size_t)s].d_data + off, host, (size_t)len,
                             hipMemcpyHostToDevice, st));
    Event e = take_event();
    HIP_CHECK(hipEventRecord(e, st));
    return e;
  }
  bool copied(Event e) { return query(e); }
  void recycle(Event e) {
    if (e) free_events_.push_back(e);
  }
  // A slot's parts went over any of the copy streams: mark the end of what each has queued.
  void close_copies(int s) {
    Slot& sl = slots_[(size_t)s];
    for (size_t k = 0; k < copies_.size(); ++k) HIP_CHECK(hipEventRecord(sl.copied[k], copies_[k]));
  }
  int64_t launch_lanes() const { return launch_lanes_; }
  // One sha1_lanes kernel over the lanes of `nslots` slots, in order: the lane table of the
  // launch (offset in the arena + length per lane) is built in the stream's pinned table
  // (free: the stream's previous launch, its H2D included, finished before this one is made),
  // copied behind the slots' copy markers, and the digests come back with one D2H.
  void launch(int stream, const int* slots, const int* lanes, int nslots, int total,
              bool align16) {
    if (total <= 0 || total > launch_lanes_) throw std::runtime_error("PartHasher: bad launch");
    Run& r = runs_[(size_t)stream];
    hipStream_t st = streams_[(size_t)stream];
    int64_t* ho = r.h_tab;
    int64_t* hl = r.h_tab + total;
    int i = 0;
    for (int k = 0; k < nslots; ++k) {
      Slot& sl = slots_[(size_t)slots[k]];
      for (size_t c = 0; c < copies_.size(); ++c) HIP_CHECK(hipStreamWaitEvent(st, sl.copied[c], 0));
      const int64_t base = (int64_t)(sl.d_data - arena_);
      for (int l = 0; l < lanes[k]; ++l, ++i) {
        ho[i] = base + sl.h_lane[l];
        hl[i] = sl.h_lane[max_lanes_ + l];
      }
    }
    if (i != total) throw std::runtime_error("PartHasher: lane count mismatch");
    HIP_CHECK(hipMemcpyAsync(r.d_tab, r.h_tab, (size_t)total * 2 * sizeof(int64_t),
                             hipMemcpyHostToDevice, st));
    const int64_t* dp = r.d_tab;
    const int64_t* dl = r.d_tab + total;
    const int block = 64, grid = (total + block - 1) / block;
    if (align16 && split_)
      hipLaunchKernelGGL(sha1_lanes_split, dim3(grid), dim3(kSplitThreads), 0, st, arena_, dp,
                         dl, total, r.d_dig);
    else if (align16)
      hipLaunchKernelGGL(sha1_lanes<16>, dim3(grid), dim3(block), 0, st, arena_, dp, dl, total,
                         r.d_dig);
    else
      hipLaunchKernelGGL(sha1_lanes<1>, dim3(grid), dim3(block), 0, st, arena_, dp, dl, total,
                         r.d_dig);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(r.h_dig, r.d_dig, (size_t)total * 20, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipEventRecord(r.done, st));
  }
  bool finished(int stream) { return query(runs_[(size_t)stream].done); }
  const uint8_t* digests(int stream) { return runs_[(size_t)stream].h_dig; }
  void drain_copies() noexcept {
    for (auto c : copies_) hipStreamSynchronize(c);
  }
  int reg(void* p, size_t n) {
    if (hipSetDevice(device_) != hipSuccess) return -1;
    return hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess ? 0 : -1;
  }
  void unreg(void* p) {
    hipSetDevice(device_);
    hipHostUnregister(p);
  }

 private:
  struct Slot {
    uint8_t* d_data = nullptr;
    int64_t* h_lane = nullptr;   // [off x max_lanes][len x max_lanes], offsets in the slot
    hipEvent_t copied[4] = {nullptr, nullptr, nullptr, nullptr};   // one per copy stream
  };
  struct Run {                   // a compute stream's launch: lane table and digests
    int64_t* h_tab = nullptr;    // pinned [offset in the arena x total][len x total]
    int64_t* d_tab = nullptr;
    uint8_t* d_dig = nullptr;
    uint8_t* h_dig = nullptr;
    hipEvent_t done = nullptr;
  };

  static bool query(hipEvent_t e) {
    hipError_t q = hipEventQuery(e);
    if (q == hipErrorNotReady) return false;
    HIP_CHECK(q);
    return true;
  }

  void create(int slots, int streams, int copy_streams) {
    // Parts are DMA'd round-robin over copy_streams streams: each is its own hardware queue,
    // so H2D copies of consecutive parts run on separate SDMA engines instead of queueing
    // behind one another (a part's host buffer is held until its copy ends).
    copies_.resize((size_t)copy_streams);
    for (auto& c : copies_) HIP_CHECK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
    // Every HIP stream is mapped onto one of GPU_MAX_HW_QUEUES (4) hardware queues; a copy
    // stream that shares a queue with a compute stream has its copy-completion marker wait
    // behind a ~77 ms sha1_lanes kernel, and the part's host buffer with it. streams <= 0:
    // as many compute streams as the queues left over by the copy streams.
    const int hwq = hw_queues();
    const int compute = streams > 0 ? std::min(streams, 4) : std::max(1, hwq - copy_streams);
    streams_.resize((size_t)compute);
    for (auto& st : streams_) HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    slots_.resize((size_t)slots);
    // one arena, a window per slot: lane offsets from its base keep the kernel's loads global
    // + a pad: sha1_lanes_split reads a lane's tail block as 64 raw bytes, which may run past
    // the last slot's end
    HIP_CHECK(hipMalloc((void**)&arena_, (size_t)slot_bytes_ * (size_t)slots + kArenaPad));
    for (size_t k = 0; k < slots_.size(); ++k) {
      Slot& sl = slots_[k];
      sl.d_data = arena_ + (size_t)slot_bytes_ * k;
      HIP_CHECK(hipHostMalloc((void**)&sl.h_lane, (size_t)max_lanes_ * 2 * sizeof(int64_t),
                              hipHostMallocDefault));
      for (auto& e : sl.copied) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // a launch may carry every slot's lanes
    launch_lanes_ = (int64_t)max_lanes_ * (int64_t)slots;
    runs_.resize((size_t)compute);
    for (auto& r : runs_) {
      HIP_CHECK(hipHostMalloc((void**)&r.h_tab, (size_t)launch_lanes_ * 2 * sizeof(int64_t),
                              hipHostMallocDefault));
      HIP_CHECK(hipMalloc((void**)&r.d_tab, (size_t)launch_lanes_ * 2 * sizeof(int64_t)));
      HIP_CHECK(hipMalloc((void**)&r.d_dig, (size_t)launch_lanes_ * 20));
      HIP_CHECK(hipHostMalloc((void**)&r.h_dig, (size_t)launch_lanes_ * 20, hipHostMallocDefault));
      HIP_CHECK(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
    }
  }

  // Everything create() made, also when it stopped half-way (null handles are skipped).
  void release() {
    hipSetDevice(device_);
    for (auto c : copies_)
      if (c) hipStreamSynchronize(c);
    for (auto st : streams_)
      if (st) {
        hipStreamSynchronize(st);
        hipStreamDestroy(st);
      }
    for (auto c : copies_)
      if (c) hipStreamDestroy(c);
    if (arena_) hipFree(arena_);
    arena_ = nullptr;
    for (auto& sl : slots_) {
      if (sl.h_lane) hipHostFree(sl.h_lane);
      for (auto e : sl.copied)
        if (e) hipEventDestroy(e);
    }
    for (auto& r : runs_) {
      if (r.h_tab) hipHostFree(r.h_tab);
      if (r.d_tab) hipFree(r.d_tab);
      if (r.d_dig) hipFree(r.d_dig);
      if (r.h_dig) hipHostFree(r.h_dig);
      if (r.done) hipEventDestroy(r.done);
    }
    for (hipEvent_t e : free_events_) hipEventDestroy(e);
    copies_.clear();
    streams_.clear();
    slots_.clear();
    runs_.clear();
    free_events_.clear();
  }

  hipEvent_t take_event() {
    if (!free_events_.empty()) {
      hipEvent_t e = free_events_.back();
      free_events_.pop_back();
      return e;
    }
    hipEvent_t e;
    HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }

  int device_;
  int64_t slot_bytes_;
  int max_lanes_;
  bool split_ = split_default();
  int64_t launch_lanes_ = 0;
  uint8_t* arena_ = nullptr;     // slots x slot_bytes of HBM
  std::vector<hipStream_t> copies_;
  std::vector<hipStream_t> streams_;
  std::vector<Slot> slots_;
  std::vector<Run> runs_;
  std::vector<hipEvent_t> free_events_;   // dispatcher thread only
};

using PartHasher = stager::PartDispatcher<HipPartDevice>;

py::dict part_stats(PartHasher& h) {
  const stager::PartDispatchStats s = h.stats();
  py::dict d;
  d["submitted"] = s.submitted;
  d["launches"] = s.launches;
  d["lanes"] = s.lanes;
  d["max_batch_lanes"] = s.max_batch_lanes;
  d["multi_slot_launches"] = s.multi_slot_launches;   // launches spanning >= 2 HBM slots
  d["max_launch_slots"] = s.max_launch_slots;
  d["broken"] = s.broken;
  d["pending"] = s.pending;
  d["registered"] = s.registered;       // part buffers page-locked (hipHostRegister)
  d["unregistered"] = s.unregistered;
  d["register_s"] = s.register_s;
  d["copy_streams"] = s.copy_streams;
  d["compute_streams"] = s.compute_streams;
  d["kernel"] = h.device().split() ? "sha1_lanes_split" : "sha1_lanes";
  return d;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // namespace

PYBIND11_MODULE(_gpuhash, m) {
  m.doc() = "gfx950 batched SHA-1 piece verification (one lane per piece)";
  m.def("device_count", &device_count);
  m.def(
      "mem_info",
      [](int device) {
        size_t free_b = 0, total_b = 0;
        HIP_CHECK(hipSetDevice(device));
        HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        return py::make_tuple(free_b, total_b);
      },
      py::arg("device") = 0, "(free, total) bytes of device memory (hipMemGetInfo)");
  m.def("arch", [] {
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, 0));
    return std::string(p.gcnArchName);
  });
  py::class_<GpuVerifier>(m, "GpuVerifier")
      .def(py::init([](int device, int64_t batch_bytes, int readers) {
             py::gil_scoped_release rel;
             return new GpuVerifier(device, batch_bytes, readers);
           }),
           py::arg("device") = 0, py::arg("batch_bytes") = (int64_t)256 << 20,
           py::arg("reader_threads") = 8)
      .def(
          "hash_buffer",
          [](GpuVerifier& g, const py::buffer& b, int64_t piece_len) {
            py::buffer_info info = b.request();
            int64_t n = (int64_t)info.size * (int64_t)info.itemsize;
            if (piece_len <= 0) throw std::invalid_argument("piece_len must be > 0");
            std::string out;
            {
              py::gil_scoped_release rel;
              out = g.hash_buffer((const uint8_t*)info.ptr, n, piece_len);
            }
            return py::bytes(out);
          },
          py::arg("data"), py::arg("piece_len"))
      .def(
          "verify_files",
          [](GpuVerifier& g, const std::vector<std::pair<std::string, int64_t>>& files,
             int64_t piece_len, const py::bytes& hashes) {
            std::string hs = hashes;
            if (piece_len <= 0) throw std::invalid_argument("piece_len must be > 0");
            std::vector<uint8_t> ok;
            {
              py::gil_scoped_release rel;
              ok = g.verify_files(files, piece_len, hs);
            }
            return py::bytes((const char*)ok.data(), ok.size());
          },
          py::arg("files"), py::arg("piece_len"), py::arg("hashes"))
      .def(
          "verify_files_streamed",
          [](GpuVerifier& g, const std::vector<std::pair<std::string, int64_t>>& files,
             int64_t piece_len, const py::bytes& hashes, int64_t chunk,
             const std::vector<int>& which) {
            std::string hs = hashes;
            if (piece_len <= 0) throw std::invalid_argument("piece_len must be > 0");
            std::vector<uint8_t> ok;
            std::vector<double> timing;
            {
              py::gil_scoped_release rel;
              ok = g.verify_files_streamed(files, piece_len, hs, chunk, &timing, which);
            }
            return py::make_tuple(py::bytes((const char*)ok.data(), ok.size()),
                                  py::make_tuple(timing[0], timing[1]));
          },
          py::arg("files"), py::arg("piece_len"), py::arg("hashes"), py::arg("chunk") = 65536,
          py::arg("which") = std::vector<int>{},
          "Chunk-streamed SHA-1 verification: returns (ok bytes, (host_fill_s, host_wait_s)); "
          "with `which`, one ok byte per listed piece in list order.")
      .def(
          "kernel_bench",
          [](GpuVerifier& g, int64_t piece_len, int n_pieces, int iters) {
            if (piece_len <= 0 || piece_len % 16 || n_pieces <= 0 || iters <= 0)
              throw std::invalid_argument("piece_len must be a positive multiple of 16");
            std::vector<double> r;
            {
              py::gil_scoped_release rel;
              r = g.kernel_bench(piece_len, n_pieces, iters);
            }
            return py::make_tuple(r[0], r[1]);
          },
          py::arg("piece_len"), py::arg("n_pieces"), py::arg("iters") = 5,
          "(ms_bitop3, ms_plain): kernel time per launch, device-resident data")
      .def(
          "kernel_bench_prefetch",
          [](GpuVerifier& g, int64_t piece_len, int n_pieces, int iters) {
            if (piece_len <= 0 || piece_len % 16 || n_pieces <= 0 || iters <= 0)
              throw std::invalid_argument("piece_len must be a positive multiple of 16");
            std::vector<double> r;
            {
              py::gil_scoped_release rel;
              r = g.kernel_bench_prefetch(piece_len, n_pieces, iters);
            }
            return py::make_tuple(r[0], r[1]);
          },
          py::arg("piece_len"), py::arg("n_pieces"), py::arg("iters") = 5,
          "(ms_prefetch, ms_no_prefetch): kernel time per launch, device-resident data")
      .def(
          "kernel_bench_concurrent",
          [](GpuVerifier& g, int64_t piece_len, int n0, int n1, int iters, int mode) {
            if (piece_len < 256 || piece_len % 16 || n0 <= 0 || n1 < 0 || iters <= 0 ||
                mode < 0 || mode > 2)
              throw std::invalid_argument("piece_len must be a multiple of 16, >= 256");
            std::vector<double> r;
            {
              py::gil_scoped_release rel;
              r = g.kernel_bench_concurrent(piece_len, n0, n1, iters, mode);
            }
            return py::make_tuple(r[0], r[1], r[2]);
          },
          py::arg("piece_len"), py::arg("n0"), py::arg("n1"), py::arg("iters") = 3,
          py::arg("mode") = 0,
          "(ms alone, ms on stream 0, ms on stream 1): sha1_lanes_split launches of n0 and n1 "
          "lanes side by side (mode 0), n0 beside 48 x 64 MiB H2D copies (1), after 40 ms idle "
          "(2)")
      .def(
          "kernel_bench_split",
          [](GpuVerifier& g, int64_t piece_len, int n_pieces, int iters, bool dup) {
            if (piece_len < 256 || piece_len % 16 || n_pieces <= 0 || iters <= 0)
              throw std::invalid_argument("piece_len must be a multiple of 16, >= 256");
            std::vector<double> r;
            {
              py::gil_scoped_release rel;
              r = g.kernel_bench_split(piece_len, n_pieces, iters, dup);
            }
            return py::make_tuple(r[0], r[1], r[2] != 0.0);
          },
          py::arg("piece_len"), py::arg("n_pieces"), py::arg("iters") = 3, py::arg("dup") = true,
          "(ms_split, ms_lanes, digests_equal): the PartHasher's two kernels on one lane table "
          "(dup=False: the split kernel with its idle lanes left idle)")
      .def_property_readonly("batch_bytes", &GpuVerifier::batch_bytes);
  py::class_<PartHasher>(m, "PartHasher")
      .def(py::init([](int device, int64_t slot_bytes, int slots, int streams, int max_lanes,
                       int copy_streams) {
             py::gil_scoped_release rel;
             return new PartHasher(slot_bytes, max_lanes, device, slot_bytes, slots, streams,
                                   max_lanes, copy_streams);
           }),
           py::arg("device") = 0, py::arg("slot_bytes") = (int64_t)1 << 30, py::arg("slots") = 8,
           py::arg("streams") = 0, py::arg("max_lanes") = 16384, py::arg("copy_streams") = 2)
      .def(
          "api",
          [](PartHasher& h) {
            return py::capsule((void*)h.api(), "downloader_amd.gpu_part_api");
          },
          "PyCapsule of the C ABI (gpu_part_api.h) for _native.set_gpu_part_hasher; the "
          "PartHasher must outlive every user of the capsule (ops.hashing keeps it for good)")
      .def(
          "hash",
          [](PartHasher& h, const py::buffer& b, int64_t piece_len) {
            // test / bench entry: the buffer is registered, submitted and waited for here
            py::buffer_info info = b.request();
            const int64_t n = (int64_t)info.size * (int64_t)info.itemsize;
            const int64_t np = piece_len > 0 ? (n + piece_len - 1) / piece_len : 0;
            std::string out((size_t)np * 20, '\0');
            char err[256] = {0};
            int rc;
            {
              py::gil_scoped_release rel;
              void* p = info.ptr;
              bool r = h.reg(p, (size_t)n) == 0;
              uint64_t t = h.submit((const uint8_t*)p, n, piece_len);
              rc = t ? h.wait(t, GPU_PART_DONE, (uint8_t*)out.data(), out.size(), err, sizeof err)
                     : -1;
              if (r) h.unreg(p);
            }
            if (rc != 0) throw std::runtime_error(err[0] ? err : "PartHasher refused the part");
            return py::bytes(out);
          },
          py::arg("data"), py::arg("piece_len"))
      .def("stats", &part_stats);
}
