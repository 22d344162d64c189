// C ABI between the host module (_native: the hashed relay owns the part buffers) and the
// gfx950 module (_gpuhash: the PartHasher batches relayed parts' pieces onto the GPU).
//
// The relay hands a finished part buffer to `submit` instead of hashing it with the host
// multi-buffer SHA-1; `wait(ticket, GPU_PART_COPIED)` returns once the DMA out of the buffer
// is done (the relay's buffer lease is released then), `wait(ticket, GPU_PART_DONE)` once the
// digests are back. Buffers are page-locked once with `reg` (hipHostRegister) and unlocked
// with `unreg` before the pool unmaps them. Passed from Python to _native as a PyCapsule
// named "downloader_amd.gpu_part_api".
#pragma once

#include <stddef.h>
#include <stdint.h>

#define GPU_PART_API_ABI 1u
#define GPU_PART_COPIED 1
#define GPU_PART_DONE 2

struct GpuPartHashApi {
  uint32_t abi;
  void* ctx;
  // page-lock [p, p + n) for DMA: 0 on success
  int (*reg)(void* ctx, void* p, size_t n);
  void (*unreg)(void* ctx, void* p);
  // queue `len` bytes at `data` (registered memory) as pieces of `piece_len` (the last one
  // may be short): a ticket, 0 if refused (broken device, shutting down)
  uint64_t (*submit)(void* ctx, const uint8_t* data, int64_t len, int64_t piece_len);
  // block until `phase`; for GPU_PART_DONE copy 20 B per piece to `out` (out_len bytes) and
  // forget the ticket. 0 on success, else an error message in err (errlen bytes).
  int (*wait)(void* ctx, uint64_t ticket, int phase, uint8_t* out, size_t out_len, char* err,
              size_t errlen);
};
