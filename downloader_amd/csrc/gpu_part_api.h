// C ABI between the host module (_native: the hashed relay owns the part buffers) and the
// gfx950 module (_gpuhash: the PartHasher batches relayed parts' pieces onto the GPU).
//
// The relay hands a finished part buffer to `submit` instead of hashing it with the host
// multi-buffer SHA-1. The hasher then reports each job's progress through the `notify`
// callback installed with `set_notify`: GPU_PART_COPIED once the DMA out of the buffer is done
// (the relay's buffer lease ends then - the bytes live in HBM from here on), GPU_PART_DONE
// once the digests are back. A job that fails is notified at the phase it failed in; `wait`
// for that phase then returns the error. `notify` is always called WITHOUT the hasher's own
// lock held, from the hasher's thread, so it may call `wait` (ready: never blocks) and `unreg`.
//
// Buffers are page-locked once with `reg` (hipHostRegister) and unlocked with `unreg` before
// the pool unmaps them. Passed from Python to _native as a PyCapsule named
// "downloader_amd.gpu_part_api".
#pragma once

#include <stddef.h>
#include <stdint.h>

#define GPU_PART_API_ABI 2u
#define GPU_PART_COPIED 1
#define GPU_PART_DONE 2

typedef void (*gpu_part_notify_fn)(void* arg, uint64_t ticket, int phase);

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
  // install the completion callback (null: none); jobs submitted later are notified
  void (*set_notify)(void* ctx, gpu_part_notify_fn fn, void* arg);
};
