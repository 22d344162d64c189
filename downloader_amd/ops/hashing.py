"""Hashing front-end: CPU (OpenSSL EVP, threaded) and GPU (gfx950 SHA-1) backends.

Used by: torrent piece verification (reference: webtorrent's per-piece SHA-1),
torrent creation (bench fixtures), S3 SigV4 payload hashes and Content-MD5 / ETag checks.
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence, Tuple

from . import gpu_available, gpuhash, native

FileList = Sequence[Tuple[str, int]]

# Below this much data, or with few pieces, the PCIe round trip is not worth it.
GPU_MIN_BYTES = 256 << 20
GPU_MIN_PIECES = 256


def digest(algo: str, data) -> bytes:
    return native().digest(algo, data)


def sha1(data) -> bytes:
    return native().digest("sha1", data)


def sha256_hex(data) -> str:
    return native().digest("sha256", data).hex()


def md5(data) -> bytes:
    return native().digest("md5", data)


def new(algo: str):
    return native().Hasher(algo)


def hash_pieces(data, piece_len: int, algo: str = "sha1", threads: int = 0,
                backend: str = "cpu") -> bytes:
    if backend == "gpu":
        if algo != "sha1":
            raise ValueError("GPU backend implements SHA-1 only")
        return _verifier().hash_buffer(data, piece_len)
    return native().hash_pieces(algo, data, piece_len, threads)


def hash_storage_pieces(files: FileList, piece_len: int, algo: str = "sha1",
                        threads: int = 0) -> bytes:
    return native().hash_storage_pieces(list(files), piece_len, algo, threads)


def hash_file_ranges(path: str, ranges: Sequence[Tuple[int, int]], algo: str,
                     threads: int = 0) -> List[bytes]:
    return list(native().hash_file_ranges(path, list(ranges), algo, threads))


_gpu_lock = threading.Lock()
_gpu_verifier = None
# A cold verifier pays HIP init + 2 pinned staging slots (~0.3-1 s): "auto" uses the GPU for
# a cold start only when the recheck is big enough to amortise it.
GPU_COLD_MIN_BYTES = 32 << 30


def gpu_device() -> int:
    """One worker per GPU: ``STAGER_GPU_DEVICE``, else worker index / LOCAL_RANK modulo the
    visible device count."""
    if os.environ.get("STAGER_GPU_DEVICE"):
        return int(os.environ["STAGER_GPU_DEVICE"])
    idx = int(os.environ.get("STAGER_WORKER_INDEX", os.environ.get("LOCAL_RANK", "0")) or 0)
    try:
        n = gpuhash().device_count()
    except Exception:
        n = 1
    return idx % max(1, n)


def _verifier():
    global _gpu_verifier
    with _gpu_lock:
        if _gpu_verifier is None:
            _gpu_verifier = gpuhash().GpuVerifier(gpu_device(), 256 << 20, 8)
        return _gpu_verifier


def prewarm_gpu() -> bool:
    """Create the verifier now (worker start-up) so later rechecks see a warm device."""
    if not gpu_available():
        return False
    _verifier()
    return True


def choose_backend(requested: str, total_bytes: int, n_pieces: int) -> str:
    if requested == "cpu":
        return "cpu"
    if requested == "gpu":
        if not gpu_available():
            raise RuntimeError("verify_backend=gpu but no HIP device is available")
        return "gpu"
    if total_bytes < GPU_MIN_BYTES or n_pieces < GPU_MIN_PIECES:
        return "cpu"
    warm = _gpu_verifier is not None
    if (warm or total_bytes >= GPU_COLD_MIN_BYTES) and gpu_available():
        return "gpu"
    return "cpu"


def verify_pieces(files: FileList, piece_len: int, hashes: bytes,
                  which: Optional[Sequence[int]] = None, threads: int = 0,
                  backend: str = "cpu") -> bytes:
    """One byte per piece (1 = SHA-1 matches). ``which`` restricts the CPU check to a subset;
    the GPU backend always checks the full storage (recheck use case)."""
    files = [(str(p), int(n)) for p, n in files]
    total = sum(n for _, n in files)
    n_pieces = (total + piece_len - 1) // piece_len if total else 0
    be = choose_backend(backend, total, n_pieces) if which is None else "cpu"
    if be == "gpu":
        ok, _timing = _verifier().verify_files_streamed(files, piece_len, hashes)
        return ok
    return native().verify_pieces(files, piece_len, hashes, list(which or []), threads)
