"""Hashing front-end: CPU (OpenSSL EVP + AVX-512 multi-buffer SHA-1, threaded) and GPU
(gfx950 SHA-1) backends.

``verify_backend=auto`` follows measurements on the MI355X box (EPYC 9575F, 16-CPU quota,
``profiles/archive/s2_r1/``): with the 16-lane multi-buffer SHA-1 the host verifies a 4 GiB recheck at
57-62 GB/s vs 41-52 GB/s for the chunk-streamed gfx950 path (both bound by reading the bytes,
the GPU additionally by the pinned H2D hop), and a disk-staged 20 GB torrent at 13.1-13.8 vs
12.3-13.0 GB/s with less worker CPU. So auto keeps SHA-1 on the host whenever it has AVX-512
and uses the GPU on hosts without it; ``gpu`` forces the device.

Used by: torrent piece verification (reference: webtorrent's per-piece SHA-1),
torrent creation (bench fixtures), S3 SigV4 payload hashes and Content-MD5 / ETag checks.
"""
from __future__ import annotations

import collections
import os
import threading
import weakref
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


def crc32c(data, crc: int = 0) -> int:
    """CRC32C (Castagnoli), continuing from ``crc``: S3's x-amz-checksum-crc32c."""
    return native().crc32c(data, crc)


def crc32c_b64(data) -> str:
    """``x-amz-checksum-crc32c`` header value of ``data`` (base64 of the big-endian CRC)."""
    n = native()
    return n.crc32c_base64(n.crc32c(data))


def crc32c_fd_b64(fd: int, offset: int, length: int) -> str:
    n = native()
    return n.crc32c_base64(n.crc32c_fd(fd, offset, length))


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


_part_hasher = None
_part_hasher_failed = False
_retired_hashers: list = []      # replaced hashers: kept alive while their parts may be pending

# PartHasher geometry: device slots of slot_bytes each. A part's host buffer is only held
# until its DMA into a slot completes, so enough slots that a DMA never waits for a kernel to
# free one keeps host memory at a few parts (the slots are HBM: 16 x 1 GiB of 288 GB).
PART_SLOT_BYTES = 1 << 30
PART_SLOTS = 16


def gpu_relay_hashing(min_pieces: int = 8, slots: int = PART_SLOTS,
                      slot_bytes: int = PART_SLOT_BYTES, copy_streams: int = 2,
                      compute_streams: int = 0) -> bool:
    """Route the hashed relay's parts to the gfx950 ``PartHasher`` (batched, one lane per
    piece; csrc/gpu_sha1.hip) instead of the host multi-buffer SHA-1. Created once per
    process on the worker's GPU; False (host hashing) when no HIP device is usable."""
    global _part_hasher, _part_hasher_failed
    with _gpu_lock:
        if _part_hasher is not None:
            return True
        if _part_hasher_failed or not gpu_available():
            return False
        try:
            ph = gpuhash().PartHasher(gpu_device(), int(slot_bytes), int(slots),
                                      int(compute_streams), 16384, int(copy_streams))
            native().set_gpu_part_hasher(ph.api(), min_pieces)
        except Exception:
            _part_hasher_failed = True
            raise
        _part_hasher = ph
        return True


def use_part_hasher(hasher, min_pieces: int = 8) -> None:
    """Install ``hasher`` (anything with ``api()`` returning the gpu_part_api.h capsule, e.g.
    ``_native.CpuPartHasher`` in tests) as the relay's part hasher; None restores host
    hashing. The object is kept alive here (a replaced one too: its parts may be pending)."""
    global _part_hasher
    with _gpu_lock:
        native().set_gpu_part_hasher(hasher.api() if hasher is not None else None, min_pieces)
        if _part_hasher is not None and _part_hasher is not hasher:
            _retired_hashers.append(_part_hasher)
        _part_hasher = hasher


class GpuPart:
    """Completion of one part handed to the GPU hasher: ``copied`` resolves when the DMA out
    of its buffer is over (the buffer is back in the relay pool), ``done`` with its digests
    (or a RuntimeError when the device failed after the DMA)."""

    def __init__(self, loop: "asyncio.AbstractEventLoop"):
        self.loop = loop
        self.copied = loop.create_future()
        self.done = loop.create_future()
        self.done.add_done_callback(_retrieve)

    def _deliver(self, kind: int, data: bytes) -> None:
        if not self.copied.done():
            self.copied.set_result(None)
        if self.done.done():
            return
        if kind == 2:
            self.done.set_result(data)
        elif kind == 3:
            self.done.set_exception(RuntimeError(data.decode(errors="replace")))


def _retrieve(fut) -> None:
    if not fut.cancelled():
        fut.exception()


EARLY_MAX = 4096


class _GpuParts:
    """Routes the native completion queue (``gpu_part_poll``, signalled through an eventfd
    the event loop watches) to per-part futures: no thread blocks per part."""

    def __init__(self):
        self._lock = threading.Lock()
        self._parts: dict = {}
        self._early: dict = {}        # news for a part not tracked yet
        self._evicted: "collections.OrderedDict" = collections.OrderedDict()  # ids whose news
        self._loops: "weakref.WeakSet" = weakref.WeakSet()                     # were dropped

    def track(self, gid: int) -> GpuPart:
        import asyncio
        loop = asyncio.get_running_loop()
        self._watch(loop)
        part = GpuPart(loop)
        with self._lock:
            lost = self._evicted.pop(gid, None) is not None
            if not lost:
                self._parts[gid] = part
            early = self._early.pop(gid, [])
        if lost:
            # its news was dropped from a full _early buffer (gpu_part_poll had already
            # collected the part natively): fail it now instead of waiting for good - the
            # caller refetches the part
            part._deliver(3, b"GPU part completion lost before it was tracked")
            return part
        for kind, data in early:
            self._dispatch(gid, part, kind, data)
        self.drain()                  # news that came before this loop watched the fd
        return part

    def _watch(self, loop) -> None:
        if loop in self._loops:
            return
        loop.add_reader(native().gpu_part_eventfd(), self.drain)
        self._loops.add(loop)

    def _dispatch(self, gid: int, part: GpuPart, kind: int, data: bytes) -> None:
        if kind != 1:
            with self._lock:
                self._parts.pop(gid, None)
        import asyncio
        try:
            running = asyncio.get_running_loop()
        except RuntimeError:
            running = None
        if running is part.loop:
            part._deliver(kind, data)
        elif not part.loop.is_closed():
            part.loop.call_soon_threadsafe(part._deliver, kind, data)

    def drain(self) -> None:
        for gid, kind, data in native().gpu_part_poll():
            with self._lock:
                part = self._parts.get(gid)
                if part is None:
                    # news before track() (the relay's executor thread returned the id, the
                    # loop has not run the tracker yet); bounded: an id nobody tracks (a
                    # caller that waits with gpu_part_wait) must not grow it for good
                    self._early.setdefault(gid, []).append((kind, data))
                    while len(self._early) > EARLY_MAX:
                        old = next(iter(self._early))
                        self._early.pop(old)
                        self._evicted[old] = True          # track(old) fails it fast
                        while len(self._evicted) > 4 * EARLY_MAX:
                            self._evicted.popitem(last=False)
                    continue
            self._dispatch(gid, part, kind, data)

    def pending(self) -> int:
        with self._lock:
            return len(self._parts)


_gpu_parts = _GpuParts()


def gpu_part_track(gid: int) -> GpuPart:
    """Futures of a part the relay queued to the GPU (``gpu_ticket``). Track every id once:
    a tracked part's buffer returns to the pool whether or not anybody awaits it."""
    return _gpu_parts.track(gid)


async def gpu_part_digests(gid: int) -> bytes:
    """Digests of a part the relay queued to the GPU (``gpu_ticket``)."""
    return await gpu_part_track(gid).done


def gpu_relay_stats() -> dict:
    d = dict(native().gpu_part_stats())
    d["tracked"] = _gpu_parts.pending()
    if _part_hasher is not None and hasattr(_part_hasher, "stats"):
        d.update({f"device_{k}": v for k, v in _part_hasher.stats().items()})
    return d


def host_multibuffer() -> bool:
    """The host runs the AVX-512 16-lane SHA-1 (``csrc/sha1_mb.cpp``)."""
    return bool(native().sha1_mb_supported())


def auto_may_use_gpu() -> bool:
    """Whether ``verify_backend=auto`` ever sends work to the GPU on this host."""
    return not host_multibuffer() and gpu_available()


def swarm_backend(requested: str, total_bytes: int, gpu_min_bytes: int) -> str:
    """Where the native peer wire SHA-1s a swarm torrent's pieces. ``auto``: the device when
    the host lacks the AVX-512 multi-buffer SHA-1, or for a torrent of at least
    ``gpu_min_bytes`` (0: never): on config 6 at 16 GB the device runs within ~5 % of the
    host's rate at 35 % less leech CPU per byte; at 2 GB its ~75 ms per piece costs 35 - 40 %
    of the rate (profiles/archive/r5/swarm/backpressure/)."""
    if requested == "cpu":
        return "cpu"
    if requested == "gpu":
        return "gpu"
    if host_multibuffer() and not (gpu_min_bytes and total_bytes >= gpu_min_bytes):
        return "cpu"
    return "gpu" if gpu_available() else "cpu"


def choose_backend(requested: str, total_bytes: int, n_pieces: int) -> str:
    if requested == "cpu":
        return "cpu"
    if requested == "gpu":
        if not gpu_available():
            raise RuntimeError("verify_backend=gpu but no HIP device is available")
        return "gpu"
    if host_multibuffer() or total_bytes < GPU_MIN_BYTES or n_pieces < GPU_MIN_PIECES:
        return "cpu"
    warm = _gpu_verifier is not None
    if (warm or total_bytes >= GPU_COLD_MIN_BYTES) and gpu_available():
        return "gpu"
    return "cpu"


def verify_pieces(files: FileList, piece_len: int, hashes: bytes,
                  which: Optional[Sequence[int]] = None, threads: int = 0,
                  backend: str = "cpu") -> bytes:
    """One byte per piece (1 = SHA-1 matches). With ``which``, one byte per listed piece in
    list order. ``backend="auto"`` picks the GPU only for a whole-storage recheck; a subset
    goes to the GPU when asked for explicitly (see ``GpuBatcher`` for the batched path).
    Only ``which=None`` asks for a full recheck: an empty ``which`` verifies nothing (the
    native calls read an empty list as "every piece")."""
    if which is not None:
        which = [int(i) for i in which]
        if not which:
            return b""
    files = [(str(p), int(n)) for p, n in files]
    total = sum(n for _, n in files)
    n_pieces = (total + piece_len - 1) // piece_len if total else 0
    if which is None:
        be = choose_backend(backend, total, n_pieces)
    else:
        be = "gpu" if backend == "gpu" and choose_backend("gpu", total, n_pieces) == "gpu" \
            else "cpu"
    if be == "gpu":
        v = _verifier()
        with _gpu_call_lock:
            ok, _timing = v.verify_files_streamed(files, piece_len, hashes,
                                                  which=which or [])
        return ok
    return native().verify_pieces(files, piece_len, hashes, which or [], threads)


# One GpuVerifier per process owns two pinned slots and two streams: calls are serialised.
_gpu_call_lock = threading.Lock()


class GpuBatcher:
    """Coalesces incremental piece checks (webseed runs, peer pieces) into few GPU launches.

    A lane hashes ~41 MB/s (SHA-1 is serial within a piece), so the GPU pays off only with
    hundreds of pieces in flight: every caller submits its pieces and gets a future; one
    thread takes everything pending for the same storage, verifies the union in ONE
    chunk-streamed call and resolves the futures. While a batch runs, the next one fills.
    Host cost per byte is a pread into pinned memory instead of a SHA-1 pass on a core.
    """

    def __init__(self, max_pieces: int = 8192):
        self.max_pieces = max_pieces
        self._cv = threading.Condition()
        self._pending: List[tuple] = []
        self._thread: Optional[threading.Thread] = None
        self.batches = 0
        self.pieces = 0

    def submit(self, files: FileList, piece_len: int, hashes: bytes, pieces: Sequence[int]):
        from concurrent.futures import Future
        fut: Future = Future()
        key = (tuple((str(p), int(n)) for p, n in files), int(piece_len), hashes)
        with self._cv:
            self._pending.append((key, list(pieces), fut))
            if self._thread is None:
                self._thread = threading.Thread(target=self._loop, name="gpu-verify",
                                                daemon=True)
                self._thread.start()
            self._cv.notify()
        return fut

    def _take(self):
        with self._cv:
            while not self._pending:
                self._cv.wait()
            key = self._pending[0][0]
            batch, rest, n = [], [], 0
            for item in self._pending:
                if item[0] == key and (n == 0 or n + len(item[1]) <= self.max_pieces):
                    batch.append(item)
                    n += len(item[1])
                else:
                    rest.append(item)
            self._pending = rest
            return key, batch

    def _loop(self) -> None:
        while True:
            key, batch = self._take()
            files, piece_len, hashes = key
            union = sorted({i for _, ps, _ in batch for i in ps})
            if not union:           # nothing to verify (never a whole-storage recheck)
                for _, _, fut in batch:
                    if fut.set_running_or_notify_cancel():
                        fut.set_result([])
                continue
            try:
                v = _verifier()
                with _gpu_call_lock:
                    ok, _t = v.verify_files_streamed(list(files), piece_len, hashes, which=union)
                pos = {p: ok[j] for j, p in enumerate(union)}
                self.batches += 1
                self.pieces += len(union)
                for _, ps, fut in batch:
                    if fut.set_running_or_notify_cancel():
                        fut.set_result([bool(pos[i]) for i in ps])
            except BaseException as e:  # surface to every waiter, keep serving
                for _, _, fut in batch:
                    if not fut.done():
                        fut.set_exception(e)


_batcher: Optional[GpuBatcher] = None


def gpu_batcher() -> GpuBatcher:
    global _batcher
    with _gpu_lock:
        if _batcher is None:
            _batcher = GpuBatcher()
        return _batcher
