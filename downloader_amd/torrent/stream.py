"""Streamed staging of webseed-only torrents: webseed -> S3, pieces verified on the way, no disk.

The reference downloads the whole torrent into ``<download_path>/<id>`` with webtorrent
(lib/download.js:43-123), walks it (lib/process.js) and uploads the media files
(lib/upload.js:34-52). When the torrent's only source is BEP-19 webseeds and the process
stage's answer is already known from the metainfo (``MediaSelector.find_virtual``), the
bytes need not land on disk at all:

* every multipart part of every selected file is ONE Range GET on the file's webseed URL,
  relayed into its UploadPart through L2-sized user-space chunks that are SHA-1'd in flight
  (``HttpConn::relay_body_hashed``): whole pieces inside the part are verified by the relay
  itself;
* a piece that straddles a part's end (or a file boundary) is assembled from the neighbouring
  parts' edge fragments plus - where it reaches into a file the selector drops - "gap" bytes
  fetched into memory, and verified once complete;
* a part whose pieces fail is fetched and uploaded again (S3 replaces a part number); a file
  becomes visible only at ``CompleteMultipartUpload``, issued after every piece covering it
  verified - and the job's commit point stays the done marker written by the upload stage.

Files the selector drops are never fetched (apart from gap bytes). Measured on the build box:
page-cache writes of ONE file top out at ~8 GB/s (inode lock, page allocation; tmpfs is
slower still, ``profiles/archive/s2_r1/stage_fs.jsonl``), which capped the 4 GB single-file config.
"""
from __future__ import annotations

import asyncio
import hashlib
import os
import time
import weakref
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set, Tuple

from ..models import keys
from ..stages.base import media_type
from ..net.http import TransportError
from ..utils.aio import gather_strict
from ..utils import membudget
from ..utils.log import redact_url
from .metainfo import Metainfo
from .session import TorrentError, webseed_url


@dataclass(eq=False)
class _Target:
    """One selected file and its staging object."""
    path: str
    key: str
    index: int                  # file index in the metainfo
    offset: int                 # torrent offset of the file's first byte
    size: int
    single: bool                # one PUT (<= multipart threshold) instead of multipart
    upload_id: str = ""
    etags: Dict[int, str] = field(default_factory=dict)
    completed: bool = False     # CompleteMultipartUpload succeeded (abort deletes the object)


@dataclass(eq=False)
class _Unit:
    """A contiguous torrent byte range fetched in one go: an S3 part of a target (relayed
    and hashed) or a gap (bytes of unselected files, fetched into memory for a boundary
    piece)."""
    uid: int
    start: int
    length: int
    target: Optional[_Target] = None
    num: int = 0                # part number (multipart targets)
    file_off: int = 0           # offset of the part inside its file
    skip: int = 0               # bytes before the first whole piece
    full: int = 0               # bytes of whole pieces
    attempts: int = 0
    state: str = "queued"       # queued | running | done - a unit is in the queue at most once
    again: bool = False         # fetch once more when the running fetch ends (bad neighbour piece)
    counted: bool = False       # its bytes are in StreamStager.done_bytes

    @property
    def end(self) -> int:
        return self.start + self.length

    def fragments(self) -> List[Tuple[int, int]]:
        """Torrent ranges of this unit that belong to boundary pieces (head, tail; a gap is
        one fragment)."""
        if self.target is None:
            return [(self.start, self.end)]
        out = []
        if self.skip:
            out.append((self.start, self.start + self.skip))
        t0 = self.start + self.skip + self.full
        if t0 < self.end:
            out.append((t0, self.end))
        return out


_active_stagers = 0
_trim_handle: Optional[asyncio.TimerHandle] = None


def _trim_relay_buffers() -> None:
    """Unmap the idle pooled part buffers of the hashed relay (as large as a part, one per
    relay that was in flight) - unless stream staging started again meanwhile."""
    global _trim_handle
    _trim_handle = None
    if _active_stagers:
        return
    try:
        from ..ops import native
        native().relay_pool_trim()
    except Exception:
        pass


# Idle part buffers are bounded in BYTES by the part budget (utils/membudget.py: leased +
# idle <= budget, enforced by the native pool), so their count needs no cap of its own.
POOL_IDLE_MAX = 4096
_gpu_pending_sems: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _gpu_pending_sem(n: int) -> asyncio.Semaphore:
    """Parts awaiting GPU digests, shared by every stream stager of the process (one per
    event loop): the device needs ~128 - 160 parts in flight to hide its per-piece latency,
    whether they come from one job or several. Since round 4 such a part holds no host memory
    once its DMA is over - only HBM (profiles/archive/r3_relayhash3/ for the count)."""
    loop = asyncio.get_running_loop()
    sem = _gpu_pending_sems.get(loop)
    if sem is None:
        sem = _gpu_pending_sems[loop] = asyncio.Semaphore(n)
    return sem


_gpu_init_started = False


def start_gpu_init(min_pieces: int, slots: int = 16, copy_streams: int = 2,
                   compute_streams: int = 0, slot_bytes: int = 1 << 30) -> None:
    """``auto``: set up the gfx950 PartHasher on an executor thread (HIP init and the device
    slots take a moment; the event loop keeps relaying meanwhile). Once per process; a
    missing device or a failed init leaves every part on the host."""
    global _gpu_init_started
    from ..ops import hashing
    if _gpu_init_started or hashing._part_hasher is not None or hashing._part_hasher_failed:
        return
    _gpu_init_started = True

    def init() -> bool:
        from ..ops import gpu_available
        return gpu_available() and hashing.gpu_relay_hashing(min_pieces, slots, slot_bytes,
                                                             copy_streams=copy_streams,
                                                             compute_streams=compute_streams)
    fut = asyncio.get_running_loop().run_in_executor(None, init)
    fut.add_done_callback(lambda f: f.cancelled() or f.exception())   # retrieved


def _schedule_trim(idle_s: float, keep_bytes: int = 0) -> None:
    """Last stream stager of the process finished: at once, idle buffers beyond ``keep_bytes``
    (what one job's relays in flight use) are unmapped; the rest after ``idle_s`` quiet
    seconds (0 = now), so back-to-back jobs reuse warm buffers while an idle worker holds
    none."""
    global _trim_handle
    if _trim_handle is not None:
        _trim_handle.cancel()
        _trim_handle = None
    if idle_s > 0 and keep_bytes > 0:
        try:
            from ..ops import native
            native().relay_pool_trim(keep_bytes)
        except Exception:
            pass
    if idle_s <= 0:
        _trim_relay_buffers()
    else:
        _trim_handle = asyncio.get_running_loop().call_later(idle_s, _trim_relay_buffers)


def piece_split(meta: Metainfo, start: int, length: int) -> Tuple[int, int]:
    """(skip, full) of the torrent range [start, start+length): ``skip`` bytes before the
    first whole piece, then ``full`` bytes of whole pieces (the torrent's short last piece
    counts as whole when the range reaches the end)."""
    plen, end = meta.piece_length, start + length
    ps = -(-start // plen) * plen
    pe = end if end == meta.total_length else (end // plen) * plen
    if pe <= ps:
        return min(ps - start, length), 0
    return ps - start, pe - ps


class StreamStager:
    def __init__(self, meta: Metainfo, job, cfg, sv, selected: List[str], root: str,
                 webseeds: List[str], parallel: int = 16, max_failures: int = 5):
        self.meta = meta
        self.job = job
        self.sv = sv
        self.s3 = sv.s3
        self.bucket = cfg.s3.bucket
        self.webseeds = list(webseeds)
        self.plen = meta.piece_length
        self.parallel = max(1, parallel)
        self.max_failures = max(1, max_failures)
        self.cfg = cfg
        self.trim_idle_s = float(getattr(getattr(cfg, "download", None),
                                         "relay_pool_idle_trim_s", 0.0) or 0.0)
        # every relayed part draws its buffer's bytes from the process-wide budget
        self.budget_bytes = membudget.relay_budget_bytes(getattr(cfg, "download", None))
        self._budget: Optional[membudget.PartBudget] = None
        index = {os.path.abspath(p): i for i, (p, _) in enumerate(meta.local_files(root))}
        self.selected = [os.path.abspath(f) for f in selected]
        self.sizes = {f: meta.files[index[f]].length for f in self.selected}
        owner: Dict[str, str] = {}
        for f in self.selected:
            owner[keys.object_key(job.id, f)] = f       # the later file wins the key (App. A #10)
        self.targets: List[_Target] = []
        self.units: List[_Unit] = []
        for key, f in owner.items():
            fe = meta.files[index[f]]
            t = _Target(f, key, index[f], fe.offset, fe.length,
                        fe.length <= self.s3.multipart_threshold)
            self.targets.append(t)
            if t.size == 0:
                continue
            parts = [(0, 0, t.size)] if t.single else \
                self.s3.plan_parts(t.size, fe.offset, meta.piece_length)
            for num, off, ln in parts:
                skip, full = piece_split(meta, t.offset + off, ln)
                self.units.append(_Unit(len(self.units), t.offset + off, ln, t, num, off,
                                        skip, full))
        # boundary pieces: piece -> {torrent offset: fragment}, and the units supplying them
        self.frags: Dict[int, Dict[int, bytes]] = {}
        self.suppliers: Dict[int, Set[int]] = {}
        self._plan_gaps()
        self.verified: Set[int] = set()
        self._checking: Set[int] = set()
        # boundary piece -> version of its fragment set, bumped whenever a fragment is
        # stored, replaced or dropped: a check whose snapshot is stale does not count
        self.frag_ver: Dict[int, int] = {}
        self.piece_fails: Dict[int, int] = {}
        self.total = sum(t.size for t in self.targets)
        self.fetched_bytes = 0
        self.done_bytes = 0
        self.hash_fails = 0
        self.error: Optional[BaseException] = None
        self._outstanding = 0
        self._finished = asyncio.Event()
        self.stats = {"relay_s": 0.0, "gap_bytes": 0, "units": 0}
        # seconds since run() began: uploads created, first / last relay over, last device
        # digest in, every unit settled, uploads completed (where a job's time goes)
        self.timeline: Dict[str, float] = {}
        self._t0 = time.monotonic()
        # GPU piece hashing of relayed parts: at most this many parts awaiting digests,
        # across every stream stager of the process
        self._gpu_slots: Optional[asyncio.Semaphore] = None
        self.gpu_pending = 0
        self._continuations: Set[asyncio.Task] = set()
        d = getattr(cfg, "download", None)
        gpu_pending = int(getattr(d, "stream_gpu_pending", 0) or 0)
        self.verify_mode = getattr(d, "stream_verify_backend", "cpu") if gpu_pending > 0 else "cpu"
        self._min_pieces = int(getattr(d, "stream_gpu_min_pieces", 8) or 8)
        self._gpu_dev_slots = int(getattr(d, "stream_gpu_slots", 16) or 16)
        self._gpu_copy_streams = int(getattr(d, "stream_gpu_copy_streams", 2) or 2)
        self._gpu_compute_streams = int(getattr(d, "stream_gpu_compute_streams", 0) or 0)
        self._gpu_slot_bytes = int(getattr(d, "stream_gpu_slot_mb", 1024) or 1024) << 20
        # parts still queued below which the rest hash on the host
        self.gpu_tail = int(getattr(d, "stream_gpu_tail", 0) or 0)
        self._n_parts = sum(1 for u in self.units if u.target is not None)
        from ..ops import hashing
        try:
            self._host_mb = hashing.host_multibuffer()
        except Exception:
            self._host_mb = False
        if self.verify_mode == "auto":
            # the device is set up off the event loop when it is first wanted (run()); parts
            # go to it once it is ready
            self.gpu_pending = gpu_pending
            self.stats["verify"] = "auto"
        if self.verify_mode == "gpu":
            why = _gpu_relay_on(cfg)
            if why is None:
                self.gpu_pending = gpu_pending    # the process-wide budget (run())
                self.stats["verify"] = "gpu"
            else:
                self.stats["verify_fallback"] = why
                job.logger.warn("GPU piece hashing unavailable, hashing on the host", err=why)

    # ---------------------------------------------------------------- planning
    def _piece_range(self, p: int) -> Tuple[int, int]:
        return p * self.plen, p * self.plen + self.meta.piece_size(p)

    def _plan_gaps(self) -> None:
        covered: Dict[int, List[Tuple[int, int]]] = {}
        for u in self.units:
            for a, b in u.fragments():
                p = a // self.plen
                covered.setdefault(p, []).append((a, b))
                self.suppliers.setdefault(p, set()).add(u.uid)
        for p in sorted(covered):
            lo, hi = self._piece_range(p)
            pos = lo
            for a, b in sorted(covered[p]) + [(hi, hi)]:
                if a > pos:
                    g = _Unit(len(self.units), pos, a - pos)
                    self.units.append(g)
                    self.suppliers[p].add(g.uid)
                pos = max(pos, b)
            self.frags[p] = {}

    @property
    def progress(self) -> float:
        """Fraction of the selected bytes relayed and verified (the ticker / stall watchdog
        of lib/download.js:78-101 sample it like webtorrent's ``torrent.progress``)."""
        return 1.0 if self.total == 0 else min(1.0, self.done_bytes / self.total)

    def skipped_bytes(self) -> int:
        """Torrent bytes never fetched (files the selector drops)."""
        return self.meta.total_length - sum(u.length for u in self.units)

    # ---------------------------------------------------------------- execution
    async def run(self) -> List[dict]:
        """Stage every selected file; return the ``streamed`` entries (walk order, every
        selected file - the upload stage resolves key ownership) for the later stages."""
        global _active_stagers
        multi = [t for t in self.targets if not t.single and t.size]
        _active_stagers += 1
        if _trim_handle is not None:           # a job started inside the warm window
            _trim_handle.cancel()
        self._budget = membudget.part_budget(self.budget_bytes)
        self._t0 = time.monotonic()
        self.stats["timeline"] = self.timeline
        try:
            from ..ops import native
            native().relay_pool_set_max_idle(POOL_IDLE_MAX)
        except Exception:
            pass
        if self.verify_mode == "auto" and self._gpu_wanted():
            start_gpu_init(self._min_pieces, self._gpu_dev_slots, self._gpu_copy_streams,
                           self._gpu_compute_streams, self._gpu_slot_bytes)
        try:
            for t in self.targets:
                if t.size == 0:
                    await self.s3.put_object(self.bucket, t.key, b"", self._ctype(t))
            async def create(t: _Target) -> None:
                t.upload_id = await self.s3.create_multipart_upload(
                    self.bucket, t.key, self._ctype(t),
                    checksum=self.s3.want_checksum(relay=True, hashed=True))
            # all creations settle before a failure propagates: abort() then sees every
            # upload that was opened (none is left behind on the bucket)
            await gather_strict(*(create(t) for t in multi), cancel=False)
            self._mark("created_s")
            queue: "asyncio.Queue[_Unit]" = asyncio.Queue()
            for u in self.units:
                queue.put_nowait(u)
            self._outstanding = len(self.units)
            if not self.units:
                self._finished.set()
            workers = [asyncio.ensure_future(self._worker(queue)) for _ in range(self.parallel)]
            try:
                await self._finished.wait()
                self._mark("settled_s")
            finally:
                for w in workers + list(self._continuations):
                    w.cancel()
                await asyncio.gather(*workers, *self._continuations, return_exceptions=True)
            if self.error is not None:
                raise self.error
            unverified = [p for p in self.frags if p not in self.verified]
            if unverified:
                raise TorrentError(f"pieces {unverified[:5]} never verified")
            async def complete(t: _Target) -> None:
                await self.s3.complete_multipart_upload(self.bucket, t.key, t.upload_id,
                                                        sorted(t.etags.items()))
                t.completed = True
            await gather_strict(*(complete(t) for t in multi), cancel=False)
            self._mark("completed_s")
        except BaseException:
            await asyncio.shield(self.abort())
            raise
        finally:
            _active_stagers -= 1
            self.stats["budget"] = self._budget.stats()
            if _active_stagers == 0:
                # keep warm what one job's relays take, the rest goes now
                _schedule_trim(self.trim_idle_s,
                               self.parallel * membudget.buffer_bytes(self.s3.part_size))
        return [{"file": f, "key": keys.object_key(self.job.id, f), "size": self.sizes[f],
                 "virtual": True} for f in self.selected]

    async def _worker(self, queue: "asyncio.Queue[_Unit]") -> None:
        while True:
            u = await queue.get()
            u.state = "running"
            if u.target is not None and self._gpu_sem() is not None:
                # GPU piece hashing: this worker only moves the part's bytes; waiting for the
                # digests (~piece_len / 58 MB/s on the device) and the checks run in a
                # continuation, so the relay slots stay busy relaying meanwhile
                await self._gpu_slots.acquire()
                try:
                    nb = await self._budget.acquire(u.length)
                except BaseException:
                    self._gpu_slots.release()
                    raise
                # the job's last parts hash on the host: their GPU latency (~piece_len / 58
                # MB/s) would land on the end of the job with nothing left to overlap it
                gpu = self._gpu_now() and queue.qsize() >= self.gpu_tail
                try:
                    res = await self._relay_part(u, gpu)
                except BaseException as e:
                    self._release_after(e, nb)
                    self._gpu_slots.release()
                    if not await self._unit_failed(u, e, queue):
                        return
                    continue
                gid = res[1].get("gpu_ticket")
                if gid:
                    from ..ops import hashing
                    try:
                        part = hashing.gpu_part_track(gid)
                    except BaseException as e:
                        # untracked, the part would keep its budget bytes, its GPU slot and
                        # its native record for good: drop it - the bytes come
                        # back once its DMA is over - then fail the unit as usual
                        await self._forget_part(gid)
                        self._budget.release(nb)
                        self._gpu_slots.release()
                        if not await self._unit_failed(u, e, queue):
                            return
                        continue
                    # the buffer is back in the pool once the DMA is over: so are its bytes
                    part.copied.add_done_callback(lambda _f, nb=nb: self._budget.release(nb))
                    t = asyncio.ensure_future(self._complete(u, res, part, queue))
                    self._continuations.add(t)
                    t.add_done_callback(self._continuations.discard)
                    continue
                self._budget.release(nb)
                self._gpu_slots.release()         # hashed on the host after all (refused)
                try:
                    requeue = await self._after_fetch(u, self._accept(u, *res,
                                                                       res[1]["digests"]))
                except BaseException as e:
                    if not await self._unit_failed(u, e, queue):
                        return
                    continue
            else:
                try:
                    requeue = await self._process(u)
                except BaseException as e:
                    if not await self._unit_failed(u, e, queue):
                        return
                    continue
            if self.error is not None:
                return
            self._settle(u, requeue, queue)

    def _mark(self, key: str, first: bool = False) -> None:
        t = round(time.monotonic() - self._t0, 4)
        if not first or key not in self.timeline:
            self.timeline[key] = t

    def _release_after(self, e: BaseException, nb: int) -> None:
        """A failed / cancelled relay's budget bytes: back now, or - when the cancellation
        could not wait for the GPU hasher to hand the part's buffer back (``held_until``, set
        by the transport) - once it has."""
        held = getattr(e, "held_until", None)
        if held is not None and not held.done():
            held.add_done_callback(lambda _f, nb=nb: self._budget.release(nb))
        else:
            self._budget.release(nb)

    async def _forget_part(self, gid: int) -> None:
        """Drop a queued GPU part nobody will collect (blocks until its DMA is over, so on a
        thread)."""
        from ..ops import native
        try:
            await asyncio.get_running_loop().run_in_executor(None, native().gpu_part_forget, gid)
        except Exception:
            pass

    def _gpu_wanted(self) -> bool:
        """``auto``: is the device worth it? When the host lacks the AVX-512 SHA-1, when jobs
        share the worker, or when this job has more parts than the host-hashed tail - config
        4 on the MI355X box, steady reps: one job 26.3 - 28.0 GB/s at 6.5 - 6.6 worker CPU-s
        with the last 96 parts on the host vs 24.8 - 25.4 at 7.7 - 8.2 all on the host, two
        jobs 26.5 - 28.4 vs 23.7 - 25.5 at 13 - 14 vs 17 - 18 CPU-s (profiles/archive/r3_tail2/)."""
        return not self._host_mb or _active_stagers >= 2 or self._n_parts > self.gpu_tail

    def _gpu_sem(self) -> Optional[asyncio.Semaphore]:
        """The process-wide budget of parts awaiting GPU digests, once a hasher is ready
        (``gpu``: set up in __init__; ``auto``: by ``start_gpu_init``); None = host only."""
        if self._gpu_slots is None and self.gpu_pending:
            from ..ops import hashing
            if hashing._part_hasher is not None:
                self._gpu_slots = _gpu_pending_sem(self.gpu_pending)
        return self._gpu_slots

    def _gpu_now(self) -> bool:
        """Hash this part's pieces on the device? ``gpu``: always; ``auto``: _gpu_wanted().
        (Either way the job's last ``stream_gpu_tail`` queued parts stay on the host.)"""
        if self.verify_mode == "gpu":
            return True
        if self._gpu_wanted():
            return True
        return False

    async def _unit_failed(self, u: _Unit, e: BaseException,
                           queue: "asyncio.Queue[_Unit]") -> bool:
        """A unit's fetch raised: transport errors are retried (backoff, then the unit goes
        back to the queue), anything else - or too many attempts - fails the stager.
        False = the caller's loop must stop."""
        if not isinstance(e, (TransportError, OSError)):
            self._fail(e)
            return False
        u.attempts += 1
        if u.attempts >= self.max_failures:
            self._fail(TorrentError(f"webseed failed: {e}"))
            return False
        await asyncio.sleep(min(5.0, 0.1 * (2 ** u.attempts)))
        if self.error is not None:
            return False
        self._settle(u, [u], queue)
        return True

    async def _complete(self, u: _Unit, res, part, queue: "asyncio.Queue[_Unit]") -> None:
        """Continuation of a part whose pieces the GPU hashes: digests, checks, settle."""
        etag, h = res
        try:
            try:
                digests = await part.done
            except RuntimeError as e:
                # the device failed after the part's buffer went back to the pool: the
                # bytes are gone, so the part is fetched (and relayed) again - its next
                # relay hashes on the host if the hasher now refuses work
                self.stats["gpu_failures"] = self.stats.get("gpu_failures", 0) + 1
                raise TransportError(f"part {u.num}: {e}") from e
            self.stats["gpu_parts"] = self.stats.get("gpu_parts", 0) + 1
            self._mark("last_gpu_digest_s")
            requeue = await self._after_fetch(u, self._accept(u, etag, h, digests))
        except BaseException as e:
            self._gpu_slots.release()
            await self._unit_failed(u, e, queue)
            return
        self._gpu_slots.release()
        if self.error is None:
            self._settle(u, requeue, queue)

    def _settle(self, u: _Unit, requeue: List[_Unit], queue: "asyncio.Queue[_Unit]") -> None:
        """``u``'s fetch ended; ``requeue`` = units whose bytes must be fetched again. A unit
        is never queued twice: a queued one stays as it is, a running one is flagged
        ``again`` (it goes back to the queue when its fetch ends), a done one returns to the
        queue and counts as outstanding again."""
        redo = {r.uid: r for r in requeue}
        if u.again:
            u.again = False
            redo[u.uid] = u
        for r in redo.values():
            for a, _ in r.fragments():               # its fragments are fetched again
                p = a // self.plen
                self.frags[p].pop(a, None)
                self.frag_ver[p] = self.frag_ver.get(p, 0) + 1
                self.verified.discard(p)
            if r.counted:
                r.counted = False
                self.done_bytes -= r.length
        for r in redo.values():
            if r is u:
                continue
            if r.state == "done":
                r.state = "queued"
                self._outstanding += 1
                queue.put_nowait(r)
            elif r.state == "running":
                r.again = True
        if u.uid in redo:
            u.state = "queued"
            queue.put_nowait(u)
        else:
            u.state = "done"
            self._outstanding -= 1
        if self._outstanding == 0:
            self._finished.set()

    def _fail(self, e: BaseException) -> None:
        if self.error is None:
            self.error = e
        self._finished.set()

    def _ctype(self, t: _Target) -> str:
        return media_type(self.cfg, t.path)

    def _base(self, u: _Unit) -> str:
        return self.webseeds[(u.uid + u.attempts) % len(self.webseeds)]

    async def _process(self, u: _Unit) -> List[_Unit]:
        """Fetch one unit; return the units that must be fetched again (bad pieces)."""
        if u.target is None:
            return await self._after_fetch(u, [(u.start, await self._fetch_gap(u))])
        nb = await self._budget.acquire(u.length)
        try:
            etag, h = await self._relay_part(u)
        finally:
            self._budget.release(nb)
        return await self._after_fetch(u, self._accept(u, etag, h, h["digests"]))

    async def _after_fetch(self, u: _Unit, got: Optional[List[Tuple[int, bytes]]]) -> List[_Unit]:
        """Fragments of a fetched unit into the boundary pieces (checked once complete);
        ``got`` None = a whole piece inside the part failed its hash."""
        if got is None:
            u.attempts += 1
            if u.attempts >= self.max_failures:
                raise TorrentError("webseed served corrupt pieces")
            return [u]
        pieces = got
        self.stats["units"] += 1
        requeue: List[_Unit] = []
        for a, data in pieces:
            p = a // self.plen
            self.frags[p][a] = data
            self.frag_ver[p] = self.frag_ver.get(p, 0) + 1
            if await self._check_piece(p):
                requeue += [self.units[i] for i in sorted(self.suppliers[p])]
        return requeue

    async def _relay_part(self, u: _Unit, gpu: bool = False):
        """Relay one part webseed -> S3 (its whole pieces hashed on the way - by the host
        multi-buffer SHA-1, or queued to the GPU: then ``h["gpu_ticket"]``)."""
        t = u.target
        url = webseed_url(self.meta, self._base(u), t.index)
        whole = u.file_off == 0 and u.length == t.size
        t0 = time.perf_counter()
        etag, h = await self.s3.relay_hashed(
            self.bucket, t.key, url, u.file_off, u.length, whole, (u.skip, u.full, self.plen),
            part=None if t.single else (u.num, t.upload_id), content_type=self._ctype(t),
            gpu=gpu)
        self.stats["relay_s"] += time.perf_counter() - t0
        self._mark("first_relay_s", first=True)
        self._mark("last_relay_s")
        if gpu and h.get("gpu_ticket"):
            self._mark("last_gpu_relay_s")
        self.fetched_bytes += u.length
        return etag, h

    def _accept(self, u: _Unit, etag: str, h: dict,
                digests: bytes) -> Optional[List[Tuple[int, bytes]]]:
        """Check a relayed part's whole pieces; None = one failed (refetch the part)."""
        t = u.target
        first = (u.start + u.skip) // self.plen
        if len(digests) != 20 * (-(-u.full // self.plen)):
            # never accept a part whose pieces were not all hashed
            raise TorrentError(f"part {u.num}: {len(digests) // 20} digests for "
                               f"{-(-u.full // self.plen)} pieces")
        for k in range(len(digests) // 20):
            if digests[20 * k:20 * k + 20] != self.meta.piece_hash(first + k):
                self.hash_fails += 1
                return None
        if not t.single:
            t.etags[u.num] = etag
        if not u.counted:
            u.counted = True
            self.done_bytes += u.length
        out = []
        if u.skip:
            out.append((u.start, h["head"]))
        if h["tail"]:
            out.append((u.start + u.skip + u.full, h["tail"]))
        return out

    async def _fetch_gap(self, u: _Unit) -> bytes:
        buf = bytearray()
        for fi, foff, ln in self.meta.file_spans(u.start, u.length):
            url = webseed_url(self.meta, self._base(u), fi)
            r = await self.sv.transports.request(
                "GET", url, headers=[("Range", f"bytes={foff}-{foff + ln - 1}")])
            if r.status != 206 or len(r.body) != ln:
                raise TransportError(f"webseed {redact_url(url)}: HTTP {r.status}, "
                                     f"{len(r.body)}/{ln} B",
                                     r.status)
            buf += r.body
        self.fetched_bytes += u.length
        self.stats["gap_bytes"] += u.length
        return bytes(buf)

    async def _check_piece(self, p: int) -> bool:
        """Verify boundary piece ``p`` once all its fragments are in; True = it failed. A
        piece already being hashed (its last fragment arrived twice) is not checked again
        here: the running check sees the version bump and re-checks. Large pieces are hashed
        in an executor while the loop runs on, so ``_settle`` may drop or replace a fragment
        meanwhile; the verdict only counts if the fragment set is still the hashed one."""
        while True:
            got = self.frags[p]
            lo, hi = self._piece_range(p)
            if p in self.verified or p in self._checking or \
                    sum(len(b) for b in got.values()) != hi - lo:
                return False
            ver = self.frag_ver.get(p, 0)
            # the fragments in order, hashed where they lie (joining them first copied every
            # boundary piece once more on the event loop: ~0.05 CPU-s/GB of a 50-file torrent)
            frags = [got[a] for a in sorted(got)]
            self._checking.add(p)
            try:
                if hi - lo >= 1 << 20:
                    digest = await asyncio.get_running_loop().run_in_executor(None, _sha1v, frags)
                else:
                    digest = _sha1v(frags)
            finally:
                self._checking.discard(p)
            if self.frag_ver.get(p, 0) != ver:
                continue                     # fragments changed while hashing: check again
            if digest == self.meta.piece_hash(p):
                self.verified.add(p)
                return False
            self.hash_fails += 1
            self.piece_fails[p] = self.piece_fails.get(p, 0) + 1
            if self.piece_fails[p] >= self.max_failures:
                raise TorrentError(f"webseed served corrupt data for piece {p}")
            return True

    async def abort(self) -> None:
        """Drop what a failed attempt staged: open multipart uploads, single-PUT objects."""
        for t in self.targets:
            try:
                if t.upload_id and not t.completed:
                    await self.s3.abort_multipart_upload(self.bucket, t.key, t.upload_id)
                elif t.single or t.completed:
                    await self.s3.delete_object(self.bucket, t.key)
            except Exception:
                pass


def _sha1(b: bytes) -> bytes:
    return hashlib.sha1(b).digest()


def _sha1v(parts) -> bytes:
    """SHA-1 of the concatenation of ``parts`` without building it (hashlib drops the GIL on
    large updates)."""
    h = hashlib.sha1()
    for b in parts:
        h.update(b)
    return h.digest()


def _gpu_relay_on(cfg) -> Optional[str]:
    """``download.stream_verify_backend: gpu``: set up the gfx950 PartHasher (once per
    process). None when the relayed parts' pieces will be hashed on the device, else why not
    (no HIP device, init failure) - the host multi-buffer SHA-1 then hashes them."""
    from ..ops import hashing
    d = getattr(cfg, "download", None)
    if hashing._part_hasher is not None:         # already set up (or a test double)
        return None
    try:
        if hashing.gpu_relay_hashing(getattr(d, "stream_gpu_min_pieces", 8),
                                     getattr(d, "stream_gpu_slots", 16),
                                     int(getattr(d, "stream_gpu_slot_mb", 1024) or 1024) << 20,
                                     copy_streams=getattr(d, "stream_gpu_copy_streams", 2),
                                     compute_streams=getattr(d, "stream_gpu_compute_streams",
                                                             0)):
            return None
        return "no usable HIP device"
    except Exception as e:
        return f"{type(e).__name__}: {e}"
