#!/usr/bin/env python3
"""Headline benchmark: MB/s staged end-to-end (download -> S3) + p50 job latency.

BASELINE.json names the metric "MB/s staged end-to-end (download->S3) + p50 job latency at
1/2/4/8 workers" and config 2 "100x100 MB HTTP URLs, N concurrent workers -> MinIO multipart".
One rank = one worker process (the reference's scaling unit: one consumer per container,
SURVEY §2.6). One "step" = every worker stages a batch of ``--jobs-per-step`` 100 MB
random-byte media blobs (default 64; like a training batch, it keeps the timed region long
enough to be stable), each job being the worker's full path: done-marker probe -> HTTP
origin -> (default ``--staging stream``: each multipart part relayed origin->S3 by splice;
``--staging disk``: download to the job dir first) -> media selection -> S3 multipart upload
-> done marker -> api.Convert published -> ack. Weak scaling: per-worker work is fixed as N
grows.

Launch: ``python bench.py`` (N=1) or ``python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N``. Each rank starts its own native ``blobd`` peer (origin + S3 sink;
``--peers shared`` = one on rank 0) and pins itself to its GPU slot's CPU share (the same
at every N, so the 1/2/4/8 curve is weak scaling of one slot's host resources); ranks
synchronise over gloo (the workload is host-side: there is no tensor compute).

Objects above 64 MiB go as S3 multipart uploads of 64 MiB parts (minio-js' split), so a 100 MB
job is 2 parts. Every PUT and part carries a CRC32C of its payload (``s3.checksum: always``, the
default since round 6: the relay peeks each byte once into user space for it), like minio-js
hashes every byte it uploads (lib/upload.js:45). The run fails unless the S3 peer's own
counters, sampled at "go" and after the last timed job, show (a) at least as many bytes
received as the workers claim to have staged, (b) every timed media PUT / part carrying a
CRC32C and none refused for a wrong one - the peer recomputes the CRC of a salted 1-in-8
subset of the bodies (``--sink-crc-check``), so a wrong CRC is caught without the bench's S3
re-reading every byte on the worker's CPUs - and (c) with ``--sink sample`` (default) /
``verify``, every timed object matched against the bytes the origin generated for it (sampled
windows / every byte) with zero mismatches. The origin's bytes repeat with a period of
64 MiB + 4 KiB, so a part or piece fetched from the wrong offset never matches.

Same-call extras of the line: ``unchecked_MBps`` (``s3.checksum: auto``: the plain relay
spliced with no payload checksum), ``reference_mode_MBps`` (reference-equivalent mode,
BASELINE.md: one serial prefetch-1 consumer per process, ``--ref-procs`` of them, on the same
CPUs; ``vs_baseline`` = headline / it), ``workers_curve`` (MB/s and p50 at 1/2/4/8 worker
processes of the rank), config 1's p50 (a single 10 MB job, tuned and reference mode) and the
streamed-torrent GPU vs host A/B.
"""
from __future__ import annotations

import argparse
import asyncio
import contextlib
import json
import os
import shutil
import statistics
import sys
import tempfile
import time
from typing import Optional

os.environ.setdefault("LOG_LEVEL", "warn")
REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "MB/s staged end-to-end (download->S3) + p50 job latency"


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1, help="worker processes (one per GPU slot)")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size-mb", type=float, default=100.0, help="object size in MB (1e6 B)")
    p.add_argument("--mode", choices=["tuned", "reference"], default="tuned")
    p.add_argument("--concurrency", type=int, default=4,
                   help="jobs in flight per worker process (4: with 2-part multipart jobs this "
                        "keeps 16 relays in flight per rank - 70.3 GB/s, p50 11 ms vs 49.3 GB/s, "
                        "27 ms at 8: profiles/archive/r3_mp_sweep); lowered when the uid's pipe "
                        "budget could not give every relay a 512 KiB pipe (utils/limits.relay_plan)")
    p.add_argument("--jobs-per-step", type=int, default=64,
                   help="jobs per worker per step (64: ~1 s timed at N=1 for 10 steps; 16/32/64 "
                        "give the same MB/s, profiles/archive/s2_r1/jobs_ab.jsonl)")
    p.add_argument("--stage-dir", default="", help="download_path (default: a temp dir)")
    p.add_argument("--http-streams", type=int, default=0, help="override download.http_streams")
    p.add_argument("--part-mb", type=int, default=0, help="override s3.part_size (MiB)")
    p.add_argument("--inflight-parts", type=int, default=0, help="override s3.max_inflight_parts")
    p.add_argument("--threshold-mb", type=int, default=0,
                   help="override s3.multipart_threshold (MiB; objects up to it go in one PUT)")
    p.add_argument("--staging", choices=["stream", "disk"], default="stream",
                   help="stream: single-file HTTP jobs relay origin->S3; disk: stage on disk first")
    p.add_argument("--peers", choices=["per-rank", "shared"], default="per-rank",
                   help="one blobd origin+S3 peer per worker, or one shared on rank 0")
    p.add_argument("--sink", choices=["sample", "verify", "discard", "checksum"], default="sample",
                   help="blobd S3 sink: sample = drop bodies in the kernel (MSG_TRUNC) but compare a 4 KiB "
                        "window of every MiB (and each body's tail) with the origin generator's "
                        "bytes at the object offset; verify = compare every byte (checksum of the "
                        "body vs checksum of the generated range); discard = no check; checksum "
                        "= fold every byte, no comparison")
    p.add_argument("--compare-single-put", dest="compare_single_put", action="store_true",
                   help="add a same-call run with round-2 settings (objects up to 128 MiB in one "
                        "PUT)")
    p.add_argument("--no-compare-single-put", dest="compare_single_put", action="store_false")
    p.add_argument("--no-compare-unchecked", "--no-compare-crc", dest="compare_unchecked",
                   action="store_false",
                   help="skip the same-call run of the unchecked spliced relay (--checksum auto)")
    p.add_argument("--sink-crc-check", type=int, default=8,
                   help="the S3 peer recomputes the CRC32C of 1 in N checksummed bodies (a "
                        "salted hash of key + part picks them); the rest must carry a "
                        "well-formed CRC and are dropped in the kernel")
    p.add_argument("--pipe-kb", type=int, default=0,
                   help="splice pipe KiB per transfer (0: the uid's pipe budget / workers)")
    p.add_argument("--checksum", choices=["auto", "always", "off"], default="",
                   help="s3.checksum: CRC32C per PUT/part (auto = where bytes cross user space "
                        "anyway, i.e. not this plain-http splice relay; always = the relay copies "
                        "through user space to compute it)")
    p.add_argument("--cpus-per-rank", type=int, default=0,
                   help="pin each rank (worker + its peer) to this many CPUs; 0: its GPU slot's "
                        "share, min(mask, cgroup quota) / visible GPUs; -1: no pinning")
    p.add_argument("--procs-per-rank", type=int, default=0,
                   help="worker processes per rank; 0: one per 4 CPUs of the rank's slice")
    p.add_argument("--tls", choices=["off", "native", "aiohttp"], default="off",
                   help="origin and S3 over https (self-signed blobd certificate): TLS in the "
                        "native transport's threads, or through aiohttp on the event loop")
    p.add_argument("--torrent-gb", type=float, default=20.0,
                   help="same-call GPU vs host A/B of the streamed torrent path on a config-4 "
                        "shaped torrent of this many GB (50 files, 4 MiB pieces; 0 = skip)")
    p.add_argument("--torrent-timeout", type=float, default=300.0,
                   help="seconds the torrent A/B may take before it is reported as failed")
    p.add_argument("--torrent-pairs", type=int, default=3,
                   help="timed jobs per backend in the torrent A/B (alternating)")
    p.add_argument("--no-compare-reference", dest="compare_reference", action="store_false",
                   help="skip the same-call reference-equivalent run (vs_baseline then null)")
    p.add_argument("--compare-reference", dest="compare_reference", action="store_true")
    p.add_argument("--sink-crc-salt", type=int, default=0,
                   help="salt of the sink's CRC subset (0: random per run)")
    p.add_argument("--ref-procs", type=int, default=8,
                   help="reference mode: serial prefetch-1 consumers (processes) on the rank's "
                        "CPUs - BASELINE.json config 2 runs 8 workers")
    p.add_argument("--ref-jobs", type=int, default=128, help="reference mode: timed jobs")
    p.add_argument("--ref-warmup-jobs", type=int, default=2,
                   help="reference mode: untimed jobs per process first")
    p.add_argument("--workers-curve", default="1,2,4,8",
                   help="worker-process counts of the same-call curve (MB/s + p50 at each; "
                        "'' = skip)")
    p.add_argument("--curve-steps", type=int, default=6, help="timed steps per curve point")
    p.add_argument("--no-config1", dest="config1", action="store_false",
                   help="skip the same-call config 1 (single 10 MB job) p50, tuned and reference")
    p.add_argument("--curve-warmup-jobs", type=int, default=8,
                   help="untimed jobs per worker process before each curve point")
    return p.parse_args()


@contextlib.contextmanager
def _stdout_to_stderr():
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class Dist:
    def __init__(self, want: int):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            # gloo reports "[Gloo] Rank r is connected to ..." on fd 1; the driver reads rank
            # 0's stdout for the ONE result line, so the rendezvous chatter goes to stderr.
            with _stdout_to_stderr():
                dist.init_process_group("gloo")
            self.dist = dist
        if want != self.world and self.rank == 0:
            print(f"[bench] --gpus {want} but WORLD_SIZE={self.world}; using {self.world} workers",
                  file=sys.stderr)

    def barrier(self) -> None:
        if self.world > 1:
            self.dist.barrier()

    def bcast(self, obj):
        if self.world == 1:
            return obj
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=0)
        return lst[0]

    def gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self) -> None:
        if self.world > 1:
            self.dist.destroy_process_group()


def cuda_sync() -> None:
    # The driver's contract brackets the timed region with a device sync; the staging path does
    # not use the device for HTTP jobs, so this is a no-op unless torch already initialised it.
    torch = sys.modules.get("torch")      # (never imported just for this: ~1.5 s of CPU)
    try:
        if torch is not None and torch.cuda.is_initialized():   # never initialise HIP here
            torch.cuda.synchronize()
    except Exception:
        pass


async def run_phase(worker, blob_ep_url, rank: int, first: int, count: int, size: int,
                    tag: str, media_type: str = "MOVIE"):
    from downloader_amd.models import api
    done = asyncio.Event()
    results = []

    def on_result(r):
        results.append(r)
        if len(results) >= count:
            done.set()
    worker.on_result = on_result
    t0 = time.perf_counter()
    for i in range(first, first + count):
        url = blob_ep_url(f"r{rank}-j{i}.mkv", size, rank * 1_000_003 + i)
        await worker.submit(api.make_download(f"bench-{tag}-r{rank}-j{i}", "http", url, media_type))
    if count:
        await done.wait()
    dt = time.perf_counter() - t0
    worker.on_result = None
    return dt, results


async def _start_worker(args, endpoint: str, mode: str, stage_root: str):
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.service.worker import Worker
    from downloader_amd.utils.config import load_config

    over = {
        "mode": mode,
        "concurrency": args.concurrency,
        "instance": {"download_path": stage_root},
        "s3": {"endpoint": endpoint},
        # HTTP staging never verifies torrent pieces: no GPU verifier (HIP init, pinned slots)
        "download": {"gpu_prewarm": False},
        "broker": {"backend": "memory"},
        "health": {"enabled": False},
    }
    if getattr(args, "pipe_kb_eff", 0):
        over["download"]["pipe_kb"] = args.pipe_kb_eff
    ca = getattr(args, "ca_file", "")
    if args.tls != "off":
        over["s3"]["secure"] = True
        over["tls"] = {"ca_file": ca, "native": args.tls == "native"}
    if args.checksum:
        over["s3"]["checksum"] = args.checksum
    if mode == "tuned":
        if getattr(args, "single_put", False):   # round-2 headline settings, for comparison
            over["s3"]["multipart_threshold"] = 128 << 20
        if args.http_streams:
            over["download"]["http_streams"] = args.http_streams
        if args.part_mb:
            over["s3"]["part_size"] = args.part_mb << 20
        if args.inflight_parts:
            over["s3"]["max_inflight_parts"] = args.inflight_parts
        if args.threshold_mb:
            over["s3"]["multipart_threshold"] = args.threshold_mb << 20
        over["download"]["stream_http"] = args.staging == "stream"
    cfg = load_config(overrides=over, env={})
    worker = Worker(cfg, broker=MemoryBroker())
    await worker.start(health=False)
    host, port = endpoint.split(":")

    scheme = "https" if args.tls != "off" else "http"

    def url(name, sz, seed):
        return f"{scheme}://{host}:{port}/media/{name}?size={sz}&seed={seed}"
    return worker, url


def _tag(args, mode: str) -> str:
    """Job-id tag of a measurement: each one stages fresh ids (no done-marker skips)."""
    return f"{mode}-m{getattr(args, 'measure_seq', 0)}"


def _warmup_jobs(args) -> int:
    """Untimed jobs each worker process stages before "go"."""
    w = getattr(args, "warmup_jobs", None)
    return args.warmup * args.jobs_per_step if w is None else w


async def _warmup(args, worker, url, wid: int, mode: str) -> None:
    _, wres = await run_phase(worker, url, wid, 0, _warmup_jobs(args),
                              int(args.size_mb * 1e6), _tag(args, mode))
    bad = [r for r in wres if r.outcome != "staged"]
    if bad:
        raise RuntimeError(f"warmup job failed: {bad[0]}")


def _cpu() -> tuple:
    """(user+system, system) CPU seconds of this whole process: every thread, the native
    transport's included."""
    t = os.times()
    return t.user + t.system, t.system


async def _timed(args, worker, url, wid: int, mode: str, count: int) -> dict:
    """The timed jobs of one worker process; ``elapsed`` is this process' own view and
    ``cpu_s`` / ``sys_s`` the CPU it spent inside that window only (no interpreter start,
    imports or warmup jobs)."""
    rc0 = _relay_counters()
    cpu0, sys0 = _cpu()
    t0 = time.perf_counter()
    loop_cpu0 = time.thread_time()
    dt, res = await run_phase(worker, url, wid, _warmup_jobs(args), count,
                              int(args.size_mb * 1e6), _tag(args, mode))
    loop_cpu = time.thread_time() - loop_cpu0
    t1 = time.perf_counter()
    cpu1, sys1 = _cpu()
    rc1 = _relay_counters()
    bad = [r for r in res if r.outcome != "staged"]
    pipes = _pipe_stats()
    # event-loop thread CPU / wall: ~1.0 means the Python side (one thread) is the limit
    return {"elapsed": t1 - t0, "latencies": [r.seconds for r in res],
            "bytes": sum(r.bytes for r in res), "failed": len(bad),
            "err": bad[0].error if bad else "", "loop_busy": loop_cpu / max(1e-9, t1 - t0),
            "cpu_s": cpu1 - cpu0, "sys_s": sys1 - sys0,
            "relay": {k: rc1[k] - rc0.get(k, 0) for k in rc1},
            "pipes_created": pipes.get("created", 0), "pipes_short": pipes.get("short", 0)}


def _relay_counters() -> dict:
    """The native transport's per-phase relay counters (``relay_counters``) of this process."""
    try:
        from downloader_amd.ops import native
        return dict(native().relay_counters())
    except Exception:
        return {}


def _sum_dicts(ds) -> dict:
    out: dict = {}
    for d in ds:
        for k, v in d.items():
            out[k] = out.get(k, 0) + v
    return out


def relay_breakdown(rc: dict, worker_cpu_s: float, gb: float) -> dict:
    """Where the workers' CPU per GB went, from the native relay counters: the relaying
    threads' own CPU (splice / peek-copy + CRC / copy modes), its CRC share, syscalls per MiB
    and bytes per copy call; ``other`` = the rest of the worker processes (event loop, HTTP
    heads, SigV4, job bookkeeping)."""
    gb = max(1e-9, gb)
    relay_ns = sum(rc.get(f"{m}_cpu_ns", 0) for m in ("splice", "dup", "copy"))
    moved = sum(rc.get(f"{m}_bytes", 0) for m in ("splice", "dup", "copy"))
    mib = max(1e-9, moved / (1 << 20))
    return {"relay_threads_cpu_s_per_GB": round(relay_ns / 1e9 / gb, 4),
            "crc_cpu_s_per_GB": round(rc.get("crc_ns", 0) / 1e9 / gb, 4),
            "other_worker_cpu_s_per_GB": round(max(0.0, worker_cpu_s - relay_ns / 1e9) / gb, 4),
            "splices_per_MiB": round((rc.get("splice_in_calls", 0)
                                      + rc.get("splice_out_calls", 0)) / mib, 2),
            "copy_KiB_per_call": round(rc.get("dup_copied_bytes", 0) / 1024
                                       / max(1, rc.get("dup_calls", 0)), 1),
            "relays": {m: rc.get(f"{m}_relays", 0) for m in ("splice", "dup", "copy")}}


def _pipe_stats() -> dict:
    """This process' splice pipes (``short``: created below the asked capacity because the
    user's pipe page budget, fs.pipe-user-pages-soft, was spent)."""
    try:
        from downloader_amd.ops import native
        return dict(native().pipe_stats())
    except Exception:
        return {}


async def rank_main(args, dist: Dist, endpoint: str, mode: str, stage_root: str, on_go=None,
                    on_end=None):
    worker, url = await _start_worker(args, endpoint, mode, stage_root)
    await _warmup(args, worker, url, dist.rank, mode)
    dist.barrier()
    if on_go is not None:
        on_go()                     # sink counters at "go": warmup bytes are not timed bytes
    cuda_sync()
    t0 = time.perf_counter()
    out = await _timed(args, worker, url, dist.rank, mode, args.steps * args.jobs_per_step)
    cuda_sync()
    out["elapsed"] = time.perf_counter() - t0
    if on_end is not None:
        on_end()
    await worker.stop()
    return out


def _proc_main(conn, args, endpoint: str, mode: str, stage_root: str, wid: int, cpus: list,
               count: int, pool_workers: int = 0) -> None:
    """One worker process of a rank (``--procs-per-rank``): warm up, report ready, wait for
    the rank's go, run its share of the timed jobs, report (its CPU counted from "go" to its
    last timed job only)."""
    if cpus:
        os.sched_setaffinity(0, cpus)
    os.environ.setdefault("LOG_LEVEL", "error")
    if pool_workers:     # this process' share of the node's memory (utils/membudget)
        os.environ["STAGER_POOL_WORKERS"] = str(pool_workers)

    async def go():
        worker, url = await _start_worker(args, endpoint, mode, stage_root)
        await _warmup(args, worker, url, wid, mode)
        conn.send(("ready", None))
        if conn.recv() != "go":
            await worker.stop()
            return
        out = await _timed(args, worker, url, wid, mode, count)
        conn.send(("done", out))
        await worker.stop()
    try:
        asyncio.run(go())
    except BaseException as e:   # the rank turns this into a failed run
        conn.send(("error", repr(e)))
        raise


def rank_procs(args, dist: Dist, endpoint: str, mode: str, stage_root: str, nproc: int,
               cpus: list, on_go=None, on_end=None) -> dict:
    """Run a rank as ``nproc`` worker processes (like ``downloader_amd supervisor -n`` does for
    a GPU slot): one asyncio worker saturates its event loop + GIL long before the rank's CPU
    share (two single-process ranks on one 16-CPU box: 82 GB/s vs 55 GB/s for one). Each
    process gets a contiguous sub-slice of the rank's CPUs and an equal share of the jobs; the
    rank's clock brackets "go" to the last "done"."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")            # fresh interpreters: no fork after gloo threads
    total = args.steps * args.jobs_per_step
    shares = [total // nproc + (1 if i < total % nproc else 0) for i in range(nproc)]
    per = len(cpus) // nproc if cpus else 0
    # memory: every worker process of the node takes limit / (slots x processes per slot)
    from downloader_amd.utils.cpus import gpu_slots
    pool = max(gpu_slots(), int(os.environ.get("LOCAL_WORLD_SIZE", dist.world))) * nproc
    procs, conns = [], []
    for i in range(nproc):
        a, b = ctx.Pipe()
        sub = cpus[i * per:(i + 1) * per] if per >= 1 else []
        p = ctx.Process(target=_proc_main, args=(b, args, endpoint, mode, stage_root,
                                                 dist.rank * 64 + i, sub, shares[i], pool),
                        daemon=True)
        p.start()
        procs.append(p)
        conns.append(a)

    def recv(c):
        kind, val = c.recv()
        if kind == "error":
            raise RuntimeError(f"bench worker process failed: {val}")
        return val
    try:
        for c in conns:
            recv(c)                           # all warmed up
        dist.barrier()
        if on_go is not None:
            on_go()
        cuda_sync()
        cpu0, sys0 = _cpu()                   # the rank's own process (it mostly waits)
        t0 = time.perf_counter()
        for c in conns:
            c.send("go")
        outs = [recv(c) for c in conns]
        cuda_sync()
        elapsed = time.perf_counter() - t0
        cpu1, sys1 = _cpu()
        if on_end is not None:
            on_end()
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return {"elapsed": elapsed, "latencies": [x for o in outs for x in o["latencies"]],
            "bytes": sum(o["bytes"] for o in outs), "failed": sum(o["failed"] for o in outs),
            "err": next((o["err"] for o in outs if o["err"]), ""),
            "loop_busy": max(o["loop_busy"] for o in outs),
            "pipes_created": sum(o["pipes_created"] for o in outs),
            "pipes_short": sum(o["pipes_short"] for o in outs),
            "cpu_s": cpu1 - cpu0 + sum(o["cpu_s"] for o in outs),
            "sys_s": sys1 - sys0 + sum(o["sys_s"] for o in outs),
            "relay": _sum_dicts(o["relay"] for o in outs)}


SINK_KEYS = ("bytes_received", "verify_objects", "verify_bytes", "verify_mismatches",
             "verify_unknown", "multipart_objects", "multipart_parts", "objects", "bad_digests",
             "checksummed_puts", "crc_checked_puts", "crc_unchecked_puts", "media_puts",
             "media_puts_crc")


def measure(args, dist: Dist, endpoint: str, mode: str, blob=None, nproc: int = 1,
            cpus: Optional[list] = None):
    args.measure_seq = getattr(args, "measure_seq", 0) + 1
    stage_root = args.stage_dir or tempfile.mkdtemp(prefix=f"stager-bench-r{dist.rank}-")
    at_go: dict = {}
    peer_cpu = [0.0, 0.0]

    # Timed-window CPU only: the peer's CPU from "go" to the rank's last timed job, the
    # workers' from "go" to each one's last timed job (_timed) - never start-up or warmup.
    def on_go() -> None:
        if blob is not None:
            at_go.update(blob.stats())
            peer_cpu[0] = blob.cpu_seconds()

    def on_end() -> None:
        if blob is not None:
            peer_cpu[1] = blob.cpu_seconds()
    try:
        if nproc > 1:
            out = rank_procs(args, dist, endpoint, mode, stage_root, nproc, cpus or [], on_go,
                             on_end)
        else:
            out = asyncio.run(rank_main(args, dist, endpoint, mode, stage_root, on_go, on_end))
    finally:
        if not args.stage_dir:
            shutil.rmtree(stage_root, ignore_errors=True)
    out["worker_cpu_s"] = out.pop("cpu_s")
    out["worker_sys_s"] = out.pop("sys_s")
    # with --peers shared only rank 0 has a peer: its CPU is the whole job's
    out["peer_cpu_s"] = peer_cpu[1] - peer_cpu[0]
    out["cpus"] = len(cpus) if cpus else len(os.sched_getaffinity(0))
    dist.barrier()
    # The S3 peer's own counters, between "go" and the end of the timed jobs (every rank is
    # past the barrier): bytes it received, objects it matched against the origin generator.
    end = blob.stats() if blob is not None else {}
    out["sink"] = {k: int(end.get(k, 0)) - int(at_go.get(k, 0)) for k in SINK_KEYS}
    out["sink"]["mismatches_total"] = int(end.get("verify_mismatches", 0))
    out["sink"]["unknown_total"] = int(end.get("verify_unknown", 0))
    out["sink"]["bad_digests_total"] = int(end.get("bad_digests", 0))
    allr = dist.gather(out)
    elapsed = max(r["elapsed"] for r in allr)
    total_bytes = sum(r["bytes"] for r in allr)
    sink = {k: sum(r["sink"][k] for r in allr) for k in allr[0]["sink"]}
    lats = [x for r in allr for x in r["latencies"]]
    failed = sum(r["failed"] for r in allr)
    jobs = args.steps * args.jobs_per_step * dist.world
    if failed:
        raise RuntimeError(f"{failed} timed jobs failed: {[r['err'] for r in allr if r['err']][:1]}")
    if sink["bad_digests_total"]:
        raise RuntimeError(f"S3 peer refused {sink['bad_digests_total']} bodies whose payload "
                           f"checksum did not match their bytes")
    if integrity(args, args.checksum, mode) == "crc32c" and blob is not None \
            and sink["media_puts_crc"] < sink["media_puts"]:
        raise RuntimeError(f"{sink['media_puts'] - sink['media_puts_crc']} of "
                           f"{sink['media_puts']} timed media PUTs / parts carried no CRC32C")
    if sink["bytes_received"] < total_bytes:
        raise RuntimeError(f"S3 peer received {sink['bytes_received']} bytes in the timed region "
                           f"< {total_bytes} claimed staged")
    if args.sink in ("sample", "verify"):
        if sink["mismatches_total"] or sink["unknown_total"]:
            raise RuntimeError(f"S3 peer: {sink['mismatches_total']} staged objects differ from "
                               f"the origin's bytes, {sink['unknown_total']} unmatched")
        if sink["verify_objects"] < jobs:
            raise RuntimeError(f"S3 peer checked {sink['verify_objects']} objects in the timed "
                               f"region < {jobs} timed jobs")
    gb_all = max(1e-9, sink["bytes_received"] / 1e9)
    mp = sink["multipart_objects"]
    worker_cpu = sum(r["worker_cpu_s"] for r in allr)
    peer_cpu = sum(r["peer_cpu_s"] for r in allr)
    # what the ranks' CPU slices could have delivered in their timed windows: the measured
    # CPU must fit inside it (a CPU-per-GB figure above it is an accounting error)
    capacity = sum(r["elapsed"] * r["cpus"] for r in allr)
    relay = _sum_dicts(r["relay"] for r in allr)
    return {"mbps": total_bytes / elapsed / 1e6, "elapsed": elapsed,
            "p50": statistics.median(lats) if lats else 0.0,
            "p90": sorted(lats)[int(0.9 * (len(lats) - 1))] if lats else 0.0,
            "bytes": total_bytes, "sink": sink,
            "parts_per_object": round(sink["multipart_parts"] / mp, 3) if mp else 1.0,
            "worker_cpu_s_per_GB": worker_cpu / gb_all,
            "worker_sys_share": sum(r["worker_sys_s"] for r in allr) / max(1e-9, worker_cpu),
            "peer_cpu_s_per_GB": peer_cpu / gb_all,
            "timed_cpu_s": worker_cpu + peer_cpu, "cpu_capacity_s": capacity,
            "breakdown": relay_breakdown(relay, worker_cpu, gb_all),
            "loop_busy": max(r["loop_busy"] for r in allr),
            "pipes_created": sum(r["pipes_created"] for r in allr),
            "pipes_short": sum(r["pipes_short"] for r in allr)}


def torrent_measure(args, dist: Dist) -> dict:
    """After the config-2 lines: the streamed-torrent path with its pieces hashed on this
    rank's GPU (PartHasher, ``stream_verify_backend: auto``) vs on the host (``cpu``),
    alternating, same call (``bench/torrent_ab.py``). Ranks start together; totals are summed
    over ranks (they run at once), device counters too."""
    from downloader_amd.bench.torrent_ab import torrent_ab
    dist.barrier()
    # An extra of the line: a failure (or a run past --torrent-timeout) is reported in it,
    # never allowed to cost the headline above; every rank still reaches the gather.
    try:
        r = asyncio.run(asyncio.wait_for(
            torrent_ab(total_bytes=int(args.torrent_gb * 1e9), pairs=args.torrent_pairs,
                       tag=f"ab-r{dist.rank}"), args.torrent_timeout))
    except Exception as e:   # (asyncio.TimeoutError included)
        r = {"torrent_error": f"{type(e).__name__}: {e}"[:300]}
    allr = dist.gather(r)
    failed = [x for x in allr if "torrent_error" in x]
    if failed:
        return {"torrent_error": failed[0]["torrent_error"], "torrent_ranks_failed": len(failed)}
    out = dict(allr[0])
    for k in ("torrent_gpu_MBps", "torrent_host_MBps", "gpu_parts", "gpu_host_fallbacks",
              "gpu_refused", "gpu_launches"):
        if k in out:
            out[k] = round(sum(x[k] for x in allr), 1) if "MBps" in k else sum(x[k] for x in allr)
    if len(allr) > 1:
        out["torrent_ranks"] = len(allr)
    return out


async def _config1(mode: str, jobs: int = 21, object_mb: int = 10) -> dict:
    """BASELINE config 1 in miniature: a single 10 MB HTTP job at a time through one worker
    (``bench/configs.config1``; the first job only warms the connections)."""
    from downloader_amd.bench import configs
    from downloader_amd.bench.infra import Blobd
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api
    from downloader_amd.service.worker import Worker
    stage = tempfile.mkdtemp(prefix="bench-cfg1-")
    try:
        with Blobd(sink="discard") as b:
            w = Worker(configs._cfg(mode, b.endpoint, stage, None, concurrency=1,
                                    download={"gpu_prewarm": False}), broker=MemoryBroker())
            await w.start(health=False)
            lat = []
            for i in range(jobs):
                m = api.make_download(f"cfg1-{mode}-{i}", "http",
                                      b.media_url(f"cfg1-{i}.mkv", object_mb * 10 ** 6, i))
                _, r = await configs._run_jobs(w, [m])
                if r[0].outcome != "staged":
                    raise RuntimeError(f"config 1 job failed: {r[0].error}")
                lat.append(r[0].seconds)
            await w.stop()
    finally:
        shutil.rmtree(stage, ignore_errors=True)
    lat = lat[1:] or lat
    return {"p50_s": round(statistics.median(lat), 4),
            "MBps_sequential": round(object_mb * 10 ** 6 / statistics.mean(lat) / 1e6, 1)}


def config1_measure(args, dist: Dist) -> dict:
    """Same call: config 1 (single 10 MB job, one worker) tuned and in reference mode, on
    rank 0's CPUs - the p50 half of BASELINE's metric on its own config."""
    out: dict = {}
    if dist.rank == 0:
        try:
            t = asyncio.run(_config1("tuned"))
            r = asyncio.run(_config1("reference"))
            out = {"config1_p50_s": t["p50_s"], "config1_MBps_sequential": t["MBps_sequential"],
                   "config1_reference_p50_s": r["p50_s"],
                   "config1_reference_MBps_sequential": r["MBps_sequential"]}
        except Exception as e:      # an extra of the line: never costs the headline
            out = {"config1_error": f"{type(e).__name__}: {e}"[:300]}
    dist.barrier()
    return out


def pin_rank(dist: Dist, per_rank: int = 0) -> list:
    """Give each rank (worker threads + its blobd, which inherits the mask) a disjoint slice
    of the allowed CPUs: no cross-rank cache thrash, and sockets/threads stay on a few CCDs
    of one NUMA node instead of migrating over the whole mask (build box: 256 CPUs in the
    mask, 16-CPU quota; 35.8 - 37.6 GB/s pinned vs 23.5 - 28.7 GB/s unpinned,
    profiles/archive/bench_pinning_r1.jsonl).

    ``per_rank`` 0 = auto: the rank's GPU slot share, min(mask, quota) / visible GPUs
    (``utils.cpus.pin_slot``) - NOT divided by the number of ranks, so a rank owns the same
    CPUs at N=1 as at N=8 and the driver's 1/2/4/8 curve is a weak-scaling curve (one GPU
    slot's worth of host per worker) rather than "the whole node at N=1"; -1 = off; K = K
    contiguous CPUs per local rank. Returns the slice ([] = unpinned)."""
    if per_rank < 0 or os.environ.get("STAGER_BENCH_NO_PIN") == "1":
        return []
    from downloader_amd.utils import cpus
    local = int(os.environ.get("LOCAL_RANK", dist.rank))
    nlocal = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", dist.world)))
    if per_rank == 0:
        return cpus.pin_slot(local, max(nlocal, cpus.gpu_slots()))
    return cpus.pin_share(local, nlocal, per_rank)


def integrity(args, checksum: str, mode: str = "") -> str:
    """Payload integrity of the measured uploads: ``crc32c`` when every PUT / part carries an
    x-amz-checksum-crc32c (the sink checks each one's form and recomputes a salted subset),
    ``sha256`` for reference mode over plain http (minio-js signs every payload), ``none``
    when the relay is spliced unchecked (``s3.checksum: auto`` on a plain-http relay, or
    ``off``)."""
    if (mode or args.mode) == "reference":
        return "sha256" if args.tls == "off" else "crc32c"
    pol = checksum or "always"
    if pol == "off":
        return "none"
    if pol == "always":
        return "crc32c"
    return "crc32c" if (args.tls != "off" or args.staging == "disk") else "none"


def slot_budget() -> tuple:
    """(GPU slots of the node, CPUs one slot may use = min(mask, cgroup quota) / slots): the
    CPU share a rank is pinned to (``pin_rank``), whatever N is."""
    import math
    from downloader_amd.utils import cpus
    slots = cpus.gpu_slots()
    mask = len(os.sched_getaffinity(0))
    q = cpus.cgroup_cpu_quota()
    budget = mask if q == math.inf else min(mask, max(1, math.ceil(q)))
    return slots, budget // max(1, slots)


@contextlib.contextmanager
def _override(args, **kw):
    """Run one extra measurement with some arguments changed."""
    saved = {k: getattr(args, k, None) for k in kw}
    for k, v in kw.items():
        setattr(args, k, v)
    try:
        yield
    finally:
        for k, v in saved.items():
            setattr(args, k, v)


def _plan_pipes(args, dist: Dist, nproc: int, base_conc: int) -> None:
    """Splice pipes: every worker process on the node shares one uid's pipe page budget
    (64 MiB for the unprivileged user of the GPU boxes); each relay in flight holds one."""
    from downloader_amd.utils import limits
    if args.pipe_kb:
        args.pipe_kb_eff = args.pipe_kb
        args.concurrency = base_conc
    else:
        args.concurrency, pipe = limits.relay_plan(base_conc, 2, dist.world * nproc)
        args.pipe_kb_eff = pipe >> 10


def _cpu_fields(m: dict, prefix: str = "") -> dict:
    return {f"{prefix}worker_cpu_s_per_GB": round(m["worker_cpu_s_per_GB"], 4),
            f"{prefix}peer_cpu_s_per_GB": round(m["peer_cpu_s_per_GB"], 4),
            f"{prefix}cpu_utilisation": round(m["timed_cpu_s"] / max(1e-9, m["cpu_capacity_s"]), 3)}


def main() -> int:
    args = parse()
    slots, slot_cpus = slot_budget()      # before pin_rank narrows the mask
    dist = Dist(args.gpus)
    pinned = pin_rank(dist, args.cpus_per_rank)
    from downloader_amd.bench.infra import Blobd, self_signed_cert
    blob = None
    endpoint = None
    cert = None
    if args.tls != "off":
        cert = self_signed_cert(tempfile.mkdtemp(prefix=f"stager-bench-tls-r{dist.rank}-"))
        args.ca_file = cert[0]
    if args.peers == "per-rank" or dist.rank == 0:
        # Native origin + S3 sink. per-rank: every worker gets its own peer (the external world
        # is not the bottleneck being measured); shared: one peer on rank 0 for all workers.
        blob = Blobd(default_size=int(args.size_mb * 1e6), sink=args.sink, tls=cert,
                     crc_check=args.sink_crc_check, crc_salt=args.sink_crc_salt).start()
        endpoint = blob.endpoint
    if args.peers == "shared":
        endpoint, ca = dist.bcast((endpoint, cert[0] if cert else ""))
        if cert:
            args.ca_file = ca
    # every rank's CPU slice and S3/origin peer, reported by rank 0 (placement evidence for
    # the driver's 1/2/4/8 runs: disjoint slices, one peer per rank)
    topo = dist.gather({"cpus": pinned, "peer": endpoint if blob is not None else None})
    nproc = args.procs_per_rank
    if nproc <= 0:
        # auto: one worker process per 4 CPUs of the rank's slice, at most 8. With a CRC32C on
        # every part the 16-CPU slice is CPU-bound; 4 processes x 4 jobs keep it ~94 % busy
        # vs ~83 % for 2 x 4 (48.0 - 51.3 vs 46.1 - 47.0 GB/s on two boxes, p50 32 vs 17 ms;
        # profiles/r6/sweep, profiles/r6/sweep2)
        nproc = max(1, min(8, len(pinned or os.sched_getaffinity(0)) // 4))
    if args.mode == "reference" and args.procs_per_rank <= 0:
        nproc = 1    # the reference is one serial consumer per container (explicit N: N of them)
    from downloader_amd.utils import limits
    base_conc = args.concurrency
    _plan_pipes(args, dist, nproc, base_conc)
    head_conc, head_pipe_kb = args.concurrency, args.pipe_kb_eff
    tuned_mode = args.mode == "tuned"
    try:
        tuned = measure(args, dist, endpoint, args.mode, blob, nproc, pinned)
        unchecked = single = ref = tor = None
        cfg1: dict = {}
        curve = []
        if args.compare_unchecked and tuned_mode and integrity(args, args.checksum) == "crc32c":
            with _override(args, checksum="auto"):
                if integrity(args, "auto") == "none":
                    unchecked = measure(args, dist, endpoint, args.mode, blob, nproc, pinned)
        if args.compare_single_put and tuned_mode:
            with _override(args, single_put=True):
                single = measure(args, dist, endpoint, args.mode, blob, nproc, pinned)
        if args.compare_reference and tuned_mode and args.ref_procs > 0:
            rp = args.ref_procs
            jobs = max(rp, args.ref_jobs)
            with _override(args, steps=1, jobs_per_step=jobs, warmup_jobs=args.ref_warmup_jobs):
                _plan_pipes(args, dist, rp, 1)
                ref = measure(args, dist, endpoint, "reference", blob, rp, pinned)
        for k in [int(x) for x in args.workers_curve.split(",") if x.strip()] if tuned_mode else []:
            with _override(args, steps=args.curve_steps, warmup_jobs=args.curve_warmup_jobs):
                _plan_pipes(args, dist, k, base_conc)
                m = measure(args, dist, endpoint, args.mode, blob, k, pinned)
                curve.append({"procs": k, "MBps": round(m["mbps"], 1),
                              "p50_s": round(m["p50"], 4), "p90_s": round(m["p90"], 4),
                              "concurrency_per_worker": args.concurrency,
                              "cpu_utilisation": round(m["timed_cpu_s"]
                                                       / max(1e-9, m["cpu_capacity_s"]), 3)})
        args.concurrency, args.pipe_kb_eff = head_conc, head_pipe_kb
        cfg1 = config1_measure(args, dist) if args.config1 and tuned_mode else {}
        tor = torrent_measure(args, dist) if args.torrent_gb > 0 and tuned_mode else None
    finally:
        if blob is not None:
            blob.stop()
    if dist.rank == 0:
        n = dist.world
        ts = tuned["sink"]
        line = {
            "metric": METRIC,
            "value": round(tuned["mbps"], 2),
            "unit": "MB/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tuned["elapsed"] / max(1, args.steps) * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            # headline / the same call's reference-equivalent mode (the reference
            # publishes no number; this mode stands in for it on the same CPUs)
            "vs_baseline": round(tuned["mbps"] / ref["mbps"], 3) if ref else None,
            "dtype": "bytes",
            "data": "synthetic random-byte media blobs served by the native blobd origin",
            "p50_job_latency_s": round(tuned["p50"], 4),
            # what the headline's bytes were checked with on the way to S3: crc32c = every PUT /
            # part carried an x-amz-checksum-crc32c of its payload (the sink checked that each
            # is there and well-formed, and recomputed the crc_checked_parts subset)
            "integrity": integrity(args, args.checksum),
            "sink_crc_check": f"1/{args.sink_crc_check}",
            "crc_parts": ts["media_puts_crc"],
            "media_parts": ts["media_puts"],
            "crc_checked_parts": ts["crc_checked_puts"],
            "bad_digests": ts["bad_digests"],
            # S3 side, counted by the sink itself between "go" and the end of the timed jobs
            "timed_sink_bytes": ts["bytes_received"],
            "parts_per_object": tuned["parts_per_object"],
            "sink": args.sink,
            "sink_verified_objects": ts["verify_objects"],
            "sink_verified_bytes": ts["verify_bytes"],
            "sink_mismatches": ts["mismatches_total"],
            "worker_cpu_s_per_GB": round(tuned["worker_cpu_s_per_GB"], 4),
            "worker_kernel_share": round(tuned["worker_sys_share"], 3),   # system / (user+system)
            "event_loop_busy": round(tuned["loop_busy"], 3),
            "peer_cpu_s_per_GB": round(tuned["peer_cpu_s_per_GB"], 4),
            # worker + peer CPU-seconds of the timed window / what the ranks' CPU slices could
            # give in it (elapsed x CPUs): <= 1 for physically consistent CPU figures
            "cpu_utilisation": round(tuned["timed_cpu_s"] / max(1e-9, tuned["cpu_capacity_s"]), 3),
            "worker_breakdown": tuned["breakdown"],
            # splice pipes created below their asked capacity (pipe page budget spent)
            "pipes_short": {"workers": tuned["pipes_short"], "of": tuned["pipes_created"]},
            "pipe_kb": head_pipe_kb,
            "pipe_budget_bytes": limits.pipe_budget_bytes(),
            "gpu_slots": slots,
            "slot_budget_cpus": slot_cpus,
            "peers": args.peers,
            "cpus_per_rank": len(pinned) if pinned else len(os.sched_getaffinity(0)),
            "rank_cpus": [t["cpus"] for t in topo],
            "rank_peers": [t["peer"] for t in topo],
            "p90_job_latency_s": round(tuned["p90"], 4),
            "mode": args.mode,
            "checksum": args.checksum or "always",
            "staging": args.staging if args.mode == "tuned" else "disk",
            **({"tls": args.tls} if args.tls != "off" else {}),
            "concurrency_per_worker": head_conc if args.mode == "tuned" else 1,
            "procs_per_rank": nproc,
            "config": {
                "model": "BASELINE.json config 2: HTTP media blob -> S3 multipart staging",
                "global_batch": n * args.jobs_per_step,
                "jobs_per_step_per_worker": args.jobs_per_step,
                "seq_len": int(args.size_mb * 1e6),
                "parallelism": f"ranks{n}x{nproc}procs",
                "object_bytes": int(args.size_mb * 1e6),
                "jobs_timed": n * args.steps * args.jobs_per_step,
            },
        }
        if ref is not None:      # same call: reference-equivalent mode
            line["reference_mode_MBps"] = round(ref["mbps"], 2)
            line["reference_mode_p50_s"] = round(ref["p50"], 4)
            line["reference_mode_procs"] = args.ref_procs
            line["reference_mode_jobs"] = n * max(args.ref_procs, args.ref_jobs)
            line["reference_mode_integrity"] = integrity(args, args.checksum, "reference")
            line.update(_cpu_fields(ref, "reference_mode_"))
        if curve:                # same call: MB/s and p50 at 1/2/4/8 worker processes
            line["workers_curve"] = curve
        line.update(cfg1)        # same call: config 1's p50, tuned and reference mode
        if unchecked is not None:   # same call: the spliced relay with no payload checksum
            line["unchecked_MBps"] = round(unchecked["mbps"], 2)
            line["unchecked_p50_s"] = round(unchecked["p50"], 4)
            line["unchecked_integrity"] = "none"
            line.update(_cpu_fields(unchecked, "unchecked_"))
            line["unchecked_worker_breakdown"] = unchecked["breakdown"]
        if single is not None:   # same call, round-2 settings: 100 MB objects in one PUT
            line["single_put_MBps"] = round(single["mbps"], 2)
            line["single_put_p50_s"] = round(single["p50"], 4)
            line["single_put_parts_per_object"] = single["parts_per_object"]
        if tor is not None:      # same call: streamed torrent, GPU vs host piece hashing
            line.update(tor)
        print(json.dumps(line), flush=True)
    dist.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
