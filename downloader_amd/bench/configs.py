"""Runner for the BASELINE.json benchmark configs (config 2 is the headline ``bench.py``).

  1  single 10 MB HTTP URL -> S3, 1 worker: per-job latency (p50/p90 over sequential jobs)
  3  single-file 4 GB torrent fetched from a BEP-19 webseed, piece-hash verification on
  4  multi-file 20 GB torrent (50 files), full piece verification, one S3 object per file
  5  mixed steady-state queue: HTTP + torrent jobs published at a fixed rate to the AMQP
     broker, consumed by N worker processes, 5% of HTTP jobs fail once (retry path)

Every config runs the real worker (stages, S3 client, telemetry) against the native ``blobd``
peer (origin, webseed file server and S3 sink); ``--mode reference`` runs the reference-
equivalent structure (prefetch 1, sequential parts/files, single stream, disk staging).

  python -m downloader_amd.bench.configs --config 3 [--scale 0.25] [--mode tuned|reference]

``--scale`` shrinks configs 3/4/5 proportionally for quick runs; results report the actual
sizes. Output: one JSON line per config.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import shutil
import statistics
import sys
import tempfile
import time
from typing import Dict, List

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from downloader_amd.bench.infra import Blobd  # noqa: E402
from downloader_amd.broker.memory import MemoryBroker  # noqa: E402
from downloader_amd.models import api  # noqa: E402
from downloader_amd.service.worker import Worker  # noqa: E402
from downloader_amd.utils.config import load_config  # noqa: E402
from downloader_amd.stages.jobdir import get_reaper  # noqa: E402

MB = 1_000_000


def _pct(xs: List[float], q: float) -> float:
    if not xs:
        return 0.0
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


def _rss_mb() -> Dict[str, float]:
    """This (worker) process: current RSS (/proc/self/statm) and peak RSS (ru_maxrss)."""
    import resource
    try:
        with open("/proc/self/statm") as f:
            cur = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
    except OSError:
        cur = 0
    peak = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
    return {"rss_MB": round(cur / MB, 1), "rss_peak_MB": round(peak / MB, 1)}


def _self_cpu() -> float:
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


_CERT = None


def _tls_cert(a):
    """--tls: one throwaway certificate per bench process for blobd (origin, webseed, S3)."""
    global _CERT
    if not getattr(a, "tls", False):
        return None
    if _CERT is None:
        from .infra import self_signed_cert
        _CERT = self_signed_cert(tempfile.mkdtemp(prefix="cfg-tls-"))
    return _CERT


def _cfg(mode: str, endpoint: str, stage: str, tls=None, **over) -> object:
    o: Dict = {"mode": mode, "instance": {"download_path": stage}, "s3": {"endpoint": endpoint},
               "broker": {"backend": "memory"}, "health": {"enabled": False},
               "download": {"torrent_enable_dht": False, "progress_interval_s": 5.0}}
    if tls is not None:
        o["s3"]["secure"] = True
        o["tls"] = {"ca_file": tls[0]}
    for k, v in over.items():
        if isinstance(v, dict):
            o.setdefault(k, {}).update(v)
        else:
            o[k] = v
    return load_config(overrides=o, env={})


async def _run_jobs(w: Worker, msgs, timeout: float = 3600.0):
    done = asyncio.Event()
    res = []

    def cb(r):
        res.append(r)
        if len(res) >= len(msgs):
            done.set()
    w.on_result = cb
    t0 = time.perf_counter()
    for m in msgs:
        await w.submit(m)
    await asyncio.wait_for(done.wait(), timeout)
    return time.perf_counter() - t0, res


def _write_random(path: str, n: int, seed: int) -> None:
    import numpy as np
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        left = n
        while left:
            k = min(left, 256 << 20)
            f.write(rng.bytes(k))
            left -= k


# ---------------------------------------------------------------------------- config 1
async def config1(a) -> Dict:
    stage = tempfile.mkdtemp(prefix="cfg1-")
    cert = _tls_cert(a)
    with Blobd(sink="discard", tls=cert) as b:
        w = Worker(_cfg(a.mode, b.endpoint, stage, cert, concurrency=1), broker=MemoryBroker())
        await w.start(health=False)
        lat = []
        for i in range(a.jobs):
            m = api.make_download(f"c1-{a.mode}-{i}", "http",
                                  b.media_url(f"c1-{i}.mkv", a.object_mb * MB, i))
            _, r = await _run_jobs(w, [m])
            assert r[0].outcome == "staged", r[0]
            lat.append(r[0].seconds)
        await w.stop()
    shutil.rmtree(stage, ignore_errors=True)
    lat = lat[1:] or lat   # first job warms connections
    return {"config": 1, "mode": a.mode, "jobs": len(lat), "object_MB": a.object_mb,
            **({"tls": True} if cert else {}),
            "p50_latency_s": round(statistics.median(lat), 4),
            "p90_latency_s": round(_pct(lat, 0.9), 4),
            "MBps_sequential": round(a.object_mb / statistics.mean(lat), 1)}


# ---------------------------------------------------------------------------- configs 3/4
def _make_torrent_tree(root: str, name: str, sizes: List[int], url: str, plen: int) -> bytes:
    from downloader_amd.torrent.metainfo import make_torrent
    if len(sizes) == 1:
        p = os.path.join(root, name)
        _write_random(p, sizes[0], 7)
        return make_torrent(p, plen, url_list=[url + name])
    for i, n in enumerate(sizes):
        _write_random(os.path.join(root, name, f"Season 1/{name} E{i + 1:02d}.mkv"), n, 100 + i)
    return make_torrent(os.path.join(root, name), plen, url_list=[url])


async def config_torrent(a, cfg_no: int) -> Dict:
    if cfg_no == 3:
        sizes = [int(4e9 * a.scale)]
        name = "movie.mkv"
    else:
        total = int(20e9 * a.scale)
        sizes = [total // 50 + (i * 7919) % 1000 for i in range(50)]
        name = "Show"
    total = sum(sizes)
    src = tempfile.mkdtemp(prefix=f"cfg{cfg_no}-src-", dir=a.src_dir)
    stage = tempfile.mkdtemp(prefix=f"cfg{cfg_no}-stage-", dir=a.stage_dir or None)
    try:
        cert = _tls_cert(a)
        with Blobd(sink="discard", files_root=src, tls=cert) as b:
            t0 = time.perf_counter()
            raw = _make_torrent_tree(src, name, sizes, b.files_url(), a.piece_mb << 20)
            setup_s = time.perf_counter() - t0
            with open(os.path.join(src, "job.torrent"), "wb") as f:
                f.write(raw)
            dl = {"verify_backend": a.verify_backend, "torrent_stream": a.torrent_stream}
            if a.stream_parallel:
                dl["torrent_stream_parallel"] = a.stream_parallel
            if a.webseed_streams:
                dl["webseed_streams"] = a.webseed_streams
            if a.webseed_chunk_mb:
                dl["webseed_chunk"] = a.webseed_chunk_mb << 20
            if a.webseed_verify_depth:
                dl["webseed_verify_depth"] = a.webseed_verify_depth
            if getattr(a, "webseed_verify_depth_gpu", 0):
                dl["webseed_verify_depth_gpu"] = a.webseed_verify_depth_gpu
            if getattr(a, "no_gpu_prewarm", False):
                dl["gpu_prewarm"] = False
            if getattr(a, "stream_verify", ""):
                dl["stream_verify_backend"] = a.stream_verify
            if getattr(a, "stream_gpu_pending", 0):
                dl["stream_gpu_pending"] = a.stream_gpu_pending
            if getattr(a, "stream_gpu_tail", None) is not None:
                dl["stream_gpu_tail"] = a.stream_gpu_tail
            if getattr(a, "relay_trim_s", None) is not None:
                dl["relay_pool_idle_trim_s"] = a.relay_trim_s
            if getattr(a, "relay_memory_mb", 0):
                dl["relay_memory_mb"] = a.relay_memory_mb
            if getattr(a, "stream_gpu_slots", 0):
                dl["stream_gpu_slots"] = a.stream_gpu_slots
            if getattr(a, "gpu_slot_mb", 0):
                dl["stream_gpu_slot_mb"] = a.gpu_slot_mb
            if getattr(a, "gpu_copy_streams", 0):
                dl["stream_gpu_copy_streams"] = a.gpu_copy_streams
            if getattr(a, "gpu_compute_streams", 0):
                dl["stream_gpu_compute_streams"] = a.gpu_compute_streams
            part_mb = getattr(a, "part_mb", 0)
            s3o = {"part_size": part_mb << 20} if part_mb else {}
            if getattr(a, "checksum", ""):
                s3o["checksum"] = a.checksum
            kj = max(1, int(getattr(a, "torrent_jobs", 1) or 1))
            w = Worker(_cfg(a.mode, b.endpoint, stage, cert, concurrency=kj, download=dl,
                            s3=s3o), broker=MemoryBroker())
            await w.start(health=False)
            # --reps: the same torrent staged again under a fresh media id (no done marker,
            # so every rep does the full job); one job is a sub-second sample on this box.
            reps = []
            try:
                from downloader_amd.ops import native
                native().relay_pool_reset_peak()
            except Exception:
                pass
            rss0 = _rss_mb()["rss_MB"]
            threads0 = _thread_cpu(0)
            for k in range(max(1, getattr(a, "reps", 1))):
                suffix = f"-r{k}" if k else ""
                # --torrent-jobs K: K copies of the job at once (distinct media ids)
                ms = [api.make_download(f"c{cfg_no}-{a.mode}{suffix}" + (f"-j{i}" if i else ""),
                                        "http", b.files_url("job.torrent"),
                                        "TV" if cfg_no == 4 else "MOVIE") for i in range(kj)]
                cpu0, peer0 = _self_cpu(), b.cpu_seconds()
                dt_k, r_k = await _run_jobs(w, ms)
                cpu_k, peer_k = _self_cpu() - cpu0, b.cpu_seconds() - peer0
                # job_s ends at the convert publish; the background unlink of the staged
                # files (instance.background_cleanup) is timed separately here.
                tc = time.perf_counter()
                await asyncio.get_running_loop().run_in_executor(
                    None, get_reaper(w.services).drain, 600.0)
                cleanup_k = time.perf_counter() - tc
                assert all(x.outcome == "staged" for x in r_k), r_k
                try:
                    from downloader_amd.ops import native
                    pool_k = native().relay_pool_stats()
                except Exception:
                    pool_k = {}
                reps.append((dt_k, r_k, cpu_k, peer_k, cleanup_k,
                             {"rss_MB": _rss_mb()["rss_MB"],
                              "pool_MiB": (pool_k.get("in_use_bytes", 0)
                                           + pool_k.get("idle_bytes", 0)) >> 20}))
            rss = _rss_mb()
            thread_cpu = _thread_cpu_delta(threads0, _thread_cpu(0))
            try:
                from downloader_amd.ops import native
                pool = native().relay_pool_stats()
            except Exception:
                pool = {}
            gpu_relay = {}
            if getattr(a, "stream_verify", "") in ("gpu", "auto"):
                from downloader_amd.ops import hashing
                gpu_relay = hashing.gpu_relay_stats()
            await w.stop()
            # the median rep is the one reported in full
            reps_sorted = sorted(reps, key=lambda x: x[0])
            dt, r, cpu_s, peer_cpu_s, cleanup_s, _ = reps_sorted[len(reps_sorted) // 2]
            st = b.stats()
    finally:
        shutil.rmtree(src, ignore_errors=True)
        shutil.rmtree(stage, ignore_errors=True)
    return {"config": cfg_no, "mode": a.mode, "bytes": total, "files": len(sizes),
            **({"tls": True} if cert else {}),
            "piece_len": a.piece_mb << 20, "job_s": round(dt, 3),
            "MBps": round(kj * total / dt / MB, 1), "setup_s": round(setup_s, 2),
            "s3_bytes_received": st["bytes_received"], "uploaded_bytes": r[0].bytes,
            "torrent": r[0].stats.get("torrent", {}), "stage_s": r[0].stats.get("stage_s", {}),
            "eager_upload_s": r[0].stats.get("eager_upload_s"),
            "cleanup_after_job_s": round(cleanup_s, 3),
            "worker_cpu_s": round(cpu_s, 2), "peer_cpu_s": round(peer_cpu_s, 2),
            "worker_rss_before_MB": rss0, "worker_rss_after_MB": rss["rss_MB"],
            "worker_rss_peak_MB": rss["rss_peak_MB"],
            "relay_pool_after": pool,
            "part_budget_MiB": r[0].stats.get("torrent", {}).get("budget", {}).get("capacity", 0)
            >> 20,
            "part_pool_peak_MiB": pool.get("peak_bytes", 0) >> 20,
            **({"thread_cpu": thread_cpu} if os.environ.get("STAGER_THREAD_CPU") else {}),
            **({"stream_verify": a.stream_verify, "gpu_relay": gpu_relay}
               if getattr(a, "stream_verify", "") else {}),
            **({"torrent_jobs": kj} if kj > 1 else {}),
            "reps": len(reps), "MBps_reps": [round(kj * total / x[0] / MB, 1) for x in reps],
            # per rep (the first is the worker's cold job): job seconds, summed relay seconds
            # of all parts, worker and peer CPU seconds
            "reps_detail": [{"job_s": round(x[0], 3),
                             "relay_s": x[1][0].stats.get("torrent", {}).get("webseed_fetch_s"),
                             "worker_cpu_s": round(x[2], 2), "peer_cpu_s": round(x[3], 2),
                             **x[5]}
                            for x in reps]}


# ---------------------------------------------------------------------------- config 5
async def config5(a) -> Dict:
    from downloader_amd.broker.amqp import AmqpBroker
    from downloader_amd.broker.server import BrokerServer
    from downloader_amd.parallel.supervisor import Supervisor, worker_argv
    from downloader_amd.torrent.metainfo import make_torrent
    n_jobs = max(20, int(1000 * a.scale))
    src = tempfile.mkdtemp(prefix="cfg5-src-", dir=a.src_dir)
    stage = tempfile.mkdtemp(prefix="cfg5-stage-", dir=a.stage_dir or None)
    srv = await BrokerServer(heartbeat=0).start()
    with Blobd(sink="discard", files_root=src) as b:
        # 4 distinct torrents re-used by the torrent jobs (50 MB each, webseed)
        torrents = []
        for t in range(4):
            p = os.path.join(src, f"t{t}.mkv")
            _write_random(p, 50 * MB, 500 + t)
            raw = make_torrent(p, 1 << 20, url_list=[b.files_url(f"t{t}.mkv")])
            with open(os.path.join(src, f"t{t}.torrent"), "wb") as f:
                f.write(raw)
            torrents.append(b.files_url(f"t{t}.torrent"))
        env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error",
                   STAGER_BROKER__URL=srv.url, STAGER_BROKER__BACKEND="amqp",
                   STAGER_S3__ENDPOINT=b.endpoint, STAGER_INSTANCE__DOWNLOAD_PATH=stage,
                   STAGER_HEALTH__ENABLED="false", STAGER_DOWNLOAD__TORRENT_ENABLE_DHT="false",
                   STAGER_BROKER__RETRY_BACKOFF_S=str(a.retry_backoff_s),
                   STAGER_BROKER__RETRY_DELAY=a.retry_delay, STAGER_MODE=a.mode,
                   STAGER_CONCURRENCY=str(a.concurrency))
        sup = Supervisor(a.workers, worker_argv(), env=env)
        client = AmqpBroker(srv.url)
        await client.connect()
        for q in ("v1.download", "v1.convert"):
            await client.declare(q)
        sup.start()
        rng = random.Random(5)
        published: Dict[str, float] = {}
        lat_of: Dict[str, float] = {}
        kinds: Dict[str, str] = {}
        done = asyncio.Event()

        async def on_convert(d):
            mid = api.decode(api.Convert, d.body).media.id
            if mid in published and mid not in lat_of:      # first convert of a job counts
                lat_of[mid] = time.perf_counter() - published[mid]
            await d.ack()
            if len(lat_of) >= n_jobs:
                done.set()
        await client.consume("v1.convert", on_convert, prefetch=64)
        t0 = time.perf_counter()
        fails = 0
        for i in range(n_jobs):
            target = t0 + i / a.qps
            now = time.perf_counter()
            if target > now:
                await asyncio.sleep(target - now)
            jid = f"c5-{a.mode}-{i}"
            if rng.random() < 0.2:
                m = api.make_download(jid, "http", torrents[i % 4])
                kinds[jid] = "torrent"
            else:
                url = b.media_url(f"c5-{i}.mkv", 10 * MB, i)
                failing = rng.random() < 0.05
                if failing:
                    url += "&fail=1"
                    fails += 1
                m = api.make_download(jid, "http", url)
                kinds[jid] = "http-failing" if failing else "http"
            published[jid] = time.perf_counter()
            await client.publish("v1.download", api.encode(m))
        publish_s = time.perf_counter() - t0
        try:
            await asyncio.wait_for(done.wait(), 1800)
        finally:
            wall = time.perf_counter() - t0
            codes = await asyncio.get_running_loop().run_in_executor(None, sup.stop)
            await client.close()
            await srv.stop()
            shutil.rmtree(src, ignore_errors=True)
            shutil.rmtree(stage, ignore_errors=True)
    n_torrent = sum(1 for k in kinds.values() if k == "torrent")
    total_bytes = (n_jobs - n_torrent) * 10 * MB + n_torrent * 50 * MB
    lat = list(lat_of.values())
    healthy = [v for k, v in lat_of.items() if kinds.get(k) != "http-failing"]
    return {"config": 5, "mode": a.mode, "jobs": n_jobs, "workers": a.workers,
            "retry_backoff_s": a.retry_backoff_s, "retry_delay": a.retry_delay,
            # jobs that never failed: what a backoff that holds a consumer slot delays
            "healthy_p50_s": round(statistics.median(healthy), 4),
            "healthy_p99_s": round(_pct(healthy, 0.99), 4),
            "qps_offered": a.qps, "publish_s": round(publish_s, 2), "wall_s": round(wall, 2),
            "jobs_per_s": round(n_jobs / wall, 1), "MBps": round(total_bytes / wall / MB, 1),
            "p50_latency_s": round(statistics.median(lat), 4),
            "p99_latency_s": round(_pct(lat, 0.99), 4), "injected_failures": fails,
            "torrent_jobs": n_torrent, "worker_exit_codes": codes}


# ---------------------------------------------------------------------------- config 8
async def config_bucket(a) -> Dict:
    """bucket:// source (extra; the reference fetches every object sequentially with
    fGetObject, lib/download.js:218-226, then uploads the selected ones): a season of 10
    episodes plus 2 extras in a synthetic source bucket served by blobd."""
    ep = int(1e9 * a.scale)
    objs = {f"lib/Show/Season 1/Show S01E{i + 1:02d}.mkv": ep + i for i in range(10)}
    objs.update({f"lib/Show/Extras/extra{i}.mkv": ep for i in range(2)})
    objs["lib/Show/readme.txt"] = 1000
    stage = tempfile.mkdtemp(prefix="cfg8-stage-", dir=a.stage_dir or None)
    out: Dict = {"config": 8, "mode": a.mode, "objects": len(objs),
                 "selected_bytes": sum(n for k, n in objs.items() if "Season" in k),
                 "listed_bytes": sum(objs.values())}
    try:
        with Blobd(sink="discard", synth_bucket="src", synth_objects=objs) as b:
            # blobd is source and staging endpoint but cannot copy server-side: measure the
            # relay (a same-endpoint deployment would copy without moving any bytes)
            dl = {"bucket_secure": False, "bucket_server_copy": False}
            if a.mode == "tuned":
                dl["stream_bucket"] = a.torrent_stream != "off"
            w = Worker(_cfg(a.mode, b.endpoint, stage, concurrency=1, download=dl),
                       broker=MemoryBroker())
            await w.start(health=False)
            uri = f"bucket://{b.endpoint},src,minioadmin,minioadmin,lib"
            cpu0, peer0 = _self_cpu(), b.cpu_seconds()
            dt, r = await _run_jobs(w, [api.make_download(f"c8-{a.mode}", "bucket", uri, "TV")])
            cpu, peer = _self_cpu() - cpu0, b.cpu_seconds() - peer0
            assert r[0].outcome == "staged", r[0]
            await w.stop()
            out.update({"streamed": bool(r[0].stats.get("streamed")), "job_s": round(dt, 3),
                        "MBps_selected": round(out["selected_bytes"] / dt / MB, 1),
                        "downloaded_bytes": r[0].stats.get("downloaded_bytes"),
                        "uploaded_bytes": r[0].bytes, "worker_cpu_s": round(cpu, 2),
                        "peer_cpu_s": round(peer, 2), "stage_s": r[0].stats.get("stage_s")})
    finally:
        shutil.rmtree(stage, ignore_errors=True)
    return out


def _seed_proc(conn, raw: bytes, src: str, n: int, native_wire: bool = True) -> None:
    """Seeding clients in their own process (remote peers are not on our event loop)."""
    from downloader_amd.torrent.client import TorrentClient
    from downloader_amd.torrent.metainfo import parse_torrent

    async def go():
        meta = parse_torrent(raw)
        cs = []
        for _ in range(n):
            c = await TorrentClient(max_uploads=64, native_wire=native_wire).start()
            await c.add_torrent(meta, src)
            cs.append(c)
        conn.send([c.listen_port for c in cs])
        await asyncio.get_running_loop().run_in_executor(None, conn.recv)
        for c in cs:
            await c.close()
    asyncio.run(go())


async def config_swarm(a) -> Dict:
    """Extra (not in BASELINE.json): a peer-wire-only download from ``--seeders`` seeders
    over loopback (no webseed), measuring the BEP-3 block pipeline + SHA-1 verification of
    the downloading client. The seeders run in a separate process (``--seed-inproc``: on the
    same event loop, as in round 1)."""
    import multiprocessing as mp

    from downloader_amd.torrent.client import TorrentClient
    from downloader_amd.torrent.metainfo import make_torrent, parse_torrent
    total = int(2e9 * a.scale)
    wire = getattr(a, "wire", "native") == "native"
    src = tempfile.mkdtemp(prefix="swarm-src-", dir=a.src_dir)
    dst = tempfile.mkdtemp(prefix="swarm-dst-", dir=a.stage_dir or None)
    procs: List = []
    seeders = []
    try:
        p = os.path.join(src, "swarm.mkv")
        _write_random(p, total, 99)
        raw = make_torrent(p, a.piece_mb << 20)
        meta = parse_torrent(raw)
        if getattr(a, "seed_inproc", False):
            for _ in range(a.seeders):
                c = await TorrentClient(max_uploads=64, native_wire=wire).start()
                await c.add_torrent(meta, src)
                seeders.append(c)
            ports = [c.listen_port for c in seeders]
        else:
            # one process per seeder (--seeder-procs 1: all in one, as in the first round-2
            # runs, where that process's event loop capped the leecher at ~1.4 GB/s)
            ctx = mp.get_context("spawn")
            nproc = max(1, min(a.seeders, getattr(a, "seeder_procs", 0) or a.seeders))
            share = [a.seeders // nproc + (1 if i < a.seeders % nproc else 0)
                     for i in range(nproc)]
            for n in share:
                conn, child = ctx.Pipe()
                proc = ctx.Process(target=_seed_proc, args=(child, raw, src, n, wire),
                                   daemon=True)
                proc.start()
                procs.append((proc, conn))
            ports = []
            for _, conn in procs:
                ports += await asyncio.get_running_loop().run_in_executor(None, conn.recv)
        verify = getattr(a, "swarm_verify", "auto")
        if getattr(a, "swarm_job", False):
            return await _swarm_jobs(a, meta, ports, total, dst, verify, wire, seeders, procs)
        native_req = getattr(a, "wire_requests", "native") == "native"
        extra = {}
        if getattr(a, "swarm_gpu_inflight", 0):
            extra["wire_gpu_inflight"] = a.swarm_gpu_inflight
        if getattr(a, "swarm_pool_mb", 0):
            extra["wire_pool_mb"] = a.swarm_pool_mb
        if getattr(a, "swarm_gpu_tail_x", None) is not None:
            extra["swarm_gpu_tail_x"] = a.swarm_gpu_tail_x
        if getattr(a, "swarm_gpu_tail_max", None) is not None:
            extra["swarm_gpu_tail_max"] = a.swarm_gpu_tail_max
        if getattr(a, "swarm_gpu_tail_mb", None) is not None:
            mb = a.swarm_gpu_tail_mb
            extra["swarm_gpu_tail_bytes"] = mb << 20 if mb >= 0 else -1
        leech = await TorrentClient(max_peers=64, pipeline=a.pipeline, native_wire=wire,
                                    swarm_verify=verify, wire_requests=native_req,
                                    **extra).start()
        if wire and verify == "gpu":
            # a worker sets its GPU up at start (download.gpu_prewarm), not inside a job
            from downloader_amd.ops import hashing
            await asyncio.get_running_loop().run_in_executor(None, hashing.gpu_relay_hashing)
        # --reps K: the torrent downloaded K times by the same leecher (fresh directories, a
        # new session each); the first is the process' cold one (pools, page locking), the
        # last is reported in full
        runs = []
        for k in range(max(1, getattr(a, "reps", 1) or 1)):
            d = os.path.join(dst, f"r{k}")
            threads0 = _thread_cpu(0)
            cpu0 = _self_cpu()
            t0 = time.perf_counter()
            s = await leech.add_torrent(meta, d, peers=[("127.0.0.1", port) for port in ports])
            await asyncio.wait_for(s.wait(), 1800)
            dt = time.perf_counter() - t0
            cpu_s = _self_cpu() - cpu0
            # where the leecher's CPU went (before close: the wire's threads still exist)
            per_thread = _thread_cpu_delta(threads0, _thread_cpu(0))
            stats = s.wire.stats() if s.wire is not None else None
            runs.append((dt, cpu_s, per_thread, stats, s))
            await leech.remove(s)
            shutil.rmtree(d, ignore_errors=True)
        dt, cpu_s, per_thread, stats, s = runs[-1]
        out = {"config": "swarm", "bytes": total, "seeders": a.seeders, "pipeline": a.pipeline,
               "wire": "native" if s.wire is not None else "python",
               "wire_requests": ("native" if native_req else "python") if s.wire is not None
               else "python",
               "swarm_verify": s.stats.get("swarm_verify", "python"),
               **({"wire_stats": stats} if stats is not None else {}),
               "seeders_in_process": bool(seeders), "seeder_procs": len(procs),
               "piece_len": a.piece_mb << 20,
               "s": round(dt, 3), "MBps": round(total / dt / MB, 1),
               "leech_cpu_s": round(cpu_s, 2), "hash_fails": s.stats["hash_fails"],
               "leech_cpu_s_per_GB": round(cpu_s / (total / 1e9), 3),
               "leech_thread_cpu": per_thread,
               "reps": len(runs), "MBps_reps": [round(total / r[0] / MB, 1) for r in runs],
               "leech_cpu_s_per_GB_reps": [round(r[1] / (total / 1e9), 3) for r in runs],
               # GPU mode: bytes left to start when the rest went to the host (auto tail)
               "gpu_host_tail_bytes_reps": [r[4].stats.get("gpu_host_tail_bytes", 0)
                                            for r in runs],
               # piece buffers page-locked for the GPU hasher (process-wide, so far), per rep
               "pool_locks_reps": [(r[3] or {}).get("pool_locks", 0) for r in runs]}
        await leech.close()
        return out
    finally:
        for c in seeders:
            await c.close()
        for proc, conn in procs:
            try:
                conn.send("stop")
            except (OSError, ValueError):
                pass
        for proc, _ in procs:
            proc.join(timeout=30)
            if proc.is_alive():
                proc.kill()
        shutil.rmtree(src, ignore_errors=True)
        shutil.rmtree(dst, ignore_errors=True)


async def _swarm_jobs(a, meta, ports, total: int, dst: str, verify: str, wire: bool,
                      seeders, procs) -> Dict:
    """config 6 --swarm-job: the whole job the reference runs for a magnet (download.js:64 ->
    upload.js): a worker takes a `v1.download` whose source is a magnet naming the seeders
    (x.pe), fetches the metadata from them (BEP-9), downloads the swarm, stages the file to the
    S3 sink (uploads start per completed file region while the swarm runs, eager staging),
    writes the done marker and publishes `v1.convert`. MB/s = bytes / job seconds."""
    from downloader_amd.torrent.magnet import Magnet
    dl = {"swarm_verify_backend": verify, "torrent_native_wire": wire,
          "torrent_request_pipeline": a.pipeline}
    if getattr(a, "swarm_pool_mb", 0):
        dl["swarm_pool_mb"] = a.swarm_pool_mb
    runs = []
    with Blobd(sink="discard") as b:
        w = Worker(_cfg(a.mode, b.endpoint, dst, None, download=dl), broker=MemoryBroker())
        await w.start(health=False)
        try:
            uri = Magnet(meta.info_hash, meta.name, [],
                         peers=[("127.0.0.1", p) for p in ports]).to_uri()
            for k in range(max(1, getattr(a, "reps", 1) or 1)):
                m = api.make_download(f"swarm-job-{k}", "torrent", uri, "MOVIE")
                cpu0, peer0, rx0 = _self_cpu(), b.cpu_seconds(), b.stats()["bytes_received"]
                dt, r = await _run_jobs(w, [m])
                cpu_s, peer_s = _self_cpu() - cpu0, b.cpu_seconds() - peer0
                rx = b.stats()["bytes_received"] - rx0
                await asyncio.get_running_loop().run_in_executor(
                    None, get_reaper(w.services).drain, 600.0)
                assert r[0].outcome == "staged", r[0]
                runs.append((dt, cpu_s, peer_s, rx, r[0]))
        finally:
            await w.stop()
    dt, cpu_s, peer_s, rx, r = runs[-1]
    return {"config": "swarm-job", "bytes": total, "seeders": a.seeders, "pipeline": a.pipeline,
            "wire": "native" if wire else "python", "swarm_verify": verify,
            "seeder_procs": len(procs), "seeders_in_process": bool(seeders),
            "piece_len": a.piece_mb << 20, "job_s": round(dt, 3),
            "MBps": round(total / dt / MB, 1), "s3_bytes_received": rx,
            "worker_cpu_s": round(cpu_s, 2), "worker_cpu_s_per_GB": round(cpu_s / (total / 1e9), 3),
            "sink_cpu_s": round(peer_s, 2), "stage_s": r.stats.get("stage_s", {}),
            "eager_upload_s": r.stats.get("eager_upload_s"),
            "reps": len(runs), "MBps_reps": [round(total / x[0] / MB, 1) for x in runs],
            "worker_cpu_s_per_GB_reps": [round(x[1] / (total / 1e9), 3) for x in runs]}


# ---------------------------------------------------------------------------- config 9
def _thread_cpu(top: int = 14) -> List[Dict]:
    """This process' threads (the ``top`` busiest; 0 = all): OS name or Python thread name,
    user / system CPU seconds - where a config's worker CPU goes (STAGER_THREAD_CPU=1)."""
    import threading
    names = {t.native_id: t.name for t in threading.enumerate()}
    hz = os.sysconf("SC_CLK_TCK")
    rows = []
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
            with open(f"/proc/self/task/{tid}/comm") as f:
                comm = f.read().strip()
        except OSError:
            continue
        fields = st[st.rindex(")") + 2:].split()
        rows.append({"tid": int(tid), "name": names.get(int(tid), comm),
                     "user_s": int(fields[11]) / hz, "sys_s": int(fields[12]) / hz})
    rows.sort(key=lambda r: -(r["user_s"] + r["sys_s"]))
    return rows[:top] if top else rows


def _thread_cpu_delta(before: List[Dict], after: List[Dict], top: int = 14) -> List[Dict]:
    """CPU per thread between two ``_thread_cpu(0)`` snapshots, grouped by name (threads of
    one pool share a name), busiest first; threads that exited in between are missing."""
    b = {r["tid"]: r for r in before}
    groups: Dict[str, Dict] = {}
    for r in after:
        p = b.get(r["tid"], {"user_s": 0.0, "sys_s": 0.0})
        key = r["name"].rstrip("0123456789_-")
        g = groups.setdefault(key, {"name": key, "threads": 0, "user_s": 0.0, "sys_s": 0.0})
        g["threads"] += 1
        g["user_s"] = round(g["user_s"] + r["user_s"] - p["user_s"], 2)
        g["sys_s"] = round(g["sys_s"] + r["sys_s"] - p["sys_s"], 2)
    out = sorted(groups.values(), key=lambda g: -(g["user_s"] + g["sys_s"]))
    return [g for g in out if g["user_s"] + g["sys_s"] > 0][:top]


async def config_small(a) -> Dict:
    """Control-plane ceiling (extra): ``--jobs`` tiny HTTP jobs (``--small-kb``) submitted at
    once to ONE worker process with ``--concurrency`` jobs in flight. Every job still does the
    whole protocol - done-marker check, relayed PUT, done marker, convert publish, telemetry -
    so jobs/s and CPU-ms per job are the per-process cost of a job apart from its bytes."""
    stage = tempfile.mkdtemp(prefix="cfg9-")
    n = max(100, a.jobs)
    spans = os.path.join(stage, "spans.jsonl")
    with Blobd(sink="discard") as b:
        cfg = _cfg(a.mode, b.endpoint, stage, None, concurrency=a.concurrency)
        if getattr(a, "trace", False):    # spans of every job and stage to a JSONL file
            cfg.trace.enabled, cfg.trace.path = True, spans
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        warm = [api.make_download(f"c9-w{i}", "http", b.media_url(f"w{i}.mkv", 1000, i))
                for i in range(min(100, n))]
        await _run_jobs(w, warm)
        msgs = [api.make_download(f"c9-{a.mode}-{i}", "http",
                                  b.media_url(f"c9-{i}.mkv", a.small_kb * 1000, i))
                for i in range(n)]
        c0, p0 = _self_cpu(), b.cpu_seconds()
        dt, res = await _run_jobs(w, msgs)
        cpu, peer = _self_cpu() - c0, b.cpu_seconds() - p0
        await w.stop()
    n_spans = sum(1 for _ in open(spans)) if os.path.exists(spans) else 0
    shutil.rmtree(stage, ignore_errors=True)
    staged = sum(1 for r in res if r.outcome == "staged")
    lat = [r.seconds for r in res]
    return {"config": 9, "mode": a.mode, "jobs": n, "staged": staged,
            "object_kB": a.small_kb, "concurrency": a.concurrency,
            "jobs_per_s": round(n / dt, 1), "worker_cpu_ms_per_job": round(1000 * cpu / n, 3),
            "peer_cpu_ms_per_job": round(1000 * peer / n, 3),
            "p50_latency_s": round(statistics.median(lat), 4),
            "p99_latency_s": round(_pct(lat, 0.99), 4),
            "trace": bool(getattr(a, "trace", False)), "spans_written": n_spans}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, action="append", required=True,
                    help="1, 3, 4, 5 (BASELINE.json), 6 (peer-wire swarm, extra), 7 (chaos "
                         "soak: worker kills + broker connection drops under load, extra) or "
                         "8 (bucket:// season, extra; --torrent-stream off = disk path) or 9 "
                         "(control-plane ceiling: tiny jobs through one worker, extra)")
    ap.add_argument("--small-kb", type=int, default=1,
                    help="config 9: object size in kB (jobs = --jobs, in flight = --concurrency)")
    ap.add_argument("--trace", action="store_true",
                    help="config 9: tracing on (spans to a JSONL file by the exporter thread)")
    ap.add_argument("--chaos-interval", type=float, default=2.0,
                    help="config 7: seconds between chaos actions (kill / connection drop)")
    ap.add_argument("--no-chaos-kill", dest="chaos_kill", action="store_false",
                    help="config 7: no worker kills (connection drops and S3 faults only), so "
                         "long-lived workers show RSS / fd growth")
    ap.add_argument("--s3-fail-rate", type=float, default=0.02,
                    help="config 7: share of S3 object/part PUTs the peer answers 503 SlowDown")
    ap.add_argument("--chaos-multipart-mb", type=int, default=0,
                    help="config 7: multipart threshold in MB for the workers (0 = default); "
                         "16 stages the 50 MB torrents as multipart uploads")
    ap.add_argument("--chaos-timeout", type=float, default=900.0,
                    help="config 7: give up waiting for every job's convert after this long")
    ap.add_argument("--seeders", type=int, default=4, help="config 6: seeding clients")
    ap.add_argument("--swarm-verify", choices=["auto", "gpu", "cpu"], default="auto",
                    help="config 6: piece SHA-1 of the native wire on the gfx950 or the host")
    ap.add_argument("--wire", choices=["native", "python"], default="native",
                    help="config 6: peer connections on the native wire (csrc/peerwire.cpp) or "
                         "framed in Python (torrent/peer.py), leecher and seeders alike")
    ap.add_argument("--pipeline", type=int, default=64, help="config 6: requests in flight/peer")
    ap.add_argument("--swarm-gpu-inflight", type=int, default=0,
                    help="config 6, GPU mode: pieces on the device at once (0: the default)")
    ap.add_argument("--swarm-job", action="store_true",
                    help="config 6: the whole magnet job through a worker (metadata from the "
                         "seeders, swarm download, staging to the S3 sink), not the bare leech")
    ap.add_argument("--swarm-gpu-tail-mb", type=int, default=None,
                    help="config 6, GPU mode: the last MB hashed on the host (default: config)")
    ap.add_argument("--swarm-gpu-tail-max", type=float, default=None,
                    help="config 6, GPU mode: the auto tail's largest share of the torrent")
    ap.add_argument("--swarm-gpu-tail-x", type=float, default=None,
                    help="config 6, GPU mode: the auto tail's multiple of the device latency")
    ap.add_argument("--swarm-pool-mb", type=int, default=0,
                    help="config 6: idle piece buffers kept (0: the default)")
    ap.add_argument("--wire-requests", choices=["native", "python"], default="native",
                    help="config 6, native wire: whole pieces requested by the wire itself, or "
                         "every block requested and booked in Python")
    ap.add_argument("--seeder-procs", type=int, default=0,
                    help="config 6: processes the seeders run in (0: one per seeder)")
    ap.add_argument("--seed-inproc", action="store_true",
                    help="config 6: seeders on the measuring process's event loop (round 1)")
    ap.add_argument("--mode", choices=["tuned", "reference"], default="tuned")
    ap.add_argument("--tls", action="store_true",
                    help="configs 1/3/4: origin, webseed and S3 over https (blobd certificate)")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--jobs", type=int, default=21, help="config 1: sequential jobs")
    ap.add_argument("--object-mb", type=int, default=10,
                    help="config 1: object size (BASELINE: 10 MB)")
    ap.add_argument("--piece-mb", type=int, default=4)
    ap.add_argument("--torrent-jobs", type=int, default=1,
                    help="configs 3/4: K copies of the torrent job at once per rep (aggregate "
                         "MB/s; the worker's concurrency = K)")
    ap.add_argument("--reps", type=int, default=1,
                    help="configs 3/4: stage the torrent this many times, report the median")
    ap.add_argument("--verify-backend", choices=["cpu", "gpu", "auto"], default="auto")
    ap.add_argument("--webseed-streams", type=int, default=0)
    ap.add_argument("--webseed-chunk-mb", type=int, default=0)
    ap.add_argument("--webseed-verify-depth", type=int, default=0)
    ap.add_argument("--webseed-verify-depth-gpu", type=int, default=0,
                    help="fetched runs queued per stream when the GPU batcher verifies them")
    ap.add_argument("--torrent-stream", choices=["auto", "always", "off"], default="auto",
                    help="download.torrent_stream: webseed->S3 relay (auto) or disk staging (off)")
    ap.add_argument("--stream-verify", choices=["cpu", "gpu", "auto"], default="",
                    help="download.stream_verify_backend: relayed parts' pieces hashed by the "
                         "host multi-buffer SHA-1, the gfx950 PartHasher, or auto (the device "
                         "when stream jobs share the worker)")
    ap.add_argument("--stream-gpu-pending", type=int, default=0,
                    help="download.stream_gpu_pending (parts awaiting GPU digests, all jobs)")
    ap.add_argument("--stream-gpu-tail", type=int, default=None,
                    help="download.stream_gpu_tail (queued parts below which the host hashes)")
    ap.add_argument("--stream-parallel", type=int, default=0,
                    help="download.torrent_stream_parallel (parts in flight per job)")
    ap.add_argument("--part-mb", type=int, default=0,
                    help="configs 3/4: override s3.part_size (MiB; one relayed part per unit)")
    ap.add_argument("--relay-trim-s", type=float, default=None,
                    help="configs 3/4: download.relay_pool_idle_trim_s (0: trim after every job)")
    ap.add_argument("--relay-memory-mb", type=int, default=0,
                    help="configs 3/4: download.relay_memory_mb (part-buffer budget per worker)")
    ap.add_argument("--stream-gpu-slots", type=int, default=0,
                    help="configs 3/4: download.stream_gpu_slots (PartHasher HBM slots)")
    ap.add_argument("--gpu-slot-mb", type=int, default=0,
                    help="configs 3/4: download.stream_gpu_slot_mb (PartHasher slot size)")
    ap.add_argument("--gpu-copy-streams", type=int, default=0,
                    help="configs 3/4: download.stream_gpu_copy_streams")
    ap.add_argument("--gpu-compute-streams", type=int, default=0,
                    help="configs 3/4: download.stream_gpu_compute_streams (0: the queues left)")
    ap.add_argument("--no-gpu-prewarm", action="store_true",
                    help="do not init the GPU verifier at worker start (download.gpu_prewarm)")
    ap.add_argument("--retry-backoff-s", type=float, default=0.05,
                    help="config 5: broker.retry_backoff_s (first backoff of a failed job)")
    ap.add_argument("--retry-delay", choices=["queue", "sleep"], default="queue",
                    help="config 5: broker.retry_delay (TTL holding queue vs in-consumer sleep)")
    ap.add_argument("--checksum", choices=["auto", "always", "off"], default="",
                    help="configs 1/3/4: s3.checksum (CRC32C payload integrity policy)")
    ap.add_argument("--workers", type=int, default=4, help="config 5 worker processes")
    ap.add_argument("--concurrency", type=int, default=4, help="config 5 jobs per worker")
    ap.add_argument("--qps", type=float, default=50.0, help="config 5 offered job rate")
    ap.add_argument("--src-dir", default="/dev/shm" if os.path.isdir("/dev/shm") else None)
    ap.add_argument("--stage-dir", default="")
    ap.add_argument("--cpus", type=int, default=0,
                    help="pin the bench (worker, blobd, config-5 workers) to this many CPUs; "
                         "0: the cgroup quota share, -1: no pinning")
    a = ap.parse_args(argv)
    os.environ.setdefault("LOG_LEVEL", "error")
    if a.cpus >= 0:
        from downloader_amd.utils.cpus import pin_share
        pin_share(0, 1, a.cpus)
    for c in a.config:
        if c == 1:
            out = asyncio.run(config1(a))
        elif c in (3, 4):
            out = asyncio.run(config_torrent(a, c))
        elif c == 5:
            out = asyncio.run(config5(a))
        elif c == 6:
            out = asyncio.run(config_swarm(a))
        elif c == 7:
            from .chaos import config_chaos
            out = asyncio.run(config_chaos(a))
        elif c == 8:
            out = asyncio.run(config_bucket(a))
        elif c == 9:
            out = asyncio.run(config_small(a))
        else:
            raise SystemExit(f"config {c}: use bench.py for config 2")
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
