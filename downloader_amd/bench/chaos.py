"""Config 7 (extra): chaos soak of the whole service (SURVEY §5.3 failure detection / elastic
recovery / fault injection, under load).

The config-5 mix - 10 MB HTTP jobs (5 % with an injected 503) and 50 MB webseed torrents - is
fed through the bundled AMQP broker to a supervised pool of worker processes while a chaos task
alternately SIGKILLs a random worker (the supervisor respawns it; the broker requeues its
unacked deliveries) and drops every AMQP connection (workers reconnect and re-consume); with
``--s3-fail-rate`` the S3 peer also answers that share of object/part PUTs with 503 SlowDown
(the S3 client's retries). The run passes when every published job reaches ``v1.convert``
at least once. Reported: lost jobs (must be 0), duplicate converts (at-least-once
redeliveries of jobs that were killed between their convert publish and their ack), worker
restarts, per-process RSS / open-fd high-water marks, and what is left in the staging
directory after the drain.

The reference has no equivalent: a crash there drops the in-flight job's local data and relies
on RabbitMQ redelivery with no resume; stalls ack and lose the job.
"""
from __future__ import annotations

import asyncio
import os
import random
import shutil
import signal
import statistics
import sys
import tempfile
import time
from typing import Dict

from ..models import api
from .infra import Blobd

MB = 1_000_000
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _proc_stats(pid: int) -> Dict[str, float]:
    out = {"rss_MB": 0.0, "fds": 0}
    try:
        with open(f"/proc/{pid}/status") as f:
            for ln in f:
                if ln.startswith("VmRSS:"):
                    out["rss_MB"] = int(ln.split()[1]) / 1024
        out["fds"] = len(os.listdir(f"/proc/{pid}/fd"))
    except OSError:
        pass
    return out


def _tree_bytes(root: str) -> int:
    n = 0
    for dp, _, fns in os.walk(root):
        for fn in fns:
            try:
                n += os.path.getsize(os.path.join(dp, fn))
            except OSError:
                pass
    return n


async def config_chaos(a) -> Dict:
    from ..broker.amqp import AmqpBroker
    from ..broker.server import BrokerServer
    from ..parallel.supervisor import Supervisor, worker_argv
    from ..torrent.metainfo import make_torrent
    from .configs import _write_random

    n_jobs = max(20, int(600 * a.scale))
    src = tempfile.mkdtemp(prefix="cfg7-src-", dir=a.src_dir)
    stage = tempfile.mkdtemp(prefix="cfg7-stage-", dir=a.stage_dir or None)
    srv = await BrokerServer(heartbeat=0).start()
    rng = random.Random(7)
    with Blobd(sink="discard", files_root=src, s3_fail_rate=a.s3_fail_rate) as b:
        torrents = []
        for t in range(4):
            p = os.path.join(src, f"t{t}.mkv")
            _write_random(p, 50 * MB, 700 + t)
            raw = make_torrent(p, 1 << 20, url_list=[b.files_url(f"t{t}.mkv")])
            with open(os.path.join(src, f"t{t}.torrent"), "wb") as f:
                f.write(raw)
            torrents.append(b.files_url(f"t{t}.torrent"))
        env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error",
                   STAGER_BROKER__URL=srv.url, STAGER_BROKER__BACKEND="amqp",
                   STAGER_S3__ENDPOINT=b.endpoint, STAGER_INSTANCE__DOWNLOAD_PATH=stage,
                   STAGER_HEALTH__ENABLED="false", STAGER_DOWNLOAD__TORRENT_ENABLE_DHT="false",
                   STAGER_BROKER__RETRY_BACKOFF_S="0.05", STAGER_BROKER__MAX_RETRIES="5",
                   STAGER_CONCURRENCY=str(a.concurrency))
        mp = int(getattr(a, "chaos_multipart_mb", 0) or 0)
        if mp:      # the 50 MB torrents stage as multipart uploads a SIGKILL can leave open
            env.update(STAGER_S3__MULTIPART_THRESHOLD=str(mp * MB),
                       STAGER_S3__PART_SIZE=str(max(5, mp // 2) * MB))
        sup = Supervisor(a.workers, worker_argv(), env=env, backoff=0.2,
                         max_restarts=10_000)
        client = AmqpBroker(srv.url)
        await client.connect()
        for q in ("v1.download", "v1.convert"):
            await client.declare(q)
        sup.start()
        published: Dict[str, float] = {}
        first: Dict[str, float] = {}
        converts: Dict[str, int] = {}
        done = asyncio.Event()
        hw: Dict[str, float] = {"rss_MB": 0.0, "fds": 0}
        # pid -> [(t, rss_MB, fds)] every ~5 s: growth of long-lived workers shows leaks
        series: Dict[int, list] = {}
        last_sample = [0.0]
        actions = {"kill": 0, "drop": 0}

        async def on_convert(d):
            mid = api.decode(api.Convert, d.body).media.id
            converts[mid] = converts.get(mid, 0) + 1
            if mid in published and mid not in first:
                first[mid] = time.perf_counter() - published[mid]
            await d.ack()
            if len(first) >= n_jobs:
                done.set()
        await client.consume("v1.convert", on_convert, prefetch=64)

        async def supervise():
            while not done.is_set():
                sup.poll()
                now = time.perf_counter()
                sample = now - last_sample[0] >= 5.0
                if sample:
                    last_sample[0] = now
                for s in sup.slots:
                    if s.proc is not None and s.proc.poll() is None:
                        st = _proc_stats(s.proc.pid)
                        hw["rss_MB"] = max(hw["rss_MB"], st["rss_MB"])
                        hw["fds"] = max(hw["fds"], st["fds"])
                        if sample and st["rss_MB"]:
                            series.setdefault(s.proc.pid, []).append(
                                (now, st["rss_MB"], st["fds"]))
                await asyncio.sleep(0.1)

        async def chaos():
            k = 0
            while not done.is_set():
                await asyncio.sleep(a.chaos_interval)
                if done.is_set():
                    break
                if k % 2 == 0 and a.chaos_kill:
                    live = [s for s in sup.slots if s.proc is not None and s.proc.poll() is None]
                    if live:
                        victim = rng.choice(live)
                        try:
                            os.kill(victim.proc.pid, signal.SIGKILL)
                            actions["kill"] += 1
                        except ProcessLookupError:
                            pass
                elif k % 2 == 1:
                    srv.drop_connections()
                    actions["drop"] += 1
                k += 1

        async def report():
            t_start = time.perf_counter()
            while not done.is_set():
                await asyncio.sleep(30)
                print(f"[chaos] {time.perf_counter() - t_start:.0f}s published {len(published)} "
                      f"converted {len(first)} kills {actions['kill']} drops {actions['drop']}",
                      file=sys.stderr, flush=True)

        tasks = [asyncio.ensure_future(supervise()), asyncio.ensure_future(chaos()),
                 asyncio.ensure_future(report())]
        t0 = time.perf_counter()
        for i in range(n_jobs):
            target = t0 + i / a.qps
            now = time.perf_counter()
            if target > now:
                await asyncio.sleep(target - now)
            jid = f"c7-{i}"
            if rng.random() < 0.2:
                m = api.make_download(jid, "http", torrents[i % 4])
            else:
                url = b.media_url(f"c7-{i}.mkv", 10 * MB, i)
                if rng.random() < 0.05:
                    url += "&fail=1"
                m = api.make_download(jid, "http", url)
            published[jid] = time.perf_counter()
            await client.publish("v1.download", api.encode(m))
        timed_out = False
        try:
            await asyncio.wait_for(done.wait(), a.chaos_timeout)
        except asyncio.TimeoutError:
            timed_out = True
        wall = time.perf_counter() - t0
        done.set()
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
        # drain: let redelivered duplicates settle, then stop the pool
        await asyncio.sleep(1.0)
        codes = await asyncio.get_running_loop().run_in_executor(None, sup.stop)
        bst = b.stats()
        s3_faults = bst.get("s3_faults", 0)
        # multipart uploads still open: what killed workers left and no sweep reclaimed
        open_uploads = bst.get("open_uploads", 0)
        restarts = sum(s.restarts for s in sup.slots)
        await client.close()
        await srv.stop()
        leftover = _tree_bytes(stage)
        shutil.rmtree(src, ignore_errors=True)
        shutil.rmtree(stage, ignore_errors=True)
    lat = list(first.values())
    lost = sorted(set(published) - set(first))
    # leak check: workers that lived >= 60 s, RSS / fds at their first sample >= 20 s after the
    # start of the series (warm) vs their last sample
    growth = []
    for pid, pts in series.items():
        if len(pts) < 2 or pts[-1][0] - pts[0][0] < 60:
            continue
        warm = next((p for p in pts if p[0] - pts[0][0] >= 20), pts[0])
        growth.append({"pid": pid, "lived_s": round(pts[-1][0] - pts[0][0], 1),
                       "rss_warm_MB": round(warm[1], 1), "rss_end_MB": round(pts[-1][1], 1),
                       "fds_warm": warm[2], "fds_end": pts[-1][2]})
    return {"config": 7, "jobs": n_jobs, "workers": a.workers, "qps_offered": a.qps,
            "chaos_interval_s": a.chaos_interval, "kills": actions["kill"],
            "connection_drops": actions["drop"], "worker_restarts": restarts,
            "s3_fail_rate": a.s3_fail_rate, "s3_faults_injected": s3_faults,
            "wall_s": round(wall, 2), "timed_out": timed_out,
            "lost_jobs": len(lost), "lost_examples": lost[:5],
            "duplicate_converts": sum(c - 1 for c in converts.values() if c > 1),
            "p50_latency_s": round(statistics.median(lat), 4) if lat else None,
            "p99_latency_s": round(sorted(lat)[int(0.99 * (len(lat) - 1))], 4) if lat else None,
            "worker_rss_high_MB": round(hw["rss_MB"], 1), "worker_fds_high": hw["fds"],
            "stage_leftover_bytes": leftover, "s3_open_uploads": open_uploads,
            "worker_exit_codes": codes,
            "long_lived_workers": growth}
