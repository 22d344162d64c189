"""Same-call A/B of the streamed torrent path: pieces hashed by the gfx950 PartHasher
(``download.stream_verify_backend: auto``) vs the host multi-buffer SHA-1 (``cpu``).

A config-4-shaped torrent (BASELINE.json config 4: 20 GB, 50 files, full piece verification,
one S3 object per file; 4 MiB pieces) is served by a ``blobd`` webseed from its synthetic
pool (``bench/synth_torrent.py``: no data on disk) and staged by two workers of this process,
one per backend, alternating job by job after one untimed job each (HIP initialisation,
connection pools). The reference verifies every piece with SHA-1 in webtorrent
(/root/reference/lib/download.js:64); this measures both of our ways of doing that under the
same clock, in the call that produces the driver's bench line.
"""
from __future__ import annotations

import asyncio
import os
import shutil
import statistics
import tempfile
import time
from typing import Dict, List, Optional

from .infra import Blobd
from .synth_torrent import config4_files, make_synth_torrent, served_paths

MB = 1_000_000


def _relay_counters() -> Dict:
    try:
        from ..ops import native
        return dict(native().relay_counters())
    except Exception:
        return {}


def _cpu() -> float:
    t = os.times()
    return t.user + t.system


async def _stage(w, msg) -> tuple:
    done = asyncio.get_running_loop().create_future()

    def cb(r):
        if not done.done():
            done.set_result(r)
    w.on_result = cb
    t0 = time.perf_counter()
    await w.submit(msg)
    r = await asyncio.wait_for(done, 900)
    w.on_result = None
    return time.perf_counter() - t0, r


async def torrent_ab(total_bytes: int = 20 * 10 ** 9, files: int = 50, piece_len: int = 4 << 20,
                     pairs: int = 3, stage_root: str = "", tag: str = "ab",
                     backends=("auto", "cpu"), download: Optional[Dict] = None) -> Dict:
    """Stage the torrent ``pairs`` times per backend, alternating; medians of the timed jobs.
    ``download``: extra ``download.*`` settings of both workers (A/B knobs)."""
    from ..broker.memory import MemoryBroker
    from ..models import api
    from ..ops import hashing
    from ..service.worker import Worker
    from ..utils.config import load_config

    name = "Show"
    fl = config4_files(total_bytes, files, name)
    total = sum(n for _, n, _ in fl)
    root = tempfile.mkdtemp(prefix="torrent-ab-")
    stage = stage_root or tempfile.mkdtemp(prefix="torrent-ab-stage-")
    workers = {}
    try:
        with Blobd(sink="discard", files_root=root, synth_files=served_paths(name, fl)) as b:
            t0 = time.perf_counter()
            raw = make_synth_torrent(b.pool(), name, fl, piece_len, b.files_url(),
                                     threads=min(16, os.cpu_count() or 1))
            setup_s = time.perf_counter() - t0
            with open(os.path.join(root, "job.torrent"), "wb") as f:
                f.write(raw)
            for be in backends:
                cfg = load_config(overrides={
                    "instance": {"download_path": os.path.join(stage, be)},
                    "s3": {"endpoint": b.endpoint}, "broker": {"backend": "memory"},
                    "health": {"enabled": False},
                    "download": {"torrent_enable_dht": False, "progress_interval_s": 5.0,
                                 "stream_verify_backend": be, "gpu_prewarm": be != "cpu",
                                 **(download or {})}},
                    env={})
                w = Worker(cfg, broker=MemoryBroker())
                await w.start(health=False)
                workers[be] = w
            url = b.files_url("job.torrent")
            runs: Dict[str, List[dict]] = {be: [] for be in backends}
            dev0 = None
            for k in range(pairs + 1):                 # round 0: one untimed job each
                for be in backends:
                    if be != "cpu" and k == 1:
                        dev0 = hashing.gpu_relay_stats()
                    msg = api.make_download(f"{tag}-{be}-{k}", "http", url, "TV")
                    c0, p0 = _cpu(), b.cpu_seconds()
                    rc0 = _relay_counters()
                    dt, r = await _stage(workers[be], msg)
                    c1, p1 = _cpu(), b.cpu_seconds()
                    rc1 = _relay_counters()
                    if r.outcome != "staged":
                        raise RuntimeError(f"torrent A/B job ({be}) failed: {r.error}")
                    if r.bytes != total:
                        raise RuntimeError(f"torrent A/B job ({be}) staged {r.bytes} of {total}")
                    if k:
                        t = r.stats.get("torrent", {})
                        runs[be].append({"s": dt, "worker_cpu_s": c1 - c0, "peer_cpu_s": p1 - p0,
                                         "hash_fails": t.get("hash_fails", 0),
                                         "parts": t.get("parts", 0),
                                         "gpu_parts": t.get("gpu_parts", 0),
                                         "timeline": dict(t.get("timeline", {}), job_s=dt),
                                         "relay": {k: rc1[k] - rc0.get(k, 0) for k in rc1}})
            dev1 = hashing.gpu_relay_stats() if any(be != "cpu" for be in backends) else {}
            st = b.stats()
    finally:
        for w in workers.values():
            await w.stop()
        shutil.rmtree(root, ignore_errors=True)
        if not stage_root:
            shutil.rmtree(stage, ignore_errors=True)

    out: Dict = {"torrent_bytes": total, "torrent_files": len(fl), "torrent_piece_len": piece_len,
                 "torrent_pairs": pairs, "torrent_setup_s": round(setup_s, 2),
                 "torrent_sink_bytes": st.get("bytes_received", 0)}
    for be in backends:
        xs = runs[be]
        key = "gpu" if be != "cpu" else "host"
        med = statistics.median(x["s"] for x in xs)
        out[f"torrent_{key}_MBps"] = round(total / med / MB, 1)
        out[f"torrent_{key}_MBps_runs"] = [round(total / x["s"] / MB, 1) for x in xs]
        out[f"torrent_{key}_worker_cpu_s_per_GB"] = round(
            statistics.median(x["worker_cpu_s"] for x in xs) / (total / 1e9), 4)
        out[f"torrent_{key}_hash_fails"] = sum(x["hash_fails"] for x in xs)
        # where a job's time goes (torrent/stream.py timeline, seconds from the stager's
        # start; job_s from the submit): medians over the timed jobs
        keys_t = sorted({k for x in xs for k in x["timeline"]})
        out[f"torrent_{key}_timeline_s"] = {
            k: round(statistics.median(x["timeline"][k] for x in xs if k in x["timeline"]), 4)
            for k in keys_t}
        # where the workers' CPU went (native relay counters, as the headline's
        # worker_breakdown): relaying threads, CRC, host SHA-1, the rest
        rc: Dict = {}
        for x in xs:
            for k, v in x["relay"].items():
                rc[k] = rc.get(k, 0) + v
        gb = max(1e-9, len(xs) * total / 1e9)
        cpu = sum(x["worker_cpu_s"] for x in xs)
        relay_s = sum(rc.get(f"{m}_cpu_ns", 0) for m in ("splice", "dup", "copy", "hashed")) / 1e9
        out[f"torrent_{key}_breakdown"] = {
            # relaying threads of the hashed relays (peek copy into the part buffer, CRC,
            # splice; host SHA-1 of the parts not given to the device)
            "relay_threads_cpu_s_per_GB": round(relay_s / gb, 4),
            "host_sha1_s_per_GB": round(rc.get("sha1_ns", 0) / 1e9 / gb, 4),
            "crc_cpu_s_per_GB": round(rc.get("crc_ns", 0) / 1e9 / gb, 4),
            "other_worker_cpu_s_per_GB": round(max(0.0, cpu - relay_s) / gb, 4),
            "relays": {m: rc.get(f"{m}_relays", 0) for m in ("splice", "dup", "copy", "hashed")}}
        if be != "cpu":      # parts whose pieces the device hashed / all parts, timed jobs
            parts = sum(x["parts"] for x in xs)
            out["gpu_part_share"] = round(sum(x["gpu_parts"] for x in xs) / parts, 3) \
                if parts else 0.0
    if dev0 is not None:
        d = {k: dev1.get(k, 0) - dev0.get(k, 0) for k in
             ("submitted", "host_fallbacks", "refused", "device_launches", "device_lanes")}
        out["gpu_parts"] = d["submitted"]
        out["gpu_host_fallbacks"] = d["host_fallbacks"]
        out["gpu_refused"] = d["refused"]
        out["gpu_launches"] = d["device_launches"]
        out["gpu_lanes_per_launch"] = round(d["device_lanes"] / d["device_launches"], 1) \
            if d["device_launches"] else 0.0
        out["gpu_multi_slot_launches"] = dev1.get("device_multi_slot_launches", 0) - \
            dev0.get("device_multi_slot_launches", 0)
        out["gpu_max_launch_lanes"] = dev1.get("device_max_batch_lanes", 0)
    return out


def main() -> None:
    """``python -m downloader_amd.bench.torrent_ab --gb 20 --set stream_gpu_tail=32``: the A/B
    alone, one JSON line (A/B of download.* knobs on the box)."""
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=20.0)
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--set", action="append", default=[], help="download.KEY=VALUE (both arms)")
    ap.add_argument("--no-pin", action="store_true",
                    help="run on the whole CPU mask (default: pinned like bench.py's rank)")
    a = ap.parse_args()
    # as bench.py pins a rank (and its blobd, which inherits the mask) to one GPU slot's share
    # of the CPUs: unpinned, a 16-CPU quota over a mask of hundreds throttles in bursts and
    # both arms ran ~20 - 24 GB/s instead of 27 - 34, their ratio lost in it (r6/split/)
    pinned = []
    if not a.no_pin:
        from ..utils import cpus
        pinned = cpus.pin_slot(0, max(1, cpus.gpu_slots()))
    over: Dict = {}
    for kv in a.set:
        k, _, v = kv.partition("=")
        over[k] = json.loads(v) if v[:1] in "0123456789-[{tf\"" else v
    out = asyncio.run(torrent_ab(total_bytes=int(a.gb * 1e9), pairs=a.pairs, download=over))
    out["download"] = over
    out["pinned_cpus"] = len(pinned)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
