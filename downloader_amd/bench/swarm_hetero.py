"""A heterogeneous swarm: the leecher against ``swarmd``'s fake seeders of
very different speed and latency, some of which stall mid-piece or hang up.

The reference's main torrent use is a public magnet through webtorrent
(/root/reference/lib/download.js:64-121; bittorrent-protocol, yarn.lock:389-398): up to 55
connections a torrent, to peers of every speed. Config 6's 1 - 4 loopback seeders never show
what that does to a downloader that hands whole 4 MiB pieces to one connection; here

  * every seeder has a token-bucket rate (log-uniform, default 0.2 - 50 MB/s) and answers
    each REQUEST after a delay (uniform, default 20 - 200 ms),
  * ``stall_share`` of them stop answering mid-piece (the connection stays open),
  * ``hangup_share`` of them close the connection part-way,

and the download is compared with the aggregate rate the healthy seeders offer. The leecher's
answers to it (torrent/session.py ``_rate_loop``): each connection's request pipeline follows
its bandwidth-delay product, and a peer slower than its share gives its whole pieces back.

    python -m downloader_amd.bench.swarm_hetero --gb 2 --peers 48 --wire native --wire python
"""
from __future__ import annotations

import argparse
import asyncio
import hashlib
import json
import math
import os
import random
import shutil
import subprocess
import tempfile
import time
from typing import Dict, List, Optional, Tuple

from ..ops import build

MB = 1_000_000


def hetero_specs(n: int = 48, seed: int = 1, rate_mb: Tuple[float, float] = (0.2, 50.0),
                 delay_ms: Tuple[int, int] = (20, 200), stall_share: float = 0.1,
                 hangup_share: float = 0.1, piece_len: int = 4 << 20) -> List[dict]:
    """Per seeder: rate (bytes/s), delay (ms), stall / hang-up point (payload bytes, 0 never).
    Stalls land mid-piece (a random point inside the 1st - 3rd piece's worth of bytes)."""
    rng = random.Random(seed)
    lo, hi = math.log(rate_mb[0] * MB), math.log(rate_mb[1] * MB)
    kinds = ["stall"] * round(n * stall_share) + ["hangup"] * round(n * hangup_share)
    kinds += ["ok"] * (n - len(kinds))
    rng.shuffle(kinds)
    out = []
    for k in kinds:
        rate = math.exp(rng.uniform(lo, hi))
        at = int(rng.uniform(0.3, 2.7) * piece_len)
        out.append({"rate": rate, "delay_ms": rng.randint(*delay_ms),
                    "stall": at if k == "stall" else 0, "hangup": at if k == "hangup" else 0,
                    "kind": k})
    return out


class Swarmd:
    """The native fake-seeder process (csrc/swarmd.cpp) for one single-file torrent."""

    def __init__(self, data_path: str, info_hash: bytes, pieces: int, piece_len: int,
                 specs: List[dict]):
        self.data_path = data_path
        self.info_hash = info_hash
        self.pieces = pieces
        self.piece_len = piece_len
        self.specs = specs
        self.proc: Optional[subprocess.Popen] = None
        self.ports: List[int] = []
        self.report = ""
        self._dir = ""

    def start(self, timeout: float = 30.0) -> "Swarmd":
        exe = build.build_swarmd(verbose=False)
        self._dir = tempfile.mkdtemp(prefix="swarmd-")
        spec = os.path.join(self._dir, "peers")
        with open(spec, "w") as f:
            for s in self.specs:
                f.write(f"{s['rate']:.0f} {s['delay_ms']} {s['stall']} {s['hangup']}\n")
        pf = os.path.join(self._dir, "ports")
        self.proc = subprocess.Popen(
            [str(exe), "--file", self.data_path, "--info-hash", self.info_hash.hex(),
             "--pieces", str(self.pieces), "--piece-length", str(self.piece_len),
             "--peers", spec, "--port-file", pf],
            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        t0 = time.time()
        while not os.path.exists(pf):
            if self.proc.poll() is not None:
                raise RuntimeError(f"swarmd exited: {self.proc.stderr.read().decode()}")
            if time.time() - t0 > timeout:
                self.stop()
                raise RuntimeError("swarmd did not start")
            time.sleep(0.02)
        self.ports = [int(x) for x in open(pf).read().split()]
        return self

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                _, err = self.proc.communicate(timeout=10)
                self.report = err.decode(errors="replace")
            except subprocess.TimeoutExpired:
                self.proc.kill()
        self.proc = None
        if self._dir:
            shutil.rmtree(self._dir, ignore_errors=True)

    def sent_per_seeder(self) -> List[int]:
        out = []
        for line in self.report.splitlines():
            if line.startswith("seeder "):
                out.append(int(line.split(": ", 1)[1].split(" B", 1)[0]))
        return out

    def __enter__(self) -> "Swarmd":
        return self.start()

    def __exit__(self, *a) -> None:
        self.stop()


def _write_random(path: str, total: int, seed: int) -> None:
    """Deterministic pseudo-random data, fast (SHA-256 counter blocks stretched to 1 MiB)."""
    with open(path, "wb") as f:
        left, i = total, 0
        while left > 0:
            blk = hashlib.sha256(b"%d-%d" % (seed, i)).digest() * 32768     # 1 MiB
            blk = bytes(b ^ (i & 0xFF) for b in blk[:64]) + blk[64:]
            k = min(left, len(blk))
            f.write(blk[:k])
            left -= k
            i += 1


def _threads() -> int:
    try:
        return len(os.listdir("/proc/self/task"))
    except OSError:
        return 0


async def run_hetero(total: int = 2 * 10 ** 9, piece_len: int = 4 << 20, peers: int = 48,
                     wire: str = "native", seed: int = 1, pipeline: int = 16,
                     timeout: float = 600.0, specs: Optional[List[dict]] = None,
                     src_dir: Optional[str] = None, io_threads: int = 4) -> Dict:
    """One download of a ``total``-byte single-file torrent from ``peers`` swarmd seeders."""
    from ..torrent.client import TorrentClient
    from ..torrent.metainfo import make_torrent, parse_torrent
    specs = specs or hetero_specs(peers, seed, piece_len=piece_len)
    src = tempfile.mkdtemp(prefix="hetero-src-", dir=src_dir)
    dst = tempfile.mkdtemp(prefix="hetero-dst-", dir=src_dir)
    try:
        path = os.path.join(src, "hetero.mkv")
        _write_random(path, total, seed)
        raw = make_torrent(path, piece_len)
        meta = parse_torrent(raw)
        healthy = [s for s in specs if s["kind"] == "ok"]
        offered = sum(s["rate"] for s in healthy)
        threads0 = _threads()
        with Swarmd(path, meta.info_hash, meta.num_pieces, piece_len, specs) as sd:
            leech = await TorrentClient(max_peers=max(64, peers + 8), pipeline=pipeline,
                                        native_wire=wire == "native",
                                        wire_io_threads=io_threads).start()
            try:
                t0 = time.perf_counter()
                s = await leech.add_torrent(meta, dst, peers=[("127.0.0.1", p) for p in sd.ports])
                peak = _threads()
                task = asyncio.ensure_future(s.wait())
                while not task.done():
                    await asyncio.wait([task], timeout=0.1)
                    peak = max(peak, _threads())
                    if time.perf_counter() - t0 > timeout:
                        task.cancel()
                        raise TimeoutError(f"hetero swarm: not done in {timeout} s")
                await task
                dt = time.perf_counter() - t0
                wst = s.wire.stats() if s.wire is not None else {}
                st = dict(s.stats)
                await leech.remove(s)
            finally:
                await leech.close()
            sent = None
        sent = sd.sent_per_seeder()
        with open(os.path.join(dst, "hetero.mkv"), "rb") as fa, open(path, "rb") as fb:
            same = hashlib.sha1(fa.read()).digest() == hashlib.sha1(fb.read()).digest()
    finally:
        shutil.rmtree(src, ignore_errors=True)
        shutil.rmtree(dst, ignore_errors=True)
    mbps = total / dt / MB
    # what the stalling / hanging-up seeders did deliver before they stopped, added to the
    # healthy ones' rates: the rate the swarm as a whole offered this download
    partial = sum(b for sp, b in zip(specs, sent or []) if sp["kind"] != "ok") / dt
    offered_all = offered + partial
    return {"config": "swarm-hetero", "wire": wire, "bytes": total, "piece_len": piece_len,
            "peers": peers, "seed": seed, "s": round(dt, 3), "MBps": round(mbps, 1),
            "offered_MBps": round(offered / MB, 1),
            "of_offered": round(mbps / (offered / MB), 3) if offered else None,
            "offered_incl_partial_MBps": round(offered_all / MB, 1),
            "of_offered_incl_partial": round(mbps / (offered_all / MB), 3) if offered_all else None,
            "healthy": len(healthy), "stalling": sum(s["kind"] == "stall" for s in specs),
            "hanging_up": sum(s["kind"] == "hangup" for s in specs),
            "data_ok": same, "threads_before": threads0, "threads_peak": peak,
            "wire_io_threads": wst.get("io_threads"),
            "slow_peers": st.get("slow_peers", 0),
            "slow_released_pieces": st.get("slow_released_pieces", 0),
            "slow_released_blocks": st.get("slow_released_blocks", 0),
            "max_owned_idle_s": st.get("max_owned_idle_s", 0.0),
            "max_depth": st.get("max_depth", 0), "hash_fails": st.get("hash_fails", 0),
            "endgame_pieces": st.get("wire_endgame_pieces", 0),
            "timeline": st.get("rate_timeline", []),
            "sent_per_seeder": sent}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=2.0)
    ap.add_argument("--piece-mb", type=int, default=4)
    ap.add_argument("--peers", type=int, default=48)
    ap.add_argument("--wire", action="append", default=[], choices=["native", "python"])
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--pipeline", type=int, default=16)
    ap.add_argument("--io-threads", type=int, default=4)
    ap.add_argument("--src-dir", default=None)
    a = ap.parse_args()
    for rep in range(a.reps):
        for w in a.wire or ["native", "python"]:
            r = asyncio.run(run_hetero(int(a.gb * 1e9), a.piece_mb << 20, a.peers, w,
                                       a.seed + rep, a.pipeline, src_dir=a.src_dir,
                                       io_threads=a.io_threads))
            r["rep"] = rep
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
