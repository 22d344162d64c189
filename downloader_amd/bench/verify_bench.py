"""Piece-verification benchmark: the MI355X SHA-1 kernel vs the host (OpenSSL SHA-NI) path.

Reference hot loop: webtorrent verifies every piece with SHA-1 (SURVEY §2.5, §3 hot loop 2);
BASELINE.json configs 3/4 run "full piece verification" over 4 GB / 20 GB torrents.

Reports (JSON lines):
  * ``kernel``  - device-resident data, hipEvent-timed, v_bitop3 vs plain-C rounds (A/B
    interleaved in one process), GB/s per piece size and piece count;
  * ``verify``  - end-to-end recheck of a multi-file torrent that sits in the page cache:
    CPU (threaded native SHA-1) vs GPU (pread -> pinned -> H2D -> kernel, double-buffered).

  python -m downloader_amd.bench.verify_bench --gib 4 --piece-mb 1
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time


def emit(d) -> None:
    print(json.dumps(d), flush=True)


def kernel_section(gv, sizes, counts, iters) -> None:
    for plen in sizes:
        for n in counts:
            if plen * n > (16 << 30):
                continue
            ms_b3, ms_plain = gv.kernel_bench(plen, n, iters)
            gb = plen * n / 1e9
            emit({"section": "kernel", "piece_len": plen, "pieces": n,
                  "ms_bitop3": round(ms_b3, 3), "ms_plain": round(ms_plain, 3),
                  "GBps_bitop3": round(gb / (ms_b3 / 1e3), 1),
                  "GBps_plain": round(gb / (ms_plain / 1e3), 1),
                  "speedup": round(ms_plain / ms_b3, 3)})
            if hasattr(gv, "kernel_bench_prefetch"):
                ms_pf, ms_nopf = gv.kernel_bench_prefetch(plen, n, iters)
                emit({"section": "kernel_prefetch", "piece_len": plen, "pieces": n,
                      "ms_prefetch": round(ms_pf, 3), "ms_no_prefetch": round(ms_nopf, 3),
                      "GBps_prefetch": round(gb / (ms_pf / 1e3), 1),
                      "GBps_no_prefetch": round(gb / (ms_nopf / 1e3), 1),
                      "speedup": round(ms_nopf / ms_pf, 3)})


def make_files(root: str, total: int, nfiles: int):
    import numpy as np
    rng = np.random.default_rng(1234)
    os.makedirs(root, exist_ok=True)
    files = []
    per = total // nfiles
    for i in range(nfiles):
        n = per + (total - per * nfiles if i == nfiles - 1 else 0) + (i * 4099 % 777 if i else 0)
        p = os.path.join(root, f"f{i:03d}.mkv")
        with open(p, "wb") as f:
            left = n
            while left:
                k = min(left, 256 << 20)
                f.write(rng.bytes(k))
                left -= k
        files.append((p, n))
    return files


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--piece-mb", type=float, default=1.0)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--dir", default="/dev/shm/stager-verify-bench")
    ap.add_argument("--threads", type=int, default=16, help="CPU hashing threads")
    ap.add_argument("--readers", type=int, default=8, help="GPU path pread threads")
    ap.add_argument("--batch-mb", type=int, default=512)
    ap.add_argument("--chunk-kb", type=int, default=64, help="streamed path chunk per lane")
    ap.add_argument("--kernel-only", action="store_true")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--kernel-sizes", default="256,1024,4096", help="kernel section piece KiB")
    ap.add_argument("--kernel-counts", default="1024,4096,16384", help="kernel section pieces")
    a = ap.parse_args(argv)

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from downloader_amd.ops import gpu_available, gpuhash, hashing
    if not gpu_available():
        print("no HIP device", file=sys.stderr)
        return 2
    gv = gpuhash().GpuVerifier(0, a.batch_mb << 20, a.readers)
    emit({"section": "device", "arch": gpuhash().arch()})
    kernel_section(gv, [int(k) << 10 for k in a.kernel_sizes.split(",")],
                   [int(n) for n in a.kernel_counts.split(",")], 3)
    if a.kernel_only:
        return 0

    plen = int(a.piece_mb * (1 << 20))
    total = int(a.gib * (1 << 30))
    t0 = time.perf_counter()
    files = make_files(a.dir, total, a.files)
    total = sum(n for _, n in files)
    emit({"section": "setup", "bytes": total, "files": len(files), "write_s":
          round(time.perf_counter() - t0, 2)})
    try:
        t0 = time.perf_counter()
        hashes = hashing.hash_storage_pieces(files, plen, "sha1", a.threads)
        dt = time.perf_counter() - t0
        emit({"section": "cpu_hash", "threads": a.threads, "GBps": round(total / dt / 1e9, 2)})
        npieces = len(hashes) // 20
        for r in range(a.repeat):
            t0 = time.perf_counter()
            ok = hashing.native().verify_pieces(files, plen, hashes, [], a.threads)
            dc = time.perf_counter() - t0
            assert ok == b"\x01" * npieces
            t0 = time.perf_counter()
            okg = gv.verify_files(files, plen, hashes)
            dg = time.perf_counter() - t0
            assert okg == ok, "GPU (whole-piece) and CPU verification disagree"
            t0 = time.perf_counter()
            oks, (t_fill, t_wait) = gv.verify_files_streamed(files, plen, hashes, a.chunk_kb << 10)
            ds = time.perf_counter() - t0
            assert oks == ok, "GPU (streamed) and CPU verification disagree"
            emit({"section": "verify", "round": r, "bytes": total, "pieces": npieces,
                  "piece_len": plen, "cpu_threads": a.threads, "cpu_s": round(dc, 3),
                  "cpu_GBps": round(total / dc / 1e9, 2), "gpu_readers": a.readers,
                  "gpu_whole_piece_GBps": round(total / dg / 1e9, 2),
                  "gpu_streamed_s": round(ds, 3), "gpu_streamed_GBps": round(total / ds / 1e9, 2),
                  "streamed_host_fill_s": round(t_fill, 3), "streamed_host_wait_s": round(t_wait, 3),
                  "streamed_vs_cpu": round(dc / ds, 3)})
        # corruption is still caught by the GPU path
        p0, _ = files[len(files) // 2]
        with open(p0, "r+b") as f:
            f.seek(12345)
            b = f.read(1)
            f.seek(12345)
            f.write(bytes([b[0] ^ 0xFF]))
        okg = gv.verify_files(files, plen, hashes)
        oks, _ = gv.verify_files_streamed(files, plen, hashes, a.chunk_kb << 10)
        emit({"section": "corruption", "bad_pieces": okg.count(0),
              "bad_pieces_streamed": oks.count(0)})
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
