"""Probe: aggregate page-cache write bandwidth into ONE file from T threads, via pwrite vs a
shared writable mmap (+ optional MADV_POPULATE_WRITE). Tells whether parallel webseed streams
into a single-file torrent are bound by the file's write path."""
import mmap
import os
import sys
import tempfile
import threading
import time

import numpy as np

N = int(float(sys.argv[1]) if len(sys.argv) > 1 else 4e9)
CH = 64 << 20
d = sys.argv[2] if len(sys.argv) > 2 else tempfile.gettempdir()
src = np.frombuffer(os.urandom(CH), dtype=np.uint8)


def run(mode, threads):
    path = os.path.join(d, f"probe.{os.getpid()}")
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
    os.ftruncate(fd, N)
    chunks = list(range(0, N, CH))
    lock = threading.Lock()
    mm = None
    if mode.startswith("mmap"):
        mm = mmap.mmap(fd, N, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        arr = np.frombuffer(mm, dtype=np.uint8)

    def work():
        while True:
            with lock:
                if not chunks:
                    return
                off = chunks.pop()
            ln = min(CH, N - off)
            if mode == "pwrite":
                mv = memoryview(src)[:ln]
                w = 0
                while w < ln:
                    w += os.pwrite(fd, mv[w:], off + w)
            else:
                if mode == "mmap_populate":
                    mm.madvise(23, off, ln)   # MADV_POPULATE_WRITE
                arr[off:off + ln] = src[:ln]
    t0 = time.perf_counter()
    ts = [threading.Thread(target=work) for _ in range(threads)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    dt = time.perf_counter() - t0
    if mm is not None:
        del arr
        mm.close()
    os.close(fd)
    t1 = time.perf_counter()
    os.unlink(path)
    print(f"{mode:14s} threads={threads:2d} {N / dt / 1e9:6.2f} GB/s  unlink {time.perf_counter() - t1:.3f}s",
          flush=True)


for mode in ("pwrite", "mmap", "mmap_populate"):
    for th in (1, 2, 4, 8):
        try:
            run(mode, th)
        except OSError as e:
            print(mode, th, "error", e)
