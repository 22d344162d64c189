"""Torrents whose files are the bench origin's synthetic bytes (no data on disk).

``blobd --synth-files`` serves BEP-19 webseed files made of its origin pool: byte ``o`` of a
file with seed ``s`` is ``pool[(o + 7919 s) % POOL]`` (the same rule as its ``/media/``
origin). POOL is 64 MiB + 4 KiB, an odd number of pages: no power-of-two part or piece size
divides it, so data fetched from the wrong part / piece offset never carries the right bytes
(``csrc/blobd.cpp`` kPool). This module writes the metainfo for such a file set: the piece
SHA-1s are computed over the same rule. Pieces that start at the same pool offset share their
hash (computed once); with the odd period that happens only every 16385 pieces, so the
hashing costs about the torrent's size, spread over threads, and no disk.

Used by ``bench.py`` for the config-4-shaped GPU vs host A/B (20 GB, 50 files, 4 MiB pieces)
that the driver's bench line carries, and by the tests in miniature.
"""
from __future__ import annotations

import hashlib
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Sequence, Tuple

from ..torrent.bencode import bencode

POOL = (64 << 20) + 4096     # blobd's kPool
STRIDE = 7919


def config4_files(total: int, n: int = 50, name: str = "Show") -> List[Tuple[str, int, int]]:
    """Config 4's shape (bench/configs.py): ``n`` episodes of ~total/n bytes under
    ``Season 1/``, (relative path, size, seed) each."""
    return [(f"Season 1/{name} E{i + 1:02d}.mkv", total // n + (i * 7919) % 1000, 100 + i)
            for i in range(n)]


def served_paths(name: str, files: Sequence[Tuple[str, int, int]]) -> Dict[str, Tuple[int, int]]:
    """``Blobd(synth_files=...)``: the webseed path of each file (``<name>/<rel>``, BEP-19's
    multi-file URL rule) -> (size, seed)."""
    return {f"{name}/{rel}": (size, seed) for rel, size, seed in files}


def _segments(files: Sequence[Tuple[str, int, int]], piece_len: int, period: int = POOL):
    """Per piece: the (pool offset, length) runs it is made of, in order."""
    out: List[Tuple[Tuple[int, int], ...]] = []
    cur: List[Tuple[int, int]] = []
    room = piece_len
    for _, size, seed in files:
        off = 0
        while off < size:
            k = min(room, size - off)
            cur.append(((off + seed * STRIDE) % period, k))
            off += k
            room -= k
            if room == 0:
                out.append(tuple(cur))
                cur, room = [], piece_len
    if cur:
        out.append(tuple(cur))
    return out


def piece_hashes(pool: bytes, files: Sequence[Tuple[str, int, int]], piece_len: int,
                 threads: int = 8) -> bytes:
    if len(pool) < piece_len:
        raise ValueError("piece length above the pool size")
    ring = memoryview(pool + pool[:piece_len])     # any run of <= piece_len bytes is contiguous
    segs = _segments(files, piece_len, len(pool))   # the served pool's period (POOL normally)
    uniq = list(dict.fromkeys(segs))

    def h(key) -> bytes:
        d = hashlib.sha1()
        for po, k in key:
            d.update(ring[po:po + k])
        return d.digest()
    with ThreadPoolExecutor(max(1, threads)) as ex:       # hashlib drops the GIL on big buffers
        digest = dict(zip(uniq, ex.map(h, uniq)))
    return b"".join(digest[s] for s in segs)


def make_synth_torrent(pool: bytes, name: str, files: Sequence[Tuple[str, int, int]],
                       piece_len: int, webseed_root: str, threads: int = 8) -> bytes:
    """Multi-file metainfo for ``files`` (relative paths under ``name``) with one webseed,
    ``webseed_root`` = blobd's ``files_url()``."""
    info = {"name": name, "piece length": piece_len,
            "files": [{"path": rel.split("/"), "length": size} for rel, size, _ in files],
            "pieces": piece_hashes(pool, files, piece_len, threads)}
    return bencode({"info": info, "created by": "downloader-amd bench", "url-list": [webseed_root]})
