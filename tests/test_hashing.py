"""Native host hashing vs hashlib (SURVEY §4 rebuild plan item 5)."""
from __future__ import annotations

import hashlib
import os

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from downloader_amd.ops import hashing, native


@settings(max_examples=30, deadline=None)
@given(st.binary(min_size=0, max_size=5000), st.sampled_from(["sha1", "sha256", "md5"]))
def test_digest_matches_hashlib(data, algo):
    assert native().digest(algo, data) == hashlib.new(algo, data).digest()


@pytest.mark.parametrize("piece", [1, 63, 64, 65, 16384, 1 << 20])
def test_hash_pieces(piece):
    data = os.urandom(3 * 1048576 + 777)
    want = b"".join(hashlib.sha1(data[i:i + piece]).digest() for i in range(0, len(data), piece))
    if piece >= 64:
        assert hashing.hash_pieces(data, piece, threads=4) == want


def test_streaming_hasher_and_copy():
    h = native().Hasher("sha256")
    h.update(b"abc")
    c = h.copy()
    h.update(os.urandom(100000))
    c.update(b"def")
    assert c.digest() == hashlib.sha256(b"abcdef").digest()
    assert c.hexdigest() == hashlib.sha256(b"abcdef").hexdigest()


def _storage(tmp_path, sizes):
    files, blob = [], b""
    for i, n in enumerate(sizes):
        d = os.urandom(n)
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(d)
        files.append((str(p), n))
        blob += d
    return files, blob


def test_verify_pieces_across_file_boundaries(tmp_path):
    files, blob = _storage(tmp_path, [10000, 0, 70000, 3, 40000])
    piece = 16384
    hashes = b"".join(hashlib.sha1(blob[i:i + piece]).digest() for i in range(0, len(blob), piece))
    assert hashing.hash_storage_pieces(files, piece) == hashes
    ok = hashing.verify_pieces(files, piece, hashes, threads=3)
    assert ok == b"\x01" * len(ok)
    # corrupt one byte in the third file -> exactly the pieces covering it fail
    p = files[2][0]
    b = bytearray(open(p, "rb").read())
    b[20000] ^= 0xFF
    open(p, "wb").write(bytes(b))
    bad_off = 10000 + 20000
    ok = hashing.verify_pieces(files, piece, hashes)
    assert [i for i, v in enumerate(ok) if not v] == [bad_off // piece]
    # subset check
    sub = hashing.verify_pieces(files, piece, hashes, which=[0, bad_off // piece])
    assert sub == b"\x01\x00"
    # an explicit empty subset verifies nothing (only which=None is a full recheck)
    assert hashing.verify_pieces(files, piece, hashes, which=[]) == b""
    assert hashing.verify_pieces(files, piece, hashes, which=(), backend="gpu") == b""


def test_gpu_batcher_empty_batch_never_rechecks(monkeypatch):
    calls = []

    class V:
        def verify_files_streamed(self, files, plen, hashes, which=()):
            calls.append(list(which))
            return b"\x01" * len(which), (0.0, 0.0)

    monkeypatch.setattr(hashing, "_verifier", lambda: V())
    b = hashing.GpuBatcher()
    assert b.submit([("x", 10)], 4, b"\0" * 60, []).result(5) == []
    assert b.submit([("x", 10)], 4, b"\0" * 60, [2]).result(5) == [True]
    assert calls == [[2]]


def test_verify_missing_file_reports_false(tmp_path):
    files, blob = _storage(tmp_path, [50000])
    hashes = hashing.hash_storage_pieces(files, 16384)
    os.unlink(files[0][0])
    assert hashing.verify_pieces(files, 16384, hashes) == b"\x00" * 4


def test_hash_file_ranges(tmp_path):
    d = os.urandom(300000)
    p = tmp_path / "x"
    p.write_bytes(d)
    rngs = [(0, 100), (100, 299900), (5, 0)]
    out = hashing.hash_file_ranges(str(p), rngs, "md5", threads=2)
    assert out == [hashlib.md5(d[o:o + n]).digest() for o, n in rngs]


def test_choose_backend_cpu_without_gpu():
    assert hashing.choose_backend("cpu", 1 << 40, 1 << 20) == "cpu"
    assert hashing.choose_backend("auto", 100, 1) == "cpu"


def test_auto_backend_accounts_for_cold_start(monkeypatch):
    monkeypatch.setattr(hashing, "gpu_available", lambda: True)
    monkeypatch.setattr(hashing, "_gpu_verifier", object())
    # a host with the AVX-512 multi-buffer SHA-1 out-runs the device: auto stays on the host
    monkeypatch.setattr(hashing, "host_multibuffer", lambda: True)
    assert hashing.choose_backend("auto", hashing.GPU_COLD_MIN_BYTES, 1 << 20) == "cpu"
    assert not hashing.auto_may_use_gpu()
    assert hashing.choose_backend("gpu", 1, 1) == "gpu"
    monkeypatch.setattr(hashing, "host_multibuffer", lambda: False)
    monkeypatch.setattr(hashing, "_gpu_verifier", None)
    big, cold = hashing.GPU_MIN_BYTES, hashing.GPU_COLD_MIN_BYTES
    # Cold device: only a recheck large enough to amortise HIP init goes to the GPU.
    assert hashing.choose_backend("auto", big, 1024) == "cpu"
    assert hashing.choose_backend("auto", cold, 1024) == "gpu"
    # Few pieces never pay off, warm or not.
    assert hashing.choose_backend("auto", cold, 8) == "cpu"
    monkeypatch.setattr(hashing, "_gpu_verifier", object())
    assert hashing.choose_backend("auto", big, 1024) == "gpu"
    assert hashing.choose_backend("auto", big - 1, 1024) == "cpu"


def test_gpu_device_from_worker_index(monkeypatch):
    class _G:
        @staticmethod
        def device_count():
            return 8
    monkeypatch.setattr(hashing, "gpuhash", lambda: _G)
    monkeypatch.delenv("STAGER_GPU_DEVICE", raising=False)
    monkeypatch.setenv("STAGER_WORKER_INDEX", "11")
    assert hashing.gpu_device() == 3
    monkeypatch.setenv("STAGER_GPU_DEVICE", "5")
    assert hashing.gpu_device() == 5


@pytest.mark.parametrize("piece", [300_001, 262_144, 4096 + 64])
def test_multibuffer_verify_and_hash_storage(tmp_path, piece):
    """The AVX-512 16-lane path (``csrc/sha1_mb.cpp``): pieces longer than one 256 KiB lane
    step with a sub-block tail, groups of 16 plus a remainder, a file missing mid-torrent,
    corrupt pieces, the short last piece and an arbitrary ``which`` list - vs hashlib."""
    files, blob = _storage(tmp_path, [1_234_567, 2_000_000, 777_777, 0, 3_000_001])
    want = b"".join(hashlib.sha1(blob[i:i + piece]).digest() for i in range(0, len(blob), piece))
    n = len(want) // 20
    assert hashing.hash_storage_pieces(files, piece, threads=3) == want
    assert hashing.verify_pieces(files, piece, want, threads=2) == b"\x01" * n
    p = files[4][0]
    b = bytearray(open(p, "rb").read())
    for off in (5, 1_500_000, len(b) - 1):          # incl. the torrent's short last piece
        b[off] ^= 1
    open(p, "wb").write(bytes(b))
    base = sum(f[1] for f in files[:4])
    bad = sorted({(base + off) // piece for off in (5, 1_500_000, len(b) - 1)})
    os.unlink(files[2][0])                          # 777_777 bytes missing mid-torrent
    lost = set(range(sum(f[1] for f in files[:2]) // piece,
                     (sum(f[1] for f in files[:3]) - 1) // piece + 1))
    ok = hashing.verify_pieces(files, piece, want)
    assert [i for i in range(n) if not ok[i]] == sorted(lost | set(bad))
    which = [n - 1, 0, bad[0], n - 1, n + 5] + sorted(lost)[:1]
    sub = hashing.verify_pieces(files, piece, want, which=which)
    expect = [i not in lost and i not in bad and 0 <= i < n for i in which]
    assert list(sub) == [int(x) for x in expect]
