"""The bench's own integrity checks.

* The origin's bytes repeat with a period of 64 MiB + 4 KiB (``csrc/blobd.cpp`` kPool), which
  no power-of-two part or piece size divides: a multipart part sent from the wrong Range, or a
  webseed read shifted by whole 64 MiB parts, no longer carries the bytes it should. With the
  round-5 period (exactly 64 MiB = the part size = 16 pieces of 4 MiB) both errors passed the
  sink's compare and the piece SHA-1s (checked with ``STAGER_BLOBD_EXE`` pointed at the old
  build: profiles/r6/aliasing/).
* The S3 peer recomputes the CRC32C of a salted 1-in-N subset of the checksummed bodies
  (``--crc-check``) and checks the others' trailers for form; a wrong CRC inside the subset is
  refused (400 BadDigest) and fails the bench run.
"""
from __future__ import annotations

import base64
import http.client
import json
import os
import re
import subprocess
import sys
import urllib.request
from urllib.parse import quote

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MiB = 1 << 20


def _req(port, method, path, body=b"", headers=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request(method, path, body=body, headers=headers or {})
    r = c.getresponse()
    data = r.read()
    c.close()
    return r.status, data


def _origin_range(b, name, size, seed, start, length) -> bytes:
    req = urllib.request.Request(b.media_url(name, size, seed),
                                 headers={"Range": f"bytes={start}-{start + length - 1}"})
    with urllib.request.urlopen(req, timeout=60) as r:
        assert r.status == 206
        return r.read()


def _multipart(b, key, parts) -> None:
    path = "/triton-staging/" + quote(key, safe="/")
    _req(b.port, "PUT", "/triton-staging")
    st, x = _req(b.port, "POST", path + "?uploads")
    assert st == 200
    uid = re.search(rb"<UploadId>([^<]+)</UploadId>", x).group(1).decode()
    for i, body in enumerate(parts, 1):
        assert _req(b.port, "PUT", f"{path}?partNumber={i}&uploadId={uid}", body)[0] == 200
    assert _req(b.port, "POST", f"{path}?uploadId={uid}", b"<CompleteMultipartUpload/>")[0] == 200


@pytest.mark.parametrize("wrong", [False, True])
def test_sink_catches_a_part_relayed_from_the_previous_parts_range(wrong):
    """A 100 MB object in 64 MiB parts (the headline's shape) whose part 2 carries the bytes of
    part 1's Range start: the sample sink's windows no longer match the origin's bytes."""
    from downloader_amd.bench.infra import Blobd
    size, seed, part = 100_000_000, 11, 64 * MiB
    with Blobd(sink="sample") as b:
        p1 = _origin_range(b, "alias.mkv", size, seed, 0, part)
        p2 = _origin_range(b, "alias.mkv", size, seed, 0 if wrong else part, size - part)
        key = "job-alias-%d/original/%s" % (wrong, base64.b64encode(b"alias.mkv").decode())
        _multipart(b, key, [p1, p2])
        st = b.stats()
        assert st["verify_objects"] == 1 and st["verify_unknown"] == 0
        assert st["verify_mismatches"] == (1 if wrong else 0)


def test_origin_period_is_not_a_part_or_piece_multiple():
    """Byte o and byte o + k x 4 MiB of one object differ for every k up to a 20 GB torrent."""
    from downloader_amd.bench.infra import Blobd
    from downloader_amd.bench.synth_torrent import POOL
    assert POOL % (4 * MiB) and (POOL // 4096) % 2 == 1
    with Blobd(sink="discard") as b:
        pool = b.pool()
    assert len(pool) == POOL
    win = 4096
    for k in (1, 16, 32, 1000, 4768):              # 4 MiB .. 20 GB offsets
        o = (k * 4 * MiB) % POOL
        ring = pool + pool[:win]
        assert ring[o:o + win] != pool[:win], k


def test_webseed_shifted_by_one_part_fails_the_piece_hashes(run, tmp_path):
    """A webseed whose files are served 64 MiB off (a whole part / 16 pieces): the streamed
    torrent job's piece SHA-1s fail and the job is not staged."""
    from downloader_amd.bench.infra import Blobd
    from downloader_amd.bench.synth_torrent import make_synth_torrent, served_paths
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api
    from downloader_amd.service.worker import Worker
    from downloader_amd.utils.config import load_config

    name = "Shift"
    files = [("Season 1/Shift E01.mkv", 80 * MiB + 123, 5)]
    root = tmp_path / "seed"
    root.mkdir()

    async def go(b):
        raw = make_synth_torrent(b.pool(), name, files, 4 * MiB, b.files_url(), threads=4)
        (root / "job.torrent").write_bytes(raw)
        cfg = load_config(overrides={
            "instance": {"download_path": str(tmp_path / "dl")},
            "s3": {"endpoint": b.endpoint}, "health": {"enabled": False},
            "broker": {"backend": "memory", "max_retries": 0, "retry_backoff_s": 0.01},
            "download": {"torrent_enable_dht": False, "stream_verify_backend": "cpu",
                         "gpu_prewarm": False}}, env={})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        try:
            await w.submit(api.make_download("shifted", "http", b.files_url("job.torrent"), "TV"))
            import asyncio
            for _ in range(1200):
                if w.results:
                    break
                await asyncio.sleep(0.05)
            return w.results[0]
        finally:
            await w.stop()

    with Blobd(sink="discard", files_root=str(root), synth_files=served_paths(name, files),
               synth_shift=64 * MiB) as b:
        r = run(go(b), timeout=120)
    assert r.outcome != "staged", r
    assert "corrupt" in r.error or "hash" in r.error.lower() or "piece" in r.error, r.error


def test_blobd_crc_subset_recomputes_only_selected_bodies():
    """--crc-check 8: a wrong CRC in a selected body is refused; outside the subset the body is
    dropped in the kernel and only the trailer's form is checked (a malformed one is refused)."""
    from downloader_amd.bench.infra import Blobd
    from downloader_amd.ops import hashing
    data = os.urandom(256 * 1024)
    good = hashing.crc32c_b64(data)
    bad = hashing.crc32c_b64(data[:-1] + bytes([data[-1] ^ 1]))

    def chunked(crc):
        return (f"{len(data):x}\r\n".encode() + data + b"\r\n0\r\n" +
                f"x-amz-checksum-crc32c:{crc}\r\n\r\n".encode())
    hdr = {"Content-Encoding": "aws-chunked", "x-amz-decoded-content-length": str(len(data)),
           "x-amz-trailer": "x-amz-checksum-crc32c"}
    with Blobd(sink="discard", keep_bytes=0, crc_check=8, crc_salt=12345) as b:
        _req(b.port, "PUT", "/bk")
        keys = [f"k{i}/original/eA==" for i in range(64)]
        sel = [k for k in keys if b.crc_selected(k)]
        unsel = [k for k in keys if not b.crc_selected(k)]
        assert 0 < len(sel) < len(keys) // 2                     # ~1 in 8
        assert _req(b.port, "PUT", "/bk/" + sel[0], chunked(bad), hdr)[0] == 400
        assert _req(b.port, "PUT", "/bk/" + sel[1], chunked(good), hdr)[0] == 200
        assert _req(b.port, "PUT", "/bk/" + unsel[0], chunked(bad), hdr)[0] == 200   # sampled out
        assert _req(b.port, "PUT", "/bk/" + unsel[1], chunked("nope"), hdr)[0] == 400
        st = b.stats()
        assert st["crc_check"] == 8 and st["crc_checked_puts"] == 2
        assert st["crc_unchecked_puts"] == 2 and st["bad_digests"] == 2
        assert st["media_puts"] == 4 and st["media_puts_crc"] == 4


def _bench(extra, env_extra=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error", **(env_extra or {}))
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1",
                           "--warmup", "1", "--jobs-per-step", "6", "--size-mb", "12",
                           "--part-mb", "5", "--threshold-mb", "5", "--procs-per-rank", "1",
                           "--torrent-gb", "0", "--no-compare-unchecked",
                           "--no-compare-reference", "--workers-curve", ""] + extra,
                          env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.slow
def test_bench_fails_on_a_wrong_crc_inside_the_checked_subset():
    """The worker sends one wrong CRC32C trailer (STAGER_FAULT_BAD_CRC) on a part the sink's
    salted subset recomputes: the sink refuses it, the worker's retry stages the job, and the
    bench run fails on the refused body. The same fault on a part outside the subset goes
    through (the price of checking 1 in 8)."""
    from downloader_amd.bench.infra import Blobd
    salt = 987654321
    # job ids of the timed jobs: bench-tuned-m1-r0-j<i>, i = 6..11 (6 warmup jobs first)
    with Blobd(sink="discard", crc_check=8, crc_salt=salt) as b:
        def key(i):
            return f"bench-tuned-m1-r0-j{i}/original/" + base64.b64encode(
                f"r0-j{i}.mkv".encode()).decode()
        cand = [(i, p) for i in range(6, 12) for p in (1, 2, 3)]
        sel = [(i, p) for i, p in cand if b.crc_selected(key(i), p)]
        unsel = [(i, p) for i, p in cand if not b.crc_selected(key(i), p)]
    assert sel and unsel, "salt gives no selected part among the timed ones: pick another"
    common = ["--sink-crc-check", "8", "--sink-crc-salt", str(salt)]
    i, p = sel[0]
    r = _bench(common, {"STAGER_FAULT_BAD_CRC": f"bench-tuned-m1-r0-j{i}/*partNumber={p}&"})
    assert r.returncode != 0
    assert "refused 1 bodies" in r.stderr, r.stderr[-2000:]
    i, p = unsel[0]
    r = _bench(common, {"STAGER_FAULT_BAD_CRC": f"bench-tuned-m1-r0-j{i}/*partNumber={p}&"})
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["integrity"] == "crc32c" and j["bad_digests"] == 0
    assert j["crc_parts"] == j["media_parts"] == 6 * 3 and j["sink_crc_check"] == "1/8"
