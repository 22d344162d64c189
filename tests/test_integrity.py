"""Payload integrity end to end (S3 flexible checksums, CRC32C): a byte flipped between the
worker and S3 is refused with 400 BadDigest and the upload is sent again, on every upload path
- in-memory PUT, disk PUT, disk multipart part, socket relay (aws-chunked trailer), TLS relay,
piece-hashed torrent relay - against both S3 peers (Python FakeS3, native blobd). With
``checksum: off`` the same corruption is stored silently (why the default is on)."""
from __future__ import annotations

import asyncio
import base64
import hashlib
import os
import shutil
import socket
import subprocess
import urllib.request

import pytest

from downloader_amd.s3.client import S3Client, S3Error
from downloader_amd.s3.fake_server import FakeS3, decode_aws_chunked

CREDS = ("minioadmin", "minioadmin")


def _crc_ref(b: bytes) -> int:
    c = 0xFFFFFFFF
    for x in b:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def test_crc32c_matches_reference_and_streams():
    from downloader_amd.ops import native
    n = native()
    assert n.crc32c(b"123456789") == 0xE3069283                  # the CRC-32C check value
    assert n.crc32c_base64(0xE3069283) == base64.b64encode(bytes.fromhex("e3069283")).decode()
    # short inputs (crc32 chains), and >= 1 KiB with odd lengths and misaligned starts (the
    # AVX-512 VPCLMULQDQ folding path where the CPU has it: 256-byte blocks, 16-byte tail)
    for size in (0, 1, 7, 9, 255, 256, 769, 1023, 1024, 1025, 1279, 1281, 4103, 8191, 24577,
                 50_001):
        for off in (0, 3):
            b = os.urandom(size + off)[off:]
            assert n.crc32c(b) == _crc_ref(b), (size, off)
            k = size // 3
            assert n.crc32c(b[k:], n.crc32c(b[:k])) == _crc_ref(b), (size, off)


def test_decode_aws_chunked():
    body = b"5\r\nhello\r\n3;ext=1\r\nabc\r\n0\r\nx-amz-checksum-crc32c:AAAAAA==\r\n\r\n"
    data, tr = decode_aws_chunked(body)
    assert data == b"helloabc" and tr == {"x-amz-checksum-crc32c": "AAAAAA=="}
    assert decode_aws_chunked(b"5\r\nhel") is None


def test_memory_disk_and_multipart_uploads_survive_corruption(run, tmp_path):
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        c = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20)
        await c.ensure_bucket("b")
        s3.corrupt_next = 1
        await c.put_object("b", "mem", b"x" * 1000)
        assert s3.get("b", "mem") == b"x" * 1000
        assert (s3.corrupted, s3.bad_digests) == (1, 1)
        small = tmp_path / "small.bin"
        small.write_bytes(os.urandom(1_000_000))
        s3.corrupt_next = 1
        await c.fput_object("b", "disk", str(small))
        assert s3.get("b", "disk") == small.read_bytes() and s3.bad_digests == 2
        big = tmp_path / "big.bin"
        big.write_bytes(os.urandom(12_000_000))                     # 3 parts
        s3.corrupt_next = 2
        await c.fput_object("b", "mp", str(big))
        assert s3.get("b", "mp") == big.read_bytes() and s3.bad_digests == 4
        assert s3.objects("b")["mp"].etag.endswith("-3")
        await c.close()
        await s3.stop()
    run(go())


def test_multipart_declares_its_checksum_algorithm(run, tmp_path, origin_cls):
    """parts that carry x-amz-checksum-crc32c belong to an upload created with
    x-amz-checksum-algorithm: CRC32C, and CompleteMultipartUpload lists each part's checksum.
    FakeS3 refuses a part checksum the upload did not declare (S3's "Checksum Type mismatch")
    and checks Complete's <ChecksumCRC32C> against the stored parts - for disk uploads,
    relayed parts and resumed relays alike."""
    from downloader_amd.s3.client import PartTag

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(13_000_000)
        origin.blobs["/r.mkv"] = blob
        c = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20,
                     checksum="always")
        await c.ensure_bucket("b")
        big = tmp_path / "big.bin"
        big.write_bytes(blob)
        await c.fput_object("b", "disk", str(big))
        await c.relay_object("b", "relay", origin.url("/r.mkv"), len(blob))
        for k in ("disk", "relay"):
            assert s3.get("b", k) == blob
        assert s3.complete_part_checksums == 6 and s3.checksum_type_mismatches == 0
        # an upload created WITHOUT the algorithm refuses checksummed parts
        uid = await c.create_multipart_upload("b", "legacy")
        with pytest.raises(S3Error) as ei:
            await c.upload_part("b", "legacy", uid, 1, b"q" * 100)
        assert ei.value.code == "InvalidRequest" and s3.checksum_type_mismatches == 1
        # ... and a Complete whose part checksum differs from the stored one is refused
        uid = await c.create_multipart_upload("b", "wrong", checksum=True)
        tag = await c.upload_part("b", "wrong", uid, 1, b"w" * 100)
        assert isinstance(tag, PartTag) and tag.crc32c
        with pytest.raises(S3Error) as ei:
            await c.complete_multipart_upload("b", "wrong", uid,
                                              [(1, PartTag.of(str(tag), "AAAAAA=="))])
        assert ei.value.code == "InvalidPart"
        # list_parts carries the checksums (a resumed relay completes with them)
        parts = await c.list_parts("b", "wrong", uid)
        assert parts[0][1].crc32c == tag.crc32c
        assert await c.complete_multipart_upload("b", "wrong", uid, [(1, parts[0][1])])
        assert s3.get("b", "wrong") == b"w" * 100
        await c.close(); await origin.stop(); await s3.stop()
    run(go())


def test_checksum_off_stores_corruption_silently(run):
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        c = S3Client(ep, *CREDS, checksum="off")
        await c.ensure_bucket("b")
        s3.corrupt_next = 1
        await c.put_object("b", "k", b"y" * 100)
        assert s3.corrupted == 0 and s3.checksummed == 0          # nothing to check against
        await c.close()
        await s3.stop()
    run(go())


def test_bad_digest_is_refused_then_retried_out(run):
    """Persistent corruption: every attempt is refused, the client gives up with BadDigest."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        c = S3Client(ep, *CREDS, retries=2)
        await c.ensure_bucket("b")
        s3.corrupt_next = 10
        with pytest.raises(S3Error) as ei:
            await c.put_object("b", "k", b"z" * 10)
        assert ei.value.code == "BadDigest" and s3.bad_digests == 3
        assert s3.get("b", "k") is None
        await c.close()
        await s3.stop()
    run(go())


@pytest.mark.parametrize("policy,expect_crc", [("auto", False), ("always", True)])
def test_plain_relay_checksum_policy(run, origin_cls, policy, expect_crc):
    """The plain-http splice relay carries a CRC only when asked (``always``: the bytes then
    go through user space, aws-chunked with the CRC32C as trailer); corruption is then caught
    on single PUTs and on parts."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(13_000_000)
        origin.blobs["/r.mkv"] = blob
        c = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20, checksum=policy)
        await c.ensure_bucket("b")
        s3.corrupt_next = 2 if expect_crc else 0
        await c.relay_object("b", "mp", origin.url("/r.mkv"), len(blob))
        assert s3.get("b", "mp") == blob
        assert s3.checksummed == (3 + 2 if expect_crc else 0)      # 3 parts + 2 refused
        assert s3.bad_digests == (2 if expect_crc else 0)
        c.multipart_threshold = 64 << 20
        await c.relay_object("b", "one", origin.url("/r.mkv"), len(blob))
        assert s3.get("b", "one") == blob
        from downloader_amd.ops import native
        ps = native().pipe_stats()      # pipes are leased per transfer, all returned
        assert ps["in_use"] == 0 and ps["idle"] <= 32
        await c.close()
        await origin.stop()
        await s3.stop()
    run(go())


@pytest.mark.skipif(shutil.which("openssl") is None, reason="needs the openssl CLI")
def test_tls_relay_checksummed_by_default(run, tmp_path, origin_cls):
    async def go():
        import ssl
        crt, key = str(tmp_path / "c.pem"), str(tmp_path / "k.pem")
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                        "-out", crt, "-days", "1", "-subj", "/CN=127.0.0.1",
                        "-addext", "subjectAltName=IP:127.0.0.1"], check=True, capture_output=True)
        sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        sctx.load_cert_chain(crt, key)
        s3 = FakeS3(ssl_context=sctx)
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(3_000_000)
        origin.blobs["/t.mkv"] = blob
        c = S3Client(ep, *CREDS, secure=True, ca_file=crt)
        await c.ensure_bucket("b")
        s3.corrupt_next = 1
        await c.relay_object("b", "t", origin.url("/t.mkv"), len(blob))
        assert s3.get("b", "t") == blob and s3.bad_digests == 1
        await c.close()
        await origin.stop()
        await s3.stop()
    run(go())


def test_torrent_stream_relay_checksummed(run, tmp_path, make_cfg, origin_cls):
    """Webseed torrent staged part by part with in-flight SHA-1: the S3 leg carries a CRC32C
    trailer too, so a byte flipped after the piece check is still caught (refused, resent)."""
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.service.worker import Worker
    from downloader_amd.torrent.metainfo import make_torrent

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(7_000_003)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 65536, url_list=[origin.url("/ws/")])
        w = Worker(make_cfg(ep, download={"torrent_enable_dht": False}), broker=MemoryBroker())
        await w.start(health=False)
        s3.corrupt_next = 1
        await w.submit(api.make_download("tc", "http", origin.url("/t/m.torrent")))
        for _ in range(1500):
            if w.results:
                break
            await asyncio.sleep(0.02)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert r.stats["torrent"]["staging"] == "stream"
        assert s3.get("triton-staging", keys.object_key("tc", "m.mkv")) == data
        assert s3.bad_digests == 1
        await w.stop()
        await origin.stop()
        await s3.stop()
    run(go())


# ---------------------------------------------------------------- native S3 sink (blobd)
def _put(port, path, body, headers):
    s = socket.create_connection(("127.0.0.1", port))
    head = f"PUT {path} HTTP/1.1\r\nHost: x\r\nContent-Length: {len(body)}\r\n"
    head += "".join(f"{k}: {v}\r\n" for k, v in headers.items()) + "Connection: close\r\n\r\n"
    s.sendall(head.encode() + body)
    resp = b""
    while True:
        d = s.recv(65536)
        if not d:
            break
        resp += d
    s.close()
    return int(resp.split(b" ", 2)[1]), resp


def test_blobd_verifies_payload_checksums():
    from downloader_amd.bench.infra import Blobd
    from downloader_amd.ops import hashing
    with Blobd() as b:
        port = b.port
        assert _put(port, "/bk", b"", {})[0] == 200
        data = os.urandom(300_000)
        good = hashing.crc32c_b64(data)
        bad = hashing.crc32c_b64(data[:-1] + b"\0")
        assert _put(port, "/bk/a", data, {"x-amz-checksum-crc32c": good})[0] == 200
        st, resp = _put(port, "/bk/b", data, {"x-amz-checksum-crc32c": bad})
        assert st == 400 and b"BadDigest" in resp
        md5 = base64.b64encode(hashlib.md5(data).digest()).decode()
        assert _put(port, "/bk/c", data, {"Content-MD5": md5})[0] == 200
        assert _put(port, "/bk/d", data + b"!", {"Content-MD5": md5})[0] == 400

        def chunked(crc):
            return (f"{len(data):x}\r\n".encode() + data + b"\r\n0\r\n" +
                    f"x-amz-checksum-crc32c:{crc}\r\n\r\n".encode())
        hdr = {"Content-Encoding": "aws-chunked", "x-amz-decoded-content-length": str(len(data)),
               "x-amz-trailer": "x-amz-checksum-crc32c"}
        assert _put(port, "/bk/e", chunked(good), hdr)[0] == 200
        assert _put(port, "/bk/f", chunked(bad), hdr)[0] == 400
        st = b.stats()
        assert st["bad_digests"] == 3 and st["checksummed_puts"] == 6
        with urllib.request.urlopen(f"http://{b.endpoint}/bk/e") as r:
            assert r.read() == data                                  # decoded, not the framing


def test_worker_with_corrupting_blobd_sink(run, tmp_path):
    """Worker -> native sink that corrupts 30 % of the checksummed bodies on arrival, with
    the verify sink on: every job is staged, the sink refused the corrupted bodies, and every
    stored object matches what the origin generated."""
    from downloader_amd.bench.infra import Blobd
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api
    from downloader_amd.service.worker import Worker
    from downloader_amd.utils.config import load_config

    async def go(b):
        cfg = load_config(overrides={
            "instance": {"download_path": str(tmp_path / "dl")},
            "s3": {"endpoint": b.endpoint, "part_size": 5 << 20, "multipart_threshold": 6 << 20,
                   "checksum": "always", "retries": 8},
            "broker": {"backend": "memory"}, "health": {"enabled": False},
            "download": {"gpu_prewarm": False}}, env={})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        n = 6
        for i in range(n):
            await w.submit(api.make_download(f"c{i}", "http",
                                             b.media_url(f"c{i}.mkv", 11_000_000 + i, 50 + i)))
        for _ in range(3000):
            if len(w.results) >= n:
                break
            await asyncio.sleep(0.02)
        assert [r.outcome for r in w.results] == ["staged"] * n
        await w.stop()
    with Blobd(sink="verify", s3_corrupt_rate=0.3) as b:
        run(go(b))
        st = b.stats()
        assert st["verify_objects"] == 6 and st["verify_mismatches"] == 0
        assert st["bad_digests"] == st["corrupted"] > 0


# ---------------------------------------------------------------- origin version pinning
def _swap_after_first_range(origin, path, new):
    seen = []

    def hook(method, p):
        if p == path and method == "GET":
            seen.append(1)
            if len(seen) == 2:              # the second part's GET sees the new version
                origin.blobs[path] = new
    origin.hooks.append(hook)


@pytest.mark.parametrize("staging,ignore_if_match", [("stream", False), ("stream", True),
                                                     ("disk", False), ("disk", True)])
def test_origin_swap_mid_job_stages_one_coherent_version(run, make_cfg, origin_cls, staging,
                                                         ignore_if_match):
    """The origin's object changes after the first part was fetched: every split GET is
    pinned to the probed version (If-Match; If-Range for servers that ignore If-Match), the
    change is noticed, and the job restarts from the new version - the staged object is
    exactly v2, never v1's first part glued to v2's rest."""
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.service.worker import Worker

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        origin.ignore_if_match = ignore_if_match
        v1, v2 = os.urandom(13_000_000), os.urandom(13_000_000)
        origin.blobs["/v.mkv"] = v1
        _swap_after_first_range(origin, "/v.mkv", v2)
        cfg = make_cfg(ep, s3={"endpoint": ep, "part_size": 5 << 20, "multipart_threshold": 6 << 20,
                               "max_inflight_parts": 1},
                       download={"stream_http": staging == "stream", "http_streams": 3,
                                 "http_min_split": 4 << 20})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        await w.submit(api.make_download("sw", "http", origin.url("/v.mkv")))
        for _ in range(1500):
            if w.results:
                break
            await asyncio.sleep(0.02)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert s3.get("triton-staging", keys.object_key("sw", "v.mkv")) == v2
        gets = [h for m, p, h in origin.requests if p == "/v.mkv" and m == "GET"]
        assert len(gets) > 3                 # the restart fetched v2 again
        await w.stop()
        await origin.stop()
        await s3.stop()
    run(go())


def test_bucket_relay_parts_pinned_to_listed_etag(run, origin_cls):
    """S3 -> S3 relay of a listed object: parts carry If-Match of the listed ETag, so an
    object overwritten between the listing and the last part fails instead of mixing."""
    async def go():
        from downloader_amd.net.http import SourceChanged
        s3 = FakeS3()
        ep = await s3.start()
        c = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20,
                     max_inflight_parts=1)
        await c.ensure_bucket("src")
        await c.ensure_bucket("dst")
        await c.put_object("src", "o", os.urandom(11_000_000))
        (info,) = await c.list_objects("src")
        url = c.presign("GET", "src", "o")
        await c.put_object("src", "o", os.urandom(11_000_000))     # overwritten
        with pytest.raises(SourceChanged):
            await c.relay_object("dst", "o", url, info.size, validator=f'"{info.etag}"')
        assert s3.get("dst", "o") is None and not s3.uploads.get("dst")
        await c.close()
        await s3.stop()
    run(go())


@pytest.mark.parametrize("sink", ["sample", "verify"])
def test_blobd_sink_detects_wrong_torn_and_reordered_objects(sink):
    """The bench's S3 sink compares each staged object with what its origin generated: an
    exact copy passes; other bytes, a truncated object and swapped multipart parts are all
    counted as mismatches (so the headline cannot pass while staging wrong bytes)."""
    from downloader_amd.bench.infra import Blobd
    n = 3 * 1_048_576 + 5
    key = "/bk/job/original/" + base64.b64encode(b"x.mkv").decode()
    with Blobd(sink=sink) as b:
        port = b.port
        assert _put(port, "/bk", b"", {})[0] == 200
        with urllib.request.urlopen(b.media_url("x.mkv", n, 7)) as r:
            good = r.read()

        def mp(parts):
            s = socket.create_connection(("127.0.0.1", port))
            s.sendall(f"POST {key}?uploads HTTP/1.1\r\nHost: x\r\nContent-Length: 0\r\n"
                      "Connection: close\r\n\r\n".encode())
            resp = b""
            while True:
                d = s.recv(65536)
                if not d:
                    break
                resp += d
            uid = resp.split(b"<UploadId>")[1].split(b"</UploadId>")[0].decode()
            for num, body in parts:
                assert _put(port, f"{key}?partNumber={num}&uploadId={uid}", body, {})[0] == 200
            s = socket.create_connection(("127.0.0.1", port))
            s.sendall(f"POST {key}?uploadId={uid} HTTP/1.1\r\nHost: x\r\nContent-Length: 0\r\n"
                      "Connection: close\r\n\r\n".encode())
            while s.recv(65536):
                pass
        assert _put(port, key, good, {})[0] == 200
        assert b.stats()["verify_mismatches"] == 0
        bad = bytearray(good)
        bad[2_000_000] ^= 0xFF          # a byte outside every sampled window still differs in
        bad[0] ^= 0xFF                  # ... and one inside the first window
        assert _put(port, key, bytes(bad), {})[0] == 200
        assert _put(port, key, good[:-1], {})[0] == 200                    # truncated
        h = 1 << 21
        mp([(1, good[:h]), (2, good[h:])])                                   # coherent
        mp([(1, good[h:2 * h]), (2, good[:h] + good[2 * h:])])              # parts swapped
        st = b.stats()
        assert st["verify_objects"] == 5 and st["verify_mismatches"] == 3, st


@pytest.mark.parametrize("dup", ["peek", "tee"])
@pytest.mark.parametrize("main_kb,tee_kb", [(64, 64), (1024, 64), (64, 1024)])
def test_teed_relays_with_small_and_uneven_pipes(run, origin_cls, main_kb, tee_kb, dup):
    """The CRC'd and piece-hashed relays splice through a pipe and copy the same bytes out -
    peeked from the socket (default) or read from a tee()d duplicate: with small or uneven
    pipes a chunk is copied and sent in several rounds - the CRC the sink checks and the piece
    digests must still cover exactly the bytes sent."""
    from downloader_amd.ops import native

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(5_000_003)
        origin.blobs["/u.bin"] = blob
        c = S3Client(ep, *CREDS, checksum="always", part_size=5 << 20,
                     multipart_threshold=64 << 20)
        await c.ensure_bucket("b")
        s3.corrupt_next = 1                       # the first PUT is refused: CRC must differ
        await c.relay_object("b", "plain", origin.url("/u.bin"), len(blob))
        assert s3.get("b", "plain") == blob and s3.bad_digests == 1
        plen = 1 << 18
        full = ((len(blob) - 777) // plen) * plen
        _, h = await c.relay_hashed("b", "h", origin.url("/u.bin"), 0, len(blob), True,
                                    (777, full, plen))
        assert h["digests"] == b"".join(hashlib.sha1(blob[777 + i:777 + i + plen]).digest()
                                        for i in range(0, full, plen))
        assert h["head"] == blob[:777] and h["tail"] == blob[777 + full:]
        assert s3.get("b", "h") == blob
        await c.close(); await origin.stop(); await s3.stop()

    n = native()
    n.set_pipe_sizes(main_kb << 10, tee_kb << 10)
    n.set_relay_dup(dup)
    try:
        run(go())
    finally:
        n.set_relay_dup("peek")
        n.set_pipe_sizes(1 << 20, 256 << 10)
