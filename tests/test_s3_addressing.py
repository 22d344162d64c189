"""S3 addressing (minio-js 7 semantics): virtual-hosted style ``<bucket>.<endpoint>/<key>`` for
AWS endpoints, path style ``<endpoint>/<bucket>/<key>`` elsewhere; both signed correctly."""
from __future__ import annotations

import os
import socket

import pytest

from downloader_amd.s3.client import S3Client
from downloader_amd.s3.fake_server import FakeS3

CREDS = ("minioadmin", "minioadmin")


@pytest.mark.parametrize("endpoint,secure,bucket,virtual", [
    ("s3.amazonaws.com", True, "examplebucket", True),
    ("s3.eu-west-1.amazonaws.com", True, "triton-staging", True),
    ("s3.amazonaws.com", True, "my.dotted.bucket", False),    # dots break the *.s3 cert
    ("s3.amazonaws.com", False, "my.dotted.bucket", True),
    ("s3.amazonaws.com", True, "Bad_Name", False),             # not DNS-compatible
    ("minio.internal:9000", False, "triton-staging", False),   # non-AWS: path style
    ("127.0.0.1:9000", False, "b", False),
])
def test_auto_addressing(endpoint, secure, bucket, virtual):
    c = S3Client(endpoint, *CREDS, secure=secure)
    assert c.virtual_host(bucket) is virtual
    host, path = c._address(bucket, "k/x.mkv")
    if virtual:
        assert (host, path) == (f"{bucket}.{endpoint}", "/k/x.mkv")
    else:
        assert (host, path) == (endpoint, f"/{bucket}/k/x.mkv")
    assert S3Client(endpoint, *CREDS, addressing="path").virtual_host(bucket) is False
    with pytest.raises(ValueError):
        S3Client(endpoint, *CREDS, addressing="dns")


class _StaticResolver:
    """aiohttp resolver mapping every name to 127.0.0.1 (no DNS for <bucket>.s3.test here)."""

    async def resolve(self, host, port=0, family=socket.AF_INET):
        return [{"hostname": host, "host": "127.0.0.1", "port": port, "family": socket.AF_INET,
                 "proto": 0, "flags": socket.AI_NUMERICHOST}]

    async def close(self):
        pass


def test_virtual_hosted_round_trip(run, tmp_path):
    """Forced virtual-hosted style against FakeS3: bucket ops, PUT/GET, multipart, list -
    every request signed over the <bucket>.<endpoint> host and the bucket-less path."""
    import aiohttp

    from downloader_amd.net.http import AiohttpTransport, TransportSet

    async def go():
        s3 = FakeS3(virtual_host_suffix="s3.test")
        await s3.start()
        fb = AiohttpTransport()
        fb._session = aiohttp.ClientSession(
            connector=aiohttp.TCPConnector(resolver=_StaticResolver()), auto_decompress=False)
        c = S3Client(f"s3.test:{s3.port}", *CREDS, transports=TransportSet(None, fb),
                     addressing="virtual", part_size=5 << 20, multipart_threshold=6 << 20)
        await c.ensure_bucket("media")
        assert "media" in s3.buckets
        await c.put_object("media", "a/b.txt", b"hello")
        assert await c.get_object("media", "a/b.txt") == b"hello"
        blob = os.urandom((11 << 20) + 5)
        p = tmp_path / "big.bin"
        p.write_bytes(blob)
        await c.fput_object("media", "big.bin", str(p))
        assert s3.get("media", "big.bin") == blob
        names = sorted(o.name for o in await c.list_objects("media", "", recursive=True))
        assert names == ["a/b.txt", "big.bin"]
        assert all(path.startswith("/media") for _, path in s3.requests)
        await fb.close()
        await s3.stop()
    run(go())


def test_bucket_region_learnt_from_refusal(run, tmp_path, origin_cls):
    """A bucket in another region: the first request is refused (400 AuthorizationHeader-
    Malformed + x-amz-bucket-region), the client re-signs for that region at once and keeps
    using it - for plain requests, multipart uploads, HEADs and the socket relay."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        s3.buckets["eu"] = {}
        s3.bucket_regions["eu"] = "eu-west-1"
        origin = await origin_cls().start()
        blob = os.urandom((11 << 20) + 3)
        origin.blobs["/m.mkv"] = blob
        c = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20, retries=0)
        assert await c.bucket_exists("eu")                      # HEAD: header-only hint
        assert c.region_of("eu") == "eu-west-1" and c.region_of("other") == "us-east-1"
        c2 = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20, retries=0)
        await c2.put_object("eu", "small", b"x")                # body hint (<Region>)
        p = tmp_path / "f.bin"
        p.write_bytes(blob)
        await c2.fput_object("eu", "big", str(p))
        assert s3.get("eu", "big") == blob
        c3 = S3Client(ep, *CREDS, part_size=5 << 20, multipart_threshold=6 << 20, retries=0)
        assert c3.can_relay(origin.url("/m.mkv"))
        await c3.relay_object("eu", "relayed", origin.url("/m.mkv"), len(blob))
        assert s3.get("eu", "relayed") == blob and c3.region_of("eu") == "eu-west-1"
        s3.bucket_regions["eu"] = "ap-south-1"                  # moved again: learnt again
        assert await c3.get_object("eu", "small") == b"x"
        for x in (c, c2, c3):
            await x.close()
        await origin.stop()
        await s3.stop()
    run(go())


def test_session_token_signed(run, make_cfg):
    """Temporary credentials: s3.session_token travels as a signed x-amz-security-token."""
    from downloader_amd.s3.client import S3Error

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        s3.session_tokens["minioadmin"] = "tok/123=="
        c = S3Client.from_config(make_cfg(ep, s3={"session_token": "tok/123=="}).s3)
        await c.ensure_bucket("b")
        await c.put_object("b", "k", b"v")
        assert await c.get_object("b", "k") == b"v"
        await c.close()
        bad = S3Client(ep, *CREDS, retries=0)
        with pytest.raises(S3Error) as ei:
            await bad.get_object("b", "k")
        assert ei.value.code == "InvalidToken"
        await bad.close()
        await s3.stop()
    run(go())
