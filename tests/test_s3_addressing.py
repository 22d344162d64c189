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
