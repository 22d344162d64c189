"""TLS end to end: S3 with ``secure: true``, bucket:// sources (always TLS in the reference,
lib/download.js:210 ``useSSL: true``) and https:// origins, against in-process servers with a
throwaway self-signed certificate; trust comes from ``tls.ca_file``."""
from __future__ import annotations

import asyncio
import os
import shutil
import ssl
import subprocess

import pytest

from downloader_amd.broker.memory import MemoryBroker
from downloader_amd.models import api, keys
from downloader_amd.net.http import TransportError
from downloader_amd.s3.client import S3Client, S3Error
from downloader_amd.s3.fake_server import FakeS3
from downloader_amd.service.worker import Worker

CREDS = ("minioadmin", "minioadmin")
pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="needs the openssl CLI")


@pytest.fixture(scope="module")
def cert(tmp_path_factory):
    d = tmp_path_factory.mktemp("tls")
    crt, key = str(d / "c.pem"), str(d / "k.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", crt, "-days", "1", "-subj", "/CN=127.0.0.1",
                    "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, capture_output=True, timeout=60)
    return crt, key


def _server_ctx(cert):
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(*cert)
    return ctx


async def _wait(w, n=1, timeout=30.0):
    t = 0.0
    while len(w.results) < n and t < timeout:
        await asyncio.sleep(0.02)
        t += 0.02
    assert len(w.results) >= n, w.results


def test_s3_client_over_tls(run, cert, tmp_path):
    async def go():
        s3 = FakeS3(ssl_context=_server_ctx(cert))
        ep = await s3.start()
        c = S3Client(ep, *CREDS, secure=True, ca_file=cert[0], part_size=5 << 20,
                     multipart_threshold=6 << 20)
        assert c.base.startswith("https://")
        await c.ensure_bucket("b")
        await c.put_object("b", "small", b"hello")
        assert await c.get_object("b", "small") == b"hello"
        blob = os.urandom((12 << 20) + 7)                      # multipart: 3 parts
        src = tmp_path / "big.bin"
        src.write_bytes(blob)
        await c.fput_object("b", "big", str(src))
        assert s3.get("b", "big") == blob
        dst = tmp_path / "back.bin"
        await c.fget_object("b", "big", str(dst), streams=2)
        assert dst.read_bytes() == blob
        await c.close()
        # the system store alone does not trust the throwaway CA; verify=False does
        untrusted = S3Client(ep, *CREDS, secure=True, retries=0)
        with pytest.raises((TransportError, S3Error)):
            await untrusted.get_object("b", "small")
        await untrusted.close()
        lax = S3Client(ep, *CREDS, secure=True, ssl_verify=False)
        assert await lax.get_object("b", "small") == b"hello"
        await lax.close()
        await s3.stop()
    run(go())


def test_worker_https_origin_tls_s3_and_bucket_source(run, make_cfg, origin_cls, cert):
    """Both data planes over TLS in one worker: an https:// origin staged into a TLS S3, and a
    bucket:// source with the reference's always-on TLS (download.bucket_secure default)."""
    async def go():
        s3 = FakeS3(ssl_context=_server_ctx(cert))
        ep = await s3.start()
        origin = await origin_cls(ssl_context=_server_ctx(cert)).start()
        blob = os.urandom((7 << 20) + 11)
        origin.blobs["/Movie.mkv"] = blob
        cfg = make_cfg(ep, s3={"secure": True}, tls={"ca_file": cert[0]})
        assert cfg.download.bucket_secure is True
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        url = origin.url("/Movie.mkv")
        assert url.startswith("https://")
        await w.submit(api.make_download("t1", "http", url, "MOVIE"))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("t1", "Movie.mkv")) == blob
        plain = await origin_cls().start()         # http origin -> TLS S3: no socket relay
        plain.blobs["/Film.mkv"] = blob[::-1]
        await w.submit(api.make_download("t0", "http", plain.url("/Film.mkv"), "MOVIE"))
        await _wait(w, 2)
        assert w.results[1].outcome == "staged", w.results[1]
        assert s3.get("triton-staging", keys.object_key("t0", "Film.mkv")) == blob[::-1]
        await plain.stop()
        s3.buckets["src"] = {}
        s3.put("src", "show/S1/ep1.mkv", b"one" * 1000)
        s3.put("src", "show/S1/ep2.mkv", b"two" * 1000)
        await w.submit(api.make_download(
            "t2", "bucket", f"bucket://{ep},src,minioadmin,minioadmin,show", "TV"))
        await _wait(w, 3)
        assert w.results[2].outcome == "staged", w.results[2]
        assert s3.get("triton-staging", keys.object_key("t2", "ep2.mkv")) == b"two" * 1000
        await w.stop()
        await origin.stop()
        await s3.stop()
    run(go())


def test_worker_rejects_untrusted_origin(run, make_cfg, origin_cls, cert):
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls(ssl_context=_server_ctx(cert)).start()
        origin.blobs["/x.mkv"] = b"x" * 1000
        w = Worker(make_cfg(ep, broker={"max_retries": 0}), broker=MemoryBroker())
        await w.start(health=False)
        await w.submit(api.make_download("t3", "http", origin.url("/x.mkv")))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "dead" and "certificate" in r.error.lower(), r
        assert not s3.buckets.get("triton-staging")
        await w.stop()
        await origin.stop()
        await s3.stop()
    run(go())
