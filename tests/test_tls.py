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


@pytest.mark.parametrize("native_tls", [True, False])
def test_s3_client_over_tls(run, cert, tmp_path, native_tls):
    """Same S3 traffic through the native OpenSSL transport (pread + SSL_write for file
    bodies, SSL_read + pwrite into sinks) and through aiohttp."""
    async def go():
        s3 = FakeS3(ssl_context=_server_ctx(cert))
        ep = await s3.start()
        c = S3Client(ep, *CREDS, secure=True, ca_file=cert[0], part_size=5 << 20,
                     multipart_threshold=6 << 20, native_tls=native_tls)
        assert c.base.startswith("https://")
        used = type(c.t.for_url(c.base)).__name__
        assert used == ("NativeTransport" if native_tls else "AiohttpTransport")
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
        untrusted = S3Client(ep, *CREDS, secure=True, retries=0, native_tls=native_tls)
        with pytest.raises((TransportError, S3Error)) as ei:
            await untrusted.get_object("b", "small")
        assert "certificate" in str(ei.value).lower()
        await untrusted.close()
        lax = S3Client(ep, *CREDS, secure=True, ssl_verify=False, native_tls=native_tls)
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
        assert w.results[0].stats.get("streamed")     # https -> https socket relay, no disk
        plain = await origin_cls().start()         # http origin -> TLS S3
        plain.blobs["/Film.mkv"] = blob[::-1]
        await w.submit(api.make_download("t0", "http", plain.url("/Film.mkv"), "MOVIE"))
        await _wait(w, 2)
        assert w.results[1].outcome == "staged", w.results[1]
        assert s3.get("triton-staging", keys.object_key("t0", "Film.mkv")) == blob[::-1]
        assert w.results[1].stats.get("streamed")     # http -> https relay
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


def test_stream_torrent_over_tls(run, tmp_path, make_cfg, origin_cls, cert):
    """Webseed-only torrent on an https webseed, staged into a TLS S3 by the hashed relay
    (SSL_read -> buffer -> SSL_write, pieces SHA-1'd in flight); a corrupt piece is caught
    and refetched, nothing touches the disk."""
    from downloader_amd.torrent.metainfo import make_torrent, parse_torrent

    async def go():
        s3 = FakeS3(ssl_context=_server_ctx(cert))
        ep = await s3.start()
        origin = await origin_cls(ssl_context=_server_ctx(cert)).start()
        src = tmp_path / "src" / "Show" / "Season 1"
        src.mkdir(parents=True)
        data = {"e1.mkv": os.urandom(6_500_001), "e2.mkv": os.urandom(300_007)}
        for n, d in data.items():
            (src / n).write_bytes(d)
            origin.blobs["/ws/Show/Season 1/" + n] = d
        raw = make_torrent(str(tmp_path / "src" / "Show"), 131072, url_list=[origin.url("/ws/")])
        origin.blobs["/t/show.torrent"] = raw
        origin.corrupt["/ws/Show/Season 1/e1.mkv"] = [3_000_000, 1]
        assert parse_torrent(raw).url_list[0].startswith("https://")
        w = Worker(make_cfg(ep, s3={"secure": True}, tls={"ca_file": cert[0]},
                            download={"torrent_enable_dht": False}), broker=MemoryBroker())
        await w.start(health=False)
        await w.submit(api.make_download("ts", "http", origin.url("/t/show.torrent"), "TV"))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert r.stats["torrent"]["staging"] == "stream" and r.stats["torrent"]["hash_fails"] >= 1
        for n, d in data.items():
            assert s3.get("triton-staging", keys.object_key("ts", n)) == d
        for dp, _, fns in os.walk(tmp_path / "dl"):
            assert not [f for f in fns if f.endswith(".mkv")], (dp, fns)
        await w.stop()
        await origin.stop()
        await s3.stop()
    run(go())


@pytest.mark.parametrize("native_tls", [True, False])
def test_tls_host_name_checked(run, tmp_path, native_tls):
    """DNS names: SNI is sent and the certificate must name the host (SSL_set1_host), like
    Node's checkServerIdentity; a certificate for another name is refused."""
    def mk(name):
        d = tmp_path / name
        d.mkdir()
        crt, key = str(d / "c.pem"), str(d / "k.pem")
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout",
                        key, "-out", crt, "-days", "1", "-subj", f"/CN={name}",
                        "-addext", f"subjectAltName=DNS:{name}"],
                       check=True, capture_output=True, timeout=60)
        return crt, key

    async def go():
        for name, ok in (("localhost", True), ("other.example", False)):
            cert = mk(name)
            s3 = FakeS3(ssl_context=_server_ctx(cert))
            await s3.start()
            c = S3Client(f"localhost:{s3.port}", *CREDS, secure=True, ca_file=cert[0],
                         retries=0, native_tls=native_tls)
            if ok:
                await c.ensure_bucket("b")
                await c.put_object("b", "k", b"v")
                assert await c.get_object("b", "k") == b"v"
            else:
                with pytest.raises((TransportError, S3Error)) as ei:
                    await c.get_object("b", "k")
                msg = str(ei.value).lower()
                assert "certificate" in msg or "hostname" in msg, msg
            await c.close()
            await s3.stop()
    run(go())


def test_https_source_through_connect_proxy(run, make_cfg, origin_cls, cert):
    """https sources behind download.http_proxy: a CONNECT tunnel on the native transport,
    TLS inside it (stream relay and disk path); S3 traffic is not proxied."""
    from test_worker import _ForwardProxy

    async def go():
        proxy = await _ForwardProxy().start()
        purl = f"http://user:pw@127.0.0.1:{proxy.port}"
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls(ssl_context=_server_ctx(cert)).start()
        big = os.urandom((13 << 20) + 1)
        origin.blobs["/p/big.mkv"] = big
        for job, stream in (("cp1", True), ("cp2", False)):
            cfg = make_cfg(ep, tls={"ca_file": cert[0]},
                           download={"http_proxy": purl, "stream_http": stream})
            w = Worker(cfg, broker=MemoryBroker())
            await w.start(health=False)
            assert type(w.transports.for_url(origin.url("/"), True)).__name__ == "NativeTransport"
            await w.submit(api.make_download(job, "http", origin.url("/p/big.mkv")))
            await _wait(w)
            r = w.results[0]
            assert r.outcome == "staged", r
            assert bool(r.stats.get("streamed")) == stream
            assert s3.get("triton-staging", keys.object_key(job, "big.mkv")) == big
            await w.stop()
        lines = [ln for ln, _ in proxy.seen]
        assert lines and all(ln == f"CONNECT 127.0.0.1:{origin.port} HTTP/1.1" for ln in lines)
        assert {a for _, a in proxy.seen} == {"Basic dXNlcjpwdw=="}
        await proxy.stop()
        await origin.stop()
        await s3.stop()
    run(go())


def test_connect_refused_by_proxy(run):
    """A proxy that refuses the tunnel (407) fails the request with the proxy's answer."""
    from downloader_amd.net.http import NativeTransport
    from downloader_amd.net.proxy import Proxy

    async def go():
        async def deny(r, w):
            await r.readuntil(b"\r\n\r\n")
            w.write(b"HTTP/1.1 407 Proxy Authentication Required\r\nContent-Length: 0\r\n\r\n")
            await w.drain()
            w.close()
        srv = await asyncio.start_server(deny, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        t = NativeTransport(4)
        with pytest.raises(TransportError) as ei:
            await t.request("GET", "https://example.invalid/x",
                            proxy=Proxy(f"http://127.0.0.1:{port}", "127.0.0.1", port))
        assert "407" in str(ei.value) and "CONNECT example.invalid:443" in str(ei.value)
        await t.close()
        srv.close()
        await srv.wait_closed()
    run(go())


def test_tls_relay_split_into_parallel_parts(run, cert, origin_cls):
    """Over TLS an object under the multipart threshold but above 6 MiB is relayed as parallel
    parts (one thread's AES-GCM bounds a single relay); plain http keeps one PUT."""
    async def go():
        s3 = FakeS3(ssl_context=_server_ctx(cert))
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(8_000_000)
        origin.blobs["/o.mkv"] = blob
        c = S3Client(ep, *CREDS, secure=True, ca_file=cert[0], max_inflight_parts=4)
        await c.ensure_bucket("b")
        await c.relay_object("b", "split", origin.url("/o.mkv"), len(blob))
        assert s3.get("b", "split") == blob
        assert s3.objects("b")["split"].etag.endswith("-2")        # 5 MiB + the rest
        c.split_tls_relays = False
        await c.relay_object("b", "one", origin.url("/o.mkv"), len(blob))
        assert "-" not in s3.objects("b")["one"].etag
        await c.relay_object("b", "small", origin.url("/o.mkv"), len(blob), ranges=False)
        await c.close()
        await origin.stop()
        await s3.stop()
    run(go())
