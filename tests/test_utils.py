"""Config (triton-core/config), dynamics, pino-style logging, tracing, metrics."""
from __future__ import annotations

import asyncio
import io
import json
import os

import pytest

from downloader_amd.utils.config import load_config
from downloader_amd.utils.dynamics import dyn
from downloader_amd.utils.log import Logger, ListSink, Sink
from downloader_amd.utils.metrics import Metrics
from downloader_amd.utils.trace import Tracer, parse_traceparent

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defaults_pin_reference_constants():
    c = load_config(env={})
    assert c.download.torrent_metadata_timeout_s == 240        # lib/download.js:21
    assert c.download.torrent_stall_timeout_s == 240
    assert c.download.progress_interval_s == 30                # lib/download.js:88
    assert c.s3.bucket == "triton-staging"                     # lib/upload.js:29
    assert c.process.media_exts == [".mp4", ".mkv", ".mov", ".webm"]   # lib/process.js:15-20
    assert c.broker.download_queue == "v1.download" and c.broker.convert_queue == "v1.convert"
    assert c.health.port == 3401                               # lib/main.js:194
    assert c.stages == ["download", "process", "upload"]       # lib/main.js:28-32


def test_env_overrides_and_reference_env_flags():
    env = {"STAGER_S3__ENDPOINT": "s3:9", "STAGER_CONCURRENCY": "7", "PORT": "4000",
           "ALLOW_FILE_URLS": "true", "STAGER_DOWNLOAD__HTTP_STREAMS": "2"}
    c = load_config(env=env)
    assert c.s3.endpoint == "s3:9" and c.concurrency == 7 and c.broker.prefetch == 7
    assert c.health.port == 4000 and c.download.allow_file_urls is True
    assert c.download.http_streams == 2
    assert load_config(env={"ALLOW_FILE_URLS": "1"}).download.allow_file_urls is False


def test_reference_mode_is_serial():
    c = load_config(env={}, overrides={"mode": "reference"})
    assert (c.concurrency, c.broker.prefetch, c.s3.max_inflight_parts, c.s3.concurrent_files,
            c.download.http_streams) == (1, 1, 1, 1, 1)
    assert not c.download.stream_http and not c.download.eager_upload


def test_yaml_file_and_converter_alias(tmp_path):
    d = tmp_path / "config"
    d.mkdir()
    (d / "converter.yaml").write_text("instance:\n  download_path: /data/dl\n")
    from downloader_amd.utils import config as cfgmod
    p = cfgmod.find_config_file("downloader", [d])
    assert p is not None and p.name == "converter.yaml"        # index.js:18 legacy name
    c = load_config(path=str(p), env={})
    assert str(c.resolved_download_root()) == "/data/dl"
    ex = load_config(path=os.path.join(REPO, "config", "downloader.example.yaml"), env={})
    assert ex.s3.bucket == "triton-staging"


def test_relative_download_path_resolves_against_project_root():
    c = load_config(env={}, overrides={"instance": {"download_path": "dl"}})
    assert str(c.resolved_download_root()) == os.path.join(REPO, "dl")


def test_dynamics_lookup_order():
    assert dyn("rabbitmq", {"RABBITMQ_URL": "amqp://x"}) == "amqp://x"
    assert dyn("rabbitmq", {"RABBITMQ_SERVICE_HOST": "10.0.0.1",
                            "RABBITMQ_SERVICE_PORT": "5673"}) == "amqp://guest:guest@10.0.0.1:5673/"
    assert dyn("rabbitmq", {}).startswith("amqp://")


def test_pino_line_format_and_child_bindings():
    buf = io.StringIO()
    lg = Logger("main.js", sink=Sink(buf), level=20)
    lg.child(jobId="j", fileId="f").info("hello", "world", extra=1)
    rec = json.loads(buf.getvalue())
    assert rec["level"] == 30 and rec["name"] == "main.js" and rec["msg"] == "hello world"
    assert rec["jobId"] == "j" and rec["fileId"] == "f" and rec["extra"] == 1
    assert {"time", "pid", "hostname"} <= set(rec)
    sink = ListSink()
    Logger("x", sink=sink, level=40).info("dropped")
    assert sink.records == []


def test_trace_spans_nest_and_propagate():
    t = Tracer("downloader", enabled=False)
    t.keep = True
    with t.span("job") as job:
        with t.span("stage.download"):
            pass
        tp = job.traceparent()
    assert [s.name for s in t.finished] == ["stage.download", "job"]
    assert t.finished[0].parent_id == t.finished[1].span_id
    trace_id, span_id = parse_traceparent(tp)
    with t.span("convert", traceparent=tp) as c:
        pass
    assert c.trace_id == trace_id and c.parent_id == span_id
    assert parse_traceparent("garbage") is None


def test_trace_export_off_the_calling_thread(tmp_path, monkeypatch):
    """Spans are serialised and written by the exporter thread through one open file: the
    thread that finishes a span (the event loop) neither opens the trace file nor
    json-encodes; flush() waits for the queue, close() drains it."""
    import builtins
    import threading

    import downloader_amd.utils.trace as T
    path = str(tmp_path / "spans.jsonl")
    caller = threading.current_thread()
    opens, dumps = [], []
    real_open, real_dumps = builtins.open, T.json.dumps

    def spy_open(*a, **kw):
        opens.append(threading.current_thread() is caller)
        return real_open(*a, **kw)

    def spy_dumps(*a, **kw):
        dumps.append(threading.current_thread() is caller)
        return real_dumps(*a, **kw)
    monkeypatch.setattr(builtins, "open", spy_open)
    monkeypatch.setattr(T.json, "dumps", spy_dumps)
    t = Tracer("downloader", enabled=True, path=path)
    for i in range(500):
        with t.span("job", n=i):
            with t.span("stage.upload"):
                pass
    assert t.flush(10)
    t.close()
    monkeypatch.setattr(builtins, "open", real_open)
    lines = real_open(path).read().splitlines()
    assert len(lines) == 1000 and not any(opens) and not any(dumps) and opens
    assert [json.loads(x)["name"] for x in lines[:2]] == ["stage.upload", "job"]


def test_metrics_registry_exposition():
    m = Metrics()
    m.bytes_downloaded.labels("http").inc(10)
    with m.time_stage("download"):
        pass
    text = m.exposition().decode()
    assert 'downloader_bytes_downloaded_total{proto="http"} 10.0' in text
    assert "downloader_stage_duration_seconds_count" in text
    assert m.sample("downloader_bytes_downloaded_total", proto="http") == 10


def test_effective_cpus_respects_cgroup_quota(tmp_path, monkeypatch):
    from downloader_amd.utils import cpus
    f = tmp_path / "cpu.max"
    f.write_text("1600000 100000\n")
    assert cpus.cgroup_cpu_quota(str(f)) == 16
    f.write_text("max 100000\n")
    assert cpus.cgroup_cpu_quota(str(f)) == float("inf")
    assert cpus.cgroup_cpu_quota(str(tmp_path / "missing")) == float("inf")
    cpus.effective_cpus.cache_clear()
    monkeypatch.setattr(cpus, "cgroup_cpu_quota", lambda path="": 2.5)
    assert cpus.effective_cpus() == min(3, len(os.sched_getaffinity(0)))
    cpus.effective_cpus.cache_clear()


def test_native_effective_cpus_matches_python():
    from downloader_amd.ops import native
    from downloader_amd.utils.cpus import effective_cpus
    assert native().effective_cpus() == effective_cpus()


def test_cancelled_native_request_frees_its_thread(run):
    """A request stuck on a silent server: cancelling it aborts the socket, so the single
    executor thread is free again at once instead of after io_timeout."""
    import asyncio
    import socket
    import time
    from downloader_amd.net.http import NativeTransport

    async def go():
        srv = socket.socket()
        srv.bind(("127.0.0.1", 0))
        srv.listen(4)
        port = srv.getsockname()[1]
        t = NativeTransport(max_workers=1, connect_timeout=5, io_timeout=60)
        task = asyncio.ensure_future(t.request("GET", f"http://127.0.0.1:{port}/x"))
        await asyncio.sleep(0.3)
        task.cancel()
        t0 = time.perf_counter()
        await asyncio.get_running_loop().run_in_executor(t._exec, lambda: None)
        assert time.perf_counter() - t0 < 5
        await t.close()
        srv.close()
    run(go(), timeout=30)


def test_redirect_target_and_headers():
    from downloader_amd.net.http import Response, redirect_headers, redirect_target
    r = Response(302, [("location", "../b/c d.mkv?x=1")])
    assert redirect_target("http://h:1/a/x/y.mkv", r) == "http://h:1/a/b/c%20d.mkv?x=1"
    assert redirect_target("http://h/a", Response(200, [("location", "/x")])) is None
    assert redirect_target("http://h/a", Response(301, [])) is None
    assert redirect_target("http://h/a", Response(302, [("location", "ftp://x/y")])) is None
    assert redirect_target("http://h/a", Response(302, [("location", "/p%20q")])) == "http://h/p%20q"
    hdrs = [("Range", "bytes=0-9"), ("Authorization", "AWS4 x"), ("Host", "h")]
    assert redirect_headers("http://h/a", "http://h/b", hdrs) == hdrs[:2]
    assert redirect_headers("http://h/a", "http://other/b", hdrs) == hdrs[:1]


def test_long_running_worker_state_is_bounded(make_cfg):
    """Per-job records a worker keeps for tests and debugging (results, telemetry history)
    are bounded, so a worker staging millions of jobs does not grow without limit."""
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.service import worker as wmod
    from downloader_amd.service.telemetry import Telemetry
    w = wmod.Worker(make_cfg(), broker=MemoryBroker())
    assert w.results.maxlen == wmod.RESULTS_MAX
    for i in range(wmod.RESULTS_MAX + 5):
        w.results.append(i)
    assert len(w.results) == wmod.RESULTS_MAX and w.results[0] == 5
    t = Telemetry(None, history_max=3)
    import asyncio as _a
    for i in range(5):
        _a.run(t.emit_progress("m", 2, i))
    assert t.progress_of("m") == [2, 3, 4]


def test_native_pool_idle_ttl_and_global_cap(run, origin_cls):
    """Idle keep-alive sockets are capped over all hosts and expire after idle_ttl."""
    from downloader_amd.net.http import NativeTransport

    async def go():
        origins = [await origin_cls().start() for _ in range(3)]
        for o in origins:
            o.blobs["/x"] = b"y" * 100
        t = NativeTransport(max_workers=4, idle_ttl=0.3, max_idle_total=2)
        for o in origins:
            r = await t.request("GET", o.url("/x"))
            assert r.status == 200 and r.body == b"y" * 100
        assert t.idle_connections() == 2                    # global cap
        r = await t.request("GET", origins[2].url("/x"))    # reuses a pooled socket
        assert r.status == 200 and t.idle_connections() == 2
        await asyncio.sleep(0.4)
        r = await t.request("GET", origins[2].url("/x"))    # expired: dropped, fresh socket
        assert r.status == 200 and t.idle_connections() <= 2
        await t.close()
        for o in origins:
            await o.stop()
    run(go())


def test_redact_url_for_logs():
    from downloader_amd.utils.log import redact_url
    u = ("https://u:pw@cdn.example.com:8443/m/x.mkv?X-Amz-Algorithm=AWS4-HMAC-SHA256"
         "&X-Amz-Credential=AKIA%2F2024&X-Amz-Signature=abc123&partNumber=2&token=t0k")
    r = redact_url(u)
    assert "pw" not in r and "abc123" not in r and "AKIA" not in r and "t0k" not in r
    assert r.startswith("https://u:***@cdn.example.com:8443/m/x.mkv?")
    assert "X-Amz-Algorithm=AWS4-HMAC-SHA256" in r and "partNumber=2" in r
    assert redact_url("http://o/x.mkv?size=1") == "http://o/x.mkv?size=1"
    assert redact_url("magnet:?xt=urn:btih:abc") == "magnet:?xt=urn:btih:abc"


def test_native_transport_ipv6_literal(run):
    """http://[::1]:port/ - bracketed IPv6 literals reach the native transport (getaddrinfo
    AF_UNSPEC) with a bracketed Host header."""
    import socket

    from aiohttp import web

    from downloader_amd.net.http import NativeTransport
    if not socket.has_ipv6:
        pytest.skip("no IPv6")

    async def go():
        seen = {}

        async def h(r):
            seen["host"] = r.headers.get("Host")
            return web.Response(body=b"v6" * 1000)
        app = web.Application()
        app.router.add_get("/x", h)
        runner = web.AppRunner(app)
        await runner.setup()
        try:
            site = web.TCPSite(runner, "::1", 0)
            await site.start()
        except OSError:
            await runner.cleanup()
            pytest.skip("no IPv6 loopback")
        port = site._server.sockets[0].getsockname()[1]
        t = NativeTransport(2)
        r = await t.request("GET", f"http://[::1]:{port}/x")
        assert r.status == 200 and r.body == b"v6" * 1000
        assert seen["host"] == f"[::1]:{port}"
        await t.close()
        await runner.cleanup()
    run(go())


def test_native_http_parser_survives_garbage(run, tmp_path):
    """Malformed / truncated / hostile responses (bad status lines, negative or non-hex chunk
    sizes, lying Content-Length, early close) end in an HttpError / TransportError - never a
    crash of the native parser, never a hang - for bodies read into memory and into files."""
    import random

    from downloader_amd.net.http import FileSink, HttpError, NativeTransport
    rng = random.Random(1234)
    pieces = [b"HTTP/1.1 200 OK\r\n", b"HTTP/1.0 206 Partial\r\n", b"HTTP/1.1 abc\r\n",
              b"garbage\r\n", b"Content-Length: 10\r\n", b"Content-Length: -4\r\n",
              b"Content-Length: 99999999999999999999\r\n", b"Transfer-Encoding: chunked\r\n",
              b"Connection: close\r\n", b"X: " + b"y" * 70000 + b"\r\n", b"\r\n",
              b"5\r\nhello\r\n", b"-5\r\nhello\r\n", b"zz\r\n", b"0\r\n\r\n",
              b"fffffffffffffffffffffff\r\n", b"abcdefghij", b"\x00\xff" * 20]
    cases = [b"".join(rng.choice(pieces) for _ in range(rng.randint(1, 6))) for _ in range(150)]
    cases += [b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n-5\r\nhello\r\n0\r\n\r\n",
              b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n",
              b"HTTP/1.1 200 OK\r\nContent-Length: 100\r\n\r\nshort"]

    async def go():
        i = {"n": 0}

        async def serve(r, w):
            payload = cases[i["n"] % len(cases)]
            try:
                await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
                w.write(payload)
                await w.drain()
            except Exception:
                pass
            w.close()
        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        t = NativeTransport(4, connect_timeout=2, io_timeout=2)
        outcomes = {"ok": 0, "err": 0}
        fd = os.open(str(tmp_path / "sink"), os.O_WRONLY | os.O_CREAT, 0o600)
        for k in range(len(cases)):
            i["n"] = k
            for sink in (None, FileSink(fd, 0, 1 << 20)):
                try:
                    await asyncio.wait_for(
                        t.request("GET", f"http://127.0.0.1:{port}/f", sink=sink), 10)
                    outcomes["ok"] += 1
                except (HttpError, ValueError):
                    outcomes["err"] += 1
        os.close(fd)
        assert outcomes["err"] > 50 and sum(outcomes.values()) == 2 * len(cases)
        await t.close()
        srv.close()
        await srv.wait_closed()
    run(go(), timeout=300)


def test_native_http_head_limits_and_strict_lengths(run):
    """The native parser refuses what it cannot delimit safely instead of guessing: a
    Content-Length that is not plain decimal, conflicting Content-Length values, a status code
    that is not three digits in 100-599, and a head of more than 1,024 lines / 256 KiB (an
    origin streaming headers forever would otherwise grow memory without bound). Identical
    repeated lengths (RFC 9110) are accepted."""
    from downloader_amd.net.http import HttpError, NativeTransport
    hdrs = b"".join(b"X-%d: v\r\n" % i for i in range(2000))
    cases = {
        "bad_len": (b"HTTP/1.1 200 OK\r\nContent-Length: 0x10\r\n\r\n" + b"a" * 16, None),
        "plus_len": (b"HTTP/1.1 200 OK\r\nContent-Length: +5\r\n\r\nhello", None),
        "conflict": (b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\nContent-Length: 6\r\n\r\n"
                     b"hello!", None),
        "list_conflict": (b"HTTP/1.1 200 OK\r\nContent-Length: 5, 6\r\n\r\nhello!", None),
        "list_same": (b"HTTP/1.1 200 OK\r\nContent-Length: 5, 5\r\n\r\nhello", b"hello"),
        "code4": (b"HTTP/1.1 2000 OK\r\nContent-Length: 1\r\n\r\nx", None),
        "code99": (b"HTTP/1.1 099 Odd\r\nContent-Length: 1\r\n\r\nx", None),
        "nocode": (b"HTTP/1.1\r\nContent-Length: 1\r\n\r\nx", None),
        "many_headers": (b"HTTP/1.1 200 OK\r\n" + hdrs + b"Content-Length: 1\r\n\r\nx", None),
        "big_trailer": (b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n1\r\nx\r\n0\r\n"
                        + (b"T: " + b"t" * 60000 + b"\r\n") * 5 + b"\r\n", None),
        "ok": (b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\n\r\nhello", b"hello"),
    }

    async def go():
        current = {"k": None}

        async def serve(r, w):
            try:
                await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
                w.write(cases[current["k"]][0])
                await w.drain()
                await asyncio.sleep(0.05)
            except Exception:
                pass
            w.close()
        srv = await asyncio.start_server(serve, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        t = NativeTransport(2, connect_timeout=2, io_timeout=2)
        for k, (_, want) in cases.items():
            current["k"] = k
            if want is None:
                with pytest.raises(HttpError):
                    await asyncio.wait_for(t.request("GET", f"http://127.0.0.1:{port}/{k}"), 10)
            else:
                r = await asyncio.wait_for(t.request("GET", f"http://127.0.0.1:{port}/{k}"), 10)
                assert r.status == 200 and r.body == want, k
        await t.close()
        srv.close()
        await srv.wait_closed()
    run(go(), timeout=120)


def test_nofile_limit_raised_and_storage_headroom_checked(tmp_path):
    """A torrent with more files than RLIMIT_NOFILE leaves fails up front with EMFILE and a
    clear message (not halfway through the job); ``raise_nofile`` (worker start) lifts the
    soft limit to the hard one so the same torrent opens."""
    import errno
    import resource

    from downloader_amd.torrent.bencode import bencode
    from downloader_amd.torrent.metainfo import parse_torrent
    from downloader_amd.torrent.storage import Storage
    from downloader_amd.utils import limits
    files = [{b"length": 10, b"path": [b"f%04d.mkv" % i]} for i in range(600)]
    info = {b"name": b"many", b"piece length": 16384, b"pieces": b"\0" * 20, b"files": files}
    meta = parse_torrent(bencode({b"info": info}))
    soft0, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if hard != resource.RLIM_INFINITY and hard < 1400:
        pytest.skip(f"hard RLIMIT_NOFILE {hard} too low for this test")
    try:
        resource.setrlimit(resource.RLIMIT_NOFILE, (512, hard))
        with pytest.raises(OSError) as ei:
            Storage(meta, str(tmp_path / "a"))
        assert ei.value.errno == errno.EMFILE and "600 files" in str(ei.value)
        soft, _ = limits.raise_nofile()
        assert soft >= min(hard, limits.NOFILE_CAP) and soft > 512
        st = Storage(meta, str(tmp_path / "b"))
        assert len(st.fds) == 600
        st.close()
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft0, hard))


def test_cancelled_native_download_never_writes_after_cancel(run, tmp_path):
    """Cancelling a native download into a file returns only once the transfer thread has
    let go of the descriptor: a file opened right after (reusing the fd number, as a torrent
    session's next storage would) receives none of the old transfer's bytes."""
    from downloader_amd.net.http import FileSink, NativeTransport

    async def go():
        async def slow(r, w):
            await r.readuntil(b"\r\n\r\n")
            w.write(b"HTTP/1.1 200 OK\r\nContent-Length: 100000000\r\n\r\n")
            try:
                for _ in range(400):
                    w.write(b"x" * 65536)
                    await w.drain()
                    await asyncio.sleep(0.005)
            except Exception:
                pass
            w.close()
        srv = await asyncio.start_server(slow, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        t = NativeTransport(2, connect_timeout=2, io_timeout=10)
        loop = asyncio.get_running_loop()
        futs = []
        orig = loop.run_in_executor

        def capture(ex, fn, *a):
            f = orig(ex, fn, *a)
            futs.append(f)
            return f
        loop.run_in_executor = capture
        fd = os.open(str(tmp_path / "old"), os.O_WRONLY | os.O_CREAT, 0o600)
        task = asyncio.ensure_future(t.request("GET", f"http://127.0.0.1:{port}/big",
                                               sink=FileSink(fd, 0, 100_000_000)))
        await asyncio.sleep(0.3)
        task.cancel()
        with pytest.raises(asyncio.CancelledError):
            await task
        assert futs and all(f.done() for f in futs)    # the thread has returned
        loop.run_in_executor = orig
        os.close(fd)
        fd2 = os.open(str(tmp_path / "new"), os.O_WRONLY | os.O_CREAT, 0o600)
        await asyncio.sleep(0.5)
        os.close(fd2)
        assert os.path.getsize(tmp_path / "new") == 0
        assert os.path.getsize(tmp_path / "old") > 0
        await t.close()
        srv.close()
        await srv.wait_closed()
    run(go(), timeout=60)


def test_pipe_size_follows_the_uid_budget():
    """Splice pipes are sized so every worker of the uid fits in the pipe page budget
    (64 MiB default for non-root): 1 MiB when unbounded, power-of-two steps down to 64 KiB."""
    from downloader_amd.utils import limits
    mib = 1 << 20
    assert limits.pipe_size(budget=0) == mib                       # root / no soft limit
    assert limits.pipe_size(pipe_kb=300) == 300 << 10              # explicit
    b = 64 * mib
    assert limits.pipe_size(sharers=2, per_proc=10, budget=b) == mib
    assert limits.pipe_size(sharers=4, per_proc=10, budget=b) == mib
    assert limits.pipe_size(sharers=8, per_proc=10, budget=b) == 512 << 10
    assert limits.pipe_size(sharers=16, per_proc=10, budget=b) == 256 << 10
    assert limits.pipe_size(sharers=1000, per_proc=16, budget=b) == 64 << 10   # floor
    for sharers in (1, 2, 4, 8, 16, 32):
        sz = limits.pipe_size(sharers=sharers, per_proc=10, budget=b)
        assert sz & (sz - 1) == 0 and (sz == 64 << 10 or sharers * 10 * sz <= b * 3 // 4)


def test_transfers_copy_when_no_pipe_can_be_had(run, origin_cls):
    """With the pipe budget spent, relays (plain, CRC'd, piece-hashed) and bodies to disk
    copy through user space instead of splicing through two-page pipes - same bytes."""
    import hashlib
    import os

    from downloader_amd.ops import native
    from downloader_amd.s3.client import S3Client
    from downloader_amd.s3.fake_server import FakeS3

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(9_000_000)
        origin.blobs["/x.bin"] = blob
        for policy in ("auto", "always"):
            c = S3Client(ep, "minioadmin", "minioadmin", checksum=policy)
            await c.ensure_bucket("b")
            await c.relay_object("b", f"plain-{policy}", origin.url("/x.bin"), len(blob))
            assert s3.get("b", f"plain-{policy}") == blob
            _, h = await c.relay_hashed("b", f"h-{policy}", origin.url("/x.bin"), 0, len(blob),
                                        True, (1000, 8 << 20, 1 << 20))
            assert h["digests"] == b"".join(hashlib.sha1(blob[1000 + i:1000 + i + (1 << 20)])
                                            .digest() for i in range(0, 8 << 20, 1 << 20))
            assert h["head"] == blob[:1000] and h["tail"] == blob[1000 + (8 << 20):]
            await c.close()
        await origin.stop(); await s3.stop()

    n = native()
    before = n.pipe_stats()["created"]
    n.set_pipes_refused(True)
    try:
        run(go())
    finally:
        n.set_pipes_refused(False)
    assert n.pipe_stats()["created"] == before and n.pipe_stats()["in_use"] == 0


def test_trace_summary_counts_lanes_and_overlap(tmp_path):
    """bench/trace_summary.py on a rocprofv3 kernel-trace CSV: launches, duration stats,
    grid threads per launch (lanes for sha1_lanes) and the peak of overlapping launches."""
    from downloader_amd.bench.trace_summary import summarise
    hdr = ('"Kind","Kernel_Name","Start_Timestamp","End_Timestamp","Grid_Size_X",'
           '"Grid_Size_Y"\n')
    k16 = 'void (anonymous namespace)::sha1_lanes<16>(unsigned char const*, long)'
    rows = [(k16, 0, 10_000_000, 128), (k16, 5_000_000, 20_000_000, 256),
            ('__amd_rocclr_copyBuffer', 30_000_000, 30_000_100, 512)]
    p = tmp_path / "t.csv"
    p.write_text(hdr + "".join(f'"KERNEL_DISPATCH","{n}",{s},{e},{g},1\n' for n, s, e, g in rows))
    s = summarise(str(p))
    k = s["sha1_lanes<16>"]
    assert k["launches"] == 2 and k["grid_threads_min"] == 128 and k["grid_threads_max"] == 256
    assert k["max_concurrent"] == 2 and k["ms_max"] == 15.0 and k["device_busy_share"] == 1.0
    assert s["__amd_rocclr_copyBuffer"]["launches"] == 1


def test_relay_plan_keeps_pipes_at_512k_under_the_uid_budget():
    """bench.py's splice plan for N ranks x 2 processes on a 64 MiB uid pipe budget: 1 MiB
    pipes while they fit, 512 KiB at 4 ranks, and at 8 ranks 3 jobs per process on 512 KiB
    pipes rather than 4 on 256 KiB (measured 13 % slower); root / no budget: unchanged."""
    from downloader_amd.utils.limits import PIPE_GOOD, PIPE_MAX, relay_plan
    b = 64 << 20
    assert relay_plan(4, 2, 2, b) == (4, PIPE_MAX)
    assert relay_plan(4, 2, 4, b) == (4, PIPE_MAX)
    assert relay_plan(4, 2, 8, b) == (4, PIPE_GOOD)
    assert relay_plan(4, 2, 16, b) == (3, PIPE_GOOD)
    for sharers in (2, 4, 8, 16):
        c, p = relay_plan(4, 2, sharers, b)
        assert sharers * c * 2 * p <= b * 7 // 8
    assert relay_plan(4, 2, 64, b)[0] == 2                # never below 2 jobs
    assert relay_plan(4, 2, 16, 0) == (4, PIPE_MAX)


def test_part_budget_fifo_oversize_and_cancellation(run):
    """utils/membudget.PartBudget: grants in arrival order (a big request is not starved by
    later small ones), a request larger than the whole budget runs alone, and a cancelled
    waiter neither leaks bytes nor blocks the ones behind it."""
    import asyncio

    from downloader_amd.utils.membudget import BUFFER_ALIGN, PartBudget, buffer_bytes
    MiB = 1 << 20
    assert buffer_bytes(1) == BUFFER_ALIGN and buffer_bytes(5 * MiB) == 6 * MiB

    async def go():
        b = PartBudget(8 * MiB)
        a = await b.acquire(6 * MiB)                 # 6 of 8 used
        order = []

        async def want(tag, n):
            got = await b.acquire(n)
            order.append(tag)
            return got
        big = asyncio.ensure_future(want("big", 4 * MiB))
        await asyncio.sleep(0)
        small = asyncio.ensure_future(want("small", 2 * MiB))   # would fit now, but queues
        await asyncio.sleep(0.01)
        assert order == [] and b.stats()["queued"] == 2
        b.release(a)                                   # big first, then small fits too
        await big
        await small
        assert order == ["big", "small"] and b.used == 6 * MiB
        b.release(4 * MiB)
        b.release(2 * MiB)
        huge = await b.acquire(20 * MiB)               # alone: granted past the capacity
        assert b.used == 20 * MiB
        w1 = asyncio.ensure_future(b.acquire(2 * MiB))
        w2 = asyncio.ensure_future(b.acquire(2 * MiB))
        await asyncio.sleep(0.01)
        w1.cancel()
        await asyncio.sleep(0)
        b.release(huge)
        assert await w2 == 2 * MiB and b.used == 2 * MiB
        assert w1.cancelled() and b.stats()["queued"] == 0 and b.peak == 20 * MiB
    run(go())


def test_relay_budget_follows_the_memory_limit(monkeypatch):
    from downloader_amd.utils import membudget
    from downloader_amd.utils.config import DownloadConfig
    MiB = 1 << 20
    monkeypatch.setattr(membudget, "memory_limit", lambda: 32 << 30)
    monkeypatch.setenv("STAGER_POOL_WORKERS", "2")
    assert membudget.relay_budget_bytes(DownloadConfig()) == 4 << 30          # 32 / 2 / 4
    assert membudget.relay_budget_bytes(DownloadConfig(relay_memory_mb=300)) == 300 * MiB
    monkeypatch.setattr(membudget, "memory_limit", lambda: 256 * MiB)
    assert membudget.relay_budget_bytes(DownloadConfig()) == membudget.MIN_BUDGET


def test_relay_budget_is_a_per_slot_share(monkeypatch):
    """No STAGER_POOL_WORKERS (bench ranks, standalone workers on a shared 8-GPU node): the
    divisor is GPU slots x worker processes per slot, as for the CPU budget."""
    from downloader_amd.utils import membudget
    from downloader_amd.utils.config import DownloadConfig
    lim = 1536 << 30
    monkeypatch.setattr(membudget, "memory_limit", lambda: lim)
    monkeypatch.delenv("STAGER_POOL_WORKERS", raising=False)
    monkeypatch.setenv("STAGER_GPU_SLOTS", "8")
    monkeypatch.setenv("STAGER_PROCS_PER_SLOT", "2")
    assert membudget.pool_workers() == 16
    assert membudget.relay_budget_bytes(DownloadConfig()) == int(lim // 16 * 0.25)
    monkeypatch.delenv("STAGER_PROCS_PER_SLOT")
    assert membudget.pool_workers() == 8
    monkeypatch.setenv("STAGER_POOL_WORKERS", "3")                 # explicit wins
    assert membudget.pool_workers() == 3


def test_supervisor_and_bench_children_declare_procs_per_slot(monkeypatch):
    from downloader_amd.parallel.supervisor import Supervisor
    monkeypatch.delenv("STAGER_PROCS_PER_SLOT", raising=False)
    seen = {}

    class P:
        def __init__(self, argv, env, preexec_fn):
            seen.update(env)
    monkeypatch.setattr("subprocess.Popen", P)
    s = Supervisor(2, ["true"], env={})
    s._spawn(s.slots[0])
    assert seen["STAGER_PROCS_PER_SLOT"] == "2" and "STAGER_POOL_WORKERS" not in seen


def test_cgroup_memory_limit_v1_v2(tmp_path):
    from downloader_amd.utils.membudget import cgroup_memory_limit
    (tmp_path / "memory.max").write_text("max\n")
    assert cgroup_memory_limit(str(tmp_path)) == 0
    (tmp_path / "memory.max").write_text("34359738368\n")
    assert cgroup_memory_limit(str(tmp_path)) == 32 << 30
    v1 = tmp_path / "v1"
    (v1 / "memory").mkdir(parents=True)
    (v1 / "memory" / "memory.limit_in_bytes").write_text("9223372036854771712\n")   # unlimited
    assert cgroup_memory_limit(str(v1)) == 0
    (v1 / "memory" / "memory.limit_in_bytes").write_text("8589934592\n")
    assert cgroup_memory_limit(str(v1)) == 8 << 30


def test_swarm_memory_defaults_follow_the_worker_share(monkeypatch):
    """download.swarm_pool_mb / swarm_backlog_mb 0: 1/8 of the worker's share of the memory
    limit, capped at 4 GiB, at least 256 MiB; an explicit value wins."""
    from downloader_amd.utils import membudget
    gib = 1 << 30
    monkeypatch.setenv("STAGER_POOL_WORKERS", "2")
    monkeypatch.setattr(membudget, "memory_limit", lambda: 300 * gib)
    assert membudget.swarm_bytes(0) == 4 * gib
    monkeypatch.setattr(membudget, "memory_limit", lambda: 8 * gib)
    assert membudget.swarm_bytes(0) == gib // 2
    monkeypatch.setattr(membudget, "memory_limit", lambda: 1 * gib)
    assert membudget.swarm_bytes(0) == 256 << 20
    assert membudget.swarm_bytes(100) == 100 << 20
