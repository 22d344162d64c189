"""Service kernel end-to-end on in-process fakes (SURVEY §7.3 minimum slice + §3.4 failure
paths): memory broker -> worker -> HTTP origin -> selector -> FakeS3 -> convert publish."""
from __future__ import annotations

import asyncio
import base64
import os

import pytest

from downloader_amd.broker.memory import MemoryBroker
from downloader_amd.models import api, keys
from downloader_amd.s3.fake_server import FakeS3, FaultRule
from downloader_amd.service.worker import Worker
from downloader_amd.stages.base import DownloadStalled, Stage


async def _wait(w, n=1, timeout=30.0):
    t = 0.0
    while len(w.results) < n and t < timeout:
        await asyncio.sleep(0.02)
        t += 0.02
    assert len(w.results) >= n, w.results


async def _setup(make_cfg, origin_cls, **over):
    s3 = FakeS3()
    ep = await s3.start()
    origin = await origin_cls().start()
    cfg = make_cfg(ep, **over)
    b = MemoryBroker()
    w = Worker(cfg, broker=b)
    await w.start(health=False)
    return s3, origin, b, w


def test_minimum_slice_http_to_s3(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls)
        blob = os.urandom(10 * 1024 * 1024 + 3)
        origin.blobs["/media/blob.mkv"] = blob
        await w.submit(api.make_download("job1", "http", origin.url("/media/blob.mkv?x=1")))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "staged" and r.bytes == len(blob)
        key = "job1/original/" + base64.b64encode(b"blob.mkv").decode()
        assert s3.get("triton-staging", key) == blob
        assert s3.get("triton-staging", "job1/original/done") == b"true"
        assert w.telemetry.statuses_of("job1") == [2]
        assert w.telemetry.progress_of("job1") == [0, 50, 100]
        conv = b.drain("v1.convert")
        assert len(conv) == 1
        c = api.decode(api.Convert, conv[0])
        assert c.media.id == "job1" and c.media.sourceURI.endswith("blob.mkv?x=1")
        # job directory released at once (renamed into .trash), unlinked by the reaper
        root = w.cfg.instance.download_path
        assert not os.path.exists(os.path.join(root, "job1"))
        code = await w.stop()
        assert code == 0
        assert os.listdir(os.path.join(root, ".trash")) == []
        await s3.stop()
        await origin.stop()
    run(go())


def test_done_marker_skips_stages(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls)
        s3.buckets["triton-staging"] = {}
        s3.put("triton-staging", "job2/original/done", b"true")
        await w.submit(api.make_download("job2", "http", origin.url("/nothing.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "skipped"
        assert origin.requests == []
        assert len(b.drain("v1.convert")) == 1
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_done_marker_probe_error_is_not_treated_as_missing(run, make_cfg, origin_cls):
    # App. A #5: only NoSuchKey means "not staged"; an auth error must retry, not re-download
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0})
        s3.faults.add(FaultRule(method="GET", path_contains="/done", status=403,
                                code="AccessDenied", times=1))
        origin.blobs["/a.mkv"] = b"x" * 100
        await w.submit(api.make_download("job3", "http", origin.url("/a.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "dead"
        assert origin.requests == []
        assert w.telemetry.statuses_of("job3") == [2, 6]
        assert len(b.drain("v1.download.dead")) == 1
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_http_error_status_fails_job_then_retries_then_dead_letters(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 2})
        origin.fail_status["/bad.mkv"] = 500
        await w.submit(api.make_download("job4", "http", origin.url("/bad.mkv")))
        await _wait(w, 3)
        assert [r.outcome for r in w.results] == ["retried", "retried", "dead"]
        dead = b.drain("v1.download.dead")
        assert len(dead) == 1
        assert b.drain("v1.convert") == []
        assert w.telemetry.statuses_of("job4") == [2, 6, 2, 6, 2, 6]
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_reference_mode_nacks_on_failure(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, mode="reference")
        origin.fail_status["/bad.mkv"] = 404
        await w.submit(api.make_download("job5", "http", origin.url("/bad.mkv")))
        await _wait(w, 2)
        assert w.results[0].outcome == "failed"
        assert w.results[1].outcome == "failed"   # redelivered (nack requeue)
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_no_media_files_fails(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0})
        origin.blobs["/notes.txt"] = b"hello"
        await w.submit(api.make_download("job6", "http", origin.url("/notes.txt")))
        await _wait(w)
        assert w.results[0].outcome == "dead"
        assert "suitable media" in w.results[0].error
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


class _StallStage(Stage):
    async def run(self, job):
        raise DownloadStalled()


async def stall_factory(cfg, services):
    return _StallStage()


def test_stall_acks_and_drops(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(
            make_cfg, origin_cls, stages=["tests.test_worker:stall_factory"])
        await w.submit(api.make_download("job7", "http", origin.url("/x.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "stalled"
        assert await b.queue_size("v1.download") == 0
        assert w.telemetry.statuses_of("job7") == [2]      # reference: no ERRORED on stall
        assert w.metrics.sample("downloader_stall_total") == 1
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_convert_publish_failure_nacks(run, make_cfg, origin_cls):
    # App. A #8: a failed convert publish must not leave the delivery unacked forever.
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls)
        origin.blobs["/m.mkv"] = b"m" * 1000
        await w.submit(api.make_download("job8", "http", origin.url("/m.mkv")))
        # fail only the convert publish (telemetry is disabled on a memory-broker? no: count)
        orig = b.publish

        async def flaky(queue, body, headers=None):
            if queue == "v1.convert" and not getattr(flaky, "done", False):
                flaky.done = True
                raise ConnectionError("broker down")
            return await orig(queue, body, headers)
        b.publish = flaky
        await _wait(w, 2)
        assert w.results[0].outcome == "publish_failed"
        assert w.results[1].outcome == "skipped"   # redelivered; done marker present
        assert len(b.drain("v1.convert")) == 1
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_health_endpoint_semantics(run, make_cfg, origin_cls):
    async def go():
        import aiohttp
        s3, origin, b, w = await _setup(make_cfg, origin_cls)
        from downloader_amd.service.health import HealthServer
        w.cfg.health.port = 0
        hs = HealthServer(w, w.cfg.health)
        port = await hs.start()
        async with aiohttp.ClientSession() as sess:
            async with sess.get(f"http://127.0.0.1:{port}/health") as r:
                assert r.status == 500
                assert await r.json() == {"message": "Not Running Jobs"}
            from downloader_amd.service.worker import ActiveJob
            w.active[99] = ActiveJob("j", "c")
            async with sess.get(f"http://127.0.0.1:{port}/health") as r:
                body = await r.json()
                assert r.status == 200 and body["data"]["active"] == 1
                assert body["metadata"]["success"] is True
            async with sess.get(f"http://127.0.0.1:{port}/readyz") as r:
                assert r.status == 200
            async with sess.get(f"http://127.0.0.1:{port}/metrics") as r:
                txt = await r.text()
                assert "downloader_jobs_total" in txt
                assert "downloader_http_idle_connections" in txt       # native runtime gauges
                assert "downloader_relay_pool_idle_bytes" in txt
                assert "downloader_splice_pipes_short_total" in txt    # pipe budget signal
                assert "downloader_relay_pool_budget_bytes" in txt     # part-buffer budget
                assert "downloader_relay_pool_over_budget_total" in txt
                assert "downloader_gpu_parts_pending" in txt
                assert "downloader_telemetry_buffered" in txt
        w.active.clear()
        await hs.stop()
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


@pytest.mark.parametrize("stream", [True, False])
def test_multi_file_bucket_source_with_collisions(run, make_cfg, origin_cls, stream):
    """Same outcome on the streamed (presigned relay) and the disk path."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={
            "bucket_secure": False, "stream_bucket": stream})
        s3.buckets["src"] = {}
        s3.put("src", "show/S1/KonoSuba S1E1.mkv", b"one")
        s3.put("src", "show/Season 1/KonoSuba S1E1.mkv", b"two")
        s3.put("src", "show/Extras/ova.mkv", b"x")
        uri = f"bucket://{s3.endpoint},src,minioadmin,minioadmin,show"
        await w.submit(api.make_download("job9", "bucket", uri, "TV"))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        k = keys.object_key("job9", "KonoSuba S1E1.mkv")
        assert s3.get("triton-staging", k) == b"two"   # last in walk order wins (App. A #10)
        assert w.metrics.sample("downloader_key_collisions_total") == 1
        assert w.telemetry.progress_of("job9") == [0, 50, 75, 100]
        assert bool(w.results[0].stats.get("streamed")) == stream
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


@pytest.mark.parametrize("server_copy", [False, True])
def test_bucket_source_streams_selected_objects_only(run, make_cfg, origin_cls, tmp_path,
                                                     server_copy, monkeypatch):
    """bucket:// fast path: the selector runs on the object listing; selected objects (one
    above the multipart threshold: Range parts in parallel) are relayed source -> staging
    through presigned GETs - or, the source being on the staging endpoint with the same
    credentials, copied server-side (CopyObject; UploadPartCopy ranges above the copy
    limit, shrunk here to 5 MiB) - extras are never fetched and nothing touches the disk."""
    from downloader_amd.s3 import client as s3client
    monkeypatch.setattr(s3client, "COPY_MAX", 5 << 20)
    monkeypatch.setattr(s3client, "COPY_PART", 5 << 20)

    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={
            "bucket_secure": False, "bucket_server_copy": server_copy})
        s3.buckets["src"] = {}
        big = os.urandom((13 << 20) + 7)
        s3.put("src", "lib/Show/Season 1/e1.mkv", big)
        s3.put("src", "lib/Show/Season 1/e2.mkv", b"e2" * 5000)
        s3.put("src", "lib/Show/Extras/making-of.mkv", os.urandom(3 << 20))
        s3.put("src", "lib/Show/notes.txt", b"n")
        s3.put("src", "lib/Show/Season 1/e0.mkv", b"")                # empty object
        uri = f"bucket://{s3.endpoint},src,minioadmin,minioadmin,lib"
        await w.submit(api.make_download("bs1", "bucket", uri, "TV"))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert [os.path.basename(x["file"]) for x in r.stats["streamed"]] == \
            ["e0.mkv", "e1.mkv", "e2.mkv"]
        assert s3.get("triton-staging", keys.object_key("bs1", "e0.mkv")) == b""
        assert r.stats["bucket_skipped_bytes"] == (3 << 20) + 1
        assert s3.get("triton-staging", keys.object_key("bs1", "e1.mkv")) == big
        assert s3.objects("triton-staging")[keys.object_key("bs1", "e1.mkv")].etag.endswith("-3")
        assert s3.get("triton-staging", keys.object_key("bs1", "e2.mkv")) == b"e2" * 5000
        assert s3.get("triton-staging", keys.object_key("bs1", "making-of.mkv")) is None
        gets = [p for m, p in s3.requests if m == "GET" and p.startswith("/src/")]
        assert r.stats["bucket_server_copy"] is server_copy
        if server_copy:
            assert not gets and s3.server_copies == 3 + 2      # e0, e2 + e1's 3 ranges
        else:
            assert gets and not any("Extras" in p or "notes" in p for p in gets)
            assert s3.server_copies == 0
        assert s3.get("triton-staging", keys.done_key("bs1")) is not None
        for dp, _, fns in os.walk(tmp_path / "dl"):
            assert not [f for f in fns if f.endswith(".mkv")], (dp, fns)
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_file_urls_gated(run, make_cfg, origin_cls, tmp_path):
    async def go():
        src = tmp_path / "in.mkv"
        src.write_bytes(b"f" * 12345)
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0})
        await w.submit(api.make_download("j10", "file", f"file://{src}"))
        await _wait(w)
        assert w.results[0].outcome == "dead" and "not allowed" in w.results[0].error
        await w.stop()
        s3b, origin2, b2, w2 = s3, origin, MemoryBroker(), None
        cfg = make_cfg(s3.endpoint, download={"allow_file_urls": True})
        w2 = Worker(cfg, broker=b2)
        await w2.start(health=False)
        await w2.submit(api.make_download("j11", "file", f"file://{src}"))
        await _wait(w2)
        assert w2.results[0].outcome == "staged"
        assert s3.get("triton-staging", keys.object_key("j11", "in.mkv")) == b"f" * 12345
        assert w2.results[0].stats.get("streamed")          # uploaded from its own path
        assert src.read_bytes() == b"f" * 12345               # source untouched
        await w2.stop()
        # disk path (stream_file off) and a non-media name: copied, then selected as usual
        w3 = Worker(make_cfg(s3.endpoint, download={"allow_file_urls": True,
                                                    "stream_file": False}), broker=b2)
        await w3.start(health=False)
        await w3.submit(api.make_download("j12", "file", f"file://{src}"))
        await _wait(w3)
        assert w3.results[0].outcome == "staged" and not w3.results[0].stats.get("streamed")
        assert s3.get("triton-staging", keys.object_key("j12", "in.mkv")) == b"f" * 12345
        await w3.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_concurrent_jobs_prefetch(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, concurrency=3)
        for i in range(6):
            origin.blobs[f"/c{i}.mp4"] = os.urandom(200_000)
            await w.submit(api.make_download(f"cj{i}", "http", origin.url(f"/c{i}.mp4")))
        await _wait(w, 6)
        assert all(r.outcome == "staged" for r in w.results)
        assert w.cfg.broker.prefetch == 3
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_unsupported_protocol_and_bad_message(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0})
        d = api.make_download("j12", "http", "x")
        d.media.source = 3  # BUCKET with a malformed URI
        d.media.sourceURI = "bucket://nope"
        await w.submit(d)
        await b.publish("v1.download", b"\xff\xff\xff garbage")
        # a publisher's junk x-attempt header is attempt 0, not a stuck unacked delivery
        origin.blobs["/ok.mkv"] = b"m" * 1000
        await w.submit(api.make_download("j13", "http", origin.url("/ok.mkv")),
                       {"x-attempt": "not-a-number"})
        await _wait(w, 3)
        outs = sorted(r.outcome for r in w.results)
        assert outs == ["dead", "dead", "staged"]
        assert len(b.drain("v1.download.dead")) == 2
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_stream_path_and_disk_fallback(run, make_cfg, origin_cls):
    """Single selector-approved HTTP file -> relayed origin->S3 (no disk); without Range
    support (multipart size) or with stream_http off it falls back to the disk path."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls)
        blob = os.urandom(13 * 1024 * 1024 + 11)
        origin.blobs["/v/big.mkv"] = blob
        await w.submit(api.make_download("st1", "http", origin.url("/v/big.mkv")))
        await _wait(w)
        key = keys.object_key("st1", "big.mkv")
        assert w.results[0].outcome == "staged" and s3.get("triton-staging", key) == blob
        ranged = [r for r in origin.requests if r[2]]
        assert len(ranged) == 3                     # 5 MiB parts -> 3 Range GETs relayed
        assert w.telemetry.progress_of("st1") == [0, 50, 100]
        # no Range support -> disk path (single GET)
        origin.no_ranges = True
        origin.requests.clear()
        await w.submit(api.make_download("st2", "http", origin.url("/v/big.mkv")))
        await _wait(w, 2)
        assert w.results[1].outcome == "staged"
        assert s3.get("triton-staging", keys.object_key("st2", "big.mkv")) == blob
        assert [r for r in origin.requests if r[0] == "GET" and r[2]] == []
        # non-media name -> never streamed, job fails in the process stage
        origin.no_ranges = False
        origin.blobs["/v/readme.txt"] = b"x" * 100
        w.cfg.broker.max_retries = 0
        await w.submit(api.make_download("st3", "http", origin.url("/v/readme.txt")))
        await _wait(w, 3)
        assert w.results[2].outcome == "dead"
        assert s3.get("triton-staging", keys.object_key("st3", "readme.txt")) is None
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_stream_source_failure_retries_cleanly(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 1})
        origin.blobs["/f.mkv"] = os.urandom(8 * 1024 * 1024)
        # part 2 fails 5 times: the client's 4 tries fail the first job attempt, the retry passes
        s3.faults.add(FaultRule(method="PUT", query_contains="partNumber=2", times=5,
                                status=500, code="InternalError"))
        await w.submit(api.make_download("st4", "http", origin.url("/f.mkv")))
        await _wait(w, 2)
        assert [r.outcome for r in w.results] == ["retried", "staged"]
        assert s3.get("triton-staging", keys.object_key("st4", "f.mkv")) == origin.blobs["/f.mkv"]
        assert not s3.uploads.get("triton-staging")   # failed attempt's upload was aborted
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_http_resume_after_truncated_transfer(run, make_cfg, origin_cls):
    """Attempt 1 is cut mid-body; the retry re-uses the job directory and continues with a
    Range request from the partial length (the reference restarts from 0)."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={"stream_http": False,
                                                                         "http_streams": 1})
        blob = os.urandom(3 * 1024 * 1024 + 5)
        origin.blobs["/r.mkv"] = blob
        origin.truncate.add("/r.mkv")
        await w.submit(api.make_download("rs1", "http", origin.url("/r.mkv")))
        await _wait(w, 1)
        assert w.results[0].outcome == "retried"
        origin.truncate.discard("/r.mkv")
        await _wait(w, 2)
        assert w.results[1].outcome == "staged"
        gets = [r for r in origin.requests if r[0] == "GET"]
        assert gets[-1][2] and gets[-1][2].startswith("bytes=") and gets[-1][2] != "bytes=0-"
        assert s3.get("triton-staging", keys.object_key("rs1", "r.mkv")) == blob
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_parallel_range_resume_skips_done_ranges(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={
            "stream_http": False, "http_streams": 4, "http_min_split": 1 << 20})
        blob = os.urandom(8 * 1024 * 1024)
        origin.blobs["/p.mkv"] = blob
        # the last of 4 ranges fails once: 3 ranges complete in attempt 1
        bad = f"bytes={3 * 2 * 1024 * 1024}-{len(blob) - 1}"
        origin.fail_ranges[bad] = 1
        await w.submit(api.make_download("rs2", "http", origin.url("/p.mkv")))
        await _wait(w, 2)
        assert [r.outcome for r in w.results] == ["retried", "staged"]
        ranged = [c[2] for c in origin.requests if c[0] == "GET" and c[2]]
        assert ranged.count("bytes=0-2097151") == 1       # done in attempt 1, skipped after
        assert ranged.count(bad) == 2
        assert s3.get("triton-staging", keys.object_key("rs2", "p.mkv")) == blob
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_multipart_upload_resume_reuses_parts(run, make_cfg, origin_cls):
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={"stream_http": False})
        blob = os.urandom(16 * 1024 * 1024 + 7)
        origin.blobs["/u.mkv"] = blob
        # part 3 fails on every try of attempt 1 (client retries 3 -> 4 faults)
        s3.faults.add(FaultRule(method="PUT", query_contains="partNumber=3", times=4,
                                status=500, code="InternalError"))
        part_puts = []
        s3.hooks.append(lambda m, p: part_puts.append(m))
        await w.submit(api.make_download("rs3", "http", origin.url("/u.mkv")))
        await _wait(w, 2)
        assert [r.outcome for r in w.results] == ["retried", "staged"]
        assert s3.get("triton-staging", keys.object_key("rs3", "u.mkv")) == blob
        # attempt 2 listed the open upload and only re-sent the missing part(s)
        assert any(m == "GET" for m in part_puts)
        assert not s3.uploads.get("triton-staging")
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_http_stall_floor_fails_slow_transfer(run, make_cfg, origin_cls):
    """A bytes/s floor (``download.http_min_rate``) turns a crawling origin into a failure the
    retry policy can handle (the reference has no HTTP stall detection at all)."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0},
                                        download={"stream_http": False, "http_streams": 1,
                                                  "http_min_rate": 1e6, "http_timeout_s": 0.5})
        origin.blobs["/crawl.mkv"] = os.urandom(4 * 1024 * 1024)
        origin.slow["/crawl.mkv"] = 100_000          # 100 kB/s < the 1 MB/s floor
        await w.submit(api.make_download("sl1", "http", origin.url("/crawl.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "dead"
        assert "B/s" in w.results[0].error
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_reaper_renames_then_unlinks_and_sweeps(tmp_path):
    from downloader_amd.stages.jobdir import Reaper
    root = tmp_path / "dl"
    job = root / "j1" / "Season 1"
    job.mkdir(parents=True)
    (job / "e1.mkv").write_bytes(os.urandom(1 << 20))
    r = Reaper(str(root))
    fut = r.reap(str(root / "j1"))
    assert not (root / "j1").exists()           # path free before the unlink finished
    fut.result(10)
    assert r.drain(10) and os.listdir(root / ".trash") == []
    # leftovers of a crashed worker are swept
    (root / ".trash" / "old.abcd" / "x").mkdir(parents=True)
    assert r.sweep() == 1 and r.drain(10)
    assert os.listdir(root / ".trash") == []
    r.close()
    # reference mode: inline removal, no trash
    (root / "j2").mkdir()
    inline = Reaper(str(root), background=False)
    assert inline.reap(str(root / "j2")) is None and not (root / "j2").exists()
    assert inline.reap(str(root / "missing")) is None


def test_signed_payload_staging(run, make_cfg, origin_cls):
    """s3.unsigned_payload=False (minio-js over plain HTTP; reference mode): every PUT and
    part carries its SHA-256, which FakeS3 checks against the body it received."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls,
                                        s3={"unsigned_payload": False},
                                        download={"stream_http": False})
        blob = os.urandom(13 * 1024 * 1024 + 7)           # > threshold: multipart, 3 parts
        origin.blobs["/m/signed.mkv"] = blob
        await w.submit(api.make_download("sig1", "http", origin.url("/m/signed.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        key = "sig1/original/" + base64.b64encode(b"signed.mkv").decode()
        assert s3.get("triton-staging", key) == blob
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_job_dir_names_stay_inside_the_root(tmp_path):
    """media.id comes from the queue: '', '.', '..', ids with '/' or NUL, dot-ids (which
    could hit .locks / .trash) and over-long ids get an encoded single component; plain ids
    keep the reference layout <root>/<id>."""
    from downloader_amd.stages.jobdir import JobDir, Reaper, dir_name, inside
    root = tmp_path / "dl"
    root.mkdir()
    assert dir_name("job1") == "job1" and dir_name("Some Movie (2019)") == "Some Movie (2019)"
    seen = set()
    for bad in ("", ".", "..", "../x", "a/b", "/", "x\0y", ".trash", ".locks", "%41",
                "é" * 300):
        n = dir_name(bad)
        assert n.startswith("%") and "/" not in n and "\0" not in n and len(n) <= 200, n
        assert n not in seen
        seen.add(n)
        jd = JobDir(str(root), bad)
        p = jd.acquire()
        assert inside(str(root), p) and os.path.dirname(p) == str(root)
        jd.release()
    # the reaper never removes the root, its parent or its own bookkeeping dirs
    (root / "other").mkdir()
    r = Reaper(str(root), background=False)
    for p in (str(root), str(tmp_path), str(root / "."), str(root / ".."),
              str(root / ".locks"), str(root / ".trash")):
        os.makedirs(root / ".trash", exist_ok=True)
        with pytest.raises(ValueError):
            r.reap(p)
    assert (root / "other").is_dir() and (root / ".locks").is_dir()
    jd = JobDir(str(root), "..")
    jd.path = str(root)          # a corrupted path is still not removed
    jd.remove()
    assert (root / "other").is_dir()


def test_dotdot_job_id_does_not_wipe_other_jobs(run, make_cfg, origin_cls, tmp_path):
    """A job whose id is '..' stages normally and its cleanup removes only its own dir."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls)
        keep = tmp_path / "dl" / "other-job"
        keep.mkdir(parents=True)
        (keep / "x.mkv").write_bytes(b"x")
        origin.blobs["/d.mkv"] = os.urandom(100_000)
        for jid in ("..", "."):
            await w.submit(api.make_download(jid, "http", origin.url("/d.mkv")))
        await _wait(w, 2)
        assert [r.outcome for r in w.results] == ["staged", "staged"], w.results
        reaper = w.services.extra.get("reaper")
        if reaper is not None:
            assert reaper.drain(10)
        assert (keep / "x.mkv").read_bytes() == b"x"
        assert (tmp_path / "dl").is_dir()
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_source_names_cannot_leave_the_job_dir(run, tmp_path):
    """bucket:// object names are joined under the job dir: '../<sibling>/x' passes a plain
    string-prefix check ('/dl/job' is a prefix of '/dl/job2') and must still be refused. An
    HTTP URL path ending in '..' names no file (Node's URL parser drops the segment)."""
    from downloader_amd.fetch.bucket import fetch_bucket
    from downloader_amd.fetch.http import output_name

    assert output_name("http://h/a/..") == "index" and output_name("http://h/a/%2E%2e") == "index"
    assert output_name("http://h/a/.") == "index" and output_name("http://h/x/m.mkv?q") == "m.mkv"

    async def go():
        s3 = FakeS3()
        await s3.start()
        s3.buckets["src"] = {}
        s3.put("src", "show/../job2/evil.mkv", b"evil")
        job = tmp_path / "dl" / "job"
        (tmp_path / "dl" / "job2").mkdir(parents=True)
        job.mkdir()
        uri = f"bucket://{s3.endpoint},src,minioadmin,minioadmin,show"
        with pytest.raises(ValueError, match="escapes"):
            await fetch_bucket(uri, str(job), secure=False)
        assert not (tmp_path / "dl" / "job2" / "evil.mkv").exists()
        await s3.stop()
    run(go())


def test_http_sources_follow_redirects(run, make_cfg, origin_cls):
    """request@2 follows up to 10 GET redirects (relative Locations too, Range kept). The
    stream relay, the disk path (parallel Range GETs) and .torrent URLs all land on the final
    URL; an 11-hop loop fails the job."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0})
        big = os.urandom(13 * 1024 * 1024 + 5)          # multipart: relayed in Range parts
        origin.blobs["/cdn/real/big.mkv"] = big
        origin.redirect["/v/big.mkv"] = (302, "/cdn/hop.mkv")
        origin.redirect["/cdn/hop.mkv"] = (307, "real/big.mkv")          # relative
        await w.submit(api.make_download("rd1", "http", origin.url("/v/big.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert w.results[0].stats.get("streamed")                  # relayed, no disk hop
        assert s3.get("triton-staging", keys.object_key("rd1", "big.mkv")) == big
        # disk path with parallel ranges: every Range GET carries its Range through the hops
        await w.stop()
        cfg = make_cfg(s3.endpoint, download={"stream_http": False, "http_streams": 3,
                                              "http_min_split": 4 << 20},
                       broker={"max_retries": 0})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        await w.submit(api.make_download("rd2", "http", origin.url("/v/big.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("rd2", "big.mkv")) == big
        ranged = [rg for m, p, rg in origin.requests if p == "/cdn/real/big.mkv" and m == "GET"]
        assert ranged and all(rg for rg in ranged)
        # a redirect loop is an error, not a hang
        for i in range(12):
            origin.redirect[f"/loop/{i}.mkv"] = (302, f"/loop/{i + 1}.mkv")
        await w.submit(api.make_download("rd3", "http", origin.url("/loop/0.mkv")))
        await _wait(w, 2)
        assert w.results[1].outcome == "dead" and "redirect" in w.results[1].error
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


class _ForwardProxy:
    """Minimal HTTP/1.1 forward proxy for tests: absolute-form requests (one per client
    connection, answered with Connection: close) and CONNECT tunnels; records what it saw."""

    def __init__(self):
        self.seen = []          # (request line, Proxy-Authorization)
        self.server = None
        self.port = 0

    async def start(self):
        self.server = await asyncio.start_server(self._client, "127.0.0.1", 0)
        self.port = self.server.sockets[0].getsockname()[1]
        return self

    async def _client(self, r, w):
        from urllib.parse import urlsplit
        try:
            head = await r.readuntil(b"\r\n\r\n")
            lines = head.decode("latin-1").split("\r\n")
            method, target, ver = lines[0].split(" ")
            auth = next((ln.split(":", 1)[1].strip() for ln in lines[1:]
                         if ln.lower().startswith("proxy-authorization:")), "")
            self.seen.append((lines[0], auth))
            if method == "CONNECT":
                host, _, port = target.rpartition(":")
                orr, ow = await asyncio.open_connection(host.strip("[]"), int(port))
                w.write(b"HTTP/1.1 200 Connection established\r\n\r\n")
                await w.drain()

                async def pump(src, dst):
                    try:
                        while True:
                            chunk = await src.read(1 << 16)
                            if not chunk:
                                break
                            dst.write(chunk)
                            await dst.drain()
                    finally:
                        dst.close()
                await asyncio.gather(pump(r, ow), pump(orr, w), return_exceptions=True)
                return
            u = urlsplit(target)
            keep = [ln for ln in lines[1:] if ln and not ln.lower().startswith(
                ("proxy-authorization:", "connection:"))]
            path = (u.path or "/") + ("?" + u.query if u.query else "")
            req = "\r\n".join([f"{method} {path} {ver}"] + keep + ["Connection: close", "", ""])
            orr, ow = await asyncio.open_connection(u.hostname, u.port or 80)
            ow.write(req.encode("latin-1"))
            await ow.drain()
            while True:
                chunk = await orr.read(1 << 16)
                if not chunk:
                    break
                w.write(chunk)
                await w.drain()
            ow.close()
        except Exception:
            pass
        finally:
            w.close()

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()


def test_http_source_through_forward_proxy(run, make_cfg, origin_cls):
    """download.http_proxy (request@2 honours HTTP_PROXY): source GETs - stream relay and
    disk path - go through the proxy in absolute form with Proxy-Authorization; S3 traffic
    does not."""
    async def go():
        proxy = await _ForwardProxy().start()
        purl = f"http://user:pw@127.0.0.1:{proxy.port}"
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={"http_proxy": purl})
        big = os.urandom(13 * 1024 * 1024 + 1)
        origin.blobs["/p/big.mkv"] = big
        await w.submit(api.make_download("px1", "http", origin.url("/p/big.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert w.results[0].stats.get("streamed")
        assert s3.get("triton-staging", keys.object_key("px1", "big.mkv")) == big
        await w.stop()
        cfg = make_cfg(s3.endpoint, download={"http_proxy": purl, "stream_http": False})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        await w.submit(api.make_download("px2", "http", origin.url("/p/big.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("px2", "big.mkv")) == big
        lines = [ln for ln, _ in proxy.seen]
        assert lines and all(f"http://127.0.0.1:{origin.port}/p/big.mkv" in ln for ln in lines)
        assert {a for _, a in proxy.seen} == {"Basic dXNlcjpwdw=="}
        assert any(ln.startswith("HEAD ") for ln in lines) and any(ln.startswith("GET ") for ln in lines)
        assert not any("triton-staging" in ln for ln in lines)
        await w.stop(); await proxy.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_proxy_env_selection():
    from downloader_amd.net.proxy import ProxyConfig, proxy_from_env
    env = {"HTTP_PROXY": "http://p:3128", "NO_PROXY": ".internal, cdn.example.com:8080,x.org"}
    assert proxy_from_env("http://a.example.com/x", env).port == 3128
    assert proxy_from_env("http://h.internal/x", env) is None
    assert proxy_from_env("http://internal/x", env) is None
    assert proxy_from_env("http://cdn.example.com:8080/x", env) is None
    assert proxy_from_env("http://cdn.example.com/x", env) is not None        # port differs
    assert proxy_from_env("http://sub.x.org/x", env) is None
    assert proxy_from_env("http://127.0.0.1:9/x", env) is None                 # loopback
    assert proxy_from_env("https://a.example.com/x", env).host == "p"          # https -> HTTP_PROXY
    assert proxy_from_env("https://a.b/x", {"HTTPS_PROXY": "s:1", "HTTP_PROXY": "p:2"}).host == "s"
    assert proxy_from_env("http://a.b/x", {"http_proxy": "p:2", "NO_PROXY": "*"}) is None
    assert proxy_from_env("http://a.b/x", {}) is None
    assert ProxyConfig("").for_url("http://a.b/") is None
    assert ProxyConfig("http://u:p@q:8").for_url("http://127.0.0.1/").auth.startswith("Basic ")
    assert ProxyConfig("env", {"HTTP_PROXY": "p:1"}).for_url("http://a.b/").port == 1


def test_complete_multipart_with_lost_reply(run, make_cfg, origin_cls):
    """CompleteMultipartUpload succeeds on the server but its reply is lost: the client's
    retry gets NoSuchUpload, finds the object with the matching multipart ETag, and the job
    is staged instead of failing (and retrying a job whose object is already in place)."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0},
                                        download={"stream_http": False})
        blob = os.urandom(13 * 1024 * 1024 + 9)
        origin.blobs["/lost/reply.mkv"] = blob
        s3.faults.add(FaultRule(method="POST", query_contains="uploadId", times=1,
                                drop_after=True))
        await w.submit(api.make_download("lr1", "http", origin.url("/lost/reply.mkv")))
        await _wait(w)
        assert w.results[0].outcome == "staged", w.results[0]
        o = s3.objects("triton-staging")[keys.object_key("lr1", "reply.mkv")]
        assert o.data == blob and o.etag.endswith("-3")
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


@pytest.mark.parametrize("validators", [True, False])
def test_http_resume_discards_partial_data_of_a_changed_origin(run, make_cfg, origin_cls,
                                                               validators):
    """Attempt 1 is cut mid-body; before the retry the origin serves ANOTHER file of the same
    size (new ETag). The partial data must not be spliced with the new bytes: the retry
    starts from 0. Without validators nothing is resumed at all."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls,
                                        download={"stream_http": False, "http_streams": 1})
        origin.no_validators = not validators
        old = os.urandom(3 * 1024 * 1024 + 5)
        new = os.urandom(len(old))
        origin.blobs["/v.mkv"] = old
        origin.truncate.add("/v.mkv")
        heads = []

        def swap(method, path):     # the retry's first request sees the new file
            if method == "HEAD" and path == "/v.mkv":
                heads.append(1)
                if len(heads) == 2:
                    origin.blobs["/v.mkv"] = new
                    origin.truncate.discard("/v.mkv")
        origin.hooks.append(swap)
        await w.submit(api.make_download("rv1", "http", origin.url("/v.mkv")))
        await _wait(w, 2)
        assert w.results[0].outcome == "retried"
        assert w.results[1].outcome == "staged", w.results[1]
        gets = [r for r in origin.requests if r[0] == "GET"]
        assert not gets[-1][2]                      # a full GET, no Range
        assert s3.get("triton-staging", keys.object_key("rv1", "v.mkv")) == new
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_complete_download_reused_only_for_the_same_origin_version(run, make_cfg, origin_cls):
    """Attempt 1 downloads the whole file but its upload fails; the retry reuses the file on
    disk only if the origin still reports the same ETag - here it changed, so it refetches."""
    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls,
                                        download={"stream_http": False, "http_streams": 1})
        old = os.urandom(2 * 1024 * 1024 + 1)
        new = os.urandom(len(old))
        origin.blobs["/c.mkv"] = old
        s3.faults.add(FaultRule(method="PUT", path_contains="/rc1/original/Yy5ta3Y=",
                                times=1, status=403, code="AccessDenied"))
        heads = []

        def swap(method, path):
            if method == "HEAD" and path == "/c.mkv":
                heads.append(1)
                if len(heads) == 2:
                    origin.blobs["/c.mkv"] = new
        origin.hooks.append(swap)
        await w.submit(api.make_download("rc1", "http", origin.url("/c.mkv")))
        await _wait(w, 2)
        assert [r.outcome for r in w.results] == ["retried", "staged"], w.results
        assert s3.get("triton-staging", keys.object_key("rc1", "c.mkv")) == new
        assert len([r for r in origin.requests if r[0] == "GET"]) == 2
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_not_enough_space_fails_before_fetching(run, make_cfg, origin_cls, tmp_path, monkeypatch):
    """Disk paths check free space first (stages/space.py): an HTTP file and a torrent that
    cannot fit fail with ENOSPC before their payload is fetched; stream staging is unaffected."""
    import collections
    import shutil as _shutil

    from downloader_amd.torrent.metainfo import make_torrent
    real = _shutil.disk_usage
    Usage = collections.namedtuple("Usage", "total used free")
    monkeypatch.setattr(_shutil, "disk_usage",
                        lambda p: Usage(real(p).total, real(p).used, 1_000_000))

    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, broker={"max_retries": 0},
                                        download={"stream_http": False,
                                                  "torrent_stream": "off"})
        origin.blobs["/big.mkv"] = os.urandom(3_000_000)
        src = tmp_path / "t.mkv"
        src.write_bytes(os.urandom(2_000_000))
        origin.blobs["/ws/t.mkv"] = src.read_bytes()
        origin.blobs["/t.torrent"] = make_torrent(str(src), 65536,
                                                  url_list=[origin.url("/ws/t.mkv")])
        await w.submit(api.make_download("ns1", "http", origin.url("/big.mkv")))
        await w.submit(api.make_download("ns2", "http", origin.url("/t.torrent")))
        await _wait(w, 2)
        for r in w.results:
            assert r.outcome == "dead" and "not enough space" in r.error, r
        gets = [(m, p) for m, p, *_ in origin.requests if m == "GET"]
        assert ("GET", "/big.mkv") not in gets
        assert not any(p.startswith("/ws/") for _, p in gets)
        await w.stop()
        # plenty of room again: the same HTTP job stages normally
        monkeypatch.setattr(_shutil, "disk_usage", real)
        w2 = Worker(make_cfg(s3.endpoint, download={"stream_http": False}), broker=MemoryBroker())
        await w2.start(health=False)
        await w2.submit(api.make_download("ns3", "http", origin.url("/big.mkv")))
        await _wait(w2)
        assert w2.results[0].outcome == "staged", w2.results[0]
        await w2.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_failed_bucket_relay_does_not_log_presigned_signature(run, make_cfg, origin_cls):
    """a bucket:// relay whose presigned source GET fails must not put the
    X-Amz-Signature / X-Amz-Credential of that URL into logs or the retry headers."""
    from downloader_amd.s3.fake_server import FaultRule
    from downloader_amd.utils.log import ListSink, set_default_sink, _default_sink

    async def go():
        s3, origin, b, w = await _setup(make_cfg, origin_cls, download={
            "bucket_secure": False, "bucket_server_copy": False}, broker={"max_retries": 0})
        s3.buckets["src"] = {}
        s3.put("src", "lib/Movie/m.mkv", os.urandom(100_000))
        s3.faults.add(FaultRule(method="GET", path_contains="/src/lib/Movie/m.mkv", times=10,
                                status=403, code="AccessDenied"))
        uri = f"bucket://{s3.endpoint},src,minioadmin,minioadmin,lib"
        await w.submit(api.make_download("leak", "bucket", uri, "MOVIE"))
        await _wait(w)
        assert w.results[0].outcome in ("dead", "failed"), w.results[0]
        dead = b.queues.get("v1.download.dead") or []
        await w.stop(); await s3.stop(); await origin.stop()
        return dead
    saved = _default_sink
    sink = ListSink()
    set_default_sink(sink)
    try:
        import os as _os
        old = _os.environ.get("LOG_LEVEL")
        _os.environ["LOG_LEVEL"] = "info"
        try:
            dead = run(go())
        finally:
            if old is None:
                _os.environ.pop("LOG_LEVEL", None)
            else:
                _os.environ["LOG_LEVEL"] = old
    finally:
        set_default_sink(saved)
    text = "\n".join(str(r) for r in sink.records)
    assert "answered HTTP 403" in text                       # the failure is logged ...
    assert "X-Amz-Signature=***" in text
    import re
    for m in re.finditer(r"X-Amz-(Signature|Credential)=([^&\s'\"]*)", text):
        assert m.group(2) == "***", text[m.start():m.start() + 80]
    for m in dead:
        err = m.headers.get("x-last-error", "")
        assert "X-Amz-Signature=" not in err or "X-Amz-Signature=***" in err


def test_lost_complete_reply_with_non_md5_part_etags_keeps_the_s3_error(run):
    """SSE-KMS / SSE-C part ETags are not MD5 hex; the NoSuchUpload recovery must
    re-raise the S3 error instead of a ValueError from computing the multipart ETag."""
    from downloader_amd.s3.client import ObjectInfo, S3Client, S3Error

    class Stub(S3Client):
        async def _request(self, *a, **kw):
            raise S3Error("NoSuchUpload", "gone", 404, "k", "b")

        async def head_object(self, bucket, key):
            return ObjectInfo(key, 10, "whatever-2")

    async def go():
        c = Stub("127.0.0.1:9", "a", "b")
        with pytest.raises(S3Error) as ei:
            await c.complete_multipart_upload("b", "k", "u", [(1, "kms-opaque-1"), (2, "x")])
        assert ei.value.code == "NoSuchUpload"
    run(go())
