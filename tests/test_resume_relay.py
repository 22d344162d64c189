"""Resumable streamed relays (SURVEY §5.4 "resumable multipart (list parts on retry)"): a
relayed multipart upload that fails part-way keeps its upload and a journal; the retry of the
same object and source version relays only the parts the upload does not hold yet."""
from __future__ import annotations

import os

import pytest

from downloader_amd.s3.client import S3Client, S3Error
from downloader_amd.s3.fake_server import FakeS3
from downloader_amd.net.http import TransportError

CREDS = ("minioadmin", "minioadmin")
MiB = 1 << 20


def _rng(off: int, ln: int) -> str:
    return f"bytes={off}-{off + ln - 1}"


async def _setup(origin_cls, size=24 * MiB + 77):
    s3 = FakeS3()
    ep = await s3.start()
    origin = await origin_cls().start()
    blob = os.urandom(size)
    origin.blobs["/big.mkv"] = blob
    c = S3Client(ep, *CREDS, part_size=5 * MiB, multipart_threshold=6 * MiB, retries=1,
                 max_inflight_parts=2)
    await c.ensure_bucket("b")
    return s3, origin, c, blob


def test_failed_relay_resumes_from_the_journal(run, origin_cls):
    async def go():
        s3, origin, c, blob = await _setup(origin_cls)
        parts = c.plan_parts(len(blob))
        n, off, ln = parts[-1]
        origin.fail_ranges[_rng(off, ln)] = 99             # the last part's GET keeps failing
        v = origin._etag("/big.mkv", blob)
        with pytest.raises((TransportError, S3Error)):
            await c.relay_object("b", "o", origin.url("/big.mkv"), len(blob), validator=v,
                                 journal="j/o.json", keep_on_error=True)
        assert s3.get("b", "o") is None and s3.get("b", "j/o.json") is not None
        served = len(origin.requests)
        origin.fail_ranges.clear()
        st: dict = {}
        await c.relay_object("b", "o", origin.url("/big.mkv"), len(blob), validator=v,
                             journal="j/o.json", keep_on_error=True, stats=st)
        assert s3.get("b", "o") == blob
        assert st["resumed_parts"] == len(parts) - 1           # only the failed part again
        assert len(origin.requests) - served == 1
        assert s3.get("b", "j/o.json") is None                  # journal gone with the upload
        assert await c.find_upload("b", "o") is None
        await c.close(); await origin.stop(); await s3.stop()
    run(go())


def test_changed_version_or_no_keep_starts_over_and_cleans_up(run, origin_cls):
    async def go():
        s3, origin, c, blob = await _setup(origin_cls)
        parts = c.plan_parts(len(blob))
        n, off, ln = parts[-1]
        origin.fail_ranges[_rng(off, ln)] = 99
        with pytest.raises((TransportError, S3Error)):
            await c.relay_object("b", "o", origin.url("/big.mkv"), len(blob),
                                 validator=origin._etag("/big.mkv", blob),
                                 journal="j/o.json", keep_on_error=True)
        old = await c.find_upload("b", "o")
        assert old is not None
        origin.fail_ranges.clear()
        # the origin moved on to another version: nothing of the old upload is reused, and
        # the old upload is aborted rather than left behind
        blob = os.urandom(len(blob))
        origin.blobs["/big.mkv"] = blob
        st: dict = {}
        await c.relay_object("b", "o", origin.url("/big.mkv"), len(blob),
                             validator=origin._etag("/big.mkv", blob),
                             journal="j/o.json", keep_on_error=True, stats=st)
        assert s3.get("b", "o") == blob and "resumed_parts" not in st
        assert await c.find_upload("b", "o") is None
        # keep_on_error=False (the job's last attempt): a failure aborts and drops the journal
        origin.fail_ranges[_rng(off, ln)] = 99
        with pytest.raises((TransportError, S3Error)):
            await c.relay_object("b", "o2", origin.url("/big.mkv"), len(blob),
                                 validator=origin._etag("/big.mkv", blob),
                                 journal="j/o2.json", keep_on_error=False)
        assert await c.find_upload("b", "o2") is None and s3.get("b", "j/o2.json") is None
        await c.close(); await origin.stop(); await s3.stop()
    run(go())


def test_worker_retry_resumes_a_streamed_http_object(run, tmp_path, make_cfg, origin_cls):
    """End to end: the job's first attempt fails on one part, the broker-held retry resumes
    the upload (only that part is relayed again) and the staged object is byte-exact."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.service.worker import Worker

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(24 * MiB + 5)
        origin.blobs["/movie.mkv"] = blob
        cfg = make_cfg(ep, s3={"part_size": 5 * MiB, "multipart_threshold": 6 * MiB,
                               "retries": 0, "relay_resume_min_bytes": 10 * MiB},
                       broker={"retry_backoff_s": 0.05})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        c = w.s3
        parts = c.plan_parts(len(blob))
        n, off, ln = parts[2]
        origin.fail_ranges[_rng(off, ln)] = 1                  # one failure of part 3
        await w.submit(api.make_download("rs", "http", origin.url("/movie.mkv")))
        for _ in range(1500):
            if any(r.outcome == "staged" for r in w.results):
                break
            await asyncio.sleep(0.02)
        staged = [r for r in w.results if r.outcome == "staged"]
        assert staged, w.results
        assert s3.get("triton-staging", keys.object_key("rs", "movie.mkv")) == blob
        assert staged[0].stats.get("resumed_parts", 0) >= 1
        assert s3.get("triton-staging", keys.relay_journal_key("rs", "movie.mkv")) is None
        assert not [k for k in s3.objects("triton-staging") if "/original/" in k
                    and k != keys.object_key("rs", "movie.mkv") and not k.endswith("/done")]
        await w.stop(); await origin.stop(); await s3.stop()
    run(go())


def test_bucket_retry_skips_objects_already_staged(run, make_cfg, origin_cls):
    """A bucket:// season whose first attempt fails on one object: the retry HEADs the
    staged keys and skips the objects an earlier attempt staged from the same source version
    (x-amz-meta-stager-source), relaying only the rest; a changed source object is redone."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.service.worker import Worker

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        s3.buckets["src"] = {}
        eps = {f"e{i}.mkv": os.urandom((2 << 20) + i) for i in range(1, 5)}
        for n, d in eps.items():
            s3.put("src", f"lib/Show/Season 1/{n}", d)
        cfg = make_cfg(ep, download={"bucket_secure": False, "bucket_server_copy": False,
                                     "bucket_concurrency": 1},
                       s3={"retries": 0}, broker={"retry_backoff_s": 0.05})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        # e3's source GET fails (503) once: attempt 1 stages e1 and e2 (objects one at a
        # time), then fails; with S3 retries off the job itself is retried
        from downloader_amd.s3.fake_server import FaultRule
        s3.faults.add(FaultRule(method="GET", path_contains="e3.mkv", times=1))
        uri = f"bucket://{s3.endpoint},src,minioadmin,minioadmin,lib"
        await w.submit(api.make_download("bk", "bucket", uri, "TV"))
        for _ in range(1500):
            if any(r.outcome == "staged" for r in w.results):
                break
            await asyncio.sleep(0.02)
        staged = [r for r in w.results if r.outcome == "staged"]
        assert staged, w.results
        for n, d in eps.items():
            assert s3.get("triton-staging", keys.object_key("bk", n)) == d
        assert staged[0].stats.get("reused_objects", 0) >= 1
        await w.stop(); await origin.stop(); await s3.stop()
    run(go())


def test_bucket_failure_lets_objects_in_flight_finish(run, make_cfg, origin_cls):
    """Objects relayed in parallel: one fails while another is still moving. With a retry to
    come, the one in flight finishes (not cancelled), so the retry reuses it."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.s3.fake_server import FaultRule
    from downloader_amd.service.worker import Worker

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        s3.buckets["src"] = {}
        eps = {f"e{i}.mkv": os.urandom((2 << 20) + i) for i in range(1, 5)}
        for n, d in eps.items():
            s3.put("src", f"lib/Show/Season 1/{n}", d)
        cfg = make_cfg(ep, download={"bucket_secure": False, "bucket_server_copy": False,
                                     "bucket_concurrency": 4},
                       s3={"retries": 0}, broker={"retry_backoff_s": 0.05})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        s3.faults.add(FaultRule(method="GET", path_contains="e1.mkv", status=0, delay_s=0.4,
                                times=1))                  # e1 still moving when e3 fails
        s3.faults.add(FaultRule(method="GET", path_contains="e3.mkv", times=1))
        uri = f"bucket://{s3.endpoint},src,minioadmin,minioadmin,lib"
        await w.submit(api.make_download("bf", "bucket", uri, "TV"))
        for _ in range(1500):
            if any(r.outcome == "staged" for r in w.results):
                break
            await asyncio.sleep(0.02)
        staged = [r for r in w.results if r.outcome == "staged"]
        assert staged, w.results
        for n, d in eps.items():
            assert s3.get("triton-staging", keys.object_key("bf", n)) == d
        assert staged[0].stats.get("reused_objects", 0) == 3     # e1, e2, e4
        await w.stop(); await s3.stop()
    run(go())


def test_finished_jobs_sweep_stale_uploads(run, make_cfg, origin_cls):
    """Uploads a killed worker left open under a job's originals are aborted when the
    redelivered job is staged, and a dead-lettered job leaves neither uploads nor journals."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.service.worker import Worker

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(3 << 20)
        origin.blobs["/a.mkv"] = blob
        cfg = make_cfg(ep, s3={"retries": 0}, broker={"max_retries": 0})
        broker = MemoryBroker()
        w = Worker(cfg, broker=broker)
        await w.start(health=False)
        c = w.s3
        await c.ensure_bucket("triton-staging")
        # what a worker killed mid-relay leaves: an open upload (+ a journal)
        await c.create_multipart_upload("triton-staging", keys.object_key("sw", "a.mkv"))
        await c.put_object("triton-staging", keys.relay_journal_key("sw", "a.mkv"), b"{}")
        await c.create_multipart_upload("triton-staging", keys.object_key("swx", "a.mkv"))
        msg = api.make_download("sw", "http", origin.url("/a.mkv"))
        from collections import deque

        from downloader_amd.broker.memory import _Msg
        q = cfg.broker.download_queue      # redelivered: its first consumer died mid-job
        broker.queues.setdefault(q, deque()).append(_Msg(api.encode(msg), {}, redelivered=True))
        broker._pump(q)
        for _ in range(500):
            if w.results:
                break
            await asyncio.sleep(0.02)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert s3.get("triton-staging", keys.object_key("sw", "a.mkv")) == blob
        left = await c.list_uploads("triton-staging", "")
        assert [k for k, _ in left] == [keys.object_key("swx", "a.mkv")]   # other job untouched
        assert s3.get("triton-staging", keys.relay_journal_key("sw", "a.mkv")) is None
        assert r.stats["stale_uploads_aborted"] == 1
        assert w.metrics.sample("downloader_stale_uploads_aborted_total") == 1
        # a job that fails for good cleans up after itself too
        await c.create_multipart_upload("triton-staging", keys.object_key("sd", "b.mkv"))
        await w.submit(api.make_download("sd", "http", origin.url("/missing.mkv")))
        for _ in range(500):
            if len(w.results) > 1:
                break
            await asyncio.sleep(0.02)
        assert w.results[1].outcome == "dead", w.results
        assert [k for k, _ in await c.list_uploads("triton-staging", "")] == \
            [keys.object_key("swx", "a.mkv")]
        await w.stop(); await origin.stop(); await s3.stop()
    run(go())


def test_list_uploads_pages(run):
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        c = S3Client(ep, *CREDS)
        await c.ensure_bucket("b")
        ids = set()
        for i in range(7):
            k = f"j/original/k{i % 3}"
            ids.add((k, await c.create_multipart_upload("b", k)))
        await c.create_multipart_upload("b", "other/original/x")
        got = await c.list_uploads("b", "j/original/", page=2)
        assert sorted(got) == sorted(ids) and len(got) == 7
        assert (await c.find_upload("b", "other/original/x")) is not None
        await c.close(); await s3.stop()
    run(go())


def test_blobd_lists_open_uploads(run):
    """The bench peer answers ListMultipartUploads, so the stale-upload sweep works against it
    (and the chaos soak's open_uploads count is what the sweeps left)."""
    from downloader_amd.bench.infra import Blobd

    async def go():
        with Blobd(default_size=1 << 20) as blob:
            c = S3Client(blob.endpoint, *CREDS)
            await c.ensure_bucket("bk")
            a = await c.create_multipart_upload("bk", "j1/original/a")
            await c.create_multipart_upload("bk", "j2/original/b")
            assert await c.list_uploads("bk", "j1/original/") == [("j1/original/a", a)]
            await c.abort_multipart_upload("bk", "j1/original/a", a)
            assert await c.list_uploads("bk", "j1/") == []
            assert blob.stats()["open_uploads"] == 1
            await c.close()
    run(go())
