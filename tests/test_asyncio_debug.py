"""Python-side race/leak detection (SURVEY §5.2 asks for sanitizers on the native code; this
is the asyncio counterpart): whole jobs - HTTP relay, disk path, webseed torrent stream and
session staging, a failing job - run under asyncio debug mode, and nothing may be reported
as a never-awaited coroutine, a never-retrieved task exception, an unclosed transport or an
exception that reached the event loop's handler."""
from __future__ import annotations

import asyncio
import gc
import logging
import os
import warnings

from downloader_amd.broker.memory import MemoryBroker
from downloader_amd.models import api
from downloader_amd.s3.fake_server import FakeS3
from downloader_amd.service.worker import Worker
from downloader_amd.torrent.metainfo import make_torrent


def test_jobs_clean_under_asyncio_debug(tmp_path, make_cfg, origin_cls, caplog):
    problems = []

    async def go():
        loop = asyncio.get_running_loop()
        loop.set_debug(True)
        loop.slow_callback_duration = 10.0          # only correctness reports, not timing
        loop.set_exception_handler(lambda lp, ctx: problems.append(ctx.get("message")))
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        origin.blobs["/a/big.mkv"] = os.urandom(7 << 20)
        origin.blobs["/a/small.mkv"] = os.urandom(100_000)
        src = tmp_path / "src" / "Show" / "Season 1"
        src.mkdir(parents=True)
        (src / "e1.mkv").write_bytes(os.urandom(700_000))
        origin.blobs["/ws/Show/Season 1/e1.mkv"] = (src / "e1.mkv").read_bytes()
        origin.blobs["/t/s.torrent"] = make_torrent(str(tmp_path / "src" / "Show"), 65536,
                                                    url_list=[origin.url("/ws/")])
        jobs = [("d1", {}, "/a/big.mkv", "MOVIE"), ("d2", {"stream_http": False}, "/a/small.mkv", "MOVIE"),
                ("d3", {}, "/t/s.torrent", "TV"), ("d4", {"torrent_stream": "off"}, "/t/s.torrent", "TV"),
                ("d5", {}, "/a/missing.mkv", "MOVIE")]
        for jid, dl, path, typ in jobs:
            d = {"torrent_enable_dht": False, "progress_interval_s": 0.05}
            d.update(dl)
            w = Worker(make_cfg(ep, download=d, broker={"max_retries": 0}), broker=MemoryBroker())
            await w.start(health=False)
            await w.submit(api.make_download(jid, "http", origin.url(path), typ))
            for _ in range(1500):
                if w.results:
                    break
                await asyncio.sleep(0.02)
            want = "dead" if jid == "d5" else "staged"
            assert w.results and w.results[0].outcome == want, (jid, w.results)
            await w.stop()
        await s3.stop()
        await origin.stop()

    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        with caplog.at_level(logging.ERROR, logger="asyncio"):
            asyncio.run(asyncio.wait_for(go(), 120))
            gc.collect()
    bad = [str(w.message) for w in caught
           if "never awaited" in str(w.message) or "unclosed" in str(w.message).lower()]
    bad += [r.getMessage() for r in caplog.records if r.name == "asyncio"]
    assert not problems and not bad, (problems, bad)
