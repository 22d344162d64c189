"""utils/aio.gather_strict: a failed fan-out leaves no sibling running (sibling Range GETs
would otherwise keep writing into a file descriptor the caller closes, sibling parts land in
an upload being aborted)."""
from __future__ import annotations

import asyncio

import pytest

from downloader_amd.utils.aio import gather_strict


def test_failure_cancels_and_awaits_siblings(run):
    async def go():
        state = {"started": 0, "finished": 0, "cancelled": 0}

        async def slow():
            state["started"] += 1
            try:
                await asyncio.sleep(5)
                state["finished"] += 1
            except asyncio.CancelledError:
                await asyncio.sleep(0.01)          # cleanup takes a moment
                state["cancelled"] += 1
                raise

        async def bad():
            await asyncio.sleep(0.01)
            raise ValueError("boom")

        with pytest.raises(ValueError):
            await gather_strict(slow(), bad(), slow())
        # both siblings have finished their cleanup by the time the error surfaces
        assert state == {"started": 2, "finished": 0, "cancelled": 2}
    run(go())


def test_keep_lets_siblings_finish(run):
    async def go():
        done = []

        async def ok(i):
            await asyncio.sleep(0.05)
            done.append(i)

        async def bad():
            raise RuntimeError("x")

        with pytest.raises(RuntimeError):
            await gather_strict(ok(1), bad(), ok(2), cancel=False)
        assert sorted(done) == [1, 2]
        assert await gather_strict(ok(3), ok(4)) == [None, None]
    run(go())


def test_outer_cancel_still_waits(run):
    async def go():
        state = {"cleaned": 0}

        async def slow():
            try:
                await asyncio.sleep(5)
            except asyncio.CancelledError:
                await asyncio.sleep(0.02)
                state["cleaned"] += 1
                raise

        t = asyncio.ensure_future(gather_strict(slow(), slow()))
        await asyncio.sleep(0.01)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        assert state["cleaned"] == 2
    run(go())


def test_failed_range_download_leaves_no_transfer_behind(run, tmp_path, origin_cls):
    """Parallel Range GETs, one of which fails: when download_to raises, no sibling GET is
    still running (it would keep writing into the closed .part descriptor)."""
    import os

    from downloader_amd.fetch.http import download_to
    from downloader_amd.net.http import make_transports

    async def go():
        origin = await origin_cls().start()
        blob = os.urandom(12 << 20)
        origin.blobs["/m.mkv"] = blob
        origin.slow["/m.mkv"] = 8 << 20                  # siblings trickle for ~0.5 s
        step = len(blob) // 3
        origin.fail_ranges[f"bytes={step}-{2 * step - 1}"] = 99
        t = make_transports()

        def ours():       # client-side tasks (the origin's own handler tasks excluded)
            return [x for x in asyncio.all_tasks() if "downloader_amd" in
                    getattr(getattr(x.get_coro(), "cr_code", None), "co_filename", "")]
        before = set(ours())
        with pytest.raises(Exception):
            await download_to(t, origin.url("/m.mkv"), str(tmp_path / "m.mkv"), streams=3,
                              min_split=1 << 20)
        assert not set(ours()) - before, ours()      # nothing new left running
        await t.close(); await origin.stop()
    run(go())


def test_run_settled_waits_and_discards(run):
    import threading
    import time

    from downloader_amd.utils.aio import run_settled

    async def go():
        done, discarded = threading.Event(), []

        def work():
            time.sleep(0.1)
            done.set()
            return "opened"

        t = asyncio.ensure_future(run_settled(work, discard=discarded.append))
        await asyncio.sleep(0.02)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        assert done.is_set() and discarded == ["opened"]     # waited, result handed back
        assert await run_settled(lambda: 7) == 7
    run(go())
