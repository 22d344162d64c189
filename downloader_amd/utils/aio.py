"""Structured fan-out for the staging paths.

``asyncio.gather`` raises the first failure but leaves the other awaitables running. For
the stager that is a resource bug, not a style point: sibling Range GETs keep splicing
into a file descriptor the caller closes on the way out (and the kernel may hand that fd
number to something else), sibling parts land in a multipart upload that is being aborted,
or a retry lists an upload's parts while the previous attempt is still adding to it.

``gather_strict`` waits for every sibling before it re-raises, so a failed fan-out has no
work left behind when it returns. The reference has no fan-out (one GET per file,
lib/download.js:159-160; uploads in a sequential loop, lib/upload.js:40-56); this is the
contract the parallel paths keep instead.
"""
from __future__ import annotations

import asyncio
from typing import Any, Awaitable, Callable, Iterable, List, Optional


async def drain(tasks: Iterable[asyncio.Future]) -> bool:
    """Wait until every task is done, whatever happens to the caller meanwhile. Returns True
    when the caller was cancelled during the wait (the caller re-raises after cleanup)."""
    tasks = list(tasks)
    interrupted = False
    while True:
        pending = [t for t in tasks if not t.done()]
        if not pending:
            break
        try:
            await asyncio.wait(pending)
        except asyncio.CancelledError:
            interrupted = True
    for t in tasks:                      # mark secondary failures as retrieved
        if not t.cancelled():
            t.exception()
    return interrupted


async def gather_strict(*aws: Awaitable[Any], cancel: bool = True) -> List[Any]:
    """Like ``asyncio.gather`` (results in order, first failure raised), but when one branch
    fails the others are cancelled (``cancel=True``) or allowed to finish (``cancel=False``)
    - and in both cases awaited - before the exception propagates. A cancellation of the
    caller always cancels every branch (``gather`` forwards it) and likewise waits for them."""
    tasks = [asyncio.ensure_future(a) for a in aws]
    try:
        return list(await asyncio.gather(*tasks))      # noqa: settled below
    except BaseException:
        if cancel:
            for t in tasks:
                t.cancel()
        await drain(tasks)
        raise


async def run_settled(fn: Callable[..., Any], *args: Any,
                      discard: Optional[Callable[[Any], None]] = None) -> Any:
    """``fn(*args)`` on the default executor. A cancellation of the caller returns only
    after the thread is done (it may be writing into a directory or descriptor the caller
    releases next); a result that arrives after the cancellation goes to ``discard`` (e.g.
    close the files it opened) instead of being dropped."""
    fut = asyncio.get_running_loop().run_in_executor(None, fn, *args)
    try:
        return await asyncio.shield(fut)
    except asyncio.CancelledError:
        await drain([fut])
        if discard is not None and not fut.cancelled() and fut.exception() is None:
            discard(fut.result())
        raise
