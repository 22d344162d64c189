"""Shared fixtures: fake S3, a local HTTP origin, config factory, gpu marker."""
from __future__ import annotations

import asyncio
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

os.environ.setdefault("LOG_LEVEL", "error")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture
def run():
    """Run a coroutine to completion on a fresh loop."""
    def _run(coro, timeout: float = 120.0):
        return asyncio.run(asyncio.wait_for(coro, timeout))
    return _run


class Origin:
    """aiohttp origin serving named blobs (Range + HEAD), optional faults."""

    def __init__(self, ssl_context=None):
        self.ssl_context = ssl_context
        self.blobs = {}
        self.runner = None
        self.port = 0
        self.requests = []
        self.fail_status = {}   # path -> status
        self.truncate = set()   # paths whose body is cut short
        self.no_ranges = False
        self.fail_ranges = {}   # Range header value -> remaining injected 503s
        self.slow = {}          # path -> bytes/s trickle rate
        self.chunked = set()
        self.corrupt = {}       # path -> [file offset, responses left]: flip that byte
        self.redirect = {}      # path -> (status, Location): answered before anything else
        self.no_validators = False   # True: no ETag (resume cannot be validated)
        self.hooks = []              # callables(method, path) run before each request
        self.ignore_if_match = False  # True: like servers that only honour If-Range
        self._etags = {}

    def _body(self, path: str, data: bytes, s: int, e: int) -> bytes:
        """data[s:e+1], with the byte of an armed ``corrupt`` fault flipped if covered."""
        body = data[s:e + 1]
        c = self.corrupt.get(path)
        if c and c[1] > 0 and s <= c[0] <= e:
            c[1] -= 1
            i = c[0] - s
            body = body[:i] + bytes([body[i] ^ 0xFF]) + body[i + 1:]
        return body

    def _etag(self, path, data):
        import hashlib
        hit = self._etags.get(path)
        if hit is None or hit[0] is not data:
            hit = (data, '"%s"' % hashlib.md5(data).hexdigest())
            self._etags[path] = hit
        return hit[1]

    async def _trickle(self, req, status, body, hdrs):
        from aiohttp import web
        rate = self.slow[req.path]
        resp = web.StreamResponse(status=status,
                                  headers=dict(hdrs, **{"Content-Length": str(len(body))}))
        await resp.prepare(req)
        step = max(1, int(rate / 20))
        for i in range(0, len(body), step):
            await resp.write(body[i:i + step])
            await asyncio.sleep(0.05)
        return resp

    async def start(self):
        from aiohttp import web

        async def handler(req: web.Request):
            self.requests.append((req.method, req.path_qs, req.headers.get("Range")))
            for h in self.hooks:
                h(req.method, req.path)
            if req.path in self.redirect:
                st, loc = self.redirect[req.path]
                return web.Response(status=st, headers={"Location": loc}, text="moved")
            if req.path in self.fail_status:
                return web.Response(status=self.fail_status[req.path], text="nope")
            data = self.blobs.get(req.path)
            if data is None:
                return web.Response(status=404, text="not found")
            hdrs = {} if self.no_ranges else {"Accept-Ranges": "bytes"}
            rng = req.headers.get("Range")
            if not self.no_validators:
                etag = hdrs["ETag"] = self._etag(req.path, data)
                im = req.headers.get("If-Match")
                if im and not self.ignore_if_match and im not in ("*", etag):
                    return web.Response(status=412, text="precondition failed")
                ir = req.headers.get("If-Range")
                if rng and ir and ir != etag:
                    rng = None                   # RFC 9110: changed -> the whole new body
            if rng and self.fail_ranges.get(rng, 0) > 0:
                self.fail_ranges[rng] -= 1
                return web.Response(status=503, text="injected range failure")
            if rng and not self.no_ranges:
                a, _, b = rng[6:].partition("-")
                s, e = int(a), int(b) if b else len(data) - 1
                hdrs["Content-Range"] = f"bytes {s}-{e}/{len(data)}"
                body = self._body(req.path, data, s, e)
                if req.path in self.slow:
                    return await self._trickle(req, 206, body, hdrs)
                return web.Response(status=206, body=body, headers=hdrs)
            if req.method == "HEAD":
                hdrs["Content-Length"] = str(len(data))
                return web.Response(status=200, headers=hdrs)
            if req.path in self.truncate:
                resp = web.StreamResponse(status=200, headers={"Content-Length": str(len(data))})
                await resp.prepare(req)
                await resp.write(data[: len(data) // 2])
                req.transport.close()
                return resp
            if req.path in self.slow:            # trickle the body at `slow[path]` bytes/s
                return await self._trickle(req, 200, data, {})
            if req.path in self.chunked:
                resp = web.StreamResponse(status=200)
                resp.enable_chunked_encoding()
                await resp.prepare(req)
                for i in range(0, len(data), 7777):
                    await resp.write(data[i:i + 7777])
                await resp.write_eof()
                return resp
            return web.Response(body=self._body(req.path, data, 0, len(data) - 1), headers=hdrs)

        app = web.Application()
        app.router.add_route("*", "/{tail:.*}", handler)
        self.runner = web.AppRunner(app, access_log=None)
        await self.runner.setup()
        site = web.TCPSite(self.runner, "127.0.0.1", 0, ssl_context=self.ssl_context)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]
        return self

    def url(self, path: str) -> str:
        scheme = "https" if self.ssl_context is not None else "http"
        return f"{scheme}://127.0.0.1:{self.port}{path}"

    async def stop(self):
        if self.runner is not None:
            await self.runner.cleanup()


@pytest.fixture
def origin_cls():
    return Origin


@pytest.fixture
def make_cfg(tmp_path):
    from downloader_amd.utils.config import load_config

    def _make(s3_endpoint: str = "127.0.0.1:9", **over):
        base = {"instance": {"download_path": str(tmp_path / "dl")},
                "s3": {"endpoint": s3_endpoint, "part_size": 5 << 20,
                       "multipart_threshold": 6 << 20},
                "broker": {"backend": "memory", "retry_backoff_s": 0.01},
                "health": {"enabled": False}}
        for k, v in over.items():
            if isinstance(v, dict) and isinstance(base.get(k), dict):
                base[k].update(v)
            else:
                base[k] = v
        return load_config(overrides=base, env={})
    return _make
