"""Health / readiness / metrics HTTP server (reference lib/main.js:174-194, express).

``GET /health`` keeps the reference contract: 500 ``{"message":"Not Running Jobs"}`` when idle
(App. A #9, switchable with ``health.legacy_idle_500``), otherwise 200 ``{"metadata":
{"success": true, "host": <hostname>}, "data": {"active": n}}``. Added: ``/healthz`` (liveness),
``/readyz`` (broker connected, download consumer live, not draining) and ``/metrics`` (Prometheus exposition).
"""
from __future__ import annotations

from aiohttp import web

from ..utils.metrics import CONTENT_TYPE_LATEST


class HealthServer:
    def __init__(self, worker, hcfg):
        self.worker = worker
        self.cfg = hcfg
        self._runner = None
        self.port = hcfg.port

    async def start(self) -> int:
        app = web.Application()
        app.router.add_get("/health", self._health)
        app.router.add_get("/healthz", self._healthz)
        app.router.add_get("/readyz", self._readyz)
        app.router.add_get("/metrics", self._metrics)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.cfg.host, self.cfg.port, reuse_address=True)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        return self.port

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None

    async def _health(self, req: web.Request) -> web.Response:
        status, body = self.worker.health()
        return web.json_response(body, status=status)

    async def _healthz(self, req: web.Request) -> web.Response:
        return web.json_response({"ok": True})

    async def _readyz(self, req: web.Request) -> web.Response:
        """Ready = the broker connection is up AND the ``v1.download`` consumer is subscribed
        at the broker (a consumer cancelled by the broker, or whose channel the broker
        closed, receives nothing while the connection looks healthy) AND not draining."""
        b = self.worker.broker
        connected = bool(getattr(b, "connected", False))
        tag = self.worker._consumer
        consuming = connected and tag is not None and b.consumer_live(tag)
        ready = consuming and not self.worker._stopping
        return web.json_response({"ready": ready, "broker": connected, "consumer": consuming},
                                 status=200 if ready else 503)

    async def _metrics(self, req: web.Request) -> web.Response:
        return web.Response(body=self.worker.metrics.exposition(),
                            headers={"Content-Type": CONTENT_TYPE_LATEST})
