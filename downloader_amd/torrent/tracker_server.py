"""Minimal BitTorrent tracker (HTTP ``/announce`` + UDP BEP-15) for tests and benches - the
reference has no test infrastructure for its swarm path."""
from __future__ import annotations

import asyncio
import random
import struct
import time
from typing import Dict, Optional, Tuple
from urllib.parse import parse_qsl, unquote_to_bytes

from aiohttp import web

from .bencode import bencode
from .tracker import UDP_MAGIC, encode_compact

Peer = Tuple[str, int]


class Tracker:
    def __init__(self, host: str = "127.0.0.1", interval: int = 5):
        self.host = host
        self.interval = interval
        self.swarms: Dict[bytes, Dict[Peer, Tuple[float, int]]] = {}
        self.announces = 0
        self.http_port = 0
        self.udp_port = 0
        self._runner: Optional[web.AppRunner] = None
        self._udp: Optional[asyncio.DatagramTransport] = None
        self._conn_ids: Dict[int, float] = {}

    @property
    def http_url(self) -> str:
        return f"http://{self.host}:{self.http_port}/announce"

    @property
    def udp_url(self) -> str:
        return f"udp://{self.host}:{self.udp_port}/announce"

    def _record(self, ih: bytes, peer: Peer, left: int, event: str) -> list:
        self.announces += 1
        sw = self.swarms.setdefault(ih, {})
        if event == "stopped":
            sw.pop(peer, None)
        else:
            sw[peer] = (time.monotonic(), left)
        return [p for p in sw if p != peer]

    async def start(self) -> "Tracker":
        app = web.Application()
        app.router.add_get("/announce", self._http)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, 0)
        await site.start()
        self.http_port = site._server.sockets[0].getsockname()[1]
        loop = asyncio.get_running_loop()
        tracker = self

        class P(asyncio.DatagramProtocol):
            def connection_made(self, tr):
                self.tr = tr

            def datagram_received(self, data, addr):
                tracker._udp_packet(self.tr, data, addr)

        self._udp, _ = await loop.create_datagram_endpoint(P, local_addr=(self.host, 0))
        self.udp_port = self._udp.get_extra_info("sockname")[1]
        return self

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
        if self._udp is not None:
            self._udp.close()

    async def _http(self, req: web.Request) -> web.Response:
        raw = req.rel_url.raw_query_string
        q = {}
        for part in raw.split("&"):
            k, _, v = part.partition("=")
            q[k] = unquote_to_bytes(v)
        try:
            ih = q["info_hash"]
            port = int(q["port"])
            left = int(q.get("left", b"0"))
        except (KeyError, ValueError):
            return web.Response(body=bencode({"failure reason": "bad announce"}))
        ip = q.get("ip", b"").decode() or req.remote or "127.0.0.1"
        ev = q.get("event", b"").decode()
        peers = self._record(ih, (ip, port), left, ev)
        sw = self.swarms.get(ih, {})
        body = {"interval": self.interval, "peers": encode_compact(peers),
                "complete": sum(1 for _, l in sw.values() if l == 0),
                "incomplete": sum(1 for _, l in sw.values() if l > 0)}
        return web.Response(body=bencode(body), content_type="text/plain")

    def _udp_packet(self, tr, data: bytes, addr) -> None:
        if len(data) < 16:
            return
        conn, action, tid = struct.unpack(">QII", data[:16])
        if action == 0 and conn == UDP_MAGIC:
            cid = random.getrandbits(63)
            self._conn_ids[cid] = time.monotonic()
            tr.sendto(struct.pack(">IIQ", 0, tid, cid), addr)
        elif action == 1 and conn in self._conn_ids and len(data) >= 98:
            ih = data[16:36]
            left = struct.unpack(">Q", data[64:72])[0]
            ev = {1: "completed", 2: "started", 3: "stopped"}.get(struct.unpack(">I", data[80:84])[0], "")
            port = struct.unpack(">H", data[96:98])[0]
            peers = self._record(ih, (addr[0], port), left, ev)
            sw = self.swarms.get(ih, {})
            seed = sum(1 for _, l in sw.values() if l == 0)
            tr.sendto(struct.pack(">IIIII", 1, tid, self.interval, len(sw) - seed, seed)
                      + encode_compact(peers), addr)
        else:
            tr.sendto(struct.pack(">II", 3, tid) + b"bad request", addr)


def _unused(x) -> None:  # keep parse_qsl import for callers extending the tracker
    parse_qsl(x)
