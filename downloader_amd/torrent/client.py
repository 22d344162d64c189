"""Torrent client: one per worker process (the reference keeps a module-level
``new Webtorrent()`` singleton, lib/download.js:19, shared by every job). It owns the TCP
listener for incoming peers, the optional DHT node and the transports; each job gets its own
``TorrentSession`` (no shared ``torrents`` map keyed by magnet, App. A #3/#7)."""
from __future__ import annotations

import asyncio
from typing import Dict, List, Optional, Sequence, Tuple

from .magnet import Magnet
from .metainfo import Metainfo
from .peer import PeerConn, handshake_bytes, read_handshake
from .session import TorrentError, TorrentSession
from .tracker import random_peer_id
from ..utils import membudget

Peer = Tuple[str, int]

# StreamReader buffer limit of a peer connection: reading pauses at 2x this. The default
# (64 KiB) paused/resumed the socket every few 16 KiB blocks - a recv and two epoll
# updates per ~80 KB at full rate.
PEER_READ_LIMIT = 4 << 20


class TorrentClient:
    def __init__(self, transports=None, peer_id: Optional[bytes] = None,
                 listen_host: str = "0.0.0.0", listen_port: int = 0, public_host: str = "",
                 max_peers: int = 32, max_uploads: int = 8, pipeline: int = 16,
                 enable_dht: bool = False, dht_bootstrap: Sequence[Peer] = (),
                 dht_port: int = 0, verify_backend: str = "auto", webseed_streams: int = 4,
                 webseed_chunk: int = 32 << 20, webseed_verify_depth: int = 2,
                 webseed_verify_depth_gpu: int = 32, verify_threads: int = 0,
                 webseed_max_failures: int = 5,
                 idle_timeout: float = 120.0, connect_timeout: float = 10.0,
                 seed_after_done: bool = False, listen: bool = True,
                 native_wire: bool = True, wire_verify_threads: int = 4,
                 swarm_verify: str = "auto", wire_requests: bool = True,
                 wire_pool_mb: int = 4096, wire_gpu_inflight: int = 1024,
                 swarm_gpu_min_bytes: int = 3 << 29, swarm_gpu_tail_bytes: int = -1,
                 swarm_backlog_bytes: int = 4 << 30, wire_io_threads: int = 4,
                 swarm_gpu_tail_x: float = 3.0, swarm_gpu_tail_max: float = 0.85):
        from ..net.http import make_transports
        self._own_transports = transports is None
        self.transports = transports or make_transports()
        self.peer_id = peer_id or random_peer_id()
        self.listen_host = listen_host
        self.listen_port = listen_port
        self.public_host = public_host
        self.max_peers = max_peers
        self.max_uploads = max_uploads
        self.pipeline = pipeline
        self.enable_dht = enable_dht
        self.dht_bootstrap = list(dht_bootstrap)
        self.dht_port = dht_port
        self.dht = None
        self.verify_backend = verify_backend
        self.webseed_streams = webseed_streams
        self.webseed_chunk = webseed_chunk
        self.webseed_verify_depth = webseed_verify_depth
        self.webseed_verify_depth_gpu = webseed_verify_depth_gpu
        self.verify_threads = verify_threads
        self.webseed_max_failures = webseed_max_failures
        self.idle_timeout = idle_timeout
        self.connect_timeout = connect_timeout
        self.seed_after_done = seed_after_done
        self.listen = listen
        # peer connections handed to the native wire after the handshake (csrc/peerwire.cpp)
        self.native_wire = native_wire
        self.wire_verify_threads = wire_verify_threads
        self.wire_io_threads = wire_io_threads    # epoll threads of a session's native wire
        self.swarm_verify = swarm_verify          # auto / gpu / cpu (native wire only)
        # whole pieces requested by the native wire itself (SwarmWire.assign), not per block
        self.wire_requests = wire_requests
        self.wire_gpu_inflight = wire_gpu_inflight   # device-verified pieces at once (GPU mode)
        self.swarm_gpu_min_bytes = swarm_gpu_min_bytes   # `auto`: device from this size up
        # GPU mode: the last bytes on the host (-1: sized by the measured device latency)
        self.swarm_gpu_tail_bytes = swarm_gpu_tail_bytes
        self.swarm_gpu_tail_x = swarm_gpu_tail_x         # auto tail: x the device's latency
        self.swarm_gpu_tail_max = swarm_gpu_tail_max     # auto tail: share of the torrent, max
        self.swarm_backlog_bytes = swarm_backlog_bytes   # complete, unverified pieces at most
        if native_wire:
            try:
                from ..ops import native
                native().swarm_piece_pool_limit(max(0, wire_pool_mb) << 20)
            except Exception:
                pass
        self.pex_interval = 60.0
        self.piece_cache_bytes = 64 << 20   # per-session LRU of pieces being served to peers
        self.dht_interval = 30.0
        self.max_announce_interval = 300.0
        self.sessions: Dict[bytes, TorrentSession] = {}
        self._server: Optional[asyncio.AbstractServer] = None
        self._conn_tasks: set = set()

    @classmethod
    def from_config(cls, cfg, transports=None, **kw) -> "TorrentClient":
        d = cfg.download
        boot = kw.pop("dht_bootstrap", None)
        if boot is None and d.torrent_dht_bootstrap:
            boot = [_hostport(x) for x in d.torrent_dht_bootstrap]
        return cls(transports=transports, listen_port=d.torrent_listen_port,
                   max_peers=d.torrent_max_peers, pipeline=d.torrent_request_pipeline,
                   enable_dht=d.torrent_enable_dht, verify_backend=d.verify_backend,
                   webseed_streams=max(1, d.webseed_streams or d.http_streams),
                   webseed_chunk=d.webseed_chunk, webseed_verify_depth=d.webseed_verify_depth,
                   webseed_verify_depth_gpu=d.webseed_verify_depth_gpu,
                   verify_threads=d.verify_threads,
                   native_wire=d.torrent_native_wire,
                   swarm_verify=d.swarm_verify_backend,
                   wire_requests=d.torrent_wire_requests,
                   wire_verify_threads=d.swarm_verify_threads,
                   wire_io_threads=d.swarm_wire_io_threads,
                   wire_pool_mb=membudget.swarm_bytes(d.swarm_pool_mb) >> 20,
                   wire_gpu_inflight=d.swarm_gpu_inflight,
                   swarm_gpu_min_bytes=int(d.swarm_gpu_min_gb * (1 << 30)),
                   swarm_gpu_tail_bytes=(d.swarm_gpu_tail_mb << 20) if d.swarm_gpu_tail_mb >= 0
                   else -1, swarm_gpu_tail_x=d.swarm_gpu_tail_x,
                   swarm_gpu_tail_max=d.swarm_gpu_tail_max,
                   swarm_backlog_bytes=membudget.swarm_bytes(d.swarm_backlog_mb),
                   dht_bootstrap=boot if boot is not None else DEFAULT_BOOTSTRAP, **kw)

    async def start(self) -> "TorrentClient":
        if self.listen:
            self._server = await asyncio.start_server(self._incoming, self.listen_host,
                                                      self.listen_port, reuse_address=True,
                                                      limit=PEER_READ_LIMIT)
            self.listen_port = self._server.sockets[0].getsockname()[1]
        if self.enable_dht:
            from .dht import DHTNode
            self.dht = DHTNode(port=self.dht_port, bootstrap=self.dht_bootstrap)
            await self.dht.start()
        return self

    async def close(self) -> None:
        for s in list(self.sessions.values()):
            await s.close()
        self.sessions.clear()
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()
        for t in list(self._conn_tasks):
            t.cancel()
        if self.dht is not None:
            await self.dht.close()
        if self._own_transports:
            await self.transports.close()

    # ---------------------------------------------------------------- sessions
    def _register(self, s: TorrentSession) -> TorrentSession:
        if s.info_hash in self.sessions:
            raise TorrentError("torrent already active in this worker")
        self.sessions[s.info_hash] = s
        return s

    async def add_torrent(self, meta: Metainfo, root: str, peers: Sequence[Peer] = (),
                          extra_webseeds: Sequence[str] = ()) -> TorrentSession:
        s = self._register(TorrentSession(self, meta.info_hash, root, meta, peers=peers,
                                          webseeds=extra_webseeds))
        await s.start()
        return s

    async def add_magnet(self, m: Magnet, root: str) -> TorrentSession:
        s = self._register(TorrentSession(self, m.info_hash, root, None, m.trackers, m.webseeds,
                                          m.peers, m.name, m.exact_sources))
        await s.start()
        return s

    async def remove(self, s: TorrentSession) -> None:
        self.sessions.pop(s.info_hash, None)
        await s.close()

    # ---------------------------------------------------------------- peers
    async def connect_peer(self, s: TorrentSession, addr: Peer) -> PeerConn:
        r, w = await asyncio.wait_for(asyncio.open_connection(addr[0], addr[1],
                                                              limit=PEER_READ_LIMIT),
                                      self.connect_timeout)
        try:
            w.write(handshake_bytes(s.info_hash, self.peer_id, True, self.dht is not None))
            await w.drain()
            reserved, ih, pid = await read_handshake(r, self.connect_timeout)
            if ih != s.info_hash:
                raise TorrentError("peer answered for another torrent")
        except BaseException:
            w.close()
            raise
        pc = PeerConn(s, r, w, addr, pid, reserved, outgoing=True)
        if not s.register_peer(pc):
            w.close()
            raise TorrentError("peer rejected (duplicate or full)")
        return pc

    async def _incoming(self, r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
        t = asyncio.current_task()
        self._conn_tasks.add(t)
        try:
            try:
                reserved, ih, pid = await read_handshake(r, self.connect_timeout)
            except Exception:
                w.close()
                return
            s = self.sessions.get(ih)
            if s is None or s._closed:
                w.close()
                return
            w.write(handshake_bytes(ih, self.peer_id, True, self.dht is not None))
            peer = w.get_extra_info("peername") or ("?", 0)
            pc = PeerConn(s, r, w, (peer[0], peer[1]), pid, reserved, outgoing=False)
            if not s.register_peer(pc):
                w.close()
                return
            await pc.run()
        except Exception:
            # never let a remote connection's failure reach the loop's exception handler
            # (it stops the worker): drop the connection
            w.close()
        finally:
            self._conn_tasks.discard(t)


DEFAULT_BOOTSTRAP: List[Peer] = [("router.bittorrent.com", 6881), ("dht.transmissionbt.com", 6881),
                                 ("router.utorrent.com", 6881)]


def _hostport(s: str) -> Peer:
    """``host:port`` (``[v6]:port``) of a DHT bootstrap node."""
    h, _, p = s.strip().rpartition(":")
    return h.strip("[]"), int(p)
