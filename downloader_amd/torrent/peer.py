"""BitTorrent peer wire protocol (BEP-3) with the extension protocol (BEP-10), ut_metadata
(BEP-9) and ut_pex (BEP-11) - replaces ``bittorrent-protocol@3``, ``ut_metadata`` and ``ut_pex``
from the reference's webtorrent stack (yarn.lock:389-398).

A ``PeerConn`` owns one TCP connection: it keeps a request pipeline full while unchoked and
interested, serves blocks of verified pieces to peers it has unchoked, and forwards
metadata/PEX traffic to the session.

With the session's native wire (``csrc/peerwire.cpp``, ``download.torrent_native_wire``) the
socket is handed over right after the handshake: native threads frame the messages, copy
PIECE payloads into the assembling piece and send what this class queues; this class keeps
every protocol decision (what to request, interest, choking, serving, extensions) and gets
the other messages, and the blocks that arrived, as events (``_wq``). Whole pieces the session
assigns to the connection are requested by the wire itself (``SwarmWire.assign``).
"""
from __future__ import annotations

import asyncio
import itertools
import os
import struct
import time
from typing import TYPE_CHECKING, Dict, Optional, Set, Tuple

from .bencode import bdecode_prefix, bencode
from .storage import Bitfield

if TYPE_CHECKING:  # pragma: no cover
    from .session import TorrentSession

PSTR = b"\x13BitTorrent protocol"
BLOCK = 16384
MAX_MSG = 2 * 1024 * 1024
CHOKE, UNCHOKE, INTERESTED, NOT_INTERESTED, HAVE, BITFIELD, REQUEST, PIECE, CANCEL, PORT = range(10)
EXTENDED = 20
# native wire event kinds (SwarmWire.poll) and this class' own queue markers
EV_MSG, EV_BLOCKS, EV_CLOSED, EV_PIECE, EV_NEED = 1, 2, 3, 4, 5
EV_FILL, EV_CANCEL_DUPS = 101, 102
# our extension message ids (what peers must use when talking to us)
UT_METADATA_ID = 1
UT_PEX_ID = 2
METADATA_PIECE = 16384


class ProtocolError(Exception):
    pass


def handshake_bytes(info_hash: bytes, peer_id: bytes, ext: bool = True, dht: bool = False) -> bytes:
    reserved = bytearray(8)
    if ext:
        reserved[5] |= 0x10
    if dht:
        reserved[7] |= 0x01
    return PSTR + bytes(reserved) + info_hash + peer_id


async def read_handshake(reader: asyncio.StreamReader, timeout: float = 10.0) -> Tuple[bytes, bytes, bytes]:
    data = await asyncio.wait_for(reader.readexactly(68), timeout)
    if data[:20] != PSTR:
        raise ProtocolError("not a BitTorrent handshake")
    return data[20:28], data[28:48], data[48:68]


# Connection ids (the native wire's connection key, session.peers and picker ownership):
# process-wide and never reused. self.cid was reused by CPython as soon as a PeerConn was
# freed, so a new connection could receive the events a detached one left behind.
_CONN_IDS = itertools.count(1)


class PeerConn:
    def __init__(self, session: "TorrentSession", reader: asyncio.StreamReader,
                 writer: asyncio.StreamWriter, addr: Tuple[str, int], remote_id: bytes,
                 reserved: bytes, outgoing: bool):
        self.cid = next(_CONN_IDS)
        self.s = session
        self.reader = reader
        self.writer = writer
        self.addr = addr
        self.remote_id = remote_id
        self.outgoing = outgoing
        self.supports_ext = bool(reserved[5] & 0x10)
        self.supports_dht = bool(reserved[7] & 0x01)
        self.ext: Dict[bytes, int] = {}
        self.metadata_size = 0
        self.listen_port = 0
        self.am_choking = True
        self.am_interested = False
        self.peer_choking = True
        self.peer_interested = False
        self.bitfield: Optional[Bitfield] = None
        self._raw_bitfield: Optional[bytes] = None
        self._early_haves: Set[int] = set()
        self.inflight: Dict[Tuple[int, int], float] = {}
        self.closed = False
        self.down_bytes = 0
        # receive rate (TorrentSession._rate_loop): the request pipeline is sized to the
        # peer's bandwidth-delay product, and a peer far slower than its share of the swarm
        # stops owning whole pieces (``slow``)
        self.rx_mark = 0
        self.rate: Optional[float] = None
        self.last_rate = 0.0
        # a new connection starts at 8 pipelines (slow start: the rate loop sizes it after its
        # first samples; a slow peer gives its requests back within ~1 s)
        self.depth = 8 * session.client.pipeline
        self.reqq = 0                  # the peer's advertised request queue (0: not said)
        self.slow = False
        self.slow_ticks = 0
        self.progress_t: Optional[float] = None   # last rate sample with bytes received
        self.up_bytes = 0
        self.hash_fails = 0
        self.connected_at = time.monotonic()
        self.last_rx = self.connected_at
        self._wlock = asyncio.Lock()
        self._out: list = []
        self._out_bytes = 0
        self._flush_due = False
        self.wire = None               # the session's SwarmWire once the socket is handed over
        self._wq: Optional[asyncio.Queue] = None
        self.fill_queued = False

    def attach_wire(self, wire) -> None:
        """Hand the socket to the native wire: asyncio stops reading it (what its buffer
        already holds goes along as the first bytes), native threads read and write it from
        here on, and events come back through the session (``TorrentSession._wire_drain``)."""
        transport = self.writer.transport
        sock = transport.get_extra_info("socket")
        if sock is None or transport.get_write_buffer_size():
            return          # (unsent asyncio bytes would be overtaken: stay on the Python path)
        transport.pause_reading()
        buf = getattr(self.reader, "_buffer", None)
        prefix = bytes(buf) if buf else b""
        if buf:
            buf.clear()
        fd = os.dup(sock.fileno())
        try:
            wire.attach(fd, self.cid, prefix)
        except Exception:
            os.close(fd)
            transport.resume_reading()
            raise
        self.wire = wire
        self._wq = asyncio.Queue()
        try:
            wire.set_conn_pipeline(self.cid, self.depth)
        except Exception:
            pass

    # ---------------------------------------------------------------- sending
    # Every message goes through one small output queue that is written out when the
    # connection's task next waits for input (``call_soon``), or at 256 KiB: a batch of
    # REQUESTs answered with 64 PIECE messages leaves in one write instead of 64 syscalls,
    # and message order is kept.
    def _frame(self, mid: int, payload: bytes = b"") -> bytes:
        return struct.pack(">IB", len(payload) + 1, mid) + payload

    def _queue(self, *parts) -> None:
        self._out.extend(parts)
        self._out_bytes += sum(len(x) for x in parts)
        if self._out_bytes >= 1 << 18:
            self._flush()
        elif not self._flush_due:
            self._flush_due = True
            asyncio.get_running_loop().call_soon(self._flush)

    def _flush(self) -> None:
        self._flush_due = False
        if self._out and not self.closed:
            if self.wire is not None:
                self.wire.sendv(self.cid, self._out)     # one copy, into the native queue
            else:
                self.writer.write(b"".join(self._out))
        self._out.clear()
        self._out_bytes = 0

    async def _maybe_drain(self) -> None:
        if self.wire is not None:
            while not self.closed and self.wire.pending_out(self.cid) > 1 << 20:
                await asyncio.sleep(0.001)
            return
        if self.writer.transport.get_write_buffer_size() > 1 << 20:
            async with self._wlock:
                await self.writer.drain()

    async def send(self, mid: int, payload: bytes = b"") -> None:
        if self.closed:
            return
        self._queue(self._frame(mid, payload))
        await self._maybe_drain()

    async def send_block(self, idx: int, begin: int, block: memoryview) -> None:
        """PIECE message with the block taken as a view of the cached piece (copied once,
        into the output write)."""
        if self.closed:
            return
        self._queue(struct.pack(">IBII", len(block) + 9, PIECE, idx, begin), block)
        await self._maybe_drain()

    async def send_ext(self, name: bytes, payload: bytes) -> None:
        mid = self.ext.get(name)
        if mid:
            await self.send(EXTENDED, bytes([mid]) + payload)

    async def send_ext_handshake(self) -> None:
        # reqq: the requests the native wire queues per connection before it calls it a flood
        # (csrc/peerwire.cpp kMaxServeQueue)
        d = {"m": {"ut_metadata": UT_METADATA_ID, "ut_pex": UT_PEX_ID}, "v": "downloader-amd 0.1",
             "reqq": 2048}
        if self.s.client.listen_port:
            d["p"] = self.s.client.listen_port
        if self.s.meta is not None:
            d["metadata_size"] = len(self.s.meta.raw_info)
        await self.send(EXTENDED, b"\x00" + bencode(d))

    async def send_bitfield(self) -> None:
        if self.s.have is not None and self.s.have.count:
            await self.send(BITFIELD, self.s.have.to_bytes())

    async def send_have(self, i: int) -> None:
        await self.send(HAVE, struct.pack(">I", i))

    async def set_interested(self, v: bool) -> None:
        if v != self.am_interested:
            self.am_interested = v
            await self.send(INTERESTED if v else NOT_INTERESTED)

    async def set_choking(self, v: bool) -> None:
        if v != self.am_choking:
            self.am_choking = v
            if self.wire is not None and v:
                self.wire.set_serving(self.cid, False)    # before the CHOKE is queued
            await self.send(CHOKE if v else UNCHOKE)
            if self.wire is not None and not v:
                self._flush()                             # the UNCHOKE goes out first, then
                self.wire.set_serving(self.cid, True)     # REQUESTs are served natively

    async def request(self, piece: int, begin: int, length: int) -> None:
        self.inflight[(piece, begin)] = time.monotonic()
        await self.send(REQUEST, struct.pack(">III", piece, begin, length))

    async def request_many(self, blocks) -> None:
        now = time.monotonic()
        frames = []
        for piece, begin, length in blocks:
            self.inflight[(piece, begin)] = now
            frames.append(self._frame(REQUEST, struct.pack(">III", piece, begin, length)))
        if self.closed:
            return
        self._queue(*frames)
        await self._maybe_drain()

    async def cancel(self, piece: int, begin: int, length: int) -> None:
        if self.inflight.pop((piece, begin), None) is not None:
            await self.send(CANCEL, struct.pack(">III", piece, begin, length))

    # ---------------------------------------------------------------- lifecycle
    def close(self) -> None:
        if self.closed:
            return
        try:
            self._flush()                 # queued messages still go out before the FIN
        except Exception:
            pass
        self.closed = True
        if self.wire is not None:
            try:
                self.wire.detach(self.cid)        # FIN, threads joined, its fd closed
            except Exception:
                pass
        try:
            self.writer.close()
        except Exception:
            pass

    async def _idle_watchdog(self) -> None:
        # One timer per connection instead of a wait_for() around every read (which costs a
        # task + timer handle per message on the hot path).
        period = max(1.0, self.s.idle_timeout / 4)
        while not self.closed:
            await asyncio.sleep(period)
            idle = time.monotonic() - self.last_rx
            if self.wire is not None and idle > self.s.idle_timeout:
                # blocks of a piece the wire requests itself are not reported one by one: ask
                # the wire when the socket last received
                try:
                    idle = min(idle, self.wire.rx_idle(self.cid))
                except Exception:
                    pass
            if idle > self.s.idle_timeout:
                self.close()
                return

    async def run(self) -> None:
        wd = asyncio.get_running_loop().create_task(self._idle_watchdog())
        read = self.reader.readexactly
        try:
            if self.supports_ext:
                await self.send_ext_handshake()
            await self.send_bitfield()
            if self.s.client.dht is not None and self.supports_dht:
                await self.send(PORT, struct.pack(">H", self.s.client.dht.port))
            if self._wq is not None:
                await self._run_wire()            # returns when the wire closed
            else:
                while not self.closed:
                    await self._read_batch(read)
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.TimeoutError, OSError,
                ProtocolError):
            pass
        except Exception:
            # A malformed message from the remote (short REQUEST/HAVE -> struct.error, a bad
            # bitfield, odd bencoding) ends this connection only. Escaping run() it would fail
            # the whole torrent session (outgoing peers) or reach the event loop's exception
            # handler and stop the worker (incoming peers).
            self.s.stats["peer_protocol_errors"] = self.s.stats.get("peer_protocol_errors", 0) + 1
        finally:
            wd.cancel()
            self.close()
            self.s.peer_closed(self)

    async def _read_batch(self, readexactly) -> None:
        """Read whatever the socket has (up to 1 MiB) and dispatch every message in it as a
        view of that one immutable chunk: no await and no copy per message (a 16 KiB block
        is copied once, into its piece). A message cut by the chunk's end is completed with
        ``readexactly`` and copied once."""
        data = await self.reader.read(1 << 20)
        if not data:
            raise asyncio.IncompleteReadError(b"", 4)
        self.last_rx = time.monotonic()
        mv = memoryview(data)
        end, pos = len(data), 0
        while pos < end:
            if end - pos < 4:                              # a cut length prefix
                hdr = bytes(mv[pos:]) + await readexactly(4 - (end - pos))
                n = int.from_bytes(hdr, "big")
                if n > MAX_MSG:
                    raise ProtocolError(f"message too large ({n})")
                if n:
                    body = await readexactly(n)
                    await self._dispatch(body[0], memoryview(body)[1:])
                return
            n = int.from_bytes(mv[pos:pos + 4], "big")
            if n > MAX_MSG:
                raise ProtocolError(f"message too large ({n})")
            pos += 4
            if n == 0:                                     # keep-alive
                continue
            if end - pos >= n:
                await self._dispatch(mv[pos], mv[pos + 1:pos + n])
                pos += n
            else:                                          # a cut message body
                body = bytes(mv[pos:]) + await readexactly(n - (end - pos))
                await self._dispatch(body[0], memoryview(body)[1:])
                return

    async def _run_wire(self) -> None:
        """Events of the native wire, in wire order: messages, endgame cancels and refills
        the session's drain queued for this connection, and the close."""
        q = self._wq
        while not self.closed:
            kind, data = await q.get()
            if kind == EV_MSG:
                if data:
                    await self._dispatch(data[0], memoryview(data)[1:])
            elif kind == EV_FILL:
                self.fill_queued = False
                await self.s.fill(self)
            elif kind == EV_CANCEL_DUPS:
                await self.s.cancel_dups(self, *data)
            elif kind == EV_CLOSED:
                return

    def attach_meta(self) -> None:
        """Called when metadata becomes known (magnet): materialise the bitfield."""
        if self.bitfield is not None or self.s.meta is None:
            return
        self.bitfield = Bitfield(self.s.meta.num_pieces)
        if self._raw_bitfield is not None:
            try:
                self.bitfield.load(self._raw_bitfield)
            except ValueError:
                pass
        for i in self._early_haves:
            if i < self.bitfield.n:
                self.bitfield.set(i)
        self._raw_bitfield = None
        self._early_haves.clear()
        self.s.picker.add_peer(self.bitfield, self.cid)

    # ---------------------------------------------------------------- receiving
    async def _dispatch(self, mid: int, p: memoryview) -> None:
        s = self.s
        if mid == PIECE:
            if len(p) < 8:
                raise ProtocolError("short piece message")
            idx, begin = struct.unpack(">II", p[:8])
            if self.inflight.pop((idx, begin), None) is not None or s.picker is not None:
                self.down_bytes += len(p) - 8
                # synchronous fast path (copy into the piece); a coroutine only for endgame
                # cancels or a completed piece
                if s.take_block(self, idx, begin, p[8:]):   # copied once, into the piece
                    await s.block_followup(self, idx, begin, len(p) - 8)
            if s.refill_due(self):
                await s.fill(self)
        elif mid == REQUEST:
            idx, begin, ln = struct.unpack(">III", p[:12])
            await s.serve_request(self, idx, begin, ln)
        elif mid == HAVE:
            idx = struct.unpack(">I", p[:4])[0]
            if self.bitfield is None:
                self._early_haves.add(idx)
            elif idx < self.bitfield.n and self.bitfield.set(idx):
                s.picker.inc(idx, self.cid)
                await s.update_interest(self)
                await s.fill(self)
        elif mid == BITFIELD:
            if s.meta is None:
                self._raw_bitfield = bytes(p)
            else:
                if self.bitfield is not None:
                    s.picker.remove_peer(self.bitfield, self.cid)
                self.bitfield = Bitfield(s.meta.num_pieces)
                self.bitfield.load(bytes(p))
                s.picker.add_peer(self.bitfield, self.cid)
                await s.update_interest(self)
                await s.fill(self)
        elif mid == UNCHOKE:
            self.peer_choking = False
            await s.fill(self)
        elif mid == CHOKE:
            self.peer_choking = True
            s.release_inflight(self)
        elif mid == INTERESTED:
            self.peer_interested = True
            await s.maybe_unchoke(self)
        elif mid == NOT_INTERESTED:
            self.peer_interested = False
        elif mid == CANCEL:
            pass  # blocks are sent as soon as they are read; nothing queued to cancel
        elif mid == PORT:
            port = struct.unpack(">H", p[:2])[0] if len(p) >= 2 else 0
            if s.client.dht is not None and port:
                s.client.dht.add_node_addr((self.addr[0], port))
        elif mid == EXTENDED:
            await self._extended(p)

    async def _extended(self, p: memoryview) -> None:
        if not p:
            return
        eid = p[0]
        if eid == 0:
            d, _ = bdecode_prefix(bytes(p[1:]))
            if not isinstance(d, dict):
                return
            m = d.get(b"m", {})
            if isinstance(m, dict):
                self.ext = {k: int(v) for k, v in m.items() if isinstance(v, int) and v > 0}
            # untrusted: a negative size or an out-of-range port counts as absent
            ms, lp = d.get(b"metadata_size", 0), d.get(b"p", 0)
            rq = d.get(b"reqq", 0)
            # BEP-10 reqq: requests it keeps without dropping; our pipeline to it stays below
            self.reqq = rq if isinstance(rq, int) and 0 < rq < 1 << 20 else 0
            self.metadata_size = ms if isinstance(ms, int) and ms > 0 else 0
            self.listen_port = lp if isinstance(lp, int) and 0 < lp < 65536 else 0
            if self.listen_port and not self.outgoing:
                self.s.add_peers([(self.addr[0], self.listen_port)], source="incoming")
            await self.s.on_ext_handshake(self)
        elif eid == UT_METADATA_ID:
            d, used = bdecode_prefix(bytes(p[1:]))
            await self.s.on_metadata_msg(self, d, bytes(p[1 + used:]))
        elif eid == UT_PEX_ID:
            d, _ = bdecode_prefix(bytes(p[1:]))
            self.s.on_pex(self, d)
