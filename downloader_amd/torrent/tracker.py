"""Tracker clients: HTTP (BEP-3, compact peers BEP-23) and UDP (BEP-15).

Replaces ``bittorrent-tracker@9`` (yarn.lock:402-430). WebSocket trackers (``ws://``,
``wss://``) only hand out WebRTC peers; bittorrent-tracker in Node without ``wrtc`` drops them
from the announce list, and so does ``supported`` here: a torrent whose only
trackers are WebSocket ones is treated as tracker-less instead of announcing to them forever.
"""
from __future__ import annotations

import asyncio
import random
import socket
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple
from urllib.parse import quote_from_bytes, urlsplit

from .bencode import bdecode

Peer = Tuple[str, int]


class TrackerError(Exception):
    pass


@dataclass
class AnnounceResult:
    interval: int = 1800
    peers: List[Peer] = field(default_factory=list)
    seeders: int = 0
    leechers: int = 0


def decode_compact(b: bytes) -> List[Peer]:
    return [(socket.inet_ntoa(b[i:i + 4]), struct.unpack(">H", b[i + 4:i + 6])[0])
            for i in range(0, len(b) - len(b) % 6, 6)]


def decode_compact6(b: bytes) -> List[Peer]:
    return [(socket.inet_ntop(socket.AF_INET6, b[i:i + 16]), struct.unpack(">H", b[i + 16:i + 18])[0])
            for i in range(0, len(b) - len(b) % 18, 18)]


def encode_compact(peers: List[Peer]) -> bytes:
    out = b""
    for h, p in peers:
        try:
            out += socket.inet_aton(h) + struct.pack(">H", p)
        except OSError:
            continue
    return out


async def announce_http(url: str, info_hash: bytes, peer_id: bytes, port: int, uploaded: int,
                        downloaded: int, left: int, event: str = "", numwant: int = 50,
                        transports=None, timeout: float = 15.0) -> AnnounceResult:
    q = (f"info_hash={quote_from_bytes(info_hash)}&peer_id={quote_from_bytes(peer_id)}"
         f"&port={port}&uploaded={uploaded}&downloaded={downloaded}&left={left}"
         f"&compact=1&numwant={numwant}")
    if event:
        q += f"&event={event}"
    full = url + ("&" if "?" in url else "?") + q
    if transports is not None:
        r = await asyncio.wait_for(transports.request("GET", full), timeout)
        status, body = r.status, r.body
    else:
        import aiohttp
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=timeout)) as s:
            async with s.get(full) as resp:
                status, body = resp.status, await resp.read()
    if status != 200:
        raise TrackerError(f"tracker HTTP {status}")
    return parse_announce_response(body)


def parse_announce_response(body: bytes) -> AnnounceResult:
    """BEP-3 / BEP-23 / BEP-7 announce response -> AnnounceResult. The body is untrusted:
    anything malformed (not a dict, wrong value types) is a TrackerError."""
    try:
        d = bdecode(body)
    except ValueError as e:
        raise TrackerError(f"bad tracker response: {e}") from e
    if not isinstance(d, dict):
        raise TrackerError("bad tracker response: not a dictionary")
    try:
        if b"failure reason" in d:
            raise TrackerError(bytes(d[b"failure reason"]).decode("utf-8", "replace"))
        res = AnnounceResult(int(d.get(b"interval", 1800)), [], int(d.get(b"complete", 0)),
                             int(d.get(b"incomplete", 0)))
    except (TypeError, ValueError) as e:
        raise TrackerError(f"bad tracker response: {e}") from e
    peers = d.get(b"peers", b"")
    if isinstance(peers, bytes):
        res.peers = decode_compact(peers)
    elif isinstance(peers, list):
        for p in peers:
            try:
                res.peers.append((bytes(p[b"ip"]).decode(), int(p[b"port"])))
            except (KeyError, ValueError, TypeError):
                continue
    if isinstance(d.get(b"peers6"), bytes):
        res.peers += decode_compact6(d[b"peers6"])
    return res


class _UdpProto(asyncio.DatagramProtocol):
    def __init__(self) -> None:
        self.q: asyncio.Queue = asyncio.Queue()

    def datagram_received(self, data: bytes, addr) -> None:
        self.q.put_nowait(data)

    def error_received(self, exc) -> None:
        self.q.put_nowait(exc)


UDP_MAGIC = 0x41727101980
EVENTS = {"": 0, "completed": 1, "started": 2, "stopped": 3}


async def announce_udp(url: str, info_hash: bytes, peer_id: bytes, port: int, uploaded: int,
                       downloaded: int, left: int, event: str = "", numwant: int = 50,
                       timeout: float = 3.0, retries: int = 2) -> AnnounceResult:
    u = urlsplit(url)
    loop = asyncio.get_running_loop()
    tr, proto = await loop.create_datagram_endpoint(_UdpProto, remote_addr=(u.hostname, u.port or 80))
    try:
        async def rt(packet: bytes, tid: int, want: int, min_len: int) -> bytes:
            for attempt in range(retries + 1):
                tr.sendto(packet)
                try:
                    while True:
                        data = await asyncio.wait_for(proto.q.get(), timeout * (2 ** attempt))
                        if isinstance(data, Exception):
                            raise TrackerError(str(data))
                        if len(data) >= 8 and struct.unpack(">I", data[4:8])[0] == tid:
                            action = struct.unpack(">I", data[:4])[0]
                            if action == 3:
                                raise TrackerError(data[8:].decode("utf-8", "replace"))
                            if action != want:
                                raise TrackerError(f"UDP tracker replied action {action}, "
                                                   f"expected {want}")
                            if len(data) < min_len:
                                raise TrackerError("short UDP tracker reply")
                            return data
                except asyncio.TimeoutError:
                    continue
            raise TrackerError("UDP tracker timeout")

        tid = random.getrandbits(32)
        data = await rt(struct.pack(">QII", UDP_MAGIC, 0, tid), tid, 0, 16)
        conn_id = struct.unpack(">Q", data[8:16])[0]
        tid = random.getrandbits(32)
        pkt = struct.pack(">QII20s20sQQQIIIiH", conn_id, 1, tid, info_hash, peer_id, downloaded,
                          left, uploaded, EVENTS.get(event, 0), 0, random.getrandbits(32),
                          numwant, port)
        data = await rt(pkt, tid, 1, 20)
        interval, leechers, seeders = struct.unpack(">III", data[8:20])
        # BEP-15: the peer list's address family is the one the tracker was reached over
        v6 = tr.get_extra_info("socket").family == socket.AF_INET6
        peers = (decode_compact6 if v6 else decode_compact)(data[20:])
        return AnnounceResult(interval, peers, seeders, leechers)
    finally:
        tr.close()


SCHEMES = ("http", "https", "udp")


def supported(url: str) -> bool:
    """True for tracker URLs this client can announce to (HTTP(S) and UDP)."""
    try:
        return urlsplit(url).scheme in SCHEMES
    except ValueError:
        return False


async def announce(url: str, *a, transports=None, **kw) -> AnnounceResult:
    scheme = urlsplit(url).scheme
    if scheme in ("http", "https"):
        return await announce_http(url, *a, transports=transports, **kw)
    if scheme == "udp":
        return await announce_udp(url, *a, **kw)
    raise TrackerError(f"unsupported tracker scheme {scheme!r}")


def random_peer_id(prefix: bytes = b"-DA0100-") -> bytes:
    return prefix + bytes(random.choice(b"0123456789abcdefghijklmnopqrstuvwxyz")
                          for _ in range(20 - len(prefix)))


def parse_peer(s: str) -> Optional[Peer]:
    h, _, p = s.rpartition(":")
    try:
        return h.strip("[]"), int(p)
    except ValueError:
        return None
