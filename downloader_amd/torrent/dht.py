"""Mainline DHT node (BEP-5) - replaces ``bittorrent-dht@9`` + ``k-rpc`` + ``k-bucket``
(yarn.lock:367,1912-1936).

KRPC over UDP with bencoded ``ping`` / ``find_node`` / ``get_peers`` / ``announce_peer`` in both
directions. The routing table keeps up to ``k`` nodes per XOR-distance bucket (160 buckets).
BEP-5 keeps good nodes over new ones: a full bucket only admits a newcomer by evicting a node
not heard from for ``STALE_S`` (the "ping the questionable node" step is simplified to "a
questionable node loses its slot"), so a flood of queries under fresh ids cannot flush the
nodes a lookup relies on. ``get_peers`` runs the iterative alpha=3 lookup, collects ``values``
and then announces to the closest nodes that returned tokens. A reply is accepted only from
the address the query went to (a guessed 16-bit transaction id from elsewhere is dropped), and
announced peers expire after ``PEER_TTL_S`` as in BEP-5.
"""
from __future__ import annotations

import asyncio
import hashlib
import os
import socket
import struct
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Set, Tuple

from .bencode import BencodeError, bdecode, bencode

Addr = Tuple[str, int]
K = 8
ALPHA = 3
STORE_MAX_TORRENTS = 10000      # announce_peer store bounds (any node can announce)
STORE_MAX_PEERS = 200
STALE_S = 15 * 60               # BEP-5: a node unheard-from for 15 minutes is questionable
PEER_TTL_S = 30 * 60            # announced peers are forgotten after 30 minutes


def distance(a: bytes, b: bytes) -> int:
    return int.from_bytes(a, "big") ^ int.from_bytes(b, "big")


def bucket_index(own: bytes, other: bytes) -> int:
    d = distance(own, other)
    return d.bit_length() - 1 if d else 0


@dataclass
class Node:
    id: bytes
    addr: Addr
    seen: float


def _is_id(x) -> bool:
    return isinstance(x, bytes) and len(x) == 20


def pack_nodes(nodes: Sequence[Node]) -> bytes:
    out = b""
    for n in nodes:
        try:
            out += n.id + socket.inet_aton(n.addr[0]) + struct.pack(">H", n.addr[1])
        except OSError:
            continue
    return out


def unpack_nodes(b: bytes) -> List[Node]:
    """Compact node info from a reply. These nodes are second-hand (a third party vouches
    for them), so they carry ``seen=0`` - questionable - and are lookup candidates only: a
    node enters the routing table when it answers us itself (``query``) or queries us."""
    return [Node(b[i:i + 20], (socket.inet_ntoa(b[i + 20:i + 24]),
                               struct.unpack(">H", b[i + 24:i + 26])[0]), 0.0)
            for i in range(0, len(b) - len(b) % 26, 26)]


def pack_peer(addr: Addr) -> bytes:
    return socket.inet_aton(addr[0]) + struct.pack(">H", addr[1])


def unpack_peer(b: bytes) -> Optional[Addr]:
    if len(b) != 6:
        return None
    return socket.inet_ntoa(b[:4]), struct.unpack(">H", b[4:])[0]


class RoutingTable:
    def __init__(self, own: bytes, k: int = K):
        self.own = own
        self.k = k
        self.buckets: List[List[Node]] = [[] for _ in range(160)]

    def add(self, n: Node) -> None:
        """Insert / refresh ``n``, which must have been heard from directly (it answered or
        queried us from ``n.addr``). A known id keeps its address while that entry is good:
        another host claiming the id cannot re-point it (BEP-5 node-id hijack)."""
        if n.id == self.own or len(n.id) != 20 or n.addr[1] == 0 or n.seen <= 0:
            return
        b = self.buckets[bucket_index(self.own, n.id)]
        for i, x in enumerate(b):
            if x.id == n.id:
                if x.addr != n.addr and n.seen - x.seen < STALE_S:
                    return
                b[i] = n
                return
        if len(b) >= self.k:
            oldest = min(range(len(b)), key=lambda i: b[i].seen)
            if n.seen - b[oldest].seen < STALE_S:
                return                   # every resident node is still good: keep them
            b.pop(oldest)
        b.append(n)

    def remove(self, node_id: bytes) -> None:
        b = self.buckets[bucket_index(self.own, node_id)]
        b[:] = [x for x in b if x.id != node_id]

    def closest(self, target: bytes, n: int = K) -> List[Node]:
        allnodes = [x for b in self.buckets for x in b]
        allnodes.sort(key=lambda x: distance(x.id, target))
        return allnodes[:n]

    def __len__(self) -> int:
        return sum(len(b) for b in self.buckets)


class DHTNode(asyncio.DatagramProtocol):
    def __init__(self, node_id: Optional[bytes] = None, host: str = "0.0.0.0", port: int = 0,
                 bootstrap: Sequence[Addr] = (), timeout: float = 2.0):
        self.id = node_id or hashlib.sha1(os.urandom(20)).digest()
        self.host = host
        self.port = port
        self.bootstrap_nodes = list(bootstrap)
        self.timeout = timeout
        self.table = RoutingTable(self.id)
        self.store: Dict[bytes, Dict[Addr, float]] = {}
        self._pending: Dict[bytes, Tuple[asyncio.Future, Addr]] = {}
        self._tasks: Set[asyncio.Task] = set()
        self._tid = 0
        self._secret = os.urandom(16)
        self._old_secret = self._secret
        self._secret_t = time.monotonic()
        self.transport: Optional[asyncio.DatagramTransport] = None
        self.queries_served = 0
        self.bad_packets = 0

    # ---------------------------------------------------------------- lifecycle
    async def start(self) -> "DHTNode":
        loop = asyncio.get_running_loop()
        self.transport, _ = await loop.create_datagram_endpoint(
            lambda: self, local_addr=(self.host, self.port))
        self.port = self.transport.get_extra_info("sockname")[1]
        if self.bootstrap_nodes:
            await self.bootstrap()
        return self

    async def bootstrap(self) -> None:
        loop = asyncio.get_running_loop()
        addrs: List[Addr] = []
        for h, p in self.bootstrap_nodes:
            try:
                infos = await asyncio.wait_for(loop.getaddrinfo(h, p, type=socket.SOCK_DGRAM,
                                                                family=socket.AF_INET), 2.0)
                addrs += [(i[4][0], i[4][1]) for i in infos[:1]]
            except Exception:
                continue
        await asyncio.gather(*(self._find_node_at(a, self.id) for a in addrs),
                             return_exceptions=True)
        if len(self.table):
            await self.lookup(self.id, want_peers=False)

    async def close(self) -> None:
        for f, _a in self._pending.values():
            if not f.done():
                f.cancel()
        for task in list(self._tasks):
            task.cancel()
        if self.transport is not None:
            self.transport.close()

    # ---------------------------------------------------------------- KRPC plumbing
    def _token(self, ip: str, secret: Optional[bytes] = None) -> bytes:
        if time.monotonic() - self._secret_t > 300:
            self._old_secret, self._secret = self._secret, os.urandom(16)
            self._secret_t = time.monotonic()
        return hashlib.sha1((secret or self._secret) + ip.encode()).digest()[:8]

    def _valid_token(self, ip: str, tok: bytes) -> bool:
        return tok in (self._token(ip), self._token(ip, self._old_secret))

    def _send(self, msg: dict, addr: Addr) -> None:
        if self.transport is not None:
            self.transport.sendto(bencode(msg), addr)

    async def query(self, addr: Addr, q: str, args: dict) -> dict:
        self._tid = (self._tid + 1) & 0xFFFF
        t = struct.pack(">H", self._tid)
        fut = asyncio.get_running_loop().create_future()
        self._pending[t] = (fut, (addr[0], addr[1]))
        a = dict(args)
        a["id"] = self.id
        self._send({"t": t, "y": "q", "q": q, "a": a}, addr)
        try:
            r = await asyncio.wait_for(fut, self.timeout)
        finally:
            self._pending.pop(t, None)
        nid = r.get(b"id")
        if isinstance(nid, bytes) and len(nid) == 20:
            self.table.add(Node(nid, addr, time.monotonic()))
        return r

    def datagram_received(self, data: bytes, addr) -> None:
        # Anything may arrive on a public UDP port: a packet that does not parse or that
        # breaks a handler is dropped. An exception escaping a protocol callback would reach
        # the event loop's exception handler, which stops the worker process.
        try:
            self._datagram(data, addr)
        except Exception:
            self.bad_packets += 1

    def _datagram(self, data: bytes, addr) -> None:
        try:
            msg = bdecode(data)
        except BencodeError:
            self.bad_packets += 1
            return
        if not isinstance(msg, dict):
            return
        y = msg.get(b"y")
        t = msg.get(b"t", b"")
        if not isinstance(t, bytes):
            self.bad_packets += 1
            return
        addr = (addr[0], addr[1])
        if y == b"r" or y == b"e":
            ent = self._pending.get(t)
            if ent is None or ent[1] != addr:      # unknown tid, or a reply from elsewhere
                if ent is not None:
                    self.bad_packets += 1
                return
            f = ent[0]
            if not f.done():
                if y == b"r" and isinstance(msg.get(b"r"), dict):
                    f.set_result(msg[b"r"])
                else:
                    f.set_exception(RuntimeError(f"KRPC error {msg.get(b'e')}"))
            return
        if y == b"q":
            self._handle_query(msg, t, addr)

    def _handle_query(self, msg: dict, t: bytes, addr: Addr) -> None:
        q = msg.get(b"q")
        a = msg.get(b"a") or {}
        if not isinstance(a, dict):
            self._send({"t": t, "y": "e", "e": [203, "bad arguments"]}, addr)
            return
        nid = a.get(b"id")
        if not isinstance(nid, bytes) or len(nid) != 20:
            self._send({"t": t, "y": "e", "e": [203, "bad id"]}, addr)
            return
        self.queries_served += 1
        self.table.add(Node(nid, addr, time.monotonic()))
        r: Dict[str, object] = {"id": self.id}
        if q == b"ping":
            pass
        elif q in (b"find_node", b"get_peers") and not _is_id(
                a.get(b"target" if q == b"find_node" else b"info_hash")):
            self._send({"t": t, "y": "e", "e": [203, "bad target"]}, addr)
            return
        elif q == b"find_node":
            target = a.get(b"target", b"")
            r["nodes"] = pack_nodes(self.table.closest(target))
        elif q == b"get_peers":
            ih = a.get(b"info_hash", b"")
            r["token"] = self._token(addr[0])
            peers = self._live_peers(ih)
            if peers:
                r["values"] = [pack_peer(p) for p in list(peers)[:50]]
            else:
                r["nodes"] = pack_nodes(self.table.closest(ih))
        elif q == b"announce_peer":
            ih = a.get(b"info_hash", b"")
            if not self._valid_token(addr[0], a.get(b"token", b"")):
                self._send({"t": t, "y": "e", "e": [203, "bad token"]}, addr)
                return
            port = addr[1] if a.get(b"implied_port") else a.get(b"port", 0)
            if not isinstance(ih, bytes) or len(ih) != 20 or not isinstance(port, int) \
                    or not 0 < port < 65536:
                self._send({"t": t, "y": "e", "e": [203, "bad announce"]}, addr)
                return
            peers = self.store.get(ih)
            if peers is None:
                if len(self.store) >= STORE_MAX_TORRENTS:      # bounded: forget the oldest
                    self.store.pop(next(iter(self.store)))
                peers = self.store[ih] = {}
            peers[(addr[0], port)] = time.monotonic()
            while len(peers) > STORE_MAX_PEERS:
                peers.pop(min(peers, key=peers.get))
        else:
            self._send({"t": t, "y": "e", "e": [204, "method unknown"]}, addr)
            return
        self._send({"t": t, "y": "r", "r": r}, addr)

    def _live_peers(self, ih: bytes) -> Dict[Addr, float]:
        """Peers announced for ``ih`` within ``PEER_TTL_S``; expired ones are dropped."""
        peers = self.store.get(ih)
        if not peers:
            return {}
        cut = time.monotonic() - PEER_TTL_S
        for p in [p for p, ts in peers.items() if ts < cut]:
            del peers[p]
        if not peers:
            del self.store[ih]
        return peers

    # ---------------------------------------------------------------- client operations
    async def ping(self, addr: Addr) -> bytes:
        r = await self.query(addr, "ping", {})
        return r.get(b"id", b"")

    def add_node_addr(self, addr: Addr) -> None:
        async def _p():
            try:
                await self.ping(addr)
            except Exception:
                pass
        task = asyncio.get_running_loop().create_task(_p())
        self._tasks.add(task)                  # the loop holds only weak task references
        task.add_done_callback(self._tasks.discard)

    async def _find_node_at(self, addr: Addr, target: bytes) -> List[Node]:
        """find_node at ``addr``; the responder itself enters the table (``query``), the
        nodes it names do not - they are pinged so the ones that answer get in."""
        r = await self.query(addr, "find_node", {"target": target})
        nodes = unpack_nodes(r.get(b"nodes", b""))
        for n in nodes[:K]:
            if n.id != self.id:
                self.add_node_addr(n.addr)
        return nodes

    async def lookup(self, target: bytes, want_peers: bool = True
                     ) -> Tuple[List[Addr], List[Tuple[Node, bytes]]]:
        """Iterative lookup; returns (peers, [(node, token)] of the closest responders)."""
        shortlist: Dict[bytes, Node] = {n.id: n for n in self.table.closest(target, K * 2)}
        queried: Set[bytes] = set()
        peers: Dict[Addr, None] = {}
        tokens: Dict[bytes, Tuple[Node, bytes]] = {}
        for _ in range(20):
            cands = sorted((n for n in shortlist.values() if n.id not in queried),
                           key=lambda n: distance(n.id, target))[:ALPHA]
            if not cands:
                break
            closest_before = sorted(shortlist, key=lambda i: distance(i, target))[:K]
            results = await asyncio.gather(*(self._lookup_one(n, target, want_peers) for n in cands),
                                           return_exceptions=True)
            for n, res in zip(cands, results):
                queried.add(n.id)
                if isinstance(res, BaseException):
                    self.table.remove(n.id)
                    shortlist.pop(n.id, None)
                    continue
                found_nodes, vals, tok = res
                for fn in found_nodes:
                    if fn.id != self.id:
                        shortlist.setdefault(fn.id, fn)
                for v in vals:
                    peers[v] = None
                if tok:
                    tokens[n.id] = (n, tok)
            closest_after = sorted(shortlist, key=lambda i: distance(i, target))[:K]
            if closest_after == closest_before and all(i in queried for i in closest_after):
                break
        best = sorted(tokens.values(), key=lambda nt: distance(nt[0].id, target))[:K]
        return list(peers), best

    async def _lookup_one(self, n: Node, target: bytes, want_peers: bool):
        if want_peers:
            r = await self.query(n.addr, "get_peers", {"info_hash": target})
            vals = [p for p in (unpack_peer(v) for v in r.get(b"values", []) if isinstance(v, bytes)) if p]
            return unpack_nodes(r.get(b"nodes", b"")), vals, r.get(b"token", b"")
        r = await self.query(n.addr, "find_node", {"target": target})
        return unpack_nodes(r.get(b"nodes", b"")), [], b""

    async def get_peers(self, info_hash: bytes, announce_port: int = 0) -> List[Addr]:
        peers, best = await self.lookup(info_hash, want_peers=True)
        local = list(self._live_peers(info_hash))
        if announce_port:
            await asyncio.gather(*(self.query(n.addr, "announce_peer", {
                "info_hash": info_hash, "port": announce_port, "token": tok, "implied_port": 0})
                for n, tok in best), return_exceptions=True)
        return list(dict.fromkeys(peers + local))
