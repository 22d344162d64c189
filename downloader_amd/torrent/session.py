"""One torrent being downloaded (and seeded while it runs).

Replaces webtorrent's ``Torrent`` (reference: ``client.add(magnet, {path}, cb)`` lib/download.js:64,
``torrent.progress`` :79, ``'done'`` :110, ``'error'`` :103). Sources of data:

* peers (BEP-3) found through trackers, DHT (BEP-5), PEX (BEP-11), magnet ``x.pe`` and
  incoming connections - rarest-first piece picking, 16 KiB block pipelining, endgame mode,
  per-piece SHA-1 verification before anything is written;
* webseeds (BEP-19 ``url-list`` / magnet ``ws``) - runs of whole pieces are fetched with HTTP
  Range GETs spliced directly into the files (native transport), then verified in place by the
  threaded native SHA-1; failed pieces are released back to the picker.

Metadata for magnets is fetched with ut_metadata (BEP-9) - or from the magnet's ``xs`` exact
sources over HTTP, as webtorrent does - and checked against the infohash.
"""
from __future__ import annotations

import asyncio
import hashlib
import os
import random
import struct
import time
from collections import OrderedDict
from typing import TYPE_CHECKING, Dict, List, Optional, Set, Tuple
from urllib.parse import quote

from ..net.http import FileSink, TransportError
from ..ops import hashing
from ..utils.aio import drain, gather_strict, run_settled
from ..utils.log import redact_url
from .bencode import bencode
from .metainfo import Metainfo, MetainfoError, parse_info
from .peer import (BLOCK, EV_BLOCKS, EV_CANCEL_DUPS, EV_FILL, EV_NEED, EV_PIECE, METADATA_PIECE,
                   PeerConn)
from .storage import Bitfield, Storage
from .tracker import decode_compact, encode_compact, supported as tracker_supported

# Below this torrent size "auto" keeps incremental verification on the host: a GPU batch takes
# ~100 ms whatever its size (a lane hashes a 4 MiB piece serially), so a short job pays that as
# a tail. Measured on the build box with OpenSSL host hashing: 4 GB single file 6.7 GB/s host
# vs 5.0 GB/s GPU; 20 GB / 50 files 12.1 vs 14.7 GB/s. With the AVX-512 multi-buffer SHA-1
# the host wins both (20 GB: 13.1-13.8 vs 12.3-13.0 GB/s, profiles/archive/s2_r1/verify_ab.jsonl), so
# auto uses the GPU only on hosts without it (``hashing.auto_may_use_gpu``).
GPU_INCREMENTAL_MIN_BYTES = 8 << 30

if TYPE_CHECKING:  # pragma: no cover
    from .client import TorrentClient

Peer = Tuple[str, int]


class TorrentError(Exception):
    pass


class _Active:
    __slots__ = ("idx", "size", "nblocks", "buf", "state", "req", "got", "peers", "owner")

    def __init__(self, idx: int, size: int, buffered: bool = True):
        self.idx = idx
        self.size = size
        self.nblocks = (size + BLOCK - 1) // BLOCK
        # with the native wire the piece is assembled (and verified, written) natively
        self.buf = bytearray(size) if buffered else None
        self.state = bytearray(self.nblocks)   # 0 free, 1 requested, 2 received
        self.req: Dict[int, Set[int]] = {}     # block -> ids of peers that requested it
        self.got = 0
        self.peers: Set[int] = set()           # peers that contributed blocks
        # native wire: the connection whose wire requests this piece by itself (its blocks
        # are then not booked here: ``state`` reads all-requested until it is released)
        self.owner: Optional[int] = None

    def block_len(self, b: int) -> int:
        return min(BLOCK, self.size - b * BLOCK)


class PiecePicker:
    """Rarest-first picker over pieces; blocks inside active pieces; endgame duplicates.

    Candidates (pieces not had, not active, not being verified, not claimed by a webseed
    stream) sit in availability buckets, so starting a new piece costs O(1) expected instead
    of a scan over every piece (quadratic over a 20k-piece torrent). Buckets are maintained
    lazily: an entry whose piece changed availability or stopped being a candidate is
    dropped when met. Each peer's count of pieces it has that we still want is kept up to
    date too, so "is this peer interesting?" is O(1) instead of a scan per completed piece
    per peer."""

    def __init__(self, meta: Metainfo, have: Bitfield):
        self.meta = meta
        self.have = have
        self.n = meta.num_pieces
        self.avail = [0] * self.n
        self.active: Dict[int, _Active] = {}
        # the active pieces requested block by block (not owned by a connection's native
        # wire): the only ones the block loops below walk - with owned pieces, active also
        # holds every piece awaiting its native verification
        self.loose: Dict[int, _Active] = {}
        self.claimed: Set[int] = set()       # pieces owned by webseed workers
        self.verifying: Set[int] = set()     # all blocks in, SHA-1 / write in progress
        self.failed: Dict[int, int] = {}
        self._buckets: Dict[int, List[int]] = {}
        self._slot = [-1] * self.n            # bucket a piece's live entry sits in (-1: none)
        self._peers: Dict[int, Bitfield] = {}
        self.want_count: Dict[int, int] = {}      # peer id -> pieces it has that we lack
        # native wire: called when a piece becomes active (its native buffer starts over)
        self.on_activate = None
        for i in range(self.n):
            self._push(i)

    # ---------------------------------------------------------------- candidates
    def _cand(self, i: int) -> bool:
        return not (i in self.have or i in self.active or i in self.claimed
                    or i in self.verifying)

    def _push(self, i: int) -> None:
        a = self.avail[i]
        if self._slot[i] == a or not self._cand(i):
            return
        self._slot[i] = a
        b = self._buckets.get(a)
        if b is None:
            b = self._buckets[a] = []
        b.append(i)

    def requeue(self, i: int) -> None:
        """Piece ``i`` is wanted again (failed its hash check, or a claim was released)."""
        self.verifying.discard(i)
        self._slot[i] = -1
        self._push(i)

    def _take_rarest(self, bf: Bitfield) -> int:
        """Remove and return a random piece of the lowest availability that ``bf`` has."""
        for a in sorted(self._buckets):
            if a <= 0:
                continue                      # nobody has those
            lst = self._buckets[a]
            misses = 0
            while lst:
                r = random.randrange(len(lst)) if len(lst) > 1 else 0
                i = lst[r]
                stale = self._slot[i] != a or not self._cand(i)
                if stale or i in bf:
                    lst[r] = lst[-1]
                    lst.pop()
                    if self._slot[i] == a:
                        self._slot[i] = -1
                    if stale:
                        continue
                    return i
                misses += 1
                if misses >= 16:             # a sparse peer: scan this bucket once
                    for r, i in enumerate(lst):
                        if self._slot[i] == a and self._cand(i) and i in bf:
                            lst[r] = lst[-1]
                            lst.pop()
                            self._slot[i] = -1
                            return i
                    break
        return -1

    # ---------------------------------------------------------------- peers
    def add_peer(self, bf: Bitfield, pid: Optional[int] = None) -> None:
        want = 0
        for i in range(self.n):
            if i in bf:
                self.avail[i] += 1
                self._push(i)
                if i not in self.have:
                    want += 1
        if pid is not None:
            self._peers[pid] = bf
            self.want_count[pid] = want

    def remove_peer(self, bf: Bitfield, pid: Optional[int] = None) -> None:
        for i in range(self.n):
            if i in bf:
                self.avail[i] -= 1
                self._push(i)
        if pid is not None:
            self._peers.pop(pid, None)
            self.want_count.pop(pid, None)

    def inc(self, i: int, pid: Optional[int] = None) -> None:
        """A peer announced piece ``i`` (HAVE)."""
        self.avail[i] += 1
        self._push(i)
        if pid is not None and pid in self.want_count and i not in self.have:
            self.want_count[pid] += 1

    def piece_done(self, i: int) -> None:
        """``i`` was just added to ``have``: peers holding it are less interesting."""
        self.verifying.discard(i)
        for pid, bf in self._peers.items():
            if i in bf:
                self.want_count[pid] -= 1

    def peer_has_wanted(self, bf: Bitfield, pid: Optional[int] = None) -> bool:
        if self.have.complete:
            return False
        if pid is not None and pid in self.want_count:
            return self.want_count[pid] > 0
        return any(i in bf and i not in self.have for i in range(self.n))

    # ---------------------------------------------------------------- blocks
    def next_block(self, peer_id: int, bf: Bitfield, fresh: bool = True,
                   dups: bool = True) -> Optional[Tuple[int, int, int]]:
        # 1. a free block of an active piece this peer has
        for ap in self.loose.values():
            if ap.idx in bf:
                for b in range(ap.nblocks):
                    if ap.state[b] == 0:
                        ap.state[b] = 1
                        ap.req.setdefault(b, set()).add(peer_id)
                        return ap.idx, b * BLOCK, ap.block_len(b)
        # 2. start the rarest piece this peer has
        best = self._take_rarest(bf) if fresh else -1
        if best >= 0:
            ap = _Active(best, self.meta.piece_size(best), self.on_activate is None)
            if self.on_activate is not None:
                self.on_activate(best)
            self.active[best] = ap
            self.loose[best] = ap
            ap.state[0] = 1
            ap.req[0] = {peer_id}
            return best, 0, ap.block_len(0)
        # 3. endgame: duplicate an outstanding block this peer has not requested yet
        if not dups:
            return None
        for ap in self.loose.values():
            if ap.idx in bf:
                for b in range(ap.nblocks):
                    if ap.state[b] == 1 and peer_id not in ap.req.get(b, ()):
                        ap.req.setdefault(b, set()).add(peer_id)
                        return ap.idx, b * BLOCK, ap.block_len(b)
        return None

    def next_blocks(self, peer_id: int, bf: Bitfield, k: int, fresh: bool = True,
                    dups: bool = True) -> List[Tuple[int, int, int]]:
        """Up to ``k`` blocks for one peer in one pass: free blocks of active pieces first,
        then whole new (rarest) pieces (``fresh``), then endgame duplicates (``dups``)."""
        out: List[Tuple[int, int, int]] = []
        if not fresh and not dups and not self.loose:
            return out                  # (owned pieces only: nothing to request per block)
        for ap in self.loose.values():
            if len(out) >= k:
                return out
            if ap.idx not in bf or ap.got + len(ap.req) >= ap.nblocks and 0 not in ap.state:
                continue
            for b in range(ap.nblocks):
                if ap.state[b] == 0:
                    ap.state[b] = 1
                    ap.req.setdefault(b, set()).add(peer_id)
                    out.append((ap.idx, b * BLOCK, ap.block_len(b)))
                    if len(out) >= k:
                        return out
        # whole new pieces (rarest first), each taken block by block
        while fresh and len(out) < k:
            best = self._take_rarest(bf)
            if best < 0:
                break
            ap = _Active(best, self.meta.piece_size(best), self.on_activate is None)
            if self.on_activate is not None:
                self.on_activate(best)
            self.active[best] = ap
            self.loose[best] = ap
            for b in range(ap.nblocks):
                if len(out) >= k:
                    break
                ap.state[b] = 1
                ap.req[b] = {peer_id}
                out.append((best, b * BLOCK, ap.block_len(b)))
        # endgame: duplicates of outstanding blocks this peer has not requested yet - one pass
        # (next_block per duplicate rescanned every loose piece: quadratic in the pipeline
        # depth, seconds of event loop per fill once depths reached ~1000 blocks)
        if dups and len(out) < k:
            for ap in self.loose.values():
                if ap.idx not in bf:
                    continue
                for b in range(ap.nblocks):
                    if ap.state[b] == 1:
                        rs = ap.req.setdefault(b, set())
                        if peer_id not in rs:
                            rs.add(peer_id)
                            out.append((ap.idx, b * BLOCK, ap.block_len(b)))
                            if len(out) >= k:
                                return out
        return out

    def take_piece(self, peer_id: int, bf: Bitfield) -> int:
        """The rarest piece ``bf`` has, activated whole for one connection's native wire to
        request (-1: none)."""
        best = self._take_rarest(bf)
        if best < 0:
            return -1
        ap = _Active(best, self.meta.piece_size(best), False)
        if self.on_activate is not None:
            self.on_activate(best)
        ap.owner = peer_id
        ap.state = bytearray(b"\x01") * ap.nblocks
        self.active[best] = ap
        return best

    def unstarted(self) -> int:
        """Missing pieces not active, not being verified and not claimed by a webseed."""
        return self.n - self.have.count - len(self.active) - len(self.verifying) \
            - len(self.claimed)

    def no_candidates(self) -> bool:
        """Every missing piece is active, being verified or claimed by a webseed: the
        endgame."""
        return self.unstarted() <= 0

    def complete_blocks(self, idx: int) -> bool:
        """All blocks of active piece ``idx`` arrived: it leaves ``active`` for ``verifying``
        (not a candidate again unless its hash check fails -> ``requeue``). False when it was
        not active any more: another follow-up (an endgame duplicate finishing the same
        piece) got there first and owns the verification."""
        self.loose.pop(idx, None)
        if self.active.pop(idx, None) is None:
            return False
        self.verifying.add(idx)
        return True

    def release(self, peer_id: int, piece: int, begin: int) -> None:
        ap = self.active.get(piece)
        if ap is None:
            return
        b = begin // BLOCK
        rs = ap.req.get(b)
        if rs is not None:
            rs.discard(peer_id)
            if not rs and ap.state[b] == 1:
                ap.state[b] = 0

    def claim_run(self, max_bytes: int, busy_files: Optional[Dict[int, int]] = None
                  ) -> Optional[Tuple[int, int]]:
        """Claim a run of contiguous free pieces (<= max_bytes) for a webseed stream. With
        ``busy_files`` (file index -> streams writing it) the first run that starts in a file
        no other stream is writing wins: page-cache writes into ONE file serialise on its
        inode (~10 GB/s per file on the build box), so streams spread over files."""
        plen = self.meta.piece_length
        maxp = max(1, max_bytes // plen)
        fallback = None
        i = 0
        while i < self.n:
            if i in self.have or i in self.active or i in self.claimed or i in self.verifying:
                i += 1
                continue
            j = i
            while j < self.n and j - i < maxp and j not in self.have and j not in self.active \
                    and j not in self.claimed and j not in self.verifying:
                j += 1
            if not busy_files or not busy_files.get(self.meta.file_at(i * plen), 0):
                fallback = (i, j)
                break
            if fallback is None:
                fallback = (i, j)
            i = self._next_file_piece(i, j)
        if fallback is None:
            return None
        i, j = fallback
        for k in range(i, j):
            self.claimed.add(k)
        return i, j - i

    def _next_file_piece(self, i: int, j: int) -> int:
        """First piece index at or after j that starts beyond the file holding piece i."""
        m = self.meta
        f = m.files[m.file_at(i * m.piece_length)]
        end = f.offset + f.length
        return max(j, end // m.piece_length)

    def unclaim(self, pieces) -> None:
        for p in pieces:
            self.claimed.discard(p)
            self.requeue(p)

    def settle_claim(self, p: int, good: bool) -> None:
        """A claimed webseed piece was verified: done (caller sets ``have``) or wanted again."""
        self.claimed.discard(p)
        if not good:
            self.requeue(p)

    def remaining(self) -> int:
        return self.n - self.have.count


class MetadataFetch:
    def __init__(self, info_hash: bytes):
        self.info_hash = info_hash
        self.size = 0
        self.pieces: Dict[int, bytes] = {}
        self.pending: Dict[int, float] = {}

    def n(self) -> int:
        return (self.size + METADATA_PIECE - 1) // METADATA_PIECE

    def next_piece(self) -> Optional[int]:
        now = time.monotonic()
        for i in range(self.n()):
            if i not in self.pieces and now - self.pending.get(i, 0) > 5.0:
                self.pending[i] = now
                return i
        return None

    def assemble(self) -> Optional[bytes]:
        if self.size == 0 or len(self.pieces) < self.n():
            return None
        data = b"".join(self.pieces[i] for i in range(self.n()))[: self.size]
        if hashlib.sha1(data).digest() != self.info_hash:
            self.pieces.clear()
            self.pending.clear()
            return None
        return data


# Per-peer rates (TorrentSession._rate_loop): sampled every RATE_S; each connection keeps
# QUEUE_S of its rate requested (at least the client's pipeline, at most MAX_DEPTH blocks =
# 16 MiB), so a 50 MB/s peer 200 ms away is not capped at pipeline x 16 KiB / RTT; a peer below
# SLOW_SHARE of the busy peers' mean rate for SLOW_TICKS samples in a row - or one that
# received nothing for SLOW_TICKS samples while holding work (stalled) - gives back the whole
# pieces it owns and only helps with loose blocks until it speeds up (above 2 x SLOW_SHARE).
RATE_S = 0.25
QUEUE_S = 0.5
MAX_DEPTH = 1024
SLOW_SHARE = 1 / 8
SLOW_TICKS = 2
# endgame: an owner keeps its piece if it would finish half a piece within this at its rate
# (heterogeneous swarm on the CPU, 1 GB, 3 seeds: 3.15 - 3.68 s vs 3.44 - 4.07 s with the
# mean/2 rule alone; 0.5 s: 3.33 - 3.38)
ENDGAME_KEEP_S = 0.25


class TorrentSession:
    def __init__(self, client: "TorrentClient", info_hash: bytes, root: str,
                 meta: Optional[Metainfo] = None, trackers=(), webseeds=(), peers=(), name: str = "",
                 exact_sources=()):
        self.client = client
        self.info_hash = info_hash
        self.root = root
        self.meta = meta
        self.name = name
        self.trackers: List[str] = [t for t in trackers if tracker_supported(t)]
        self.webseeds: List[str] = list(webseeds)
        self.exact_sources: List[str] = [x for x in exact_sources
                                          if x.startswith(("http://", "https://"))]
        self.known: Dict[Peer, float] = {}
        self.failed_peers: Dict[Peer, Tuple[int, float]] = {}
        self.peers: Dict[int, PeerConn] = {}
        self.storage: Optional[Storage] = None
        self.have: Optional[Bitfield] = None
        self.picker: Optional[PiecePicker] = None
        self.metafetch = MetadataFetch(info_hash)
        self.meta_ready = asyncio.Event()
        self.done = asyncio.Event()
        self.error: Optional[BaseException] = None
        self.failed = asyncio.Event()
        self.idle_timeout = client.idle_timeout
        self.downloaded = 0
        self.uploaded = 0
        self.verified_bytes = 0
        self.webseed_bytes = 0
        self._tasks: List[asyncio.Task] = []
        self._wake = asyncio.Event()
        self._closed = False
        self._ws_dead = 0
        self._ws_live = 0                      # webseed stream tasks still running
        self._ws_error: Optional[BaseException] = None
        self._ws_files: Dict[int, int] = {}   # file index -> webseed streams writing into it
        self._gpu_verify: Optional[bool] = None
        self.piece_listeners: List = []   # callbacks(piece index) after a piece is verified
        self._piece_cache: "OrderedDict[int, bytes]" = OrderedDict()   # LRU of served pieces
        # (piece, block) -> (active piece, endgame duplicates) between take_block and
        # block_followup of the same dispatch
        self._followup: Dict[Tuple[int, int], tuple] = {}
        self._piece_cache_bytes = 0
        # native peer wire (csrc/peerwire.cpp): sockets handed over after the handshake
        self.wire = None
        self._wire_loop = None
        self._wire_pieces: "asyncio.Queue" = asyncio.Queue()
        self._verifying_ap: Dict[int, _Active] = {}   # natively verified pieces: contributors
        # whole pieces requested by the wire itself (SwarmWire.assign) until the endgame
        self._owned_mode = bool(client.native_wire and client.wire_requests)
        self._endgame = False
        # GPU mode: the wire's pieces go to the GPU part hasher, except once no more than
        # _tail_bytes are left to start (_host_tail)
        self._host_tail = False
        self._tail_bytes = 0
        self._tail_auto = False            # _tail_bytes follows rate x device latency
        self._tail_t = 0.0                 # last auto check
        self._tail_rx0: Optional[Tuple[float, int]] = None   # (time, bytes) at the first rx
        if client.native_wire:
            try:
                from ..ops import native
                self.wire = native().SwarmWire(max(1, client.wire_verify_threads),
                                               max(1, getattr(client, "wire_io_threads", 4)))
            except Exception:
                self.wire = None
        self.stats = {"hash_fails": 0, "peers_connected": 0, "webseed_failures": 0,
                      # native wire: owned pieces handed back by a choking / closing peer, and
                      # made ordinary when the endgame began
                      "wire_released": 0, "wire_endgame_pieces": 0,
                      # ... and fills that started no piece: the verify / write backlog was full
                      "wire_backlogged": 0,
                      # peers marked slow (their owned pieces / requests given back) and the
                      # owned pieces / requested blocks they gave back
                      "slow_peers": 0, "slow_released_pieces": 0, "slow_released_blocks": 0,
                      "max_depth": 0,
                      # longest time a peer held owned pieces / requested blocks without
                      # receiving anything (a stalled peer is shed after SLOW_TICKS samples)
                      "max_owned_idle_s": 0.0,
                      # summed over webseed streams: time in Range GETs / in piece verification
                      "webseed_fetch_s": 0.0, "webseed_verify_s": 0.0}
        self.add_peers(list(peers), "magnet")
        if meta is not None:
            self.trackers += [t for t in meta.trackers()
                              if t not in self.trackers and tracker_supported(t)]
            self.webseeds += [w for w in meta.url_list if w not in self.webseeds]

    # ---------------------------------------------------------------- state
    @property
    def progress(self) -> float:
        """Fraction of verified bytes, 0..1 (webtorrent ``torrent.progress``)."""
        if self.meta is None or self.meta.total_length == 0:
            return 1.0 if self.done.is_set() else 0.0
        return self.verified_bytes / self.meta.total_length

    @property
    def left(self) -> int:
        if self.meta is None:
            return 1 << 40
        return self.meta.total_length - self.verified_bytes

    async def start(self) -> None:
        if self.wire is not None:
            self._wire_loop = asyncio.get_running_loop()
            self._wire_loop.add_reader(self.wire.eventfd(), self._wire_drain)
            self._spawn(self._wire_piece_loop())
        if self.meta is not None:
            await self._init_storage()
        self._spawn(self._connector())
        if self.meta is None and self.exact_sources:
            self._spawn(self._xs_fetch())
        for t in self.trackers:
            self._spawn(self._announce_loop(t))
        if self.client.dht is not None and not (self.meta and self.meta.private):
            self._spawn(self._dht_loop())
        self._spawn(self._pex_loop())
        self._spawn(self._rate_loop())

    def _peer_rx(self, p: PeerConn) -> int:
        if p.wire is not None:
            try:
                return int(self.wire.conn_rx(p.cid))
            except Exception:
                return p.down_bytes
        return p.down_bytes

    def _tail_due(self, unstarted: int) -> bool:
        """GPU mode: hash the rest on the host now? Fixed tail: once no more than _tail_bytes
        are left to start. Auto (VERDICT r5 item 6 - the device's per-piece latency landing
        on the end of a small torrent): once what is left would download in less than the
        device's submission -> digest time (measured by the wire, 0.12 s before the first
        digest) x swarm_gpu_tail_x (3), at the rate the download has run since its first
        byte; at most swarm_gpu_tail_max (0.85) of the torrent. Checked at most every 5 ms
        (it runs per piece assigned)."""
        if not self._tail_auto:
            return unstarted <= self._tail_bytes
        if unstarted <= 0:
            return True
        now = time.monotonic()
        if now - self._tail_t < 0.005:
            return False
        self._tail_t = now
        rx = self.wire.rx_total()
        if self._tail_rx0 is None:
            if rx > 0:
                self._tail_rx0 = (now, rx)
            return False
        t0, b0 = self._tail_rx0
        if now - t0 < 0.02:
            return False
        rate = (rx - b0) / (now - t0)
        lat = self.wire.gpu_latency() or 0.12
        x = getattr(self.client, "swarm_gpu_tail_x", 3.0)
        tail = min(self._tail_bytes, int(rate * lat * x))
        return unstarted <= tail

    async def _rate_loop(self) -> None:
        """Per-peer receive rates every RATE_S: each connection's request pipeline follows its
        bandwidth-delay product (BEP-3 leaves the depth to the client; libtorrent keeps ~3 s
        of a peer's rate requested), and a peer far slower than its share of the swarm - or
        stalled mid-piece - hands its owned pieces and requested blocks back so faster peers
        finish them (a 100 KB/s peer sat on a whole 4 MiB piece until the
        endgame)."""
        last = self._t_start = time.monotonic()
        while not self._closed and not self.done.is_set():
            await asyncio.sleep(RATE_S)
            now = time.monotonic()
            dt, last = max(1e-3, now - last), now
            if self.picker is None:
                continue
            tl = self.stats.setdefault("rate_timeline", [])
            if len(tl) < 600:      # (t, MB verified, endgame) per sample: the bench's ramp / tail
                tl.append((round(now - self._t_start, 2), round(self.verified_bytes / 1e6, 1),
                           int(self._endgame)))
            busy = []
            total = 0.0
            for p in list(self.peers.values()):
                if p.closed:
                    continue
                rx = self._peer_rx(p)
                r = max(0, rx - p.rx_mark) / dt
                p.rx_mark = rx
                p.rate = r if p.rate is None else 0.5 * p.rate + 0.5 * r
                p.last_rate = r
                if r > 0 or p.progress_t is None:
                    p.progress_t = now
                elif not p.slow and (p.inflight or self._owns(p)):
                    self.stats["max_owned_idle_s"] = max(self.stats["max_owned_idle_s"],
                                                         round(now - p.progress_t, 2))
                if not p.peer_choking and p.am_interested and p.bitfield is not None:
                    busy.append(p)
                    total += p.rate
            if len(busy) < 2 or total <= 0:
                continue
            share = total / len(busy)
            base = self.client.pipeline
            shed = False
            for p in busy:
                # grow at once (the last sample), shrink with the average
                cap = min(MAX_DEPTH, p.reqq) if p.reqq else MAX_DEPTH
                depth = int(min(cap, max(min(base, cap), max(p.rate, p.last_rate) * QUEUE_S / BLOCK)))
                if depth != p.depth:
                    p.depth = depth
                    self.stats["max_depth"] = max(self.stats["max_depth"], depth)
                    if p.wire is not None:
                        try:
                            self.wire.set_conn_pipeline(p.cid, depth)
                        except Exception:
                            pass
                stalled = p.progress_t is not None and now - p.progress_t >= SLOW_TICKS * RATE_S
                if (p.rate < share * SLOW_SHARE or stalled) and (p.inflight or self._owns(p)):
                    p.slow_ticks = SLOW_TICKS if stalled else p.slow_ticks + 1
                    if p.slow_ticks >= SLOW_TICKS and not p.slow:
                        p.slow = True
                        self.stats["slow_peers"] += 1
                        self._shed(p)
                        shed = True
                else:
                    p.slow_ticks = 0
                    if p.slow and p.rate >= 2 * share * SLOW_SHARE:
                        p.slow = False
            if shed:
                self._refill_all()
            elif self.wire is not None and self._owned_mode and not self._endgame:
                # safety net: a connection whose native queue ran below its pipeline without
                # Python hearing of it (NEED is sent once per fill) gets a fill now
                for p in busy:
                    if p.wire is not None and not p.fill_queued and not p.slow and \
                            p._wq is not None and self.wire.todo(p.cid) < p.depth:
                        p.fill_queued = True
                        p._wq.put_nowait((EV_FILL, None))

    def _owns(self, p: PeerConn) -> bool:
        return any(ap.owner == p.cid for ap in self.picker.active.values())

    def _shed(self, p: PeerConn) -> None:
        """A slow peer's work goes back: its owned pieces become ordinary (blocks received
        kept, its outstanding requests still its own), and its outstanding block requests
        may be asked of others too (its late answers are then duplicates)."""
        if self.wire is not None and self._owned_mode:
            for idx, ap in list(self.picker.active.items()):
                if ap.owner != p.cid:
                    continue
                r = self.wire.release_piece(idx)
                if r is None:
                    continue            # complete, being verified
                _, states = r
                self._to_block_mode(ap, states, p)
                self.stats["slow_released_pieces"] += 1
        for (piece, begin) in list(p.inflight):
            ap = self.picker.active.get(piece)
            if ap is None:
                continue
            b = begin // BLOCK
            if ap.state[b] == 1:
                ap.state[b] = 0         # free for others; p's request stays in ap.req
                self.stats["slow_released_blocks"] += 1

    def _spawn(self, coro) -> asyncio.Task:
        t = asyncio.get_running_loop().create_task(coro)
        self._tasks.append(t)
        t.add_done_callback(self._task_done)
        return t

    def _task_done(self, t: asyncio.Task) -> None:
        if t.cancelled():
            return
        e = t.exception()
        if e is not None and not isinstance(e, (asyncio.CancelledError,)):
            self.fail(e)

    def fail(self, e: BaseException) -> None:
        if self.error is None and not self.done.is_set():
            self.error = e
            self.failed.set()

    async def _init_storage(self) -> None:
        loop = asyncio.get_running_loop()
        meta = self.meta
        assert meta is not None
        # a cancel during the opens waits for them and closes what was opened
        self.storage = await run_settled(Storage, meta, self.root,
                                         discard=lambda st: st.close())
        self.have = await loop.run_in_executor(None, self.storage.recheck,
                                               self.client.verify_backend)
        self.verified_bytes = sum(meta.piece_size(i) for i in range(meta.num_pieces)
                                  if i in self.have)
        self.picker = PiecePicker(meta, self.have)
        want_gpu = False
        if self.wire is not None and meta.num_pieces > 1:
            # swarm pieces SHA-1'd by the gfx950 PartHasher (set up once per worker, off the
            # loop): asked for, or `auto` on a torrent big enough to hide the device's
            # per-piece latency (hashing.swarm_backend; the device check itself off the loop)
            v = self.client.swarm_verify
            want_gpu = v == "gpu" or (v == "auto" and await loop.run_in_executor(
                None, hashing.swarm_backend, v, meta.total_length,
                self.client.swarm_gpu_min_bytes) == "gpu")
        if want_gpu:
            try:
                on = await loop.run_in_executor(None, hashing.gpu_relay_hashing)
            except Exception:
                on = False
            if not on and self.client.swarm_verify == "gpu":
                raise TorrentError("swarm_verify_backend=gpu but no GPU part hasher")
            self.wire.set_gpu(bool(on), self.client.wire_gpu_inflight)
            # fixed: at most a quarter of the torrent (a small one stays mostly on the device);
            # auto: rate x device latency, at most swarm_gpu_tail_max of it (_tail_due)
            tb = self.client.swarm_gpu_tail_bytes
            self._tail_auto = bool(on) and tb < 0
            cap = int(meta.total_length * min(1.0, max(0.0, getattr(
                self.client, "swarm_gpu_tail_max", 0.85))))
            self._tail_bytes = (cap if tb < 0 else min(tb, meta.total_length // 4)) if on else 0
            self.stats["swarm_verify"] = "gpu" if on else "cpu"
        if self.wire is not None:
            self.wire.set_storage(meta.piece_length, meta.total_length, meta.pieces,
                                  [(fd, n) for fd, (_, n) in zip(self.storage.fds,
                                                                  self.storage.paths)])
            self.picker.on_activate = self.wire.begin_piece
            self.wire.set_pipeline(self.client.pipeline)
            self.wire.set_backlog_cap(self.client.swarm_backlog_bytes)
            self.wire.set_have(self.have.to_bytes())     # what unchoked peers may be served
        self.meta_ready.set()
        for p in list(self.peers.values()):
            p.attach_meta()
            await self.update_interest(p)
            await p.send_bitfield()
            await self.fill(p)
        for url in self.webseeds:
            for _ in range(self.client.webseed_streams):
                self._spawn(self._webseed_worker(url))
        if self.have.complete:
            self._finish()

    def _finish(self) -> None:
        # No fsync here: staged files are uploaded and deleted right after, and a crashed
        # attempt is recovered by re-verifying what is on disk (recheck), not by durability.
        if not self.done.is_set():
            self.done.set()
            for t in self.trackers:
                self._spawn(self._announce_once(t, "completed"))

    # ---------------------------------------------------------------- peers
    def add_peers(self, peers: List[Peer], source: str = "") -> None:
        new = False
        for p in peers:
            if p[1] <= 0 or p[1] > 65535:
                continue
            if p == (self.client.public_host, self.client.listen_port) or \
                    (p[1] == self.client.listen_port and p[0] in ("127.0.0.1", "0.0.0.0", "::1")
                     and self.client.listen_port):
                continue
            if p not in self.known:
                self.known[p] = time.monotonic()
                new = True
        if new:
            self._wake.set()

    def connected_addrs(self) -> Set[Peer]:
        return {p.addr for p in self.peers.values()}

    async def _connector(self) -> None:
        while not self._closed:
            if not self.done.is_set() or self.client.seed_after_done:
                conn = self.connected_addrs()
                now = time.monotonic()
                cands = [p for p in self.known if p not in conn and
                         now >= self.failed_peers.get(p, (0, 0.0))[1]]
                random.shuffle(cands)
                room = self.client.max_peers - len(self.peers)
                for p in cands[:max(0, room)]:
                    self._spawn(self._connect(p))
            self._wake.clear()
            try:
                await asyncio.wait_for(self._wake.wait(), 2.0)
            except asyncio.TimeoutError:
                pass

    async def _connect(self, addr: Peer) -> None:
        try:
            pc = await self.client.connect_peer(self, addr)
        except Exception:
            n, _ = self.failed_peers.get(addr, (0, 0.0))
            self.failed_peers[addr] = (n + 1, time.monotonic() + min(300.0, 2.0 * (2 ** n)))
            return
        self.failed_peers.pop(addr, None)
        await pc.run()

    def register_peer(self, pc: PeerConn) -> bool:
        if len(self.peers) >= self.client.max_peers + 8 or self._closed:
            return False
        if pc.addr in self.connected_addrs() or pc.remote_id == self.client.peer_id:
            return False
        self.peers[pc.cid] = pc
        self.stats["peers_connected"] += 1
        if self.wire is not None:
            try:
                pc.attach_wire(self.wire)
            except Exception:
                pass                      # this connection stays on the Python path
        if self.meta is not None and pc.bitfield is None:
            pc.bitfield = Bitfield(self.meta.num_pieces)
        return True

    def peer_closed(self, pc: PeerConn) -> None:
        if self.peers.pop(pc.cid, None) is None:
            return
        if pc.bitfield is not None and self.picker is not None:
            self.picker.remove_peer(pc.bitfield, pc.cid)
        self.release_inflight(pc)
        self._wake.set()

    def release_inflight(self, pc: PeerConn) -> None:
        """The peer choked us or went away: what it was asked for is free again - its block
        requests, and the pieces its native wire was requesting (made ordinary, their received
        blocks kept). Every other connection is offered them."""
        released = bool(pc.inflight)
        if self.picker is not None:
            for (piece, begin) in list(pc.inflight):
                self.picker.release(pc.cid, piece, begin)
            if pc.wire is not None and self._owned_mode:
                try:
                    back = self.wire.release(pc.cid)
                except Exception:
                    back = []
                for idx, states in back:
                    ap = self.picker.active.get(idx)
                    if ap is not None and ap.owner == pc.cid:
                        self._to_block_mode(ap, states, None)
                        self.stats["wire_released"] += 1
                        released = True
        pc.inflight.clear()
        if released and not self._closed:
            self._refill_all()

    def _to_block_mode(self, ap: "_Active", states: bytes, owner: Optional[PeerConn]) -> None:
        """An owned piece goes back to per-block requesting: received blocks stay, blocks the
        owner still has requests out for stay its (``owner``: endgame) or are freed."""
        oid = ap.owner
        ap.owner = None
        self.picker.loose[ap.idx] = ap
        ap.state = bytearray(states)
        ap.req = {}
        ap.got = 0
        now = time.monotonic()
        for b, st in enumerate(ap.state):
            if st == 2:
                ap.got += 1
            elif st == 1:
                if owner is not None and not owner.closed:
                    ap.req[b] = {oid}
                    owner.inflight[(ap.idx, b * BLOCK)] = now
                else:
                    ap.state[b] = 0
        if ap.got:
            ap.peers.add(oid)
            self.downloaded += min(ap.size, ap.got * BLOCK)

    def _assign(self, pc: PeerConn) -> bool:
        """Keep two pipelines of blocks queued on the connection's native wire, a whole piece
        at a time. False when no piece was left for it (the endgame may begin)."""
        # blocks queued beyond those in flight: one pipeline (NEED asks for more when the
        # queue runs below it) - a connection owns ~2 x its depth, ~2 x QUEUE_S of its rate
        me, want = pc.cid, pc.depth
        wire, picker = self.wire, self.picker
        if pc.slow:
            return False                 # a slow peer helps with loose blocks only
        try:
            t = wire.todo(me)
            while t < want:
                if wire.backlogged():
                    # complete pieces waiting for their hash / write hold their buffers: no new
                    # piece until half of them are through (NEED on conn 0 refills everyone)
                    self.stats["wire_backlogged"] += 1
                    return True
                idx = picker.take_piece(me, pc.bitfield)
                if idx < 0:
                    # nothing left to start: once this connection is down to its last
                    # pipeline, the endgame begins (the others' queues become duplicable)
                    if t < pc.depth and picker.no_candidates():
                        self._enter_endgame()
                    return False
                if self._tail_bytes and not self._host_tail and \
                        self._tail_due(picker.unstarted() * self.meta.piece_length):
                    # the last pieces are hashed on the host: on the device each would add its
                    # submission -> digest time to the end of the job
                    self._host_tail = True
                    wire.set_host_tail(True)
                    self.stats["gpu_host_tail_bytes"] = picker.unstarted() * self.meta.piece_length
                try:
                    t = wire.assign(me, idx)
                except Exception:
                    # the connection is gone: the piece stays active, all blocks free
                    ap = picker.active[idx]
                    ap.owner = None
                    ap.state = bytearray(ap.nblocks)
                    picker.loose[idx] = ap
                    raise
        except Exception:
            return False
        return True

    def _enter_endgame(self) -> None:
        """Every missing piece is being fetched: owned pieces go back to per-block requesting
        (their outstanding requests kept as the owner's), so idle connections can duplicate
        the last blocks like on the Python wire."""
        if self._endgame or self.wire is None:
            return
        self._endgame = True
        # pieces of connections at least half the swarm's mean rate stay theirs (they finish
        # them sooner than duplicates would: a heterogeneous swarm spent 2/3 of its endgame on
        # per-block duplicates of fast owners' pieces); slower owners' pieces go back to
        # per-block requesting, where idle connections duplicate their missing blocks
        rates = [p.rate for p in self.peers.values() if not p.closed and p.rate]
        mean = sum(rates) / len(rates) if rates else 0.0
        # ... and only when they would finish it soon: half a piece within ENDGAME_KEEP_S at
        # their rate (a 5 MB/s owner of a fresh 4 MiB piece kept the endgame waiting ~0.8 s)
        keep_s = float(os.environ.get("STAGER_ENDGAME_KEEP_S", ENDGAME_KEEP_S))
        keep = max(mean / 2, self.meta.piece_length / 2 / keep_s if keep_s > 0 else 0.0)
        for idx, ap in list(self.picker.active.items()):
            if ap.owner is None:
                continue
            owner = self.peers.get(ap.owner)
            if owner is not None and not owner.closed and not owner.slow and mean > 0 and \
                    (owner.rate or 0.0) >= keep:
                continue
            r = self.wire.release_piece(idx)
            if r is None:
                continue            # complete, being verified: its result still finds the owner
            oid, states = r
            self._to_block_mode(ap, states, self.peers.get(oid))
            self.stats["wire_endgame_pieces"] += 1
        self._refill_all()

    async def update_interest(self, pc: PeerConn) -> None:
        if self.picker is None or pc.bitfield is None:
            return
        await pc.set_interested(self.picker.peer_has_wanted(pc.bitfield, pc.cid))

    async def maybe_unchoke(self, pc: PeerConn) -> None:
        unchoked = sum(1 for p in self.peers.values() if not p.am_choking)
        if pc.am_choking and unchoked < self.client.max_uploads and self.have is not None:
            await pc.set_choking(False)

    # ---------------------------------------------------------------- native wire
    def _wire_drain(self) -> None:
        """eventfd readable: route the wire's events. Block arrivals are booked right here
        (no await, no copy: the bytes are already in their native piece); messages, endgame
        cancels and refills go to the connection's own queue, piece results to the piece
        task."""
        if self.wire is None:
            return
        now = time.monotonic()
        for conn, kind, data in self.wire.poll():
            if kind == EV_PIECE:
                self._wire_pieces.put_nowait(data)
                continue
            if conn == 0:                        # NEED on conn 0: the backlog drained
                self._refill_all()
                continue
            pc = self.peers.get(conn)
            if pc is None or pc._wq is None:
                continue
            pc.last_rx = now
            if kind == EV_BLOCKS:
                self._wire_blocks(pc, data)
            elif kind == EV_NEED:
                if not pc.fill_queued:
                    pc.fill_queued = True
                    pc._wq.put_nowait((EV_FILL, None))
            else:
                pc._wq.put_nowait((kind, data))

    def _wire_blocks(self, pc: PeerConn, data: bytes) -> None:
        """Book one batch of arrivals (16-byte records: piece, begin, length, status). The
        per-block work is what the Python wire did minus the copy and the framing: ~1.6 us a
        block, 0.1 CPU-s per GB (profiles/archive/r5/swarm/wire/)."""
        picker = self.picker
        if picker is None:
            return
        inflight_pop = pc.inflight.pop
        active_get = picker.active.get
        me = pc.cid
        got_bytes = 0
        last_idx, ap = -1, None
        for idx, begin, ln, st in struct.iter_unpack(">IIII", data):
            inflight_pop((idx, begin), None)
            if not st:
                # not taken (a duplicate, a bad length, a piece no longer assembling): if this
                # peer was the one asked, the block is free again rather than stuck requested
                picker.release(me, idx, begin)
                continue
            got_bytes += ln
            if idx != last_idx:                    # blocks of one piece come in runs
                last_idx, ap = idx, active_get(idx)
                if ap is not None:
                    ap.peers.add(me)
            if ap is None:
                continue
            b = begin >> 14                        # BLOCK = 16 KiB
            if ap.state[b] != 2:
                ap.state[b] = 2
                ap.got += 1
            rs = ap.req.pop(b, None)
            if rs is not None and (len(rs) > 1 or me not in rs):     # endgame duplicates
                pc._wq.put_nowait((EV_CANCEL_DUPS, (rs, idx, begin, ln)))
            if st == 2 and picker.complete_blocks(idx):
                self._verifying_ap[idx] = ap          # verified + written natively
                last_idx, ap = -1, None
        self.downloaded += got_bytes
        pc.down_bytes += got_bytes
        if not pc.fill_queued and self.refill_due(pc):
            pc.fill_queued = True
            pc._wq.put_nowait((EV_FILL, None))

    async def cancel_dups(self, pc: PeerConn, dup: Set[int], idx: int, begin: int,
                          ln: int) -> None:
        for other_id in dup:
            if other_id != pc.cid:
                other = self.peers.get(other_id)
                if other is not None:
                    await other.cancel(idx, begin, ln)

    async def _wire_piece_loop(self) -> None:
        """Native verification results, in order: 1 verified and written, 0 hash mismatch,
        2 storage write failed."""
        while True:
            data = await self._wire_pieces.get()
            idx, status = struct.unpack(">IB", data[:5])
            ap = self._verifying_ap.pop(idx, None)
            if self.picker is None:
                continue
            if ap is None:
                # an owned piece (or one released with every block already in): its blocks
                # were never booked one by one, this result is the first Python hears of it
                ap = self.picker.active.get(idx)
                if ap is not None:
                    self.picker.complete_blocks(idx)
                    if ap.owner is not None:
                        ap.peers.add(ap.owner)
                        self.downloaded += ap.size
                        owner = self.peers.get(ap.owner)
                        if owner is not None:
                            owner.down_bytes += ap.size
            if status == 1:
                await self._piece_complete(idx)
            elif status == 2:
                self.picker.requeue(idx)
                self.fail(TorrentError(f"storage write of piece {idx} failed: "
                                       f"{data[5:].decode(errors='replace')}"))
            else:
                self.stats["hash_fails"] += 1
                self.picker.requeue(idx)
                for pid in (ap.peers if ap is not None else ()):
                    p = self.peers.get(pid)
                    if p is not None:
                        p.hash_fails += 1
                        if p.hash_fails >= 3:
                            p.close()
                # the verdict came after the blocks: no arrival will refill the pipelines, so
                # the requeued piece is offered to every connection now
                self._refill_all()

    def _refill_all(self) -> None:
        """Offer freed blocks (a requeued piece, a closed peer's requests) to every
        connection: an idle pipeline is otherwise only refilled by its own next arrival."""
        for p in list(self.peers.values()):
            if p.closed or p.fill_queued:
                continue
            p.fill_queued = True
            if p._wq is not None:
                p._wq.put_nowait((EV_FILL, None))
            else:
                self._spawn(self._fill_once(p))

    async def _fill_once(self, pc: PeerConn) -> None:
        pc.fill_queued = False
        if not pc.closed:
            await self.fill(pc)

    def refill_due(self, pc: PeerConn) -> bool:
        """Whether ``fill`` would send anything (checked without a coroutine per block)."""
        return pc.depth - len(pc.inflight) >= max(1, pc.depth // 4)

    def take_block(self, pc: PeerConn, idx: int, begin: int, data) -> bool:
        """Synchronous part of ``on_block``: copy a block into its piece. True when
        ``block_followup`` has work (endgame duplicates to cancel, or the piece is complete)."""
        if self.picker is None or self.have is None:
            return False
        ap = self.picker.active.get(idx)
        if ap is None or begin % BLOCK or begin >= ap.size:
            return False
        b = begin // BLOCK
        if ap.state[b] == 2 or len(data) != ap.block_len(b):
            return False
        if ap.buf is None:
            # a Python-framed connection of a native-wire session (its socket could not be
            # handed over): the piece is assembled natively
            self._native_take(pc, ap, idx, begin, data)
            return False
        ap.buf[begin:begin + len(data)] = data
        ap.state[b] = 2
        ap.got += 1
        ap.peers.add(pc.cid)
        self.downloaded += len(data)
        rs = ap.req.pop(b, None)
        others = rs is not None and (len(rs) > 1 or pc.cid not in rs)   # endgame duplicates
        if others or ap.got >= ap.nblocks:
            self._followup[(idx, b)] = (ap, rs if others else None)
            return True
        return False

    def _native_take(self, pc: PeerConn, ap: "_Active", idx: int, begin: int, data) -> None:
        st = self.wire.take_block(idx, begin, data) if self.wire is not None else 0
        if not st:
            return
        b = begin // BLOCK
        ap.state[b] = 2
        ap.got += 1
        ap.peers.add(pc.cid)
        self.downloaded += len(data)
        rs = ap.req.pop(b, None)
        if rs is not None and (len(rs) > 1 or pc.cid not in rs):
            self._spawn(self.cancel_dups(pc, rs, idx, begin, len(data)))
        if st == 2 and self.picker.complete_blocks(idx):
            self._verifying_ap[idx] = ap

    async def block_followup(self, pc: PeerConn, idx: int, begin: int, ln: int) -> None:
        ent = self._followup.pop((idx, begin // BLOCK), None)
        if ent is not None:
            await self._block_done(pc, ent[0], ent[1], idx, begin, ln)

    async def fill(self, pc: PeerConn) -> None:
        if self.picker is None or pc.closed or pc.peer_choking or not pc.am_interested \
                or pc.bitfield is None:
            return
        fresh = dups = True
        if self.wire is not None and self.wire.backlogged():
            fresh = False                        # (per-block requests of started pieces only)
        if pc.wire is not None and self._owned_mode and not self._endgame:
            # whole pieces go to the wire; below, only free blocks of ordinary pieces (one a
            # choked or closed peer left) are requested per block, and duplicates once every
            # missing piece is being fetched
            fresh = False
            dups = not self._assign(pc) and self._endgame
        room = pc.depth - len(pc.inflight)
        # Refill in batches (at least a quarter of the pipeline) so one write carries many
        # REQUEST messages instead of one syscall per 17-byte message.
        if room < max(1, pc.depth // 4):
            return
        if pc.slow:
            fresh = False                # no new pieces for a slow peer: loose blocks only
        blocks = self.picker.next_blocks(pc.cid, pc.bitfield, room, fresh, dups)
        if blocks:
            await pc.request_many(blocks)

    async def on_block(self, pc: PeerConn, idx: int, begin: int, data) -> None:
        """``data``: the block (bytes or a memoryview of the receive buffer - it is copied
        into the piece before anything awaits)."""
        if self.take_block(pc, idx, begin, data):
            await self.block_followup(pc, idx, begin, len(data))

    async def _block_done(self, pc: PeerConn, ap: "_Active", dup: Optional[Set[int]], idx: int,
                          begin: int, ln: int) -> None:
        # endgame: cancel the duplicates requested from other peers
        if dup:
            for other_id in dup:
                if other_id != pc.cid:
                    other = self.peers.get(other_id)
                    if other is not None:
                        await other.cancel(idx, begin, ln)
        if ap.got < ap.nblocks or not self.picker.complete_blocks(idx):
            return                  # not complete, or the other follow-up verifies it
        # The piece's buffer is complete and no longer written (every block is state 2), so it
        # is hashed and, if good, written to storage in place - one executor hop, no copy.
        buf = ap.buf
        loop = asyncio.get_running_loop()
        off = idx * self.meta.piece_length
        want = self.meta.piece_hash(idx)
        try:
            if len(buf) >= 262144:
                good = await loop.run_in_executor(None, self._verify_write, buf, off, want)
            else:
                good = self._verify_write(buf, off, want)
        except OSError as e:   # our disk, not the peer: ENOSPC/EIO fail the job (retried)
            self.picker.requeue(idx)
            self.fail(TorrentError(f"storage write of piece {idx} failed: {e}"))
            return
        if not good:
            self.stats["hash_fails"] += 1
            self.picker.requeue(idx)
            for pid in ap.peers:
                p = self.peers.get(pid)
                if p is not None:
                    p.hash_fails += 1
                    if p.hash_fails >= 3:
                        p.close()
            return
        await self._piece_complete(idx)

    def _verify_write(self, buf, off: int, want: bytes) -> bool:
        if hashing.sha1(buf) != want:
            return False
        self.storage.write(off, buf)
        return True

    async def _piece_complete(self, idx: int) -> None:
        if not self.have.set(idx):
            return
        if self.wire is not None:
            self.wire.set_have_piece(idx)        # (natively verified pieces are set already)
        self.picker.piece_done(idx)
        self.verified_bytes += self.meta.piece_size(idx)
        for cb in self.piece_listeners:
            cb(idx)
        for p in list(self.peers.values()):
            # (not to a peer that has the piece: a seed gains nothing from it, and it costs a
            # message per piece per seed)
            if p.bitfield is None or idx not in p.bitfield:
                await p.send_have(idx)
            if p.am_interested and p.bitfield is not None and \
                    not self.picker.peer_has_wanted(p.bitfield, p.cid):
                await p.set_interested(False)
        if self.have.complete:
            self._finish()

    async def serve_request(self, pc: PeerConn, idx: int, begin: int, ln: int) -> None:
        if pc.am_choking or self.have is None or idx >= self.have.n or idx not in self.have:
            return
        if ln > 131072 or begin + ln > self.meta.piece_size(idx):
            return
        piece = self._piece_cache.get(idx)
        if piece is None:
            # Read the whole piece once (one thread-pool hop) and serve its blocks from memory.
            piece = await asyncio.get_running_loop().run_in_executor(
                None, self.storage.read, idx * self.meta.piece_length, self.meta.piece_size(idx))
            self._piece_cache[idx] = piece
            self._piece_cache_bytes += len(piece)
            while self._piece_cache_bytes > self.client.piece_cache_bytes and self._piece_cache:
                old = next(iter(self._piece_cache))
                self._piece_cache_bytes -= len(self._piece_cache.pop(old))
        else:
            self._piece_cache.move_to_end(idx)
        pc.up_bytes += ln
        self.uploaded += ln
        await pc.send_block(idx, begin, memoryview(piece)[begin:begin + ln])

    # ---------------------------------------------------------------- metadata (BEP-9)
    async def on_ext_handshake(self, pc: PeerConn) -> None:
        if self.meta is None and pc.metadata_size and b"ut_metadata" in pc.ext:
            if pc.metadata_size > 64 << 20:
                return
            if self.metafetch.size == 0:
                self.metafetch.size = pc.metadata_size
            await self._request_metadata(pc)

    async def _request_metadata(self, pc: PeerConn) -> None:
        if self.meta is not None or b"ut_metadata" not in pc.ext:
            return
        for _ in range(4):
            i = self.metafetch.next_piece()
            if i is None:
                return
            await pc.send_ext(b"ut_metadata", bencode({"msg_type": 0, "piece": i}))

    async def on_metadata_msg(self, pc: PeerConn, d, tail: bytes) -> None:
        if not isinstance(d, dict):
            return
        t = d.get(b"msg_type")
        piece = int(d.get(b"piece", -1))
        if t == 0:  # request
            if self.meta is None:
                await pc.send_ext(b"ut_metadata", bencode({"msg_type": 2, "piece": piece}))
                return
            raw = self.meta.raw_info
            chunk = raw[piece * METADATA_PIECE:(piece + 1) * METADATA_PIECE]
            if not chunk:
                await pc.send_ext(b"ut_metadata", bencode({"msg_type": 2, "piece": piece}))
                return
            await pc.send_ext(b"ut_metadata", bencode({"msg_type": 1, "piece": piece,
                                                       "total_size": len(raw)}) + chunk)
        elif t == 1 and self.meta is None:
            if 0 <= piece < self.metafetch.n():
                self.metafetch.pieces[piece] = tail
            data = self.metafetch.assemble()
            if data is not None:
                await self.set_metadata(data)
            else:
                await self._request_metadata(pc)
        elif t == 2:
            self.metafetch.pending.pop(piece, None)

    async def set_metadata(self, info_bytes: bytes) -> None:
        if self.meta is not None:
            return
        try:
            m = parse_info(info_bytes, self.info_hash)
        except MetainfoError as e:
            self.fail(TorrentError(f"bad metadata: {e}"))
            return
        self.meta = m
        self.name = m.name
        await self._init_storage()

    async def _xs_fetch(self) -> None:
        """Magnet ``xs``: fetch the ``.torrent`` from each exact source in turn while peers
        are asked over ut_metadata; the first file whose info dict hashes to the magnet's
        infohash wins. A source that fails or serves another torrent is skipped."""
        from ..fetch.http import fetch_bytes
        from .metainfo import parse_torrent
        for url in self.exact_sources:
            if self.meta is not None or self._closed:
                return
            try:
                m = parse_torrent(await fetch_bytes(self.client.transports, url))
            except Exception:
                continue
            if m.info_hash == self.info_hash and self.meta is None:
                # the .torrent may carry trackers / webseeds the magnet did not list
                new = [t for t in m.trackers() if t not in self.trackers and tracker_supported(t)]
                self.trackers += new
                for t in new:
                    self._spawn(self._announce_loop(t))
                for w in m.url_list:
                    if w not in self.webseeds:
                        self.webseeds.append(w)
                await self.set_metadata(m.raw_info)
                return

    # ---------------------------------------------------------------- PEX (BEP-11)
    def on_pex(self, pc: PeerConn, d) -> None:
        if not isinstance(d, dict) or (self.meta is not None and self.meta.private):
            return
        added = d.get(b"added", b"")
        if isinstance(added, bytes):
            self.add_peers(decode_compact(added), "pex")

    async def _pex_loop(self) -> None:
        while not self._closed:
            await asyncio.sleep(self.client.pex_interval)
            if self.meta is not None and self.meta.private:
                continue
            addrs = [p.addr if p.outgoing else (p.addr[0], p.listen_port)
                     for p in self.peers.values() if p.outgoing or p.listen_port]
            msg = bencode({"added": encode_compact(addrs[:50]), "added.f": b"\x00" * min(50, len(addrs)),
                           "dropped": b""})
            for p in list(self.peers.values()):
                await p.send_ext(b"ut_pex", msg)

    # ---------------------------------------------------------------- trackers / DHT
    async def _announce_once(self, url: str, event: str = "") -> int:
        from .tracker import announce
        try:
            r = await announce(url, self.info_hash, self.client.peer_id, self.client.listen_port,
                               self.uploaded, self.downloaded, self.left, event,
                               transports=self.client.transports)
        except Exception:
            return 30
        self.add_peers(r.peers, "tracker")
        return max(5, min(r.interval, 1800))

    async def _announce_loop(self, url: str) -> None:
        interval = await self._announce_once(url, "started")
        while not self._closed:  # keep announcing while seeding too
            await asyncio.sleep(min(interval, self.client.max_announce_interval))
            interval = await self._announce_once(url)

    async def _dht_loop(self) -> None:
        dht = self.client.dht
        while not self._closed:  # a complete session keeps announcing itself as a seed
            try:
                peers = await dht.get_peers(self.info_hash, announce_port=self.client.listen_port)
                self.add_peers(peers, "dht")
            except Exception:
                pass
            await asyncio.sleep(self.client.dht_interval)

    # ---------------------------------------------------------------- webseeds (BEP-19)
    def _webseed_url(self, base: str, file_idx: int) -> str:
        assert self.meta is not None
        return webseed_url(self.meta, base, file_idx)

    async def _webseed_worker(self, base: str) -> None:
        """One BEP-19 stream: claim a run of whole pieces (``webseed_chunk`` bytes), GET it
        straight into the storage files (splice), hand the run to verification and go on with
        the next run while it is hashed - fetch and SHA-1 overlap within the stream, so a few
        streams saturate the path (parallel writers into one file contend on its inode lock)."""
        st = {"failures": 0, "seen": 0}
        verifying: Set[asyncio.Task] = set()
        loop = asyncio.get_running_loop()
        depth = max(1, self.client.webseed_verify_depth_gpu if self._use_gpu_verify()
                    else self.client.webseed_verify_depth)
        self._ws_live += 1
        try:
            while not self._closed and not self.done.is_set():
                if st["failures"] >= self.client.webseed_max_failures:
                    self._webseed_gave_up(TorrentError("webseed served corrupt pieces"))
                    return
                if st["failures"] > st["seen"]:       # a run failed its hash check: back off
                    st["seen"] = st["failures"]
                    await asyncio.sleep(min(10.0, 0.2 * (2 ** st["failures"])))
                    continue
                run = self.picker.claim_run(self.client.webseed_chunk, self._ws_files)
                if run is None:
                    if not verifying:
                        return
                    # a failing verification hands its pieces back: wait, then look again
                    await asyncio.wait(verifying, return_when=asyncio.FIRST_COMPLETED)
                    continue
                first, count = run
                pieces = list(range(first, first + count))
                fidx = self.meta.file_at(first * self.meta.piece_length)
                self._ws_files[fidx] = self._ws_files.get(fidx, 0) + 1
                try:
                    await self._webseed_fetch(base, first, pieces)
                except (TransportError, OSError) as e:
                    self.picker.unclaim(pieces)
                    st["failures"] += 1
                    st["seen"] = st["failures"]
                    self.stats["webseed_failures"] += 1
                    if st["failures"] >= self.client.webseed_max_failures:
                        self._webseed_gave_up(e)
                        return
                    await asyncio.sleep(min(10.0, 0.2 * (2 ** st["failures"])))
                    continue
                finally:
                    self._ws_files[fidx] -= 1
                t = loop.create_task(self._webseed_verify(pieces, st))
                verifying.add(t)
                t.add_done_callback(verifying.discard)
                while len(verifying) >= depth:
                    await asyncio.wait(verifying, return_when=asyncio.FIRST_COMPLETED)
            if verifying:
                await gather_strict(*verifying)
        finally:
            pending = list(verifying)
            for t in pending:
                t.cancel()
            # a verification may sit in an executor reading the storage fds: it finishes
            # before this webseed loop counts as gone (the session closes those fds after)
            interrupted = await drain(pending)
            self._webseed_exit()
            if interrupted:
                raise asyncio.CancelledError()

    async def _webseed_fetch(self, base: str, first: int, pieces: List[int]) -> None:
        off = first * self.meta.piece_length
        length = sum(self.meta.piece_size(i) for i in pieces)
        t_fetch = time.perf_counter()
        for fd, foff, ln, fidx in self.storage.segments(off, length):
            url = self._webseed_url(base, fidx)
            flen = self.meta.files[fidx].length
            hdrs = [] if (foff == 0 and ln == flen) else \
                [("Range", f"bytes={foff}-{foff + ln - 1}")]
            r = await self.client.transports.request("GET", url, headers=hdrs,
                                                     sink=FileSink(fd, foff, ln))
            if r.status not in (200, 206) or (r.status == 200 and hdrs) or r.written != ln:
                raise TransportError(f"webseed {redact_url(url)}: HTTP {r.status}, "
                                     f"{r.written}/{ln} B",
                                     r.status)
            self.webseed_bytes += ln
            self.downloaded += ln
        self.stats["webseed_fetch_s"] += time.perf_counter() - t_fetch

    def _use_gpu_verify(self) -> bool:
        """Incremental (per-run) verification on the GPU: always for ``verify_backend=gpu``;
        for ``auto`` only when the verifier is already warm (``download.gpu_prewarm``) and the
        torrent is big enough to keep hundreds of pieces in flight."""
        if self._gpu_verify is None:
            be = self.client.verify_backend
            if be == "gpu":
                self._gpu_verify = True
            elif be == "auto":
                self._gpu_verify = (hashing._gpu_verifier is not None and
                                    self.meta.total_length >= GPU_INCREMENTAL_MIN_BYTES and
                                    hashing.auto_may_use_gpu())
            else:
                self._gpu_verify = False
        return self._gpu_verify

    async def _host_verify(self, pieces: List[int]) -> List[bool]:
        return await asyncio.get_running_loop().run_in_executor(
            None, self.storage.verify, pieces, self.client.verify_threads)

    async def _webseed_verify(self, pieces: List[int], st: Dict[str, int]) -> None:
        """Verify one fetched run. It runs as a plain task next to its stream, so nothing may
        escape it: every error hands the pieces back to the picker (otherwise they stay
        claimed and nobody fetches them again). A transient read error counts as a stream
        failure; a verifier fault (HIP error, OOM, no device) falls back to the host under
        ``verify_backend=auto`` and fails the session under an explicit ``gpu``."""
        t_verify = time.perf_counter()
        try:
            if self._use_gpu_verify():
                try:
                    fut = hashing.gpu_batcher().submit(self.storage.paths, self.meta.piece_length,
                                                       self.meta.pieces, pieces)
                    ok = await asyncio.wrap_future(fut)
                except OSError:
                    raise
                except Exception:
                    if self.client.verify_backend == "gpu":
                        raise
                    self._gpu_verify = False          # auto: this session stays on the host
                    ok = await self._host_verify(pieces)
            else:
                ok = await self._host_verify(pieces)
        except OSError:
            self.picker.unclaim(pieces)
            st["failures"] += 1
            return
        except Exception as e:
            self.picker.unclaim(pieces)
            st["failures"] += 1
            self.fail(TorrentError(f"piece verification failed: {e!r}"))
            return
        self.stats["webseed_verify_s"] += time.perf_counter() - t_verify
        for i, good in zip(pieces, ok):
            self.picker.settle_claim(i, bool(good))
            if good:
                await self._piece_complete(i)
            else:
                self.stats["hash_fails"] += 1
        if not all(ok):
            st["failures"] += 1

    def _webseed_gave_up(self, e: BaseException) -> None:
        self._ws_dead += 1
        self._ws_error = e

    def _webseed_exit(self) -> None:
        """A stream ended. Streams that found nothing left to claim end normally, so when the
        LAST one ends after another gave up, pieces may be left that nobody fetches: with no
        other source (peers, trackers, DHT) the session fails instead of waiting forever."""
        self._ws_live -= 1
        if self._ws_live == 0 and self._ws_error is not None and not self.done.is_set() \
                and not self.peers and not self.known and not self.trackers \
                and self.client.dht is None:
            self.fail(TorrentError(f"webseed failed: {self._ws_error}"))

    # ---------------------------------------------------------------- shutdown
    async def wait(self) -> None:
        """Wait until complete; raise the session error if one happens first."""
        d = asyncio.ensure_future(self.done.wait())
        f = asyncio.ensure_future(self.failed.wait())
        try:
            await asyncio.wait({d, f}, return_when=asyncio.FIRST_COMPLETED)
        finally:
            d.cancel()
            f.cancel()
        if not self.done.is_set() and self.error is not None:
            raise self.error

    async def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        for t in self._tasks:
            t.cancel()
        for p in list(self.peers.values()):
            p.close()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        if self.wire is not None:
            # its verifiers write into the storage's fds: stopped before those close
            if self._wire_loop is not None and not self._wire_loop.is_closed():
                self._wire_loop.remove_reader(self.wire.eventfd())
            await asyncio.get_running_loop().run_in_executor(None, self.wire.close)
        if self.storage is not None:
            # may wait for a piece write still on an executor thread: not on the loop
            await asyncio.get_running_loop().run_in_executor(None, self.storage.close)
        stop = [self._announce_once(t, "stopped") for t in self.trackers]
        if stop:
            try:
                await asyncio.wait_for(asyncio.gather(*stop, return_exceptions=True), 2.0)
            except asyncio.TimeoutError:
                pass

    def local_files(self) -> List[str]:
        return [p for p, _ in self.meta.local_files(self.root)] if self.meta else []

    def total_bytes(self) -> int:
        return self.meta.total_length if self.meta else 0


def webseed_url(m: Metainfo, base: str, file_idx: int) -> str:
    """BEP-19 URL of file ``file_idx``: a single-file torrent's url-list entry is the file
    itself (or a directory, when it ends in ``/``); multi-file entries are the parent of
    ``<name>/<path...>``."""
    if not m.multi_file:
        return base + quote(m.name) if base.endswith("/") else base
    f = m.files[file_idx]
    return base.rstrip("/") + "/" + "/".join(quote(x) for x in [m.name] + f.path)


def webseed_file_size(path: str) -> int:
    return os.path.getsize(path)
