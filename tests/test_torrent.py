"""BitTorrent subsystem: bencode, metainfo, magnet, trackers, swarm, ut_metadata, webseeds,
DHT, resume, and the worker-level torrent job with the reference watchdogs."""
from __future__ import annotations

import asyncio
import hashlib
import os
import shutil
import struct

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from downloader_amd.torrent.bencode import BencodeError, bdecode, bencode, decode_torrent
from downloader_amd.torrent.client import TorrentClient
from downloader_amd.torrent.magnet import Magnet, MagnetError, parse_magnet
from downloader_amd.torrent.metainfo import MetainfoError, make_torrent, parse_torrent
from downloader_amd.torrent.session import TorrentError
from downloader_amd.torrent.tracker import announce
from downloader_amd.torrent.tracker_server import Tracker

_bval = st.recursive(
    st.one_of(st.integers(-10**12, 10**12), st.binary(max_size=20)),
    lambda ch: st.one_of(st.lists(ch, max_size=4),
                         st.dictionaries(st.binary(max_size=6), ch, max_size=4)),
    max_leaves=12)


@settings(max_examples=60, deadline=None)
@given(_bval)
def test_bencode_roundtrip(v):
    assert bdecode(bencode(v)) == v


@pytest.mark.parametrize("bad", [b"i01e", b"i-0e", b"ie", b"5:abc", b"l", b"d1:ae", b"x", b"i1ei2e"])
def test_bdecode_rejects(bad):
    with pytest.raises(BencodeError):
        bdecode(bad)


def test_info_span_is_exact():
    raw = b"d8:announce3:abc4:infod6:lengthi5e4:name1:x12:piece lengthi16384e6:pieces20:" + \
        b"A" * 20 + b"ee"
    top, info = decode_torrent(raw)
    assert info.startswith(b"d6:length") and info.endswith(b"e")
    assert parse_torrent(raw).info_hash == hashlib.sha1(info).digest()


def _tree(root, sizes):
    data = {}
    for rel, n in sizes.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        d = os.urandom(n)
        with open(p, "wb") as f:
            f.write(d)
        data[rel] = d
    return data


def test_make_and_parse_multi_file(tmp_path):
    _tree(tmp_path / "src" / "Show", {"S1/a.mkv": 100_000, "S1/b.mkv": 1, "c.txt": 70_000})
    t = make_torrent(str(tmp_path / "src" / "Show"), 16384, trackers=["http://t/a", "udp://u:1"],
                     url_list=["http://ws/"])
    m = parse_torrent(t)
    assert m.multi_file and m.name == "Show" and m.total_length == 170_001
    assert [f.path for f in m.files] == [["S1", "a.mkv"], ["S1", "b.mkv"], ["c.txt"]]
    assert m.num_pieces == (170_001 + 16383) // 16384
    assert m.trackers() == ["http://t/a", "udp://u:1"] and m.url_list == ["http://ws/"]
    lf = m.local_files("/dl")
    assert lf[0] == ("/dl/Show/S1/a.mkv", 100_000)
    assert m.file_spans(99_999, 3) == [(0, 99_999, 1), (1, 0, 1), (2, 0, 1)]


def test_metainfo_rejects_bad_piece_count():
    raw = bencode({"info": {"name": "x", "length": 100000, "piece length": 16384,
                            "pieces": b"A" * 20}})
    with pytest.raises(MetainfoError):
        parse_torrent(raw)


@pytest.mark.parametrize("bad", [
    {"announce": "x"},                                                       # no info
    {"info": {"name": "x", "piece length": 16384, "pieces": b"A" * 20, "files": [1, 2]}},
    {"info": {"name": "x", "piece length": 16384, "pieces": b"A" * 20, "files": [{"path": ["a"]}]}},
    {"info": {"name": "x", "piece length": 16384, "pieces": b"A" * 20, "length": "big"}},
    {"info": {"name": "x", "piece length": 1 << 30, "pieces": b"A" * 20, "length": 10}},
    {"info": {"name": "x", "piece length": 16384, "pieces": 7, "length": 10}},
])
def test_malformed_metainfo_is_a_metainfo_error(bad):
    """.torrent files and ut_metadata come from the network: every malformation is a
    MetainfoError (the job fails cleanly / the peer's metadata is dropped), and a piece
    length that would make the peer path buffer gigabytes per piece is refused."""
    with pytest.raises(MetainfoError):
        parse_torrent(bencode(bad))
    good = {"info": {"name": "x", "piece length": 16384, "pieces": b"A" * 20, "length": 10},
            "announce-list": [5, ["http://t/a"]], "url-list": 3}
    m = parse_torrent(bencode(good))
    assert m.announce == [["http://t/a"]] and m.url_list == []


def test_path_traversal_is_neutralised(tmp_path):
    raw = bencode({"info": {"name": "..", "piece length": 16384, "pieces": b"A" * 20,
                            "files": [{"path": ["..", "etc", "passwd"], "length": 5}]}})
    m = parse_torrent(raw)
    for p, _ in m.local_files(str(tmp_path)):
        assert os.path.abspath(p).startswith(str(tmp_path))


def test_magnet_parse():
    ih = bytes(range(20))
    m = parse_magnet(f"magnet:?xt=urn:btih:{ih.hex()}&dn=My%20Show&tr=udp%3A%2F%2Ft%3A1"
                     f"&ws=http%3A%2F%2Fw%2F&x.pe=1.2.3.4:5&xl=99")
    assert m.info_hash == ih and m.name == "My Show" and m.trackers == ["udp://t:1"]
    assert m.webseeds == ["http://w/"] and m.peers == [("1.2.3.4", 5)] and m.exact_length == 99
    import base64
    b32 = base64.b32encode(ih).decode()
    assert parse_magnet(f"magnet:?xt=urn:btih:{b32}").info_hash == ih
    assert parse_magnet(Magnet(ih, "n", ["http://t"]).to_uri()).trackers == ["http://t"]
    with pytest.raises(MagnetError):
        parse_magnet("magnet:?dn=x")
    # magnet-uri folds ``as`` into the webseed list; ``xs`` = .torrent exact sources
    m = parse_magnet(f"magnet:?xt=urn:btih:{ih.hex()}&as=http%3A%2F%2Fa%2F&ws=http%3A%2F%2Fa%2F"
                     f"&xs=http%3A%2F%2Fo%2Fx.torrent&kt=movie+2019")
    assert m.webseeds == ["http://a/"] and m.exact_sources == ["http://o/x.torrent"]
    assert m.keywords == ["movie", "2019"]
    assert parse_magnet(m.to_uri()).exact_sources == ["http://o/x.torrent"]


def test_http_and_udp_tracker(run):
    async def go():
        tr = await Tracker().start()
        ih, a, b = b"I" * 20, b"A" * 20, b"B" * 20
        r1 = await announce(tr.http_url, ih, a, 1111, 0, 0, 10, "started")
        assert r1.peers == []
        r2 = await announce(tr.udp_url, ih, b, 2222, 0, 0, 0, "started")
        assert ("127.0.0.1", 1111) in r2.peers and r2.interval == 5
        r3 = await announce(tr.http_url, ih, a, 1111, 0, 0, 10)
        assert ("127.0.0.1", 2222) in r3.peers and r3.seeders == 1
        await tr.stop()
    run(go())


async def _seed(tmp_path, sizes, piece=32768, **mk):
    src = tmp_path / "seed"
    data = _tree(src / "Pack", sizes)
    raw = make_torrent(str(src / "Pack"), piece, **mk)
    seeder = await TorrentClient().start()
    await seeder.add_torrent(parse_torrent(raw), str(src))
    return raw, data, seeder, src


def _check(dst, data, name="Pack"):
    for rel, d in data.items():
        with open(os.path.join(dst, name, rel), "rb") as f:
            assert f.read() == d, rel


def test_swarm_download_from_seeder(run, tmp_path):
    async def go():
        tr = await Tracker().start()
        raw, data, seeder, _ = await _seed(tmp_path, {"a.mkv": 700_000, "S1/b.mkv": 123_457},
                                           trackers=[tr.http_url])
        leech = await TorrentClient().start()
        s = await leech.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        await asyncio.wait_for(s.wait(), 30)
        assert s.progress == 1.0 and s.stats["hash_fails"] == 0
        _check(tmp_path / "dl", data)
        await leech.close(); await seeder.close(); await tr.stop()
    run(go())


def test_magnet_metadata_over_peers(run, tmp_path):
    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 400_000})
        m = parse_torrent(raw)
        leech = await TorrentClient().start()
        mag = Magnet(m.info_hash, peers=[("127.0.0.1", seeder.listen_port)])
        s = await leech.add_magnet(parse_magnet(mag.to_uri()), str(tmp_path / "dl"))
        await asyncio.wait_for(s.wait(), 30)
        assert s.meta.info_hash == m.info_hash
        _check(tmp_path / "dl", data)
        await leech.close(); await seeder.close()
    run(go())


def test_magnet_metadata_from_exact_source(run, tmp_path, origin_cls):
    """A magnet with no peers, trackers or DHT but an ``xs`` URL: the .torrent is fetched over
    HTTP (a first source serving ANOTHER torrent is skipped), its webseeds are adopted, and
    the payload arrives from them (webtorrent's exact-source path)."""
    async def go():
        origin = await origin_cls().start()
        src = tmp_path / "ws"
        data = _tree(src / "Pack", {"a.mkv": 300_000})
        raw = make_torrent(str(src / "Pack"), 65536, url_list=[origin.url("/seed/")])
        other = make_torrent(str(src / "Pack"), 32768)
        origin.blobs["/seed/Pack/a.mkv"] = data["a.mkv"]
        origin.blobs["/t/other.torrent"] = other
        origin.blobs["/t/pack.torrent"] = raw
        m = parse_torrent(raw)
        c = await TorrentClient(webseed_chunk=65536, webseed_streams=2).start()
        mag = Magnet(m.info_hash, exact_sources=[origin.url("/t/missing.torrent"),
                                                 origin.url("/t/other.torrent"),
                                                 origin.url("/t/pack.torrent")])
        s = await c.add_magnet(parse_magnet(mag.to_uri()), str(tmp_path / "dl"))
        await asyncio.wait_for(s.wait(), 30)
        assert s.meta.info_hash == m.info_hash and s.webseed_bytes == 300_000
        _check(tmp_path / "dl", data)
        await c.close(); await origin.stop()
    run(go())


def test_bad_peer_data_is_rejected_and_refetched(run, tmp_path):
    async def go():
        raw, data, seeder, src = await _seed(tmp_path, {"x.mkv": 300_000})
        # corrupt the seeder's file AFTER it verified: it will serve a bad piece 0
        p = src / "Pack" / "x.mkv"
        b = bytearray(p.read_bytes())
        b[10] ^= 0xFF
        p.write_bytes(bytes(b))
        good = await TorrentClient().start()
        gdir = tmp_path / "good"
        _tree(gdir / "Pack", {})
        shutil.copytree(src / "Pack", gdir / "Pack", dirs_exist_ok=True)
        (gdir / "Pack" / "x.mkv").write_bytes(data["x.mkv"])
        await good.add_torrent(parse_torrent(raw), str(gdir))
        leech = await TorrentClient().start()
        s = await leech.add_torrent(parse_torrent(raw), str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", seeder.listen_port),
                                           ("127.0.0.1", good.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        await leech.close(); await seeder.close(); await good.close()
    run(go(), timeout=90)


@pytest.mark.parametrize("native_wire,wire_requests", [(True, True), (True, False),
                                                       (False, False)])
def test_swarm_native_and_python_wire(run, tmp_path, native_wire, wire_requests):
    """The peer wire both ways (download.torrent_native_wire): multi-file pieces straddling
    file boundaries from two seeders. Natively every piece is assembled, SHA-1'd and written
    by csrc/peerwire.cpp (its counters say so), its blocks requested by the wire itself
    (download.torrent_wire_requests) or one by one from Python; in Python by
    peer.py/session.py."""
    async def go():
        src = tmp_path / "seed"
        data = _tree(src / "Pack", {"a.mkv": 1_000_003, "S1/b.mkv": 377_777, "S1/c.mkv": 5})
        raw = make_torrent(str(src / "Pack"), 65536)
        seeders = []
        for _ in range(2):
            c = await TorrentClient(native_wire=native_wire).start()
            await c.add_torrent(parse_torrent(raw), str(src))
            seeders.append(c)
        leech = await TorrentClient(native_wire=native_wire, pipeline=32,
                                    wire_requests=wire_requests).start()
        meta = parse_torrent(raw)
        s = await leech.add_torrent(meta, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", c.listen_port) for c in seeders])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        assert s.stats["hash_fails"] == 0
        if native_wire:
            st = s.wire.stats()
            assert st["verified"] == meta.num_pieces and st["hash_fails"] == 0
            assert st["block_bytes"] == meta.total_length and st["active_pieces"] == 0
            assert all(p.wire is not None for p in s.peers.values())
            # the seeders served every block from their storage files natively (sendfile)
            served = sum(ss.wire.stats()["served_bytes"] for c in seeders
                         for ss in c.sessions.values())
            assert served >= meta.total_length
            if wire_requests:
                # whole pieces were handed to the wire, which asked for their blocks itself
                # (on a torrent this small every piece is handed out at once, and the endgame
                # soon turns most back to per-block requests; config 6 has the wire request
                # 99.6 % of the blocks of 2 GB itself, profiles/archive/r5/)
                assert st["assigned"] > 0 and st["requests"] > 0
            else:
                assert st["assigned"] == 0 and st["requests"] == 0
        else:
            assert s.wire is None
        await leech.close()
        for c in seeders:
            await c.close()
    run(go(), timeout=90)


def test_native_wire_pieces_verified_on_the_part_hasher(run, tmp_path):
    """swarm_verify_backend=gpu: complete pieces go from page-locked pooled buffers to the
    installed GPU part hasher (here its host double, the same C ABI as the gfx950 PartHasher),
    the digests come back in order and every piece is verified and written; a corrupt piece
    is caught from the device's digest."""
    from downloader_amd.ops import hashing, native

    async def go():
        raw, data, seeder, src = await _seed(tmp_path, {"a.mkv": 900_000, "b.mkv": 300_001})
        p = src / "Pack" / "a.mkv"
        b = bytearray(p.read_bytes())
        b[100_000] ^= 0xFF                       # piece 3 served corrupt by this seeder
        p.write_bytes(bytes(b))
        good = await TorrentClient().start()
        gdir = tmp_path / "good"
        (gdir / "Pack").mkdir(parents=True)
        for rel, d in data.items():
            (gdir / "Pack" / rel).write_bytes(d)
        await good.add_torrent(parse_torrent(raw), str(gdir))
        leech = await TorrentClient(swarm_verify="gpu", pipeline=64,
                                    swarm_gpu_tail_bytes=0).start()
        meta = parse_torrent(raw)
        s = await leech.add_torrent(meta, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.sleep(0.5)
        s.add_peers([("127.0.0.1", good.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        st = s.wire.stats()
        assert s.stats["swarm_verify"] == "gpu"
        assert st["gpu_pieces"] >= meta.num_pieces and st["gpu_errors"] == 0
        assert st["hash_fails"] >= 1 and st["verified"] == meta.num_pieces
        await leech.close(); await seeder.close(); await good.close()
        assert s.wire.stats()["pool_in_use"] == 0       # every piece buffer back in the pool

    hashing.use_part_hasher(native().CpuPartHasher(0.002), 4)
    try:
        run(go(), timeout=90)
    finally:
        hashing.use_part_hasher(None)


def test_native_wire_gpu_overflow_is_hashed_on_the_host(run, tmp_path):
    """GPU mode with at most one piece on the (slow) device: the pieces that complete while it
    is busy are SHA-1'd on the host instead of queueing behind it; every piece verifies."""
    from downloader_amd.ops import hashing, native

    async def go():
        raw, data, seeder, src = await _seed(tmp_path, {"a.mkv": 1_500_000}, piece=65536)
        leech = await TorrentClient(swarm_verify="gpu", pipeline=64,
                                    wire_gpu_inflight=1, swarm_gpu_tail_bytes=0).start()
        meta = parse_torrent(raw)
        s = await leech.add_torrent(meta, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        st = s.wire.stats()
        assert st["gpu_pieces"] >= 1 and st["gpu_overflow"] >= 1
        assert st["gpu_pieces"] + st["gpu_overflow"] >= meta.num_pieces
        assert st["verified"] == meta.num_pieces and st["hash_fails"] == 0
        await leech.close(); await seeder.close()

    hashing.use_part_hasher(native().CpuPartHasher(0.05), 4)
    try:
        run(go(), timeout=90)
    finally:
        hashing.use_part_hasher(None)


def test_native_wire_bad_piece_is_refetched_and_peer_blamed(run, tmp_path):
    """A seeder serving a corrupt piece over the native wire: the native verifier rejects
    it (hash_fails), the session requeues it and gets it from the good seeder."""
    async def go():
        raw, data, seeder, src = await _seed(tmp_path, {"x.mkv": 300_000})
        p = src / "Pack" / "x.mkv"
        b = bytearray(p.read_bytes())
        b[40_000] ^= 0xFF                        # piece 1 of 32 KiB pieces
        p.write_bytes(bytes(b))
        good = await TorrentClient().start()
        gdir = tmp_path / "good"
        (gdir / "Pack").mkdir(parents=True)
        (gdir / "Pack" / "x.mkv").write_bytes(data["x.mkv"])
        await good.add_torrent(parse_torrent(raw), str(gdir))
        leech = await TorrentClient(pipeline=64).start()
        s = await leech.add_torrent(parse_torrent(raw), str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.sleep(0.5)                 # the bad seeder alone first: piece 1 fails
        s.add_peers([("127.0.0.1", good.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        assert s.wire.stats()["hash_fails"] >= 1 and s.stats["hash_fails"] >= 1
        await leech.close(); await seeder.close(); await good.close()
    run(go(), timeout=90)


@pytest.mark.parametrize("then", ["choke", "close"])
def test_native_wire_choked_or_closed_owner_releases_its_pieces(run, tmp_path, then):
    """Pieces the native wire requests by itself for one connection go back to per-block
    requesting when that peer chokes us or hangs up half-way: the blocks it delivered are
    kept, the rest are fetched from the other seeder, and every piece verifies."""
    from downloader_amd.torrent.peer import handshake_bytes

    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 3_000_000}, piece=65536)
        m = parse_torrent(raw)
        blob = data["x.mkv"]
        answered = []

        async def fake_peer(r, w):
            # handshake, all pieces, unchoke; answer 10 requests, then choke (or close)
            await r.readexactly(68)
            w.write(handshake_bytes(m.info_hash, b"-XX0001-" + b"2" * 12, False))
            bits = bytearray((m.num_pieces + 7) // 8)
            for i in range(m.num_pieces):
                bits[i // 8] |= 0x80 >> (i % 8)
            w.write(struct.pack(">IB", 1 + len(bits), 5) + bytes(bits))
            w.write(struct.pack(">IB", 1, 1))
            try:
                while True:
                    n = int.from_bytes(await r.readexactly(4), "big")
                    body = await r.readexactly(n) if n else b""
                    if not body or body[0] != 6:
                        continue
                    if len(answered) >= 10:
                        if then == "close":
                            w.close()
                            return
                        if len(answered) == 10:
                            answered.append(None)
                            w.write(struct.pack(">IB", 1, 0))          # CHOKE
                        continue
                    idx, begin, ln = struct.unpack(">III", body[1:13])
                    off = idx * m.piece_length + begin
                    w.write(struct.pack(">IBII", 9 + ln, 7, idx, begin) + blob[off:off + ln])
                    answered.append((idx, begin))
                    await w.drain()
            except (asyncio.IncompleteReadError, ConnectionError):
                pass

        srv = await asyncio.start_server(fake_peer, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        leech = await TorrentClient(pipeline=8).start()
        s = await leech.add_torrent(m, str(tmp_path / "dl"), peers=[("127.0.0.1", port)])
        while len(answered) < 10:
            await asyncio.sleep(0.01)
        await asyncio.sleep(0.2)
        assert not s.done.is_set()
        s.add_peers([("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        assert s.stats["wire_released"] >= 1 and s.stats["hash_fails"] == 0
        assert s.wire.stats()["assigned"] >= 2
        await leech.close(); await seeder.close()
        srv.close()
    run(go(), timeout=90)


def test_webseed_single_and_multi_file(run, tmp_path, origin_cls):
    async def go():
        origin = await origin_cls().start()
        src = tmp_path / "ws"
        data = _tree(src / "Pack", {"a.mkv": 1_000_003, "dir/b.mkv": 77_777, "dir/c.mp4": 5})
        for rel, d in data.items():
            origin.blobs["/seed/Pack/" + rel] = d
        raw = make_torrent(str(src / "Pack"), 65536, url_list=[origin.url("/seed/")])
        c = TorrentClient(webseed_chunk=200_000, webseed_streams=3)
        await c.start()
        s = await c.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        await asyncio.wait_for(s.wait(), 30)
        _check(tmp_path / "dl", data)
        assert s.webseed_bytes == sum(len(d) for d in data.values())
        # single-file torrent with a URL pointing at the file itself
        one = os.urandom(333_333)
        (src / "one.mkv").write_bytes(one)
        origin.blobs["/direct/one.mkv"] = one
        raw1 = make_torrent(str(src / "one.mkv"), 16384, url_list=[origin.url("/direct/one.mkv")])
        s1 = await c.add_torrent(parse_torrent(raw1), str(tmp_path / "dl1"))
        await asyncio.wait_for(s1.wait(), 30)
        assert (tmp_path / "dl1" / "one.mkv").read_bytes() == one
        await c.close(); await origin.stop()
    run(go())


def test_resume_rechecks_existing_data(run, tmp_path, origin_cls):
    async def go():
        origin = await origin_cls().start()
        src = tmp_path / "ws"
        data = _tree(src / "Pack", {"a.mkv": 500_000})
        origin.blobs["/s/Pack/a.mkv"] = data["a.mkv"]
        raw = make_torrent(str(src / "Pack"), 16384, url_list=[origin.url("/s/")])
        dl = tmp_path / "dl" / "Pack"
        dl.mkdir(parents=True)
        partial = bytearray(data["a.mkv"])
        partial[400_000:] = b"\x00" * 100_000
        (dl / "a.mkv").write_bytes(bytes(partial))
        c = await TorrentClient().start()
        s = await c.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        have0 = s.have.count
        await asyncio.wait_for(s.wait(), 30)
        assert have0 == 400_000 // 16384
        assert s.webseed_bytes < 150_000
        _check(tmp_path / "dl", data)
        await c.close(); await origin.stop()
    run(go())


def test_dht_peer_discovery(run, tmp_path):
    async def go():
        from downloader_amd.torrent.dht import DHTNode
        boot = await DHTNode(host="127.0.0.1").start()
        nodes = [await DHTNode(host="127.0.0.1", bootstrap=[("127.0.0.1", boot.port)]).start()
                 for _ in range(6)]
        ih = hashlib.sha1(b"x").digest()
        assert await nodes[0].get_peers(ih, announce_port=4242) == []
        found = await nodes[5].get_peers(ih)
        assert ("127.0.0.1", 4242) in found
        # full client path: seeder announces via DHT, leecher finds it with no tracker
        raw, data, _, src = await _seed(tmp_path, {"d.mkv": 200_000})
        seeder = TorrentClient(enable_dht=True, dht_bootstrap=[("127.0.0.1", boot.port)])
        seeder.dht_interval = 0.5
        await seeder.start()
        await seeder.add_torrent(parse_torrent(raw), str(src))
        leech = TorrentClient(enable_dht=True, dht_bootstrap=[("127.0.0.1", boot.port)])
        leech.dht_interval = 0.5
        await leech.start()
        await asyncio.sleep(1.0)
        s = await leech.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        await asyncio.wait_for(s.wait(), 30)
        _check(tmp_path / "dl", data)
        await leech.close(); await seeder.close()
        for n in nodes + [boot]:
            await n.close()
    run(go(), timeout=60)


def test_pex_spreads_peers(run, tmp_path):
    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"p.mkv": 100_000})
        a = await TorrentClient().start()
        a.pex_interval = 0.3
        sa = await a.add_torrent(parse_torrent(raw), str(tmp_path / "a"),
                                 peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(sa.wait(), 30)
        b = await TorrentClient().start()
        sb = await b.add_torrent(parse_torrent(raw), str(tmp_path / "b"),
                                 peers=[("127.0.0.1", a.listen_port)])
        await asyncio.wait_for(sb.wait(), 30)
        for _ in range(30):
            if ("127.0.0.1", seeder.listen_port) in sb.known:
                break
            await asyncio.sleep(0.1)
        assert ("127.0.0.1", seeder.listen_port) in sb.known
        await a.close(); await b.close(); await seeder.close()
    run(go())


# ------------------------------------------------------------------ worker-level torrent jobs
def _worker(make_cfg, s3_ep, **over):
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.service.worker import Worker
    d = {"torrent_enable_dht": False, "progress_interval_s": 0.05}
    d.update(over.pop("download", {}))
    cfg = make_cfg(s3_ep, download=d, **over)
    return Worker(cfg, broker=MemoryBroker())


async def _wait_results(w, n=1, timeout=30.0):
    for _ in range(int(timeout / 0.02)):
        if len(w.results) >= n:
            return
        await asyncio.sleep(0.02)
    raise AssertionError(w.results)


def test_worker_torrent_over_http_with_webseed(run, tmp_path, make_cfg, origin_cls):
    """Reference path lib/download.js:143-155: a .torrent URL chains to the torrent backend."""
    async def go():
        from downloader_amd.models import api, keys
        from downloader_amd.s3.fake_server import FakeS3
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src"
        data = _tree(src / "My Show", {"Season 1/e1.mkv": 400_000, "Season 1/e2.mkv": 300_000,
                                       "Extras/x.mkv": 1000, "readme.txt": 10})
        for rel, d in data.items():
            origin.blobs["/ws/My Show/" + rel] = d
        raw = make_torrent(str(src / "My Show"), 32768, url_list=[origin.url("/ws/")])
        origin.blobs["/t/show.torrent"] = raw
        w = _worker(make_cfg, ep)
        await w.start(health=False)
        await w.submit(api.make_download("tj1", "http", origin.url("/t/show.torrent"), "TV"))
        await _wait_results(w)
        r = w.results[0]
        assert r.outcome == "staged", r
        for rel in ("Season 1/e1.mkv", "Season 1/e2.mkv"):
            assert s3.get("triton-staging", keys.object_key("tj1", rel)) == data[rel]
        assert s3.get("triton-staging", keys.object_key("tj1", "x.mkv")) is None  # extras dropped
        prog = w.telemetry.progress_of("tj1")
        assert prog[0] == 0 and 50 in prog and prog[-1] == 100
        assert all(p <= 50 for p in prog[:prog.index(50)])
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_worker_magnet_job(run, tmp_path, make_cfg):
    async def go():
        from downloader_amd.models import api, keys
        from downloader_amd.s3.fake_server import FakeS3
        s3 = FakeS3()
        ep = await s3.start()
        tr = await Tracker().start()
        raw, data, seeder, _ = await _seed(tmp_path, {"movie.mkv": 250_000}, trackers=[tr.http_url])
        m = parse_torrent(raw)
        w = _worker(make_cfg, ep)
        await w.start(health=False)
        await w.submit(api.make_download("tj2", "torrent", Magnet(m.info_hash, "Pack",
                                                                  [tr.udp_url]).to_uri()))
        await _wait_results(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("tj2", "movie.mkv")) == data["movie.mkv"]
        await w.stop(); await seeder.close(); await tr.stop(); await s3.stop()
    run(go())


def test_worker_metadata_stall_fails_job(run, tmp_path, make_cfg):
    async def go():
        from downloader_amd.models import api
        from downloader_amd.s3.fake_server import FakeS3
        s3 = FakeS3()
        ep = await s3.start()
        w = _worker(make_cfg, ep, download={"torrent_metadata_timeout_s": 0.3},
                    broker={"max_retries": 0})
        await w.start(health=False)
        await w.submit(api.make_download("tj3", "torrent", Magnet(b"\x01" * 20).to_uri()))
        await _wait_results(w)
        assert w.results[0].outcome == "dead"
        assert "Metadata fetch stalled" in w.results[0].error
        assert w.telemetry.statuses_of("tj3") == [2, 6]
        await w.stop(); await s3.stop()
    run(go())


def test_worker_progress_stall_acks(run, tmp_path, make_cfg, origin_cls):
    """A torrent whose only source never delivers -> ERRDLSTALL -> acked and dropped."""
    async def go():
        from downloader_amd.models import api
        from downloader_amd.s3.fake_server import FakeS3
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src"
        _tree(src / "P", {"a.mkv": 100_000})
        raw = make_torrent(str(src / "P"), 16384, url_list=[origin.url("/missing/")])
        origin.blobs["/t.torrent"] = raw
        w = _worker(make_cfg, ep, download={"torrent_stall_timeout_s": 0.4})
        await w.start(health=False)
        await w.submit(api.make_download("tj4", "http", origin.url("/t.torrent")))
        await _wait_results(w)
        assert w.results[0].outcome == "stalled"
        assert w.telemetry.statuses_of("tj4") == [2]
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_worker_torrent_eager_upload_collision_and_parts(run, tmp_path, make_cfg, origin_cls):
    """Eager staging while downloading keeps the reference's key-collision rule (the later
    file in walk order owns the key) and multipart objects are complete and correct."""
    async def go():
        from downloader_amd.models import api, keys
        from downloader_amd.s3.fake_server import FakeS3
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src"
        data = _tree(src / "Show", {"S1/ep.mkv": 9_000_001, "Season 1/ep.mkv": 7_000_003,
                                    "Extras/ep.mkv": 1000})
        for rel, d in data.items():
            origin.blobs["/ws/Show/" + rel] = d
        raw = make_torrent(str(src / "Show"), 65536, url_list=[origin.url("/ws/")])
        origin.blobs["/t/s.torrent"] = raw
        w = _worker(make_cfg, ep)
        await w.start(health=False)
        await w.submit(api.make_download("eg1", "http", origin.url("/t/s.torrent"), "TV"))
        await _wait_results(w)
        assert w.results[0].outcome == "staged", w.results[0]
        k = keys.object_key("eg1", "ep.mkv")
        assert s3.get("triton-staging", k) == data["Season 1/ep.mkv"]
        assert s3.objects("triton-staging")[k].etag.endswith("-2")   # multipart (5 MiB parts)
        assert w.metrics.sample("downloader_key_collisions_total") == 1
        assert not s3.uploads.get("triton-staging")
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_eager_upload_failure_fails_the_job_before_the_download_ends(run, tmp_path, make_cfg,
                                                                     origin_cls):
    """An eager part upload that fails for good (S3 403) fails the job at once; the rest of
    the torrent is not downloaded first (ADVICE-style audit: errors were only surfaced by
    finish(), after the whole payload had arrived)."""
    async def go():
        import time as _time

        from downloader_amd.models import api
        from downloader_amd.s3.fake_server import FakeS3, FaultRule
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src"
        data = _tree(src / "Show", {"Season 1/a.mkv": 1_000_000, "Season 1/b.mkv": 8_000_000})
        for rel, d in data.items():
            origin.blobs["/ws/Show/" + rel] = d
        origin.slow["/ws/Show/Season 1/b.mkv"] = 200_000       # b alone takes ~10 s
        raw = make_torrent(str(src / "Show"), 65536, url_list=[origin.url("/ws/")])
        origin.blobs["/t/s.torrent"] = raw
        s3.faults.add(FaultRule(method="PUT", path_contains="/eg2/", times=100, status=403,
                                code="AccessDenied"))
        w = _worker(make_cfg, ep, download={"torrent_stream": "off", "webseed_chunk": 262144},
                    broker={"max_retries": 0})
        await w.start(health=False)
        t0 = _time.perf_counter()
        await w.submit(api.make_download("eg2", "http", origin.url("/t/s.torrent"), "TV"))
        await _wait_results(w)
        assert w.results[0].outcome == "dead", w.results[0]
        assert _time.perf_counter() - t0 < 3.0
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_webseed_claims_spread_over_files():
    """Streams prefer runs in files no other stream is writing (one file's page-cache write
    path serialises), and fall back to any free run."""
    from downloader_amd.torrent.metainfo import FileEntry, Metainfo
    from downloader_amd.torrent.session import PiecePicker
    from downloader_amd.torrent.storage import Bitfield
    files, off = [], 0
    for i, n in enumerate([16, 0, 16, 16]):
        files.append(FileEntry([f"f{i}"], n, off))
        off += n
    m = Metainfo(b"x" * 20, "t", 4, b"\0" * 20 * (off // 4), files, off, multi_file=True)
    assert [m.file_at(o) for o in (0, 15, 16, 31, 32, 47)] == [0, 0, 2, 2, 3, 3]
    pp = PiecePicker(m, Bitfield(m.num_pieces))
    busy = {}
    got = []
    for _ in range(6):
        first, count = pp.claim_run(8, busy)
        f = m.file_at(first * 4)
        busy[f] = busy.get(f, 0) + 1
        got.append((first, count, f))
    assert [g[2] for g in got[:3]] == [0, 2, 3]            # one stream per file first
    assert sorted(p for g in got for p in range(g[0], g[0] + g[1])) == list(range(12))
    assert pp.claim_run(8, busy) is None


def test_webseed_gpu_verify_path_through_batcher(run, tmp_path, origin_cls, monkeypatch):
    """verify_backend=gpu routes every fetched run through GpuBatcher. The device is stood in
    for by the host verifier here (the real kernel: tests/test_gpu_hash.py), so the CPU tier
    covers the batching, result mapping and a corrupt-run refetch."""
    from downloader_amd.ops import hashing, native

    class HostVerifier:
        def verify_files_streamed(self, files, plen, hashes, chunk=65536, which=()):
            return native().verify_pieces(files, plen, hashes, list(which), 0), (0.0, 0.0)

    monkeypatch.setattr(hashing, "_verifier", lambda: HostVerifier())
    monkeypatch.setattr(hashing, "gpu_available", lambda: True)
    batcher = hashing.GpuBatcher()
    monkeypatch.setattr(hashing, "gpu_batcher", lambda: batcher)

    async def go():
        origin = await origin_cls().start()
        src = tmp_path / "ws"
        data = _tree(src / "Pack", {"a.mkv": 1_000_003, "dir/b.mkv": 377_777})
        raw = make_torrent(str(src / "Pack"), 65536, url_list=[origin.url("/seed/")])
        for rel, d in data.items():
            origin.blobs["/seed/Pack/" + rel] = d
        # the first GET of a.mkv's head serves a corrupt byte -> hash fail -> refetch
        good = data["a.mkv"]
        origin.blobs["/seed/Pack/a.mkv"] = bytes([good[0] ^ 0xFF]) + good[1:]
        c = TorrentClient(webseed_chunk=200_000, webseed_streams=3, verify_backend="gpu")
        await c.start()
        s = await c.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        await asyncio.sleep(0.3)
        origin.blobs["/seed/Pack/a.mkv"] = good
        await asyncio.wait_for(s.wait(), 30)
        _check(tmp_path / "dl", data)
        assert s._gpu_verify is True and batcher.pieces >= s.meta.num_pieces
        assert s.stats["hash_fails"] >= 1
        await c.close(); await origin.stop()
    run(go())


@pytest.mark.parametrize("backend", ["gpu", "auto"])
def test_webseed_verifier_fault_is_never_lost(run, tmp_path, origin_cls, monkeypatch, backend):
    """The GPU verifier raises (HIP fault, OOM, no device) inside a run's verify task. Under
    an explicit ``gpu`` the session fails at once with that error - the pieces are handed
    back, nothing waits for the 240 s stall watchdog; under ``auto`` the run is verified on
    the host instead and the job completes."""
    from concurrent.futures import Future

    from downloader_amd.ops import hashing

    class Broken:
        submitted = 0

        def submit(self, files, plen, hashes, pieces):
            Broken.submitted += 1
            f: Future = Future()
            f.set_exception(RuntimeError("hipErrorIllegalAddress"))
            return f

    monkeypatch.setattr(hashing, "gpu_available", lambda: True)
    monkeypatch.setattr(hashing, "gpu_batcher", lambda: Broken())
    monkeypatch.setattr(hashing, "_gpu_verifier", object())

    async def go():
        origin = await origin_cls().start()
        src = tmp_path / "ws"
        data = _tree(src / "Pack", {"a.mkv": 400_000})
        raw = make_torrent(str(src / "Pack"), 65536, url_list=[origin.url("/seed/")])
        origin.blobs["/seed/Pack/a.mkv"] = data["a.mkv"]
        c = TorrentClient(webseed_chunk=131072, webseed_streams=2, verify_backend=backend)
        await c.start()
        s = await c.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        if backend == "auto":
            s._gpu_verify = True          # as if the warm-verifier policy had picked the GPU
            await asyncio.wait_for(s.wait(), 30)
            _check(tmp_path / "dl", data)
            assert s._gpu_verify is False and Broken.submitted >= 1
        else:
            with pytest.raises(TorrentError, match="hipErrorIllegalAddress"):
                await asyncio.wait_for(s.wait(), 10)
            assert not s.picker.claimed or all(i not in s.have for i in s.picker.claimed)
        await c.close(); await origin.stop()
    run(go())


def test_webseed_serving_corrupt_data_fails_session(run, tmp_path, origin_cls):
    """A webseed that keeps serving a bad piece: the owning stream backs off, gives up after
    webseed_max_failures, and - with no peers/trackers/DHT - the session fails instead of
    waiting forever for a piece nobody fetches."""
    async def go():
        origin = await origin_cls().start()
        src = tmp_path / "ws"
        data = _tree(src / "Pack", {"a.mkv": 300_000})
        raw = make_torrent(str(src / "Pack"), 65536, url_list=[origin.url("/seed/")])
        bad = bytearray(data["a.mkv"])
        bad[70_000] ^= 0xFF                  # flip, never a no-op (writing a constant is 1/256)
        origin.blobs["/seed/Pack/a.mkv"] = bytes(bad)
        c = TorrentClient(webseed_chunk=65536, webseed_streams=2, webseed_max_failures=2)
        await c.start()
        s = await c.add_torrent(parse_torrent(raw), str(tmp_path / "dl"))
        with pytest.raises(TorrentError, match="webseed failed"):
            await asyncio.wait_for(s.wait(), 30)
        assert s.stats["hash_fails"] >= 2 and 1 not in s.have
        await c.close(); await origin.stop()
    run(go())


def test_auto_incremental_verify_policy(monkeypatch):
    """auto: GPU batches only with a warm verifier AND a torrent big enough to amortise the
    ~100 ms batch latency; reference mode never (host, one thread)."""
    from downloader_amd.ops import hashing
    from downloader_amd.torrent import session as S
    from downloader_amd.torrent.metainfo import FileEntry, Metainfo
    monkeypatch.setattr(hashing, "gpu_available", lambda: True)
    monkeypatch.setattr(hashing, "host_multibuffer", lambda: False)   # host without AVX-512

    def sess(backend, total):
        c = TorrentClient(verify_backend=backend, listen=False)
        m = Metainfo(b"y" * 20, "t", 1 << 22, b"\0" * 20, [FileEntry(["t"], total, 0)], total)
        return S.TorrentSession(c, m.info_hash, "/nonexistent", m)
    big, small = S.GPU_INCREMENTAL_MIN_BYTES, S.GPU_INCREMENTAL_MIN_BYTES - 1
    monkeypatch.setattr(hashing, "_gpu_verifier", None)
    assert sess("auto", big)._use_gpu_verify() is False          # cold device
    monkeypatch.setattr(hashing, "_gpu_verifier", object())
    assert sess("auto", big)._use_gpu_verify() is True
    assert sess("auto", small)._use_gpu_verify() is False
    assert sess("cpu", big)._use_gpu_verify() is False
    assert sess("gpu", 1)._use_gpu_verify() is True
    monkeypatch.setattr(hashing, "host_multibuffer", lambda: True)    # AVX-512 host: CPU wins
    assert sess("auto", big)._use_gpu_verify() is False
    assert sess("gpu", 1)._use_gpu_verify() is True
    from downloader_amd.utils.config import load_config
    ref = load_config(overrides={"mode": "reference"}, env={})
    assert ref.download.verify_backend == "cpu" and ref.download.verify_threads == 1
    assert ref.download.webseed_verify_depth == 1 and not ref.s3.unsigned_payload


def test_websocket_only_trackers_are_dropped(run, tmp_path):
    """ws:// / wss:// trackers hand out WebRTC peers only; like bittorrent-tracker in Node
    without wrtc they are dropped, so a torrent whose only trackers are WebSocket ones and
    whose webseed is dead fails instead of waiting for the 240 s stall watchdog."""
    from downloader_amd.torrent.tracker import supported
    assert supported("http://t/a") and supported("udp://u:1") and supported("https://t/a")
    assert not supported("wss://tracker.example/announce") and not supported("ws://t")
    _tree(tmp_path / "src", {"movie.mkv": 100_000})
    meta = parse_torrent(make_torrent(str(tmp_path / "src" / "movie.mkv"), 16384,
                                      trackers=["wss://tracker.example/announce", "ws://t/a"],
                                      url_list=["http://127.0.0.1:1/"]))

    async def go():
        c = await TorrentClient(listen=False, webseed_max_failures=2).start()
        try:
            s = await c.add_torrent(meta, str(tmp_path / "dl"))
            assert s.trackers == []
            with pytest.raises(TorrentError):
                await asyncio.wait_for(s.wait(), 60)
        finally:
            await c.close()
    run(go())


def test_malformed_remote_input_never_escapes(run, tmp_path):
    """Garbage from the network ends one connection / drops one packet and nothing else:
    a peer's short REQUEST (struct.error) and a DHT query whose ``a`` is a list / whose ``t``
    is a dict. Escaping, they would fail the session or hit the event loop's exception
    handler, which stops the worker."""
    from downloader_amd.torrent.bencode import bencode
    from downloader_amd.torrent.dht import DHTNode
    from downloader_amd.torrent.peer import handshake_bytes, read_handshake

    async def go():
        loop_errors = []
        asyncio.get_running_loop().set_exception_handler(lambda lp, ctx: loop_errors.append(ctx))
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 200_000})
        m = parse_torrent(raw)
        sess = seeder.sessions[m.info_hash]
        r, w = await asyncio.open_connection("127.0.0.1", seeder.listen_port)
        w.write(handshake_bytes(m.info_hash, b"-XX0001-" + b"0" * 12, True))
        await read_handshake(r)
        w.write(struct.pack(">IB", 5, 6) + b"\0\0\0\0")       # REQUEST with 4 of 12 bytes
        await w.drain()
        await asyncio.wait_for(r.read(), 5)                    # the seeder hangs up on us
        w.close()
        assert sess.error is None and not sess.failed.is_set()
        assert sess.stats.get("peer_protocol_errors", 0) >= 1
        # the seeder still serves a well-behaved leecher
        leech = await TorrentClient().start()
        s = await leech.add_torrent(m, str(tmp_path / "dl"), peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 30)
        _check(tmp_path / "dl", data)
        await leech.close(); await seeder.close()
        node = await DHTNode(host="127.0.0.1").start()
        probe = await DHTNode(host="127.0.0.1").start()
        for pkt in (bencode({"t": "aa", "y": "q", "q": "ping", "a": [1, 2]}),
                    bencode({"t": {"x": 1}, "y": "r", "r": {}}),
                    bencode({"t": "ab", "y": "q", "q": "announce_peer",
                             "a": {"id": b"i" * 20, "info_hash": [1], "port": "x", "token": b""}}),
                    b"d1:y1:qe", b"\xff" * 40):
            probe.transport.sendto(pkt, ("127.0.0.1", node.port))
        await asyncio.sleep(0.2)
        assert await probe.ping(("127.0.0.1", node.port)) == node.id    # still answering
        await node.close(); await probe.close()
        assert not loop_errors, loop_errors
    run(go())


def test_native_wire_hostile_peer(run, tmp_path):
    """Garbage over the native wire ends that connection only: a length prefix past 2 MiB is
    refused by the native framer, PIECE messages for pieces nobody asked for are dropped, a
    REQUEST while choked or for a piece out of range never reaches the storage; the seeder
    keeps serving a well-behaved leecher."""
    from downloader_amd.torrent.peer import handshake_bytes, read_handshake

    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 200_000})
        m = parse_torrent(raw)
        sess = seeder.sessions[m.info_hash]
        assert sess.wire is not None
        for bad in (struct.pack(">I", 0xFFFFFFF0) + b"x" * 64,              # oversize frame
                    struct.pack(">IBII", 9 + 5, 7, 3, 0) + b"junk!" +      # unrequested PIECE
                    struct.pack(">IBIII", 13, 6, 99, 0, 16384) +            # REQUEST, choked
                    struct.pack(">IBIII", 13, 6, 0, 0, 1 << 30) +           # absurd length
                    struct.pack(">I", 0xFFFFFFF0)):
            r, w = await asyncio.open_connection("127.0.0.1", seeder.listen_port)
            w.write(handshake_bytes(m.info_hash, b"-XX0001-" + b"1" * 12, True))
            await read_handshake(r)
            w.write(bad)
            await w.drain()
            got = await asyncio.wait_for(r.read(), 5)          # the seeder hangs up on us
            assert struct.pack(">IB", 9 + 16384, 7) not in got   # nothing was served
            w.close()
        assert sess.error is None and not sess.failed.is_set()
        assert sess.wire.stats()["served_bytes"] == 0
        leech = await TorrentClient().start()
        s = await leech.add_torrent(m, str(tmp_path / "dl"), peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 30)
        _check(tmp_path / "dl", data)
        assert sess.wire.stats()["served_bytes"] >= m.total_length
        await leech.close(); await seeder.close()
    run(go())


async def _unchoked_raw_peer(seeder, m):
    """A raw BEP-3 connection to the seeder that asked to be unchoked and was."""
    from downloader_amd.torrent.peer import handshake_bytes, read_handshake
    r, w = await asyncio.open_connection("127.0.0.1", seeder.listen_port)
    w.write(handshake_bytes(m.info_hash, b"-XX0001-" + b"2" * 12, False))
    await read_handshake(r)
    w.write(struct.pack(">IB", 1, 2))                           # INTERESTED
    await w.drain()
    while True:                                                  # until UNCHOKE (id 1)
        n = struct.unpack(">I", await asyncio.wait_for(r.readexactly(4), 10))[0]
        body = await r.readexactly(n) if n else b""
        if body[:1] == b"\x01":
            return r, w


def test_native_wire_request_flood_is_bounded(run, tmp_path):
    """an unchoked peer that floods REQUESTs faster than the blocks go out (it never
    reads) is disconnected once kMaxServeQueue blocks wait on its connection, instead of the
    queue growing without bound; the seeder keeps serving others."""
    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 8 << 20}, piece=1 << 20)
        m = parse_torrent(raw)
        sess = seeder.sessions[m.info_hash]
        assert sess.wire is not None
        r, w = await _unchoked_raw_peer(seeder, m)
        flood = b"".join(struct.pack(">IBIII", 13, 6, i % 8, 0, 131072) for i in range(5000))
        w.write(flood)
        try:
            await w.drain()
        except ConnectionError:
            pass
        for _ in range(200):
            if sess.wire.stats()["serve_floods"]:
                break
            await asyncio.sleep(0.05)
        st = sess.wire.stats()
        assert st["serve_floods"] == 1
        assert st["served_bytes"] < 5000 * 131072 // 4      # far from every request answered
        w.close()
        leech = await TorrentClient().start()
        s = await leech.add_torrent(m, str(tmp_path / "dl"), peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 30)
        _check(tmp_path / "dl", data)
        await leech.close(); await seeder.close()
    run(go())


def test_native_wire_cancel_drops_a_queued_block(run, tmp_path):
    """A CANCEL for a block still queued on the native wire (the peer is not reading, so the
    socket is full) removes it: it is never sent, and the others are."""
    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 8 << 20}, piece=1 << 20)
        m = parse_torrent(raw)
        sess = seeder.sessions[m.info_hash]
        r, w = await _unchoked_raw_peer(seeder, m)
        reqs = [(i % 8, (i // 8) * 131072, 131072) for i in range(64)]   # 8 MiB, not read yet
        w.write(b"".join(struct.pack(">IBIII", 13, 6, *q) for q in reqs))
        await w.drain()
        await asyncio.sleep(0.3)                   # the socket buffers fill, the rest queue
        cancelled = reqs[-16:]
        w.write(b"".join(struct.pack(">IBIII", 13, 8, *q) for q in cancelled))
        await w.drain()
        got = set()
        while len(got) < len(reqs):
            try:
                n = struct.unpack(">I", await asyncio.wait_for(r.readexactly(4), 2))[0]
            except asyncio.TimeoutError:
                break
            body = await r.readexactly(n) if n else b""
            if body[:1] == b"\x07":
                idx, begin = struct.unpack(">II", body[1:9])
                got.add((idx, begin))
        st = sess.wire.stats()
        assert st["serve_cancels"] >= 1
        assert len(got) == len(reqs) - st["serve_cancels"]
        assert all((q[0], q[1]) not in got for q in cancelled[-st["serve_cancels"]:])
        w.close()
        await seeder.close()
    run(go())


def test_piece_picker_buckets_and_interest_counts():
    """Randomised check of the bucketed rarest-first picker against brute force: every piece
    started is a candidate of minimal availability among those the peer has; per-peer
    interest counts match a full recount; a 20k-piece torrent is picked in O(1) per piece."""
    import random as _r
    import time as _t

    from downloader_amd.torrent.metainfo import FileEntry, Metainfo
    from downloader_amd.torrent.session import PiecePicker
    from downloader_amd.torrent.storage import Bitfield

    rng = _r.Random(7)
    n = 300
    m = Metainfo(b"x" * 20, "t", 16384, b"\0" * 20 * n, [FileEntry(["t"], n * 16384, 0)],
                 n * 16384)
    have = Bitfield(n)
    pk = PiecePicker(m, have)
    peers = {}
    for step in range(1500):
        op = rng.random()
        if op < 0.08 or not peers:
            bf = Bitfield(n)
            for i in rng.sample(range(n), rng.randrange(1, n)):
                bf.set(i)
            pid = step
            peers[pid] = bf
            pk.add_peer(bf, pid)
        elif op < 0.12 and len(peers) > 1:
            pid = rng.choice(list(peers))
            pk.remove_peer(peers.pop(pid), pid)
        elif op < 0.3:
            pid = rng.choice(list(peers))
            i = rng.randrange(n)
            if peers[pid].set(i):
                pk.inc(i, pid)
        elif op < 0.8:
            pid = rng.choice(list(peers))
            bf = peers[pid]
            cands = [i for i in range(n) if i in bf and i not in have and i not in pk.active
                     and i not in pk.verifying and i not in pk.claimed]
            got = pk._take_rarest(bf)
            if not cands:
                assert got == -1
                continue
            assert got in cands and pk.avail[got] == min(pk.avail[i] for i in cands)
            pk.active[got] = object()          # started
        elif op < 0.95 and pk.active:
            i = rng.choice(list(pk.active))
            pk.complete_blocks(i)
            if rng.random() < 0.2:
                pk.requeue(i)                   # hash failure
            else:
                have.set(i)
                pk.piece_done(i)
        else:
            i = rng.randrange(n)
            if pk._cand(i):
                pk.claimed.add(i)
                pk.unclaim([i]) if rng.random() < 0.5 else None
        for pid, bf in peers.items():
            assert pk.want_count[pid] == sum(1 for i in range(n) if i in bf and i not in have)
    # scale: 20k pieces, 32 full seeders
    n = 20000
    m = Metainfo(b"x" * 20, "t", 16384, b"\0" * 20 * n, [FileEntry(["t"], n * 16384, 0)],
                 n * 16384)
    have = Bitfield(n)
    pk = PiecePicker(m, have)
    full = Bitfield(n, b"\xff" * ((n + 7) // 8))
    for pid in range(32):
        pk.add_peer(full, pid)
    t0 = _t.perf_counter()
    seen = set()
    for _ in range(n):
        i = pk._take_rarest(full)
        assert i >= 0 and i not in seen
        seen.add(i)
        pk.active[i] = object()
        pk.complete_blocks(i)
        have.set(i)
        pk.piece_done(i)
    assert pk._take_rarest(full) == -1 and not pk.peer_has_wanted(full, 0)
    assert _t.perf_counter() - t0 < 2.0


def test_peer_read_batch_handles_every_split(run):
    """Messages cut anywhere by the socket (inside the length prefix, inside the body,
    keep-alives in between) come out whole and in order from the chunk parser."""
    from downloader_amd.torrent.peer import PeerConn

    msgs = [(7, b"\x00\x00\x00\x01\x00\x00\x40\x00" + bytes(range(256)) * 64), (4, b"\x00\x00\x00\x09"),
            (1, b""), (20, b"\x00d1:md11:ut_metadatai1eee"), (7, b"\x00" * 8 + b"z" * 100)]
    wire = b""
    for mid, body in msgs:
        wire += len(body + b"x").to_bytes(4, "big") + bytes([mid]) + body
        wire += b"\x00\x00\x00\x00"                                  # keep-alive

    async def go():
        for cut in list(range(1, 12)) + [4096, 16393, 16400, len(wire) - 3]:
            reader = asyncio.StreamReader(limit=1 << 22)
            pc = PeerConn.__new__(PeerConn)
            pc.reader = reader
            got = []

            async def disp(mid, p, got=got):
                got.append((mid, bytes(p)))
            pc._dispatch = disp
            parts = [wire[i:i + cut] for i in range(0, len(wire), cut)]

            async def feed():
                for part in parts:
                    reader.feed_data(part)
                    await asyncio.sleep(0)
                reader.feed_eof()
            f = asyncio.ensure_future(feed())
            with pytest.raises(asyncio.IncompleteReadError):
                while True:
                    await pc._read_batch(reader.readexactly)
            await f
            assert got == msgs, cut
    run(go())


def test_file_spans_bisect_matches_linear_scan():
    """file_spans starts at the first file ending after the offset (bisect) and returns what
    a scan over every file returns, zero-length files included."""
    import random

    from downloader_amd.torrent.bencode import bencode
    from downloader_amd.torrent.metainfo import parse_torrent
    rng = random.Random(7)
    lengths = [rng.choice([0, 1, 5, 16384, 70000, 1 << 20]) for _ in range(300)]
    lengths[0] = max(lengths[0], 1)
    files = [{b"length": n, b"path": [b"f%03d.mkv" % i]} for i, n in enumerate(lengths)]
    total = sum(lengths)
    npieces = -(-total // 16384)
    meta = parse_torrent(bencode({b"info": {b"name": b"t", b"piece length": 16384,
                                            b"pieces": b"\0" * 20 * npieces, b"files": files}}))

    def linear(offset, length):
        out, end = [], offset + length
        for idx, f in enumerate(meta.files):
            fs, fe = f.offset, f.offset + f.length
            if fe <= offset or f.length == 0:
                continue
            if fs >= end:
                break
            out.append((idx, max(fs, offset) - fs, min(fe, end) - max(fs, offset)))
        return out
    for _ in range(2000):
        off = rng.randrange(total)
        ln = rng.randrange(1, min(total - off, 3 << 20) + 1)
        assert meta.file_spans(off, ln) == linear(off, ln)


def test_overlong_path_components_are_shortened():
    """A torrent path component longer than NAME_MAX (255 bytes) would fail with
    ENAMETOOLONG on disk: it is cut to fit, keeping the extension, with a digest of the full
    name so two long names sharing a prefix stay distinct; multi-byte characters are not
    split."""
    from downloader_amd.torrent.metainfo import NAME_MAX, _safe
    a, b = "é" * 200 + "A.mkv", "é" * 200 + "B.mkv"
    sa, sb = _safe(a), _safe(b)
    assert sa != sb and sa.endswith(".mkv") and sb.endswith(".mkv")
    assert len(sa.encode()) <= NAME_MAX and len(sb.encode()) <= NAME_MAX
    sa.encode("utf-8")                                   # still valid UTF-8
    assert _safe("short.mkv") == "short.mkv"
    assert len(_safe("x" * 300).encode()) <= NAME_MAX


def test_dht_table_store_and_reply_source(run):
    """DHT hardening (BEP-5): a full bucket keeps its good nodes and only gives up a stale
    one; announced peers expire after PEER_TTL_S; a reply whose transaction id matches but
    that comes from another address is dropped (the query still times out / gets the real
    answer); find_node / get_peers with a malformed target get a KRPC error."""
    import time as _t

    from downloader_amd.torrent import dht as D
    from downloader_amd.torrent.bencode import bdecode, bencode

    own = b"\0" * 20
    rt = D.RoutingTable(own, k=2)
    now = _t.monotonic()
    ids = [bytes([0x80]) + bytes([i]) * 19 for i in range(1, 4)]     # all in bucket 159
    rt.add(D.Node(ids[0], ("10.0.0.1", 1), now))
    rt.add(D.Node(ids[1], ("10.0.0.2", 1), now))
    rt.add(D.Node(ids[2], ("10.0.0.3", 1), now + 1))                 # bucket full of good nodes
    assert {n.id for n in rt.buckets[159]} == {ids[0], ids[1]}
    rt.buckets[159][0].seen = now - D.STALE_S - 1                     # ids[0] goes questionable
    rt.add(D.Node(ids[2], ("10.0.0.3", 1), now + 1))
    assert {n.id for n in rt.buckets[159]} == {ids[1], ids[2]}

    async def go():
        node = await D.DHTNode(host="127.0.0.1").start()
        probe = await D.DHTNode(host="127.0.0.1", timeout=0.5).start()
        spoof = await D.DHTNode(host="127.0.0.1").start()
        ih = b"h" * 20
        node.store[ih] = {("1.2.3.4", 5): _t.monotonic() - D.PEER_TTL_S - 1,
                          ("1.2.3.5", 6): _t.monotonic()}
        r = await probe.query(("127.0.0.1", node.port), "get_peers", {"info_hash": ih})
        assert [D.unpack_peer(v) for v in r[b"values"]] == [("1.2.3.5", 6)]
        assert list(node.store[ih]) == [("1.2.3.5", 6)]
        # a reply with the next transaction id, sent from a third socket, must not resolve it
        nxt = (probe._tid + 1) & 0xFFFF
        silent = ("127.0.0.1", spoof.port)                 # spoof never answers queries...
        spoof.datagram_received = lambda data, addr: None
        q = asyncio.ensure_future(probe.query(silent, "ping", {}))
        await asyncio.sleep(0.05)
        fake = bencode({"t": struct.pack(">H", nxt), "y": "r", "r": {"id": b"z" * 20}})
        node.transport.sendto(fake, ("127.0.0.1", probe.port))   # ...so this is a forgery
        with pytest.raises(asyncio.TimeoutError):
            await q
        assert probe.bad_packets >= 1 and all(n.id != b"z" * 20 for b in probe.table.buckets for n in b)
        # malformed targets answer 203
        got = asyncio.get_running_loop().create_future()
        probe.datagram_received = lambda data, addr: got.done() or got.set_result(bdecode(data))
        probe.transport.sendto(bencode({"t": b"xy", "y": "q", "q": "find_node",
                                        "a": {"id": b"i" * 20, "target": [1]}}), ("127.0.0.1", node.port))
        e = await asyncio.wait_for(got, 2)
        assert e[b"y"] == b"e" and e[b"e"][0] == 203
        for n in (node, probe, spoof):
            await n.close()
    run(go())


def test_udp_tracker_reply_action_checked(run):
    """BEP-15: a reply whose transaction id matches but whose action is not the one asked
    for (here a scrape reply, action 2, to a connect) is a TrackerError, not a connection
    id read out of the wrong fields."""
    from downloader_amd.torrent.tracker import TrackerError, announce_udp

    class Bad(asyncio.DatagramProtocol):
        def connection_made(self, tr):
            self.tr = tr

        def datagram_received(self, data, addr):
            self.tr.sendto(struct.pack(">II", 2, struct.unpack(">I", data[12:16])[0]) + b"\0" * 12, addr)

    async def go():
        tr, _ = await asyncio.get_running_loop().create_datagram_endpoint(
            Bad, local_addr=("127.0.0.1", 0))
        port = tr.get_extra_info("sockname")[1]
        with pytest.raises(TrackerError, match="action 2"):
            await announce_udp(f"udp://127.0.0.1:{port}/announce", b"h" * 20, b"p" * 20,
                               1, 0, 0, 0, timeout=1.0, retries=0)
        tr.close()
    run(go())


def test_dht_second_hand_nodes_and_id_hijack(run):
    """nodes named in someone else's reply carry seen=0 and never enter the
    routing table by themselves (only after answering us); a known id's address is not
    re-pointed by another host while the entry is good."""
    import time as _t

    from downloader_amd.torrent import dht as D

    own = b"\0" * 20
    rt = D.RoutingTable(own, k=2)
    nid = bytes([0x80]) + b"\1" * 19
    second = D.unpack_nodes(nid + bytes([10, 0, 0, 9]) + struct.pack(">H", 7))
    assert second[0].seen == 0
    rt.add(second[0])
    assert len(rt) == 0                                     # hearsay is not a table entry
    now = _t.monotonic()
    rt.add(D.Node(nid, ("10.0.0.1", 1), now))
    rt.add(D.Node(nid, ("6.6.6.6", 1), now + 1))           # same id, other host: refused
    assert rt.buckets[159][0].addr == ("10.0.0.1", 1)
    rt.add(D.Node(nid, ("6.6.6.6", 1), now + D.STALE_S + 1))   # the old entry went stale
    assert rt.buckets[159][0].addr == ("6.6.6.6", 1)

    async def go():
        a = await D.DHTNode(host="127.0.0.1").start()
        b = await D.DHTNode(host="127.0.0.1").start()
        fake = bytes([0x40]) + b"\2" * 19              # a node b claims exists, that is nobody
        b.table.add(D.Node(fake, ("127.0.0.1", 9), _t.monotonic()))
        await a._find_node_at(("127.0.0.1", b.port), fake)
        await asyncio.sleep(a.timeout + 0.3)            # the ping of the named node times out
        ids = {n.id for bk in a.table.buckets for n in bk}
        assert b.id in ids and fake not in ids
        await a.close()
        await b.close()
    run(go(), timeout=30)


def test_picker_verifying_pieces_are_not_reclaimed_or_verified_twice():
    """a piece whose blocks are all in (being hashed / written) is not handed to
    a webseed run, and the second of two racing follow-ups does not verify it again."""
    from downloader_amd.torrent.metainfo import FileEntry, Metainfo
    from downloader_amd.torrent.session import PiecePicker
    from downloader_amd.torrent.storage import Bitfield
    n = 8
    m = Metainfo(b"x" * 20, "t", 16384, b"\0" * 20 * n, [FileEntry(["t"], n * 16384, 0)],
                 n * 16384)
    pk = PiecePicker(m, Bitfield(n))
    pk.active[3] = object()
    assert pk.complete_blocks(3) is True and 3 in pk.verifying
    assert pk.complete_blocks(3) is False           # the racing follow-up backs off
    start, count = pk.claim_run(8 * 16384)
    claimed = set(range(start, start + count))
    assert 3 not in claimed and claimed == {0, 1, 2}
    start, count = pk.claim_run(8 * 16384)
    assert set(range(start, start + count)) == {4, 5, 6, 7}


def test_storage_close_waits_for_inflight_writes(tmp_path):
    """A piece write running on an executor thread when the session closes its storage
    finishes before the fds are closed; later I/O fails with EBADF, not on a reused fd."""
    import errno
    import threading
    import time

    from downloader_amd.torrent.metainfo import FileEntry, Metainfo
    from downloader_amd.torrent.storage import Storage

    m = Metainfo(b"x" * 20, "t", 1 << 20, b"\0" * 20 * 4, [FileEntry(["t.bin"], 4 << 20, 0)],
                 4 << 20)
    st = Storage(m, str(tmp_path))
    entered = threading.Event()
    real_pwrite = os.pwrite

    def slow_pwrite(fd, data, off):
        entered.set()
        time.sleep(0.2)
        return real_pwrite(fd, data, off)

    os.pwrite = slow_pwrite
    try:
        t = threading.Thread(target=st.write, args=(0, b"a" * (1 << 20)))
        t.start()
        entered.wait(5)
        st.close()                         # waits for the write above
        assert not t.is_alive()
    finally:
        os.pwrite = real_pwrite
    with open(st.paths[0][0], "rb") as f:
        assert f.read(1 << 20) == b"a" * (1 << 20)
    with pytest.raises(OSError) as ei:
        st.write(0, b"b")
    assert ei.value.errno == errno.EBADF


def test_bare_infohash_torrent_ids():
    """parse-torrent 7 (/root/reference/yarn.lock:2519) accepts a bare infohash as the
    torrent id of client.add (/root/reference/lib/download.js:64): 40 hex or 32 base32."""
    import base64

    from downloader_amd.torrent.magnet import bare_infohash, parse_magnet, torrent_id_uri
    ih = hashlib.sha1(b"bare").digest()
    assert bare_infohash(ih.hex()) == ih
    assert bare_infohash(ih.hex().upper()) == ih
    assert bare_infohash(base64.b32encode(ih).decode()) == ih
    assert bare_infohash(base64.b32encode(ih).decode().lower()) == ih
    for other in ("magnet:?xt=urn:btih:" + ih.hex(), "http://x/" + ih.hex() + ".torrent",
                  "/tmp/" + ih.hex(), ih.hex()[:39], ih.hex() + "0", "z" * 40):
        assert bare_infohash(other) is None
        assert torrent_id_uri(other) == other
    m = parse_magnet(torrent_id_uri(ih.hex(), ["udp://127.0.0.1:1/announce"]))
    assert m.info_hash == ih and m.trackers == ["udp://127.0.0.1:1/announce"]
    assert parse_magnet(torrent_id_uri(ih.hex())).trackers == []


def test_worker_stages_a_bare_infohash_via_configured_tracker(run, tmp_path, make_cfg):
    async def go():
        from downloader_amd.models import api, keys
        from downloader_amd.s3.fake_server import FakeS3
        s3 = FakeS3()
        ep = await s3.start()
        tr = await Tracker().start()
        raw, data, seeder, _ = await _seed(tmp_path, {"movie.mkv": 250_000}, trackers=[tr.http_url])
        m = parse_torrent(raw)
        w = _worker(make_cfg, ep, download={"torrent_default_trackers": [tr.http_url]})
        await w.start(health=False)
        await w.submit(api.make_download("bih", "torrent", m.info_hash.hex()))
        await _wait_results(w)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("bih", "movie.mkv")) == data["movie.mkv"]
        await w.stop(); await seeder.close(); await tr.stop(); await s3.stop()
    run(go())


def test_worker_stages_a_base32_infohash_via_the_dht(run, tmp_path, make_cfg):
    """No tracker anywhere: the seeder announces on a local DHT, the worker's client finds
    it from the base32 infohash alone (metadata over ut_metadata, then the pieces)."""
    import base64

    async def go():
        from downloader_amd.models import api, keys
        from downloader_amd.s3.fake_server import FakeS3
        from downloader_amd.torrent.dht import DHTNode
        s3 = FakeS3()
        ep = await s3.start()
        boot = await DHTNode(host="127.0.0.1").start()
        raw, data, _, src = await _seed(tmp_path, {"film.mkv": 180_000})
        seeder = TorrentClient(enable_dht=True, dht_bootstrap=[("127.0.0.1", boot.port)])
        seeder.dht_interval = 0.5
        await seeder.start()
        await seeder.add_torrent(parse_torrent(raw), str(src))
        await asyncio.sleep(1.0)
        ih = parse_torrent(raw).info_hash
        w = _worker(make_cfg, ep, download={"torrent_enable_dht": True,
                                            "torrent_dht_bootstrap": [f"127.0.0.1:{boot.port}"],
                                            "torrent_metadata_timeout_s": 30})
        await w.start(health=False)
        await w.submit(api.make_download("b32", "torrent", base64.b32encode(ih).decode()))
        await _wait_results(w, timeout=45)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("b32", "film.mkv")) == data["film.mkv"]
        await w.stop(); await seeder.close(); await boot.close(); await s3.stop()
    run(go(), timeout=60)


def test_swarm_piece_pool_is_bounded_in_bytes():
    """The native wire's process-wide piece pool keeps released buffers for reuse up to
    download.swarm_pool_mb; lowering the limit frees the idle ones beyond it at once."""
    from downloader_amd.ops import native
    n = native()
    w = n.SwarmWire(1)
    w.set_storage(65536, 4 * 65536, b"\0" * 80, [])
    n.swarm_piece_pool_limit(1 << 30)
    try:
        for i in range(4):
            w.begin_piece(i)
        for i in range(4):
            w.drop_piece(i)
        st = w.stats()
        assert st["pool_in_use"] == 0 and st["pool_idle_bytes"] >= 4 * 65536
        n.swarm_piece_pool_limit(65536)
        assert w.stats()["pool_idle_bytes"] <= 65536
        w.begin_piece(0)
        w.begin_piece(1)
        w.drop_piece(0)
        w.drop_piece(1)
        assert w.stats()["pool_idle_bytes"] <= 65536
    finally:
        n.swarm_piece_pool_limit(1 << 30)
        w.close()


def test_swarm_verify_backend_policy(monkeypatch):
    """`auto` keeps small swarm torrents on the host's multi-buffer SHA-1 and sends big ones
    (or any, on a host without it) to the device when there is one."""
    from downloader_amd.ops import hashing
    gb = 1 << 30
    for mb, dev, size, want in [(True, True, 2 * gb, "cpu"), (True, True, 8 * gb, "gpu"),
                                (True, False, 8 * gb, "cpu"), (False, True, 1 * gb, "gpu"),
                                (False, False, 1 * gb, "cpu")]:
        monkeypatch.setattr(hashing, "host_multibuffer", lambda mb=mb: mb)
        monkeypatch.setattr(hashing, "gpu_available", lambda dev=dev: dev)
        assert hashing.swarm_backend("auto", size, 4 * gb) == want, (mb, dev, size)
    monkeypatch.setattr(hashing, "host_multibuffer", lambda: True)
    monkeypatch.setattr(hashing, "gpu_available", lambda: True)
    assert hashing.swarm_backend("auto", 100 * gb, 0) == "cpu"      # 0: never by size
    assert hashing.swarm_backend("cpu", 100 * gb, 4 * gb) == "cpu"
    assert hashing.swarm_backend("gpu", 1, 4 * gb) == "gpu"


def test_native_wire_gpu_mode_hashes_the_tail_on_the_host(run, tmp_path):
    """GPU mode hands the last pieces of a download (swarm_gpu_tail_bytes, at most a quarter
    of the torrent) to the host SHA-1, so the job does not end waiting out the device."""
    from downloader_amd.ops import hashing, native

    async def go():
        raw, data, seeder, src = await _seed(tmp_path, {"a.mkv": 4_000_000}, piece=65536)
        # (pipeline 2: pieces are started a few at a time, so the first ones are verified
        # before the last quarter is reached - with 16 half the torrent was requested at once
        # and, on a loaded host, completed only after the switch: no piece on the device)
        leech = await TorrentClient(swarm_verify="gpu", pipeline=2,
                                    swarm_gpu_tail_bytes=1 << 30).start()
        meta = parse_torrent(raw)
        s = await leech.add_torrent(meta, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        st = s.wire.stats()
        assert s._host_tail and st["verified"] == meta.num_pieces
        assert 0 < st["gpu_pieces"] < meta.num_pieces and st["verify_batches"] > 0
        # the wire timed the device's pieces (submission -> digest; the auto tail's input)
        assert s.wire.gpu_latency() > 0 and st["gpu_latency_ms_max"] >= st["gpu_latency_ms_mean"] > 0
        await leech.remove(s)
        # a second download reuses the pool's page-locked buffers for its device pieces
        # instead of locking fresh ones (they are taken first, r6/tail)
        locks = st["pool_locks"]
        s = await leech.add_torrent(meta, str(tmp_path / "dl2"),
                                    peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl2", data)
        st2 = s.wire.stats()
        assert st2["gpu_pieces"] > 0 and st2["pool_locks"] - locks <= st2["gpu_pieces"] // 2, \
            (locks, st2["pool_locks"], st2["gpu_pieces"])
        await leech.close(); await seeder.close()

    hashing.use_part_hasher(native().CpuPartHasher(0.002), 4)
    try:
        run(go(), timeout=90)
    finally:
        hashing.use_part_hasher(None)


def test_native_wire_backlog_holds_back_new_pieces(run, tmp_path):
    """Complete pieces waiting for a slow hasher hold their buffers: at swarm_backlog_bytes no
    new piece is started until half of them are through (NEED on conn 0 refills everyone),
    and the download still completes."""
    from downloader_amd.ops import hashing, native

    async def go():
        raw, data, seeder, src = await _seed(tmp_path, {"a.mkv": 3_000_000}, piece=65536)
        # (pipeline 2: a connection starts at 8 pipelines = 16 blocks = 4 pieces queued, so
        # pieces are started a few at a time and the backlog is met)
        leech = await TorrentClient(swarm_verify="gpu", pipeline=2, swarm_gpu_tail_bytes=0,
                                    swarm_backlog_bytes=4 * 65536).start()
        meta = parse_torrent(raw)
        s = await leech.add_torrent(meta, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        st = s.wire.stats()
        assert s.stats["wire_backlogged"] > 0 and st["verified"] == meta.num_pieces
        assert st["backlog_bytes"] == 0
        await leech.close(); await seeder.close()

    hashing.use_part_hasher(native().CpuPartHasher(0.02), 4)
    try:
        run(go(), timeout=90)
    finally:
        hashing.use_part_hasher(None)


@pytest.mark.parametrize("mode", ["host", "device"])
def test_native_wire_fickle_peers_never_stall_the_download(run, tmp_path, mode):
    """Stress of the owned-piece bookkeeping: three peers that choke and unchoke at random
    (dropping what was asked, as BEP-3 allows), answer out of order, send stray blocks, and
    hang up; a good seeder joins late. Every piece must verify, with nothing left stuck as
    requested. ``device``: the same with the pieces on a slow GPU part hasher (its host
    double), a 4-piece verify backlog and the last quarter hashed on the host."""
    import random as _r
    from downloader_amd.ops import hashing, native
    from downloader_amd.torrent.peer import handshake_bytes

    async def go():
        raw, data, seeder, _ = await _seed(tmp_path, {"x.mkv": 6_000_000}, piece=65536)
        m = parse_torrent(raw)
        blob = data["x.mkv"]

        def fake(seed):
            rnd = _r.Random(seed)

            async def peer(r, w):
                await r.readexactly(68)
                w.write(handshake_bytes(m.info_hash, b"-XX0001-" + bytes([48 + seed]) * 12,
                                        False))
                bits = bytearray((m.num_pieces + 7) // 8)
                for i in range(m.num_pieces):
                    bits[i // 8] |= 0x80 >> (i % 8)
                w.write(struct.pack(">IB", 1 + len(bits), 5) + bytes(bits))
                w.write(struct.pack(">IB", 1, 1))
                choked, pending = False, []
                try:
                    while True:
                        n = int.from_bytes(await r.readexactly(4), "big")
                        body = await r.readexactly(n) if n else b""
                        if not body or body[0] != 6:
                            continue
                        if choked:
                            if rnd.random() < 0.05:
                                choked = False
                                w.write(struct.pack(">IB", 1, 1))          # UNCHOKE
                            continue                                       # dropped
                        pending.append(struct.unpack(">III", body[1:13]))
                        if len(pending) < 4 and rnd.random() < 0.7:
                            continue
                        rnd.shuffle(pending)                               # out of order
                        for idx, begin, ln in pending:
                            off = idx * m.piece_length + begin
                            w.write(struct.pack(">IBII", 9 + ln, 7, idx, begin) +
                                    blob[off:off + ln])
                        pending = []
                        x = rnd.random()
                        if x < 0.03:
                            w.close()
                            return
                        if x < 0.10:
                            choked = True
                            w.write(struct.pack(">IB", 1, 0))              # CHOKE
                        elif x < 0.13:                                     # stray block
                            i = rnd.randrange(m.num_pieces)
                            w.write(struct.pack(">IBII", 9 + 16384, 7, i, 0) + b"z" * 16384)
                        await w.drain()
                except (asyncio.IncompleteReadError, ConnectionError):
                    pass
            return peer

        servers = [await asyncio.start_server(fake(k), "127.0.0.1", 0) for k in range(3)]
        extra = {} if mode == "host" else dict(swarm_verify="gpu", swarm_gpu_tail_bytes=1 << 30,
                                                 swarm_backlog_bytes=4 * 65536)
        # (pipeline 2: a connection starts at 8 pipelines = 16 blocks, as round 5's 8 x 2 did,
        # so the fickle peers own pieces when they choke or hang up)
        leech = await TorrentClient(pipeline=2, idle_timeout=5.0, **extra).start()
        s = await leech.add_torrent(m, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", sv.sockets[0].getsockname()[1])
                                           for sv in servers])
        await asyncio.sleep(0.5)
        s.add_peers([("127.0.0.1", seeder.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        _check(tmp_path / "dl", data)
        assert s.wire.stats()["verified"] == m.num_pieces
        assert not s.picker.active and not s.picker.loose
        # owned pieces were handed back: by a choking / closing peer, or by the rate loop's
        # slow-peer rule (a fickle peer is often shed before it chokes)
        assert s.stats["wire_released"] + s.stats["slow_released_pieces"] >= 1, (s.stats, s.wire.stats())
        assert s.wire.stats()["assigned"] >= 1
        if mode == "device":
            assert s.wire.stats()["gpu_pieces"] > 0 and s.wire.stats()["backlog_bytes"] == 0
        await leech.close(); await seeder.close()
        for sv in servers:
            sv.close()

    if mode == "device":
        hashing.use_part_hasher(native().CpuPartHasher(0.005), 4)
    try:
        run(go(), timeout=90)
    finally:
        if mode == "device":
            hashing.use_part_hasher(None)


def test_swarm_wire_rx_idle_tracks_the_socket():
    """The idle watchdog asks the native wire when a connection last received (blocks of
    owned pieces are not reported one by one, so Python's own clock would go stale)."""
    import socket as _s
    import time as _t
    from downloader_amd.ops import native
    w = native().SwarmWire(1)
    a, b = _s.socketpair()
    try:
        w.attach(os.dup(a.fileno()), 7, b"")
        _t.sleep(0.3)
        assert w.rx_idle(7) >= 0.25
        b.sendall(struct.pack(">IB", 1, 2))              # INTERESTED
        deadline = _t.monotonic() + 5
        while w.rx_idle(7) > 0.2 and _t.monotonic() < deadline:
            _t.sleep(0.01)
        assert w.rx_idle(7) < 0.2
        assert any(kind == 1 for _, kind, _ in w.poll())   # the message went up
        assert w.rx_idle(12345) == 0.0                   # unknown connection
    finally:
        w.close()
        a.close()
        b.close()
