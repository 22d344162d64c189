"""Streamed staging of webseed-only torrents (torrent/stream.py): webseed -> S3 relay with
in-flight piece verification, boundary pieces assembled from neighbouring parts and gap
fetches, refetch of corrupt data, clean abort, and the gate that picks this path."""
from __future__ import annotations

import asyncio
import hashlib
import os
import types

import pytest

from downloader_amd.models import api, keys
from downloader_amd.s3.fake_server import FakeS3
from downloader_amd.torrent.metainfo import FileEntry, Metainfo, make_torrent, parse_torrent
from downloader_amd.torrent.stream import piece_split


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


def _worker(make_cfg, s3_ep, **over):
    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.service.worker import Worker
    d = {"torrent_enable_dht": False, "progress_interval_s": 0.05}
    d.update(over.pop("download", {}))
    return Worker(make_cfg(s3_ep, download=d, **over), broker=MemoryBroker())


async def _wait(w, n=1, timeout=30.0):
    for _ in range(int(timeout / 0.02)):
        if len(w.results) >= n:
            return
        await asyncio.sleep(0.02)
    raise AssertionError(w.results)


def test_piece_split():
    m = Metainfo(b"x" * 20, "t", 4, b"\0" * 100, [FileEntry(["t"], 18, 0)], 18)
    assert piece_split(m, 0, 8) == (0, 8)        # aligned: two whole pieces
    assert piece_split(m, 1, 8) == (3, 4)        # head 1..4, piece 4..8, tail 8..9
    assert piece_split(m, 5, 2) == (2, 0)        # inside one piece: all head
    assert piece_split(m, 6, 4) == (2, 0)        # straddles 8 without a whole piece
    assert piece_split(m, 14, 4) == (2, 2)       # reaches the end: short last piece is whole
    assert piece_split(m, 17, 1) == (1, 0)


SHOW = {"Extras/x.mkv": 150_000, "Season 1/e1.mkv": 6_500_001, "Season 1/e2.mkv": 300_007,
        "readme.txt": 1_000}


async def _show(tmp_path, origin, plen=131072):
    src = tmp_path / "src"
    data = _tree(src / "Show", SHOW)
    for rel, d in data.items():
        origin.blobs["/ws/Show/" + rel] = d
    raw = make_torrent(str(src / "Show"), plen, url_list=[origin.url("/ws/")])
    origin.blobs["/t/show.torrent"] = raw
    return data, parse_torrent(raw)


def test_stream_job_unaligned_files_gaps_and_refetch(run, tmp_path, make_cfg, origin_cls):
    """Selected files start and end mid-piece; the pieces they share with dropped files
    (Extras, readme) are completed with gap fetches. One corrupt byte inside a part's whole
    pieces and one inside a gap are both caught and refetched; the result is byte-exact and
    the dropped files are (almost) never fetched."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        data, meta = await _show(tmp_path, origin)
        origin.corrupt["/ws/Show/Season 1/e1.mkv"] = [3_000_000, 1]    # whole piece, part 1
        origin.corrupt["/ws/Show/Extras/x.mkv"] = [140_000, 1]          # gap of a boundary piece
        w = _worker(make_cfg, ep)
        await w.start(health=False)
        await w.submit(api.make_download("st1", "http", origin.url("/t/show.torrent"), "TV"))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "staged", r
        t = r.stats["torrent"]
        assert t["staging"] == "stream" and t["hash_fails"] >= 2
        for rel in ("Season 1/e1.mkv", "Season 1/e2.mkv"):
            assert s3.get("triton-staging", keys.object_key("st1", rel)) == data[rel]
        assert s3.objects("triton-staging")[keys.object_key("st1", "e1.mkv")].etag.endswith("-2")
        assert s3.get("triton-staging", keys.object_key("st1", "x.mkv")) is None
        assert not s3.uploads.get("triton-staging")
        # dropped bytes: only the gap slices of the two boundary pieces were fetched
        assert t["gap_bytes"] < 2 * meta.piece_length
        assert t["skipped_bytes"] >= SHOW["Extras/x.mkv"] - meta.piece_length
        ranges = [rg for _, p, rg in origin.requests if p.startswith("/ws/Show/Extras")]
        assert ranges and all(rg and rg.startswith("bytes=") for rg in ranges)
        assert w.metrics.sample("downloader_bytes_verified_total", backend="host") == \
            t["webseed_bytes"] >= SHOW["Season 1/e1.mkv"] + SHOW["Season 1/e2.mkv"]
        prog = w.telemetry.progress_of("st1")
        assert prog[0] == 0 and 50 in prog and prog[-1] == 100
        for dp, _, fns in os.walk(tmp_path / "dl"):
            assert not [f for f in fns if f.endswith(".mkv")], (dp, fns)   # nothing on disk
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_stream_job_persistent_corruption_aborts_cleanly(run, tmp_path, make_cfg, origin_cls):
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        data, _ = await _show(tmp_path, origin)
        origin.corrupt["/ws/Show/Season 1/e1.mkv"] = [6_000_000, 1000]   # part 2, always bad
        w = _worker(make_cfg, ep, broker={"max_retries": 0})
        await w.start(health=False)
        await w.submit(api.make_download("st2", "http", origin.url("/t/show.torrent"), "TV"))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "dead" and "corrupt" in r.error, r
        assert s3.get("triton-staging", keys.object_key("st2", "e1.mkv")) is None
        assert s3.get("triton-staging", keys.object_key("st2", "e2.mkv")) is None   # deleted
        assert s3.get("triton-staging", keys.done_key("st2")) is None
        assert not s3.uploads.get("triton-staging")
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


@pytest.mark.parametrize("plen", [16384, 1 << 20])
def test_stream_matches_disk_path(run, tmp_path, make_cfg, origin_cls, plen):
    """Same job through both staging paths -> identical objects and progress endpoints."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        data, _ = await _show(tmp_path, origin, plen)
        got = {}
        for mode in ("auto", "off"):
            w = _worker(make_cfg, ep, download={"torrent_stream": mode,
                                                "relay_pool_idle_trim_s": 0.3})
            await w.start(health=False)
            jid = f"cmp-{mode}"
            await w.submit(api.make_download(jid, "http", origin.url("/t/show.torrent"), "TV"))
            await _wait(w)
            r = w.results[0]
            assert r.outcome == "staged", r
            assert r.stats["torrent"]["staging"] == ("stream" if mode == "auto" else "disk")
            if mode == "off":   # the whole torrent was downloaded and verified
                assert w.metrics.sample("downloader_bytes_verified_total", backend="host") == \
                    sum(SHOW.values())
            got[mode] = {rel: s3.get("triton-staging", keys.object_key(jid, rel))
                         for rel in ("Season 1/e1.mkv", "Season 1/e2.mkv", "Extras/x.mkv")}
            await w.stop()
        assert got["auto"] == got["off"]
        assert got["auto"]["Season 1/e1.mkv"] == data["Season 1/e1.mkv"]
        # the hashed relay's pooled part buffers are all back after the job, and unmapped
        # once the worker has been idle for relay_pool_idle_trim_s
        from downloader_amd.ops import native
        pool = native().relay_pool_stats()
        assert pool["in_use"] == 0, pool
        await asyncio.sleep(0.5)
        assert native().relay_pool_stats()["idle_bytes"] == 0
        await s3.stop(); await origin.stop()
    run(go())


def test_stream_gate():
    from downloader_amd.torrent.backend import stream_webseeds
    from downloader_amd.utils.config import load_config

    class S3:
        def can_relay(self, u):
            return u.startswith("http://")
    sv = types.SimpleNamespace(s3=S3())
    m = Metainfo(b"x" * 20, "t", 4, b"\0" * 20, [FileEntry(["t"], 4, 0)], 4,
                 url_list=["http://a/t"])
    job = types.SimpleNamespace(attempt=0)
    cfg = load_config(env={})
    assert stream_webseeds(m, job, cfg, sv) == ["http://a/t"]
    assert stream_webseeds(m, types.SimpleNamespace(attempt=1), cfg, sv) == []  # retry: disk
    m.announce = [["http://tracker/announce"]]
    assert stream_webseeds(m, job, cfg, sv) == []                # peers may be the source
    cfg.download.torrent_stream = "always"
    assert stream_webseeds(m, job, cfg, sv) == ["http://a/t"]
    m.url_list.append("https://b/t")                              # TLS seed: no native relay
    assert stream_webseeds(m, job, cfg, sv) == []
    ref = load_config(overrides={"mode": "reference"}, env={})
    m.url_list.pop()
    assert stream_webseeds(m, job, ref, sv) == []


def test_settle_never_queues_a_unit_twice(tmp_path):
    """Boundary piece 2 ([8, 12)) is supplied by file a's tail and file b's head. When it
    fails while a neighbour is still being fetched, the neighbour is flagged and re-fetched
    once its current fetch ends - it is never in the queue twice, and the outstanding count
    that ends the job stays exact."""
    from downloader_amd.torrent.stream import StreamStager
    files = [FileEntry(["a.mkv"], 10, 0), FileEntry(["b.mkv"], 10, 10)]
    m = Metainfo(b"x" * 20, "P", 4, b"\0" * 100, files, 20, multi_file=True)
    s3 = types.SimpleNamespace(multipart_threshold=1 << 20, plan_parts=lambda n, *a: [(1, 0, n)])
    root = str(tmp_path)
    sel = [os.path.join(root, "P", "a.mkv"), os.path.join(root, "P", "b.mkv")]
    st = StreamStager(m, types.SimpleNamespace(id="j"),
                      types.SimpleNamespace(s3=types.SimpleNamespace(bucket="b")),
                      types.SimpleNamespace(s3=s3), sel, root, ["http://x/"])
    a, b = st.units
    assert len(st.units) == 2 and st.suppliers[2] == {a.uid, b.uid}   # no gaps needed
    q = asyncio.Queue()
    st._outstanding = 2
    a.state = b.state = "running"
    for u in (a, b):
        u.counted = True
        st.done_bytes += u.length
    st._settle(a, [], q)                      # a done
    assert (a.state, st._outstanding, q.qsize()) == ("done", 1, 0)
    st._settle(b, [a, b], q)                  # piece 2 failed when b delivered: both again
    assert (a.state, b.state, st._outstanding, q.qsize()) == ("queued", "queued", 2, 2)
    assert st.done_bytes == 0 and not a.counted
    q.get_nowait(), q.get_nowait()
    a.state = b.state = "running"
    st._settle(a, [a, b], q)                  # fails again while b is still running
    assert (a.state, b.again, q.qsize(), st._outstanding) == ("queued", True, 1, 2)
    st._settle(b, [], q)                      # b's stale fetch ends: re-queued, not done
    assert (b.state, b.again, q.qsize(), st._outstanding) == ("queued", False, 2, 2)
    q.get_nowait(), q.get_nowait()
    a.state = b.state = "running"
    st._settle(a, [], q)
    st._settle(b, [], q)
    assert st._outstanding == 0 and st._finished.is_set() and q.qsize() == 0


def test_check_piece_discards_stale_verdict(run, tmp_path, monkeypatch):
    """A 1 MiB boundary piece is hashed in an executor. While that hash runs, ``_settle``
    requeues one supplier (dropping its fragment). The in-flight verdict is stale and must
    not mark the piece verified: otherwise the supplier's re-fetched - here corrupt - bytes
    would never be checked (version counter per piece)."""
    import hashlib
    import threading

    from downloader_amd.torrent import stream as stream_mod
    from downloader_amd.torrent.stream import StreamStager

    plen = 1 << 20
    data = os.urandom(3 * plen)
    half = 3 * plen // 2
    files = [FileEntry(["a.mkv"], half, 0), FileEntry(["b.mkv"], half, half)]
    pieces = b"".join(hashlib.sha1(data[i:i + plen]).digest() for i in range(0, 3 * plen, plen))
    m = Metainfo(b"x" * 20, "P", plen, pieces, files, 3 * plen, multi_file=True)
    s3 = types.SimpleNamespace(multipart_threshold=1 << 30, plan_parts=lambda n, *a: [(1, 0, n)])
    root = str(tmp_path)
    sel = [os.path.join(root, "P", "a.mkv"), os.path.join(root, "P", "b.mkv")]
    st = StreamStager(m, types.SimpleNamespace(id="j"),
                      types.SimpleNamespace(s3=types.SimpleNamespace(bucket="b")),
                      types.SimpleNamespace(s3=s3), sel, root, ["http://x/"])
    a, b = st.units
    assert st.suppliers[1] == {a.uid, b.uid}
    gate, entered = threading.Event(), threading.Event()
    real = stream_mod._sha1v

    def slow_sha1(parts):
        entered.set()
        gate.wait(10)
        return real(parts)

    async def go():
        q = asyncio.Queue()
        st._outstanding = 2
        a.state, b.state = "done", "running"
        st.frags[1][plen] = data[plen:half]                 # a's tail
        st.frags[1][half] = data[half:2 * plen]             # b's head
        st.frag_ver[1] = 2
        monkeypatch.setattr(stream_mod, "_sha1v", slow_sha1)
        chk = asyncio.ensure_future(st._check_piece(1))
        while not entered.is_set():
            await asyncio.sleep(0.005)
        st._settle(b, [b], q)                               # b's fragment dropped mid-hash
        gate.set()
        assert await chk is False and 1 not in st.verified
        monkeypatch.setattr(stream_mod, "_sha1v", real)
        bad = bytearray(data[half:2 * plen])
        bad[7] ^= 0xFF
        st.frags[1][half] = bytes(bad)                      # the re-fetch brings bad bytes
        st.frag_ver[1] += 1
        assert await st._check_piece(1) is True             # ... and they ARE checked
        assert 1 not in st.verified and st.hash_fails == 1
        st.frags[1][half] = data[half:2 * plen]
        st.frag_ver[1] += 1
        assert await st._check_piece(1) is False and 1 in st.verified
    run(go())


@pytest.mark.parametrize("mode", ["auto", "off"])
def test_webseeds_that_redirect(run, tmp_path, make_cfg, origin_cls, mode):
    """Webseed file URLs answering 302 to a mirror: the hashed relay (stream staging) and the
    session's spliced Range GETs (disk staging) both follow to the mirror."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        data, _ = await _show(tmp_path, origin)
        for rel in SHOW:
            origin.blobs["/mirror/Show/" + rel] = origin.blobs.pop("/ws/Show/" + rel)
            origin.redirect["/ws/Show/" + rel] = (302, origin.url("/mirror/Show/" + rel))
        w = _worker(make_cfg, ep, download={"torrent_stream": mode})
        await w.start(health=False)
        await w.submit(api.make_download("rdt", "http", origin.url("/t/show.torrent"), "TV"))
        await _wait(w)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert r.stats["torrent"]["staging"] == ("stream" if mode == "auto" else "disk")
        for rel in ("Season 1/e1.mkv", "Season 1/e2.mkv"):
            assert s3.get("triton-staging", keys.object_key("rdt", rel)) == data[rel]
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


def test_piece_aligned_part_plan():
    """Interior part boundaries of a file at an unaligned torrent offset land on piece
    boundaries (only the file's two end pieces straddle a part/file edge); parts stay >= 5 MiB
    except the last, and cover the file exactly."""
    from downloader_amd.s3.client import MIN_PART, S3Client
    c = S3Client("127.0.0.1:9", "a", "b", part_size=64 << 20)
    plen = 4 << 20
    for off, size in ((12345, 300 << 20), (0, 200 << 20), (plen - 1, 129 << 20),
                      (7 << 20, (64 << 20) + 1), (123, 64 << 20)):
        parts = c.plan_parts(size, off, plen)
        assert parts[0][1] == 0 and sum(ln for _, _, ln in parts) == size
        assert all(o1 + l1 == o2 for (_, o1, l1), (_, o2, _) in zip(parts, parts[1:]))
        assert [n for n, _, _ in parts] == list(range(1, len(parts) + 1))
        assert all(ln >= MIN_PART for _, _, ln in parts[:-1])
        for _, o, _ in parts[1:]:
            assert (off + o) % plen == 0, (off, size, parts)
    # part size not a multiple of the piece length: the plain plan
    assert c.plan_parts(200 << 20, 5, 3 << 20) == c.plan_parts(200 << 20)


def test_staged_objects_carry_media_content_types(run, tmp_path, make_cfg, origin_cls):
    """minio-js fPutObject sets Content-Type from the file name (mime-types): every staging
    path - HTTP stream relay, HTTP disk + upload stage, torrent stream staging, torrent eager
    staging - stores video/x-matroska for .mkv (and octet-stream with the flag off)."""
    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        data, _ = await _show(tmp_path, origin)
        origin.blobs["/h/movie.mkv"] = os.urandom(7 << 20)
        origin.blobs["/h/clip.mp4"] = os.urandom(1 << 20)
        jobs = [("ct1", {}, "/h/movie.mkv", "MOVIE"),
                ("ct2", {"stream_http": False}, "/h/clip.mp4", "MOVIE"),
                ("ct3", {}, "/t/show.torrent", "TV"),
                ("ct4", {"torrent_stream": "off"}, "/t/show.torrent", "TV")]
        for jid, dl, path, typ in jobs:
            w = _worker(make_cfg, ep, download=dl)
            await w.start(health=False)
            await w.submit(api.make_download(jid, "http", origin.url(path), typ))
            await _wait(w)
            assert w.results[0].outcome == "staged", w.results[0]
            await w.stop()
        objs = s3.objects("triton-staging")
        assert objs[keys.object_key("ct1", "movie.mkv")].content_type == "video/x-matroska"
        assert objs[keys.object_key("ct2", "clip.mp4")].content_type == "video/mp4"
        for jid in ("ct3", "ct4"):
            assert objs[keys.object_key(jid, "e1.mkv")].content_type == "video/x-matroska"
            assert objs[keys.object_key(jid, "e2.mkv")].content_type == "video/x-matroska"
        w = _worker(make_cfg, ep, s3={"content_type_by_extension": False})
        await w.start(health=False)
        await w.submit(api.make_download("ct5", "http", origin.url("/h/movie.mkv")))
        await _wait(w)
        await w.stop()
        assert objs is not None and s3.objects("triton-staging")[
            keys.object_key("ct5", "movie.mkv")].content_type == "application/octet-stream"
        assert keys.content_type("a/B.MKV") == "video/x-matroska"
        assert keys.content_type("x.webm") == "video/webm" and keys.content_type("x") == \
            "application/octet-stream"
        await s3.stop(); await origin.stop()
    run(go())


@pytest.mark.parametrize("corrupt", [False, True])
def test_stream_async_part_hashing_with_host_double(run, tmp_path, make_cfg, origin_cls, corrupt):
    """The GPU relay-hashing path (stream_verify_backend: gpu) on a host: the native
    CpuPartHasher serves the same C ABI as the gfx950 PartHasher (copy and hash each finish
    later on its own thread). Relay slots are freed after the bytes move, parts are finished in
    continuations, a corrupt piece is caught from the late digests and the part refetched,
    and every buffer lease returns to the pool."""
    from downloader_amd.ops import hashing, native

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(23 * (1 << 20) + 12345)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        if corrupt:
            origin.corrupt["/ws/Movie/m.mkv"] = [9 * (1 << 20) + 5, 1]
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        w = _worker(make_cfg, ep, download={"stream_verify_backend": "gpu",
                                            "stream_gpu_min_pieces": 4, "stream_gpu_tail": 0})
        await w.start(health=False)
        before = native().gpu_part_stats()
        await w.submit(api.make_download("ah", "http", origin.url("/t/m.torrent")))
        await _wait(w, timeout=60)
        r = w.results[0]
        assert r.outcome == "staged", r
        t = r.stats["torrent"]
        assert t["verify"] == "gpu" and t["gpu_parts"] >= 4
        assert s3.get("triton-staging", keys.object_key("ah", "m.mkv")) == data
        assert (t["hash_fails"] >= 1) == corrupt
        after = native().gpu_part_stats()
        assert after["submitted"] - before["submitted"] >= 4 + corrupt
        assert after["host_fallbacks"] == before["host_fallbacks"]
        assert native().relay_pool_stats()["in_use"] == 0        # every lease came back
        await w.stop(); await s3.stop(); await origin.stop()

    hashing.use_part_hasher(native().CpuPartHasher(0.01), 4)
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)


def test_gpu_part_track_failure_releases_budget_and_refetches(run, tmp_path, make_cfg,
                                                            origin_cls, monkeypatch):
    """when tracking a queued GPU part raises (e.g. the eventfd cannot be watched),
    the part is forgotten natively, its budget bytes and GPU slot come back, and the unit is
    refetched - the job still stages every byte and nothing stays leased or pending."""
    from downloader_amd.ops import hashing, native
    real = hashing.gpu_part_track
    calls = {"n": 0}

    def flaky(gid):
        calls["n"] += 1
        if calls["n"] <= 2:
            raise OSError("add_reader failed")
        return real(gid)
    monkeypatch.setattr(hashing, "gpu_part_track", flaky)

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(23 * (1 << 20) + 12345)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        w = _worker(make_cfg, ep, download={"stream_verify_backend": "gpu",
                                            "stream_gpu_min_pieces": 4, "stream_gpu_tail": 0})
        await w.start(health=False)
        await w.submit(api.make_download("tf", "http", origin.url("/t/m.torrent")))
        await _wait(w, timeout=60)
        r = w.results[0]
        assert r.outcome == "staged", r
        assert s3.get("triton-staging", keys.object_key("tf", "m.mkv")) == data
        budget = r.stats["torrent"]["budget"]
        assert budget["used"] == 0 and budget["queued"] == 0     # every byte came back
        assert native().relay_pool_stats()["in_use"] == 0
        assert native().gpu_part_stats()["pending"] == 0
        await w.stop(); await s3.stop(); await origin.stop()

    hashing.use_part_hasher(native().CpuPartHasher(0.01), 4)
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)
    assert calls["n"] >= 3


def test_gpu_part_news_evicted_before_tracking_fails_fast(monkeypatch):
    """news for more untracked parts than the early buffer holds is dropped oldest
    first; tracking such a part later fails it at once (the caller refetches) instead of
    waiting forever for news that already went."""
    import asyncio
    from downloader_amd.ops import hashing

    class FakeNative:
        def __init__(self):
            self.batch = []
            self.rfd, self.wfd = os.pipe()

        def gpu_part_poll(self):
            b, self.batch = self.batch, []
            return b

        def gpu_part_eventfd(self):
            return self.rfd
    fake = FakeNative()
    monkeypatch.setattr(hashing, "native", lambda: fake)
    monkeypatch.setattr(hashing, "EARLY_MAX", 8)
    parts = hashing._GpuParts()
    fake.batch = [(gid, 2, b"d" * 20) for gid in range(1, 13)]     # 12 parts, room for 8
    parts.drain()

    async def go():
        lost = parts.track(1)                   # evicted: fails now
        with pytest.raises(RuntimeError, match="lost"):
            await asyncio.wait_for(lost.done, 1)
        assert lost.copied.done()
        kept = parts.track(12)                  # still buffered: delivered normally
        assert await asyncio.wait_for(kept.done, 1) == b"d" * 20
    asyncio.run(go())
    os.close(fake.rfd); os.close(fake.wfd)


def test_untracked_gpu_parts_still_return_their_buffers(run, origin_cls):
    """Parts queued to the hasher return their buffers to the pool when their DMA is over,
    whether or not anybody waits for the digests (an aborted job cancels its waits): no
    thread blocks per part - completions come through the native eventfd."""
    from downloader_amd.ops import hashing, native
    from downloader_amd.s3.client import S3Client
    from downloader_amd.s3.fake_server import FakeS3

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(4 << 20)
        origin.blobs["/p.bin"] = blob
        c = S3Client(ep, "minioadmin", "minioadmin")
        await c.ensure_bucket("b")
        ids = []
        for i in range(3):
            _, h = await c.relay_hashed("b", f"k{i}", origin.url("/p.bin"), 0, len(blob), True,
                                        (0, len(blob), 1 << 18), gpu=True)
            assert h["gpu_ticket"] and not h["digests"]
            ids.append(h["gpu_ticket"])
        assert len(set(ids)) == 3
        parts = [hashing.gpu_part_track(i) for i in ids]
        waits = [asyncio.ensure_future(p.done) for p in parts]
        await asyncio.sleep(0.01)
        for w in waits[1:]:
            w.cancel()                        # nobody asks for these digests any more
        want = b"".join(hashlib.sha1(blob[i:i + (1 << 18)]).digest()
                        for i in range(0, len(blob), 1 << 18))
        assert await waits[0] == want
        for p in parts:
            await p.copied
        assert native().relay_pool_stats()["in_use"] == 0
        for _ in range(300):
            if native().gpu_part_stats()["pending"] == 0 and hashing._gpu_parts.pending() == 0:
                break
            await asyncio.sleep(0.02)
        assert native().gpu_part_stats()["pending"] == 0
        assert hashing._gpu_parts.pending() == 0
        await c.close(); await origin.stop(); await s3.stop()

    hashing.use_part_hasher(native().CpuPartHasher(0.2), 4)
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)


def test_refused_put_releases_its_queued_part(run, origin_cls):
    """A relayed part the S3 peer refuses (400 BadDigest after a flipped byte) had already been
    queued to the part hasher: the relay waits that ticket out itself, the retry queues a new
    one, and no buffer stays leased."""
    from downloader_amd.ops import hashing, native
    from downloader_amd.s3.client import S3Client
    from downloader_amd.s3.fake_server import FakeS3

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blob = os.urandom(4 << 20)
        origin.blobs["/p.bin"] = blob
        c = S3Client(ep, "minioadmin", "minioadmin")
        await c.ensure_bucket("b")
        before = native().gpu_part_stats()["submitted"]
        s3.corrupt_next = 1
        _, h = await c.relay_hashed("b", "k", origin.url("/p.bin"), 0, len(blob), True,
                                    (0, len(blob), 1 << 18), gpu=True)
        assert s3.bad_digests == 1 and s3.get("b", "k") == blob
        assert native().gpu_part_stats()["submitted"] - before == 2      # refused + retry
        # the retry's lease ends when its DMA does, digests asked for or not
        assert native().relay_pool_stats()["in_use"] <= 1
        digests = await hashing.gpu_part_digests(h["gpu_ticket"])
        assert digests == b"".join(hashlib.sha1(blob[i:i + (1 << 18)]).digest()
                                   for i in range(0, len(blob), 1 << 18))
        assert native().relay_pool_stats()["in_use"] == 0
        await c.close(); await origin.stop(); await s3.stop()

    hashing.use_part_hasher(native().CpuPartHasher(0.01), 4)
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)


def test_stream_survives_part_hasher_failures(run, tmp_path, make_cfg, origin_cls):
    """A device that fails before the DMA out of a part buffer (the relay hashes that part on
    the host) or after it (the bytes are gone: the part is fetched again) still stages the
    exact bytes, and every buffer lease comes back."""
    from downloader_amd.ops import hashing, native

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(19 * (1 << 20) + 4321)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        w = _worker(make_cfg, ep, download={"stream_verify_backend": "gpu",
                                            "stream_gpu_min_pieces": 4, "stream_gpu_tail": 0})
        await w.start(health=False)
        before = native().gpu_part_stats()
        await w.submit(api.make_download("hf", "http", origin.url("/t/m.torrent")))
        await _wait(w, timeout=60)
        r = w.results[0]
        assert r.outcome == "staged", r
        t = r.stats["torrent"]
        assert s3.get("triton-staging", keys.object_key("hf", "m.mkv")) == data
        after = native().gpu_part_stats()
        assert after["host_fallbacks"] > before["host_fallbacks"]      # copy failures
        assert t.get("gpu_failures", 0) >= 1                           # hash failures
        assert native().relay_pool_stats()["in_use"] == 0
        await w.stop(); await s3.stop(); await origin.stop()

    hashing.use_part_hasher(native().CpuPartHasher(0.005, fail_copy_every=3, fail_done_every=4), 4)
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)


@pytest.mark.parametrize("jobs,tail", [(1, 99), (2, 0), (1, 0)])
def test_stream_verify_auto_uses_the_device_when_it_pays(run, tmp_path, make_cfg,
                                                         origin_cls, jobs, tail):
    """``stream_verify_backend: auto`` with a hasher ready: a job with no more parts than the
    host-hashed tail stays on the host; jobs with parts beyond the tail - alone or two at
    once - send those parts to the device (profiles/archive/r3_relayhash4/, r3_tail2/)."""
    from downloader_amd.ops import hashing, native

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(24 * (1 << 20) + 777)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        # 5 MiB parts one at a time: each job is several sequential relays, so two jobs
        # submitted together overlap for most of their parts
        w = _worker(make_cfg, ep, concurrency=2, s3={"part_size": 5 << 20},
                    download={"stream_verify_backend": "auto", "stream_gpu_min_pieces": 4,
                              "stream_gpu_tail": tail, "gpu_prewarm": False,
                              "torrent_stream_parallel": 1})
        await w.start(health=False)
        for i in range(jobs):
            await w.submit(api.make_download(f"au{jobs}-{i}", "http",
                                             origin.url("/t/m.torrent")))
        await _wait(w, n=jobs, timeout=60)
        for i, r in enumerate(sorted(w.results, key=lambda r: r.job_id)):
            assert r.outcome == "staged", r
            assert s3.get("triton-staging", keys.object_key(f"au{jobs}-{i}", "m.mkv")) == data
        gpu_parts = sum(r.stats["torrent"]["gpu_parts"] for r in w.results)
        assert {r.stats["torrent"]["verify"] for r in w.results} == {"auto"}
        if jobs == 1 and tail and hashing.host_multibuffer():
            assert gpu_parts == 0
        else:
            assert gpu_parts > 0
        assert native().relay_pool_stats()["in_use"] == 0
        await w.stop(); await s3.stop(); await origin.stop()

    hashing.use_part_hasher(native().CpuPartHasher(0.01), 4)    # "set up at worker start"
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)


def test_stream_verify_auto_without_a_device_stays_on_the_host(run, tmp_path, make_cfg,
                                                               origin_cls):
    from downloader_amd.ops import hashing

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(6 * (1 << 20) + 5)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        w = _worker(make_cfg, ep, download={"stream_verify_backend": "auto"})
        await w.start(health=False)
        await w.submit(api.make_download("an", "http", origin.url("/t/m.torrent")))
        await _wait(w, timeout=60)
        r = w.results[0]
        assert r.outcome == "staged" and r.stats["torrent"]["verify"] == "auto"
        assert r.stats["torrent"]["gpu_parts"] == 0
        if hashing.host_multibuffer():           # one job on an AVX-512 host: no HIP init
            assert hashing._part_hasher is None
        await w.stop(); await s3.stop(); await origin.stop()

    assert hashing._part_hasher is None
    run(go())


def test_failed_upload_creation_leaves_no_open_upload(run, tmp_path, make_cfg, origin_cls):
    """One file's CreateMultipartUpload fails while another's is still in flight: the job
    fails and every upload that was opened is aborted (the slow creation is not orphaned)."""
    from downloader_amd.s3.fake_server import FaultRule

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        await _show(tmp_path, origin)
        s3.faults.add(FaultRule(method="POST", path_contains=keys.object_key("st9", "e1.mkv"),
                                query_contains="uploads",
                                status=0, delay_s=0.3, times=1))
        s3.faults.add(FaultRule(method="POST", path_contains=keys.object_key("st9", "e2.mkv"),
                                query_contains="uploads",
                                status=500, code="InternalError", times=99))
        w = _worker(make_cfg, ep, broker={"max_retries": 0},
                    s3={"multipart_threshold": 200_000, "retries": 0})
        await w.start(health=False)
        await w.submit(api.make_download("st9", "http", origin.url("/t/show.torrent"), "TV"))
        await _wait(w)
        assert w.results[0].outcome == "dead", w.results
        await asyncio.sleep(0.5)
        assert not s3.uploads.get("triton-staging"), s3.uploads
        await w.stop(); await s3.stop(); await origin.stop()
    run(go())


@pytest.mark.parametrize("backend", ["cpu", "gpu"])
def test_two_streamed_torrents_stay_inside_the_part_budget(run, tmp_path, make_cfg, origin_cls,
                                                           backend):
    """Two streamed torrents at once, 16 relays in flight each, 5 MiB parts (6 MiB buffers):
    unbounded they would lease 192 MiB of part buffers. Under a 24 MiB budget the native pool's
    high-water mark (leased + idle) never passes it, no lease is granted past it, and both jobs
    stage the exact bytes - on the host path and on the asynchronous GPU path (host double),
    where a part's bytes return to the budget when its DMA is over."""
    from downloader_amd.ops import hashing, native

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blobs = {}
        for j in range(2):
            src = tmp_path / f"src{j}" / "Movie"
            src.mkdir(parents=True)
            data = os.urandom(40 * (1 << 20) + 4321 * j)
            (src / "m.mkv").write_bytes(data)
            origin.blobs[f"/ws{j}/Movie/m.mkv"] = data
            origin.blobs[f"/t/m{j}.torrent"] = make_torrent(str(src), 1 << 18,
                                                           url_list=[origin.url(f"/ws{j}/")])
            blobs[j] = data
        native().relay_pool_trim()
        native().relay_pool_reset_peak()
        w = _worker(make_cfg, ep, concurrency=2, s3={"part_size": 5 << 20},
                    download={"stream_verify_backend": backend, "stream_gpu_min_pieces": 4,
                              "stream_gpu_tail": 0, "torrent_stream_parallel": 16,
                              "relay_memory_mb": 24, "relay_pool_idle_trim_s": 0})
        await w.start(health=False)
        for j in range(2):
            await w.submit(api.make_download(f"bud{j}", "http", origin.url(f"/t/m{j}.torrent")))
        await _wait(w, n=2, timeout=120)
        for r in w.results:
            assert r.outcome == "staged", r
        for j in range(2):
            assert s3.get("triton-staging", keys.object_key(f"bud{j}", "m.mkv")) == blobs[j]
        st = native().relay_pool_stats()
        assert st["budget"] == 24 << 20
        assert 0 < st["peak_bytes"] <= 24 << 20, st
        assert st["over_budget"] == 0, st
        assert st["in_use"] == 0 and st["idle_bytes"] == 0      # trimmed after the last job
        tstats = [r.stats["torrent"] for r in w.results]
        assert sum(t["budget"]["waits"] for t in tstats) > 0     # the budget did the bounding
        assert all(t["budget"]["peak"] <= 24 << 20 for t in tstats)
        if backend == "gpu":
            assert sum(t["gpu_parts"] for t in tstats) > 0
        await w.stop(); await s3.stop(); await origin.stop()
        native().relay_pool_set_budget(0)

    if backend == "gpu":
        hashing.use_part_hasher(native().CpuPartHasher(0.01), 4)
    try:
        run(go())
    finally:
        if backend == "gpu":
            hashing.use_part_hasher(None)


def test_job_end_trims_idle_buffers_to_one_jobs_worth(run, tmp_path, make_cfg, origin_cls):
    """When the last streamed job ends, idle part buffers beyond what one job's relays in
    flight use are unmapped at once (6.8 GB stayed idle until the 60 s trim);
    the rest stays warm for the next job until relay_pool_idle_trim_s. Parts awaiting their
    (slow, host-double) DMA hold buffers beyond the relays in flight, so the pool grows past
    one job's worth during the job."""
    from downloader_amd.ops import hashing, native

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(40 * (1 << 20) + 99)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        native().relay_pool_trim()
        native().relay_pool_reset_peak()
        w = _worker(make_cfg, ep, s3={"part_size": 5 << 20},
                    download={"stream_verify_backend": "gpu", "stream_gpu_min_pieces": 4,
                              "stream_gpu_tail": 0, "torrent_stream_parallel": 2,
                              "relay_memory_mb": 64, "relay_pool_idle_trim_s": 60})
        await w.start(health=False)
        await w.submit(api.make_download("tr", "http", origin.url("/t/m.torrent")))
        await _wait(w, timeout=120)
        assert w.results[0].outcome == "staged", w.results[0]
        assert s3.get("triton-staging", keys.object_key("tr", "m.mkv")) == data
        st = native().relay_pool_stats()
        assert st["peak_bytes"] > 2 * (6 << 20), st         # parts awaiting DMA held more
        assert 0 < st["idle_bytes"] <= 2 * (6 << 20), st     # one job's worth kept warm
        await w.stop(); await s3.stop(); await origin.stop()
        native().relay_pool_trim()
        native().relay_pool_set_budget(0)

    hashing.use_part_hasher(native().CpuPartHasher(0.08), 4)
    try:
        run(go())
    finally:
        hashing.use_part_hasher(None)


def test_part_hasher_layout_comes_from_the_config(monkeypatch):
    """``download.stream_gpu_slots / _slot_mb / _copy_streams / _compute_streams`` reach the
    PartHasher's constructor arguments (slot size sets how many lanes one launch can hash)."""
    from downloader_amd.ops import hashing
    from downloader_amd.torrent import stream
    from downloader_amd.utils.config import Config
    seen = []
    monkeypatch.setattr(hashing, "_part_hasher", None)
    monkeypatch.setattr(hashing, "gpu_relay_hashing",
                        lambda *a, **k: seen.append((a, k)) or True)
    cfg = Config.model_validate({"download": {"stream_gpu_slots": 8, "stream_gpu_slot_mb": 2048,
                                              "stream_gpu_copy_streams": 1,
                                              "stream_gpu_compute_streams": 3}})
    assert stream._gpu_relay_on(cfg) is None
    (a, k), = seen
    assert a[1:] == (8, 2 << 30) and k == {"copy_streams": 1, "compute_streams": 3}


def test_cancelled_relay_does_not_hang_on_a_stuck_gpu_forget(run):
    """a cancelled relay waits for gpu_part_forget (its part's buffer must be back
    before the budget is), but only FORGET_WAIT_S: a device that stopped answering returns the
    future of the forget instead, and the caller keeps the part's budget bytes until it ends."""
    import threading

    from downloader_amd.net.http import NativeTransport

    release = threading.Event()
    calls = []

    class SlowNative:
        def gpu_part_forget(self, gid):
            calls.append(gid)
            release.wait(10)

    t = NativeTransport.__new__(NativeTransport)
    t._n = SlowNative()
    t.FORGET_WAIT_S = 0.2

    async def go():
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        fut.set_result((None, None, None, {"gpu_ticket": 42}))
        t0 = loop.time()
        held = await t._forget_ticket(fut)
        assert loop.time() - t0 < 2 and held is not None and not held.done()
        released = []
        from downloader_amd.torrent.stream import StreamStager

        class Budget:
            def release(self, nb):
                released.append(nb)
        st = StreamStager.__new__(StreamStager)
        st._budget = Budget()
        e = asyncio.CancelledError()
        e.held_until = held
        st._release_after(e, 7)
        assert released == []                      # held while the forget is blocked
        release.set()
        await asyncio.wait_for(held, 5)
        await asyncio.sleep(0)
        assert released == [7] and calls == [42]
        st._release_after(RuntimeError("x"), 3)     # no hold: back at once
        assert released == [7, 3]
    run(go(), timeout=30)


@pytest.mark.parametrize("mode", ["0", "1", "2"])
def test_streamed_part_staging_keeps_bytes_and_digests(mode):
    """STAGER_PART_NT (csrc/transfer.cpp ``part_nt_mode``): parts peeked into an L2-sized
    buffer and streamed into the part buffer with non-temporal stores relay, hash and catch
    corruption exactly like parts peeked straight into it (0; 1, the default: device-bound
    parts, which the host double stands in for; 2: every hashed part). The mode is read once
    per process, so the stream tests run again in a child with it set."""
    import subprocess
    import sys
    env = dict(os.environ, STAGER_PART_NT=mode)
    code = ("import sys, pytest\n"
            f"rc = pytest.main(['-q', '-x', '-m', 'not gpu', '-p', 'no:cacheprovider', {__file__!r},"
            " '-k', 'stream_matches_disk_path or async_part_hashing_with_host_double'])\n"
            "from downloader_amd.ops import native\n"
            "print('NT_STAGED', native().relay_counters()['nt_staged_bytes'])\n"
            "sys.exit(int(rc))\n")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    staged = int(r.stdout.split("NT_STAGED")[1].split()[0])
    if mode == "0":
        assert staged == 0
    else:
        assert staged >= 23 << 20, r.stdout[-1000:]    # at least the host double's torrent
