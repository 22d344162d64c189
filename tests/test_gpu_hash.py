"""gfx950 batched SHA-1 kernel vs a CPU reference (hashlib) - needs a real MI355X."""
from __future__ import annotations

import hashlib
import os
import time

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gv():
    from downloader_amd.ops import gpu_available, gpuhash
    if not gpu_available():
        pytest.fail("HIP device not visible: the GPU test tier must run on a MI355X")
    assert "gfx950" in gpuhash().arch()
    return gpuhash().GpuVerifier(0, 64 << 20, 8)


def ref(data, piece):
    return b"".join(hashlib.sha1(data[i:i + piece]).digest() for i in range(0, len(data), piece))


@pytest.mark.parametrize("piece,n", [
    (16384, 64 * 16384),            # one full wavefront, aligned
    (16384, 100 * 16384 + 5),       # short last piece (5 bytes)
    (262144, 33 * 262144 + 55),     # tail that needs 1 padding block
    (262144, 7 * 262144 + 60),      # tail >= 56 -> 2 padding blocks
    (1000, 257 * 1000 + 999),       # piece_len % 16 != 0 -> dword path
    (999, 300 * 999),               # odd piece length -> byte path
    (64, 64 * 5000),                # many tiny pieces, > 1 workgroup
    (192, 192 * 200 + 64 * 3 + 7),  # odd block count (3): prefetch pair loop + odd block
    (1008, 1008 * 129 + 330),       # 15 whole blocks + tail, last piece 5 blocks
])
def test_hash_buffer_matches_hashlib(gv, piece, n):
    data = os.urandom(n)
    assert gv.hash_buffer(data, piece) == ref(data, piece)


def test_kernel_ab_timings(gv):
    """The prefetch / no-prefetch kernel A/B used by verify_bench runs and times both."""
    pf, nopf = gv.kernel_bench_prefetch(65536, 256, 1)
    b3, plain = gv.kernel_bench(65536, 256, 1)
    assert min(pf, nopf, b3, plain) > 0
    with pytest.raises(ValueError):
        gv.kernel_bench_prefetch(1000, 256, 1)


def test_kernel_prefetch_keeps_its_speedup(gv):
    """Perf guard for the block prefetch (profiles/archive/r2_kpf: 1.37x per lane, A/B in one
    process, so box-to-box variance cancels)."""
    pf, nopf = gv.kernel_bench_prefetch(1 << 20, 4096, 2)
    assert nopf / pf > 1.15, (pf, nopf)
    b3, plain = gv.kernel_bench(1 << 20, 4096, 2)
    assert plain / b3 > 1.05, (b3, plain)


def test_multi_batch_pipeline(gv):
    # 64 MiB staging slots, 200 MiB of data -> 4 batches through both streams
    piece = 1 << 20
    data = os.urandom(200 * piece + 12345)
    assert gv.hash_buffer(data, piece) == ref(data, piece)


def test_verify_files_detects_corruption(gv, tmp_path):
    piece = 65536
    sizes = [3_000_000, 1, 5_000_000, 777_777]
    files, blob = [], b""
    for i, n in enumerate(sizes):
        d = os.urandom(n)
        p = tmp_path / f"f{i}"
        p.write_bytes(d)
        files.append((str(p), n))
        blob += d
    hashes = ref(blob, piece)
    ok = gv.verify_files(files, piece, hashes)
    assert ok == b"\x01" * (len(hashes) // 20)
    b = bytearray(open(files[2][0], "rb").read())
    b[123456] ^= 1
    open(files[2][0], "wb").write(bytes(b))
    ok = gv.verify_files(files, piece, hashes)
    bad = (3_000_001 + 123456) // piece
    assert [i for i, v in enumerate(ok) if not v] == [bad]


@pytest.mark.parametrize("piece,sizes,chunk", [
    (1 << 20, [3_000_000, 1, 5_000_000, 777_777], 65536),   # short last piece, file spans
    (65536, [200_000, 333_333], 65536),                     # chunk == piece
    (262144, [1_048_576], 65536),                           # exact multiple, no tail
    (100_000, [950_001], 65536),                            # piece not a multiple of the chunk
    (1 << 20, [4_500_000], 4096),                           # many rounds per piece
])
def test_streamed_verify_matches_cpu(gv, tmp_path, piece, sizes, chunk):
    from downloader_amd.ops import hashing
    files, blob = [], b""
    for i, n in enumerate(sizes):
        d = os.urandom(n)
        p = tmp_path / f"s{i}"
        p.write_bytes(d)
        files.append((str(p), n))
        blob += d
    hashes = ref(blob, piece)
    ok, _ = gv.verify_files_streamed(files, piece, hashes, chunk)
    assert ok == b"\x01" * (len(hashes) // 20)
    assert hashing.verify_pieces(files, piece, hashes, backend="gpu") == ok
    # corrupt the last byte of the storage -> only the last piece fails
    last = files[-1][0]
    b = bytearray(open(last, "rb").read())
    b[-1] ^= 0x01
    open(last, "wb").write(bytes(b))
    ok, _ = gv.verify_files_streamed(files, piece, hashes, chunk)
    n = len(hashes) // 20
    assert [i for i, v in enumerate(ok) if not v] == [n - 1]


def test_streamed_window_smaller_than_piece_count(gv, tmp_path):
    """A tiny pinned slot forces several windows of lanes (W < pieces)."""
    from downloader_amd.ops import gpuhash
    g = gpuhash().GpuVerifier(0, 1 << 20, 4)   # 1 MiB slot / 64 KiB chunk -> 16 lanes/window
    d = os.urandom(70 * 65536 + 123)
    p = tmp_path / "w"
    p.write_bytes(d)
    hashes = ref(d, 65536)
    ok, _ = g.verify_files_streamed([(str(p), len(d))], 65536, hashes, 65536)
    assert ok == b"\x01" * 71


def test_gpu_matches_cpu_backend_and_reports_throughput(gv, tmp_path):
    from downloader_amd.ops import hashing
    piece = 1 << 20
    data = os.urandom(256 * piece)
    p = tmp_path / "big"
    p.write_bytes(data)
    hashes = hashing.hash_pieces(data, piece)
    t0 = time.perf_counter()
    g = hashing.verify_pieces([(str(p), len(data))], piece, hashes, backend="gpu")
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    c = hashing.verify_pieces([(str(p), len(data))], piece, hashes, backend="cpu")
    tc = time.perf_counter() - t0
    assert g == c == b"\x01" * 256
    print(f"verify 256 MiB: gpu {len(data) / tg / 1e9:.2f} GB/s, cpu {len(data) / tc / 1e9:.2f} GB/s")


def test_prewarm_makes_auto_pick_gpu(monkeypatch):
    """On a host without the AVX-512 multi-buffer SHA-1 a warm device takes auto rechecks."""
    from downloader_amd.ops import hashing
    assert hashing.prewarm_gpu() is True
    monkeypatch.setattr(hashing, "host_multibuffer", lambda: False)
    assert hashing.choose_backend("auto", hashing.GPU_MIN_BYTES, 1024) == "gpu"


def test_streamed_verify_subset_in_list_order(gv, tmp_path):
    """``which`` = piece list (unsorted, includes the short last piece, several windows)."""
    from downloader_amd.ops import gpuhash
    piece = 65536
    d = bytearray(os.urandom(90 * piece + 777))
    p = tmp_path / "sub"
    hashes = ref(bytes(d), piece)
    d[5 * piece + 9] ^= 0x40                       # piece 5 corrupt
    p.write_bytes(bytes(d))
    which = [90, 5, 0, 44, 89, 6, 17]
    g = gpuhash().GpuVerifier(0, 4 * piece, 4)     # 4 lanes per window -> 2 windows
    ok, _ = g.verify_files_streamed([(str(p), len(d))], piece, hashes, 65536, which=which)
    assert list(ok) == [1, 0, 1, 1, 1, 1, 1]
    with pytest.raises(ValueError):
        g.verify_files_streamed([(str(p), len(d))], piece, hashes, 65536, which=[91])


def test_gpu_batcher_coalesces_concurrent_runs(tmp_path):
    from concurrent.futures import wait
    from downloader_amd.ops import hashing
    piece = 1 << 20
    d = bytearray(os.urandom(64 * piece + 5))
    hashes = ref(bytes(d), piece)
    d[33 * piece] ^= 1
    p = tmp_path / "b"
    p.write_bytes(bytes(d))
    files = [(str(p), len(d))]
    b = hashing.GpuBatcher()
    runs = [list(range(i, min(i + 8, 65))) for i in range(0, 65, 8)]
    futs = [b.submit(files, piece, hashes, r) for r in runs]
    wait(futs, timeout=60)
    got = [v for f in futs for v in f.result()]
    assert got == [i != 33 for i in range(65)]
    assert b.batches < len(runs) and b.pieces == 65
    # subset through the front-end too
    assert hashing.verify_pieces(files, piece, hashes, which=[33, 64], backend="gpu") == b"\x00\x01"


def test_torrent_job_with_gpu_piece_verification(run):
    """Config-4 shape at 1/50 scale, disk staging (the stream path hashes in the relay):
    webseed torrent -> eager S3 staging, every downloaded run verified by the gfx950 kernel
    through the batcher."""
    import argparse
    from downloader_amd.bench import configs
    from downloader_amd.ops import hashing
    a = argparse.Namespace(mode="tuned", scale=0.02, piece_mb=1, verify_backend="gpu",
                           webseed_streams=4, webseed_chunk_mb=8, webseed_verify_depth=4,
                           src_dir=None, stage_dir="", torrent_stream="off", stream_parallel=0)
    before = hashing.gpu_batcher().pieces
    r = run(configs.config_torrent(a, 4), timeout=300)
    assert r["uploaded_bytes"] == r["bytes"] and r["s3_bytes_received"] >= r["bytes"]
    assert r["torrent"]["hash_fails"] == 0 and r["torrent"]["staging"] == "disk"
    assert hashing.gpu_batcher().pieces - before >= r["bytes"] // (1 << 20)


# ---------------------------------------------------------------- relayed-part hashing
@pytest.fixture(scope="module")
def part_hasher():
    from downloader_amd.ops import gpu_available, gpuhash
    if not gpu_available():
        pytest.fail("HIP device not visible: the GPU test tier must run on a MI355X")
    return gpuhash().PartHasher(0, 64 << 20, 4, 4, 4096)


@pytest.mark.parametrize("piece,n", [
    (16384, 16 * 16384),            # aligned, whole pieces
    (262144, 9 * 262144 + 77),      # short last piece
    (1000, 40 * 1000 + 3),          # piece_len % 16 != 0 -> byte path
    (65536, 65536 * 300),           # several hundred lanes in one launch
])
def test_part_hasher_matches_hashlib(part_hasher, piece, n):
    data = os.urandom(n)
    assert part_hasher.hash(data, piece) == ref(data, piece)


def test_split_kernel_matches_lanes_kernel_and_is_faster(gv):
    """sha1_lanes_split (two schedule waves + a rounds wave per 64 pieces) vs sha1_lanes<16> on
    one lane table whose lanes end at different blocks and with every tail shape: identical
    digests, and a 4 MiB piece's latency cut (~618 -> ~410 VALU ops per block on its chain:
    73 -> 53 ms measured, profiles/r6/split/)."""
    ms_s, ms_l, same = gv.kernel_bench_split(65536 + 48, 200, 1)
    assert same, (ms_s, ms_l)
    ms_s, ms_l, same = gv.kernel_bench_split(4 << 20, 128, 2)
    assert same and ms_l / ms_s > 1.25, (ms_s, ms_l)
    with pytest.raises(ValueError):
        gv.kernel_bench_split(1000, 16, 1)


def test_split_kernel_small_launches(gv):
    """A launch of one part (16 lanes of a 64-lane workgroup), with its idle lanes hashing live
    lanes' pieces again (the default) or left idle: right digests either way, and the default
    no slower (left idle it took 72 - 96 ms per 4 MiB piece on one box, 57 on another, against
    57 with every lane busy; profiles/r6/split/small_launch_dup.jsonl)."""
    dup, _, same = gv.kernel_bench_split(4 << 20, 16, 2, True)
    idle, _, same2 = gv.kernel_bench_split(4 << 20, 16, 2, False)
    assert same and same2
    assert dup < idle * 1.1, (dup, idle)


@pytest.mark.parametrize("kernel", ["sha1_lanes_split", "sha1_lanes"])
def test_part_hasher_kernels_match_hashlib(monkeypatch, kernel):
    from downloader_amd.ops import gpuhash
    monkeypatch.setenv("STAGER_SHA1_KERNEL", "lanes" if kernel == "sha1_lanes" else "split")
    h = gpuhash().PartHasher(0, 16 << 20, 2, 1, 256)
    assert h.stats()["kernel"] == kernel
    for piece, n in [(16384, 40 * 16384 + 60), (65536, 65536 * 7 + 55), (262144, 262144 * 3)]:
        data = os.urandom(n)
        assert h.hash(data, piece) == ref(data, piece), (kernel, piece, n)


def test_part_hasher_batches_concurrent_parts(part_hasher):
    """Parts submitted from many threads at once share launches (the batching that gives
    one-lane-per-piece hashing its throughput), and each gets its own digests back."""
    from concurrent.futures import ThreadPoolExecutor
    parts = [os.urandom(16 * 65536 + (i % 3) * 65536) for i in range(48)]
    before = part_hasher.stats()
    with ThreadPoolExecutor(48) as ex:
        got = list(ex.map(lambda d: part_hasher.hash(d, 65536), parts))
    assert got == [ref(d, 65536) for d in parts]
    st = part_hasher.stats()
    launches = st["launches"] - before["launches"]
    assert 1 <= launches < 48 and st["max_batch_lanes"] > 18 and not st["broken"], st


def _disp_threads():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                if f.read().strip() == "gpu-part-disp":
                    with open(f"/proc/self/task/{tid}/stat") as g:
                        st = g.read().rsplit(")", 1)[1].split()
                    out[tid] = (int(st[11]) + int(st[12])) / os.sysconf("SC_CLK_TCK")
        except OSError:
            pass
    return out


def test_part_hasher_dispatcher_idles_while_every_slot_is_busy():
    """with every device slot busy, queued parts used to keep the dispatcher thread
    spinning on its lock and hipEventQuery. 2 slots of one 4 MiB piece each, one stream, 16
    parts from 16 threads: ~1 s of kernels with parts waiting for a slot most of the time -
    the dispatcher must sleep between polls (its CPU well under the wall time)."""
    import time
    from concurrent.futures import ThreadPoolExecutor

    from downloader_amd.ops import gpuhash
    before = set(_disp_threads())
    h = gpuhash().PartHasher(0, 4 << 20, 2, 1, 64)
    tid = next(t for t in _disp_threads() if t not in before)
    parts = [os.urandom(4 << 20) for _ in range(16)]
    cpu0, t0 = _disp_threads()[tid], time.perf_counter()
    with ThreadPoolExecutor(16) as ex:
        got = list(ex.map(lambda d: h.hash(d, 4 << 20), parts))
    wall = time.perf_counter() - t0
    cpu = _disp_threads()[tid] - cpu0
    assert got == [ref(d, 4 << 20) for d in parts]
    st = h.stats()
    assert st["launches"] >= 8 and not st["broken"], st
    assert wall > 0.3 and cpu < 0.35 * wall, (cpu, wall)
    del h


def test_part_hasher_failed_setup_frees_what_it_allocated():
    """A PartHasher whose slots do not fit in HBM fails to construct - and hands back the
    slots, streams and events it had already made (no HBM leaked for the process's life
    while the relay carries on hashing on the host)."""
    from downloader_amd.ops import gpuhash
    free0, total = gpuhash().mem_info(0)
    slot = 32 << 30
    with pytest.raises(Exception):
        gpuhash().PartHasher(0, slot, int(total // slot) + 2, 1, 64)
    free1, _ = gpuhash().mem_info(0)
    assert free1 > free0 - (1 << 30), (free0, free1)


def test_part_hasher_small_parts_through_the_relay(run, origin_cls):
    """Many small parts (64 pieces of 4 KiB: kernels of well under a millisecond) through the
    relay's asynchronous path. A kernel can then finish between the dispatcher's poll of its
    copies and its poll of the kernels, so a part's DONE may be the first news of its copy:
    every part still completes with the right digests, every buffer returns to the pool, and
    the hasher neither hangs nor breaks."""
    import asyncio

    from downloader_amd.ops import gpu_available, gpuhash, hashing, native
    from downloader_amd.s3.client import S3Client
    from downloader_amd.s3.fake_server import FakeS3
    from downloader_amd.utils.aio import gather_strict

    if not gpu_available():
        pytest.fail("HIP device not visible: the GPU test tier must run on a MI355X")
    piece, size = 4096, 256 << 10

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blobs = [os.urandom(size) for _ in range(8)]
        for i, b in enumerate(blobs):
            origin.blobs[f"/p{i}.bin"] = b
        c = S3Client(ep, "minioadmin", "minioadmin")
        await c.ensure_bucket("b")

        async def one(k):
            b = k % len(blobs)
            _, h = await c.relay_hashed("b", f"k{k}", origin.url(f"/p{b}.bin"), 0, size, True,
                                        (0, size, piece), gpu=True)
            assert h["gpu_ticket"] and not h["digests"]
            return b, await asyncio.wait_for(hashing.gpu_part_digests(h["gpu_ticket"]), 30)

        got = []
        for r in range(12):
            got += await gather_strict(*(one(r * 16 + i) for i in range(16)))
        want = [b"".join(hashlib.sha1(x[i:i + piece]).digest() for i in range(0, size, piece))
                for x in blobs]
        assert all(d == want[b] for b, d in got)
        st = ph.stats()
        assert st["submitted"] >= 192 and not st["broken"] and st["pending"] == 0, st
        assert native().relay_pool_stats()["in_use"] == 0
        await c.close(); await origin.stop(); await s3.stop()

    prev = hashing._part_hasher
    ph = gpuhash().PartHasher(0, 64 << 20, 4, 0, 4096, 2)
    hashing.use_part_hasher(ph, 4)
    try:
        run(go(), timeout=120)
    finally:
        hashing.use_part_hasher(prev)


@pytest.mark.parametrize("corrupt", [False, True])
def test_stream_torrent_with_gpu_relay_hashing(run, tmp_path, make_cfg, origin_cls, corrupt):
    """Webseed torrent staged webseed -> S3 with the relayed parts' pieces hashed by the
    PartHasher (stream_verify_backend: gpu): byte-exact objects, parts really went to the
    device, and a corrupt byte inside a part's pieces is caught by the GPU digest and the
    part refetched."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.ops import hashing, native
    from downloader_amd.s3.fake_server import FakeS3
    from downloader_amd.service.worker import Worker
    from downloader_amd.torrent.metainfo import make_torrent

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
        cfg = make_cfg(ep, download={"torrent_enable_dht": False, "stream_verify_backend": "gpu",
                                     "stream_gpu_min_pieces": 4, "stream_gpu_tail": 0})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        before = native().gpu_part_stats()["submitted"]
        await w.submit(api.make_download("gs", "http", origin.url("/t/m.torrent")))
        for _ in range(3000):
            if w.results:
                break
            await asyncio.sleep(0.02)
        r = w.results[0]
        assert r.outcome == "staged", r
        t = r.stats["torrent"]
        assert t["staging"] == "stream" and t.get("verify") == "gpu", t.get("verify_fallback")
        assert s3.get("triton-staging", keys.object_key("gs", "m.mkv")) == data
        assert native().gpu_part_stats()["submitted"] - before >= 4
        assert (t["hash_fails"] >= 1) == corrupt
        st = hashing.gpu_relay_stats()
        assert st["host_fallbacks"] == 0 and not st["device_broken"]
        await w.stop(); await origin.stop(); await s3.stop()
    run(go(), timeout=120)


def test_stream_torrent_auto_sets_the_device_up_lazily(run, tmp_path, make_cfg, origin_cls):
    """The default ``stream_verify_backend: auto`` on a HIP box: the first job with parts
    beyond the host-hashed tail starts the PartHasher on an executor thread (its first parts
    hash on the host meanwhile); the next such job sends its parts to the gfx950 kernel, and
    the objects are byte-exact."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.ops import hashing
    from downloader_amd.s3.fake_server import FakeS3
    from downloader_amd.service.worker import Worker
    from downloader_amd.torrent.metainfo import make_torrent

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        src = tmp_path / "src" / "Movie"
        src.mkdir(parents=True)
        data = os.urandom(40 * (1 << 20) + 999)
        (src / "m.mkv").write_bytes(data)
        origin.blobs["/ws/Movie/m.mkv"] = data
        origin.blobs["/t/m.torrent"] = make_torrent(str(src), 1 << 18,
                                                    url_list=[origin.url("/ws/")])
        cfg = make_cfg(ep, s3={"part_size": 5 << 20},
                       download={"torrent_enable_dht": False, "stream_gpu_min_pieces": 4,
                                 "stream_gpu_tail": 2, "torrent_stream_parallel": 2})
        assert cfg.download.stream_verify_backend == "auto"
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)

        async def job(jid: str):
            n = len(w.results)
            await w.submit(api.make_download(jid, "http", origin.url("/t/m.torrent")))
            for _ in range(3000):
                if len(w.results) > n:
                    break
                await asyncio.sleep(0.02)
            r = w.results[-1]
            assert r.outcome == "staged", r
            assert s3.get("triton-staging", keys.object_key(jid, "m.mkv")) == data
            return r.stats["torrent"]
        await job("ga1")                           # starts the set-up (HIP init)
        for _ in range(1500):
            if hashing._part_hasher is not None:
                break
            await asyncio.sleep(0.02)
        assert hashing._part_hasher is not None
        t = await job("ga2")
        assert t["verify"] == "auto" and t["gpu_parts"] >= 1, t
        await w.stop(); await origin.stop(); await s3.stop()
    run(go(), timeout=120)


def test_two_stream_torrents_inside_the_part_budget_on_the_device(run, tmp_path, make_cfg,
                                                                  origin_cls):
    """The gfx950 PartHasher under a part-buffer budget: two streamed torrents at once, 16
    relays in flight each, 24 MiB budget. A part's bytes return to the budget when the
    hasher notifies its DMA's end (eventfd, no waiting thread), so the pool's high-water mark
    stays inside the budget while both jobs' parts are hashed on the device."""
    import asyncio

    from downloader_amd.broker.memory import MemoryBroker
    from downloader_amd.models import api, keys
    from downloader_amd.ops import hashing, native
    from downloader_amd.s3.fake_server import FakeS3
    from downloader_amd.service.worker import Worker
    from downloader_amd.torrent.metainfo import make_torrent

    async def go():
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        blobs = {}
        for j in range(2):
            src = tmp_path / f"src{j}" / "Movie"
            src.mkdir(parents=True)
            data = os.urandom(40 * (1 << 20) + 777 * j)
            (src / "m.mkv").write_bytes(data)
            origin.blobs[f"/ws{j}/Movie/m.mkv"] = data
            origin.blobs[f"/t/m{j}.torrent"] = make_torrent(str(src), 1 << 18,
                                                           url_list=[origin.url(f"/ws{j}/")])
            blobs[j] = data
        native().relay_pool_trim()
        native().relay_pool_reset_peak()
        cfg = make_cfg(ep, concurrency=2, s3={"part_size": 5 << 20},
                       download={"torrent_enable_dht": False, "stream_verify_backend": "gpu",
                                 "stream_gpu_min_pieces": 4, "stream_gpu_tail": 0,
                                 "torrent_stream_parallel": 16, "relay_memory_mb": 24,
                                 "relay_pool_idle_trim_s": 0})
        w = Worker(cfg, broker=MemoryBroker())
        await w.start(health=False)
        for j in range(2):
            await w.submit(api.make_download(f"gb{j}", "http", origin.url(f"/t/m{j}.torrent")))
        for _ in range(3000):
            if len(w.results) >= 2:
                break
            await asyncio.sleep(0.02)
        assert len(w.results) == 2
        for r in w.results:
            assert r.outcome == "staged", r
            assert r.stats["torrent"]["verify"] == "gpu"
        for j in range(2):
            assert s3.get("triton-staging", keys.object_key(f"gb{j}", "m.mkv")) == blobs[j]
        assert sum(r.stats["torrent"]["gpu_parts"] for r in w.results) >= 8
        st = native().relay_pool_stats()
        assert 0 < st["peak_bytes"] <= 24 << 20 and st["over_budget"] == 0, st
        assert st["in_use"] == 0
        gs = hashing.gpu_relay_stats()
        assert gs["host_fallbacks"] == 0 and not gs["device_broken"] and gs["pending"] == 0
        await w.stop(); await origin.stop(); await s3.stop()
        native().relay_pool_set_budget(0)
    run(go(), timeout=120)


def test_swarm_pieces_verified_on_the_gfx950_part_hasher(run, tmp_path):
    """Native peer wire with swarm_verify_backend=gpu on the real device: a swarm download's
    complete pieces go from page-locked pooled buffers to the gfx950 PartHasher, their
    digests are compared natively, a corrupt piece from one seeder is caught by the device's
    digest and fetched again, and every piece lands on disk."""
    import asyncio

    from downloader_amd.ops import gpu_available, gpuhash, hashing
    from downloader_amd.torrent.client import TorrentClient
    from downloader_amd.torrent.metainfo import make_torrent, parse_torrent

    if not gpu_available():
        pytest.fail("HIP device not visible: the GPU test tier must run on a MI355X")
    piece = 1 << 20
    data = os.urandom(24 * piece + 4321)

    async def go():
        src = tmp_path / "seed" / "Pack"
        src.mkdir(parents=True)
        (src / "m.mkv").write_bytes(data)
        raw = make_torrent(str(src), piece)
        meta = parse_torrent(raw)
        bad = await TorrentClient().start()
        await bad.add_torrent(meta, str(tmp_path / "seed"))
        b = bytearray(data)
        b[5 * piece + 17] ^= 0x01                       # piece 5 served corrupt by `bad`
        (src / "m.mkv").write_bytes(bytes(b))
        good_dir = tmp_path / "good" / "Pack"
        good_dir.mkdir(parents=True)
        (good_dir / "m.mkv").write_bytes(data)
        good = await TorrentClient().start()
        await good.add_torrent(meta, str(tmp_path / "good"))
        leech = await TorrentClient(swarm_verify="gpu", pipeline=64,
                                    swarm_gpu_tail_bytes=0).start()
        s = await leech.add_torrent(meta, str(tmp_path / "dl"),
                                    peers=[("127.0.0.1", bad.listen_port)])
        await asyncio.sleep(0.5)
        s.add_peers([("127.0.0.1", good.listen_port)])
        await asyncio.wait_for(s.wait(), 60)
        assert (tmp_path / "dl" / "Pack" / "m.mkv").read_bytes() == data
        st = s.wire.stats()
        assert s.stats["swarm_verify"] == "gpu"
        assert st["gpu_pieces"] >= meta.num_pieces and st["gpu_errors"] == 0, st
        assert st["verified"] == meta.num_pieces and st["hash_fails"] >= 1, st
        await leech.close(); await bad.close(); await good.close()

    prev = hashing._part_hasher
    ph = gpuhash().PartHasher(0, 64 << 20, 4, 0, 4096, 2)
    hashing.use_part_hasher(ph, 4)
    try:
        run(go(), timeout=120)
        assert not ph.stats()["broken"]
    finally:
        hashing.use_part_hasher(prev)
