"""A heterogeneous swarm on the CPU (bench/swarm_hetero.py, csrc/swarmd.cpp):
>= 32 fake seeders with per-peer token-bucket rates (0.2 - 50 MB/s), 20 - 200 ms answer
delays, 10 % stalling mid-piece and 10 % hanging up. The download must complete with the right
bytes, no piece may stay owned by (or requested from) a peer that has stopped sending for
longer than the stall rule allows, and the native wire's threads stay bounded whatever the
number of peers (it used to run two per connection)."""
from __future__ import annotations

import pytest

from downloader_amd.bench.swarm_hetero import hetero_specs, run_hetero


def test_hetero_specs_shape():
    sp = hetero_specs(48, seed=3)
    assert len(sp) == 48
    assert sum(s["kind"] == "stall" for s in sp) == 5 and sum(s["kind"] == "hangup" for s in sp) == 5
    assert all(0.2e6 * 0.999 <= s["rate"] <= 50e6 * 1.001 for s in sp)
    assert all(20 <= s["delay_ms"] <= 200 for s in sp)
    # stalls / hang-ups land inside a piece, not on its boundary
    assert all(s["stall"] % (4 << 20) for s in sp if s["kind"] == "stall")


@pytest.mark.slow
@pytest.mark.parametrize("wire", ["native", "python"])
def test_hetero_swarm_completes_without_stuck_pieces(run, tmp_path, wire):
    r = run(run_hetero(total=96 << 20, piece_len=1 << 20, peers=36, wire=wire, seed=5,
                       src_dir=str(tmp_path), timeout=120), timeout=180)
    assert r["data_ok"] and r["hash_fails"] == 0
    assert r["stalling"] >= 3 and r["hanging_up"] >= 3
    # a peer that stopped sending gave its owned pieces / requested blocks back within the
    # stall rule (SLOW_TICKS x RATE_S = 0.5 s) plus a sampling period of slack
    assert r["max_owned_idle_s"] <= 1.5, r
    assert r["slow_peers"] >= r["stalling"]
    if wire == "native":
        # 4 epoll I/O threads, verifiers, digest collectors and the writer: not 2 per peer
        assert r["wire_io_threads"] == 4
        assert r["threads_peak"] - r["threads_before"] <= 24, r
    assert r["MBps"] > 0


@pytest.mark.slow
def test_fast_seeders_pipeline_growth_never_idles_a_connection(run, tmp_path):
    """Config 6's shape on swarmd: 4 unthrottled seeders, the rate loop growing every
    connection's pipeline mid-download. A deeper pipeline drains the connection's queue of
    blocks to request below it; that NEED must reach Python (it was dropped once, leaving all
    four connections idle at 160 MiB of 256)."""
    specs = [{"rate": 0, "delay_ms": 0, "stall": 0, "hangup": 0, "kind": "ok"} for _ in range(4)]
    r = run(run_hetero(total=256 << 20, piece_len=4 << 20, peers=4, specs=specs, pipeline=64,
                       src_dir=str(tmp_path), timeout=60), timeout=120)
    assert r["data_ok"] and r["hash_fails"] == 0 and r["slow_peers"] == 0
    assert r["max_depth"] > 8 * 64                     # the pipelines did grow
