"""BASELINE config benches on the CPU: the torrent configs (3/4) through the native blobd
peer at a tiny scale, including ``--reps`` (same torrent staged again under fresh media ids,
median reported)."""
import argparse

from downloader_amd.bench import configs


def _ns(**over):
    a = argparse.Namespace(mode="tuned", scale=0.002, piece_mb=1, verify_backend="cpu",
                           webseed_streams=0, webseed_chunk_mb=0, webseed_verify_depth=0,
                           src_dir=None, stage_dir="", torrent_stream="auto", stream_parallel=0)
    vars(a).update(over)
    return a


def test_config3_reps_report_median(run):
    r = run(configs.config_torrent(_ns(reps=3), 3), timeout=120)
    assert r["reps"] == 3 and len(r["MBps_reps"]) == 3
    assert sorted(r["MBps_reps"])[1] == r["MBps"]
    assert r["uploaded_bytes"] == r["bytes"]
    assert r["s3_bytes_received"] >= 3 * r["bytes"]      # every rep re-staged the object
    assert r["torrent"]["hash_fails"] == 0


def test_config4_single_rep_default(run):
    """Namespace callers without ``reps`` (e.g. older scripts) still get one job."""
    r = run(configs.config_torrent(_ns(), 4), timeout=120)
    assert r["reps"] == 1 and r["files"] == 50
    assert r["uploaded_bytes"] == r["bytes"]


def test_config9_control_plane_ceiling(run):
    """Config 9: tiny jobs through one worker; every job is staged and the per-job CPU cost
    is reported."""
    r = run(configs.config_small(_ns(jobs=150, concurrency=16, small_kb=1)), timeout=120)
    assert r["staged"] == r["jobs"] == 150
    assert r["jobs_per_s"] > 0 and r["worker_cpu_ms_per_job"] > 0
    assert r["p99_latency_s"] >= r["p50_latency_s"]


def test_config6_swarm_leech_and_whole_magnet_job(run):
    """Config 6 at a tiny scale, seeders in-process: the bare leech on the native wire (every
    piece assigned to and requested by the wire), then the whole magnet job through a worker
    (--swarm-job), whose S3 sink receives every byte of every rep."""
    base = dict(scale=0.01, piece_mb=1, seeders=2, seed_inproc=True, seeder_procs=0,
                pipeline=16, reps=2, wire="native", swarm_verify="cpu", wire_requests="native",
                swarm_gpu_inflight=0, swarm_pool_mb=0)
    r = run(configs.config_swarm(_ns(**base)), timeout=120)
    assert r["reps"] == 2 and r["hash_fails"] == 0 and r["wire"] == "native"
    assert r["wire_stats"]["verified"] == r["bytes"] // (1 << 20) + 1
    assert r["wire_stats"]["assigned"] > 0
    j = run(configs.config_swarm(_ns(swarm_job=True, **base)), timeout=120)
    assert j["config"] == "swarm-job" and j["reps"] == 2
    assert j["s3_bytes_received"] >= j["bytes"]
