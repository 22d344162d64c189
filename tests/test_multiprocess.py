"""Multi-process: the supervisor runs N worker processes (CLI entrypoint) against the bundled
AMQP broker; jobs are spread across workers; SIGTERM drains them cleanly. Plus the bench
contract on 2 ranks over gloo (torch.distributed.run)."""
from __future__ import annotations

import asyncio
import json
import os
import shutil
import ssl
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.parametrize("tls", [False, True], ids=["amqp", "amqps"])
def test_supervisor_two_workers_over_amqp(run, tmp_path, origin_cls, tls):
    if tls and shutil.which("openssl") is None:
        pytest.skip("needs the openssl CLI")

    async def go():
        from downloader_amd.broker.amqp import AmqpBroker, client_ssl_context
        from downloader_amd.broker.server import BrokerServer
        from downloader_amd.models import api, keys
        from downloader_amd.parallel.supervisor import Supervisor, worker_argv
        from downloader_amd.s3.fake_server import FakeS3
        sctx, cctx, extra = None, None, {}
        if tls:     # amqps://: private CA handed to the workers through the config env
            key, crt = str(tmp_path / "k.pem"), str(tmp_path / "c.pem")
            subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes",
                            "-keyout", key, "-out", crt, "-days", "1", "-subj", "/CN=127.0.0.1",
                            "-addext", "subjectAltName=IP:127.0.0.1"], check=True,
                           capture_output=True)
            sctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            sctx.load_cert_chain(crt, key)
            cctx = client_ssl_context(True, crt)
            extra = {"STAGER_BROKER__CA_FILE": crt}
        srv = await BrokerServer(ssl_context=sctx).start()
        s3 = FakeS3()
        ep = await s3.start()
        origin = await origin_cls().start()
        env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error",
                   STAGER_BROKER__URL=srv.url, STAGER_BROKER__BACKEND="amqp",
                   STAGER_S3__ENDPOINT=ep, STAGER_INSTANCE__DOWNLOAD_PATH=str(tmp_path / "dl"),
                   STAGER_HEALTH__ENABLED="false", STAGER_DOWNLOAD__TORRENT_ENABLE_DHT="false",
                   STAGER_CONCURRENCY="1", **extra)
        sup = Supervisor(2, worker_argv(), env=env)
        sup.start()
        client = AmqpBroker(srv.url, ssl_context=cctx)
        await client.connect()
        await client.declare("v1.download")   # unroutable publishes are dropped, like RabbitMQ
        # both worker processes subscribed before the jobs go out (a loaded CI box may start
        # the second interpreter after the first has drained all 8 jobs)
        for _ in range(3000):
            q = srv.queues.get("v1.download")
            if q is not None and len(q.consumers) == 2:
                break
            await asyncio.sleep(0.02)
        n = 8
        for i in range(n):
            origin.blobs[f"/m{i}.mkv"] = os.urandom(30_000 + i)
            await client.publish("v1.download", api.encode(
                api.make_download(f"mp{i}", "http", origin.url(f"/m{i}.mkv"))))
        got = []
        for _ in range(1500):
            d = await client.get("v1.convert")
            if d is not None:
                got.append(api.decode(api.Convert, d.body).media.id)
                await d.ack()
                if len(got) == n:
                    break
            else:
                await asyncio.sleep(0.02)
        assert sorted(got) == sorted(f"mp{i}" for i in range(n))
        for i in range(n):
            assert s3.get("triton-staging", keys.object_key(f"mp{i}", f"m{i}.mkv")) == \
                origin.blobs[f"/m{i}.mkv"]
        # both workers consumed (prefetch=1 round-robin)
        assert len(srv.queues["v1.download"].consumers) == 2
        codes = await asyncio.get_running_loop().run_in_executor(None, sup.stop)
        assert codes == [0, 0]
        await client.close(); await srv.stop(); await s3.stop(); await origin.stop()
    run(go(), timeout=120)


@pytest.mark.slow
def test_bench_contract_two_ranks_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--size-mb", "4", "--jobs-per-step", "2",
           "--torrent-gb", "0.05", "--torrent-pairs", "1", "--ref-jobs", "16",
           "--curve-steps", "1"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout   # ONE line, nothing else
    j = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in j
    assert j["n_gpus"] == 2 and j["steps"] == 2 and j["value"] > 0
    assert j["config"]["jobs_timed"] == 2 * 2 * 2   # ranks x steps x jobs-per-step
    # the default extras ran on both ranks (the driver launches N>1 with the defaults)
    assert j["reference_mode_MBps"] > 0 and j["vs_baseline"] > 0 and len(j["workers_curve"]) == 4
    assert j["integrity"] == "crc32c" and j["crc_parts"] == j["media_parts"] == 2 * 2 * 2
    # the torrent A/B ran on both ranks at once: rates and device counters are summed
    assert j["torrent_ranks"] == 2 and j["torrent_gpu_MBps"] > 0 and j["torrent_host_MBps"] > 0


def test_bench_single_rank_defaults_are_valid(tmp_path):
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2",
                        "--warmup", "1", "--size-mb", "2", "--torrent-gb", "0.2",
                        "--torrent-pairs", "1", "--curve-steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["n_gpus"] == 1 and j["higher_is_better"] is True and j["scaling"] == "weak"
    # the headline's bytes are checked: every timed media PUT carried a CRC32C (2 MB objects:
    # one PUT per job, 2 steps x 64 jobs), the sink recomputed a salted 1-in-8 subset of them
    # and refused none
    assert j["integrity"] == "crc32c" and j["checksum"] == "always"
    assert j["crc_parts"] == j["media_parts"] == 2 * 64 and j["bad_digests"] == 0
    assert 0 < j["crc_checked_parts"] < j["crc_parts"] and j["sink_crc_check"] == "1/8"
    # same call: the unchecked spliced relay, labelled as such
    assert j["unchecked_MBps"] > 0 and j["unchecked_integrity"] == "none"
    # same call: reference-equivalent mode (8 serial prefetch-1 consumers, SHA-256-signed
    # payloads) on the same CPUs, and vs_baseline is the headline over it
    assert j["reference_mode_MBps"] > 0 and j["reference_mode_procs"] == 8
    assert j["reference_mode_integrity"] == "sha256"
    assert j["vs_baseline"] == round(j["value"] / j["reference_mode_MBps"], 3)
    # the BASELINE metric's curve: MB/s and p50 at 1/2/4/8 worker processes
    assert [c["procs"] for c in j["workers_curve"]] == [1, 2, 4, 8]
    assert all(c["MBps"] > 0 and c["p50_s"] > 0 for c in j["workers_curve"])
    assert j["gpu_slots"] >= 1 and j["slot_budget_cpus"] >= 1
    # CPU counted over the timed window only: worker + peer CPU fits in elapsed x the
    # rank's CPUs (BENCH_r04 claimed 19.9 CPU-s per second on a 16-CPU slice)
    assert 0 < j["cpu_utilisation"] <= 1.05 and 0 < j["unchecked_cpu_utilisation"] <= 1.05
    assert j["worker_cpu_s_per_GB"] > 0 and j["peer_cpu_s_per_GB"] > 0
    # the same-call torrent A/B (config 4's shape in miniature; no GPU here: both backends
    # hash on the host, so the device counters stay 0 - on a GPU box gpu_parts > 0)
    assert j["torrent_files"] == 50 and j["torrent_gpu_MBps"] > 0 and j["torrent_host_MBps"] > 0
    assert j["torrent_gpu_hash_fails"] == 0 and j["torrent_host_hash_fails"] == 0
    assert j["gpu_host_fallbacks"] == 0


def test_supervisor_auto_pinning_quota_share():
    from downloader_amd.parallel.supervisor import auto_cpus_per_worker, cpu_slices
    mask = list(range(256))
    assert auto_cpus_per_worker(4, mask, 16.0) == 4
    assert auto_cpus_per_worker(1, mask, 16.0) == 16
    assert auto_cpus_per_worker(4, mask, float("inf")) == 0
    assert auto_cpus_per_worker(1, list(range(8)), 16.0) == 0     # share = whole mask
    assert cpu_slices(2, 3, list(range(8))) == [[0, 1, 2], [3, 4, 5]]
    assert cpu_slices(2, -1, list(range(8))) == [[], []]


@pytest.mark.slow
def test_bench_torrent_ab_failure_never_costs_the_headline(tmp_path):
    """The torrent A/B is an extra of the line: when it fails or overruns --torrent-timeout
    the line still prints, with the headline and the error."""
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1",
                        "--warmup", "0", "--size-mb", "2", "--no-compare-single-put",
                        "--no-compare-crc", "--no-compare-reference", "--workers-curve", "",
                        "--torrent-gb", "0.2", "--torrent-timeout", "0.001"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["value"] > 0 and "TimeoutError" in j["torrent_error"]
    assert j["torrent_ranks_failed"] == 1 and "torrent_gpu_MBps" not in j


def test_bench_four_ranks_disjoint_cpus_and_own_peers(tmp_path):
    """The driver's N=4 launch rehearsed on CPU: 4 ranks over gloo, each pinned to its own
    GPU-slot CPU slice (disjoint, same size) with its own blobd peer, one JSON line whose
    totals cover all four ranks."""
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error", STAGER_GPU_SLOTS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(REPO, "bench.py"),
           "--gpus", "4", "--steps", "2", "--warmup", "1", "--size-mb", "2", "--jobs-per-step", "2",
           "--no-compare-single-put", "--torrent-gb", "0", "--no-compare-reference",
           "--workers-curve", ""]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["n_gpus"] == 4 and j["config"]["jobs_timed"] == 4 * 2 * 2
    cpus = [set(c) for c in j["rank_cpus"]]
    if len(os.sched_getaffinity(0)) >= 4:
        assert all(cpus) and len({len(c) for c in cpus}) == 1
        assert sum(len(c) for c in cpus) == len(set().union(*cpus))      # pairwise disjoint
    peers = j["rank_peers"]
    assert len(peers) == 4 and all(peers) and len(set(peers)) == 4
    assert j["timed_sink_bytes"] >= 4 * 2 * 2 * 2_000_000 and j["sink_mismatches"] == 0


@pytest.mark.slow
def test_bench_eight_ranks_as_the_driver_launches_them(tmp_path):
    """The driver's N=8 scaling launch rehearsed on CPU (gloo, 8 ranks, STAGER_GPU_SLOTS=8)
    with the GPU boxes' unprivileged pipe budget (64 MiB for the uid): every rank pinned to
    its own equal CPU slice, 8 distinct blobd peers, splice pipes of the size the budget math
    predicts for 8 ranks x their worker processes with none created short, and every timed
    object checked by its rank's sink."""
    from downloader_amd.utils import limits
    budget = 64 << 20
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error", STAGER_GPU_SLOTS="8",
               STAGER_PIPE_BUDGET_BYTES=str(budget), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(REPO, "bench.py"),
           "--gpus", "8", "--steps", "2", "--warmup", "1", "--size-mb", "2", "--jobs-per-step", "2",
           "--no-compare-unchecked", "--no-compare-reference", "--workers-curve", "",
           "--torrent-gb", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout                        # rank 0 prints the one line
    j = json.loads(lines[0])
    assert j["n_gpus"] == 8 and j["config"]["jobs_timed"] == 8 * 2 * 2
    assert j["gpu_slots"] == 8 and j["integrity"] == "crc32c" and j["bad_digests"] == 0
    assert j["crc_parts"] == j["media_parts"] == 8 * 2 * 2
    cpus = [set(c) for c in j["rank_cpus"]]
    assert len(cpus) == 8
    if len(os.sched_getaffinity(0)) >= 8:
        assert all(cpus) and len({len(c) for c in cpus}) == 1
        assert sum(len(c) for c in cpus) == len(set().union(*cpus))      # pairwise disjoint
        assert j["cpus_per_rank"] == j["slot_budget_cpus"]
    peers = j["rank_peers"]
    assert len(peers) == 8 and all(peers) and len(set(peers)) == 8
    nproc = j["procs_per_rank"]
    conc, pipe = limits.relay_plan(4, 2, 8 * nproc, budget)
    assert j["pipe_budget_bytes"] == budget
    assert (j["concurrency_per_worker"], j["pipe_kb"]) == (conc, pipe >> 10)
    assert pipe >= limits.PIPE_GOOD
    assert j["pipes_short"]["workers"] == 0
    assert j["timed_sink_bytes"] >= 8 * 2 * 2 * 2_000_000 and j["sink_mismatches"] == 0
    assert j["sink_verified_objects"] >= 8 * 2 * 2


@pytest.mark.slow
def test_bench_rank_with_two_worker_processes(tmp_path):
    """--procs-per-rank 2: the rank spawns two worker processes, splits the timed jobs, and
    still prints exactly one JSON line whose byte count the S3 peer confirmed."""
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2",
                        "--warmup", "1", "--jobs-per-step", "3", "--size-mb", "4",
                        "--procs-per-rank", "2", "--torrent-gb", "0", "--compare-single-put",
                        "--no-compare-reference", "--workers-curve", ""],
                       env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    j = json.loads(lines[0])
    assert j["procs_per_rank"] == 2 and j["config"]["jobs_timed"] == 6
    assert j["timed_sink_bytes"] >= 6 * 4_000_000 and j["value"] > 0
    assert j["sink"] == "sample" and j["sink_mismatches"] == 0
    assert j["sink_verified_objects"] >= 6
    assert "single_put_MBps" in j


@pytest.mark.slow
@pytest.mark.parametrize("sink", ["sample", "verify"])
def test_bench_multipart_objects_checked_against_the_origin(tmp_path, sink):
    """The headline shape in miniature: objects above the threshold go as multipart uploads
    (here 12 MB in 5 MiB parts = 3 parts), and the S3 peer matches every timed object, part by
    part at its offset, against the bytes its origin generated (sampled windows / every byte);
    the sink counters are taken inside the timed bracket."""
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2",
                        "--warmup", "1", "--jobs-per-step", "2", "--size-mb", "12",
                        "--part-mb", "5", "--threshold-mb", "5", "--sink", sink,
                        "--no-compare-single-put", "--torrent-gb", "0",
                        "--no-compare-reference", "--workers-curve", ""],
                       env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    assert j["parts_per_object"] == 3.0
    assert j["sink_verified_objects"] == 4 and j["sink_mismatches"] == 0
    assert 4 * 12_000_000 <= j["timed_sink_bytes"] < 2 * 4 * 12_000_000   # no warmup bytes
    if sink == "verify":
        assert j["sink_verified_bytes"] == 4 * 12_000_000
    else:
        assert 0 < j["sink_verified_bytes"] < 4 * 12_000_000
    assert "single_put_MBps" not in j


@pytest.mark.slow
def test_bench_reference_mode_worker_count():
    """Reference mode defaults to one serial consumer per rank; an explicit --procs-per-rank N
    runs N of them (N reference containers, the worker sweep's reference column)."""
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    base = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1", "--warmup", "0",
            "--jobs-per-step", "2", "--size-mb", "2", "--mode", "reference"]
    for extra, want in (([], 1), (["--procs-per-rank", "2"], 2)):
        r = subprocess.run(base + extra, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        j = json.loads(r.stdout.strip().splitlines()[-1])
        assert j["mode"] == "reference" and j["procs_per_rank"] == want
        assert j["config"]["jobs_timed"] == 2        # jobs per step are per rank, split over procs


def test_supervisor_restarts_crashed_workers_without_blocking():
    """A worker that keeps crashing is respawned with exponential backoff up to max_restarts
    and then left down, each exit is recorded once, and a healthy sibling is untouched;
    poll() never sleeps (the old loop slept through the backoff)."""
    import time as _t

    from downloader_amd.parallel.supervisor import Supervisor
    code = ("import os, sys, time\n"
            "if os.environ['STAGER_WORKER_INDEX'] == '1': time.sleep(30)\n"
            "sys.exit(3)\n")
    sup = Supervisor(2, [sys.executable, "-c", code], cpus_per_worker=-1, max_restarts=2,
                     backoff=0.05)
    sup.start()
    t0 = _t.monotonic()
    while not sup.slots[0].done and _t.monotonic() - t0 < 20:
        t1 = _t.monotonic()
        sup.poll()
        assert _t.monotonic() - t1 < 0.5
        _t.sleep(0.02)
    s0, s1 = sup.slots
    assert s0.done and s0.restarts == 2 and s0.exit_codes == [3, 3, 3]
    assert s1.proc is not None and s1.proc.poll() is None and not s1.exit_codes
    assert sup.stop(timeout=10) != []


def test_chaos_soak_loses_no_job(tmp_path):
    """Config 7 in miniature: supervised workers over the bundled AMQP broker while workers are
    SIGKILLed and every AMQP connection is dropped; every job still reaches v1.convert and
    nothing is left in the staging directory."""
    env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="critical")
    r = subprocess.run([sys.executable, "-m", "downloader_amd.bench.configs", "--config", "7",
                        "--scale", "0.1", "--workers", "2", "--concurrency", "2", "--qps", "20",
                        "--chaos-interval", "0.7", "--chaos-timeout", "120", "--cpus", "-1",
                        "--src-dir", str(tmp_path), "--stage-dir", str(tmp_path)],
                       capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["config"] == 7 and out["jobs"] == 60 and not out["timed_out"]
    assert out["lost_jobs"] == 0, out
    assert out["kills"] >= 1 and out["connection_drops"] >= 1
    assert out["stage_leftover_bytes"] == 0
