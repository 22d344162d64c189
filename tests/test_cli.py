"""Command-line entrypoint (reference index.js + operational tools)."""
from __future__ import annotations

import asyncio
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(*args, env=None, timeout=120):
    e = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error")
    e.update(env or {})
    return subprocess.run([sys.executable, "-m", "downloader_amd", *args], capture_output=True,
                          text=True, timeout=timeout, env=e, cwd=REPO)


def test_make_torrent_and_verify_roundtrip(tmp_path):
    src = tmp_path / "Show"
    (src / "S1").mkdir(parents=True)
    (src / "S1" / "a.mkv").write_bytes(os.urandom(300_000))
    (src / "b.mkv").write_bytes(os.urandom(5))
    out = tmp_path / "show.torrent"
    r = _cli("make-torrent", str(src), "-o", str(out), "--piece-length", "16384",
             "--webseed", "http://ws/", "--tracker", "udp://t:1")
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout)
    assert info["bytes"] == 300_005 and info["pieces"] == (300_005 + 16383) // 16384
    r = _cli("verify", str(out), str(tmp_path), "--backend", "cpu")
    assert r.returncode == 0, r.stderr
    v = json.loads(r.stdout)
    assert v["good"] == v["pieces"] and v["backend"] == "cpu"
    with open(src / "S1" / "a.mkv", "r+b") as f:
        f.write(b"\x00\x01")
    r = _cli("verify", str(out), str(tmp_path), "--backend", "cpu")
    assert r.returncode == 1 and json.loads(r.stdout)["good"] == v["pieces"] - 1


def test_config_command_prints_effective_config():
    r = _cli("config", env={"STAGER_S3__BUCKET": "other", "PORT": "4123",
                            "STAGER_S3__SECRET_KEY": "hunter2",
                            "STAGER_BROKER__URL": "amqp://u:pw@mq:5672/"})
    assert r.returncode == 0, r.stderr
    c = json.loads(r.stdout)
    assert c["s3"]["bucket"] == "other" and c["health"]["port"] == 4123
    assert "hunter2" not in r.stdout and ":pw@" not in r.stdout     # masked by default
    assert c["broker"]["url"] == "amqp://u:***@mq:5672/"
    r = _cli("config", "--show-secrets", env={"STAGER_S3__SECRET_KEY": "hunter2"})
    assert json.loads(r.stdout)["s3"]["secret_key"] == "hunter2"


def test_submit_publishes_download(run):
    async def go():
        from downloader_amd.broker.amqp import AmqpBroker
        from downloader_amd.broker.server import BrokerServer
        from downloader_amd.models import api
        srv = await BrokerServer().start()
        c = AmqpBroker(srv.url)
        await c.connect()
        await c.declare("v1.download")
        r = await asyncio.get_running_loop().run_in_executor(None, lambda: _cli(
            "submit", "m42", "http", "http://o/x.mkv", "--type", "TV", "--creator", "card7",
            env={"STAGER_BROKER__URL": srv.url}))
        assert r.returncode == 0, r.stderr
        d = await c.get("v1.download")
        m = api.decode(api.Download, d.body)
        assert (m.media.id, m.media.creatorId, m.media.sourceURI) == ("m42", "card7", "http://o/x.mkv")
        assert m.media.type == api.string_to_enum("MediaType", "TV")
        await c.close()
        await srv.stop()
    run(go())


def test_worker_exits_zero_on_sigterm_when_idle(run, tmp_path):
    async def go():
        import signal
        from downloader_amd.broker.server import BrokerServer
        srv = await BrokerServer().start()
        env = dict(os.environ, PYTHONPATH=REPO, LOG_LEVEL="error", STAGER_BROKER__URL=srv.url,
                   STAGER_HEALTH__PORT="0", STAGER_INSTANCE__DOWNLOAD_PATH=str(tmp_path),
                   STAGER_DOWNLOAD__TORRENT_ENABLE_DHT="false")
        p = await asyncio.create_subprocess_exec(sys.executable, "-m", "downloader_amd", "worker",
                                                 env=env, cwd=REPO)
        for _ in range(200):
            q = srv.queues.get("v1.download")
            if q is not None and q.consumers:
                break
            await asyncio.sleep(0.05)
        p.send_signal(signal.SIGTERM)
        code = await asyncio.wait_for(p.wait(), 30)
        assert code == 0            # termHandler: exit(0) when no job is in flight
        await srv.stop()
    run(go(), timeout=60)


def test_bench_pin_rank_quota_share(monkeypatch):
    """bench.py pins each rank to its share of the CPU quota (contiguous, disjoint)."""
    import os
    import types

    import bench
    from downloader_amd.utils import cpus
    got = {}
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, s: got.setdefault("mask", list(s)))
    monkeypatch.delenv("STAGER_BENCH_NO_PIN", raising=False)
    monkeypatch.setattr(cpus, "cgroup_cpu_quota", lambda path="": 16.0)
    one = types.SimpleNamespace(world=1, rank=0)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    # the build pool's EPYC 9575F: CPU c and c+128 are SMT siblings, cores 0-63 on package 0
    monkeypatch.setattr(cpus, "_core_of", lambda c, root: (c % 128 // 64, c % 64))
    monkeypatch.setenv("STAGER_GPU_SLOTS", "1")                  # 1-GPU box
    assert bench.pin_rank(one) == list(range(16))
    assert bench.pin_rank(one, -1) == []
    # 8-GPU node, quota 128: 16 CPUs per GPU slot whatever the number of ranks
    monkeypatch.setenv("STAGER_GPU_SLOTS", "8")
    monkeypatch.setattr(cpus, "cgroup_cpu_quota", lambda path="": 128.0)
    assert bench.pin_rank(one) == list(range(16))               # N=1: slot 0, not the node
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    eight = types.SimpleNamespace(world=8, rank=3)
    assert bench.pin_rank(eight) == list(range(48, 64))
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert bench.pin_rank(eight) == list(range(80, 96))         # package 1
    # no quota: 32 CPUs per slot = 16 cores with both SMT threads, never shared across slots
    monkeypatch.setattr(cpus, "cgroup_cpu_quota", lambda path="": float("inf"))
    assert bench.pin_rank(eight) == list(range(80, 96)) + list(range(208, 224))
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setenv("STAGER_GPU_SLOTS", "1")
    assert bench.pin_rank(one) == []                            # no quota, one slot: leave it
    assert bench.pin_rank(one, 4) == [0, 1, 2, 3]               # K > 0: K contiguous per rank


def test_gpu_slots_from_env(monkeypatch):
    from downloader_amd.utils import cpus
    monkeypatch.delenv("STAGER_GPU_SLOTS", raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    assert cpus.gpu_slots() == 8
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "3")
    assert cpus.gpu_slots() == 1
    monkeypatch.setenv("STAGER_GPU_SLOTS", "4")
    assert cpus.gpu_slots() == 4


def test_config_reference_doc_is_current():
    """docs/CONFIG.md is the generated reference of every key (config --reference)."""
    from downloader_amd.utils.config import Config
    from downloader_amd.utils.config_doc import reference_markdown
    md = reference_markdown()
    with open(os.path.join(REPO, "docs", "CONFIG.md")) as f:
        assert f.read().strip() == md.strip(), \
            "regenerate: python -m downloader_amd config --reference > docs/CONFIG.md"
    for sec, f in Config.model_fields.items():
        sub = getattr(f.annotation, "model_fields", None)
        for k in (sub or {sec: None}):
            key = f"{sec}.{k}" if sub else sec
            assert f"| `{key}` |" in md, key


def test_k8s_manifest_matches_the_cli_and_probes():
    """deploy/k8s/downloader.yaml: valid YAML, its embedded config loads, the command parses,
    and the probes point at endpoints the health server serves."""
    import yaml

    from downloader_amd.utils.config import load_config
    with open(os.path.join(REPO, "deploy", "k8s", "downloader.yaml")) as f:
        docs = list(yaml.safe_load_all(f))
    cm = next(d for d in docs if d["kind"] == "ConfigMap")
    cfg = load_config(overrides=yaml.safe_load(cm["data"]["downloader.yaml"]), env={})
    assert cfg.concurrency == 8 and cfg.instance.download_path == "/data/downloads"
    dep = next(d for d in docs if d["kind"] == "Deployment")
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][:4] == ["python3", "-m", "downloader_amd", "supervisor"]
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"
    src = open(os.path.join(REPO, "downloader_amd", "service", "health.py")).read()
    assert '"/readyz"' in src and '"/healthz"' in src and '"/metrics"' in src
    # memory: the request covers every worker's worst case - fixed part (interpreter, native
    # modules, HIP runtime) + its part-buffer budget, which the worker derives from the limit
    from downloader_amd.utils import membudget

    def gib(q: str) -> float:
        assert q.endswith("Gi"), q
        return float(q[:-2])
    n = int(c["command"][c["command"].index("-n") + 1])
    res = c["resources"]
    limit, request = gib(res["limits"]["memory"]), gib(res["requests"]["memory"])
    budget = limit / n * cfg.download.relay_memory_fraction
    assert cfg.download.relay_memory_mb == 0          # the budget follows the limit
    assert request >= n * (2.3 + budget), (request, n, budget)
    assert limit >= request
    assert membudget.MIN_BUDGET <= budget * (1 << 30)


def test_concurrent_builds_never_leave_a_broken_binary(tmp_path):
    """Ranks of a multi-GPU bench may find a stale blobd together: each builder writes a
    private temporary file that atomically replaces the binary."""
    code = ("import sys; sys.path.insert(0, %r); from downloader_amd.ops import build; "
            "build.build_blobd(force=True, verbose=False)" % REPO)
    procs = [subprocess.Popen([sys.executable, "-c", code]) for _ in range(3)]
    assert all(p.wait(timeout=300) == 0 for p in procs)
    exe = os.path.join(REPO, "downloader_amd", "bin", "blobd")
    r = subprocess.run([exe, "--bogus"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "usage: blobd" in r.stderr
    assert not [f for f in os.listdir(os.path.dirname(exe)) if ".tmp." in f]


def test_doctor_reports_host_readiness():
    """``doctor``: native SIMD paths, CPUs, open-file limit, the uid's pipe budget and the
    pipe size the worker would pick, THP, GPUs - as JSON with a warnings list."""
    import subprocess
    r = subprocess.run([sys.executable, "-m", "downloader_amd", "doctor", "--sharers", "8"],
                       capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=REPO))
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout)
    assert d["native"]["loaded"] and d["native"]["crc32c"] in ("avx512-vpclmulqdq",
                                                               "sse4.2-3way")
    assert d["pipes"]["sharers"] == 8 and d["pipes"]["pipe_bytes"] >= 64 << 10
    assert d["cpus"]["effective"] >= 1 and isinstance(d["warnings"], list)
    m = d["memory"]
    assert m["part_budget_bytes"] > 0 and m["worst_case_worker_bytes"] > m["part_budget_bytes"]
    assert "devices" in d["gpu"]
