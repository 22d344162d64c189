# Probe: config 3 at 2 GB staged 3x on one worker, with 1 s of all-CPU spin before the first
# job; prints wall/CPU/peer CPU per rep (docs/PERFORMANCE.md, "Configs 3/4 over repeated jobs").
import asyncio, json, sys, time, argparse, resource, threading
from downloader_amd.bench import configs
inst = {}
class B(configs.Blobd):
    def __enter__(self):
        r = super().__enter__(); inst['b'] = self; return r
configs.Blobd = B
orig = configs._run_jobs
import subprocess
first=[True]
async def wrapped(w, msgs, timeout=3600.0):
    if first[0]:
        first[0]=False
        ps=[subprocess.Popen([sys.executable,'-c','import time\nt=time.time()\nwhile time.time()-t<1.0: pass']) for _ in range(8)]
        [p.wait() for p in ps]
    ru0=resource.getrusage(resource.RUSAGE_SELF); p0 = inst['b'].cpu_seconds(); th0 = threading.active_count()
    dt, r = await orig(w, msgs, timeout)
    ru1=resource.getrusage(resource.RUSAGE_SELF)
    print(json.dumps({"dt": round(dt,3), "sys": round(ru1.ru_stime-ru0.ru_stime,2), "usr": round(ru1.ru_utime-ru0.ru_utime,2),
        "peer": round(inst['b'].cpu_seconds()-p0,2), "threads": (th0, threading.active_count()), "fetch": r[0].stats["torrent"]["webseed_fetch_s"]}), file=sys.stderr)
    return dt, r
configs._run_jobs = wrapped
a = argparse.Namespace(mode="tuned", scale=0.5, piece_mb=4, verify_backend="auto", webseed_streams=0, webseed_chunk_mb=0, webseed_verify_depth=0, src_dir="/dev/shm", stage_dir="", torrent_stream="auto", stream_parallel=0, reps=3)
asyncio.run(configs.config_torrent(a, 3))
