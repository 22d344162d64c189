#!/bin/bash
# Probe: per-user pipe page limits on the box (an unprivileged user's pipes past
# pipe-user-pages-soft are created with one page) and config 3's first-rep cost with the
# tee()d relay on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=${OUT:-gpurun_out/probe_pipes}
mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp PYTHONPATH=${GRAFT_REPO_ROOT:-$PWD}
for f in pipe-max-size pipe-user-pages-soft pipe-user-pages-hard; do echo "$f $(cat /proc/sys/fs/$f)"; done | tee $F/limits.txt
id | tee -a $F/limits.txt
python - <<'PY' | tee -a $F/limits.txt
import fcntl, os
F_SETPIPE_SZ, F_GETPIPE_SZ = 1031, 1032
pipes, sizes = [], []
for i in range(200):
    r, w = os.pipe()
    try:
        fcntl.fcntl(w, F_SETPIPE_SZ, 1 << 20)
    except OSError as e:
        pass
    sizes.append(fcntl.fcntl(w, F_GETPIPE_SZ))
    pipes.append((r, w))
print("first 1 MiB refusal at pipe", next((i for i, s in enumerate(sizes) if s < (1 << 20)), None),
      "sizes seen", sorted(set(sizes)))
PY
for tee in 1 0 1; do
  STAGER_RELAY_TEE=$tee timeout -k 10 300 python -m downloader_amd.bench.configs --config 3 --reps 4 > $F/c3_tee${tee}.json 2>> $F/err.txt || exit 1
  python -c "import json;j=json.loads(open('$F/c3_tee${tee}.json').read().strip().splitlines()[-1]);print('tee $tee', j['MBps_reps'], j['worker_cpu_s'])"
done
timeout -k 10 200 python bench.py --no-compare-single-put > $F/c2.json 2>> $F/err.txt || exit 1
python -c "import json;j=json.loads(open('$F/c2.json').read().strip().splitlines()[-1]);print('headline', j['value'], j['worker_cpu_s_per_GB'], j['peer_cpu_s_per_GB'], j['pipes_short'])"
