#!/bin/bash
# Config 1 (10 MB single jobs) A/B: this tree vs the round-2 morning tree (.abtree, commit
# c7330fb, same native modules), alternating, 61 jobs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
F=gpurun_out/c1_ab
mkdir -p $F
export LOG_LEVEL=error
for i in 1 2 3; do
  for t in .abtree .; do
    ( cd /tmp && PYTHONPATH=$GRAFT_REPO_ROOT/$t timeout -k 10 120 python -m downloader_amd.bench.configs --config 1 --jobs 61 ) > $F/c1_${i}_$( [ $t = . ] && echo new || echo old ).json 2>> $F/err.txt || exit 1
  done
done
for f in $F/c1_*.json; do echo "$f $(cat $f)"; done
