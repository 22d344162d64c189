#!/bin/bash
# Same-box A/B of the default bench: an older tree in ./ab_old (git archive <commit> |
# tar -x -C ab_old, native modules built in it; git-ignored) vs this tree, alternating.
set -o pipefail
F=gpurun_out/r3_ab_regress; mkdir -p $F
export LOG_LEVEL=error TMPDIR=/tmp
for i in 1 2 3; do
  (cd ab_old && timeout -k 10 300 python bench.py > ../$F/old_$i.json 2>> ../$F/err.txt) || exit 1
  timeout -k 10 300 python bench.py > $F/new_$i.json 2>> $F/err.txt || exit 1
  python -c "import json;a=json.load(open('$F/old_$i.json'));b=json.load(open('$F/new_$i.json'));print('old', a['value'], a['single_put_MBps'], 'new', b['value'], b['single_put_MBps'])"
done
