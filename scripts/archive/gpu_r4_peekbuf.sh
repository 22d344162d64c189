#!/bin/bash
# Round 4: does the CRC staging buffer size matter for the peeked relay? relaybench peekcrc at
# 8 relay threads with 64 KiB .. 1 MiB buffers (1 MiB pipes), alternating, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
F=${OUT:-gpurun_out/r4_peekbuf}
mkdir -p $F
for r in 1 2; do
  for b in 64 128 256 512 1024; do
    timeout -k 5 120 taskset -c 0-15 ./downloader_amd/bin/relaybench --mode peekcrc --gb 8 --threads 8 --buf-kb $b >> $F/peekbuf.jsonl || exit 1
  done
  for b in 256 1024; do
    timeout -k 5 120 taskset -c 0-15 ./downloader_amd/bin/relaybench --mode teecrc --gb 8 --threads 8 --buf-kb $b >> $F/peekbuf.jsonl || exit 1
  done
done
cat $F/peekbuf.jsonl
