#!/bin/bash
# What a box exposes about GPU slots and CPU topology (no kernels launched).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/probe
O=gpurun_out/probe/slots.txt
{
  echo "== env"; env | grep -E 'VISIBLE|ROCR|HIP|CUDA|OMP|LOCAL' | sort
  echo "== cpu.max"; cat /sys/fs/cgroup/cpu.max
  echo "== affinity"; python3 -c 'import os; s=sorted(os.sched_getaffinity(0)); print(len(s), s[:4], s[-4:])'
  echo "== dri"; ls /dev/dri 2>&1
  echo "== kfd nodes"
  for n in /sys/class/kfd/kfd/topology/nodes/*; do
    printf '%s simd=%s cpu_cores=%s numa=%s\n' "$n" \
      "$(grep -m1 simd_count "$n/properties" | awk '{print $2}')" \
      "$(grep -m1 cpu_cores_count "$n/properties" | awk '{print $2}')" \
      "$(cat "$n/properties" | grep -m1 -E '^location_id' | awk '{print $2}')"
  done
  echo "== torch"; timeout -k 5 120 python3 -c 'import torch; print("device_count", torch.cuda.device_count())'
  echo "== topology cpu0,1,64,128"
  for c in 0 1 64 128 192; do
    d=/sys/devices/system/cpu/cpu$c/topology
    echo "cpu$c pkg=$(cat $d/physical_package_id) core=$(cat $d/core_id) sib=$(cat $d/thread_siblings_list)"
  done
  echo "== numa"; ls /sys/devices/system/node | grep node; cat /sys/devices/system/node/node*/cpulist
} > $O 2>&1
cat $O
