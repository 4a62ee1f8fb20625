#!/bin/bash
# Round 6 A/B: the fixed-slot occupancy variant at 6 waves per SIMD (this tree: 3 x 8-wave
# workgroups per CU) against 7 (ab7/: 7 x 4-wave workgroups, SGPRs capped at 96) -- one stream,
# HIP-event us per 1 Mi-packet batch, alternating builds (tools/ab_lib.py).
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
out="$root/gpurun_out/r6_ab7"
mkdir -p "$out"
for rep in 1 2 3; do
  for cfg in acl_rules acl; do
    for pkg in ebpf-emu_amd ab7/ebpf-emu_amd; do
      timeout -k 10 120 python3 tools/ab_lib.py "$pkg" --fixed --config $cfg --steps 200 >> "$out/ab.log" 2>> "$out/ab.err"
    done
  done
done
echo done
