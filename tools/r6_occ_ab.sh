#!/bin/bash
# Round 6: the fixed-slot kernel's occupancy variant -- its GPU tests, then A/B bench lines
# (EBPFEMU_FIXED_OCC=0 vs the default) for the issue-bound configs, and a kernel trace of each.
# Every GPU step under its own time limit; the first failure ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_occ"
mkdir -p "$out"
cd "$root"
timeout -k 10 600 python -u -m pytest tests/test_occ.py tests/test_store_mode.py \
  tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1
for cfg in nat; do
  for g in "" "--generic"; do
    timeout -k 10 200 python -u bench.py --config $cfg --steps 100 --warmup 10 --cpu-seconds 0 \
      --streams 1 $g > "$out/bench_${cfg}${g}.json" 2> "$out/bench_${cfg}${g}.err"
  done
done
for cfg in acl_rules acl; do
  for occ in 0 1; do
    EBPFEMU_FIXED_OCC=$occ timeout -k 10 200 python -u bench.py --config $cfg --steps 200 \
      --warmup 20 --cpu-seconds 0 > "$out/bench_${cfg}_occ$occ.json" 2> "$out/bench_${cfg}_occ$occ.err"
    EBPFEMU_FIXED_OCC=$occ timeout -k 10 200 python -u bench.py --config $cfg --steps 200 \
      --warmup 20 --cpu-seconds 0 --streams 1 > "$out/bench_${cfg}_occ${occ}_s1.json" \
      2> "$out/bench_${cfg}_occ${occ}_s1.err"
  done
done
cd /tmp && export TMPDIR=/tmp
for occ in 0 1; do
  EBPFEMU_FIXED_OCC=$occ timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof_occ$occ" \
    -o run -- python3 "$root/bench.py" --config acl_rules --steps 50 --warmup 5 --cpu-seconds 0 \
    --streams 1 > "$out/prof_occ$occ.log" 2>&1
done
echo done
