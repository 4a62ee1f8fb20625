#!/bin/bash
# Round 6: the fixed-slot kernel's occupancy variant -- its GPU tests, then A/B bench lines
# (EBPFEMU_FIXED_OCC=0 vs the default) for the issue-bound configs, and a kernel trace of each.
# Every GPU step under its own time limit; the first failure ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_occ"
mkdir -p "$out"
cd "$root"
timeout -k 10 240 python -u tools/debug_store.py 7118000000000000570800001f00000007080000140000000f18000000000000bf8700000000000007070000080000006b283c00000000007176280000000000a40200003cf7214e61804200000000007a010500d6a85b681413000007000000b60400000000000069753d000000000071a0ffff0000000047350000000000002f83000064000000ce3508004100000071150f0000000000bf850000fc0300007a07ffff0000008079753d000000000079823300000000006b473c00000000007b283e00000000005760000019224db1af30000000000000af40000000000000af50000000000000af600000000000009500000000000000 128 > "$out/dbg.log" 2>&1
timeout -k 10 800 python -u -m pytest tests/test_occ.py tests/test_store_far.py tests/test_store_mode.py \
  tests/test_gpu_xdp_md.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > "$out/tests.log" 2>&1
for fb in 64 1504; do
  timeout -k 10 200 python -u bench.py --config responder --frame-bytes $fb --steps 100 --warmup 10 \
    --cpu-seconds 0 > "$out/bench_responder_$fb.json" 2> "$out/bench_responder_$fb.err"
done
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
