#!/bin/bash
# Round 6: the wide occupancy form (ebpf_tile_jit_fixed_occw) -- the forward-program suites, then
# an A/B against the previous commit's build in abA/ (tools/ab_lib.py, alternating). Outputs
# under gpurun_out/r6_occw/. The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_occw"
mkdir -p "$out"
cd "$root"
timeout -k 10 700 python -u -m pytest tests/test_occ.py tests/test_gpu_jit.py tests/test_big_programs.py \
  tests/test_gpu_parity.py tests/test_calls.py tests/test_varl.py -m gpu -x -q --timeout 300 \
  --timeout-method thread --durations=10 > "$out/suite.log" 2>&1
for rep in 1 2; do
  for cfg in acl_rules acl 5tuple; do
    for pkg in ebpf-emu_amd abA/ebpf-emu_amd; do
      echo "$pkg $cfg" >> "$out/ab.log"
      timeout -k 10 120 python3 tools/ab_lib.py "$pkg" --fixed --config $cfg --steps 200 >> "$out/ab.log" 2>> "$out/ab.err"
    done
  done
done
for cfg in acl_rules acl 5tuple; do
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config $cfg >> "$out/lines.jsonl" 2>> "$out/lines.err"
  (cd abA && timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config $cfg >> "$out/lines_A.jsonl" 2>> "$out/lines.err")
done
echo done
