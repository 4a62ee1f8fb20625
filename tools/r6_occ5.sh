#!/bin/bash
# Round 6: the occupancy variant on short programs (EBPFEMU_FIXED_OCC=1) against the fixed-slot
# kernel, alternating in one box: the bench default (two streams, 200 steps) and the driver's
# style (--steps 20 --warmup 5) for the 5-tuple and drop-all; then the PMC passes and a kernel
# trace of acl_rules on the round's final rule-chain code (pending masks). Outputs under
# gpurun_out/r6_occ5/ and gpurun_out/pmc/. The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_occ5"
mkdir -p "$out"
cd "$root"
b() {  # tag, bench args
  local tag="$1"; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" >> "$out/$tag.jsonl" 2>> "$out/$tag.err"
}
for rep in 1 2 3; do
  for cfg in 5tuple drop; do
    EBPFEMU_FIXED_OCC=0 b ${cfg}_fixed --config $cfg
    EBPFEMU_FIXED_OCC=1 b ${cfg}_occ --config $cfg
    EBPFEMU_FIXED_OCC=0 b ${cfg}_fixed_d20 --config $cfg --steps 20 --warmup 5
    EBPFEMU_FIXED_OCC=1 b ${cfg}_occ_d20 --config $cfg --steps 20 --warmup 5
  done
done
bash tools/pmc.sh acl_rules_pm --config acl_rules --streams 1
python3 tools/pmc_summary.py gpurun_out/pmc/acl_rules_pm ebpf_tile_jit_fixed_occ > gpurun_out/pmc/acl_rules_pm.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/pmc/acl_rules_pm_prof" -o run -- \
  python3 "$root/bench.py" --steps 50 --warmup 5 --cpu-seconds 0 --config acl_rules --streams 1 \
  > "$root/gpurun_out/pmc/acl_rules_pm_prof.log" 2>&1
echo done
