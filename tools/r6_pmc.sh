#!/bin/bash
# Round 6: PMC passes (tools/pmc.sh, one counter group per rocprofv3 run) and kernel traces of
# the lines round 6 changed: the general interpreter (--generic: nat on tier 1, acl_rules on
# tier 0), acl_rules on the occupancy variant, NAT in store mode. Summaries into
# gpurun_out/pmc/<tag>.json (tools/pmc_summary.py). The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
run() {  # tag kernel-substring bench-args...
  local tag="$1" k="$2"; shift 2
  bash tools/pmc.sh "$tag" "$@"
  python3 tools/pmc_summary.py "gpurun_out/pmc/$tag" "$k" > "gpurun_out/pmc/$tag.json"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/pmc/${tag}_prof" -o run -- \
    python3 "$root/bench.py" --steps 50 --warmup 5 --cpu-seconds 0 "$@" \
    > "$root/gpurun_out/pmc/${tag}_prof.log" 2>&1
  cd "$root"
}
run nat_generic interp_kernel --config nat --generic --streams 1
run acl_rules_generic interp_kernel --config acl_rules --generic --streams 1
run acl_rules ebpf_tile_jit_fixed_occ --config acl_rules --streams 1
run nat ebpf_tile_jit_varl_stack --config nat --streams 1
echo done
