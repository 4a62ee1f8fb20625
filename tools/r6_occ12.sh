#!/bin/bash
# Round 6 A/B: the occupancy variant's workgroups of 12 waves x 2 per CU (this tree) against 8 x 3
# (abA/, the last commit): one launch (tools/ab_lib.py) and the bench's two-stream and
# driver-style lines, alternating. Outputs under gpurun_out/r6_occ12/.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_occ12"
mkdir -p "$out"
cd "$root"
timeout -k 10 300 python -u -m pytest tests/test_occ.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/suite.log" 2>&1
for rep in 1 2; do
  for cfg in 5tuple acl_rules drop; do
    for pkg in ebpf-emu_amd abA/ebpf-emu_amd; do
      echo "$pkg $cfg" >> "$out/ab.log"
      timeout -k 10 120 python3 tools/ab_lib.py "$pkg" --fixed --config $cfg --steps 200 >> "$out/ab.log" 2>> "$out/ab.err"
    done
  done
  for t in B A; do
    d=$root; [ $t = A ] && d=$root/abA
    (cd "$d" && timeout -k 10 200 python -u bench.py --cpu-seconds 0 >> "$out/$t.jsonl" 2>> "$out/$t.err")
    (cd "$d" && timeout -k 10 200 python -u bench.py --cpu-seconds 0 --steps 20 --warmup 5 >> "$out/${t}_d20.jsonl" 2>> "$out/$t.err")
    (cd "$d" && timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config acl_rules >> "$out/${t}_acl.jsonl" 2>> "$out/$t.err")
  done
done
echo done
