#!/bin/bash
# Round 6: the whole GPU suite (with its timing) on the current tree, then the lines the round's
# compiler changes move: acl_rules / acl (occupancy variant, sunk high-half moves, narrowed
# compares), the responder on 1504-byte slots (store mode's overflow blocks), NAT, and the
# 5-tuple on the occupancy variant as an A/B (EBPFEMU_FIXED_OCC=1). The first failure ends it.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_check"
mkdir -p "$out"
cd "$root"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --durations=25 > "$out/suite.log" 2>&1
# A/B against the build of the previous commit in abA/ (the pending masks, the compare rewrites)
for rep in 1 2; do
  for cfg in acl_rules acl 5tuple; do
    for pkg in ebpf-emu_amd abA/ebpf-emu_amd; do
      echo "$pkg $cfg" >> "$out/ab.log"
      timeout -k 10 120 python3 tools/ab_lib.py "$pkg" --fixed --config $cfg --steps 200 >> "$out/ab.log" 2>> "$out/ab.err"
    done
  done
done
b() {  # tag, bench args
  local tag="$1"; shift
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 "$@" > "$out/$tag.json" 2> "$out/$tag.err"
}
b acl_rules --config acl_rules
b acl_rules_s1 --config acl_rules --streams 1
b acl --config acl
b responder_1504 --config responder --frame-bytes 1504
b responder_1504_s1 --config responder --frame-bytes 1504 --streams 1
b nat_s1 --config nat --streams 1
b 5tuple_s1 --config 5tuple --streams 1
export EBPFEMU_FIXED_OCC=1
b 5tuple_occ_s1 --config 5tuple --streams 1
b 5tuple_occ --config 5tuple
unset EBPFEMU_FIXED_OCC
echo done
