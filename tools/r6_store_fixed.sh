#!/bin/bash
# Round 6: store mode on the fixed-slot statement (gen_tile.py STORE_DEOPT_FIXED, marker st=1) --
# the store / stack suites, then NAT and the responder on fixed slots (one launch and two
# streams). Outputs under gpurun_out/r6_store/. The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_store"
mkdir -p "$out"
cd "$root"
timeout -k 10 600 python -u -m pytest tests/test_store_mode.py tests/test_store_far.py \
  tests/test_stack_tier.py tests/test_gpu_xdp_md.py tests/test_knobs.py -m gpu -x -q --timeout 300 \
  --timeout-method thread --durations=10 > "$out/suite.log" 2>&1
b() {  # tag, bench args
  local tag="$1"; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" >> "$out/$tag.jsonl" 2>> "$out/$tag.err"
}
b nat --config nat
b nat_s1 --config nat --streams 1
b responder --config responder
b responder_1504 --config responder --frame-bytes 1504
b responder_1504_s1 --config responder --frame-bytes 1504 --streams 1
b tier1 --config tier1
bash tools/prof.sh r6_nat_fixed_s1 --config nat --steps 200 --warmup 20
echo done
