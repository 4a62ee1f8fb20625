#!/bin/bash
# Round 6: the overflow fill with 16-byte loads for whole chunks -- the store suites, then the
# responder on 1504-byte slots and NAT. Outputs under gpurun_out/r6_fill/.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_fill"
mkdir -p "$out"
cd "$root"
timeout -k 10 600 python -u -m pytest tests/test_store_mode.py tests/test_store_far.py tests/test_stack_tier.py \
  tests/test_big_programs.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/suite.log" 2>&1
b() { local tag="$1"; shift; timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" >> "$out/$tag.jsonl" 2>> "$out/$tag.err"; }
b r1504 --config responder --frame-bytes 1504
b r1504_s1 --config responder --frame-bytes 1504 --streams 1
b nat --config nat
echo done
