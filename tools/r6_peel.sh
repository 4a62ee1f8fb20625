#!/bin/bash
# Round 6: loop-invariant bound loads peeled (host.cpp peel_invariant_loads) -- the peel tests and
# the loop / xdp_md / long-program suites, then the reload checksum's lines. Outputs under
# gpurun_out/r6_peel/. The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_peel"
mkdir -p "$out"
cd "$root"
timeout -k 10 600 python -u -m pytest tests/test_peel.py tests/test_gpu_xdp_md.py tests/test_gpu_loops.py \
  tests/test_big_programs.py tests/test_calls.py -m gpu -x -q --timeout 300 --timeout-method thread \
  --durations=10 > "$out/suite.log" 2>&1
b() {  # tag, bench args
  local tag="$1"; shift
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 "$@" >> "$out/$tag.jsonl" 2>> "$out/$tag.err"
}
b reload --config checksum_xdp_reload --steps 50
b reload_s1 --config checksum_xdp_reload --streams 1 --steps 50
b xdp --config checksum_xdp --steps 50
echo done
