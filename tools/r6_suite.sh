#!/bin/bash
# Round 6: the GPU suite with its timing summary and the smoke test (gpurun_out/r6_suite/).
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_suite"
mkdir -p "$out"
cd "$root"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --durations=30 > "$out/suite.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/default.json" 2> "$out/default.err"
echo done
