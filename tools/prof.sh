#!/bin/bash
# rocprofv3 kernel-trace summary of one bench.py workload (one stream: the per-kernel average is
# one launch's duration). Output: gpurun_out/prof/<tag>/run_kernel_stats.csv (+ the trace).
#   usage: tools/prof.sh <tag> <bench args...>     (run on the GPU box, e.g. via gpu_session.sh)
set -e
tag="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/prof/$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 "$root/bench.py" --cpu-seconds 0 --streams 1 "$@" > "$out/bench.json" 2> "$out/stderr.log"
find "$out" -name "*kernel_stats.csv" -exec cp {} "$out/stats.csv" \;
head -5 "$out/stats.csv"
