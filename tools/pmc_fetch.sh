#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes only (HBM traffic), one rocprofv3 run each, over a short bench run.
#   usage: tools/pmc_fetch.sh <tag> <bench args...>
set -e
tag="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/pmc/$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 "$root/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 "$@" > "$out/p$i.log" 2>&1 || {
    rc=$?; echo "pass $i ($grp) failed rc=$rc"; tail -5 "$out/p$i.log"; exit $rc; }
done
