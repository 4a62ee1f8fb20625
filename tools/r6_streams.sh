#!/bin/bash
# Round 6: how many streams the bench's batches should alternate over on the round's kernel --
# 2 (the default), 3 and 4, alternating on one box, default and driver-style runs. Outputs under
# gpurun_out/r6_streams/. The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_streams"
mkdir -p "$out"
cd "$root"
for rep in 1 2; do
  for s in 2 3 4; do
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --streams $s >> "$out/s$s.jsonl" 2>> "$out/s$s.err"
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --streams $s --steps 20 --warmup 5 >> "$out/s${s}_d20.jsonl" 2>> "$out/s${s}_d20.err"
  done
done
echo done
