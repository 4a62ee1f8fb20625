#!/bin/bash
# Round 6: the headline (5-tuple, 1 Mi x 64 B, ebpf_tile_jit_fixed_occ since late round 6) -- one launch's kernel trace
# at one stream, the two-stream union (the bench line's per-batch time), the per-wave stamp
# breakdown (EBPFEMU_TRACE=1: ramp, tiles, last-tile spread, counter tail) with and without the
# counters, and driver-style 20-step lines. Outputs under gpurun_out/r6_head/. Every GPU step
# under its own limit; the first failure ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_head"
mkdir -p "$out"
cd "$root"
bash tools/prof.sh r6_5tuple_s1 --config 5tuple --steps 200 --warmup 20
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/s2" -o run -- \
  python3 "$root/bench.py" --cpu-seconds 0 --config 5tuple --steps 200 --warmup 20 \
  > "$out/s2_bench.json" 2> "$out/s2_stderr.log"
cd "$root"
f=$(find "$out/s2" -name "*kernel_trace.csv" | head -1)
python3 tools/rocprof_union.py "$f" ebpf_tile_jit_fixed --skip 20 --count 200 > "$out/s2_union.json"
timeout -k 10 200 python3 tools/trace_tiles.py --config 5tuple > "$out/trace_5tuple.json" 2> "$out/trace.err"
timeout -k 10 200 python3 tools/trace_tiles.py --config 5tuple --no-counters > "$out/trace_5tuple_nocnt.json" 2>> "$out/trace.err"
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > "$out/driver20_$i.json" 2> "$out/driver20_$i.err"
done
timeout -k 10 300 python3 bench.py > "$out/default.json" 2> "$out/default.err"
echo done
