# bench.py with consecutive batches on two streams (the default) vs one: 5-tuple, drop-all,
# config 5, config 4; rocprof kernel traces of the 5-tuple both ways
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
P="rocprofv3 --kernel-trace --stats --output-format csv"
bash tools/gpu_session.sh \
  "s2|200|python bench.py --cpu-seconds 0" "s1|200|python bench.py --cpu-seconds 0 --streams 1" \
  "s2d|120|python bench.py --steps 20 --warmup 5 --cpu-seconds 0" "s1d|120|python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --streams 1" \
  "d2|120|python bench.py --config drop --cpu-seconds 0" "d1|120|python bench.py --config drop --cpu-seconds 0 --streams 1" \
  "c2|200|python bench.py --config checksum --cpu-seconds 0 --steps 50" "c1|200|python bench.py --config checksum --cpu-seconds 0 --steps 50 --streams 1" \
  "g2|300|python bench.py --total-packets 100000000 --steps 10 --warmup 2 --cpu-seconds 0" "g1|300|python bench.py --total-packets 100000000 --steps 10 --warmup 2 --cpu-seconds 0 --streams 1" \
  "p2|200|cd /tmp && $P -d $R/gpurun_out/p2 -o run -- python3 $R/bench.py --cpu-seconds 0" \
  "p1|200|cd /tmp && $P -d $R/gpurun_out/p1 -o run -- python3 $R/bench.py --cpu-seconds 0 --streams 1"
