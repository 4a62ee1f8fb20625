# round-3 headline set: the default bench line (two streams, CPU baseline), its rocprof summary,
# drop-all and config 5 lines with CPU baselines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
P="rocprofv3 --kernel-trace --stats --output-format csv"
bash tools/gpu_session.sh \
  "h5|300|python bench.py" \
  "hp5|200|cd /tmp && $P -d $R/gpurun_out/hp5 -o run -- python3 $R/bench.py --cpu-seconds 0" \
  "hd|300|python bench.py --config drop" \
  "hc|300|python bench.py --config checksum" \
  "hpc|200|cd /tmp && $P -d $R/gpurun_out/hpc -o run -- python3 $R/bench.py --cpu-seconds 0 --config checksum --steps 50"
