# rocprofv3 kernel-trace summaries + bench lines (with the CPU baseline) of the bench workloads
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
B="$R/bench.py --cpu-seconds 0"
bash tools/gpu_session.sh \
  "prof5|180|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof5 -o run -- python3 $B --steps 100" \
  "profd|180|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profd -o run -- python3 $B --steps 100 --config drop" \
  "profc|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profc -o run -- python3 $B --steps 20 --warmup 3 --config checksum" \
  "bench5|240|python bench.py" \
  "benchd|240|python bench.py --config drop" \
  "benchc|300|python bench.py --config checksum" \
  "bench4|300|python bench.py --total-packets 100000000 --steps 20 --warmup 3 --cpu-seconds 0"
