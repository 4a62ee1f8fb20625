# coop_sum (the byte sum of whole ranges, transposed): the loop parity tests, config 5's golden
# counters, then the checksum batch with and without it (A/B on one box) and its rocprof summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "tloops|500|python -u -m pytest tests/test_gpu_loops.py -x -v -m gpu --timeout 120 --timeout-method thread" \
  "tgold|300|python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k 'golden' --timeout 200 --timeout-method thread" \
  "ca|120|$B" "cna|120|EBPFEMU_NO_COOP_SUM=1 $B" "cb|120|$B" "cnb|120|EBPFEMU_NO_COOP_SUM=1 $B" \
  "pcs|180|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pcoop -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 50 --config checksum"
