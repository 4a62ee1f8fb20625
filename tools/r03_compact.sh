# coop_sum_compact (config 5 on the deep kernel, batch order): the loop parity tests, the
# full-size golden counters, then the A/B against the strided sum, and the SOL scan.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "tcoop|400|python -u -m pytest tests/test_gpu_loops.py -x -v -m gpu -k 'coop' --timeout 120 --timeout-method thread" \
  "k0|120|$B" "ks|120|EBPFEMU_LOOP_DEEP=1 EBPFEMU_COOP_STRIDED=1 EBPFEMU_BIN=0 $B" "k0b|120|$B" "ksb|120|EBPFEMU_LOOP_DEEP=1 EBPFEMU_COOP_STRIDED=1 EBPFEMU_BIN=0 $B" \
  "tloops|500|python -u -m pytest tests/test_gpu_loops.py -x -q -m gpu --timeout 120 --timeout-method thread" \
  "tgold|300|python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k 'golden' --timeout 200 --timeout-method thread" \
  "sol|200|./build/scan_sol"
