# coop_sum_compact with the window's part summed from LDS: coop parity tests, A/B vs
# EBPFEMU_COOP_NO_WINDOW, the loop suite, config 5's golden counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "tcoop|400|python -u -m pytest tests/test_gpu_loops.py -x -v -m gpu -k 'coop' --timeout 120 --timeout-method thread" \
  "w0|120|$B" "wd2|120|EBPFEMU_COOP_DEPTH=2 $B" "w0b|120|$B" "wd2b|120|EBPFEMU_COOP_DEPTH=2 $B" \
  "tloops|500|python -u -m pytest tests/test_gpu_loops.py -x -q -m gpu --timeout 120 --timeout-method thread" \
  "tgold|300|python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k 'golden' --timeout 200 --timeout-method thread"
