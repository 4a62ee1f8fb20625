# Config 5 (coop_sum, unbinned, deep kernel): one tile per wave vs balanced persistent waves
# (EBPFEMU_LOOP_GRID=persist), A/B, and the persistent grid's timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
E="EBPFEMU_BIN=0 EBPFEMU_LOOP_DEEP=1"
bash tools/gpu_session.sh \
  "tgrid|300|EBPFEMU_LOOP_GRID=persist python -u -m pytest tests/test_gpu_loops.py -x -v -m gpu -k 'coop or binned or budget_exact' --timeout 120 --timeout-method thread" \
  "g1|120|$E $B" "gp|120|$E EBPFEMU_LOOP_GRID=persist $B" \
  "g1b|120|$E $B" "gpb|120|$E EBPFEMU_LOOP_GRID=persist $B" \
  "gp5|120|EBPFEMU_BIN=0 EBPFEMU_LOOP_GRID=persist $B" \
  "tr2|200|$E EBPFEMU_LOOP_GRID=persist python tools/trace_loop.py"
