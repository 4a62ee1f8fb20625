# metadata pipeline (var kernels; loop kernels with a persistent grid) + the var kernels' own-
# occupancy grid: GPU tests, then A/B of the knobs (offsets + lens batches, one and two streams;
# config 5), then the settle A/B of the driver-style run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "t|300|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jit.py tests/test_gpu_xdp_md.py tests/test_gpu_loops.py -x -q --timeout 240 --timeout-method thread -k \"var or layout or xdp or loop or golden\"" \
  "ab1|240|bash tools/ab_env.sh 3 '--layout offsets --streams 1' EBPFEMU_VAR_PIPE=1 'EBPFEMU_VAR_PIPE=0 EBPFEMU_VAR_GRID=tile' EBPFEMU_VAR_PIPE=0 EBPFEMU_VAR_GRID=tile" \
  "ab2|240|bash tools/ab_env.sh 3 '--layout offsets' EBPFEMU_VAR_PIPE=1 'EBPFEMU_VAR_PIPE=0 EBPFEMU_VAR_GRID=tile'" \
  "ab3|240|bash tools/ab_env.sh 2 '--layout offsets --config stack --streams 1' EBPFEMU_VAR_PIPE=1 'EBPFEMU_VAR_PIPE=0 EBPFEMU_VAR_GRID=tile'" \
  "tp|300|EBPFEMU_LOOP_GRID=persist python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loops.py -x -q --timeout 240 --timeout-method thread -k \"golden or sample or loop or checksum\"" \
  "ab5|300|bash tools/ab_env.sh 2 '--config checksum --steps 50 --streams 1' EBPFEMU_LOOP_PIPE=1 EBPFEMU_LOOP_GRID=persist 'EBPFEMU_LOOP_GRID=persist EBPFEMU_LOOP_PIPE=0'" \
  && bash tools/r03_settle.sh
