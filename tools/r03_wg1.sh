# the deep loop kernel in one-wave workgroups (EBPFEMU_LOOP_WG=1) vs four-wave ones: coop parity
# tests on both, then config 5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "tcoop|400|python -u -m pytest tests/test_gpu_loops.py -x -v -m gpu -k 'coop' --timeout 120 --timeout-method thread" \
  "g4|120|EBPFEMU_LOOP_WG=4 $B" "g1|120|EBPFEMU_LOOP_WG=1 $B" "g4b|120|EBPFEMU_LOOP_WG=4 $B" "g1b|120|EBPFEMU_LOOP_WG=1 $B"
