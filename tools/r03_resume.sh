# Round-3 resume: the whole -m gpu suite, then config 5's loop-kernel variants A/B on one box
# (coop_sum on/off, the deep kernel, binned vs unbinned, persistent grid), then the 5-tuple's
# driver-style 20-step line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "tgpu|780|python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread" \
  "c0|120|$B" "cnc|120|EBPFEMU_NO_COOP_SUM=1 $B" "cd|120|EBPFEMU_LOOP_DEEP=1 $B" \
  "cdu|120|EBPFEMU_LOOP_DEEP=1 EBPFEMU_BIN=0 $B" "cdp|120|EBPFEMU_LOOP_DEEP=1 EBPFEMU_BIN=0 EBPFEMU_LOOP_GRID=persist $B" \
  "c0b|120|$B" "cdb|120|EBPFEMU_LOOP_DEEP=1 $B" \
  "b5|120|python bench.py --steps 20 --warmup 20 --cpu-seconds 0"
