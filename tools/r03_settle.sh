# A/B on one box: the driver-style run (20 steps, 5 warmup) with and without an untimed
# clock-settling run before the warmup steps (bench.py --settle-ms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --cpu-seconds-1core 0"
bash tools/gpu_session.sh \
  "s0a|120|$B" "s50a|120|$B --settle-ms 50" \
  "s0b|120|$B" "s50b|120|$B --settle-ms 50" \
  "s0c|120|$B" "s50c|120|$B --settle-ms 50" \
  "s200|120|$B --settle-ms 200" "s10|120|$B --settle-ms 10"
