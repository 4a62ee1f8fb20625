# driver-style runs (20 steps) with warmup 5 / 8 / 16: does the 20-step device time per batch
# (12.9 vs 10.9 us at 200 steps) come from pool batches first touched inside the timed region?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --steps 20 --cpu-seconds 0 --cpu-seconds-1core 0"
bash tools/gpu_session.sh \
  "w5a|120|$B --warmup 5" "w8a|120|$B --warmup 8" "w16a|120|$B --warmup 16" \
  "w5b|120|$B --warmup 5" "w8b|120|$B --warmup 8" "w16b|120|$B --warmup 16" \
  "w5s1|120|$B --warmup 5 --streams 1" "w8s1|120|$B --warmup 8 --streams 1" \
  "w5c|120|$B --warmup 5 --steps 50" "w8c|120|$B --warmup 8 --steps 50"
