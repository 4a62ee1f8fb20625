# every bench workload at the two-stream default (CPU baselines skipped; the headline set has them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --cpu-seconds 0"
bash tools/gpu_session.sh \
  "x_stack|120|$B --config stack" "x_tier1|120|$B --config tier1" "x_acl|120|$B --config acl" \
  "x_xdp|120|$B --config xdp" "x_call|120|$B --config call" \
  "x_5o|120|$B --layout offsets" "x_stko|120|$B --config stack --layout offsets" \
  "x_5t1500|200|$B --frame-bytes 1500 --steps 50" "x_drop1500|200|$B --config drop --frame-bytes 1500 --steps 50" \
  "x_cstk|300|$B --config checksum_stack --steps 20 --warmup 3"
