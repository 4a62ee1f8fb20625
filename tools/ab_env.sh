#!/bin/bash
# A/B of environment settings of the in-tree library on one box: bench.py alternating between
# settings, `rounds` times; prints, per run, value (Mpkt/s), HIP-event us per batch, one launch
# at a time (us) and the wall clock's fixed part (us).
#   usage: tools/ab_env.sh <rounds> "<bench args>" "VAR=a" "VAR=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
rounds="$1"; args="$2"; shift 2
for r in $(seq "$rounds"); do
  for e in "$@"; do
    line=$(env $e python bench.py --cpu-seconds 0 $args | tail -n 1) || exit $?
    echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(sys.argv[1], "round", sys.argv[2], "value", d["value"], "event_us", r["kernel_avg_us"], "single_us", r["kernel_single_us"], "fixed_us", d["wall_fixed_us"])' "$e" "$r" || exit $?
  done
done
