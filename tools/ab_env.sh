#!/bin/bash
# A/B of environment settings of the in-tree library on one box: bench.py alternating between
# settings, `rounds` times; prints HIP-event us per batch per run.
#   usage: tools/ab_env.sh <rounds> "<bench args>" "VAR=a" "VAR=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
rounds="$1"; args="$2"; shift 2
for r in $(seq "$rounds"); do
  for e in "$@"; do
    us=$(env $e python bench.py --cpu-seconds 0 $args | python -c 'import json,sys; d=json.loads(sys.stdin.read().splitlines()[-1]); print(d["roofline"]["kernel_avg_us"])') || exit $?
    echo "$e round $r: $us us"
  done
done
