#!/bin/bash
# Runs GPU steps in order on the gpurun box. Each step has its own time limit. Any failing step
# ends the session (a failed test may be a GPU fault: nothing further touches the GPU); so does a
# log that reports a GPU fault even where the step's exit status is 0.
#   usage: tools/gpu_session.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rc_all=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] || grep -qi "illegal memory access\|memory access fault\|hipErrorIllegalAddress" "gpurun_out/$name.log"; then
    echo "=== stopping after [$name]: exit $rc" | tee -a gpurun_out/session.log
    exit $(( rc ? rc : 1 ))
  fi
done
exit 0
