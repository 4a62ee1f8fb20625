#!/bin/bash
# Runs GPU steps in order on the gpurun box. Each step has its own time limit. A test failure
# (exit 1) does not stop the session; a crash-type exit (timeout 124/137, abort 134, segfault
# 139, or anything >= 128) ends it immediately and nothing further touches the GPU.
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
  if [ $rc -ge 124 ] && [ $rc -ne 0 ]; then
    echo "=== stopping: crash-type exit $rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
  [ $rc -ne 0 ] && rc_all=$rc
done
exit $rc_all
