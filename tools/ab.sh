# Summarise bench logs of a gpu_session run: name value kernel_us frac
for f in "$@"; do echo -n "$f "; tail -1 gpurun_out/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])" 2>/dev/null || echo "(no json)"; done
