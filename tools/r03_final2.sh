# end of round 3 (session 3): the full GPU suite, smoke, the default bench line, two driver-style
# 20-step runs, then HBM-traffic PMC passes of the var kernel (5-tuple and stack 5-tuple on an
# offsets + lens batch, one stream)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "t|800|python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread" \
  "s|120|python -c \"import __graft_entry__ as g; g.smoke()\"" \
  "b|200|python bench.py" \
  "b20|120|python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --cpu-seconds-1core 0" \
  "b20b|120|python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --cpu-seconds-1core 0" \
  "pv|300|bash tools/pmc_fetch.sh 5tuple_offsets --layout offsets --streams 1 --cpu-seconds-1core 0" \
  "ps|300|bash tools/pmc_fetch.sh stack_offsets --layout offsets --config stack --streams 1 --cpu-seconds-1core 0"
