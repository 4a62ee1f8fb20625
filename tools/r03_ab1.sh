# config 5 (coop_sum_compact): the counters' cost (--no-counters), the fold kernel, persistent grid
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "a0|120|$B" "anc|120|$B --no-counters" "afk|120|EBPFEMU_FOLD=kernel $B" "ap|120|EBPFEMU_LOOP_GRID=persist $B" \
  "a0b|120|$B" "ancb|120|$B --no-counters" "afkb|120|EBPFEMU_FOLD=kernel $B" "apb|120|EBPFEMU_LOOP_GRID=persist $B"
