# Checksum loop kernel: PMC of the plain loop kernel (5 waves per SIMD) and of the same code on the
# deep kernel (4 waves, EBPFEMU_LOOP_DEEP=1), and the A/B of the two.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "c1a|120|$B" "c1da|120|EBPFEMU_LOOP_DEEP=1 $B" "c1b|120|$B" "c1db|120|EBPFEMU_LOOP_DEEP=1 $B" \
  "pmc1|300|bash tools/pmc.sh cs1 --config checksum" \
  "pmc1d|300|EBPFEMU_LOOP_DEEP=1 bash tools/pmc.sh cs1d --config checksum"
