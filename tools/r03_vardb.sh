# var kernels with double-buffered windows (EBPFEMU_VAR_DB, default on) vs the metadata prefetch
# alone: the var/xdp/stack/layout GPU tests, then A/B on offsets + lens batches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "t|300|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jit.py tests/test_gpu_xdp_md.py tests/test_stack_tier.py tests/test_calls.py tests/test_pcap.py -x -q --timeout 240 --timeout-method thread -m gpu" \
  "ab1|240|bash tools/ab_env.sh 3 '--layout offsets --streams 1' EBPFEMU_VAR_DB=1 EBPFEMU_VAR_DB=0" \
  "ab2|240|bash tools/ab_env.sh 3 '--layout offsets' EBPFEMU_VAR_DB=1 EBPFEMU_VAR_DB=0" \
  "ab3|240|bash tools/ab_env.sh 2 '--layout offsets --config stack --streams 1' EBPFEMU_VAR_DB=1 EBPFEMU_VAR_DB=0" \
  "ab4|240|bash tools/ab_env.sh 2 '--layout offsets --config xdp --streams 1' EBPFEMU_VAR_DB=1 EBPFEMU_VAR_DB=0" \
  "ab6|240|bash tools/ab_env.sh 2 '--layout offsets --config acl --streams 1' EBPFEMU_VAR_DB=1 EBPFEMU_VAR_DB=0"
