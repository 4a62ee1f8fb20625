# the var kernel (offsets + lens batches): round-2's build (worktree under build/r2) vs this one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "v2|120|python tools/ab_lib.py build/r2/ebpf-emu_amd" "v3|120|python tools/ab_lib.py ebpf-emu_amd" \
  "v2b|120|python tools/ab_lib.py build/r2/ebpf-emu_amd" "v3b|120|python tools/ab_lib.py ebpf-emu_amd" \
  "f2|120|python tools/ab_lib.py build/r2/ebpf-emu_amd --fixed" "f3|120|python tools/ab_lib.py ebpf-emu_amd --fixed"
