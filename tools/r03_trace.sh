# config 5 on the deep kernel (coop_sum_compact, batch order): the per-wave timeline and PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "tr|200|python tools/trace_loop.py" \
  "pmc|400|PMC_GROUPS='FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS;GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum' bash tools/pmc.sh cs3 --config checksum"
