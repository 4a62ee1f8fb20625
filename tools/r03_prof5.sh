# config 5 profile set: rocprof kernel-trace summary, PMC passes, an occupancy probe (LDS pad to
# 3 waves per SIMD), the per-wave timeline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
B="python bench.py --config checksum --cpu-seconds 0 --steps 50 --warmup 5"
bash tools/gpu_session.sh \
  "p5|180|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p5 -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 50 --config checksum" \
  "pmc|400|PMC_GROUPS='FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS;GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum' bash tools/pmc.sh cs4 --config checksum" \
  "o3|120|EBPFEMU_LDS_PAD=12288 $B" "o4|120|$B" \
  "tr|200|python tools/trace_loop.py"
