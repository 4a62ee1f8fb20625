#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only; never combined with
# sys/runtime traces) over a short bench run. Output CSVs under gpurun_out/pmc/<tag>/.
#   usage: tools/pmc.sh <tag> <bench args...>
set -e
tag="$1"; shift
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/pmc/$tag"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
# PMC_GROUPS (groups separated by ";") replaces the default passes
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -ra GROUPS_ <<< "$PMC_GROUPS"; else GROUPS_=(
  "FETCH_SIZE" "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
  "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_INT64 TCC_HIT_sum TCC_MISS_sum"); fi
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$out/p$i" -o run -- python3 "$root/bench.py" --steps 20 --warmup 3 --cpu-seconds 0 "$@" > "$out/p$i.log" 2>&1 || {
    rc=$?; echo "pass $i ($grp) failed rc=$rc"; tail -5 "$out/p$i.log"
    [ $rc -ge 124 ] && exit $rc  # timeout / abort / fault: nothing more on the GPU
  }
done
ls -R "$out" | head -50
