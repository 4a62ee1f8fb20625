# Round-3 profiles: rocprofv3 kernel-trace summaries of the new paths (xdp_md in place on fixed
# slots, the stack-window programs on an offsets + lens batch and on the loop kernel), PMC HBM
# traffic of the xdp_md batch, and their bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
B="$R/bench.py --cpu-seconds 0"
P="rocprofv3 --kernel-trace --stats --output-format csv"
bash tools/gpu_session.sh \
  "tcall|300|python -u -m pytest tests/test_calls.py tests/test_gpu_xdp_md.py -x -v -m gpu --timeout 120 --timeout-method thread" \
  "pxdp|180|cd /tmp && $P -d $R/gpurun_out/pxdp -o run -- python3 $B --steps 100 --config xdp" \
  "pstko|180|cd /tmp && $P -d $R/gpurun_out/pstko -o run -- python3 $B --steps 100 --config stack --layout offsets" \
  "pcs|240|cd /tmp && $P -d $R/gpurun_out/pcs -o run -- python3 $B --steps 20 --warmup 3 --config checksum_stack" \
  "pmcx|200|PMC_GROUPS='FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS' bash tools/pmc.sh xdp --config xdp" \
  "bxdp|200|python bench.py --config xdp" \
  "bstko|200|python bench.py --config stack --layout offsets" \
  "bstkog|200|python bench.py --config stack --layout offsets --generic --steps 20 --warmup 3 --cpu-seconds 0" \
  "b5o|200|python bench.py --layout offsets --cpu-seconds 0" \
  "pcall|180|cd /tmp && $P -d $R/gpurun_out/pcall -o run -- python3 $B --steps 100 --config call" \
  "bcall|200|python bench.py --config call" \
  "bcallg|200|python bench.py --config call --generic --steps 20 --warmup 3 --cpu-seconds 0" \
  "b5|200|python bench.py --cpu-seconds 0" \
  "b5spin|200|EBPFEMU_BENCH_SPIN=1 python bench.py --cpu-seconds 0"
