# The loop kernel's refill-pattern speed-of-light (tools/scan_sol.hip, built in-tree under build/),
# and a rocprof summary of config 5 on the deep kernel without length binning.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
bash tools/gpu_session.sh \
  "sol|200|./build/scan_sol" \
  "pcdu|180|cd /tmp && EBPFEMU_LOOP_DEEP=1 EBPFEMU_BIN=0 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pcdu -o run -- python3 $R/bench.py --cpu-seconds 0 --steps 50 --config checksum"
