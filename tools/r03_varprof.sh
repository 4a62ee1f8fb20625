# round-3 var-kernel lines after the metadata prefetch: offsets + lens batches (5-tuple, stack,
# xdp_md, ACL) at two streams and one, and the rocprof summary of the one-stream 5-tuple
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$PWD
P="rocprofv3 --kernel-trace --stats --output-format csv"
B="python bench.py --layout offsets --cpu-seconds 0 --cpu-seconds-1core 0"
bash tools/gpu_session.sh \
  "vo2|120|$B" "vo1|120|$B --streams 1" \
  "vs2|120|$B --config stack" "vx2|120|$B --config xdp" "va2|120|$B --config acl" \
  "vop|200|cd /tmp && $P -d $R/gpurun_out/vop -o run -- python3 $R/bench.py --layout offsets --streams 1 --cpu-seconds 0 --cpu-seconds-1core 0"
