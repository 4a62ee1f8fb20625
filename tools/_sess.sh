B="python bench.py --steps 200 --warmup 20 --cpu-seconds 0"
P="cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --cpu-seconds 0"
bash tools/gpu_session.sh "tests|400|python -m pytest tests -m gpu -x -q" "b5|120|$B --config 5tuple" "bd|120|$B --config drop" "bc|120|$B --config checksum" "prof5|240|$P" "pmc5|600|bash tools/pmc.sh t5 --config 5tuple" "bench|300|python bench.py"
