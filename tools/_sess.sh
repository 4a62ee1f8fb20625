B="python bench.py --cpu-seconds 0 --steps 100"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "jit|300|$T tests/test_gpu_jit.py -m gpu" "b5|120|$B" "b5f|120|EBPFEMU_GRID=full $B" "bd|120|$B --config drop" "bdf|120|EBPFEMU_GRID=full $B --config drop" "b5_8m|120|$B --packets 8388608" "b5p|120|EBPFEMU_LDS_PAD=8192 $B" "bdp|120|EBPFEMU_LDS_PAD=8192 $B --config drop"
