B="python bench.py --cpu-seconds 0 --steps 100"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "tests|400|$T tests -m gpu" "b5|120|$B" "bd|120|$B --config drop" "b5_8m|120|$B --packets 8388608" "bd_8m|120|$B --packets 8388608 --config drop" "b5k|120|EBPFEMU_FOLD=kernel $B" "b5p|120|EBPFEMU_LDS_PAD=8192 $B"
