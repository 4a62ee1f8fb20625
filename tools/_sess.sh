B="python bench.py --cpu-seconds 0 --steps 100"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "jit|300|$T tests/test_gpu_jit.py tests/test_gpu_parity.py -m gpu" "b5|120|$B" "bd|120|$B --config drop" "b5_8m|120|$B --packets 8388608" "bd_8m|120|$B --packets 8388608 --config drop"
