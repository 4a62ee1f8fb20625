B="python bench.py --cpu-seconds 0"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "jit|400|$T tests/test_gpu_jit.py tests/test_gpu_parity.py -m gpu" "b5|120|$B --steps 100" "b5b|120|$B --steps 100" "bd|120|$B --steps 100 --config drop"
