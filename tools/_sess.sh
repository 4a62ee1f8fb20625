B="python bench.py --cpu-seconds 0"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "loops|400|$T tests/test_gpu_loops.py tests/test_gpu_parity.py -m gpu" "bc|200|$B --steps 20 --warmup 3 --config checksum" "b5|120|$B --steps 100"
