B="python bench.py --cpu-seconds 0"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "loops|400|$T tests/test_gpu_loops.py -m gpu" "tests|400|$T tests -m gpu" "bc|200|$B --steps 20 --warmup 3 --config checksum" "bcn|200|EBPFEMU_NO_JIT=1 $B --steps 20 --warmup 3 --config checksum" "b5|120|$B --steps 100"
