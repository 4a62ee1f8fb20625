B="python bench.py --cpu-seconds 0 --steps 100"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "jit|300|$T tests/test_gpu_jit.py -m gpu" "tests|400|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" "b5|120|$B" "b5n|120|EBPFEMU_NO_JIT=1 $B" "b5b|120|$B" "b5nb|120|EBPFEMU_NO_JIT=1 $B"
