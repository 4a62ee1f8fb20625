B="python bench.py --cpu-seconds 0 --steps 100"
bash tools/gpu_session.sh "tests|300|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" "b5|120|$B" "bd|120|$B --config drop" "b5k|120|EBPFEMU_FOLD=kernel $B"
