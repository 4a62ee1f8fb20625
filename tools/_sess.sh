B="python bench.py --cpu-seconds 0 --steps 100"
bash tools/gpu_session.sh "tests|400|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" "b5|120|$B" "b5n|120|EBPFEMU_TILE_PREFETCH=0 $B" "bd|120|$B --config drop" "bdn|120|EBPFEMU_TILE_PREFETCH=0 $B --config drop" "b5b|120|$B" "b5nb|120|EBPFEMU_TILE_PREFETCH=0 $B"
