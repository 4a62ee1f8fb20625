B="python bench.py --cpu-seconds 0 --steps 100"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_session.sh "tests|400|$T tests -m gpu" "b5|120|$B" "bd|120|$B --config drop" "b5_8m|120|$B --packets 8388608" "s5|120|$B --packets 65536" "s5_4k|120|$B --packets 4096" "tr5|120|python tools/trace_tiles.py"
