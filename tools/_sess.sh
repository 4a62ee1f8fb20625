B="python bench.py --cpu-seconds 0"
bash tools/gpu_session.sh "b15|200|$B --steps 50 --frame-bytes 1500" "bd15|200|$B --steps 50 --frame-bytes 1500 --config drop" "b5|120|$B --steps 100"
