B="python bench.py --cpu-seconds 0 --steps 100"
bash tools/gpu_session.sh "b5|120|$B" "b5nt|120|EBPFEMU_DMA_POLICY=nt $B" "bd|120|$B --config drop" "bdnt|120|EBPFEMU_DMA_POLICY=nt $B --config drop" "b5_8m|120|$B --packets 8388608" "b5nt_8m|120|EBPFEMU_DMA_POLICY=nt $B --packets 8388608" "b5sc|120|EBPFEMU_DMA_POLICY='sc0 sc1 nt' $B" "bdnc|120|$B --config drop --no-counters"
