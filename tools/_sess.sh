bash tools/gpu_session.sh "pcap|300|python tools/e2e_bench.py --pcap" "pcapc|300|python tools/e2e_bench.py --pcap --chunk 4194304"
