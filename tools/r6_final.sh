#!/bin/bash
# Round 6, on the round's last code: the GPU suite (durations), the smoke test, every bench config
# (two streams, the default), the headline's driver-style lines, one-launch lines, and the rocprof
# kernel summaries + PMC of the headline on its new kernel (ebpf_tile_jit_fixed_occ). Outputs
# under gpurun_out/r6_final/ (PMC: gpurun_out/pmc/). The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/r6_final"
mkdir -p "$out"
cd "$root"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --durations=30 > "$out/suite.log" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > "$out/smoke.log" 2>&1
b() {  # tag, bench args
  local tag="$1"; shift
  timeout -k 10 300 python -u bench.py "$@" >> "$out/$tag.jsonl" 2>> "$out/$tag.err"
}
b default
for cfg in 5tuple drop stack tier1 acl xdp call nat acl_rules checksum checksum_stack checksum_xdp checksum_xdp_reload; do
  b all --config $cfg --cpu-seconds 0
done
b all --config responder --frame-bytes 1504 --cpu-seconds 0
for i in 1 2 3; do b driver20 --steps 20 --warmup 5; done
for cfg in 5tuple acl_rules nat checksum_xdp_reload; do b s1 --config $cfg --streams 1 --cpu-seconds 0; done
bash tools/prof.sh r6_5tuple_occ_s1 --config 5tuple --steps 200 --warmup 20
bash tools/pmc.sh 5tuple_occ --config 5tuple --streams 1
python3 tools/pmc_summary.py gpurun_out/pmc/5tuple_occ ebpf_tile_jit_fixed_occ > gpurun_out/pmc/5tuple_occ.json
bash tools/pmc.sh acl_rules_occw --config acl_rules --streams 1
python3 tools/pmc_summary.py gpurun_out/pmc/acl_rules_occw ebpf_tile_jit_fixed_occw > gpurun_out/pmc/acl_rules_occw.json
bash tools/pmc.sh drop_occ --config drop --streams 1
python3 tools/pmc_summary.py gpurun_out/pmc/drop_occ ebpf_tile_jit_fixed_occ > gpurun_out/pmc/drop_occ.json
echo done
