#!/bin/bash
# Round 6: PMC passes and a kernel summary of acl_rules on the round's last code (complement
# regions). Summaries into gpurun_out/pmc/. The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
bash tools/pmc.sh acl_rules_cm --config acl_rules --streams 1
python3 tools/pmc_summary.py gpurun_out/pmc/acl_rules_cm ebpf_tile_jit_fixed_occ > gpurun_out/pmc/acl_rules_cm.json
bash tools/prof.sh r6_acl_rules_cm_s1 --config acl_rules --steps 200 --warmup 20
echo done
