#!/bin/bash
# Round 6: PMC of NAT on the fixed-slot statement's store mode, then the headline's breakdown on
# its round-6 kernel (tools/r6_headline.sh: one-stream trace, two-stream union, stamps, driver-style
# lines). The first failing step ends the script.
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
bash tools/pmc.sh nat_fixed --config nat --streams 1
python3 tools/pmc_summary.py gpurun_out/pmc/nat_fixed ebpf_tile_jit_fixed > gpurun_out/pmc/nat_fixed.json
bash tools/r6_headline.sh
echo done
