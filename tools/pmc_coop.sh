cd "${GRAFT_REPO_ROOT}" || exit 2
timeout -k 10 120 ./build/scan_sol && \
PMC_GROUPS='SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH' bash tools/pmc.sh coop --config checksum
