# Round 5 GPU call 35: kernel trace + PMC passes of config 5 on the final
# binary (16 workgroups per CU, slot-global latency placement).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/profile.sh r05final2_cfg5 --no-secondary --config cfg5
