# Round 5 GPU call 27: kernel trace + PMC passes of config 3 on the final
# (fast-tail) binary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/profile.sh r05final2_cfg3 --no-secondary --config cfg3
