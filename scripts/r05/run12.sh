# Round 5 GPU call 12: kernel traces + PMC passes of the round-5 binary,
# configs 3 and 2 (scripts/profile.sh; run13.sh: configs 4 and 5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in cfg3 cfg2; do
  echo "== $c"
  bash scripts/profile.sh r05final_$c --no-secondary --config $c || exit $?
done
