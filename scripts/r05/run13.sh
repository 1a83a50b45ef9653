# Round 5 GPU call 13: kernel traces + PMC passes of the round-5 binary,
# configs 4 and 5 (scripts/profile.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in cfg4 cfg5; do
  echo "== $c"
  bash scripts/profile.sh r05final_$c --no-secondary --config $c || exit $?
done
