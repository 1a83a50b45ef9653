# Round-4 final binary: smoke, GPU suite, default bench, config-3 profile
# (full.sh), then the config 2 / 5 / 4 profiles (final_prof2.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/r04/full.sh r04_final3 prof || exit $?
bash scripts/r04/final_prof2.sh
