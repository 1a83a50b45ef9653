#!/bin/bash
# Profile every BASELINE config's decode kernel at HEAD (run through gpurun):
#   bash scripts/profile_all.sh TAG
# gpurun_out/prof_TAG_<cfg>/ per config (scripts/profile.sh), stops at the first failure.
set -o pipefail
TAG=${1:-head}
R="$GRAFT_REPO_ROOT"
for c in cfg3 cfg2 cfg4 cfg5; do
  echo "== $c"
  bash "$R/scripts/profile.sh" "${TAG}_$c" --no-secondary --config $c || exit $?
done
echo "all profiles done"
