# Round 4 final binary: kernel trace + PMC passes of configs 2, 5 and 4 (the
# config-3 profile is in full.sh r04_final prof).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in cfg2 cfg5; do
  bash scripts/profile.sh r04_final3_$c --config $c > gpurun_out/prof_r04_final3_$c.log 2>&1
  s=$?; echo "$c profile exit $s"; tail -1 gpurun_out/prof_r04_final3_$c.log; [ $s -eq 0 ] || exit $s
done
bash scripts/profile.sh r04_final3_cfg4 --config cfg4 --no-gather > gpurun_out/prof_r04_final3_cfg4.log 2>&1
s=$?; echo "cfg4 profile exit $s"; tail -1 gpurun_out/prof_r04_final3_cfg4.log; exit $s
