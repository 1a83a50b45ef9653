# Round-4 baseline on the round-3 binary: default bench line, then cfg2 / cfg5
# kernel traces + PMC passes on the HEAD binary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_base
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 120 ./scripts/ubench/issue_ubench > $O/issue_ubench.jsonl 2> $O/issue_ubench.err
s=$?; echo "ubench exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench exit $s"; cut -c1-400 $O/bench.json; [ $s -eq 0 ] || exit $s
bash scripts/profile.sh r04_base_cfg2 --config cfg2 > $O/profile_cfg2.log 2>&1
s=$?; echo "profile cfg2 exit $s"; tail -2 $O/profile_cfg2.log; [ $s -eq 0 ] || exit $s
bash scripts/profile.sh r04_base_cfg5 --config cfg5 > $O/profile_cfg5.log 2>&1
s=$?; echo "profile cfg5 exit $s"; tail -2 $O/profile_cfg5.log
exit $s
