# default bench line on the shipped binary, reading the round-3 profile
# summaries (profiles/pmc_cfg3.json, traffic_cfg3.json, pmc_cfg4.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03w
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > gpurun_out/r03w/binary.sha256
timeout -k 10 500 python -u bench.py > gpurun_out/r03w/bench.json 2> gpurun_out/r03w/bench.err
s=$?; echo "bench exit $s"; cut -c1-300 gpurun_out/r03w/bench.json; exit $s
