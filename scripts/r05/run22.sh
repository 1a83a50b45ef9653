# Round 5 GPU call 22: the final binary -- smoke, the whole GPU suite, the
# default bench line (with the secondary configs) and a rocprofv3 kernel trace
# of one lone LzmaDecode caller.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run22
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
s=$?; echo "smoke exit $s: $(tail -1 $O/smoke.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1
s=$?; echo "pytest exit $s: $(tail -1 $O/pytest_gpu.log)"; [ $s -eq 0 ] || exit $s
timeout -k 10 600 python bench.py > $O/bench_line.json 2> $O/bench.err
s=$?; echo "bench exit $s: $(python -c "import json;d=json.load(open('$O/bench_line.json'));print(d['value'], d['ms_per_step'], d['verified'], {k:(v['value'],v['verified']) for k,v in d['secondary'].items()})")"; [ $s -eq 0 ] || exit $s
F=$(python scripts/r05/stream_set.py $O/set 512) || exit 1
B=$GRAFT_REPO_ROOT/tests/c_host/build/lzma_c_threads
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_1 -o kt --output-format csv -- \
  $B 1 $F 1 one > $GRAFT_REPO_ROOT/$O/kt_1.out 2> $GRAFT_REPO_ROOT/$O/kt_1.err
s=$?; echo "kt 1 exit $s"; exit $s
