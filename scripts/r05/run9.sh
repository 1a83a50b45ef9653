# Round 5 GPU call 9: the default bench line on the 32-lane one-stream build,
# config 2 with 16 / 32 / 64 lanes per stream, the time-sliced config 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run9
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so > $O/binary.sha256
timeout -k 10 600 python bench.py > $O/bench_line.json 2> $O/bench.err
s=$?; echo "bench exit $s: $(python -c "import json;d=json.load(open('$O/bench_line.json'));print(d['value'], d['ms_per_step'], d['verified'], {k:(v['value'],v['verified']) for k,v in d['secondary'].items()})")"; [ $s -eq 0 ] || exit $s
for D in 16 32 64; do
  LZGPU_DUP=$D timeout -k 10 300 python bench.py --config cfg2 --steps 5 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-crc --no-secondary --sliced 16384 > $O/cfg2_dup$D.json 2>> $O/ab.err || exit $?
  echo "cfg2 dup $D: $(python -c "import json;d=json.load(open('$O/cfg2_dup$D.json'));print(d['value'], d['ms_per_step'], d['verified'], d['sliced']['MBps'], d['sliced']['vs_one_shot'])")"
done
