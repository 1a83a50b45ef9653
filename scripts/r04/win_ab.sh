# Round 4: the LDS history window of the cooperative kernels -- GPU parity of
# every path that runs them, then A/B (LZGPU_WIN=0 vs default) on configs 1 and 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_win
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py \
  tests/test_cfg1.py tests/test_dropin_mirror.py tests/test_sessions.py tests/test_c_host.py \
  tests/test_coalesce.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "coop or parity or cfg1 or mirror or session or c_host or coalesce or streaming or goldens or walker or threads or cfg4" \
  > $O/pytest.log 2>&1
s=$?; echo "pytest exit $s"; tail -2 $O/pytest.log; [ $s -eq 0 ] || exit $s
for round in 1 2; do
  for w in 0 1; do
    LZGPU_WIN=$w timeout -k 10 300 python bench.py --config cfg1 --steps 3 --warmup 1 --no-cpu-baseline \
      > $O/cfg1_w${w}_r$round.json 2>> $O/ab.err || exit $?
    echo "cfg1 win=$w r$round: $(python -c "import json;d=json.load(open('$O/cfg1_w${w}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
    LZGPU_WIN=$w timeout -k 10 300 python bench.py --config cfg4 --steps 5 --warmup 1 --no-cpu-baseline --no-gather \
      > $O/cfg4_w${w}_r$round.json 2>> $O/ab.err || exit $?
    echo "cfg4 win=$w r$round: $(python -c "import json;d=json.load(open('$O/cfg4_w${w}_r$round.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
  done
done
