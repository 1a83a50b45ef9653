#!/bin/bash
# A/B bench runs on the GPU box: COMBOS="variant:lanes:occ[:VAR=v,VAR=v] ..."
# (variant = a lib/variants/liblzmagpu_<variant>.so, or "main" for
# lib/liblzmagpu.so; lanes/occ 0 = planner default; optional extra env).
# Two interleaved rounds; stops on a crash.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-ab}; shift
BARGS="$*"
for round in 1 2; do
for c in $COMBOS; do
  v=$(echo $c | cut -d: -f1); l=$(echo $c | cut -d: -f2); o=$(echo $c | cut -d: -f3)
  x=$(echo $c | cut -d: -f4 -s | tr ',' ' ')
  if [ "$v" = main ]; then lib=$PWD/lzma-sdk-zliblike_amd/lib/liblzmagpu.so; else lib=$PWD/lzma-sdk-zliblike_amd/lib/variants/liblzmagpu_$v.so; fi
  envs="LZGPU_LIB=$lib"
  [ "$l" != 0 ] && envs="$envs LZGPU_LANES=$l"
  [ "$o" != 0 ] && envs="$envs LZGPU_OCC=$o"
  [ -n "$x" ] && envs="$envs $x"
  xt=$(echo "$x" | tr -cd 'A-Za-z0-9')
  out=gpurun_out/${TAG}_${v}_l${l}o${o}${xt}_$round.json
  env $envs timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $BARGS > $out 2>> gpurun_out/${TAG}.err
  s=$?; echo "$v lanes=$l occ=$o $x r$round exit $s: $(python -c "import json;d=json.load(open('$out'));print(d['value'], d['ms_per_step'], d['config']['kernel_plan'], d['verified'])")"
  [ $s -eq 0 ] || exit $s
done
done
