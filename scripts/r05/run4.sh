# Round 5 GPU call 4: the cooperative kernel's decision
# chain -- A/B of the default build against batched bit trees (cb), batched
# trees with the checkpoint reader (cbq), plus NORMALIZE as selects (cbqs),
# and the checkpoint reader + select NORMALIZE alone (qs), on config 4 (two
# rounds), the xz leg and config 1 (every bench leg verifies its output
# bit-exactly); config-4 region profiles of the default and cb builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05_run4
V=lzma-sdk-zliblike_amd/lib/variants
mkdir -p $O
sha256sum lzma-sdk-zliblike_amd/lib/liblzmagpu.so $V/*.so > $O/binary.sha256
run() {  # config variant tag [extra args]
  local c=$1 v=$2 t=$3; shift 3
  local L=""; [ $v != base ] && L=$V/liblzmagpu_$v.so
  LZGPU_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline "$@" \
    > $O/${c}_${v}_$t.json 2>> $O/ab.err || return $?
  echo "$c $v $t: $(python -c "import json;d=json.load(open('$O/${c}_${v}_$t.json'));print(d['value'], d['ms_per_step'], d['verified'])")"
}
for round in 1 2; do
  for v in base cb cbq cbqs qs; do run cfg4 $v r$round --no-gather || exit $?; done
done
for v in base cb cbq cbqs qs; do run xz $v r1 || exit $?; done
for v in base cb cbq cbqs qs; do run cfg1 $v r1 || exit $?; done
for v in prof cbprof; do
  LZGPU_LIB=$V/liblzmagpu_$v.so timeout -k 10 300 python -u bench.py --config cfg4 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-gather > $O/prof_cfg4_$v.json 2> $O/prof_cfg4_$v.err || exit $?
  echo "prof $v: $(grep PROF $O/prof_cfg4_$v.err | cut -c1-1500)"
done
