#!/bin/bash
# The one GPU-box runner (round 6; replaces the per-call scripts/r04/, r05/
# runners).  Run through gpurun from the repo root:
#   gpurun --timeout 1200 -- bash scripts/gpu.sh TAG STEP [STEP ...]
# Every step writes under gpurun_out/TAG/, runs under its own time limit, and
# the first failing step ends the call (no GPU work after a fault or timeout).
# Steps:
#   ab:CFGS:VARIANTS[:ROUNDS]  bench A/B: every config of CFGS (cfg2,cfg3,...)
#                              on every library of VARIANTS (base = the shipped
#                              lib/liblzmagpu.so, NAME = lib/variants/
#                              liblzmagpu_NAME.so from `make variants`),
#                              ROUNDS rounds (default 2), interleaved
#   suite[:VARIANT]            the GPU test suite (on a variant library)
#   bench[:ARGS]               the default bench line (ARGS: comma-separated
#                              extra bench.py arguments)
#   profile:CFG[:VARIANT]      kernel trace + separate PMC passes of CFG
#                              (scripts/profile.sh) -> TAG/prof_CFG
#   shares:CFG:S1,S2,...[:ENV] bench --streams S of CFG: one GPU's share of a
#                              strong-scaling run (ENV: K=V,K2=V2 planner
#                              variables for every run of the step)
#   pmci:CFG:VARIANTS          one PMC pass of instruction counters per
#                              library (SQ_INSTS_*, waves) -> TAG/pmci_CFG_V
#   smoke                      __graft_entry__.smoke()
#   coalesce                   the drop-in's concurrent-caller bench
#   fuzz:N[:VARIANT]           N LZMA (N/5 LZMA2) fuzz cases through every
#                              instantiation against the oracle
#                              (tests/test_gpu_kernels.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
L=lzma-sdk-zliblike_amd/lib
V=$L/variants
sha256sum $L/liblzmagpu.so $V/*.so > "$O/binary.sha256" 2>/dev/null
lib_of() {  # variant name -> LZGPU_LIB value ("" = the shipped library)
  if [ "$1" = base ] || [ -z "$1" ]; then echo ""; else echo "$V/liblzmagpu_$1.so"; fi
}
R0=$PWD
lib_abs() {  # the same as an absolute path (for runs from /tmp)
  if [ "$1" = base ] || [ -z "$1" ]; then echo ""; else echo "$R0/$V/liblzmagpu_$1.so"; fi
}
summ() {  # bench json -> one line
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'], d['ms_per_step'], d['verified'])" "$1"
}
BA0="--no-cpu-baseline --no-e2e --no-crc --no-secondary"
BA="--steps 5 --warmup 1 $BA0"
for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  case $kind in
    ab)
      rounds=${c:-2}
      for r in $(seq 1 "$rounds"); do
        for cfg in ${a//,/ }; do
          for v in ${b//,/ }; do
            f=$O/${cfg}_${v}_r$r.json
            LZGPU_LIB=$(lib_of "$v") timeout -k 10 300 python3 bench.py --config "$cfg" $BA \
              > "$f" 2>> "$O/ab.err" || exit $?
            echo "$cfg $v r$r: $(summ "$f")"
          done
        done
      done ;;
    suite)
      LZGPU_LIB=$(lib_of "$a") timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q \
        --timeout 120 --timeout-method thread > "$O/suite_${a:-base}.log" 2>&1
      s=$?; echo "suite ${a:-base} exit $s: $(tail -1 "$O/suite_${a:-base}.log")"; [ $s -eq 0 ] || exit $s ;;
    bench)
      timeout -k 10 600 python3 bench.py ${a//,/ } > "$O/bench_line.json" 2> "$O/bench.err" || exit $?
      echo "bench: $(python3 -c "import json;d=json.load(open('$O/bench_line.json'));print(d['value'], d['ms_per_step'], d['verified'], {k:(v['value'],v['verified']) for k,v in d.get('secondary',{}).items()})")" ;;
    profile)
      LZGPU_LIB=$(lib_abs "$b") bash scripts/profile.sh "$O/prof_$a" --config "$a" || exit $? ;;
    shares)
      for s in ${b//,/ }; do
        f=$O/share_${a}_$s${c:+_${c//[=,]/_}}.json
        env ${c//,/ } timeout -k 10 300 python3 bench.py --config "$a" --streams "$s" $BA > "$f" \
          2>> "$O/shares.err" || exit $?
        echo "$a share $s ${c}: $(summ "$f")"
      done ;;
    pmci)
      for v in ${b//,/ }; do
        d=$R0/$O/pmci_${a}_$v
        ( cd /tmp && export TMPDIR=/tmp && LZGPU_LIB=$(lib_abs "$v") timeout -s KILL 300 rocprofv3 --pmc \
            SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD \
            SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d "$d" -o pmc --output-format csv -- \
            python3 "$R0/bench.py" --config "$a" --steps 2 --warmup 0 $BA0 > "$d.json" 2> "$d.err" ) || exit $?
        echo "pmci $a $v: $(summ "$d.json")"
      done ;;
    smoke)
      timeout -k 10 400 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
      echo "smoke: $(tail -1 "$O/smoke.log")" ;;
    coalesce)
      timeout -k 10 600 python3 bench.py --config coalesce > "$O/coalesce.json" 2> "$O/coalesce.err" || exit $?
      echo "coalesce: $(head -c 400 "$O/coalesce.json")" ;;
    fuzz)
      LZGPU_LIB=$(lib_of "$b") LZGPU_FUZZ_CASES=$a LZGPU_FUZZ2_CASES=$((a / 5)) timeout -k 10 900 \
        python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k fuzz --timeout 800 \
        --timeout-method thread > "$O/fuzz_$a.log" 2>&1
      s=$?; echo "fuzz $a exit $s: $(tail -1 "$O/fuzz_$a.log")"; [ $s -eq 0 ] || exit $s ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG done"
