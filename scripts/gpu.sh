#!/bin/bash
# One parameterised GPU-box wrapper (replaces the round-2 one-off r2_*.sh scripts).
# usage: bash scripts/gpu.sh TAG STEP [STEP ...]; every step writes gpurun_out/TAG_<step>.* and runs
# under its own time limit; the first failing step ends the call (no GPU work after a failure).
#   tests            python -m pytest tests -m gpu (thread timeout per test)
#   tests:EXPR       the same with -k EXPR (commas for spaces: tests:a,or,b)
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     python bench.py ARGS (comma-separated, e.g. bench:--config,5,--steps,2)
#   prof[:ARGS]      rocprofv3 --kernel-trace --stats of bench.py ARGS (--steps 3 --warmup 1 by default)
#   bin:PROGRAM[:ARGS] a built program (e.g. scripts/mfma_round_probe)
#   env:NAME=VALUE   export NAME=VALUE for the steps after it (env:NAME= unsets it)
#   ab:MODE,ROUNDS,LIB1,LIB2,...  scripts/ab.sh (same-box A/B of library variants)
#   py:SCRIPT[:ARGS] python SCRIPT ARGS
#   kprof:SCRIPT[:ARGS] rocprofv3 --kernel-trace --stats of python3 SCRIPT ARGS
#   pmc[:ARGS]       scripts/pmc_passes.sh over scripts/pmc_target.py ARGS
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
n=0
for step in "$@"; do
  n=$((n+1))
  name=${step%%:*}; arg=""; [[ "$step" == *:* ]] && arg=${step#*:}
  IFS=',' read -r -a A <<< "$arg"
  out=gpurun_out/${TAG}_${n}_${name}
  echo "[$(date +%T)] step $n: $step" >&2
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "${arg//,/ }")   # commas stand for spaces: tests:a,or,b -> -k "a or b"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "${K[@]}" > $out.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out.log 2>&1 ;;
    bench)
      timeout -k 10 600 python bench.py "${A[@]}" > $out.json 2> $out.err ;;
    prof)
      [ ${#A[@]} -eq 0 ] && A=(--steps 3 --warmup 1 --no-cpu-baseline)
      rm -rf $out
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- python3 bench.py "${A[@]}" > $out.log 2>&1 ;;
    bin)
      s=${A[0]}; timeout -k 10 120 $s "${A[@]:1}" > $out.out 2> $out.err ;;
    env)
      k=${arg%%=*}; v=${arg#*=}
      if [ -n "$v" ]; then export "$k=$v"; else unset "$k"; fi
      true ;;
    ab)
      timeout -k 10 900 bash scripts/ab.sh "${A[@]}" > $out.log 2>&1 ;;
    py)
      s=${A[0]}; timeout -k 10 600 python -u $s "${A[@]:1}" > $out.out 2> $out.err ;;
    kprof)
      s=${A[0]}; rm -rf $out
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- python3 $s "${A[@]:1}" > $out.log 2>&1 ;;
    pmc)
      bash scripts/pmc_passes.sh $out "${A[@]}" > $out.log 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
  rc=$?
  echo "[$(date +%T)] step $n rc=$rc" >&2
  [ $rc -ne 0 ] && exit $rc
done
exit 0
