#!/bin/bash
# One parametrised GPU-box script for a round's checks (run from the repo root through gpurun);
# replaces the per-lease r04*/r05* scripts. Every GPU step has its own time limit and the first
# failure ends the script (set -e); outputs go under gpurun_out/<tag>/.
#
#   bash tools/gpu_round.sh tests  <tag> [pytest selection...]    -m gpu suite (+ smoke() when no selection)
#   bash tools/gpu_round.sh bench  <tag> <name> "<bench args>" [<name> "<bench args>" ...]
#   bash tools/gpu_round.sh ab     <tag> "<bench args>" <libA> <libB> [reps]
#                                  interleaved A/B of two built libraries (MPCCBF_LIB), reps x (A B)
#   bash tools/gpu_round.sh prof   <tag> <name> "<bench args>"    rocprofv3 --kernel-trace --stats
#   bash tools/gpu_round.sh stamps <tag> <lib> <agents> <steps> [variant]
#                                  phase stamps (tools/stamp_profile.py) with a stamps build
# Several commands can be chained with "--": bash tools/gpu_round.sh tests t -- ab t "..." a b
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
step() { echo "[$(date +%T)] $*"; }

run_one() {
  local cmd=$1 tag=$2
  shift 2
  local O=$ROOT/gpurun_out/$tag
  mkdir -p "$O"
  case "$cmd" in
    tests)
      if [ $# -eq 0 ]; then
        step pytest
        timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
          > "$O/pytest.log" 2>&1
        step smoke
        timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      else
        step pytest "$@"
        timeout -k 10 600 python3 -u -m pytest -m gpu -v -x --timeout 200 --timeout-method thread "$@" \
          > "$O/pytest_sel.log" 2>&1
      fi
      ;;
    bench)
      while [ $# -ge 2 ]; do
        step bench "$1" "$2"
        timeout -k 10 300 python3 bench.py $2 > "$O/$1.json" 2> "$O/$1.err"
        shift 2
      done
      ;;
    ab)
      local args=$1 la=$2 lb=$3 reps=${4:-2}
      for r in $(seq 1 "$reps"); do
        for v in a b; do
          local L=$la
          [ $v = b ] && L=$lb
          step ab $v $r
          MPCCBF_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > "$O/${v}_$r.json" 2> "$O/${v}_$r.err"
        done
      done
      ;;
    prof)
      local name=$1 args=$2
      step prof "$name"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/prof_$name" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline $args \
        > "$O/prof_$name.json" 2> "$O/prof_$name.err")
      ;;
    stamps)
      local lib=$1 n=$2 st=$3 var=${4:-0}
      step stamps "$lib" "$n" "$st" "$var"
      MPCCBF_LIB=$lib timeout -k 10 200 python3 -u tools/stamp_profile.py "$n" "$st" "$var" > "$O/stamps_$n.log" 2>&1
      ;;
    *)
      echo "unknown command $cmd" >&2
      exit 2
      ;;
  esac
}

# split the arguments at "--" into commands
cmd=()
for a in "$@"; do
  if [ "$a" = "--" ]; then
    run_one "${cmd[@]}"
    cmd=()
  else
    cmd+=("$a")
  fi
done
[ ${#cmd[@]} -gt 0 ] && run_one "${cmd[@]}"
step done
