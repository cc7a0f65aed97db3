#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel trace. Each GPU step has its
# own time limit; a step only runs if the previous one ended normally (exit 0 or 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-smoke,pytest,bench,prof}
rc=0
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
}
case ",$STEPS," in *,smoke,*) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()";; esac
if [ $rc -le 1 ]; then case ",$STEPS," in *,pytest,*) run pytest_gpu 1100 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS};; esac; fi
if [ $rc -le 1 ]; then case ",$STEPS," in *,bench,*) run bench 600 python bench.py ${BENCH_ARGS};; esac; fi
if [ $rc -le 1 ]; then case ",$STEPS," in *,prof,*)
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o rx -- python3 "$R/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1
  if [ $rc -le 1 ]; then
    run prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof5" -o rx -- python3 "$R/bench.py" --config 5 --steps 50 --warmup 5 --no-cpu-baseline --no-extra --no-scale --no-strong --pipeline 1
  fi
;; esac; fi
exit $rc
