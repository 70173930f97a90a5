#!/bin/bash
# One gpurun call: smoke -> gpu tests -> bench -> rocprof kernel trace.
# Each GPU step has its own time limit; the script stops at the first step that
# ends by a signal / timeout / abort (exit >= 124), never retries.
set -u
OUT=gpurun_out
mkdir -p $OUT
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-smoke,tests,bench,prof}
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
[[ $STEPS == *bench* ]] && run bench 600 python bench.py ${BENCH_ARGS:-}
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-}
exit 0
