#!/bin/bash
# One gpurun call: GPU parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
    if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
    return $rc
}
export PYTHONUNBUFFERED=1
STEPS=${STEPS:-pytest,smoke,bench,prof}
[[ $STEPS == *pytest* ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
[[ $STEPS == *smoke* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* ]] && step bench 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-}
if [[ $STEPS == *prof* ]]; then
    export TMPDIR=/tmp
    step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extra ${BENCH_ARGS:-}
    find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
exit 0
