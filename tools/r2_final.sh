#!/bin/bash
# round 2 end: whole -m gpu suite, default bench line, rocprofv3 kernel stats of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/final
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench.err
rc=$?; cat $O/bench_line.json; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-extra > $O/bench_under_rocprof.json 2> $O/bench_prof.err
rc=$?; [ $rc = 0 ] || exit $rc
cd $R && python3 tools/trace_summary.py $(ls $O/prof/run_kernel_trace.csv $O/prof/*/run_kernel_trace.csv 2>/dev/null | head -1) > $O/trace_summary.txt 2>&1 || true
