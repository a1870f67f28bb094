set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r05/gputest1.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r05/gputest1.log
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/r05/bench1.json 2> gpurun_out/r05/bench1.err
echo "bench rc=$?"
tail -3 gpurun_out/r05/gputest1.log
