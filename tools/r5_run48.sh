# The fitted tile rule: parity tests, then the tile sweep again (auto against both forced tiles)
set -o pipefail
O=gpurun_out/r05; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gemm9 or gemm8 or wide or auto_tile or sibling or image" > $O/rule.tests.log 2>&1; rc=$?; tail -1 $O/rule.tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/g9_tile_sweep.py > $O/g9_tile_sweep2.jsonl 2> $O/g9_tile_sweep2.err
