#!/bin/bash
# exact-mode (algo 4) per-launch time (quantize + exact kernel) vs N, tools/shape_sweep.py graph replay
set -e
ALGO=4 timeout -k 10 120 python tools/shape_sweep.py 4096:4096 4096:11008 11008:4096 4544:4672 4544:18176 18176:4544 2>&1 | grep '^{'
for n in 2 4 8 40 512; do
  ALGO=4 NTOK=$n timeout -k 10 200 python tools/shape_sweep.py 4096:4096 2>&1 | grep '^{'
done
