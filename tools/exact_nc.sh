#!/bin/bash
# exact-mode columns-per-workgroup choice at larger N
set -e
for n in 8 40 512; do for nc in 1 2 4 8; do
  GGML_HIP_EXACT_NC=$nc ALGO=4 NTOK=$n timeout -k 10 200 python tools/shape_sweep.py 4096:4096 2>&1 | grep '^{' | sed "s/^/nc=$nc /"
done; done
