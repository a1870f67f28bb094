# the tile sweep with every call streaming its weight image from HBM (COLD=1), mixed launches and small halves on
set -o pipefail
O=gpurun_out/r05; mkdir -p $O
COLD=1 NS="128 256 384 512 768 1024" timeout -k 10 900 python tools/g9_tile_sweep.py > $O/g9_tile_sweep_cold.jsonl 2> $O/g9_tile_sweep_cold.err
