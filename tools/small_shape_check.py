"""Per-algorithm error against the oracle at small K / M (the tiny GGJT model's shapes) over the N
range where the auto policy switches kernels.  Prints max |y - y_oracle| / max |y_oracle|.
Usage (GPU box): python tools/small_shape_check.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from test_gpu_parity import gpu_mul_mat, make_case  # noqa: E402

for K, M in [(256, 256), (256, 768), (768, 256), (256, 320), (4096, 4096)]:
    for N in [1, 8, 9, 32, 40, 64, 128, 129]:
        wq, x = make_case(K, M, N, seed=K * 7 + M + N)
        ref = O.mul_mat(wq, K, x)
        row = {"K": K, "M": M, "N": N}
        for algo in [0, 1, 2, 3]:
            if algo == 1 and N > 8:
                continue
            y, _ = gpu_mul_mat(wq, K, x, algo=algo)
            row[f"a{algo}"] = float(np.abs(y - ref).max() / np.abs(ref).max())
        print(json.dumps(row), flush=True)
