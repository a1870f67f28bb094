"""One gloo rank of tests/test_dist.py (CPU, torch.distributed).  argv: rank world port cases.json.
This process imports torch but never loads libggml_hip.so (a second HIP runtime next to torch's
bundled one corrupts a process); the row partitions come precomputed from the parent, which got
them from the library's ggml_hip_split_rows."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(os.path.dirname(HERE), "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle as O  # noqa: E402


def main():
    rank, world, port, cases_path = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cases = json.load(open(cases_path))
    for K, M, N, rb, seed in cases:
        rb = np.asarray(rb, np.int64)
        wf = O.gaussian(M * K, seed, 0.0, 0.02).reshape(M, K)
        wq, _ = O.quantize_q4_0(wf)
        x = O.gaussian(N * K, seed + 1, 0.0, 1.0).reshape(N, K)
        lo, hi = int(rb[rank]), int(rb[rank + 1])
        max_rows = int(np.diff(rb).max())
        slab = np.zeros((N, max_rows), np.float32)                 # padded send slab [N][max_rows]
        if hi > lo:
            slab[:, :hi - lo] = O.mul_mat(wq[lo:hi], K, x)
        gathered = [torch.zeros(N, max_rows) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(slab))
        y = np.empty((N, M), np.float32)                           # compaction (k_scatter_slabs)
        for r in range(world):
            rows = int(rb[r + 1] - rb[r])
            y[:, rb[r]:rb[r] + rows] = gathered[r].numpy()[:, :rows]
        y_full = O.mul_mat(wq, K, x)
        assert np.array_equal(y.view(np.uint32), y_full.view(np.uint32)), (K, M, N, rb.tolist())
    dist.barrier()
    dist.destroy_process_group()
    print(f"DIST_OK rank {rank}", flush=True)


if __name__ == "__main__":
    main()
