"""One rank of tests/test_dist.py::test_file_comm_ranks_drive_product_host_code (CPU, no torch, no GPU
work).  argv: rank world dir cases.json.  The rank loads libggml_hip.so and drives the product's
multi-rank host code in its own process: the file-rendezvous comm (ggml_hip_comm_init_file), its row
partition (ggml_hip_split_rows, the reference's tensor_split rule, ggml-cuda.cu:1874-1881,
2361-2368), and its host collectives (ggml_hip_comm_allgather_host, _allreduce_host).  The shard
product of its rows is the oracle's (the GPU kernels run in tests/test_gpu_split.py); the padded slabs
[N][max_rows] that the split path all-gathers are exchanged through the comm and compacted here as
k_scatter_slabs does, and y must equal the unsharded product bitwise."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "llama.cpp-q_4_0_amd", "python"), HERE,
                os.path.join(os.path.dirname(HERE), "oracle")]
import ggml_hip as gh  # noqa: E402
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402


def main():
    rank, world, cdir, cases_path = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    L = gh.load()
    comm = ctypes.c_void_p()
    gh.check(L.ggml_hip_comm_init_file(ctypes.byref(comm), world, rank, cdir.encode()), "comm_init_file")
    r_, n_ = ctypes.c_int(), ctypes.c_int()
    gh.check(L.ggml_hip_comm_rank(comm, ctypes.byref(r_), ctypes.byref(n_)))
    assert (r_.value, n_.value) == (rank, world)
    for K, M, N, fr, seed in json.load(open(cases_path)):
        rb = np.zeros(world + 1, np.int64)
        fa = np.asarray(fr, np.float32) if fr is not None else None
        gh.check(L.ggml_hip_split_rows(M, world, fa.ctypes.data_as(ctypes.c_void_p) if fa is not None else None,
                                       rb.ctypes.data_as(ctypes.c_void_p)))
        # every rank computed the same partition
        allrb = np.zeros((world, world + 1), np.int64)
        gh.check(L.ggml_hip_comm_allgather_host(comm, rb.ctypes.data_as(ctypes.c_void_p), rb.nbytes,
                                                allrb.ctypes.data_as(ctypes.c_void_p)))
        assert (allrb == rb).all(), allrb
        wq, _ = O.quantize_q4_0(O.gaussian(M * K, seed, 0.0, 0.02).reshape(M, K))
        x = O.gaussian(N * K, seed + 1, 0.0, 1.0).reshape(N, K)
        lo, hi = int(rb[rank]), int(rb[rank + 1])
        max_rows = int(np.diff(rb).max())
        slab = np.zeros((N, max_rows), np.float32)
        if hi > lo:
            slab[:, :hi - lo] = O.mul_mat(wq[lo:hi], K, x)
        slabs = np.zeros((world, N, max_rows), np.float32)
        gh.check(L.ggml_hip_comm_allgather_host(comm, slab.ctypes.data_as(ctypes.c_void_p), slab.nbytes,
                                                slabs.ctypes.data_as(ctypes.c_void_p)))
        y = np.empty((N, M), np.float32)
        for r in range(world):
            y[:, rb[r]:rb[r + 1]] = slabs[r, :, :rb[r + 1] - rb[r]]
        assert np.array_equal(y.view(np.uint32), O.mul_mat(wq, K, x).view(np.uint32)), (K, M, N, rb.tolist())
    vals = (ctypes.c_double * 3)(rank + 1.0, -rank, 10.0 * rank)
    for op, want in ((0, [sum(r + 1.0 for r in range(world)), -sum(range(world)), 10.0 * sum(range(world))]),
                     (1, [float(world), 0.0, 10.0 * (world - 1)]), (2, [1.0, -(world - 1.0), 0.0])):
        v = (ctypes.c_double * 3)(*vals)
        gh.check(L.ggml_hip_comm_allreduce_host(comm, v, 3, op))
        assert list(v) == want, (op, list(v), want)
    gh.check(L.ggml_hip_comm_destroy(comm))
    print(f"FILE_COMM_OK rank {rank}", flush=True)


if __name__ == "__main__":
    main()
