"""One rank of tests/test_gpu_split.py::test_split_rccl_multiprocess (RCCL transport, one process
per GPU).  argv: rank world idfile.  The backend is loaded before anything else (no torch), rank 0
writes the RCCL unique id to idfile, the others poll for it.  Each rank runs
ggml_hip_mul_mat_q4_0_split / _split_multi on the LLaMA-13B shapes (equal and uneven splits) and
compares its gathered y_full bitwise against the concatenation of the per-slice products, which it
computes itself on its own device (every rank knows every slice's weights: same seeds)."""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "llama.cpp-q_4_0_amd", "python"), HERE,
                os.path.join(os.path.dirname(HERE), "oracle")]
import ggml_hip as gh  # noqa: E402  (loads libggml_hip.so + /opt/rocm's librccl first)
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402


def main():
    rank, world, idfile = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    L = gh.load()
    gh.check(L.ggml_hip_set_device(rank % L.ggml_hip_device_count()), "set_device")
    uid = ctypes.create_string_buffer(128)
    if rank == 0:
        gh.check(L.ggml_hip_comm_unique_id(uid))
        with open(idfile + ".tmp", "wb") as f:
            f.write(uid.raw)
        os.replace(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile):
            if time.time() - t0 > 120:
                raise SystemExit("no unique id")
            time.sleep(0.05)
        uid = ctypes.create_string_buffer(open(idfile, "rb").read(), 128)
    comm = ctypes.c_void_p()
    gh.check(L.ggml_hip_comm_init(ctypes.byref(comm), world, rank, uid), "comm_init")
    s = L.ggml_hip_default_stream()

    def slice_products(wq, rb, K, x):
        N = x.shape[0]
        xd = gh.DeviceBuffer.from_array(x)
        outs = []
        for r in range(world):
            w = wq[rb[r]:rb[r + 1]]
            if len(w) == 0:
                outs.append(np.zeros((N, 0), np.float32))
                continue
            wd, yd = gh.DeviceBuffer.from_array(w), gh.DeviceBuffer(N * len(w) * 4)
            gh.mul_mat(wd, K, len(w), xd, N, yd)
            outs.append(yd.download((N, len(w)), np.float32))
        return np.concatenate(outs, axis=1)

    def rows(M, fr):
        rb = np.zeros(world + 1, np.int64)
        fp = None
        if fr is not None:
            fa = np.asarray(fr, np.float32)
            fp = fa.ctypes.data_as(ctypes.c_void_p)
        gh.check(L.ggml_hip_split_rows(M, world, fp, rb.ctypes.data_as(ctypes.c_void_p)))
        return rb

    uneven = [1.0 + (r % 3) for r in range(world)]
    nchecks = 0
    for (K, M, N, fr) in [(5120, 5120, 1, None), (5120, 13824, 1, None), (13824, 5120, 1, None),
                          (5120, 5120, 3, None), (5120, 5120, 1, uneven), (4096, 1000, 40, uneven)]:
        wf = O.gaussian(M * K, 0x5EED6000 + K + M, 0.0, 0.02).reshape(M, K)
        wq, _ = O.quantize_q4_0(wf)
        x = O.gaussian(N * K, 0x5EED7000 + N, 0.0, 1.0).reshape(N, K)
        rb = rows(M, fr)
        expect = slice_products(wq, rb, K, x)
        mine = wq[rb[rank]:rb[rank + 1]]
        wd = gh.DeviceBuffer.from_array(mine) if len(mine) else gh.DeviceBuffer(16)
        xd, yd = gh.DeviceBuffer.from_array(x), gh.DeviceBuffer(N * M * 4)
        gh.check(L.ggml_hip_mul_mat_q4_0_split(comm, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N,
                                               yd.ptr, s), "split")
        got = yd.download((N, M), np.float32, stream=s)
        assert np.array_equal(got.view(np.uint32), expect.view(np.uint32)), (K, M, N, fr)
        nchecks += 1
    # siblings: wq|wk|wv of 13B, one GEMV launch + one grouped all-gather
    K, Ms = 5120, (5120, 5120, 5120)
    x = O.gaussian(K, 0x5EED7100, 0.0, 1.0).reshape(1, K)
    xd = gh.DeviceBuffer.from_array(x)
    rbs = [rows(M, None) for M in Ms]
    ws = [O.quantize_q4_0(O.gaussian(M * K, 0x5EED7200 + i, 0.0, 0.02).reshape(M, K))[0] for i, M in enumerate(Ms)]
    expects = [slice_products(w, rb, K, x) for w, rb in zip(ws, rbs)]
    wds = [gh.DeviceBuffer.from_array(w[rb[rank]:rb[rank + 1]]) for w, rb in zip(ws, rbs)]
    yds = [gh.DeviceBuffer(M * 4) for M in Ms]
    n = len(Ms)
    gh.check(L.ggml_hip_mul_mat_q4_0_split_multi(comm, n, (ctypes.c_void_p * n)(*[w.ptr for w in wds]),
                                                 (ctypes.c_int64 * n)(*Ms),
                                                 (ctypes.c_void_p * n)(*[rb.ctypes.data for rb in rbs]), K, xd.ptr, 1,
                                                 (ctypes.c_void_p * n)(*[y.ptr for y in yds]), s), "split_multi")
    for y, e, M in zip(yds, expects, Ms):
        got = y.download((1, M), np.float32, stream=s)
        assert np.array_equal(got.view(np.uint32), e.view(np.uint32))
        nchecks += 1
    gh.check(L.ggml_hip_comm_destroy(comm))
    print(f"SPLIT_OK rank {rank}/{world}: {nchecks} checks", flush=True)


if __name__ == "__main__":
    main()
