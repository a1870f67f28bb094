"""One rank of tests/test_gpu_split.py::test_split_rccl_multiprocess (RCCL transport, one process
per GPU) or ::test_split_p2p_ipc_two_processes (mode "ipc": the file-rendezvous comm,
ggml_hip_comm_init_file, with the direct-store P2P all-gather across processes, any number of ranks
per device: hipIpcGetMemHandle / hipIpcOpenMemHandle of the fine-grained landing buffers and the
system-scope flag protocol of p2p_gather.hip).  argv: rank world idfile [mode].  The backend is loaded
before anything else (no torch); in RCCL mode rank 0 writes the unique id to idfile, the others poll
for it; in ipc mode the comm's files live in idfile's directory.  Each rank runs
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
    mode = sys.argv[4] if len(sys.argv) > 4 else "rccl"
    L = gh.load()
    gh.check(L.ggml_hip_set_device(rank % L.ggml_hip_device_count()), "set_device")
    if mode == "ipc":
        return main_ipc(L, rank, world, os.path.dirname(idfile))
    if mode == "abort":
        return main_abort(L, rank, world, os.path.dirname(idfile))
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


def main_ipc(L, rank, world, cdir):
    comm = ctypes.c_void_p()
    gh.check(L.ggml_hip_comm_init_file(ctypes.byref(comm), world, rank, cdir.encode()), "comm_init_file")
    s = L.ggml_hip_stream_create()
    cases = [(4096, 1024, 1, None), (4096, 1000, 1, [0.3, 0.7]), (4096, 1024, 3, None), (4096, 1000, 40, [1.0, 2.0])]
    gh.check(L.ggml_hip_comm_enable_p2p(comm, max(N * M for _, M, N, _ in cases)), "enable_p2p (IPC)")
    nchecks = 0
    for (K, M, N, fr) in cases:
        fr = fr if fr is None or len(fr) == world else None
        wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED6100 + M + N, 0.0, 0.02).reshape(M, K))
        x = O.gaussian(N * K, 0x5EED7300 + N, 0.0, 1.0).reshape(N, K)
        rb = np.zeros(world + 1, np.int64)
        fa = np.asarray(fr, np.float32) if fr is not None else None
        gh.check(L.ggml_hip_split_rows(M, world, fa.ctypes.data_as(ctypes.c_void_p) if fa is not None else None,
                                       rb.ctypes.data_as(ctypes.c_void_p)))
        xd = gh.DeviceBuffer.from_array(x)
        expect = []
        for r in range(world):                 # every slice's product, computed alone on this device
            wd_r, yd_r = gh.DeviceBuffer.from_array(wq[rb[r]:rb[r + 1]]), gh.DeviceBuffer(N * int(rb[r + 1] - rb[r]) * 4)
            gh.mul_mat(wd_r, K, int(rb[r + 1] - rb[r]), xd, N, yd_r)
            expect.append(yd_r.download((N, int(rb[r + 1] - rb[r])), np.float32))
        expect = np.concatenate(expect, axis=1)
        wd = gh.DeviceBuffer.from_array(wq[rb[rank]:rb[rank + 1]])
        yd = gh.DeviceBuffer(N * M * 4)
        for it in range(5):                    # epochs cycle through both landing slots
            L.ggml_hip_memset(yd.ptr, 0x7F, yd.nbytes, s)
            gh.check(L.ggml_hip_mul_mat_q4_0_split(comm, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N,
                                                   yd.ptr, s), f"split (IPC P2P) {K}x{M} N={N} it {it}")
            got = yd.download((N, M), np.float32, stream=s)
            assert np.array_equal(got.view(np.uint32), expect.view(np.uint32)), (K, M, N, fr, it)
            nchecks += 1
        if N == 1 and fr is None:              # the oracle on the gathered rows (tests/parity.py bound)
            from parity import block_terms, check_y
            _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
            check_y(got, O.mul_mat(wq, K, x, nthreads=4), s_abs, 1e-3, 1e-6)
    st = L.ggml_hip_comm_p2p_status(comm)
    assert st == 0, f"p2p status {st}"
    L.ggml_hip_stream_destroy(s)
    gh.check(L.ggml_hip_comm_destroy(comm))
    print(f"P2P_IPC_OK rank {rank}/{world}: {nchecks} checks", flush=True)


def main_abort(L, rank, world, cdir):
    """Active failure propagation across processes: one good split, a barrier, then rank 0 aborts its comm
    0.3 s later while rank 1 runs the next split; rank 1's gather must be released by the notice."""
    comm = ctypes.c_void_p()
    gh.check(L.ggml_hip_comm_init_file(ctypes.byref(comm), world, rank, cdir.encode()), "comm_init_file")
    s = L.ggml_hip_stream_create()
    K, M, N = 4096, 1024, 1
    wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED6200, 0.0, 0.02).reshape(M, K))
    x = O.gaussian(N * K, 0x5EED7400, 0.0, 1.0).reshape(N, K)
    rb = np.array([M * r // world for r in range(world + 1)], np.int64)
    gh.check(L.ggml_hip_comm_enable_p2p(comm, N * M), "enable_p2p (IPC)")
    xd = gh.DeviceBuffer.from_array(x)
    wd = gh.DeviceBuffer.from_array(wq[rb[rank]:rb[rank + 1]])
    yd = gh.DeviceBuffer(N * M * 4)

    def split():
        return L.ggml_hip_mul_mat_q4_0_split(comm, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N, yd.ptr, s)
    gh.check(split(), "good split")
    gh.check(L.ggml_hip_stream_synchronize(s))
    assert L.ggml_hip_comm_p2p_status(comm) == 0
    own = yd.download((N, M), np.float32, stream=s)[:, rb[rank]:rb[rank + 1]].copy()
    v = (ctypes.c_double * 1)(0.0)
    gh.check(L.ggml_hip_comm_allreduce_host(comm, v, 1, 0), "barrier")
    if rank == 0:
        time.sleep(0.3)
        gh.check(L.ggml_hip_comm_abort(comm), "abort")
        assert split() == gh.ERR_COMM
        print("ABORT_OK rank 0 sent the notice", flush=True)
    else:
        L.ggml_hip_memset(yd.ptr, 0, yd.nbytes, s)
        t0 = time.time()
        gh.check(split(), "split after the peer's abort")
        gh.check(L.ggml_hip_stream_synchronize(s))
        waited = time.time() - t0
        got = yd.download((N, M), np.float32, stream=s)
        assert np.array_equal(got[:, rb[1]:rb[2]].view(np.uint32), own.view(np.uint32))
        assert np.all(np.isnan(got[:, rb[0]:rb[1]])), "rank 0's segment must read NaN"
        assert L.ggml_hip_comm_p2p_status(comm) & 1
        assert split() == gh.ERR_COMM
        assert waited < 2.0, f"rank 1 waited {waited:.3f} s (timeout 10 s): the notice did not release it"
        print(f"ABORT_OK rank 1 released after {waited:.3f} s (0.3 s abort delay, 10 s timeout)", flush=True)
    L.ggml_hip_stream_destroy(s)
    gh.check(L.ggml_hip_comm_destroy(comm))


if __name__ == "__main__":
    main()
