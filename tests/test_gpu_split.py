"""Multi-GPU row split (BASELINE config 4) through the product's own split code.

* LLaMA-13B per-rank shard shapes of the 8-way split (K=5120 -> M/8 = 640 / 1728, K=13824 -> 640)
  against the oracle, decode and small/large batches.
* R = 2..8 ranks through ggml_hip_mul_mat_q4_0_split / _split_multi on ONE device: the
  in-process loopback transport (ggml_hip_comm_init_local, one host thread per rank, each on its
  own stream) has ncclAllGather's semantics, so the partition, the in-place gather, the padded
  slabs and the compaction kernel (k_scatter_slabs) run exactly as on 8 GPUs, with equal and
  uneven (reference tensor_split, ggml-cuda.cu:1863-1882) partitions.  Every rank's y_full must
  equal, bitwise, the concatenation of the per-slice products computed alone.
* The RCCL transport with one process per GPU (skipped below 2 visible devices): tests/
  split_worker.py ranks, unique id through a file, no torch import.
"""
import ctypes
import os
import subprocess
import sys
import tempfile
import threading

import numpy as np
import pytest

import oracle as O
from hip_env import ggml_hip, gpu_available
from parity import block_terms, check_y

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer
RTOL, ATOL_BLOCKS = 1e-3, 1e-6
HERE = os.path.dirname(os.path.abspath(__file__))


def make_case(K, M, N, seed):
    wf = O.gaussian(M * K, 0x5EED3000 + seed, 0.0, 0.02).reshape(M, K)
    wq, _ = O.quantize_q4_0(wf)
    x = O.gaussian(N * K, 0x5EED4000 + seed, 0.0, 1.0).reshape(N, K)
    return wq, x


def split_rows(M, R, fractions=None):
    L = ggml_hip.load()
    rb = np.zeros(R + 1, np.int64)
    fp = None
    if fractions is not None:
        fr = np.asarray(fractions, np.float32)
        fp = fr.ctypes.data_as(ctypes.c_void_p)
    ggml_hip.check(L.ggml_hip_split_rows(M, R, fp, rb.ctypes.data_as(ctypes.c_void_p)))
    return rb


def gpu_y(wq, K, x):
    N, M = x.shape[0], wq.shape[0]
    wd, xd, yd = DB.from_array(wq), DB.from_array(x), DB(max(N * M, 1) * 4)
    ggml_hip.mul_mat(wd, K, M, xd, N, yd)
    return yd.download((N, M), np.float32)


# ------------------------------------------------------------------ 13B per-rank shard shapes
@pytest.mark.parametrize("K,M", [(5120, 640), (5120, 1728), (13824, 640)])
@pytest.mark.parametrize("N", [1, 3, 64])
def test_llama13b_shard_shapes(K, M, N):
    """One rank's slice of the LLaMA-13B 8-way split (wq/wk/wv/wo 5120/8, w1/w3 13824/8, w2 at
    K=13824): y within the parity bound of the oracle (ggml.c:11226-11424 semantics)."""
    wq, x = make_case(K, M, N, seed=K + M + N)
    y = gpu_y(wq, K, x)
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
    check_y(y, O.mul_mat(wq, K, x, nthreads=8), s_abs, RTOL, ATOL_BLOCKS)


# ------------------------------------------------------------------ R ranks, loopback transport
def run_ranks(R, fn):
    """fn(rank, comm, stream) in R threads (ctypes releases the GIL); re-raises the first error."""
    L = ggml_hip.load()
    comms = (ctypes.c_void_p * R)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, R, None), "comm_init_local")
    streams = [L.ggml_hip_stream_create() for _ in range(R)]
    errs = [None] * R
    out = [None] * R

    def body(r):
        try:
            out[r] = fn(r, ctypes.c_void_p(comms[r]), streams[r])
            ggml_hip.check(L.ggml_hip_stream_synchronize(streams[r]))
        except BaseException as e:           # noqa: BLE001 - reported below
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    alive = any(t.is_alive() for t in th)
    for s in streams:
        L.ggml_hip_stream_destroy(s)
    for r in range(R):
        L.ggml_hip_comm_destroy(ctypes.c_void_p(comms[r]))
    assert not alive, "a rank thread hung"
    for e in errs:
        if e is not None:
            raise e
    return out


FRACTIONS = {2: [0.3, 0.7], 3: [1.0, 2.0, 1.0], 4: [0.1, 0.2, 0.3, 0.4],
             8: [1.0, 1.0, 2.0, 0.5, 0.5, 1.0, 3.0, 1.0]}


@pytest.mark.parametrize("R", [2, 3, 4, 8])
@pytest.mark.parametrize("uneven", [False, True])
@pytest.mark.parametrize("N", [1, 3, 40])
def test_split_loopback_ranks(R, uneven, N):
    """ggml_hip_mul_mat_q4_0_split at R ranks: equal N=1 takes the in-place all-gather, the rest the
    padded slabs + k_scatter_slabs.  y_full on EVERY rank == concat of the slice products, bitwise."""
    if uneven and R not in FRACTIONS:
        pytest.skip("no uneven split for this R")
    K, M = 4096, 1000 if uneven else 1024
    wq, x = make_case(K, M, N, seed=100 * R + N + uneven)
    rb = split_rows(M, R, FRACTIONS[R] if uneven else None)
    assert rb[0] == 0 and rb[-1] == M and np.all(np.diff(rb) >= 0)
    slices = [wq[rb[r]:rb[r + 1]] for r in range(R)]
    expect = np.concatenate([gpu_y(s, K, x) if len(s) else np.zeros((N, 0), np.float32) for s in slices], axis=1)
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wds = [DB.from_array(s) if len(s) else DB(16) for s in slices]
    yds = [DB(N * M * 4) for _ in range(R)]
    for y in yds:
        L.ggml_hip_memset(y.ptr, 0x7F, y.nbytes, None)
    ggml_hip.synchronize()

    def rank(r, comm, stream):
        ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split(comm, wds[r].ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p),
                                                     xd.ptr, N, yds[r].ptr, stream), f"split rank {r}")

    run_ranks(R, rank)
    for r in range(R):
        got = yds[r].download((N, M), np.float32)
        assert np.array_equal(got.view(np.uint32), expect.view(np.uint32)), f"rank {r}"
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
    check_y(expect, O.mul_mat(wq, K, x, nthreads=8), s_abs, RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("R", [2, 4, 8])
@pytest.mark.parametrize("N,Ms,uneven", [(1, (5120, 5120, 5120), False), (1, (13824, 13824), False),
                                         (1, (4096, 1000), True), (3, (1024, 2048), False)])
def test_split_multi_loopback_ranks(R, N, Ms, uneven):
    """Sibling form (one multi-matrix GEMV + one grouped all-gather per rank; per-matrix split
    otherwise), 13B QKV / w1|w3 shard shapes at R=8: every rank's outputs == per-slice products."""
    K = 5120 if Ms[0] in (5120, 13824) else 4096
    n = len(Ms)
    x = O.gaussian(N * K, 0x5EED5000 + R + N, 0.0, 1.0).reshape(N, K)
    fr = FRACTIONS.get(R) if uneven else None
    rbs = [split_rows(M, R, fr) for M in Ms]
    ws = [make_case(K, M, 1, seed=7 * i + R)[0] for i, M in enumerate(Ms)]
    expect = []
    for w, rb in zip(ws, rbs):
        expect.append(np.concatenate([gpu_y(w[rb[r]:rb[r + 1]], K, x) for r in range(R)], axis=1))
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wds = [[DB.from_array(w[rb[r]:rb[r + 1]]) for w, rb in zip(ws, rbs)] for r in range(R)]
    yds = [[DB(N * M * 4) for M in Ms] for _ in range(R)]
    ggml_hip.synchronize()
    mt = (ctypes.c_int64 * n)(*Ms)
    rp = (ctypes.c_void_p * n)(*[rb.ctypes.data for rb in rbs])

    def rank(r, comm, stream):
        wp = (ctypes.c_void_p * n)(*[w.ptr for w in wds[r]])
        yp = (ctypes.c_void_p * n)(*[y.ptr for y in yds[r]])
        ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split_multi(comm, n, wp, mt, rp, K, xd.ptr, N, yp, stream),
                       f"split_multi rank {r}")

    run_ranks(R, rank)
    for r in range(R):
        for i, M in enumerate(Ms):
            got = yds[r][i].download((N, M), np.float32)
            assert np.array_equal(got.view(np.uint32), expect[i].view(np.uint32)), (r, i)
    xq = O.quantize_q8_0(x, "avx2")             # and the gathered product against the oracle
    for w, e in zip(ws, expect):
        _, s_abs = block_terms(w, xq, K)
        check_y(e, O.mul_mat(w, K, x, nthreads=8), s_abs, RTOL, ATOL_BLOCKS)


def test_split_slab_path_graph_capture():
    """A split call on the padded-slab path captured in a HIP graph (the bench's form) replays the
    same gather: the compaction kernel takes row_begin by value, nothing host-side is read at
    replay.  (Loopback ranks need a host thread each, so the capture runs one rank.)"""
    K, M, N = 4096, 1000, 3
    wq, x = make_case(K, M, N, seed=9)
    expect = gpu_y(wq, K, x)
    L = ggml_hip.load()
    xd, wd, y = DB.from_array(x), DB.from_array(wq), DB(N * M * 4)
    comms = (ctypes.c_void_p * 1)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, 1, None))
    comm = ctypes.c_void_p(comms[0])
    s = L.ggml_hip_stream_create()
    rb = np.array([0, M], np.int64)
    try:
        def call():
            ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split(comm, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p),
                                                         xd.ptr, N, y.ptr, s), "split")
        call()                                   # grows the slab outside capture
        g = ggml_hip.Graph(s)
        with g:
            call()
        L.ggml_hip_memset(y.ptr, 0, y.nbytes, s)
        g.launch()
        got = y.download((N, M), np.float32, stream=s)
        assert np.array_equal(got.view(np.uint32), expect.view(np.uint32))
    finally:
        L.ggml_hip_stream_destroy(s)
        L.ggml_hip_comm_destroy(comm)


# ------------------------------------------------------------------ RCCL, one process per GPU
def _device_count_subprocess():
    code = ("import sys; sys.path.insert(0, %r); import ggml_hip; print(ggml_hip.load().ggml_hip_device_count())"
            % os.path.join(os.path.dirname(HERE), "llama.cpp-q_4_0_amd", "python"))
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        return int(out.stdout.strip().splitlines()[-1])
    except Exception:
        return 0


@pytest.mark.parametrize("R", [2, 4, 8])
def test_split_rccl_multiprocess(R):
    """RCCL transport: R processes (tests/split_worker.py), one GPU each; every rank runs split and
    split_multi (13B shard shapes, equal and uneven) and checks itself against the unsharded
    per-slice products it computes locally; unique id via a file."""
    ndev = _device_count_subprocess()
    if ndev < R:
        pytest.skip(f"needs {R} visible devices (have {ndev})")
    with tempfile.TemporaryDirectory() as td:
        idfile = os.path.join(td, "uid")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "split_worker.py"), str(r), str(R), idfile],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                 for r in range(R)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=240)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        for r, (p, o) in enumerate(zip(procs, outs)):
            assert p.returncode == 0, f"rank {r} failed:\n{o[-3000:]}"
            assert "SPLIT_OK" in o, o[-2000:]


# ------------------------------------------------------------------ direct-store (P2P) all-gather
@pytest.mark.parametrize("R", [2])
@pytest.mark.parametrize("N,uneven", [(1, False), (1, True), (3, False), (40, True)])
def test_split_p2p_loopback_ranks(R, N, uneven):
    """ggml_hip_comm_enable_p2p: the same split calls with the all-gather done by direct stores into
    the peers' landing buffers + flags (p2p_gather.hip) instead of copies; repeated calls cycle the
    device-side epoch through both landing slots.  Every rank's y_full == the slice products, bitwise,
    and no peer wait timed out.  (The ranks share one device: their waiting gathers must run
    concurrently, so each rank's stream needs its own hardware queue; the product allows at most 2
    loopback ranks per device for P2P, test_p2p_api_errors.)"""
    K, M = 4096, 1000 if uneven else 1024
    wq, x = make_case(K, M, N, seed=300 * R + N + uneven)
    rb = split_rows(M, R, FRACTIONS[R] if uneven else None)
    slices = [wq[rb[r]:rb[r + 1]] for r in range(R)]
    expect = np.concatenate([gpu_y(s, K, x) for s in slices], axis=1)
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wds = [DB.from_array(s) for s in slices]
    yds = [DB(N * M * 4) for _ in range(R)]
    ggml_hip.synchronize()

    def rank(r, comm, stream):
        ggml_hip.check(L.ggml_hip_comm_enable_p2p(comm, N * M), f"enable_p2p rank {r}")
        for it in range(7):
            L.ggml_hip_memset(yds[r].ptr, 0x7F, yds[r].nbytes, stream)
            ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split(comm, wds[r].ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p),
                                                         xd.ptr, N, yds[r].ptr, stream), f"split rank {r}")
        return L.ggml_hip_comm_p2p_status(comm)

    status = run_ranks(R, rank)
    assert status == [0] * R, status
    for r in range(R):
        got = yds[r].download((N, M), np.float32)
        assert np.array_equal(got.view(np.uint32), expect.view(np.uint32)), f"rank {r}"


@pytest.mark.parametrize("R", [2])
def test_split_multi_p2p_graph_replay(R):
    """Sibling group (one GEMV + one all-gather per matrix) over P2P stores, captured in a HIP graph on
    every rank and replayed: the epoch advances on the device, so replays keep alternating slots."""
    K, N, Ms = 4096, 1, (1024, 2048, 512)
    n = len(Ms)
    x = O.gaussian(N * K, 0x5EED5100 + R, 0.0, 1.0).reshape(N, K)
    rbs = [split_rows(M, R) for M in Ms]
    ws = [make_case(K, M, 1, seed=17 * i + R)[0] for i, M in enumerate(Ms)]
    expect = [np.concatenate([gpu_y(w[rb[r]:rb[r + 1]], K, x) for r in range(R)], axis=1) for w, rb in zip(ws, rbs)]
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wds = [[DB.from_array(w[rb[r]:rb[r + 1]]) for w, rb in zip(ws, rbs)] for r in range(R)]
    yds = [[DB(N * M * 4) for M in Ms] for _ in range(R)]
    ggml_hip.synchronize()
    mt = (ctypes.c_int64 * n)(*Ms)
    rp = (ctypes.c_void_p * n)(*[rb.ctypes.data for rb in rbs])

    def rank(r, comm, stream):
        ggml_hip.check(L.ggml_hip_comm_enable_p2p(comm, max(Ms)), f"enable_p2p rank {r}")
        wp = (ctypes.c_void_p * n)(*[w.ptr for w in wds[r]])
        yp = (ctypes.c_void_p * n)(*[y.ptr for y in yds[r]])

        def call():
            ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split_multi(comm, n, wp, mt, rp, K, xd.ptr, N, yp, stream),
                           f"split_multi rank {r}")
        call()
        g = ggml_hip.Graph(stream)
        with g:
            call()
        for _ in range(4):
            for y in yds[r]:
                L.ggml_hip_memset(y.ptr, 0, y.nbytes, stream)
            g.launch()
        ggml_hip.check(L.ggml_hip_stream_synchronize(stream))
        del g
        return L.ggml_hip_comm_p2p_status(comm)

    status = run_ranks(R, rank)
    assert status == [0] * R, status
    for r in range(R):
        for i, M in enumerate(Ms):
            got = yds[r][i].download((N, M), np.float32)
            assert np.array_equal(got.view(np.uint32), expect[i].view(np.uint32)), (r, i)


def test_split_p2p_ipc_two_processes_one_gpu():
    """The cross-process P2P path on one MI355X: two fresh processes (tests/split_worker.py, mode ipc)
    share device 0 through the file-rendezvous comm (RCCL refuses two ranks on one device), exchange
    IPC handles of their fine-grained landing buffers (hipIpcGetMemHandle / hipIpcOpenMemHandle) and
    run split mul_mats whose all-gather is the direct-store kernel with system-scope flags across the
    process boundary: y_full bitwise the per-slice products (equal / uneven partitions, N = 1 / 3 / 40,
    five epochs each), the oracle bound on the gathered rows, no peer wait timed out."""
    R = 2
    with tempfile.TemporaryDirectory() as td:
        idfile = os.path.join(td, "uid")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "split_worker.py"), str(r), str(R), idfile, "ipc"],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                 for r in range(R)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=100)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        for r, (p, o) in enumerate(zip(procs, outs)):
            assert p.returncode == 0, f"rank {r} failed:\n{o[-3000:]}"
            assert "P2P_IPC_OK" in o, o[-2000:]


def test_p2p_timeout_fails_the_comm():
    """A peer that never gathers: the waiting rank's gather gives up after the timeout, writes NaN into
    that peer's segment (never the stale landing slot), marks the comm failed (p2p_status bit), and the
    NEXT split call returns GGML_HIP_ERR_COMM before enqueueing anything; a later gather does not wait."""
    import time
    K, M, N = 4096, 1024, 1
    wq, x = make_case(K, M, N, seed=77)
    rb = split_rows(M, 2)
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wd = DB.from_array(wq[rb[0]:rb[1]])
    y = DB(N * M * 4)
    comms = (ctypes.c_void_p * 2)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, 2, None))
    c0, c1 = ctypes.c_void_p(comms[0]), ctypes.c_void_p(comms[1])
    s = L.ggml_hip_stream_create()
    try:
        th = threading.Thread(target=lambda: ggml_hip.check(L.ggml_hip_comm_enable_p2p(c1, N * M)))
        th.start()
        ggml_hip.check(L.ggml_hip_comm_enable_p2p(c0, N * M))
        th.join(timeout=60)
        ggml_hip.check(L.ggml_hip_comm_set_p2p_timeout(c0, 200.0))
        L.ggml_hip_memset(y.ptr, 0, y.nbytes, s)
        t0 = time.time()
        ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split(c0, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr,
                                                     N, y.ptr, s), "first split (rank 1 never gathers)")
        ggml_hip.check(L.ggml_hip_stream_synchronize(s))
        waited = time.time() - t0
        assert L.ggml_hip_comm_p2p_status(c0) == 1 << 1            # peer 1's data never arrived
        got = y.download((N, M), np.float32, stream=s)
        own = gpu_y(wq[rb[0]:rb[1]], K, x)
        assert np.array_equal(got[:, rb[0]:rb[1]].view(np.uint32), own.view(np.uint32))
        assert np.all(np.isnan(got[:, rb[1]:rb[2]])), "a timed-out peer segment must read NaN, not a stale slot"
        assert 0.15 < waited < 30, waited
        rc = L.ggml_hip_mul_mat_q4_0_split(c0, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N, y.ptr, s)
        assert rc == ggml_hip.ERR_COMM, rc                         # the comm is failed: error, nothing enqueued
        assert L.ggml_hip_comm_p2p_status(c0) == 1 << 1            # sticky
    finally:
        L.ggml_hip_stream_destroy(s)
        L.ggml_hip_comm_destroy(c0)
        L.ggml_hip_comm_destroy(c1)


def test_p2p_abort_notifies_a_waiting_peer():
    """Verdict r4 item 4: a failure propagates actively.  Rank 1's gather is already waiting for rank 0's
    data (default 10 s timeout) when rank 0 aborts (ggml_hip_comm_abort: bit 0 stored into rank 1's control
    block over the P2P mapping); rank 1's wait polls that word, so its launch ends within one poll, not
    after its own timeout: own rows bitwise, rank 0's segment NaN (never the stale slot), p2p_status names
    rank 0, and the next split call on either rank returns GGML_HIP_ERR_COMM."""
    import time
    K, M, N = 4096, 1024, 1
    wq, x = make_case(K, M, N, seed=78)
    rb = split_rows(M, 2)
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wds = [DB.from_array(wq[rb[r]:rb[r + 1]]) for r in range(2)]
    y = DB(N * M * 4)
    own = gpu_y(wq[rb[1]:rb[2]], K, x)
    comms = (ctypes.c_void_p * 2)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, 2, None))
    c0, c1 = ctypes.c_void_p(comms[0]), ctypes.c_void_p(comms[1])
    s = L.ggml_hip_stream_create()
    out = {}
    try:
        th = threading.Thread(target=lambda: ggml_hip.check(L.ggml_hip_comm_enable_p2p(c1, N * M)))
        th.start()
        ggml_hip.check(L.ggml_hip_comm_enable_p2p(c0, N * M))
        th.join(timeout=60)
        L.ggml_hip_memset(y.ptr, 0, y.nbytes, s)
        ggml_hip.synchronize()

        def rank1():
            t0 = time.time()
            out["rc"] = L.ggml_hip_mul_mat_q4_0_split(c1, wds[1].ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr,
                                                      N, y.ptr, s)
            out["sync"] = L.ggml_hip_stream_synchronize(s)
            out["waited"] = time.time() - t0
        th = threading.Thread(target=rank1)
        th.start()
        time.sleep(0.3)                                            # rank 1 is spinning on rank 0's flag now
        t_abort = time.time()
        ggml_hip.check(L.ggml_hip_comm_abort(c0), "abort rank 0")
        th.join(timeout=60)
        released = time.time() - t_abort
        assert not th.is_alive()
        assert out["rc"] == 0 and out["sync"] == 0, out
        assert released < 1.0, f"rank 1 released {released:.3f} s after the abort (timeout 10 s)"
        got = y.download((N, M), np.float32, stream=s)
        assert np.array_equal(got[:, rb[1]:rb[2]].view(np.uint32), own.view(np.uint32))
        assert np.all(np.isnan(got[:, rb[0]:rb[1]])), "the aborted peer's segment must read NaN"
        assert L.ggml_hip_comm_p2p_status(c1) & 1, "rank 1's status must name rank 0"
        for c, r in ((c1, 1), (c0, 0)):
            rc = L.ggml_hip_mul_mat_q4_0_split(c, wds[r].ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N,
                                               y.ptr, s)
            assert rc == ggml_hip.ERR_COMM, (r, rc)
        print(f"rank 1 waited {out['waited']:.3f} s, released {released * 1e3:.1f} ms after the abort")
    finally:
        L.ggml_hip_stream_destroy(s)
        L.ggml_hip_comm_destroy(c0)
        L.ggml_hip_comm_destroy(c1)


def test_p2p_abort_releases_own_gather_on_default_stream():
    """abort while THIS rank's own gather is blocked on a peer, on the very stream the abort's notice
    queues on (the backend's default stream, stream = NULL).  Rank 1 runs a split mul_mat whose all-gather
    waits for rank 0, which never gathers; ggml_hip_comm_abort(rank 1) sets its host-mapped request word, the
    blocked wait sees it at its next poll, notifies rank 0 and ends, so the abort returns in well under the
    10 s timeout: rank 1's own rows bitwise, rank 0's segment NaN, both ranks' status failed (rank 0 through
    the notice), and the next split call on either rank returns GGML_HIP_ERR_COMM."""
    import time
    K, M, N = 4096, 1024, 1
    wq, x = make_case(K, M, N, seed=79)
    rb = split_rows(M, 2)
    L = ggml_hip.load()
    xd = DB.from_array(x)
    wds = [DB.from_array(wq[rb[r]:rb[r + 1]]) for r in range(2)]
    y = DB(N * M * 4)
    own = gpu_y(wq[rb[1]:rb[2]], K, x)
    comms = (ctypes.c_void_p * 2)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, 2, None))
    c0, c1 = ctypes.c_void_p(comms[0]), ctypes.c_void_p(comms[1])
    try:
        th = threading.Thread(target=lambda: ggml_hip.check(L.ggml_hip_comm_enable_p2p(c1, N * M)))
        th.start()
        ggml_hip.check(L.ggml_hip_comm_enable_p2p(c0, N * M))
        th.join(timeout=60)
        L.ggml_hip_memset(y.ptr, 0, y.nbytes, None)
        ggml_hip.synchronize()
        rc = L.ggml_hip_mul_mat_q4_0_split(c1, wds[1].ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N,
                                           y.ptr, None)
        assert rc == 0
        time.sleep(0.3)                                   # rank 1's gather is spinning on rank 0's flag now
        t0 = time.time()
        ggml_hip.check(L.ggml_hip_comm_abort(c1), "abort rank 1")
        took = time.time() - t0
        assert took < 1.0, f"abort took {took:.3f} s behind its own blocked gather (timeout 10 s)"
        got = y.download((N, M), np.float32)
        assert np.array_equal(got[:, rb[1]:rb[2]].view(np.uint32), own.view(np.uint32))
        assert np.all(np.isnan(got[:, rb[0]:rb[1]])), "the never-arrived peer's segment must read NaN"
        assert L.ggml_hip_comm_p2p_status(c1) != 0
        assert L.ggml_hip_comm_p2p_status(c0) & 2, "rank 0 must hold rank 1's failure notice"
        for c, r in ((c1, 1), (c0, 0)):
            rc = L.ggml_hip_mul_mat_q4_0_split(c, wds[r].ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p), xd.ptr, N,
                                               y.ptr, None)
            assert rc == ggml_hip.ERR_COMM, (r, rc)
        print(f"abort returned {took * 1e3:.1f} ms after the call, own gather released")
    finally:
        L.ggml_hip_comm_destroy(c0)
        L.ggml_hip_comm_destroy(c1)


def test_p2p_abort_across_processes_one_gpu():
    """The same active failure across the process boundary (IPC mappings, tests/split_worker.py mode abort):
    after one good split on both ranks, rank 1 starts the next one while rank 0 aborts 0.3 s later; rank 1
    must finish within 2 s (its timeout is 10 s) with rank 0's segment NaN and then get GGML_HIP_ERR_COMM."""
    R = 2
    with tempfile.TemporaryDirectory() as td:
        idfile = os.path.join(td, "uid")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "split_worker.py"), str(r), str(R), idfile, "abort"],
                                  env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                 for r in range(R)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=100)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        for r, (p, o) in enumerate(zip(procs, outs)):
            assert p.returncode == 0, f"rank {r} failed:\n{o[-3000:]}"
            assert "ABORT_OK" in o, o[-2000:]
        print(outs[1].strip().splitlines()[-1])


def test_p2p_loopback_refusal_is_uniform():
    """Ranks on devices [0, 0, 0, 1] (or all on device 0 on a one-GPU box): every rank refuses P2P,
    including one on a device with fewer ranks (the decision was per rank before)."""
    L = ggml_hip.load()
    ndev = L.ggml_hip_device_count()
    devs = [0, 0, 0, 1 if ndev > 1 else 0]
    comms = (ctypes.c_void_p * 4)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, 4, (ctypes.c_int * 4)(*devs)))
    out = [None] * 4

    def body(r):
        L.ggml_hip_set_device(devs[r])
        out[r] = L.ggml_hip_comm_enable_p2p(ctypes.c_void_p(comms[r]), 1024)
    th = [threading.Thread(target=body, args=(r,)) for r in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    L.ggml_hip_set_device(0)
    for r in range(4):
        L.ggml_hip_comm_destroy(ctypes.c_void_p(comms[r]))
    assert out == [ggml_hip.ERR_UNSUPPORTED] * 4, out


def test_p2p_api_errors():
    L = ggml_hip.load()
    comms = (ctypes.c_void_p * 1)()
    ggml_hip.check(L.ggml_hip_comm_init_local(comms, 1, None))
    c = ctypes.c_void_p(comms[0])
    try:
        assert L.ggml_hip_comm_set_transport(c, 1) == ggml_hip.ERR_INVALID      # not enabled yet
        assert L.ggml_hip_comm_p2p_status(c) == ggml_hip.ERR_INVALID
        assert L.ggml_hip_comm_enable_p2p(c, 0) == ggml_hip.ERR_INVALID
        ggml_hip.check(L.ggml_hip_comm_enable_p2p(c, 4096))
        assert L.ggml_hip_comm_enable_p2p(c, 4096) == ggml_hip.ERR_INVALID     # twice
        ggml_hip.check(L.ggml_hip_comm_set_transport(c, 0))
        ggml_hip.check(L.ggml_hip_comm_set_transport(c, 1))
        assert L.ggml_hip_comm_p2p_status(c) == 0
    finally:
        L.ggml_hip_comm_destroy(c)
    # three loopback ranks on one device: refused (their gathers could queue behind each other)
    status = run_ranks(3, lambda r, comm, stream: L.ggml_hip_comm_enable_p2p(comm, 1024))
    assert status == [ggml_hip.ERR_UNSUPPORTED] * 3, status
