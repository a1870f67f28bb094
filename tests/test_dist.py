"""Multi-rank path on CPU (gloo, world size 2): the row partition of ggml_hip_split_rows, each
rank's shard product (oracle), the padded-slab all-gather and the compaction used by
ggml_hip_mul_mat_q4_0_split reproduce the unsharded mul_mat exactly; the RCCL unique id crosses
ranks the way bench.py ships it (torch.distributed broadcast_object_list)."""
import ctypes
import os
import socket

import numpy as np
import pytest

import oracle as O
from hip_env import ggml_hip

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _split_rows(M, world, fractions=None):
    L = ggml_hip.load()
    rb = np.zeros(world + 1, np.int64)
    fp = None
    if fractions is not None:
        fr = np.asarray(fractions, np.float32)
        fp = fr.ctypes.data_as(ctypes.c_void_p)
    ggml_hip.check(L.ggml_hip_split_rows(M, world, fp, rb.ctypes.data_as(ctypes.c_void_p)))
    return rb


def _worker(rank, world, port, cases, errq):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        uid = [b"\x07" * 128 if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        assert uid[0] == b"\x07" * 128
        for K, M, N, fractions, seed in cases:
            wf = O.gaussian(M * K, seed, 0.0, 0.02).reshape(M, K)
            wq, _ = O.quantize_q4_0(wf)
            x = O.gaussian(N * K, seed + 1, 0.0, 1.0).reshape(N, K)
            rb = _split_rows(M, world, fractions)
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
            assert np.array_equal(y.view(np.uint32), y_full.view(np.uint32)), (K, M, N, fractions)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        errq.put(f"rank {rank}: {e!r}")
        raise


@pytest.mark.parametrize("world", [2])
def test_row_split_allgather_matches_full(world):
    cases = [(4096, 256, 1, None, 11), (4544, 200, 3, None, 12), (4096, 130, 2, [3.0, 1.0], 13),
             (64, 5, 4, [0.0, 1.0], 14)]
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
