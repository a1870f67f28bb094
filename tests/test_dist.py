"""Multi-rank path on CPU (gloo, world size 2): the row partition of ggml_hip_split_rows, each
rank's shard product (oracle), the padded-slab all-gather and the compaction used by
ggml_hip_mul_mat_q4_0_split reproduce the unsharded mul_mat exactly.  The ranks are separate
processes (tests/dist_worker.py) that import torch for gloo and never load libggml_hip.so; this
process loads the library (for the partitions) and never imports torch: torch bundles its own
HIP runtime, and two runtimes in one process corrupt it.  The product's own split code at R > 1
runs on the GPU in tests/test_gpu_split.py (in-process loopback ranks)."""
import ctypes
import importlib.util
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from hip_env import ggml_hip

HERE = os.path.dirname(os.path.abspath(__file__))


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


@pytest.mark.skipif(importlib.util.find_spec("torch") is None, reason="torch (gloo) not importable")
@pytest.mark.parametrize("world", [2])
def test_row_split_allgather_matches_full(world):
    cases = [(4096, 256, 1, None, 11), (4544, 200, 3, None, 12), (4096, 130, 2, [3.0, 1.0], 13),
             (64, 5, 4, [0.0, 1.0], 14)]
    spec = [(K, M, N, _split_rows(M, world, fr).tolist(), seed) for K, M, N, fr, seed in cases]
    port = _free_port()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "cases.json")
        json.dump(spec, open(path, "w"))
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                                   path], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                 for r in range(world)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=240)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"DIST_OK rank {r}" in o, o[-3000:]


@pytest.mark.parametrize("world", [2, 3])
def test_file_comm_ranks_drive_product_host_code(world):
    """World-size 2 and 3 on CPU through the LIBRARY in every rank (tests/file_comm_worker.py: no torch,
    so libggml_hip.so loads): the file-rendezvous comm, each rank's own ggml_hip_split_rows, the padded-slab
    all-gather through ggml_hip_comm_allgather_host, ggml_hip_comm_allreduce_host sum / max / min;
    y == the unsharded oracle product bitwise."""
    cases = [(4096, 256, 1, None, 21), (4544, 200, 3, None, 22), (4096, 130, 2, [3.0, 1.0, 2.0][:world], 23),
             (64, 5, 4, [0.0, 1.0, 1.0][:world], 24)]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "cases.json")
        json.dump(cases, open(path, "w"))
        cdir = os.path.join(td, "comm")
        os.mkdir(cdir)
        env = dict(os.environ, GGML_HIP_COMM_FILE_TIMEOUT_S="60")
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "file_comm_worker.py"), str(r), str(world), cdir,
                                   path], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
                 for r in range(world)]
        outs = []
        for p in procs:
            try:
                outs.append(p.communicate(timeout=180)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    q.kill()
                raise
        for r, (p, o) in enumerate(zip(procs, outs)):
            assert p.returncode == 0, f"rank {r}:\n{o[-3000:]}"
            assert "FILE_COMM_OK" in o, o[-2000:]


def test_file_comm_session_nonce_and_reuse():
    """file-comm names carry a per-session nonce that rank 0 publishes as <dir>/session (link(2),
    refused when the name exists), so a reused directory never feeds a dead session's file of the same
    sequence number into a new one.  Two world-2 sessions run back to back in ONE directory (the first
    leaves its last files behind), and a directory holding a session file is refused loudly."""
    cases = [(4096, 64, 1, None, 31)]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "cases.json")
        json.dump(cases, open(path, "w"))
        cdir = os.path.join(td, "comm")
        os.mkdir(cdir)
        env = dict(os.environ, GGML_HIP_COMM_FILE_TIMEOUT_S="60")
        for session in range(2):
            procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "file_comm_worker.py"), str(r), "2", cdir, path],
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
                     for r in range(2)]
            outs = [p.communicate(timeout=180)[0] for p in procs]
            for r, (p, o) in enumerate(zip(procs, outs)):
                assert p.returncode == 0 and "FILE_COMM_OK" in o, f"session {session} rank {r}:\n{o[-3000:]}"
            left = sorted(os.listdir(cdir))
            assert "session" not in left, left
            nonces = {f[1:].split("_")[0] for f in left if f.startswith("c")}
            assert len(nonces) == session + 1, left          # each session's leftovers carry their own nonce
        # a directory with a session file (in use, or a crashed session's leftover): refused, not joined
        L = ggml_hip.load()
        sdir = os.path.join(td, "stale")
        os.mkdir(sdir)
        open(os.path.join(sdir, "session"), "w").write("0123456789abcdef")
        c = ctypes.c_void_p()
        assert L.ggml_hip_comm_init_file(ctypes.byref(c), 1, 0, sdir.encode()) == ggml_hip.ERR_COMM
        assert b"session" in L.ggml_hip_last_error()
        os.remove(os.path.join(sdir, "session"))
        ggml_hip.check(L.ggml_hip_comm_init_file(ctypes.byref(c), 1, 0, sdir.encode()))   # one rank: joins itself
        v = (ctypes.c_double * 1)(3.0)
        ggml_hip.check(L.ggml_hip_comm_allreduce_host(c, v, 1, 0))
        assert v[0] == 3.0
        ggml_hip.check(L.ggml_hip_comm_destroy(c))


def _bench_json(stdout):
    lines = [l for l in stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


def test_bench_launcher_deadline_with_a_stalled_rank():
    """Verdict r5 item 4: `bench.py --gpus 2` self-launched with both ranks forced to stall before any GPU
    work (GGML_HIP_BENCH_STALL_RANKS) returns within its deadline (--deadline + 30 s for the launcher), prints
    ONE JSON line with "error" and exits non-zero, instead of waiting for the driver's kill."""
    import time
    root = os.path.dirname(HERE)
    env = dict(os.environ, GGML_HIP_BENCH_STALL_RANKS="0,1")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--deadline", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    line = _bench_json(r.stdout)
    assert "deadline" in line["error"] and line["value"] is None and line["n_gpus"] == 2
    assert took < 2 + 30 + 10 + 20, took


def test_bench_rank_watchdog_under_external_launcher():
    """The driver launches N > 1 through torchrun (WORLD_SIZE set), so the launcher deadline does not apply:
    each rank's own watchdog does.  A rank started as torchrun would start it, forced to hang with its watchdog
    armed (GGML_HIP_BENCH_STALL_ARMED_RANKS: as if stuck in RCCL init or a collective), ends after --deadline:
    rank 0 prints the one JSON line with "error" and the process exits 3."""
    import time
    root = os.path.dirname(HERE)
    work = tempfile.mkdtemp(prefix="bench_wd_")
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), GGML_HIP_UID_FILE=os.path.join(work, "uid"),
               GGML_HIP_COMM_DIR=os.path.join(work, "comm"), GGML_HIP_BENCH_STALL_ARMED_RANKS="0")
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--deadline", "3"], env=env,
                       capture_output=True, text=True, timeout=120)
    took = time.time() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    line = _bench_json(r.stdout)
    assert "deadline" in line["error"] and line["value"] is None
    assert took < 3 + 30, took
