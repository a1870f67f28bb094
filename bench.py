#!/usr/bin/env python3
"""bench.py — q4_0 mul_mat on MI355X: decode tok/s (+ prefill GB/s), LLaMA-7B shapes.

Metric (BASELINE.json): "q4_0 mul_mat: decode tok/s + prefill GB/s, LLaMA-7B shapes, 1/2/4/8 GPU".

One step = one decode token through the q4_0 matmuls of LLaMA-7B: 32 layers x 7 mul_mats
(wq, wk, wv, wo: 4096->4096; w1, w3: 4096->11008; w2: 11008->4096), each including the q8_0
quantize of its activation row.  The weight stack (3.64 GB of
block_q4_0 rows, distinct memory per layer) is resident in HBM and larger than the 256 MB
Infinity Cache.  The 224 launches of a step are captured once in a HIP graph and replayed.

N GPUs (torchrun, one process per GPU): every matrix is row-sharded N ways (the reference's
GGML_BACKEND_GPU_SPLIT); siblings (wq|wk|wv, w1|w3) run as one GEMV launch per rank followed by
one grouped RCCL all-gather of their y slices over xGMI (4 collectives per layer);
value = tokens/s of the sharded model (strong scaling: total work fixed), over the faster of the two
all-gather transports (RCCL, or the direct-store P2P all-gather when its run passes its self-checks;
both are in the line).

Extra fields: per-kernel roofline of the dominant kernel (the decode GEMV) from HIP events on
the launch stream, prefill (N=512, the same sibling groups: one x quantize per group) GB/s and
int8-MFMA TOP/s, exact-mode decode, the LLaMA-13B / Falcon-7B decode shapes, and the CPU baseline
(the reference's own ggml.c built from /root/reference into oracle/_ref, on this host's cores).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "llama.cpp-q_4_0_amd", "python"))

METRIC = "q4_0 mul_mat: decode tok/s + prefill GB/s, LLaMA-7B shapes, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
INT8_PEAK_TOPS = 5000.0          # dense int8 MFMA = 2x bf16 per clock (~2.5 PF bf16 dense)
N_LAYERS = 32
# (name, K, M) in ggml terms: W [M][K] q4_0, x [N][K], y [N][M]
LAYER = [("wq", 4096, 4096), ("wk", 4096, 4096), ("wv", 4096, 4096), ("wo", 4096, 4096),
         ("w1", 4096, 11008), ("w3", 4096, 11008), ("w2", 11008, 4096)]


# other BASELINE.json configs measured on one GPU (same kernels): (name, layers, spec, sibling groups)
EXTRA_CONFIGS = [
    ("LLaMA-13B decode (config 4 shapes, 1 GPU)", 40,
     [("wq", 5120, 5120), ("wk", 5120, 5120), ("wv", 5120, 5120), ("wo", 5120, 5120),
      ("w1", 5120, 13824), ("w3", 5120, 13824), ("w2", 13824, 5120)], [[0, 1, 2], [3], [4, 5], [6]]),
    # Falcon-7B runs attention and MLP in parallel (parallel_attn = 1, arch/falcon/falcon.cpp:1334-1355): the
    # fused qkv and the MLP's fc both read the layer's one layer-norm output (outLN), so they are siblings
    ("Falcon-7B decode (config 5 shapes, arch/falcon)", 32,
     [("wqkv", 4544, 4672), ("wo", 4544, 4544), ("w1", 4544, 18176), ("w2", 18176, 4544)], [[0, 2], [1], [3]]),
    ("GPT-NeoX-20B decode (config 5 shapes, arch/gptneox: n_embd 6144, n_ff 24576)", 44,
     [("wqkv", 6144, 18432), ("wo", 6144, 6144), ("w1", 6144, 24576), ("w2", 24576, 6144)], [[0], [1], [2], [3]]),
]


def q4_bytes(K, M):
    return 18 * K // 32 * M


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------------------------
def error_line(n_gpus, msg):
    """the one JSON line of a run that could not measure (a rank stalled, failed or ran out of time)"""
    return json.dumps({"metric": METRIC, "value": None, "unit": "tok/s", "n_gpus": n_gpus, "higher_is_better": True,
                       "error": msg})


def launch_ranks(n_gpus, deadline_s):
    """`bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment): start N fresh child
    processes of this script, one per rank, before this process loads any GPU library (no exec, no
    relaunch of a process that touched the GPU).  Rank 0's stdout (the one JSON line) is this process's
    stdout, the other ranks' go to stderr.  The ranks rendezvous through a fresh directory (RCCL unique
    id file, or the file comm when ranks share a device).  Returns the exit code (the worst rank's).
    Overall deadline (verdict r5 item 4): when the ranks have not all exited `deadline_s` after the start
    (a rank stuck before or in RCCL init, or in a collective), every remaining rank is terminated (killed
    10 s later) and this process prints ONE JSON line with "error" and returns 124; a failed rank gives
    the others 60 s (or what is left of the deadline)."""
    import shutil
    import socket
    import subprocess
    import tempfile
    work = tempfile.mkdtemp(prefix="ggml_hip_bench_")
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    try:
        for r in range(n_gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n_gpus), LOCAL_WORLD_SIZE=str(n_gpus),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GGML_HIP_UID_FILE=os.path.join(work, "uid"),
                       GGML_HIP_COMM_DIR=os.path.join(work, "comm"), GGML_HIP_BENCH_SELF_LAUNCHED="1")
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                          stdout=None if r == 0 else sys.stderr))
        rcs = [None] * n_gpus
        t_fail = None
        t_start = time.time()
        while any(rc is None for rc in rcs):
            if time.time() - t_start > deadline_s:
                stuck = [r for r in range(n_gpus) if rcs[r] is None]
                log(f"[launcher] deadline {deadline_s:.0f} s passed: terminating ranks {stuck}")
                for r in stuck:
                    procs[r].terminate()
                t_kill = time.time()
                while any(procs[r].poll() is None for r in stuck) and time.time() - t_kill < 10:
                    time.sleep(0.05)
                for r in stuck:
                    if procs[r].poll() is None:
                        procs[r].kill()
                print(error_line(n_gpus, f"launcher deadline {deadline_s:.0f} s passed with ranks {stuck} still running "
                                         f"(exit codes so far: {rcs})"), flush=True)
                return 124
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
                    if rcs[r] not in (None, 0) and t_fail is None:
                        t_fail = time.time()
                        log(f"[launcher] rank {r} exited with {rcs[r]}")
            if t_fail is not None and time.time() - t_fail > 60:     # a failed rank: the others get 60 s
                for r, p in enumerate(procs):
                    if rcs[r] is None:
                        log(f"[launcher] terminating rank {r}")
                        p.terminate()
                t_fail = time.time() + 1e9
            time.sleep(0.05)
        return max(abs(rc) for rc in rcs)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        shutil.rmtree(work, ignore_errors=True)


def rank_watchdog(L, rank, world, deadline_s, get_comm):
    """N > 1 ranks (torchrun's or the self-launcher's): if this rank has not finished `deadline_s` after it
    started, a timer thread aborts its communicator (ncclCommAbort releases a collective stuck on the device;
    the P2P notice tells the peers), rank 0 prints the one JSON line with "error", and the process exits 3
    (torchrun then stops the other ranks).  RCCL init and every RCCL call are bounded inside the library too
    (GGML_HIP_COMM_TIMEOUT_MS, default 120 s)."""
    import threading

    def fire():
        log(f"[rank {rank}] deadline {deadline_s:.0f} s passed: aborting the communicator and exiting")
        c = get_comm()
        if c is not None and c.value:            # bounded: the exit below happens even if the abort blocks
            ab = threading.Thread(target=L.ggml_hip_comm_abort, args=(c,), daemon=True)
            ab.start()
            ab.join(15.0)
        if rank == 0:
            print(error_line(world, f"rank deadline {deadline_s:.0f} s passed (stuck in init or a collective)"),
                  flush=True)
        sys.stderr.flush()
        os._exit(3)

    t = threading.Timer(deadline_s, fire)
    t.daemon = True
    t.start()
    return t


def setup_dist():
    """launcher env -> (rank, world, local_rank).  No torch in this process: torch bundles its own
    libamdhip64 / librccl, and a second HIP runtime next to /opt/rocm's (which libggml_hip.so is
    built against) corrupts the process; ranks talk through RCCL or the file comm only."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", rank))
    return rank, world, local


def _rendezvous_path(kind):
    """a path every rank of this node derives alike: the launcher's (self-launch sets it), else one named
    after torchrun's agent (every worker's parent) and its rendezvous port"""
    env = {"uid": "GGML_HIP_UID_FILE", "comm": "GGML_HIP_COMM_DIR"}[kind]
    return os.environ.get(env) or os.path.join(
        "/tmp", f"ggml_hip_{kind}_{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}")


def exchange_unique_id(gh, L, rank, world):
    """RCCL unique id from rank 0 to the other ranks of this node through a file."""
    path = _rendezvous_path("uid")
    uid = ctypes.create_string_buffer(128)
    if rank == 0:
        gh.check(L.ggml_hip_comm_unique_id(uid))
        with open(path + ".tmp", "wb") as f:
            f.write(uid.raw)
        os.replace(path + ".tmp", path)
    elif world > 1:
        t0 = time.time()
        while not os.path.exists(path):
            if time.time() - t0 > 300:
                raise SystemExit(f"rank {rank}: no RCCL unique id at {path}")
            time.sleep(0.02)
        time.sleep(0.05)
        uid = ctypes.create_string_buffer(open(path, "rb").read(), 128)
    return uid, path


def weight_std(K):
    """W ~ N(0, 1/sqrt(K)): y = W x keeps x's scale, so the decode chain (each launch reads the previous
    launch's y) stays O(1) over 32 layers (at N(0, 0.02) it grew ~4.4x per layer and overflowed the fp16
    q8_0 scale by layer ~10); LLaMA-7B's init scale 0.02 is 1.28/sqrt(4096)"""
    return 1.0 / float(np.sqrt(K))


class Stack:
    """Resident weight stack for one rank: per layer per matrix the rank's row slice."""

    def __init__(self, gh, L, rank, world, layers, seed_base=0x5EED0000, spec=None):
        spec = LAYER if spec is None else spec
        self.mats = []
        self.bufs = []
        tmp = gh.DeviceBuffer(max(K * M for _, K, M in spec) * 4)
        total = 0
        for li in range(layers):
            row = []
            for mi, (name, K, M) in enumerate(spec):
                rb = np.zeros(world + 1, np.int64)
                gh.check(L.ggml_hip_split_rows(M, world, None, rb.ctypes.data_as(ctypes.c_void_p)))
                m_loc = int(rb[rank + 1] - rb[rank])
                nbytes = q4_bytes(K, m_loc)
                buf = gh.DeviceBuffer(max(nbytes, 16))
                seed = seed_base + li * 16 + mi
                gh.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * m_loc, seed, 0.0, weight_std(K), None))
                gh.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, m_loc, buf.ptr, None))
                row.append((name, K, M, m_loc, buf, rb))
                self.bufs.append(buf)
                total += nbytes
            self.mats.append(row)
        gh.synchronize()
        tmp.free()
        self.total_bytes = total

    def free(self):
        for b in self.bufs:
            b.free()
        self.bufs = []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layers", type=int, default=N_LAYERS)
    ap.add_argument("--config4-layers", type=int, default=40,
                    help="N > 1: layers of the LLaMA-13B row-sharded line (BASELINE config 4); 0 skips it")
    ap.add_argument("--prefill-tokens", type=int, default=512)
    ap.add_argument("--no-prefill", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    ap.add_argument("--eager", action="store_true", help="no HIP graph (launch-per-call)")
    ap.add_argument("--force-split", action="store_true",
                    help="run the multi-GPU code path (row split + RCCL all-gather) even with one rank")
    ap.add_argument("--comm", choices=("auto", "rccl", "file"), default="auto",
                    help="N > 1: RCCL communicator (one rank per GPU), or the file-rendezvous comm with the P2P "
                         "all-gather only (ranks may share a device); auto = file when ranks outnumber devices")
    ap.add_argument("--no-extra", action="store_true", help="skip the LLaMA-13B / Falcon-7B decode lines")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-mode (bit-identical) decode line")
    ap.add_argument("--no-p2p", action="store_true",
                    help="N > 1: skip the direct-store (P2P) all-gather line next to RCCL's")
    ap.add_argument("--no-batch-siblings", action="store_true",
                    help="one launch per mul_mat (7 per layer) instead of batching wq/wk/wv and w1/w3")
    ap.add_argument("--decode", choices=("auto", "engine", "launches"), default="auto",
                    help="headline decode path: the persistent LDS-DMA engine (one launch per token, "
                         "ggml_hip_chain_set_engine), the per-launch graph (4 sibling GEMVs per layer), or auto = "
                         "the engine when its outputs are bitwise the launches' and it ran faster (both are timed)")
    ap.add_argument("--no-roofline-replays", action="store_true",
                    help="skip the per-position isolated replays of the roofline (profiling runs: the rocprof summary "
                         "then holds the timed replays' GEMVs only)")
    ap.add_argument("--no-aql", action="store_true",
                    help="decode: skip the form issued through the library's own AQL queue (launch mode 3)")
    ap.add_argument("--deadline", type=float, default=300.0,
                    help="N > 1: seconds after which a rank that has not finished aborts its communicator and exits "
                         "(rank 0 prints an error line); the self-launcher terminates its ranks 30 s later")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, args.deadline + 30.0))
    stall = os.environ.get("GGML_HIP_BENCH_STALL_RANKS")     # test hook: these ranks hang before any GPU work
    if stall and os.environ.get("RANK", "0") in stall.split(","):
        log(f"[rank {os.environ.get('RANK')}] GGML_HIP_BENCH_STALL_RANKS: stalling before GPU init")
        while True:
            time.sleep(1)

    import ggml_hip as gh
    L = gh.load()                            # /opt/rocm HIP + RCCL (no torch in this process)
    rank, world, local = setup_dist()
    if world > 1 and args.gpus != world:
        log(f"[rank {rank}] --gpus {args.gpus} but WORLD_SIZE {world}: using {world} ranks")
    comm = None
    watchdog = rank_watchdog(L, rank, world, args.deadline, lambda: comm) if world > 1 else None
    armed = os.environ.get("GGML_HIP_BENCH_STALL_ARMED_RANKS")   # test hook: hang with the watchdog armed
    if armed and str(rank) in armed.split(","):
        log(f"[rank {rank}] GGML_HIP_BENCH_STALL_ARMED_RANKS: stalling with the watchdog armed")
        while True:
            time.sleep(1)
    ndev = L.ggml_hip_device_count()
    if ndev < 1:
        raise SystemExit("no HIP device")
    gh.check(L.ggml_hip_set_device(local % ndev), "set_device")
    stream = L.ggml_hip_default_stream()

    comm_kind = None
    if world > 1 or args.force_split:
        comm_kind = args.comm if args.comm != "auto" else ("file" if world > ndev else "rccl")
        comm = ctypes.c_void_p()
        if comm_kind == "file":
            cdir = _rendezvous_path("comm")
            os.makedirs(cdir, exist_ok=True)
            gh.check(L.ggml_hip_comm_init_file(ctypes.byref(comm), world, rank, cdir.encode()), "comm_init_file")
        else:
            uid, uid_path = exchange_unique_id(gh, L, rank, world)
            # RCCL prints a version banner on fd 1 at init: keep stdout to the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                gh.check(L.ggml_hip_comm_init(ctypes.byref(comm), world, rank, uid), "comm_init")
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            if rank == 0 and world > 1:
                try:
                    os.remove(uid_path)      # every rank has joined (comm init is collective)
                except OSError:
                    pass

    def allreduce(vals, op):
        """sum (0) / max (1) / min (2) of host doubles over the ranks (RCCL or files; also a barrier)"""
        if comm is None:
            return list(vals)
        buf = (ctypes.c_double * len(vals))(*vals)
        gh.check(L.ggml_hip_comm_allreduce_host(comm, buf, len(vals), op), "allreduce")
        return list(buf)

    def barrier():
        gh.check(L.ggml_hip_device_synchronize())
        allreduce([0.0], 0)

    if comm is not None:
        result = sharded_main(gh, L, comm, comm_kind, rank, world, args, stream, allreduce, barrier)
        if watchdog is not None:
            watchdog.cancel()
        if rank == 0:
            print(json.dumps(result), flush=True)
        L.ggml_hip_comm_destroy(comm)
        return

    t0 = time.time()
    stack = Stack(gh, L, 0, 1, args.layers)
    log(f"weight stack {stack.total_bytes / 1e9:.3f} GB resident in {time.time() - t0:.1f}s")

    # activations (one x per K; synthetic N(0,1)) and outputs (one y per M)
    xs = {}
    for K in (4096, 11008):
        b = gh.DeviceBuffer(K * 4 * max(1, args.prefill_tokens))
        gh.check(L.ggml_hip_fill_gaussian(b.ptr, K * max(1, args.prefill_tokens), 0x5EED1000 + K, 0.0, 1.0, None))
        xs[K] = b
    ys = {M: gh.DeviceBuffer(M * 4 * max(1, args.prefill_tokens)) for M in (4096, 11008)}
    for K, M in ((4096, 11008), (11008, 4096)):     # prefill: the GEMM's per-call weight image of M rows
        gh.check(L.ggml_hip_reserve_workspace_mm(K, max(1, args.prefill_tokens), M))
    gh.synchronize()

    batch = not args.no_batch_siblings
    # sibling groups that share src1 in the LLaMA graph: (wq, wk, wv) and (w1, w3)
    groups = [[0, 1, 2], [3], [4, 5], [6]] if batch else [[i] for i in range(len(LAYER))]
    yb = {i: gh.DeviceBuffer(LAYER[i][2] * 4) for i in range(len(LAYER))}
    # the decode's real data dependencies (each launch reads the y of the launch before it): wq|wk|wv read
    # the previous layer's w2 output (layer 0: the fixed input row), wo reads q, w1|w3 read wo's output,
    # w2 reads w1's output
    DEP = {0: 6, 1: 6, 2: 6, 3: 0, 4: 3, 5: 3, 6: 4}

    def x_of(li, i):
        K = LAYER[i][1]
        if li == 0 and DEP[i] == 6:
            return xs[K].ptr
        return yb[DEP[i]].ptr

    launch_args = []
    for li, row in enumerate(stack.mats):
        for g in groups:
            if len(g) == 1 or not batch:
                launch_args.append(("local", tuple(row[g[0]]) + (yb[g[0]], None, x_of(li, g[0]))))
            else:
                n = len(g)
                wp = (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g])
                yp = (ctypes.c_void_p * n)(*[yb[i].ptr for i in g])
                mp = (ctypes.c_int64 * n)(*[row[i][3] for i in g])
                launch_args.append(("multi", (n, wp, mp, row[g[0]][1], yp, x_of(li, g[0]))))

    def decode_step():
        for kind, a in launch_args:
            if kind == "multi":
                n, wp, mp, K, yp, xp = a
                gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xp, 1, yp, stream))
            else:
                name, K, M, m_loc, buf, rb, ylocal, _, xp = a
                gh.check(L.ggml_hip_mul_mat_q4_0_ex(buf.ptr, K, m_loc, xp, 1, ylocal.ptr, m_loc, 0, stream))

    graph = None
    if not args.eager:
        decode_step()                        # first call outside capture (workspace, lazy init)
        gh.check(L.ggml_hip_stream_synchronize(stream))
        graph = gh.Graph(stream)
        with graph:
            decode_step()

    def run_step():
        if graph is not None:
            graph.launch()
        else:
            decode_step()

    def timed(step_fn):
        for _ in range(args.warmup):
            step_fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_fn()
        barrier()
        return time.perf_counter() - t0

    # the per-launch chain two ways, interleaved twice, best of each: replayed as one HIP graph per token, and
    # issued eagerly from the host (128 launches at ~2.7 us of host time each stay ahead of the ~0.93 ms device
    # step; tools/prefetch_ab.py measured the eager form 1-2 % faster on the device)
    # A third form: the same eager launches through the library's own AQL queue (launch mode 3, ggml-hip-aql.cpp:
    # 0.2-0.3 us of host time per dispatch, kernargs in VRAM, agent-scope fences between kernels); it must give the
    # graph's outputs bit for bit to count
    # (not under a profiler: rocprofv3 wraps HSA queues, and this form writes its packets into its queue directly)
    profiled = "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)
    aql_ok = hasattr(L, "ggml_hip_debug_set_stream_launch_mode") and not args.eager and not args.no_aql and not profiled

    def timed_aql():                  # the stream's launches through the queue for the whole timed block
        gh.check(L.ggml_hip_debug_set_stream_launch_mode(stream, 3))
        try:
            return timed(decode_step)
        finally:
            gh.check(L.ggml_hip_debug_set_stream_launch_mode(stream, 0))

    if graph is not None:
        t_graph, t_eager, t_aql = [], [], []
        for _ in range(2):
            t_graph.append(timed(run_step))
            t_eager.append(timed(decode_step))
            if aql_ok:
                t_aql.append(timed_aql())
        elapsed_graph, elapsed_eager = min(t_graph), min(t_eager)
        elapsed_aql = min(t_aql) if t_aql else None
        eager_wins = elapsed_eager < elapsed_graph
        elapsed_launches = min(elapsed_graph, elapsed_eager)
    else:
        elapsed_graph, elapsed_eager, eager_wins, elapsed_aql = None, timed(run_step), True, None
        elapsed_launches = elapsed_eager
    last = yb[6].download((LAYER[6][2],), np.float32, stream=stream)          # the step's last output
    finite = bool(np.all(np.isfinite(last)))
    if not finite:
        log("WARNING: the decode chain's last output is not finite")
    outs_launches = [yb[i].download((LAYER[i][2],), np.float32, stream=stream) for i in range(len(LAYER))]
    aql_form = None
    if elapsed_aql is not None:                # bitwise self-check of the AQL form against the graph's outputs
        for i in range(len(LAYER)):
            gh.check(L.ggml_hip_memset(yb[i].ptr, 0xFF, LAYER[i][2] * 4, stream))
        gh.check(L.ggml_hip_debug_set_stream_launch_mode(stream, 3))
        try:
            decode_step()
        finally:
            gh.check(L.ggml_hip_debug_set_stream_launch_mode(stream, 0))
        same = all(np.array_equal(yb[i].download((LAYER[i][2],), np.float32, stream=stream).view(np.uint32),
                                  outs_launches[i].view(np.uint32)) for i in range(len(LAYER)))
        aql_form = {"tok_s": round(args.steps / elapsed_aql * 32 / args.layers, 2),
                    "ms_per_step": round(elapsed_aql / args.steps * 1e3, 4), "bitwise_vs_graph": bool(same)}
        if same and elapsed_aql < elapsed_launches:
            elapsed_launches = elapsed_aql
            eager_wins = "aql"
    engine = None
    if args.decode != "launches" and graph is not None and batch:
        engine = engine_decode(gh, L, launch_args, yb, outs_launches, stream, timed)
        if args.decode == "engine" and not engine.get("on"):
            raise SystemExit(f"--decode engine: the engine declined the chain: {engine.get('declined')}")
    # the engine is the headline only when asked for, or (auto) when it checked bitwise AND ran faster than the
    # per-launch graph; round 6 measured it slower (profiles/r06_engine_variants.txt), so auto keeps
    # the launches and the line carries both
    engine_ok = engine is not None and engine.get("on") and engine["bitwise_vs_launches"] and engine["status"] == 0
    use_engine = engine_ok and (args.decode == "engine" or engine["elapsed_s"] < elapsed_launches)
    if engine is not None and engine.get("on"):
        engine["tok_s"] = round(args.steps / engine["elapsed_s"] * 32 / args.layers, 2)
        engine["ms_per_step"] = round(engine["elapsed_s"] / args.steps * 1e3, 4)
    elapsed = engine["elapsed_s"] if use_engine else elapsed_launches
    ms_per_step = elapsed / args.steps * 1e3
    tok_s = args.steps / elapsed * 32 / args.layers if args.layers else 0.0   # per full 32-layer token

    result = {
        "metric": METRIC, "value": round(tok_s, 2), "unit": "tok/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "q4_0 x q8_0 (int8 dot, f32 acc)",
        "data": ("synthetic: W ~ N(0, 1/sqrt(K)) -> q4_0 (ggml A3 rule, on device), x ~ N(0,1); random-init, no "
                 "checkpoint; departs from SURVEY 8d's N(0, 0.02): with each launch reading the previous launch's y "
                 "(wo <- q, w1|w3 <- wo, w2 <- w1, next layer <- w2) 0.02 grows the activations ~4.4x per layer and "
                 "overflows the fp16 q8_0 scale by layer ~10, 1/sqrt(K) keeps them O(1) (bytes and time do not depend "
                 f"on it); last output finite: {finite}"),
        "config": {"workload": "LLaMA-7B q4_0 decode, 32 layers x 7 mul_mats (wq,wk,wv,wo 4096x4096; w1,w3 "
                               "4096->11008; w2 11008->4096), N=1, q8_0 quantize of x included, lm_head excluded",
                   "layers": args.layers, "weights_bytes_per_rank": stack.total_bytes,
                   "graph": graph is not None,
                   "decode_path": ("persistent LDS-DMA engine: ONE launch per token (ggml_hip_chain_set_engine), "
                                   "outputs bitwise the per-launch GEMVs'" if use_engine else
                                   "per-launch GEMVs, " + (
                                       "issued through the library's own AQL queue (launch mode 3; the fastest form here, "
                                       "bitwise the graph's outputs)" if eager_wins == "aql" else
                                       "issued eagerly (faster than the per-token HIP graph here)" if eager_wins else
                                       "one HIP graph per token")),
                   "launches_per_layer": 0.0 if use_engine else len(groups),
                   "sibling_batching": "wq|wk|wv and w1|w3 share src1 -> one launch each" if batch else "off",
                   "collectives_per_layer": 0, "parallelism": "single GPU", "activations_finite": finite},
    }
    result["config"]["runtime_libs"] = gh.mapped_runtime_libs()
    if elapsed_graph is not None:
        result["launches_graph"] = {"tok_s": round(args.steps / elapsed_graph * 32 / args.layers, 2),
                                    "ms_per_step": round(elapsed_graph / args.steps * 1e3, 4),
                                    "launches_per_layer": len(groups)}
    result["launches_eager"] = {"tok_s": round(args.steps / elapsed_eager * 32 / args.layers, 2),
                                "ms_per_step": round(elapsed_eager / args.steps * 1e3, 4),
                                "launches_per_layer": len(groups)}
    if aql_form is not None:
        result["launches_aql"] = aql_form
    if engine is not None:
        result["engine"] = {k: v for k, v in engine.items() if k != "elapsed_s"}
    result["roofline"] = kernel_roofline(gh, L, launch_args, xs, stream, len(groups),
                                         elapsed_launches / args.steps * 1e3, args.layers,
                                         engine_step_ms=result.get("engine", {}).get("ms_per_step"),
                                         isolated=not args.no_roofline_replays)
    if not args.no_prefill and args.prefill_tokens > 0:
        result["prefill"] = prefill_bench(gh, L, stack, xs, ys, stream, args.prefill_tokens,
                                          groups=[tuple(g) for g in groups])
    if not args.no_exact:
        result["exact_mode"] = exact_decode(gh, L, decode_step, stream, args)
    if not args.no_extra:
        result["other_configs"] = [extra_decode(gh, L, stream, *c, steps=args.steps, warmup=args.warmup)
                                   for c in EXTRA_CONFIGS]
    if not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    print(json.dumps(result), flush=True)


# ---------------------------------------------------------------------------------------------
LLAMA13B = [("wq", 5120, 5120), ("wk", 5120, 5120), ("wv", 5120, 5120), ("wo", 5120, 5120),
            ("w1", 5120, 13824), ("w3", 5120, 13824), ("w2", 13824, 5120)]


def sharded_main(gh, L, comm, comm_kind, rank, world, args, stream, allreduce, barrier):
    """N ranks (one process each): every matrix row-sharded N ways (GGML_BACKEND_GPU_SPLIT); per layer 4
    launches (siblings batched) each followed by one grouped all-gather.  The headline is LLaMA-7B (32
    layers) over the faster self-checked transport; the BASELINE config-4 line (LLaMA-13B, 40 layers) rides
    along.  File comm: the RCCL transport is unavailable (ranks may share a device), P2P only."""
    use_p2p = comm_kind == "file" or (world > 1 and not args.no_p2p)
    p2p_state = {"on": False, "error": None}
    if use_p2p:
        max_floats = max(M for _, K, M in LAYER + LLAMA13B)
        rc = L.ggml_hip_comm_enable_p2p(comm, max_floats)
        if allreduce([float(rc)], 2)[0] != 0.0:             # any rank failed (the outcome is collective)
            p2p_state["error"] = f"enable_p2p rc={rc}: {L.ggml_hip_last_error().decode(errors='replace')}"
            if comm_kind == "file":
                raise SystemExit(f"[rank {rank}] file comm needs the P2P transport: {p2p_state['error']}")
        else:
            p2p_state["on"] = True
    batch = not args.no_batch_siblings
    groups = [[0, 1, 2], [3], [4, 5], [6]] if batch else [[i] for i in range(len(LAYER))]
    line = sharded_decode(gh, L, comm, comm_kind, rank, world, LAYER, args.layers, groups, args, stream, allreduce,
                          barrier, p2p_state, 0x5EED0000)
    tok_s, ms = line["tok_s"], line["ms_per_step"]
    result = {
        "metric": METRIC, "value": tok_s, "unit": "tok/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "q4_0 x q8_0 (int8 dot, f32 acc)",
        "data": ("synthetic: W ~ N(0, 1/sqrt(K)) -> q4_0 (ggml A3 rule, on device), x ~ N(0,1); random-init, no "
                 "checkpoint; departs from SURVEY 8d's N(0, 0.02) as the single-GPU line does (activations O(1) over "
                 "the chained layers)"),
        "config": {"workload": "LLaMA-7B q4_0 decode, 32 layers x 7 mul_mats (wq,wk,wv,wo 4096x4096; w1,w3 "
                               "4096->11008; w2 11008->4096), N=1, q8_0 quantize of x included, lm_head excluded",
                   "layers": args.layers, "weights_bytes_per_rank": line["weights_bytes_per_rank"],
                   "graph": True, "launches_per_layer": len(groups), "comm": comm_kind,
                   "sibling_batching": ("wq|wk|wv and w1|w3 share src1 -> one launch + one grouped all-gather each"
                                        if batch else "off"),
                   "collectives_per_layer": len(groups),
                   "parallelism": f"row-split x{world} + {line['transport']} all-gather",
                   "transport": line["transport"], "transports": line["transports"],
                   "compute_only_tok_s": line["compute_only_tok_s"], "split_check": line["split_check"],
                   "self_launched": os.environ.get("GGML_HIP_BENCH_SELF_LAUNCHED") == "1"},
    }
    if "rccl" in line["transports"]:
        r = line["transports"]["rccl"]
        result["config"]["collective_us_per_token"] = r.get("collective_us_per_token")
    if "p2p" in line["transports"]:
        result["config"]["p2p_transport"] = line["transports"]["p2p"]
    if p2p_state["error"]:
        result["config"]["p2p_transport"] = {"error": p2p_state["error"]}
    if args.config4_layers > 0 and world > 1:
        c4 = sharded_decode(gh, L, comm, comm_kind, rank, world, LLAMA13B, args.config4_layers, groups, args, stream,
                            allreduce, barrier, p2p_state, 0x5EEF0000, tokens_per=40)
        result["config4_llama13b_sharded"] = dict(
            {"config": f"LLaMA-13B q4_0 decode, weight rows sharded {world}-way + all-gather over xGMI (BASELINE "
                       "config 4): 40 layers x 7 mul_mats (5120x5120 x4, 5120->13824 x2, 13824->5120), 4 grouped "
                       "all-gathers per layer", "layers": args.config4_layers}, **c4)
    result["config"]["runtime_libs"] = gh.mapped_runtime_libs()
    return result


def sharded_decode(gh, L, comm, comm_kind, rank, world, spec, n_layers, groups, args, stream, allreduce, barrier,
                   p2p_state, seed_base, tokens_per=32):
    """One model's row-sharded decode: the split graph on each available transport (RCCL, P2P), the same
    shards without collectives (compute only), and the bitwise split self-check.  tok/s per full model
    (`tokens_per` layers), max over ranks of the timed region."""
    stack = Stack(gh, L, rank, world, n_layers, seed_base=seed_base, spec=spec)
    Ks = sorted({K for _, K, _ in spec})
    xs = {}
    for K in Ks:
        xs[K] = gh.DeviceBuffer(K * 4)
        gh.check(L.ggml_hip_fill_gaussian(xs[K].ptr, K, 0x5EED1000 + K, 0.0, 1.0, None))
    yb = {i: gh.DeviceBuffer(max(spec[i][2] // world + 1, 1) * 4 + 64) for i in range(len(spec))}
    ysplit = {i: gh.DeviceBuffer(spec[i][2] * 4) for i in range(len(spec))}     # full-M gathered outputs
    gh.synchronize()
    keep = []

    def build(use_comm):
        out = []
        for row in stack.mats:
            for g in groups:
                n = len(g)
                K = row[g[0]][1]
                if not use_comm:
                    wp = (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g])
                    yp = (ctypes.c_void_p * n)(*[yb[i].ptr for i in g])
                    mp = (ctypes.c_int64 * n)(*[row[i][3] for i in g])
                    keep.append((wp, yp, mp))
                    out.append(("multi", (n, wp, mp, K, yp)))
                else:                # split siblings: one GEMV launch + one grouped all-gather
                    wp = (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g])
                    mt = (ctypes.c_int64 * n)(*[row[i][2] for i in g])
                    rp = (ctypes.c_void_p * n)(*[row[i][5].ctypes.data for i in g])
                    yp = (ctypes.c_void_p * n)(*[ysplit[i].ptr for i in g])
                    keep.append((wp, mt, rp, yp))
                    out.append(("split_multi", (n, wp, mt, rp, K, yp)))
        return out

    split_args, local_args = build(True), build(False)

    def step(launch_args):
        for kind, a in launch_args:
            if kind == "multi":
                n, wp, mp, K, yp = a
                gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xs[K].ptr, 1, yp, stream))
            else:
                n, wp, mt, rp, K, yp = a
                gh.check(L.ggml_hip_mul_mat_q4_0_split_multi(comm, n, wp, mt, rp, K, xs[K].ptr, 1, yp, stream))

    def timed_graph(launch_args):
        step(launch_args)                    # outside capture first (workspaces, lazy init)
        gh.check(L.ggml_hip_stream_synchronize(stream))
        g = gh.Graph(stream)
        with g:
            step(launch_args)
        for _ in range(args.warmup):
            g.launch()
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.launch()
        barrier()
        el = allreduce([time.perf_counter() - t0], 1)[0]     # max over ranks
        del g
        return el

    el_local = timed_graph(local_args)
    tokens = tokens_per / n_layers
    out = {"weights_bytes_per_rank": stack.total_bytes,
           "compute_only_tok_s": round(args.steps / el_local * tokens, 2), "transports": {}}
    runs = []
    if comm_kind == "rccl":
        gh.check(L.ggml_hip_comm_set_transport(comm, 0))
        el = timed_graph(split_args)
        chk = split_check(gh, L, stack, ysplit, yb, rank, allreduce, stream)
        out["transports"]["rccl"] = {"tok_s": round(args.steps / el * tokens, 2),
                                     "ms_per_step": round(el / args.steps * 1e3, 4), "split_check": chk,
                                     "collective_us_per_token": round((el - el_local) / args.steps * 1e6 * tokens, 1)}
        runs.append(("rccl", el, chk, True))
    if p2p_state["on"]:
        gh.check(L.ggml_hip_comm_set_transport(comm, 1))
        try:
            # one eager step first: a transport that cannot run here (IPC, peer access) is reported, not timed;
            # a peer wait that times out fails the comm for good and the next split call raises, but every
            # rank still reaches the allreduce below (the waits are time-bounded)
            try:
                step(split_args)
                local_ok = True
            except gh.GgmlHipError as e:
                log(f"[rank {rank}] P2P step failed: {e}")
                local_ok = False
            gh.check(L.ggml_hip_device_synchronize(), "device synchronize")
            st = L.ggml_hip_comm_p2p_status(comm)
            if allreduce([float(st) if local_ok else 1.0], 1)[0] != 0.0:
                out["transports"]["p2p"] = {"error": f"peer waits failed (status {st}, this rank's step "
                                                     f"{'ok' if local_ok else 'failed'})"}
                p2p_state["on"] = False
            else:
                el = timed_graph(split_args)
                st = L.ggml_hip_comm_p2p_status(comm)
                ok = allreduce([float(st)], 1)[0] == 0.0
                chk = split_check(gh, L, stack, ysplit, yb, rank, allreduce, stream)
                out["transports"]["p2p"] = {"tok_s": round(args.steps / el * tokens, 2),
                                            "ms_per_step": round(el / args.steps * 1e3, 4), "status_ok": ok,
                                            "split_check": chk,
                                            "collective_us_per_token": round((el - el_local) / args.steps * 1e6 * tokens, 1)}
                runs.append(("p2p", el, chk, ok))
        finally:
            if comm_kind == "rccl":
                L.ggml_hip_comm_set_transport(comm, 0)
    # the faster transport whose run passed its own checks (bitwise own rows, gathered checksum, no
    # peer-wait failure); every transport's figures stay in the line
    good = [r for r in runs if r[3] and r[2]["own_rows_bitwise"] and r[2]["gather_checksum"]]
    best = min(good or runs, key=lambda r: r[1]) if runs else None
    if best is None:
        raise SystemExit(f"[rank {rank}] no all-gather transport ran")
    out["transport"] = {"rccl": "RCCL", "p2p": "direct-store P2P"}[best[0]]
    out["tok_s"] = round(args.steps / best[1] * tokens, 2)
    out["ms_per_step"] = round(best[1] / args.steps * 1e3, 4)
    out["split_check"] = best[2]
    out["self_checks_passed"] = bool(good)
    stack.free()
    return out


# ---------------------------------------------------------------------------------------------
def _bits_checksum(a, offset):
    """order-independent exact checksum of float32 values at global positions offset + i"""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64).ravel()
    pos = np.arange(offset, offset + u.size, dtype=np.uint64)
    return int(np.sum((u + np.uint64(1)) * (pos * np.uint64(2654435761) + np.uint64(97)), dtype=np.uint64))


def split_check(gh, L, stack, ysplit, yb, rank, allreduce, stream):
    """Self-check of the sharded run (after its timed region): the split step leaves the last layer's
    gathered outputs in ysplit and the local-only graph (run before it, same x) its slices in yb.  (1) this
    rank's rows of every gathered y equal its own slice bitwise; (2) the exact checksum of every gathered y
    equals the sum over ranks of the slice checksums (every rank's slice landed at its rows)."""
    MOD = 1 << 44                            # sums of <= 256 ranks stay exact in a double
    row = stack.mats[-1]
    ok_own, mine, full = True, [], []
    for i, (name, K, M, m_loc, buf, rb) in enumerate(row):
        g = ysplit[i].download((M,), np.float32, stream=stream)
        loc = yb[i].download((m_loc,), np.float32, stream=stream)
        lo = int(rb[rank])
        ok_own &= bool(np.array_equal(g[lo:lo + m_loc].view(np.uint32), loc.view(np.uint32)))
        mine.append(float(_bits_checksum(loc, lo) % MOD))
        full.append(_bits_checksum(g, 0) % MOD)
    tot = allreduce(mine, 0)
    ok_own = allreduce([1.0 if ok_own else 0.0], 2)[0] == 1.0
    ok_sum = all((fu - int(tt)) % MOD == 0 for fu, tt in zip(full, tot))
    return {"own_rows_bitwise": ok_own, "gather_checksum": ok_sum, "matrices": len(row)}


def newest_profile(suffix):
    """the newest round's committed profile with this suffix (profiles/rNN_<suffix>), or None"""
    fs = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith(suffix))
    return os.path.join(ROOT, "profiles", fs[-1]) if fs else None


def rocprof_stats(path):
    """{kernel name: (calls, total ns)} of a rocprofv3 --stats kernel summary (csv)"""
    import csv
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            out[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]))
    return out


def kernel_roofline(gh, L, launch_args, xs, stream, per_layer, ms_per_step, n_layers, engine_step_ms=None,
                    isolated=True, reps=10):
    """The decode roofline, priced on the TIMED step itself (verdict r5 item 5: the dominant kernel's time per step
    cannot exceed the step).  Every launch of a step is the decode GEMV (k_gemv_q4_0<1,...>): 4 sibling launches
    per layer, back to back (one HIP graph per token, or issued eagerly: the faster), so achieved = the step's algorithmic bytes / ms_per_step (the launch
    boundaries inside the step are charged to the GEMVs; avg_launch_us = step / launches).  Algorithmic bytes of a
    launch = sum over its matrices of 18*M*K/32 (q4_0) + 4*K (f32 x) + 4*M (f32 y).  Beside it:
      rocprof_check: from the newest committed rocprofv3 summary of this bench's own timed replays
        (profiles/rNN_bench_rocprofv3_kernel_stats.csv, tools/run.sh PARTS=prof): the GEMV kernels' busy
        time per step (total ns / (calls / launches per step)) <= ms_per_step, the rest being boundaries;
      per_shape_isolated: each launch position's 32 launches replayed in a graph of their own (the shape's own
        rate; their sum exceeds the step by the shape-mixing of the real sequence, so they are not the headline)."""
    launches = len(launch_args)
    step_bytes = 0
    for kind, a in launch_args:
        if kind == "multi":
            n, wp, mp, K, yp, _ = a
            Ms = [mp[i] for i in range(n)]
        else:
            K, Ms = a[1], [a[3]]
        step_bytes += sum(q4_bytes(K, M) + 4 * K + 4 * M for M in Ms)
    t_step = ms_per_step * 1e-3                              # one step = this run's n_layers layers
    achieved = step_bytes / t_step / 1e9
    traffic, src = None, None
    pmc = newest_profile("_gemv_pmc_traffic.json")
    if pmc:
        try:
            traffic = round(json.load(open(pmc))["traffic_bytes_per_launch_mean"])
            src = f"{os.path.relpath(pmc, ROOT)}: 2*FETCH_SIZE+WRITE_SIZE (x1024) per GEMV launch, mean"
        except Exception:
            traffic = None
    out = {"bound": "hbm", "kernel": "k_gemv_q4_0<NT=1,...> (fused q8_0 quantize + q4_0.q8_0 GEMV, one row item per wave "
                                     "ring slot), 4 sibling launches per layer",
           "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
           "traffic": traffic, "traffic_source": src,
           "algorithmic_bytes_per_launch_mean": round(step_bytes / launches), "algorithmic_bytes_per_step": step_bytes,
           "launches_per_step": launches, "avg_launch_us": round(t_step / launches * 1e6, 3),
           "timing": "the timed step: ms_per_step of the per-launch chain, graph or eager, the faster (barrier + synchronize around `steps` steps)",
           "bytes_per_launch_def": "sum over the launch's matrices of 18*M*K/32 (q4_0) + 4*K (f32 x) + 4*M (f32 y)"}
    prof = newest_profile("_bench_rocprofv3_kernel_stats.csv")
    if prof:
        try:
            st = rocprof_stats(prof)
            calls = sum(c for k, (c, _) in st.items() if "k_gemv_q4_0<1," in k)
            ns = sum(t for k, (c, t) in st.items() if "k_gemv_q4_0<1," in k)
            steps_seen = calls / launches if launches else 0
            busy = ns / steps_seen / 1e3 if steps_seen else None      # us per step
            out["rocprof_check"] = {"source": os.path.relpath(prof, ROOT), "gemv_calls": calls,
                                    "gemv_busy_us_per_step": round(busy, 1) if busy else None,
                                    "gemv_avg_us": round(ns / calls / 1e3, 3) if calls else None,
                                    "ms_per_step_us": round(t_step * 1e6, 1),
                                    "busy_le_step": bool(busy is not None and busy <= t_step * 1e6),
                                    "kernel_only_GBps": round(step_bytes / (busy * 1e-6) / 1e9, 1) if busy else None}
            # the tracer's own effect: it separates dispatches by tens of us, so every GEMV starts on an idle GPU
            # (no overlap with the previous kernel's drain); the one-launch engine has no such boundaries and is
            # the calibration (its traced average against its untraced step in this run)
            eng = [(c, t) for k, (c, t) in st.items() if "k_engine_q4_0" in k]
            if eng and engine_step_ms:
                traced = eng[0][1] / eng[0][0] / 1e3
                out["rocprof_check"]["engine_traced_avg_us"] = round(traced, 1)
                out["rocprof_check"]["engine_untraced_step_us"] = round(engine_step_ms * 1e3, 1)
            # the same check inside the traced run (tools/trace_steps.py): its own step, and the device span of its
            # gap-free 128-launch windows against their summed durations
            sp = newest_profile("_bench_rocprofv3_step_spans.json")
            if sp and busy:
                j = json.load(open(sp))
                rc = out["rocprof_check"]
                rc["spans_source"] = os.path.relpath(sp, ROOT)
                if j.get("traced_ms_per_step"):
                    rc["traced_step_us"] = round(j["traced_ms_per_step"] * 1e3, 1)
                    rc["busy_le_traced_step"] = bool(busy <= j["traced_ms_per_step"] * 1e3)
                gf = j.get("gap_free")
                if gf:
                    rc["device_bound_windows"] = j["gap_free_windows"]
                    rc["window_sum_us_median"] = gf["sum_us_median"]
                    rc["window_span_us_median"] = gf["span_us_median"]
                    rc["window_sum_le_span"] = bool(gf["sum_us_median"] <= gf["span_us_median"])
                rc["note"] = ("busy_le_step compares traced kernel durations with the UNtraced step; the tracer "
                              "stamps every dispatch and its durations run ~2-5 % long, so the like-for-like checks "
                              "are busy_le_traced_step and window_sum_le_span (both inside the traced run)")
        except Exception as e:       # a malformed summary must not cost the line
            out["rocprof_check"] = {"source": os.path.relpath(prof, ROOT), "error": str(e)}
    if engine_step_ms is not None:
        te = engine_step_ms * 1e-3
        out["engine"] = {"kernel": "k_engine_q4_0 (one launch per step)", "achieved": round(step_bytes / te / 1e9, 1),
                         "frac": round(step_bytes / te / 1e9 / HBM_PEAK_GBPS, 4)}
    if not isolated:
        return out
    shapes = {}
    for pos in range(per_layer):
        sel = launch_args[pos::per_layer]
        g = gh.Graph(stream)
        with g:
            for kind, a in sel:
                run_launch(gh, L, kind, a, xs, stream)
        g.launch()
        gh.check(L.ggml_hip_stream_synchronize(stream))
        e0, e1 = gh.Event(), gh.Event()
        e0.record(stream)
        for _ in range(reps):
            g.launch()
        e1.record(stream)
        t = e0.elapsed_ms(e1) * 1e-3 / (reps * len(sel))
        kind, a = sel[0]
        if kind == "multi":
            n, wp, mp, K, yp, _ = a
            Ms = [mp[i] for i in range(n)]
        else:
            K, Ms = a[1], [a[3]]
        nbytes = sum(q4_bytes(K, M) + 4 * K + 4 * M for M in Ms)
        shapes[f"K{K}->M{'+'.join(map(str, Ms))}"] = {"us": round(t * 1e6, 3), "GBps": round(nbytes / t / 1e9, 1),
                                                       "bytes": nbytes}
    out["per_shape_isolated"] = shapes
    return out


def engine_decode(gh, L, launch_args, yb, outs_launches, stream, timed):
    """The same decode chain (the bench's 128 launches per token with their real data dependencies) on the
    persistent LDS-DMA engine: one launch per token (q4_0_engine.hip).  Timed like the per-launch graph
    (barrier + synchronize around `steps` replays of a graph holding the one launch); self-check: every
    output of the last layer bitwise equal to the per-launch graph's (same weights, same input)."""
    tasks = []
    for kind, a in launch_args:
        if kind == "multi":
            n, wp, mp, K, yp, xp = a
            tasks.append(([wp[i] for i in range(n)], [mp[i] for i in range(n)], K, xp, [yp[i] for i in range(n)]))
        else:
            name, K, M, m_loc, buf, rb, ylocal, _, xp = a
            tasks.append(([buf.ptr], [m_loc], K, xp, [ylocal.ptr]))
    ch = gh.Chain(tasks)
    on = ch.set_engine(1)
    out = {"on": bool(on)}
    if not on:
        out["declined"] = L.ggml_hip_last_error().decode(errors="replace")
        return out
    for i in range(len(outs_launches)):          # the engine must write every output itself
        gh.check(L.ggml_hip_memset(yb[i].ptr, 0xFF, outs_launches[i].size * 4, stream))
    ch.launch(stream)
    gh.check(L.ggml_hip_stream_synchronize(stream))
    g = gh.Graph(stream)
    with g:
        ch.launch(stream)
    el = timed(g.launch)
    st = ch.status()
    same = all(np.array_equal(yb[i].download((o.size,), np.float32, stream=stream).view(np.uint32), o.view(np.uint32))
               for i, o in enumerate(outs_launches))
    info = ch.engine_info()
    out.update({"elapsed_s": el, "status": st, "bitwise_vs_launches": bool(same), "units": info["units"],
                "cus": info["cus"], "max_cu_stream_bytes": info["max_stream_bytes"],
                "weight_bytes": info["weight_bytes"],
                "structure": "per CU: 1 loader wave (global_load_lds_dwordx4, 40 x 1 KiB in flight, 128 KiB LDS ring) + "
                             "4 consumer waves (the decode GEMV's per-row arithmetic); edges = q8_0 granules "
                             "quantized once by the producing CU, swept by one consumer wave per CU"})
    if st != 0:
        out["error"] = L.ggml_hip_last_error().decode(errors="replace")
    del g
    return out


def exact_decode(gh, L, decode_step, stream, args):
    """The headline decode graph re-captured in exact mode (ggml_hip_set_exact): every mul_mat runs
    algorithm 4, bit-identical to the reference's AVX2 ggml_vec_dot_q4_0_q8_0 (tests/test_gpu_exact.py)."""
    prev = L.ggml_hip_get_exact()
    gh.check(L.ggml_hip_set_exact(1))
    try:
        decode_step()
        gh.check(L.ggml_hip_stream_synchronize(stream))
        g = gh.Graph(stream)
        with g:
            decode_step()
        for _ in range(args.warmup):
            g.launch()
        gh.check(L.ggml_hip_stream_synchronize(stream))
        a, b = gh.Event(), gh.Event()
        a.record(stream)
        for _ in range(args.steps):
            g.launch()
        b.record(stream)
        t = a.elapsed_ms(b) * 1e-3 / args.steps * 32 / args.layers
        del g
    finally:
        L.ggml_hip_set_exact(prev)
    return {"tok_s": round(1.0 / t, 2), "ms_per_token": round(t * 1e3, 4),
            "numerics": "every y bit-identical to the reference's AVX2 ggml_vec_dot_q4_0_q8_0 (algo 4)"}


def extra_decode(gh, L, stream, name, n_layers, spec, groups, steps=20, warmup=5):
    """Decode tok/s of another model's q4_0 matmul stack on this GPU: same graph-replayed launch
    chain as the headline (siblings batched), distinct weights per layer (> Infinity Cache)."""
    stack = Stack(gh, L, 0, 1, n_layers, seed_base=0x5EEE0000, spec=spec)
    Ks = sorted({K for _, K, _ in spec})
    xs = {K: gh.DeviceBuffer(K * 4) for K in Ks}
    for K in Ks:
        gh.check(L.ggml_hip_fill_gaussian(xs[K].ptr, K, 0x5EED1000 + K, 0.0, 1.0, None))
    yb = {i: gh.DeviceBuffer(spec[i][2] * 4) for i in range(len(spec))}
    keep = []

    def step():
        for row in stack.mats:
            for g in groups:
                n = len(g)
                wp = (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g])
                yp = (ctypes.c_void_p * n)(*[yb[i].ptr for i in g])
                mp = (ctypes.c_int64 * n)(*[row[i][3] for i in g])
                keep.append((wp, yp, mp))
                gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, row[g[0]][1], xs[row[g[0]][1]].ptr, 1, yp, stream))
    step()
    gh.check(L.ggml_hip_stream_synchronize(stream))
    g = gh.Graph(stream)
    with g:
        step()
    for _ in range(warmup):
        g.launch()
    gh.check(L.ggml_hip_stream_synchronize(stream))
    a, b = gh.Event(), gh.Event()
    a.record(stream)
    for _ in range(steps):
        g.launch()
    b.record(stream)
    t = a.elapsed_ms(b) * 1e-3 / steps
    nbytes = n_layers * sum(q4_bytes(K, M) + 4 * K + 4 * M for _, K, M in spec)
    del g
    for buf in stack.bufs:
        buf.free()
    return {"config": name, "tok_s": round(1.0 / t, 2), "ms_per_token": round(t * 1e3, 4),
            "weights_bytes": stack.total_bytes, "launches_per_layer": len(groups),
            "GBps": round(nbytes / t / 1e9, 1), "hbm_frac": round(nbytes / t / 1e9 / HBM_PEAK_GBPS, 4)}


def run_launch(gh, L, kind, a, xs, stream):
    if kind == "multi":
        n, wp, mp, K, yp, _ = a
        gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xs[K].ptr, 1, yp, stream))
    else:
        name, K, M, m_loc, buf, rb, yb, _, _ = a
        gh.check(L.ggml_hip_mul_mat_q4_0_ex(buf.ptr, K, m_loc, xs[K].ptr, 1, yb.ptr, m_loc, 1, stream))


SETTLE_PASSES = 60       # prefill: back-to-back passes before the first timed one (~65 ms of load)


def prefill_bench(gh, L, stack, xs, ys, stream, N, layers=4, reps=10, warm=3, groups=((0, 1, 2), (3,), (4, 5), (6,))):
    """N-token prefill through `layers` layers of the stack (7 mul_mats each), sibling groups as in decode
    (wq|wk|wv and w1|w3 share src1: one launch per group, ggml_hip_mul_mat_q4_0_multi's grouping).
    Headline: the layers as ONE dependent chain (ggml_hip_chain_create_n), the decode's data dependencies at N
    tokens: wq|wk|wv read the previous layer's w2 output (layer 0: a fixed N x 4096 input), wo reads q, w1|w3
    read wo's output, w2 reads w1's output (verdict r5 item 6); each task's fp6 x image by k_prep9_x.  Beside
    it: the same chain with each k_gemm9 epilogue writing the next launch's x image (opt-in: bitwise the same,
    measured slower), and the round-5 figure (each group on a fixed input x).  GB/s = (W + 4KN + 4MN) / t
    (SURVEY.md §8d config 3)."""
    mats = [m for row in stack.mats[:layers] for m in row]
    ybuf = {}
    calls = []
    for row in stack.mats[:layers]:
        for g in groups:
            K = row[g[0]][1]
            n = len(g)
            for i in g:                                  # one output per sibling (distinct buffers)
                ybuf.setdefault(i, gh.DeviceBuffer(row[i][3] * 4 * N))
            wp = (ctypes.c_void_p * n)(*[row[i][4].ptr for i in g])
            mp = (ctypes.c_int64 * n)(*[row[i][3] for i in g])
            yp = (ctypes.c_void_p * n)(*[ybuf[i].ptr for i in g])
            calls.append((n, wp, mp, K, yp))
    # the dependent chain: the group's x = the y of the group's producer (DEP by the group's first matrix)
    DEP = {0: 6, 3: 0, 4: 3, 6: 4}
    chain_tasks = []
    for li, row in enumerate(stack.mats[:layers]):
        for g in groups:
            K = row[g[0]][1]
            x = xs[K].ptr if (li == 0 and g[0] == 0) else ybuf[DEP[g[0]]].ptr
            chain_tasks.append(([row[i][4].ptr for i in g], [row[i][3] for i in g], K, x, [ybuf[i].ptr for i in g]))

    def run():
        for n, wp, mp, K, yp in calls:
            gh.check(L.ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xs[K].ptr, N, yp, stream))

    def timed(fn=run):
        for _ in range(warm):           # clocks and TLBs settle over the first passes (tools/prefill_chain_ab.py)
            fn()
        gh.check(L.ggml_hip_stream_synchronize(stream))
        a, b = gh.Event(), gh.Event()
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        return a.elapsed_ms(b) * 1e-3 / reps

    nbytes = sum(q4_bytes(K, m) + 4 * K * N + 4 * m * N for _, K, M, m, _, _ in mats)
    ops = sum(2 * K * m * N for _, K, M, m, _, _ in mats)
    chain = {}

    def chain_timed():
        ch = gh.Chain(chain_tasks, N=N)
        chain["epilogue_links"] = ch.engine_info()["epilogue_images"]
        go = lambda: ch.launch(stream)
        # sustained load first: the clocks settle only after ~25 ms of back-to-back passes (the first of
        # tools/prefill_chain_ab.py's interleaved rounds runs up to 15 % slow), then the two chain forms
        # interleaved twice, best of each
        for _ in range(SETTLE_PASSES):
            go()
            gh.check(L.ggml_hip_stream_synchronize(stream))
        t_prep, t_fold = [], []
        try:
            for _ in range(2):
                gh.check(L.ggml_hip_debug_set_chain_x9(0))         # the default: every x image by k_prep9_x
                t_prep.append(timed(go))
                last_prep = ybuf[6].download((N, 4096), np.float32, stream)
                gh.check(L.ggml_hip_debug_set_chain_x9(1))         # opt-in: the producers' epilogues write them
                t_fold.append(timed(go))
                last = ybuf[6].download((N, 4096), np.float32, stream)
        finally:
            gh.check(L.ggml_hip_debug_set_chain_x9(-1))
        chain["t_fold"] = min(t_fold)
        chain["bitwise_fold_vs_prep"] = bool(np.array_equal(last.view(np.uint32), last_prep.view(np.uint32)))
        chain["t_indep"] = timed(run)
        del ch
        return min(t_prep)

    # default path: each weight's image built once, as the hook does on a resident weight's first
    # prefill (ggml_hip_weight_image_create): fp6 images + k_gemm9 (GEMM version 10, the
    # default); for comparison the int8 images + k_gemm8 (version 8) and no image (k_gemm7 on the q4_0
    # bytes in place), both on the fixed-input groups
    def with_images(version, fn):
        gh.check(L.ggml_hip_debug_set_gemm_version(version))
        try:
            for _, K, M, m, buf, _ in mats:
                gh.check(L.ggml_hip_weight_image_create(buf.ptr, K, m, stream))
            nbytes_img = L.ggml_hip_weight_image_bytes()
            try:
                return fn(), nbytes_img
            finally:
                for _, K, M, m, buf, _ in mats:
                    L.ggml_hip_weight_image_free(buf.ptr)
        finally:
            gh.check(L.ggml_hip_debug_set_gemm_version(-1))

    t, image_bytes = with_images(10, chain_timed)
    t8, image_bytes8 = with_images(8, timed)
    t7 = timed()                                      # no images: k_gemm7 on the q4_0 bytes in place

    def alt(kernel, tt):
        return {"kernel": kernel, "ms_per_layer": round(tt / layers * 1e3, 4), "TOPs": round(ops / tt / 1e12, 1),
                "mfma_frac": round(ops / tt / 1e12 / INT8_PEAK_TOPS, 4)}
    # the prefill GEMM's own roofline (verdict r5 item 5): its instruction and that instruction's peak, named.
    # v_mfma_scale_f32_32x32x64_f8f6f4 with e2m3 operands runs at ~10 PF dense (MI355X_MICROARCH.md, FP6 row);
    # k_gemm9 puts each q8_0 value into it as TWO e2m3 digits (q = 16 (q >> 4) + (q & 15), one per K half), so
    # one instruction advances the algorithm's K by 32, not 64: the effective peak of 2*M*K*N is 5 POP/s.
    # achieved = 2*M*K*N over the dependent layer chain (its x image preps included); kernel_only from the
    # newest committed rocprofv3 summary of this bench (k_gemm9* durations of the fp6 passes: `warm` + `reps`
    # of the chain, then the same of the chain with the epilogue fold and of the fixed-input groups)
    roof = {"bound": "mfma", "kernel": "k_gemm9_q4_0 / k_gemm9w_q4_0",
            "instruction": "v_mfma_scale_f32_32x32x64_f8f6f4 (e2m3 x e2m3, block scales 2^1 / 2^5)",
            "instruction_peak": 10000.0, "effective_peak": 5000.0, "unit": "TOP/s",
            "peak_note": "10 PF fp6 dense; two e2m3 digits per q8_0 value -> 5 POP/s of the algorithm's 2*M*K*N",
            "achieved": round(ops / t / 1e12, 1), "frac": round(ops / t / 1e12 / 5000.0, 4),
            "timing": "the 4-layer dependent prefill chain (HIP events over `reps` passes after `warm`), x image preps included"}
    prof = newest_profile("_bench_rocprofv3_kernel_stats.csv")
    if prof:
        try:
            st = rocprof_stats(prof)
            g9 = sum(tt_ for k, (c, tt_) in st.items() if "k_gemm9" in k)
            if g9 > 0:
                passes = SETTLE_PASSES + 5 * (reps + warm)   # every pass of the stack on k_gemm9 in this bench
                roof["kernel_only_TOPs"] = round(ops * passes / (g9 * 1e-9) / 1e12, 1)
                roof["kernel_only_frac"] = round(ops * passes / (g9 * 1e-9) / 1e12 / 5000.0, 4)
                roof["kernel_only_source"] = (f"{os.path.relpath(prof, ROOT)}: sum of k_gemm9* durations over the "
                                              f"{passes} passes of the 4-layer stack in this bench (the chain with and "
                                              "without the epilogue fold, the fixed-input groups)")
        except Exception as e:
            roof["kernel_only_error"] = str(e)
    return {"tokens": N, "layers": layers, "ms_per_layer": round(t / layers * 1e3, 4), "roofline": roof,
            "GBps": round(nbytes / t / 1e9, 1), "TOPs": round(ops / t / 1e12, 1),
            "mfma_frac": round(ops / t / 1e12 / INT8_PEAK_TOPS, 4), "peak_TOPs": INT8_PEAK_TOPS,
            "stack_7B_prefill_ms": round(t / layers * 32 * 1e3, 3),
            "dependency": ("one dependent chain (ggml_hip_chain_create_n): wq|wk|wv <- previous w2 (layer 0: fixed "
                           "N x 4096 input), wo <- wq, w1|w3 <- wo, w2 <- w1; each task's fp6 x image by k_prep9_x "
                           "from its producer's y (the default; the epilogue fold below is opt-in)"),
            "chain_epilogue_images": dict(alt("the same chain, each k_gemm9 epilogue writing the next launch's x image "
                                              f"({chain.get('epilogue_links')} of {len(chain_tasks)} tasks; "
                                              "ggml_hip_debug_set_chain_x9(1))", chain["t_fold"]),
                                          bitwise_vs_default=chain.get("bitwise_fold_vs_prep")),
            "kernel": "k_gemm9_q4_0 / k_gemm9w_q4_0: exact block sums on the block-scaled fp6 MFMA, 128x64 or "
                      "128x128 workgroup tiles chosen per launch by rounds of CUs, per-weight e2m3 images built "
                      f"once (26 B per 32 weights; image bytes {image_bytes} for {layers} layers)",
            "independent_x": alt("each group on a fixed input x, one k_prep9_x per group (the round-5 figure)",
                                 chain["t_indep"]),
            "int8_images": alt("k_gemm8_q4_0: i8 MFMA on per-weight int8 images, fixed-input groups (34 B per 32 "
                               f"weights; image bytes {image_bytes8})", t8),
            "q4_0_in_place": alt("k_gemm7_q4_0 (no image: the q4_0 blocks read in place), fixed-input groups", t7)}


def _cpu_name():
    import platform
    cpu = platform.processor() or "x86_64"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def _cpu_flags():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                return set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return set()


def _stats(vals):
    v = np.asarray(vals, np.float64)
    return {"median": float(np.median(v)), "min": float(v.min()), "max": float(v.max()), "n": int(v.size)}


def _loadavg():
    try:
        return float(open("/proc/loadavg").read().split()[0])
    except (OSError, ValueError, IndexError):
        return None


def _cg_throttled():
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            if line.startswith("throttled_usec"):
                return int(line.split()[1])
    except (OSError, ValueError, IndexError):
        pass
    return None


def _cpu_share():
    """P for the CPU baseline: BASELINE.md §3 asks for the physical cores of one socket; a job on the GPU
    box runs under a CPU quota (cgroup cpu.max / affinity / OMP_NUM_THREADS, 16 for one GPU), and
    threads beyond the quota only time-slice, so P = min(cores per socket, quota), both reported."""
    per_socket = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("cpu cores"):
                per_socket = int(line.split(":")[1])
                break
    except OSError:
        pass
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit() else None
    limits = {k: v for k, v in (("cgroup_cpu_max", quota), ("affinity", affinity), ("OMP_NUM_THREADS", omp)) if v}
    cap = min(limits.values()) if limits else (os.cpu_count() or 1)
    P = min(per_socket or cap, cap)
    binding = min(limits, key=limits.get) if limits and cap < (per_socket or cap + 1) else "cores_per_socket"
    lim = ", ".join(f"{k}={v}" for k, v in limits.items())
    rule = (f"P = min(physical cores per socket {per_socket}, this job's CPU limit {cap} ({lim}))"
            if per_socket else f"P = this job's CPU limit {cap} ({lim})")
    return {"P": P, "cores_per_socket": per_socket, "limits": limits, "binding": binding, "rule": rule}


def cpu_baseline(budget_s):
    """CPU path timed beside the GPU path on this host.

    kind "reference": the reference's own ggml.c (oracle/_ref, compiled from /root/reference by
    oracle/Makefile): the "native" build (AVX-512 + AVX-VNNI: ggml.c's __AVXVNNI__ dpbusd branch,
    what -march=native selects on the EPYC host) when the host has those extensions, else the AVX2
    build (-march=x86-64-v3).  Decode = the 7 q4_0 mul_mats of a LLaMA-7B layer over 6 rotating layer
    copies (> LLC), one ggml graph per pass as llama.cpp computes one graph per token (threads spawned
    once per graph compute, ggml.c:17540-17571), tok/s = 1 / (32 x layer time), at P threads (P = this
    process's CPU share) and at 1 thread; plus the spawn-per-mul_mat form (one graph per mul_mat), the
    persistent-pool form (the oracle's AVX2 restatement of the same path, kind "port"), a 512-token
    prefill layer, and BASELINE config 1 (test-quantize-perf q4_0 vec_dot over 4096 x 4096 values, one
    thread).  Median / min / max over the samples.  kind "port" only when oracle/_ref was not built."""
    share = _cpu_share()
    P = int(os.environ.get("CPU_BASELINE_THREADS", share["P"]))
    n_copies = 6                                   # ~680 MB of weights: beyond any host LLC
    flags = _cpu_flags()
    native_ok = {"avx512f", "avx512bw", "avx512vl", "avx_vnni"} <= flags
    ref_dir = os.path.join(ROOT, "oracle", "_ref")
    ref_so = os.path.join(ref_dir, "libref_bench_native.so" if native_ok else "libref_bench.so")
    if not (os.path.exists(ref_so) and os.environ.get("CPU_BASELINE_KIND", "reference") == "reference"):
        return cpu_baseline_port(budget_s, P, n_copies)
    R = ctypes.CDLL(ref_so)
    R.ref_layers_create.restype = ctypes.c_void_p
    R.ref_layers_create.argtypes = [ctypes.c_int, ctypes.c_int]
    for fn in (R.ref_layer_run, R.ref_stack_run):
        fn.restype = ctypes.c_double
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    R.ref_layers_destroy.argtypes = [ctypes.c_void_p, ctypes.c_int]
    R.ref_vec_dot_bench.restype = ctypes.c_float
    R.ref_vec_dot_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    t_start = time.time()

    def samples(run, sample_s, n_min, n_max, budget):
        """per-layer seconds of >= n_min samples of >= sample_s each, within budget seconds"""
        out, t0 = [], time.time()
        while len(out) < n_max and (len(out) < n_min or time.time() - t0 < budget):
            tot, layers = 0.0, 0
            while tot < sample_s or layers == 0:
                dt, nl = run()
                tot += dt
                layers += nl
            out.append(tot / layers)
        return out

    h = R.ref_layers_create(n_copies, 1)
    R.ref_stack_run(h, n_copies, P)              # warm: page in every layer copy
    load0, thr0 = _loadavg(), _cg_throttled()
    r0, w0 = os.times(), time.perf_counter()
    dec_p = samples(lambda: (R.ref_stack_run(h, n_copies, P), n_copies), 0.8, 5, 12, 0.45 * budget_s)
    r1, w1 = os.times(), time.perf_counter()
    load1, thr1 = _loadavg(), _cg_throttled()
    host_load = {
        "loadavg_1m_before": load0, "loadavg_1m_after": load1, "host_cpus": os.cpu_count(),
        # CPU time this process got during the P-thread samples / (wall x P): < 1 when its threads waited
        "cpu_utilisation_of_P": round(((r1.user - r0.user) + (r1.system - r0.system)) / max(1e-9, (w1 - w0) * P), 3),
        "cgroup_throttled_usec": (thr1 - thr0) if thr0 is not None and thr1 is not None else None,
        "note": "the box's host is shared with other jobs: compare CPU numbers across runs with these fields"}
    dec_1 = samples(lambda: (R.ref_stack_run(h, n_copies, 1), n_copies), 0.2, 3, 5, 0.08 * budget_s)
    k = [0]

    def per_call():
        k[0] += 1
        return R.ref_layer_run(h, k[0] % n_copies, P), 1
    dec_spawn = samples(per_call, 0.3, 3, 5, 0.1 * budget_s)
    R.ref_layers_destroy(h, n_copies)
    hp = R.ref_layers_create(1, 512)
    R.ref_stack_run(hp, 1, P)
    pre = samples(lambda: (R.ref_stack_run(hp, 1, P), 1), 0.0, 3, 3, 0.0)
    R.ref_layers_destroy(hp, 1)
    vd = np.zeros(20, np.float64)
    R.ref_vec_dot_bench(4096 * 4096, vd.size, vd.ctypes.data_as(ctypes.c_void_p))
    pool = cpu_baseline_port(0.1 * budget_s, P, 2, pool=True, n_min=3)

    def tok(t):
        return 1.0 / (32 * t)
    dP, d1, dS = _stats(dec_p), _stats(dec_1), _stats(dec_spawn)
    pre_s = _stats(pre)
    pre_ops = 2 * 512 * sum(K * M for _, K, M in LAYER)
    vd_s = _stats(vd)
    build = ("-march=x86-64-v4 -mavxvnni (AVX-512 + AVX-VNNI: the __AVXVNNI__ dpbusd branch of ggml.c:647-657; "
             "the host's -march=native set)" if native_ok else
             "-march=x86-64-v3 (AVX2/FMA/F16C branches; the host lacks AVX-512/AVX-VNNI)")
    return {
        "value": round(tok(dP["median"]), 3), "unit": "tok/s", "cores": P, "kind": "reference",
        "value_min": round(tok(dP["max"]), 3), "value_max": round(tok(dP["min"]), 3), "host_load": host_load,
        "sample": (f"LLaMA-7B decode layers (7 q4_0 mul_mats, N=1) over {n_copies} rotating layer copies through the "
                   f"reference ggml.c (oracle/_ref, {build}); one ggml graph per pass, one ggml_graph_compute with "
                   f"{P} threads ({share['rule']}); {dP['n']} samples of >= 0.8 s, median; "
                   f"tok/s = 1/(32 x layer time)"),
        "cpu": _cpu_name(), "host_cpus": os.cpu_count(), "build": build, "cpu_share": share,
        "decode": {
            "threads_P": {"threads": P, "tok_s_median": round(tok(dP["median"]), 3),
                          "tok_s_min": round(tok(dP["max"]), 3), "tok_s_max": round(tok(dP["min"]), 3),
                          "ms_per_layer": round(dP["median"] * 1e3, 4), "samples": dP["n"]},
            "threads_1": {"threads": 1, "tok_s_median": round(tok(d1["median"]), 3),
                          "tok_s_min": round(tok(d1["max"]), 3), "tok_s_max": round(tok(d1["min"]), 3),
                          "ms_per_layer": round(d1["median"] * 1e3, 4), "samples": d1["n"]},
            "spawn_per_mul_mat_P": {"threads": P, "tok_s": round(tok(dS["median"]), 3),
                                    "ms_per_layer": round(dS["median"] * 1e3, 4), "samples": dS["n"],
                                    "note": "one ggml graph (one thread spawn) per mul_mat, ggml.c:17540-17571"},
            "persistent_pool_P": pool,
        },
        "prefill_512": {"threads": P, "ms_per_layer": round(pre_s["median"] * 1e3, 2),
                        "TOPs": round(pre_ops / pre_s["median"] / 1e12, 4),
                        "stack_7B_ms": round(pre_s["median"] * 32 * 1e3, 1), "samples": pre_s["n"]},
        "config1_vec_dot_4096x4096": {
            "threads": 1, "us": round(vd_s["median"] * 1e6, 1), "us_min": round(vd_s["min"] * 1e6, 1),
            "q4_0_GiB_s": round(4096 * 4096 // 32 * 18 / vd_s["min"] / 2**30, 3),
            "ns_per_32_values": round(vd_s["min"] / (4096 * 4096 / 32) * 1e9, 3),
            "note": "tests/test-quantize-perf.cpp --type q4_0 --op vec_dot_q --size 16777216; GiB/s of the q4_0 "
                    "operand at the fastest of 20 calls, as that test reports"},
        "seconds": round(time.time() - t_start, 1),
    }


def cpu_baseline_port(budget_s, nthreads, n_copies, pool=False, n_min=1):
    """The oracle's AVX2 restatement of the same path (kind "port"): per mul_mat the q8_0 quantize
    and the row-split vec_dot, threads spawned per call (ggml.c:17540-17571) or, with pool, a
    persistent pool."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    base = []
    for mi, (name, K, M) in enumerate(LAYER):
        wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED0000 + mi, 0.0, 0.02).reshape(M, K))
        base.append((K, wq))
    layers = [[(K, wq.copy()) for K, wq in base] for _ in range(n_copies)]
    x = {K: O.gaussian(K, 0x5EED1000 + K, 0.0, 1.0).reshape(1, K) for K in (4096, 11008)}
    O.mul_mat(base[0][1], 4096, x[4096], nthreads=nthreads, mode="avx2", pool=pool)   # warm
    per = []
    t_all = time.perf_counter()
    while len(per) < n_min or time.perf_counter() - t_all < budget_s:
        t0 = time.perf_counter()
        for K, wq in layers[len(per) % n_copies]:
            O.mul_mat(wq, K, x[K], nthreads=nthreads, mode="avx2", pool=pool)
        per.append(time.perf_counter() - t0)
    st = _stats(per)
    note = (f"oracle AVX2 restatement of quantize_row_q8_0 + ggml_vec_dot_q4_0_q8_0 + the row split, "
            f"{nthreads} threads {'in a persistent pool' if pool else 'spawned per mul_mat'}, "
            f"AVX2={bool(O.lib().oracle_have_avx2())}")
    if pool:
        return {"threads": nthreads, "tok_s": round(1.0 / (32 * st["median"]), 3),
                "ms_per_layer": round(st["median"] * 1e3, 4), "samples": st["n"], "kind": "port", "note": note}
    return {"value": round(1.0 / (32 * st["median"]), 3), "unit": "tok/s", "cores": nthreads, "kind": "port",
            "ms_per_layer": round(st["median"] * 1e3, 4), "samples": st["n"], "sample": note, "cpu": _cpu_name()}


if __name__ == "__main__":
    main()
