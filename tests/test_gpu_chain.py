"""Decode chains (ggml_hip_chain_*): a sequence of dependent N = 1 q4_0 mul_mats as one persistent
launch, against the same mul_mats launched one by one (stream order) and against the oracle.

Bar: bitwise equal to separate ggml_hip_mul_mat_q4_0_multi calls (the chain runs the same per-row
arithmetic), every dependency honoured (task t's x is an earlier task's y, re-randomised between
launches so a stale read shows), oracle within the north-star bound (tests/parity.py).
"""
import ctypes

import numpy as np
import pytest

import oracle as O
from hip_env import ggml_hip, gpu_available
from parity import block_terms, check_y

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer


def dev_weights(K, M, seed):
    L = ggml_hip.load()
    tmp = DB(K * M * 4)
    w = DB(18 * K // 32 * M)
    ggml_hip.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, seed, 0.0, 0.02, None))
    ggml_hip.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, w.ptr, None))
    tmp.free()
    return w


class ChainCase:
    """spec: list of (K, [M...], src) with src = index of an earlier task whose first output feeds
    x (its first K values), or None for an independent input buffer."""

    def __init__(self, spec, seed=0):
        self.spec = spec
        self.w = [[dev_weights(K, M, 0x7000 + seed * 97 + 8 * t + i) for i, M in enumerate(Ms)]
                  for t, (K, Ms, _) in enumerate(spec)]
        self.sets = [self._buffers() for _ in range(2)]      # [0] chain, [1] one launch per task

    def _buffers(self):
        ys = [[DB(M * 4) for M in Ms] for (_, Ms, _) in self.spec]
        xs = []
        for t, (K, Ms, src) in enumerate(self.spec):
            if src is None:
                xs.append(DB(K * 4))
            else:
                assert self.spec[src][1][0] >= K and src < t
                xs.append(ys[src][0])
        return xs, ys

    def randomize(self, seed):
        for xs, _ in self.sets:
            for t, (K, _, src) in enumerate(self.spec):
                if src is None:
                    ggml_hip.check(ggml_hip.load().ggml_hip_fill_gaussian(xs[t].ptr, K, 0x9000 + seed * 131 + t,
                                                                         0.0, 1.0, None))
        ggml_hip.synchronize()

    def tasks(self, which=0):
        xs, ys = self.sets[which]
        return [(self.w[t], Ms, K, xs[t], ys[t]) for t, (K, Ms, _) in enumerate(self.spec)]

    def run_separate(self):
        for ws, Ms, K, x, ys in self.tasks(1):
            ggml_hip.mul_mat_multi(ws, Ms, K, x, 1, ys)
        ggml_hip.synchronize()

    def outputs(self, which):
        _, ys = self.sets[which]
        return [[y.download((M,), np.float32) for y, M in zip(yt, Ms)] for yt, (_, Ms, _) in zip(ys, self.spec)]


def assert_bitwise(a, b):
    for t, (ya, yb) in enumerate(zip(a, b)):
        for i, (u, v) in enumerate(zip(ya, yb)):
            assert np.array_equal(u.view(np.uint32), v.view(np.uint32)), f"task {t} matrix {i} differs"


def llama_layers(n, K=4096, F=11008, src0=None):
    spec = []
    prev = src0
    for _ in range(n):
        q = len(spec)
        spec.append((K, [K, K, K], prev))              # wq | wk | wv
        spec.append((K, [K], q))                       # wo  (x = q output)
        spec.append((K, [F, F], q + 1))                # w1 | w3
        spec.append((F, [K], q + 2))                   # w2  (x = w1 output)
        prev = q + 3
    return spec


def test_chain_llama7b_two_layers_bitwise():
    c = ChainCase(llama_layers(2))
    ch = ggml_hip.Chain(c.tasks(0))
    for rep in range(3):                               # fresh x each launch: stale reads would show
        c.randomize(rep)
        ch.launch()
        c.run_separate()
        assert ch.status() == 0
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_chain_ragged_shapes_bitwise():
    spec = [(4096, [4100], None),          # M not a multiple of the grid
            (4096, [1, 33, 777], 0),       # tiny siblings, x = prefix of task 0's y
            (64, [5], None),               # K = 64: one block pair per row
            (256, [300], 0),               # partial 64-pair chunk (4 pairs)
             (4544, [4544], None),         # Falcon K (71 pairs: two chunks)
             (13824, [640], None),         # > 12288: chunked path of the per-launch GEMV
             (640, [4544], 5),             # x = task 5's y (640 values)
             (4544, [18176], 4),           # Falcon w1
             (18176, [300], 7)]            # K = 18176 (284 pairs, 5 chunks), x = w1 output
    c = ChainCase(spec, seed=1)
    ch = ggml_hip.Chain(c.tasks(0))
    for rep in range(2):
        c.randomize(10 + rep)
        ch.launch()
        c.run_separate()
        assert ch.status() == 0
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_chain_against_oracle():
    """Each task's y against the oracle on the task's actual input (the previous y)."""
    L = ggml_hip.load()
    spec = [(256, [200], None), (192, [320, 64], 0), (320, [256], 1), (256, [96], 2)]
    wq = []
    ws = []
    for t, (K, Ms, _) in enumerate(spec):
        row = []
        wrow = []
        for i, M in enumerate(Ms):
            q, _ = O.quantize_q4_0(O.gaussian(M * K, 0xA000 + 8 * t + i, 0.0, 0.05).reshape(M, K))
            row.append(q)
            wrow.append(DB.from_array(q))
        wq.append(row)
        ws.append(wrow)
    ys = [[DB(M * 4) for M in Ms] for (_, Ms, _) in spec]
    x0 = O.gaussian(256, 0xB000, 0.0, 1.0).astype(np.float32)
    xd0 = DB.from_array(x0)
    xs = [xd0 if src is None else ys[src][0] for (_, _, src) in spec]
    ch = ggml_hip.Chain([(ws[t], Ms, K, xs[t], ys[t]) for t, (K, Ms, _) in enumerate(spec)])
    ch.launch()
    assert ch.status() == 0
    x = x0
    for t, (K, Ms, src) in enumerate(spec):
        xin = x0 if src is None else ys[src][0].download((spec[src][1][0],), np.float32)[:K]
        xq = O.quantize_q8_0(xin.reshape(1, K), "avx2")
        for i, M in enumerate(Ms):
            y = ys[t][i].download((1, M), np.float32)
            y_ref = O.mul_mat(wq[t][i], K, xin.reshape(1, K), nthreads=1)
            _, s_abs = block_terms(wq[t][i], xq, K)
            check_y(y, y_ref, s_abs, rtol=1e-3, atol_blocks=1e-6)


def test_chain_graph_replay_bitwise():
    c = ChainCase(llama_layers(1, K=1024, F=2816), seed=2)
    ch = ggml_hip.Chain(c.tasks(0))
    c.randomize(20)
    ch.launch()
    ggml_hip.synchronize()
    eager = c.outputs(0)
    g = ggml_hip.Graph(None)
    with g:
        ch.launch(ggml_hip.load().ggml_hip_default_stream())
    for _ in range(3):
        g.launch()
    ggml_hip.synchronize()
    assert ch.status() == 0
    assert_bitwise(c.outputs(0), eager)
    c.randomize(21)                       # replay after the inputs changed
    g.launch()
    c.run_separate()
    assert_bitwise(c.outputs(0), c.outputs(1))


def test_chain_many_tasks_segments():
    """More tasks than one launch's LDS table holds: several launches, stream ordered."""
    spec = [(128, [128], None)] + [(128, [128], t) for t in range(599)]
    c = ChainCase(spec, seed=3)
    ch = ggml_hip.Chain(c.tasks(0))
    c.randomize(30)
    ch.launch()
    c.run_separate()
    assert ch.status() == 0
    assert_bitwise(c.outputs(0), c.outputs(1))


def test_chain_exact_mode_bitwise():
    L = ggml_hip.load()
    c = ChainCase(llama_layers(1, K=512, F=1408), seed=4)
    ch = ggml_hip.Chain(c.tasks(0))
    c.randomize(40)
    L.ggml_hip_set_exact(1)
    try:
        ch.launch()
        c.run_separate()
    finally:
        L.ggml_hip_set_exact(0)
    assert_bitwise(c.outputs(0), c.outputs(1))


def test_chain_invalid_arguments():
    L = ggml_hip.load()
    h = ctypes.c_void_p()
    t = (ggml_hip.ChainTask * 1)()
    t[0].nmat = 5
    assert L.ggml_hip_chain_create(1, t, ctypes.byref(h)) == ggml_hip.ERR_INVALID
    w = DB(18 * 2 * 64)
    x = DB(64 * 4)
    y = DB(64 * 4)
    t[0].nmat, t[0].K, t[0].x = 1, 96, x.ptr           # K % 64 != 0
    t[0].W[0], t[0].M[0], t[0].y[0] = w.ptr, 64, y.ptr
    assert L.ggml_hip_chain_create(1, t, ctypes.byref(h)) == ggml_hip.ERR_INVALID
    t[0].K = 64
    t[0].M[0] = 0
    assert L.ggml_hip_chain_create(1, t, ctypes.byref(h)) == ggml_hip.ERR_INVALID
    t[0].M[0] = 64
    assert L.ggml_hip_chain_create(0, t, ctypes.byref(h)) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_chain_create(1, t, ctypes.byref(h)) == ggml_hip.OK
    assert L.ggml_hip_chain_launch(h, None) == ggml_hip.OK
    assert L.ggml_hip_chain_status(h) == 0
    assert L.ggml_hip_chain_destroy(h) == ggml_hip.OK


# ---- the persistent decode engine (ggml_hip_chain_set_engine; q4_0_engine.hip) -----------------------------
def _engine_chain(spec, seed):
    c = ChainCase(spec, seed=seed)
    ch = ggml_hip.Chain(c.tasks(0))
    on = ch.set_engine(1)
    return c, ch, on


def test_engine_llama7b_two_layers_bitwise():
    """Full LLaMA-7B layer shapes (wq|wk|wv -> wo -> w1|w3 -> w2, x of each task = an output of the previous
    one, as llama.cpp:1334-1500 chains them): the engine's ONE launch reproduces the per-launch GEMVs bit for
    bit over three launches with fresh inputs (stale granules or stale x would show)."""
    c, ch, on = _engine_chain(llama_layers(2), 5)
    assert on, ggml_hip.load().ggml_hip_last_error()
    info = ch.engine_info()
    assert info["on"] == 1 and info["units"] > 0
    for rep in range(3):
        c.randomize(50 + rep)
        ch.launch()
        c.run_separate()
        assert ch.status() == 0, ggml_hip.load().ggml_hip_last_error()
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_engine_ragged_linear_chain_bitwise():
    """Ragged shapes on a linear chain: M not a multiple of 32 (partial units), prefix x (K < M of the
    producer), one-row and 33-row siblings, K = 64 (one pair per row), K = 4544 (2 pairs per lane), K = 11008 and
    12288 (3 per lane), rows that wrap the LDS ring."""
    spec = [(4096, [4100, 1, 33], None),      # consumed: the 4100-row output (prefix 4096 read next)
            (4096, [777, 64], 0),            # x = task 0's first output, prefix
            (640, [4544], 1),                # K 640 < 777: prefix of task 1's output 0
            (4544, [12288, 5], 2),           # Falcon K
            (12288, [256], 3),               # K = 12288: 3 pairs per lane, 6912-byte rows
            (256, [11008], 4),
            (11008, [96, 3], 5),
            (64, [64], 6)]                   # K = 64: one pair, lanes 1..63 idle
    c, ch, on = _engine_chain(spec, 6)
    assert on, ggml_hip.load().ggml_hip_last_error()
    for rep in range(2):
        c.randomize(60 + rep)
        ch.launch()
        c.run_separate()
        assert ch.status() == 0, ggml_hip.load().ggml_hip_last_error()
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_engine_many_tasks_and_replays():
    """600 dependent tasks (the epoch tags of 600 x 4 units' granules), eager and as a replayed HIP graph."""
    spec = [(128, [128], None)] + [(128, [128], t) for t in range(599)]
    c, ch, on = _engine_chain(spec, 7)
    assert on
    c.randomize(70)
    ch.launch()
    c.run_separate()
    assert ch.status() == 0
    assert_bitwise(c.outputs(0), c.outputs(1))
    g = ggml_hip.Graph(None)
    with g:
        ch.launch(ggml_hip.load().ggml_hip_default_stream())
    for rep in range(3):
        c.randomize(71 + rep)
        g.launch()
        c.run_separate()
        assert ch.status() == 0
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_engine_graph_replay_llama_layer():
    c, ch, on = _engine_chain(llama_layers(1, K=1024, F=2816), 8)
    assert on
    g = ggml_hip.Graph(None)
    with g:
        ch.launch(ggml_hip.load().ggml_hip_default_stream())
    for rep in range(4):
        c.randomize(80 + rep)
        g.launch()
        c.run_separate()
        assert ch.status() == 0
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_engine_declines_nonlinear_chains_and_stays_correct():
    """A task whose x is not an output of the task before it (or a first x the chain writes): the engine
    declines (ggml_hip_last_error says why) and the chain runs per launch, bitwise as before."""
    spec = [(4096, [4100], None), (4096, [1, 33, 777], 0), (4096, [64], 0)]
    c, ch, on = _engine_chain(spec, 9)
    assert not on
    assert b"not an output of task" in ggml_hip.load().ggml_hip_last_error()
    assert ch.engine_info()["on"] == 0
    c.randomize(90)
    ch.launch()
    c.run_separate()
    assert ch.status() == 0
    assert_bitwise(c.outputs(0), c.outputs(1))


def test_engine_exact_mode_runs_per_launch():
    L = ggml_hip.load()
    c, ch, on = _engine_chain(llama_layers(1, K=512, F=1408), 10)
    assert on
    c.randomize(100)
    L.ggml_hip_set_exact(1)
    try:
        ch.launch()
        c.run_separate()
    finally:
        L.ggml_hip_set_exact(0)
    assert ch.status() == 0
    assert_bitwise(c.outputs(0), c.outputs(1))


def test_engine_against_oracle():
    """Every task's y of a small linear chain against the oracle on its actual input (the previous y)."""
    spec = [(256, [224], None), (192, [320, 64], 0), (320, [256], 1), (256, [96], 2)]
    wq, ws = [], []
    for t, (K, Ms, _) in enumerate(spec):
        row, wrow = [], []
        for i, M in enumerate(Ms):
            q, _ = O.quantize_q4_0(O.gaussian(M * K, 0xA100 + 8 * t + i, 0.0, 0.05).reshape(M, K))
            row.append(q)
            wrow.append(DB.from_array(q))
        wq.append(row)
        ws.append(wrow)
    ys = [[DB(M * 4) for M in Ms] for (_, Ms, _) in spec]
    x0 = O.gaussian(256, 0xB100, 0.0, 1.0).astype(np.float32)
    xd0 = DB.from_array(x0)
    xs = [xd0 if src is None else ys[src][0] for (_, _, src) in spec]
    ch = ggml_hip.Chain([(ws[t], Ms, K, xs[t], ys[t]) for t, (K, Ms, _) in enumerate(spec)], engine=1)
    assert ch.engine_info()["on"] == 1
    ch.launch()
    assert ch.status() == 0
    for t, (K, Ms, src) in enumerate(spec):
        xin = x0 if src is None else ys[src][0].download((spec[src][1][0],), np.float32)[:K]
        xq = O.quantize_q8_0(xin.reshape(1, K), "avx2")
        for i, M in enumerate(Ms):
            y = ys[t][i].download((1, M), np.float32)
            y_ref = O.mul_mat(wq[t][i], K, xin.reshape(1, K), nthreads=1)
            _, s_abs = block_terms(wq[t][i], xq, K)
            check_y(y, y_ref, s_abs, rtol=1e-3, atol_blocks=1e-6)


def test_chain_through_aql_launch_mode_bitwise():
    """The tensor-free launches of a stream routed through the own AQL queue (launch mode 3,
    ggml_hip_debug_set_stream_launch_mode): the per-launch decode chain stays bitwise the separate calls',
    over launches with fresh inputs (HIP fills / copies between them order against the queue)."""
    L = ggml_hip.load()
    L.ggml_hip_debug_set_stream_launch_mode.argtypes = [ctypes.c_void_p, ctypes.c_int]
    c = ChainCase(llama_layers(2), seed=12)
    ch = ggml_hip.Chain(c.tasks(0))
    s = L.ggml_hip_default_stream()
    for rep in range(3):
        c.randomize(120 + rep)
        ggml_hip.check(L.ggml_hip_debug_set_stream_launch_mode(s, 3), "launch mode 3")
        try:
            ch.launch(s)
        finally:
            ggml_hip.check(L.ggml_hip_debug_set_stream_launch_mode(s, 0), "launch mode 0")
        c.run_separate()
        assert ch.status() == 0
        assert_bitwise(c.outputs(0), c.outputs(1))
