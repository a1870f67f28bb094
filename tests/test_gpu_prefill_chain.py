"""N-token chains (ggml_hip_chain_create_n, verdict r5 item 6): dependent prefill mul_mats where each k_gemm9
launch's epilogue writes the next launch's fp6 x image beside its f32 y (no k_prep9_x between them).

Bar: bitwise equal to separate ggml_hip_mul_mat_q4_0_multi calls at the same N (the image is bitwise
k_prep9_x's of y, so the consumer's GEMM reads the same codes); bitwise equal with the fold switched off
(ggml_hip_debug_set_chain_x9(0)); every dependency honoured (inputs re-randomised between launches); the
oracle within the north-star bound (tests/parity.py) on each task's actual input.
"""
import numpy as np
import pytest

import oracle as O
from hip_env import ggml_hip, gpu_available
from parity import block_terms, check_y

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer


@pytest.fixture(autouse=True)
def epilogue_fold_on():
    """the fold is opt-in (measured slower, include/ggml-hip.h): these tests run it, and restore the default"""
    L = ggml_hip.load()
    ggml_hip.check(L.ggml_hip_debug_set_chain_x9(1))
    yield
    L.ggml_hip_debug_set_chain_x9(-1)


def dev_weights(K, M, seed):
    L = ggml_hip.load()
    tmp = DB(K * M * 4)
    w = DB(18 * K // 32 * M)
    ggml_hip.check(L.ggml_hip_fill_gaussian(tmp.ptr, K * M, seed, 0.0, 0.02, None))
    ggml_hip.check(L.ggml_hip_quantize_q4_0(tmp.ptr, K, M, w.ptr, None))
    tmp.free()
    return w


class PrefillCase:
    """spec: list of (K, [M...], src); src = (task, matrix) whose y (N x M) is this task's x, or None for an
    independent input.  Every weight gets its fp6 image (k_gemm9) unless images=False."""

    def __init__(self, spec, N, seed=0, images=True):
        self.spec, self.N = spec, N
        L = ggml_hip.load()
        self.w = [[dev_weights(K, M, 0x5100 + seed * 97 + 8 * t + i) for i, M in enumerate(Ms)]
                  for t, (K, Ms, _) in enumerate(spec)]
        self.images = images
        if images:
            for t, (K, Ms, _) in enumerate(spec):
                for i, M in enumerate(Ms):
                    ggml_hip.check(L.ggml_hip_weight_image_create(self.w[t][i].ptr, K, M, None), "image")
        self.sets = [self._buffers() for _ in range(2)]      # [0] chain, [1] separate calls

    def close(self):
        if self.images:
            L = ggml_hip.load()
            for row in self.w:
                for w in row:
                    L.ggml_hip_weight_image_free(w.ptr)

    def _buffers(self):
        ys = [[DB(M * 4 * self.N) for M in Ms] for (_, Ms, _) in self.spec]
        xs = []
        for t, (K, Ms, src) in enumerate(self.spec):
            if src is None:
                xs.append(DB(K * 4 * self.N))
            else:
                u, i = src
                assert u < t and self.spec[u][1][i] == K
                xs.append(ys[u][i])
        return xs, ys

    def randomize(self, seed):
        L = ggml_hip.load()
        for xs, _ in self.sets:
            for t, (K, _, src) in enumerate(self.spec):
                if src is None:
                    ggml_hip.check(L.ggml_hip_fill_gaussian(xs[t].ptr, K * self.N, 0x9100 + seed * 131 + t, 0.0, 1.0,
                                                            None))
        ggml_hip.synchronize()

    def tasks(self, which=0):
        xs, ys = self.sets[which]
        return [(self.w[t], Ms, K, xs[t], ys[t]) for t, (K, Ms, _) in enumerate(self.spec)]

    def run_separate(self):
        for ws, Ms, K, x, ys in self.tasks(1):
            ggml_hip.mul_mat_multi(ws, Ms, K, x, self.N, ys)
        ggml_hip.synchronize()

    def outputs(self, which):
        _, ys = self.sets[which]
        return [[y.download((self.N, M), np.float32) for y, M in zip(yt, Ms)]
                for yt, (_, Ms, _) in zip(ys, self.spec)]


def assert_bitwise(a, b):
    for t, (ya, yb) in enumerate(zip(a, b)):
        for i, (u, v) in enumerate(zip(ya, yb)):
            if not np.array_equal(u.view(np.uint32), v.view(np.uint32)):
                bad = np.argwhere(u.view(np.uint32) != v.view(np.uint32))
                raise AssertionError(f"task {t} matrix {i} differs at {len(bad)} places, first {bad[0]}")


def llama_layers(n, K=4096, F=11008):
    """wq|wk|wv -> wo (x = q) -> w1|w3 -> w2 (x = w1) -> next layer's wq|wk|wv (x = w2): the bench's chain"""
    spec = []
    prev = None
    for _ in range(n):
        q = len(spec)
        spec.append((K, [K, K, K], prev))
        spec.append((K, [K], (q, 0)))
        spec.append((K, [F, F], (q + 1, 0)))
        spec.append((F, [K], (q + 2, 0)))
        prev = (q + 3, 0)
    return spec


def _run_case(c, ch, seeds):
    for s in seeds:
        c.randomize(s)
        ch.launch()
        c.run_separate()
        assert ch.status() == 0
        assert_bitwise(c.outputs(0), c.outputs(1))


def test_prefill_chain_llama7b_layers_bitwise():
    """Full LLaMA-7B shapes at N = 512 (the bench's prefill chain): 8 tasks, 7 of them fed by an epilogue."""
    c = PrefillCase(llama_layers(2), 512, seed=1)
    try:
        ch = ggml_hip.Chain(c.tasks(0), N=512)
        assert ch.engine_info()["epilogue_images"] == 7
        _run_case(c, ch, [0, 1])
        L = ggml_hip.load()
        ggml_hip.check(L.ggml_hip_debug_set_chain_x9(0))          # every image by k_prep9_x: the same y
        try:
            _run_case(c, ch, [2])
        finally:
            L.ggml_hip_debug_set_chain_x9(1)
    finally:
        c.close()


@pytest.mark.parametrize("N", [65, 300, 777])
def test_prefill_chain_ragged_bitwise(N):
    """Token counts off the 64 / 128-token tiles (half tiles, wide and mixed launches), M = 4160 (a partial
    128-row tile feeding K = 4160), x = y of a sibling other than the first, two consumers sharing one image,
    a consumer of another matrix of the same producer (its own k_prep9_x), a task in between that overwrites
    part of the producer's output (no epilogue link: k_prep9_x on the new values)."""
    spec = [(1024, [4160, 1024, 192], None),     # 0
            (4160, [2048], (0, 0)),              # 1: x = task 0 matrix 0 (M = 4160, a partial 128-row tile)
            (4160, [64], (0, 0)),                # 2: second consumer of (0, 0): shares the image
            (1024, [1024], (0, 1)),              # 3: x = sibling 1: task 0 writes (0, 0)'s image, so k_prep9_x
            (192, [1024], (0, 2)),               # 4: likewise (K = 192)
            (2048, [1024], (1, 0)),              # 5: x = task 1's y
            (1024, [1024], None),                # 6: y = the first half of task 1's output buffer (below)
            (2048, [128], (1, 0))]               # 7: x = task 1's buffer after task 6 wrote into it: no link
    c = PrefillCase(spec, N, seed=2)
    for s in c.sets:
        s[1][6][0] = s[1][1][0]                  # task 6 writes rows [N][1024] over task 1's [N][2048] output
    try:
        ch = ggml_hip.Chain(c.tasks(0), N=N)
        links = ch.engine_info()["epilogue_images"]
        assert links == 3, links                  # tasks 1, 2, 5
        _run_case(c, ch, [10, 11])
    finally:
        c.close()


def test_prefill_chain_mixed_paths_bitwise():
    """Tasks off the k_gemm9 path keep the sibling calls: weights without images (split-K / LDS GEMM),
    N <= 8 (GEMVs), exact mode; a consumer whose producer did not run on k_gemm9 preps its own image."""
    spec = [(1024, [1024], None), (1024, [2048], (0, 0)), (2048, [1024], (1, 0))]
    c = PrefillCase(spec, 200, seed=3)
    L = ggml_hip.load()
    try:
        L.ggml_hip_weight_image_free(c.w[0][0].ptr)       # task 0 without an image: task 1 preps
        ch = ggml_hip.Chain(c.tasks(0), N=200)
        _run_case(c, ch, [20])
        L.ggml_hip_set_exact(1)
        try:
            _run_case(c, ch, [21])
        finally:
            L.ggml_hip_set_exact(0)
    finally:
        c.close()
    c = PrefillCase(spec, 6, seed=4, images=False)         # N = 6: GEMVs
    ch = ggml_hip.Chain(c.tasks(0), N=6)
    assert ch.engine_info()["epilogue_images"] == 0
    _run_case(c, ch, [22])


def test_prefill_chain_graph_replay():
    c = PrefillCase(llama_layers(1, K=1024, F=2816), 384, seed=5)
    try:
        ch = ggml_hip.Chain(c.tasks(0), N=384)
        c.randomize(30)
        ch.launch()
        ggml_hip.synchronize()
        eager = c.outputs(0)
        g = ggml_hip.Graph(None)
        with g:
            ch.launch(ggml_hip.load().ggml_hip_default_stream())
        g.launch()
        ggml_hip.synchronize()
        assert_bitwise(c.outputs(0), eager)
        c.randomize(31)
        g.launch()
        c.run_separate()
        assert_bitwise(c.outputs(0), c.outputs(1))
    finally:
        c.close()


def test_prefill_chain_against_oracle():
    """Each task's y against the oracle on its actual input (the producer's y), N = 96."""
    N = 96
    spec = [(256, [192, 256], None), (192, [320], (0, 0)), (320, [256], (1, 0)), (256, [128], (0, 1))]
    wq, ws = [], []
    L = ggml_hip.load()
    for t, (K, Ms, _) in enumerate(spec):
        row, wrow = [], []
        for i, M in enumerate(Ms):
            q, _ = O.quantize_q4_0(O.gaussian(M * K, 0xA200 + 8 * t + i, 0.0, 0.05).reshape(M, K))
            row.append(q)
            d = DB.from_array(q)
            ggml_hip.check(L.ggml_hip_weight_image_create(d.ptr, K, M, None), "image")
            wrow.append(d)
        wq.append(row)
        ws.append(wrow)
    try:
        ys = [[DB(M * 4 * N) for M in Ms] for (_, Ms, _) in spec]
        x0 = O.gaussian(256 * N, 0xB200, 0.0, 1.0).astype(np.float32).reshape(N, 256)
        xd0 = DB.from_array(x0)
        xs = [xd0 if src is None else ys[src[0]][src[1]] for (_, _, src) in spec]
        ch = ggml_hip.Chain([(ws[t], Ms, K, xs[t], ys[t]) for t, (K, Ms, _) in enumerate(spec)], N=N)
        assert ch.engine_info()["epilogue_images"] == 2       # tasks 1, 2 (task 3 reads sibling 1: k_prep9_x)
        ch.launch()
        assert ch.status() == 0
        for t, (K, Ms, src) in enumerate(spec):
            xin = x0 if src is None else ys[src[0]][src[1]].download((N, K), np.float32)
            xq = O.quantize_q8_0(xin, "avx2")
            for i, M in enumerate(Ms):
                y = ys[t][i].download((N, M), np.float32)
                y_ref = O.mul_mat(wq[t][i], K, xin, nthreads=4)
                _, s_abs = block_terms(wq[t][i], xq, K)
                check_y(y, y_ref, s_abs, rtol=1e-3, atol_blocks=1e-6)
    finally:
        for row in ws:
            for d in row:
                L.ggml_hip_weight_image_free(d.ptr)


def test_prefill_chain_invalid_and_engine_declines():
    import ctypes
    L = ggml_hip.load()
    w = DB(18 * 2 * 64)
    x = DB(64 * 4 * 100)
    y = DB(64 * 4 * 100)
    t = (ggml_hip.ChainTask * 1)()
    t[0].nmat, t[0].K, t[0].x = 1, 64, x.ptr
    t[0].W[0], t[0].M[0], t[0].y[0] = w.ptr, 64, y.ptr
    h = ctypes.c_void_p()
    assert L.ggml_hip_chain_create_n(1, t, 0, ctypes.byref(h)) == ggml_hip.ERR_INVALID
    t[0].y[0] = x.ptr + 64 * 4 * 50                  # y overlaps x at N = 100 (not at N = 1)
    assert L.ggml_hip_chain_create_n(1, t, 100, ctypes.byref(h)) == ggml_hip.ERR_INVALID
    t[0].y[0] = y.ptr
    assert L.ggml_hip_chain_create_n(1, t, 100, ctypes.byref(h)) == ggml_hip.OK
    assert L.ggml_hip_chain_set_engine(h, 1) == 0
    assert b"N = 1" in L.ggml_hip_last_error()
    assert L.ggml_hip_chain_launch(h, None) == ggml_hip.OK
    assert L.ggml_hip_chain_status(h) == 0
    assert L.ggml_hip_chain_destroy(h) == ggml_hip.OK
