"""Exact mode (algorithm 4): every y BIT-IDENTICAL to the reference's x86 AVX2+FMA
ggml_vec_dot_q4_0_q8_0 (ggml.c:2412-2435) — the golden vectors the reference itself produced,
and the oracle's restatement of that fp32 schedule (oracle/q4_0_oracle.c:209-240) on random
shapes, ragged tails (K/32 not a multiple of the kernel's 32-block chunk, M not a multiple of
its 16-row tile), every N regime, and the process-wide switch that routes the auto-selected,
sibling-matrix and ggml-tensor entry points through it."""
import ctypes

import numpy as np
import pytest

import oracle as O
from golden_io import load
from hip_env import ggml_hip, gpu_available
from test_gpu_parity import DB, gpu_mul_mat, make_case

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_bitwise(got, ref):
    diff = np.flatnonzero(bits(got) != bits(ref))
    assert diff.size == 0, f"{diff.size} of {got.size} differ; first at {diff[:4]}: {got.ravel()[diff[:4]]} vs " \
                           f"{ref.ravel()[diff[:4]]}"


@pytest.fixture
def exact_off():
    L = ggml_hip.load()
    prev = L.ggml_hip_get_exact()
    L.ggml_hip_set_exact(0)
    yield L
    L.ggml_hip_set_exact(prev)


def test_exact_golden_vectors_bitwise():
    """The reference's own mul_mat outputs (tests/golden, produced by ggml.c built -march=x86-64-v3)."""
    for K, tag in ((4096, "4096"), (4544, "4544")):
        wq, x = load("avx2", f"w{tag}_q4_0"), load("avx2", f"x{tag}_f32")
        y, _ = gpu_mul_mat(wq, K, x, algo=4)
        assert_bitwise(y, load("avx2", f"y{tag}_mul_mat"))


@pytest.mark.parametrize("K,M,N", [
    (64, 1, 1), (64, 33, 3), (128, 100, 8), (1088, 17, 1), (1024, 16, 2), (1088, 31, 5),
    (4096, 257, 2), (4544, 4672 // 8, 1), (11008, 96, 4), (64, 130, 9), (256, 129, 31),
    (4096, 128, 33), (4544, 200, 65), (11008, 40, 64), (768, 256, 40), (256, 320, 40), (2048, 48, 129),
])
def test_exact_vs_oracle_bitwise(K, M, N):
    wq, x = make_case(K, M, N, seed=K * 3 + M * 5 + N)
    y, _ = gpu_mul_mat(wq, K, x, algo=4)
    assert_bitwise(y, O.mul_mat(wq, K, x, nthreads=4))


def test_exact_no_writes_outside_rows():
    wq, x = make_case(4096, 100, 3, seed=11)
    y, yfull = gpu_mul_mat(wq, 4096, x, algo=4, ldy=128)
    assert np.all(yfull[:, 100:].view(np.uint32) == 0x7F7F7F7F)
    assert_bitwise(y, O.mul_mat(wq, 4096, x))


def test_exact_zero_and_extreme_activations():
    K, M = 4096, 64
    wq, _ = make_case(K, M, 1, seed=3)
    x = np.zeros((4, K), np.float32)
    x[1, ::7] = 3.0e4
    x[2] = -1e-30
    x[3, 5] = -65000.0
    y, _ = gpu_mul_mat(wq, K, x, algo=4)
    assert_bitwise(y, O.mul_mat(wq, K, x))


@pytest.mark.parametrize("K,M", [(4096, 4096), (11008, 4096)])
def test_exact_llama7b_decode_full_shape(K, M):
    wq, x = make_case(K, M, 1, seed=K + M + 1)
    y, _ = gpu_mul_mat(wq, K, x, algo=4)
    assert_bitwise(y, O.mul_mat(wq, K, x, nthreads=8))


def test_exact_switch_routes_auto_multi_and_tensor_paths(exact_off):
    L = exact_off
    K, Ms, N = 4096, [256, 128, 300], 3
    cases = [make_case(K, M, N, seed=70 + i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    refs = [O.mul_mat(wq, K, x) for wq, _ in cases]
    # off: the fast kernels (not bitwise in general), on: bitwise through every entry point
    assert L.ggml_hip_set_exact(1) == 0 and L.ggml_hip_get_exact() == 1
    for (wq, _), ref in zip(cases, refs):
        y, _ = gpu_mul_mat(wq, K, x, algo=0)
        assert_bitwise(y, ref)
    wds, xd = [DB.from_array(c[0]) for c in cases], DB.from_array(x)
    ys = [DB(N * M * 4) for M in Ms]
    ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
    for yd, M, ref in zip(ys, Ms, refs):
        assert_bitwise(yd.download((N, M), np.float32), ref)
    # ggml tensor ABI, host tensors: the hook path ggml.c's compute_forward takes (ggml.c:15645)
    wq = np.ascontiguousarray(cases[0][0])
    N2 = 40
    x2 = np.ascontiguousarray(O.gaussian(N2 * K, 123, 0.0, 1.0).reshape(N2, K))
    y2 = np.zeros((N2, Ms[0]), np.float32)
    w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, Ms[0]), wq)
    xt = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, N2), x2)
    yt = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (Ms[0], N2), y2)
    yt.op = ggml_hip.GGML_OP_MUL_MAT
    yt.src0, yt.src1 = ctypes.pointer(w), ctypes.pointer(xt)
    p = ggml_hip.GgmlComputeParams(ggml_hip.GGML_TASK_COMPUTE, 0, 1, 0, None)
    assert L.ggml_hip_compute_forward(ctypes.byref(p), ctypes.byref(yt))
    assert_bitwise(y2, O.mul_mat(wq, K, x2))
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")


@pytest.mark.parametrize("N", [1, 8, 40])
def test_exact_sibling_group_one_launch_bitwise(exact_off, N):
    """Exact mode runs a sibling group (ggml_hip_mul_mat_q4_0_multi) as ONE exact launch over the
    concatenated 16-row workgroups of up to four matrices: every y still bit-identical to the
    oracle's AVX2 schedule, ragged M (a matrix that ends mid-workgroup) included."""
    L = exact_off
    K, Ms = 1024, [512, 48, 300, 16]
    cases = [make_case(K, M, N, seed=90 + i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    assert L.ggml_hip_set_exact(1) == 0
    wds, xd = [DB.from_array(c[0]) for c in cases], DB.from_array(x)
    ys = [DB(N * M * 4) for M in Ms]
    ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
    for (wq, _), yd, M in zip(cases, ys, Ms):
        assert_bitwise(yd.download((N, M), np.float32), O.mul_mat(wq, K, x))


@pytest.mark.parametrize("K", [64, 4544, 11008, 18176, 22528, 22592])
def test_exact_n1_long_rows_bitwise(exact_off, K):
    """Exact-mode decode (N = 1) up to K = 22592 (Falcon's 18176 and past it, ragged final chunks):
    single matrices, a sibling group, and the extreme rows the quantizer's tests cover — all
    bitwise to the oracle's AVX2 schedule."""
    L = exact_off
    Ms = [48, 17, 33]
    cases = [make_case(K, M, 1, seed=K + 7 * i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    for wq, _ in cases[:1]:
        y, _ = gpu_mul_mat(wq, K, x, algo=4)
        assert_bitwise(y, O.mul_mat(wq, K, x, nthreads=4))
    for row in (np.where(np.arange(K) % 7 == 0, 3.0e4, 0.0), np.full(K, -1e-30), np.zeros(K)):
        xr = np.ascontiguousarray(row.reshape(1, K), np.float32)
        y, _ = gpu_mul_mat(cases[0][0], K, xr, algo=4)
        assert_bitwise(y, O.mul_mat(cases[0][0], K, xr))
    assert L.ggml_hip_set_exact(1) == 0
    wds, xd = [DB.from_array(c[0]) for c in cases], DB.from_array(x)
    ys = [DB(M * 4) for M in Ms]
    ggml_hip.mul_mat_multi(wds, Ms, K, xd, 1, ys)
    for (wq, _), yd, M in zip(cases, ys, Ms):
        assert_bitwise(yd.download((1, M), np.float32), O.mul_mat(wq, K, x))
