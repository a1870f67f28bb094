"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bar (BASELINE.json north_star): q8_0 activation bytes bit-exact to the reference's AVX2
branch; y within 1e-3 relative on the fp32 accumulator, with the cancellation-safe bound of
tests/parity.py (|dy| <= 1e-3|y| + atol_blocks * sum_b |d_w d_x sumi|).  q4_0 weight
quantization and dequantization are bit-exact.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
from golden_io import load
from hip_env import ggml_hip, gpu_available
from parity import block_terms, check_y, s_abs_exact

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer
RTOL, ATOL_BLOCKS = 1e-3, 1e-6


def gpu_q8(x):
    x = np.ascontiguousarray(x, np.float32)
    N, K = x.shape
    xd = DB.from_array(x)
    xq = DB(N * K // 32 * 34)
    ggml_hip.quantize_q8_0(xd, K, N, xq)
    return xq.download((N, K // 32 * 34), np.uint8)


def gpu_mul_mat(wq, K, x, algo=0, ldy=None):
    x = np.ascontiguousarray(x, np.float32)
    N = x.shape[0]
    M = wq.shape[0]
    ldy = M if ldy is None else ldy
    wd, xd = DB.from_array(wq), DB.from_array(x)
    yd = DB(max(N, 1) * ldy * 4)
    ggml_hip.load().ggml_hip_memset(yd.ptr, 0x7F, yd.nbytes, None)
    ggml_hip.mul_mat(wd, K, M, xd, N, yd, algo=algo, ldy=ldy)
    y = yd.download((max(N, 1), ldy), np.float32)
    return y[:N, :M], y


def upper_s_abs(wq, xq, K):
    """sum_b |d_w d_x sumi|, exact (tests/parity.py s_abs_exact, chunked over blocks)."""
    return s_abs_exact(wq, xq, K)


def make_case(K, M, N, seed, wstd=0.02, xscale=1.0):
    wf = O.gaussian(M * K, 0x5EED0000 + seed, 0.0, wstd).reshape(M, K)
    wq, _ = O.quantize_q4_0(wf)
    x = O.gaussian(N * K, 0x5EED1000 + seed, 0.0, xscale).reshape(N, K)
    return wq, x


# ------------------------------------------------------------------------------- q8_0 (A5)
def test_q8_0_bitexact_golden():
    x = load("avx2", "x4096_f32")
    assert np.array_equal(gpu_q8(x), load("avx2", "x4096_q8_0"))
    t = load("avx2", "tie_x_f32").reshape(1, -1)
    assert np.array_equal(gpu_q8(t).reshape(8, 34), load("avx2", "tie_q8_0"))


@pytest.mark.parametrize("K,N", [(64, 1), (4096, 7), (4544, 3), (11008, 5), (13824, 2)])
def test_q8_0_bitexact_random_scales(K, N):
    rng = np.random.default_rng(K + N)
    x = (rng.standard_normal((N, K)) * np.exp(rng.uniform(-12, 10, (N, K // 32))).repeat(32, 1)).astype(np.float32)
    x[0, :32] = 0.0                                   # amax == 0 block
    x[-1, 32:64] = np.float32(1e-30)                  # d underflows fp16
    assert np.array_equal(gpu_q8(x), O.quantize_q8_0(x, "avx2"))


def test_q8_0_half_integer_ties_round_to_even():
    """Blocks with amax = 127 (id = 1 exactly) and half-integer values: every element is a tie."""
    K = 128
    x = np.zeros((1, K), np.float32)
    for b in range(3):
        x[0, 32 * b:32 * b + 32] = (np.arange(32) - 16).astype(np.float32) + 0.5 * (b + 1) % 2 + 0.5 * (b == 1)
        x[0, 32 * b + 7] = 127.0 if b != 1 else -127.0
    x[0, 96:128] = np.linspace(-126.5, 126.5, 32).astype(np.float32)
    x[0, 100] = 127.0
    assert np.array_equal(gpu_q8(x), O.quantize_q8_0(x, "avx2"))
    assert not np.array_equal(O.quantize_q8_0(x, "avx2"), O.quantize_q8_0(x, "ref"))   # ties do differ


# ------------------------------------------------------------------------------- q4_0 (A3/A4)
@pytest.mark.parametrize("K,M", [(128, 1), (4096, 64), (4544, 8)])
def test_q4_0_quantize_bitexact(K, M):
    w = O.gaussian(M * K, 0x5EED0001 if (K, M) == (4096, 64) else 77 + K, 0.0, 0.02).reshape(M, K)
    wd = DB.from_array(w)
    qd = DB(M * K // 32 * 18)
    ggml_hip.quantize_q4_0(wd, K, M, qd)
    got = qd.download((M, K // 32 * 18), np.uint8)
    ref, _ = O.quantize_q4_0(w)
    assert np.array_equal(got, ref)
    if (K, M) == (4096, 64):
        assert np.array_equal(got, load("avx2", "w4096_q4_0"))


def test_q4_0_quantize_ties_golden():
    w = load("avx2", "q4tie_w_f32").reshape(1, 128)
    wd = DB.from_array(w)
    qd = DB(4 * 18)
    ggml_hip.quantize_q4_0(wd, 128, 1, qd)
    assert np.array_equal(qd.download((4, 18), np.uint8), load("avx2", "q4tie_q4_0"))


def test_dequantize_bitexact_golden():
    wq = load("avx2", "w4096_q4_0")[:2]
    qd = DB.from_array(wq)
    od = DB(2 * 4096 * 4)
    ggml_hip.dequantize_q4_0(qd, 4096, 2, od)
    got = od.download((2, 4096), np.float32)
    assert np.array_equal(got.view(np.uint32), load("avx2", "w4096_dequant_rows01").view(np.uint32))


# ------------------------------------------------------------------------------- mul_mat vs golden
@pytest.mark.parametrize("algo", [1, 2, 3])
def test_mul_mat_golden_llama_slice(algo):
    wq, x = load("avx2", "w4096_q4_0"), load("avx2", "x4096_f32")
    y, _ = gpu_mul_mat(wq, 4096, x, algo=algo)
    y_ref = load("avx2", "y4096_mul_mat")
    _, s_abs = block_terms(wq, load("avx2", "x4096_q8_0"), 4096)
    rel, _ = check_y(y, y_ref, s_abs, RTOL, ATOL_BLOCKS)
    assert rel < 1e-3


@pytest.mark.parametrize("algo", [1, 2, 3])
def test_mul_mat_golden_falcon_k4544(algo):
    wq, x = load("avx2", "w4544_q4_0"), load("avx2", "x4544_f32")
    y, _ = gpu_mul_mat(wq, 4544, x, algo=algo)
    xq = O.quantize_q8_0(x, "avx2")
    _, s_abs = block_terms(wq, xq, 4544)
    check_y(y, load("avx2", "y4544_mul_mat"), s_abs, RTOL, ATOL_BLOCKS)


# ------------------------------------------------------------------------------- mul_mat vs oracle
EDGE_SHAPES = [(64, 1, 1), (64, 33, 3), (128, 100, 8), (4096, 257, 2), (4544, 4672 // 8, 1), (11008, 96, 4),
               (64, 130, 9), (256, 129, 31), (4096, 128, 33), (4544, 200, 65), (11008, 130, 64), (4096, 64, 100)]


@pytest.mark.parametrize("K,M,N,algo", [s + (0,) for s in EDGE_SHAPES] + [s + (2,) for s in EDGE_SHAPES if s[2] > 8])
def test_mul_mat_vs_oracle_edges(K, M, N, algo):
    """auto (GEMV N <= 8, split-K N <= 128, GEMM above) and the LDS-staged GEMM forced (N > 8)."""
    wq, x = make_case(K, M, N, seed=K * 7 + M + N)
    y, yfull = gpu_mul_mat(wq, K, x, algo=algo)
    xq = O.quantize_q8_0(x, "avx2")
    y_ref = O.mul_mat(wq, K, x, nthreads=4)
    _, s_abs = block_terms(wq, xq, K)
    check_y(y, y_ref, s_abs, RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("N", [1, 2, 5, 8])
def test_gemv_and_gemm_agree(N):
    wq, x = make_case(4096, 192, N, seed=N)
    y1, _ = gpu_mul_mat(wq, 4096, x, algo=1)
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), 4096)
    for algo in (2, 3):
        y2, _ = gpu_mul_mat(wq, 4096, x, algo=algo)
        check_y(y1, y2, s_abs, RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("N", [1, 3, 8, 20, 200, 512])
def test_multi_matrix_siblings_match_single_calls(N):
    """wq|wk|wv-style sibling batch (shared x, different M) == separate calls, bitwise: one GEMV launch
    (N <= 8), one x quantize + a GEMM per matrix (split-K range), one GEMM launch over the concatenated
    row tiles (N > 128; M = 300 ends mid-tile)."""
    K = 4096
    Ms = [256, 128, 300]
    cases = [make_case(K, M, N, seed=40 + i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    wds = [DB.from_array(c[0]) for c in cases]
    xd = DB.from_array(x)
    ys = [DB(N * M * 4) for M in Ms]
    ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
    for (wq, _), yd, M, wd in zip(cases, ys, Ms, wds):
        got = yd.download((N, M), np.float32)
        single, _ = gpu_mul_mat(wq, K, x)
        assert np.array_equal(got.view(np.uint32), single.view(np.uint32))


def test_ldy_stride_and_no_out_of_bounds_writes():
    wq, x = make_case(4096, 100, 3, seed=5)
    for algo in (1, 2, 3):
        y, yfull = gpu_mul_mat(wq, 4096, x, algo=algo, ldy=128)
        assert np.all(yfull[:, 100:].view(np.uint32) == 0x7F7F7F7F), "wrote outside [0, M) of a row"
        y_ref = O.mul_mat(wq, 4096, x)
        _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), 4096)
        check_y(y, y_ref, s_abs, RTOL, ATOL_BLOCKS)


def test_zero_and_extreme_activations():
    K, M = 4096, 64
    wq, _ = make_case(K, M, 1, seed=9)
    x = np.zeros((4, K), np.float32)
    x[1] = 1e-20
    x[2, ::7] = 3e4
    x[3] = O.gaussian(K, 3, 0.0, 1.0) * np.float32(1e-3)
    y, _ = gpu_mul_mat(wq, K, x)
    assert np.all(y[0] == 0.0)
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
    check_y(y, O.mul_mat(wq, K, x), s_abs, RTOL, ATOL_BLOCKS)


def test_invalid_arguments_fail_loudly():
    L = ggml_hip.load()
    wq, x = make_case(128, 4, 1, seed=1)
    wd, xd, yd = DB.from_array(wq), DB.from_array(x), DB(4 * 4)
    assert L.ggml_hip_mul_mat_q4_0(wd.ptr, 96, 4, xd.ptr, 1, yd.ptr, None) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_mul_mat_q4_0(wd.ptr + 4, 128, 4, xd.ptr, 1, yd.ptr, None) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_mul_mat_q4_0_ex(wd.ptr, 128, 4, xd.ptr, 9, yd.ptr, 4, 1, None) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_mul_mat_q4_0(wd.ptr, 128, 4, xd.ptr, 0, yd.ptr, None) == ggml_hip.OK   # N == 0: no-op


# ------------------------------------------------------------------------------- full LLaMA shapes
@pytest.mark.parametrize("K,M", [(4096, 4096), (4096, 11008), (11008, 4096)])
def test_llama7b_decode_full_shape(K, M):
    wq, x = make_case(K, M, 1, seed=K + M)
    y, _ = gpu_mul_mat(wq, K, x)
    y_ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=False)
    xq = O.quantize_q8_0(x, "avx2")
    assert np.array_equal(gpu_q8(x), xq)
    check_y(y, y_ref, upper_s_abs(wq, xq, K), RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("K,M", [(4544, 4672), (4544, 4544), (4544, 18176), (18176, 4544),
                                 (6144, 18432), (6144, 24576), (24576, 6144),
                                 (4096, 4096), (4096, 16384), (16384, 4096)],
                         ids=["falcon-qkv", "falcon-dense", "falcon-h_to_4h", "falcon-4h_to_h",
                              "neox-qkv", "neox-h_to_4h", "neox-4h_to_h",
                              "rwkv-att_kvro", "rwkv-ff_k", "rwkv-ff_v"])
@pytest.mark.parametrize("N", [1, 4])
def test_arch_decode_full_shapes(K, M, N):
    """BASELINE config 5 at full size: Falcon-7B (arch/falcon/falcon.cpp:995-1025; K = 4544 rows are
    only 4-byte aligned, K = 18176 takes the 64-pair-chunk items) and GPT-NeoX / StableLM-7B
    (n_embd 6144: QKV {n_embd, 3 n_embd}, MLP {n_embd, 4 n_embd}, arch/gptneox/gptneox.cpp:1014-1024)
    and RWKV-4 at n_embd 4096 (att k/v/r/out {n_embd, n_embd}, ff_k {n_embd, 4 n_embd}, ff_v {4 n_embd,
    n_embd}: K = 16384 is a long-row chunk-item launch; arch/rwkv/rwkv.cpp:1194-1217).
    q8_0 bytes bit-exact, y within the parity bound."""
    wq, x = make_case(K, M, N, seed=5 * K + M + N)
    y, _ = gpu_mul_mat(wq, K, x)
    y_ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=False)
    xq = O.quantize_q8_0(x, "avx2")
    assert np.array_equal(gpu_q8(x), xq)
    check_y(y, y_ref, upper_s_abs(wq, xq, K), RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("K,M", [(4096, 4096), (4096, 11008)])
def test_llama7b_prefill_512_full_shape(K, M):
    wq, x = make_case(K, M, 512, seed=3 * K + M)
    y, _ = gpu_mul_mat(wq, K, x)
    y_ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=True)
    xq = O.quantize_q8_0(x, "avx2")
    rel, _ = check_y(y, y_ref, upper_s_abs(wq, xq, K), RTOL, ATOL_BLOCKS)
    assert rel < 1e-3
    # size-independent property: linearity in x (x -> 2x doubles q8 scales exactly); same kernel
    # (auto sends N = 64 to the split-K path, whose fp32 summation order differs)
    y2, _ = gpu_mul_mat(wq, K, 2 * x[:64], algo=2)
    assert np.array_equal(y2.view(np.uint32), (2 * y[:64]).view(np.uint32))


@pytest.mark.parametrize("K,M,N", [(4096, 11008, 64), (11008, 4096, 17)])
def test_llama7b_small_batch_split_k_full_shape(K, M, N):
    """Split-K MFMA path (9 <= N <= 128) at full LLaMA shapes; linearity x -> 2x bitwise."""
    wq, x = make_case(K, M, N, seed=5 * K + M + N)
    y, _ = gpu_mul_mat(wq, K, x, algo=3)
    xq = O.quantize_q8_0(x, "avx2")
    y_ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=True)
    rel, _ = check_y(y, y_ref, upper_s_abs(wq, xq, K), RTOL, ATOL_BLOCKS)
    assert rel < 1e-3
    y2, _ = gpu_mul_mat(wq, K, 2 * x, algo=3)
    assert np.array_equal(y2.view(np.uint32), (2 * y).view(np.uint32))


# ------------------------------------------------------------------------------- tensor ABI (host tensors)
def test_can_mul_mat_rule():
    """Q4_0 x F32 -> F32 with ne0, ne1, ne10 >= 32 (ggml-cuda.cu:2595-2610); other types: no."""
    L = ggml_hip.load()
    K, M = 4096, 64
    for N, expect in ((32, True), (31, False), (512, True)):
        w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, M))
        x = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, N))
        y = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, N))
        assert bool(L.ggml_hip_can_mul_mat(ctypes.byref(w), ctypes.byref(x), ctypes.byref(y))) == expect
    wf = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, M))
    assert not L.ggml_hip_can_mul_mat(ctypes.byref(wf), ctypes.byref(x), ctypes.byref(y))
    w96 = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (96, M))     # K % 64 != 0 -> CPU path
    x96 = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (96, 64))
    y96 = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, 64))
    assert not L.ggml_hip_can_mul_mat(ctypes.byref(w96), ctypes.byref(x96), ctypes.byref(y96))
    assert L.ggml_hip_mul_mat_get_wsize(ctypes.byref(w), ctypes.byref(x), ctypes.byref(y)) == 0



def test_tensor_abi_compute_forward_host_tensors():
    """ggml.c:15645-15652 hook: node taken, only ith == 0 / COMPUTE computes; batch dim ne2 = 2."""
    L = ggml_hip.load()
    K, M, N = 4096, 96, 40
    wq, x = make_case(K, M * 2, N * 2, seed=11)
    w_np = np.ascontiguousarray(wq)
    x_np = np.ascontiguousarray(x)
    y_np = np.zeros((2, N, M), np.float32)
    w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, M, 2), w_np)
    xt = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, N, 2), x_np)
    y = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, N, 2), y_np)
    y.op = ggml_hip.GGML_OP_MUL_MAT
    y.src0 = ctypes.pointer(w)
    y.src1 = ctypes.pointer(xt)
    for phase, ith in ((ggml_hip.GGML_TASK_INIT, 0), (ggml_hip.GGML_TASK_COMPUTE, 1)):
        p = ggml_hip.GgmlComputeParams(phase, ith, 2, 0, None)
        assert L.ggml_hip_compute_forward(ctypes.byref(p), ctypes.byref(y))
    assert np.all(y_np == 0.0)                      # nothing computed yet
    p = ggml_hip.GgmlComputeParams(ggml_hip.GGML_TASK_COMPUTE, 0, 2, 0, None)
    assert L.ggml_hip_compute_forward(ctypes.byref(p), ctypes.byref(y))
    for b in range(2):
        wb = w_np[b * M:(b + 1) * M]
        xb = x_np[b * N:(b + 1) * N]
        _, s_abs = block_terms(wb, O.quantize_q8_0(xb, "avx2"), K)
        check_y(y_np[b], O.mul_mat(wb, K, xb), s_abs, RTOL, ATOL_BLOCKS)


def test_tensor_abi_transform_tensor_resident_weights():
    """ggml_cuda_transform_tensor equivalent: upload once, extra->data_device[main]; decode N=1."""
    L = ggml_hip.load()
    K, M = 4096, 256
    wq, x = make_case(K, M, 1, seed=12)
    w_np, x_np = np.ascontiguousarray(wq), np.ascontiguousarray(x)
    y_np = np.zeros((1, M), np.float32)
    w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, M), w_np, backend=ggml_hip.GGML_BACKEND_GPU)
    L.ggml_hip_transform_tensor(w_np.ctypes.data_as(ctypes.c_void_p), ctypes.byref(w))
    assert w.extra
    xt = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, 1), x_np)
    y = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, 1), y_np)
    y.op = ggml_hip.GGML_OP_MUL_MAT
    y.src0 = ctypes.pointer(w)
    y.src1 = ctypes.pointer(xt)
    p = ggml_hip.GgmlComputeParams(ggml_hip.GGML_TASK_COMPUTE, 0, 1, 0, None)
    assert L.ggml_hip_compute_forward(ctypes.byref(p), ctypes.byref(y))   # any_on_device -> taken at N=1
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
    check_y(y_np, O.mul_mat(wq, K, x), s_abs, RTOL, ATOL_BLOCKS)
    L.ggml_hip_free_data(ctypes.byref(w))
    assert not w.extra


def test_graph_capture_replays_gemv():
    K, M = 4096, 512
    wq, x = make_case(K, M, 1, seed=13)
    wd, xd, yd = DB.from_array(wq), DB.from_array(x), DB(M * 4)
    L = ggml_hip.load()
    s = L.ggml_hip_default_stream()
    g = ggml_hip.Graph(s)
    with g:
        ggml_hip.mul_mat(wd, K, M, xd, 1, yd, stream=s)
    L.ggml_hip_memset(yd.ptr, 0, M * 4, s)
    g.launch()
    y = yd.download((1, M), np.float32, stream=s)
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
    check_y(y, O.mul_mat(wq, K, x), s_abs, RTOL, ATOL_BLOCKS)


# ------------------------------------------------------------------------------- RCCL split path (1 rank)
@pytest.mark.parametrize("N", [1, 3, 12])
def test_split_path_single_rank_rccl(N):
    """ggml_hip_mul_mat_q4_0_split through a real 1-rank RCCL communicator: the in-place
    all-gather (N=1) and the padded-slab + compaction path (N>1) equal the plain mul_mat."""
    L = ggml_hip.load()
    uid = ctypes.create_string_buffer(128)
    ggml_hip.check(L.ggml_hip_comm_unique_id(uid))
    comm = ctypes.c_void_p()
    ggml_hip.check(L.ggml_hip_comm_init(ctypes.byref(comm), 1, 0, uid), "comm_init")
    try:
        K, M = 4096, 320
        wq, x = make_case(K, M, N, seed=77 + N)
        wd, xd, yd = DB.from_array(wq), DB.from_array(x), DB(N * M * 4)
        rb = np.array([0, M], np.int64)
        ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split(comm, wd.ptr, K, M, rb.ctypes.data_as(ctypes.c_void_p),
                                                     xd.ptr, N, yd.ptr, None), "split")
        ggml_hip.check(L.ggml_hip_stream_synchronize(None))
        y = yd.download((N, M), np.float32)
        single, _ = gpu_mul_mat(wq, K, x)
        assert np.array_equal(y.view(np.uint32), single.view(np.uint32))
    finally:
        L.ggml_hip_comm_destroy(comm)


@pytest.mark.parametrize("N,Ms", [(1, (256, 256, 256)), (1, (512, 1376)), (3, (320, 64))])
def test_split_multi_single_rank_rccl(N, Ms):
    """ggml_hip_mul_mat_q4_0_split_multi (one multi-matrix GEMV + one grouped all-gather for the
    siblings; per-matrix split for N > 1) equals separate plain mul_mats bitwise."""
    L = ggml_hip.load()
    uid = ctypes.create_string_buffer(128)
    ggml_hip.check(L.ggml_hip_comm_unique_id(uid))
    comm = ctypes.c_void_p()
    ggml_hip.check(L.ggml_hip_comm_init(ctypes.byref(comm), 1, 0, uid), "comm_init")
    try:
        K, n = 4096, len(Ms)
        x = O.gaussian(N * K, 0x5EED2200 + N, 0.0, 1.0).reshape(N, K)
        cases = [make_case(K, M, N, seed=90 + i)[0] for i, M in enumerate(Ms)]
        wds = [DB.from_array(w) for w in cases]
        yds = [DB(N * M * 4) for M in Ms]
        rbs = [np.array([0, M], np.int64) for M in Ms]
        xd = DB.from_array(x)
        wp = (ctypes.c_void_p * n)(*[w.ptr for w in wds])
        mp = (ctypes.c_int64 * n)(*Ms)
        rp = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rbs])
        yp = (ctypes.c_void_p * n)(*[y.ptr for y in yds])
        ggml_hip.check(L.ggml_hip_mul_mat_q4_0_split_multi(comm, n, wp, mp, rp, K, xd.ptr, N, yp, None),
                       "split_multi")
        ggml_hip.check(L.ggml_hip_stream_synchronize(None))
        for w, M, yd in zip(cases, Ms, yds):
            single, _ = gpu_mul_mat(w, K, x)
            assert np.array_equal(yd.download((N, M), np.float32).view(np.uint32), single.view(np.uint32))
    finally:
        L.ggml_hip_comm_destroy(comm)


# ------------------------------------------------------------------------------- GEMV launch policies
@pytest.mark.parametrize("K,M,N", [(4096, 4544, 1), (4544, 4672, 1), (4096, 12288, 1), (11008, 300, 1),
                                   (13824, 333, 1), (4096, 9000, 2), (64, 37, 3)])
def test_gemv_launch_policies_bitwise_identical(K, M, N):
    """Every GEMV launch policy (row mapping strided / interleaved / blocked, ring depth 1 / 2, row
    items on / off, 1 / 2 workgroups per CU) does the same per-row fp32 arithmetic in the same
    order: y must be bitwise identical across all of them, and within the bound of the oracle."""
    L = ggml_hip.load()
    L.ggml_hip_debug_set_gemv_policy.argtypes = [ctypes.c_int] * 4
    wq, x = make_case(K, M, N, seed=K + 3 * M + N)
    ref = None
    try:
        for mp in (0, 1, 2):
            for depth in (1, 2):
                for rowitems in (0, 1):
                    for wg in (1, 2):
                        ggml_hip.check(L.ggml_hip_debug_set_gemv_policy(mp, depth, rowitems, wg), "policy")
                        y, _ = gpu_mul_mat(wq, K, x, algo=1)
                        if ref is None:
                            ref = y
                            _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
                            check_y(y, O.mul_mat(wq, K, x, nthreads=8), s_abs, RTOL, ATOL_BLOCKS)
                        else:
                            assert np.array_equal(y.view(np.uint32), ref.view(np.uint32)), (mp, depth, rowitems, wg)
    finally:
        ggml_hip.check(L.ggml_hip_debug_set_gemv_policy(-1, 0, 1, 0), "policy reset")


@pytest.mark.parametrize("K,M", [(18176, 4544), (13824, 5120), (12352, 333), (13824, 17), (24576, 6144),
                                 (16384, 4096), (16384, 4100), (49152, 600), (52224, 600)],
                         ids=["falcon-4h_to_h", "llama13b-w2", "k12352-ragged", "m17", "neox-4h_to_h",
                              "rwkv-ff_v", "rwkv-ff_v-row-tail", "lds-61k", "lds-over-64k-falls-back"])
def test_gemv_balanced_chunks(K, M):
    """The chunk-balanced decode GEMV (BAL, K > 12288: (row, chunk) items round-robin over a
    workgroup's waves, per-item sums combined in chunk order) against the oracle, forced on and off;
    deterministic (two runs bitwise equal), and independent of the row mapping: a sibling batch
    whose rows straddle workgroups gives the single calls' y bitwise."""
    L = ggml_hip.load()
    L.ggml_hip_debug_set_gemv_bal.argtypes = [ctypes.c_int]
    wq, x = make_case(K, M, 1, seed=7 * K + M)
    y_ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=False)
    s_abs = upper_s_abs(wq, O.quantize_q8_0(x, "avx2"), K)
    try:
        ys = {}
        for bal in (1, 0):
            ggml_hip.check(L.ggml_hip_debug_set_gemv_bal(bal), "bal")
            ys[bal], _ = gpu_mul_mat(wq, K, x, algo=1)
            check_y(ys[bal], y_ref, s_abs, RTOL, ATOL_BLOCKS)
        ggml_hip.check(L.ggml_hip_debug_set_gemv_bal(1), "bal")
        again, _ = gpu_mul_mat(wq, K, x, algo=1)
        assert np.array_equal(again.view(np.uint32), ys[1].view(np.uint32))
        if M >= 64:
            Ms = [M // 3, M - M // 3]
            parts = [np.ascontiguousarray(wq[:Ms[0]]), np.ascontiguousarray(wq[Ms[0]:])]
            wds = [DB.from_array(p) for p in parts]
            xd = DB.from_array(x)
            yds = [DB(m * 4) for m in Ms]
            ggml_hip.mul_mat_multi(wds, Ms, K, xd, 1, yds)
            got = np.concatenate([yd.download((1, m), np.float32) for yd, m in zip(yds, Ms)], axis=1)
            assert np.array_equal(got.view(np.uint32), ys[1].view(np.uint32))
    finally:
        ggml_hip.check(L.ggml_hip_debug_set_gemv_bal(-1), "bal reset")


# ------------------------------------------------------------------------------- weight-residency cache
def test_weight_cache_reuses_and_revalidates_host_weights():
    """a CPU-backend Q4_0 src0 is uploaded once per device and reused (bitwise
    same y); rewriting the host bytes in place is detected and re-uploaded (y follows the data)."""
    L = ggml_hip.load()
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    K, M, N = 4096, 192, 40
    wq, x = make_case(K, M, N, seed=21)
    w_np, x_np = np.ascontiguousarray(wq).copy(), np.ascontiguousarray(x)

    def stats():
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
        return h.value, m.value, r.value

    def run():
        y_np = np.zeros((N, M), np.float32)
        w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, M), w_np)
        xt = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, N), x_np)
        y = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, N), y_np)
        L.ggml_hip_mul_mat(ctypes.byref(w), ctypes.byref(xt), ctypes.byref(y))
        return y_np

    y1 = run()
    assert stats()[:2] == (0, 1) and stats()[2] == w_np.nbytes
    y2 = run()
    assert stats()[:2] == (1, 1)
    assert np.array_equal(y1.view(np.uint32), y2.view(np.uint32))
    _, s_abs = block_terms(wq, O.quantize_q8_0(x, "avx2"), K)
    check_y(y1, O.mul_mat(wq, K, x), s_abs, RTOL, ATOL_BLOCKS)
    wq2, _ = make_case(K, M, 1, seed=22)                 # same address, new bytes
    w_np[...] = wq2
    y3 = run()
    assert stats()[:2] == (1, 2)
    _, s_abs2 = block_terms(wq2, O.quantize_q8_0(x, "avx2"), K)
    check_y(y3, O.mul_mat(wq2, K, x), s_abs2, RTOL, ATOL_BLOCKS)
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    assert stats() == (0, 0, 0)


def test_weight_cache_invalidate_and_full_verify():
    """In-place edits the sampled fingerprint cannot see (one block between its sample points):
    ggml_hip_weight_cache_invalidate(ptr, bytes) drops the copy exactly (the next call re-uploads
    and y follows the new bytes), and GGML_HIP_WEIGHT_CACHE_VERIFY=full (set_verify(1)) detects the
    edit without any call.  Reference: the LoRA apply rewrites weights in place, llama.cpp:2950-2967."""
    L = ggml_hip.load()
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    K, M, N = 4096, 192, 40
    wq, x = make_case(K, M, N, seed=23)
    w_np, x_np = np.ascontiguousarray(wq).copy(), np.ascontiguousarray(x)
    n = w_np.nbytes
    flat = w_np.reshape(-1)

    def sampled(lo, hi):            # wcache_fingerprint's sampled byte windows
        win = [(0, 32), (n - 32, n)] + [((n // 64) * i + n // 128, (n // 64) * i + n // 128 + 8) for i in range(64)]
        return any(a < hi and lo < b for a, b in win)

    def stats():
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
        return h.value, m.value

    def run():
        y_np = np.zeros((N, M), np.float32)
        w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, M), w_np)
        xt = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, N), x_np)
        y = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, N), y_np)
        L.ggml_hip_mul_mat(ctypes.byref(w), ctypes.byref(xt), ctypes.byref(y))
        return y_np

    def expect(y):
        w2 = w_np.reshape(M, -1)
        _, s_abs = block_terms(w2, O.quantize_q8_0(x, "avx2"), K)
        check_y(y, O.mul_mat(w2, K, x), s_abs, RTOL, ATOL_BLOCKS)

    def edit_block(off):            # double the block's fp16 scale (exponent + 1): y of its row moves
        assert off % 18 == 0 and not sampled(off, off + 18)
        d = flat[off:off + 2].view(np.uint16)
        d[0] = np.uint16(d[0] + 0x0400) if (d[0] & 0x7C00) < 0x7800 else d[0]
        return off // (18 * K // 32)

    try:
        y0 = run()
        assert stats() == (0, 1)
        row = edit_block(18 * 4000)
        y_stale = run()                                   # sampled fingerprint: same bytes seen
        assert stats() == (1, 1)
        assert np.array_equal(y_stale.view(np.uint32), y0.view(np.uint32))
        dropped = L.ggml_hip_weight_cache_invalidate(ctypes.c_void_p(w_np.ctypes.data + 18 * 4000), 18)
        assert dropped == 1
        y1 = run()
        assert stats() == (1, 2)
        assert not np.array_equal(y1[:, row], y0[:, row])
        expect(y1)
        assert L.ggml_hip_weight_cache_invalidate(ctypes.c_void_p(w_np.ctypes.data + n + 4096), 16) == 0
        ggml_hip.check(L.ggml_hip_weight_cache_set_verify(1), "verify full")
        row2 = edit_block(18 * 9000)
        y2 = run()                                        # full fingerprint: the edit is a miss
        assert stats() == (1, 3)
        assert not np.array_equal(y2[:, row2], y1[:, row2])
        expect(y2)
        y3 = run()
        assert stats() == (2, 3)
        assert np.array_equal(y3.view(np.uint32), y2.view(np.uint32))
    finally:
        ggml_hip.check(L.ggml_hip_weight_cache_set_verify(-1), "verify reset")
        ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")


# ---------------------------------------------------- prefill GEMM v8 (int8 images) and v9 (fp6 images)
def _gemm_version(v):
    ggml_hip.check(ggml_hip.load().ggml_hip_debug_set_gemm_version(v), "gemm version")


GEMM_PER_CALL = {8: 9, 10: 11}          # image version -> the version that builds that image per call


def _image_bytes(K, M, v):
    return (M + 63) // 64 * 64 * K // 32 * 34 if v == 8 else (M + 127) // 128 * 128 * K // 32 * 26


@pytest.mark.parametrize("v", [9, 11], ids=["gemm8-int8", "gemm9-fp6"])
@pytest.mark.parametrize("K,M,N", [s for s in EDGE_SHAPES if s[2] > 8] + [(4544, 4672 // 8, 130), (128, 1, 200)])
def test_gemm8_per_call_image_vs_oracle(K, M, N, v):
    """k_gemm8 / k_gemm9 with the weight converted into the workspace per call (version 9 / 11): ragged M
    (images padded to 64 / 128 rows with d = 0), ragged N, K = 64 (one half-stage), K = 4544 (a partial
    last stage)."""
    wq, x = make_case(K, M, N, seed=K * 3 + M + N)
    _gemm_version(v)
    try:
        y, _ = gpu_mul_mat(wq, K, x, algo=2)
    finally:
        _gemm_version(-1)
    xq = O.quantize_q8_0(x, "avx2")
    _, s_abs = block_terms(wq, xq, K)
    check_y(y, O.mul_mat(wq, K, x, nthreads=4), s_abs, RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("K,M,N", [s for s in EDGE_SHAPES if s[2] > 8] +
                         [(4544, 4672, 130), (128, 1, 200), (4096, 4096, 512), (11008, 4096, 300), (4096, 11008, 257)])
def test_gemm9_fp6_bitwise_equals_gemm8_int8(K, M, N):
    """The fp6 block sums (v_mfma_scale_f32_32x32x64_f8f6f4 on e2m3 images, k_gemm9) are the same integers
    as the i8 MFMA's, and the two kernels share the block order, the workgroup-half K split and the scale
    product: y is bitwise equal, at edge shapes and full LLaMA-7B prefill shapes (q8_0 values over the
    whole int8 range, so the (q >> 4, q & 15) split sees every code)."""
    wq, x = make_case(K, M, N, seed=K * 5 + M + N)
    ys = {}
    _gemm9_wide(0)                                       # the 128 x 64 tile: k_gemm8's block order
    try:
        for v in (9, 11):
            _gemm_version(v)
            ys[v], _ = gpu_mul_mat(wq, K, x, algo=2)
    finally:
        _gemm_version(-1)
        _gemm9_wide(-1)
    assert np.array_equal(ys[9].view(np.uint32), ys[11].view(np.uint32))


def _gemm9_wide(mode):
    L = ggml_hip.load()
    L.ggml_hip_debug_set_gemm9_wide.argtypes = [ctypes.c_int]
    ggml_hip.check(L.ggml_hip_debug_set_gemm9_wide(mode), "gemm9 wide")


@pytest.mark.parametrize("K,M,N", [s for s in EDGE_SHAPES if s[2] > 8] +
                         [(4544, 4672, 130), (128, 1, 200), (4096, 4096, 1024), (11008, 4096, 300), (4096, 11008, 257)])
def test_gemm9_wide_tile_vs_oracle(K, M, N):
    """The 128 x 128 k_gemm9 tile (k_gemm9w_q4_0, forced): ragged M / N, K = 64 (one partial stage), K = 4544
    (a partial last stage), full LLaMA shapes; within the oracle bound, and within it of the 128 x 64 tile."""
    wq, x = make_case(K, M, N, seed=K * 7 + M + N)
    ys = {}
    try:
        _gemm_version(11)
        for mode in (0, 1):
            _gemm9_wide(mode)
            ys[mode], _ = gpu_mul_mat(wq, K, x, algo=2)
    finally:
        _gemm_version(-1)
        _gemm9_wide(-1)
    xq = O.quantize_q8_0(x, "avx2")
    _, s_abs = block_terms(wq, xq, K)
    ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=True)
    check_y(ys[1], ref, s_abs, RTOL, ATOL_BLOCKS)
    check_y(ys[1], ys[0], s_abs, RTOL, ATOL_BLOCKS)


def g9_wide_rows(Ms, N, cus=256):
    """csrc/q4_0_gemm.hip gemm9_run_multi's tile plan, restated: how many leading rows of the concatenated row tiles
    run the 128 x 128 tile (the rest 128 x 64): none when the 128 x 64 tiles fit one round; one or more whole
    128 x 128 rounds' row tiles when the 128 x 128 tiles would leave a last round at most half full (mixed); all
    otherwise (wide_pays)."""
    Mt = sum((M + 127) // 128 for M in Ms)
    tiles, tiles_w = Mt * ((N + 63) // 64), Mt * ((N + 127) // 128)
    total = sum(Ms)
    if tiles <= cus:
        return 0
    rem_w = tiles_w % cus
    if tiles_w > cus and rem_w > 0 and 2 * rem_w <= cus:
        return min(total, 128 * ((tiles_w // cus) * cus // ((N + 127) // 128)))
    if tiles_w <= cus or tiles_w >= 2 * cus or 2 * (tiles_w - cus) > cus:
        return total
    return 0


def test_gemm9_auto_tile_takes_wide_for_llama_w1w3():
    """The automatic tile plan (256 CUs): the LLaMA-7B w1|w3 group at 512 tokens (1,376 128 x 64 tiles; 688
    128 x 128 = 2.7 rounds) and q|k|v at 256 tokens (192 128 x 128 tiles: one round) run the wide tile; q|k|v at
    512 tokens (384 wide tiles: a last round half full) runs one round of it (wq, wk) and wv as 128 x 64; wo at 512
    tokens (256 128 x 64 tiles: one round) keeps 128 x 64.  Every row bitwise the forced result of its tile."""
    L = ggml_hip.load()
    K = 4096
    x = make_case(K, 8, 512, seed=77)[1]
    for Ms, N in (([11008, 11008], 512), ([4096, 4096, 4096], 512), ([4096, 4096, 4096], 256), ([4096], 512)):
        xd = DB.from_array(np.ascontiguousarray(x[:N]))
        cases = [make_case(K, M, 1, seed=900 + 3 * i + M)[0] for i, M in enumerate(Ms)]
        wds = [DB.from_array(c) for c in cases]
        for wd, M in zip(wds, Ms):
            ggml_hip.check(L.ggml_hip_weight_image_create(wd.ptr, K, M, None), "image")
        try:
            out = {}
            for mode in (-1, 0, 1):
                _gemm9_wide(mode)
                ys = [DB(N * M * 4) for M in Ms]
                ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
                out[mode] = np.concatenate([y.download((N, M), np.float32).view(np.uint32) for y, M in zip(ys, Ms)], 1)
        finally:
            _gemm9_wide(-1)
            for wd in wds:
                L.ggml_hip_weight_image_free(wd.ptr)
        cut = g9_wide_rows(Ms, N)
        assert np.array_equal(out[-1][:, :cut], out[1][:, :cut]), (Ms, N, cut)
        assert np.array_equal(out[-1][:, cut:], out[0][:, cut:]), (Ms, N, cut)
    assert [g9_wide_rows(*c) for c in (([11008, 11008], 512), ([4096] * 3, 512), ([4096] * 3, 256), ([4096], 512))] == \
        [22016, 8192, 12288, 0]


def test_gemm9_fp6_extreme_blocks_exact():
    """Blocks whose q8_0 values hit -128 / 127 / 0 and whose nibbles are all 0 (w = -8) or all 15 (w = 7):
    the largest block sums (|sumi| = 32 * 8 * 128) and every e2m3 code at its extremes, against the oracle."""
    K, M, N = 256, 64, 160
    rng = np.random.default_rng(7)
    w = rng.standard_normal((M, K)).astype(np.float32) * 0.02
    w[:8] = -1.0                                        # d = +0.125: all nibbles 0 -> w = -8
    w[8:16] = np.where(np.arange(K) % 32 == 0, -1.0, 0.875).astype(np.float32)
    wq, _ = O.quantize_q4_0(w)
    x = rng.standard_normal((N, K)).astype(np.float32)
    x[:8] = 1.0
    x[8:16] = -1.0
    x[16:24, ::2] = 0.0
    xq = O.quantize_q8_0(x, "avx2")
    _gemm_version(11)
    try:
        y, _ = gpu_mul_mat(wq, K, x, algo=2)
    finally:
        _gemm_version(-1)
    _, s_abs = block_terms(wq, xq, K)
    check_y(y, O.mul_mat(wq, K, x, nthreads=4), s_abs, RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("v", [8, 10], ids=["int8-image", "fp6-image"])
@pytest.mark.parametrize("K,M", [(4096, 4096), (11008, 4096)])
def test_gemm8_registered_image_prefill_512(K, M, v):
    """A registered weight image (ggml_hip_weight_image_create; int8 under version 8, fp6 under the
    default 10) is used by every later prefill call of that weight: bitwise equal to the per-call image,
    within the bound of the oracle at full LLaMA-7B shape, x -> 2x bitwise; freeing the image returns the
    GEMM to the q4_0 bytes (k_gemm7)."""
    L = ggml_hip.load()
    wq, x = make_case(K, M, 512, seed=11 * K + M)
    wd, xd = DB.from_array(wq), DB.from_array(x)
    yd = DB(512 * M * 4)
    before = L.ggml_hip_weight_image_bytes()
    _gemm_version(v)
    ggml_hip.check(L.ggml_hip_weight_image_create(wd.ptr, K, M, None), "image")
    assert L.ggml_hip_weight_image_bytes() - before == _image_bytes(K, M, v)
    try:
        ggml_hip.mul_mat(wd, K, M, xd, 512, yd, algo=2)
        y_img = yd.download((512, M), np.float32)
        _gemm_version(GEMM_PER_CALL[v])
        y_call, _ = gpu_mul_mat(wq, K, x, algo=2)
        _gemm_version(v)
        assert np.array_equal(y_img.view(np.uint32), y_call.view(np.uint32))
        xq = O.quantize_q8_0(x, "avx2")
        y_ref = O.mul_mat(wq, K, x, nthreads=8, mode="avx2", pool=True)
        rel, _ = check_y(y_img, y_ref, upper_s_abs(wq, xq, K), RTOL, ATOL_BLOCKS)
        assert rel < 1e-3
        x2 = DB.from_array(2 * x)
        ggml_hip.mul_mat(wd, K, M, x2, 512, yd, algo=2)
        assert np.array_equal(yd.download((512, M), np.float32).view(np.uint32), (2 * y_img).view(np.uint32))
    finally:
        _gemm_version(-1)
        assert L.ggml_hip_weight_image_free(wd.ptr) == 1
    assert L.ggml_hip_weight_image_bytes() == before
    ggml_hip.mul_mat(wd, K, M, xd, 512, yd, algo=2)                       # k_gemm7 again
    y7 = yd.download((512, M), np.float32)
    check_y(y7, y_ref, upper_s_abs(wq, xq, K), RTOL, ATOL_BLOCKS)


@pytest.mark.parametrize("K,M,N", [(4096, 4096, 96), (4096, 11008, 65), (11008, 4096, 128), (4544, 584, 100),
                                   (4096, 11008, 16), (5120, 13824, 9)])
def test_image_gemm_below_prefill_threshold(K, M, N):
    """A weight with an image takes the image GEMM (k_gemm9) from N > 64, and tall ones (M >= 8192) at
    any N above the GEMV's, in auto mode (otherwise, and without an image, the split-K GEMM on the q4_0
    bytes): bitwise equal to the forced per-call fp6 image (version 11, algo 2), within the bound of the
    oracle; without the image auto mode is the split-K result."""
    L = ggml_hip.load()
    wq, x = make_case(K, M, N, seed=13 * K + M + N)
    wd, xd = DB.from_array(wq), DB.from_array(x)
    yd = DB(N * M * 4)
    ggml_hip.mul_mat(wd, K, M, xd, N, yd)                                   # auto, no image: split-K
    y_sk = yd.download((N, M), np.float32)
    y_sk3, _ = gpu_mul_mat(wq, K, x, algo=3)
    assert np.array_equal(y_sk.view(np.uint32), y_sk3.view(np.uint32))
    ggml_hip.check(L.ggml_hip_weight_image_create(wd.ptr, K, M, None), "image")
    try:
        ggml_hip.mul_mat(wd, K, M, xd, N, yd)                               # auto with the image
        y_img = yd.download((N, M), np.float32)
        _gemm_version(11)
        try:
            y_call, _ = gpu_mul_mat(wq, K, x, algo=2)
        finally:
            _gemm_version(-1)
        assert np.array_equal(y_img.view(np.uint32), y_call.view(np.uint32))
        xq = O.quantize_q8_0(x, "avx2")
        _, s_abs = block_terms(wq, xq, K)
        check_y(y_img, O.mul_mat(wq, K, x, nthreads=4), s_abs, RTOL, ATOL_BLOCKS)
    finally:
        assert L.ggml_hip_weight_image_free(wd.ptr) == 1


def test_mixed_sibling_group_at_96_tokens_bitwise():
    """N = 96: a sibling group whose weights have / lack images runs k_gemm9 and the split-K GEMM side
    by side on one x (two x forms), bitwise equal to separate calls."""
    L = ggml_hip.load()
    K, N = 4096, 96
    Ms = [256, 4096, 300]
    cases = [make_case(K, M, N, seed=90 + i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    wds = [DB.from_array(c[0]) for c in cases]
    ggml_hip.check(L.ggml_hip_weight_image_create(wds[1].ptr, K, Ms[1], None), "image")
    try:
        xd = DB.from_array(x)
        ys = [DB(N * M * 4) for M in Ms]
        ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
        for wd, yd, M in zip(wds, ys, Ms):
            single = DB(N * M * 4)
            ggml_hip.mul_mat(wd, K, M, xd, N, single)
            assert np.array_equal(yd.download((N, M), np.float32).view(np.uint32),
                                  single.download((N, M), np.float32).view(np.uint32))
    finally:
        L.ggml_hip_weight_image_free(wds[1].ptr)


def test_gemm8_mixed_sibling_group_bitwise():
    """A sibling group (one x quantization per form) where the weights have an fp6 image, an int8 image,
    none, and an fp6 image again: the k_gemm9, k_gemm8 and k_gemm7 siblings each read their own x form (the
    fp6 and int8 x images share one region, rewritten when the form changes), bitwise equal to separate
    calls."""
    L = ggml_hip.load()
    K, N = 4096, 200
    Ms = [256, 128, 300, 192]
    cases = [make_case(K, M, N, seed=60 + i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    wds = [DB.from_array(c[0]) for c in cases]
    try:
        for i, v in ((0, 10), (1, 8), (3, 10)):
            _gemm_version(v)
            ggml_hip.check(L.ggml_hip_weight_image_create(wds[i].ptr, K, Ms[i], None), "image")
        _gemm_version(-1)
        xd = DB.from_array(x)
        ys = [DB(N * M * 4) for M in Ms]
        ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
        for wd, yd, M in zip(wds, ys, Ms):
            single = DB(N * M * 4)
            ggml_hip.mul_mat(wd, K, M, xd, N, single)
            assert np.array_equal(yd.download((N, M), np.float32).view(np.uint32),
                                  single.download((N, M), np.float32).view(np.uint32))
        xq = O.quantize_q8_0(x, "avx2")
        for i in (0, 1):
            _, s_abs = block_terms(cases[i][0], xq, K)
            check_y(ys[i].download((N, Ms[i]), np.float32), O.mul_mat(cases[i][0], K, x, nthreads=4), s_abs, RTOL,
                    ATOL_BLOCKS)
    finally:
        _gemm_version(-1)
        for i in (0, 1, 3):
            L.ggml_hip_weight_image_free(wds[i].ptr)


@pytest.mark.parametrize("K,Ms,N", [
    (4096, [4096, 4096, 4096], 512),          # LLaMA-7B wq|wk|wv prefill: one k_gemm9 launch, 768 tiles
    (4096, [11008, 11008], 512),              # w1|w3: 1376 tiles (XCD-aware order, C = 172)
    (4096, [300, 128, 4096, 200], 200),       # ragged row tiles, 4 siblings, ragged token tile
    (4544, [4672, 4544], 100),                # Falcon shapes, N just above IMG_MIN_N
    (4096, [129, 11008], 40),                 # tall sibling below IMG_MIN_N with a short one (both imaged)
])
@pytest.mark.parametrize("wide", [0, 1], ids=["tile128x64", "tile128x128"])
def test_gemm9_sibling_group_one_launch_bitwise(K, Ms, N, wide):
    """Siblings that all have fp6 images run as ONE k_gemm9 launch over their row tiles (the x image built
    once): every y bitwise equal to a separate call per matrix with the same tile, within the oracle bound."""
    L = ggml_hip.load()
    _gemm9_wide(wide)
    cases = [make_case(K, M, N, seed=700 + 7 * i + M) for i, M in enumerate(Ms)]
    x = cases[0][1]
    wds = [DB.from_array(c[0]) for c in cases]
    for wd, M in zip(wds, Ms):
        ggml_hip.check(L.ggml_hip_weight_image_create(wd.ptr, K, M, None), "image")
    try:
        xd = DB.from_array(x)
        ys = [DB(N * M * 4) for M in Ms]
        ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys)
        outs = [yd.download((N, M), np.float32) for yd, M in zip(ys, Ms)]
        for wd, y, M in zip(wds, outs, Ms):
            single = DB(N * M * 4)
            ggml_hip.mul_mat(wd, K, M, xd, N, single)
            assert np.array_equal(y.view(np.uint32), single.download((N, M), np.float32).view(np.uint32))
        i = min(range(len(Ms)), key=lambda k: Ms[k])            # the oracle on the smallest sibling
        xq = O.quantize_q8_0(x, "avx2")
        check_y(outs[i], O.mul_mat(cases[i][0], K, x, nthreads=8, mode="avx2", pool=True),
                s_abs_exact(cases[i][0], xq, K), RTOL, ATOL_BLOCKS)
    finally:
        _gemm9_wide(-1)
        for wd in wds:
            L.ggml_hip_weight_image_free(wd.ptr)


def test_multi_mixed_image_siblings_fresh_stream_workspace():
    """a sibling group at a split-K N (gemv_max < N <= 64) whose tall middle sibling has an fp6
    image takes the image GEMM, which needs the larger workspace; on a fresh stream (empty workspace) the
    group must size it before the first sibling quantizes x into it, or the third sibling reads a freed
    buffer.  Every y bitwise equal to one call per matrix on the default stream."""
    L = ggml_hip.load()
    K, N, Ms = 4096, 32, (4096, 11008, 4096)
    cases = [make_case(K, M, N, seed=900 + i) for i, M in enumerate(Ms)]
    x = cases[0][1]
    wds = [DB.from_array(c[0]) for c in cases]
    ggml_hip.check(L.ggml_hip_weight_image_create(wds[1].ptr, K, Ms[1], None), "image")
    s = L.ggml_hip_stream_create()
    try:
        xd = DB.from_array(x)
        ys = [DB(N * M * 4) for M in Ms]
        for y in ys:
            L.ggml_hip_memset(y.ptr, 0x7F, y.nbytes, s)
        ggml_hip.mul_mat_multi(wds, Ms, K, xd, N, ys, stream=s)
        ggml_hip.check(L.ggml_hip_stream_synchronize(s))
        for wd, y, M in zip(wds, ys, Ms):
            single = DB(N * M * 4)
            ggml_hip.mul_mat(wd, K, M, xd, N, single)
            got = y.download((N, M), np.float32, stream=s)
            assert np.array_equal(got.view(np.uint32), single.download((N, M), np.float32).view(np.uint32)), M
    finally:
        L.ggml_hip_stream_destroy(s)
        L.ggml_hip_weight_image_free(wds[1].ptr)


def test_gemm8_image_api_errors():
    L = ggml_hip.load()
    wq, _ = make_case(128, 64, 1, seed=3)
    wd = DB.from_array(wq)
    assert L.ggml_hip_weight_image_create(wd.ptr, 96, 64, None) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_weight_image_create(None, 128, 64, None) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_weight_image_free(wd.ptr) == 0
    assert L.ggml_hip_debug_set_gemm_version(5) == ggml_hip.ERR_INVALID
    assert L.ggml_hip_debug_set_gemm_version(12) == ggml_hip.ERR_INVALID
