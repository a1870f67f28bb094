"""The reference's own ggml.c drives the MI355X backend through its own GPU hooks.

oracle/_ref/libggml_ref_hip.so is the reference ggml.c compiled unmodified with -DGGML_USE_CUBLAS
and linked against libggml_hip_cuda.so (include/ggml-hip-cuda-abi.h, the ggml-cuda.h names as
aliases of ggml-hip.h).  A q4_0 mul_mat graph built and computed by ggml (ggml_init ->
ggml_init_cublas, planner can_mul_mat, ggml_compute_forward -> ggml_cuda_compute_forward) must:
  * run on the GPU when the weight is offloaded (llama.cpp's loader: backend = GPU, then
    ggml_cuda_transform_tensor) or when N >= 32 (can_mul_mat, weights uploaded per call), with y
    within the north-star bound of the reference's CPU result (the golden vectors / the oracle,
    which is bit-exact to the reference's AVX2 build);
  * fall back to ggml's own CPU op, bit-exact to the AVX2 reference, for what the backend
    declines (a CPU weight with N < 32), exactly like the CUDA backend.
The library is built in this container from /root/reference (oracle/Makefile `ref`); the test is
skipped where it was not built.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from golden_io import load
from hip_env import ROOT, gpu_available
from parity import block_terms, check_y

LIB = os.path.join(ROOT, "oracle", "_ref", "libggml_ref_hip.so")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so"),
              pytest.mark.skipif(not os.path.exists(LIB), reason="oracle/_ref/libggml_ref_hip.so not built")]

RTOL, ATOL_BLOCKS = 1e-3, 1e-6
GGML_BACKEND_CPU = 0


@pytest.fixture(scope="module")
def ref():
    lib = ctypes.CDLL(LIB)
    lib.refhip_mul_mat.restype = ctypes.c_int
    lib.refhip_mul_mat.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.refhip_has_gpublas.restype = ctypes.c_int
    return lib


def ggml_mul_mat(ref, wq, K, x, offload, n_threads):
    wq = np.ascontiguousarray(wq, np.uint8)
    x = np.ascontiguousarray(x, np.float32)
    M, N = wq.shape[0], x.shape[0]
    y = np.full((N, M), np.nan, np.float32)
    be = ref.refhip_mul_mat(wq.ctypes.data, K, M, x.ctypes.data, N, y.ctypes.data, offload, n_threads)
    assert be >= 0
    return y, be


def assert_close(wq, x, K, y, y_ref):
    xq = O.quantize_q8_0(x)
    _, s_abs = block_terms(wq, xq, K)
    rel, _ = check_y(y, y_ref, s_abs, rtol=RTOL, atol_blocks=ATOL_BLOCKS)
    assert rel < RTOL


def test_hooks_present(ref):
    assert ref.refhip_has_gpublas() == 1          # ggml_cpu_has_cublas(): built with the GPU hooks


@pytest.mark.parametrize("n_threads", [1, 4])
@pytest.mark.parametrize("offload", [1, 2])
def test_offloaded_weight_golden(ref, offload, n_threads):
    wq, x = load("avx2", "w4096_q4_0"), load("avx2", "x4096_f32")
    y, _ = ggml_mul_mat(ref, wq, 4096, x, offload, n_threads)
    assert np.isfinite(y).all()
    assert_close(wq, x, 4096, y, load("avx2", "y4096_mul_mat"))


def test_offloaded_weight_falcon_golden(ref):
    wq, x = load("avx2", "w4544_q4_0"), load("avx2", "x4544_f32")
    y, _ = ggml_mul_mat(ref, wq, 4544, x, 1, 2)
    assert_close(wq, x, 4544, y, load("avx2", "y4544_mul_mat"))


@pytest.mark.parametrize("K,M,N,offload", [(4096, 256, 32, 0), (4096, 512, 64, 0), (11008, 128, 48, 1),
                                           (4096, 300, 512, 1), (4544, 4672 // 8, 33, 0)])
def test_prefill_through_ggml(ref, K, M, N, offload):
    """Prefill through ggml's own hooks; an offloaded weight at N > 128 gets its weight image on first use
    (fp6, k_gemm9, under the default GEMM version), released with the tensor by ggml_cuda_free_data."""
    from hip_env import ggml_hip
    L = ggml_hip.load()
    before = L.ggml_hip_weight_image_bytes()
    wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED7000 + K + M, 0.0, 0.02).reshape(M, K))
    x = O.gaussian(N * K, 0x5EED7100 + N, 0.0, 1.0).reshape(N, K)
    y, _ = ggml_mul_mat(ref, wq, K, x, offload, 4)
    assert_close(wq, x, K, y, O.mul_mat(wq, K, x))
    assert L.ggml_hip_weight_image_bytes() == before        # the driver frees the weight: image dropped


def test_declined_node_runs_reference_cpu_op(ref):
    """CPU weight and N < 32: can_mul_mat is false, ggml computes it itself (AVX2 vec_dot), so
    the result is the reference's CPU result bit for bit."""
    wq, x = load("avx2", "w4096_q4_0"), load("avx2", "x4096_f32")
    y, be = ggml_mul_mat(ref, wq, 4096, x, 0, 2)
    assert be == GGML_BACKEND_CPU
    assert np.array_equal(y.view(np.uint32), load("avx2", "y4096_mul_mat").view(np.uint32))


@pytest.mark.parametrize("N", [1, 4, 31])
def test_large_cpu_weight_taken_at_decode(ref, N):
    """The deliberate deviation from ggml-cuda.cu:2595-2610: a CPU-backend Q4_0
    weight of >= GGML_HIP_DECODE_MIN_WEIGHTS (2^19) elements is taken at N < 32 (the reference would
    decline it, since it re-uploads host weights per call, ggml-cuda.cu:2496-2502).  The node must
    reach the backend (one residency-cache upload, then hits), with y within the bound of the oracle."""
    from hip_env import ggml_hip
    L = ggml_hip.load()
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    K, M = 4096, 128                                       # 2^19 elements: exactly the threshold
    wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED7500 + N, 0.0, 0.02).reshape(M, K))
    x = O.gaussian(N * K, 0x5EED7600 + N, 0.0, 1.0).reshape(N, K)

    def stats():
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
        return h.value, m.value

    try:
        y, be = ggml_mul_mat(ref, wq, K, x, 0, 2)
        assert be == GGML_BACKEND_CPU
        assert stats() == (0, 1)                            # taken: the weight was uploaded once
        y2, _ = ggml_mul_mat(ref, wq, K, x, 0, 2)
        assert stats() == (1, 1)                            # and reused on the next call
        assert np.array_equal(y.view(np.uint32), y2.view(np.uint32))
        assert_close(wq, x, K, y, O.mul_mat(wq, K, x))
        # one row short of the threshold: declined, ggml's own CPU op (bitwise the oracle)
        w_small = np.ascontiguousarray(wq[:M - 1])
        ys, _ = ggml_mul_mat(ref, w_small, K, x, 0, 2)
        assert stats() == (1, 1)
        assert np.array_equal(ys.view(np.uint32), O.mul_mat(w_small, K, x).view(np.uint32))
    finally:
        ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")


def test_cached_weight_image_counted_in_cache_budget(ref):
    """a residency-cache copy of a host weight that gets its fp6 image at its first prefill
    (N > 64 through can_mul_mat) counts the image's bytes in the cache's resident total, the quantity the
    LRU budget GGML_HIP_WEIGHT_CACHE_MB bounds; clearing the cache releases copy and image together."""
    from hip_env import ggml_hip
    L = ggml_hip.load()
    L.ggml_hip_weight_image_bytes.restype = ctypes.c_int64
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    K, M, N = 4096, 256, 96
    wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED7700, 0.0, 0.02).reshape(M, K))
    x = O.gaussian(N * K, 0x5EED7800, 0.0, 1.0).reshape(N, K)

    def resident():
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
        return r.value

    img0 = L.ggml_hip_weight_image_bytes()
    try:
        y, be = ggml_mul_mat(ref, wq, K, x, 0, 2)
        assert be == GGML_BACKEND_CPU
        assert_close(wq, x, K, y, O.mul_mat(wq, K, x))
        img = L.ggml_hip_weight_image_bytes() - img0
        assert img == ((M + 127) // 128) * (K // 32) * 128 * 26        # the fp6 image (26 B per 32 weights)
        assert resident() == M * K // 32 * 18 + img
    finally:
        ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    assert resident() == 0
    assert L.ggml_hip_weight_image_bytes() == img0


def _device_count():
    try:
        from hip_env import ggml_hip
        return ggml_hip.device_count()
    except Exception:
        return 0


@pytest.mark.skipif(_device_count() < 2, reason="needs >= 2 HIP devices (GPU_SPLIT across devices)")
@pytest.mark.parametrize("fractions", [None, (1.0, 3.0)])
@pytest.mark.parametrize("N", [4, 64])
def test_gpu_split_across_devices(ref, fractions, N):
    """GGML_BACKEND_GPU_SPLIT with the rows on 2+ devices (llama.cpp -ts, ggml-cuda.cu:2286-2567):
    every device's slice is enqueued before the single per-device synchronize, slices gathered
    by one peer copy + one 2-D copy each; y within the bound of the reference's CPU result."""
    ndev = _device_count()
    if fractions is not None:
        fr = (ctypes.c_float * 16)(*(list(fractions) + [0.0] * (16 - len(fractions))))
        ref.ggml_cuda_set_tensor_split(fr)
    try:
        K, M = 4096, 1000 + 8 * ndev
        wq, _ = O.quantize_q4_0(O.gaussian(M * K, 0x5EED7300 + N, 0.0, 0.02).reshape(M, K))
        x = O.gaussian(N * K, 0x5EED7400 + N, 0.0, 1.0).reshape(N, K)
        y, _ = ggml_mul_mat(ref, wq, K, x, 2, 4)
        assert_close(wq, x, K, y, O.mul_mat(wq, K, x))
    finally:
        if fractions is not None:
            ref.ggml_cuda_set_tensor_split((ctypes.c_float * 16)(*([1.0] * ndev + [0.0] * (16 - ndev))))


def test_lora_in_place_add_invalidates_cached_weight(ref):
    """The reference's LoRA apply (llama.cpp:2935-2967): ggml_add_inplace(W_q4_0, delta) runs on
    ggml's CPU op (add_q_f32 requantizes every block in place).  The backend sees that node's INIT
    (ggml.c:17112-17116), drops the cached device copy of W, and the next mul_mat through ggml
    (N >= 32, can_mul_mat) uses the new bytes: y within the bound of the oracle on W_after."""
    L = __import__("hip_env").ggml_hip.load()
    __import__("hip_env").ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    K, M, N = 4096, 128, 40
    wf = O.gaussian(M * K, 0x5EED5100, 0.0, 0.02).reshape(M, K)
    wq, _ = O.quantize_q4_0(wf)
    x = O.gaussian(N * K, 0x5EED5200, 0.0, 1.0).reshape(N, K)
    delta = O.gaussian(M * K, 0x5EED5300, 0.0, 0.01).reshape(M, K)
    wq = np.ascontiguousarray(wq, np.uint8)
    y0 = np.full((N, M), np.nan, np.float32)
    y1 = np.full((N, M), np.nan, np.float32)
    w_after = np.zeros_like(wq)
    counts = np.zeros(3, np.int64)
    ref.refhip_lora_add.restype = ctypes.c_int
    ref.refhip_lora_add.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int]
    rc = ref.refhip_lora_add(wq.ctypes.data, K, M, np.ascontiguousarray(x, np.float32).ctypes.data, N,
                             np.ascontiguousarray(delta, np.float32).ctypes.data, y0.ctypes.data, y1.ctypes.data,
                             w_after.ctypes.data, counts.ctypes.data, 4)
    assert rc == 0
    assert not np.array_equal(w_after, wq)                 # the CPU op rewrote W in place
    assert counts[2] >= 1, counts                          # the add node invalidated the cached copy
    assert counts[1] == 2, counts                          # two uploads: before and after the edit
    assert_close(wq, x, K, y0, O.mul_mat(wq, K, x))
    assert_close(w_after, x, K, y1, O.mul_mat(w_after, K, x))


@pytest.mark.parametrize("poison", [0, 1])
def test_graph_ending_on_held_device_node_survives_ggml_free(ref, poison):
    """A graph whose final node is device-only (silu of an offloaded rms_norm) leaves that node held
    by the backend's launch fusion when ggml_graph_compute returns.  The caller frees the context
    (and here overwrites its arena) before synchronizing: the held node runs from the backend's own
    snapshot, and y is bitwise equal to ggml's CPU ops (rms_norm ggml.c:10389, silu 10188)."""
    n, rows = 4096, 3
    x = O.gaussian(n * rows, 0x5EED5400, 0.0, 1.0).astype(np.float32)
    y = np.full(n * rows, np.nan, np.float32)
    y_cpu = np.full(n * rows, np.nan, np.float32)
    ref.refhip_device_tail.restype = ctypes.c_int
    ref.refhip_device_tail.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int, ctypes.c_int]
    assert ref.refhip_device_tail(x.ctypes.data, n, rows, y.ctypes.data, y_cpu.ctypes.data, poison, 2) == 0
    assert np.all(np.isfinite(y_cpu))
    assert np.array_equal(y.view(np.uint32), y_cpu.view(np.uint32))
