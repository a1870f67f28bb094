"""The prefill producers that write the k_gemm9 x image beside their f32 output (csrc/ggml_ops.hip
k_row_norm4<true>, k_silu_mul_x9; used by the hook's x image fold): their output is
bitwise the chain's own kernel's, and their image is bitwise what gemm9_prep_x (k_prep9_x) makes of that
output, at ragged token counts (grids padded to 64 rows with the XCD-local row mapping, Np = N rounded up
to 4) and the LLaMA / 13B / Falcon widths.  The chains themselves are pinned against the reference's CPU
ops end to end (tests/test_gpu_llama_ggjt.py)."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer


@pytest.mark.parametrize("kind,K,N,with_add", [(1, 4096, 65, True), (1, 4096, 512, False), (1, 5120, 97, True),
                                               (1, 64, 130, False), (1, 16384, 67, True), (2, 11008, 97, False),
                                               (2, 11008, 512, False), (2, 13824, 66, False), (2, 128, 200, False)])
def test_x9_producers_bitwise(kind, K, N, with_add):
    L = ggml_hip.load()
    L.ggml_hip_debug_x9_producer.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 7 + [ctypes.c_int64] * 2 + \
        [ctypes.c_void_p] * 2
    rng = np.random.default_rng(kind * 100000 + K + N)
    if kind == 1:
        a = DB.from_array(rng.standard_normal((N, K)).astype(np.float32)) if with_add else None
        b = DB.from_array(rng.standard_normal((N, K)).astype(np.float32))
        w = DB.from_array((1.0 + 0.1 * rng.standard_normal(K)).astype(np.float32))
        s_, n_ = (DB(N * K * 4), DB(N * K * 4)) if with_add else (None, None)
    else:
        a = DB.from_array((3.0 * rng.standard_normal((N, K))).astype(np.float32))
        b = DB.from_array(rng.standard_normal((N, K)).astype(np.float32))
        w, s_, n_ = None, None, DB(N * K * 4)
    out, out_ref = DB(N * K * 4), DB(N * K * 4)
    nbytes = (K // 32) * ((N + 3) & ~3) * 50
    img = DB.from_array(np.zeros(nbytes, np.uint8))
    img_ref = DB.from_array(np.zeros(nbytes, np.uint8))
    p = lambda x: x.ptr if x is not None else None
    ggml_hip.check(L.ggml_hip_debug_x9_producer(kind, p(a), p(b), p(w), p(s_), p(n_), out.ptr, out_ref.ptr, K, N,
                                                img.ptr, img_ref.ptr), "x9 producer")
    o = out.download((N, K), np.float32)
    assert np.isfinite(o).all()
    assert np.array_equal(o.view(np.uint32), out_ref.download((N, K), np.float32).view(np.uint32))
    got, ref = img.download((nbytes,), np.uint8), img_ref.download((nbytes,), np.uint8)
    assert ref.any()
    assert np.array_equal(got, ref), int(np.flatnonzero(got != ref)[0])
