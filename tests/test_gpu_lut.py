"""ggml's fp16 lookup tables (table_silu_f16 / table_exp_f16, ggml.c:4246-4254) evaluated directly on the
device (csrc/q4_0_device.h lut_silu / lut_exp): the backend checks the direct evaluation against the host-built
tables over every finite fp16 input when it builds them, and only then tags the kernels' table pointers for
direct evaluation.  Here: the check found no difference on this MI355X (every one of the 63,488 finite inputs
of each table reproduced bit for bit), and the silu consumers give bitwise the same outputs with gathers and
with direct evaluation.  The ops stay pinned against the reference's CPU ops end to end in exact mode
(tests/test_gpu_llama_ggjt.py, tests/test_gpu_ggml_hook.py)."""
import ctypes

import numpy as np
import pytest

from hip_env import ggml_hip, gpu_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so")]

DB = ggml_hip.DeviceBuffer


def lut_state(L, on=-1):
    L.ggml_hip_debug_lut_direct.argtypes = [ctypes.c_int, ctypes.c_void_p]
    out = np.zeros(4, np.int32)
    ggml_hip.check(L.ggml_hip_debug_lut_direct(on, out.ctypes.data), "lut_direct")
    return [int(v) for v in out]


def test_direct_evaluation_reproduces_every_finite_table_entry():
    L = ggml_hip.load()
    silu_mode, silu_bad, exp_mode, exp_bad = lut_state(L, 1)
    assert (silu_bad, exp_bad) == (0, 0), (silu_bad, exp_bad)
    assert (silu_mode, exp_mode) == (1, 1)
    assert lut_state(L, 0)[0::2] == [0, 0]                 # switched off: gathers
    assert lut_state(L, 1)[0::2] == [1, 1]


@pytest.mark.parametrize("K,N", [(11008, 97), (128, 200), (4096, 1)])
def test_silu_consumers_direct_equals_gather(K, N):
    """k_silu_mul_x9 (image + output) and k_silu_mul with the table gathers and with direct evaluation:
    bitwise the same outputs, inputs spread over the whole fp16 range (large, tiny, negative)."""
    L = ggml_hip.load()
    L.ggml_hip_debug_x9_producer.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 7 + [ctypes.c_int64] * 2 + \
        [ctypes.c_void_p] * 2
    rng = np.random.default_rng(K + N)
    av = (rng.standard_normal((N, K)) * np.exp2(rng.integers(-14, 15, (N, K)))).astype(np.float32)
    a = DB.from_array(av)
    b = DB.from_array(rng.standard_normal((N, K)).astype(np.float32))
    nbytes = (K // 32) * ((N + 3) & ~3) * 50
    res = {}
    try:
        for on in (0, 1):
            lut_state(L, on)
            n_, out, out_ref = DB(N * K * 4), DB(N * K * 4), DB(N * K * 4)
            img = DB.from_array(np.zeros(nbytes, np.uint8))
            img_ref = DB.from_array(np.zeros(nbytes, np.uint8))
            ggml_hip.check(L.ggml_hip_debug_x9_producer(2, a.ptr, b.ptr, None, None, n_.ptr, out.ptr, out_ref.ptr, K, N,
                                                        img.ptr, img_ref.ptr), "x9 producer")
            res[on] = [x.download((N, K), np.float32).view(np.uint32) for x in (n_, out, out_ref)] + \
                      [img.download((nbytes,), np.uint8)]
    finally:
        lut_state(L, 1)
    for g, d in zip(res[0], res[1]):
        assert np.array_equal(g, d)
