"""Phase times of the fused decode attention (diagnostic library built with -DATTN_STAMPS):
  FILE=ggml_ops bash tools/build_variant.sh astamps -DATTN_STAMPS
  GGML_HIP_LIB=variants/libggml_hip_astamps.so python tools/attn_stamps.py
Per workgroup (thread 0): start, KQ row in LDS, softmax done, end (s_memrealtime, 100 MHz), relative to the
first workgroup's start; medians over workgroups and 20 calls."""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "llama.cpp-q_4_0_amd", "python"), os.path.join(HERE, "..", "tests")]
import ggml_hip  # noqa: E402
from test_gpu_attn_decode import attn, caches  # noqa: E402

L = ggml_hip.load()
L.ggml_hip_debug_attn_stamps.argtypes = [ctypes.c_void_p]
kc, q, vc = caches(128, 32, 2048, 1)
st = ggml_hip.DeviceBuffer(4096 * 8 * 8)
ggml_hip.check(L.ggml_hip_debug_attn_stamps(st.ptr))
for nkv in (40, 72, 136, 512):
    rows = []
    for rep in range(22):
        st.upload(np.zeros(4096 * 8, np.uint64))
        attn(L, 1, kc, q, vc, 128, 32, 2048, nkv, reps=3)    # stamps of the last of 4 back-to-back calls
        a = st.download((4096, 8), np.uint64)
        a = a[a[:, 0] != 0][:, :4].astype(np.int64)
        if rep < 2:
            continue
        t0 = a[:, 0].min()
        r = (a - t0) / 100.0
        rows.append([np.median(r[:, 0]), r[:, 0].max(), np.median(r[:, 1] - r[:, 0]), np.median(r[:, 2] - r[:, 1]),
                     np.median(r[:, 3] - r[:, 2]), r[:, 3].max()])
    m = np.mean(rows, 0)
    print(f"n_kv {nkv:4d} ({len(a)} WGs): start p50 {m[0]:.2f} max {m[1]:.2f} | KQ {m[2]:.2f} | softmax {m[3]:.2f} | "
          f"KQV {m[4]:.2f} | end max {m[5]:.2f} us", flush=True)
L.ggml_hip_debug_attn_stamps(None)
