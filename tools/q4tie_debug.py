import sys, numpy as np
sys.path[:0] = ["tests", "oracle"]
from hip_env import ggml_hip
from golden_io import load
w = load("avx2", "q4tie_w_f32").reshape(1, 128)
wd = ggml_hip.DeviceBuffer.from_array(w); qd = ggml_hip.DeviceBuffer(72)
ggml_hip.quantize_q4_0(wd, 128, 1, qd)
got = qd.download((4, 18), np.uint8); ref = load("avx2", "q4tie_q4_0")
print("got\n", got, "\nref\n", ref, "\ndiff at", np.argwhere(got != ref).tolist())
