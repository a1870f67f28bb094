import os, sys, tempfile
sys.path[:0] = ["tests", "oracle", "tests/golden", "llama.cpp-q_4_0_amd/python"]
import ggjt_model as G
import ggml_hip
ggml_hip.load()
from gen_llama_golden import ref_logits
d = tempfile.mkdtemp()
mp = os.path.join(d, "m.ggjt"); G.write(mp)
ref_logits("oracle/_ref/libllama_ref_hip.so", mp, n_evals=1, n_gpu_layers=99, with_decode=True)
