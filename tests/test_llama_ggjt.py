"""The reference's own llama.cpp (GGJT v3 loader + eval graph) on a deterministic tiny LLaMA file.

CPU (this container): the writer reproduces the committed model hash, and the reference's CPU-only
build (oracle/_ref/libllama_ref_cpu.so) reproduces the golden logits bit for bit — pinning the
fixture.  GPU (tests/test_gpu_llama_ggjt.py): the same llama.cpp built with its GPU hooks runs
every Q4_0 mul_mat of the 40-token prompt on the MI355X backend."""
import json
import os

import numpy as np
import pytest

import ggjt_model as G
from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")
CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_cpu.so")


def test_writer_reproduces_fixture_model(tmp_path):
    man = json.load(open(os.path.join(GOLD, "llama_tiny_manifest.json")))
    assert G.write(str(tmp_path / "m.ggjt")) == man["model_sha256"]
    assert man["prompt"] == G.PROMPT and man["n_ff"] == G.n_ff() == 768


@pytest.mark.skipif(not os.path.exists(CPU_LIB), reason="oracle/_ref/libllama_ref_cpu.so not built")
def test_reference_llama_cpu_reproduces_golden_logits(tmp_path):
    import sys
    sys.path.insert(0, GOLD)
    from gen_llama_golden import ref_logits
    mp = str(tmp_path / "m.ggjt")
    G.write(mp)
    got, dec = ref_logits(CPU_LIB, mp, with_decode=True)
    gold = np.load(os.path.join(GOLD, "llama_tiny_logits.npy"))
    assert np.array_equal(got.view(np.uint32), gold.view(np.uint32))
    dgold = np.load(os.path.join(GOLD, "llama_tiny_decode_logits.npy"))
    assert np.array_equal(dec.view(np.uint32), dgold.view(np.uint32))


HIP_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_hip.so")


@pytest.mark.skipif(not os.path.exists(HIP_LIB), reason="oracle/_ref/libllama_ref_hip.so not built")
def test_reference_llama_gpu_build_without_device_declines_to_cpu(tmp_path):
    """The -DGGML_USE_CUBLAS build linked against libggml_hip_cuda.so, on a host with no HIP device:
    the loader and context run through every hook (host_malloc, set_scratch_size, set_tensor_split,
    ...), can_mul_mat declines every node, and ggml's CPU ops reproduce the golden logits bitwise."""
    from hip_env import ggml_hip
    if ggml_hip.load().ggml_hip_device_count() > 0:
        pytest.skip("a HIP device is present (tests/test_gpu_llama_ggjt.py covers it)")
    import sys
    sys.path.insert(0, GOLD)
    from gen_llama_golden import ref_logits
    mp = str(tmp_path / "m.ggjt")
    G.write(mp)
    got, dec = ref_logits(HIP_LIB, mp, n_evals=2, with_decode=True)
    gold = np.load(os.path.join(GOLD, "llama_tiny_logits.npy"))
    assert np.array_equal(got.view(np.uint32), gold.view(np.uint32))
    dgold = np.load(os.path.join(GOLD, "llama_tiny_decode_logits.npy"))
    assert np.array_equal(dec.view(np.uint32), dgold.view(np.uint32))
