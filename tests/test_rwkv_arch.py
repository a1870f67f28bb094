"""The reference's RWKV-4 frontend (arch/rwkv/rwkv.cpp: GGJT v1 loader + its recurrent one-token graph,
time mixing with the max-trick state, channel mixing, ggml_map_* custom ops, softmax output) on a
deterministic small RWKV file (tests/rwkv_model.py).

CPU (this container): the writer reproduces the committed model hash, and the reference's CPU-only
build (oracle/_ref/librwkv_ref_cpu.so) reproduces the golden outputs bit for bit (its graph runs on one
thread) —
pinning the fixture.  GPU (tests/test_gpu_rwkv_arch.py): the same frontend built with ggml.c's GPU
hooks sends its Q4_0 mul_mats, prompt and decode, to the MI355X backend."""
import json
import os
import sys

import numpy as np
import pytest

import rwkv_model as G
from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")
CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "librwkv_ref_cpu.so")


def test_gptneox_writer_reproduces_fixture_model(tmp_path):
    man = json.load(open(os.path.join(GOLD, "rwkv_small_manifest.json")))
    assert G.write(str(tmp_path / "r.ggjt")) == man["model_sha256"]
    assert man["prompt"] == G.PROMPT and man["decode"] == G.DECODE and man["hparams"] == G.HP


def test_gptneox_golden_logits_are_informative():
    gold = np.load(os.path.join(GOLD, "rwkv_small_logits.npy"))
    dgold = np.load(os.path.join(GOLD, "rwkv_small_decode_logits.npy"))
    assert gold.shape == (G.HP["n_vocab"],) and dgold.shape == (len(G.DECODE), G.HP["n_vocab"])
    assert np.isfinite(gold).all() and np.isfinite(dgold).all()
    # the frontend's output is softmax probabilities (rwkv.cpp:1655): a distribution, not flat
    assert abs(float(gold.sum()) - 1.0) < 1e-3 and gold.max() > 5.0 / G.HP["n_vocab"]
    assert dgold.max(1).min() > 5.0 / G.HP["n_vocab"]
    assert len(set(int(r.argmax()) for r in np.vstack([gold[None], dgold]))) >= 2


@pytest.mark.skipif(not os.path.exists(CPU_LIB), reason="oracle/_ref/librwkv_ref_cpu.so not built")
@pytest.mark.parametrize("threads", [1, 4])
def test_reference_gptneox_cpu_reproduces_golden_logits(tmp_path, threads):
    sys.path.insert(0, GOLD)
    from gen_rwkv_golden import ref_logits
    mp = str(tmp_path / "r.ggjt")
    G.write(mp)
    got, dec = ref_logits(CPU_LIB, mp)
    assert np.array_equal(got.view(np.uint32), np.load(os.path.join(GOLD, "rwkv_small_logits.npy")).view(np.uint32))
    assert np.array_equal(dec.view(np.uint32),
                          np.load(os.path.join(GOLD, "rwkv_small_decode_logits.npy")).view(np.uint32))
