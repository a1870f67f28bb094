"""The reference's GPT-NeoX frontend (arch/gptneox/gptneox.cpp: GGJT v1 loader + eval graph, fused QKV
with biases, NeoX rope on n_rot dims, parallel residual) on a deterministic small GPT-NeoX file
(tests/gptneox_model.py).

CPU (this container): the writer reproduces the committed model hash, and the reference's CPU-only
build (oracle/_ref/libgptneox_ref_cpu.so) reproduces the golden logits bit for bit at 1 and 4 threads —
pinning the fixture.  GPU (tests/test_gpu_gptneox_arch.py): the same frontend built with ggml.c's GPU
hooks sends its Q4_0 mul_mats, prompt and decode, to the MI355X backend."""
import json
import os
import sys

import numpy as np
import pytest

import gptneox_model as G
from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")
CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "libgptneox_ref_cpu.so")


def test_gptneox_writer_reproduces_fixture_model(tmp_path):
    man = json.load(open(os.path.join(GOLD, "gptneox_small_manifest.json")))
    assert G.write(str(tmp_path / "n.ggjt")) == man["model_sha256"]
    assert man["prompt"] == G.PROMPT and man["decode"] == G.DECODE and man["hparams"] == G.HP


def test_gptneox_golden_logits_are_informative():
    gold = np.load(os.path.join(GOLD, "gptneox_small_logits.npy"))
    dgold = np.load(os.path.join(GOLD, "gptneox_small_decode_logits.npy"))
    assert gold.shape == (G.HP["n_vocab"],) and dgold.shape == (len(G.DECODE), G.HP["n_vocab"])
    assert np.isfinite(gold).all() and np.isfinite(dgold).all()
    assert gold.std() > 0.1 and dgold.std(1).min() > 0.1
    assert len(set(int(r.argmax()) for r in np.vstack([gold[None], dgold]))) >= 2


@pytest.mark.skipif(not os.path.exists(CPU_LIB), reason="oracle/_ref/libgptneox_ref_cpu.so not built")
@pytest.mark.parametrize("threads", [1, 4])
def test_reference_gptneox_cpu_reproduces_golden_logits(tmp_path, threads):
    sys.path.insert(0, GOLD)
    from gen_gptneox_golden import ref_logits
    mp = str(tmp_path / "n.ggjt")
    G.write(mp)
    got, dec = ref_logits(CPU_LIB, mp, n_threads=threads)
    assert np.array_equal(got.view(np.uint32), np.load(os.path.join(GOLD, "gptneox_small_logits.npy")).view(np.uint32))
    assert np.array_equal(dec.view(np.uint32),
                          np.load(os.path.join(GOLD, "gptneox_small_decode_logits.npy")).view(np.uint32))
