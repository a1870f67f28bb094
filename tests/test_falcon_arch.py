"""The reference's Falcon frontend (arch/falcon/falcon.cpp: GGJT v1 loader + eval graph, multi-query
attention, parallel attention/MLP) on a deterministic small Falcon file (tests/falcon_model.py).

CPU (this container): the writer reproduces the committed model hash, and the reference's CPU-only
build (oracle/_ref/libfalcon_ref_cpu.so) reproduces the golden logits bit for bit at 1 and 4
threads — pinning the fixture.  GPU (tests/test_gpu_falcon_arch.py): the same frontend built with
ggml.c's GPU hooks sends its Q4_0 mul_mats, prompt and decode, to the MI355X backend."""
import json
import os
import sys

import numpy as np
import pytest

import falcon_model as F
from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")
CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "libfalcon_ref_cpu.so")


def test_falcon_writer_reproduces_fixture_model(tmp_path):
    man = json.load(open(os.path.join(GOLD, "falcon_small_manifest.json")))
    assert F.write(str(tmp_path / "f.ggjt")) == man["model_sha256"]
    assert man["prompt"] == F.PROMPT and man["decode"] == F.DECODE and man["qkv_dim"] == F.qkv_dim() == 640


def test_falcon_golden_logits_are_informative():
    gold = np.load(os.path.join(GOLD, "falcon_small_logits.npy"))
    dgold = np.load(os.path.join(GOLD, "falcon_small_decode_logits.npy"))
    assert gold.shape == (F.HP["n_vocab"],) and dgold.shape == (len(F.DECODE), F.HP["n_vocab"])
    assert np.isfinite(gold).all() and np.isfinite(dgold).all()
    assert gold.std() > 0.1 and dgold.std(1).min() > 0.1          # not a degenerate (constant) output
    assert len(set(int(r.argmax()) for r in np.vstack([gold[None], dgold]))) >= 2


@pytest.mark.skipif(not os.path.exists(CPU_LIB), reason="oracle/_ref/libfalcon_ref_cpu.so not built")
@pytest.mark.parametrize("threads", [1, 4])
def test_reference_falcon_cpu_reproduces_golden_logits(tmp_path, threads):
    sys.path.insert(0, GOLD)
    from gen_falcon_golden import ref_logits
    mp = str(tmp_path / "f.ggjt")
    F.write(mp)
    got, dec = ref_logits(CPU_LIB, mp, n_threads=threads)
    assert np.array_equal(got.view(np.uint32), np.load(os.path.join(GOLD, "falcon_small_logits.npy")).view(np.uint32))
    assert np.array_equal(dec.view(np.uint32),
                          np.load(os.path.join(GOLD, "falcon_small_decode_logits.npy")).view(np.uint32))
