"""The reference's unmodified llama.cpp (built with -DGGML_USE_CUBLAS, linked against
libggml_hip_cuda.so) loads the tiny GGJT v3 LLaMA file with its own loader and evaluates a
40-token prompt and three decode steps.  At n_gpu_layers 0 ggml.c's can_mul_mat sends every Q4_0
mul_mat of the batch (2 layers x 7 + the output projection, N = 40) to the MI355X backend through
the weight-residency cache and everything else stays on ggml's CPU ops; with more offloaded layers
the loader uploads their weights and norms and the graph's nodes run on the device (SURVEY §8f
row 4: rms_norm, mul, add, silu, rope, scale, diag_mask_inf, soft_max, cpy into the KV cache, the
f16 attention mul_mats), up to the whole layer stack with a device KV cache.  In exact mode the
logits are bit-identical to the reference's CPU-only golden logits at every offload level; the
fast kernels stay within the propagated north-star tolerance."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

import ggjt_model as G
from conftest import ROOT
from hip_env import ggml_hip, gpu_available

GOLD = os.path.join(ROOT, "tests", "golden")
HIP_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_hip.so")

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not gpu_available(), reason="needs a HIP device and libggml_hip.so"),
              pytest.mark.skipif(not os.path.exists(HIP_LIB), reason="oracle/_ref/libllama_ref_hip.so not built")]


OPS = json.load(open(os.path.join(GOLD, "ggml_op_enum.json")))


N_FUSED = 15  # ggml-hip.h, ggml_hip_debug_op_stats: fused launches per chain in the last slots


def op_stats(L, reset=True, fused=False):
    L.ggml_hip_debug_op_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    n = OPS["GGML_OP_COUNT"]
    c = np.zeros(2 * n + 1 + N_FUSED, np.int64)
    ggml_hip.check(L.ggml_hip_debug_op_stats(c.ctypes.data, c.size, 1 if reset else 0), "op stats")
    return (c[:n], c[2 * n + 1:]) if fused else c[:n]


def run_llama(tmp_path, exact, ngl, stats=None):
    sys.path.insert(0, GOLD)
    from gen_llama_golden import ref_logits
    L = ggml_hip.load()
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(1 if exact else 0), "set_exact")
    ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
    mp = str(tmp_path / "m.ggjt")
    assert G.write(mp) == json.load(open(os.path.join(GOLD, "llama_tiny_manifest.json")))["model_sha256"]
    op_stats(L)
    try:
        got, dec = ref_logits(HIP_LIB, mp, n_evals=2, n_gpu_layers=ngl, with_decode=True)
        h, m, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        ggml_hip.check(L.ggml_hip_weight_cache_stats(ctypes.byref(h), ctypes.byref(m), ctypes.byref(r)))
        if stats is not None:
            stats.append(op_stats(L))
    finally:
        ggml_hip.check(L.ggml_hip_weight_cache_clear(), "cache clear")
        L.ggml_hip_set_exact(prev)
    # Q4_0 mul_mats whose weights stayed CPU tensors (llama.cpp:1053-1070: the last ngl layers, and
    # the output matrix from ngl > n_layer, are offloaded through transform_tensor); those go through
    # the residency cache on the two prompt evals (N = 40 >= 32); decode steps (N = 1) run them on the
    # CPU (can_mul_mat), offloaded ones on the backend
    nl = G.HP["n_layer"]
    cpu_q4 = 7 * max(0, nl - ngl) + (1 if ngl <= nl else 0)
    assert (m.value, h.value) == (cpu_q4, cpu_q4)
    return (got, dec), (np.load(os.path.join(GOLD, "llama_tiny_logits.npy")),
                        np.load(os.path.join(GOLD, "llama_tiny_decode_logits.npy")))


# n_gpu_layers (llama.cpp:1029-1076, 1117-1147, 1294-1313; n_layer = 2): 0 (weights in the cache),
# 1 (one layer's weights and norms on the device, its activations in the VRAM scratch), 2 (all
# layers), 3 (+ the final norm and the row-split output matrix), 4 (+ the V cache and the attention
# ops that read it), 5 = 99 (+ the K cache: the whole graph but get_rows and the last mul on the device)
@pytest.mark.parametrize("ngl", [0, 1, 2, 3, 4, 99])
def test_reference_llama_on_backend_exact_mode_bitwise(tmp_path, ngl):
    stats = []
    (got, dec), (gold, dgold) = run_llama(tmp_path, exact=True, ngl=ngl, stats=stats)
    assert np.array_equal(got.view(np.uint32), gold.view(np.uint32))
    assert np.array_equal(dec.view(np.uint32), dgold.view(np.uint32))
    ran = stats[0]
    nl = G.HP["n_layer"]
    if ngl >= 1:     # an offloaded layer's norms, residual adds and FFN ops ran on the device
        for op in ("GGML_OP_RMS_NORM", "GGML_OP_MUL", "GGML_OP_ADD", "GGML_OP_SILU"):
            assert ran[OPS[op]] > 0, op
    if ngl > nl + 2:  # full offload: the attention ops on the device KV cache too
        for op in ("GGML_OP_ROPE", "GGML_OP_SCALE", "GGML_OP_DIAG_MASK_INF", "GGML_OP_SOFT_MAX", "GGML_OP_CPY"):
            assert ran[OPS[op]] > 0, op


@pytest.mark.parametrize("ngl", [0, 99])
def test_reference_llama_on_backend_fast_kernels(tmp_path, ngl):
    (got, dec), (gold, dgold) = run_llama(tmp_path, exact=False, ngl=ngl)
    assert np.isfinite(got).all() and np.isfinite(dec).all()
    scale = np.abs(gold).max()
    row = np.abs(got - gold).max(1) / scale
    assert (row < 1e-5).mean() >= 0.75, row
    assert row.max() < 2e-2, row
    assert (got.argmax(1) == gold.argmax(1)).mean() >= 0.95
    assert np.abs(dec - dgold).max() / scale < 2e-2


CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_cpu.so")


HP128 = dict(n_vocab=1000, n_embd=512, n_mult=256, n_head=4, n_layer=2, n_rot=128, ftype=2)   # head_dim 128


@pytest.mark.skipif(not os.path.exists(CPU_LIB), reason="oracle/_ref/libllama_ref_cpu.so not built")
@pytest.mark.parametrize("fuse", [1, 0], ids=["fused", "unfused"])
@pytest.mark.parametrize("hp,n_prompt,n_decode", [(G.HP, 8, 600), (HP128, 40, 300), (HP128, 300, 20)],
                         ids=["head64", "head128", "head128_prompt300"])
def test_long_decode_full_offload_exact_bitwise(tmp_path, hp, n_prompt, n_decode, fuse):
    """Hundreds of single-token steps at full offload (KV cache, rope positions and soft_max rows up
    to 608, the rope table regrown past its first 512 positions; LLaMA's head_dim 128 and a
    40-token batched prompt in the second case; a 300-token prompt, whose attention runs through the
    LDS-tiled f16 mul_mat over several K stages with a tail, in the third): the last logits equal the reference's CPU-only
    build bit for bit (both run live on this host through refllama_bench)."""
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]

    def run(lib_path, ngl):
        lib = ctypes.CDLL(lib_path)
        lib.refllama_bench.restype = ctypes.c_int
        lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
        out = np.zeros(3, np.float64)
        lg = np.zeros(nv, np.float32)
        assert lib.refllama_bench(mp.encode(), n_prompt, n_decode, 1, ngl, 1024, 1, out.ctypes.data,
                                  lg.ctypes.data) == nv
        return lg

    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(1), "set_exact")
    L.ggml_hip_debug_set_fuse.argtypes = [ctypes.c_int]
    ggml_hip.check(L.ggml_hip_debug_set_fuse(fuse), "set_fuse")
    op_stats(L)
    try:
        got = run(HIP_LIB, 99)
        ran, fused = op_stats(L, fused=True)
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_fuse(1)
    ref = run(CPU_LIB, 0)
    assert np.isfinite(ref).all()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert ran[OPS["GGML_OP_SOFT_MAX"]] >= n_decode * hp["n_layer"]
    # every chain of a LLaMA layer fused once per layer and eval when fusion is on, never when off:
    # add/rms_norm/mul, scale/mask/soft_max, silu/mul, rope/cpy (K cache), KQV/merge; the decode
    # q4_0 siblings as groups (wq|wk|wv and w1|w3: two per layer and decode eval; slot 5, w3 run
    # under a pending silu, is what the prompt eval's unfused-group path leaves)
    evals = n_decode + 1
    if fuse:
        assert (fused[[0, 2]] >= evals * hp["n_layer"]).all(), fused
        # scale/mask/soft_max and the KQV merge: alone (prompt) or as the decode softmax+KQV launch
        assert fused[1] + fused[8] >= evals * hp["n_layer"] and fused[4] + fused[8] >= evals * hp["n_layer"], fused
        assert fused[8] >= n_decode * hp["n_layer"], fused
        assert fused[3] + fused[7] >= evals * hp["n_layer"], fused   # rope->cpy alone or in a batch
        assert fused[6] >= 2 * n_decode * hp["n_layer"], fused
        assert fused[7] >= n_decode * hp["n_layer"], fused      # rope K->cache, V->cache, rope Q
        # KQ inside the soft_max -> KQV launch while the row has <= 192 keys (GGML_HIP_KQ_FOLD_MAX), own launch after
        short = sum(1 for i in range(n_decode) if n_prompt + i + 1 <= 192)
        assert fused[14] >= short * hp["n_layer"], fused
    else:
        assert (fused == 0).all(), fused


@pytest.mark.parametrize("hp,n_prompt,n_decode", [(HP128, 40, 60), (G.HP, 8, 40)], ids=["head128", "head64"])
def test_fast_mode_fusion_bitwise_vs_unfused(tmp_path, hp, n_prompt, n_decode):
    """Fast kernels at full offload: every launch fusion (the chains, the sibling GEMV groups, the
    rope/cpy batch, soft_max+KQV) gives the same logits bit for bit as one launch per node."""
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_fuse.argtypes = [ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(0), "set_exact")
    out = {}
    try:
        for fuse in (1, 0):
            ggml_hip.check(L.ggml_hip_debug_set_fuse(fuse), "set_fuse")
            op_stats(L)
            lg = np.zeros(nv, np.float32)
            res = np.zeros(3, np.float64)
            assert lib.refllama_bench(mp.encode(), n_prompt, n_decode, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
            out[fuse] = (lg, op_stats(L, fused=True)[1])
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_fuse(1)
    assert np.isfinite(out[1][0]).all()
    assert np.array_equal(out[1][0].view(np.uint32), out[0][0].view(np.uint32))
    fused = out[1][1]
    assert fused[6] >= 2 * n_decode * hp["n_layer"] and fused[8] >= n_decode * hp["n_layer"], fused
    # slot 9: the decode norm chains (attention and ffn norm; layer 0's attention norm reads the host
    # embedding row, so it is no device chain) run in the q4_0 GEMVs' x prologue
    assert fused[9] >= (2 * hp["n_layer"] - 1) * n_decode, fused
    assert (out[0][1] == 0).all()


@pytest.mark.parametrize("hp,n_prompt,n_decode", [(HP128, 40, 60), (G.HP, 8, 40)], ids=["head128", "head64"])
def test_norm_fold_bitwise_vs_own_launch(tmp_path, hp, n_prompt, n_decode):
    """The decode [add ->] rms_norm -> mul and silu -> mul chains folded into the x prologue of the
    q4_0 GEMVs that consume them (ghip::gemv_q4_0_multi_norm): the same logits bit for bit as the
    chains' own launches followed by the GEMVs, and the folds fire for every device chain of a decode
    eval (q|k|v and w1|w3 behind the norms, w2 behind silu -> mul)."""
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_norm_fold.argtypes = [ctypes.c_int]
    L.ggml_hip_debug_set_epi_fold.argtypes = [ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(0), "set_exact")
    # the GEMV epilogues off: w1|w3 would take silu -> mul before the w2 prologue sees it
    ggml_hip.check(L.ggml_hip_debug_set_epi_fold(0), "set_epi_fold")
    out = {}
    try:
        for fold in (1, 0):
            ggml_hip.check(L.ggml_hip_debug_set_norm_fold(fold), "set_norm_fold")
            op_stats(L)
            lg = np.zeros(nv, np.float32)
            res = np.zeros(3, np.float64)
            assert lib.refllama_bench(mp.encode(), n_prompt, n_decode, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
            out[fold] = (lg, op_stats(L, fused=True)[1])
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_norm_fold(1)
        L.ggml_hip_debug_set_epi_fold(1)
    assert np.isfinite(out[1][0]).all()
    assert np.array_equal(out[1][0].view(np.uint32), out[0][0].view(np.uint32))
    assert out[1][1][9] >= (2 * hp["n_layer"] - 1) * n_decode, out[1][1]
    assert out[1][1][10] >= hp["n_layer"] * n_decode, out[1][1]      # silu -> mul in the w2 prologue
    assert out[0][1][9] == 0 and out[0][1][10] == 0, out[0][1]
    for k in (0, 2):                                                 # every chain still counted once
        assert out[1][1][k] == out[0][1][k], (out[1][1], out[0][1])


@pytest.mark.parametrize("hp,n_prompt,n_decode", [(HP128, 40, 60), (G.HP, 8, 40)], ids=["head128", "head64"])
def test_gemv_epilogue_bitwise_vs_elem_batch(tmp_path, hp, n_prompt, n_decode):
    """The decode GEMVs finish the nodes ggml holds behind them in their epilogue (ghip::GemvEpi): q|k|v
    the rope K -> the F16 K cache, V -> the transposed V cache, rope Q; w1|w3 (as interleaved gate / up
    rows) silu -> mul.  The same logits bit for bit as the batched elementwise launch after the GEMV
    (k_elem_batch) and silu -> mul in the w2 GEMV's prologue, and the epilogues fire for every device
    group of a decode eval (layer 0's q|k|v reads the host embedding row: no device norm chain, no group
    with a prologue, so its nodes stay in the batch)."""
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_epi_fold.argtypes = [ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(0), "set_exact")
    out = {}
    try:
        for epi in (1, 0):
            ggml_hip.check(L.ggml_hip_debug_set_epi_fold(epi), "set_epi_fold")
            op_stats(L)
            lg = np.zeros(nv, np.float32)
            res = np.zeros(3, np.float64)
            assert lib.refllama_bench(mp.encode(), n_prompt, n_decode, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
            out[epi] = (lg, op_stats(L, reset=False, fused=True))
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_epi_fold(1)
    assert np.isfinite(out[1][0]).all()
    assert np.array_equal(out[1][0].view(np.uint32), out[0][0].view(np.uint32))
    (ran1, f1), (ran0, f0) = out[1][1], out[0][1]
    assert f1[12] >= (hp["n_layer"] - 1) * n_decode, f1
    assert f1[13] >= hp["n_layer"] * n_decode, f1
    assert f0[12] == 0 and f0[13] == 0, f0
    assert f0[7] - f1[7] >= (hp["n_layer"] - 1) * n_decode, (f1, f0)   # the batches it replaced
    assert np.array_equal(ran1, ran0)                                  # every node still counted once


@pytest.mark.parametrize("exact", [0, 1], ids=["fast", "exact"])
@pytest.mark.parametrize("hp,n_prompt,n_decode", [(HP128, 40, 60), (G.HP, 8, 40)], ids=["head128", "head64"])
def test_kq_fold_bitwise_vs_own_launch(tmp_path, hp, n_prompt, n_decode, exact):
    """The decode KQ (f16 K cache view . fp16(q), one query row per head) computed by the scale ->
    diag_mask_inf -> soft_max -> KQV -> merge launch (op_kq_softmax_kqv, the head's KQ row in LDS): the
    same logits bit for bit as KQ's own launch (k_mul_mat_f16_f32) before the chain, in both modes, and
    the fold fires for every layer of every decode eval."""
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_kq_fold.argtypes = [ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(exact), "set_exact")
    out = {}
    try:
        for fold in (1, 0):
            ggml_hip.check(L.ggml_hip_debug_set_kq_fold(fold), "set_kq_fold")
            op_stats(L)
            lg = np.zeros(nv, np.float32)
            res = np.zeros(3, np.float64)
            assert lib.refllama_bench(mp.encode(), n_prompt, n_decode, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
            out[fold] = (lg, op_stats(L, reset=False, fused=True))
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_kq_fold(1)
    assert np.isfinite(out[1][0]).all()
    assert np.array_equal(out[1][0].view(np.uint32), out[0][0].view(np.uint32))
    (ran1, f1), (ran0, f0) = out[1][1], out[0][1]
    assert f1[14] >= hp["n_layer"] * n_decode and f0[14] == 0, (f1, f0)
    assert np.array_equal(ran1, ran0)


@pytest.mark.parametrize("n_prompt", [300, 97])
def test_prefill_x_image_fold_bitwise_vs_prep(tmp_path, n_prompt):
    """Prefill (N > 64 tokens) at full offload: the [add ->] rms_norm -> mul and silu -> mul chains whose
    q4_0 consumers all take k_gemm9 on fp6 weight images write the x image in their own launch (no
    k_prep9_x): the same logits bit for bit as the chains' own launches followed by the mul_mats' x prep,
    and the fold fires for every device chain of the prompt eval (q|k|v and w1|w3 behind the norms, w2
    behind silu -> mul; layer 0's attention norm reads the host embedding rows, so it is no device chain)."""
    hp = HP128
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_x9_fold.argtypes = [ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(0), "set_exact")
    out = {}
    try:
        for fold in (1, 0):
            ggml_hip.check(L.ggml_hip_debug_set_x9_fold(fold), "set_x9_fold")
            op_stats(L)
            lg = np.zeros(nv, np.float32)
            res = np.zeros(3, np.float64)
            assert lib.refllama_bench(mp.encode(), n_prompt, 2, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
            out[fold] = (lg, op_stats(L, fused=True)[1])
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_x9_fold(1)
    assert np.isfinite(out[1][0]).all()
    assert np.array_equal(out[1][0].view(np.uint32), out[0][0].view(np.uint32))
    assert out[1][1][11] >= 3 * hp["n_layer"] - 1, out[1][1]
    assert out[0][1][11] == 0, out[0][1]
    for k in (0, 2):                                                 # every chain still counted once
        assert out[1][1][k] == out[0][1][k], (out[1][1], out[0][1])


@pytest.mark.parametrize("mode", [1, 2], ids=["graphs", "thread"])
@pytest.mark.parametrize("exact", [0, 1], ids=["fast", "exact"])
def test_launch_recorder_bitwise_vs_eager(tmp_path, exact, mode):
    """The launch recorder (csrc/launch.h): GGML_HIP_GRAPH=1 records every kernel of a full-offload
    eval and submits cached HIP graphs whose position-dependent nodes are updated in place;
    GGML_HIP_GRAPH=2 hands the launches to a launcher thread.  Prompt + 120 decode steps give the same
    logits bit for bit as one launch at a time; in graph mode the counters show replays with in-place
    updates rather than one instantiation per run."""
    hp = HP128
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_graph.argtypes = [ctypes.c_int]
    L.ggml_hip_debug_graph_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    prev = L.ggml_hip_get_exact()
    ggml_hip.check(L.ggml_hip_set_exact(exact), "set_exact")
    out, stats = {}, {}
    try:
        for graph in (mode, 0):
            ggml_hip.check(L.ggml_hip_debug_set_graph(graph), "set_graph")
            g0 = np.zeros(5, np.int64)
            L.ggml_hip_debug_graph_stats(g0.ctypes.data, 1)
            lg = np.zeros(nv, np.float32)
            res = np.zeros(3, np.float64)
            assert lib.refllama_bench(mp.encode(), 24, 120, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
            g1 = np.zeros(5, np.int64)
            L.ggml_hip_debug_graph_stats(g1.ctypes.data, 0)
            out[graph], stats[graph] = lg, g1 - g0
    finally:
        L.ggml_hip_set_exact(prev)
        L.ggml_hip_debug_set_graph(0)
    assert np.isfinite(out[mode]).all()
    assert np.array_equal(out[mode].view(np.uint32), out[0].view(np.uint32))
    assert (stats[0][:4] == 0).all(), stats[0]    # recorder off: nothing recorded
    if mode == 2:
        return
    runs, kernels, updated, built = stats[1][:4]
    assert runs >= 120 and kernels >= 120 * 5 * hp["n_layer"], stats[1]   # >= 5 launches per decode layer
    assert updated > 0, stats[1]                  # n_past-dependent nodes change every step
    assert built * 10 < runs, stats[1]            # replayed, not re-instantiated per run


@pytest.mark.parametrize("hp,n_prompt,n_decode", [(HP128, 40, 30), (G.HP, 8, 20)], ids=["head128", "head64"])
def test_aql_launch_mode_bitwise(tmp_path, hp, n_prompt, n_decode):
    """Launch mode 3 (ggml-hip-aql.cpp: the hook path's kernels into an own AQL queue, kernargs in VRAM) gives the
    same logits bit for bit as eager hipLaunchKernel, prompt and decode, fast and exact kernels; the queue took the
    launches (dispatch counter) and the fallbacks stay few."""
    L = ggml_hip.load()
    mp = str(tmp_path / "m.ggjt")
    G.write(mp, hp=hp)
    nv = hp["n_vocab"]
    lib = ctypes.CDLL(HIP_LIB)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    L.ggml_hip_debug_set_graph.argtypes = [ctypes.c_int]
    L.ggml_hip_debug_aql_stats.argtypes = [ctypes.c_void_p]
    prev = L.ggml_hip_get_exact()
    out = {}
    try:
        for exact in (0, 1):
            ggml_hip.check(L.ggml_hip_set_exact(exact), "set_exact")
            for mode in (0, 3):
                ggml_hip.check(L.ggml_hip_debug_set_graph(mode), "set_graph")
                s0 = np.zeros(4, np.int64)
                L.ggml_hip_debug_aql_stats(s0.ctypes.data)
                lg = np.zeros(nv, np.float32)
                res = np.zeros(3, np.float64)
                assert lib.refllama_bench(mp.encode(), n_prompt, n_decode, 1, 99, 1024, 1, res.ctypes.data, lg.ctypes.data) == nv
                s1 = np.zeros(4, np.int64)
                L.ggml_hip_debug_aql_stats(s1.ctypes.data)
                out[(exact, mode)] = (lg, s1 - s0)
    finally:
        L.ggml_hip_debug_set_graph(0)
        L.ggml_hip_set_exact(prev)
    for exact in (0, 1):
        a, b = out[(exact, 0)][0], out[(exact, 3)][0]
        assert np.isfinite(a).all()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), f"exact={exact}"
        disp, fb = out[(exact, 3)][1][:2]
        assert disp > n_decode * hp["n_layer"], (disp, fb)
        assert fb <= disp // 10, (disp, fb)
