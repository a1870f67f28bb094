"""Deterministic tiny LLaMA model in the GGJT v3 file format (test fixture writer).

Layout as the reference's reader parses it (llama.cpp:383-503 of Fcucgvhhhvjv/llama.cpp-q_4_0):
u32 magic 'ggjt' (0x67676a74), u32 version 3; hparams n_vocab, n_embd, n_mult, n_head, n_layer,
n_rot, ftype (u32 each); vocab: per token u32 length, bytes, f32 score; then per tensor u32
n_dims, u32 name length, u32 ggml type, u32 ne[n_dims], name, zero padding to a 32-byte file
offset, data (ggml layout, q4_0 blocks verbatim).  Names and shapes as llama_model_load_internal
requests them (llama.cpp:1023-1076).  Q4_0 tensors are quantized with the oracle's restatement of
quantize_row_q4_0_reference (bit-exact to ggml_quantize_q4_0, tests/test_oracle.py)."""
import hashlib
import struct

import numpy as np

import oracle as O

GGML_TYPE_F32, GGML_TYPE_Q4_0 = 0, 2
HP = dict(n_vocab=320, n_embd=256, n_mult=256, n_head=4, n_layer=2, n_rot=64, ftype=2)


def n_ff(hp=HP):
    return ((2 * (4 * hp["n_embd"]) // 3 + hp["n_mult"] - 1) // hp["n_mult"]) * hp["n_mult"]   # llama.cpp:935


def tensors(hp=HP, seed=0x5EED9000):
    """[(name, ggml_type, ne (ggml order), bytes)] of the model, deterministic in seed."""
    E, V, F = hp["n_embd"], hp["n_vocab"], n_ff(hp)
    out = []
    k = [0]

    def q4(ne, std):
        k[0] += 1
        K, M = ne
        w = O.gaussian(M * K, seed + k[0], 0.0, std).reshape(M, K)
        return (GGML_TYPE_Q4_0, ne, O.quantize_q4_0(w)[0].tobytes())

    def f32(ne, mean, std):
        k[0] += 1
        v = (O.gaussian(int(np.prod(ne)), seed + k[0], mean, std)).astype(np.float32)
        return (GGML_TYPE_F32, ne, v.tobytes())

    out.append(("tok_embeddings.weight",) + q4((E, V), 1.0))
    out.append(("norm.weight",) + f32((E,), 1.0, 0.05))
    out.append(("output.weight",) + q4((E, V), 0.05))
    for i in range(hp["n_layer"]):
        p = f"layers.{i}."
        out.append((p + "attention_norm.weight",) + f32((E,), 1.0, 0.05))
        for w in ("wq", "wk", "wv", "wo"):
            out.append((p + f"attention.{w}.weight",) + q4((E, E), 0.05))
        out.append((p + "ffn_norm.weight",) + f32((E,), 1.0, 0.05))
        out.append((p + "feed_forward.w1.weight",) + q4((E, F), 0.05))
        out.append((p + "feed_forward.w2.weight",) + q4((F, E), 0.05))
        out.append((p + "feed_forward.w3.weight",) + q4((E, F), 0.05))
    return out


def write(path, hp=HP, seed=0x5EED9000):
    """Write the model; returns the file's sha256."""
    buf = bytearray()
    buf += struct.pack("<II", 0x67676A74, 3)
    buf += struct.pack("<7I", hp["n_vocab"], hp["n_embd"], hp["n_mult"], hp["n_head"], hp["n_layer"], hp["n_rot"],
                       hp["ftype"])
    for i in range(hp["n_vocab"]):
        tok = f"<t{i}>".encode()
        buf += struct.pack("<I", len(tok)) + tok + struct.pack("<f", -float(i))
    for name, typ, ne, data in tensors(hp, seed):
        nb = name.encode()
        buf += struct.pack("<III", len(ne), len(nb), typ) + struct.pack(f"<{len(ne)}I", *ne) + nb
        buf += b"\0" * (-len(buf) & 31)
        buf += data
    with open(path, "wb") as f:
        f.write(buf)
    return hashlib.sha256(bytes(buf)).hexdigest()


# 40 tokens (N >= 32: the reference's can_mul_mat sends the batch to the backend); BOS first
# (llama_eval_internal requires it)
PROMPT = [1] + [int(t) for t in (np.arange(1, 40) * 37 + 11) % HP["n_vocab"]]
DECODE = [7, 123, 301]                      # single-token steps after the prompt (n_past = 40, 41, 42)
