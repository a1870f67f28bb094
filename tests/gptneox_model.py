"""Deterministic small GPT-NeoX model in the reference GPT-NeoX frontend's GGJT v1 file format (test
fixture writer).

Layout as arch/gptneox/gptneox.cpp of Fcucgvhhhvjv/llama.cpp-q_4_0 parses it: u32 magic 'ggjt'
(0x67676a74), u32 version 1 (gptneox.cpp:440-458); hparams n_vocab, n_ctx, n_embd, n_head, n_layer,
n_rot, use_parallel_residual, ftype (u32 each, :460-467); vocab: per token u32 length, bytes, f32 score
(:469-484); then per tensor u32 n_dims, u32 name length, u32 ggml type, u32 ne[n_dims], name, zero
padding to a 32-byte file offset, data (:487-520).  Tensor names and shapes as gptneox_model_load_internal
requests them (:1000-1026): fused QKV {n_embd, 3 n_embd} + bias, attention output {n_embd, n_embd} +
bias, MLP {n_embd, 4 n_embd} / {4 n_embd, n_embd} + biases, two layer norms per layer, parallel
residual.  n_layer must be 16 (with n_embd < 6144 the frontend picks its 3B row of the scratch/KV size
tables, :910-921; other layer counts have no row and the loader throws).  Q4_0 tensors are quantized
with the oracle's restatement of quantize_row_q4_0_reference (bit-exact to ggml_quantize_q4_0,
tests/test_oracle.py)."""
import hashlib
import struct

import numpy as np

import oracle as O

GGML_TYPE_F32, GGML_TYPE_Q4_0 = 0, 2
HP = dict(n_vocab=512, n_ctx=2048, n_embd=512, n_head=8, n_layer=16, n_rot=16, use_parallel_residual=1, ftype=2)


def tensors(hp=HP, seed=0x5EED6000):
    """[(name, ggml_type, ne (ggml order), bytes)], deterministic in seed."""
    E, V = hp["n_embd"], hp["n_vocab"]
    k = [0]

    def q4(ne, std):
        k[0] += 1
        K, M = ne
        w = O.gaussian(M * K, seed + k[0], 0.0, std).reshape(M, K)
        return (GGML_TYPE_Q4_0, ne, O.quantize_q4_0(w)[0].tobytes())

    def f32(ne, mean, std):
        k[0] += 1
        v = O.gaussian(int(np.prod(ne)), seed + k[0], mean, std).astype(np.float32)
        return (GGML_TYPE_F32, ne, v.tobytes())

    out = [("gpt_neox.embed_in.weight",) + q4((E, V), 1.0),
           ("gpt_neox.final_layer_norm.weight",) + f32((E,), 1.0, 0.05),
           ("gpt_neox.final_layer_norm.bias",) + f32((E,), 0.0, 0.05),
           ("embed_out.weight",) + q4((E, V), 0.05)]
    for i in range(hp["n_layer"]):
        p = f"gpt_neox.layers.{i}."
        out.append((p + "input_layernorm.weight",) + f32((E,), 1.0, 0.05))
        out.append((p + "input_layernorm.bias",) + f32((E,), 0.0, 0.05))
        out.append((p + "attention.query_key_value.weight",) + q4((E, 3 * E), 0.04))
        out.append((p + "attention.query_key_value.bias",) + f32((3 * E,), 0.0, 0.02))
        out.append((p + "attention.dense.weight",) + q4((E, E), 0.04))
        out.append((p + "attention.dense.bias",) + f32((E,), 0.0, 0.02))
        out.append((p + "post_attention_layernorm.weight",) + f32((E,), 1.0, 0.05))
        out.append((p + "post_attention_layernorm.bias",) + f32((E,), 0.0, 0.05))
        out.append((p + "mlp.dense_h_to_4h.weight",) + q4((E, 4 * E), 0.04))
        out.append((p + "mlp.dense_h_to_4h.bias",) + f32((4 * E,), 0.0, 0.02))
        out.append((p + "mlp.dense_4h_to_h.weight",) + q4((4 * E, E), 0.02))
        out.append((p + "mlp.dense_4h_to_h.bias",) + f32((E,), 0.0, 0.02))
    return out


def write(path, hp=HP, seed=0x5EED6000):
    """Write the model; returns the file's sha256."""
    h = hashlib.sha256()
    with open(path, "wb") as f:
        def put(b):
            f.write(b)
            h.update(b)
        put(struct.pack("<II", 0x67676A74, 1))
        put(struct.pack("<8I", hp["n_vocab"], hp["n_ctx"], hp["n_embd"], hp["n_head"], hp["n_layer"], hp["n_rot"],
                        hp["use_parallel_residual"], hp["ftype"]))
        for i in range(hp["n_vocab"]):
            tok = f"<n{i}>".encode()
            put(struct.pack("<I", len(tok)) + tok + struct.pack("<f", -float(i)))
        for name, typ, ne, data in tensors(hp, seed):
            nb = name.encode()
            put(struct.pack("<III", len(ne), len(nb), typ) + struct.pack(f"<{len(ne)}I", *ne) + nb)
            put(b"\0" * (-f.tell() & 31))
            put(data)
    return h.hexdigest()


PROMPT = [int(t) for t in (np.arange(12) * 71 + 3) % HP["n_vocab"]]   # 12 tokens at n_past = 0
DECODE = [29, 310, 471]                                                # then n_past = 12, 13, 14
