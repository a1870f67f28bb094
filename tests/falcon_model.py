"""Deterministic small Falcon model in the reference Falcon frontend's GGJT v1 file format (test
fixture writer).

Layout as arch/falcon/falcon.cpp of Fcucgvhhhvjv/llama.cpp-q_4_0 parses it: u32 magic 'ggjt'
(0x67676a74), u32 version 1 (falcon.cpp:437-454); hparams n_vocab, n_embd, n_head, n_layer,
parallel_attn, ftype (u32 each, :456-465); vocab: per token u32 length, bytes, f32 score (:466-484);
then per tensor u32 n_dims, u32 name length, u32 ggml type, u32 ne[n_dims], name, zero padding to a
32-byte file offset, data (:485-535).  Tensor names and shapes as falcon_model_load_internal requests
them (:1001-1026): multi-query QKV {n_embd, n_embd + 2 head_dim}, MLP {n_embd, 4 n_embd} and
{4 n_embd, n_embd}, parallel attention (parallel_attn = 1, the 7B layout; the post-attention norm is
not loaded by this frontend).  n_layer must be 32: the frontend sizes its scratch buffers from a
table keyed by model type (3B / 7B by n_embd, :906-918), and n_embd < 4544 selects the 3B row.
Q4_0 tensors are quantized with the oracle's restatement of quantize_row_q4_0_reference (bit-exact
to ggml_quantize_q4_0, tests/test_oracle.py)."""
import hashlib
import struct

import numpy as np

import oracle as O

GGML_TYPE_F32, GGML_TYPE_Q4_0 = 0, 2
HP = dict(n_vocab=512, n_embd=512, n_head=8, n_layer=32, parallel_attn=1, ftype=2)


def qkv_dim(hp=HP):
    return hp["n_embd"] + 2 * (hp["n_embd"] // hp["n_head"])    # falcon.cpp:995-997


def tensors(hp=HP, seed=0x5EEDF000):
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

    out = [("transformer.word_embeddings.weight",) + q4((E, V), 1.0),
           ("transformer.ln_f.weight",) + f32((E,), 1.0, 0.05),
           ("transformer.ln_f.bias",) + f32((E,), 0.0, 0.05),
           ("lm_head.weight",) + q4((E, V), 0.05)]
    for i in range(hp["n_layer"]):
        p = f"transformer.h.{i}."
        out.append((p + "input_layernorm.weight",) + f32((E,), 1.0, 0.05))
        out.append((p + "input_layernorm.bias",) + f32((E,), 0.0, 0.05))
        out.append((p + "self_attention.query_key_value.weight",) + q4((E, qkv_dim(hp)), 0.04))
        out.append((p + "self_attention.dense.weight",) + q4((E, E), 0.04))
        out.append((p + "mlp.dense_h_to_4h.weight",) + q4((E, 4 * E), 0.04))
        out.append((p + "mlp.dense_4h_to_h.weight",) + q4((4 * E, E), 0.02))
    return out


def write(path, hp=HP, seed=0x5EEDF000):
    """Write the model; returns the file's sha256."""
    h = hashlib.sha256()
    with open(path, "wb") as f:
        def put(b):
            f.write(b)
            h.update(b)
        put(struct.pack("<II", 0x67676A74, 1))
        put(struct.pack("<6I", hp["n_vocab"], hp["n_embd"], hp["n_head"], hp["n_layer"], hp["parallel_attn"],
                        hp["ftype"]))
        for i in range(hp["n_vocab"]):
            tok = f"<f{i}>".encode()
            put(struct.pack("<I", len(tok)) + tok + struct.pack("<f", -float(i)))
        for name, typ, ne, data in tensors(hp, seed):
            nb = name.encode()
            put(struct.pack("<III", len(ne), len(nb), typ) + struct.pack(f"<{len(ne)}I", *ne) + nb)
            put(b"\0" * (-f.tell() & 31))
            put(data)
    return h.hexdigest()


PROMPT = [int(t) for t in (np.arange(12) * 53 + 5) % HP["n_vocab"]]   # 12 tokens at n_past = 0
DECODE = [17, 300, 444]                                                # then n_past = 12, 13, 14
