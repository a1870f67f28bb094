"""Deterministic small RWKV-4 model in the reference RWKV frontend's GGJT v1 file format (test fixture
writer).

Layout as arch/rwkv/rwkv.cpp of Fcucgvhhhvjv/llama.cpp-q_4_0 parses it: u32 magic 'ggjt' (0x67676a74),
u32 version 1 (rwkv.cpp:509-527); hparams n_vocab, n_ctx, n_embd, n_layer, rescale_every, ftype (u32
each, :529-537); vocab: per token u32 length, bytes (no score, :539-558); then per tensor u32 n_dims, u32
name length, u32 ggml type, u32 ne[n_dims], name, zero padding to a 32-byte file offset, data
(:562-600).  Tensor names and shapes as rwkv_model_load_internal requests them (:1152-1219): per block
ln1/ln2, time-mix vectors, time_first, time_decay (stored negative, as the converter's -exp(w)), the
four attention matrices {n_embd, n_embd} and the channel-mix matrices key {n_embd, 4 n_embd},
receptance {n_embd, n_embd}, value {4 n_embd, n_embd}; block 0 also carries pre_ln.  n_layer must be 12
or 24 (the frontend's 169M / 430M rows of its scratch tables, :1062-1073).  Q4_0 tensors are quantized
with the oracle's restatement of quantize_row_q4_0_reference (bit-exact to ggml_quantize_q4_0)."""
import hashlib
import struct

import numpy as np

import oracle as O

GGML_TYPE_F32, GGML_TYPE_Q4_0 = 0, 2
HP = dict(n_vocab=512, n_ctx=1024, n_embd=512, n_layer=12, rescale_every=6, ftype=2)


def tensors(hp=HP, seed=0x5EED7000):
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

    out = [("rwkv.embeddings.weight",) + q4((E, V), 1.0),
           ("rwkv.blocks.0.pre_ln.weight",) + f32((E,), 1.0, 0.05),
           ("rwkv.blocks.0.pre_ln.bias",) + f32((E,), 0.0, 0.05),
           ("rwkv.ln_out.weight",) + f32((E,), 1.0, 0.05),
           ("rwkv.ln_out.bias",) + f32((E,), 0.0, 0.05),
           ("head.weight",) + q4((E, V), 0.05)]
    for i in range(hp["n_layer"]):
        p = f"rwkv.blocks.{i}."
        out.append((p + "ln1.weight",) + f32((E,), 1.0, 0.05))
        out.append((p + "ln1.bias",) + f32((E,), 0.0, 0.05))
        out.append((p + "attention.time_mix_key",) + f32((E,), 0.5, 0.15))
        out.append((p + "attention.time_mix_value",) + f32((E,), 0.5, 0.15))
        out.append((p + "attention.time_mix_receptance",) + f32((E,), 0.5, 0.15))
        out.append((p + "attention.time_first",) + f32((E,), 0.0, 0.5))
        out.append((p + "attention.time_decay",) + f32((E,), -1.0, 0.3))
        out.append((p + "attention.key.weight",) + q4((E, E), 0.04))
        out.append((p + "attention.value.weight",) + q4((E, E), 0.04))
        out.append((p + "attention.receptance.weight",) + q4((E, E), 0.04))
        out.append((p + "attention.output.weight",) + q4((E, E), 0.04))
        out.append((p + "ln2.weight",) + f32((E,), 1.0, 0.05))
        out.append((p + "ln2.bias",) + f32((E,), 0.0, 0.05))
        out.append((p + "feed_forward.time_mix_key",) + f32((E,), 0.5, 0.15))
        out.append((p + "feed_forward.time_mix_receptance",) + f32((E,), 0.5, 0.15))
        out.append((p + "feed_forward.key.weight",) + q4((E, 4 * E), 0.04))
        out.append((p + "feed_forward.receptance.weight",) + q4((E, E), 0.04))
        out.append((p + "feed_forward.value.weight",) + q4((4 * E, E), 0.02))
    return out


def write(path, hp=HP, seed=0x5EED7000):
    """Write the model; returns the file's sha256."""
    h = hashlib.sha256()
    with open(path, "wb") as f:
        def put(b):
            f.write(b)
            h.update(b)
        put(struct.pack("<II", 0x67676A74, 1))
        put(struct.pack("<6I", hp["n_vocab"], hp["n_ctx"], hp["n_embd"], hp["n_layer"], hp["rescale_every"],
                        hp["ftype"]))
        for i in range(hp["n_vocab"]):
            tok = f"<r{i}>".encode()
            put(struct.pack("<I", len(tok)) + tok)
        for name, typ, ne, data in tensors(hp, seed):
            nb = name.encode()
            put(struct.pack("<III", len(ne), len(nb), typ) + struct.pack(f"<{len(ne)}I", *ne) + nb)
            put(b"\0" * (-f.tell() & 31))
            put(data)
    return h.hexdigest()


PROMPT = [int(t) for t in (np.arange(6) * 89 + 11) % HP["n_vocab"]]   # one token per eval (recurrent)
DECODE = [41, 290, 433]
