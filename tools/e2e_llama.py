"""End-to-end LLaMA-7B-shaped decode through the reference's own llama.cpp on the backend.

Writes a GGJT v3 q4_0 model of LLaMA-7B shape (n_vocab 32000, n_embd 4096, n_head 32, n_layer 32,
n_ff 11008; random valid q4_0 blocks, F32 norms ~ 1; no checkpoint exists offline) and evaluates it
with oracle/_ref's builds of the reference llama.cpp + ggml.c (the caller side, unmodified):
  cpu     libllama_ref_cpu.so  (ggml.c's AVX2 path, N_CPU threads)
  offload libllama_ref_hip.so  n_gpu_layers = 99: weights, norms, KV cache and every node but the
          token embedding lookup on the MI355X, fast and exact mode.
Reports load time, prompt ms, decode ms/token and tok/s; checks that exact mode's last logits are
bitwise equal to the CPU's (and the fast kernels' within tolerance).
This measures the reference's host executor around the backend (graph build + ggml_graph_compute
per token), not a kernel: the kernel numbers are bench.py's.

  python tools/e2e_llama.py [--decode 64] [--threads-cpu 16] [--out profiles/r01_e2e_llama7b.json]
"""
import argparse
import ctypes
import json
import os
import struct
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "llama.cpp-q_4_0_amd", "python")]
CPU_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_cpu.so")
HIP_LIB = os.path.join(ROOT, "oracle", "_ref", "libllama_ref_hip.so")
HP7B = dict(n_vocab=32000, n_embd=4096, n_mult=256, n_head=32, n_layer=32, n_rot=128, ftype=2)
# the same graph (32 layers, 1,187 nodes per decode eval, head dim 128) with little device work: the host
# walk of the hook path measured on its own (--shape host)
HPHOST = dict(n_vocab=32000, n_embd=512, n_mult=256, n_head=4, n_layer=32, n_rot=128, ftype=2)


def n_ff(hp):
    return ((2 * (4 * hp["n_embd"]) // 3 + hp["n_mult"] - 1) // hp["n_mult"]) * hp["n_mult"]   # llama.cpp:935


def write_model(path, hp, seed=7):
    """GGJT v3 (llama.cpp:383-503): header, vocab, then per tensor a record and 32-byte aligned data."""
    rng = np.random.default_rng(seed)
    E, V, F = hp["n_embd"], hp["n_vocab"], n_ff(hp)

    def q4(ne):
        nblk = ne[0] * ne[1] // 32
        b = np.frombuffer(rng.bytes(nblk * 18), np.uint8).reshape(nblk, 18).copy()
        d = rng.uniform(0.0015, 0.0035, nblk).astype(np.float16).view(np.uint8).reshape(nblk, 2)
        b[:, :2] = d
        return 2, ne, b

    def f32(ne):
        return 0, ne, (1.0 + 0.05 * rng.standard_normal(int(np.prod(ne)))).astype(np.float32)

    specs = [("tok_embeddings.weight", lambda: q4((E, V))), ("norm.weight", lambda: f32((E,))),
             ("output.weight", lambda: q4((E, V)))]
    for i in range(hp["n_layer"]):
        p = f"layers.{i}."
        specs.append((p + "attention_norm.weight", lambda: f32((E,))))
        for w in ("wq", "wk", "wv", "wo"):
            specs.append((p + f"attention.{w}.weight", lambda: q4((E, E))))
        specs.append((p + "ffn_norm.weight", lambda: f32((E,))))
        specs.append((p + "feed_forward.w1.weight", lambda: q4((E, F))))
        specs.append((p + "feed_forward.w2.weight", lambda: q4((F, E))))
        specs.append((p + "feed_forward.w3.weight", lambda: q4((E, F))))
    with open(path, "wb") as f:
        f.write(struct.pack("<II", 0x67676A74, 3))
        f.write(struct.pack("<7I", hp["n_vocab"], hp["n_embd"], hp["n_mult"], hp["n_head"], hp["n_layer"],
                            hp["n_rot"], hp["ftype"]))
        for i in range(hp["n_vocab"]):
            tok = f"<t{i}>".encode()
            f.write(struct.pack("<I", len(tok)) + tok + struct.pack("<f", -float(i)))
        for name, gen in specs:
            typ, ne, data = gen()
            nb = name.encode()
            f.write(struct.pack("<III", len(ne), len(nb), typ) + struct.pack(f"<{len(ne)}I", *ne) + nb)
            f.write(b"\0" * (-f.tell() & 31))
            f.write(data.tobytes())
    return os.path.getsize(path)


def bench(lib_path, model, n_prompt, n_decode, threads, ngl, reps, nv):
    lib = ctypes.CDLL(lib_path)
    lib.refllama_bench.restype = ctypes.c_int
    lib.refllama_bench.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p, ctypes.c_void_p]
    out = np.zeros(3, np.float64)
    logits = np.zeros(nv, np.float32)
    # the KV cache must hold every position (llama.cpp does not check n_past + N <= n_ctx)
    n_ctx = max(512, -(-(n_prompt + n_decode) // 512) * 512)
    rc = lib.refllama_bench(model.encode(), n_prompt, n_decode, threads, ngl, n_ctx, reps, out.ctypes.data,
                            logits.ctypes.data)
    if rc != nv:
        raise RuntimeError(f"refllama_bench({lib_path}) failed: {rc}")
    lo, hi = ctypes.c_double(), ctypes.c_double()
    lib.refllama_last_prompt_range(ctypes.byref(lo), ctypes.byref(hi))
    return {"load_s": round(out[0], 2), "prompt_tokens": n_prompt, "prompt_ms": round(out[1], 2),
            "prompt_ms_min": round(lo.value, 2), "prompt_ms_max": round(hi.value, 2),
            "decode_tokens": n_decode, "decode_ms_per_token": round(out[2], 3),
            "decode_tok_s": round(1e3 / out[2], 2) if out[2] > 0 else None, "threads": threads,
            "n_gpu_layers": ngl}, logits


OP_NAMES = {2: "add", 6: "mul", 23: "silu", 26: "rms_norm", 32: "mul_mat", 34: "scale", 36: "cpy", 38: "reshape",
            39: "view", 40: "permute", 41: "transpose", 45: "diag_mask_inf", 47: "soft_max", 49: "rope"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--decode", type=int, default=64)
    ap.add_argument("--decode-cpu", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=8)
    ap.add_argument("--threads-cpu", type=int, default=16)
    ap.add_argument("--threads-gpu", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-warm", action="store_true", help="no untimed warm-up run per mode")
    ap.add_argument("--modes", default="fast,exact")
    ap.add_argument("--out", default="")
    ap.add_argument("--shape", choices=("7b", "host"), default="7b")
    ap.add_argument("--maps", action="store_true",
                    help="record the libggml_hip files mapped into this process (one copy expected; GGML_HIP_LIB)")
    ap.add_argument("--hostprof", default="", help="sample the host walk of each mode (tools/hostprof.c) into PATH.<mode>")
    args = ap.parse_args()
    hp = HP7B if args.shape == "7b" else HPHOST
    import ggml_hip as gh
    L = gh.load()
    d = tempfile.mkdtemp(prefix="e2e7b_", dir=os.environ.get("E2E_DIR", "/tmp"))
    model = os.path.join(d, "llama7b-q4_0-synthetic.ggjt")
    t0 = time.time()
    size = write_model(model, hp)
    print(f"model {size / 1e9:.2f} GB written in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    nv = hp["n_vocab"]
    res = {"model": ("LLaMA-7B shape" if args.shape == "7b" else f"host-walk shape {hp}") + ", GGJT v3 q4_0, random valid blocks (synthetic)", "model_bytes": size,
           "caller": "reference llama.cpp + ggml.c (oracle/_ref builds, unmodified sources)",
           "n_ctx": max(512, -(-(args.prompt + args.decode) // 512) * 512)}
    try:
        if not args.no_cpu:
            res["cpu"], lg_cpu = bench(CPU_LIB, model, args.prompt, args.decode_cpu, args.threads_cpu, 0, 1, nv)
            print("cpu", res["cpu"], file=sys.stderr, flush=True)
        L.ggml_hip_debug_graph_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
        for mode in args.modes.split(","):
            # modes: fast, exact; "-noepi" (below); suffix "-graph": launch recorder with HIP graphs (GGML_HIP_GRAPH=1),
            # "-thread": launcher thread (GGML_HIP_GRAPH=2), "-aql": own AQL queue (GGML_HIP_GRAPH=3)
            gh.check(L.ggml_hip_set_exact(1 if mode.startswith("exact") else 0))
            gh.check(L.ggml_hip_debug_set_graph(1 if mode.endswith("-graph") else 2 if mode.endswith("-thread") else
                                                3 if "-aql" in mode else 0))
            # "-noepi": the decode q|k|v GEMV epilogue off (the held rope / copy nodes as their own batch)
            L.ggml_hip_debug_set_epi_fold.argtypes = [ctypes.c_int]
            gh.check(L.ggml_hip_debug_set_epi_fold(0 if "-noepi" in mode else 1))
            # "-nokq": the decode KQ as its own launch
            L.ggml_hip_debug_set_kq_fold.argtypes = [ctypes.c_int]
            gh.check(L.ggml_hip_debug_set_kq_fold(0 if "-nokq" in mode else 1))
            # "-padN": a busy wait of N ns after every eager launch (the token time's dependence on launch cost)
            pad = int(mode.split("-pad")[1].split("-")[0]) if "-pad" in mode else 0
            L.ggml_hip_debug_set_launch_pad.argtypes = [ctypes.c_int]
            gh.check(L.ggml_hip_debug_set_launch_pad(pad))
            if not args.no_warm:
                # a short untimed run in this mode first: the first evals of a process (code-object loads, the
                # AQL queue and kernel lookups, pool growth) otherwise land in whichever mode is listed first
                bench(HIP_LIB, model, args.prompt, 4, args.threads_gpu, 99, 1, nv)
            g0 = np.zeros(5, np.int64)
            L.ggml_hip_debug_graph_stats(g0.ctypes.data, 0)
            L.ggml_hip_debug_op_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            st = np.zeros(2 * 68 + 1 + 15, np.int64)
            L.ggml_hip_debug_op_stats(st.ctypes.data, st.size, 1)
            L.ggml_hip_debug_launch_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
            ls = np.zeros(2, np.int64)
            L.ggml_hip_debug_launch_stats(ls.ctypes.data, 1)
            if args.hostprof:
                # a warm run first: the sampler's signals must not interrupt the HIP runtime's start-up
                # (device discovery, code-object loads), which then finds no device
                bench(HIP_LIB, model, args.prompt, 4, args.threads_gpu, 99, 1, nv)
                hp_lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhostprof.so"))
                hp_lib.hostprof_stop.argtypes = [ctypes.c_char_p]
                hp_lib.hostprof_start(50)
            L.ggml_hip_debug_aql_stats.argtypes = [ctypes.c_void_p]
            aq0 = np.zeros(4, np.int64)
            L.ggml_hip_debug_aql_stats(aq0.ctypes.data)
            r, lg = bench(HIP_LIB, model, args.prompt, args.decode, args.threads_gpu, 99, 3, nv)
            aq1 = np.zeros(4, np.int64)
            L.ggml_hip_debug_aql_stats(aq1.ctypes.data)
            if "-aql" in mode:       # per eval: dispatches, fallbacks, queue drains, HIP-stream waits
                r["aql_per_eval"] = [round(float(v) / (3 + args.decode), 1) for v in (aq1 - aq0)]
            if args.hostprof:
                r["hostprof_samples"] = hp_lib.hostprof_stop(f"{args.hostprof}.{mode}".encode())
            L.ggml_hip_debug_op_stats(st.ctypes.data, st.size, 1)
            L.ggml_hip_debug_launch_stats(ls.ctypes.data, 0)
            r["eager_launches_per_eval"] = round(float(ls[0]) / (3 + args.decode), 1)
            r["eager_launch_host_ms_per_eval"] = round(float(ls[1]) / 1e6 / (3 + args.decode), 3)
            ntok = 3 * args.prompt + args.decode      # evals: 3 prompt reps + decode steps
            r["backend_nodes_per_eval"] = round(float(st[:68].sum()) / (3 + args.decode), 1)
            r["backend_host_ms_per_eval"] = round(float(st[68]) / 1e6 / (3 + args.decode), 3)
            # per op of the arriving node: nodes per eval and host us per eval (fused chains are
            # charged to the node that completes them)
            r["backend_per_op"] = {OP_NAMES.get(i, str(i)): [round(float(st[i]) / (3 + args.decode), 1),
                                                             round(float(st[69 + i]) / 1e3 / (3 + args.decode), 1)]
                                   for i in range(68) if st[i] or st[69 + i]}
            g1 = np.zeros(5, np.int64)
            L.ggml_hip_debug_graph_stats(g1.ctypes.data, 0)
            g = (g1 - g0) / (3 + args.decode)
            r["graph_per_eval"] = {"runs": round(float(g[0]), 2), "kernels": round(float(g[1]), 1),
                                   "nodes_updated": round(float(g[2]), 1), "instantiated": round(float(g[3]), 2),
                                   "submit_ms": round(float(g[4]) / 1e6, 3)}
            r["finite"] = bool(np.isfinite(lg).all())
            if not args.no_cpu:       # same token sequence as the CPU run: compare the last logits
                _, lg8 = bench(HIP_LIB, model, args.prompt, args.decode_cpu, args.threads_gpu, 99, 1, nv)
                scale = float(np.abs(lg_cpu).max())
                r["last_logits_vs_cpu"] = ("bitwise" if np.array_equal(lg8.view(np.uint32), lg_cpu.view(np.uint32))
                                           else f"max |d|/max|y| {float(np.abs(lg8 - lg_cpu).max()) / scale:.2e}")
            key, k = f"offload_{mode}", 2
            while key in res:                      # a mode listed twice (interleaved repeats)
                key, k = f"offload_{mode}#{k}", k + 1
            res[key] = r
            print(mode, r, file=sys.stderr, flush=True)
        gh.check(L.ggml_hip_set_exact(0))
        gh.check(L.ggml_hip_debug_set_graph(0))
        gh.check(L.ggml_hip_debug_set_launch_pad(0))
    finally:
        os.remove(model)
        os.rmdir(d)
    if args.maps:      # after the evals: every library the reference llama.cpp pulled in is mapped by now
        mapped = {l.split()[-1] for l in open("/proc/self/maps") if "/" in l}
        res["libggml_hip_mapped"] = sorted(m for m in mapped if os.path.basename(m).startswith("libggml_hip")
                                           and "_cuda" not in m)
        res["ggml_hip_lib_env"] = os.environ.get("GGML_HIP_LIB")
    if "cpu" in res:
        res["cpu_cpu_name"] = open("/proc/cpuinfo").read().split("model name")[1].split(":")[1].split("\n")[0].strip()
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
