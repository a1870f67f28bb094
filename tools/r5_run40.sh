# End-of-round e2e evidence: the reference llama.cpp fully offloaded (LLaMA-7B shape): decode 128 (fast, exact,
# CPU), the launch recorder modes, a 500-token prompt with the k_gemm9 tile automatic vs forced 128 x 64, and a
# kernel trace of fast decode.
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python tools/e2e_llama.py --decode 128 --modes fast,exact --out $O/e2e_7b.json > $O/e2e_7b.log 2>&1; echo "e2e rc=$?"
timeout -k 10 500 python tools/e2e_llama.py --decode 128 --no-cpu --modes fast,fast-graph,fast-thread --out $O/e2e_7b_modes.json > $O/e2e_7b_modes.log 2>&1; echo "modes rc=$?"
for r in 1 2; do
  for w in -1 0; do
    GGML_HIP_GEMM9_WIDE=$w timeout -k 10 300 python tools/e2e_llama.py --prompt 500 --decode 8 --no-cpu --modes fast --out $O/e2e_p500_w${w}_$r.json > $O/e2e_p500_w${w}_$r.log 2>&1; echo "p500 w$w r$r rc=$?"
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_e2e -o e2e --output-format csv -- python3 tools/e2e_llama.py --decode 64 --no-cpu --modes fast > $O/e2e_prof.log 2>&1; echo "prof rc=$?"
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05e/*.json")):
    r = json.load(open(f))
    for k, v in r.items():
        if isinstance(v, dict) and "decode_tok_s" in v:
            print(f.split("/")[-1], k, "decode", v["decode_tok_s"], "tok/s; prompt", v["prompt_tokens"], v["prompt_ms"], "ms (min", v.get("prompt_ms_min"), ")")
PY
