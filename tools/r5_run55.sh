# final e2e: decode 128 (fast, exact, CPU) and the 500-token prompt, at the final launch plan
set -o pipefail
O=gpurun_out/r05e2; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python tools/e2e_llama.py --decode 128 --modes fast,exact --out $O/e2e_7b.json > $O/e2e_7b.log 2>&1; echo "e2e rc=$?"
for r in 1 2; do
  timeout -k 10 300 python tools/e2e_llama.py --prompt 500 --decode 8 --no-cpu --modes fast --out $O/e2e_p500_$r.json > $O/e2e_p500_$r.log 2>&1; echo "p500 r$r rc=$?"
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05e2/*.json")):
    r = json.load(open(f))
    for k, v in r.items():
        if isinstance(v, dict) and "decode_tok_s" in v:
            print(f.split("/")[-1], k, "decode", v["decode_tok_s"], "tok/s; prompt", v["prompt_tokens"], v["prompt_ms"], "ms (min", v.get("prompt_ms_min"), ")")
PY
