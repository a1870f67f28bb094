import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(" ".join(f"{r['N']}:{r['us']}" for r in rows if r["path"] == "gemm_sk"))
