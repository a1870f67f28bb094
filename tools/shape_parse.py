import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(" ".join(f"{r['K']}x{r['M']}:{r['us']}" for r in rows))
