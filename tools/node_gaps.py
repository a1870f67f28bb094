"""Host timeline of the hook from a GGML_HIP_TRACE_NODES=1 log (stderr of tools/e2e_llama.py): per decode eval,
the time inside the hook (taken nodes), the time between taken nodes (the caller: ggml's loop and its CPU
nodes), and the gap between one eval's last taken node and the next eval's first (the caller's graph build)."""
import re
import sys

import numpy as np


def main(path):
    t, d, names = [], [], []
    last = None
    for line in open(path, errors="replace"):
        if line.startswith("node op="):
            last = line.split()[2] if len(line.split()) > 2 else "?"
        elif line.startswith("node_ns "):
            p = line.split()
            d.append(int(p[1]))
            t.append(int(p[2]))
            names.append(last)
    t, d = np.array(t, np.int64), np.array(d, np.int64)
    end = t + d
    gaps = t[1:] - end[:-1]
    cut = np.flatnonzero(gaps > 200_000) + 1          # > 200 us between taken nodes: an eval boundary
    evals = np.split(np.arange(len(t)), cut)
    rows = []
    for i in range(1, len(evals) - 1):
        e = evals[i]
        inside = d[e].sum() / 1e3
        span = (end[e[-1]] - t[e[0]]) / 1e3
        boundary = (t[evals[i + 1][0]] - end[e[-1]]) / 1e3
        rows.append((len(e), span, inside, span - inside, boundary))
    r = np.array(rows)
    print(f"evals {len(r)} (taken nodes {r[:, 0].mean():.0f}): span first..last taken node {r[:, 1].mean():.0f} us, "
          f"inside the hook {r[:, 2].mean():.0f} us, caller between nodes {r[:, 3].mean():.0f} us, "
          f"boundary to the next eval {np.median(r[:, 4]):.0f} us (median)")
    e = evals[len(evals) // 2]
    big = sorted(((t[j + 1] - end[j]) / 1e3, names[j], names[j + 1]) for j in e[:-1])[-6:]
    print("largest caller gaps inside one eval (us, after -> before):", [(round(g, 1), a, b) for g, a, b in big])


if __name__ == "__main__":
    main(sys.argv[1])
