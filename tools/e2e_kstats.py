"""Per-kernel decode-phase summary of a rocprofv3 --kernel-trace database of tools/e2e_llama.py (sqlite
rocpd output): kernels per eval, average duration, device busy vs wall per eval, one layer's sequence."""
import collections
import re
import sqlite3
import sys


def short(n):
    n = re.sub(r"^void ", "", n)
    n = n.replace("(anonymous namespace)::", "")
    depth, out = 0, ""
    for ch in n:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out += ch
    return out


def main(db, n_dec=62, marker="k_gemv_q4_0<1, 16, 1, 15, 1, 1, 0, 1>"):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if marker in short(r[0])]
    per = max(1, len(idx) // (n_dec + 5))
    seg = rows[idx[-n_dec * per]:]
    t0, t1 = seg[0][1], seg[-1][2]
    busy = sum(e - s for _, s, e in seg)
    print(f"evals {n_dec}: wall/eval {(t1 - t0) / n_dec / 1e3:.1f} us, busy {busy / n_dec / 1e3:.1f} us, "
          f"kernels/eval {len(seg) / n_dec:.1f}")
    agg = collections.defaultdict(list)
    for n, s, e in seg:
        agg[short(n)].append(e - s)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v) / n_dec:6.1f}/eval {sum(v) / len(v) / 1e3:8.2f} us {sum(v) / n_dec / 1e3:8.1f} us/eval  {k[:90]}")
    i0, i1 = idx[-10], idx[-9]
    print("one layer:")
    for n, s, e in rows[i0:i1 + 1]:
        print(f"  {(e - s) / 1e3:7.2f} us at {(s - rows[i0][1]) / 1e3:8.2f}  {short(n)[:80]}")


if __name__ == "__main__":
    main(*sys.argv[1:2])
