"""Discrete-event model of a persistent decode engine (one LDS-DMA loader per CU running ahead through a
ring, consumers gated by the all-to-all edge of each op), used to decide whether to build it and with
which unit schedule.  Per-CU stream rate R (GB/s = KB/us), ring capacity RING (KB), edge latency E (us:
last producer done -> every consumer has x), consumer rate RC.

  python tools/engine_sim.py
"""
import heapq
import sys

CUS = 256
LAYER = [  # (op, units, unit_kb)  LLaMA-7B: 32-row units (one q8_0 block of the op's output)
    ("qkv", 384, 32 * 2304 / 1000), ("wo", 128, 32 * 2304 / 1000),
    ("w13", 688, 32 * 2304 / 1000), ("w2", 128, 32 * 6192 / 1000)]


def schedule(kind, layers, unit_rows=32):
    """per CU: list of (op_index, kb)"""
    per = [[] for _ in range(CUS)]
    load = [0.0] * CUS
    opi = 0
    for _ in range(layers):
        for name, units, kb in LAYER:
            u = units * 32 // unit_rows
            kbu = kb * unit_rows / 32
            if kind == "greedy":      # least cumulative bytes first
                order = sorted(range(CUS), key=lambda c: (load[c], c))
                for i in range(u):
                    c = order[i % CUS] if u >= CUS else order[i]
                    if u > CUS and i >= CUS:
                        order2 = sorted(range(CUS), key=lambda c: (load[c], c))
                        c = order2[0]
                    per[c].append((opi, kbu))
                    load[c] += kbu
            else:                     # round robin per op from CU 0
                for i in range(u):
                    per[i % CUS].append((opi, kbu))
                    load[i % CUS] += kbu
            opi += 1
    return per, opi


def simulate(per, nops, R=25.0, RING=128.0, E=3.0, RC=80.0, CH=16.0):
    """chunk-level: the loader streams CH-KB chunks in order at R, chunk i starts only after the consumer
    freed chunk i - RING/CH; the consumer takes chunks in order at RC, a unit's first chunk no earlier
    than its op's input edge (previous op's last unit done + E)"""
    slots = max(1, int(RING // CH))
    done_op = [0.0] * nops
    # per CU state
    lt = [0.0] * CUS               # loader time
    ct = [0.0] * CUS               # consumer time
    cfree = [[] for _ in range(CUS)]   # consumer finish time of each chunk, in order
    idx = [0] * CUS
    for op in range(nops):
        ready = 0.0 if op == 0 else done_op[op - 1] + E
        fin = 0.0
        for c in range(CUS):
            while idx[c] < len(per[c]) and per[c][idx[c]][0] == op:
                kb = per[c][idx[c]][1]
                first = True
                while kb > 1e-9:
                    ch = min(CH, kb)
                    kb -= ch
                    n = len(cfree[c])
                    start = lt[c]
                    if n - slots >= 0:
                        start = max(start, cfree[c][n - slots])
                    lt[c] = start + ch / R
                    cs = max(ct[c], lt[c], ready if first else 0.0)
                    first = False
                    ct[c] = cs + ch / RC
                    cfree[c].append(ct[c])
                fin = max(fin, ct[c])
                idx[c] += 1
        done_op[op] = fin
    return done_op


def main():
    layers = 8
    for kind in ("rr", "greedy"):
        for unit_rows in (32, 16):
            per, nops = schedule(kind, layers, unit_rows)
            for E in (1.5, 3.0, 4.0):
                for RING in (64, 128):
                    d = simulate(per, nops, E=E, RING=RING)
                    per_layer = (d[-1] - d[4 * 2 - 1]) / (layers - 2)
                    print(f"{kind:6s} unit {unit_rows:2d} rows  E {E:.1f}  ring {RING:3d} KB: {per_layer:5.1f} us/layer"
                          f" = {1e6 / (32 * per_layer):6.0f} tok/s")


if __name__ == "__main__":
    main()
