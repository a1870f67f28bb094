"""Resolve tools/hostprof.c samples: self and inclusive time per function (busiest thread first).
usage: hostprof_report.py samples.txt [top]"""
import collections
import gzip
import os
import subprocess
import sys


def main(path, top=40):
    maps, samples = [], []
    for line in (gzip.open(path, "rt") if path.endswith(".gz") else open(path)):
        if line.startswith("M "):
            p = line[2:].split()
            if len(p) >= 6 and "x" in p[1]:
                lo, hi = (int(x, 16) for x in p[0].split("-"))
                maps.append((lo, hi, int(p[2], 16), p[5]))
        elif line.startswith("S "):
            p = line[2:].split()
            samples.append((int(p[0]), [int(x, 16) for x in p[1:]]))
    tids = collections.Counter(t for t, _ in samples)
    print("samples per thread:", tids.most_common(6))
    main_tid = tids.most_common(1)[0][0]
    addrs = set(a for t, st in samples if t == main_tid for a in st)

    def where(a):
        for lo, hi, off, mod in maps:
            if lo <= a < hi:
                return mod, a - lo + off
        return "?", a
    bymod = collections.defaultdict(set)
    loc = {}
    for a in addrs:
        mod, off = where(a)
        loc[a] = (mod, off)
        bymod[mod].add(off)
    name = {}

    def to_vaddr(mod2, offs):     # file offset -> ELF virtual address (lld puts .text at offset + 0x1000)
        segs = []
        out = subprocess.run(["readelf", "-lW", mod2], capture_output=True, text=True).stdout
        for ln in out.splitlines():
            p = ln.split()
            if p and p[0] == "LOAD":
                segs.append((int(p[1], 16), int(p[2], 16), int(p[4], 16)))
        res = []
        for o in offs:
            v = o
            for po, pv, sz in segs:
                if po <= o < po + sz:
                    v = o - po + pv
            res.append(v)
        return res
    for mod, offs in bymod.items():
        offs = sorted(offs)
        if not os.path.exists(mod):             # a path on the GPU box: the same file in this tree
            for part in ("/oracle/", "/llama.cpp-q_4_0_amd/", "/tools/"):
                if part in mod and os.path.exists("/root/repo" + part + mod.split(part, 1)[1]):
                    mod2 = "/root/repo" + part + mod.split(part, 1)[1]
                    break
            else:
                mod2 = None
        else:
            mod2 = mod
        if mod2 is None:
            for o in offs:
                name[(mod, o)] = os.path.basename(mod) + "+?"
            continue
        out = subprocess.run(["addr2line", "-f", "-C", "-e", mod2] + [hex(o) for o in to_vaddr(mod2, offs)], capture_output=True,
                             text=True).stdout.split("\n")
        for i, o in enumerate(offs):
            fn = out[2 * i] if 2 * i < len(out) else "?"
            name[(mod, o)] = (fn if fn != "??" else "?") + " [" + os.path.basename(mod) + "]"
    selfc, incl = collections.Counter(), collections.Counter()
    n = 0
    for t, st in samples:
        if t != main_tid or not st:
            continue
        n += 1
        fns = [name[loc[a]] for a in st]
        selfc[fns[0]] += 1
        for f in set(fns):
            incl[f] += 1
    print(f"main thread {main_tid}: {n} samples")
    print("--- self")
    for f, c in selfc.most_common(top):
        print(f"{100 * c / n:6.2f}%  {f[:150]}")
    print("--- inclusive")
    for f, c in incl.most_common(top):
        print(f"{100 * c / n:6.2f}%  {f[:150]}")
    mods = collections.Counter()
    for t, st in samples:
        if t == main_tid and st:
            mods[os.path.basename(loc[st[0]][0])] += 1
    print("--- self by module")
    for m, c in mods.most_common(12):
        print(f"{100 * c / n:6.2f}%  {m}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
