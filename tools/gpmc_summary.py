"""Summary of the prefill GEMM counter passes (tools/run.sh PARTS=gpmc: rocprofv3 --pmc, one pass per counter set,
tools/gemm_one.py = k_gemm9 at K = M = 4096, N = 512): mean per dispatch of every counter, and the derived figures
DESIGN.md cites: MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x SIMDs) with cycles = GRBM_GUI_ACTIVE / 8 XCDs,
VALU instructions per MFMA, HBM read = 2 x FETCH_SIZE KiB (the gfx950 half count), SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES.

usage: python tools/gpmc_summary.py <gpmc dir> [SIMDs, default 1024]"""
import collections
import csv
import glob
import os
import statistics
import sys


def main(d, simds=1024):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)            # (dispatch, counter) -> value summed over dimensions
        for r in csv.DictReader(open(f)):
            if "k_gemm9" not in r.get("Kernel_Name", ""):
                continue
            per[(r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    m = {c: statistics.mean(v) for c, v in vals.items()}
    print("k_gemm9_q4_0 (registered fp6 image, tools/gemm_one.py), K=M=4096, N=512; mean per dispatch")
    for c in sorted(m):
        print(f"{c:28s} n={len(vals[c]):3d} mean={m[c]:.4g}")
    out = []
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        out.append(f"MFMA busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * simds):.3f} of {cyc:.0f} cycles")
    if "FETCH_SIZE" in m:
        out.append(f"HBM read {2 * m['FETCH_SIZE'] * 1024 / 1e6:.1f} MB (2 x FETCH_SIZE, gfx950 half count)")
    if "WRITE_SIZE" in m:
        out.append(f"write {m['WRITE_SIZE'] * 1024 / 1e6:.1f} MB")
    if "SQ_INSTS_VALU" in m and "SQ_INSTS_MFMA" in m:
        out.append(f"VALU per MFMA {m['SQ_INSTS_VALU'] / m['SQ_INSTS_MFMA']:.1f}")
    if "SQ_WAIT_INST_ANY" in m and "SQ_WAVE_CYCLES" in m:
        out.append(f"WAIT_INST_ANY / WAVE_CYCLES {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
    print("derived: " + "; ".join(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1024)
