#!/bin/bash
# copy the evidence of the last tools/r3_final.sh run (gpurun_out/r03) into profiles/ (run here, not on the box)
cd "$(dirname "$0")/.."
O=gpurun_out/r03
L=$O/gputest.log
{ echo "Round 3 final GPU test run (one MI355X, gpurun box), commit $(git rev-parse --short HEAD)"
  echo "command: python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread   (tools/r3_final.sh)"
  echo; grep -E "^=+ .*(passed|failed)" $L | tail -n 1
  echo; echo "== skipped (id: reason) =="; grep "^SKIPPED" $L
  echo; echo "== parity report (conftest terminal summary) =="
  sed -n '/parity report/,$p' $L | grep -v -E "^=+ .*passed"
  echo; echo "== smoke (__graft_entry__.smoke on cuda:0) =="; cat $O/smoke.log
  echo; echo "== per-test results =="; grep -E "PASSED|SKIPPED|FAILED|ERROR" $L | grep "::" | sed 's/ *\[ *[0-9]*%\]//'
} > profiles/r03_gputest_summary.txt
tail -n 1 $O/bench.log > profiles/r03_bench_line.json
cp $O/prof/run_kernel_stats.csv profiles/r03_bench_rocprofv3_kernel_stats.csv
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv > profiles/r03_bench_rocprofv3_trace_summary.txt
cp $O/gemv_pmc_traffic.json profiles/r03_gemv_pmc_traffic.json
python3 - <<'PY'
import re
t = open('gpurun_out/r03/gemm9_pmc.txt').read()
v = {m.group(1): float(m.group(2)) for m in re.finditer(r"^(\w+)\s+n=\s*\d+ mean=(\S+)", t, re.M)}
cyc = v['GRBM_GUI_ACTIVE'] / 8
t += ("\nderived: MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); LDS conflicts = "
      "SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; HBM = 2*FETCH_SIZE (gfx950 half count) + WRITE_SIZE, KiB\n")
t += (f"MFMA busy {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f} of {cyc:.0f} cycles; LDS bank conflicts "
      f"{v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.3f}; HBM read {2 * v['FETCH_SIZE'] * 1024 / 1e6:.1f} MB "
      f"(fp6 images: 13.6 MB weights + 3.4 MB x per dispatch; x is fetched once per XCD L2) write "
      f"{v['WRITE_SIZE'] * 1024 / 1e6:.1f} MB; VALU per MFMA {v['SQ_INSTS_VALU'] / v['SQ_INSTS_MFMA']:.1f}; "
      f"WAIT_INST_ANY/WAVE_CYCLES {v['SQ_WAIT_INST_ANY'] / v['SQ_WAVE_CYCLES']:.3f}, WAIT_ANY/WAVE_CYCLES "
      f"{v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']:.3f}\n")
open('profiles/r03_gemm9_pmc.txt', 'w').write(t)
print(t[-420:])
PY
