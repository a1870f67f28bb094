import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def pytest_terminal_summary(terminalreporter):
    """Parity report: per check_y call, the worst relative error (well-conditioned elements) and the
    smallest atol_blocks that would still pass (the bound is 1e-3|y| + atol_blocks * S_abs)."""
    try:
        from parity import REPORT
    except ImportError:
        return
    if not REPORT:
        return
    tr = terminalreporter
    tr.write_sep("-", f"parity report ({len(REPORT)} y checks; bound 1e-3|y| + atol_blocks*S_abs)")
    for tid, n, rel, need in REPORT:
        tr.write_line(f"{tid:<110s} n={n:<9d} max_rel={rel:.2e} atol_blocks_needed={need:.2e}")
    worst = max(r[3] for r in REPORT)
    tr.write_line(f"worst atol_blocks needed over the run: {worst:.2e}")
