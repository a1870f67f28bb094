"""bench.py's multi-rank flow end to end on one MI355X (verdict r4 item 1): `bench.py --gpus 2` with no
launcher in the environment starts two fresh rank processes itself (no exec, before any GPU library is
loaded), both on device 0.  RCCL refuses two ranks on one device, so the ranks pick the file-rendezvous
comm and the direct-store P2P all-gather across the process boundary (IPC mappings) — the same sharded
decode code, self-checks and JSON line the driver's 8-GPU run produces (there with RCCL and P2P both).
Also the BASELINE config-4 line (LLaMA-13B row-sharded) rides along at reduced depth."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_self_launched_two_ranks_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--layers", "2", "--config4-layers", "2",
           "--steps", "2", "--warmup", "1", "--no-prefill", "--no-cpu", "--no-extra", "--no-exact"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout[-2000:]            # rank 0's one JSON line, nothing else on stdout
    r = json.loads(lines[0])
    cfg = r["config"]
    assert r["n_gpus"] == 2 and cfg["self_launched"] and cfg["comm"] == "file", cfg
    assert r["value"] > 0 and cfg["transport"] == "direct-store P2P"
    assert cfg["split_check"]["own_rows_bitwise"] and cfg["split_check"]["gather_checksum"], cfg["split_check"]
    p2p = cfg["p2p_transport"]
    assert p2p["status_ok"] and p2p["split_check"]["own_rows_bitwise"] and p2p["split_check"]["gather_checksum"], p2p
    c4 = r["config4_llama13b_sharded"]
    assert c4["self_checks_passed"] and c4["split_check"]["own_rows_bitwise"] and c4["split_check"]["gather_checksum"]
    assert c4["tok_s"] > 0 and c4["compute_only_tok_s"] > 0
    print(json.dumps({"value": r["value"], "compute_only_tok_s": cfg["compute_only_tok_s"],
                      "config4_tok_s": c4["tok_s"]}))
