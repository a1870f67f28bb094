"""CPU-side checks of the drop-in boundary: the C-ABI library builds, loads and exports every
symbol include/ggml-hip.h declares; the ggml_tensor mirror matches ggml.h; host-only logic
(row split, can_mul_mat rule) behaves like the reference.  No compute calls (no GPU here)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from hip_env import LIB_PATH, PKG, ggml_hip


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", PKG, "-j4"])
    return ggml_hip.load()


def test_library_exports_every_declared_symbol(lib):
    declared = ggml_hip.declared_symbols()
    assert len(declared) >= 50
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    for s in declared:
        assert hasattr(lib, s)


def test_library_targets_gfx950_only():
    out = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", LIB_PATH], text=True,
                                  stderr=subprocess.STDOUT) if False else ""
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert other not in blob


def test_no_oracle_linkage():
    """The product must never route through the oracle / a CPU fallback."""
    out = subprocess.check_output(["nm", "-D", LIB_PATH], text=True)
    assert "oracle_" not in out
    deps = subprocess.check_output(["readelf", "-d", LIB_PATH], text=True)
    assert "oracle" not in deps
    assert "libamdhip64" in deps and "librccl" in deps


def test_device_code_uses_no_runtime_services():
    """The AQL launch mode (csrc/ggml-hip-aql.cpp) fills only the dispatch-geometry hidden arguments: no kernel may
    use device printf, malloc / free or assert, whose hostcall / heap pointers would stay zero there."""
    import re
    csrc = os.path.join(PKG, "csrc")
    pat = re.compile(r"\b(printf|malloc|free|assert|__assert_fail)\s*\(")
    for f in sorted(os.listdir(csrc)):
        if not (f.endswith(".hip") or f in ("q4_0_device.h",)):
            continue
        for i, line in enumerate(open(os.path.join(csrc, f)), 1):
            code = line.split("//")[0]
            hits = [m for m in pat.findall(code) if m]
            assert not hits, f"{f}:{i}: {line.strip()}"


def test_ggml_tensor_mirror_layout():
    T = ggml_hip.GgmlTensor
    assert ctypes.sizeof(T) == 240
    off = {name: getattr(T, name).offset for name, _ in T._fields_}
    assert (off["ne"], off["nb"], off["op"], off["src0"], off["src1"], off["n_tasks"], off["data"],
            off["name"], off["extra"]) == (16, 48, 80, 96, 104, 144, 168, 176, 224)
    assert ctypes.sizeof(ggml_hip.GgmlComputeParams) == 32


@pytest.mark.parametrize("M,n", [(4096, 8), (11008, 8), (5120, 8), (13824, 8), (4672, 3), (7, 4), (0, 2)])
def test_split_rows_equal(lib, M, n):
    rb = np.zeros(n + 1, np.int64)
    ggml_hip.check(lib.ggml_hip_split_rows(M, n, None, rb.ctypes.data_as(ctypes.c_void_p)))
    assert rb[0] == 0 and rb[-1] == M and np.all(np.diff(rb) >= 0)
    assert np.diff(rb).max() - np.diff(rb).min() <= 1


def test_split_rows_fractions_match_reference_rule(lib):
    """ggml-cuda.cu:1863-1882 normalises cumulative fractions; rows = (int)(nrows*split[id])."""
    ts = np.array([3.0, 1.0, 2.0, 2.0], np.float32)
    M = 11008
    rb = np.zeros(5, np.int64)
    ggml_hip.check(lib.ggml_hip_split_rows(M, 4, ts.ctypes.data_as(ctypes.c_void_p), rb.ctypes.data_as(ctypes.c_void_p)))
    cum = np.concatenate([[0], np.cumsum(ts)[:-1]]).astype(np.float32) / np.float32(ts.sum())
    expect = [0] + [int(np.float32(M) * c) for c in cum[1:]] + [M]
    assert list(rb) == expect


def _reference_split_rows_f32(M, ts):
    """float32 restatement of ggml-cuda.cu:1874-1881 (cumulative start fractions summed and divided
    in float) and :2363-2364 (row_low = nrows0*g_tensor_split[id], an int64*float product truncated)."""
    s = np.float32(0)
    starts = []
    for t in np.asarray(ts, np.float32):
        starts.append(s)
        s = np.float32(s + t)
    frac = [np.float32(c / s) for c in starts]
    return [0] + [int(np.float32(np.float32(M) * f)) for f in frac[1:]] + [M]


SPLITS = [[0.1, 0.2, 0.3, 0.4], [1 / 3, 1 / 3, 1 / 3], [0.3, 0.3, 0.4], [0.7, 0.1, 0.1, 0.1],
          [0.125] * 8, [0.15, 0.05, 0.2, 0.1, 0.1, 0.1, 0.1, 0.1], [1 / 7] * 7, [0.6, 0.4]]


@pytest.mark.parametrize("ts", SPLITS, ids=lambda t: "x".join(f"{v:.3g}" for v in t))
def test_split_rows_non_representable_fractions_bit_exact(lib, ts):
    """Non-representable fractions: every boundary row equals the reference's float rule bit for
    bit (a double-precision sum puts some boundaries one row away, e.g. M=9 with the 8-way split).
    The LLaMA/Falcon/13B row counts plus every M < 2048."""
    n = len(ts)
    tsa = np.asarray(ts, np.float32)
    for M in list(range(0, 2048)) + [4096, 4544, 4672, 5120, 11008, 13824, 18176, 32000]:
        rb = np.zeros(n + 1, np.int64)
        ggml_hip.check(lib.ggml_hip_split_rows(M, n, tsa.ctypes.data_as(ctypes.c_void_p),
                                               rb.ctypes.data_as(ctypes.c_void_p)))
        assert list(rb) == _reference_split_rows_f32(M, tsa), (M, ts)


def test_can_mul_mat_declines_without_device(lib):
    """No HIP device: every node is declined, so ggml.c plans and runs its own CPU mul_mat (the
    shape rule itself, ggml-cuda.cu:2595-2610, is tests/test_gpu_parity.py::test_can_mul_mat_rule)."""
    if lib.ggml_hip_device_count() > 0:
        pytest.skip("a HIP device is present")
    K, M, N = 4096, 64, 512
    w = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_Q4_0, (K, M))
    x = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (K, N))
    y = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (M, N))
    assert not lib.ggml_hip_can_mul_mat(ctypes.byref(w), ctypes.byref(x), ctypes.byref(y))
    assert lib.ggml_hip_mul_mat_get_wsize(ctypes.byref(w), ctypes.byref(x), ctypes.byref(y)) == 0


def test_compute_forward_declines_other_ops_without_device(lib):
    """Non-MUL_MAT nodes are never taken (ggml.c falls through to its CPU op)."""
    t = ggml_hip.make_tensor(ggml_hip.GGML_TYPE_F32, (64, 64))
    t.op = 5   # not MUL_MAT
    p = ggml_hip.GgmlComputeParams(ggml_hip.GGML_TASK_COMPUTE, 0, 1, 0, None)
    assert not lib.ggml_hip_compute_forward(ctypes.byref(p), ctypes.byref(t))


def test_version(lib):
    assert b"gfx950" in lib.ggml_hip_version()


def test_cuda_abi_shim_exports_reference_names():
    """libggml_hip_cuda.so exports every ggml-cuda.h name declared in include/ggml-hip-cuda-abi.h
    (the full reference list, ggml-cuda.h:15-36) and forwards to libggml_hip.so."""
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(LIB_PATH)), "include", "ggml-hip-cuda-abi.h")
    shim = os.path.join(os.path.dirname(LIB_PATH), "libggml_hip_cuda.so")
    src = re.sub(r"/\*.*?\*/", "", open(hdr).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(ggml_(?:cuda|init_cublas)\w*)\s*\(", src)))
    assert len(declared) == 17
    out = subprocess.check_output(["nm", "-D", "--defined-only", shim], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not [s for s in declared if s not in exported]
    deps = subprocess.check_output(["readelf", "-d", shim], text=True)
    assert "libggml_hip.so" in deps and "oracle" not in deps


def test_op_enum_mirror_matches_reference_header():
    """csrc/ggml_abi.h's GGML_OP_* / GGML_TYPE_* values equal the reference ggml.h's (the fork shifts
    MUL_MAT and later ops by four EXT ops); the fixture was generated from the reference header by
    tests/golden/gen_ggml_enum.c."""
    import json
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ref = json.load(open(os.path.join(root, "tests", "golden", "ggml_op_enum.json")))
    src = open(os.path.join(root, "llama.cpp-q_4_0_amd", "csrc", "ggml_abi.h")).read()
    mine = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(OP_\w+|TYPE_\w+) = (\d+)", src)}
    for name, v in ref.items():
        key = name.replace("GGML_", "")
        assert mine[key] == v, (name, mine.get(key), v)


def test_library_identity_soname_and_exports():
    """libggml_hip.so carries SONAME libggml_hip.so and exports the C ABI only (ggml_*): no internal
    C++ symbol (ghip:: / ghh:: globals) can be interposed by, or interpose onto, another copy."""
    dyn = subprocess.check_output(["readelf", "-d", LIB_PATH], text=True)
    assert "Library soname: [libggml_hip.so]" in dyn
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH], text=True)
    exported = [line.split()[-1] for line in out.splitlines() if line.strip()]
    assert exported and all(s.startswith("ggml_") for s in exported), [s for s in exported if not s.startswith("ggml_")][:5]


_MAPS_PROBE = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
import ggml_hip
ggml_hip.load()
for p in sys.argv[2:]:
    ctypes.CDLL(p)            # the caller side: NEEDED libggml_hip_cuda.so -> NEEDED libggml_hip.so
maps = {l.split()[-1] for l in open("/proc/self/maps") if "/" in l}
copies = sorted(m for m in maps if os.path.basename(m).startswith("libggml_hip") and "_cuda" not in m)
print("\n".join(copies))
"""


def test_variant_library_is_the_only_mapped_copy(tmp_path):
    """GGML_HIP_LIB pointing at a variant build (another file name) and the reference's hooked llama.cpp
    (or the ggml-cuda.h shim) loaded after it: exactly ONE libggml_hip is mapped.  Without a SONAME the
    shim's NEEDED libggml_hip.so resolved through its RUNPATH to the in-tree file, a second copy whose
    default-visibility globals interposed onto the first and whose static destructors ran on the same
    objects at exit (round 5's `double free or corruption` after the e2e line)."""
    import shutil
    variant = tmp_path / "libggml_hip_variant.so"
    shutil.copy(LIB_PATH, variant)
    callers = [os.path.join(os.path.dirname(LIB_PATH), "libggml_hip_cuda.so")]
    ref = os.path.join(os.path.dirname(PKG), "oracle", "_ref", "libllama_ref_hip.so")
    if os.path.exists(ref):
        callers.append(ref)
    env = dict(os.environ, GGML_HIP_LIB=str(variant))
    r = subprocess.run([os.sys.executable, "-c", _MAPS_PROBE, os.path.join(PKG, "python")] + callers, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    copies = r.stdout.split()
    assert copies == [str(variant)], copies
