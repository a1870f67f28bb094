"""ctypes binding of libggml_hip.so (include/ggml-hip.h) for tests and bench.py.

This is the ctypes stub a Python host would add for the backend (INTEGRATION.md shows the
same for ggml.c itself).  Nothing here computes: every operation is a C-ABI call into the
HIP library, and loading fails loudly when the library is missing.

Runtime note: the library links libamdhip64.so.7 / librccl.so.1 from /opt/rocm (its RUNPATH), the
runtime it was built against.  torch bundles its own copies; a process that loads this library
must not import torch first (the first mapped soname wins process-wide).  bench.py and the GPU
tests never import torch (tests/conftest.py loads this library before any test module).
"""
import ctypes
import os
import sys

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GGML_HIP_LIB") or os.path.join(PKG, "libggml_hip.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "ggml-hip.h")

OK = 0
ERR_INVALID, ERR_UNSUPPORTED, ERR_DEVICE, ERR_NOMEM, ERR_COMM = -1, -2, -3, -4, -5

_lib = None


class GgmlHipError(RuntimeError):
    pass


def _bind(L):
    vp, i32, i64, sz, fl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float
    cp = ctypes.c_char_p
    sigs = {
        "ggml_init_hip": ([], None),
        "ggml_hip_set_tensor_split": ([vp], None),
        "ggml_hip_can_mul_mat": ([vp, vp, vp], ctypes.c_bool),
        "ggml_hip_mul_mat_get_wsize": ([vp, vp, vp], sz),
        "ggml_hip_mul_mat": ([vp, vp, vp], None),
        "ggml_hip_host_malloc": ([sz], vp),
        "ggml_hip_host_free": ([vp], None),
        "ggml_hip_transform_tensor": ([vp, vp], None),
        "ggml_hip_free_data": ([vp], None),
        "ggml_hip_assign_buffers": ([vp], None),
        "ggml_hip_assign_buffers_no_scratch": ([vp], None),
        "ggml_hip_assign_buffers_force_inplace": ([vp], None),
        "ggml_hip_set_main_device": ([i32], None),
        "ggml_hip_set_scratch_size": ([sz], None),
        "ggml_hip_free_scratch": ([], None),
        "ggml_hip_compute_forward": ([vp, vp], ctypes.c_bool),
        "ggml_cpu_has_hipblas": ([], i32),
        "ggml_hip_quantize_q8_0": ([vp, i64, i64, vp, vp], i32),
        "ggml_hip_quantize_q4_0": ([vp, i64, i64, vp, vp], i32),
        "ggml_hip_dequantize_q4_0": ([vp, i64, i64, vp, vp], i32),
        "ggml_hip_mul_mat_q4_0": ([vp, i64, i64, vp, i64, vp, vp], i32),
        "ggml_hip_mul_mat_q4_0_ex": ([vp, i64, i64, vp, i64, vp, i64, i32, vp], i32),
        "ggml_hip_reserve_workspace": ([i64, i64], i32),
        "ggml_hip_reserve_workspace_mm": ([i64, i64, i64], i32),
        "ggml_hip_weight_image_create": ([vp, i64, i64, vp], i32),
        "ggml_hip_comm_enable_p2p": ([vp, i64], i32),
        "ggml_hip_comm_set_transport": ([vp, i32], i32),
        "ggml_hip_comm_p2p_status": ([vp], i32),
        "ggml_hip_comm_set_p2p_timeout": ([vp, ctypes.c_double], i32),
        "ggml_hip_comm_abort": ([vp], i32),
        "ggml_hip_comm_init_file": ([vp, i32, i32, cp], i32),
        "ggml_hip_weight_image_free": ([vp], i32),
        "ggml_hip_weight_image_bytes": ([], i64),
        "ggml_hip_debug_set_gemm_version": ([i32], i32),
        "ggml_hip_mul_mat_q4_0_multi": ([i32, vp, vp, i64, vp, i64, vp, vp], i32),
        "ggml_hip_comm_unique_id": ([vp], i32),
        "ggml_hip_comm_init": ([vp, i32, i32, vp], i32),
        "ggml_hip_comm_destroy": ([vp], i32),
        "ggml_hip_comm_init_local": ([vp, i32, vp], i32),
        "ggml_hip_comm_rank": ([vp, vp, vp], i32),
        "ggml_hip_comm_allreduce_host": ([vp, vp, i32, i32], i32),
        "ggml_hip_comm_allgather_host": ([vp, vp, sz, vp], i32),
        "ggml_hip_stream_create": ([], vp),
        "ggml_hip_stream_destroy": ([vp], i32),
        "ggml_hip_split_rows": ([i64, i32, vp, vp], i32),
        "ggml_hip_mul_mat_q4_0_split": ([vp, vp, i64, i64, vp, vp, i64, vp, vp], i32),
        "ggml_hip_mul_mat_q4_0_split_multi": ([vp, i32, vp, vp, vp, i64, vp, i64, vp, vp], i32),
        "ggml_hip_weight_cache_stats": ([vp, vp, vp], i32),
        "ggml_hip_weight_cache_clear": ([], i32),
        "ggml_hip_weight_cache_invalidate": ([vp, sz], i64),
        "ggml_hip_weight_cache_set_verify": ([i32], i32),
        "ggml_hip_weight_cache_invalidations": ([], i64),
        "ggml_hip_set_exact": ([i32], i32),
        "ggml_hip_get_exact": ([], i32),
        "ggml_hip_device_count": ([], i32),
        "ggml_hip_set_device": ([i32], i32),
        "ggml_hip_get_device": ([], i32),
        "ggml_hip_dev_malloc": ([sz], vp),
        "ggml_hip_dev_free": ([vp], None),
        "ggml_hip_memcpy_h2d": ([vp, vp, sz, vp], i32),
        "ggml_hip_memcpy_d2h": ([vp, vp, sz, vp], i32),
        "ggml_hip_memcpy_d2d": ([vp, vp, sz, vp], i32),
        "ggml_hip_memset": ([vp, i32, sz, vp], i32),
        "ggml_hip_stream_synchronize": ([vp], i32),
        "ggml_hip_device_synchronize": ([], i32),
        "ggml_hip_default_stream": ([], vp),
        "ggml_hip_fill_gaussian": ([vp, i64, ctypes.c_uint64, fl, fl, vp], i32),
        "ggml_hip_event_create": ([], vp),
        "ggml_hip_event_record": ([vp, vp], i32),
        "ggml_hip_event_elapsed_ms": ([vp, vp], fl),
        "ggml_hip_event_destroy": ([vp], None),
        "ggml_hip_graph_begin": ([vp], i32),
        "ggml_hip_graph_end": ([vp, vp], i32),
        "ggml_hip_graph_launch": ([vp, vp], i32),
        "ggml_hip_graph_destroy": ([vp], i32),
        "ggml_hip_chain_create": ([i32, vp, vp], i32),
        "ggml_hip_chain_create_n": ([i32, vp, i64, vp], i32),
        "ggml_hip_debug_set_chain_x9": ([i32], i32),
        "ggml_hip_debug_chain_links": ([i32, vp, i64, vp, vp], i32),
        "ggml_hip_chain_launch": ([vp, vp], i32),
        "ggml_hip_chain_status": ([vp], i32),
        "ggml_hip_chain_destroy": ([vp], i32),
        "ggml_hip_chain_set_engine": ([vp, i32], i32),
        "ggml_hip_debug_set_stream_launch_mode": ([vp, i32], i32),
        "ggml_hip_chain_engine_info": ([vp, vp, i32], i32),
        "ggml_hip_last_error": ([], cp),
        "ggml_hip_version": ([], cp),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return sigs


def declared_symbols():
    """Function names declared in include/ggml-hip.h (parsed, for the ABI export test)."""
    import re
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(ggml_\w+|ggml_cpu_has_hipblas)\s*\(", src)
    return sorted(set(n for n in names if n not in ("ggml_tensor",)))


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GgmlHipError(f"{LIB_PATH} not built: run `make -C llama.cpp-q_4_0_amd` (or __graft_entry__.build())")
    if "torch" in sys.modules and os.environ.get("GGML_HIP_ALLOW_TORCH_RUNTIME") != "1":
        import warnings
        warnings.warn("torch was imported before libggml_hip.so: the process may run on torch's bundled "
                      "HIP/RCCL runtime instead of /opt/rocm's (see ggml_hip module doc)")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    _bind(L)
    _lib = L
    return L


def check(rc, what="ggml_hip"):
    if rc != OK:
        raise GgmlHipError(f"{what} failed ({rc}): {load().ggml_hip_last_error().decode()}")


def device_count():
    return load().ggml_hip_device_count()


def mapped_runtime_libs():
    """Paths of the HIP / RCCL runtime libraries mapped into this process (/proc/self/maps)."""
    libs = set()
    try:
        for line in open("/proc/self/maps"):
            p = line.split()[-1] if "/" in line else ""
            if any(n in p for n in ("librccl", "libamdhip64", "libhsa-runtime64", "libggml_hip")):
                libs.add(p)
    except OSError:
        pass
    return sorted(libs)


class DeviceBuffer:
    """Owning device allocation (hipMalloc through the C ABI)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self.ptr = load().ggml_hip_dev_malloc(max(self.nbytes, 1))
        if not self.ptr:
            raise GgmlHipError(f"device allocation of {nbytes} bytes failed")

    @classmethod
    def from_array(cls, a, stream=None):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a, stream)
        return b

    def upload(self, a, stream=None):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        check(load().ggml_hip_memcpy_h2d(self.ptr, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, stream), "h2d")

    def download(self, shape, dtype, stream=None, offset=0):
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes + offset <= self.nbytes
        check(load().ggml_hip_memcpy_d2h(out.ctypes.data_as(ctypes.c_void_p), self.ptr + offset, out.nbytes, stream),
              "d2h")
        return out

    def free(self):
        if self.ptr:
            load().ggml_hip_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ---------------------------------------------------------------------------------------------
# thin wrappers of the tensor-free entry points

def quantize_q8_0(x_dev, K, N, xq_dev, stream=None):
    check(load().ggml_hip_quantize_q8_0(x_dev.ptr, K, N, xq_dev.ptr, stream), "quantize_q8_0")


def quantize_q4_0(w_dev, K, M, wq_dev, stream=None):
    check(load().ggml_hip_quantize_q4_0(w_dev.ptr, K, M, wq_dev.ptr, stream), "quantize_q4_0")


def dequantize_q4_0(wq_dev, K, M, w_dev, stream=None):
    check(load().ggml_hip_dequantize_q4_0(wq_dev.ptr, K, M, w_dev.ptr, stream), "dequantize_q4_0")


def mul_mat(w_dev, K, M, x_dev, N, y_dev, algo=0, ldy=None, stream=None, w_off=0, x_off=0, y_off=0):
    wp = w_dev if isinstance(w_dev, int) else w_dev.ptr
    xp = x_dev if isinstance(x_dev, int) else x_dev.ptr
    yp = y_dev if isinstance(y_dev, int) else y_dev.ptr
    check(load().ggml_hip_mul_mat_q4_0_ex(wp + w_off, K, M, xp + x_off, N, yp + y_off, M if ldy is None else ldy,
                                          algo, stream), "mul_mat_q4_0")


def mul_mat_multi(ws, Ms, K, x_dev, N, ys, stream=None):
    """Sibling mul_mats sharing x: ws / ys are DeviceBuffers (or raw pointers)."""
    n = len(ws)
    wp = (ctypes.c_void_p * n)(*[w if isinstance(w, int) else w.ptr for w in ws])
    yp = (ctypes.c_void_p * n)(*[y if isinstance(y, int) else y.ptr for y in ys])
    mp = (ctypes.c_int64 * n)(*Ms)
    xp = x_dev if isinstance(x_dev, int) else x_dev.ptr
    check(load().ggml_hip_mul_mat_q4_0_multi(n, wp, mp, K, xp, N, yp, stream), "mul_mat_q4_0_multi")


class ChainTask(ctypes.Structure):
    """struct ggml_hip_chain_task (include/ggml-hip.h)"""
    _fields_ = [("nmat", ctypes.c_int), ("K", ctypes.c_int64), ("x", ctypes.c_void_p),
                ("W", ctypes.c_void_p * 4), ("M", ctypes.c_int64 * 4), ("y", ctypes.c_void_p * 4)]


def _ptr(b):
    return b if isinstance(b, int) else b.ptr


class Chain:
    """A chain (ggml_hip_chain_*): tasks = [(ws, Ms, K, x, ys), ...] run in stream order, one sibling
    launch per task; task t reads x after every earlier task wrote its y.  N = 1: decode (GEMVs, optional
    engine); N > 1: ggml_hip_chain_create_n (prefill: GEMM epilogues write the next task's x image)."""

    def __init__(self, tasks, engine=None, N=1):
        L = load()
        arr = (ChainTask * len(tasks))()
        for t, (ws, Ms, K, x, ys) in enumerate(tasks):
            arr[t].nmat = len(ws)
            arr[t].K = K
            arr[t].x = _ptr(x)
            for i in range(len(ws)):
                arr[t].W[i] = _ptr(ws[i])
                arr[t].M[i] = Ms[i]
                arr[t].y[i] = _ptr(ys[i])
        self.h = ctypes.c_void_p()
        if N == 1:
            check(L.ggml_hip_chain_create(len(tasks), arr, ctypes.byref(self.h)), "chain_create")
        else:
            check(L.ggml_hip_chain_create_n(len(tasks), arr, N, ctypes.byref(self.h)), "chain_create_n")
        if engine is not None:
            self.set_engine(engine)

    def set_engine(self, on):
        """1 on (returns True when the persistent engine runs the chain), 0 off; the reason of a decline is
        in ggml_hip_last_error()"""
        rc = load().ggml_hip_chain_set_engine(self.h, 1 if on else 0)
        if rc < 0:
            check(rc, "chain_set_engine")
        return rc == 1

    def engine_info(self):
        """{on, units, max_stream_bytes, weight_bytes, cus} of the engine's plan (on = 0: per-launch path), and
        epilogue_images: tasks of an N-token chain whose x image a producer's GEMM epilogue writes"""
        v = (ctypes.c_int64 * 6)()
        check(load().ggml_hip_chain_engine_info(self.h, v, 6), "chain_engine_info")
        return dict(zip(("on", "units", "max_stream_bytes", "weight_bytes", "cus", "epilogue_images"), list(v)))

    def launch(self, stream=None):
        check(load().ggml_hip_chain_launch(self.h, stream), "chain_launch")

    def status(self):
        return load().ggml_hip_chain_status(self.h)

    def __del__(self):
        if _lib is not None and getattr(self, "h", None):
            _lib.ggml_hip_chain_destroy(self.h)
            self.h = None


def synchronize():
    check(load().ggml_hip_device_synchronize(), "device_synchronize")


class Event:
    def __init__(self):
        self.e = load().ggml_hip_event_create()

    def record(self, stream=None):
        check(load().ggml_hip_event_record(self.e, stream), "event_record")

    def elapsed_ms(self, stop):
        return load().ggml_hip_event_elapsed_ms(self.e, stop.e)

    def __del__(self):
        try:
            load().ggml_hip_event_destroy(self.e)
        except Exception:
            pass


class Graph:
    """HIP graph captured from the backend stream."""

    def __init__(self, stream=None):
        self.stream = stream
        self.g = ctypes.c_void_p()

    def __enter__(self):
        check(load().ggml_hip_graph_begin(self.stream), "graph_begin")
        return self

    def __exit__(self, *exc):
        check(load().ggml_hip_graph_end(self.stream, ctypes.byref(self.g)), "graph_end")

    def launch(self):
        check(load().ggml_hip_graph_launch(self.g, self.stream), "graph_launch")

    def __del__(self):
        try:
            if self.g:
                load().ggml_hip_graph_destroy(self.g)
        except Exception:
            pass


# ---------------------------------------------------------------------------------------------
# ggml_tensor mirror (ggml.h:378-414) for driving the tensor ABI from tests

GGML_TYPE_F32, GGML_TYPE_Q4_0 = 0, 2
GGML_BACKEND_CPU, GGML_BACKEND_GPU, GGML_BACKEND_GPU_SPLIT = 0, 10, 20
GGML_OP_MUL_MAT = 32
GGML_TASK_INIT, GGML_TASK_COMPUTE, GGML_TASK_FINALIZE = 0, 1, 2


class GgmlTensor(ctypes.Structure):
    pass


GgmlTensor._fields_ = [
    ("type", ctypes.c_int), ("backend", ctypes.c_int), ("n_dims", ctypes.c_int),
    ("ne", ctypes.c_int64 * 4), ("nb", ctypes.c_size_t * 4), ("op", ctypes.c_int), ("is_param", ctypes.c_bool),
    ("grad", ctypes.POINTER(GgmlTensor)), ("src0", ctypes.POINTER(GgmlTensor)), ("src1", ctypes.POINTER(GgmlTensor)),
    ("opt", ctypes.POINTER(GgmlTensor) * 4), ("n_tasks", ctypes.c_int), ("perf_runs", ctypes.c_int),
    ("perf_cycles", ctypes.c_int64), ("perf_time_us", ctypes.c_int64), ("data", ctypes.c_void_p),
    ("name", ctypes.c_char * 48), ("extra", ctypes.c_void_p), ("padding", ctypes.c_char * 4),
]
assert ctypes.sizeof(GgmlTensor) == 240


class GgmlComputeParams(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("ith", ctypes.c_int), ("nth", ctypes.c_int),
                ("wsize", ctypes.c_size_t), ("wdata", ctypes.c_void_p)]


def make_tensor(gtype, ne, data=None, backend=GGML_BACKEND_CPU):
    """2-D contiguous tensor {ne0, ne1} (ggml order); data: numpy array kept alive by the caller."""
    t = GgmlTensor()
    t.type = gtype
    t.backend = backend
    t.n_dims = 2
    ne = list(ne) + [1] * (4 - len(ne))
    for i in range(4):
        t.ne[i] = ne[i]
    if gtype == GGML_TYPE_Q4_0:
        t.nb[0] = 18
        t.nb[1] = 18 * ne[0] // 32
    else:
        t.nb[0] = 4
        t.nb[1] = 4 * ne[0]
    t.nb[2] = t.nb[1] * ne[1]
    t.nb[3] = t.nb[2] * ne[2]
    if data is not None:
        t.data = data.ctypes.data_as(ctypes.c_void_p).value
    return t
