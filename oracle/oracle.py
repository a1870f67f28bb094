"""ctypes binding of oracle/liboracle_q4_0.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference q4_0 x q8_0 mul_mat path (see
q4_0_oracle.h for the function -> reference ggml.c file:line map).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / the CPU baseline; the product library
(llama.cpp-q_4_0_amd/, libggml_hip.so) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_q4_0.so")
REF_DIR = os.path.join(HERE, "_ref")

QK = 32
Q4_0_BYTES = 18
Q8_0_BYTES = 34

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle_q4_0.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, ip, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.oracle_fp32_to_fp16.argtypes = [fp]
        L.oracle_fp32_to_fp16.restype = ctypes.c_uint16
        L.oracle_fp16_to_fp32.argtypes = [ctypes.c_uint16]
        L.oracle_fp16_to_fp32.restype = fp
        for name in ("oracle_quantize_row_q4_0", "oracle_dequantize_row_q4_0",
                     "oracle_quantize_row_q8_0_avx2", "oracle_quantize_row_q8_0_ref",
                     "oracle_quantize_row_q8_0_avx2_simd"):
            getattr(L, name).argtypes = [vp, vp, ip]
            getattr(L, name).restype = None
        L.oracle_quantize_q4_0.argtypes = [vp, vp, ip, ip, vp]
        L.oracle_quantize_q4_0.restype = ctypes.c_size_t
        for name in ("oracle_vec_dot_q4_0_q8_0_avx2", "oracle_vec_dot_q4_0_q8_0_scalar",
                     "oracle_vec_dot_q4_0_q8_0_avx2_simd"):
            getattr(L, name).argtypes = [ip, vp, vp]
            getattr(L, name).restype = fp
        L.oracle_have_avx2.restype = ip
        L.oracle_mul_mat_q4_0_f32.argtypes = [vp, ip, ip, vp, ip, vp, ip, ip, ip]
        L.oracle_mul_mat_q4_0_f32.restype = ip
        L.oracle_fill_gaussian.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint64, fp, fp]
        L.oracle_fill_gaussian.restype = None
        L.oracle_pool_shutdown.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gaussian(n, seed, mean=0.0, std=1.0):
    out = np.empty(n, dtype=np.float32)
    lib().oracle_fill_gaussian(_p(out), n, seed, mean, std)
    return out


def quantize_q4_0(w):
    """w: float32 [M, K] -> uint8 [M, K/32*18] (ggml_quantize_q4_0, A3)."""
    w = np.ascontiguousarray(w, dtype=np.float32)
    M, K = w.shape
    out = np.empty((M, K // QK * Q4_0_BYTES), dtype=np.uint8)
    hist = np.zeros(16, dtype=np.int64)
    lib().oracle_quantize_q4_0(_p(w), _p(out), M * K, K, _p(hist))
    return out, hist


def dequantize_q4_0(wq, K):
    wq = np.ascontiguousarray(wq, dtype=np.uint8)
    rows = wq.size // (K // QK * Q4_0_BYTES)
    out = np.empty((rows, K), dtype=np.float32)
    lib().oracle_dequantize_row_q4_0(_p(wq), _p(out), rows * K)
    return out


def quantize_q8_0(x, mode="avx2"):
    """x: float32 [N, K] -> uint8 [N, K/32*34].  mode: avx2 | ref | avx2_simd."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    if x.ndim == 1:
        x = x[None, :]
    N, K = x.shape
    out = np.empty((N, K // QK * Q8_0_BYTES), dtype=np.uint8)
    fn = {"avx2": lib().oracle_quantize_row_q8_0_avx2,
          "ref": lib().oracle_quantize_row_q8_0_ref,
          "avx2_simd": lib().oracle_quantize_row_q8_0_avx2_simd}[mode]
    fn(_p(x), _p(out), N * K)
    return out


def vec_dot(K, wrow, xrow, mode="avx2"):
    fn = {"avx2": lib().oracle_vec_dot_q4_0_q8_0_avx2,
          "scalar": lib().oracle_vec_dot_q4_0_q8_0_scalar,
          "avx2_simd": lib().oracle_vec_dot_q4_0_q8_0_avx2_simd}[mode]
    wrow = np.ascontiguousarray(wrow, dtype=np.uint8)
    xrow = np.ascontiguousarray(xrow, dtype=np.uint8)
    return fn(K, _p(wrow), _p(xrow))


def mul_mat(wq, K, x, nthreads=1, mode="avx2", pool=False):
    """A10: wq uint8 [M, K/32*18], x f32 [N, K] -> y f32 [N, M]."""
    wq = np.ascontiguousarray(wq, dtype=np.uint8)
    x = np.ascontiguousarray(x, dtype=np.float32)
    if x.ndim == 1:
        x = x[None, :]
    N = x.shape[0]
    M = wq.size // (K // QK * Q4_0_BYTES)
    y = np.empty((N, M), dtype=np.float32)
    rc = lib().oracle_mul_mat_q4_0_f32(_p(wq), K, M, _p(x), N, _p(y), nthreads,
                                       0 if mode == "avx2" else 1, 1 if pool else 0)
    if rc != 0:
        raise RuntimeError(f"oracle_mul_mat_q4_0_f32 failed: {rc}")
    return y
