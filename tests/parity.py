"""Shared parity helpers (numpy): block decoding and the fp32-accumulator bound.

The north-star tolerance is "within 1e-3 relative on the fp32 accumulator".
A bare relative error is ill-conditioned where y ~ 0 (cancellation), so every
y comparison uses the per-element bound of SURVEY.md §7.3:

    |y_gpu - y_ref| <= rtol * |y_ref| + atol_blocks * S_abs,
    S_abs[n, m] = sum_b |d_w[m,b] * d_x[n,b] * sumi[n,m,b]|

and also reports max relative error over |y_ref| > 1e-3 * max|y_ref|.
"""
import numpy as np

QK = 32


def split_q4_0(wq, K):
    """uint8 [M, K/32*18] -> (d_w f32 [M, nb], w int8 [M, nb, 32]) with w = nib - 8."""
    nb = K // QK
    b = np.ascontiguousarray(wq).reshape(-1, nb, 18)
    d = b[:, :, 0:2].copy().view(np.float16)[:, :, 0].astype(np.float32)
    qs = b[:, :, 2:18]
    lo = (qs & 0x0F).astype(np.int8) - 8
    hi = (qs >> 4).astype(np.int8) - 8
    return d, np.concatenate([lo, hi], axis=2)


def split_q8_0(xq, K):
    """uint8 [N, K/32*34] -> (d_x f32 [N, nb], q int8 [N, nb, 32])."""
    nb = K // QK
    b = np.ascontiguousarray(xq).reshape(-1, nb, 34)
    d = b[:, :, 0:2].copy().view(np.float16)[:, :, 0].astype(np.float32)
    q = b[:, :, 2:34].copy().view(np.int8)
    return d, q


def block_terms(wq, xq, K):
    """(y_exact f64 [N, M], S_abs f64 [N, M]) from the integer block sums."""
    dw, w = split_q4_0(wq, K)
    dx, q = split_q8_0(xq, K)
    sumi = np.einsum("mbj,nbj->nmb", w.astype(np.int32), q.astype(np.int32))
    d = dx.astype(np.float64)[:, None, :] * dw.astype(np.float64)[None, :, :]
    t = d * sumi
    return t.sum(axis=2), np.abs(t).sum(axis=2)


def check_y(y_got, y_ref, s_abs, rtol=1e-3, atol_blocks=1e-6):
    """Assert the per-element bound; return (max_rel_well_conditioned, max_abs_err)."""
    y_got = np.asarray(y_got, dtype=np.float64)
    y_ref = np.asarray(y_ref, dtype=np.float64)
    err = np.abs(y_got - y_ref)
    bound = rtol * np.abs(y_ref) + atol_blocks * s_abs
    bad = err > bound
    if bad.any():
        i = np.argwhere(bad)[0]
        raise AssertionError(f"{bad.sum()} elements out of bound; first {tuple(i)}: got {y_got[tuple(i)]} "
                             f"ref {y_ref[tuple(i)]} bound {bound[tuple(i)]}")
    big = np.abs(y_ref) > 1e-3 * np.abs(y_ref).max()
    rel = (err[big] / np.abs(y_ref[big])).max() if big.any() else 0.0
    return float(rel), float(err.max())
