"""Host logic of N-token chains (ggml_hip_chain_create_n): which task's GEMM epilogue writes which consumer's
x image.  ggml_hip_debug_chain_links runs the planner alone (no device, pointers never dereferenced), so these
run on the CPU; tests/test_gpu_prefill_chain.py runs the same shapes on the GPU, bitwise."""
import ctypes
import os

import pytest

from hip_env import LIB_PATH, ggml_hip

pytestmark = pytest.mark.skipif(not os.path.exists(LIB_PATH), reason="libggml_hip.so not built")

BASE = 1 << 32          # fake device addresses, far apart


class Alloc:
    def __init__(self):
        self.next = BASE

    def __call__(self, nbytes):
        p = self.next
        self.next += (nbytes + 4095) // 4096 * 4096 + 4096
        return p


def links(tasks, N):
    """tasks: [(K, [M...], x_ptr, [y_ptr...])] -> (prod, share)"""
    arr = (ggml_hip.ChainTask * len(tasks))()
    for t, (K, Ms, x, ys) in enumerate(tasks):
        arr[t].nmat, arr[t].K, arr[t].x = len(Ms), K, x
        for i, M in enumerate(Ms):
            arr[t].W[i] = BASE // 2 + 64 * (8 * t + i)
            arr[t].M[i] = M
            arr[t].y[i] = ys[i]
    prod = (ctypes.c_int * len(tasks))()
    share = (ctypes.c_int * len(tasks))()
    ggml_hip.check(ggml_hip.load().ggml_hip_debug_chain_links(len(tasks), arr, N, prod, share), "chain_links")
    return list(prod), list(share)


def llama(n, N, K=4096, F=11008):
    a = Alloc()
    x0 = a(4 * K * N)
    ys = {i: a(4 * (F if i in (4, 5) else K) * N) for i in range(7)}
    tasks = []
    for li in range(n):
        tasks.append((K, [K, K, K], x0 if li == 0 else ys[6], [ys[0], ys[1], ys[2]]))
        tasks.append((K, [K], ys[0], [ys[3]]))
        tasks.append((K, [F, F], ys[3], [ys[4], ys[5]]))
        tasks.append((F, [K], ys[4], [ys[6]]))
    return tasks


def test_llama_chain_links_every_task_after_the_first():
    prod, share = links(llama(2, 512), 512)
    assert prod == [-1, 0, 1, 2, 3, 4, 5, 6]
    assert share == [-1] * 8


def test_gemv_sized_chains_have_no_links():
    prod, _ = links(llama(1, 4), 4)                  # N <= gemv_max_tokens: GEMVs, no images
    assert prod == [-1] * 4
    prod, _ = links(llama(1, 8), 8)                  # w2 (K = 11008) leaves the GEMV at N = 8; its producer not
    assert prod == [-1] * 4
    prod, _ = links(llama(1, 9), 9)
    assert prod == [-1, 0, 1, 2]


def test_shared_images_other_siblings_and_clashes():
    N = 300
    a = Alloc()
    x0 = a(4 * 1024 * N)
    y00, y01, y02 = a(4 * 4160 * N), a(4 * 1024 * N), a(4 * 192 * N)
    y1, y2, y3, y4, y5, y7 = (a(4 * m * N) for m in (2048, 64, 1024, 1024, 1024, 128))
    x6 = a(4 * 1024 * N)
    tasks = [(1024, [4160, 1024, 192], x0, [y00, y01, y02]),
             (4160, [2048], y00, [y1]),              # first consumer of (0, 0): link
             (4160, [64], y00, [y2]),                # second consumer: shares task 1's image
             (1024, [1024], y01, [y3]),              # (0, 1): task 0 already writes (0, 0)'s image
             (192, [1024], y02, [y4]),               # (0, 2): likewise
             (2048, [1024], y1, [y5]),               # link to task 1
             (1024, [1024], x6, [y1]),               # writes the first half of task 1's output
             (2048, [128], y1, [y7])]                # overlapping write in between, M != K: no link
    prod, share = links(tasks, N)
    assert prod == [-1, 0, 0, -1, -1, 1, -1, -1]
    assert share == [-1, -1, 1, -1, -1, -1, -1, -1]


def test_exact_producer_rewrite_relinks_and_prefix_does_not():
    N = 128
    a = Alloc()
    x0, ya, yb = a(4 * 4096 * N), a(4 * 4096 * N), a(4 * 4096 * N)
    tasks = [(4096, [4096], x0, [ya]),
             (4096, [4096], x0, [ya]),               # rewrites ya completely (same M): the latest writer links
             (4096, [4096], ya, [yb]),
             (2048, [64], yb, [a(4 * 64 * N)])]      # K < M of the producer: x is not its [N][K] y
    prod, _ = links(tasks, N)
    assert prod == [-1, -1, 1, -1]
