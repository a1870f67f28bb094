// The empty kernel tools/aql_dispatch_cost.hip dispatches through its own AQL queue (same argument list as its
// hipLaunchKernelGGL twin).  A bare code object ELF (not an offload bundle): see tools/aql_dispatch_cost.hip
#include <hip/hip_runtime.h>

extern "C" __global__ void k_empty_aql(const float *x, const unsigned char *w0, const unsigned char *w1,
                                       const unsigned char *w2, int a, int b, int c, int d, int e, int f, float *y, long ldy) {
    if (a == -12345 && threadIdx.x == 0) y[ldy] = x[0] + (float)(w0[0] + w1[0] + w2[0] + b + c + d + e + f);
}
