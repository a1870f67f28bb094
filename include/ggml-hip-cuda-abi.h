/*
 * ggml-hip-cuda-abi.h — the reference's ggml-cuda.h function set (ggml-cuda.h:15-36 of
 * Fcucgvhhhvjv/llama.cpp-q_4_0), exported by libggml_hip_cuda.so as thin aliases of the
 * ggml_hip_* entry points in ggml-hip.h.
 *
 * Purpose: an UNMODIFIED reference tree built with -DGGML_USE_CUBLAS (ggml.c:233-234, 4282-4283,
 * 15645-15652, 17283-17288; llama.cpp's offload calls) links against libggml_hip_cuda.so instead
 * of the CUDA backend and runs its q4_0 mul_mats on the MI355X ("optional
 * GGML_HIP_CUDA_ABI alias shim").  Same names, same argument meaning, same error behaviour.
 */
#ifndef GGML_HIP_CUDA_ABI_H
#define GGML_HIP_CUDA_ABI_H

#include "ggml-hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GGML_CUDA_MAX_DEVICES GGML_HIP_MAX_DEVICES   /* ggml-cuda.h:9 */

void   ggml_init_cublas(void);                                           /* ggml-cuda.h:15 */
void   ggml_cuda_set_tensor_split(const float *tensor_split);            /* ggml-cuda.h:16 */
void   ggml_cuda_mul(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                     struct ggml_tensor *dst);                           /* ggml-cuda.h:18 */
bool   ggml_cuda_can_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                             struct ggml_tensor *dst);                   /* ggml-cuda.h:19 */
size_t ggml_cuda_mul_mat_get_wsize(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                                   struct ggml_tensor *dst);             /* ggml-cuda.h:20 */
void   ggml_cuda_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                         struct ggml_tensor *dst, void *wdata, size_t wsize);   /* ggml-cuda.h:21 */
void  *ggml_cuda_host_malloc(size_t size);                               /* ggml-cuda.h:24 */
void   ggml_cuda_host_free(void *ptr);                                   /* ggml-cuda.h:25 */
void   ggml_cuda_transform_tensor(void *data, struct ggml_tensor *tensor);        /* ggml-cuda.h:27 */
void   ggml_cuda_free_data(struct ggml_tensor *tensor);                  /* ggml-cuda.h:29 */
void   ggml_cuda_assign_buffers(struct ggml_tensor *tensor);             /* ggml-cuda.h:30 */
void   ggml_cuda_assign_buffers_no_scratch(struct ggml_tensor *tensor);  /* ggml-cuda.h:31 */
void   ggml_cuda_assign_buffers_force_inplace(struct ggml_tensor *tensor);        /* ggml-cuda.h:32 */
void   ggml_cuda_set_main_device(int main_device);                       /* ggml-cuda.h:33 */
void   ggml_cuda_set_scratch_size(size_t scratch_size);                  /* ggml-cuda.h:34 */
void   ggml_cuda_free_scratch(void);                                     /* ggml-cuda.h:35 */
bool   ggml_cuda_compute_forward(struct ggml_compute_params *params, struct ggml_tensor *tensor); /* :36 */

#ifdef __cplusplus
}
#endif

#endif /* GGML_HIP_CUDA_ABI_H */
