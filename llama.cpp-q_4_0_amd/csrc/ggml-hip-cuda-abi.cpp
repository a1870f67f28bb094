// libggml_hip_cuda.so: the ggml-cuda.h names (ggml-cuda.h:15-36) as aliases of ggml-hip.h, so an
// unmodified -DGGML_USE_CUBLAS ggml.c / llama.cpp links against the MI355X backend.
#include "ggml-hip-cuda-abi.h"

#include <cstdio>
#include <cstdlib>

extern "C" {

void ggml_init_cublas(void) { ggml_init_hip(); }
void ggml_cuda_set_tensor_split(const float *tensor_split) { ggml_hip_set_tensor_split(tensor_split); }
void ggml_cuda_mul(const struct ggml_tensor *src0, const struct ggml_tensor *src1, struct ggml_tensor *dst) {
    ggml_hip_mul(src0, src1, dst);
}
bool ggml_cuda_can_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1, struct ggml_tensor *dst) {
    return ggml_hip_can_mul_mat(src0, src1, dst);
}
size_t ggml_cuda_mul_mat_get_wsize(const struct ggml_tensor *src0, const struct ggml_tensor *src1,
                                   struct ggml_tensor *dst) {
    return ggml_hip_mul_mat_get_wsize(src0, src1, dst);
}
void ggml_cuda_mul_mat(const struct ggml_tensor *src0, const struct ggml_tensor *src1, struct ggml_tensor *dst,
                       void * /*wdata*/, size_t /*wsize*/) {
    ggml_hip_mul_mat(src0, src1, dst);
}
void *ggml_cuda_host_malloc(size_t size) { return ggml_hip_host_malloc(size); }
void ggml_cuda_host_free(void *ptr) { ggml_hip_host_free(ptr); }
void ggml_cuda_transform_tensor(void *data, struct ggml_tensor *tensor) { ggml_hip_transform_tensor(data, tensor); }
void ggml_cuda_free_data(struct ggml_tensor *tensor) { ggml_hip_free_data(tensor); }
void ggml_cuda_assign_buffers(struct ggml_tensor *tensor) { ggml_hip_assign_buffers(tensor); }
void ggml_cuda_assign_buffers_no_scratch(struct ggml_tensor *tensor) { ggml_hip_assign_buffers_no_scratch(tensor); }
void ggml_cuda_assign_buffers_force_inplace(struct ggml_tensor *tensor) { ggml_hip_assign_buffers_force_inplace(tensor); }
void ggml_cuda_set_main_device(int main_device) { ggml_hip_set_main_device(main_device); }
void ggml_cuda_set_scratch_size(size_t scratch_size) { ggml_hip_set_scratch_size(scratch_size); }
void ggml_cuda_free_scratch(void) { ggml_hip_free_scratch(); }
bool ggml_cuda_compute_forward(struct ggml_compute_params *params, struct ggml_tensor *tensor) {
    return ggml_hip_compute_forward(params, tensor);
}

}  // extern "C"
