// hip-smoke: the functional analogue of the reference validator's CUDA-samples
// `vectorAdd` (validator/cuda-workload-validation.yaml:20). fp32
// C = A + B over 50,000 elements; the host verifies every element. Vectorised
// float4 loads (16 B/lane) so the kernel also reports a meaningful bandwidth figure
// when run on large buffers.
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace {
__global__ void vector_add_f32(const float* __restrict__ a, const float* __restrict__ b,
                               float* __restrict__ c, size_t n) {
  const size_t n4 = n / 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 x = reinterpret_cast<const float4*>(a)[i];
    const float4 y = reinterpret_cast<const float4*>(b)[i];
    reinterpret_cast<float4*>(c)[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
  // tail
  const size_t t = n4 * 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) c[t] = a[t] + b[t];
}
}  // namespace

extern "C" int amdgo_vector_add_f32(const float* a, const float* b, float* c, size_t n,
                                    void* stream) {
  size_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(vector_add_f32, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     a, b, c, n);
  return (int)hipGetLastError();
}
