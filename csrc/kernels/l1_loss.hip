// Fused L1 loss: mean |a - b| and its gradient in ONE read of a and b (the perceptual loss's feature-map terms,
// models/losses.py -- Stoke-DDP.py:224's feat_loss).  Under autocast torch runs l1_loss in fp32: every bf16 feature
// map is copied to fp32, subtracted, abs'd, reduced, and the backward re-reads the fp32 difference for its sign --
// ~4 ms of fp32 elementwise passes per SwinIR-S step at 18 x 64 x 256 x 256.  Here a grid-stride kernel reads
// 8 bf16 (16 bytes) of each operand per lane, accumulates |a - b| in fp32, and (when a gradient is wanted) writes
// sign(a - b) / n straight away; one fp32 partial per workgroup, summed in a fixed order by a second launch.
#include "common.h"

using namespace pdt;

namespace {

constexpr int NT = 256;

template <typename T>
__global__ __launch_bounds__(NT) void l1_fwd_grad_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                         T* __restrict__ g, float* __restrict__ part, int64_t n,
                                                         float inv_n) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  const int64_t n8 = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * NT) {
    float av[8], bv[8], gv[8];
    Vec8<T>::load(a + 8 * i, av);
    Vec8<T>::load(b + 8 * i, bv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = av[k] - bv[k];
      s += fabsf(d);
      gv[k] = d > 0.f ? inv_n : (d < 0.f ? -inv_n : 0.f);
    }
    if (g != nullptr) Vec8<T>::store(g + 8 * i, gv);
  }
  // the n % 8 tail (first workgroup)
  if (blockIdx.x == 0) {
    for (int64_t i = 8 * n8 + threadIdx.x; i < n; i += NT) {
      const float d = to_f<T>(a[i]) - to_f<T>(b[i]);
      s += fabsf(d);
      if (g != nullptr) g[i] = from_f<T>(d > 0.f ? inv_n : (d < 0.f ? -inv_n : 0.f));
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    part[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(NT) void l1_finish_kernel(const float* __restrict__ part, int np, float inv_n,
                                                       float* __restrict__ out) {
  __shared__ float red[NT / 64];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += NT) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    out[0] = t * inv_n;
  }
}

}  // namespace

PDT_API int pdt_l1_partials(int64_t n) { return grid_for(n / 8 + 1, NT, 256 * 8); }

// out[0] (fp32) = mean |a - b| over n elements; g (nullable, a's dtype) = sign(a - b) / n.  a, b, g share one dense
// layout, 16-byte aligned.  ws: >= pdt_l1_partials(n) floats.
PDT_API int pdt_l1_fwd_grad(const void* a, const void* b, void* g, float* out, float* ws, int64_t n, int dt,
                            hipStream_t st) {
  if (n <= 0 || (((uintptr_t)a | (uintptr_t)b | (uintptr_t)g) & 15)) return (int)hipErrorInvalidValue;
  const int grid = pdt_l1_partials(n);
  const float inv_n = 1.f / (float)n;
  if (dt == kBF16)
    l1_fwd_grad_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)a, (const bf16_t*)b, (bf16_t*)g, ws, n, inv_n);
  else if (dt == kF32)
    l1_fwd_grad_kernel<float><<<grid, NT, 0, st>>>((const float*)a, (const float*)b, (float*)g, ws, n, inv_n);
  else
    return (int)hipErrorInvalidValue;
  l1_finish_kernel<<<1, NT, 0, st>>>(ws, grid, inv_n, out);
  return (int)hipGetLastError();
}
