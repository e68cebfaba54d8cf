// Embedding backward for gfx950 with shapes that do not depend on the data: dW[idx[i], :] += dY[i, :].
//
// torch's dense embedding backward sorts the indices (rocprim radix sort) and compacts them into
// segments with a device-wide unique/partition whose output size is data dependent -- above 3,072
// indices it is the path GPT-2 / Llama take, and it is what faulted when a DDP-wrapped GPT-2 124M step
// (16,384 indices, vocab 50,257) was replayed as a HIP graph.  This kernel has no data-dependent sizes,
// no temporary storage and no host interaction, so a step that contains it captures and replays:
//   1. the fp32 accumulator [V, D] is zeroed (hipMemsetAsync),
//   2. one workgroup per 4 index rows, 16-B loads of dY, hardware fp32 atomic adds
//      (global_atomic_add_f32, -munsafe-fp-atomics) into the accumulator -- a repeated token simply
//      lands several times on the same row; out-of-range indices are skipped,
//   3. the accumulator is cast to the weight's dtype (or handed over as is for fp32 weights).
// Atomics make the summation order of a repeated token non-deterministic (last-bit differences only).
#include "common.h"

using namespace pdt;

namespace {

constexpr int EB_THREADS = 256;
constexpr int EB_ROWS = 4;   // index rows per workgroup

template <typename T>
__global__ __launch_bounds__(EB_THREADS) void embedding_bwd_atomic_kernel(const int64_t* __restrict__ idx,
                                                                          const T* __restrict__ dy,
                                                                          float* __restrict__ acc, int64_t n,
                                                                          int d, int64_t v) {
  const int64_t r0 = (int64_t)blockIdx.x * EB_ROWS;
  for (int rr = 0; rr < EB_ROWS; ++rr) {
    const int64_t r = r0 + rr;
    if (r >= n) return;
    const int64_t row = idx[r];
    if (row < 0 || row >= v) continue;
    const T* __restrict__ src = dy + r * (int64_t)d;
    float* __restrict__ dst = acc + row * (int64_t)d;
    if ((d & 7) == 0) {
      for (int c = threadIdx.x * 8; c < d; c += EB_THREADS * 8) {
        float x[8];
        Vec8<T>::load(src + c, x);
#pragma unroll
        for (int k = 0; k < 8; ++k) unsafeAtomicAdd(dst + c + k, x[k]);
      }
    } else {
      for (int c = threadIdx.x; c < d; c += EB_THREADS) unsafeAtomicAdd(dst + c, to_f<T>(src[c]));
    }
  }
}

template <typename O>
__global__ __launch_bounds__(EB_THREADS) void cast_from_f32_kernel(const float* __restrict__ s, O* __restrict__ o,
                                                                   int64_t n) {
  for (int64_t i = (blockIdx.x * (int64_t)EB_THREADS + threadIdx.x) * 8; i < n;
       i += (int64_t)gridDim.x * EB_THREADS * 8) {
    if (i + 8 <= n) {
      float x[8];
      Vec8<float>::load(s + i, x);
      Vec8<O>::store(o + i, x);
    } else {
      for (int64_t j = i; j < n; ++j) o[j] = from_f<O>(s[j]);
    }
  }
}

}  // namespace

// acc: fp32 [v, d] scratch (zeroed here); out: [v, d] in out_dtype (may alias acc when out_dtype is fp32).
PDT_API int pdt_embedding_bwd(const int64_t* idx, const void* dy, int dy_dtype, float* acc, void* out,
                              int out_dtype, int64_t n, int d, int64_t v, hipStream_t stream) {
  if (n < 0 || d <= 0 || v <= 0) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(acc, 0, (size_t)v * d * sizeof(float), stream);
  if (e != hipSuccess) return (int)e;
  if (n > 0) {
    const unsigned grid = (unsigned)((n + EB_ROWS - 1) / EB_ROWS);
    if (dy_dtype == kF32)
      embedding_bwd_atomic_kernel<float><<<grid, EB_THREADS, 0, stream>>>(idx, (const float*)dy, acc, n, d, v);
    else if (dy_dtype == kBF16)
      embedding_bwd_atomic_kernel<bf16_t><<<grid, EB_THREADS, 0, stream>>>(idx, (const bf16_t*)dy, acc, n, d, v);
    else
      return (int)hipErrorInvalidValue;
  }
  if (out_dtype != kF32 || out != (void*)acc) {
    const int64_t total = v * (int64_t)d;
    int64_t g = (total / 8 + EB_THREADS - 1) / EB_THREADS;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    if (out_dtype == kBF16)
      cast_from_f32_kernel<bf16_t><<<(unsigned)g, EB_THREADS, 0, stream>>>(acc, (bf16_t*)out, total);
    else if (out_dtype == kF32)
      cast_from_f32_kernel<float><<<(unsigned)g, EB_THREADS, 0, stream>>>(acc, (float*)out, total);
    else
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
