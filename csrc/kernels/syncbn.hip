// Synchronized BatchNorm kernels for gfx950 (ResNet configs with
// DDPConfig(convert_to_sync_batch_norm=True), Stoke-DDP.py:190-193).
//
// x is viewed as [outer, C, inner]: NCHW -> (N, C, H*W); channels_last NHWC -> (N*H*W, C, 1).
// Forward:  per-channel (sum, sumsq) of the local batch -> fp64 [2C] (partials combined in fp64 so the
//           variance does not cancel) -> ONE all-reduce of 2C+1 doubles across ranks (caller) ->
//           finalize (mean, invstd, running-stat update) -> normalise+affine (16-B vector path).
// Backward: per-channel (sum dy, sum dy*(x-mean)) -> one all-reduce -> dx elementwise.
// Semantics: torch/nn/modules/_functions.py:36-200 (SyncBatchNorm), running var unbiased.
#include "common.h"
#include <algorithm>

using namespace pdt;

namespace {
constexpr int NT = 256;

// MODE 0: (x, x^2)    MODE 1: (dy, dy * (x - mean[c]))
template <typename T, int MODE>
__device__ __forceinline__ void acc_pair(float xv, float dv, float mean, float& a, float& b) {
  if (MODE == 0) { a += xv; b += xv * xv; }
  else { a += dv; b += dv * (xv - mean); }
}

// channels-last (inner == 1): rows = outer, C contiguous.  Thread = 8 channels; the block's threads
// that share a channel group split the rows; grid = (channel-group blocks, row splits).
template <typename T, int MODE>
__global__ __launch_bounds__(NT) void stats_nhwc_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const float* __restrict__ mean, int64_t rows, int C,
                                                        int64_t rows_per, float* __restrict__ part) {
  const int groups = C / 8;
  const int tpr = groups < NT ? groups : NT;          // threads per row
  const int rl = threadIdx.x / tpr, rlanes = NT / tpr;
  const int cg = blockIdx.x * tpr + (threadIdx.x % tpr);
  const bool active = cg < groups && rl < rlanes;
  const int64_t r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  __shared__ float sa[NT * 8], sb[NT * 8];
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0}, mu[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (active) {
    if (MODE == 1) Vec8<float>::load(mean + cg * 8, mu);
    for (int64_t r = r0 + rl; r < r1; r += rlanes) {
      float xv[8], dv[8];
      Vec8<T>::load(x + r * C + cg * 8, xv);
      if (MODE == 1) Vec8<T>::load(dy + r * C + cg * 8, dv);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc_pair<T, MODE>(xv[k], MODE == 1 ? dv[k] : 0.f, mu[k], a[k], b[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { sa[threadIdx.x * 8 + k] = a[k]; sb[threadIdx.x * 8 + k] = b[k]; }
  __syncthreads();
  if (rl == 0 && cg < groups) {
    for (int j = 1; j < rlanes; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) { a[k] += sa[(threadIdx.x + j * tpr) * 8 + k]; b[k] += sb[(threadIdx.x + j * tpr) * 8 + k]; }
    float* pa = part + (int64_t)blockIdx.y * 2 * C;
#pragma unroll
    for (int k = 0; k < 8; ++k) { pa[cg * 8 + k] = a[k]; pa[C + cg * 8 + k] = b[k]; }
  }
}

// NCHW (inner > 1): block = (channel, split of the outer index)
template <typename T, int MODE>
__global__ __launch_bounds__(NT) void stats_nchw_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const float* __restrict__ mean, int64_t outer, int C,
                                                        int64_t inner, int64_t outer_per, float* __restrict__ part) {
  __shared__ float red[NT / 64];
  const int c = blockIdx.x;
  const int64_t o0 = blockIdx.y * outer_per, o1 = min(outer, o0 + outer_per);
  const float mu = MODE == 1 ? mean[c] : 0.f;
  float a = 0.f, b = 0.f;
  const bool vec = (inner % 8) == 0;
  for (int64_t o = o0; o < o1; ++o) {
    const T* px = x + (o * C + c) * inner;
    const T* pd = MODE == 1 ? dy + (o * C + c) * inner : nullptr;
    if (vec) {
      for (int64_t i = threadIdx.x * 8; i < inner; i += NT * 8) {
        float xv[8], dv[8];
        Vec8<T>::load(px + i, xv);
        if (MODE == 1) Vec8<T>::load(pd + i, dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc_pair<T, MODE>(xv[k], MODE == 1 ? dv[k] : 0.f, mu, a, b);
      }
    } else {
      for (int64_t i = threadIdx.x; i < inner; i += NT)
        acc_pair<T, MODE>(to_f<T>(px[i]), MODE == 1 ? to_f<T>(pd[i]) : 0.f, mu, a, b);
    }
  }
  a = block_sum<NT / 64>(a, red);
  b = block_sum<NT / 64>(b, red);
  if (threadIdx.x == 0) {
    float* pa = part + (int64_t)blockIdx.y * 2 * C;
    pa[c] = a;
    pa[C + c] = b;
  }
}

// fold [splits, 2C] fp32 partials into out[2C] fp64
__global__ void combine_kernel(const float* __restrict__ part, int splits, int C, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * C) return;
  double s = 0.0;
  for (int j = 0; j < splits; ++j) s += (double)part[(int64_t)j * 2 * C + i];
  out[i] = s;
}

// stats[0:2C] = global (sum, sumsq); stats[2C] = global element count per channel (device-side, so
// ranks may hold different batch sizes without a host sync)
__global__ void finalize_kernel(const double* __restrict__ stats, int C, float eps, float momentum,
                                float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ rmean,
                                float* __restrict__ rvar) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double count = stats[2 * C];
  const double mu = stats[c] / count;
  double var = stats[C + c] / count - mu * mu;
  if (var < 0) var = 0;
  mean[c] = (float)mu;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    const double unbiased = count > 1 ? var * count / (count - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mu);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
}

// y = (x - mean) * invstd * w + b       (MODE 0)
// dx = (dy - mdy - (x-mean) * invstd^2 * mdyx) * invstd * w   (MODE 1; mdy, mdyx = global means)
template <typename T, typename W, int MODE>
__global__ __launch_bounds__(NT) void elemt_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                   T* __restrict__ out, const float* __restrict__ mean,
                                                   const float* __restrict__ invstd, const W* __restrict__ w,
                                                   const W* __restrict__ b, const double* __restrict__ gsum,
                                                   const double* __restrict__ count_ptr, int64_t total, int C,
                                                   int64_t inner) {
  const double inv_count = MODE == 1 ? 1.0 / count_ptr[0] : 0.0;
  const bool nhwc = inner == 1;
  const bool vec = nhwc ? (C % 8 == 0) : (inner % 8 == 0);
  if (vec) {
    for (int64_t i = (blockIdx.x * (int64_t)NT + threadIdx.x) * 8; i < total; i += (int64_t)gridDim.x * NT * 8) {
      float xv[8], dv[8], o[8];
      Vec8<T>::load(x + i, xv);
      if (MODE == 1) Vec8<T>::load(dy + i, dv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = nhwc ? (int)((i + k) % C) : (int)(((i) / inner) % C);
        const float mu = mean[c], is = invstd[c];
        const float wc = w ? to_f<W>(w[c]) : 1.f;
        if (MODE == 0) {
          o[k] = (xv[k] - mu) * is * wc + (b ? to_f<W>(b[c]) : 0.f);
        } else {
          const float mdy = (float)(gsum[c] * inv_count), mdyx = (float)(gsum[C + c] * inv_count);
          o[k] = (dv[k] - mdy - (xv[k] - mu) * is * is * mdyx) * is * wc;
        }
      }
      Vec8<T>::store(out + i, o);
    }
  } else {
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
      const int c = nhwc ? (int)(i % C) : (int)((i / inner) % C);
      const float mu = mean[c], is = invstd[c], xv = to_f<T>(x[i]);
      const float wc = w ? to_f<W>(w[c]) : 1.f;
      float o;
      if (MODE == 0) {
        o = (xv - mu) * is * wc + (b ? to_f<W>(b[c]) : 0.f);
      } else {
        const float mdy = (float)(gsum[c] * inv_count), mdyx = (float)(gsum[C + c] * inv_count);
        o = (to_f<T>(dy[i]) - mdy - (xv - mu) * is * is * mdyx) * is * wc;
      }
      out[i] = from_f<T>(o);
    }
  }
}

template <typename T, int MODE>
int launch_stats(const void* x, const void* dy, const float* mean, int64_t outer, int C, int64_t inner, float* ws,
                 double* out, hipStream_t st) {
  int splits;
  if (inner == 1 && C % 8 == 0) {
    const int groups = C / 8;
    const int tpr = groups < NT ? groups : NT;
    const int gx = (groups + tpr - 1) / tpr;
    splits = (int)std::min<int64_t>((int64_t)(1024 / gx > 1 ? 1024 / gx : 1), (int64_t)(outer / 64 > 1 ? outer / 64 : 1));
    const int64_t rows_per = (outer + splits - 1) / splits;
    splits = (int)((outer + rows_per - 1) / rows_per);
    stats_nhwc_kernel<T, MODE><<<dim3(gx, splits), NT, 0, st>>>((const T*)x, (const T*)dy, mean, outer, C, rows_per, ws);
  } else {
    // treat NHWC with C % 8 != 0 as NCHW with inner=1 (scalar path)
    splits = (int)std::min<int64_t>((int64_t)(2048 / C > 1 ? 2048 / C : 1), outer);
    const int64_t per = (outer + splits - 1) / splits;
    splits = (int)((outer + per - 1) / per);
    stats_nchw_kernel<T, MODE><<<dim3(C, splits), NT, 0, st>>>((const T*)x, (const T*)dy, mean, outer, C, inner, per, ws);
  }
  combine_kernel<<<(2 * C + 255) / 256, 256, 0, st>>>(ws, splits, C, out);
  return (int)hipGetLastError();
}

}  // namespace

// workspace for stats / bwd_reduce: 2 * C * 1024 floats is always enough
PDT_API int pdt_syncbn_stats(const void* x, int64_t outer, int C, int64_t inner, int dt, float* ws, double* out,
                             hipStream_t st) {
  if (dt == kBF16) return launch_stats<bf16_t, 0>(x, nullptr, nullptr, outer, C, inner, ws, out, st);
  return launch_stats<float, 0>(x, nullptr, nullptr, outer, C, inner, ws, out, st);
}

PDT_API int pdt_syncbn_finalize(const double* stats, int C, float eps, float momentum, float* mean, float* invstd,
                                float* rmean, float* rvar, hipStream_t st) {
  finalize_kernel<<<(C + 255) / 256, 256, 0, st>>>(stats, C, eps, momentum, mean, invstd, rmean, rvar);
  return (int)hipGetLastError();
}

PDT_API int pdt_syncbn_elemt(const void* x, void* y, const float* mean, const float* invstd, const void* w,
                             const void* b, int64_t outer, int C, int64_t inner, int dt, int wdt, hipStream_t st) {
  const int64_t total = outer * C * inner;
  const int grid = grid_for(total / 8 + 1, NT, 256 * 16);
#define PDT_L(T, W) elemt_kernel<T, W, 0><<<grid, NT, 0, st>>>((const T*)x, nullptr, (T*)y, mean, invstd, (const W*)w, \
                                                             (const W*)b, nullptr, nullptr, total, C, inner)
  if (dt == kBF16) { if (wdt == kBF16) PDT_L(bf16_t, bf16_t); else PDT_L(bf16_t, float); }
  else { if (wdt == kBF16) PDT_L(float, bf16_t); else PDT_L(float, float); }
#undef PDT_L
  return (int)hipGetLastError();
}

PDT_API int pdt_syncbn_bwd_reduce(const void* dy, const void* x, const float* mean, int64_t outer, int C,
                                  int64_t inner, int dt, float* ws, double* out, hipStream_t st) {
  if (dt == kBF16) return launch_stats<bf16_t, 1>(x, dy, mean, outer, C, inner, ws, out, st);
  return launch_stats<float, 1>(x, dy, mean, outer, C, inner, ws, out, st);
}

PDT_API int pdt_syncbn_bwd_elemt(const void* dy, const void* x, void* dx, const float* mean, const float* invstd,
                                 const void* w, const double* gsum, const double* count, int64_t outer, int C,
                                 int64_t inner, int dt, int wdt, hipStream_t st) {
  const int64_t total = outer * C * inner;
  const int grid = grid_for(total / 8 + 1, NT, 256 * 16);
#define PDT_L(T, W) elemt_kernel<T, W, 1><<<grid, NT, 0, st>>>((const T*)x, (const T*)dy, (T*)dx, mean, invstd, \
                                                             (const W*)w, nullptr, gsum, count, total, C, inner)
  if (dt == kBF16) { if (wdt == kBF16) PDT_L(bf16_t, bf16_t); else PDT_L(bf16_t, float); }
  else { if (wdt == kBF16) PDT_L(float, bf16_t); else PDT_L(float, float); }
#undef PDT_L
  return (int)hipGetLastError();
}
