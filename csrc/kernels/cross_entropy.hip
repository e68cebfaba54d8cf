// Fused softmax cross-entropy for gfx950 (LM heads: GPT-2 vocab 50304, Llama-3 vocab 128256).
//
// Forward: one workgroup per row, a single streaming pass with an online (max, sum-exp) merge per
// lane -> wave -> workgroup, so the [tokens, vocab] logits are read exactly once; writes the
// per-row loss and log-sum-exp.  Backward: one more read of the logits, writes
// (softmax - onehot) * g, optionally in place over the logits (the logits are dead after the loss,
// which saves a [tokens, vocab] allocation: 0.8 GB at GPT-2 1.3B's 8192 tokens/GPU).
#include "common.h"

using namespace pdt;

namespace {
constexpr int NT = 256;
constexpr int NW = NT / 64;

template <typename T>
__global__ __launch_bounds__(NT) void ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                    float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                    int64_t ldl, int ignore_index) {
  __shared__ float sm[NW], ss[NW];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ldl;
  float m = -INFINITY, s = 0.f;
  const bool vec = (V % 8 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
  if (vec) {
    for (int c = threadIdx.x * 8; c < V; c += NT * 8) {
      float v[8];
      Vec8<T>::load(x + c, v);
      float bm = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) bm = fmaxf(bm, v[k]);
      if (bm == -INFINITY) continue;  // fully masked slab
      float bs = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) bs += __expf(v[k] - bm);
      lse_merge(m, s, bm, bs);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += NT) lse_merge(m, s, to_f<T>(x[c]), 1.f);
  }
  wave_lse(m, s);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) lse_merge(M, S, sm[i], ss[i]);
    const float lse = M + __logf(S);
    const int64_t t = target[row];
    lse_out[row] = lse;
    loss[row] = (t == ignore_index || t < 0 || t >= V) ? 0.f : lse - to_f<T>(x[t]);
  }
}

// grad[row, j] = (exp(x - lse) - [j == t]) * g_row ;  g_row = (grow ? grow[row] : 1) * (gscale ? *gscale : 1)
template <typename T>
__global__ __launch_bounds__(NT) void ce_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ target,
                                                    const float* __restrict__ lse_in, const float* __restrict__ grow,
                                                    const float* __restrict__ gscale, T* __restrict__ grad, int V,
                                                    int64_t ldl, int64_t ldg, int ignore_index) {
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ldl;
  T* g = grad + row * ldg;
  const int64_t t = target[row];
  float gr = (grow ? grow[row] : 1.f) * (gscale ? *gscale : 1.f);
  if (t == ignore_index) gr = 0.f;
  const float lse = lse_in[row];
  const bool vec = (V % 8 == 0) && (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g)) & 15) == 0);
  if (vec) {
    for (int c = threadIdx.x * 8; c < V; c += NT * 8) {
      float v[8];
      Vec8<T>::load(x + c, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (__expf(v[k] - lse) - (c + k == t ? 1.f : 0.f)) * gr;
      Vec8<T>::store(g + c, v);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += NT) g[c] = from_f<T>((__expf(to_f<T>(x[c]) - lse) - (c == t ? 1.f : 0.f)) * gr);
  }
}
// Forward with the gradient (the LM heads' case: the logits are dead after the loss and its upstream gradient is
// a scalar): one workgroup per row holds the whole row in registers (NTH threads x IT 16-byte slabs), so the
// logits are read ONCE and the gradient (softmax - onehot) * scale (scale = *inv_count for a mean, 1 for a sum)
// is written over them in the same pass -- the separate backward's second read of the [tokens, vocab] logits and
// its launch disappear (ce_scale_kernel applies a non-unit upstream gradient later).  bf16 (kept packed in
// registers: IT x 4 VGPRs), V % 8 == 0, V <= NTH * 8 * IT.
template <int NTH, int IT>
__global__ __launch_bounds__(NTH) void ce_fwd_grad_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ target,
                                                          float* __restrict__ loss, float* __restrict__ lse_out,
                                                          const float* __restrict__ inv_count, int V, int64_t ldl,
                                                          int ignore_index) {
  constexpr int W = NTH / 64;
  __shared__ float sm[W], ss[W], sl;
  const int64_t row = blockIdx.x;
  bf16_t* x = logits + row * ldl;
  uint4 raw[IT];
  float m = -INFINITY, s = 0.f;
  auto unpack = [](const uint4& r, float (&f)[8]) {
    const uint32_t w4[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = __uint_as_float(w4[k] << 16);
      f[2 * k + 1] = __uint_as_float(w4[k] & 0xffff0000u);
    }
  };
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (it * NTH + (int)threadIdx.x) * 8;
    if (c < V) raw[it] = *reinterpret_cast<const uint4*>(x + c);
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (it * NTH + (int)threadIdx.x) * 8;
    if (c < V) {
      float v[8];
      unpack(raw[it], v);
      float bm = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) bm = fmaxf(bm, v[k]);
      if (bm != -INFINITY) {
        float bs = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) bs += __expf(v[k] - bm);
        lse_merge(m, s, bm, bs);
      }
    }
  }
  wave_lse(m, s);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  const int64_t t = target[row];
  const bool ign = t == ignore_index || t < 0 || t >= V;
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
#pragma unroll
    for (int i = 1; i < W; ++i) lse_merge(M, S, sm[i], ss[i]);
    const float lse = M + __logf(S);
    sl = lse;
    lse_out[row] = lse;
    loss[row] = ign ? 0.f : lse - bf2f(x[t]);   // (read before any thread's gradient store: the barrier below)
  }
  __syncthreads();
  const float lse = sl;
  const float gr = ign ? 0.f : (inv_count ? *inv_count : 1.f);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = (it * NTH + (int)threadIdx.x) * 8;
    if (c < V) {
      float v[8];
      unpack(raw[it], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (__expf(v[k] - lse) - (c + k == t ? 1.f : 0.f)) * gr;
      Vec8<bf16_t>::store(x + c, v);
    }
  }
}

// g *= *scale unless *scale == 1 (every block reads the scalar and leaves at once in the common case)
template <typename T>
__global__ __launch_bounds__(256) void ce_scale_kernel(T* __restrict__ g, const float* __restrict__ scale, int64_t rows,
                                                       int V, int64_t ld) {
  const float sc = *scale;
  if (sc == 1.f) return;
  const int64_t n8 = rows * (V / 8);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n8; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / (V / 8);
    const int c = (int)(e - r * (V / 8)) * 8;
    float v[8];
    Vec8<T>::load(g + r * ld + c, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= sc;
    Vec8<T>::store(g + r * ld + c, v);
  }
}
}  // namespace

// Forward + gradient in one pass (see ce_fwd_grad_kernel); 0 or a hipError_t, -1 when the shape does not qualify
// (the caller then runs pdt_ce_fwd / pdt_ce_bwd).
PDT_API int pdt_ce_fwd_grad(void* logits, const int64_t* target, float* loss, float* lse, const float* inv_count,
                            int64_t rows, int V, int64_t ldl, int dt, int ignore_index, hipStream_t st) {
  if (rows <= 0) return 0;
  // up to 65,536 columns (GPT-2's 50,304; 16 slabs of 1,024 threads for Llama-3's 128,256 spilled at 128 VGPRs).
  // 1,024 threads x 8 slabs (106 VGPRs: 16 waves per CU) or 512 x 16 (180 VGPRs: 8 waves); PDT_CE_FUSED_NTH
  static const int nth = [] { const char* e = getenv("PDT_CE_FUSED_NTH"); return e ? atoi(e) : 1024; }();
  if (V % 8 || ldl % 8 || (reinterpret_cast<uintptr_t>(logits) & 15) || V > 512 * 8 * 16) return -1;
  if (dt != kBF16) return -1;   // fp32 logits: 2x the registers per element; the two-pass path
  if (nth == 512)
    ce_fwd_grad_kernel<512, 16><<<rows, 512, 0, st>>>((bf16_t*)logits, target, loss, lse, inv_count, V, ldl,
                                                       ignore_index);
  else
    ce_fwd_grad_kernel<1024, 8><<<rows, 1024, 0, st>>>((bf16_t*)logits, target, loss, lse, inv_count, V, ldl,
                                                        ignore_index);
  return (int)hipGetLastError();
}

PDT_API int pdt_ce_scale(void* grad, const float* scale, int64_t rows, int V, int64_t ld, int dt, hipStream_t st) {
  if (rows <= 0) return 0;
  if (V % 8 || ld % 8) return (int)hipErrorInvalidValue;
  const int grid = grid_for(rows * (V / 8), 256, 256 * 8);
  if (dt == kBF16) ce_scale_kernel<bf16_t><<<grid, 256, 0, st>>>((bf16_t*)grad, scale, rows, V, ld);
  else ce_scale_kernel<float><<<grid, 256, 0, st>>>((float*)grad, scale, rows, V, ld);
  return (int)hipGetLastError();
}

PDT_API int pdt_ce_fwd(const void* logits, const int64_t* target, float* loss, float* lse, int64_t rows, int V,
                       int64_t ldl, int dt, int ignore_index, hipStream_t st) {
  if (rows <= 0) return 0;
  if (dt == kBF16)
    ce_fwd_kernel<bf16_t><<<rows, NT, 0, st>>>((const bf16_t*)logits, target, loss, lse, V, ldl, ignore_index);
  else
    ce_fwd_kernel<float><<<rows, NT, 0, st>>>((const float*)logits, target, loss, lse, V, ldl, ignore_index);
  return (int)hipGetLastError();
}

PDT_API int pdt_ce_bwd(const void* logits, const int64_t* target, const float* lse, const float* grow,
                       const float* gscale, void* grad, int64_t rows, int V, int64_t ldl, int64_t ldg, int dt,
                       int ignore_index, hipStream_t st) {
  if (rows <= 0) return 0;
  if (dt == kBF16)
    ce_bwd_kernel<bf16_t><<<rows, NT, 0, st>>>((const bf16_t*)logits, target, lse, grow, gscale, (bf16_t*)grad, V, ldl,
                                               ldg, ignore_index);
  else
    ce_bwd_kernel<float><<<rows, NT, 0, st>>>((const float*)logits, target, lse, grow, gscale, (float*)grad, V, ldl, ldg,
                                              ignore_index);
  return (int)hipGetLastError();
}
