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
}  // namespace

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
