// Multi-tensor optimizer-side kernels for gfx950: fused AdamW, fused L2-norm / non-finite check,
// clip-coefficient, and in-place scale.  One launch covers every tensor in a list.
//
// Replaces the per-parameter foreach chain torch runs for the reference's AdamW + clip_grad_norm_
// (reference: Stoke-DDP.py:226-235 AdamW(lr, betas=(0.9,0.99), eps, wd), Stoke-DDP.py:253
// ClipGradNormConfig(max_norm, norm_type=2); Fairscale-DDP.py:78-86) -- the math order follows
// torch/optim/adam.py:419-547 / torch's fused AdamW so checkpoints interoperate.
//
// Tensor lists are described by a device int64 table, 6 words per tensor:
//   [ptr0, ptr1, ptr2, ptr3, ptr4, numel]
// and a block table (int32 pairs: tensor index, chunk index).  The engines keep parameters in flat
// buffers, so the common case is a 1-entry table whose chunks tile the whole shard; the table form
// is what lets a user hand the optimizer arbitrary parameter lists and still get ONE launch.
//
// Sync-free step: the grad multiplier (1/loss_scale * clip coefficient) and the found_inf flag live in
// device memory, produced by pdt_l2norm_* + pdt_clip_coef, so no host round trip sits between
// backward and the optimizer.
#include "common.h"

using namespace pdt;

namespace {

constexpr int MT_META = 6;
constexpr int MT_THREADS = 256;

struct AdamHyper {
  float lr, beta1, beta2, eps, wd;
  float step_size;  // lr / (1 - beta1^t)
  float bc2_sqrt;   // sqrt(1 - beta2^t)
  int decoupled;    // 1 = AdamW, 0 = Adam (L2 added to the gradient)
};

template <typename G>
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamHyper& h) {
  if (h.decoupled) {
    p *= 1.f - h.lr * h.wd;
  } else if (h.wd != 0.f) {
    g += h.wd * p;
  }
  m = h.beta1 * m + (1.f - h.beta1) * g;
  v = h.beta2 * v + (1.f - h.beta2) * g * g;
  const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
  p -= h.step_size * m / denom;
}

// One block processes one chunk of one tensor; 4 elements per thread per iteration (16-B loads).
template <typename G>
__global__ __launch_bounds__(MT_THREADS) void adamw_mt_kernel(
    const int64_t* __restrict__ meta, const int* __restrict__ blk, int chunk, AdamHyper h,
    const float* __restrict__ gscale, const int* __restrict__ found_inf, const float* __restrict__ dstep) {
  if (found_inf != nullptr && *found_inf != 0) return;  // GradScaler semantics: skip the step
  const float gs = gscale ? *gscale : 1.f;
  if (dstep != nullptr) {   // graph-capturable: the step count lives on the device, bias corrections here
    const float t = *dstep;
    h.step_size = h.lr / (1.f - powf(h.beta1, t));
    h.bc2_sqrt = sqrtf(1.f - powf(h.beta2, t));
  }
  const int t = blk[2 * blockIdx.x], c = blk[2 * blockIdx.x + 1];
  const int64_t* mt = meta + (int64_t)t * MT_META;
  float* __restrict__ P = reinterpret_cast<float*>(mt[0]);
  const G* __restrict__ Gr = reinterpret_cast<const G*>(mt[1]);
  float* __restrict__ M = reinterpret_cast<float*>(mt[2]);
  float* __restrict__ V = reinterpret_cast<float*>(mt[3]);
  bf16_t* __restrict__ O = reinterpret_cast<bf16_t*>(mt[4]);
  const int64_t n = mt[5];
  const int64_t beg = (int64_t)c * chunk;
  const int64_t end = beg + chunk < n ? beg + chunk : n;
  const bool vec_ok = ((mt[0] | mt[1] | mt[2] | mt[3]) & 15) == 0 && (mt[4] & 7) == 0 &&
                      (sizeof(G) == 4 || (mt[1] & 7) == 0);
  int64_t i = beg + (int64_t)threadIdx.x * 4;
  if (vec_ok) {
    for (; i + 3 < end; i += MT_THREADS * 4) {
      f32x4 p = *reinterpret_cast<f32x4*>(P + i);
      f32x4 m = *reinterpret_cast<f32x4*>(M + i);
      f32x4 v = *reinterpret_cast<f32x4*>(V + i);
      float g[4];
      if constexpr (sizeof(G) == 4) {
        f32x4 gg = *reinterpret_cast<const f32x4*>(Gr + i);
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = gg[k];
      } else {
        u16x4 gg = *reinterpret_cast<const u16x4*>(Gr + i);
#pragma unroll
        for (int k = 0; k < 4; ++k) g[k] = bf2f(gg[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float pk = p[k], mk = m[k], vk = v[k];
        adam_elem<G>(pk, mk, vk, g[k] * gs, h);
        p[k] = pk; m[k] = mk; v[k] = vk;
      }
      *reinterpret_cast<f32x4*>(P + i) = p;
      *reinterpret_cast<f32x4*>(M + i) = m;
      *reinterpret_cast<f32x4*>(V + i) = v;
      if (O) {
        u16x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f2bf(p[k]);
        *reinterpret_cast<u16x4*>(O + i) = o;
      }
    }
    // tail (fewer than 4 left for this thread)
    for (; i < end; ++i) {
      float p = P[i], m = M[i], v = V[i];
      adam_elem<G>(p, m, v, to_f<G>(Gr[i]) * gs, h);
      P[i] = p; M[i] = m; V[i] = v;
      if (O) O[i] = f2bf(p);
    }
  } else {
    for (int64_t j = beg + threadIdx.x; j < end; j += MT_THREADS) {
      float p = P[j], m = M[j], v = V[j];
      adam_elem<G>(p, m, v, to_f<G>(Gr[j]) * gs, h);
      P[j] = p; M[j] = m; V[j] = v;
      if (O) O[j] = f2bf(p);
    }
  }
}

// Sum of squares per block (ptr0 of each tensor), written to partial[blockIdx.x].
template <typename G>
__global__ __launch_bounds__(MT_THREADS) void l2norm_mt_kernel(const int64_t* __restrict__ meta,
                                                               const int* __restrict__ blk, int chunk,
                                                               float* __restrict__ partial) {
  __shared__ float red[MT_THREADS / 64];
  const int t = blk[2 * blockIdx.x], c = blk[2 * blockIdx.x + 1];
  const int64_t* mt = meta + (int64_t)t * MT_META;
  const G* __restrict__ X = reinterpret_cast<const G*>(mt[0]);
  const int64_t n = mt[5];
  const int64_t beg = (int64_t)c * chunk;
  const int64_t end = beg + chunk < n ? beg + chunk : n;
  float acc = 0.f;
  const bool vec_ok = (mt[0] & 15) == 0;
  int64_t i = beg + (int64_t)threadIdx.x * 8;
  if (vec_ok) {
    for (; i + 7 < end; i += MT_THREADS * 8) {
      float x[8];
      Vec8<G>::load(X + i, x);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += x[k] * x[k];
    }
    for (; i < end; ++i) { float x = to_f<G>(X[i]); acc += x * x; }
  } else {
    for (int64_t j = beg + threadIdx.x; j < end; j += MT_THREADS) { float x = to_f<G>(X[j]); acc += x * x; }
  }
  acc = block_sum<MT_THREADS / 64>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Deterministic final reduction of the per-block partials (fixed order: bitwise reproducible).
__global__ __launch_bounds__(1024) void reduce_partials_kernel(const float* __restrict__ partial, int n,
                                                               float* __restrict__ out, int accumulate) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) acc += partial[i];
  acc = block_sum<16>(acc, red);
  if (threadIdx.x == 0) out[0] = accumulate ? out[0] + acc : acc;
}

// total_sq holds the (already globally all-reduced) sum of squares of the *scaled* gradients.
// Writes: norm_out = ||g|| / loss_scale, coef_out = grad multiplier = clip_coef / loss_scale,
// found_inf = !isfinite(total).  clip_coef = min(1, max_norm / (norm + 1e-6))
// (torch/nn/utils/clip_grad.py:165-174).  max_norm <= 0 disables clipping.
__global__ void clip_coef_kernel(const float* __restrict__ total_sq, float max_norm, const float* inv_scale_ptr,
                                 float inv_scale_val, float* __restrict__ norm_out, float* __restrict__ coef_out,
                                 int* __restrict__ found_inf) {
  const float inv_scale = inv_scale_ptr ? *inv_scale_ptr : inv_scale_val;
  const float sq = total_sq[0];
  const float norm = sqrtf(sq) * inv_scale;
  const bool finite = isfinite(sq);
  float coef = 1.f;
  if (max_norm > 0.f && finite) coef = fminf(max_norm / (norm + 1e-6f), 1.f);
  if (norm_out) norm_out[0] = norm;
  if (coef_out) coef_out[0] = coef * inv_scale;
  if (found_inf) found_inf[0] = finite ? 0 : 1;
}

template <typename G>
__global__ __launch_bounds__(MT_THREADS) void scale_mt_kernel(const int64_t* __restrict__ meta,
                                                              const int* __restrict__ blk, int chunk,
                                                              const float* __restrict__ s_ptr) {
  const float s = *s_ptr;
  const int t = blk[2 * blockIdx.x], c = blk[2 * blockIdx.x + 1];
  const int64_t* mt = meta + (int64_t)t * MT_META;
  G* __restrict__ X = reinterpret_cast<G*>(mt[0]);
  const int64_t n = mt[5];
  const int64_t beg = (int64_t)c * chunk;
  const int64_t end = beg + chunk < n ? beg + chunk : n;
  for (int64_t j = beg + threadIdx.x; j < end; j += MT_THREADS) X[j] = from_f<G>(to_f<G>(X[j]) * s);
}

// fp32 -> bf16 copy over a tensor list (ptr0 = src fp32, ptr1 = dst bf16): used to refresh the
// low-precision compute copy of parameters outside the optimizer (e.g. after load_state_dict).
__global__ __launch_bounds__(MT_THREADS) void cast_f32_bf16_mt_kernel(const int64_t* __restrict__ meta,
                                                                      const int* __restrict__ blk, int chunk) {
  const int t = blk[2 * blockIdx.x], c = blk[2 * blockIdx.x + 1];
  const int64_t* mt = meta + (int64_t)t * MT_META;
  const float* __restrict__ S = reinterpret_cast<const float*>(mt[0]);
  bf16_t* __restrict__ D = reinterpret_cast<bf16_t*>(mt[1]);
  const int64_t n = mt[5];
  const int64_t beg = (int64_t)c * chunk;
  const int64_t end = beg + chunk < n ? beg + chunk : n;
  for (int64_t j = beg + threadIdx.x; j < end; j += MT_THREADS) D[j] = f2bf(S[j]);
}

// dst <- src over a tensor list (ptr0 = dst, ptr1 = src, same element type; src 0 -> dst zero-filled): gathers
// per-parameter gradients into a flat buffer in ONE launch (parallel/ddp.py, single-process compute-copy mode)
template <typename T>
__global__ __launch_bounds__(MT_THREADS) void copy_mt_kernel(const int64_t* __restrict__ meta, const int* __restrict__ blk,
                                                             int chunk) {
  const int t = blk[2 * blockIdx.x], c = blk[2 * blockIdx.x + 1];
  const int64_t* mt = meta + (int64_t)t * MT_META;
  T* __restrict__ D = reinterpret_cast<T*>(mt[0]);
  const T* __restrict__ S = reinterpret_cast<const T*>(mt[1]);
  const int64_t n = mt[5];
  const int64_t beg = (int64_t)c * chunk;
  const int64_t end = beg + chunk < n ? beg + chunk : n;
  for (int64_t j = beg + threadIdx.x; j < end; j += MT_THREADS) D[j] = S ? S[j] : T(0);
}

// dst += src for every (dst, src) pair of the table (fp32 arithmetic; a null src adds nothing) -- per-parameter
// gradients accumulated into a flat buffer in ONE launch (DDP gradient stealing across accumulation micro-steps)
template <typename T>
__global__ __launch_bounds__(MT_THREADS) void add_mt_kernel(const int64_t* __restrict__ meta, const int* __restrict__ blk,
                                                            int chunk) {
  const int t = blk[2 * blockIdx.x], c = blk[2 * blockIdx.x + 1];
  const int64_t* mt = meta + (int64_t)t * MT_META;
  T* __restrict__ D = reinterpret_cast<T*>(mt[0]);
  const T* __restrict__ S = reinterpret_cast<const T*>(mt[1]);
  if (S == nullptr) return;
  const int64_t n = mt[5];
  const int64_t beg = (int64_t)c * chunk;
  const int64_t end = beg + chunk < n ? beg + chunk : n;
  for (int64_t j = beg + threadIdx.x; j < end; j += MT_THREADS) D[j] = from_f<T>(to_f<T>(D[j]) + to_f<T>(S[j]));
}

// Device step counter of a param group: +1 unless the (all-reduced) found_inf flag says the step is skipped
// (torch.amp.GradScaler skips optimizer.step() on overflow, so Adam's bias-correction step must not move).
__global__ void step_inc_kernel(float* __restrict__ dstep, const int* __restrict__ found_inf) {
  if (threadIdx.x == 0 && (found_inf == nullptr || *found_inf == 0)) dstep[0] = dstep[0] + 1.f;
}

}  // namespace

PDT_API int pdt_step_inc(float* dstep, const int* found_inf, hipStream_t stream) {
  step_inc_kernel<<<1, 64, 0, stream>>>(dstep, found_inf);
  return (int)hipGetLastError();
}

PDT_API int pdt_adamw_mt(const int64_t* meta, const int* blk, int nblocks, int chunk, int grad_dtype, float lr,
                         float beta1, float beta2, float eps, float wd, float step_size, float bc2_sqrt,
                         int decoupled, const float* gscale, const int* found_inf, const float* dstep,
                         hipStream_t stream) {
  AdamHyper h{lr, beta1, beta2, eps, wd, step_size, bc2_sqrt, decoupled};
  if (nblocks <= 0) return 0;
  if (grad_dtype == kF32)
    adamw_mt_kernel<float><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk, h, gscale, found_inf, dstep);
  else
    adamw_mt_kernel<bf16_t><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk, h, gscale, found_inf, dstep);
  return (int)hipGetLastError();
}

// partial must hold nblocks floats.  out[0] = sum of squares (accumulate=1 adds to out[0]).
PDT_API int pdt_l2norm_mt(const int64_t* meta, const int* blk, int nblocks, int chunk, int dtype, float* partial,
                          float* out, int accumulate, hipStream_t stream) {
  if (nblocks <= 0) {
    if (!accumulate) return (int)hipMemsetAsync(out, 0, sizeof(float), stream);
    return 0;
  }
  if (dtype == kF32)
    l2norm_mt_kernel<float><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk, partial);
  else
    l2norm_mt_kernel<bf16_t><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk, partial);
  reduce_partials_kernel<<<1, 1024, 0, stream>>>(partial, nblocks, out, accumulate);
  return (int)hipGetLastError();
}

PDT_API int pdt_clip_coef(const float* total_sq, float max_norm, const float* inv_scale_ptr, float inv_scale_val,
                          float* norm_out, float* coef_out, int* found_inf, hipStream_t stream) {
  clip_coef_kernel<<<1, 1, 0, stream>>>(total_sq, max_norm, inv_scale_ptr, inv_scale_val, norm_out, coef_out,
                                        found_inf);
  return (int)hipGetLastError();
}

PDT_API int pdt_scale_mt(const int64_t* meta, const int* blk, int nblocks, int chunk, int dtype, const float* s,
                         hipStream_t stream) {
  if (nblocks <= 0) return 0;
  if (dtype == kF32)
    scale_mt_kernel<float><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk, s);
  else
    scale_mt_kernel<bf16_t><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk, s);
  return (int)hipGetLastError();
}

PDT_API int pdt_cast_f32_bf16_mt(const int64_t* meta, const int* blk, int nblocks, int chunk, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  cast_f32_bf16_mt_kernel<<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk);
  return (int)hipGetLastError();
}

// dt: kBF16 or kF32
PDT_API int pdt_add_mt(const int64_t* meta, const int* blk, int nblocks, int chunk, int dt, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  if (dt == kF32)
    add_mt_kernel<float><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk);
  else if (dt == kBF16)
    add_mt_kernel<bf16_t><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// elem_bytes 2 (bf16 / fp16) or 4 (fp32)
PDT_API int pdt_copy_mt(const int64_t* meta, const int* blk, int nblocks, int chunk, int elem_bytes, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  if (elem_bytes == 4)
    copy_mt_kernel<uint32_t><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk);
  else if (elem_bytes == 2)
    copy_mt_kernel<uint16_t><<<nblocks, MT_THREADS, 0, stream>>>(meta, blk, chunk);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
