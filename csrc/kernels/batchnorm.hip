// Fused BatchNorm (+ residual add) (+ ReLU) for channels-last (NHWC) activations on gfx950 -- the
// ResNet-50 DDP config (BASELINE.json config 2).  A bf16 ResNet-50 step spends ~35 % of
// its time in BatchNorm and another ~8 % in ReLU (scripts/bench_resnet_breakdown.py: 42.2 ms -> 27.3 ms without
// BN, -> 24.0 ms without BN and ReLU); stock PyTorch runs BN, the residual add and ReLU as separate
// passes over HBM.  Here:
//
//   forward   stats  : per-channel (sum, sum^2) partials over row chunks (fp32) -> fp64 combine
//             apply  : y = relu(x * scale[c] + shift[c] (+ res))         ONE pass (reads x (+res), writes y)
//   backward  reduce : (sum dy', sum dy' * xhat) with dy' = dy * relu'(.)  (ReLU mask: recomputed from x, or a
//                      1-bit-per-element mask the forward apply wrote after a residual add)
//             apply  : dx = (dy' - s1/M - xhat * s2/M) * invstd * w ; dres = dy' (residual branch)
//
// x is [R rows, C] contiguous (R = N*H*W), C % 8 == 0.  A thread owns 8 consecutive channels for the
// whole launch (scale / shift / mean / invstd live in registers, no per-element channel index math) and
// walks rows; a workgroup covers 256 / (C/8) rows per pass (coalesced 16-byte accesses).  Cross-rank
// SyncBN = one all-reduce of the fp64 sums between the combine and finalize kernels (caller).
#include "common.h"

using namespace pdt;

namespace {

constexpr int NT = 256;

struct Tile {
  int G, rpb, rl, cg;   // channel groups, rows per block pass, this thread's row lane, channel group
  bool act;
  __device__ Tile(int C) {
    G = C >> 3;
    rpb = NT / G;
    rl = threadIdx.x / G;
    cg = threadIdx.x - rl * G;
    act = rl < rpb;
  }
};

// MODE 0: (x, x^2)  MODE 1: (dy', dy' * xhat), dy' = dy * relu'(.) per MASK:
//   MASK 0: no ReLU;  1: mask = (y > 0) from the saved output;
//   2: mask = (x * scale + shift > 0) recomputed from x with the forward's own coefficients (BN -> ReLU with
//      no residual: y is then never read -- one bf16 stream less in both backward passes);
//   3: mask bits written by the forward apply (after a residual add, where x alone does not determine it): one
//      byte per (row, 8-channel group), bit k = channel 8g + k -- 1/16 of the bytes of reading y back
template <int MASK>
__device__ __forceinline__ void relu_mask(float (&g)[8], const float (&xv)[8], const float* yv, const float (&sc)[8],
                                          const float (&sh)[8], unsigned bits) {
  if constexpr (MASK == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
  } else if constexpr (MASK == 2) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = xv[k] * sc[k] + sh[k] > 0.f ? g[k] : 0.f;
  } else if constexpr (MASK == 3) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = (bits >> k) & 1u ? g[k] : 0.f;
  }
}

template <int MODE, int MASK>
__global__ __launch_bounds__(NT) void bn_reduce_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                       const bf16_t* __restrict__ y, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ scsh, int64_t R, int C,
                                                       float* __restrict__ part) {
  constexpr bool RELU = MASK == 1;   // y is read
  const uint8_t* __restrict__ mbits = reinterpret_cast<const uint8_t*>(y);   // MASK 3: y is the bit mask
  __shared__ __attribute__((aligned(16))) float sa[NT * 8];
  __shared__ __attribute__((aligned(16))) float sb[NT * 8];
  const Tile t(C);
  float a[8], b[8], mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { a[k] = 0.f; b[k] = 0.f; mu[k] = 0.f; is[k] = 0.f; sc[k] = 0.f; sh[k] = 0.f; }
  if (t.act) {
    if (MODE == 1) {
      Vec8<float>::load(mean + t.cg * 8, mu);
      Vec8<float>::load(invstd + t.cg * 8, is);
    }
    if (MASK == 2) {
      Vec8<float>::load(scsh + t.cg * 8, sc);
      Vec8<float>::load(scsh + C + t.cg * 8, sh);
    }
    const int64_t stride = (int64_t)gridDim.x * t.rpb;
    int64_t r = (int64_t)blockIdx.x * t.rpb + t.rl;
    // two rows in flight per thread (all loads issued before the first use)
    for (; r + stride < R; r += 2 * stride) {
      const int64_t off0 = r * C + t.cg * 8, off1 = (r + stride) * C + t.cg * 8;
      typename Vec8<bf16_t>::raw_t x0 = Vec8<bf16_t>::load_raw(x + off0), x1 = Vec8<bf16_t>::load_raw(x + off1);
      typename Vec8<bf16_t>::raw_t g0, g1, y0, y1;
      unsigned b0 = 0, b1 = 0;
      if (MODE == 1) { g0 = Vec8<bf16_t>::load_raw(dy + off0); g1 = Vec8<bf16_t>::load_raw(dy + off1); }
      if (MODE == 1 && RELU) { y0 = Vec8<bf16_t>::load_raw(y + off0); y1 = Vec8<bf16_t>::load_raw(y + off1); }
      if (MODE == 1 && MASK == 3) { b0 = mbits[r * t.G + t.cg]; b1 = mbits[(r + stride) * t.G + t.cg]; }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float xv[8];
        Vec8<bf16_t>::unpack(u ? x1 : x0, xv);
        if (MODE == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { a[k] += xv[k]; b[k] += xv[k] * xv[k]; }
        } else {
          float g[8], yv[8];
          Vec8<bf16_t>::unpack(u ? g1 : g0, g);
          if (RELU) Vec8<bf16_t>::unpack(u ? y1 : y0, yv);
          relu_mask<MASK>(g, xv, yv, sc, sh, u ? b1 : b0);
#pragma unroll
          for (int k = 0; k < 8; ++k) { a[k] += g[k]; b[k] += g[k] * (xv[k] - mu[k]) * is[k]; }
        }
      }
    }
    for (; r < R; r += stride) {
      const int64_t off = r * C + t.cg * 8;
      float xv[8];
      Vec8<bf16_t>::load(x + off, xv);
      if (MODE == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { a[k] += xv[k]; b[k] += xv[k] * xv[k]; }
      } else {
        float g[8], yv[8];
        Vec8<bf16_t>::load(dy + off, g);
        if (RELU) Vec8<bf16_t>::load(y + off, yv);
        relu_mask<MASK>(g, xv, yv, sc, sh, MASK == 3 ? (unsigned)mbits[r * t.G + t.cg] : 0u);
#pragma unroll
        for (int k = 0; k < 8; ++k) { a[k] += g[k]; b[k] += g[k] * (xv[k] - mu[k]) * is[k]; }
      }
    }
  }
  Vec8<float>::store(sa + threadIdx.x * 8, a);
  Vec8<float>::store(sb + threadIdx.x * 8, b);
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int g = c >> 3, k = c & 7;
    float s1 = 0.f, s2 = 0.f;
    for (int q = 0; q < t.rpb; ++q) { s1 += sa[(q * t.G + g) * 8 + k]; s2 += sb[(q * t.G + g) * 8 + k]; }
    part[(int64_t)blockIdx.x * 2 * C + c] = s1;
    part[(int64_t)blockIdx.x * 2 * C + C + c] = s2;
  }
}

// [P, 2C] fp32 partials -> out[2C] fp64.  Workgroup = 64 outputs x 16 waves; each wave sums a sixteenth of
// the P partial rows (lanes read consecutive outputs: coalesced), 8 loads in flight per lane, folded through
// LDS.  (4 waves and 4 loads left the ~100 combines of a ResNet-50 step latency-bound at ~11 us each: the
// narrow layers have only 2-4 workgroups here.)
//   count > 0: out[2C] = count (forward);  dw / db (nullable): fp32 copies of the two halves (backward)
constexpr int CW = 16;
__global__ __launch_bounds__(64 * CW) void bn_combine_kernel(const float* __restrict__ part, int P, int C, double count,
                                                             double* __restrict__ out, float* __restrict__ dw,
                                                             float* __restrict__ db) {
  __shared__ double red[CW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  double s = 0.0;
  if (i < 2 * C) {
    const int per = (P + CW - 1) / CW, j0 = wv * per, j1 = min(P, j0 + per);
    int j = j0;
    for (; j + 8 <= j1; j += 8) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = part[(int64_t)(j + u) * 2 * C + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)a[u];
    }
    for (; j < j1; ++j) s += (double)part[(int64_t)j * 2 * C + i];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && i < 2 * C) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < CW; ++q) t += red[q][lane];
    out[i] = t;
    if (i < C) { if (db) db[i] = (float)t; }
    else if (dw) dw[i - C] = (float)t;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && count > 0) out[2 * C] = count;
}

// bn_combine_kernel + bn_finalize_kernel in one launch for the single-process statistics (no all-reduce between
// them): a workgroup owns 64 channels and sums BOTH halves of their partial rows, so the finalize needs no
// second pass (ResNet-50 runs ~50 forward batch norms per step: one ~4 us launch less each)
__global__ __launch_bounds__(64 * CW) void bn_combine_finalize_kernel(const float* __restrict__ part, int P, int C,
                                                                      double count, double* __restrict__ out,
                                                                      float eps, float momentum,
                                                                      const float* __restrict__ w,
                                                                      const float* __restrict__ b,
                                                                      float* __restrict__ mean, float* __restrict__ invstd,
                                                                      float* __restrict__ scale, float* __restrict__ shift,
                                                                      float* __restrict__ rmean, float* __restrict__ rvar) {
  __shared__ double red[2][CW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const int per = (P + CW - 1) / CW, j0 = wv * per, j1 = min(P, j0 + per);
    int j = j0;
    for (; j + 4 <= j1; j += 4) {
      float a[4], q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) { a[u] = part[(int64_t)(j + u) * 2 * C + c]; q[u] = part[(int64_t)(j + u) * 2 * C + C + c]; }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s1 += (double)a[u]; s2 += (double)q[u]; }
    }
    for (; j < j1; ++j) { s1 += (double)part[(int64_t)j * 2 * C + c]; s2 += (double)part[(int64_t)j * 2 * C + C + c]; }
  }
  red[0][wv][lane] = s1;
  red[1][wv][lane] = s2;
  __syncthreads();
  if (wv == 0 && c < C) {
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int q = 0; q < CW; ++q) { t1 += red[0][q][lane]; t2 += red[1][q][lane]; }
    out[c] = t1;
    out[C + c] = t2;
    const double mu = t1 / count;
    double var = t2 / count - mu * mu;
    if (var < 0) var = 0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
    mean[c] = (float)mu;
    invstd[c] = is;
    scale[c] = is * wc;
    shift[c] = bc - (float)mu * is * wc;
    if (rmean) {
      const double unbiased = count > 1 ? var * count / (count - 1) : var;
      rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mu);
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[2 * C] = count;
}

// stats (global sums + count) -> mean, invstd, scale = invstd * w, shift = b - mean * scale; running stats
__global__ void bn_finalize_kernel(const double* __restrict__ stats, int C, float eps, float momentum,
                                   const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ mean,
                                   float* __restrict__ invstd, float* __restrict__ scale, float* __restrict__ shift,
                                   float* __restrict__ rmean, float* __restrict__ rvar) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double n = stats[2 * C];
  const double mu = stats[c] / n;
  double var = stats[C + c] / n - mu * mu;
  if (var < 0) var = 0;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
  mean[c] = (float)mu;
  invstd[c] = is;
  scale[c] = is * wc;
  shift[c] = bc - (float)mu * is * wc;
  if (rmean) {
    const double unbiased = n > 1 ? var * n / (n - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mu);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unbiased);
  }
}

// eval mode: scale / shift from the running statistics
__global__ void bn_eval_coef_kernel(const float* __restrict__ rmean, const float* __restrict__ rvar, int C, float eps,
                                    const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ scale,
                                    float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = rsqrtf(rvar[c] + eps), wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
  scale[c] = is * wc;
  shift[c] = bc - rmean[c] * is * wc;
}

template <bool RES, bool RELU, bool MOUT = false>
__global__ __launch_bounds__(NT) void bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      bf16_t* __restrict__ y, int64_t R, int C,
                                                      uint8_t* __restrict__ mask_out) {
  const Tile t(C);
  if (!t.act) return;
  float sc[8], sh[8];
  Vec8<float>::load(scale + t.cg * 8, sc);
  Vec8<float>::load(shift + t.cg * 8, sh);
  const int64_t stride = (int64_t)gridDim.x * t.rpb;
#pragma unroll 2
  for (int64_t r = (int64_t)blockIdx.x * t.rpb + t.rl; r < R; r += stride) {
    const int64_t off = r * C + t.cg * 8;
    float v[8];
    Vec8<bf16_t>::load(x + off, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] * sc[k] + sh[k];
    if (RES) {
      float rv[8];
      Vec8<bf16_t>::load(res + off, rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += rv[k];
    }
    if (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
    }
    if (MOUT) {   // relu'(pre) = (pre > 0) = (y > 0): the backward's MASK 3 bits
      unsigned bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) bits |= (v[k] > 0.f ? 1u : 0u) << k;
      mask_out[r * t.G + t.cg] = (uint8_t)bits;
    }
    Vec8<bf16_t>::store(y + off, v);
  }
}

// dx = (dy' - s1 / M - xhat * s2 / M) * invstd * w ; dres = dy'   (MASK as bn_reduce_kernel)
template <int MASK, bool DRES>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                          const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, const float* __restrict__ w,
                                                          const float* __restrict__ scsh,
                                                          const double* __restrict__ sums, const double* __restrict__ count,
                                                          bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, int64_t R,
                                                          int C) {
  constexpr bool RELU = MASK == 1;
  const uint8_t* __restrict__ mbits = reinterpret_cast<const uint8_t*>(y);   // MASK 3: y is the bit mask
  const Tile t(C);
  if (!t.act) return;
  const double inv_m = 1.0 / count[0];
  float mu[8], is[8], k1[8], k2[8], k3[8], sc[8], sh[8];
  if (MASK == 2) {
    Vec8<float>::load(scsh + t.cg * 8, sc);
    Vec8<float>::load(scsh + C + t.cg * 8, sh);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = t.cg * 8 + k;
    mu[k] = mean[c];
    is[k] = invstd[c];
    const float wc = w ? w[c] : 1.f;
    k1[k] = is[k] * wc;                               // dy' coefficient
    k2[k] = (float)(sums[c] * inv_m) * k1[k];         // mean(dy') term
    k3[k] = (float)(sums[C + c] * inv_m) * k1[k];     // mean(dy' xhat) term (times xhat)
  }
  const int64_t stride = (int64_t)gridDim.x * t.rpb;
#pragma unroll 2
  for (int64_t r = (int64_t)blockIdx.x * t.rpb + t.rl; r < R; r += stride) {
    const int64_t off = r * C + t.cg * 8;
    float g[8], xv[8], o[8], yv[8];
    Vec8<bf16_t>::load(dy + off, g);
    Vec8<bf16_t>::load(x + off, xv);
    if (RELU) Vec8<bf16_t>::load(y + off, yv);
    relu_mask<MASK>(g, xv, yv, sc, sh, MASK == 3 ? (unsigned)mbits[r * t.G + t.cg] : 0u);
    if (DRES) Vec8<bf16_t>::store(dres + off, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * k1[k] - k2[k] - (xv[k] - mu[k]) * is[k] * k3[k];
    Vec8<bf16_t>::store(dx + off, o);
  }
}

int reduce_grid(int64_t R, int C) {
  const int rpb = NT / (C >> 3);
  int64_t g = (R + (int64_t)rpb * 16 - 1) / ((int64_t)rpb * 16);   // >= 16 rows per thread
  if (g < 1) g = 1;
  if (g > 512) g = 512;
  return (int)g;
}
int apply_grid(int64_t R, int C) {
  const int rpb = NT / (C >> 3);
  int64_t g = (R + (int64_t)rpb * 8 - 1) / ((int64_t)rpb * 8);
  if (g < 1) g = 1;
  if (g > 256 * 8) g = 256 * 8;
  return (int)g;
}

}  // namespace

// workspace (fp32) for the partial sums: 2 * C * 1024 floats
PDT_API int pdt_bn_ws_floats(int C) { return 2 * C * 1024; }

PDT_API int pdt_bn_ok(int C) { return (C % 8 == 0 && C >= 8 && C <= 2048) ? 1 : 0; }

// forward statistics: out[0:2C] = (sum, sum^2) fp64, out[2C] = R (count)
PDT_API int pdt_bn_stats(const void* x, int64_t R, int C, float* ws, double* out, hipStream_t st) {
  if (!pdt_bn_ok(C)) return (int)hipErrorInvalidValue;
  const int P = reduce_grid(R, C);
  bn_reduce_kernel<0, 0><<<P, NT, 0, st>>>((const bf16_t*)x, nullptr, nullptr, nullptr, nullptr, nullptr, R, C, ws);
  bn_combine_kernel<<<(2 * C + 63) / 64, 64 * CW, 0, st>>>(ws, P, C, (double)R, out, nullptr, nullptr);
  return (int)hipGetLastError();
}

// pdt_bn_stats + pdt_bn_finalize with no cross-rank reduction in between (two launches instead of three)
PDT_API int pdt_bn_stats_finalize(const void* x, int64_t R, int C, float* ws, double* out, float eps, float momentum,
                                  const float* w, const float* b, float* mean, float* invstd, float* scale,
                                  float* shift, float* rmean, float* rvar, hipStream_t st) {
  if (!pdt_bn_ok(C)) return (int)hipErrorInvalidValue;
  const int P = reduce_grid(R, C);
  bn_reduce_kernel<0, 0><<<P, NT, 0, st>>>((const bf16_t*)x, nullptr, nullptr, nullptr, nullptr, nullptr, R, C, ws);
  bn_combine_finalize_kernel<<<(C + 63) / 64, 64 * CW, 0, st>>>(ws, P, C, (double)R, out, eps, momentum, w, b, mean,
                                                                invstd, scale, shift, rmean, rvar);
  return (int)hipGetLastError();
}

PDT_API int pdt_bn_finalize(const double* stats, int C, float eps, float momentum, const float* w, const float* b,
                            float* mean, float* invstd, float* scale, float* shift, float* rmean, float* rvar,
                            hipStream_t st) {
  bn_finalize_kernel<<<(C + 255) / 256, 256, 0, st>>>(stats, C, eps, momentum, w, b, mean, invstd, scale, shift, rmean,
                                                      rvar);
  return (int)hipGetLastError();
}

PDT_API int pdt_bn_eval_coef(const float* rmean, const float* rvar, int C, float eps, const float* w, const float* b,
                             float* scale, float* shift, hipStream_t st) {
  bn_eval_coef_kernel<<<(C + 255) / 256, 256, 0, st>>>(rmean, rvar, C, eps, w, b, scale, shift);
  return (int)hipGetLastError();
}

// y = act(x * scale + shift (+ res)); act: 0 none, 1 relu.  mask_out (nullable, relu only): [R, C / 8] bytes of
// relu'(.) bits for the backward's relu = 3 mode
PDT_API int pdt_bn_apply(const void* x, const void* res, const float* scale, const float* shift, void* y, int64_t R,
                         int C, int relu, void* mask_out, hipStream_t st) {
  if (!pdt_bn_ok(C) || (mask_out && !relu)) return (int)hipErrorInvalidValue;
  const int g = apply_grid(R, C);
#define PDT_L(RS, RL, MO) bn_apply_kernel<RS, RL, MO><<<g, NT, 0, st>>>((const bf16_t*)x, (const bf16_t*)res, scale, \
                                                                        shift, (bf16_t*)y, R, C, (uint8_t*)mask_out)
  if (mask_out) { if (res) PDT_L(true, true, true); else PDT_L(false, true, true); }
  else if (res) { if (relu) PDT_L(true, true, false); else PDT_L(true, false, false); }
  else { if (relu) PDT_L(false, true, false); else PDT_L(false, false, false); }
#undef PDT_L
  return (int)hipGetLastError();
}

// backward sums: out[0:2C] = (sum dy', sum dy' * xhat) fp64 (local; caller all-reduces for SyncBN);
// dw / db (fp32, nullable) receive the local parameter gradients.  relu: 0 none, 1 mask from y, 2 mask from
// x * scale + shift (scsh = [scale C | shift C], the forward's coefficients; y is not read), 3 mask bits from
// pdt_bn_apply's mask_out (passed as y)
PDT_API int pdt_bn_bwd_reduce(const void* dy, const void* y, const void* x, const float* mean, const float* invstd,
                              const float* scsh, int64_t R, int C, int relu, float* ws, double* out, float* dw,
                              float* db, hipStream_t st) {
  if (!pdt_bn_ok(C) || relu < 0 || relu > 3 || (relu == 2 && !scsh)) return (int)hipErrorInvalidValue;
  const int P = reduce_grid(R, C);
#define PDT_L(M) bn_reduce_kernel<1, M><<<P, NT, 0, st>>>((const bf16_t*)x, (const bf16_t*)dy, (const bf16_t*)y, mean, \
                                                          invstd, scsh, R, C, ws)
  if (relu == 1) PDT_L(1);
  else if (relu == 2) PDT_L(2);
  else if (relu == 3) PDT_L(3);
  else PDT_L(0);
#undef PDT_L
  bn_combine_kernel<<<(2 * C + 63) / 64, 64 * CW, 0, st>>>(ws, P, C, 0.0, out, dw, db);
  return (int)hipGetLastError();
}

// dx (and dres = masked dy when dres != null); sums = global (sum dy', sum dy' xhat); count = global M
PDT_API int pdt_bn_bwd_apply(const void* dy, const void* y, const void* x, const float* mean, const float* invstd,
                             const float* w, const float* scsh, const double* sums, const double* count, void* dx,
                             void* dres, int64_t R, int C, int relu, hipStream_t st) {
  if (!pdt_bn_ok(C) || relu < 0 || relu > 3 || (relu == 2 && !scsh)) return (int)hipErrorInvalidValue;
  const int g = apply_grid(R, C);
#define PDT_L(M, DR) bn_bwd_apply_kernel<M, DR><<<g, NT, 0, st>>>((const bf16_t*)dy, (const bf16_t*)y, \
      (const bf16_t*)x, mean, invstd, w, scsh, sums, count, (bf16_t*)dx, (bf16_t*)dres, R, C)
  if (relu == 1) { if (dres) PDT_L(1, true); else PDT_L(1, false); }
  else if (relu == 2) { if (dres) PDT_L(2, true); else PDT_L(2, false); }
  else if (relu == 3) { if (dres) PDT_L(3, true); else PDT_L(3, false); }
  else { if (dres) PDT_L(0, true); else PDT_L(0, false); }
#undef PDT_L
  return (int)hipGetLastError();
}
