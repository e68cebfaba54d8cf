// Fused shifted-window attention (SwinIR / Swin) for gfx950: softmax(q k^T * scale + B_rel + M_shift) v
// for every (window, head), forward and backward, reading the fused qkv projection [Bw, N, 3C] in place
// and writing o as [Bw, N, C] (the layout the output projection consumes -- no permute/contiguous).
//
// SURVEY.md K4 (window attention: `q·kᵀ·scale + rel_pos_bias[idx] (+mask)` → softmax → `·v`, 4,608
// windows × 6 heads of [64×10]·[10×64] per SwinIR-S block at the Stoke config, Stoke-DDP.py:206-208)
// and K6 (the window partition permutes are folded into the addressing).  The stock path
// materialises the expanded bias+mask [Bw, h, N, N] and the score matrix in HBM; here nothing of
// size N×N leaves the CU.
//
// Shape regime: N ≤ 64 tokens per window, head_dim d ≤ 32 (SwinIR-S: N = 64, d = 10).  With d = 10 an
// MFMA tile would be > 60% padding, so the math runs on the VALU in fp32: one wave per head, one
// lane per query (forward / dQ) or per key (dK/dV); the window's K/V (and Q/dO in backward) are staged
// in LDS as fp32 rows padded to DP floats and read as wave-uniform broadcasts (conflict-free).
// A workgroup = one window × all heads (64·H threads) and walks windows grid-stride.
//
// Backward phase A (lane = query i): recompute p_ij, dS_ij, dQ_i; the per-(head, i, j) dS sums
// (relative-position-bias gradient) accumulate in registers across the windows the workgroup visits
// and are written as one fp32 partial [H, N, N] per workgroup (summed on the host side of the op).
// Phase B (lane = key j): recompute p_ij, dS_ij from the staged Q/dO/lse/delta, accumulate dK_j, dV_j.
#include "common.h"

using namespace pdt;

namespace {

constexpr int NMAX = 64;

template <int DP>
struct WinSmem {
  // [H][NMAX][DP] fp32 row blocks
  static __device__ __forceinline__ float* blk(float* base, int which, int H, int h) {
    return base + ((int64_t)which * H + h) * NMAX * DP;
  }
};

template <int DP>
__device__ __forceinline__ float dotp(const float (&a)[DP], const float* row) {
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < DP; c += 4) {
    const f32x4 r = *reinterpret_cast<const f32x4*>(row + c);
    acc += a[c] * r[0] + a[c + 1] * r[1] + a[c + 2] * r[2] + a[c + 3] * r[3];
  }
  return acc;
}

// cooperative load of `nblk` of the q/k/v thirds (which = 0,1,2) of one window into LDS blocks
template <typename T, int DP>
__device__ __forceinline__ void stage(const T* base, int N, int H, int d, float* sm, int which, int slot,
                                      float mul) {
  const int C = H * d;
  for (int e = threadIdx.x; e < N * C; e += blockDim.x) {
    const int t = e / C, c = e % C, hh = c / d, cc = c % d;
    WinSmem<DP>::blk(sm, slot, H, hh)[t * DP + cc] = to_f<T>(base[(int64_t)t * 3 * C + which * C + c]) * mul;
  }
}

template <typename T, int DP>
__global__ __launch_bounds__(1024) void win_attn_fwd_kernel(const T* __restrict__ qkv, const float* __restrict__ bias_t,
                                                            const float* __restrict__ mask_t, int nw,
                                                            T* __restrict__ o, float* __restrict__ lse, int Bw, int N,
                                                            int H, int d, float scale) {
  extern __shared__ __attribute__((aligned(16))) float sm[];   // K, V: [2][H][NMAX][DP]
  const int lane = threadIdx.x & 63, h = threadIdx.x >> 6;
  const int C = H * d;
  for (int e = threadIdx.x; e < 2 * H * NMAX * DP; e += blockDim.x) sm[e] = 0.f;   // zero pads once
  for (int bw = blockIdx.x; bw < Bw; bw += gridDim.x) {
    const T* base = qkv + (int64_t)bw * N * 3 * C;
    __syncthreads();
    stage<T, DP>(base, N, H, d, sm, 1, 0, 1.f);
    stage<T, DP>(base, N, H, d, sm, 2, 1, 1.f);
    __syncthreads();
    if (lane < N) {
      float q[DP];
#pragma unroll
      for (int c = 0; c < DP; ++c) q[c] = c < d ? to_f<T>(base[(int64_t)lane * 3 * C + h * d + c]) * scale : 0.f;
      const float* Kh = WinSmem<DP>::blk(sm, 0, H, h);
      const float* Vh = WinSmem<DP>::blk(sm, 1, H, h);
      const float* bt = bias_t + (int64_t)h * N * N;
      const float* mt = mask_t ? mask_t + (int64_t)(bw % nw) * N * N : nullptr;
      float s[NMAX];
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < NMAX; ++j) {
        if (j < N) {
          float a = dotp<DP>(q, Kh + j * DP) + bt[j * N + lane];
          if (mt) a += mt[j * N + lane];
          s[j] = a;
          m = fmaxf(m, a);
        }
      }
      float l = 0.f, acc[DP];
#pragma unroll
      for (int c = 0; c < DP; ++c) acc[c] = 0.f;
#pragma unroll
      for (int j = 0; j < NMAX; ++j) {
        if (j < N) {
          const float p = __expf(s[j] - m);
          l += p;
#pragma unroll
          for (int c = 0; c < DP; c += 4) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(Vh + j * DP + c);
            acc[c] += p * v[0]; acc[c + 1] += p * v[1]; acc[c + 2] += p * v[2]; acc[c + 3] += p * v[3];
          }
        }
      }
      const float il = 1.f / l;
      T* orow = o + ((int64_t)bw * N + lane) * C + h * d;
#pragma unroll
      for (int c = 0; c < DP; ++c)
        if (c < d) orow[c] = from_f<T>(acc[c] * il);
      lse[((int64_t)bw * H + h) * N + lane] = m + __logf(l);
    }
  }
}

template <typename T, int DP>
__global__ __launch_bounds__(1024) void win_attn_bwd_kernel(const T* __restrict__ qkv, const float* __restrict__ bias,
                                                            const float* __restrict__ bias_t,
                                                            const float* __restrict__ mask,
                                                            const float* __restrict__ mask_t, int nw,
                                                            const T* __restrict__ o, const T* __restrict__ dout,
                                                            const float* __restrict__ lse, T* __restrict__ dqkv,
                                                            float* __restrict__ dbias_part, int Bw, int N, int H, int d,
                                                            float scale) {
  // LDS: Q(scaled), K, V, dO as [4][H][NMAX][DP]; lse, delta as [2][H][NMAX]
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* sstat = sm + 4 * H * NMAX * DP;
  const int lane = threadIdx.x & 63, h = threadIdx.x >> 6;
  const int C = H * d;
  for (int e = threadIdx.x; e < 4 * H * NMAX * DP; e += blockDim.x) sm[e] = 0.f;
  float dsacc[NMAX];
#pragma unroll
  for (int j = 0; j < NMAX; ++j) dsacc[j] = 0.f;
  const float* Qh = WinSmem<DP>::blk(sm, 0, H, h);
  const float* Kh = WinSmem<DP>::blk(sm, 1, H, h);
  const float* Vh = WinSmem<DP>::blk(sm, 2, H, h);
  const float* Gh = WinSmem<DP>::blk(sm, 3, H, h);
  float* Lh = sstat + h * NMAX;
  float* Dh = sstat + (H + h) * NMAX;

  for (int bw = blockIdx.x; bw < Bw; bw += gridDim.x) {
    const T* base = qkv + (int64_t)bw * N * 3 * C;
    T* dbase = dqkv + (int64_t)bw * N * 3 * C;
    __syncthreads();
    stage<T, DP>(base, N, H, d, sm, 0, 0, scale);
    stage<T, DP>(base, N, H, d, sm, 1, 1, 1.f);
    stage<T, DP>(base, N, H, d, sm, 2, 2, 1.f);
    for (int e = threadIdx.x; e < N * C; e += blockDim.x) {   // dO [Bw, N, C] -> slot 3
      const int t = e / C, c = e % C, hh = c / d, cc = c % d;
      WinSmem<DP>::blk(sm, 3, H, hh)[t * DP + cc] = to_f<T>(dout[((int64_t)bw * N + t) * C + c]);
    }
    __syncthreads();
    const float* mrow = mask ? mask + (int64_t)(bw % nw) * N * N : nullptr;
    const float* mcol = mask_t ? mask_t + (int64_t)(bw % nw) * N * N : nullptr;
    // ---- phase A: lane = query i
    if (lane < N) {
      float q[DP], g[DP];
      float dl = 0.f;
#pragma unroll
      for (int c = 0; c < DP; ++c) {
        q[c] = Qh[lane * DP + c];
        g[c] = Gh[lane * DP + c];
        if (c < d) dl += g[c] * to_f<T>(o[((int64_t)bw * N + lane) * C + h * d + c]);
      }
      const float ls = lse[((int64_t)bw * H + h) * N + lane];
      Lh[lane] = ls;
      Dh[lane] = dl;
      const float* bt = bias_t + (int64_t)h * N * N;
      float dq[DP];
#pragma unroll
      for (int c = 0; c < DP; ++c) dq[c] = 0.f;
#pragma unroll
      for (int j = 0; j < NMAX; ++j) {
        if (j < N) {
          float a = dotp<DP>(q, Kh + j * DP) + bt[j * N + lane];
          if (mcol) a += mcol[j * N + lane];
          const float p = __expf(a - ls);
          const float dp = dotp<DP>(g, Vh + j * DP);
          const float ds = p * (dp - dl);
          dsacc[j] += ds;
#pragma unroll
          for (int c = 0; c < DP; c += 4) {
            const f32x4 k = *reinterpret_cast<const f32x4*>(Kh + j * DP + c);
            dq[c] += ds * k[0]; dq[c + 1] += ds * k[1]; dq[c + 2] += ds * k[2]; dq[c + 3] += ds * k[3];
          }
        }
      }
      T* dqrow = dbase + (int64_t)lane * 3 * C + h * d;
#pragma unroll
      for (int c = 0; c < DP; ++c)
        if (c < d) dqrow[c] = from_f<T>(dq[c] * scale);
    }
    __syncthreads();
    // ---- phase B: lane = key j
    if (lane < N) {
      float k[DP], v[DP], dk[DP], dv[DP];
#pragma unroll
      for (int c = 0; c < DP; ++c) { k[c] = Kh[lane * DP + c]; v[c] = Vh[lane * DP + c]; dk[c] = 0.f; dv[c] = 0.f; }
      const float* br = bias + (int64_t)h * N * N;
#pragma unroll 4
      for (int i = 0; i < N; ++i) {
        float a = dotp<DP>(k, Qh + i * DP) + br[i * N + lane];
        if (mrow) a += mrow[i * N + lane];
        const float p = __expf(a - Lh[i]);
        const float dp = dotp<DP>(v, Gh + i * DP);
        const float ds = p * (dp - Dh[i]);
#pragma unroll
        for (int c = 0; c < DP; c += 4) {
          const f32x4 qq = *reinterpret_cast<const f32x4*>(Qh + i * DP + c);
          const f32x4 gg = *reinterpret_cast<const f32x4*>(Gh + i * DP + c);
          dk[c] += ds * qq[0]; dk[c + 1] += ds * qq[1]; dk[c + 2] += ds * qq[2]; dk[c + 3] += ds * qq[3];
          dv[c] += p * gg[0]; dv[c + 1] += p * gg[1]; dv[c + 2] += p * gg[2]; dv[c + 3] += p * gg[3];
        }
      }
      T* dkrow = dbase + (int64_t)lane * 3 * C + C + h * d;
      T* dvrow = dbase + (int64_t)lane * 3 * C + 2 * C + h * d;
#pragma unroll
      for (int c = 0; c < DP; ++c)
        if (c < d) { dkrow[c] = from_f<T>(dk[c]); dvrow[c] = from_f<T>(dv[c]); }
    }
  }
  // relative-position-bias gradient partial of this workgroup: [H][N(i)][N(j)]
  if (lane < N) {
    float* dst = dbias_part + ((int64_t)blockIdx.x * H + h) * N * N + (int64_t)lane * N;
#pragma unroll
    for (int j = 0; j < NMAX; ++j)
      if (j < N) dst[j] = dsacc[j];
  }
}

template <int DP>
int dp_ok(int d) { return d <= DP; }

}  // namespace

// grid size the launcher uses (also the number of dbias partials the caller must allocate)
PDT_API int pdt_win_attn_grid(int Bw) { return Bw < 512 ? Bw : 512; }

// qkv [Bw, N, 3, H, d] (= [Bw, N, 3C]); bias_t [H, N(j), N(i)] fp32 (dense relative-position bias,
// transposed); mask_t [nw, N(j), N(i)] fp32 or null (window bw uses mask bw % nw); o [Bw, N, C]; lse [Bw, H, N]
PDT_API int pdt_win_attn_fwd(const void* qkv, const float* bias_t, const float* mask_t, int nw, void* o, float* lse,
                             int Bw, int N, int H, int d, float scale, int dt, hipStream_t st) {
  if (N > NMAX || d > 32 || H > 16 || N <= 0) return (int)hipErrorInvalidValue;
  const int grid = pdt_win_attn_grid(Bw);
#define PDT_L(T, DP)                                                                                       \
  win_attn_fwd_kernel<T, DP><<<grid, 64 * H, 2 * H * NMAX * DP * sizeof(float), st>>>(                     \
      (const T*)qkv, bias_t, mask_t, nw, (T*)o, lse, Bw, N, H, d, scale)
#define PDT_D(T) \
  if (d <= 4) PDT_L(T, 4); else if (d <= 12) PDT_L(T, 12); else if (d <= 16) PDT_L(T, 16); else PDT_L(T, 32);
  if (dt == kBF16) { PDT_D(bf16_t) } else { PDT_D(float) }
#undef PDT_D
#undef PDT_L
  return (int)hipGetLastError();
}

// dqkv [Bw, N, 3C] (fully written); dbias_part [pdt_win_attn_grid(Bw), H, N, N] fp32 (fully written)
PDT_API int pdt_win_attn_bwd(const void* qkv, const float* bias, const float* bias_t, const float* mask,
                             const float* mask_t, int nw, const void* o, const void* dout, const float* lse,
                             void* dqkv, float* dbias_part, int Bw, int N, int H, int d, float scale, int dt,
                             hipStream_t st) {
  if (N > NMAX || d > 32 || H > 16 || N <= 0) return (int)hipErrorInvalidValue;
  const int grid = pdt_win_attn_grid(Bw);
#define PDT_L(T, DP)                                                                                          \
  win_attn_bwd_kernel<T, DP><<<grid, 64 * H, (4 * H * NMAX * DP + 2 * H * NMAX) * sizeof(float), st>>>(      \
      (const T*)qkv, bias, bias_t, mask, mask_t, nw, (const T*)o, (const T*)dout, lse, (T*)dqkv, dbias_part, Bw, N, \
      H, d, scale)
#define PDT_D(T) \
  if (d <= 4) PDT_L(T, 4); else if (d <= 12) PDT_L(T, 12); else if (d <= 16) PDT_L(T, 16); else PDT_L(T, 32);
  if (dt == kBF16) { PDT_D(bf16_t) } else { PDT_D(float) }
#undef PDT_D
#undef PDT_L
  return (int)hipGetLastError();
}
