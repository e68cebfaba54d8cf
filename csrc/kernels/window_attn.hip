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

// ================================================================================================
// MFMA path (bf16, head_dim <= 16, N <= 64; SwinIR-S: N = 64, d = 10): the window's 64 x 64 score tile
// per head is 4 v_mfma_f32_32x32x16_bf16 (head_dim zero-padded to the K = 16 of one MFMA), with the
// "accumulator as the next MFMA's operand" idiom of flash_attn.hip: scores are produced transposed
// (S^T = K Q^T: lane = query, registers = keys), so the softmax is lane-local plus one xor-32 exchange
// and the probability registers feed O^T = V^T P^T directly (keys in the permuted order
// key = 16 s + 8 (j >> 2) + 4 hh + (j & 3), matched by the gathered V^T operand).  The backward runs a
// lane = query pass (dQ, relative-bias gradient) and a lane = key pass (S recomputed untransposed:
// dK, dV), 40 MFMAs per (window, head).
//
// Workgroup = 64 * H threads (one wave per head, H <= 8: <= 2 waves per SIMD, 256 VGPRs each), grid-strides
// over windows.  LDS holds the window's
// qkv rows (16-B vector staged), the output tile (written back with 16-B stores), and the dense
// relative-position bias of all heads + the window's shift mask as bf16 rows padded to 68 elements
// (34-dword stride: conflict-free 8-byte reads of 4 consecutive entries and 2-byte column reads).  The
// forward stores them row-major ([q][key]: a lane = query reads 4 keys per ds_read_b64); the backward
// stores them transposed ([key][q]) for its lane = key pass (4 queries per read), the pass with 2x the
// lookups.  Masks are a template parameter: the unshifted half of the blocks does no mask lookups.
// ================================================================================================
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

constexpr int BP = 68;   // padded bias / mask row (bf16 elements, 8-byte aligned rows)

__device__ __forceinline__ f32x16 mfma32(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}
// accumulator register r, lane half hh -> row inside the 32 x 32 tile (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }
// token feeding k-element j of the permuted-k operand at k-step s (16 tokens per step), lane half hh
__device__ __forceinline__ int perm_k(int s, int j, int hh) { return 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3); }

// A zero the compiler cannot see through: re-derived per window so the 64+ per-register LDS addresses
// of the bias / mask / lse lookups are not hoisted out of the window loop (that hoist spills VGPRs).
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// row fragment: token t, head columns [off, off + d), elements 8hh .. 8hh+7 (zero past d)
__device__ __forceinline__ u16x8 rowfrag(const u16* s, int t, int stride, int off, int hh, int d) {
  u16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = 8 * hh + i;
    r[i] = e < d ? s[t * stride + off + e] : (u16)0;
  }
  return r;
}
// permuted column fragment (A operand of X^T P^T): row dd of the head slice, tokens perm_k(ks, j, hh)
__device__ __forceinline__ u16x8 colfrag(const u16* s, int ks, int hh, int dd, int stride, int off, int d) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = dd < d ? s[perm_k(ks, j, hh) * stride + off + dd] : (u16)0;
  return r;
}
__device__ __forceinline__ u16x8 pack8(const f32x16& x, int s) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(x[8 * s + j]);
  return r;
}

// stage rows [0, N) of a contiguous [N, width] bf16 block into LDS [64][width], zero rows N..63
__device__ __forceinline__ void stage_rows(const bf16_t* g, u16* s, int N, int width) {
  const int nv = N * width / 8;
  const u16x8* src = reinterpret_cast<const u16x8*>(g);
  for (int i = threadIdx.x; i < nv; i += blockDim.x) reinterpret_cast<u16x8*>(s)[i] = src[i];
  for (int i = N * width + threadIdx.x; i < 64 * width; i += blockDim.x) s[i] = 0;
}
__device__ __forceinline__ void zero_lds(u16* s, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) s[i] = 0;
}
// dense fp32 [mats][N][N] -> bf16 LDS [mats][64][BP] (each matrix padded to 64 rows of BP elements),
// TRANSPOSE: element (row, col) stored at [col][row]
template <bool TRANSPOSE>
__device__ __forceinline__ void stage_bias(const float* g, u16* s, int mats, int N) {
  for (int e = threadIdx.x; e < mats * N * N; e += blockDim.x) {
    const int r = e / N, c = e - r * N;          // r = matrix * N + row
    const int mat = r / N, row = r - mat * N;
    s[(mat * 64 + (TRANSPOSE ? c : row)) * BP + (TRANSPOSE ? row : c)] = f2bf(g[e]);
  }
}
__device__ __forceinline__ u16x4 ld4(const u16* p) { return *reinterpret_cast<const u16x4*>(p); }

template <bool HAS_MASK>
__global__ __launch_bounds__(512) void win_attn_fwd_mfma(const bf16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                         const float* __restrict__ mask, int nw, bf16_t* __restrict__ o,
                                                         float* __restrict__ lse, int Bw, int N, int H, int d,
                                                         float scale) {
  extern __shared__ __attribute__((aligned(16))) u16 smf[];
  const int C = H * d, C3 = 3 * C;
  u16* sq = smf;                       // [64][C3]
  u16* so = sq + 64 * C3;              // [64][C]
  u16* sb = so + 64 * C;               // [H][64][BP]
  u16* sm = sb + H * 64 * BP;          // [64][BP]
  const int lane = threadIdx.x & 63, h = threadIdx.x >> 6, hh = lane >> 5, l32 = lane & 31;
  zero_lds(sb, (H + 1) * 64 * BP);   // bias + mask rows incl. padding
  __syncthreads();
  stage_bias<false>(bias, sb, H, N);
  for (int bw = blockIdx.x; bw < Bw; bw += gridDim.x) {
    __syncthreads();
    stage_rows(qkv + (int64_t)bw * N * C3, sq, N, C3);
    if (HAS_MASK) stage_bias<false>(mask + (int64_t)(bw % nw) * N * N, sm, 1, N);
    __syncthreads();
    u16x8 kf[2], qf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      kf[t] = rowfrag(sq, 32 * t + l32, C3, C + h * d, hh, d);
      qf[t] = rowfrag(sq, 32 * t + l32, C3, h * d, hh, d);
    }
    const int z0 = opaque_zero();
    const u16* bh = sb + h * 64 * BP + z0;
    const u16* smw = sm + z0;
    f32x16 p[2][2];
    float msum[2], mmax[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = 32 * qt + l32;
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        p[qt][kt] = mfma32(kf[kt], qf[qt], zero16());
#pragma unroll
        for (int i = 0; i < 4; ++i) {          // registers 4i..4i+3 = keys base..base+3
          const int base = 32 * kt + 8 * i + 4 * hh;
          const u16x4 bv = ld4(bh + q * BP + base);
          u16x4 mv = {0, 0, 0, 0};
          if (HAS_MASK) mv = ld4(smw + q * BP + base);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * i + j;
            float a = p[qt][kt][r] * scale + bf2f(bv[j]);
            if (HAS_MASK) a += bf2f(mv[j]);
            p[qt][kt][r] = (base + j < N && q < N) ? a : -INFINITY;
            m = fmaxf(m, p[qt][kt][r]);
          }
        }
      }
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float a = p[qt][kt][r];
          const float e = a == -INFINITY ? 0.f : __expf(a - m);
          p[qt][kt][r] = e;
          l += e;
        }
      l += __shfl_xor(l, 32, 64);
      msum[qt] = l;
      mmax[qt] = m;
    }
    u16x8 vt[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) vt[ks] = colfrag(sq, ks, hh, l32, C3, 2 * C + h * d, d);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 acc = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma32(vt[ks], pack8(p[qt][ks >> 1], ks & 1), acc);
      const int q = 32 * qt + l32;
      if (q < N) {
        const float il = 1.f / msum[qt];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dd = acc_row(r, hh);
          if (dd < d) so[q * C + h * d + dd] = f2bf(acc[r] * il);
        }
        if (hh == 0) lse[((int64_t)bw * H + h) * N + q] = mmax[qt] + __logf(msum[qt]);
      }
    }
    __syncthreads();
    u16x8* dst = reinterpret_cast<u16x8*>(o + (int64_t)bw * N * C);
    for (int i = threadIdx.x; i < N * C / 8; i += blockDim.x) dst[i] = reinterpret_cast<const u16x8*>(so)[i];
  }
}

// Backward, split in two launches so neither holds more than one pass's registers (one kernel spilled the
// 64-register relative-bias accumulator):
//   PASS 1 (lane = query, S^T layout): delta = rowsum(dO o O) (written for pass 2), dS^T, dQ, and the
//          relative-bias gradient accumulated in registers across the workgroup's windows;
//   PASS 2 (lane = key, S layout): dV = P^T dO and dK = dS^T Q (S / dP recomputed per sub-pass).
// Each pass writes its own column range of the [N, 3C] dqkv rows (8-byte stores).
template <bool HAS_MASK, int PASS>
__global__ __launch_bounds__(512) void win_attn_bwd_mfma(const bf16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                         const float* __restrict__ mask, int nw,
                                                         const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout,
                                                         const float* __restrict__ lse, float* __restrict__ delta,
                                                         bf16_t* __restrict__ dqkv, float* __restrict__ dbias_part,
                                                         int Bw, int N, int H, int d, float scale) {
  extern __shared__ __attribute__((aligned(16))) u16 smb[];
  const int C = H * d, C3 = 3 * C;
  u16* sq = smb;                        // [64][C3] qkv
  u16* sd = sq + 64 * C3;               // [64][C3] output tile (PASS 1: first [64][C] holds O until delta is formed)
  u16* sg = sd + 64 * C3;               // [64][C] dO
  u16* sb = sg + 64 * C;                // [H][64][BP] bias (PASS 1 row-major [q][key], PASS 2 transposed [key][q])
  u16* sm = sb + H * 64 * BP;           // [64][BP] mask (same layout)
  float* slse = reinterpret_cast<float*>(sm + 64 * BP);   // [H][64]
  float* sdel = slse + H * 64;                            // [H][64]
  constexpr bool TR = PASS == 2;
  const int lane = threadIdx.x & 63, h = threadIdx.x >> 6, hh = lane >> 5, l32 = lane & 31;
  zero_lds(sb, (H + 1) * 64 * BP);
  __syncthreads();
  stage_bias<TR>(bias, sb, H, N);
  f32x16 dsacc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) dsacc[x][y] = zero16();

  for (int bw = blockIdx.x; bw < Bw; bw += gridDim.x) {
    __syncthreads();
    stage_rows(qkv + (int64_t)bw * N * C3, sq, N, C3);
    stage_rows(dout + (int64_t)bw * N * C, sg, N, C);
    if (PASS == 1) stage_rows(o + (int64_t)bw * N * C, sd, N, C);
    if (HAS_MASK) stage_bias<TR>(mask + (int64_t)(bw % nw) * N * N, sm, 1, N);
    if (PASS == 1) __syncthreads();
    {   // lse (both passes), delta = <dO_q, O_q> (pass 1 computes and publishes it, pass 2 reads it)
      float dl = 0.f, ls = INFINITY;
      if (lane < N) {
        const int64_t idx = ((int64_t)bw * H + h) * N + lane;
        ls = lse[idx];
        if (PASS == 1) {
          for (int dd = 0; dd < d; ++dd) dl += bf2f(sg[lane * C + h * d + dd]) * bf2f(sd[lane * C + h * d + dd]);
          delta[idx] = dl;
        } else {
          dl = delta[idx];
        }
      }
      sdel[h * 64 + lane] = dl;
      slse[h * 64 + lane] = ls;
    }
    __syncthreads();
    const int z0 = opaque_zero();
    const float* Lh = slse + h * 64 + z0;
    const float* Dh = sdel + h * 64 + z0;
    const u16* bh = sb + h * 64 * BP + z0;
    const u16* smw = sm + z0;
    const u16* tq = sq + z0;   // per-window views: the fragment addresses are rebuilt, not kept live
    const u16* tg = sg + z0;
    if (PASS == 1) {
      // ---- lane = query (S^T layout) -> dS^T, dQ, relative-bias gradient
      u16x8 ktf[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) ktf[ks] = colfrag(tq, ks, hh, l32, C3, C + h * d, d);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q = 32 * qt + l32;
        const float L = Lh[q], D = Dh[q];
        const u16x8 qf = rowfrag(tq, q, C3, h * d, hh, d);
        const u16x8 gf = rowfrag(tg, q, C, h * d, hh, d);
        u16x8 dsk[4];   // dS^T packed to bf16 as the next MFMA's B operand
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const f32x16 sc = mfma32(rowfrag(tq, 32 * kt + l32, C3, C + h * d, hh, d), qf, zero16());
          const f32x16 dp = mfma32(rowfrag(tq, 32 * kt + l32, C3, 2 * C + h * d, hh, d), gf, zero16());
          f32x16 ds;
#pragma unroll
          for (int i = 0; i < 4; ++i) {        // registers 4i..4i+3 = keys base..base+3
            const int base = 32 * kt + 8 * i + 4 * hh;
            const u16x4 bv = ld4(bh + q * BP + base);
            u16x4 mv = {0, 0, 0, 0};
            if (HAS_MASK) mv = ld4(smw + q * BP + base);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              float a = sc[r] * scale + bf2f(bv[j]);
              if (HAS_MASK) a += bf2f(mv[j]);
              const float v = __expf(a - L) * (dp[r] - D);
              ds[r] = (base + j < N && q < N) ? v : 0.f;
            }
          }
          dsacc[qt][kt] += ds;
          dsk[2 * kt] = pack8(ds, 0);
          dsk[2 * kt + 1] = pack8(ds, 1);
        }
        f32x16 acc = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mfma32(ktf[ks], dsk[ks], acc);
        if (q < N) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int dd = acc_row(r, hh);
            if (dd < d) sd[q * C3 + h * d + dd] = f2bf(acc[r] * scale);
          }
        }
      }
    } else {
      // ---- lane = key (S layout) -> dV = P^T dO (sub-pass 0), dK = dS^T Q (sub-pass 1)
#pragma unroll 1
      for (int it = 0; it < 4; ++it) {
        const int kt = it >> 1, part = it & 1;
        const int key = 32 * kt + l32;
        const int zk = opaque_zero();
        const u16* bk = bh + zk;
        const u16* mk = smw + zk;
        const float* Lk = Lh + zk;
        const float* Dk = Dh + zk;
        const u16* uq = tq + zk;
        const u16* ug = tg + zk;
        const u16x8 kf = rowfrag(uq, key, C3, C + h * d, hh, d);
        const u16x8 vf = rowfrag(uq, key, C3, 2 * C + h * d, hh, d);
        u16x8 opk[4];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const f32x16 sc = mfma32(rowfrag(uq, 32 * qt + l32, C3, h * d, hh, d), kf, zero16());
          const f32x16 dp = mfma32(rowfrag(ug, 32 * qt + l32, C, h * d, hh, d), vf, zero16());
          f32x16 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) {        // registers 4i..4i+3 = queries base..base+3
            const int base = 32 * qt + 8 * i + 4 * hh;
            const u16x4 bv = ld4(bk + key * BP + base);
            u16x4 mv = {0, 0, 0, 0};
            if (HAS_MASK) mv = ld4(mk + key * BP + base);
            const f32x4 L4 = *reinterpret_cast<const f32x4*>(Lk + base);
            const f32x4 D4 = *reinterpret_cast<const f32x4*>(Dk + base);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              float a = sc[r] * scale + bf2f(bv[j]);
              if (HAS_MASK) a += bf2f(mv[j]);
              float pv = __expf(a - L4[j]);
              if (part) pv *= dp[r] - D4[j];
              v[r] = (key < N && base + j < N) ? pv : 0.f;
            }
          }
          opk[2 * qt] = pack8(v, 0);
          opk[2 * qt + 1] = pack8(v, 1);
        }
        f32x16 acc = zero16();
#pragma unroll
        for (int qs = 0; qs < 4; ++qs)
          acc = mfma32(part ? colfrag(uq, qs, hh, l32, C3, h * d, d) : colfrag(ug, qs, hh, l32, C, h * d, d), opk[qs], acc);
        if (key < N) {
          const float mul = part ? scale : 1.f;
          const int off = (part ? C : 2 * C) + h * d;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int dd = acc_row(r, hh);
            if (dd < d) sd[key * C3 + off + dd] = f2bf(acc[r] * mul);
          }
        }
      }
    }
    __syncthreads();
    // write this pass's column range [c0, c1) of the window's dqkv rows (8-byte stores; C % 4 == 0)
    const int c0 = PASS == 1 ? 0 : C, w4 = (PASS == 1 ? C : 2 * C) / 4;
    bf16_t* dst = dqkv + (int64_t)bw * N * C3;
    for (int i = threadIdx.x; i < N * w4; i += blockDim.x) {
      const int t = i / w4, c = c0 + (i - t * w4) * 4;
      *reinterpret_cast<u16x4*>(dst + t * C3 + c) = *reinterpret_cast<const u16x4*>(sd + t * C3 + c);
    }
  }
  if (PASS == 1) {
    // relative-position-bias gradient partial [H][N(q)][N(key)] of this workgroup
    float* dstb = dbias_part + ((int64_t)blockIdx.x * H + h) * N * N;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = 32 * qt + l32;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = 32 * kt + acc_row(r, hh);
          if (q < N && key < N) dstb[q * N + key] = dsacc[qt][kt][r];
        }
    }
  }
}

size_t fwd_mfma_lds(int N, int H, int d) { const int C = H * d; return (size_t)2 * (64 * 3 * C + 64 * C + (H + 1) * 64 * BP); }
size_t bwd_mfma_lds(int N, int H, int d) {
  const int C = H * d;
  return (size_t)2 * (2 * 64 * 3 * C + 64 * C + (H + 1) * 64 * BP) + (size_t)2 * H * 64 * sizeof(float);
}
bool mfma_ok(int N, int H, int d, int dt) {
  return dt == kBF16 && d <= 16 && N <= 64 && (N * H * d) % 8 == 0 && (H * d) % 4 == 0 && H <= 8 &&
         bwd_mfma_lds(N, H, d) <= 160 * 1024;
}

}  // namespace

// grid size the launcher uses (also the number of dbias partials the caller must allocate)
PDT_API int pdt_win_attn_grid(int Bw) { return Bw < 512 ? Bw : 512; }

// ---- MFMA path: bias [H, N(q), N(key)] fp32 (dense relative-position bias), mask [nw, N, N] fp32 or null
PDT_API int pdt_win_attn_mfma_ok(int N, int H, int d, int dt) { return mfma_ok(N, H, d, dt) ? 1 : 0; }
// one workgroup per CU (LDS-bound), grid-stride over windows; also the dbias partial count
PDT_API int pdt_win_attn_mfma_grid(int Bw) { return Bw < 256 ? Bw : 256; }

PDT_API int pdt_win_attn_mfma_fwd(const void* qkv, const float* bias, const float* mask, int nw, void* o, float* lse,
                                  int Bw, int N, int H, int d, float scale, hipStream_t st) {
  if (!mfma_ok(N, H, d, kBF16) || N <= 0 || Bw <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = fwd_mfma_lds(N, H, d);
  static bool attr = [] {
    return hipFuncSetAttribute((const void*)win_attn_fwd_mfma<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024) == hipSuccess &&
           hipFuncSetAttribute((const void*)win_attn_fwd_mfma<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024) == hipSuccess;
  }();
  (void)attr;
  if (mask)
    win_attn_fwd_mfma<true><<<pdt_win_attn_mfma_grid(Bw), 64 * H, lds, st>>>((const bf16_t*)qkv, bias, mask, nw,
                                                                             (bf16_t*)o, lse, Bw, N, H, d, scale);
  else
    win_attn_fwd_mfma<false><<<pdt_win_attn_mfma_grid(Bw), 64 * H, lds, st>>>((const bf16_t*)qkv, bias, mask, nw,
                                                                              (bf16_t*)o, lse, Bw, N, H, d, scale);
  return (int)hipGetLastError();
}

// dqkv [Bw, N, 3C] fully written; dbias_part [pdt_win_attn_mfma_grid(Bw), H, N, N] fp32 fully written;
// delta_ws [Bw, H, N] fp32 scratch (pass 1 -> pass 2)
PDT_API int pdt_win_attn_mfma_bwd(const void* qkv, const float* bias, const float* mask, int nw, const void* o,
                                  const void* dout, const float* lse, float* delta_ws, void* dqkv, float* dbias_part,
                                  int Bw, int N, int H, int d, float scale, hipStream_t st) {
  if (!mfma_ok(N, H, d, kBF16) || N <= 0 || Bw <= 0) return (int)hipErrorInvalidValue;
  const size_t lds = bwd_mfma_lds(N, H, d);
  static bool attr = [] {
    bool ok = true;
    const void* fns[4] = {(const void*)win_attn_bwd_mfma<true, 1>, (const void*)win_attn_bwd_mfma<true, 2>,
                          (const void*)win_attn_bwd_mfma<false, 1>, (const void*)win_attn_bwd_mfma<false, 2>};
    for (const void* f : fns)
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
  }();
  (void)attr;
#define PDT_WB(M, P)                                                                                        \
  win_attn_bwd_mfma<M, P><<<pdt_win_attn_mfma_grid(Bw), 64 * H, lds, st>>>(                                 \
      (const bf16_t*)qkv, bias, mask, nw, (const bf16_t*)o, (const bf16_t*)dout, lse, delta_ws, (bf16_t*)dqkv, \
      dbias_part, Bw, N, H, d, scale)
  if (mask) { PDT_WB(true, 1); PDT_WB(true, 2); }
  else { PDT_WB(false, 1); PDT_WB(false, 2); }
#undef PDT_WB
  return (int)hipGetLastError();
}

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
