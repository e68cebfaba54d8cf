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
// Two implementations.  bf16 with an even head_dim <= 16 (SwinIR-S: N = 64, d = 10) runs the MFMA kernels
// at the end of this file (one wave per (window, head), see the comment there).  Everything else
// (fp32, odd or > 16 head dims, d <= 32) runs the VALU kernels below in fp32: one wave per head, one
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
// MFMA path (bf16, even head_dim D <= 16, N <= 64; SwinIR-S: N = 64, D = 10).  ONE WAVE PER (window, head):
// a workgroup is 4 waves working on the same head h (its relative-position bias staged once in LDS, as
// bf16 rows padded to BP), each wave grid-strides over windows on its own -- no workgroup barrier in the
// window loop, so one wave's global loads overlap the other waves' MFMA/softmax work.  Per window a lane
// = token stages its d-wide Q/K/V(/dO) slices (dword loads straight from the fused [Bw, N, 3C] rows) into
// the wave's private LDS tiles:
//   row tiles  R[64][16] (dims >= D zero)          -> one ds_read_b128 per MFMA operand fragment
//   transposed T[17][TP] (rows D..16 zero)          -> two ds_read_b64 per permuted-k X^T fragment
// The 64 x 64 score tile is 4 v_mfma_f32_32x32x16_bf16 (head dim zero-padded to the MFMA K = 16), computed
// transposed (S^T = K Q^T: lane = query, registers = keys) so the softmax is lane-local plus one xor-32
// exchange and the probability registers feed O^T = V^T P^T directly (keys in the permuted order
// key = 16 s + 8 (j >> 2) + 4 hh + (j & 3), matched by the transposed-tile fragment).  Outputs go straight
// from the accumulators to global memory (4 consecutive head dims per register group = 2 dword stores).
// Backward, per (window, head) in one wave: delta = rowsum(dO o O) at staging time; pass 1 (lane = query):
// dS^T, dQ, dS accumulated in registers for the relative-bias gradient; pass 2 (lane = key): S / dP
// recomputed untransposed, P and dS packed in one sweep, dV = P^T dO and dK = dS^T Q.  40 MFMAs per
// (window, head).  The shift mask ([nw, N, N] fp32, shared by every head and image) is read from global
// memory (L2-resident) only by the masked half of the blocks (template parameter).
// ================================================================================================
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int BP = 68;       // padded bias row (bf16): conflict-free 8-byte reads of 4 consecutive entries
constexpr int TP = 68;       // transposed-tile row pitch (tokens)
constexpr int TT = 17 * TP;  // transposed tile: rows 0..15 = head dims, row 16 = zeros for lanes dd >= 16
constexpr int WA_NT = 256;   // 4 waves per workgroup
constexpr int FWD_WAVE = 2 * 1024 + TT + 4 + 32;              // QR, KR, VT (u16, padded to 16 B), 64 B labels
constexpr int BWD_WAVE = 4 * 1024 + 256 + 2 * TT + 4 + 32;    // QR KR VR GR, SL SD (fp32), 2 transposed, labels
// Shift-mask modes (template MK): 0 none, 1 dense fp32 mask [nw, N, N] read from L2, 2 region labels
// [nw, N] uint8 -- Swin's mask is -100 exactly where the query's and key's image regions differ, so the
// kernel rebuilds it from 64 label bytes per window staged in LDS (one 4-byte read per 4 keys) instead of
// reading 16 KB of fp32 mask per window and head.
// q / k / v / dO addressing of the MFMA kernels (element strides inside one window's block, which starts at
// bw * N * 3C for qkv and bw * N * C for dO in both layouts):
//   token-major (the projection's output [Bw, N, 3, H, d]): qT = 3C, qH = d, qW = C;  gT = C, gH = d
//   head-major ([Bw, 3, H, N, d], written by the forward; dO [Bw, H, N, d], pdt_win_bwd_prep): qT = d, qH = N d,
//   qW = H N d;  gT = d, gH = N d -- one head's 64 token slices are then one contiguous 64 d-element run, so a
//   wave's staging loads touch ~10 lines per instruction instead of 64 (the per-lane strided slices were ~40 % of
//   the bf16 kernels' time, profiles/r6/r6p_window_attn_staging_ab.txt).
// delta: rowsum(dO o O) per (window, head, token) precomputed by pdt_win_bwd_prep (null: the backward computes it
// from O while staging).
// dQ / dK / dV are always written token-major (the qkv projection's backward reads them); O is written token-major
// ([Bw, N, C]: oT = C, oH = d) or head-major ([Bw, H, N, d]: oT = d, oH = N d) for a projection that reads it so
// (ops.linear.linear_from_head_major): one head's 64 token slices then leave as one contiguous run.
#define WA_DQKV_ADDR(p, bw, t, w) ((p) + ((int64_t)(bw) * N + (t)) * C3 + (w) * C + h * D)
#define WA_O_ADDR(p, bw, t) ((p) + (int64_t)(bw) * N * C + (t) * LY.oT + h * LY.oH)
struct WaLayout {
  int qT, qH, qW, gT, gH, oT, oH;
  const float* delta;
};
__device__ __forceinline__ f32x4 label_mask(const uint8_t* lab, int base, uint32_t mine) {
  const uint32_t four = *reinterpret_cast<const uint32_t*>(lab + base);
  f32x4 m;
#pragma unroll
  for (int j = 0; j < 4; ++j) m[j] = ((four >> (8 * j)) & 0xffu) != mine ? -100.f : 0.f;
  return m;
}

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
__device__ __forceinline__ u16x8 pack8(const f32x16& x, int s) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(x[8 * s + j]);
  return r;
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}
__device__ __forceinline__ u16x4 ld4(const u16* p) { return *reinterpret_cast<const u16x4*>(p); }
// order this wave's LDS writes before its (cross-lane) reads: LDS executes a wave's instructions in order,
// so only the compiler has to be stopped from moving them
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

template <int D>
struct Slice {
  uint32_t v[D / 2];
  __device__ __forceinline__ void load(const bf16_t* p) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < D / 2; ++i) v[i] = s[i];
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < D / 2; ++i) v[i] = 0u;
  }
  __device__ __forceinline__ void store(bf16_t* p) const {
    uint32_t* d = reinterpret_cast<uint32_t*>(p);
#pragma unroll
    for (int i = 0; i < D / 2; ++i) d[i] = v[i];
  }
  __device__ __forceinline__ float f(int e) const { return bf2f((u16)(v[e >> 1] >> (16 * (e & 1)))); }
  // row tile R[64][16]: token t's 16 dims (zero past D) as two 16-byte stores
  __device__ __forceinline__ void put_row(u16* R, int t) const {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = i < D / 2 ? v[i] : 0u;
    u32x4* dst = reinterpret_cast<u32x4*>(R + t * 16);
    dst[0] = u32x4{w[0], w[1], w[2], w[3]};
    dst[1] = u32x4{w[4], w[5], w[6], w[7]};
  }
  // transposed tile T[dd][t]
  __device__ __forceinline__ void put_col(u16* T, int t) const {
#pragma unroll
    for (int dd = 0; dd < D; ++dd) T[dd * TP + t] = (u16)(v[dd >> 1] >> (16 * (dd & 1)));
  }
};

// B/A operand fragment of a row tile: token t, dims 8hh .. 8hh+7
__device__ __forceinline__ u16x8 rfrag(const u16* R, int t, int hh) {
  return *reinterpret_cast<const u16x8*>(R + t * 16 + 8 * hh);
}
// A operand X^T for k-step ks: lane row = head dim dd (dd >= 16 -> zero row 16), k = permuted tokens
__device__ __forceinline__ u16x8 tfrag(const u16* T, int ks, int hh, int dd) {
  const u16* row = T + (dd < 16 ? dd : 16) * TP + 16 * ks + 4 * hh;
  const u16x4 a = ld4(row), b = ld4(row + 8);
  return u16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
// D-wide output row from an O^T-layout accumulator (register r = dim acc_row(r, hh), lane = token)
template <int D>
__device__ __forceinline__ void store_dims(bf16_t* row, const f32x16& acc, float mul, int hh) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int dim = 8 * g + 4 * hh + 2 * pr;
      if (dim < D)
        *reinterpret_cast<uint32_t*>(row + dim) = pack2(acc[4 * g + 2 * pr] * mul, acc[4 * g + 2 * pr + 1] * mul);
    }
}
// bias [N][N] fp32 of one head -> bf16 LDS [64][BP] (TRANSPOSE: [key][q]), zero padded
template <bool TRANSPOSE>
__device__ __forceinline__ void stage_bias(const float* g, u16* s, int N) {
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
    const int r = e >> 6, c = e & 63;
    const u16 v = (r < N && c < N) ? f2bf(g[r * N + c]) : (u16)0;
    s[(TRANSPOSE ? c : r) * BP + (TRANSPOSE ? r : c)] = v;
  }
}

template <int D, int MK, bool FULL>
__global__ __launch_bounds__(WA_NT, 2) void win_attn_fwd_mfma(const bf16_t* __restrict__ qkv,
                                                               const float* __restrict__ bias,
                                                               const float* __restrict__ mask,
                                                               const uint8_t* __restrict__ labels, int nw,
                                                               bf16_t* __restrict__ o, float* __restrict__ lse, int Bw,
                                                               int N, int H, float scale, int P, WaLayout LY,
                                                               bf16_t* __restrict__ hm_out) {
  extern __shared__ __attribute__((aligned(16))) u16 smf[];
  const int C = H * D, C3 = 3 * C;
  const int h = blockIdx.x % H, pb = blockIdx.x / H;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hh = lane >> 5, l32 = lane & 31;
  u16* BR = smf;                                    // [64][BP] bias of head h, [q][key]
  u16* QR = smf + 64 * BP + wv * FWD_WAVE;          // this wave's tiles
  u16* KR = QR + 1024;
  u16* VT = KR + 1024;
  uint8_t* LAB = reinterpret_cast<uint8_t*>(VT + TT + 4);
  stage_bias<false>(bias + (int64_t)h * N * N, BR, N);
  for (int e = lane; e < TT; e += 64) VT[e] = 0;
  __syncthreads();

  for (int bw = pb * 4 + wv; bw < Bw; bw += P * 4) {
    {
      Slice<D> q, k, v;
      if (lane < N) {
        const bf16_t* row = qkv + (int64_t)bw * N * C3 + lane * LY.qT + h * LY.qH;
        q.load(row); k.load(row + LY.qW); v.load(row + 2 * LY.qW);
        if (hm_out != nullptr) {   // the backward's head-major copy, from the slices already in registers
          bf16_t* hp = hm_out + (((int64_t)bw * 3 * H + h) * N + lane) * D;
          q.store(hp); k.store(hp + (int64_t)H * N * D); v.store(hp + 2 * (int64_t)H * N * D);
        }
      } else {
        q.zero(); k.zero(); v.zero();
      }
      q.put_row(QR, lane); k.put_row(KR, lane); v.put_col(VT, lane);
      if (MK == 2) LAB[lane] = lane < N ? labels[(int64_t)(bw % nw) * N + lane] : (uint8_t)255;
    }
    wave_sync();
    const float* mw = MK == 1 ? mask + (int64_t)(bw % nw) * N * N : nullptr;
    u16x8 kf[2], qf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      kf[t] = rfrag(KR, 32 * t + l32, hh);
      qf[t] = rfrag(QR, 32 * t + l32, hh);
    }
    f32x16 p[2][2];
    float lsum[2], mmax[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = 32 * qt + l32;
      const int qc = FULL ? q : min(q, N - 1);
      const uint32_t qlab = MK == 2 ? LAB[q] : 0u;
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        p[qt][kt] = mfma32(kf[kt], qf[qt], zero16());
#pragma unroll
        for (int i = 0; i < 4; ++i) {          // registers 4i..4i+3 = keys base..base+3
          const int base = 32 * kt + 8 * i + 4 * hh;
          const u16x4 bv = ld4(BR + q * BP + base);
          f32x4 mv = {0.f, 0.f, 0.f, 0.f};
          if (MK == 2) {
            mv = label_mask(LAB, base, qlab);
          } else if (MK == 1) {
            if (FULL) {
              mv = *reinterpret_cast<const f32x4*>(mw + q * 64 + base);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) mv[j] = base + j < N ? mw[qc * N + base + j] : 0.f;
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * i + j;
            float a = fmaf(p[qt][kt][r], scale, bf2f(bv[j]) + mv[j]);
            if (!FULL) a = (base + j < N && q < N) ? a : -INFINITY;
            p[qt][kt][r] = a;
            m = fmaxf(m, a);
          }
        }
      }
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      const float msub = m == -INFINITY ? 0.f : m;
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __expf(p[qt][kt][r] - msub);
          p[qt][kt][r] = e;
          l += e;
        }
      l += __shfl_xor(l, 32, 64);
      lsum[qt] = l;
      mmax[qt] = msub;
    }
    u16x8 vt[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) vt[ks] = tfrag(VT, ks, hh, l32);
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      f32x16 acc = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc = mfma32(vt[ks], pack8(p[qt][ks >> 1], ks & 1), acc);
      const int q = 32 * qt + l32;
      if (FULL || q < N) {
        store_dims<D>(WA_O_ADDR(o, bw, q), acc, 1.f / lsum[qt], hh);
        if (hh == 0) lse[((int64_t)bw * H + h) * N + q] = mmax[qt] + __logf(lsum[qt]);
      }
    }
    wave_sync();
  }
}

// Backward pass PASS (1: dQ + relative-bias gradient, lane = query; 2: dK, dV, lane = key).  Two launches
// rather than one so neither holds the other's registers (the 64-register bias-gradient accumulator of
// pass 1 next to pass 2's P / dS tiles spilled).  Both recompute delta = rowsum(dO o O) while staging.
template <int D, int MK, bool FULL, int PASS>
__global__ __launch_bounds__(WA_NT, 2) void win_attn_bwd_mfma(
    const bf16_t* __restrict__ qkv, const float* __restrict__ bias, const float* __restrict__ mask,
    const uint8_t* __restrict__ labels, int nw,
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    bf16_t* __restrict__ dqkv, float* __restrict__ dbias_part, int Bw, int N, int H, float scale, int P, WaLayout LY) {
  extern __shared__ __attribute__((aligned(16))) u16 smb[];
  const int C = H * D, C3 = 3 * C;
  const int h = blockIdx.x % H, pb = blockIdx.x / H;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hh = lane >> 5, l32 = lane & 31;
  u16* BB = smb;                        // [64][BP] bias: pass 1 [q][key], pass 2 [key][q]
  u16* QR = BB + 64 * BP + wv * BWD_WAVE;
  u16* KR = QR + 1024;
  u16* VR = KR + 1024;
  u16* GR = VR + 1024;
  float* SL = reinterpret_cast<float*>(GR + 1024);   // [64] lse
  float* SD = SL + 64;                               // [64] delta
  u16* T0 = GR + 1024 + 256;                         // pass 1: K^T; pass 2: Q^T
  u16* T1 = T0 + TT;                                 // pass 2: dO^T
  uint8_t* LAB = reinterpret_cast<uint8_t*>(T1 + TT + 4);
  stage_bias<PASS == 2>(bias + (int64_t)h * N * N, BB, N);
  for (int e = lane; e < 2 * TT; e += 64) T0[e] = 0;
  __syncthreads();
  f32x16 dsacc[2][2];
  if (PASS == 1) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) dsacc[x][y] = zero16();
  }

  for (int bw = pb * 4 + wv; bw < Bw; bw += P * 4) {
    {
      Slice<D> q, k, v, g, oo;
      float L = 0.f, dl = 0.f;
      if (lane < N) {
        const int64_t tok = (int64_t)bw * N + lane;
        const bf16_t* row = qkv + (int64_t)bw * N * C3 + lane * LY.qT + h * LY.qH;
        q.load(row); k.load(row + LY.qW); v.load(row + 2 * LY.qW);
        g.load(dout + (int64_t)bw * N * C + lane * LY.gT + h * LY.gH);
        L = lse[((int64_t)bw * H + h) * N + lane];
        if (LY.delta != nullptr) {
          dl = LY.delta[((int64_t)bw * H + h) * N + lane];
        } else {
          oo.load(o + tok * C + h * D);
#pragma unroll
          for (int e = 0; e < D; ++e) dl = fmaf(g.f(e), oo.f(e), dl);
        }
      } else {
        q.zero(); k.zero(); v.zero(); g.zero();
      }
      q.put_row(QR, lane); k.put_row(KR, lane); v.put_row(VR, lane); g.put_row(GR, lane);
      if (PASS == 1) {
        k.put_col(T0, lane);
      } else {
        q.put_col(T0, lane);
        g.put_col(T1, lane);
      }
      SL[lane] = L;
      SD[lane] = dl;
      if (MK == 2) LAB[lane] = lane < N ? labels[(int64_t)(bw % nw) * N + lane] : (uint8_t)255;
    }
    wave_sync();
    const float* mw = MK == 1 ? mask + (int64_t)(bw % nw) * N * N : nullptr;
    if (PASS == 1) {
      // lane = query (S^T layout): dS^T, dQ = dS K * scale, dS summed for the bias gradient
      u16x8 ktf[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) ktf[ks] = tfrag(T0, ks, hh, l32);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q = 32 * qt + l32;
        const int qc = FULL ? q : min(q, N - 1);
        const float Lq = SL[q], Dq = SD[q];
        const uint32_t qlab = MK == 2 ? LAB[q] : 0u;
        const u16x8 qf = rfrag(QR, q, hh), gf = rfrag(GR, q, hh);
        u16x8 dsk[4];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const f32x16 sc = mfma32(rfrag(KR, 32 * kt + l32, hh), qf, zero16());
          const f32x16 dp = mfma32(rfrag(VR, 32 * kt + l32, hh), gf, zero16());
          f32x16 ds;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int base = 32 * kt + 8 * i + 4 * hh;
            const u16x4 bv = ld4(BB + q * BP + base);
            f32x4 mv = {0.f, 0.f, 0.f, 0.f};
            if (MK == 2) {
              mv = label_mask(LAB, base, qlab);
            } else if (MK == 1) {
              if (FULL) {
                mv = *reinterpret_cast<const f32x4*>(mw + q * 64 + base);
              } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) mv[j] = base + j < N ? mw[qc * N + base + j] : 0.f;
              }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              const float a = fmaf(sc[r], scale, bf2f(bv[j]) + mv[j]);
              float v = __expf(a - Lq) * (dp[r] - Dq);
              if (!FULL) v = (base + j < N && q < N) ? v : 0.f;
              ds[r] = v;
            }
          }
          dsacc[qt][kt] += ds;
          dsk[2 * kt] = pack8(ds, 0);
          dsk[2 * kt + 1] = pack8(ds, 1);
        }
        f32x16 acc = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mfma32(ktf[ks], dsk[ks], acc);
        if (FULL || q < N) store_dims<D>(WA_DQKV_ADDR(dqkv, bw, q, 0), acc, scale, hh);
      }
    } else {
      // lane = key (S layout): P and dS in one sweep; dV = P^T dO, dK = dS^T Q * scale
#pragma unroll 1
      for (int kt = 0; kt < 2; ++kt) {
        const int key = 32 * kt + l32;
        const int kc = FULL ? key : min(key, N - 1);
        const u16x8 kf = rfrag(KR, key, hh), vf = rfrag(VR, key, hh);
        const uint32_t klab = MK == 2 ? LAB[key] : 0u;
        f32x16 av = zero16(), ak = zero16();
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const f32x16 sc = mfma32(rfrag(QR, 32 * qt + l32, hh), kf, zero16());
          const f32x16 dp = mfma32(rfrag(GR, 32 * qt + l32, hh), vf, zero16());
          f32x16 pv, dv;
#pragma unroll
          for (int i = 0; i < 4; ++i) {        // registers 4i..4i+3 = queries base..base+3
            const int base = 32 * qt + 8 * i + 4 * hh;
            const u16x4 bv = ld4(BB + key * BP + base);
            const f32x4 L4 = *reinterpret_cast<const f32x4*>(SL + base);
            const f32x4 D4 = *reinterpret_cast<const f32x4*>(SD + base);
            f32x4 mv = {0.f, 0.f, 0.f, 0.f};
            if (MK == 2) {
              mv = label_mask(LAB, base, klab);        // the 4 queries' labels vs this lane's key
            } else if (MK == 1) {
#pragma unroll
              for (int j = 0; j < 4; ++j) mv[j] = (FULL || base + j < N) ? mw[(base + j) * N + kc] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              const float a = fmaf(sc[r], scale, bf2f(bv[j]) + mv[j]);
              float e = __expf(a - L4[j]);
              if (!FULL) e = (key < N && base + j < N) ? e : 0.f;
              pv[r] = e;
              dv[r] = e * (dp[r] - D4[j]);
            }
          }
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            av = mfma32(tfrag(T1, 2 * qt + s2, hh, l32), pack8(pv, s2), av);
            ak = mfma32(tfrag(T0, 2 * qt + s2, hh, l32), pack8(dv, s2), ak);
          }
        }
        if (FULL || key < N) {
          store_dims<D>(WA_DQKV_ADDR(dqkv, bw, key, 1), ak, scale, hh);
          store_dims<D>(WA_DQKV_ADDR(dqkv, bw, key, 2), av, 1.f, hh);
        }
      }
    }
    wave_sync();
  }
  if (PASS == 1) {
    // relative-position-bias gradient of this workgroup's windows: the 4 waves' tiles summed in LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(BB + 64 * BP);    // [64][64] over the wave tiles
    for (int e = threadIdx.x; e < 64 * 64; e += WA_NT) red[e] = 0.f;
    __syncthreads();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          atomicAdd(red + (32 * qt + l32) * 64 + 32 * kt + acc_row(r, hh), dsacc[qt][kt][r]);
    __syncthreads();
    float* dst = dbias_part + ((int64_t)pb * H + h) * N * N;
    for (int e = threadIdx.x; e < N * N; e += WA_NT) dst[e] = red[(e / N) * 64 + e % N];
  }
}

size_t fwd_mfma_lds() { return (size_t)2 * (64 * BP + 4 * FWD_WAVE); }
size_t bwd_mfma_lds() { return (size_t)2 * (64 * BP + 4 * BWD_WAVE); }
bool mfma_ok(int N, int H, int d, int dt) {
  return dt == kBF16 && d >= 2 && d <= 16 && d % 2 == 0 && N >= 1 && N <= 64 && H >= 1;
}
// workgroups per head: 4 waves each, ~`per_cu` workgroups per CU over all heads
int mfma_blocks_per_head(int Bw, int H, int per_cu) {
  const int want = (256 * per_cu) / H;
  const int need = (Bw + 3) / 4;
  return need < want ? need : (want > 0 ? want : 1);
}


// ================================================================================================
// fp32 MFMA path -- the reference's own precision (Stoke-DDP.py:247 trains SwinIR with fp16=None).  gfx950 has
// f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32, an fmaf chain per output, 64 FLOP/clk/SIMD) and no xf32, so
// these kernels keep full fp32 numerics while moving every product off the VALU.  Same structure as the bf16
// kernels above -- one wave per (window, head), scores transposed (lane = query, registers = keys), the two-pass
// backward -- with fp32 operands: a 32x32x2 fragment is ONE float per lane (A[row = l & 31][k = l >> 5],
// B[k = l >> 5][col = l & 31]), read straight from per-wave LDS row tiles R[64][D + 1] (odd pitch for D even:
// the 32 rows of a fragment hit distinct banks).  Products whose k runs over keys take the accumulator registers
// as the B operand in the permuted key order key = acc_row(r, hh), and their A operand from the same row tile at
// [key][min(l32, D)] -- column D is kept zero, so output rows (head dims) >= D come out zero for free.
// ================================================================================================
constexpr int BPF = 68;      // fp32 bias row pitch: 16-byte reads of 4 consecutive keys

__device__ __forceinline__ f32x16 mfma2(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
template <int D> constexpr int f32_fwd_wave() { return 3 * 64 * (D + 1) + 16; }          // Q K V tiles, labels
template <int D> constexpr int f32_bwd_wave() { return 4 * 64 * (D + 1) + 128 + 16; }    // Q K V dO, L, delta, labels
template <int D> size_t f32_fwd_lds() { return sizeof(float) * (64 * BPF + 4 * f32_fwd_wave<D>()); }
// (the wave tiles double as the [64][64] bias-gradient reduction area at the end of pass 1)
template <int D> size_t f32_bwd_lds() {
  return sizeof(float) * (64 * BPF + (4 * f32_bwd_wave<D>() > 64 * 64 ? 4 * f32_bwd_wave<D>() : 64 * 64));
}

template <int D>
struct RowF {
  float v[D];
  __device__ __forceinline__ void load(const float* p) {      // 8-byte aligned: row offsets and D are even
    const float2* s = reinterpret_cast<const float2*>(p);
#pragma unroll
    for (int i = 0; i < D / 2; ++i) {
      const float2 x = s[i];
      v[2 * i] = x.x;
      v[2 * i + 1] = x.y;
    }
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < D; ++i) v[i] = 0.f;
  }
  __device__ __forceinline__ void store(float* p) const {
    float2* d = reinterpret_cast<float2*>(p);
#pragma unroll
    for (int i = 0; i < D / 2; ++i) d[i] = float2{v[2 * i], v[2 * i + 1]};
  }
  __device__ __forceinline__ void put(float* R, int t) const {
    float* d = R + t * (D + 1);
#pragma unroll
    for (int i = 0; i < D; ++i) d[i] = v[i];
    d[D] = 0.f;
  }
};
// D-wide fp32 output row from an O^T-layout accumulator (register r = dim acc_row(r, hh), lane = token)
template <int D>
__device__ __forceinline__ void store_dims_f32(float* row, const f32x16& acc, float mul, int hh) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int dim = 8 * g + 4 * hh + 2 * pr;
      if (dim < D) *reinterpret_cast<float2*>(row + dim) = float2{acc[4 * g + 2 * pr] * mul, acc[4 * g + 2 * pr + 1] * mul};
    }
}
template <bool TRANSPOSE>
__device__ __forceinline__ void stage_bias_f32(const float* g, float* s, int N) {
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
    const int r = e >> 6, c = e & 63;
    s[(TRANSPOSE ? c : r) * BPF + (TRANSPOSE ? r : c)] = (r < N && c < N) ? g[r * N + c] : 0.f;
  }
}
// S^T (or S) tile over the head dim: sum_s A[ra][2s + hh] B[rb][2s + hh]
template <int D>
__device__ __forceinline__ f32x16 dot_tile(const float* RA, int ra, const float* RB, int rb, int hh) {
  f32x16 acc = zero16();
#pragma unroll
  for (int s = 0; s < D / 2; ++s) acc = mfma2(RA[ra * (D + 1) + 2 * s + hh], RB[rb * (D + 1) + 2 * s + hh], acc);
  return acc;
}

template <int D, int MK, bool FULL>
__global__ __launch_bounds__(WA_NT, 2) void win_attn_fwd_f32(const float* __restrict__ qkv, const float* __restrict__ bias,
                                                             const float* __restrict__ mask,
                                                             const uint8_t* __restrict__ labels, int nw,
                                                             float* __restrict__ o, float* __restrict__ lse, int Bw,
                                                             int N, int H, float scale, int P, WaLayout LY,
                                                             float* __restrict__ hm_out) {
  extern __shared__ __attribute__((aligned(16))) float smf32[];
  constexpr int RP = D + 1;
  const int C = H * D, C3 = 3 * C;
  const int h = blockIdx.x % H, pb = blockIdx.x / H;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hh = lane >> 5, l32 = lane & 31;
  const int dcl = l32 < D ? l32 : D;
  float* BR = smf32;                                      // [64][BPF] bias of head h, [q][key]
  float* QR = smf32 + 64 * BPF + wv * f32_fwd_wave<D>();
  float* KR = QR + 64 * RP;
  float* VR = KR + 64 * RP;
  uint8_t* LAB = reinterpret_cast<uint8_t*>(VR + 64 * RP);
  stage_bias_f32<false>(bias + (int64_t)h * N * N, BR, N);
  __syncthreads();

  for (int bw = pb * 4 + wv; bw < Bw; bw += P * 4) {
    {
      RowF<D> q, k, v;
      if (lane < N) {
        const float* row = qkv + (int64_t)bw * N * C3 + lane * LY.qT + h * LY.qH;
        q.load(row); k.load(row + LY.qW); v.load(row + 2 * LY.qW);
        if (hm_out != nullptr) {   // the backward's head-major copy, from the slices already in registers
          float* hp = hm_out + (((int64_t)bw * 3 * H + h) * N + lane) * D;
          q.store(hp); k.store(hp + (int64_t)H * N * D); v.store(hp + 2 * (int64_t)H * N * D);
        }
      } else {
        q.zero(); k.zero(); v.zero();
      }
      q.put(QR, lane); k.put(KR, lane); v.put(VR, lane);
      if (MK == 2) LAB[lane] = lane < N ? labels[(int64_t)(bw % nw) * N + lane] : (uint8_t)255;
    }
    wave_sync();
    const float* mw = MK == 1 ? mask + (int64_t)(bw % nw) * N * N : nullptr;
    f32x16 p[2][2];
    float lsum[2], mmax[2];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = 32 * qt + l32;
      const int qc = FULL ? q : min(q, N - 1);
      const uint32_t qlab = MK == 2 ? LAB[q] : 0u;
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        p[qt][kt] = dot_tile<D>(KR, 32 * kt + l32, QR, q, hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) {          // registers 4i..4i+3 = keys base..base+3
          const int base = 32 * kt + 8 * i + 4 * hh;
          const f32x4 bv = *reinterpret_cast<const f32x4*>(BR + q * BPF + base);
          f32x4 mv = {0.f, 0.f, 0.f, 0.f};
          if (MK == 2) {
            mv = label_mask(LAB, base, qlab);
          } else if (MK == 1) {
            if (FULL) {
              mv = *reinterpret_cast<const f32x4*>(mw + q * 64 + base);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) mv[j] = base + j < N ? mw[qc * N + base + j] : 0.f;
            }
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * i + j;
            float a = fmaf(p[qt][kt][r], scale, bv[j] + mv[j]);
            if (!FULL) a = (base + j < N && q < N) ? a : -INFINITY;
            p[qt][kt][r] = a;
            m = fmaxf(m, a);
          }
        }
      }
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      const float msub = m == -INFINITY ? 0.f : m;
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __expf(p[qt][kt][r] - msub);
          p[qt][kt][r] = e;
          l += e;
        }
      l += __shfl_xor(l, 32, 64);
      lsum[qt] = l;
      mmax[qt] = msub;
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      // O^T = V^T P^T: k runs over the keys in the accumulator order (lane half hh supplies key acc_row(r, hh))
      f32x16 acc = zero16();
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc = mfma2(VR[(32 * kt + acc_row(r, hh)) * RP + dcl], p[qt][kt][r], acc);
      const int q = 32 * qt + l32;
      if (FULL || q < N) {
        store_dims_f32<D>(WA_O_ADDR(o, bw, q), acc, 1.f / lsum[qt], hh);
        if (hh == 0) lse[((int64_t)bw * H + h) * N + q] = mmax[qt] + __logf(lsum[qt]);
      }
    }
    wave_sync();
  }
}

template <int D, int MK, bool FULL, int PASS>
__global__ __launch_bounds__(WA_NT, 2) void win_attn_bwd_f32(
    const float* __restrict__ qkv, const float* __restrict__ bias, const float* __restrict__ mask,
    const uint8_t* __restrict__ labels, int nw,
    const float* __restrict__ o, const float* __restrict__ dout, const float* __restrict__ lse,
    float* __restrict__ dqkv, float* __restrict__ dbias_part, int Bw, int N, int H, float scale, int P, WaLayout LY) {
  extern __shared__ __attribute__((aligned(16))) float smb32[];
  constexpr int RP = D + 1;
  const int C = H * D, C3 = 3 * C;
  const int h = blockIdx.x % H, pb = blockIdx.x / H;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, hh = lane >> 5, l32 = lane & 31;
  const int dcl = l32 < D ? l32 : D;
  float* BB = smb32;                    // [64][BPF] bias: pass 1 [q][key], pass 2 [key][q]
  float* QR = BB + 64 * BPF + wv * f32_bwd_wave<D>();
  float* KR = QR + 64 * RP;
  float* VR = KR + 64 * RP;
  float* GR = VR + 64 * RP;
  float* SL = GR + 64 * RP;             // [64] lse
  float* SD = SL + 64;                  // [64] delta
  uint8_t* LAB = reinterpret_cast<uint8_t*>(SD + 64);
  stage_bias_f32<PASS == 2>(bias + (int64_t)h * N * N, BB, N);
  __syncthreads();
  f32x16 dsacc[2][2];
  if (PASS == 1) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) dsacc[x][y] = zero16();
  }

  for (int bw = pb * 4 + wv; bw < Bw; bw += P * 4) {
    {
      RowF<D> q, k, v, g, oo;
      float L = 0.f, dl = 0.f;
      if (lane < N) {
        const int64_t tok = (int64_t)bw * N + lane;
        const float* row = qkv + (int64_t)bw * N * C3 + lane * LY.qT + h * LY.qH;
        q.load(row); k.load(row + LY.qW); v.load(row + 2 * LY.qW);
        g.load(dout + (int64_t)bw * N * C + lane * LY.gT + h * LY.gH);
        L = lse[((int64_t)bw * H + h) * N + lane];
        if (LY.delta != nullptr) {
          dl = LY.delta[((int64_t)bw * H + h) * N + lane];
        } else {
          oo.load(o + tok * C + h * D);
#pragma unroll
          for (int e = 0; e < D; ++e) dl = fmaf(g.v[e], oo.v[e], dl);
        }
      } else {
        q.zero(); k.zero(); v.zero(); g.zero();
      }
      q.put(QR, lane); k.put(KR, lane); v.put(VR, lane); g.put(GR, lane);
      SL[lane] = L;
      SD[lane] = dl;
      if (MK == 2) LAB[lane] = lane < N ? labels[(int64_t)(bw % nw) * N + lane] : (uint8_t)255;
    }
    wave_sync();
    const float* mw = MK == 1 ? mask + (int64_t)(bw % nw) * N * N : nullptr;
    if (PASS == 1) {
      // lane = query (S^T layout): dS^T, dQ = dS K * scale, dS summed for the bias gradient
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const int q = 32 * qt + l32;
        const int qc = FULL ? q : min(q, N - 1);
        const float Lq = SL[q], Dq = SD[q];
        const uint32_t qlab = MK == 2 ? LAB[q] : 0u;
        f32x16 ds[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const f32x16 sc = dot_tile<D>(KR, 32 * kt + l32, QR, q, hh);
          const f32x16 dp = dot_tile<D>(VR, 32 * kt + l32, GR, q, hh);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int base = 32 * kt + 8 * i + 4 * hh;
            const f32x4 bv = *reinterpret_cast<const f32x4*>(BB + q * BPF + base);
            f32x4 mv = {0.f, 0.f, 0.f, 0.f};
            if (MK == 2) {
              mv = label_mask(LAB, base, qlab);
            } else if (MK == 1) {
              if (FULL) {
                mv = *reinterpret_cast<const f32x4*>(mw + q * 64 + base);
              } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) mv[j] = base + j < N ? mw[qc * N + base + j] : 0.f;
              }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              const float a = fmaf(sc[r], scale, bv[j] + mv[j]);
              float v = __expf(a - Lq) * (dp[r] - Dq);
              if (!FULL) v = (base + j < N && q < N) ? v : 0.f;
              ds[kt][r] = v;
            }
          }
          dsacc[qt][kt] += ds[kt];
        }
        f32x16 acc = zero16();
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc = mfma2(KR[(32 * kt + acc_row(r, hh)) * RP + dcl], ds[kt][r], acc);
        if (FULL || q < N) store_dims_f32<D>(dqkv + ((int64_t)bw * N + q) * C3 + h * D, acc, scale, hh);
      }
    } else {
      // lane = key (S layout): P and dS in one sweep; dV = P^T dO, dK = dS^T Q * scale
#pragma unroll 1
      for (int kt = 0; kt < 2; ++kt) {
        const int key = 32 * kt + l32;
        const int kc = FULL ? key : min(key, N - 1);
        const uint32_t klab = MK == 2 ? LAB[key] : 0u;
        f32x16 av = zero16(), ak = zero16();
#pragma unroll 1
        for (int qt = 0; qt < 2; ++qt) {
          const f32x16 sc = dot_tile<D>(QR, 32 * qt + l32, KR, key, hh);
          const f32x16 dp = dot_tile<D>(GR, 32 * qt + l32, VR, key, hh);
          f32x16 pv, dv;
#pragma unroll
          for (int i = 0; i < 4; ++i) {        // registers 4i..4i+3 = queries base..base+3
            const int base = 32 * qt + 8 * i + 4 * hh;
            const f32x4 bv = *reinterpret_cast<const f32x4*>(BB + key * BPF + base);
            const f32x4 L4 = *reinterpret_cast<const f32x4*>(SL + base);
            const f32x4 D4 = *reinterpret_cast<const f32x4*>(SD + base);
            f32x4 mv = {0.f, 0.f, 0.f, 0.f};
            if (MK == 2) {
              mv = label_mask(LAB, base, klab);
            } else if (MK == 1) {
#pragma unroll
              for (int j = 0; j < 4; ++j) mv[j] = (FULL || base + j < N) ? mw[(base + j) * N + kc] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * i + j;
              const float a = fmaf(sc[r], scale, bv[j] + mv[j]);
              float e = __expf(a - L4[j]);
              if (!FULL) e = (key < N && base + j < N) ? e : 0.f;
              pv[r] = e;
              dv[r] = e * (dp[r] - D4[j]);
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = (32 * qt + acc_row(r, hh)) * RP + dcl;
            av = mfma2(GR[row], pv[r], av);
            ak = mfma2(QR[row], dv[r], ak);
          }
        }
        if (FULL || key < N) {
          float* row = dqkv + ((int64_t)bw * N + key) * C3 + h * D;
          store_dims_f32<D>(row + C, ak, scale, hh);
          store_dims_f32<D>(row + 2 * C, av, 1.f, hh);
        }
      }
    }
    wave_sync();
  }
  if (PASS == 1) {
    __syncthreads();
    float* red = BB + 64 * BPF;          // [64][64] over the (now idle) wave tiles
    for (int e = threadIdx.x; e < 64 * 64; e += WA_NT) red[e] = 0.f;
    __syncthreads();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          atomicAdd(red + (32 * qt + l32) * 64 + 32 * kt + acc_row(r, hh), dsacc[qt][kt][r]);
    __syncthreads();
    float* dst = dbias_part + ((int64_t)pb * H + h) * N * N;
    for (int e = threadIdx.x; e < N * N; e += WA_NT) dst[e] = red[(e / N) * 64 + e % N];
  }
}

template <int D>
int wa_f32_fwd_launch(const float* qkv, const float* bias, const float* mask, const uint8_t* labels, int nw, float* o,
                      float* lse, int Bw, int N, int H, float scale, const WaLayout& LY, float* hm_out,
                      hipStream_t st) {
  const int P = mfma_blocks_per_head(Bw, H, 4);
  const size_t lds = f32_fwd_lds<D>();
  const bool full = N == 64;
#define PDT_WF(M, F) \
  win_attn_fwd_f32<D, M, F><<<P * H, WA_NT, lds, st>>>(qkv, bias, mask, labels, nw, o, lse, Bw, N, H, scale, P, LY, \
                                                       hm_out)
  if (labels) { if (full) PDT_WF(2, true); else PDT_WF(2, false); }
  else if (mask) { if (full) PDT_WF(1, true); else PDT_WF(1, false); }
  else { if (full) PDT_WF(0, true); else PDT_WF(0, false); }
#undef PDT_WF
  return (int)hipGetLastError();
}
template <int D>
int wa_f32_bwd_launch(const float* qkv, const float* bias, const float* mask, const uint8_t* labels, int nw,
                      const float* o, const float* dout, const float* lse, float* dqkv, float* dbias_part, int Bw,
                      int N, int H, float scale, const WaLayout& LY, hipStream_t st) {
  const int P = mfma_blocks_per_head(Bw, H, 2);
  const size_t lds = f32_bwd_lds<D>();
  static bool attr = [] {
    bool ok = true;
    const void* fns[12] = {
        (const void*)win_attn_bwd_f32<D, 1, true, 1>,  (const void*)win_attn_bwd_f32<D, 1, false, 1>,
        (const void*)win_attn_bwd_f32<D, 0, true, 1>,  (const void*)win_attn_bwd_f32<D, 0, false, 1>,
        (const void*)win_attn_bwd_f32<D, 1, true, 2>,  (const void*)win_attn_bwd_f32<D, 1, false, 2>,
        (const void*)win_attn_bwd_f32<D, 0, true, 2>,  (const void*)win_attn_bwd_f32<D, 0, false, 2>,
        (const void*)win_attn_bwd_f32<D, 2, true, 1>,  (const void*)win_attn_bwd_f32<D, 2, false, 1>,
        (const void*)win_attn_bwd_f32<D, 2, true, 2>,  (const void*)win_attn_bwd_f32<D, 2, false, 2>};
    for (const void* f : fns)
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)f32_bwd_lds<D>()) == hipSuccess;
    return ok;
  }();
  if (!attr) return (int)hipErrorInvalidValue;
  const bool full = N == 64;
#define PDT_WB(M, F, PS)                                                                                         \
  win_attn_bwd_f32<D, M, F, PS><<<P * H, WA_NT, lds, st>>>(qkv, bias, mask, labels, nw, o, dout, lse, dqkv, dbias_part, \
                                                           Bw, N, H, scale, P, LY)
  if (labels) {
    if (full) { PDT_WB(2, true, 1); PDT_WB(2, true, 2); }
    else { PDT_WB(2, false, 1); PDT_WB(2, false, 2); }
  } else if (mask) {
    if (full) { PDT_WB(1, true, 1); PDT_WB(1, true, 2); }
    else { PDT_WB(1, false, 1); PDT_WB(1, false, 2); }
  } else {
    if (full) { PDT_WB(0, true, 1); PDT_WB(0, true, 2); }
    else { PDT_WB(0, false, 1); PDT_WB(0, false, 2); }
  }
#undef PDT_WB
  return (int)hipGetLastError();
}

}  // namespace

namespace {
WaLayout wa_layout(int N, int H, int d, int q_hm, int g_hm, const float* delta, int o_hm = 0) {
  const int C = H * d;
  WaLayout L;
  if (o_hm) { L.oT = d; L.oH = N * d; }
  else { L.oT = C; L.oH = d; }
  if (q_hm) { L.qT = d; L.qH = N * d; L.qW = H * N * d; }
  else { L.qT = 3 * C; L.qH = d; L.qW = C; }
  if (g_hm) { L.gT = d; L.gH = N * d; }
  else { L.gT = C; L.gH = d; }
  L.delta = delta;
  return L;
}

// One workgroup per window: the window's token-major dO / O blocks ([N][C], contiguous) staged into LDS with 16-byte
// loads, dO written back head-major ([H][N][d], also contiguous) one head slice per thread (4-byte units: d, C and
// the offsets are even).  E: bytes per element.
constexpr int HM_NT = 256;
template <int E>
__device__ __forceinline__ void hm_permute(const uint32_t* __restrict__ sm, uint32_t* __restrict__ dst, int N, int H,
                                           int d, int parts) {
  const int du = d * E / 4;                     // 4-byte units per head slice
  const int row = parts * H * du;               // units per token row
  for (int i = threadIdx.x; i < parts * H * N; i += HM_NT) {
    const int wh = i / N, t = i - wh * N;       // slice i of the head-major block = (which * H + h, token t)
    const uint32_t* s = sm + t * row + wh * du;
    uint32_t* o = dst + i * du;
    for (int c = 0; c < du; ++c) o[c] = s[c];
  }
}
template <int E>
__device__ __forceinline__ void stage_block(const void* src, uint32_t* sm, int bytes) {
  const u32x4* s = reinterpret_cast<const u32x4*>(src);
  u32x4* d = reinterpret_cast<u32x4*>(sm);
  for (int i = threadIdx.x; i < bytes / 16; i += HM_NT) d[i] = s[i];
}

// dO -> head-major (unless it already is), and delta[bw][h][t] = sum_c dO[t][h d + c] O[t][h d + c] (fp32) from the
// same staged blocks; g_hm / o_hm: dO / O given head-major ([H][N][d] per window) instead of token-major ([N][C])
template <typename T>
__global__ __launch_bounds__(HM_NT) void bwd_prep_kernel(const T* __restrict__ dout, const T* __restrict__ o,
                                                        T* __restrict__ dout_hm, float* __restrict__ delta, int N,
                                                        int H, int d, int g_hm, int o_hm) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smh[];
  const int C = H * d;
  const int bytes = N * C * (int)sizeof(T);
  uint32_t* sg = smh;
  uint32_t* so = smh + bytes / 4;
  stage_block<sizeof(T)>(dout + (int64_t)blockIdx.x * N * C, sg, bytes);
  stage_block<sizeof(T)>(o + (int64_t)blockIdx.x * N * C, so, bytes);
  __syncthreads();
  if (!g_hm) hm_permute<sizeof(T)>(sg, reinterpret_cast<uint32_t*>(dout_hm + (int64_t)blockIdx.x * N * C), N, H, d, 1);
  const T* g = reinterpret_cast<const T*>(sg);
  const T* oo = reinterpret_cast<const T*>(so);
  const int gT = g_hm ? d : C, gH = g_hm ? N * d : d, oT = o_hm ? d : C, oH = o_hm ? N * d : d;
  for (int i = threadIdx.x; i < H * N; i += HM_NT) {
    const int h = i / N, t = i - h * N;
    float s = 0.f;
    for (int c = 0; c < d; ++c) s = fmaf(to_f<T>(g[t * gT + h * gH + c]), to_f<T>(oo[t * oT + h * oH + c]), s);
    delta[(int64_t)blockIdx.x * H * N + i] = s;
  }
}
}  // namespace

// dout, o [Bw, N, C] token-major -> dout_hm [Bw, H, N, d], delta [Bw, H, N] fp32.  16-byte aligned; N C elem_bytes
// a multiple of 16.
PDT_API int pdt_win_bwd_prep(const void* dout, const void* o, void* dout_hm, float* delta, int Bw, int N, int H, int d,
                             int dt, int g_hm, int o_hm, hipStream_t st) {
  const int E = dt == kF32 ? 4 : 2;
  const int64_t bytes = (int64_t)N * H * d * E;
  if (Bw <= 0 || d % 2 || bytes % 16 || 2 * bytes > 96 * 1024 ||
      (((uintptr_t)dout | (uintptr_t)o | (uintptr_t)dout_hm) & 15))
    return (int)hipErrorInvalidValue;
  if (E == 4)
    bwd_prep_kernel<float><<<Bw, HM_NT, 2 * bytes, st>>>((const float*)dout, (const float*)o, (float*)dout_hm, delta, N,
                                                         H, d, g_hm, o_hm);
  else
    bwd_prep_kernel<bf16_t><<<Bw, HM_NT, 2 * bytes, st>>>((const bf16_t*)dout, (const bf16_t*)o, (bf16_t*)dout_hm,
                                                          delta, N, H, d, g_hm, o_hm);
  return (int)hipGetLastError();
}

// grid size the launcher uses (also the number of dbias partials the caller must allocate)
PDT_API int pdt_win_attn_grid(int Bw) { return Bw < 512 ? Bw : 512; }

// ---- MFMA path: bias [H, N(q), N(key)] fp32 (dense relative-position bias), mask [nw, N, N] fp32 or null
PDT_API int pdt_win_attn_mfma_ok(int N, int H, int d, int dt) { return mfma_ok(N, H, d, dt) ? 1 : 0; }
// number of relative-bias-gradient partials [P, H, N, N] the backward writes
PDT_API int pdt_win_attn_mfma_grid(int Bw, int H) { return mfma_blocks_per_head(Bw, H, 2); }

#define PDT_WA_DISPATCH_D(d, CALL) \
  switch (d) {                      \
    case 2: CALL(2); break;         \
    case 4: CALL(4); break;         \
    case 6: CALL(6); break;         \
    case 8: CALL(8); break;         \
    case 10: CALL(10); break;       \
    case 12: CALL(12); break;       \
    case 14: CALL(14); break;       \
    default: CALL(16); break;       \
  }

namespace {
template <int D>
int wa_fwd_launch(const void* qkv, const float* bias, const float* mask, const uint8_t* labels, int nw, void* o,
                  float* lse, int Bw, int N, int H, float scale, const WaLayout& LY, void* hm_out, hipStream_t st) {
  const int P = mfma_blocks_per_head(Bw, H, 4);
  const size_t lds = fwd_mfma_lds();
  const bool full = N == 64;
#define PDT_WF(M, F)                                                                                          \
  win_attn_fwd_mfma<D, M, F><<<P * H, WA_NT, lds, st>>>((const bf16_t*)qkv, bias, mask, labels, nw, (bf16_t*)o, \
                                                        lse, Bw, N, H, scale, P, LY, (bf16_t*)hm_out)
  if (labels) { if (full) PDT_WF(2, true); else PDT_WF(2, false); }
  else if (mask) { if (full) PDT_WF(1, true); else PDT_WF(1, false); }
  else { if (full) PDT_WF(0, true); else PDT_WF(0, false); }
#undef PDT_WF
  return (int)hipGetLastError();
}
template <int D>
int wa_bwd_launch(const void* qkv, const float* bias, const float* mask, const uint8_t* labels, int nw, const void* o,
                  const void* dout, const float* lse, void* dqkv, float* dbias_part, int Bw, int N, int H, float scale,
                  const WaLayout& LY, hipStream_t st) {
  const int P = mfma_blocks_per_head(Bw, H, 2);
  const size_t lds = bwd_mfma_lds();
  static bool attr = [] {
    bool ok = true;
    const void* fns[12] = {
        (const void*)win_attn_bwd_mfma<D, 1, true, 1>,  (const void*)win_attn_bwd_mfma<D, 1, false, 1>,
        (const void*)win_attn_bwd_mfma<D, 0, true, 1>,  (const void*)win_attn_bwd_mfma<D, 0, false, 1>,
        (const void*)win_attn_bwd_mfma<D, 1, true, 2>,  (const void*)win_attn_bwd_mfma<D, 1, false, 2>,
        (const void*)win_attn_bwd_mfma<D, 0, true, 2>,  (const void*)win_attn_bwd_mfma<D, 0, false, 2>,
        (const void*)win_attn_bwd_mfma<D, 2, true, 1>,  (const void*)win_attn_bwd_mfma<D, 2, false, 1>,
        (const void*)win_attn_bwd_mfma<D, 2, true, 2>,  (const void*)win_attn_bwd_mfma<D, 2, false, 2>};
    for (const void* f : fns)
      ok = ok && hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bwd_mfma_lds()) == hipSuccess;
    return ok;
  }();
  if (!attr) return (int)hipErrorInvalidValue;
  const bool full = N == 64;
#define PDT_WB(M, F, PS)                                                                                           \
  win_attn_bwd_mfma<D, M, F, PS><<<P * H, WA_NT, lds, st>>>((const bf16_t*)qkv, bias, mask, labels, nw,              \
                                                            (const bf16_t*)o, (const bf16_t*)dout, lse, (bf16_t*)dqkv, \
                                                            dbias_part, Bw, N, H, scale, P, LY)
  if (labels) {
    if (full) { PDT_WB(2, true, 1); PDT_WB(2, true, 2); }
    else { PDT_WB(2, false, 1); PDT_WB(2, false, 2); }
  } else if (mask) {
    if (full) { PDT_WB(1, true, 1); PDT_WB(1, true, 2); }
    else { PDT_WB(1, false, 1); PDT_WB(1, false, 2); }
  } else {
    if (full) { PDT_WB(0, true, 1); PDT_WB(0, true, 2); }
    else { PDT_WB(0, false, 1); PDT_WB(0, false, 2); }
  }
#undef PDT_WB
  return (int)hipGetLastError();
}
}  // namespace

// mask [nw, N, N] fp32 or null; labels [nw, N] uint8 region labels or null (takes precedence over mask:
// mask value = -100 where the query's and key's labels differ, 0 elsewhere)
// qkv token-major [Bw, N, 3C], or head-major [Bw, 3, H, N, d] with q_hm = 1 (the narrow GEMM's head-major output);
// hm_out (nullable, token-major qkv only) [Bw, 3, H, N, d]: the head-major copy of q / k / v the backward reads
// (hm = 1), written from the staged slices
PDT_API int pdt_win_attn_mfma_fwd(const void* qkv, const float* bias, const float* mask, const void* labels, int nw,
                                  void* o, float* lse, int Bw, int N, int H, int d, float scale, void* hm_out,
                                  int q_hm, int o_hm, hipStream_t st) {
  if (!mfma_ok(N, H, d, kBF16) || Bw <= 0 || ((mask || labels) && nw <= 0) || (q_hm && hm_out))
    return (int)hipErrorInvalidValue;
  const WaLayout LY = wa_layout(N, H, d, q_hm, 0, nullptr, o_hm);
#define PDT_C(D) \
  return wa_fwd_launch<D>(qkv, bias, mask, (const uint8_t*)labels, nw, o, lse, Bw, N, H, scale, LY, hm_out, st)
  PDT_WA_DISPATCH_D(d, PDT_C)
#undef PDT_C
}

// dqkv [Bw, N, 3C] fully written; dbias_part [pdt_win_attn_mfma_grid(Bw, H), H, N, N] fp32 fully written
PDT_API int pdt_win_attn_mfma_bwd(const void* qkv, const float* bias, const float* mask, const void* labels, int nw,
                                  const void* o, const void* dout, const float* lse, void* dqkv, float* dbias_part,
                                  int Bw, int N, int H, int d, float scale, int hm, const float* delta,
                                  hipStream_t st) {
  if (!mfma_ok(N, H, d, kBF16) || Bw <= 0 || ((mask || labels) && nw <= 0) || (hm && !delta))
    return (int)hipErrorInvalidValue;
  const WaLayout LY = wa_layout(N, H, d, hm, hm, delta);
#define PDT_C(D)                                                                                                   \
  return wa_bwd_launch<D>(qkv, bias, mask, (const uint8_t*)labels, nw, o, dout, lse, dqkv, dbias_part, Bw, N, H, \
                          scale, LY, st)
  PDT_WA_DISPATCH_D(d, PDT_C)
#undef PDT_C
}
// fp32 MFMA path (same contract as the bf16 one; partials [pdt_win_attn_mfma_grid(Bw, H), H, N, N])
PDT_API int pdt_win_attn_mfma32_ok(int N, int H, int d) { return mfma_ok(N, H, d, kBF16) ? 1 : 0; }
PDT_API int pdt_win_attn_mfma32_fwd(const float* qkv, const float* bias, const float* mask, const void* labels, int nw,
                                    float* o, float* lse, int Bw, int N, int H, int d, float scale, float* hm_out,
                                    int q_hm, int o_hm, hipStream_t st) {
  if (!mfma_ok(N, H, d, kBF16) || Bw <= 0 || ((mask || labels) && nw <= 0) || (q_hm && hm_out))
    return (int)hipErrorInvalidValue;
  const WaLayout LY = wa_layout(N, H, d, q_hm, 0, nullptr, o_hm);
#define PDT_C(D) \
  return wa_f32_fwd_launch<D>(qkv, bias, mask, (const uint8_t*)labels, nw, o, lse, Bw, N, H, scale, LY, hm_out, st)
  PDT_WA_DISPATCH_D(d, PDT_C)
#undef PDT_C
}
PDT_API int pdt_win_attn_mfma32_bwd(const float* qkv, const float* bias, const float* mask, const void* labels, int nw,
                                    const float* o, const float* dout, const float* lse, float* dqkv,
                                    float* dbias_part, int Bw, int N, int H, int d, float scale, int hm,
                                    const float* delta, hipStream_t st) {
  if (!mfma_ok(N, H, d, kBF16) || Bw <= 0 || ((mask || labels) && nw <= 0) || (hm && !delta))
    return (int)hipErrorInvalidValue;
  const WaLayout LY = wa_layout(N, H, d, hm, hm, delta);
#define PDT_C(D)                                                                                                 \
  return wa_f32_bwd_launch<D>(qkv, bias, mask, (const uint8_t*)labels, nw, o, dout, lse, dqkv, dbias_part, Bw, N, \
                              H, scale, LY, st)
  PDT_WA_DISPATCH_D(d, PDT_C)
#undef PDT_C
}
#undef PDT_WA_DISPATCH_D

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
