// Narrow GEMMs for gfx950: Y[M, NO] = X[M, KI] . B[NO, KI]^T (+ bias), with KI, NO <= 192 and M in the hundreds
// of thousands -- SwinIR-S's linears at the Stoke config (SURVEY.md K2 "skinny GEMMs": 294,912 tokens x C = 60:
// qkv 60 -> 180, proj 60 -> 60; their data gradients 180 -> 60 and 60 -> 60, Stoke-DDP.py:206-208).
//
// Such a product is bandwidth-bound (qkv: 35 MB in, 106 MB out, 6.4 GFLOP), but library GEMMs tile it as if it
// were compute-bound: K = 60 is two 32-wide K-steps, so every 64 x 128 macro tile pays its prologue / epilogue
// for almost no MFMA work.  Here the whole weight lives in VGPRs as MFMA B fragments (loaded once per wave), and
// each wave streams 16-row blocks of X through a private LDS tile: contiguous 16-byte loads of the block (rows
// are contiguous, so a block is one span of 16 KI elements), 16 v_mfma_f32_16x16x32_bf16 A fragments read back
// as 16-byte LDS reads, the bias added in the epilogue, and the 16 x NO output block staged in LDS and written
// back as contiguous 16-byte stores.  The next block's loads are issued before the current block's MFMAs.  No
// workgroup barrier anywhere: waves run independently over a grid-stride of blocks.
//
// COLSUM (the data-gradient pass, where X = dY): the column sums of X over all M rows -- the Linear's bias
// gradient -- come out of the same read: every lane sums its A fragments, the 16 lanes of a fragment column
// group fold them with xor shuffles, and each wave writes one fp32 partial row (reduced by the caller with the
// fixed-order column reduce, so the result is deterministic).
#include "common.h"
#include "reduce.h"

using namespace pdt;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int NW = 4;                          // waves per workgroup (independent)

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

template <int KP, int NP>
struct NarrowCfg {
  static constexpr int XP = KP + 8;            // LDS row pitch (elements): 16-byte aligned rows, shifted banks
  static constexpr int KS = KP / 32;           // MFMA K-steps
  static constexpr int NT = NP / 16;           // output column tiles
  static constexpr int WAVE_ELEMS = 16 * XP + 16 * NP;   // X tile + output staging (bf16 elements)
  static constexpr int CH = (2 * KP + 63) / 64;          // 16-byte X chunks per lane per block (upper bound)
};

// 16-row block `blk` of X into registers: chunk c = lane + 64 i covers elements 8c .. 8c+7 of the block's span
template <int KP, int NP>
__device__ __forceinline__ void load_block(const bf16_t* __restrict__ X, int64_t M, int KI, int64_t blk, int lane,
                                           u16x8 (&ch)[NarrowCfg<KP, NP>::CH]) {
  const int64_t r0 = blk * 16;
  const int rows = M - r0 < 16 ? (int)(M - r0) : 16;
  const int n8 = (rows * KI) >> 3;             // whole chunks (rows * KI % 8 != 0 only in a tail block)
  const bf16_t* src = X + r0 * KI;
#pragma unroll
  for (int i = 0; i < NarrowCfg<KP, NP>::CH; ++i) {
    const int c = lane + 64 * i;
    if (c < n8) {
      ch[i] = *reinterpret_cast<const u16x8*>(src + 8 * c);
    } else if (8 * c < rows * KI) {            // the tail block's last partial chunk (KI % 4 == 0: whole halves)
      u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      const u16x4 lo = *reinterpret_cast<const u16x4*>(src + 8 * c);
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      ch[i] = v;
    }
  }
}

// ... the same block from a HEAD-MAJOR X ([windows][KI / a_d][a_n][a_d]: ops.window_attention's output for the
// projection after it): the block's 16 tokens of segment s are one contiguous run of 16 a_d elements at
// (w KI + s a_d) a_n + t0 a_d; chunk c = lane + 64 i covers elements 8c .. 8c+7 of the concatenated runs (16 a_d % 8
// == 0).  Blocks are always full (M % a_n == 0, a_n % 16 == 0).
__device__ __forceinline__ int fdiv_i(int a, float inv) { return __float2int_rz(((float)a + 0.5f) * inv); }
template <int KP, int NP>
__device__ __forceinline__ void load_block_hm(const bf16_t* __restrict__ X, int KI, int64_t blk, int lane, int a_n,
                                              int a_d, u16x8 (&ch)[NarrowCfg<KP, NP>::CH]) {
  const uint32_t r0 = (uint32_t)(blk * 16);             // M < 2^31 (hm_ok): 32-bit division
  const uint32_t win = r0 / (uint32_t)a_n;
  const int t0 = (int)(r0 - win * (uint32_t)a_n);
  const int run = 16 * a_d, n8 = 2 * KI;                // elements per segment run; chunks per block (16 KI / 8)
  const float inv_run = 1.f / (float)run;
  const bf16_t* base = X + (int64_t)win * a_n * KI + (int64_t)t0 * a_d;
#pragma unroll
  for (int i = 0; i < NarrowCfg<KP, NP>::CH; ++i) {
    const int c = lane + 64 * i;
    if (c < n8) {
      const int sg = fdiv_i(8 * c, inv_run), off = 8 * c - sg * run;
      ch[i] = *reinterpret_cast<const u16x8*>(base + (int64_t)sg * a_n * a_d + off);
    }
  }
}
template <int KP, int NP>
__device__ __forceinline__ void put_block_hm(bf16_t* Xs, int KI, int lane, int a_d,
                                             const u16x8 (&ch)[NarrowCfg<KP, NP>::CH]) {
  constexpr int XP = NarrowCfg<KP, NP>::XP;
  const int run = 16 * a_d, n8 = 2 * KI;
  const float inv_run = 1.f / (float)run, inv_d = 1.f / (float)a_d;
#pragma unroll
  for (int i = 0; i < NarrowCfg<KP, NP>::CH; ++i) {
    const int c = lane + 64 * i;
    if (c < n8) {
      const int sg = fdiv_i(8 * c, inv_run), off = 8 * c - sg * run;
#pragma unroll
      for (int k = 0; k < 4; ++k) {               // element pairs never straddle two tokens (a_d even)
        const int e = off + 2 * k, r = fdiv_i(e, inv_d), dd = e - r * a_d;
        *reinterpret_cast<uint32_t*>(Xs + r * XP + sg * a_d + dd) =
            (uint32_t)ch[i][2 * k] | ((uint32_t)ch[i][2 * k + 1] << 16);
      }
    }
  }
}

template <int KP, int NP>
__device__ __forceinline__ void put_block(bf16_t* Xs, int KI, int rows, int lane,
                                          const u16x8 (&ch)[NarrowCfg<KP, NP>::CH]) {
  constexpr int XP = NarrowCfg<KP, NP>::XP;
  const int tot = rows * KI;
#pragma unroll
  for (int i = 0; i < NarrowCfg<KP, NP>::CH; ++i) {
    const int c = lane + 64 * i;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = 8 * c + 4 * h;
      if (e < tot) {
        const int r = e / KI, col = e - r * KI;
        *reinterpret_cast<u16x4*>(Xs + r * XP + col) =
            u16x4{ch[i][4 * h], ch[i][4 * h + 1], ch[i][4 * h + 2], ch[i][4 * h + 3]};
      }
    }
  }
}

// Head-major output (hm_n > 0; Swin's qkv projection feeding the window attention): row m = window w, token t
// (m = w hm_n + t) and column c = segment s (= which x H + head), dim d (c = s hm_d + d) go to element
// (w NO + s hm_d) hm_n + t hm_d + d: one head's 16 staged tokens are one contiguous run of 16 hm_d elements,
// written as 16-byte chunks whose 4 dwords are gathered from the [16][NO] staging block (a dword never straddles
// two tokens: hm_d even).  Blocks are always full (M % hm_n == 0, hm_n % 16 == 0).  Integer splits by the runtime
// divisors go through a float reciprocal (exact: operands < 2^12).
__device__ __forceinline__ int fdiv(int a, float inv) { return __float2int_rz(((float)a + 0.5f) * inv); }
template <typename T>
__device__ __forceinline__ void hm_store(T* __restrict__ Y, const T* Ys, int64_t blk, int NO, int hm_n, int hm_d,
                                         int lane) {
  const int dpt = hm_d * (int)sizeof(T) / 4;            // dwords per token slice
  const int cps = 4 * dpt;                               // 16-byte chunks per segment run (16 dpt dwords)
  const int nch = (NO / hm_d) * cps;
  const int rowd = NO * (int)sizeof(T) / 4;              // dwords per staged row
  const float inv_cps = 1.f / (float)cps, inv_dpt = 1.f / (float)dpt;
  const uint32_t row0 = (uint32_t)(blk * 16);           // M < 2^31 (hm_ok): 32-bit division
  const uint32_t win = row0 / (uint32_t)hm_n;
  const int t0 = (int)(row0 - win * (uint32_t)hm_n);
  uint32_t* base = reinterpret_cast<uint32_t*>(Y + (int64_t)win * hm_n * NO + (int64_t)t0 * hm_d);
  const uint32_t* ys = reinterpret_cast<const uint32_t*>(Ys);
  const int64_t seg_stride = (int64_t)hm_n * hm_d * (int)sizeof(T) / 4;
  for (int c = lane; c < nch; c += 64) {
    const int sg = fdiv(c, inv_cps), k = c - sg * cps;
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int w = 4 * k + j, r = fdiv(w, inv_dpt), dd = w - r * dpt;
      v[j] = ys[r * rowd + sg * dpt + dd];
    }
    *reinterpret_cast<uint4*>(base + sg * seg_stride + 4 * k) = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// MODE (compile time, so the plain instantiations carry none of the optional paths' registers -- a runtime switch
// had cost the K = 180 kernel 46 spilled VGPRs): 0 plain, NG_HMY head-major output, NG_HMA head-major input,
// NG_RES residual add
enum { NG_PLAIN = 0, NG_HMY = 1, NG_HMA = 2, NG_RES = 3 };
template <int KP, int NP, int MODE>
__global__ __launch_bounds__(64 * NW, 2) void narrow_gemm_kernel(const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ B,
                                                                 const bf16_t* __restrict__ bias,
                                                                 bf16_t* __restrict__ Y, float* __restrict__ colsum_part,
                                                                 int64_t M, int KI, int NO, int hm_n, int hm_d, int a_n,
                                                                 int a_d, const bf16_t* __restrict__ R) {
  typedef NarrowCfg<KP, NP> Cfg;
  constexpr int XP = Cfg::XP, KS = Cfg::KS, NT = Cfg::NT;
  extern __shared__ __attribute__((aligned(16))) bf16_t nsm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  bf16_t* Xs = nsm + wv * Cfg::WAVE_ELEMS;
  bf16_t* Ys = Xs + 16 * XP;
  // zero the X tile once: columns KI .. KP-1 stay zero (the K padding of the last MFMA K-step)
  for (int e = lane; e < 16 * XP; e += 64) Xs[e] = 0;
  // the weight as B fragments: lane holds B[n = 16 nt + l16][k = 32 ks + 8 lg .. +7], zero outside [NO, KI]
  u16x8 bf[KS][NT];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = 16 * nt + l16, k0 = 32 * ks + 8 * lg;
      u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (n < NO) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (k0 + e < KI) v[e] = B[(int64_t)n * KI + k0 + e];
      }
      bf[ks][nt] = v;
    }
  float bcol[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = 16 * nt + l16;
    bcol[nt] = (bias != nullptr && n < NO) ? bf2f(bias[n]) : 0.f;
  }
  float cs[3] = {0.f, 0.f, 0.f};                 // COLSUM: columns lane, lane + 64, lane + 128

  const int64_t nblk = (M + 15) / 16;
  const int64_t gw = (int64_t)blockIdx.x * NW + wv, nwaves = (int64_t)gridDim.x * NW;
  u16x8 ch[Cfg::CH];
  if (gw < nblk) {
    if constexpr (MODE == NG_HMA) load_block_hm<KP, NP>(X, KI, gw, lane, a_n, a_d, ch);
    else load_block<KP, NP>(X, M, KI, gw, lane, ch);
  }
  for (int64_t blk = gw; blk < nblk; blk += nwaves) {
    const int rows = M - blk * 16 < 16 ? (int)(M - blk * 16) : 16;
    wave_sync();                                 // the previous block's LDS reads are done
    if constexpr (MODE == NG_HMA) put_block_hm<KP, NP>(Xs, KI, lane, a_d, ch);
    else put_block<KP, NP>(Xs, KI, rows, lane, ch);
    if (blk + nwaves < nblk) {                   // in flight under the MFMAs
      if constexpr (MODE == NG_HMA) load_block_hm<KP, NP>(X, KI, blk + nwaves, lane, a_n, a_d, ch);
      else load_block<KP, NP>(X, M, KI, blk + nwaves, lane, ch);
    }
    wave_sync();
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 a = *reinterpret_cast<const u16x8*>(Xs + l16 * XP + 32 * ks + 8 * lg);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16(a, bf[ks][nt], acc[nt]);
    }
    if (colsum_part != nullptr) {                // column sums of the staged block (valid rows only)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c = lane + 64 * j;
        if (c < KI)
          for (int r = 0; r < rows; ++r) cs[j] += bf2f(Xs[r * XP + c]);
      }
    }
    // C[row = 4 lg + r][col = 16 nt + l16] -> the output staging block [16][NO], then contiguous stores
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = 16 * nt + l16;
      if (n < NO) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Ys[(4 * lg + r) * NO + n] = f2bf(acc[nt][r] + bcol[nt]);
      }
    }
    wave_sync();
    if constexpr (MODE == NG_HMY) {
      hm_store(Y, Ys, blk, NO, hm_n, hm_d, lane);
    } else {
      bf16_t* dst = Y + blk * 16 * NO;
      const int tot = rows * NO, n8 = tot >> 3;
      if constexpr (MODE == NG_RES) {            // + the residual stream (same [M, NO] layout), rounded once
        const bf16_t* res = R + blk * 16 * NO;
        for (int c = lane; c < n8; c += 64) {
          const u16x8 a = *reinterpret_cast<const u16x8*>(Ys + 8 * c), b = *reinterpret_cast<const u16x8*>(res + 8 * c);
          u16x8 o;
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = f2bf(bf2f(a[k]) + bf2f(b[k]));
          *reinterpret_cast<u16x8*>(dst + 8 * c) = o;
        }
        for (int e = 8 * n8 + lane; e < tot; e += 64) dst[e] = f2bf(bf2f(Ys[e]) + bf2f(res[e]));
      } else {
        for (int c = lane; c < n8; c += 64) *reinterpret_cast<u16x8*>(dst + 8 * c) = *reinterpret_cast<const u16x8*>(Ys + 8 * c);
        for (int e = 8 * n8 + lane; e < tot; e += 64) dst[e] = Ys[e];
      }
    }
  }
  if (colsum_part != nullptr) {
    float* dstp = colsum_part + gw * KI;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = lane + 64 * j;
      if (c < KI) dstp[c] = cs[j];
    }
  }
}

// ---- weight gradient dW[NO][KI] = dY[M, NO]^T X[M, KI] (the tall-skinny product of the same narrow Linears) ----
// Both operands are token-major, and the MFMA's reduction index is the token: a workgroup of 8 waves stages 64-row
// blocks of dY and X as plain row-major LDS images (contiguous 16-byte loads, double-buffered, one barrier per
// block) and every fragment is two ds_read_b64_tr_b16 transposed reads (4 rows x 16 columns per 16-lane group,
// delivered column-major).  The NO/16 x KI/16 output tiles are dealt round-robin to the 8 waves; each workgroup
// writes one fp32 partial [NO][KI], folded by the caller's fixed-order column reduce.
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
constexpr int WG_WAVES = 8;
constexpr int WG_ROWS = 64;                    // rows per block: 2 MFMA K-steps (32 rows each)

__device__ __forceinline__ u16x8 tr_frag(const bf16_t* base, int pitch, int lg, int l16, int c0, int r0) {
  // rows r0 + 8 lg + q (first read) and r0 + 8 lg + 4 + q (second), columns c0 + 4 p, for lane 4 q + p of the
  // 16-lane group
  const int q = l16 >> 2, pp = l16 & 3;
  const bf16_t* p0 = base + (r0 + 8 * lg + q) * pitch + c0 + 4 * pp;
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)p0);
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p0 + 4 * pitch));
  return __builtin_bit_cast(u16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NP, int KP>
struct WgradCfg {
  static constexpr int PN = NP + 8, PK = KP + 8;                 // LDS row pitches (elements), 16-byte rows
  static constexpr int BUF = WG_ROWS * (PN + PK);                // one dY + X block image
  static constexpr int TILES = (NP / 16) * (KP / 16);
  static constexpr int TPW = (TILES + WG_WAVES - 1) / WG_WAVES; // tiles per wave
  static constexpr int CHY = (WG_ROWS * NP / 8 + 64 * WG_WAVES - 1) / (64 * WG_WAVES);   // 16-B chunks / thread
  static constexpr int CHX = (WG_ROWS * KP / 8 + 64 * WG_WAVES - 1) / (64 * WG_WAVES);
};

// 16-byte chunks of a 32-row block of a row-major [M, C] bf16 matrix (zero past M) -> registers
template <int CH>
__device__ __forceinline__ void wg_load(const bf16_t* __restrict__ A, int64_t M, int C, int64_t r0, int t,
                                        u16x8 (&v)[CH]) {
  const int64_t tot = (M - r0 < WG_ROWS ? M - r0 : WG_ROWS) * (int64_t)C;   // valid elements of the block
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int c = t + 64 * WG_WAVES * i;
    u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    if (8 * (int64_t)c + 8 <= tot) {
      z = *reinterpret_cast<const u16x8*>(A + r0 * C + 8 * (int64_t)c);
    } else if (8 * (int64_t)c < tot) {         // C % 4 == 0: a last half chunk
      const u16x4 lo = *reinterpret_cast<const u16x4*>(A + r0 * C + 8 * (int64_t)c);
      z[0] = lo[0]; z[1] = lo[1]; z[2] = lo[2]; z[3] = lo[3];
    }
    v[i] = z;
  }
}
template <int CH>
__device__ __forceinline__ void wg_put(bf16_t* img, int pitch, int C, int t, const u16x8 (&v)[CH]) {
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int c = t + 64 * WG_WAVES * i;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = 8 * c + 4 * h;
      if (e < WG_ROWS * C) {
        const int r = e / C, col = e - r * C;
        *reinterpret_cast<u16x4*>(img + r * pitch + col) = u16x4{v[i][4 * h], v[i][4 * h + 1], v[i][4 * h + 2], v[i][4 * h + 3]};
      }
    }
  }
}

// a 64-row block of a HEAD-MAJOR X whose windows are exactly the 64-row blocks ([M / 64][C / a_d][64][a_d]): the
// block is still one contiguous run (the same 16-byte loads), only the element order differs -- element e = segment
// s, token r, dim dd goes to image row r, column s a_d + dd (written as element pairs: a_d even)
template <int CH>
__device__ __forceinline__ void wg_put_hm(bf16_t* img, int pitch, int C, int t, int a_d, const u16x8 (&v)[CH]) {
  const float inv_run = 1.f / (float)(WG_ROWS * a_d), inv_d = 1.f / (float)a_d;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int c = t + 64 * WG_WAVES * i;
    if (8 * c < WG_ROWS * C) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = 8 * c + 2 * k;
        const int sg = fdiv_i(e, inv_run), o = e - sg * WG_ROWS * a_d;
        const int r = fdiv_i(o, inv_d), dd = o - r * a_d;
        *reinterpret_cast<uint32_t*>(img + r * pitch + sg * a_d + dd) = (uint32_t)v[i][2 * k] | ((uint32_t)v[i][2 * k + 1] << 16);
      }
    }
  }
}

template <int NP, int KP>
__global__ __launch_bounds__(64 * WG_WAVES, 1) void narrow_wgrad_kernel(const bf16_t* __restrict__ dY,
                                                                        const bf16_t* __restrict__ X,
                                                                        float* __restrict__ part, int64_t M, int NO,
                                                                        int KI, int x_hm_d) {
  typedef WgradCfg<NP, KP> Cfg;
  extern __shared__ __attribute__((aligned(16))) bf16_t wsm[];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  // zero both images once: padding columns (NO .. NP-1, KI .. KP-1) stay zero
  for (int e = t; e < 2 * Cfg::BUF; e += 64 * WG_WAVES) wsm[e] = 0;
  f32x4 acc[Cfg::TPW];
#pragma unroll
  for (int i = 0; i < Cfg::TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nblk = (M + WG_ROWS - 1) / WG_ROWS;
  u16x8 vy[Cfg::CHY], vx[Cfg::CHX];
  int64_t blk = blockIdx.x;
  if (blk < nblk) {
    wg_load<Cfg::CHY>(dY, M, NO, blk * WG_ROWS, t, vy);
    wg_load<Cfg::CHX>(X, M, KI, blk * WG_ROWS, t, vx);
  }
  __syncthreads();
  for (int it = 0; blk < nblk; blk += gridDim.x, ++it) {
    bf16_t* ys = wsm + (it & 1) * Cfg::BUF;
    bf16_t* xs = ys + WG_ROWS * Cfg::PN;
    wg_put<Cfg::CHY>(ys, Cfg::PN, NO, t, vy);
    if (x_hm_d > 0) wg_put_hm<Cfg::CHX>(xs, Cfg::PK, KI, t, x_hm_d, vx);
    else wg_put<Cfg::CHX>(xs, Cfg::PK, KI, t, vx);
    if (blk + gridDim.x < nblk) {
      wg_load<Cfg::CHY>(dY, M, NO, (blk + gridDim.x) * WG_ROWS, t, vy);
      wg_load<Cfg::CHX>(X, M, KI, (blk + gridDim.x) * WG_ROWS, t, vx);
    }
    __syncthreads();    // this block's images are written (the other buffer was last read before this barrier)
#pragma unroll
    for (int i = 0; i < Cfg::TPW; ++i) {
      const int tile = wv + WG_WAVES * i;
      if (tile < Cfg::TILES) {
        const int tn = tile / (KP / 16), tk = tile - tn * (KP / 16);
#pragma unroll
        for (int ks = 0; ks < WG_ROWS / 32; ++ks)
          acc[i] = mfma16(tr_frag(ys, Cfg::PN, lg, l16, 16 * tn, 32 * ks), tr_frag(xs, Cfg::PK, lg, l16, 16 * tk, 32 * ks),
                          acc[i]);
      }
    }
  }
  // C[n = 16 tn + 4 lg + r][k = 16 tk + l16] -> this workgroup's partial [NO][KI]
  float* dst = part + (int64_t)blockIdx.x * NO * KI;
#pragma unroll
  for (int i = 0; i < Cfg::TPW; ++i) {
    const int tile = wv + WG_WAVES * i;
    if (tile < Cfg::TILES) {
      const int tn = tile / (KP / 16), tk = tile - tn * (KP / 16);
      const int k = 16 * tk + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * tn + 4 * lg + r;
        if (n < NO && k < KI) dst[n * KI + k] = acc[i][r];
      }
    }
  }
}

template <int NP, int KP>
size_t wgrad_lds() { return sizeof(bf16_t) * 2 * (size_t)WgradCfg<NP, KP>::BUF; }

// ---- fp32 family (the reference's own precision: Stoke-DDP.py trains with fp16=None) on v_mfma_f32_16x16x4_f32,
// exact f32 (an fmaf chain per output): A / B fragments are ONE float per lane (A[row = l & 15][k = l >> 4],
// B[k = l >> 4][col = l & 15]), so the weight tile and the X / dY tiles are plain row-major fp32 LDS images with odd
// row pitches (b32 fragment reads of 16 rows land on distinct banks).  Structure as the bf16 kernels above: the
// forward / data gradient keep the weight in LDS (shared by 8 waves), each wave streams 16-row blocks; the weight
// gradient reduces 64-row blocks of dY and X, tiles dealt to the waves, one fp32 partial per workgroup.
constexpr int NW32 = 8;

__device__ __forceinline__ f32x4 mfma4(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int KP, int NP>
struct Narrow32Cfg {
  static constexpr int BPF = KP + 1;                        // weight row pitch (floats)
  static constexpr int XPF = KP + 1;                        // X tile row pitch
  static constexpr int WAVE = (16 * XPF > 16 * NP ? 16 * XPF : 16 * NP);   // X tile, aliased by the Y staging
  static constexpr int CH = (4 * KP + 63) / 64;              // 16-byte X chunks per lane per block (upper bound)
};

template <int KP, int NP>
__global__ __launch_bounds__(64 * NW32, 1) void narrow_gemm_f32_kernel(const float* __restrict__ X,
                                                                       const float* __restrict__ B,
                                                                       const float* __restrict__ bias,
                                                                       float* __restrict__ Y,
                                                                       float* __restrict__ colsum_part, int64_t M,
                                                                       int KI, int NO, int hm_n, int hm_d,
                                                                       const float* __restrict__ R) {
  typedef Narrow32Cfg<KP, NP> Cfg;
  constexpr int NT = NP / 16;
  extern __shared__ __attribute__((aligned(16))) float n32[];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  float* Bs = n32;                                           // [NP][BPF], zero outside [NO, KI]
  float* Xs = n32 + NP * Cfg::BPF + wv * Cfg::WAVE;          // [16][XPF]; after the MFMAs: Y staging [16][NO]
  for (int e = t; e < NP * Cfg::BPF; e += 64 * NW32) {
    const int n = e / Cfg::BPF, k = e - n * Cfg::BPF;
    Bs[e] = (n < NO && k < KI) ? B[(int64_t)n * KI + k] : 0.f;
  }
  float bcol[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = 16 * nt + l16;
    bcol[nt] = (bias != nullptr && n < NO) ? bias[n] : 0.f;
  }
  float cs[3] = {0.f, 0.f, 0.f};
  __syncthreads();
  const int64_t nblk = (M + 15) / 16;
  const int64_t gw = (int64_t)blockIdx.x * NW32 + wv, nwaves = (int64_t)gridDim.x * NW32;
  f32x4 ch[Cfg::CH];
  auto load = [&](int64_t blk) {
    const int64_t r0 = blk * 16;
    const int rows = M - r0 < 16 ? (int)(M - r0) : 16;
    const int n4 = rows * KI / 4;                            // KI % 4 == 0: 16-byte chunks never straddle rows
#pragma unroll
    for (int i = 0; i < Cfg::CH; ++i) {
      const int c = lane + 64 * i;
      if (c < n4) ch[i] = *reinterpret_cast<const f32x4*>(X + r0 * KI + 4 * c);
    }
  };
  if (gw < nblk) load(gw);
  for (int64_t blk = gw; blk < nblk; blk += nwaves) {
    const int rows = M - blk * 16 < 16 ? (int)(M - blk * 16) : 16;
    wave_sync();
    // the X tile: rows < `rows` from the chunks, columns KI .. KP-1 and rows >= `rows` zero
    for (int e = lane; e < 16 * Cfg::XPF; e += 64) Xs[e] = 0.f;
    wave_sync();
#pragma unroll
    for (int i = 0; i < Cfg::CH; ++i) {
      const int c = lane + 64 * i;
      if (c < rows * KI / 4) {
        const int r = (4 * c) / KI, col = 4 * c - r * KI;
#pragma unroll
        for (int e = 0; e < 4; ++e) Xs[r * Cfg::XPF + col + e] = ch[i][e];
      }
    }
    if (blk + nwaves < nblk) load(blk + nwaves);
    wave_sync();
    if (colsum_part != nullptr) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c = lane + 64 * j;
        if (c < KI)
          for (int r = 0; r < rows; ++r) cs[j] += Xs[r * Cfg::XPF + c];
      }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int ks = 0; ks < KP / 4; ++ks) {
      const float a = Xs[l16 * Cfg::XPF + 4 * ks + lg];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma4(a, Bs[(16 * nt + l16) * Cfg::BPF + 4 * ks + lg], acc[nt]);
    }
    wave_sync();                                             // X tile reads done: the staging aliases it
    float* Ys = Xs;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = 16 * nt + l16;
      if (n < NO) {
#pragma unroll
        for (int r = 0; r < 4; ++r) Ys[(4 * lg + r) * NO + n] = acc[nt][r] + bcol[nt];
      }
    }
    wave_sync();
    if (hm_n > 0) {
      hm_store(Y, Ys, blk, NO, hm_n, hm_d, lane);
    } else {
      float* dst = Y + blk * 16 * NO;
      const int n4 = rows * NO / 4;
      if (R != nullptr) {                        // + the residual stream (same [M, NO] layout)
        const float* res = R + blk * 16 * NO;
        for (int c = lane; c < n4; c += 64)
          *reinterpret_cast<f32x4*>(dst + 4 * c) =
              *reinterpret_cast<const f32x4*>(Ys + 4 * c) + *reinterpret_cast<const f32x4*>(res + 4 * c);
      } else {
        for (int c = lane; c < n4; c += 64) *reinterpret_cast<f32x4*>(dst + 4 * c) = *reinterpret_cast<const f32x4*>(Ys + 4 * c);
      }
    }
  }
  if (colsum_part != nullptr) {
    float* dstp = colsum_part + gw * KI;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = lane + 64 * j;
      if (c < KI) dstp[c] = cs[j];
    }
  }
}

template <int NP, int KP>
struct Wgrad32Cfg {
  static constexpr int PN = NP + 1, PK = KP + 1;
  static constexpr int BUF = 64 * (PN + PK);
  static constexpr int TILES = (NP / 16) * (KP / 16);
  static constexpr int TPW = (TILES + NW32 - 1) / NW32;
  static constexpr int CHY = (64 * NP / 4 + 64 * NW32 - 1) / (64 * NW32);
  static constexpr int CHX = (64 * KP / 4 + 64 * NW32 - 1) / (64 * NW32);
};

template <int CH>
__device__ __forceinline__ void w32_load(const float* __restrict__ A, int64_t M, int C, int64_t r0, int t,
                                         f32x4 (&v)[CH]) {
  const int64_t rows = M - r0 < 64 ? M - r0 : 64;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int c = t + 64 * NW32 * i;
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if (4 * (int64_t)c < rows * C) z = *reinterpret_cast<const f32x4*>(A + r0 * C + 4 * (int64_t)c);
    v[i] = z;
  }
}
template <int CH>
__device__ __forceinline__ void w32_put(float* img, int pitch, int C, int t, const f32x4 (&v)[CH]) {
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int c = t + 64 * NW32 * i;
    if (4 * c < 64 * C) {
      const int r = (4 * c) / C, col = 4 * c - r * C;
#pragma unroll
      for (int e = 0; e < 4; ++e) img[r * pitch + col + e] = v[i][e];
    }
  }
}

template <int NP, int KP>
__global__ __launch_bounds__(64 * NW32, 1) void narrow_wgrad_f32_kernel(const float* __restrict__ dY,
                                                                        const float* __restrict__ X,
                                                                        float* __restrict__ part, int64_t M, int NO,
                                                                        int KI) {
  typedef Wgrad32Cfg<NP, KP> Cfg;
  extern __shared__ __attribute__((aligned(16))) float w32[];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  for (int e = t; e < 2 * Cfg::BUF; e += 64 * NW32) w32[e] = 0.f;     // padding columns stay zero
  f32x4 acc[Cfg::TPW];
#pragma unroll
  for (int i = 0; i < Cfg::TPW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nblk = (M + 63) / 64;
  f32x4 vy[Cfg::CHY], vx[Cfg::CHX];
  int64_t blk = blockIdx.x;
  if (blk < nblk) {
    w32_load<Cfg::CHY>(dY, M, NO, blk * 64, t, vy);
    w32_load<Cfg::CHX>(X, M, KI, blk * 64, t, vx);
  }
  __syncthreads();
  for (int it = 0; blk < nblk; blk += gridDim.x, ++it) {
    float* ys = w32 + (it & 1) * Cfg::BUF;
    float* xs = ys + 64 * Cfg::PN;
    w32_put<Cfg::CHY>(ys, Cfg::PN, NO, t, vy);
    w32_put<Cfg::CHX>(xs, Cfg::PK, KI, t, vx);
    if (blk + gridDim.x < nblk) {
      w32_load<Cfg::CHY>(dY, M, NO, (blk + gridDim.x) * 64, t, vy);
      w32_load<Cfg::CHX>(X, M, KI, (blk + gridDim.x) * 64, t, vx);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < Cfg::TPW; ++i) {
      const int tile = wv + NW32 * i;
      if (tile < Cfg::TILES) {
        const int tn = tile / (KP / 16), tk = tile - tn * (KP / 16);
#pragma unroll 4
        for (int ks = 0; ks < 16; ++ks)        // 64 rows = 16 K-steps of 4 tokens
          acc[i] = mfma4(ys[(4 * ks + lg) * Cfg::PN + 16 * tn + l16], xs[(4 * ks + lg) * Cfg::PK + 16 * tk + l16],
                         acc[i]);
      }
    }
  }
  float* dst = part + (int64_t)blockIdx.x * NO * KI;
#pragma unroll
  for (int i = 0; i < Cfg::TPW; ++i) {
    const int tile = wv + NW32 * i;
    if (tile < Cfg::TILES) {
      const int tn = tile / (KP / 16), tk = tile - tn * (KP / 16);
      const int k = 16 * tk + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = 16 * tn + 4 * lg + r;
        if (n < NO && k < KI) dst[n * KI + k] = acc[i][r];
      }
    }
  }
}

template <int KP, int NP>
size_t narrow32_lds() { return sizeof(float) * ((size_t)NP * Narrow32Cfg<KP, NP>::BPF + (size_t)NW32 * Narrow32Cfg<KP, NP>::WAVE); }
template <int NP, int KP>
size_t wgrad32_lds() { return sizeof(float) * 2 * (size_t)Wgrad32Cfg<NP, KP>::BUF; }

inline int pad_to(int v, int q) { return (v + q - 1) / q * q; }

// resident workgroups: 4 per CU for the small (64 x 64) weight (115 VGPRs), 2 otherwise (up to 250 VGPRs);
// waves grid-stride over the 16-row blocks beyond that
int narrow_grid(int64_t M, int KI, int NO) {
  const int64_t nblk = (M + 15) / 16;
  const int64_t wg = (nblk + NW - 1) / NW;
  const int64_t cap = (KI <= 64 && NO <= 64) ? 256 * 4 : 256 * 2;
  return (int)(wg < cap ? wg : cap);
}

}  // namespace

// the weight stays in VGPRs as (KP / 32) x (NP / 16) B fragments: at most 24 of them (96 VGPRs)
PDT_API int pdt_narrow_gemm_ok(int64_t M, int KI, int NO) {
  if (M <= 0 || KI < 4 || KI > 192 || NO < 4 || NO > 192 || KI % 4 || NO % 4) return 0;
  const int KP = KI <= 64 ? 64 : KI <= 128 ? 128 : 192;
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  return (KP / 32) * (NP / 16) <= 24 ? 1 : 0;
}
// partial rows the COLSUM variant writes (= waves in the grid): the caller reduces [rows, KI] fp32
PDT_API int pdt_narrow_gemm_partials(int64_t M, int KI, int NO) { return narrow_grid(M, KI, NO) * NW; }

// Y [M, NO] bf16 = X [M, KI] bf16 . B [NO, KI]^T (+ bias [NO] bf16); X, Y contiguous and 16-byte aligned.
// colsum_out (nullable, fp32 [KI], W dtype by wdt): column sums of X -- written (not accumulated) -- with ws
// >= (pdt_narrow_gemm_partials(M, KI, NO) + 64) * KI floats (partials + the column reduce's second level).
// hm_n > 0: Y head-major (hm_store): M % hm_n == 0, hm_n % 16 == 0, NO % hm_d == 0, hm_d even
// and <= 32
static bool hm_ok(int64_t M, int NO, int hm_n, int hm_d) {
  return hm_n == 0 || (hm_n > 0 && hm_n % 16 == 0 && M % hm_n == 0 && M < (1ll << 31) && hm_d >= 2 && hm_d <= 32 &&
                       hm_d % 2 == 0 && NO % hm_d == 0);
}
// a_n > 0: X head-major ([M / a_n][KI / a_d][a_n][a_d], load_block_hm), same constraints as hm_n / hm_d on KI
// R (nullable): a residual [M, NO] added in the store (token-major output only; 16-byte aligned)
PDT_API int pdt_narrow_gemm(const void* X, const void* B, const void* bias, void* Y, int64_t M, int KI, int NO,
                            void* colsum_out, int wdt, float* ws, int hm_n, int hm_d, int a_n, int a_d, const void* R,
                            hipStream_t st) {
  if (!pdt_narrow_gemm_ok(M, KI, NO) || !hm_ok(M, NO, hm_n, hm_d) || !hm_ok(M, KI, a_n, a_d) || ((uintptr_t)X & 15) ||
      ((uintptr_t)Y & 15) || ((uintptr_t)R & 15) || (R && hm_n))
    return (int)hipErrorInvalidValue;
  const int KP = pad_to(KI, 64) <= 64 ? 64 : pad_to(KI, 64);
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const int grid = narrow_grid(M, KI, NO);
  float* part = colsum_out ? ws : nullptr;
  if ((hm_n > 0) + (a_n > 0) + (R != nullptr) > 1) return (int)hipErrorInvalidValue;   // one optional mode at a time
  const int mode = hm_n > 0 ? NG_HMY : a_n > 0 ? NG_HMA : R != nullptr ? NG_RES : NG_PLAIN;
#define PDT_NGM(KP_, NP_, M_)                                                                                    \
  narrow_gemm_kernel<KP_, NP_, M_><<<grid, 64 * NW, NW * NarrowCfg<KP_, NP_>::WAVE_ELEMS * sizeof(bf16_t), st>>>( \
      (const bf16_t*)X, (const bf16_t*)B, (const bf16_t*)bias, (bf16_t*)Y, part, M, KI, NO, hm_n, hm_d, a_n, a_d,  \
      (const bf16_t*)R)
#define PDT_NG(KP_, NP_)                                                                                        \
  do {                                                                                                          \
    if (mode == NG_HMY) PDT_NGM(KP_, NP_, NG_HMY);                                                              \
    else if (mode == NG_HMA) PDT_NGM(KP_, NP_, NG_HMA);                                                         \
    else if (mode == NG_RES) PDT_NGM(KP_, NP_, NG_RES);                                                         \
    else PDT_NGM(KP_, NP_, NG_PLAIN);                                                                           \
  } while (0)
#define PDT_NG_N(KP_) \
  do { if (NP == 64) PDT_NG(KP_, 64); else if (NP == 128) PDT_NG(KP_, 128); else PDT_NG(KP_, 192); } while (0)
  if (KP == 64) PDT_NG_N(64);
  else if (KP == 128) PDT_NG(128, 64);          // (the combinations pdt_narrow_gemm_ok admits)
  else PDT_NG(192, 64);
#undef PDT_NG_N
#undef PDT_NG
#undef PDT_NGM
  if (colsum_out) {
    const int R = grid * NW;
    float* ws2 = ws + (int64_t)R * KI;
    if (wdt == kBF16) red::col_reduce<bf16_t>(part, R, KI, (bf16_t*)colsum_out, ws2, 0, st);
    else red::col_reduce<float>(part, R, KI, (float*)colsum_out, ws2, 0, st);
  }
  return (int)hipGetLastError();
}

// ---- dW [NO, KI] (wdt: kF32 or kBF16) = dY[M, NO]^T X[M, KI]; dY, X contiguous, 16-byte aligned; NO, KI <= 192,
// multiples of 4.  ws >= pdt_narrow_wgrad_ws_floats(M, NO, KI) floats.
namespace {
// two workgroups per CU (their blocks' loads overlap each other's MFMAs and barriers)
int wgrad_grid(int64_t M) {
  const int64_t nblk = (M + WG_ROWS - 1) / WG_ROWS;
  return (int)(nblk < 512 ? nblk : 512);
}
}  // namespace
PDT_API int pdt_narrow_wgrad_ok(int64_t M, int NO, int KI) {
  return (M > 0 && NO >= 4 && NO <= 192 && KI >= 4 && KI <= 192 && NO % 4 == 0 && KI % 4 == 0) ? 1 : 0;
}
PDT_API int64_t pdt_narrow_wgrad_ws_floats(int64_t M, int NO, int KI) {
  return ((int64_t)wgrad_grid(M) + 64) * NO * KI;
}
// x_hm_d > 0: X head-major with 64-token windows ([M / 64][KI / x_hm_d][64][x_hm_d], wg_put_hm)
PDT_API int pdt_narrow_wgrad(const void* dY, const void* X, void* dW, int64_t M, int NO, int KI, int wdt, float* ws,
                             int x_hm_d, hipStream_t st) {
  if (!pdt_narrow_wgrad_ok(M, NO, KI) || ((uintptr_t)dY & 15) || ((uintptr_t)X & 15) ||
      (x_hm_d && (M % WG_ROWS || KI % x_hm_d || x_hm_d % 2)))
    return (int)hipErrorInvalidValue;
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const int KP = KI <= 64 ? 64 : KI <= 128 ? 128 : 192;
  const int grid = wgrad_grid(M);
#define PDT_WG(NP_, KP_)                                                                                       \
  narrow_wgrad_kernel<NP_, KP_><<<grid, 64 * WG_WAVES, wgrad_lds<NP_, KP_>(), st>>>(                          \
      (const bf16_t*)dY, (const bf16_t*)X, ws, M, NO, KI, x_hm_d)
#define PDT_WG_K(NP_) \
  do { if (KP == 64) PDT_WG(NP_, 64); else if (KP == 128) PDT_WG(NP_, 128); else PDT_WG(NP_, 192); } while (0)
  if (NP == 64) PDT_WG_K(64);
  else if (NP == 128) PDT_WG_K(128);
  else PDT_WG_K(192);
#undef PDT_WG_K
#undef PDT_WG
  float* ws2 = ws + (int64_t)grid * NO * KI;
  if (wdt == kBF16) red::col_reduce<bf16_t>(ws, grid, NO * KI, (bf16_t*)dW, ws2, 0, st);
  else red::col_reduce<float>(ws, grid, NO * KI, (float*)dW, ws2, 0, st);
  return (int)hipGetLastError();
}

// ---- fp32: Y [M, NO] = X [M, KI] . B [NO, KI]^T (+ bias [NO]); colsum_out (nullable, fp32 [KI]) as the bf16 entry,
// ws >= (pdt_narrow_gemm_f32_partials(M) + 64) * KI floats.  X, Y contiguous, 16-byte aligned; KI, NO <= 192, % 4.
namespace {
int narrow32_grid(int64_t M) {
  const int64_t nblk = (M + 15) / 16;
  const int64_t wg = (nblk + NW32 - 1) / NW32;
  return (int)(wg < 256 ? wg : 256);                         // one 8-wave workgroup per CU (the LDS weight tile)
}
template <int KP, int NP>
bool narrow32_attr() {
  static const bool ok =
      hipFuncSetAttribute((const void*)narrow_gemm_f32_kernel<KP, NP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)narrow32_lds<KP, NP>()) == hipSuccess;
  return ok;
}
template <int NP, int KP>
bool wgrad32_attr() {
  static const bool ok =
      hipFuncSetAttribute((const void*)narrow_wgrad_f32_kernel<NP, KP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)wgrad32_lds<NP, KP>()) == hipSuccess;
  return ok;
}
}  // namespace
PDT_API int pdt_narrow_gemm_f32_partials(int64_t M) { return narrow32_grid(M) * NW32; }
// the weight tile plus 8 waves' X tiles must fit the 160 KiB of LDS
PDT_API int pdt_narrow_gemm_f32_ok(int64_t M, int KI, int NO) {
  if (M <= 0 || KI < 4 || KI > 192 || NO < 4 || NO > 192 || KI % 4 || NO % 4) return 0;
  const int KP = KI <= 64 ? 64 : KI <= 128 ? 128 : 192;
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const size_t lds = sizeof(float) * ((size_t)NP * (KP + 1) + (size_t)NW32 * (16 * (KP + 1) > 16 * NP ? 16 * (KP + 1) : 16 * NP));
  return lds <= 160 * 1024 ? 1 : 0;
}
PDT_API int pdt_narrow_wgrad_f32_ok(int64_t M, int NO, int KI) {
  if (!pdt_narrow_wgrad_ok(M, NO, KI)) return 0;
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const int KP = KI <= 64 ? 64 : KI <= 128 ? 128 : 192;
  return sizeof(float) * 2 * 64 * (size_t)(NP + 1 + KP + 1) <= 160 * 1024 ? 1 : 0;
}
PDT_API int pdt_narrow_gemm_f32(const float* X, const float* B, const float* bias, float* Y, int64_t M, int KI, int NO,
                                float* colsum_out, float* ws, int hm_n, int hm_d, const float* R, hipStream_t st) {
  if (!pdt_narrow_gemm_f32_ok(M, KI, NO) || !hm_ok(M, NO, hm_n, hm_d) || ((uintptr_t)X & 15) || ((uintptr_t)Y & 15) ||
      ((uintptr_t)R & 15) || (R && hm_n))
    return (int)hipErrorInvalidValue;
  const int KP = KI <= 64 ? 64 : KI <= 128 ? 128 : 192;
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const int grid = narrow32_grid(M);
  float* part = colsum_out ? ws : nullptr;
#define PDT_N32(KP_, NP_)                                                                                         \
  do {                                                                                                            \
    if (!narrow32_attr<KP_, NP_>()) return (int)hipErrorInvalidValue;                                             \
    narrow_gemm_f32_kernel<KP_, NP_><<<grid, 64 * NW32, narrow32_lds<KP_, NP_>(), st>>>(X, B, bias, Y, part, M, KI, NO, \
                                                                                     hm_n, hm_d, R);              \
  } while (0)
#define PDT_N32_N(KP_) \
  do { if (NP == 64) PDT_N32(KP_, 64); else if (NP == 128) PDT_N32(KP_, 128); else PDT_N32(KP_, 192); } while (0)
  if (KP == 64) PDT_N32_N(64);
  else if (KP == 128) PDT_N32_N(128);
  else PDT_N32_N(192);
#undef PDT_N32_N
#undef PDT_N32
  if (colsum_out) {
    const int R = grid * NW32;
    red::col_reduce<float>(part, R, KI, colsum_out, ws + (int64_t)R * KI, 0, st);
  }
  return (int)hipGetLastError();
}
// fp32 dW [NO, KI] = dY^T X; ws >= pdt_narrow_wgrad_ws_floats(M, NO, KI) floats
PDT_API int pdt_narrow_wgrad_f32(const float* dY, const float* X, float* dW, int64_t M, int NO, int KI, float* ws,
                                 hipStream_t st) {
  if (!pdt_narrow_wgrad_f32_ok(M, NO, KI) || ((uintptr_t)dY & 15) || ((uintptr_t)X & 15))
    return (int)hipErrorInvalidValue;
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const int KP = KI <= 64 ? 64 : KI <= 128 ? 128 : 192;
  const int grid = wgrad_grid(M);
#define PDT_W32(NP_, KP_)                                                                                       \
  do {                                                                                                          \
    if (!wgrad32_attr<NP_, KP_>()) return (int)hipErrorInvalidValue;                                            \
    narrow_wgrad_f32_kernel<NP_, KP_><<<grid, 64 * NW32, wgrad32_lds<NP_, KP_>(), st>>>(dY, X, ws, M, NO, KI); \
  } while (0)
#define PDT_W32_K(NP_) \
  do { if (KP == 64) PDT_W32(NP_, 64); else if (KP == 128) PDT_W32(NP_, 128); else PDT_W32(NP_, 192); } while (0)
  if (NP == 64) PDT_W32_K(64);
  else if (NP == 128) PDT_W32_K(128);
  else PDT_W32_K(192);
#undef PDT_W32_K
#undef PDT_W32
  red::col_reduce<float>(ws, grid, NO * KI, dW, ws + (int64_t)grid * NO * KI, 0, st);
  return (int)hipGetLastError();
}
