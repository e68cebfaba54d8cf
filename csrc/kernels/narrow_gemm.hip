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

template <int KP, int NP>
__global__ __launch_bounds__(64 * NW, 2) void narrow_gemm_kernel(const bf16_t* __restrict__ X,
                                                                 const bf16_t* __restrict__ B,
                                                                 const bf16_t* __restrict__ bias,
                                                                 bf16_t* __restrict__ Y, float* __restrict__ colsum_part,
                                                                 int64_t M, int KI, int NO) {
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
  if (gw < nblk) load_block<KP, NP>(X, M, KI, gw, lane, ch);
  for (int64_t blk = gw; blk < nblk; blk += nwaves) {
    const int rows = M - blk * 16 < 16 ? (int)(M - blk * 16) : 16;
    wave_sync();                                 // the previous block's LDS reads are done
    put_block<KP, NP>(Xs, KI, rows, lane, ch);
    if (blk + nwaves < nblk) load_block<KP, NP>(X, M, KI, blk + nwaves, lane, ch);   // in flight under the MFMAs
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
    bf16_t* dst = Y + blk * 16 * NO;
    const int tot = rows * NO, n8 = tot >> 3;
    for (int c = lane; c < n8; c += 64) *reinterpret_cast<u16x8*>(dst + 8 * c) = *reinterpret_cast<const u16x8*>(Ys + 8 * c);
    for (int e = 8 * n8 + lane; e < tot; e += 64) dst[e] = Ys[e];
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
PDT_API int pdt_narrow_gemm(const void* X, const void* B, const void* bias, void* Y, int64_t M, int KI, int NO,
                            void* colsum_out, int wdt, float* ws, hipStream_t st) {
  if (!pdt_narrow_gemm_ok(M, KI, NO) || ((uintptr_t)X & 15) || ((uintptr_t)Y & 15)) return (int)hipErrorInvalidValue;
  const int KP = pad_to(KI, 64) <= 64 ? 64 : pad_to(KI, 64);
  const int NP = NO <= 64 ? 64 : NO <= 128 ? 128 : 192;
  const int grid = narrow_grid(M, KI, NO);
  float* part = colsum_out ? ws : nullptr;
#define PDT_NG(KP_, NP_)                                                                                        \
  narrow_gemm_kernel<KP_, NP_><<<grid, 64 * NW, NW * NarrowCfg<KP_, NP_>::WAVE_ELEMS * sizeof(bf16_t), st>>>(   \
      (const bf16_t*)X, (const bf16_t*)B, (const bf16_t*)bias, (bf16_t*)Y, part, M, KI, NO)
#define PDT_NG_N(KP_) \
  do { if (NP == 64) PDT_NG(KP_, 64); else if (NP == 128) PDT_NG(KP_, 128); else PDT_NG(KP_, 192); } while (0)
  if (KP == 64) PDT_NG_N(64);
  else if (KP == 128) PDT_NG(128, 64);          // (the combinations pdt_narrow_gemm_ok admits)
  else PDT_NG(192, 64);
#undef PDT_NG_N
#undef PDT_NG
  if (colsum_out) {
    const int R = grid * NW;
    float* ws2 = ws + (int64_t)R * KI;
    if (wdt == kBF16) red::col_reduce<bf16_t>(part, R, KI, (bf16_t*)colsum_out, ws2, 0, st);
    else red::col_reduce<float>(part, R, KI, (float*)colsum_out, ws2, 0, st);
  }
  return (int)hipGetLastError();
}
