// Implicit-GEMM 3x3 / stride 1 / pad 1 convolution for narrow channel counts (CI, CO <= 64, NHWC), gfx950 MFMA.
//
// SwinIR-S's body convolutions (60 -> 60 at 18 x 128 x 128 per device: the four RSTB convs and conv_after_body,
// SURVEY.md K1) ran as im2col + GEMM: the im2col matrix is 9 x the activation (318 MB bf16) written once and read
// once by a bandwidth-bound GEMM -- ~265 us per call.  Here nothing of that size exists: a workgroup keeps the
// whole weight in LDS as [CO][9 taps x 64 channels] (channels zero-padded to 64, so a 32-wide MFMA K-step never
// straddles a tap), and each wave computes 16 consecutive output pixels of one image row at a time:
//   * the 3 x 18 input pixels the block touches (halo zero-filled) are staged in the wave's LDS tile
//     [3][18][64 + 8] with 8-byte loads (pixel rows of CI bf16 are only 8-byte aligned for CI = 60),
//   * 18 K-steps (tap, channel half) x CO/16 output tiles of v_mfma_f32_16x16x32_bf16, A fragments from the
//     input tile at (kh, pixel + kw), B fragments from the weight tile,
//   * bias added, the 16 x CO block staged and written as contiguous 16-byte stores (NHWC rows are contiguous).
// The next block's input is loaded into registers before the current block's MFMAs.  The data gradient is the
// same kernel on dY with the flipped, transposed weight (prepared by the caller).
#include "common.h"

using namespace pdt;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int NWV = 8;                       // waves per workgroup (2 per SIMD; the weight tile is shared)
constexpr int CP = 64;                       // channels per tap, padded
constexpr int KT = 9 * CP;                   // 576
constexpr int BP = KT + 8;                   // weight row pitch (elements): 16-byte aligned, rows on distinct banks
constexpr int XPC = CP + 8;                  // input tile pixel pitch (elements)
constexpr int TILE_X = 3 * 18 * XPC;         // input tile (elements)
constexpr int LD_PER_LANE = (3 * 18 * (CP / 4) + 63) / 64;   // 8-byte input loads per lane per block (upper bound)

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

struct Geo {
  int N, H, W, CI, CO, relu;   // relu: max(0, .) on the biased output (a conv + ReLU pair in one pass)
};

// the 3 x 18 input pixels of block `blk` (n, h, w0) as 8-byte chunks: chunk q = lane + 64 i -> (row r, pixel p,
// channels 4c .. 4c+3); zero outside the image (the convolution's padding)
__device__ __forceinline__ void load_x(const bf16_t* __restrict__ X, const Geo& g, int64_t blk, int lane,
                                       u16x4 (&v)[LD_PER_LANE]) {
  // 32-bit divisions (blocks < 2^31, host check): 64-bit ones cost ~100 VALU each per block
  const uint32_t wb = (uint32_t)(g.W / 16), b32 = (uint32_t)blk;
  const uint32_t nh = b32 / wb;
  const int w0 = (int)(b32 - nh * wb) * 16;
  const uint32_t n32 = nh / (uint32_t)g.H;
  const int h = (int)(nh - n32 * (uint32_t)g.H);
  const int64_t n = n32;
  const int cq = g.CI / 4, tot = 3 * 18 * cq;
#pragma unroll
  for (int i = 0; i < LD_PER_LANE; ++i) {
    const int q = lane + 64 * i;
    u16x4 z = {0, 0, 0, 0};
    if (q < tot) {
      const int rp = q / cq, c = q - rp * cq;
      const int r = rp / 18, p = rp - r * 18;
      const int hh = h + r - 1, ww = w0 + p - 1;
      if (hh >= 0 && hh < g.H && ww >= 0 && ww < g.W)
        z = *reinterpret_cast<const u16x4*>(X + (((n * g.H + hh) * g.W + ww) * g.CI + 4 * c));
    }
    v[i] = z;
  }
}

__device__ __forceinline__ void put_x(bf16_t* Xs, const Geo& g, int lane, const u16x4 (&v)[LD_PER_LANE]) {
  const int cq = g.CI / 4, tot = 3 * 18 * cq;
#pragma unroll
  for (int i = 0; i < LD_PER_LANE; ++i) {
    const int q = lane + 64 * i;
    if (q < tot) {
      const int rp = q / cq, c = q - rp * cq;
      *reinterpret_cast<u16x4*>(Xs + rp * XPC + 4 * c) = v[i];
    }
  }
}

template <int NT>    // output tiles of 16 channels (CO <= 16 NT)
__global__ __launch_bounds__(64 * NWV, 1) void conv3x3_igemm_kernel(const bf16_t* __restrict__ X,
                                                                    const bf16_t* __restrict__ Wk,
                                                                    const bf16_t* __restrict__ bias,
                                                                    bf16_t* __restrict__ Y, Geo g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t csm[];
  bf16_t* Bs = csm;                                          // [16 NT][BP]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  bf16_t* Xs = csm + 16 * NT * BP + wv * (TILE_X + 16 * 16 * NT);
  bf16_t* Ys = Xs + TILE_X;                                   // [16][CO] output staging
  // the weight [CO][576] (caller-padded: channels CI .. 63 of every tap are zero) into LDS, rows >= CO zero
  for (int e = threadIdx.x; e < 16 * NT * (KT / 8); e += 64 * NWV) {
    const int n = e / (KT / 8), k8 = e - n * (KT / 8);
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (n < g.CO) v = *reinterpret_cast<const u16x8*>(Wk + (int64_t)n * KT + 8 * k8);
    *reinterpret_cast<u16x8*>(Bs + n * BP + 8 * k8) = v;
  }
  for (int e = lane; e < TILE_X; e += 64) Xs[e] = 0;          // channels CI .. 63 stay zero
  float bcol[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = 16 * nt + l16;
    bcol[nt] = (bias != nullptr && n < g.CO) ? bf2f(bias[n]) : 0.f;
  }
  __syncthreads();

  const int64_t nblk = (int64_t)g.N * g.H * (g.W / 16);
  const int64_t gw = (int64_t)blockIdx.x * NWV + wv, nwaves = (int64_t)gridDim.x * NWV;
  u16x4 v[LD_PER_LANE];
  if (gw < nblk) load_x(X, g, gw, lane, v);
  for (int64_t blk = gw; blk < nblk; blk += nwaves) {
    wave_sync();
    put_x(Xs, g, lane, v);
    if (blk + nwaves < nblk) load_x(X, g, blk + nwaves, lane, v);
    wave_sync();
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - 3 * kh;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const u16x8 a = *reinterpret_cast<const u16x8*>(Xs + (kh * 18 + l16 + kw) * XPC + 32 * half + 8 * lg);
        const int k0 = tap * CP + 32 * half + 8 * lg;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[nt] = mfma16(a, *reinterpret_cast<const u16x8*>(Bs + (16 * nt + l16) * BP + k0), acc[nt]);
      }
    }
    // C[pixel 4 lg + r][channel 16 nt + l16] -> [16][CO] staging -> contiguous NHWC rows
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = 16 * nt + l16;
      if (n < g.CO) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[nt][r] + bcol[nt];
          Ys[(4 * lg + r) * g.CO + n] = f2bf(g.relu ? fmaxf(v, 0.f) : v);
        }
      }
    }
    wave_sync();
    bf16_t* dst = Y + blk * 16 * g.CO;         // 16 consecutive pixels of one row: contiguous in NHWC
    const int n8 = 2 * g.CO;                   // 16 * CO / 8 whole chunks for any CO
    for (int c = lane; c < n8; c += 64) *reinterpret_cast<u16x8*>(dst + 8 * c) = *reinterpret_cast<const u16x8*>(Ys + 8 * c);
  }
}

template <int NT>
size_t igemm_lds() { return sizeof(bf16_t) * ((size_t)16 * NT * BP + (size_t)NWV * (TILE_X + 16 * 16 * NT)); }

}  // namespace

PDT_API int pdt_conv3x3_igemm_ok(int N, int H, int W, int CI, int CO) {
  // (any CO <= 64: a block's 16 x CO outputs are 2 CO whole 16-byte chunks -- CO = 3 is the data gradient of an
  // RGB-input conv, the perceptual loss's first VGG layer)
  return (N > 0 && H > 0 && W % 16 == 0 && CI >= 4 && CI <= 64 && CI % 4 == 0 && CO >= 1 && CO <= 64 &&
          (int64_t)N * H * (W / 16) < (1ll << 31)) ? 1 : 0;
}

// X [N, H, W, CI] bf16 NHWC-contiguous (8-byte aligned); Wk [CO][9][64] bf16 (tap-major, channels zero-padded to 64:
// Wk[co][kh*3+kw][ci] = w[co][ci][kh][kw]); bias [CO] or null; Y [N, H, W, CO] bf16 (16-byte aligned).
// relu != 0: y = max(0, conv + bias)
PDT_API int pdt_conv3x3_igemm_act(const void* X, const void* Wk, const void* bias, void* Y, int N, int H, int W,
                                  int CI, int CO, int relu, hipStream_t st) {
  if (!pdt_conv3x3_igemm_ok(N, H, W, CI, CO) || ((uintptr_t)X & 7) || ((uintptr_t)Y & 15) || ((uintptr_t)Wk & 15))
    return (int)hipErrorInvalidValue;
  const Geo g{N, H, W, CI, CO, relu};
  const int64_t nblk = (int64_t)N * H * (W / 16);
  const int64_t want = (nblk + NWV - 1) / NWV;
  const int grid = (int)(want < 256 ? want : 256);          // one 8-wave workgroup per CU (the LDS weight tile)
  static bool attr = [] {
    return hipFuncSetAttribute((const void*)conv3x3_igemm_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)igemm_lds<4>()) == hipSuccess;
  }();
  if (!attr) return (int)hipErrorInvalidValue;
  conv3x3_igemm_kernel<4><<<grid, 64 * NWV, igemm_lds<4>(), st>>>((const bf16_t*)X, (const bf16_t*)Wk,
                                                                 (const bf16_t*)bias, (bf16_t*)Y, g);
  return (int)hipGetLastError();
}

PDT_API int pdt_conv3x3_igemm(const void* X, const void* Wk, const void* bias, void* Y, int N, int H, int W, int CI,
                              int CO, hipStream_t st) {
  return pdt_conv3x3_igemm_act(X, Wk, bias, Y, N, H, W, CI, CO, 0, st);
}
