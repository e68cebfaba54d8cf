// 3x3 / stride 1 / pad 1 convolution support for the small-channel convolutions of SwinIR-S (SURVEY.md
// K1: conv_first 3->60, four RSTB convs 60->60, conv_after_body 60->60, upsample 60->12 at 18 x 128 x 128).
// MIOpen has no implicit-GEMM solver for these channel counts in bf16 and falls back to its naive
// direct kernels (hundreds of ms per weight-gradient call, profiles/r1_v5_swinir_stoke_kernel_stats.csv);
// here the convolution is lowered to ONE hipBLASLt GEMM over an explicit im2col matrix:
//
//   cols[P, Kp]  (P = N*H*W pixels, K = (kh*3 + kw)*C + c, zero columns up to Kp = roundup(9C, 8))
//   y  = cols @ Wm            (forward, Wm[Kp, Cout] = weight permuted to (kh, kw, c) rows)
//   dW = dY^T @ cols          (weight gradient: one GEMM with K = P)
//   dX = im2col(dY) @ Wflip   (data gradient = 3x3 conv of dY with the flipped / transposed weight)
//
// The im2col kernel reads ANY input strides (NCHW images, the NHWC-strided views SwinIR produces from
// [B, L, C] token tensors, channels_last gradients), so no layout copy precedes it, and writes 16-byte
// rows of 8 consecutive K entries per thread.
#include "common.h"

using namespace pdt;

namespace {

constexpr int NT = 256;

template <typename T>
__global__ __launch_bounds__(NT) void im2col3x3_kernel(const T* __restrict__ x, int64_t sn, int64_t sc, int64_t sh,
                                                       int64_t sw, int C, int H, int W, int Kp, int64_t total8,
                                                       T* __restrict__ out) {
  const int kp8 = Kp >> 3;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total8; i += (int64_t)gridDim.x * NT) {
    const int64_t p = i / kp8;
    const int k0 = (int)(i - p * kp8) * 8;
    const int w = (int)(p % W);
    const int64_t t = p / W;
    const int h = (int)(t % H);
    const int64_t n = t / H;
    int kk = k0 / C, c = k0 - kk * C;
    T v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      T val = from_f<T>(0.f);
      if (kk < 9) {
        const int ih = h + kk / 3 - 1, iw = w + kk % 3 - 1;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W) val = x[n * sn + c * sc + ih * sh + iw * sw];
      }
      v[j] = val;
      if (++c == C) { c = 0; ++kk; }
    }
    if constexpr (sizeof(T) == 2) {
      u16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = v[j];
      *reinterpret_cast<u16x8*>(out + i * 8) = r;
    } else {
      Vec8<float>::store(reinterpret_cast<float*>(out) + i * 8, reinterpret_cast<const float*>(v));
    }
  }
}

}  // namespace

// x: logical [N, C, H, W] with element strides (sn, sc, sh, sw); out: [N*H*W, Kp] row-major, Kp % 8 == 0,
// Kp >= 9C.  dtype: kF32 / kBF16.
PDT_API int pdt_im2col3x3(const void* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int N, int C, int H, int W,
                          int Kp, void* out, int dt, hipStream_t st) {
  if (Kp % 8 != 0 || Kp < 9 * C || N <= 0 || C <= 0 || H <= 0 || W <= 0) return (int)hipErrorInvalidValue;
  const int64_t total8 = (int64_t)N * H * W * (Kp / 8);
  const int grid = grid_for(total8, NT, 256 * 16);
  if (dt == kBF16)
    im2col3x3_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)x, sn, sc, sh, sw, C, H, W, Kp, total8, (bf16_t*)out);
  else if (dt == kF32)
    im2col3x3_kernel<float><<<grid, NT, 0, st>>>((const float*)x, sn, sc, sh, sw, C, H, W, Kp, total8, (float*)out);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
