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
#include <type_traits>

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

// channels-contiguous bf16 input (sc == 1, C % 4 == 0: SwinIR's [B, L, C] token tensors viewed as NHWC):
// every K run of one (kh, kw) tap is C contiguous input elements, so each thread moves 4 channels with
// one 8-byte load and one 8-byte store (coalesced both ways) instead of 8 two-byte gathers.
__global__ __launch_bounds__(NT) void im2col3x3_c4_kernel(const bf16_t* __restrict__ x, int64_t sn, int64_t sh,
                                                          int64_t sw, int C, int H, int W, int Kp, int64_t total4,
                                                          bf16_t* __restrict__ out) {
  const int kp4 = Kp >> 2, c4n = C >> 2;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < total4; i += (int64_t)gridDim.x * NT) {
    const int64_t p = i / kp4;
    const int j = (int)(i - p * kp4);
    const int kk = j / c4n, c = (j - kk * c4n) * 4;
    const int w = (int)(p % W);
    const int64_t t = p / W;
    const int h = (int)(t % H);
    const int64_t n = t / H;
    u16x4 v = {0, 0, 0, 0};
    if (kk < 9) {
      const int ih = h + kk / 3 - 1, iw = w + kk % 3 - 1;
      if (ih >= 0 && ih < H && iw >= 0 && iw < W) v = *reinterpret_cast<const u16x4*>(x + n * sn + ih * sh + iw * sw + c);
    }
    *reinterpret_cast<u16x4*>(out + i * 4) = v;
  }
}

// channels-contiguous input, a workgroup per 16 consecutive output rows (pixels): thread e of the block's
// 16 x Kp/4 four-element vectors (8 bytes bf16, 16 bytes fp32) -- consecutive threads, consecutive vectors, so loads
// and stores stay coalesced -- with its (pixel, tap, channel) split by float reciprocals of small operands (exact:
// e < 2^16) and the block's first (n, h, w) computed once; the 64-bit divisions per vector had made the c4 kernel
// VALU-bound at ~2.5 TB/s.
constexpr int IM_PIX = 16;
__device__ __forceinline__ int fdiv_small(int a, float inv) { return __float2int_rz(((float)a + 0.5f) * inv); }
template <typename T>
__global__ __launch_bounds__(NT) void im2col3x3_blk_kernel(const T* __restrict__ x, int64_t sn, int64_t sh,
                                                           int64_t sw, int C, int H, int W, int Kp, int64_t npix,
                                                           T* __restrict__ out) {
  typedef typename std::conditional<sizeof(T) == 2, u16x4, f32x4>::type V;
  const int kp4 = Kp / 4, c4n = C / 4;
  const float inv_kp4 = 1.f / (float)kp4, inv_c4n = 1.f / (float)c4n;
  for (int64_t p0 = (int64_t)blockIdx.x * IM_PIX; p0 < npix; p0 += (int64_t)gridDim.x * IM_PIX) {
    const int w0 = (int)(p0 % W);
    const int64_t t0 = p0 / W;
    const int h0 = (int)(t0 % H);
    const int64_t n0 = t0 / H;
    const int npx = npix - p0 < IM_PIX ? (int)(npix - p0) : IM_PIX;
    for (int e = threadIdx.x; e < npx * kp4; e += NT) {
      const int pl = fdiv_small(e, inv_kp4), jq = e - pl * kp4;
      int w = w0 + pl, h = h0;
      int64_t n = n0;
      while (w >= W) {
        w -= W;
        if (++h == H) { h = 0; ++n; }
      }
      V v = {};
      const int kk = fdiv_small(jq, inv_c4n);
      if (kk < 9) {
        const int c = (jq - kk * c4n) * 4;
        const int ih = h + kk / 3 - 1, iw = w + kk % 3 - 1;
        if (ih >= 0 && ih < H && iw >= 0 && iw < W) v = *reinterpret_cast<const V*>(x + n * sn + ih * sh + iw * sw + c);
      }
      reinterpret_cast<V*>(out + (p0 + pl) * Kp)[jq] = v;
    }
  }
}

}  // namespace

// x: logical [N, C, H, W] with element strides (sn, sc, sh, sw); out: [N*H*W, Kp] row-major, Kp % 8 == 0,
// Kp >= 9C.  dtype: kF32 / kBF16.
PDT_API int pdt_im2col3x3(const void* x, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int N, int C, int H, int W,
                          int Kp, void* out, int dt, hipStream_t st) {
  if (Kp % 8 != 0 || Kp < 9 * C || N <= 0 || C <= 0 || H <= 0 || W <= 0) return (int)hipErrorInvalidValue;
  const int es = dt == kBF16 ? 2 : 4;
  if ((dt == kBF16 || dt == kF32) && sc == 1 && C % 4 == 0 && sn % 4 == 0 && sh % 4 == 0 && sw % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(x) & (4 * es - 1)) == 0 && (reinterpret_cast<uintptr_t>(out) & (4 * es - 1)) == 0 &&
      IM_PIX * (Kp / 4) < (1 << 16)) {
    const int64_t npix = (int64_t)N * H * W;
    const int grid = grid_for(npix, IM_PIX, 256 * 16);
    if (dt == kBF16)
      im2col3x3_blk_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)x, sn, sh, sw, C, H, W, Kp, npix,
                                                        (bf16_t*)out);
    else
      im2col3x3_blk_kernel<float><<<grid, NT, 0, st>>>((const float*)x, sn, sh, sw, C, H, W, Kp, npix, (float*)out);
    return (int)hipGetLastError();
  }
  if (dt == kBF16 && sc == 1 && C % 4 == 0 && sn % 4 == 0 && sh % 4 == 0 && sw % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(x) & 7) == 0) {
    const int64_t total4 = (int64_t)N * H * W * (Kp / 4);
    im2col3x3_c4_kernel<<<grid_for(total4, NT, 256 * 16), NT, 0, st>>>((const bf16_t*)x, sn, sh, sw, C, H, W, Kp,
                                                                        total4, (bf16_t*)out);
    return (int)hipGetLastError();
  }
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

// ------------------------------------------------------------------------------------------------
// Shifted-window partition / reverse as ONE row permutation (SwinIR's torch.roll +
// window_partition + window_reverse + torch.roll + residual add are 3-5 passes over the activation; here
// partition is one gather pass and reverse (+ residual) one pass).  x is [B, H, W, C] (row = one token,
// C contiguous elements); windows are [B * nWh * nWw, ws * ws, C].  Window token (b, wh, ww, i, j) takes
// image token (b, (wh*ws + i + s) mod H, (ww*ws + j + s) mod W) -- torch.roll(x, (-s, -s), (1, 2)) then
// partition.  REVERSE maps back (inverse permutation) and optionally adds the residual.
// ------------------------------------------------------------------------------------------------
namespace {
// T = bf16_t (8-byte chunks of 4) or float (16-byte chunks of 4: the fp32 model, the reference's precision)
template <typename T, bool REVERSE, bool RES>
__global__ __launch_bounds__(256) void window_perm_kernel(const T* __restrict__ src, const T* __restrict__ res,
                                                          T* __restrict__ dst, int64_t rows, int C, int H, int W,
                                                          int ws, int shift) {
  typedef typename std::conditional<sizeof(T) == 2, u16x4, f32x4>::type V;
  const int cpr = C / 4;                      // 4-element chunks per row
  const int nww = W / ws, per_img = H * W;
  const int64_t total = rows * cpr;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / cpr;
    const int ch = (int)(e - r * cpr);
    int64_t img_row, win_row;
    if (!REVERSE) {                           // r = window-order row
      win_row = r;
      const int64_t b = r / per_img;
      const int t = (int)(r - b * per_img);
      const int wi = t / (ws * ws), k = t - wi * ws * ws;
      const int wh = wi / nww, ww = wi - wh * nww, i = k / ws, j = k - i * ws;
      int h = wh * ws + i + shift, w = ww * ws + j + shift;
      if (h >= H) h -= H;
      if (w >= W) w -= W;
      img_row = b * per_img + (int64_t)h * W + w;
    } else {                                  // r = image-order row
      img_row = r;
      const int64_t b = r / per_img;
      const int t = (int)(r - b * per_img);
      int h = t / W - shift, w = t % W - shift;
      if (h < 0) h += H;
      if (w < 0) w += W;
      const int wh = h / ws, i = h - wh * ws, ww = w / ws, j = w - ww * ws;
      win_row = b * per_img + (int64_t)(wh * nww + ww) * ws * ws + i * ws + j;
    }
    const int64_t so = (REVERSE ? win_row : img_row) * C + ch * 4;
    const int64_t dof = (REVERSE ? img_row : win_row) * C + ch * 4;
    V v = *reinterpret_cast<const V*>(src + so);
    if (RES) {
      const V a = *reinterpret_cast<const V*>(res + dof);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = from_f<T>(to_f<T>((T)v[k]) + to_f<T>((T)a[k]));
    }
    *reinterpret_cast<V*>(dst + dof) = v;
  }
}
}  // namespace

// reverse = 0: windows = partition(roll(x, -shift)); reverse = 1: x = roll(reverse(windows), +shift) (+ res).
// C % 4 == 0, H % ws == 0, W % ws == 0, 0 <= shift < ws.
namespace {
template <typename T>
int window_perm_launch(const void* src, const void* res, void* dst, int64_t rows, int C, int H, int W, int ws,
                       int shift, int reverse, hipStream_t st) {
  if (C % 4 || H % ws || W % ws || shift < 0 || shift >= ws || rows % ((int64_t)H * W)) return (int)hipErrorInvalidValue;
  const int64_t total = rows * (C / 4);
  const int grid = grid_for(total, 256, 256 * 16);
  if (reverse) {
    if (res) window_perm_kernel<T, true, true><<<grid, 256, 0, st>>>((const T*)src, (const T*)res, (T*)dst, rows, C, H, W, ws, shift);
    else window_perm_kernel<T, true, false><<<grid, 256, 0, st>>>((const T*)src, nullptr, (T*)dst, rows, C, H, W, ws, shift);
  } else {
    window_perm_kernel<T, false, false><<<grid, 256, 0, st>>>((const T*)src, nullptr, (T*)dst, rows, C, H, W, ws, shift);
  }
  return (int)hipGetLastError();
}
}  // namespace
PDT_API int pdt_window_perm(const void* src, const void* res, void* dst, int64_t rows, int C, int H, int W, int ws,
                            int shift, int reverse, hipStream_t st) {
  return window_perm_launch<bf16_t>(src, res, dst, rows, C, H, W, ws, shift, reverse, st);
}
PDT_API int pdt_window_perm_f32(const void* src, const void* res, void* dst, int64_t rows, int C, int H, int W, int ws,
                                int shift, int reverse, hipStream_t st) {
  return window_perm_launch<float>(src, res, dst, rows, C, H, W, ws, shift, reverse, st);
}

// ------------------------------------------------------------------------------------------------
// SwinIR 'pixelshuffledirect' tail: PixelShuffle(r) of the upsample convolution's output
// fused with the model's de-normalisation ``x / img_range + mean[c]`` -- one pass instead of a
// pixel_shuffle copy plus two elementwise passes (and their three backward passes).  The conv output
// arrives as its channels_last view (any strides), the image leaves channels_last (NHWC buffer), the
// layout torch's pixel_shuffle keeps for a channels_last input and the loss network's convolutions take:
//   out[n, c, h*r + i, w*r + j] = y[n, c*r*r + i*r + j, h, w] * a + b[c]
// Backward writes dy NHWC-contiguous ([N*H*W, C*r*r] rows), the layout the conv's backward GEMMs read
// without a copy:  dy[n, c*r*r + i*r + j, h, w] = dout[n, c, h*r + i, w*r + j] * a
// ------------------------------------------------------------------------------------------------
namespace {
template <typename T>
__global__ __launch_bounds__(256) void pixel_shuffle_affine_fwd(const T* __restrict__ y, int64_t sn, int64_t sc,
                                                                int64_t sh, int64_t sw, int C, int H, int W, int r,
                                                                float a, const float* __restrict__ b,
                                                                T* __restrict__ out, int64_t total) {
  const int Ho = H * r, Wo = W * r;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);              // NHWC order: the channels of one output pixel are adjacent
    int64_t t = e / C;
    const int wo = (int)(t % Wo);
    t /= Wo;
    const int ho = (int)(t % Ho);
    const int64_t n = t / Ho;
    const int h = ho / r, i = ho - h * r, w = wo / r, j = wo - w * r;
    const float v = to_f(y[n * sn + (int64_t)(c * r * r + i * r + j) * sc + h * sh + w * sw]);
    out[e] = from_f<T>(fmaf(v, a, b ? b[c] : 0.f));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pixel_shuffle_affine_bwd(const T* __restrict__ dout, int64_t dn, int64_t dc,
                                                                int64_t dh, int64_t dw, int C, int H, int W, int r,
                                                                float a, T* __restrict__ dy, int64_t total) {
  const int crr = C * r * r;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int ch = (int)(e % crr);
    int64_t p = e / crr;
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int64_t n = p / H;
    const int c = ch / (r * r), i = (ch / r) % r, j = ch % r;
    dy[e] = from_f<T>(to_f(dout[n * dn + c * dc + (int64_t)(h * r + i) * dh + (int64_t)(w * r + j) * dw]) * a);
  }
}
}  // namespace

// y: logical [N, C*r*r, H, W] with element strides (sn, sc, sh, sw); out: NHWC buffer [N, H*r, W*r, C].
// b: optional fp32 [C] (nullptr = 0).  dtype: kF32 / kBF16.
PDT_API int pdt_pixel_shuffle_affine_fwd(const void* y, int64_t sn, int64_t sc, int64_t sh, int64_t sw, int N, int C,
                                         int H, int W, int r, float a, const float* b, void* out, int dt,
                                         hipStream_t st) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || r <= 0) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * C * H * r * W * r;
  const int grid = grid_for(total, 256, 256 * 16);
  if (dt == kBF16)
    pixel_shuffle_affine_fwd<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)y, sn, sc, sh, sw, C, H, W, r, a, b,
                                                           (bf16_t*)out, total);
  else if (dt == kF32)
    pixel_shuffle_affine_fwd<float><<<grid, 256, 0, st>>>((const float*)y, sn, sc, sh, sw, C, H, W, r, a, b,
                                                          (float*)out, total);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// dout: logical [N, C, H*r, W*r] with element strides (dn, dc, dh, dw); dy: [N*H*W, C*r*r] contiguous.
PDT_API int pdt_pixel_shuffle_affine_bwd(const void* dout, int64_t dn, int64_t dc, int64_t dh, int64_t dw, int N,
                                         int C, int H, int W, int r, float a, void* dy, int dt, hipStream_t st) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || r <= 0) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W * C * r * r;
  const int grid = grid_for(total, 256, 256 * 16);
  if (dt == kBF16)
    pixel_shuffle_affine_bwd<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)dout, dn, dc, dh, dw, C, H, W, r, a,
                                                           (bf16_t*)dy, total);
  else if (dt == kF32)
    pixel_shuffle_affine_bwd<float><<<grid, 256, 0, st>>>((const float*)dout, dn, dc, dh, dw, C, H, W, r, a,
                                                          (float*)dy, total);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
