// Max pooling for channels-last (NHWC) bf16 activations on gfx950 -- the ResNet stem's 3x3 / stride-2 / pad-1
// pool (BASELINE.json config 2).  torch's NHWC kernels save an int64 argmax per output element (8 B, 4x the bf16
// output itself: 411 MB at batch 256) and scatter the backward through it; here:
//
//   forward  : y = max over the window, plus ONE BYTE per output element naming the winning window slot
//              (kh * k + kw; the first maximum in row-major scan order, a NaN replaces it -- torch's rule)
//   backward : gather, not scatter -- a thread owns 8 channels of one INPUT pixel and sums dy over the (at most
//              ceil(k / s)^2) windows whose recorded slot is that pixel: no atomics, bitwise deterministic
//
// Threads own 8 consecutive channels (16-byte loads / stores, 8-byte slot words).  C % 8 == 0.
#include "common.h"

using namespace pdt;

namespace {

constexpr int NT = 256;

struct PoolGeom {
  int N, C, H, W, OH, OW, k, s, p;
};

__global__ __launch_bounds__(NT) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         uint8_t* __restrict__ slot, PoolGeom g) {
  const int G = g.C >> 3;
  const int64_t total = (int64_t)g.N * g.OH * g.OW * G;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cg = (int)(t % G);
    const int64_t pix = t / G;                      // output pixel (n, oh, ow)
    const int ow = (int)(pix % g.OW);
    const int oh = (int)((pix / g.OW) % g.OH);
    const int n = (int)(pix / ((int64_t)g.OW * g.OH));
    float m[8];
    unsigned idx[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { m[c] = -INFINITY; idx[c] = 0; }
    const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
    for (int i = 0; i < g.k; ++i) {
      const int h = h0 + i;
      if (h < 0 || h >= g.H) continue;
      for (int j = 0; j < g.k; ++j) {
        const int w = w0 + j;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        Vec8<bf16_t>::load(x + (((int64_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
        const unsigned code = (unsigned)(i * g.k + j);
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (v[c] > m[c] || __builtin_isnan(v[c])) { m[c] = v[c]; idx[c] = code; }
      }
    }
    Vec8<bf16_t>::store(y + pix * g.C + cg * 8, m);
    uint2 packed;
    packed.x = idx[0] | (idx[1] << 8) | (idx[2] << 16) | (idx[3] << 24);
    packed.y = idx[4] | (idx[5] << 8) | (idx[6] << 16) | (idx[7] << 24);
    *reinterpret_cast<uint2*>(slot + pix * g.C + cg * 8) = packed;
  }
}

__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ slot,
                                                         bf16_t* __restrict__ dx, PoolGeom g) {
  const int G = g.C >> 3;
  const int64_t total = (int64_t)g.N * g.H * g.W * G;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cg = (int)(t % G);
    const int64_t pix = t / G;                      // input pixel (n, h, w)
    const int w = (int)(pix % g.W);
    const int h = (int)((pix / g.W) % g.H);
    const int n = (int)(pix / ((int64_t)g.W * g.H));
    // windows oh with oh * s - p <= h <= oh * s - p + k - 1
    const int ohs = max(0, (h + g.p - g.k + g.s) / g.s), ohe = min(g.OH - 1, (h + g.p) / g.s);
    const int ows = max(0, (w + g.p - g.k + g.s) / g.s), owe = min(g.OW - 1, (w + g.p) / g.s);
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.f;
    for (int oh = ohs; oh <= ohe; ++oh) {
      const int i = h - (oh * g.s - g.p);
      for (int ow = ows; ow <= owe; ++ow) {
        const int j = w - (ow * g.s - g.p);
        const unsigned code = (unsigned)(i * g.k + j);
        const int64_t o = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + cg * 8;
        const uint2 sl = *reinterpret_cast<const uint2*>(slot + o);
        float d[8];
        Vec8<bf16_t>::load(dy + o, d);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const unsigned sc = ((c < 4 ? sl.x : sl.y) >> (8 * (c & 3))) & 0xffu;
          acc[c] += sc == code ? d[c] : 0.f;
        }
      }
    }
    Vec8<bf16_t>::store(dx + pix * g.C + cg * 8, acc);
  }
}

}  // namespace

PDT_API int pdt_maxpool_ok(int C, int k, int s, int p) {
  return (C % 8 == 0 && k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k) ? 1 : 0;
}

// x [N, H, W, C] bf16 -> y [N, OH, OW, C] bf16 + slot [N, OH, OW, C] uint8
PDT_API int pdt_maxpool_fwd(const void* x, void* y, void* slot, int N, int C, int H, int W, int OH, int OW, int k,
                            int s, int p, hipStream_t st) {
  if (!pdt_maxpool_ok(C, k, s, p)) return (int)hipErrorInvalidValue;
  const PoolGeom g{N, C, H, W, OH, OW, k, s, p};
  const int64_t work = (int64_t)N * OH * OW * (C / 8);
  maxpool_fwd_kernel<<<grid_for(work, NT, 256 * 16), NT, 0, st>>>((const bf16_t*)x, (bf16_t*)y, (uint8_t*)slot, g);
  return (int)hipGetLastError();
}

// dy [N, OH, OW, C], slot (from the forward) -> dx [N, H, W, C]
PDT_API int pdt_maxpool_bwd(const void* dy, const void* slot, void* dx, int N, int C, int H, int W, int OH, int OW,
                            int k, int s, int p, hipStream_t st) {
  if (!pdt_maxpool_ok(C, k, s, p)) return (int)hipErrorInvalidValue;
  const PoolGeom g{N, C, H, W, OH, OW, k, s, p};
  const int64_t work = (int64_t)N * H * W * (C / 8);
  maxpool_bwd_kernel<<<grid_for(work, NT, 256 * 16), NT, 0, st>>>((const bf16_t*)dy, (const uint8_t*)slot, (bf16_t*)dx,
                                                                   g);
  return (int)hipGetLastError();
}
