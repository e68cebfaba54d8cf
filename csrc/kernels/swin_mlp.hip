// Fused transformer MLP for SwinIR-S's narrow channels (C = 60 -> hidden 120 -> 60, exact erf GELU):
//
//   forward   y  = GELU(x W1^T + b1) W2^T + b2                       one kernel, the hidden never leaves registers
//   backward  a  = x W1^T + b1 (recomputed), h = GELU(a)
//             dh = dy W2,  da = dh * GELU'(a),  dx = da W1           one kernel, per-token work in registers
//             dW1 = da^T [x | 1],  dW2 = dy^T [h | 1]                 (bias gradients ride in the pad column)
//
// The stock path is two skinny hipBLASLt GEMMs per direction (K = 60 / 120: a few percent of MFMA peak) plus
// a bias-GELU pass, moving the [tokens, 120] hidden through HBM 4x forward and 6x backward; here the per-token
// traffic is x and y forward, x, dy and dx backward.
//
// Layout (v_mfma_f32_16x16x32_bf16, lane l: r = l & 15, g = l >> 4): every GEMM is computed TRANSPOSED --
// rows = features, columns = 16 tokens -- so a wave's accumulator (lane: token r, 4 consecutive features
// 4g..4g+3 of a 16-row block) is directly the B operand of the next GEMM once the K order is permuted:
// B k-slot j of k-step s <-> feature pi(s, g, j) = 32 s + (j < 4 ? 4 g + j : 16 + 4 g + j - 4), and the
// weight fragments (A operand, held in VGPRs for the whole kernel) are loaded in that same order.
// Features are zero-padded to C_PAD = 64 / H_PAD = 128 in registers (pad weight rows / columns are zero).
// Weight gradients reduce over tokens: each workgroup stages 64 tokens of da^T, [h|1]^T, [x|1]^T and dy^T in
// LDS (feature-major, so an operand fragment is one ds_read_b128), four waves split the 64 output tiles of
// dW1 / dW2, accumulate over all the workgroup's tokens in registers and write one fp32 partial per
// workgroup; a column-sum kernel adds the partials (deterministic, no atomics).
#include "common.h"
#include <stdlib.h>

namespace pdt {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int CPAD = 64, HPAD = 128;
constexpr int LDT = 72;   // LDS row stride (bf16) of the token-minor staging tiles: 144 B rows, b128-aligned

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}
__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

__device__ __forceinline__ u16x8 pack2(uint2 a, uint2 b) {
  const u32x4 v = {a.x, a.y, b.x, b.y};
  return __builtin_bit_cast(u16x8, v);
}
__device__ __forceinline__ u16x8 pack_f(const f32x4& a, const f32x4& b) {
  u16x8 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[i] = f2bf(a[i]); v[4 + i] = f2bf(b[i]); }
  return v;
}

// 4 bf16 at (row, c..c+3) of a row-major [nrows, ld] matrix (c % 4 == 0, ld % 4 == 0); zero outside
__device__ __forceinline__ uint2 ld4(const bf16_t* __restrict__ p, int64_t row, int64_t nrows, int c, int ncols, int ld) {
  if (row < nrows && c < ncols) return *reinterpret_cast<const uint2*>(p + row * ld + c);
  return make_uint2(0u, 0u);
}

// exact-erf GELU and its derivative from one exp: erf by Abramowitz-Stegun 7.1.26 (|err| < 1.5e-7), whose
// exp(-x^2) with x = a / sqrt(2) is also the Gaussian density term of GELU'
__device__ __forceinline__ void gelu_grad(float a, float& g, float& dg) {
  const float x = a * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * fabsf(x));
  const float e = __expf(-x * x);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erf_ = copysignf(1.f - p * e, x);
  const float cdf = 0.5f * (1.f + erf_);
  g = a * cdf;
  dg = cdf + a * e * 0.39894228040143268f;
}
__device__ __forceinline__ float gelu_only(float a) {
  const float x = a * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * fabsf(x));
  const float e = __expf(-x * x);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return 0.5f * a * (1.f + copysignf(1.f - p * e, x));
}

// A fragments of W [rows, cols] (row-major, ld = cols) for a GEMM whose A rows are W's rows and whose K runs
// along W's columns in natural order: frag[rb][ks] = W[16 rb + r][32 ks + 8 g + j]
template <int RB, int KS>
__device__ __forceinline__ void frag_rows(u16x8 (&f)[RB][KS], const bf16_t* __restrict__ W, int rows, int cols, int r,
                                          int g) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int c0 = 32 * ks + 8 * g;
      f[rb][ks] = pack2(ld4(W, 16 * rb + r, rows, c0, cols, cols), ld4(W, 16 * rb + r, rows, c0 + 4, cols, cols));
    }
}
// ... K along W's columns in the permuted accumulator order pi(s, g, j)
template <int RB, int KS>
__device__ __forceinline__ void frag_rows_pi(u16x8 (&f)[RB][KS], const bf16_t* __restrict__ W, int rows, int cols,
                                             int r, int g) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      f[rb][s] = pack2(ld4(W, 16 * rb + r, rows, 32 * s + 4 * g, cols, cols),
                       ld4(W, 16 * rb + r, rows, 32 * s + 16 + 4 * g, cols, cols));
}
// A fragments of W^T (A rows = W's columns), K along W's rows: natural order (pi = false) or permuted
template <int RB, int KS, bool PI>
__device__ __forceinline__ void frag_cols(u16x8 (&f)[RB][KS], const bf16_t* __restrict__ W, int rows, int cols, int r,
                                          int g) {
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 v;
      const int col = 16 * rb + r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = PI ? 32 * s + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4) : 32 * s + 8 * g + j;
        v[j] = (k < rows && col < cols) ? W[(int64_t)k * cols + col] : (bf16_t)0;
      }
      f[rb][s] = v;
    }
}

// ------------------------------------------------------------------------------------------------ forward
__global__ __launch_bounds__(256) void swin_mlp_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w1,
                                                           const bf16_t* __restrict__ b1, const bf16_t* __restrict__ w2,
                                                           const bf16_t* __restrict__ b2,
                                                           const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
                                                           int64_t T, int C, int H) {
  __shared__ float b1s[HPAD], b2s[CPAD];
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < HPAD; i += 256) b1s[i] = i < H ? bf2f(b1[i]) : 0.f;
  for (int i = threadIdx.x; i < CPAD; i += 256) b2s[i] = i < C ? bf2f(b2[i]) : 0.f;
  u16x8 A1[8][2], A2[4][4];
  frag_rows<8, 2>(A1, w1, H, C, r, g);        // a^T = W1 x^T     (rows hidden, K = channels)
  frag_rows_pi<4, 4>(A2, w2, C, H, r, g);     // y^T = W2 h^T     (rows channels, K = hidden in pi order)
  __syncthreads();
  const int64_t ntiles = (T + 15) / 16;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint2 xn[4];
  auto load_x = [&](int64_t tl) {
    const int64_t t = tl * 16 + r;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      xn[2 * ks] = ld4(x, t, T, 32 * ks + 8 * g, C, C);
      xn[2 * ks + 1] = ld4(x, t, T, 32 * ks + 8 * g + 4, C, C);
    }
  };
  if (tile < ntiles) load_x(tile);
  for (; tile < ntiles; tile += stride) {
    const u16x8 B0 = pack2(xn[0], xn[1]), B1 = pack2(xn[2], xn[3]);
    if (tile + stride < ntiles) load_x(tile + stride);     // next tile's x in flight during this one
    f32x4 acc1[8];
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) acc1[hb] = mfma16(A1[hb][1], B1, mfma16(A1[hb][0], B0, zero4()));
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(b1s + 16 * hb + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc1[hb][i] = gelu_only(acc1[hb][i] + bb[i]);
    }
    f32x4 acc2[4];
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) acc2[ob] = zero4();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u16x8 Bh = pack_f(acc1[2 * s], acc1[2 * s + 1]);
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) acc2[ob] = mfma16(A2[ob][s], Bh, acc2[ob]);
    }
    const int64_t t = tile * 16 + r;
    if (t < T) {
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) {
        const int o = 16 * ob + 4 * g;
        if (o < C) {
          f32x4 bb = *reinterpret_cast<const f32x4*>(b2s + o);
          if (res) {                                      // fused residual add: y = res + MLP(x)
            const uint2 rv = *reinterpret_cast<const uint2*>(res + t * C + o);
            bb[0] += bf2f((bf16_t)(rv.x & 0xffff)); bb[1] += bf2f((bf16_t)(rv.x >> 16));
            bb[2] += bf2f((bf16_t)(rv.y & 0xffff)); bb[3] += bf2f((bf16_t)(rv.y >> 16));
          }
          const uint32_t lo = (uint32_t)f2bf(acc2[ob][0] + bb[0]) | ((uint32_t)f2bf(acc2[ob][1] + bb[1]) << 16);
          const uint32_t hi = (uint32_t)f2bf(acc2[ob][2] + bb[2]) | ((uint32_t)f2bf(acc2[ob][3] + bb[3]) << 16);
          *reinterpret_cast<uint2*>(y + t * C + o) = make_uint2(lo, hi);
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------- backward
struct BwdLds {
  bf16_t daT[HPAD][LDT];   // da^T        (hidden x 64 tokens)
  bf16_t hT[HPAD][LDT];    // [h | 1]^T   (ones row at hidden == H -> db2)
  bf16_t xT[CPAD][LDT];    // [x | 1]^T   (ones row at channel == C -> db1)
  bf16_t dyT[CPAD][LDT];   // dy^T
  float b1s[HPAD];
};

__global__ __launch_bounds__(256) void swin_mlp_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ w1, const bf16_t* __restrict__ b1,
                                                           const bf16_t* __restrict__ w2, bf16_t* __restrict__ dx,
                                                           float* __restrict__ ws, int64_t T, int C, int H) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BwdLds& L = *reinterpret_cast<BwdLds*>(smem);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < HPAD; i += 256) L.b1s[i] = i < H ? bf2f(b1[i]) : 0.f;
  u16x8 A1[8][2], Adh[8][2], Adx[4][4];
  frag_rows<8, 2>(A1, w1, H, C, r, g);              // a^T  = W1 x^T    rows hidden, K = channels
  frag_cols<8, 2, false>(Adh, w2, C, H, r, g);      // dh^T = W2^T dy^T rows hidden, K = channels (W2 rows)
  frag_cols<4, 4, true>(Adx, w1, H, C, r, g);       // dx^T = W1^T da^T rows channels, K = hidden (pi order)
  f32x4 gw1[2][4], gw2[4][2];                       // this wave's dW1 rows hb in {2w, 2w+1}; dW2 cols likewise
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) { gw1[a][b] = zero4(); gw2[b][a] = zero4(); }
  __syncthreads();
  const int64_t nchunks = (T + 63) / 64;
  const int tl = 16 * w + r;                        // this lane's token within the 64-token chunk
  uint2 xn[4], dyn[4];                              // next chunk's x / dy rows, loaded one chunk ahead
  auto load_rows = [&](int64_t chunk) {
    const int64_t tt = chunk * 64 + tl;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c0 = 32 * (q >> 1) + 8 * g + 4 * (q & 1);
      xn[q] = ld4(x, tt, T, c0, C, C);
      dyn[q] = ld4(dy, tt, T, c0, C, C);
    }
  };
  if ((int64_t)blockIdx.x < nchunks) load_rows(blockIdx.x);
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int64_t t = ch * 64 + tl;
    const u16x8 Bx[2] = {pack2(xn[0], xn[1]), pack2(xn[2], xn[3])};
    const u16x8 Bdy[2] = {pack2(dyn[0], dyn[1]), pack2(dyn[2], dyn[3])};
    if (ch + gridDim.x < nchunks) load_rows(ch + gridDim.x);
    // stage [x | 1]^T and dy^T (feature-major) for the weight gradients
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 32 * ks + 8 * g + j;
        L.xT[c][tl] = (c == C && t < T) ? (bf16_t)0x3F80 : Bx[ks][j];
        L.dyT[c][tl] = Bdy[ks][j];
      }
    f32x4 acc_a[8], acc_dh[8];
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      acc_a[hb] = mfma16(A1[hb][1], Bx[1], mfma16(A1[hb][0], Bx[0], zero4()));
      acc_dh[hb] = mfma16(Adh[hb][1], Bdy[1], mfma16(Adh[hb][0], Bdy[0], zero4()));
    }
    // elementwise: h = GELU(a), da = dh * GELU'(a); stage da^T and [h | 1]^T
#pragma unroll
    for (int hb = 0; hb < 8; ++hb) {
      const f32x4 bb = *reinterpret_cast<const f32x4*>(L.b1s + 16 * hb + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hid = 16 * hb + 4 * g + i;
        float gv, dg;
        gelu_grad(acc_a[hb][i] + bb[i], gv, dg);
        const float da = acc_dh[hb][i] * dg;
        acc_dh[hb][i] = da;
        L.daT[hid][tl] = f2bf(da);
        L.hT[hid][tl] = t >= T ? (bf16_t)0 : hid == H ? (bf16_t)0x3F80 : f2bf(gv);
      }
    }
    // dx^T = W1^T da^T
    f32x4 acc_dx[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc_dx[cb] = zero4();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u16x8 Bda = pack_f(acc_dh[2 * s], acc_dh[2 * s + 1]);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc_dx[cb] = mfma16(Adx[cb][s], Bda, acc_dx[cb]);
    }
    if (t < T) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int c = 16 * cb + 4 * g;
        if (c < C) {
          const uint32_t lo = (uint32_t)f2bf(acc_dx[cb][0]) | ((uint32_t)f2bf(acc_dx[cb][1]) << 16);
          const uint32_t hi = (uint32_t)f2bf(acc_dx[cb][2]) | ((uint32_t)f2bf(acc_dx[cb][3]) << 16);
          *reinterpret_cast<uint2*>(dx + t * C + c) = make_uint2(lo, hi);
        }
      }
    }
    __syncthreads();
    // weight gradients over the chunk's 64 tokens (K = 2 x 32): dW1 = da^T [x|1], dW2 = dy^T [h|1]
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int k0 = 32 * ks + 8 * g;
      u16x8 Ada[2], Bh[2], Bxx[4], Ady[4];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        Ada[a] = *reinterpret_cast<const u16x8*>(&L.daT[16 * (2 * w + a) + r][k0]);
        Bh[a] = *reinterpret_cast<const u16x8*>(&L.hT[16 * (2 * w + a) + r][k0]);
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        Bxx[b] = *reinterpret_cast<const u16x8*>(&L.xT[16 * b + r][k0]);
        Ady[b] = *reinterpret_cast<const u16x8*>(&L.dyT[16 * b + r][k0]);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          gw1[a][b] = mfma16(Ada[a], Bxx[b], gw1[a][b]);
          gw2[b][a] = mfma16(Ady[b], Bh[a], gw2[b][a]);
        }
    }
    __syncthreads();
  }
  // this workgroup's partial: ws[block][HPAD * CPAD (dW1 | db1 in col C)] then [CPAD * HPAD (dW2 | db2 in col H)]
  float* p1 = ws + (int64_t)blockIdx.x * (2 * HPAD * CPAD);
  float* p2 = p1 + HPAD * CPAD;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p1[(16 * (2 * w + a) + 4 * g + i) * CPAD + 16 * b + r] = gw1[a][b][i];   // dW1[hidden][channel]
        p2[(16 * b + 4 * g + i) * HPAD + 16 * (2 * w + a) + r] = gw2[b][a][i];   // dW2[channel][hidden]
      }
}

// stage 1 of the partial reduction: ws2[slice][e] = sum of partials 8 * slice .. 8 * slice + 7 (float4 per thread,
// 16 x ceil(nb / 8) workgroups: a single-stage column sum over 256 partials ran one wave per CU, latency-bound)
constexpr int RED_SLICE = 8;
__global__ __launch_bounds__(256) void swin_mlp_partial_sum(const float* __restrict__ ws, int nb, float* __restrict__ ws2) {
  const int e = (blockIdx.x * 256 + threadIdx.x) * 4;
  const int b0 = blockIdx.y * RED_SLICE;
  f32x4 acc = zero4();
#pragma unroll
  for (int b = 0; b < RED_SLICE; ++b)
    if (b0 + b < nb) acc += *reinterpret_cast<const f32x4*>(ws + (int64_t)(b0 + b) * (2 * HPAD * CPAD) + e);
  *reinterpret_cast<f32x4*>(ws2 + (int64_t)blockIdx.y * (2 * HPAD * CPAD) + e) = acc;
}

// sum the (stage-1) partials into dW1 [H, C], db1 [H], dW2 [C, H], db2 [C] (T_OUT = bf16 or fp32)
template <typename TO>
__global__ __launch_bounds__(256) void swin_mlp_wgrad_reduce(const float* __restrict__ ws, int nb, int C, int H,
                                                             TO* __restrict__ dw1, TO* __restrict__ db1,
                                                             TO* __restrict__ dw2, TO* __restrict__ db2) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * HPAD * CPAD) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += ws[(int64_t)b * (2 * HPAD * CPAD) + e];
  if (e < HPAD * CPAD) {
    const int h = e / CPAD, c = e % CPAD;
    if (h < H && c < C) dw1[h * C + c] = from_f<TO>(s);
    else if (h < H && c == C) db1[h] = from_f<TO>(s);
  } else {
    const int e2 = e - HPAD * CPAD, o = e2 / HPAD, h = e2 % HPAD;
    if (o < C && h < H) dw2[o * H + h] = from_f<TO>(s);
    else if (o < C && h == H) db2[o] = from_f<TO>(s);
  }
}

}  // namespace
}  // namespace pdt

using namespace pdt;

static bool swin_mlp_shape_ok(int C, int H, const void* a, const void* b) {
  return C > 0 && H > 0 && C < CPAD && H < HPAD && C % 4 == 0 && H % 4 == 0 &&
         ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 7) == 0;
}

PDT_API int pdt_swin_mlp_ok(int C, int H) { return swin_mlp_shape_ok(C, H, nullptr, nullptr) ? 1 : 0; }

// fp32 floats of backward workspace for `nb` workgroups
PDT_API int64_t pdt_swin_mlp_ws_floats(int nb) {
  return ((int64_t)nb + (nb + RED_SLICE - 1) / RED_SLICE) * 2 * HPAD * CPAD;
}
PDT_API int pdt_swin_mlp_bwd_blocks(int64_t T) {
  // one workgroup per CU by default (fp32 partials stay 16 MB); PDT_SWIN_MLP_BWD_WG overrides
  static const int cap = [] { const char* e = getenv("PDT_SWIN_MLP_BWD_WG"); return e ? atoi(e) : 256; }();
  const int64_t ch = (T + 63) / 64;
  return (int)(ch < cap ? ch : cap);
}

// y = MLP(x) (+ res when non-null, same [T, C] layout as y)
PDT_API int pdt_swin_mlp_fwd(const void* x, const void* w1, const void* b1, const void* w2, const void* b2,
                             const void* res, void* y, int64_t T, int C, int H, hipStream_t st) {
  if (T <= 0 || !swin_mlp_shape_ok(C, H, x, y) || !swin_mlp_shape_ok(C, H, res, res)) return (int)hipErrorInvalidValue;
  const int64_t tiles = (T + 15) / 16;
  int64_t grid = (tiles + 3) / 4;
  // workgroups (4 waves each; every wave loads the weights into VGPRs once): PDT_SWIN_MLP_FWD_WG overrides
  static const int cap = [] { const char* e = getenv("PDT_SWIN_MLP_FWD_WG"); return e ? atoi(e) : 1024; }();
  if (grid > cap) grid = cap;
  swin_mlp_fwd_kernel<<<(int)grid, 256, 0, st>>>((const bf16_t*)x, (const bf16_t*)w1, (const bf16_t*)b1,
                                                 (const bf16_t*)w2, (const bf16_t*)b2, (const bf16_t*)res, (bf16_t*)y,
                                                 T, C, H);
  return (int)hipGetLastError();
}

// dx [T, C] bf16; weight / bias gradients written (not accumulated) in out_dt (kBF16 / kF32)
PDT_API int pdt_swin_mlp_bwd(const void* x, const void* dy, const void* w1, const void* b1, const void* w2, void* dx,
                             void* dw1, void* db1, void* dw2, void* db2, int out_dt, float* ws, int nb, int64_t T,
                             int C, int H, hipStream_t st) {
  if (T <= 0 || nb <= 0 || !swin_mlp_shape_ok(C, H, x, dy) || !swin_mlp_shape_ok(C, H, dx, dx))
    return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)swin_mlp_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(BwdLds)) != hipSuccess)
      return (int)hipErrorInvalidValue;
    attr = true;
  }
  swin_mlp_bwd_kernel<<<nb, 256, sizeof(BwdLds), st>>>((const bf16_t*)x, (const bf16_t*)dy, (const bf16_t*)w1,
                                                       (const bf16_t*)b1, (const bf16_t*)w2, (bf16_t*)dx, ws, T, C, H);
  const int slices = (nb + RED_SLICE - 1) / RED_SLICE;
  float* ws2 = ws + (int64_t)nb * 2 * HPAD * CPAD;
  swin_mlp_partial_sum<<<dim3(2 * HPAD * CPAD / 1024, slices), 256, 0, st>>>(ws, nb, ws2);
  const int rgrid = (2 * HPAD * CPAD + 255) / 256;
  if (out_dt == kBF16)
    swin_mlp_wgrad_reduce<bf16_t><<<rgrid, 256, 0, st>>>(ws2, slices, C, H, (bf16_t*)dw1, (bf16_t*)db1, (bf16_t*)dw2,
                                                         (bf16_t*)db2);
  else
    swin_mlp_wgrad_reduce<float><<<rgrid, 256, 0, st>>>(ws2, slices, C, H, (float*)dw1, (float*)db1, (float*)dw2,
                                                        (float*)db2);
  return (int)hipGetLastError();
}
