// Memory-bound elementwise kernels for gfx950: bias+GELU (tanh / erf) fwd+bwd, SwiGLU fwd+bwd,
// rotary embedding (RoPE) fwd/bwd, fp8 (OCP e4m3fn) quantise/dequantise with per-tensor amax,
// and an fp32->bf16 cast.  All use 16-byte vector accesses (8 x bf16 per lane).
//
// Parity targets: GPT-2 MLP (bias + gelu_new), SwinIR MLP (nn.GELU = erf form),
// Llama-3 MLP (SwiGLU) and attention (RoPE, rotate-half convention), BASELINE.json north star
// "bf16/fp8 loss-scaled cast".
#include "common.h"
#include "reduce.h"
#include "gelu.h"
#include <hip/hip_fp8.h>

using namespace pdt;

namespace {

constexpr int NT = 256;
// y = gelu(h + bias); N % 8 == 0 (vector path).  bias may be null.
// The bias column advances incrementally (one compare-subtract per pass): a 64-bit `e % N` per vector is a
// ~40-instruction software division.  (4 vectors per thread per pass with every load issued first measured 4 %
// SLOWER at the GPT-2 1.3B c_fc shape; the kernel is not load-latency-bound.  A software-pipelined form -- next
// pass's loads issued before this pass's math, bias presence a template parameter -- measured equal, 676 vs 672 us;
// a plain device copy of the same bytes takes 628 us: at this 3.2 GB shape the kernel is within 7 % of copy
// bandwidth, profiles/r3_s4h_bias_gelu_fwd_vs_copy.jsonl.)
template <typename T, typename B, bool TANH>
__global__ __launch_bounds__(NT) void bias_gelu_fwd_kernel(const T* __restrict__ h, const B* __restrict__ bias,
                                                           T* __restrict__ y, int64_t n8, int N) {
  const int64_t i0 = blockIdx.x * (int64_t)NT + threadIdx.x, stride = (int64_t)gridDim.x * NT;
  int col = (int)((i0 * 8) % N);
  const int inc = (int)((stride * 8) % N);
  for (int64_t i = i0; i < n8; i += stride) {
    const int64_t e = i * 8;
    float v[8], b[8];
    Vec8<T>::load(h + e, v);
    if (bias) Vec8<B>::load(bias + col, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = gelu_f<TANH>(bias ? v[k] + b[k] : v[k]);
    Vec8<T>::store(y + e, v);
    col += inc;
    if (col >= N) col -= N;
  }
}

template <typename T, typename B, bool TANH>
__global__ __launch_bounds__(NT) void bias_gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                           const B* __restrict__ bias, T* __restrict__ dh,
                                                           int64_t n8, int N) {
  const int64_t i0 = blockIdx.x * (int64_t)NT + threadIdx.x, stride = (int64_t)gridDim.x * NT;
  int col = (int)((i0 * 8) % N);
  const int inc = (int)((stride * 8) % N);
  for (int64_t i = i0; i < n8; i += stride, col = col + inc >= N ? col + inc - N : col + inc) {
    const int64_t e = i * 8;
    float v[8], g[8], b[8];
    Vec8<T>::load(h + e, v);
    Vec8<T>::load(dy + e, g);
    if (bias) Vec8<B>::load(bias + col, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] *= gelu_grad<TANH>(bias ? v[k] + b[k] : v[k]);
    Vec8<T>::store(dh + e, g);
  }
}

// ACT 0: erf GELU, 1: tanh GELU of (h + bias); 2: h already holds the GELU derivative (gemm.hip E_GELU's kept
// output): the backward is a multiply, no transcendental, no bias
template <int ACT>
__device__ __forceinline__ float act_grad(float v, float b) {
  if constexpr (ACT == 2) return v;
  else return gelu_grad<ACT == 1>(v + b);
}

// GELU backward fused with the bias gradient: workgroups sweep (2048-column group) x (row chunk) as in
// reduce.h; each thread keeps its 8 columns' dbias partial sums in registers while it writes dh, so the
// bias gradient costs no second pass over the [rows, N] activation gradient.
template <typename T, typename B, int ACT>
__global__ __launch_bounds__(NT) void bias_gelu_bwd_db_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                              const B* __restrict__ bias, T* __restrict__ dh,
                                                              int rows, int N, int rows_per,
                                                              float* __restrict__ part) {
  const int col = (blockIdx.x * NT + threadIdx.x) * 8;
  if (col >= N) return;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
  float b[8], acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { acc[k] = 0.f; b[k] = 0.f; }
  if (ACT != 2) Vec8<B>::load(bias + col, b);
  int r = r0;
  for (; r + 4 <= r1; r += 4) {   // 8 loads in flight per thread (2 rows held it at ~5.2 TB/s)
    float v[4][8], g[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      Vec8<T>::load(h + (int64_t)(r + u) * N + col, v[u]);
      Vec8<T>::load(dy + (int64_t)(r + u) * N + col, g[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[u][k] *= act_grad<ACT>(v[u][k], b[k]);
        acc[k] += g[u][k];
      }
      Vec8<T>::store(dh + (int64_t)(r + u) * N + col, g[u]);
    }
  }
  for (; r < r1; ++r) {
    float v[8], g[8];
    Vec8<T>::load(h + (int64_t)r * N + col, v);
    Vec8<T>::load(dy + (int64_t)r * N + col, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g[k] *= act_grad<ACT>(v[k], b[k]);
      acc[k] += g[k];
    }
    Vec8<T>::store(dh + (int64_t)r * N + col, g);
  }
  Vec8<float>::store(part + (int64_t)blockIdx.y * N + col, acc);
}

// Narrow rows (N < 2048, e.g. the SwinIR-S MLP's 120): the column-group mapping above would leave all but
// N/8 threads of a workgroup idle; here the workgroup covers NT / (N/8) rows per pass (coalesced: adjacent
// rows are adjacent in memory) and folds its row groups through LDS into ONE partial row.
template <typename T, typename B, int ACT>
__global__ __launch_bounds__(NT) void bias_gelu_bwd_db_narrow(const T* __restrict__ dy, const T* __restrict__ h,
                                                              const B* __restrict__ bias, T* __restrict__ dh,
                                                              int rows, int N, int rows_per,
                                                              float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sacc[NT * 8];
  const int tpr = N >> 3, rpb = NT / tpr;
  const int rg = threadIdx.x / tpr, col = (threadIdx.x - rg * tpr) * 8;
  const bool act = rg < rpb;
  float b[8], acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { acc[k] = 0.f; b[k] = 0.f; }
  if (act && ACT != 2) Vec8<B>::load(bias + col, b);
  const int r0 = blockIdx.x * rows_per, r1 = min(rows, r0 + rows_per);
  if (act) {
    for (int r = r0 + rg; r < r1; r += rpb) {
      float v[8], g[8];
      Vec8<T>::load(h + (int64_t)r * N + col, v);
      Vec8<T>::load(dy + (int64_t)r * N + col, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[k] *= act_grad<ACT>(v[k], b[k]);
        acc[k] += g[k];
      }
      Vec8<T>::store(dh + (int64_t)r * N + col, g);
    }
  }
  Vec8<float>::store(sacc + threadIdx.x * 8, acc);
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += NT) {
    const int c8 = c >> 3, k = c & 7;
    float t = 0.f;
    for (int g = 0; g < rpb; ++g) t += sacc[(g * tpr + c8) * 8 + k];
    part[(int64_t)blockIdx.x * N + c] = t;
  }
}

// SwiGLU on a fused [rows, 2F] projection: y[r, j] = silu(x[r, j]) * x[r, F + j]
template <typename T>
__global__ __launch_bounds__(NT) void swiglu_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t rows,
                                                        int F) {
  // (row, column) advanced incrementally (one 64-bit division per thread, not per vector)
  const int f8 = F / 8;
  const int64_t n8 = rows * f8, i0 = blockIdx.x * (int64_t)NT + threadIdx.x, stride = (int64_t)gridDim.x * NT;
  const int64_t dr = stride / f8;
  const int dj = (int)(stride - dr * f8);
  int64_t r = i0 / f8;
  int j8 = (int)(i0 - r * f8);
  for (int64_t i = i0; i < n8; i += stride) {
    const int j = 8 * j8;
    float a[8], b[8], o[8];
    Vec8<T>::load(x + r * 2 * F + j, a);
    Vec8<T>::load(x + r * 2 * F + F + j, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = a[k] / (1.f + __expf(-a[k])) * b[k];
    Vec8<T>::store(y + r * F + j, o);
    r += dr;
    j8 += dj;
    if (j8 >= f8) { j8 -= f8; ++r; }
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void swiglu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                        T* __restrict__ dx, int64_t rows, int F) {
  const int f8 = F / 8;
  const int64_t n8 = rows * f8, i0 = blockIdx.x * (int64_t)NT + threadIdx.x, stride = (int64_t)gridDim.x * NT;
  const int64_t dr = stride / f8;
  const int dj = (int)(stride - dr * f8);
  int64_t r = i0 / f8;
  int j8 = (int)(i0 - r * f8);
  for (int64_t i = i0; i < n8; i += stride) {
    const int j = 8 * j8;
    float a[8], b[8], g[8], da[8], db[8];
    Vec8<T>::load(x + r * 2 * F + j, a);
    Vec8<T>::load(x + r * 2 * F + F + j, b);
    Vec8<T>::load(dy + r * F + j, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = 1.f / (1.f + __expf(-a[k]));
      const float silu = a[k] * s;
      db[k] = g[k] * silu;
      da[k] = g[k] * b[k] * (s * (1.f + a[k] * (1.f - s)));
    }
    Vec8<T>::store(dx + r * 2 * F + j, da);
    Vec8<T>::store(dx + r * 2 * F + F + j, db);
    r += dr;
    j8 += dj;
    if (j8 >= f8) { j8 -= f8; ++r; }
  }
}

// RoPE (rotate-half): rows = B*S*H head vectors, row r at position s = (r / H) % S + pos0.
// out[i] = x[i] c - x[i+D/2] s_ ; out[i+D/2] = x[i+D/2] c + x[i] s_   (sign = -1 for backward).
// cos/sin tables: [S_max, D/2] fp32.
// A "row" is one head vector: row r = (position r / H, head r % H) lives at
// (r / H) * pos_stride + (r % H) * head_stride, so the q and k heads of a packed [B, S, H + 2 Hkv, D] qkv
// projection are rotated IN PLACE (y == x, H = Hq + Hkv) and a plain [B, S, H, D] tensor is the
// pos_stride == H * head_stride case.  Each thread reads both halves before writing them: in-place safe.
template <typename T>
__global__ __launch_bounds__(NT) void rope_kernel(const T* x, T* y, int64_t rows,   // x may alias y
                                                  int64_t head_in, int64_t pos_in, int64_t head_out,
                                                  int64_t pos_out, int H, int S, int D, int pos0,
                                                  const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                  float sign) {
  const int half = D / 2, h8 = half / 8;
  const int64_t n = rows * h8;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / h8;
    const int j = (int)(i % h8) * 8;
    const int64_t pr = r / H, hr = r % H;
    const int s = (int)(pr % S) + pos0;
    const int64_t xi = pr * pos_in + hr * head_in, yi = pr * pos_out + hr * head_out;
    float a[8], b[8], c[8], sn[8], o1[8], o2[8];
    Vec8<T>::load(x + xi + j, a);
    Vec8<T>::load(x + xi + half + j, b);
    Vec8<float>::load(cosb + (int64_t)s * half + j, c);
    Vec8<float>::load(sinb + (int64_t)s * half + j, sn);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float ss = sign * sn[k];
      o1[k] = a[k] * c[k] - b[k] * ss;
      o2[k] = b[k] * c[k] + a[k] * ss;
    }
    Vec8<T>::store(y + yi + j, o1);
    Vec8<T>::store(y + yi + half + j, o2);
  }
}

// fp8 e4m3fn (OCP, gfx950) quantisation with a per-tensor scale read from device memory;
// the same pass records amax(|x|) (for delayed scaling) with an integer atomicMax on the float bits.
template <typename T>
__global__ __launch_bounds__(NT) void fp8_quant_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                       int64_t n, const float* __restrict__ scale,
                                                       unsigned int* __restrict__ amax_bits) {
  const float sc = scale ? *scale : 1.f;
  float amax = 0.f;
  for (int64_t i = (blockIdx.x * (int64_t)NT + threadIdx.x) * 8; i < n; i += (int64_t)gridDim.x * NT * 8) {
    if (i + 8 <= n) {
      float v[8];
      Vec8<T>::load(x + i, v);
      uint64_t packed = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        amax = fmaxf(amax, fabsf(v[k]));
        const __hip_fp8_storage_t b = __hip_cvt_float_to_fp8(v[k] * sc, __HIP_SATFINITE, __HIP_E4M3);
        packed |= (uint64_t)b << (8 * k);
      }
      *reinterpret_cast<uint64_t*>(q + i) = packed;
    } else {
      for (int64_t j = i; j < n; ++j) {
        const float v = to_f<T>(x[j]);
        amax = fmaxf(amax, fabsf(v));
        q[j] = __hip_cvt_float_to_fp8(v * sc, __HIP_SATFINITE, __HIP_E4M3);
      }
    }
  }
  if (amax_bits) {
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) atomicMax(amax_bits, __float_as_uint(amax));
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void fp8_dequant_kernel(const uint8_t* __restrict__ q, T* __restrict__ y, int64_t n,
                                                         const float* __restrict__ scale_inv) {
  const float si = scale_inv ? *scale_inv : 1.f;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    __hip_fp8_e4m3 v;
    v.__x = q[i];
    y[i] = from_f<T>((float)v * si);
  }
}

__global__ __launch_bounds__(NT) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                           int64_t n) {
  for (int64_t i = (blockIdx.x * (int64_t)NT + threadIdx.x) * 8; i < n; i += (int64_t)gridDim.x * NT * 8) {
    if (i + 8 <= n) {
      float v[8];
      Vec8<float>::load(x + i, v);
      Vec8<bf16_t>::store(y + i, v);
    } else {
      for (int64_t j = i; j < n; ++j) y[j] = f2bf(x[j]);
    }
  }
}

// y[C, R] = x[R, C]^T for 16-bit elements, R % 64 == 0 and C % 64 == 0, 16-byte aligned rows.  Hands
// hipBLASLt the data-gradient GEMM dX = dY W in the forward's x W^T operand layout (15-25 % faster on the
// GPT-2 1.3B / Llama-3 shapes, profiles/r1_v11_gemm_dgrad_layout.jsonl); torch's w.t().contiguous() moves
// these weights at ~0.7 TB/s.  64 x 64 tile through LDS with 16-byte global loads and stores on both sides;
// the LDS row stride is 33 words so the 8 row groups of a column gather land in 8 distinct bank groups.
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          int R, int C) {
  constexpr int TS = 64, LD = 66;
  __shared__ uint32_t tile[TS * LD / 2];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * TS, r0 = blockIdx.y * TS;
  const int lc = (tid & 7) * 8, lr = tid >> 3;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int r = lr + 32 * p;
    const uint4 v = *reinterpret_cast<const uint4*>(x + (int64_t)(r0 + r) * C + c0 + lc);
    uint32_t* dst = tile + (r * LD + lc) / 2;
    dst[0] = v.x;
    dst[1] = v.y;
    dst[2] = v.z;
    dst[3] = v.w;
  }
  __syncthreads();
  const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = lr + 32 * p;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = t16[(lc + 2 * j) * LD + c], hi = t16[(lc + 2 * j + 1) * LD + c];
      w[j] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4*>(y + (int64_t)(c0 + c) * R + r0 + lc) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

}  // namespace

PDT_API int pdt_bias_gelu_fwd(const void* h, const void* bias, void* y, int64_t rows, int N, int dt, int bdt,
                              int tanh_approx, hipStream_t st) {
  if (N % 8) return (int)hipErrorInvalidValue;
  const int64_t n8 = rows * N / 8;
  const int grid = grid_for(n8, NT, 256 * 16);
#define PDT_L(T, B, TH) bias_gelu_fwd_kernel<T, B, TH><<<grid, NT, 0, st>>>((const T*)h, (const B*)bias, (T*)y, n8, N)
  if (dt == kBF16) {
    if (bdt == kF32) { if (tanh_approx) PDT_L(bf16_t, float, true); else PDT_L(bf16_t, float, false); }
    else { if (tanh_approx) PDT_L(bf16_t, bf16_t, true); else PDT_L(bf16_t, bf16_t, false); }
  } else {
    if (bdt == kF32) { if (tanh_approx) PDT_L(float, float, true); else PDT_L(float, float, false); }
    else { if (tanh_approx) PDT_L(float, bf16_t, true); else PDT_L(float, bf16_t, false); }
  }
#undef PDT_L
  return (int)hipGetLastError();
}

PDT_API int pdt_bias_gelu_bwd(const void* dy, const void* h, const void* bias, void* dh, int64_t rows, int N, int dt,
                              int bdt, int tanh_approx, hipStream_t st) {
  if (N % 8) return (int)hipErrorInvalidValue;
  const int64_t n8 = rows * N / 8;
  const int grid = grid_for(n8, NT, 256 * 16);
#define PDT_L(T, B, TH) \
  bias_gelu_bwd_kernel<T, B, TH><<<grid, NT, 0, st>>>((const T*)dy, (const T*)h, (const B*)bias, (T*)dh, n8, N)
  if (dt == kBF16) {
    if (bdt == kF32) { if (tanh_approx) PDT_L(bf16_t, float, true); else PDT_L(bf16_t, float, false); }
    else { if (tanh_approx) PDT_L(bf16_t, bf16_t, true); else PDT_L(bf16_t, bf16_t, false); }
  } else {
    if (bdt == kF32) { if (tanh_approx) PDT_L(float, float, true); else PDT_L(float, float, false); }
    else { if (tanh_approx) PDT_L(float, bf16_t, true); else PDT_L(float, bf16_t, false); }
  }
#undef PDT_L
  return (int)hipGetLastError();
}

// dh = dy * gelu'(h + bias) and dbias[N] (+= if accumulate) in one sweep; ws: pdt_colsum_ws_floats(rows, N).
// tanh_approx: 0 erf, 1 tanh, 2 "h is gelu'(pre-activation)" (dh = dy * h; bias unused, may be null)
PDT_API int pdt_bias_gelu_bwd_db(const void* dy, const void* h, const void* bias, void* dh, void* dbias, float* ws,
                                 int rows, int N, int dt, int bdt, int tanh_approx, int accumulate, hipStream_t st) {
  if (N % 8 != 0 || (bias == nullptr && tanh_approx != 2) || tanh_approx < 0 || tanh_approx > 2)
    return (int)hipErrorInvalidValue;
  const red::ColPlan pl = red::col_plan(rows, N);
  dim3 grid(pl.col_groups, pl.R);
  const bool narrow = N < 8 * NT;   // one column group: use the row-packed kernel (same partial layout)
#define PDT_L(T, B, A)                                                                                           \
  if (narrow) bias_gelu_bwd_db_narrow<T, B, A><<<pl.R, NT, 0, st>>>((const T*)dy, (const T*)h, (const B*)bias,   \
                                                                     (T*)dh, rows, N, pl.rows_per, ws);          \
  else bias_gelu_bwd_db_kernel<T, B, A><<<grid, NT, 0, st>>>((const T*)dy, (const T*)h, (const B*)bias, (T*)dh,  \
                                                             rows, N, pl.rows_per, ws)
#define PDT_ACT(T, B)                            \
  if (tanh_approx == 2) { PDT_L(T, B, 2); }      \
  else if (tanh_approx == 1) { PDT_L(T, B, 1); } \
  else { PDT_L(T, B, 0); }
  if (dt == kBF16 && bdt == kBF16) { PDT_ACT(bf16_t, bf16_t); }
  else if (dt == kBF16 && bdt == kF32) { PDT_ACT(bf16_t, float); }
  else if (dt == kF32 && bdt == kF32) { PDT_ACT(float, float); }
  else if (dt == kF32 && bdt == kBF16) { PDT_ACT(float, bf16_t); }
  else return (int)hipErrorInvalidValue;
#undef PDT_ACT
#undef PDT_L
  float* ws2 = ws + (int64_t)pl.R * N;
  if (bdt == kBF16) red::col_reduce<bf16_t>(ws, pl.R, N, (bf16_t*)dbias, ws2, accumulate, st);
  else red::col_reduce<float>(ws, pl.R, N, (float*)dbias, ws2, accumulate, st);
  return (int)hipGetLastError();
}

PDT_API int pdt_swiglu_fwd(const void* x, void* y, int64_t rows, int F, int dt, hipStream_t st) {
  if (F % 8) return (int)hipErrorInvalidValue;
  const int grid = grid_for(rows * F / 8, NT, 256 * 16);
  if (dt == kBF16) swiglu_fwd_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)x, (bf16_t*)y, rows, F);
  else swiglu_fwd_kernel<float><<<grid, NT, 0, st>>>((const float*)x, (float*)y, rows, F);
  return (int)hipGetLastError();
}

PDT_API int pdt_swiglu_bwd(const void* dy, const void* x, void* dx, int64_t rows, int F, int dt, hipStream_t st) {
  if (F % 8) return (int)hipErrorInvalidValue;
  const int grid = grid_for(rows * F / 8, NT, 256 * 16);
  if (dt == kBF16)
    swiglu_bwd_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)dy, (const bf16_t*)x, (bf16_t*)dx, rows, F);
  else
    swiglu_bwd_kernel<float><<<grid, NT, 0, st>>>((const float*)dy, (const float*)x, (float*)dx, rows, F);
  return (int)hipGetLastError();
}

PDT_API int pdt_rope(const void* x, void* y, int64_t rows, int64_t head_in, int64_t pos_in, int64_t head_out,
                     int64_t pos_out, int H, int S, int D, int pos0, const float* cosb, const float* sinb, int backward,
                     int dt, hipStream_t st) {
  if ((D / 2) % 8 || H <= 0) return (int)hipErrorInvalidValue;
  const int grid = grid_for(rows * (D / 16), NT, 256 * 16);
  const float sign = backward ? -1.f : 1.f;
  if (dt == kBF16)
    rope_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)x, (bf16_t*)y, rows, head_in, pos_in, head_out, pos_out,
                                             H, S, D, pos0, cosb, sinb, sign);
  else
    rope_kernel<float><<<grid, NT, 0, st>>>((const float*)x, (float*)y, rows, head_in, pos_in, head_out, pos_out,
                                            H, S, D, pos0, cosb, sinb, sign);
  return (int)hipGetLastError();
}

PDT_API int pdt_fp8_quant(const void* x, void* q, int64_t n, int dt, const float* scale, unsigned int* amax_bits,
                          hipStream_t st) {
  const int grid = grid_for(n / 8 + 1, NT, 256 * 8);
  if (dt == kBF16) fp8_quant_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)x, (uint8_t*)q, n, scale, amax_bits);
  else fp8_quant_kernel<float><<<grid, NT, 0, st>>>((const float*)x, (uint8_t*)q, n, scale, amax_bits);
  return (int)hipGetLastError();
}

PDT_API int pdt_fp8_dequant(const void* q, void* y, int64_t n, int dt, const float* scale_inv, hipStream_t st) {
  const int grid = grid_for(n, NT, 256 * 8);
  if (dt == kBF16) fp8_dequant_kernel<bf16_t><<<grid, NT, 0, st>>>((const uint8_t*)q, (bf16_t*)y, n, scale_inv);
  else fp8_dequant_kernel<float><<<grid, NT, 0, st>>>((const uint8_t*)q, (float*)y, n, scale_inv);
  return (int)hipGetLastError();
}

PDT_API int pdt_cast_f32_bf16(const float* x, void* y, int64_t n, hipStream_t st) {
  const int grid = grid_for(n / 8 + 1, NT, 256 * 8);
  cast_f32_bf16_kernel<<<grid, NT, 0, st>>>(x, (bf16_t*)y, n);
  return (int)hipGetLastError();
}

PDT_API int pdt_transpose16(const void* x, void* y, int R, int C, hipStream_t st) {
  if (R % 64 || C % 64 || R <= 0 || C <= 0 || (R / 64) > 65535) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) return (int)hipErrorInvalidValue;
  transpose16_kernel<<<dim3(C / 64, R / 64), 256, 0, st>>>((const uint16_t*)x, (uint16_t*)y, R, C);
  return (int)hipGetLastError();
}
