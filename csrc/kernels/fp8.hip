// fp8 training support for gfx950 (OCP e4m3fn / e5m2 -- MI355X's encodings, not MI300's fnuz):
//
//  * fp8_cast_transpose: one HBM pass over a bf16/fp32 activation, weight or gradient [R, C] that writes
//    the scaled fp8 copy in row layout [R, C] AND its transpose [C, R] (either optional) and max-reduces
//    |x| into the tensor's delayed-scaling amax slot.  The three GEMMs of an fp8 linear need each operand
//    in two layouts (forward x W^T, data-gradient dY W, weight-gradient dY^T X: hipBLASLt takes A
//    row-major and B column-major), so producing both from one read halves the cast traffic against a
//    cast followed by a transpose.  64 x 64 tiles staged through LDS; each block walks several tiles so
//    the amax atomic is issued once per block, not once per tile.
//  * fp8_update_scales: the delayed-scaling bookkeeping (TransformerEngine's "max" recipe) for a range of
//    a module's tensor slots in ONE launch: push the last iteration's amax into the history, clear it,
//    scale = fmax / max(history) / 2^margin, scale_inv = 1 / scale.  Keeps the whole recipe on the device
//    (no host sync per layer).
#include "common.h"
#include "reduce.h"

#include <hip/hip_fp8.h>
#include <stdlib.h>

namespace pdt {
namespace {

constexpr int CT_TS = 64;       // tile edge
constexpr int CT_LD = 68;       // LDS row stride in bytes (17 words: column gathers spread over banks)

// prologue applied to each element before the cast (GPT-2 MLP, tanh-form GELU via the sigmoid identity)
enum CtOp : int { kPlain = 0, kBiasGelu = 1, kBiasGeluBwd = 2 };
__device__ __forceinline__ float sig2z(float u) {
  const float z = 0.7978845608028654f * (u + 0.044715f * u * u * u);
  return __builtin_amdgcn_rcpf(1.f + __expf(-2.f * z));
}
__device__ __forceinline__ float gelu_tanh(float u) { return u * sig2z(u); }
__device__ __forceinline__ float gelu_tanh_grad(float u) {
  const float s = sig2z(u);
  return s + 2.f * u * s * (1.f - s) * 0.7978845608028654f * (1.f + 3.f * 0.044715f * u * u);
}

template <int FMT>
__device__ __forceinline__ uint8_t to_fp8(float v) {
  return __hip_cvt_float_to_fp8(v, __HIP_SATFINITE, FMT == 0 ? __HIP_E4M3 : __HIP_E5M2);
}

// x [R, C] (T = bf16 or fp32), R % 64 == 0, C % 64 == 0.  q [R, C] and qt [C, R] may each be null;
// with both null the kernel only measures amax (first-iteration "current scaling").
// OP == kBiasGelu:    v = gelu(x + bias)            (GPT-2 MLP forward: the hidden goes straight to fp8)
// OP == kBiasGeluBwd: v = x * gelu'(aux + bias)     (x = dH, aux = the pre-activation; column sums of v per
//                                                    64-row tile -> dbias_part[R / 64, C], reduced afterwards)
template <typename T, int FMT, int OP = kPlain>
__global__ __launch_bounds__(256) void fp8_cast_transpose_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                                 uint8_t* __restrict__ qt, int R, int C,
                                                                 const float* __restrict__ scale,
                                                                 unsigned int* __restrict__ amax_bits,
                                                                 const T* __restrict__ aux = nullptr,
                                                                 const T* __restrict__ bias = nullptr,
                                                                 float* __restrict__ dbias_part = nullptr) {
  __shared__ uint32_t tile[CT_TS * CT_LD / 4];
  __shared__ float red[4];
  __shared__ float colp[OP == kBiasGeluBwd ? 32 : 1][OP == kBiasGeluBwd ? CT_TS : 1];
  const int tid = threadIdx.x;
  const int lc = (tid & 7) * 8, lr = tid >> 3;   // 8 threads x 8 columns per row, 32 rows per pass
  const float sc = scale ? *scale : 1.f;
  const int tiles_c = C / CT_TS;
  const int ntiles = tiles_c * (R / CT_TS);
  float amax = 0.f;
  uint8_t* t8 = reinterpret_cast<uint8_t*>(tile);
  // software pipeline: the next tile's rows are loaded into registers before this tile's convert / LDS /
  // barrier phases, so every wave keeps a tile of reads in flight through the barriers
  typename Vec8<T>::raw_t xr[2], ar[2];
  auto load_tile = [&](int tt) {
    const int rr0 = (tt / tiles_c) * CT_TS, cc0 = (tt % tiles_c) * CT_TS;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      xr[p] = Vec8<T>::load_raw(x + (int64_t)(rr0 + lr + 32 * p) * C + cc0 + lc);
      if (OP == kBiasGeluBwd) ar[p] = Vec8<T>::load_raw(aux + (int64_t)(rr0 + lr + 32 * p) * C + cc0 + lc);
    }
  };
  if ((int)blockIdx.x < ntiles) load_tile(blockIdx.x);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r0 = (t / tiles_c) * CT_TS, c0 = (t % tiles_c) * CT_TS;
    float vin[2][8], ain[2][8];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      Vec8<T>::unpack(xr[p], vin[p]);
      if (OP == kBiasGeluBwd) Vec8<T>::unpack(ar[p], ain[p]);
    }
    float b[8];                                 // bias before the prefetch: in-order vmcnt would otherwise
    if (OP != kPlain) Vec8<T>::load(bias + c0 + lc, b);   // make the bias wait drain the next tile's loads too
    // unconditional (clamped) prefetch: a branch around it would make hipcc's waitcnt pass drain it at the
    // merge (vmcnt(0) before the bias / first use), serialising the pipeline again
    load_tile(min(t + (int)gridDim.x, ntiles - 1));
    float cs[8];
    if (OP == kBiasGeluBwd) {
#pragma unroll
      for (int k = 0; k < 8; ++k) cs[k] = 0.f;
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int r = lr + 32 * p;
      float* v = vin[p];
      if (OP != kPlain) {
        if (OP == kBiasGelu) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = gelu_tanh(v[k] + b[k]);
        } else {
          const float* a = ain[p];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            v[k] *= gelu_tanh_grad(a[k] + b[k]);
            cs[k] += v[k];
          }
        }
      }
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        amax = fmaxf(amax, fmaxf(fabsf(v[k]), fabsf(v[k + 4])));
        lo |= (uint32_t)to_fp8<FMT>(v[k] * sc) << (8 * k);
        hi |= (uint32_t)to_fp8<FMT>(v[k + 4] * sc) << (8 * k);
      }
      if (q) *reinterpret_cast<uint2*>(q + (int64_t)(r0 + r) * C + c0 + lc) = make_uint2(lo, hi);
      if (qt) {
        uint32_t* dst = tile + (r * CT_LD + lc) / 4;
        dst[0] = lo;
        dst[1] = hi;
      }
    }
    if (OP == kBiasGeluBwd) {                   // this tile's column sums of dA (deterministic, no atomics)
#pragma unroll
      for (int k = 0; k < 8; ++k) colp[lr][lc + k] = cs[k];
      __syncthreads();
      if (tid < CT_TS) {
        float sum = 0.f;
#pragma unroll 8
        for (int i = 0; i < 32; ++i) sum += colp[i][tid];
        dbias_part[(int64_t)(r0 / CT_TS) * C + c0 + tid] = sum;
      }
      if (!qt) __syncthreads();                 // colp reused by the next tile
    }
    if (qt) {
      __syncthreads();
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int c = lr + 32 * p;              // output row (= input column)
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          lo |= (uint32_t)t8[(lc + k) * CT_LD + c] << (8 * k);
          hi |= (uint32_t)t8[(lc + 4 + k) * CT_LD + c] << (8 * k);
        }
        *reinterpret_cast<uint2*>(qt + (int64_t)(c0 + c) * R + r0 + lc) = make_uint2(lo, hi);
      }
      __syncthreads();                          // tile reused by the next iteration
    }
  }
  if (amax_bits) {
    amax = wave_max(amax);
    if ((tid & 63) == 0) red[tid >> 6] = amax;
    __syncthreads();
    if (tid == 0) atomicMax(amax_bits, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
  }
}

// 128 x 128-tile variant for R % 128 == 0 and C % 128 == 0 (every GPT-2 / Llama shape): each lane converts 16
// consecutive elements, so a wave's row store is 8 rows x 128 contiguous bytes (16 B per lane) and its transposed
// store 8 output rows x 128 B -- the 64 x 64 tiles' 8-byte-per-lane / 64-byte-segment stores capped the casts at
// ~3.5-3.75 TB/s (scripts/bench_fp8_cast.py).  LDS rows are 132 B (33 words): the transposed byte gathers of a
// wave touch 16 banks twice (2-way), the 16-byte row writes go as four ds_write_b32.
constexpr int CT2 = 128, CT2_LD = 132;
// LDS word of (tile row, 4-column word w): 33-word rows, words of rows >= 64 rotated by 8 so the transposed
// gathers (16-row stride per lane group) spread over all 64 banks
__device__ __forceinline__ int ct2_word(int row, int w) { return row * (CT2_LD / 4) + ((w + ((row >> 6) << 3)) & 31); }
template <typename T, int FMT, int OP = kPlain>
__global__ __launch_bounds__(256) void fp8_ct128_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                        uint8_t* __restrict__ qt, int R, int C,
                                                        const float* __restrict__ scale,
                                                        unsigned int* __restrict__ amax_bits,
                                                        const T* __restrict__ aux, const T* __restrict__ bias,
                                                        float* __restrict__ dbias_part) {
  __shared__ uint32_t tile[CT2 * CT2_LD / 4];
  __shared__ float red[4];
  __shared__ float colp[OP == kBiasGeluBwd ? 32 : 1][OP == kBiasGeluBwd ? CT2 : 1];
  const int tid = threadIdx.x;
  const int lc = (tid & 7) * 16, lr = tid >> 3;  // 8 lanes x 16 columns per row, 32 rows per pass, 4 passes
  const float sc = scale ? *scale : 1.f;
  const int tiles_c = C / CT2;
  const int ntiles = tiles_c * (R / CT2);
  float amax = 0.f;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r0 = (t / tiles_c) * CT2, c0 = (t % tiles_c) * CT2;
    float b[16], cs[16];
    if (OP != kPlain) {
      Vec8<T>::load(bias + c0 + lc, b);
      Vec8<T>::load(bias + c0 + lc + 8, b + 8);
    }
    if (OP == kBiasGeluBwd) {
#pragma unroll
      for (int k = 0; k < 16; ++k) cs[k] = 0.f;
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = lr + 32 * p;
      const int64_t off = (int64_t)(r0 + r) * C + c0 + lc;
      float v[16];
      Vec8<T>::load(x + off, v);
      Vec8<T>::load(x + off + 8, v + 8);
      if (OP == kBiasGelu) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = gelu_tanh(v[k] + b[k]);
      } else if (OP == kBiasGeluBwd) {
        float a[16];
        Vec8<T>::load(aux + off, a);
        Vec8<T>::load(aux + off + 8, a + 8);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          v[k] *= gelu_tanh_grad(a[k] + b[k]);
          cs[k] += v[k];
        }
      }
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[j] = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float e = v[4 * j + k];
          amax = fmaxf(amax, fabsf(e));
          w[j] |= (uint32_t)to_fp8<FMT>(e * sc) << (8 * k);
        }
      }
      if (q) *reinterpret_cast<uint4*>(q + off) = make_uint4(w[0], w[1], w[2], w[3]);
      if (qt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[ct2_word(r, lc / 4 + j)] = w[j];
      }
    }
    if (OP == kBiasGeluBwd) {
#pragma unroll
      for (int k = 0; k < 16; ++k) colp[lr][lc + k] = cs[k];
      __syncthreads();
      if (tid < CT2) {
        float sum = 0.f;
#pragma unroll 8
        for (int i = 0; i < 32; ++i) sum += colp[i][tid];
        dbias_part[(int64_t)(r0 / CT2) * C + c0 + tid] = sum;
      }
      if (!qt) __syncthreads();
    }
    if (qt) {
      __syncthreads();
      // lane: 4 output rows (input columns 4g..4g+3) x 16 input rows (16j..16j+15): 16 word reads, 4x4 byte
      // transposes in registers (v_perm_b32), 4 x 16-byte stores -- 8 lanes cover an output row's 128 bytes
      const int j = tid & 7, g = tid >> 3;
      uint32_t o[4][4];                          // o[i][m]: output row 4g + i, input rows 16j + 4m .. + 3
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = tile[ct2_word(16 * j + 4 * m + k, g)];
        const uint32_t t0 = __builtin_amdgcn_perm(w[1], w[0], 0x05010400u), t1 = __builtin_amdgcn_perm(w[3], w[2], 0x05010400u);
        const uint32_t t2 = __builtin_amdgcn_perm(w[1], w[0], 0x07030602u), t3 = __builtin_amdgcn_perm(w[3], w[2], 0x07030602u);
        o[0][m] = __builtin_amdgcn_perm(t1, t0, 0x05040100u);
        o[1][m] = __builtin_amdgcn_perm(t1, t0, 0x07060302u);
        o[2][m] = __builtin_amdgcn_perm(t3, t2, 0x05040100u);
        o[3][m] = __builtin_amdgcn_perm(t3, t2, 0x07060302u);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint4*>(qt + (int64_t)(c0 + 4 * g + i) * R + r0 + 16 * j) =
            make_uint4(o[i][0], o[i][1], o[i][2], o[i][3]);
      __syncthreads();
    }
  }
  if (amax_bits) {
    amax = wave_max(amax);
    if ((tid & 63) == 0) red[tid >> 6] = amax;
    __syncthreads();
    if (tid == 0) atomicMax(amax_bits, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
  }
}

// Slots [s0, s1) of a module's fp8 meta: hist [n_slots, H], cur [n_slots] (amax bits), scale / scale_inv
// [n_slots].  One thread per slot (a module has 3).
__global__ void fp8_update_scales_kernel(float* __restrict__ hist, unsigned int* __restrict__ cur,
                                         float* __restrict__ scale, float* __restrict__ scale_inv, int H, int s0,
                                         int s1, float fmax, float margin_mul) {
  const int s = s0 + threadIdx.x;
  if (s >= s1) return;
  float* h = hist + (int64_t)s * H;
  const float a = __uint_as_float(cur[s]);
  float m = a;
  for (int i = H - 1; i > 0; --i) {
    const float v = h[i - 1];
    h[i] = v;
    m = fmaxf(m, v);
  }
  h[0] = a;
  cur[s] = 0u;
  if (m > 0.f && isfinite(m)) {
    const float sc = fmax / m * margin_mul;
    scale[s] = sc;
    scale_inv[s] = 1.f / sc;
  }
}

}  // namespace
}  // namespace pdt

using namespace pdt;

// 128-tile kernel when the shape allows (16-byte stores), else the 64-tile one; tile-row count of the dbias
// partials follows the tile (ct_tile_rows)
static bool ct_wide(int R, int C) {
  static const bool force64 = getenv("PDT_FP8_CT64") != nullptr;
  return R % CT2 == 0 && C % CT2 == 0 && !force64;
}
static bool aligned16(const void* a, const void* b, const void* c) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) == 0;
}
static int ct_tile_rows(int R, int C) { return ct_wide(R, C) ? CT2 : CT_TS; }
template <typename T, int FMT, int OP>
static void ct_launch(const T* x, uint8_t* q, uint8_t* qt, int R, int C, const float* scale, unsigned int* amax,
                      const T* aux, const T* bias, float* dbp, hipStream_t st) {
  const int ts = ct_tile_rows(R, C);
  const long long tiles = (long long)(R / ts) * (C / ts);
  const int grid = (int)(tiles < 2048 ? tiles : 2048);
  if (ts == CT2)
    fp8_ct128_kernel<T, FMT, OP><<<grid, 256, 0, st>>>(x, q, qt, R, C, scale, amax, aux, bias, dbp);
  else
    fp8_cast_transpose_kernel<T, FMT, OP><<<grid, 256, 0, st>>>(x, q, qt, R, C, scale, amax, aux, bias, dbp);
}

// fmt: 0 = e4m3fn, 1 = e5m2; dt: kF32 / kBF16.  Returns hipErrorInvalidValue for unsupported shapes
// (the Python side then takes its torch path).
PDT_API int pdt_fp8_cast_transpose(const void* x, void* q, void* qt, int R, int C, int dt, int fmt,
                                   const float* scale, unsigned int* amax_bits, hipStream_t st) {
  if (R <= 0 || C <= 0 || R % CT_TS || C % CT_TS) return (int)hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(qt)) & 15)
    return (int)hipErrorInvalidValue;
#define PDT_L(T, F) \
  ct_launch<T, F, kPlain>((const T*)x, (uint8_t*)q, (uint8_t*)qt, R, C, scale, amax_bits, nullptr, nullptr, nullptr, st)
  if (dt == kBF16) { if (fmt == 0) PDT_L(bf16_t, 0); else PDT_L(bf16_t, 1); }
  else if (dt == kF32) { if (fmt == 0) PDT_L(float, 0); else PDT_L(float, 1); }
  else return (int)hipErrorInvalidValue;
#undef PDT_L
  return (int)hipGetLastError();
}

// GPT-2 MLP in fp8 (kernels above with the GELU prologues), bf16 tensors, bias [C] bf16:
//   fwd: q / qt = fp8(gelu(a + bias) * scale)            amax of the GELU output
//   bwd: q / qt = fp8(dh * gelu'(a + bias) * scale)     amax of dA, dbias[C] (bf16) = column sums of dA
// ws: pdt_fp8_gelu_bwd_ws_floats(R, C) floats.
PDT_API long long pdt_fp8_gelu_bwd_ws_floats(int R, int C) {
  return (long long)(R / CT_TS) * C + red::col_ws_floats(R / CT_TS, C);   // sized for the 64-row tiles (the larger)
}

PDT_API int pdt_fp8_bias_gelu_ct(const void* a, const void* bias, void* q, void* qt, int R, int C, int fmt,
                                 const float* scale, unsigned int* amax_bits, hipStream_t st) {
  if (R <= 0 || C <= 0 || R % CT_TS || C % CT_TS || !bias || !aligned16(a, q, qt)) return (int)hipErrorInvalidValue;
  if (fmt == 0)
    ct_launch<bf16_t, 0, kBiasGelu>((const bf16_t*)a, (uint8_t*)q, (uint8_t*)qt, R, C, scale, amax_bits, nullptr,
                                    (const bf16_t*)bias, nullptr, st);
  else
    ct_launch<bf16_t, 1, kBiasGelu>((const bf16_t*)a, (uint8_t*)q, (uint8_t*)qt, R, C, scale, amax_bits, nullptr,
                                    (const bf16_t*)bias, nullptr, st);
  return (int)hipGetLastError();
}

PDT_API int pdt_fp8_bias_gelu_bwd_ct(const void* dh, const void* a, const void* bias, void* q, void* qt, void* dbias,
                                     float* ws, int R, int C, int fmt, const float* scale, unsigned int* amax_bits,
                                     hipStream_t st) {
  if (R <= 0 || C <= 0 || R % CT_TS || C % CT_TS || !bias || !ws || !aligned16(dh, q, qt) || !aligned16(a, a, a))
    return (int)hipErrorInvalidValue;
  if (fmt == 0)
    ct_launch<bf16_t, 0, kBiasGeluBwd>((const bf16_t*)dh, (uint8_t*)q, (uint8_t*)qt, R, C, scale, amax_bits,
                                       (const bf16_t*)a, (const bf16_t*)bias, ws, st);
  else
    ct_launch<bf16_t, 1, kBiasGeluBwd>((const bf16_t*)dh, (uint8_t*)q, (uint8_t*)qt, R, C, scale, amax_bits,
                                       (const bf16_t*)a, (const bf16_t*)bias, ws, st);
  const int pr = R / ct_tile_rows(R, C);   // dbias partial rows
  if (dbias) red::col_reduce<bf16_t>(ws, pr, C, (bf16_t*)dbias, ws + (long long)pr * C, 0, st);
  return (int)hipGetLastError();
}

PDT_API int pdt_fp8_update_scales(float* hist, unsigned int* cur, float* scale, float* scale_inv, int H, int s0, int s1,
                                  float fmax, float margin_mul, hipStream_t st) {
  if (H <= 0 || s1 <= s0 || s1 - s0 > 64) return (int)hipErrorInvalidValue;
  fp8_update_scales_kernel<<<1, 64, 0, st>>>(hist, cur, scale, scale_inv, H, s0, s1, fmax, margin_mul);
  return (int)hipGetLastError();
}
