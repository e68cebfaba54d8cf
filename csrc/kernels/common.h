// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of pytorch_distributedtraining_amd.
//
// Conventions used by every kernel file:
//   * wave64 everywhere: lane = threadIdx.x & 63, reductions span 64 lanes.
//   * bf16 is moved as raw 16-bit words in 16-byte vectors (u16x8) -- hipcc does not vectorise
//     scalar bf16 loads (cdna_hip_programming.md Guideline 13).
//   * every host entry point is `extern "C" int pdt_<name>(..., hipStream_t)` returning the
//     hipError_t of the launch, so the Python side (ctypes) can raise on failure.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define PDT_API extern "C" __attribute__((visibility("default")))

namespace pdt {

typedef unsigned short bf16_t;  // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kF64 = 3 };

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  // v_cvt_pk_bf16_f32 on gfx950 (round-to-nearest-even, NaN preserving)
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

__device__ __forceinline__ float h2f(bf16_t h) {
  _Float16 v = *reinterpret_cast<_Float16*>(&h);
  return (float)v;
}
__device__ __forceinline__ bf16_t f2h(float f) {
  _Float16 v = (_Float16)f;
  return *reinterpret_cast<bf16_t*>(&v);
}

// Load / store 8 consecutive elements of type T as floats.
template <typename T> struct Vec8;
template <> struct Vec8<float> {
  struct raw_t { f32x4 a, b; };
  __device__ __forceinline__ static raw_t load_raw(const float* p) {
    return raw_t{*reinterpret_cast<const f32x4*>(p), *reinterpret_cast<const f32x4*>(p + 4)};
  }
  __device__ __forceinline__ static void unpack(const raw_t& r, float* o) {
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = r.a[i]; o[4 + i] = r.b[i]; }
  }
  __device__ __forceinline__ static void load(const float* p, float* o) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = a[i]; o[4 + i] = b[i]; }
  }
  __device__ __forceinline__ static void store(float* p, const float* v) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = v[i]; b[i] = v[4 + i]; }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};
template <> struct Vec8<bf16_t> {
  typedef u16x8 raw_t;
  __device__ __forceinline__ static raw_t load_raw(const bf16_t* p) { return *reinterpret_cast<const u16x8*>(p); }
  __device__ __forceinline__ static void unpack(const raw_t& r, float* o) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = bf2f(r[i]);
  }
  __device__ __forceinline__ static void load(const bf16_t* p, float* o) {
    u16x8 a = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = bf2f(a[i]);
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float* v) {
    u16x8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = f2bf(v[i]);
    *reinterpret_cast<u16x8*>(p) = a;
  }
};

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<bf16_t>(bf16_t v) { return bf2f(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) { return f2bf(v); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == 64 * NW; every thread gets the result.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* scratch /* >= NW floats */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += scratch[i];
  __syncthreads();
  return t;
}

// Online (max, sum-of-exp) pair merge used by softmax-style reductions.
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  float mn = fmaxf(m, m2);
  if (mn == -INFINITY) { m = mn; s = 0.f; return; }
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

__device__ __forceinline__ void wave_lse(float& m, float& s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
}

// Grid size helper for memory-bound kernels (Guideline 11): cap and grid-stride the rest.
inline int grid_for(long long work_items, int per_block, int cap = 256 * 8) {
  long long g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace pdt
