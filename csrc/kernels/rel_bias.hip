// Swin relative-position bias: table [T, H] (T = (2 ws - 1)^2) <-> dense fp32 bias [H, N, N] for the fused window
// attention (window_attn.hip), one launch each way.  The stock path gathers with index_select, permutes, casts to
// fp32 and, in the backward, sums the attention kernel's per-workgroup partials, casts, zero-fills and index_adds
// -- 7-9 launches of a few microseconds per block per micro-step (48 of each per SwinIR-S step).
//
// backward: the G partials summed per (head, entry) in a fixed order, then each (table row, head) sums the entries
// that use that row through a CSR list built once on the host (fixed order): deterministic, no atomics.
#include "common.h"

using namespace pdt;

namespace {

constexpr int RB_NT = 256;

template <typename T>
__global__ __launch_bounds__(RB_NT) void rel_bias_gather_kernel(const T* __restrict__ table, const int* __restrict__ idx,
                                                               float* __restrict__ out, int H, int NN) {
  const int e = blockIdx.x * RB_NT + threadIdx.x;
  if (e >= H * NN) return;
  const int h = e / NN, p = e - h * NN;
  out[e] = to_f<T>(table[(int64_t)idx[p] * H + h]);
}

// dense[e] = sum over g of part[g][e] (fixed order): a workgroup takes 64 consecutive entries e, its 8 waves the
// g = w (mod 8) slabs with 4 independent loads in flight per lane, then the 8 wave sums are added in wave order
constexpr int SUM_WAVES = 8;
__global__ __launch_bounds__(64 * SUM_WAVES) void rel_bias_sum_kernel(const float* __restrict__ part, int G, int HNN,
                                                                     float* __restrict__ dense) {
  __shared__ float red[SUM_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (e < HNN) {
    int g = w;
    for (; g + 3 * SUM_WAVES < G; g += 4 * SUM_WAVES) {
      s0 += part[(int64_t)g * HNN + e];
      s1 += part[(int64_t)(g + SUM_WAVES) * HNN + e];
      s2 += part[(int64_t)(g + 2 * SUM_WAVES) * HNN + e];
      s3 += part[(int64_t)(g + 3 * SUM_WAVES) * HNN + e];
    }
    for (; g < G; g += SUM_WAVES) s0 += part[(int64_t)g * HNN + e];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && e < HNN) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < SUM_WAVES; ++i) t += red[i][lane];
    dense[e] = t;
  }
}

// out[t][h] = sum over row t's CSR positions of dense[h][p]: one wave per (t, h), a lane per position (<= 64 per
// row for windows up to 8 x 8; longer lists loop), summed in a fixed shuffle order
template <typename T>
__global__ __launch_bounds__(RB_NT) void rel_bias_scatter_kernel(const float* __restrict__ dense, int H, int NN,
                                                                const int* __restrict__ off,
                                                                const int* __restrict__ pos, int TR,
                                                                T* __restrict__ out) {
  const int e = blockIdx.x * (RB_NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (e >= TR * H) return;
  const int t = e / H, h = e - t * H;
  const float* d = dense + (int64_t)h * NN;
  float s = 0.f;
  for (int i = off[t] + lane; i < off[t + 1]; i += 64) s += d[pos[i]];
  s = wave_sum(s);
  if (lane == 0) out[e] = from_f<T>(s);
}

}  // namespace

// out [H][NN] fp32 = table[idx[p]][h]; table [*, H] in dt (kBF16 / kF32), idx [NN] int32
PDT_API int pdt_rel_bias_gather(const void* table, const int* idx, float* out, int H, int NN, int dt, hipStream_t st) {
  if (H <= 0 || NN <= 0) return (int)hipErrorInvalidValue;
  const int grid = (H * NN + RB_NT - 1) / RB_NT;
  if (dt == kF32)
    rel_bias_gather_kernel<float><<<grid, RB_NT, 0, st>>>((const float*)table, idx, out, H, NN);
  else if (dt == kBF16)
    rel_bias_gather_kernel<bf16_t><<<grid, RB_NT, 0, st>>>((const bf16_t*)table, idx, out, H, NN);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// out [TR][H] (dt) = sum over g, p in row t's CSR list of part[g][h][p]; part [G][H][NN] fp32; off [TR + 1], pos [NN];
// ws >= H * NN floats
PDT_API int pdt_rel_bias_scatter(const float* part, int G, int H, int NN, const int* off, const int* pos, int TR,
                                 void* out, int dt, float* ws, hipStream_t st) {
  if (G <= 0 || H <= 0 || NN <= 0 || TR <= 0 || (dt != kF32 && dt != kBF16)) return (int)hipErrorInvalidValue;
  rel_bias_sum_kernel<<<(H * NN + 63) / 64, 64 * SUM_WAVES, 0, st>>>(part, G, H * NN, ws);
  const int grid = (TR * H + RB_NT / 64 - 1) / (RB_NT / 64);
  if (dt == kF32)
    rel_bias_scatter_kernel<float><<<grid, RB_NT, 0, st>>>(ws, H, NN, off, pos, TR, (float*)out);
  else
    rel_bias_scatter_kernel<bf16_t><<<grid, RB_NT, 0, st>>>(ws, H, NN, off, pos, TR, (bf16_t*)out);
  return (int)hipGetLastError();
}
