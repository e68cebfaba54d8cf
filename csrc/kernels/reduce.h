// Deterministic column reductions shared by the norm / activation / bias-gradient kernels.
//
// Layout: a producer kernel sweeps a [rows, N] matrix as (column group) x (row chunk) workgroups --
// 256 threads x 8 columns = 2048 columns per group, `rows_per` consecutive rows per chunk -- and writes
// one fp32 partial row per chunk into part[R, N]; col_reduce() folds the partials (two levels, fixed
// order, so results are bitwise reproducible run to run).
#pragma once
#include "common.h"

namespace pdt {
namespace red {

constexpr int NT = 256;
constexpr int COLS_PER_GROUP = NT * 8;

// (R, rows_per): enough workgroups to cover HBM latency (~2048), chunks of >= 8 rows, R <= 1024
struct ColPlan {
  int R, rows_per, col_groups;
};
inline ColPlan col_plan(int rows, int N) {
  ColPlan p;
  p.col_groups = (N + COLS_PER_GROUP - 1) / COLS_PER_GROUP;
  int want = 2048 / p.col_groups;
  want = want < 64 ? 64 : (want > 1024 ? 1024 : want);
  int rows_per = (rows + want - 1) / want;
  if (rows_per < 8) rows_per = 8;
  p.rows_per = rows_per;
  p.R = (rows + rows_per - 1) / rows_per;
  return p;
}
// workspace floats for col_plan partials + the second reduction level
inline long long col_ws_floats(int rows, int N) { return ((long long)col_plan(rows, N).R + 64) * N; }

template <typename W, bool FINAL>
__global__ __launch_bounds__(NT) void col_reduce_kernel(const float* __restrict__ part, int R, int N,
                                                        W* __restrict__ out, float* __restrict__ part2,
                                                        int accumulate) {
  __shared__ float sred[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int per = (R + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  float s = 0.f;
  if (col < N)
    for (int r = r0 + wid; r < r1; r += 4) s += part[(int64_t)r * N + col];
  sred[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && col < N) {
    float t = sred[0][lane] + sred[1][lane] + sred[2][lane] + sred[3][lane];
    if (FINAL) {
      if (accumulate) t += to_f<W>(out[col]);
      out[col] = from_f<W>(t);
    } else {
      part2[(int64_t)blockIdx.y * N + col] = t;
    }
  }
}

// Up to 3 [R, N] partial matrices at part + z * R * N reduced in the same launches (blockIdx.z = matrix): the
// norm backward's dgamma / dbeta / residual-bias sums are ~5 us launches each, launch-bound.
struct ColOuts3 {
  void* out[3];
  int accumulate[3];
};
template <typename W, bool FINAL>
__global__ __launch_bounds__(NT) void col_reduce3_kernel(const float* __restrict__ part, int R, int N, ColOuts3 outs,
                                                         float* __restrict__ part2) {
  __shared__ float sred[4][64];
  const int z = blockIdx.z;
  part += (int64_t)z * R * N;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int per = (R + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(R, r0 + per);
  float s = 0.f;
  if (col < N)
    for (int r = r0 + wid; r < r1; r += 4) s += part[(int64_t)r * N + col];
  sred[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && col < N) {
    float t = sred[0][lane] + sred[1][lane] + sred[2][lane] + sred[3][lane];
    if (FINAL) {
      W* out = reinterpret_cast<W*>(outs.out[z]);
      if (outs.accumulate[z]) t += to_f<W>(out[col]);
      out[col] = from_f<W>(t);
    } else {
      part2[((int64_t)z * gridDim.y + blockIdx.y) * N + col] = t;
    }
  }
}

// nz (<= 3) matrices part[z][R, N] -> outs.out[z][N]; ws2 must hold >= nz * 64 * N floats.  The same two-level
// fixed-order reduction as col_reduce (bitwise equal results).
template <typename W>
inline void col_reduce3(const float* part, int R, int N, int nz, const ColOuts3& outs, float* ws2, hipStream_t st) {
  const int cg = (N + 63) / 64;
  int rs = 1;
  while (rs < 64 && cg * rs < 512 && R / (rs * 2) >= 8) rs *= 2;
  if (rs == 1) {
    col_reduce3_kernel<W, true><<<dim3(cg, 1, nz), NT, 0, st>>>(part, R, N, outs, nullptr);
  } else {
    col_reduce3_kernel<W, false><<<dim3(cg, rs, nz), NT, 0, st>>>(part, R, N, outs, ws2);
    col_reduce3_kernel<W, true><<<dim3(cg, 1, nz), NT, 0, st>>>(ws2, rs, N, outs, nullptr);
  }
}

// part[R, N] -> out[N] (+= if accumulate).  ws2 must hold >= 64 * N floats.
template <typename W>
inline void col_reduce(const float* part, int R, int N, W* out, float* ws2, int accumulate, hipStream_t st) {
  const int cg = (N + 63) / 64;
  int rs = 1;
  while (rs < 64 && cg * rs < 512 && R / (rs * 2) >= 8) rs *= 2;
  if (rs == 1) {
    col_reduce_kernel<W, true><<<dim3(cg, 1), NT, 0, st>>>(part, R, N, out, nullptr, accumulate);
  } else {
    col_reduce_kernel<W, false><<<dim3(cg, rs), NT, 0, st>>>(part, R, N, out, ws2, accumulate);
    col_reduce_kernel<W, true><<<dim3(cg, 1), NT, 0, st>>>(ws2, rs, N, out, nullptr, accumulate);
  }
}

}  // namespace red
}  // namespace pdt
