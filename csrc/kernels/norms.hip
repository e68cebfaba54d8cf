// LayerNorm and RMSNorm forward/backward for gfx950.
//
// Fast path: one wave64 per row, the row held in registers (8 elements per lane per 512-column
// slab, ITERS slabs), 16-byte loads/stores, fp32 statistics.  Exact two-pass variance from the
// register copy (no Welford needed because the row never leaves the VGPRs).  Backward keeps
// per-lane dgamma/dbeta partial sums in registers across the rows a wave visits and writes one
// partial row per wave; a deterministic column-reduce kernel folds them.
// Narrow rows (N <= 64, N % 4 == 0, e.g. SwinIR-S C = 60): 16 lanes x 4 elements per row, 4 rows per wave.
// Fallback (other N % 8 != 0, or N > 8192): one workgroup per row streaming from global memory.
//
// Reference parity: SwinIR LayerNorm sites (Stoke-DDP.py:206-208), GPT-2/Llama norms
// (BASELINE.json configs 3-5); semantics of torch.nn.functional.layer_norm / rms_norm.
#include "common.h"
#include "reduce.h"
#include <stdlib.h>

using namespace pdt;

namespace {

constexpr int NT = 256;      // threads per block
constexpr int RPB = NT / 64; // rows per block (one per wave)

template <typename T, typename W, int ITERS, bool RMS>
__global__ __launch_bounds__(NT) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                      const W* __restrict__ rb, T* __restrict__ sum_out,
                                                      const W* __restrict__ w, const W* __restrict__ b,
                                                      T* __restrict__ y, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out, int rows, int N, float eps) {
  // optional fused residual: s = x + res (+ rb[col], the bias of the Linear that produced res) is written to
  // sum_out and normalised (saves one full pass of the residual stream per norm site)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float invN = 1.f / (float)N;
  for (int row = blockIdx.x * RPB + wid; row < rows; row += gridDim.x * RPB) {
    const T* xr = x + (int64_t)row * N;
    float v[ITERS][8];
    float s = 0.f;
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int col = it * 512 + lane * 8;
      if (col < N) {
        Vec8<T>::load(xr + col, v[it]);
        if (res != nullptr) {
          float r8[8];
          Vec8<T>::load(res + (int64_t)row * N + col, r8);
          if (rb != nullptr) {
            float b8[8];
            Vec8<W>::load(rb + col, b8);
#pragma unroll
            for (int k = 0; k < 8; ++k) r8[k] += b8[k];
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) v[it][k] += r8[k];
          Vec8<T>::store(sum_out + (int64_t)row * N + col, v[it]);
          // normalise exactly what was stored (the T-rounded sum), rounded in registers
          if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[it][k] = bf2f(f2bf(v[it][k]));
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[it][k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += RMS ? v[it][k] * v[it][k] : v[it][k];
    }
    s = wave_sum(s);
    float mean = 0.f, rstd;
    if (RMS) {
      rstd = rsqrtf(s * invN + eps);
    } else {
      mean = s * invN;
      float q = 0.f;
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int col = it * 512 + lane * 8;
        if (col < N) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { float d = v[it][k] - mean; q += d * d; }
        }
      }
      q = wave_sum(q);
      rstd = rsqrtf(q * invN + eps);
    }
    T* yr = y + (int64_t)row * N;
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int col = it * 512 + lane * 8;
      if (col < N) {
        float wv[8], bv[8], o[8];
        Vec8<W>::load(w + col, wv);
        if (!RMS && b != nullptr) Vec8<W>::load(b + col, bv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float t = (v[it][k] - mean) * rstd * wv[k];
          o[k] = (!RMS && b != nullptr) ? t + bv[k] : t;
        }
        Vec8<T>::store(yr + col, o);
      }
    }
    if (lane == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// Backward: one wave per row, single pass over HBM.  The row's x and dy stay in registers between the
// two row reductions and the dx write (no re-read), gamma is loaded once per wave, and the NEXT row's
// x / dy / dres loads are issued before the current row's reductions so every wave keeps a full row of
// 16-B loads in flight (the previous two-pass form was latency-bound at ~1.4 TB/s).  Per-lane
// dgamma/dbeta partials accumulate in registers; at the end the 4 waves of a workgroup fold them
// through one [2][N] LDS buffer (wave by wave, no atomics) and the workgroup writes ONE partial row;
// a 2-level column reduce (reduce.h) finishes dgamma/dbeta.
// DSUM: also the column sums of dx as stored (-> ds_part): the gradient of a bias folded into the forward's
// residual sum (norm_fwd's rb), so the producing Linear needs no separate column-sum pass over its dY.
template <typename T, typename W, int ITERS, bool RMS, bool DRES, int OCC, bool DSUM>
__global__ __launch_bounds__(NT, OCC) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                      const W* __restrict__ w, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, const T* __restrict__ dres,
                                                      T* __restrict__ dx, float* __restrict__ dw_part,
                                                      float* __restrict__ db_part, float* __restrict__ ds_part,
                                                      int rows, int N) {
  extern __shared__ __attribute__((aligned(16))) float sacc[];   // [2 or 3][N]
  typedef typename Vec8<T>::raw_t raw_t;
  typedef typename Vec8<W>::raw_t wraw_t;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float invN = 1.f / (float)N;
  // loads are unconditional (column clamped into the row, row clamped into the matrix); lanes past
  // the row end are masked at accumulate / store time
  int cc[ITERS];
  bool cv[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int col = it * 512 + lane * 8;
    cv[it] = col < N;
    cc[it] = cv[it] ? col : N - 8;
  }
  float dwa[ITERS][8], dba[ITERS][8], dsa[DSUM ? ITERS : 1][8];
  wraw_t wr[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { dwa[it][k] = 0.f; dba[it][k] = 0.f; if constexpr (DSUM) dsa[it][k] = 0.f; }
    wr[it] = Vec8<W>::load_raw(w + cc[it]);
  }
  const int stride = gridDim.x * RPB;
  int row = blockIdx.x * RPB + wid;
  raw_t cx[ITERS], cg[ITERS], cr[DRES ? ITERS : 1];
  {
    const int64_t r = min(row, rows - 1);
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      cx[it] = Vec8<T>::load_raw(x + r * N + cc[it]);
      cg[it] = Vec8<T>::load_raw(dy + r * N + cc[it]);
      if constexpr (DRES) cr[it] = Vec8<T>::load_raw(dres + r * N + cc[it]);
    }
  }
  for (; row < rows; row += stride) {
    // prefetch the next row (double buffer): in flight during this row's math and reductions
    raw_t nx[ITERS], ng[ITERS], nr[DRES ? ITERS : 1];
    const int64_t nrow = min(row + stride, rows - 1);
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      nx[it] = Vec8<T>::load_raw(x + nrow * N + cc[it]);
      ng[it] = Vec8<T>::load_raw(dy + nrow * N + cc[it]);
      if constexpr (DRES) nr[it] = Vec8<T>::load_raw(dres + nrow * N + cc[it]);
    }
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      float xv[8], dv[8], wv[8];
      Vec8<T>::unpack(cx[it], xv);
      Vec8<T>::unpack(cg[it], dv);
      Vec8<W>::unpack(wr[it], wv);
      const float m = cv[it] ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[k] - mean) * rstd;
        const float d = dv[k] * m;
        const float g = d * wv[k];
        a += g * xh;
        bsum += g;
        dwa[it][k] += d * xh;
        dba[it][k] += d;
      }
    }
    a = wave_sum(a) * invN;
    if (!RMS) bsum = wave_sum(bsum) * invN;
    if constexpr (sizeof(T) == 2) {
      // re-unpack the packed row for the dx pass instead of keeping fp32 copies live across the
      // reductions (halves the row's register footprint: 2 waves/SIMD at N = 2048)
#pragma unroll
      for (int it = 0; it < ITERS; ++it) asm volatile("" : "+v"(cx[it]), "+v"(cg[it]));
    }
    T* dxr = dx + (int64_t)row * N;
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      float xv[8], dv[8], wv[8], o[8];
      Vec8<T>::unpack(cx[it], xv);
      Vec8<T>::unpack(cg[it], dv);
      Vec8<W>::unpack(wr[it], wv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = rstd * (dv[k] * wv[k] - (RMS ? 0.f : bsum) - (xv[k] - mean) * rstd * a);
      if constexpr (DRES) {
        float rv[8];
        Vec8<T>::unpack(cr[it], rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] += rv[k];
      }
      if constexpr (DSUM) {   // the bias gradient sums dx as stored (masked lanes hold a clamped column)
        const float m = cv[it] ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) dsa[it][k] += m * to_f<T>(from_f<T>(o[k]));
      }
      if (cv[it]) Vec8<T>::store(dxr + cc[it], o);
      cx[it] = nx[it];
      cg[it] = ng[it];
      if constexpr (DRES) cr[it] = nr[it];
    }
  }
  // fold the 4 waves' accumulators: wave 0 stores, waves 1..3 add in turn (no atomics)
  float* sdw = sacc;
  float* sdb = sacc + N;
  float* sds = sacc + 2 * N;
#pragma unroll
  for (int turn = 0; turn < RPB; ++turn) {
    if (wid == turn) {
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int col = it * 512 + lane * 8;
        if (col < N) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (turn == 0) {
              sdw[col + k] = dwa[it][k]; sdb[col + k] = dba[it][k];
              if constexpr (DSUM) sds[col + k] = dsa[it][k];
            } else {
              sdw[col + k] += dwa[it][k]; sdb[col + k] += dba[it][k];
              if constexpr (DSUM) sds[col + k] += dsa[it][k];
            }
          }
        }
      }
    }
    __syncthreads();
  }
  for (int c = threadIdx.x * 4; c < N; c += NT * 4) {
    *reinterpret_cast<f32x4*>(dw_part + (int64_t)blockIdx.x * N + c) = *reinterpret_cast<const f32x4*>(sdw + c);
    if (db_part) *reinterpret_cast<f32x4*>(db_part + (int64_t)blockIdx.x * N + c) = *reinterpret_cast<const f32x4*>(sdb + c);
    if constexpr (DSUM)
      *reinterpret_cast<f32x4*>(ds_part + (int64_t)blockIdx.x * N + c) = *reinterpret_cast<const f32x4*>(sds + c);
  }
}

// ---- wide rows (N > 2048, e.g. Llama-3 8B's d = 4,096): one ROW per workgroup, split over its 4 waves ----
// The wave-per-row kernel above keeps a whole row (and the next one, prefetched) plus the per-column dgamma
// partials in registers: at N = 4,096 that is > 256 VGPRs and the compiler spilled 200-540 of them to scratch
// (300 us per call, ~1.8 TB/s at Llama's 16,384 x 4,096).  Here wave w owns columns [w N/4, (w+1) N/4): its
// slice of the row (IT 512-column slabs, IT = N / 2048) and of the dgamma partials stays small, the two row
// reductions cross waves through an 8-float LDS slot (double-buffered by row parity: one barrier per row), and
// since the waves own disjoint columns each workgroup writes its partial row straight from registers.
template <typename T, typename W, int IT, bool RMS, bool DRES, bool DSUM>
__global__ __launch_bounds__(NT, 2) void norm_bwd_split_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                               const W* __restrict__ w, const float* __restrict__ mean_in,
                                                               const float* __restrict__ rstd_in,
                                                               const T* __restrict__ dres, T* __restrict__ dx,
                                                               float* __restrict__ dw_part, float* __restrict__ db_part,
                                                               float* __restrict__ ds_part, int rows, int N) {
  __shared__ float red[2][2][RPB];          // [row parity][a, bsum][wave]
  typedef typename Vec8<T>::raw_t raw_t;
  typedef typename Vec8<W>::raw_t wraw_t;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float invN = 1.f / (float)N;
  const int span = N / RPB;                 // columns per wave (a multiple of 8)
  int cc[IT];
  bool cv[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 512 + lane * 8;
    cv[it] = c < span;
    cc[it] = wid * span + (cv[it] ? c : span - 8);
  }
  float dwa[IT][8], dba[IT][8], dsa[DSUM ? IT : 1][8];
  wraw_t wr[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { dwa[it][k] = 0.f; dba[it][k] = 0.f; if constexpr (DSUM) dsa[it][k] = 0.f; }
    wr[it] = Vec8<W>::load_raw(w + cc[it]);
  }
  raw_t cx[IT], cg[IT], cr[DRES ? IT : 1];
  int row = blockIdx.x;
  {
    const int64_t r = min(row, rows - 1);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      cx[it] = Vec8<T>::load_raw(x + r * N + cc[it]);
      cg[it] = Vec8<T>::load_raw(dy + r * N + cc[it]);
      if constexpr (DRES) cr[it] = Vec8<T>::load_raw(dres + r * N + cc[it]);
    }
  }
  int par = 0;
  for (; row < rows; row += gridDim.x, par ^= 1) {
    raw_t nx[IT], ng[IT], nr[DRES ? IT : 1];
    const int64_t nrow = min(row + (int)gridDim.x, rows - 1);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      nx[it] = Vec8<T>::load_raw(x + nrow * N + cc[it]);
      ng[it] = Vec8<T>::load_raw(dy + nrow * N + cc[it]);
      if constexpr (DRES) nr[it] = Vec8<T>::load_raw(dres + nrow * N + cc[it]);
    }
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      float xv[8], dv[8], wv[8];
      Vec8<T>::unpack(cx[it], xv);
      Vec8<T>::unpack(cg[it], dv);
      Vec8<W>::unpack(wr[it], wv);
      const float m = cv[it] ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[k] - mean) * rstd;
        const float d = dv[k] * m;
        const float g = d * wv[k];
        a += g * xh;
        bsum += g;
        dwa[it][k] += d * xh;
        dba[it][k] += d;
      }
    }
    a = wave_sum(a);
    if (!RMS) bsum = wave_sum(bsum);
    if (lane == 0) {
      red[par][0][wid] = a;
      red[par][1][wid] = bsum;
    }
    __syncthreads();     // the slot of this parity is rewritten two rows later, after the next barrier
    a = (red[par][0][0] + red[par][0][1] + red[par][0][2] + red[par][0][3]) * invN;
    if (!RMS) bsum = (red[par][1][0] + red[par][1][1] + red[par][1][2] + red[par][1][3]) * invN;
    T* dxr = dx + (int64_t)row * N;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      float xv[8], dv[8], wv[8], o[8];
      Vec8<T>::unpack(cx[it], xv);
      Vec8<T>::unpack(cg[it], dv);
      Vec8<W>::unpack(wr[it], wv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = rstd * (dv[k] * wv[k] - (RMS ? 0.f : bsum) - (xv[k] - mean) * rstd * a);
      if constexpr (DRES) {
        float rv[8];
        Vec8<T>::unpack(cr[it], rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] += rv[k];
      }
      if constexpr (DSUM) {
        const float m = cv[it] ? 1.f : 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) dsa[it][k] += m * to_f<T>(from_f<T>(o[k]));
      }
      if (cv[it]) Vec8<T>::store(dxr + cc[it], o);
      cx[it] = nx[it];
      cg[it] = ng[it];
      if constexpr (DRES) cr[it] = nr[it];
    }
  }
  // disjoint columns per wave: the workgroup's partial row straight from registers
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if (!cv[it]) continue;
    const int64_t o = (int64_t)blockIdx.x * N + cc[it];
    *reinterpret_cast<f32x4*>(dw_part + o) = f32x4{dwa[it][0], dwa[it][1], dwa[it][2], dwa[it][3]};
    *reinterpret_cast<f32x4*>(dw_part + o + 4) = f32x4{dwa[it][4], dwa[it][5], dwa[it][6], dwa[it][7]};
    if (db_part) {
      *reinterpret_cast<f32x4*>(db_part + o) = f32x4{dba[it][0], dba[it][1], dba[it][2], dba[it][3]};
      *reinterpret_cast<f32x4*>(db_part + o + 4) = f32x4{dba[it][4], dba[it][5], dba[it][6], dba[it][7]};
    }
    if constexpr (DSUM) {
      *reinterpret_cast<f32x4*>(ds_part + o) = f32x4{dsa[it][0], dsa[it][1], dsa[it][2], dsa[it][3]};
      *reinterpret_cast<f32x4*>(ds_part + o + 4) = f32x4{dsa[it][4], dsa[it][5], dsa[it][6], dsa[it][7]};
    }
  }
}
// the split kernel's shape contract: 4 waves x IT slabs of 512 columns, each wave's span a multiple of 8
__host__ __device__ constexpr bool split_rows_ok(int N) { return N > 2048 && N <= 16384 && N % (8 * RPB) == 0; }

// ---- fallback: one block per row, streamed from global memory ----
template <typename T, typename W, bool RMS>
__global__ __launch_bounds__(NT) void norm_fwd_generic(const T* __restrict__ x, const T* __restrict__ res,
                                                       const W* __restrict__ rb, T* __restrict__ sum_out,
                                                       const W* __restrict__ w,
                                                       const W* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int rows, int N, float eps) {
  __shared__ float red[RPB];
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    if (res != nullptr) {
      for (int c = threadIdx.x; c < N; c += NT)
        sum_out[(int64_t)row * N + c] = from_f<T>(to_f<T>(x[(int64_t)row * N + c]) +
                                                  (to_f<T>(res[(int64_t)row * N + c]) + (rb ? to_f<W>(rb[c]) : 0.f)));
      __syncthreads();
    }
    const T* xr = (res != nullptr ? sum_out : x) + (int64_t)row * N;
    float s = 0.f;
    for (int c = threadIdx.x; c < N; c += NT) { float v = to_f<T>(xr[c]); s += RMS ? v * v : v; }
    s = block_sum<RPB>(s, red);
    float mean = 0.f, rstd;
    if (RMS) {
      rstd = rsqrtf(s / N + eps);
    } else {
      mean = s / N;
      float q = 0.f;
      for (int c = threadIdx.x; c < N; c += NT) { float d = to_f<T>(xr[c]) - mean; q += d * d; }
      q = block_sum<RPB>(q, red);
      rstd = rsqrtf(q / N + eps);
    }
    T* yr = y + (int64_t)row * N;
    for (int c = threadIdx.x; c < N; c += NT) {
      float t = (to_f<T>(xr[c]) - mean) * rstd * to_f<W>(w[c]);
      if (!RMS && b != nullptr) t += to_f<W>(b[c]);
      yr[c] = from_f<T>(t);
    }
    if (threadIdx.x == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename T, typename W, bool RMS>
__global__ __launch_bounds__(NT) void norm_bwd_generic(const T* __restrict__ dy, const T* __restrict__ x,
                                                       const W* __restrict__ w, const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, const T* __restrict__ dres,
                                                       T* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       float* __restrict__ ds_part, int rows, int N) {
  // partial row per block: rows handled by this block are accumulated straight into it
  __shared__ float red[RPB];
  float* dwp = dw_part + (int64_t)blockIdx.x * N;
  float* dbp = db_part ? db_part + (int64_t)blockIdx.x * N : nullptr;
  float* dsp = ds_part ? ds_part + (int64_t)blockIdx.x * N : nullptr;
  for (int c = threadIdx.x; c < N; c += NT) { dwp[c] = 0.f; if (dbp) dbp[c] = 0.f; if (dsp) dsp[c] = 0.f; }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const T* xr = x + (int64_t)row * N;
    const T* gr = dy + (int64_t)row * N;
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float a = 0.f, bs = 0.f;
    for (int c = threadIdx.x; c < N; c += NT) {
      float xh = (to_f<T>(xr[c]) - mean) * rstd, d = to_f<T>(gr[c]);
      float g = d * to_f<W>(w[c]);
      a += g * xh; bs += g;
      dwp[c] += d * xh;
      if (dbp) dbp[c] += d;
    }
    a = block_sum<RPB>(a, red) / N;
    bs = RMS ? 0.f : block_sum<RPB>(bs, red) / N;
    T* dxr = dx + (int64_t)row * N;
    for (int c = threadIdx.x; c < N; c += NT) {
      float xh = (to_f<T>(xr[c]) - mean) * rstd;
      float g = to_f<T>(gr[c]) * to_f<W>(w[c]);
      float o = rstd * (g - bs - xh * a);
      if (dres != nullptr) o += to_f<T>(dres[(int64_t)row * N + c]);
      dxr[c] = from_f<T>(o);
      if (dsp) dsp[c] += to_f<T>(from_f<T>(o));
    }
  }
}

// ---- narrow rows (N <= 64, N % 4 == 0; SwinIR-S C = 60): 16 lanes x 4 elements per row, 4 rows per
// wave.  The generic kernel would give a 60-wide row a whole 256-thread workgroup (196 idle threads and
// two block barriers per row); here a wave normalises 4 rows per pass with shuffle-only reductions.
constexpr int SM_LPR = 16;                 // lanes per row
constexpr int SM_RPW = 64 / SM_LPR;        // rows per wave pass
constexpr int SM_RPB = SM_RPW * RPB;       // rows per block pass

__host__ __device__ __forceinline__ bool small_rows(int N) { return N <= 64 && N % 4 == 0; }

template <typename T> struct Vec4;
template <> struct Vec4<float> {
  __device__ static void load(const float* p, float* o) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(p);
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
  }
  __device__ static void store(float* p, const float* o) { *reinterpret_cast<f32x4*>(p) = f32x4{o[0], o[1], o[2], o[3]}; }
};
template <> struct Vec4<bf16_t> {
  __device__ static void load(const bf16_t* p, float* o) {
    const u16x4 v = *reinterpret_cast<const u16x4*>(p);
    o[0] = bf2f(v[0]); o[1] = bf2f(v[1]); o[2] = bf2f(v[2]); o[3] = bf2f(v[3]);
  }
  __device__ static void store(bf16_t* p, const float* o) {
    *reinterpret_cast<u16x4*>(p) = u16x4{f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
  }
};

__device__ __forceinline__ float row16_sum(float v) {   // sum over the 16 lanes of one row
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Swin's shifted-window permutation folded into the narrow-row norms (SwinIR-S, C = 60): image-order row r of
// [B, H*W, C] <-> row img_to_win(r) of the window-ordered [B*nW, ws*ws, C] (torch.roll by -shift, then window
// partition; the inverse of conv.hip's window_perm_kernel).  mode bit 0: the forward's y is written to / the
// backward's dy is read from window-order rows (the block's norm1 feeds the qkv projection in window order);
// bit 1: the forward's residual input is read from window-order rows / the backward also writes that residual's
// gradient to window-order rows (norm2's x + attention output).  Each replaces a whole permutation pass.
struct WinMap {
  int H, W, ws, shift, mode;
};
// 32-bit unsigned divisions (the host keeps rows < 2^31): the 64-bit division this was written with cost ~100 VALU
// per call, once per row in every narrow-row norm pass of a Swin block
__device__ __forceinline__ int64_t img_to_win(int64_t r, const WinMap& m) {
  const uint32_t per_img = (uint32_t)(m.H * m.W);
  const uint32_t r32 = (uint32_t)r;
  const uint32_t b = r32 / per_img;
  const uint32_t t = r32 - b * per_img;
  const uint32_t th = t / (uint32_t)m.W;
  int h = (int)th - m.shift, w = (int)(t - th * (uint32_t)m.W) - m.shift;
  if (h < 0) h += m.H;
  if (w < 0) w += m.W;
  const uint32_t ws = (uint32_t)m.ws;
  const uint32_t wh = (uint32_t)h / ws, i = (uint32_t)h - wh * ws, ww = (uint32_t)w / ws, j = (uint32_t)w - ww * ws;
  return (int64_t)b * per_img + (int64_t)((wh * ((uint32_t)m.W / ws) + ww) * ws * ws + i * ws + j);
}

template <typename T, typename W, bool RMS>
__global__ __launch_bounds__(NT) void norm_fwd_small(const T* __restrict__ x, const T* __restrict__ res,
                                                     const W* __restrict__ rb, T* __restrict__ sum_out,
                                                     const W* __restrict__ w,
                                                     const W* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, int N, float eps, WinMap wm) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sub = lane / SM_LPR, c0 = (lane % SM_LPR) * 4;
  const bool col_ok = c0 < N;
  float wr[4] = {0, 0, 0, 0}, br[4] = {0, 0, 0, 0}, rbr[4] = {0, 0, 0, 0};
  if (col_ok) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      wr[k] = to_f<W>(w[c0 + k]);
      if (!RMS && b != nullptr) br[k] = to_f<W>(b[c0 + k]);
      if (rb != nullptr) rbr[k] = to_f<W>(rb[c0 + k]);
    }
  }
  const float inv_n = 1.f / N;
  for (int64_t base = ((int64_t)blockIdx.x * RPB + wv) * SM_RPW; base < rows; base += (int64_t)gridDim.x * SM_RPB) {
    const int64_t row = base + sub;
    const bool ok = col_ok && row < rows;
    float v[4] = {0, 0, 0, 0};
    if (ok) {
      Vec4<T>::load(x + row * N + c0, v);
      if (res != nullptr) {
        float r[4];
        Vec4<T>::load(res + ((wm.mode & 2) ? img_to_win(row, wm) : row) * N + c0, r);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = to_f<T>(from_f<T>(v[k] + (r[k] + rbr[k])));   // the stored sum, rounded
        Vec4<T>::store(sum_out + row * N + c0, v);
      }
    }
    float mean = 0.f, rstd;
    if (RMS) {
      rstd = rsqrtf(row16_sum(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]) * inv_n + eps);
    } else {
      mean = row16_sum(v[0] + v[1] + v[2] + v[3]) * inv_n;
      float q = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) { const float d = ok ? v[k] - mean : 0.f; q += d * d; }
      rstd = rsqrtf(row16_sum(q) * inv_n + eps);
    }
    if (ok) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = (v[k] - mean) * rstd * wr[k] + br[k];
      Vec4<T>::store(y + ((wm.mode & 1) ? img_to_win(row, wm) : row) * N + c0, o);
    }
    if (row < rows && c0 == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename T, typename W, bool RMS>
__global__ __launch_bounds__(NT) void norm_bwd_small(const T* __restrict__ dy, const T* __restrict__ x,
                                                     const W* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const T* __restrict__ dres,
                                                     T* __restrict__ dx, float* __restrict__ dw_part,
                                                     float* __restrict__ db_part, float* __restrict__ ds_part,
                                                     int rows, int N, WinMap wm, T* __restrict__ dr_win) {
  __shared__ __attribute__((aligned(16))) float sred[3][RPB][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sub = lane / SM_LPR, c0 = (lane % SM_LPR) * 4;
  const bool col_ok = c0 < N;
  float wr[4] = {0, 0, 0, 0};
  if (col_ok) {
#pragma unroll
    for (int k = 0; k < 4; ++k) wr[k] = to_f<W>(w[c0 + k]);
  }
  float dwa[4] = {0, 0, 0, 0}, dba[4] = {0, 0, 0, 0}, dsa[4] = {0, 0, 0, 0};
  const float inv_n = 1.f / N;
  for (int64_t base = ((int64_t)blockIdx.x * RPB + wv) * SM_RPW; base < rows; base += (int64_t)gridDim.x * SM_RPB) {
    const int64_t row = base + sub;
    const bool ok = col_ok && row < rows;
    float xv[4] = {0, 0, 0, 0}, g[4] = {0, 0, 0, 0};
    float mean = 0.f, rstd = 0.f;
    if (ok) {
      Vec4<T>::load(x + row * N + c0, xv);
      Vec4<T>::load(dy + ((wm.mode & 1) ? img_to_win(row, wm) : row) * N + c0, g);
      mean = RMS ? 0.f : mean_in[row];
      rstd = rstd_in[row];
    }
    float xh[4], gw[4], a = 0.f, bs = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xh[k] = ok ? (xv[k] - mean) * rstd : 0.f;
      gw[k] = g[k] * wr[k];
      a += gw[k] * xh[k];
      bs += gw[k];
      dwa[k] += g[k] * xh[k];
      dba[k] += g[k];
    }
    a = row16_sum(a) * inv_n;
    bs = RMS ? 0.f : row16_sum(bs) * inv_n;
    if (ok) {
      float o[4];
      if (dres != nullptr) Vec4<T>::load(dres + row * N + c0, o);
      else o[0] = o[1] = o[2] = o[3] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] += rstd * (gw[k] - bs - xh[k] * a);
      Vec4<T>::store(dx + row * N + c0, o);
      if (wm.mode & 2) Vec4<T>::store(dr_win + img_to_win(row, wm) * N + c0, o);   // the residual's gradient
#pragma unroll
      for (int k = 0; k < 4; ++k) dsa[k] += to_f<T>(from_f<T>(o[k]));
    }
  }
  // fold the 4 row groups of the wave (lanes c, c+16, c+32, c+48 share columns), then the block's waves
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    dwa[k] += __shfl_xor(dwa[k], 16, 64); dwa[k] += __shfl_xor(dwa[k], 32, 64);
    dba[k] += __shfl_xor(dba[k], 16, 64); dba[k] += __shfl_xor(dba[k], 32, 64);
    dsa[k] += __shfl_xor(dsa[k], 16, 64); dsa[k] += __shfl_xor(dsa[k], 32, 64);
  }
  if (sub == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sred[0][wv][c0 + k] = dwa[k]; sred[1][wv][c0 + k] = dba[k]; sred[2][wv][c0 + k] = dsa[k];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += NT) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < RPB; ++q) { s0 += sred[0][q][c]; s1 += sred[1][q][c]; s2 += sred[2][q][c]; }
    dw_part[(int64_t)blockIdx.x * N + c] = s0;
    if (db_part) db_part[(int64_t)blockIdx.x * N + c] = s1;
    if (ds_part) ds_part[(int64_t)blockIdx.x * N + c] = s2;
  }
}

// column reductions of the [R, N] dgamma/dbeta partials: reduce.h (two-level, deterministic)
using red::col_reduce;

template <typename T, typename W, bool RMS>
int launch_fwd(const void* x, const void* res, const void* rb, void* sum_out, const void* w, const void* b, void* y,
               float* mean, float* rstd, int rows, int N, float eps, hipStream_t st, WinMap wm = {}) {
  const T* X = (const T*)x; const T* R = (const T*)res; T* S = (T*)sum_out; const W* RB = (const W*)rb;
  const W* Wt = (const W*)w; const W* B = (const W*)b; T* Y = (T*)y;
  if (wm.mode != 0 && !small_rows(N)) return (int)hipErrorInvalidValue;   // window maps: narrow rows only
  if (small_rows(N)) {
    norm_fwd_small<T, W, RMS><<<grid_for(rows, SM_RPB, 256 * 16), NT, 0, st>>>(X, R, RB, S, Wt, B, Y, mean, rstd, rows, N,
                                                                              eps, wm);
  } else if (N % 8 == 0 && N <= 8192) {
    // workgroups per CU: 64 (plain) / 96 (fused residual add) -- GPT-2 1.3B norms at 96 x 1024 tokens, 2,048
    // columns: plain 178 (16) -> 167.8 (32) -> 164.9 us (64), residual add 291 -> 250 us (96)
    // (profiles/r5/r5v_norm_grid_ab.txt)
    static const int cap_env = [] { const char* e = getenv("PDT_NORM_FWD_WG_PER_CU"); return e ? atoi(e) : 0; }();
    const int cap = cap_env > 0 ? cap_env : (res != nullptr ? 96 : 64);
    const int grid = grid_for(rows, RPB, 256 * cap);
    const int iters = (N + 511) / 512;
#define PDT_NF(I) norm_fwd_kernel<T, W, I, RMS><<<grid, NT, 0, st>>>(X, R, RB, S, Wt, B, Y, mean, rstd, rows, N, eps)
    if (iters <= 1) PDT_NF(1);
    else if (iters <= 2) PDT_NF(2);
    else if (iters <= 4) PDT_NF(4);
    else if (iters <= 8) PDT_NF(8);
    else PDT_NF(16);
#undef PDT_NF
  } else {
    norm_fwd_generic<T, W, RMS><<<grid_for(rows, 1, 256 * 8), NT, 0, st>>>(X, R, RB, S, Wt, B, Y, mean, rstd, rows, N, eps);
  }
  return (int)hipGetLastError();
}

// fast path: one partial row per workgroup (LDS-accumulated); fallback: one per block
int bwd_partial_rows(int rows, int N) {
  // enough waves to cover HBM latency (the row kernel holds ~120 VGPRs at N = 2048: 4 waves/SIMD)
  // a few rows per wave (so the row prefetch pays) while covering the chip: ~2 waves per SIMD
  if (small_rows(N)) {
    // 1024 workgroups: SwinIR-S bf16 426.3 -> 433.5 samples/s against 512 (2048: 433.1;
    // profiles/r6/r6k_grid_ab.jsonl); PDT_NORM_SMALL_BWD_WG overrides
    static const int scap = [] { const char* e = getenv("PDT_NORM_SMALL_BWD_WG"); return e ? atoi(e) : 1024; }();
    return grid_for(rows, SM_RPB * 8, scap);
  }
  // 256 partial-row workgroups: the flagship step 668.1 / 669.7 -> 664.8 / 669.3 ms against 512, the norm_pass
  // backward alone 360-405 -> 377-386 us (profiles/r5/r5v_norm_grid_ab.txt); PDT_NORM_BWD_WG overrides
  static const int cap = [] { const char* e = getenv("PDT_NORM_BWD_WG"); return e ? atoi(e) : 256; }();
  if (split_rows_ok(N)) {
    // one row per workgroup pass, 2 workgroups per CU resident: 512 partial rows (16 MB of fp32 partials at
    // N = 4,096 against ~540 MB of row traffic); PDT_NORM_SPLIT_WG overrides
    static const int scap = [] { const char* e = getenv("PDT_NORM_SPLIT_WG"); return e ? atoi(e) : 512; }();
    return grid_for(rows, 4, scap);
  }
  if (N % 8 == 0 && N <= 8192) return grid_for(rows, RPB * 4, cap);
  return grid_for(rows, 1, 512);
}

// workspace: fp32, >= (3 * bwd_partial_rows(rows, N) + 192) * N floats
template <typename T, typename W, bool RMS>
int launch_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, const void* dres,
               void* dx, void* dw, void* db, void* ds, float* ws, int rows, int N, int accumulate, hipStream_t st,
               WinMap wm = {}, void* dr_win = nullptr) {
  if (wm.mode != 0 && !small_rows(N)) return (int)hipErrorInvalidValue;
  if ((wm.mode & 2) && dr_win == nullptr) return (int)hipErrorInvalidValue;
  const T* DY = (const T*)dy; const T* X = (const T*)x; const W* Wt = (const W*)w; T* DX = (T*)dx;
  const T* DR = (const T*)dres;
  const int R = bwd_partial_rows(rows, N);
  float* dwp = ws;
  float* dbp = (db != nullptr) ? ws + (int64_t)R * N : nullptr;
  float* dsp = (ds != nullptr) ? ws + (int64_t)2 * R * N : nullptr;
  static const bool split_off = [] { const char* e = getenv("PDT_NORM_SPLIT"); return e && atoi(e) == 0; }();
  if (small_rows(N)) {
    norm_bwd_small<T, W, RMS><<<R, NT, 0, st>>>(DY, X, Wt, mean, rstd, DR, DX, dwp, dbp, dsp, rows, N, wm,
                                                 (T*)dr_win);
  } else if (split_rows_ok(N) && !split_off) {
    const int it = (N / RPB + 511) / 512;
#define PDT_NS2(I, D, S) \
  norm_bwd_split_kernel<T, W, I, RMS, D, S><<<R, NT, 0, st>>>(DY, X, Wt, mean, rstd, DR, DX, dwp, dbp, dsp, rows, N)
#define PDT_NS1(I, D) do { if (dsp) { PDT_NS2(I, D, true); } else { PDT_NS2(I, D, false); } } while (0)
#define PDT_NS(I) do { if (DR) { PDT_NS1(I, true); } else { PDT_NS1(I, false); } } while (0)
    if (it <= 2) PDT_NS(2);
    else if (it <= 4) PDT_NS(4);
    else PDT_NS(8);
#undef PDT_NS
#undef PDT_NS1
#undef PDT_NS2
  } else if (N % 8 == 0 && N <= 8192) {
    const int iters = (N + 511) / 512;
    const size_t lds = (dsp ? 3 : 2) * (size_t)N * sizeof(float);
    static const int occ2 = [] { const char* e = getenv("PDT_LN_BWD_OCC"); return e && atoi(e) == 2; }();
#define PDT_NB2(I, O, S)                                                                                                \
  if (DR) norm_bwd_kernel<T, W, I, RMS, true, O, S><<<R, NT, lds, st>>>(DY, X, Wt, mean, rstd, DR, DX, dwp, dbp, dsp, \
                                                                       rows, N);                                        \
  else norm_bwd_kernel<T, W, I, RMS, false, O, S><<<R, NT, lds, st>>>(DY, X, Wt, mean, rstd, DR, DX, dwp, dbp, dsp, rows, N)
#define PDT_NB1(I, O) \
  do { if (dsp) { PDT_NB2(I, O, true); } else { PDT_NB2(I, O, false); } } while (0)
#define PDT_NB(I) \
  do { if (occ2) { PDT_NB1(I, 2); } else { PDT_NB1(I, 1); } } while (0)
    if (iters <= 1) PDT_NB(1);
    else if (iters <= 2) PDT_NB(2);
    else if (iters <= 4) PDT_NB(4);
    else if (iters <= 8) PDT_NB(8);
    else PDT_NB(16);
#undef PDT_NB
#undef PDT_NB1
#undef PDT_NB2
  } else {
    norm_bwd_generic<T, W, RMS><<<R, NT, 0, st>>>(DY, X, Wt, mean, rstd, DR, DX, dwp, dbp, dsp, rows, N);
  }
  float* ws2 = ws + (int64_t)3 * R * N;
  // dgamma / dbeta / residual-bias partials sit at ws + z * R * N: reduced together (one launch per level)
  red::ColOuts3 outs{};
  int nz = 0;
  if (dw) { outs.out[nz] = dw; outs.accumulate[nz] = accumulate; ++nz; }
  if (db) { outs.out[nz] = db; outs.accumulate[nz] = accumulate; ++nz; }
  if (ds) { outs.out[nz] = ds; outs.accumulate[nz] = 0; ++nz; }
  const bool packed = (!db || dbp == ws + (int64_t)R * N) && (!ds || dsp == ws + (int64_t)(db ? 2 : 1) * R * N);
  if (packed && nz > 0) {
    red::col_reduce3<W>(ws, R, N, nz, outs, ws2, st);
  } else {
    if (dw) col_reduce<W>(dwp, R, N, (W*)dw, ws2, accumulate, st);
    if (db) col_reduce<W>(dbp, R, N, (W*)db, ws2 + (int64_t)64 * N, accumulate, st);
    if (ds) col_reduce<W>(dsp, R, N, (W*)ds, ws2 + (int64_t)128 * N, 0, st);
  }
  return (int)hipGetLastError();
}

}  // namespace

// dtype codes: x/y in {kF32, kBF16}; w/b in {kF32, kBF16}.  rms=1 selects RMSNorm (b ignored, mean unused).
// res/sum_out (nullable): fused residual -- sum_out = x + res is written and normalised.
// res_bias (nullable, w/b dtype, [N]): added with res (the bias of the Linear that produced res).
PDT_API int pdt_norm_fwd(const void* x, const void* res, const void* res_bias, void* sum_out, const void* w,
                         const void* b, void* y, float* mean, float* rstd, int rows, int N, float eps, int xdt, int wdt,
                         int rms, hipStream_t st) {
  if (res_bias && !res) return (int)hipErrorInvalidValue;
#define PDT_DISPATCH(R)                                                                                      \
  if (xdt == kBF16 && wdt == kBF16) return launch_fwd<bf16_t, bf16_t, R>(x, res, res_bias, sum_out, w, b, y, mean, rstd, rows, N, eps, st); \
  if (xdt == kBF16 && wdt == kF32) return launch_fwd<bf16_t, float, R>(x, res, res_bias, sum_out, w, b, y, mean, rstd, rows, N, eps, st);   \
  if (xdt == kF32 && wdt == kF32) return launch_fwd<float, float, R>(x, res, res_bias, sum_out, w, b, y, mean, rstd, rows, N, eps, st);     \
  if (xdt == kF32 && wdt == kBF16) return launch_fwd<float, bf16_t, R>(x, res, res_bias, sum_out, w, b, y, mean, rstd, rows, N, eps, st);
  if (rms) { PDT_DISPATCH(true) } else { PDT_DISPATCH(false) }
#undef PDT_DISPATCH
  return (int)hipErrorInvalidValue;
}

// The same with Swin's window permutation folded in (WinMap above; narrow rows, N <= 64): mode bit 0 = y written to
// window-order rows, bit 1 = res read from window-order rows.  rows = B * H * W image-order rows.
PDT_API int pdt_norm_fwd_win(const void* x, const void* res, void* sum_out, const void* w, const void* b, void* y,
                             float* mean, float* rstd, int rows, int N, float eps, int xdt, int wdt, int rms, int H,
                             int W_, int ws, int shift, int mode, hipStream_t st) {
  if (!small_rows(N) || ws <= 0 || H % ws || W_ % ws || shift < 0 || shift >= ws || rows % (H * W_) ||
      ((mode & 2) && (!res || !sum_out)))
    return (int)hipErrorInvalidValue;
  const WinMap wm{H, W_, ws, shift, mode};
#define PDT_DISPATCH(R)                                                                                                 \
  if (xdt == kBF16 && wdt == kBF16) return launch_fwd<bf16_t, bf16_t, R>(x, res, nullptr, sum_out, w, b, y, mean, rstd, rows, N, eps, st, wm); \
  if (xdt == kBF16 && wdt == kF32) return launch_fwd<bf16_t, float, R>(x, res, nullptr, sum_out, w, b, y, mean, rstd, rows, N, eps, st, wm);   \
  if (xdt == kF32 && wdt == kF32) return launch_fwd<float, float, R>(x, res, nullptr, sum_out, w, b, y, mean, rstd, rows, N, eps, st, wm);
  if (rms) { PDT_DISPATCH(true) } else { PDT_DISPATCH(false) }
#undef PDT_DISPATCH
  return (int)hipErrorInvalidValue;
}

// mode bit 0 = dy read from window-order rows; bit 1 = dr_win (window-order rows) also receives dx -- the gradient
// of a residual input the forward read through the map.
PDT_API int pdt_norm_bwd_win(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                             const void* dres, void* dx, void* dw, void* db, float* ws, int rows, int N, int xdt, int wdt,
                             int rms, int H, int W_, int wsz, int shift, int mode, void* dr_win, hipStream_t st) {
  if (!small_rows(N) || wsz <= 0 || H % wsz || W_ % wsz || shift < 0 || shift >= wsz || rows % (H * W_))
    return (int)hipErrorInvalidValue;
  const WinMap wm{H, W_, wsz, shift, mode};
#define PDT_DISPATCH(R)                                                                                                 \
  if (xdt == kBF16 && wdt == kBF16) return launch_bwd<bf16_t, bf16_t, R>(dy, x, w, mean, rstd, dres, dx, dw, db, nullptr, ws, rows, N, 0, st, wm, dr_win); \
  if (xdt == kBF16 && wdt == kF32) return launch_bwd<bf16_t, float, R>(dy, x, w, mean, rstd, dres, dx, dw, db, nullptr, ws, rows, N, 0, st, wm, dr_win);   \
  if (xdt == kF32 && wdt == kF32) return launch_bwd<float, float, R>(dy, x, w, mean, rstd, dres, dx, dw, db, nullptr, ws, rows, N, 0, st, wm, dr_win);
  if (rms) { PDT_DISPATCH(true) } else { PDT_DISPATCH(false) }
#undef PDT_DISPATCH
  return (int)hipErrorInvalidValue;
}

PDT_API int pdt_norm_bwd_workspace_floats(int rows, int N) { return (3 * bwd_partial_rows(rows, N) + 192) * N; }

// dres (nullable): gradient arriving at the fused residual sum, added into dx.
// ds (nullable, w dtype, [N]): column sums of dx -- the gradient of norm_fwd's res_bias (never accumulated).
PDT_API int pdt_norm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                         const void* dres, void* dx, void* dw, void* db, void* ds, float* ws, int rows, int N, int xdt,
                         int wdt, int rms, int accumulate, hipStream_t st) {
#define PDT_DISPATCH(R)                                                                                         \
  if (xdt == kBF16 && wdt == kBF16) return launch_bwd<bf16_t, bf16_t, R>(dy, x, w, mean, rstd, dres, dx, dw, db, ds, ws, rows, N, accumulate, st); \
  if (xdt == kBF16 && wdt == kF32) return launch_bwd<bf16_t, float, R>(dy, x, w, mean, rstd, dres, dx, dw, db, ds, ws, rows, N, accumulate, st);   \
  if (xdt == kF32 && wdt == kF32) return launch_bwd<float, float, R>(dy, x, w, mean, rstd, dres, dx, dw, db, ds, ws, rows, N, accumulate, st);     \
  if (xdt == kF32 && wdt == kBF16) return launch_bwd<float, bf16_t, R>(dy, x, w, mean, rstd, dres, dx, dw, db, ds, ws, rows, N, accumulate, st);
  if (rms) { PDT_DISPATCH(true) } else { PDT_DISPATCH(false) }
#undef PDT_DISPATCH
  return (int)hipErrorInvalidValue;
}

// Column sums of a [rows, N] matrix (T) into out[N] (W) -- bias gradients.  Workspace:
// pdt_colsum_ws_floats(rows, N) floats (reduce.h col_plan partials + second level).
namespace {
// narrow N (< VEC * NT): rows packed NT / (N / VEC) per workgroup pass, one partial row per workgroup.
// VEC = 8 (16-B bf16 loads) when N % 8 == 0, else 4 (SwinIR's C = 60 / 180 bias gradients).
template <typename T, int VEC>
__device__ __forceinline__ void load_vec(const T* p, float* v) {
  if constexpr (VEC == 8) {
    Vec8<T>::load(p, v);
  } else if constexpr (sizeof(T) == 2) {
    const u16x4 a = *reinterpret_cast<const u16x4*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = bf2f(a[k]);
  } else {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = a[k];
  }
}
template <typename T, int VEC>
__global__ __launch_bounds__(NT) void colsum_partial_narrow(const T* __restrict__ x, int rows, int N, int rows_per,
                                                            float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float sacc[NT * VEC];
  const int tpr = N / VEC, rpb = NT / tpr;
  const int rg = threadIdx.x / tpr, col = (threadIdx.x - rg * tpr) * VEC;
  float acc[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
  const int r0 = blockIdx.x * rows_per, r1 = min(rows, r0 + rows_per);
  if (rg < rpb) {
    for (int r = r0 + rg; r < r1; r += rpb) {
      float v[VEC];
      load_vec<T, VEC>(x + (int64_t)r * N + col, v);
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += v[k];
    }
  }
#pragma unroll
  for (int k = 0; k < VEC; ++k) sacc[threadIdx.x * VEC + k] = acc[k];
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += NT) {
    const int cv = c / VEC, k = c % VEC;
    float t = 0.f;
    for (int g = 0; g < rpb; ++g) t += sacc[(g * tpr + cv) * VEC + k];
    part[(int64_t)blockIdx.x * N + c] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void colsum_partial_kernel(const T* __restrict__ x, int rows, int N, int rows_per,
                                                            float* __restrict__ part) {
  // blockIdx.x = 2048-column group (256 threads x 8 columns), blockIdx.y = row chunk
  const int col = (blockIdx.x * NT + threadIdx.x) * 8;
  if (col >= N) return;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(rows, r0 + rows_per);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int r = r0;
  for (; r + 4 <= r1; r += 4) {   // 4 independent 16-B loads in flight per thread
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) Vec8<T>::load(x + (int64_t)(r + u) * N + col, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[u][k];
  }
  for (; r < r1; ++r) {
    float v[8];
    Vec8<T>::load(x + (int64_t)r * N + col, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += v[k];
  }
  Vec8<float>::store(part + (int64_t)blockIdx.y * N + col, acc);
}
}  // namespace

PDT_API int pdt_colsum_ws_floats(int rows, int N) { return (int)red::col_ws_floats(rows, N); }

PDT_API int pdt_colsum(const void* x, int rows, int N, int xdt, void* out, int odt, float* ws, int accumulate,
                       hipStream_t st) {
  if (N % 8 != 0 && !(N % 4 == 0 && N < 4 * NT)) return (int)hipErrorInvalidValue;
  const red::ColPlan pl = red::col_plan(rows, N);
  dim3 grid(pl.col_groups, pl.R);
  if (N % 8 != 0) {
    if (xdt == kBF16) colsum_partial_narrow<bf16_t, 4><<<pl.R, NT, 0, st>>>((const bf16_t*)x, rows, N, pl.rows_per, ws);
    else colsum_partial_narrow<float, 4><<<pl.R, NT, 0, st>>>((const float*)x, rows, N, pl.rows_per, ws);
  } else if (N < 8 * NT) {
    if (xdt == kBF16) colsum_partial_narrow<bf16_t, 8><<<pl.R, NT, 0, st>>>((const bf16_t*)x, rows, N, pl.rows_per, ws);
    else colsum_partial_narrow<float, 8><<<pl.R, NT, 0, st>>>((const float*)x, rows, N, pl.rows_per, ws);
  } else if (xdt == kBF16) {
    colsum_partial_kernel<bf16_t><<<grid, NT, 0, st>>>((const bf16_t*)x, rows, N, pl.rows_per, ws);
  } else {
    colsum_partial_kernel<float><<<grid, NT, 0, st>>>((const float*)x, rows, N, pl.rows_per, ws);
  }
  float* ws2 = ws + (int64_t)pl.R * N;
  if (odt == kBF16) red::col_reduce<bf16_t>(ws, pl.R, N, (bf16_t*)out, ws2, accumulate, st);
  else red::col_reduce<float>(ws, pl.R, N, (float*)out, ws2, accumulate, st);
  return (int)hipGetLastError();
}
