// bf16 GEMM family for gfx950 with fused epilogues: C[M, N] = sum_k A(m, k) B(k, n), fp32 accumulate.
//
//   layout NT : A[m * lda + k], B[n * ldb + k]  -- Linear forward x W^T, and dgrad dY (W^T)^T with the
//               weight transposed once (ops.linear: hipBLASLt's NN kernels ran 10-25 % below NT there)
//   layout TT : A[k * lda + m], B[k * ldb + n]  -- weight gradient dW = dY^T X (both token-major)
//
// Epilogues (the reason this kernel exists next to hipBLASLt, whose GELU_AUX_BIAS / DGELU_BGRAD epilogues
// are unsupported on gfx950, profiles/r2_hipblaslt_epilogue_probe.txt):
//   PLAIN   C = bf16(acc)                         BIAS   C = bf16(acc + bias[n])
//   GELU    pre = acc + bias[n] -> aux_out (bf16), C = gelu_tanh(pre)   (GPT-2 c_fc: one pass, no bias_gelu)
//   DGELU   g = acc * gelu_tanh'(aux[m, n]) -> C, per-tile column sums of g -> ws (fp32) -> dbias
//           (GPT-2 c_proj dgrad + GELU backward + bias gradient of c_fc: no bias_gelu_bwd_db pass)
//   F32     fp32 split-K partial slab (reduced by splitk_reduce_kernel)
//
// Main loop (cdna_hip_programming.md §5): 256 x 256 output tile per 512-thread workgroup, 8 waves as
// 2 (m) x 4 (n), each wave 128 x 64 = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (the 16x16 shape holds a
// higher clock under load than 32x32x16 at equal cycles per FLOP, MI355X_MICROARCH.md DVFS item 7).
// K advances 32 per step through a 4-stage LDS ring (4 x 32 KiB) filled by LDS-DMA
// (buffer_load_dwordx4 ... lds, issued from inline asm so hipcc's waitcnt pass cannot drain it); a tile is
// issued 3 steps before it is consumed, each step waits only for the NEXT tile with a counted vmcnt and
// one raw barrier, and the next tile's fragments are read during the current tile's MFMAs -- no
// ds_read -> MFMA bubble at the step boundary.
//
// LDS images (16-B chunk XOR swizzles applied to the DMA SOURCE address, rule 21):
//   NT operand: [256 rows][32 k] (64-B rows), chunk ^= ((row >> 3) & 1) << 1: the 16x16x32 fragment read
//               (ds_read_b128, rows r..r+15, chunk = lane >> 4) hits 16 distinct 16-B bank slots per group.
//   TT operand: [32 k][256 cols] (512-B rows), chunk ^= 2 * ((row & 3) | ((row >> 1) & 4)): the transposed
//               fragment read (ds_read_b64_tr_b16, rows 8g+q, 16 columns) hits 8 distinct 32-B slots per half.
//
// The MFMA runs with the B fragment as its first operand: the accumulator is C^T, so each lane holds 4
// consecutive columns n of one row m and the epilogue stores 8 (bf16) or 16 (fp32) bytes per lane.
#include "common.h"
#include "gelu.h"
#include <stdlib.h>
#include <type_traits>

using namespace pdt;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((address_space(3))) u16x8 lds_u16x8;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int TM = 256, TN = 256, KB = 64, NTH = 512;
constexpr int OPB = TM * KB * 2;           // bytes of one operand tile of one K-step (32 KiB)
constexpr int STB = 2 * OPB;               // one ring slot: A tile then B tile (2 slots = 128 KiB)
constexpr int PIECES = OPB / (NTH * 16);   // LDS-DMA instructions per thread per operand per K-step (4)

enum { L_NT = 0, L_TT = 1 };
enum { E_PLAIN = 0, E_BIAS = 1, E_GELU = 2, E_DGELU = 3, E_F32 = 4 };

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

// TT image swizzle: 16-B chunk c of k-row r is stored at chunk c ^ tt_f(r)
__device__ __forceinline__ int tt_f(int r) { return 2 * ((r & 3) | ((r >> 1) & 4)); }

// One operand's LDS-DMA: per-lane source byte offsets (relative to the K-step's tile origin) of this
// thread's PIECES wave-instructions (1 KiB each, lane-linear LDS destination, swizzle on the source).
template <int LAYOUT>
struct Dma {
  uint32_t off[PIECES];
  __device__ __forceinline__ void init(int64_t ld, int w, int lane) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const int q = i * 8 + w;   // 1-KiB piece index within the operand tile (0..31)
      int row, c;
      if (LAYOUT == L_NT) {      // 8 rows x 128 B per piece; chunk ^= (row >> 1) & 7
        row = 8 * q + (lane >> 3);
        c = (lane & 7) ^ ((row >> 1) & 7);
      } else {                   // 2 k-rows x 512 B per piece
        row = 2 * q + (lane >> 5);
        c = (lane & 31) ^ tt_f(row);
      }
      off[i] = (uint32_t)(row * ld * 2 + c * 16);
    }
  }
  // pieces [i0, i1) of the tile at byte address `tile` (wave-uniform) into the LDS tile `lds_op`
  template <int I0, int I1>
  __device__ __forceinline__ void issue(const char* tile, uint32_t nbytes, const char* lds_op, int w) const {
    const uint64_t addr = (uint64_t)(uintptr_t)tile;
    v4i rsrc;
    rsrc[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)addr);
    rsrc[1] = __builtin_amdgcn_readfirstlane((int)((addr >> 32) & 0xffff));
    rsrc[2] = __builtin_amdgcn_readfirstlane((int)nbytes);
    rsrc[3] = 0x00020000;
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(lds_void*)(lds_op + (i * 8 + w) * 1024));
      asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
                   :: "s"(m0), "v"(off[i]), "s"(rsrc) : "memory");
    }
  }
};

// Fragment of 16 rows (NT: rows of the operand tile; TT: columns) x 32 k (k-substep s of the 64-deep
// K-step) for the 16x16x32 MFMA: lane l gets row/col (l & 15), k = 32 s + 8 (l >> 4) + e, e = 0..7.
template <int LAYOUT>
struct Frag {
  uint32_t o0, o1;   // NT: byte offsets of block 0 for s = 0 / 1;  TT: row offset, swizzle term
  __device__ __forceinline__ void init(int lane) {
    const int x = lane & 15, g = lane >> 4;
    if (LAYOUT == L_NT) {
      const int h = (x >> 1) & 7;
      o0 = (uint32_t)(x * 128 + 16 * (g ^ h));
      o1 = (uint32_t)(x * 128 + 16 * ((4 + g) ^ h));
    } else {
      const int q = (lane >> 2) & 3, p = lane & 3;
      o0 = (uint32_t)((8 * g + q) * 512 + 16 * (p >> 1) + 8 * (p & 1));
      o1 = (uint32_t)tt_f(8 * g + q);
    }
  }
  template <int S>
  __device__ __forceinline__ u16x8 read(const char* op, int blk) const {
    if (LAYOUT == L_NT) {
      return *(const lds_u16x8*)(lds_void*)(op + blk * 16 * 128 + (S ? o1 : o0));
    } else {
      const uint32_t a = o0 + S * 32 * 512 + 16 * ((uint32_t)(2 * blk) ^ o1);
      const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds_void*)(op + a));
      const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds_void*)(op + a + 2048));
      return __builtin_bit_cast(u16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const bf16_t* bias;     // E_BIAS / E_GELU: [N]
  const bf16_t* aux;      // E_DGELU: pre-activation [M, ldc]
  bf16_t* aux_out;        // E_GELU: pre-activation out [M, ldc]
  float* ws;              // E_F32: slabs [splits][M][N]; E_DGELU: column partials [M / 256][N]
  int M, N, K;
  int64_t lda, ldb, ldc;
  int k_per_split;
  int xpr;                // XCD block cut (see tile_of)
};

__device__ __forceinline__ void tile_of(const GemmArgs& p, int& tm, int& tn) {
  // XCD-aware tile order (speed only): workgroups b and b + 8 share an XCD under round-robin dispatch.
  // xpr > 0: the tile grid is cut into xpr x (8 / xpr) blocks, one per XCD (host picks the cut that
  // minimises the A + B panels an XCD's L2 holds); else each XCD takes a contiguous run of tiles.
  const int mt = p.M / TM, nt = p.N / TN, ntiles = gridDim.x;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  if (p.xpr > 0) {
    const int xpc = 8 / p.xpr, rb = mt / p.xpr, cb = nt / xpc;
    tm = (xcd / xpc) * rb + loc / cb;
    tn = (xcd % xpc) * cb + loc % cb;
  } else {
    const int q8 = ntiles >> 3, r8 = ntiles & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    tm = t / nt;
    tn = t % nt;
  }
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Main-loop schedule (per K-step of 64, 2-slot LDS ring, 8 waves as two groups of four: g = wave >> 2,
// one wave of each group per SIMD).  A wave's 128 x 64 output is cut into four quadrants of 64 x 32
// (16 MFMAs each: 4 m-blocks x 2 n-blocks x 2 k-substeps); every quadrant is one PHASE = {R: its
// fragment reads (+ DMA pieces of the next K-step), barrier, M: its 16 MFMAs, barrier}.  Group 1 runs
// one barrier behind group 0, so in every barrier interval one wave of each SIMD is in M while its
// partner is in R: the matrix pipe never waits for the fragment reads (cdna_hip_programming.md §5,
// the 8-phase template's stagger).  Quadrant order (A0,B0) (A0,B1) (A1,B1) (A1,B0) re-reads only one
// operand per phase.
//   DMA of K-step t+1 into the other slot: phases 1 and 2 of step t (a slot is free once both groups'
//   phase-3 reads of step t-1 have been waited for, which every wave does before the first barrier of
//   step t's phase 1); each wave drains its own pieces (vmcnt(0)) before the barrier that precedes the
//   first read of step t+1 -- group 0 after M of phase 3, group 1 after R of phase 3.
template <int LAYOUT, int EPI>
__global__ __launch_bounds__(NTH, 1) void gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STB];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wr = w >> 2, wc = w & 3;
  int tm, tn;
  tile_of(p, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int T = min(p.K - kbeg, p.k_per_split) / KB;

  Dma<LAYOUT> da, db;
  da.init(p.lda, w, lane);
  db.init(p.ldb, w, lane);
  Frag<LAYOUT> fr;
  fr.init(lane);
  const char* Ab = reinterpret_cast<const char*>(p.A);
  const char* Bb = reinterpret_cast<const char*>(p.B);
  int64_t a0, b0, astep, bstep;
  uint32_t abytes, bbytes;
  if (LAYOUT == L_NT) {
    a0 = ((int64_t)m0 * p.lda + kbeg) * 2; b0 = ((int64_t)n0 * p.ldb + kbeg) * 2;
    astep = bstep = KB * 2;
    abytes = (uint32_t)((TM - 1) * p.lda * 2 + KB * 2); bbytes = (uint32_t)((TN - 1) * p.ldb * 2 + KB * 2);
  } else {
    a0 = ((int64_t)kbeg * p.lda + m0) * 2; b0 = ((int64_t)kbeg * p.ldb + n0) * 2;
    astep = KB * p.lda * 2; bstep = KB * p.ldb * 2;
    abytes = (uint32_t)((KB - 1) * p.lda * 2 + TM * 2); bbytes = (uint32_t)((KB - 1) * p.ldb * 2 + TN * 2);
  }
  // pieces [I0, I1) of both operands of K-step t into slot t & 1
  auto issue_a = [&](auto i0, auto i1, int t) {
    da.template issue<decltype(i0)::value, decltype(i1)::value>(Ab + a0 + t * astep, abytes, smem + (t & 1) * STB, w);
  };
  auto issue_b = [&](auto i0, auto i1, int t) {
    db.template issue<decltype(i0)::value, decltype(i1)::value>(Bb + b0 + t * bstep, bbytes,
                                                                smem + (t & 1) * STB + OPB, w);
  };
  using I0 = std::integral_constant<int, 0>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 fa[4][2], fb[2][2];   // the current phase's fragments: 4 m-blocks / 2 n-blocks x 2 k-substeps

  // prologue: K-step 0 in flight, landed and visible; group 1 falls one barrier behind
  issue_a(I0{}, I4{}, 0);
  issue_b(I0{}, I4{}, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
  if (__builtin_amdgcn_readfirstlane(wr) == 1) bar();

  // phase body: R (reads of this quadrant + DMA), barrier, M (16 MFMAs), barrier
  for (int t = 0; t < T; ++t) {
    const char* sa = smem + (t & 1) * STB;
    const char* sb = sa + OPB;
    const bool more = t + 1 < T;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mh = (q == 0 || q == 1) ? 0 : 1;
      const int nh = (q == 0 || q == 3) ? 0 : 1;
      // ---- R
      if (q == 0 || q == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          fa[i][0] = fr.template read<0>(sa, 8 * wr + 4 * mh + i);
          fa[i][1] = fr.template read<1>(sa, 8 * wr + 4 * mh + i);
        }
      }
      if (q != 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          fb[j][0] = fr.template read<0>(sb, 4 * wc + 2 * nh + j);
          fb[j][1] = fr.template read<1>(sb, 4 * wc + 2 * nh + j);
        }
      }
      if (more) {
        if (q == 1) { issue_a(I0{}, I4{}, t + 1); }
        if (q == 2) { issue_b(I0{}, I4{}, t + 1); }
      }
      if (q == 3 && __builtin_amdgcn_readfirstlane(wr) == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      // ---- M
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[4 * mh + i][2 * nh + j] = mfma16(fb[j][s], fa[i][s], acc[4 * mh + i][2 * nh + j]);
      __builtin_amdgcn_s_setprio(0);
      if (q == 3 && __builtin_amdgcn_readfirstlane(wr) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
  }
  if (__builtin_amdgcn_readfirstlane(wr) == 0) bar();   // group 0 catches up: equal barrier counts

  // ---------------------------------------------------------------- epilogue
  // acc[i][j][r] = C[m0 + 128 wr + 16 i + (lane & 15)][n0 + 64 wc + 16 j + 4 (lane >> 4) + r]
  const int mrow = m0 + 128 * wr + (lane & 15);
  const int ncol = n0 + 64 * wc + 4 * (lane >> 4);
  if constexpr (EPI == E_F32) {
    float* C = p.ws + (int64_t)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<f32x4*>(C + (int64_t)(mrow + 16 * i) * p.N + ncol + 16 * j) = acc[i][j];
    return;
  } else {
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
    float bj[4][4];
    if constexpr (EPI == E_BIAS || EPI == E_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u16x4 b = *reinterpret_cast<const u16x4*>(p.bias + ncol + 16 * j);
#pragma unroll
        for (int r = 0; r < 4; ++r) bj[j][r] = bf2f(b[r]);
      }
    }
    float cs[4][4];   // E_DGELU: this lane's column sums over its 8 rows
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t rowoff = (int64_t)(mrow + 16 * i) * p.ldc;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t e = rowoff + ncol + 16 * j;
        u16x4 o;
        if constexpr (EPI == E_PLAIN) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        } else if constexpr (EPI == E_BIAS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bj[j][r]);
        } else if constexpr (EPI == E_GELU) {
          u16x4 pre;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bf16_t h = f2bf(acc[i][j][r] + bj[j][r]);
            pre[r] = h;
            o[r] = f2bf(gelu_f<true>(bf2f(h)));   // GELU of the stored (rounded) pre-activation
          }
          *reinterpret_cast<u16x4*>(p.aux_out + e) = pre;
        } else {   // E_DGELU
          const u16x4 h = *reinterpret_cast<const u16x4*>(p.aux + e);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float g = acc[i][j][r] * gelu_grad<true>(bf2f(h[r]));
            const bf16_t gb = f2bf(g);
            o[r] = gb;
            cs[j][r] += bf2f(gb);   // the bias gradient sums the gradient as stored
          }
        }
        *reinterpret_cast<u16x4*>(C + e) = o;
      }
    }
    if constexpr (EPI == E_DGELU) {
      // sum over the 16 lanes that share (lane >> 4) (rows), then over the two wave rows through LDS;
      // one fp32 partial per column per 256-row tile (deterministic; reduced by colpart_reduce_kernel)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = cs[j][r];
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          cs[j][r] = v;
        }
      __syncthreads();                                   // the ring is no longer read: reuse its LDS
      float* red = reinterpret_cast<float*>(smem);       // [2 wave rows][256 columns]
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[wr * 256 + 64 * wc + 16 * j + 4 * (lane >> 4) + r] = cs[j][r];
      }
      __syncthreads();
      if (tid < 256) p.ws[(int64_t)tm * p.N + n0 + tid] = red[tid] + red[256 + tid];
    }
  }
}

// out[e] = sum over S slices of part[s][e] (fp32 slabs) -> bf16, 4 elements per thread
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(const float* __restrict__ part,
                                                                 bf16_t* __restrict__ out, int64_t n4, int S,
                                                                 int64_t slab) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
    f32x4 s = reinterpret_cast<const f32x4*>(part)[e];
    for (int k = 1; k < S; ++k) s += reinterpret_cast<const f32x4*>(part + k * slab)[e];
    u16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = f2bf(s[r]);
    reinterpret_cast<u16x4*>(out)[e] = o;
  }
}

// dbias[n] = sum over R row tiles of part[r][n] (fixed order: deterministic)
__global__ __launch_bounds__(256) void colpart_reduce_kernel(const float* __restrict__ part, int R, int N,
                                                             bf16_t* __restrict__ out) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += part[(int64_t)r * N + n];
  out[n] = f2bf(s);
}

int xcd_cut(int mt, int nt) {
  int xpr = 0, best = 1 << 30;
  for (int pr = 1; pr <= 8; pr *= 2) {
    const int pc = 8 / pr;
    if (mt % pr || nt % pc) continue;
    const int cost = mt / pr + nt / pc;
    if (cost < best) { best = cost; xpr = pr; }
  }
  return xpr;
}

template <int LAYOUT>
int launch_layout(int epi, const GemmArgs& a, int splits, hipStream_t s) {
  const dim3 grid((a.M / TM) * (a.N / TN), splits);
  switch (epi) {
    case E_PLAIN: gemm_kernel<LAYOUT, E_PLAIN><<<grid, NTH, 0, s>>>(a); break;
    case E_BIAS: gemm_kernel<LAYOUT, E_BIAS><<<grid, NTH, 0, s>>>(a); break;
    case E_GELU: gemm_kernel<LAYOUT, E_GELU><<<grid, NTH, 0, s>>>(a); break;
    case E_DGELU: gemm_kernel<LAYOUT, E_DGELU><<<grid, NTH, 0, s>>>(a); break;
    case E_F32: gemm_kernel<LAYOUT, E_F32><<<grid, NTH, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

// Shapes the kernel takes (checked by the host before any launch): M, N multiples of 256, K a multiple of
// 32 * splits, 16-B aligned rows, every byte offset of a stage tile below 2^32 (buffer resources).
PDT_API int pdt_gemm_ok(int layout, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int splits) {
  if (layout != L_NT && layout != L_TT) return 0;
  if (splits < 1 || M <= 0 || N <= 0 || K <= 0 || M % TM || N % TN || K % ((int64_t)KB * splits)) return 0;
  if ((M / TM) * (N / TN) > (1LL << 24) || lda % 8 || ldb % 8) return 0;
  if (layout == L_NT && (lda < K || ldb < K || (TM - 1) * lda * 2 + KB * 2 >= (1LL << 32) ||
                         (TN - 1) * ldb * 2 + KB * 2 >= (1LL << 32)))
    return 0;
  if (layout == L_TT && (lda < M || ldb < N || (KB - 1) * lda * 2 + TM * 2 >= (1LL << 32) ||
                         (KB - 1) * ldb * 2 + TN * 2 >= (1LL << 32)))
    return 0;
  return M <= (1LL << 30) && N <= (1LL << 30) && K <= (1LL << 30) ? 1 : 0;
}

// Fused-epilogue GEMM.  epi: 0 plain, 1 bias, 2 bias+GELU (aux_out = pre-activation), 3 dGELU (aux = the
// pre-activation, dbias = column sums of the result; ws >= (M / 256) * N floats), 4 is internal.
// splits > 1 (plain only): fp32 slabs in ws (splits * M * N floats) + a reduce pass.
PDT_API int pdt_gemm_bf16(int layout, int epi, const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K,
                          int64_t lda, int64_t ldb, int64_t ldc, const void* bias, const void* aux, void* aux_out,
                          void* dbias, float* ws, int splits, hipStream_t s) {
  if (!pdt_gemm_ok(layout, M, N, K, lda, ldb, splits) || ldc < N || ldc % 4) return (int)hipErrorInvalidValue;
  if (epi < 0 || epi > E_DGELU) return (int)hipErrorInvalidValue;
  if (splits > 1 && (epi != E_PLAIN || !ws)) return (int)hipErrorInvalidValue;
  if ((epi == E_BIAS || epi == E_GELU) && !bias) return (int)hipErrorInvalidValue;
  if (epi == E_GELU && !aux_out) return (int)hipErrorInvalidValue;
  if (epi == E_DGELU && (!aux || !ws || !dbias)) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C;
  a.bias = (const bf16_t*)bias; a.aux = (const bf16_t*)aux; a.aux_out = (bf16_t*)aux_out; a.ws = ws;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.k_per_split = (int)(K / splits);
  a.xpr = xcd_cut((int)(M / TM), (int)(N / TN));
  const int run_epi = splits > 1 ? E_F32 : epi;
  if (splits > 1) a.ldc = N;
  int err = layout == L_NT ? launch_layout<L_NT>(run_epi, a, splits, s) : launch_layout<L_TT>(run_epi, a, splits, s);
  if (err) return err;
  if (splits > 1) {
    const int64_t n4 = M * N / 4;
    gemm_splitk_reduce_kernel<<<grid_for(n4, 256, 256 * 16), 256, 0, s>>>(ws, (bf16_t*)C, n4, splits, M * N);
    if (ldc != N) return (int)hipErrorInvalidValue;   // slab reduce writes a dense [M, N]
  }
  if (epi == E_DGELU) {
    colpart_reduce_kernel<<<(int)((N + 255) / 256), 256, 0, s>>>(ws, (int)(M / TM), (int)N, (bf16_t*)dbias);
  }
  return (int)hipGetLastError();
}
