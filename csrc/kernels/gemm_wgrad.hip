// Weight-gradient GEMM for gfx950: C[Nr, Nc] = sum_m A[m, Nr] * B[m, Nc]  (dW = dY^T X), bf16 in,
// fp32 accumulate, bf16 out (or fp32 split-K partials).
//
// Why a hand kernel: both operands of a weight gradient are stored reduction-major (the token index m is
// the ROW of dY [M, N] and of X [M, K]), the layout hipBLASLt runs ~25 % below its forward GEMMs on the
// GPT-2 1.3B / Llama shapes (1.0-1.15 vs 1.45-1.55 PFLOP/s, profiles/r2_gpt2_1.3b_fsdp1_mb64_kernel_stats.csv).
// On MFMA the layout costs nothing: the LDS tile is filled row-major straight from HBM and BOTH fragments
// are read transposed with ds_read_b64_tr_b16 -- the idiom of the attention kernel's V^T operand
// (flash_attn.hip): a lane gets one column (an output row n / output column k) and 8 token rows.  A and B
// use the same token permutation inside each 16-deep step, so the sum is exact.
//
// Structure (cdna_hip_programming.md §5, 256^2 tile): 512 threads = 8 waves as 2 (rows) x 4 (cols), each
// wave a 128 x 64 output block = 4 x 2 v_mfma_f32_32x32x16_bf16 tiles (128 accumulators); BK = 64 tokens
// per K-step; K/V-style LDS-DMA (global_load_lds_dwordx4) into a 2-stage ring (2 x 64 KiB), ONE barrier per
// K-step that retires the stage (explicit vmcnt(0): a workgroup barrier does not wait for LDS-DMA loads),
// the next stage's DMA issued right after it; fragment reads one 16-deep step ahead of their MFMAs, each
// in a scheduling region of its own.  LDS rows are 512 B; a 16-B-chunk XOR swizzle (chunk ^= (row & 3) << 2,
// applied to the DMA source address, rule 21) makes the transposed reads conflict-free (4 rows x 64 B per
// 32-lane group land on 4 distinct 64-B bank groups).  Split-K over the tokens (fp32 partial slabs + a
// reduce pass) keeps >= 256 workgroups for small outputs (GPT-2 1.3B attention projection: 64 tiles).
#include "common.h"
#include <stdlib.h>

using namespace pdt;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BR = 256, BC = 256;
constexpr int BK = 64;                        // token granularity every split / M must respect

__device__ __forceinline__ f32x16 mfma32(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// Accumulate into an AGPR-resident tile (the 4-wave variant's 256 accumulators do not fit beside the
// fragments in the 256 arch VGPRs).  acc_fence() before any VALU read: the hazard recognizer does not
// see through inline asm.
__device__ __forceinline__ void mfma32_acc(f32x16& acc, const u16x8& a, const u16x8& b) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void acc_fence() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"); }

// 16-B chunk swizzle of a 512-B LDS row (32 chunks)
__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r & 3) << 2); }

// LDS-DMA of one 64 x 256 operand tile (rows m0.., columns c0..) of a row-major [M, ld] matrix: 2048 chunks
// of 16 B, 4 per thread (piece i = 0..3); a wave-instruction fills 64 consecutive LDS chunks (two 512-B
// rows), each lane's SOURCE chunk pre-swizzled so LDS chunk c of row r holds logical chunk swz(r, c).
// Issued as `buffer_load_dwordx4 ... offen lds` through a buffer resource whose base is the tile's first
// element (T8): per K-step only the SGPR descriptor moves, the per-lane byte offsets are computed once.
// (global_load_lds through a plain pointer made hipcc wait vmcnt(0) before the first LDS read after it --
// it cannot tell the DMA target stage from the stage being read -- which serialised every prefetch.)
template <int BKT, int NTH>
struct DmaOp {
  static constexpr int NP = BKT * 32 / NTH;   // 16-B chunks per thread per operand tile (BKT rows x 512 B)
  uint32_t off[NP];
  __device__ __forceinline__ void init(int64_t ld, int tid) {
    const int w = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int ci = i * NTH + w * 64 + lane;
      const int r = ci >> 5, c = ci & 31;
      off[i] = (uint32_t)((r * ld + swz(r, c) * 8) * 2);
    }
  }
  // Issued from inline asm: for a builtin LDS-DMA, hipcc's waitcnt pass cannot tell the target stage from the
  // stage being read and drains the whole prefetch (vmcnt(0)) before the next ds_read -- which serialised
  // every K-step.  Hidden from it, the DMA is ordered only by the K-loop's explicit counted vmcnt + barrier.
  __device__ __forceinline__ void piece(const bf16_t* tile0, int64_t ld, bf16_t* lds, int tid, int i) const {
    typedef int v4i __attribute__((ext_vector_type(4)));
    const uint64_t addr = (uint64_t)(uintptr_t)tile0;
    v4i rsrc;
    rsrc[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)addr);
    rsrc[1] = __builtin_amdgcn_readfirstlane((int)((addr >> 32) & 0xffff));
    rsrc[2] = __builtin_amdgcn_readfirstlane((int)((BKT - 1) * ld * 2 + 512));   // num_records (bytes)
    rsrc[3] = 0x00020000;
    const int w = tid >> 6;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(lds_void*)(lds + (i * NTH + w * 64) * 8));
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
                 :: "s"(m0), "v"(off[i]), "s"(rsrc) : "memory");   // m0: reserved, never allocated
  }
};

// s_waitcnt vmcnt(n) for the few counts the ring uses (the count must be an immediate)
__device__ __forceinline__ void wait_vm(int n) {
  if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Transposed fragment: lane l gets column (col0 + (l & 31)) of token rows {kb + 4h + j} (j < 4) and
// {kb + 8 + 4h + j - 4} (j >= 4), h = l >> 5 -- the 32x32x16 operand layout with the permuted k order.
struct FragAddr {
  int o1, o2;   // element offsets of the two 8-byte reads for col0 = 0, kb = 0
};
__device__ __forceinline__ FragAddr frag_addr(int lane, int col0, int kb) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int r1 = kb + 4 * (g >> 1) + q, r2 = r1 + 8;
  FragAddr a;
  a.o1 = r1 * 256 + swz(r1, col >> 3) * 8 + (col & 7);
  a.o2 = r2 * 256 + swz(r2, col >> 3) * 8 + (col & 7);
  return a;
}
__device__ __forceinline__ u16x8 frag(const bf16_t* lds, const FragAddr& a) {
  const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds + a.o1));
  const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(lds + a.o2));
  return __builtin_bit_cast(u16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
}

// grid.x = row tiles * col tiles (XCD-aware order), grid.y = split-K slices.
// BKT tokens per K-step, NST ring stages: the DMA of stage t + NST - 1 is issued in K-step t, so a stage has
// NST - 1 K-steps to land; the barrier of K-step t waits only for stage t (counted vmcnt: the younger
// stages' pieces may stay in flight across it).
// OPT bit 0: s_setprio 1 around each step's MFMAs; bit 1: plain (non-XCD-aware) tile order.
// NTH = 512: 8 waves as 2 x 4, each a 128 x 64 block (4 x 2 MFMA tiles, 2 waves per SIMD);
// NTH = 256: 4 waves as 2 x 2, each a 128 x 128 block (4 x 4 MFMA tiles, 256 accumulators, 1 wave per SIMD).
template <bool PARTIAL, int BKT, int NST, int OPT, int NTH>
__global__ __launch_bounds__(NTH, 1) void wgrad_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                       void* __restrict__ C, int M, int Nr, int Nc, int m_per_split,
                                                       int xpr) {
  constexpr int TILE_ELEMS = BKT * 256, STAGE = 2 * TILE_ELEMS, KS = BKT / 16;
  constexpr int P = 2 * DmaOp<BKT, NTH>::NP;                         // DMA instructions per stage per thread
  constexpr int WN = NTH == 512 ? 4 : 2, JB = NTH == 512 ? 2 : 4;    // wave columns, 32-col blocks per wave
  static_assert(NST * STAGE * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NST * STAGE];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane >> 5;
  const int wr = w / WN, wc = w % WN;                              // wave: rows 128*wr.., cols 32*JB*wc..
  // XCD-aware tile order (speed only): workgroups b and b + 8 share an XCD under round-robin dispatch.
  // xpr > 0: the R x C tile grid is cut into xpr x (8 / xpr) blocks, one per XCD, the cut chosen on the
  // host to minimise the A row tiles + B column tiles an XCD's L2 must hold per K-step (GPT-2 1.3B fc1
  // 32 x 8 tiles -> 4 x 2 blocks of 8 x 4; fc2 8 x 32 -> 1 x 8 blocks of 8 x 4).  xpr == 0: each XCD takes
  // a contiguous run of tiles (grids the cut does not divide).
  const int ctiles = Nc / BC, rtiles = Nr / BR;
  const int ntiles = gridDim.x, xcd = blockIdx.x & 7, loc = blockIdx.x >> 3;
  int tr, tc;
  if (OPT & 2) {
    tr = blockIdx.x / ctiles; tc = blockIdx.x % ctiles;
  } else if (xpr > 0) {
    const int xpc = 8 / xpr, rb = rtiles / xpr, cb = ctiles / xpc;
    tr = (xcd / xpc) * rb + loc / cb;
    tc = (xcd % xpc) * cb + loc % cb;
  } else {
    const int q8 = ntiles >> 3, r8 = ntiles & 7;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    tr = tile / ctiles; tc = tile % ctiles;
  }
  const int n0 = tr * BR, c0 = tc * BC;
  const int mbeg = blockIdx.y * m_per_split, mend = min(M, mbeg + m_per_split);
  const int T = (mend - mbeg) / BKT;

  // per-lane fragment offsets of token step 0: 4 A blocks (rows), 2 B blocks (cols).  Step s adds exactly
  // 16 * s rows (the swizzle depends on row & 3 only), a compile-time immediate on the ds_read.
  FragAddr fa[4], fb[JB];
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[i] = frag_addr(lane, 128 * wr + 32 * i, 0);
#pragma unroll
  for (int j = 0; j < JB; ++j) fb[j] = frag_addr(lane, 32 * JB * wc + 32 * j, 0);
  f32x16 acc[4][JB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  DmaOp<BKT, NTH> da, db;
  da.init(Nr, tid);
  db.init(Nc, tid);
  const bf16_t* Ab = A + n0;   // column offset of this tile; rows advance per K-step
  const bf16_t* Bb = B + c0;
  auto issue = [&](int stage_t, bf16_t* buf, int i) {   // piece i of both operands of stage stage_t
    const int m = mbeg + stage_t * BKT;
    da.piece(Ab + (int64_t)m * Nr, Nr, buf, tid, i);
    db.piece(Bb + (int64_t)m * Nc, Nc, buf + TILE_ELEMS, tid, i);
  };
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < T) {
#pragma unroll
      for (int i = 0; i < P / 2; ++i) issue(st, smem + st * STAGE, i);
    }

  // K-loop unrolled by the ring so every LDS address (read stage and DMA target stage) is compile-time
  auto kstep = [&](const int t, const bf16_t* as, bf16_t* nb) {
    wait_vm(min(NST - 2, T - 1 - t) * P);   // stage t landed (this wave's pieces) ...
    __syncthreads();                         // ... for every wave; all done reading stage t-1's buffer (= nb)
    const bool more = t + NST - 1 < T;
    const bf16_t* bs = as + TILE_ELEMS;
    u16x8 a[4], b[JB];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag(as, fa[i]);
#pragma unroll
    for (int j = 0; j < JB; ++j) b[j] = frag(bs, fb[j]);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      u16x8 an[4], bn[JB];
      // the new stage's DMA pieces ride in the first steps' MFMA shadow (an LDS-DMA issue costs ~60 cycles
      // beside bare MFMAs; issued back to back after the barrier they were ~500 exposed cycles)
      if (more) {
#pragma unroll
        for (int i = 0; i < P / 2; ++i)
          if (i * (KS > 1 ? KS / 2 : 1) / (P / 2) == s) issue(t + NST - 1, nb, i);   // first half of the K-step
      }
      if (s + 1 < KS) {   // next step's fragments issue ahead of this step's MFMAs, in their own region
#pragma unroll
        for (int i = 0; i < 4; ++i) an[i] = frag(as + (s + 1) * 16 * 256, fa[i]);
#pragma unroll
        for (int j = 0; j < JB; ++j) bn[j] = frag(bs + (s + 1) * 16 * 256, fb[j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < JB; ++j) {
          if constexpr (NTH == 256) mfma32_acc(acc[i][j], a[i], b[j]);
          else acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
        }
      if constexpr (OPT & 1) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < KS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = an[i];
#pragma unroll
        for (int j = 0; j < JB; ++j) b[j] = bn[j];
      }
    }
  };
  for (int t = 0; t < T; t += NST) {
#pragma unroll
    for (int u = 0; u < NST; ++u)
      if (t + u < T) kstep(t + u, smem + u * STAGE, smem + ((u + NST - 1) % NST) * STAGE);
  }
  if constexpr (NTH == 256) acc_fence();
  // epilogue: acc[i][j] register r, lane l -> C[n0 + 128wr + 32i + acc_row(r, h)][c0 + 32JB wc + 32j + (l & 31)]
  const int col = c0 + 32 * JB * wc + (lane & 31);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = n0 + 128 * wr + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        if constexpr (PARTIAL) {
          float* Cp = reinterpret_cast<float*>(C) + (int64_t)blockIdx.y * Nr * Nc;
          Cp[(int64_t)row * Nc + col + 32 * j] = acc[i][j][r];
        } else {
          reinterpret_cast<bf16_t*>(C)[(int64_t)row * Nc + col + 32 * j] = f2bf(acc[i][j][r]);
        }
      }
    }
}

// out[e] = sum over S slices of part[s][e] (fp32 slabs) -> bf16, 4 elements per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, bf16_t* __restrict__ out,
                                                            int64_t n4, int S, int64_t slab) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
    float4 s = reinterpret_cast<const float4*>(part)[e];
    for (int k = 1; k < S; ++k) {
      const float4 v = reinterpret_cast<const float4*>(part + k * slab)[e];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    u16x4 o;
    o[0] = f2bf(s.x); o[1] = f2bf(s.y); o[2] = f2bf(s.z); o[3] = f2bf(s.w);
    reinterpret_cast<u16x4*>(out)[e] = o;
  }
}


}  // namespace

// Shapes the kernel takes: Nr % 256 == 0, Nc % 256 == 0, M % (64 * splits) == 0, 16-B aligned rows.
PDT_API int pdt_wgrad_ok(int64_t M, int64_t Nr, int64_t Nc, int splits) {
  return splits >= 1 && M > 0 && Nr % BR == 0 && Nc % BC == 0 && M % ((int64_t)BK * splits) == 0 &&
         (Nr / BR) * (Nc / BC) <= 65535 && M <= (1LL << 30) && Nr * Nc <= (1LL << 31);
}

// C[Nr, Nc] (bf16) = A[M, Nr]^T B[M, Nc]; splits > 1 needs an fp32 workspace of splits * Nr * Nc floats.
namespace {

// kernel variant: 1 = BK 64 x 2 stages (default), 2 = BK 32 x 4 stages (measured 1-6 % slower), 3 = 1 + s_setprio
// around the MFMAs, 4 = 1 in plain row-major tile order (no XCD blocking).  (A 4-wave variant with 128 x 128
// blocks per wave, NTH = 256, needs 256 AGPR accumulators + ~300 VGPRs and hipcc spills 234 of them: not
// launched); PDT_WGRAD_VARIANT or pdt_wgrad_set_variant
int g_wgrad_variant = -1;
int wgrad_variant() {
  if (g_wgrad_variant < 0) { const char* e = getenv("PDT_WGRAD_VARIANT"); g_wgrad_variant = e ? atoi(e) : 1; }
  return g_wgrad_variant;
}

template <int BKT, int NST, int OPT, int NTH = 512>
void launch_wgrad(const void* A, const void* B, void* C, int64_t M, int64_t Nr, int64_t Nc, int splits, float* ws,
                  hipStream_t st) {
  const int R = (int)(Nr / BR), Cc = (int)(Nc / BC), tiles = R * Cc;
  const int mps = (int)(M / splits);
  dim3 grid(tiles, splits);
  int xpr = 0, best = 1 << 30;   // XCD block cut: xpr row parts x (8 / xpr) column parts
  for (int pr = 1; pr <= 8; pr *= 2) {
    const int pc = 8 / pr;
    if (R % pr || Cc % pc) continue;
    const int cost = R / pr + Cc / pc;
    if (cost < best) { best = cost; xpr = pr; }
  }
  if (splits == 1) {
    wgrad_kernel<false, BKT, NST, OPT, NTH><<<grid, NTH, 0, st>>>((const bf16_t*)A, (const bf16_t*)B, C, (int)M, (int)Nr,
                                                        (int)Nc, mps, xpr);
  } else {
    wgrad_kernel<true, BKT, NST, OPT, NTH><<<grid, NTH, 0, st>>>((const bf16_t*)A, (const bf16_t*)B, ws, (int)M, (int)Nr,
                                                       (int)Nc, mps, xpr);
    const int64_t n4 = Nr * Nc / 4;
    splitk_reduce_kernel<<<grid_for(n4, 256, 256 * 16), 256, 0, st>>>(ws, (bf16_t*)C, n4, splits, Nr * Nc);
  }
}

}  // namespace

PDT_API int pdt_wgrad_set_variant(int v) {
  if (v > 0) g_wgrad_variant = v;
  return wgrad_variant();
}

// C[Nr, Nc] (bf16) = A[M, Nr]^T B[M, Nc]; splits > 1 needs an fp32 workspace of splits * Nr * Nc floats.
PDT_API int pdt_wgrad_bf16(const void* A, const void* B, void* C, int64_t M, int64_t Nr, int64_t Nc, int splits,
                           float* ws, hipStream_t st) {
  if (!pdt_wgrad_ok(M, Nr, Nc, splits)) return (int)hipErrorInvalidValue;
  if (splits > 1 && !ws) return (int)hipErrorInvalidValue;
  switch (wgrad_variant()) {
    case 2: launch_wgrad<32, 4, 0>(A, B, C, M, Nr, Nc, splits, ws, st); break;
    case 3: launch_wgrad<64, 2, 1>(A, B, C, M, Nr, Nc, splits, ws, st); break;
    case 4: launch_wgrad<64, 2, 2>(A, B, C, M, Nr, Nc, splits, ws, st); break;
    default: launch_wgrad<64, 2, 0>(A, B, C, M, Nr, Nc, splits, ws, st); break;
  }
  return (int)hipGetLastError();
}
