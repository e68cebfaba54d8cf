// bf16 GEMM family for gfx950 with fused epilogues: C[M, N] = sum_k A(m, k) B(k, n), fp32 accumulate.
//
//   layout NT : A[m * lda + k], B[n * ldb + k]  -- Linear forward x W^T, and dgrad dY (W^T)^T with the
//               weight transposed once (ops.linear: hipBLASLt's NN kernels ran 10-25 % below NT there)
//   layout TT : A[k * lda + m], B[k * ldb + n]  -- weight gradient dW = dY^T X (both token-major)
//
// Epilogues (the reason this kernel exists next to hipBLASLt, whose GELU_AUX_BIAS / DGELU_BGRAD epilogues
// are unsupported on gfx950, profiles/r2_hipblaslt_epilogue_probe.txt):
//   PLAIN   C = bf16(acc)                         BIAS   C = bf16(acc + bias[n])
//   GELU    h = bf16(acc + bias[n]); C = gelu_tanh(h), aux_out = gelu_tanh'(h) (bf16)   (GPT-2 c_fc: one pass,
//           the derivative -- not the pre-activation -- is what the backward keeps)
//   DGELU   g = acc * aux[m, n] (the stored derivative) -> C, per-tile column sums of g -> ws (fp32) -> dbias
//           (GPT-2 c_proj dgrad + GELU backward + bias gradient of c_fc: no bias_gelu_bwd_db pass, and no
//           transcendental in an epilogue that runs while the matrix pipe idles)
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
#include "reduce.h"
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
typedef __attribute__((address_space(3))) const char lds_cchar;

constexpr int TM = 256, TN = 256, KB = 64, NTH = 256;
constexpr int OPB = TM * KB * 2;           // bytes of one operand tile of one K-step (32 KiB)
constexpr int STB = 2 * OPB;               // one ring slot: A tile then B tile (2 slots = 128 KiB)
constexpr int PIECES = OPB / (NTH * 16);   // LDS-DMA instructions per thread per operand per K-step (8)

enum { L_NT = 0, L_TT = 1 };
enum { E_PLAIN = 0, E_BIAS = 1, E_GELU = 2, E_DGELU = 3, E_F32 = 4 };

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

// TT image swizzle: 16-B chunk c of k-row r is stored at chunk c ^ tt_f(r)
__device__ __forceinline__ int tt_f(int r) { return 2 * ((r & 3) | ((r >> 1) & 4)); }

// One operand's LDS-DMA for one K-step: PIECES wave-instructions of 1 KiB (lane-linear LDS destination,
// swizzle on the per-lane SOURCE offset).  Piece i of wave w is 1-KiB block q = 4 i + w of the tile; its
// per-lane byte offset is a lane term (the same for every piece, or one per piece parity for TT) plus a
// wave-uniform row term passed as the buffer instruction's scalar offset.
template <int LAYOUT>
struct Dma {
  uint32_t off0, off1;   // lane terms (NT: off1 unused)
  uint32_t rowstep;      // bytes between consecutive pieces' first rows x 2 (scalar offsets are i * rowstep / 2)
  __device__ __forceinline__ void init(int64_t ld, int w, int lane) {
    if (LAYOUT == L_NT) {        // 8 rows x 128 B per piece: rows 8 q + (lane >> 3); piece i: +32 i rows
      const int row = 8 * w + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);      // (row >> 1) & 7 does not depend on i (32 i rows)
      off0 = off1 = (uint32_t)(row * ld * 2 + c * 16);
      rowstep = (uint32_t)(32 * ld * 2);
    } else {                     // 2 k-rows x 512 B per piece: rows 8 i + 2 w + (lane >> 5)
      const int r0 = 2 * w + (lane >> 5);
      off0 = (uint32_t)(r0 * ld * 2 + ((lane & 31) ^ tt_f(r0)) * 16);        // even i (row bit 3 clear)
      off1 = (uint32_t)(r0 * ld * 2 + ((lane & 31) ^ tt_f(r0 + 8)) * 16);    // odd i
      rowstep = (uint32_t)(8 * ld * 2);
    }
  }
  // wave-uniform state of one tile's DMA (descriptor, LDS base, row step), then single pieces
  struct Tile {
    v4i rsrc;
    uint32_t lds0, rs;
  };
  __device__ __forceinline__ Tile tile(const char* t, uint32_t nbytes, uint32_t lds_op, int w) const {
    const uint64_t addr = (uint64_t)(uintptr_t)t;
    Tile d;
    d.rsrc[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)addr);
    d.rsrc[1] = __builtin_amdgcn_readfirstlane((int)((addr >> 32) & 0xffff));
    d.rsrc[2] = __builtin_amdgcn_readfirstlane((int)nbytes);
    d.rsrc[3] = 0x00020000;
    d.lds0 = __builtin_amdgcn_readfirstlane(lds_op + w * 1024);
    d.rs = __builtin_amdgcn_readfirstlane(rowstep);
    return d;
  }
  template <int I>
  __device__ __forceinline__ void piece(const Tile& d) const {
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(d.lds0 + I * 4096), "v"((I & 1) ? off1 : off0), "s"(d.rsrc), "s"(I * d.rs) : "memory");
  }
  // pieces [I0, I1) of the tile at byte address `tile` (wave-uniform) into the LDS tile at byte address `lds_op`
  template <int I0, int I1>
  __device__ __forceinline__ void issue(const char* tile, uint32_t nbytes, uint32_t lds_op, int w) const {
    const uint64_t addr = (uint64_t)(uintptr_t)tile;
    v4i rsrc;
    rsrc[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)addr);
    rsrc[1] = __builtin_amdgcn_readfirstlane((int)((addr >> 32) & 0xffff));
    rsrc[2] = __builtin_amdgcn_readfirstlane((int)nbytes);
    rsrc[3] = 0x00020000;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_op + w * 1024);
    const uint32_t rs = __builtin_amdgcn_readfirstlane(rowstep);
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      const uint32_t m0 = lds0 + i * 4096;
      asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(m0), "v"((i & 1) ? off1 : off0), "s"(rsrc), "s"(i * rs) : "memory");
    }
  }
};

// Fragment of 16 rows (NT: rows of the operand tile; TT: columns) x 32 k (k-substep S of the 64-deep
// K-step) for the 16x16x32 MFMA: lane l gets row/col (l & 15), k = 32 S + 8 (l >> 4) + e, e = 0..7.
template <int LAYOUT>
struct Frag {
  uint32_t o0, o1;   // NT: byte offsets of block 0 for S = 0 / 1;  TT: row offset, swizzle term
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
  __device__ __forceinline__ u16x8 read(lds_cchar* op, int blk) const {
    if (LAYOUT == L_NT) {
      return *(const lds_u16x8*)(op + blk * 16 * 128 + (S ? o1 : o0));
    } else {
      const uint32_t a = o0 + S * 32 * 512 + 16 * ((uint32_t)(2 * blk) ^ o1);
      const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(op + a));
      const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(op + a + 2048));
      return __builtin_bit_cast(u16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const bf16_t* bias;     // E_BIAS / E_GELU: [N]
  const bf16_t* aux;      // E_DGELU: gelu'(pre-activation) [M, ldc], as E_GELU wrote it
  bf16_t* aux_out;        // E_GELU: gelu'(pre-activation) out [M, ldc]
  float* ws;              // E_F32: slabs [splits][M][N]; E_DGELU: column partials [M / 256][N]
  int M, N, K;
  int64_t lda, ldb, ldc;
  int k_per_split;
  int xpr;                // XCD block cut (see tile_of)
  int grp;                // tile rows per group inside an XCD block (see tile_of)
};

__device__ __forceinline__ void tile_of(const GemmArgs& p, int id, int ntiles, int& tm, int& tn) {
  // XCD-aware tile order (speed only): tile ids b and b + 8 share an XCD under round-robin dispatch (a
  // persistent workgroup b walks ids b, b + G, ... with G % 8 == 0, so all of them stay on its XCD).
  // xpr > 0: the tile grid is cut into xpr x (8 / xpr) blocks, one per XCD (host picks the cut that
  // minimises the A + B panels an XCD's L2 holds); else each XCD takes a contiguous run of tiles.
  const int mt = p.M / TM, nt = p.N / TN;
  const int xcd = id & 7, loc = id >> 3;
  if (p.xpr > 0) {
    // inside the block, groups of grp tile rows walked column-major within the group: the ~32 tiles an XCD's
    // CUs hold at once form a grp x (32 / grp) rectangle (4 x 8 for GPT-2's c_fc: 4 A panels + 8 B panels per
    // K-step in its L2) instead of one row of tiles that streams every B panel (1 A + 32 B at c_fc)
    const int xpc = 8 / p.xpr, rb = mt / p.xpr, cb = nt / xpc, g = p.grp, per = g * cb;
    tm = (xcd / xpc) * rb + (loc / per) * g + loc % g;
    tn = (xcd % xpc) * cb + (loc % per) / g;
  } else {
    const int q8 = ntiles >> 3, r8 = ntiles & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    tm = t / nt;
    tn = t % nt;
  }
}

// Main loop: 4 waves (one per SIMD: the accumulators of a 128 x 128 wave tile -- 8 x 8 MFMA tiles, 256
// registers -- plus two fragment sets fill its register file), K-step 64 = two 32-deep substeps, 2-slot
// LDS ring (2 x 64 KiB) filled by LDS-DMA.  Software pipeline per K-step t (one barrier):
//   A : 64 MFMAs of substep 0 (fragments F0)  ||  ds_reads of substep 1 of tile t -> F1
//   B1: 32 MFMAs of substep 1 (rows 0-63)
//       s_waitcnt vmcnt(0) (tile t+1 landed) + lgkmcnt(0) + barrier: tile t+1 visible to all waves, and every
//       wave is done reading tile t's slot
//   B2: 32 MFMAs of substep 1 (rows 64-127)  ||  ds_reads of substep 0 of tile t+1 -> F0  ||  LDS-DMA of
//       tile t+2 into tile t's slot (half of its pieces; the other half rides in the next step's A)
// A tile's DMA therefore has ~1.5 K-steps of MFMAs to land, no ds_read ever waits at a step boundary, and
// the matrix pipe of a SIMD sees 128 MFMAs per barrier (cf. the 2-wave-per-SIMD staggered variant: 56 %
// MFMA busy against hipBLASLt's 85 % at 8192^3, profiles/r3_pmc_gemm_v2_vs_hipblaslt.txt).
// (This compiler-scheduled kernel is the alternative path -- PDT_GEMM_KERNEL=hip -- and the bitwise reference
// of the hand-scheduled gemm_asm_kernel below: the same MFMA order per accumulator.)
template <int LAYOUT, int EPI>
__global__ __launch_bounds__(NTH, 1) void gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STB];
  lds_cchar* const lds = (lds_cchar*)(lds_void*)smem;                 // the ring, LDS address space
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_void*)smem;     // its LDS byte address (LDS-DMA m0)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  const int ntiles = (int)gridDim.x;
  int tm, tn;
  tile_of(p, blockIdx.x, ntiles, tm, tn);
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
  int64_t astep, bstep;
  uint32_t abytes, bbytes;
  auto tile_base = [&](int mm, int nn, int64_t& ao, int64_t& bo) {
    if (LAYOUT == L_NT) {
      ao = ((int64_t)mm * p.lda + kbeg) * 2; bo = ((int64_t)nn * p.ldb + kbeg) * 2;
    } else {
      ao = ((int64_t)kbeg * p.lda + mm) * 2; bo = ((int64_t)kbeg * p.ldb + nn) * 2;
    }
  };
  if (LAYOUT == L_NT) {
    astep = bstep = KB * 2;
    abytes = (uint32_t)((TM - 1) * p.lda * 2 + KB * 2); bbytes = (uint32_t)((TN - 1) * p.ldb * 2 + KB * 2);
  } else {
    astep = KB * p.lda * 2; bstep = KB * p.ldb * 2;
    abytes = (uint32_t)((KB - 1) * p.lda * 2 + TM * 2); bbytes = (uint32_t)((KB - 1) * p.ldb * 2 + TN * 2);
  }
  int64_t a0, b0;
  tile_base(m0, n0, a0, b0);
  // pieces [I0, I1) of BOTH operands of K-step t into slot t & 1
  auto issue = [&](auto i0, auto i1, int t) {
    constexpr int J0 = decltype(i0)::value, J1 = decltype(i1)::value;
    da.template issue<J0, J1>(Ab + a0 + t * astep, abytes, lds_addr + (t & 1) * STB, w);
    db.template issue<J0, J1>(Bb + b0 + t * bstep, bbytes, lds_addr + (t & 1) * STB + OPB, w);
  };
  using P0 = std::integral_constant<int, 0>;
  using PH = std::integral_constant<int, PIECES / 2>;
  using PE = std::integral_constant<int, PIECES>;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 fa0[8], fb0[8], fa1[8], fb1[8];   // F0 / F1: 8 A blocks (rows 128 wr..) + 8 B blocks (128 wc..)

  // prologue: tiles 0 and 1 in flight, tile 0 landed + visible, its substep-0 fragments in F0
  issue(P0{}, PE{}, 0);
  if (T > 1) issue(P0{}, PE{}, 1);
  if (T > 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * PIECES) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = fr.template read<0>(lds, 8 * wr + i);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = fr.template read<0>(lds + OPB, 8 * wc + j);

  // one K-step; G (guarded) only for the last two steps, so the steady state is branch-free and its
  // instruction interleave can be pinned with sched_group_barrier (hipcc otherwise issues a stage's reads
  // just in time and waits on them between MFMAs).  Measured: this form (DMA pieces issued as one group
  // ahead of each MFMA stretch, reads interleaved 1 : 4 / 1 : 2 with the MFMAs) beat spreading the DMA
  // pieces between 8-MFMA groups by 8 % on the weight-gradient (TT) shapes (profiles/r3_gemm_variants.txt).
  auto kstep = [&](auto guarded, const int t) {
    constexpr bool G = decltype(guarded)::value;
    lds_cchar* sa = lds + (t & 1) * STB;
    lds_cchar* na = lds + ((t + 1) & 1) * STB;
    // ---- A: substep 0 MFMAs || substep 1 reads (tile t) || second half of tile t+1's DMA
    if (t >= 1 && (!G || t + 1 < T)) issue(PH{}, PE{}, t + 1);
    // read order = order of first use: every B block (all of B1's MFMAs need them), then A blocks 0..7
#pragma unroll
    for (int j = 0; j < 8; ++j) fb1[j] = fr.template read<1>(sa + OPB, 8 * wc + j);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa1[i] = fr.template read<1>(sa, 8 * wr + i);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(fb0[j], fa0[i], acc[i][j]);
    if (!G) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 LDS read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // 4 MFMAs
      }
    }
    // ---- B1: substep 1, rows 0-63
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(fb1[j], fa1[i], acc[i][j]);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    // ---- B2: substep 1, rows 64-127 || tile t+1 substep-0 reads || first half of tile t+2's DMA
    //      (issuing all of t+2 here -- a full K-step to land, as hipBLASLt's loop does -- made hipcc shuffle the
    //      256 accumulators between AGPRs and VGPRs every step, with or without unrolling: kept split)
    if (!G || t + 2 < T) issue(P0{}, PH{}, t + 2);
    const bool more = !G || t + 1 < T;
    if (more) {   // the next step's A needs every B block first, then A blocks in order
#pragma unroll
      for (int j = 0; j < 8; ++j) fb0[j] = fr.template read<0>(na + OPB, 8 * wc + j);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa0[i] = fr.template read<0>(na, 8 * wr + i);
    }
#pragma unroll
    for (int i = 4; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(fb1[j], fa1[i], acc[i][j]);
    if (!G) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);   // 1 LDS read
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 1);   // 2 MFMAs
      }
    }
  };
  using Steady = std::integral_constant<bool, false>;
  using Guarded = std::integral_constant<bool, true>;
  int t = 0;
  for (; t + 2 < T; ++t) kstep(Steady{}, t);
  for (; t < T; ++t) kstep(Guarded{}, t);

  // ---------------------------------------------------------------- epilogue
  {
  // acc[i][j][r] = C[m0 + 128 wr + 16 i + (lane & 15)][n0 + 128 wc + 16 j + 4 (lane >> 4) + r]
  const int mrow = m0 + 128 * wr + (lane & 15);
  const int ncol = n0 + 128 * wc + 4 * (lane >> 4);
  if constexpr (EPI == E_F32) {
    float* C = p.ws + (int64_t)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<f32x4*>(C + (int64_t)(mrow + 16 * i) * p.N + ncol + 16 * j) = acc[i][j];
  } else {
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
    float bj[8][4];
    if constexpr (EPI == E_BIAS || EPI == E_GELU) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const u16x4 b = *reinterpret_cast<const u16x4*>(p.bias + ncol + 16 * j);
#pragma unroll
        for (int r = 0; r < 4; ++r) bj[j][r] = bf2f(b[r]);
      }
    }
    float cs[8][4];   // E_DGELU: this lane's column sums over its 8 rows
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t rowoff = (int64_t)(mrow + 16 * i) * p.ldc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t e = rowoff + ncol + 16 * j;
        u16x4 o;
        if constexpr (EPI == E_PLAIN) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r]);
        } else if constexpr (EPI == E_BIAS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] + bj[j][r]);
        } else if constexpr (EPI == E_GELU) {
          // GELU and its derivative of the ROUNDED (bf16) pre-activation, as an unfused bf16 Linear + GELU
          // computes them; the derivative is kept for the backward (aux_out)
          u16x4 dd;
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            gelu_f32x2 y2, d2;
            gelu_fwd_grad2(gelu_f32x2{bf2f(f2bf(acc[i][j][r] + bj[j][r])), bf2f(f2bf(acc[i][j][r + 1] + bj[j][r + 1]))},
                           y2, d2);
            o[r] = f2bf(y2[0]); o[r + 1] = f2bf(y2[1]);
            dd[r] = f2bf(d2[0]); dd[r + 1] = f2bf(d2[1]);
          }
          *reinterpret_cast<u16x4*>(p.aux_out + e) = dd;
        } else {   // E_DGELU: aux holds gelu'(pre) as E_GELU stored it
          const u16x4 h = *reinterpret_cast<const u16x4*>(p.aux + e);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float g = acc[i][j][r] * bf2f(h[r]);
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
      for (int j = 0; j < 8; ++j)
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
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[wr * 256 + 128 * wc + 16 * j + 4 * (lane >> 4) + r] = cs[j][r];
      }
      __syncthreads();
      p.ws[(int64_t)tm * p.N + n0 + tid] = red[tid] + red[256 + tid];
    }
  }
  }
}

// ============================================================================================================
// Hand-scheduled main loop (round 4): the whole K-loop is ONE inline-asm statement generated by
// gen_gemm_kloop.py (gemm_kloop.inc) -- same tile, LDS images and DMA pieces as gemm_kernel above, but every
// MFMA, LDS read, LDS-DMA piece, wait and barrier placed by hand with the accumulators pinned in a[0:255].
// Epilogue: accumulator tiles are read back (v_accvgpr_read), the epilogue math runs in fp32, and bf16 results
// are staged through LDS (528-byte rows) so every global store is a full 512-byte row segment
// (32 lanes x 16 B; the compiler-scheduled kernel's 8-byte stores touched 16 rows per instruction).
// ============================================================================================================
}  // namespace
#include "gemm_kloop.inc"
namespace {

constexpr int RING = 2 * STB;                // the two ring stages (128 KiB)
constexpr int STAGE_BYTES = 32768;          // epilogue staging: LDS past the ring, 64 rows x 512 B per round
constexpr int SMEM3 = RING + STAGE_BYTES;   // 160 KiB: all of the CU's LDS

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// accumulator tile k = 8 i + j (4 fp32) out of a[4k .. 4k + 3]
template <int K>
__device__ __forceinline__ f32x4 acc_tile() {
  float x, y, z, w;
  asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
               "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
               : "=v"(x), "=v"(y), "=v"(z), "=v"(w)
               : "i"(4 * K), "i"(4 * K + 1), "i"(4 * K + 2), "i"(4 * K + 3));
  return f32x4{x, y, z, w};
}

// Epilogue staging (round r = 0..3): every wave's accumulator tiles i = 2r, 2r + 1 (32 rows x 128 columns), i.e.
// rows {32 r .. 32 r + 31} and {128 + 32 r ..} of the 256 x 256 tile: 64 rows x 512 B at LDS offset RING.  Image row
// q = 32 wr + (row & 31); its 16-byte chunks are XOR-swizzled with (q & 15) (the 16 lanes of an accumulator
// column write 16 consecutive rows: without the swizzle one bank).  Each wave then reads 16 whole rows back (two
// rows = 1 KiB per instruction) and stores them as full 512-byte row segments.
__device__ __forceinline__ uint32_t stg_off(int q, int col) {   // byte offset of (image row q, column col)
  return (uint32_t)(q * 512 + ((((col >> 3) ^ q) & 15) | ((col >> 3) & 16)) * 16 + (col & 7) * 2);
}
// global row of image row q in round r
__device__ __forceinline__ int stg_row(int r, int q) { return 128 * (q >> 5) + 32 * r + (q & 31); }
__device__ __forceinline__ void stg_read(const char* img, u16x8 (&buf)[8], int w, int lane) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int q = 16 * w + 2 * it + (lane >> 5), c16 = lane & 31;
    buf[it] = *reinterpret_cast<const u16x8*>(img + q * 512 + ((c16 ^ (q & 15)) & 15 | (c16 & 16)) * 16);
  }
}
// Global side of the staging rounds through buffer instructions: ONE per-lane byte offset (lane term + the wave's
// rows) and a scalar per-(round, row pair) offset, instead of a 64-bit address per row and round that the compiler
// precomputes and keeps live (the DGELU epilogue spilled those).  Resource = the 256 x 256 tile at (m0, n0).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const bf16_t* base, int64_t ldc, int m0, int n0) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)m0 * ldc + n0), (short)0,
                                           (int)((255 * ldc + 256) * 2), 0x00020000);
}
// lane offset of image row q = 16 w + 2 it + (lane >> 5), chunk lane & 31 (it = 0); global row stg_row(r, q)
__device__ __forceinline__ uint32_t stg_voff(int64_t ldc, int w, int lane) {
  return (uint32_t)(128 * (w >> 1) + 16 * (w & 1) + (lane >> 5)) * ((uint32_t)ldc * 2u) + (uint32_t)(lane & 31) * 16u;
}
// sum over the 16 lanes of a DPP row (quad swaps, then half-row and row mirrors): no lane-index registers, unlike
// __shfl_xor's ds_bpermute (whose hoisted index VGPRs spilled in the DGELU kernel)
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));    // quad (1,0,3,2)
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));    // quad (2,3,0,1)
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));   // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));   // row_mirror
  return v;
}
__device__ __forceinline__ void stg_write_out(const u16x8 (&buf)[8], __amdgpu_buffer_rsrc_t rs, uint32_t vo,
                                              uint32_t ldc2, int r) {
#pragma unroll
  for (int it = 0; it < 8; ++it)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, buf[it]), rs, (int)vo,
                                           (int)((32 * r + 2 * it) * ldc2), 0);
}
// DGELU: the aux rows of round r (the same mapping as the write-out, reversed): fetched into registers a round
// ahead (stg_fetch), put into the image when the round starts (stg_put)
__device__ __forceinline__ void stg_fetch(u16x8 (&t)[8], __amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t ldc2, int r) {
#pragma unroll
  for (int it = 0; it < 8; ++it)
    t[it] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo,
                                                                            (int)((32 * r + 2 * it) * ldc2), 0));
}
__device__ __forceinline__ void stg_put(char* img, const u16x8 (&t)[8], int w, int lane) {
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int q = 16 * w + 2 * it + (lane >> 5), c16 = lane & 31;
    *reinterpret_cast<u16x8*>(img + q * 512 + ((c16 ^ (q & 15)) & 15 | (c16 & 16)) * 16) = t[it];
  }
}
// DGELU round 0 by LDS-DMA, issued BEFORE the item's main loop: the aux rows of round 0 land straight in the
// staging image (idle during the loop) under the first K-step, so the epilogue's first round waits on nothing.
// Piece i of wave w fills image rows q = 16 w + 2 i + (lane >> 5), lane-linear 16-byte positions p = lane & 31;
// position p of row q holds the image's swizzled chunk, i.e. logical chunk ((p ^ q) & 15) | (p & 16) (the XOR is
// an involution), whose global row is stg_row(0, q): the swizzle rides on the per-lane source offset (rule 21).
// Every wave waits for these 8 pieces (vmcnt, in order) and passes a barrier inside the main loop before the
// epilogue reads the image.
__device__ __forceinline__ void stg_dma_round0(const bf16_t* src, int64_t ldc, int m0, int n0, uint32_t img_lds,
                                               int w, int lane) {
  const uint64_t base = (uint64_t)(uintptr_t)(src + (int64_t)m0 * ldc + n0);
  v4i rsrc;                                       // (kernel arguments and item coordinates: already scalar)
  rsrc[0] = (int)(uint32_t)base;
  rsrc[1] = (int)((base >> 32) & 0xffff);
  rsrc[2] = (int)(uint32_t)((255 * ldc + 256) * 2);
  rsrc[3] = 0x00020000;
  const int hi = lane >> 5, p = lane & 31;
  const uint32_t row0 = (uint32_t)(128 * (w >> 1) + 16 * (w & 1));
  const uint32_t ldc2 = (uint32_t)ldc * 2u;       // 32-bit lane math (a 64-bit product wants a VGPR copy of ldc)
  uint32_t vo[8], so[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t c16 = (uint32_t)(((p ^ (2 * i + hi)) & 15) | (p & 16));
    vo[i] = (uint32_t)hi * ldc2 + c16 * 16u;
    so[i] = __builtin_amdgcn_readfirstlane((row0 + 2 * i) * ldc2);
  }
  const uint32_t m = __builtin_amdgcn_readfirstlane(img_lds + 16 * w * 512);
  asm volatile(
      "s_mov_b32 m0, %[m]\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v0], %[rs], %[s0] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v1], %[rs], %[s1] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v2], %[rs], %[s2] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v3], %[rs], %[s3] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v4], %[rs], %[s4] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v5], %[rs], %[s5] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v6], %[rs], %[s6] offen lds\n\t"
      "s_add_u32 m0, m0, 1024\n\ts_nop 0\n\tbuffer_load_dwordx4 %[v7], %[rs], %[s7] offen lds"
      :
      : [m] "s"(m), [rs] "s"(rsrc), [v0] "v"(vo[0]), [v1] "v"(vo[1]), [v2] "v"(vo[2]), [v3] "v"(vo[3]),
        [v4] "v"(vo[4]), [v5] "v"(vo[5]), [v6] "v"(vo[6]), [v7] "v"(vo[7]), [s0] "s"(so[0]), [s1] "s"(so[1]),
        [s2] "s"(so[2]), [s3] "s"(so[3]), [s4] "s"(so[4]), [s5] "s"(so[5]), [s6] "s"(so[6]), [s7] "s"(so[7])
      : "memory", "scc");
}

// The thread id for one item's per-lane terms, rebuilt from the wave index (SGPR) and the lane id (v_mbcnt) behind an
// opaque asm: no VGPR -- not even threadIdx.x -- has to stay live across the persistent loop's main-loop statements
// (a spilled one is reloaded from scratch with a vmcnt(0) that drains the prefetched K-tiles and epilogue stores).
__device__ __forceinline__ int item_tid(int wv) {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return wv * 64 + l;
}
// A scalar the compiler must treat as unknown at this point: integer divisions by it are expanded here, per item,
// instead of hoisting their (VGPR) float reciprocals out of the persistent loop.
__device__ __forceinline__ int opaque_s(int x) {
  asm volatile("" : "+s"(x));
  return x;
}

// Epilogue operands loaded BEFORE an item's main loop by inline-asm buffer loads, i.e. invisible to the compiler's
// waitcnt pass: a compiler-issued load pending across the main-loop statement is waited for with vmcnt(0) after it,
// which drains the next item's prefetched K-tiles (gen_gemm_kloop.py next_tail).  Every path through the main loop
// waits (in order) for all vector-memory ops older than its last DMA, so these have landed when it ends; `settle`
// (an empty volatile asm after the main loop, ordered after it like every volatile asm) makes each use depend on
// that point.  Bias: the lane's 8 x 4 columns (immediate offsets 32 B apart); DGELU: round 1 of the derivative rows.
__device__ __forceinline__ v4i scalar_rsrc(const void* base, uint32_t nbytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  v4i r;
  r[0] = (int)(uint32_t)a; r[1] = (int)((a >> 32) & 0xffff); r[2] = (int)nbytes; r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void preload_bias(u16x4 (&b)[8], const bf16_t* bias, int n0, int lcol) {
  const v4i rs = scalar_rsrc(bias + n0, 512);
  const uint32_t vo = (uint32_t)lcol * 2u;
  asm volatile("buffer_load_dwordx2 %0, %8, %9, 0 offen offset:0\n\t"
               "buffer_load_dwordx2 %1, %8, %9, 0 offen offset:32\n\t"
               "buffer_load_dwordx2 %2, %8, %9, 0 offen offset:64\n\t"
               "buffer_load_dwordx2 %3, %8, %9, 0 offen offset:96\n\t"
               "buffer_load_dwordx2 %4, %8, %9, 0 offen offset:128\n\t"
               "buffer_load_dwordx2 %5, %8, %9, 0 offen offset:160\n\t"
               "buffer_load_dwordx2 %6, %8, %9, 0 offen offset:192\n\t"
               "buffer_load_dwordx2 %7, %8, %9, 0 offen offset:224"
               : "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4]), "=&v"(b[5]), "=&v"(b[6]),
                 "=&v"(b[7])
               : "v"(vo), "s"(rs)
               : "memory");
}
__device__ __forceinline__ void preload_round1(u16x8 (&t)[8], const bf16_t* src, int64_t ldc, int m0, int n0,
                                               uint32_t vo) {
  const v4i rs = scalar_rsrc(src + (int64_t)m0 * ldc + n0, (uint32_t)((255 * ldc + 256) * 2));
  const uint32_t l2 = (uint32_t)ldc * 2u;
  asm volatile("buffer_load_dwordx4 %0, %8, %9, %10 offen\n\t"
               "buffer_load_dwordx4 %1, %8, %9, %11 offen\n\t"
               "buffer_load_dwordx4 %2, %8, %9, %12 offen\n\t"
               "buffer_load_dwordx4 %3, %8, %9, %13 offen\n\t"
               "buffer_load_dwordx4 %4, %8, %9, %14 offen\n\t"
               "buffer_load_dwordx4 %5, %8, %9, %15 offen\n\t"
               "buffer_load_dwordx4 %6, %8, %9, %16 offen\n\t"
               "buffer_load_dwordx4 %7, %8, %9, %17 offen"
               : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6]),
                 "=&v"(t[7])
               : "v"(vo), "s"(rs), "s"(32 * l2), "s"(34 * l2), "s"(36 * l2), "s"(38 * l2), "s"(40 * l2),
                 "s"(42 * l2), "s"(44 * l2), "s"(46 * l2)
               : "memory");
}
template <class V, int N>
__device__ __forceinline__ void settle(V (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(x[i]));
}

// Per-item operands of the main-loop / next-item statements (gen_gemm_kloop.py): buffer resources of the item's
// A and B K-tile 0 (every value wave-uniform: kernel arguments, blockIdx, the item index, the wave index).
template <int LAYOUT>
struct ItemOps {
  int tm, tn, m0, n0, split, T;
  uint32_t alo, ahi, blo, bhi;
  __device__ __forceinline__ void init(const GemmArgs& p, int item, int ntiles) {
    split = item / ntiles;
    tile_of(p, item - split * ntiles, ntiles, tm, tn);
    m0 = tm * TM; n0 = tn * TN;
    const int kbeg = split * p.k_per_split;
    T = min(p.K - kbeg, p.k_per_split) / KB;
    uint64_t a0, b0;
    if (LAYOUT == L_NT) {
      a0 = (uint64_t)(uintptr_t)p.A + ((uint64_t)m0 * p.lda + kbeg) * 2;
      b0 = (uint64_t)(uintptr_t)p.B + ((uint64_t)n0 * p.ldb + kbeg) * 2;
    } else {
      a0 = (uint64_t)(uintptr_t)p.A + ((uint64_t)kbeg * p.lda + m0) * 2;
      b0 = (uint64_t)(uintptr_t)p.B + ((uint64_t)kbeg * p.ldb + n0) * 2;
    }
    alo = (uint32_t)a0; ahi = (uint32_t)(a0 >> 32) & 0xffffu;
    blo = (uint32_t)b0; bhi = (uint32_t)(b0 >> 32) & 0xffffu;
  }
  // the same item's K-tile n (skip2: its tiles 0 and 1 were issued by the previous item's epilogue)
  __device__ __forceinline__ void skip2(uint64_t astep, uint64_t bstep) { skipn(2 * astep, 2 * bstep); }
  __device__ __forceinline__ void skip1(uint64_t astep, uint64_t bstep) { skipn(astep, bstep); }
  __device__ __forceinline__ void skipn(uint64_t da, uint64_t dbb) {
    const uint64_t a = (((uint64_t)ahi << 32) | alo) + da, b = (((uint64_t)bhi << 32) | blo) + dbb;
    alo = (uint32_t)a; ahi = (uint32_t)(a >> 32) & 0xffffu;
    blo = (uint32_t)b; bhi = (uint32_t)(b >> 32) & 0xffffu;
  }
};

// Persistent: a workgroup walks items (tile, K split) id = blockIdx.x + i * gridDim.x.  When the K-step count is
// even, an item's last two K-steps DMA the NEXT item's K-tiles 0 and 1 into the ring (gen_gemm_kloop.py
// next_tail), so those loads fly under this item's last MFMAs and its epilogue; the epilogue stages its bf16
// results through the 32 KiB of LDS past the ring (4 rounds of 64 rows, full-row 16-byte stores) and the stores
// drain under the next item's first K-steps (its first wait counts them: vmcnt(16 + stores)).
// DIAG = 1 (diagnostic builds only, pdt_gemm_stamps_bf16): wave 0 stamps s_memtime at each item's start, after
// its main loop and after its epilogue into p.ws (uint64 [item][8]: [3] = s_memrealtime at item start, [4..7] =
// the stamped loop's own phase stamps: start, prologue wait done, first K-step done, tail entry)
// -- for the phase shares of an item, never for timing the production kernel.
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  return t;
}

template <int LAYOUT, int EPI, int DIAG = 0, bool P3 = false>
__global__ __launch_bounds__(NTH, 1) void gemm_asm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM3];
  const uint32_t lds_addr = (uint32_t)(uintptr_t)(lds_void*)smem;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wr = w >> 1, wc = w & 1;
  const int wv = __builtin_amdgcn_readfirstlane(w);   // the wave index in an SGPR (see item_tid)
  const int ntiles = (p.M / TM) * (p.N / TN);
  const int splits = (p.K + p.k_per_split - 1) / p.k_per_split;
  const int nall = ntiles * splits;

  // ---- item-independent operands (scalar)
  uint64_t astep, bstep;
  uint32_t abytes, bbytes, rsa, rsb;
  int32_t db;
  if (LAYOUT == L_NT) {
    astep = bstep = KB * 2;
    abytes = (uint32_t)((TM - 1) * p.lda * 2 + KB * 2);
    bbytes = (uint32_t)((TN - 1) * p.ldb * 2 + KB * 2);
    rsa = (uint32_t)(32 * p.lda * 2);
    rsb = (uint32_t)(32 * p.ldb * 2);
    db = OPB + 16384 * (wc - wr);
  } else {
    astep = (uint64_t)KB * p.lda * 2;
    bstep = (uint64_t)KB * p.ldb * 2;
    abytes = (uint32_t)((KB - 1) * p.lda * 2 + TM * 2);
    bbytes = (uint32_t)((KB - 1) * p.ldb * 2 + TN * 2);
    rsa = (uint32_t)(8 * p.lda * 2);
    rsb = (uint32_t)(8 * p.ldb * 2);
    db = OPB + 256 * (wc - wr);
  }
  // per-lane operands of the main-loop statement (DMA source offsets, LDS read addresses) from thread id t --
  // evaluated every item from an opaque copy of the thread id, so nothing per-lane stays live across the epilogue
  // (where it would be spilled, and its reload's vmcnt(0) would drain the next item's prefetched K-tiles and the
  // epilogue's stores in front of every main loop)
  auto lane_ops = [&](int t, uint32_t& voa0, uint32_t& voa1, uint32_t& vob0, uint32_t& vob1, uint32_t& rd0,
                      uint32_t& rd1) {
    const int lw = t >> 6, ll = t & 63, lwr = lw >> 1;
    if (LAYOUT == L_NT) {
      const int row = 8 * lw + (ll >> 3);
      const int c = (ll & 7) ^ ((row >> 1) & 7);
      voa0 = voa1 = (uint32_t)(row * p.lda * 2 + c * 16);
      vob0 = vob1 = (uint32_t)(row * p.ldb * 2 + c * 16);
      const int x = ll & 15, g = ll >> 4, h = (x >> 1) & 7;
      rd0 = lds_addr + 16384 * lwr + (uint32_t)(x * 128 + 16 * (g ^ h));
      rd1 = lds_addr + 16384 * lwr + (uint32_t)(x * 128 + 16 * ((4 + g) ^ h));
    } else {
      const int r0 = 2 * lw + (ll >> 5);
      voa0 = (uint32_t)(r0 * p.lda * 2 + ((ll & 31) ^ tt_f(r0)) * 16);
      voa1 = (uint32_t)(r0 * p.lda * 2 + ((ll & 31) ^ tt_f(r0 + 8)) * 16);
      vob0 = (uint32_t)(r0 * p.ldb * 2 + ((ll & 31) ^ tt_f(r0)) * 16);
      vob1 = (uint32_t)(r0 * p.ldb * 2 + ((ll & 31) ^ tt_f(r0 + 8)) * 16);
      const int g = ll >> 4, q = (ll >> 2) & 3, pp = ll & 3;
      rd0 = lds_addr + 256 * lwr + (uint32_t)((8 * g + q) * 512 + 16 * (pp >> 1) + 8 * (pp & 1));
      rd1 = (uint32_t)tt_f(8 * g + q);     // the block XOR term
    }
  };
  const uint32_t m0b = __builtin_amdgcn_readfirstlane(lds_addr + w * 1024);
  const int dbs = __builtin_amdgcn_readfirstlane(db);
  const uint32_t asl = (uint32_t)astep, ash = (uint32_t)(astep >> 32);
  const uint32_t bsl = (uint32_t)bstep, bsh = (uint32_t)(bstep >> 32);
  // vector-memory ops an epilogue (and the next item's pre-loop loads: round-0 aux DMA + round-1 rows, bias) issues
  // after the next item's first DMA: the next main loop's first wait skips them (vmcnt counts in issue order; a
  // smaller count only waits more)
  constexpr int NST = EPI == E_F32 ? 64 : EPI == E_GELU ? 64 + 8 : EPI == E_DGELU ? 32 + 1 + 8 + 8 : EPI == E_BIAS ? 40 : 32;
  constexpr int WNX = 16 + NST < 63 ? 16 + NST : 63;
  char* const img = smem + RING;

#define PDT_KLOOP_CLOBBERS                                                                                      \
  "memory", "scc", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91",         \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78",     \
  "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93",     \
  "v94", "v95", "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", "v138", "v139", \
  "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151", "v152",      \
  "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163", "v164", "v165",      \
  "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", "v174", "v175", "v176", "v177", "v178",      \
  "v179", "v180", "v181", "v182", "v183", "v184", "v185", "v186", "v187", "v188", "v189", "v190", "v191",      \
  "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199", "v200", "v201", "v202", "v203", "v204",      \
  "v205", "v206", "v207", "v208", "v209", "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217",      \
  "v218", "v219", "v220", "v221", "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230",      \
  "v231", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243",      \
  "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255",              \
  PDT_AGPR_CLOBBERS
#define PDT_ITEM_OPS                                                                                            \
  [alo] "s"(lo.alo), [ahi] "s"(lo.ahi), [anr] "s"(abytes), [blo] "s"(lo.blo), [bhi] "s"(lo.bhi),               \
      [bnr] "s"(bbytes), [m0b] "s"(m0b), [rsa] "s"(rsa), [rsb] "s"(rsb), [asl] "s"(asl), [ash] "s"(ash),         \
      [bsl] "s"(bsl), [bsh] "s"(bsh), [cnt] "s"(cnt), [first] "s"(first), [wnx] "i"(WNX), [hnx] "s"(hnx),        \
      [nalo] "s"(nxt.alo), [nahi] "s"(nxt.ahi), [nblo] "s"(nxt.blo), [nbhi] "s"(nxt.bhi), [db] "s"(dbs)
#define PDT_KLOOP_NT_ASM(MAC)                                                                                     \
  asm volatile(MAC : : PDT_ITEM_OPS, [voa] "v"(voa0), [vob] "v"(vob0), [rd0] "v"(rd0), [rd1] "v"(rd1)           \
               : PDT_KLOOP_CLOBBERS)
#define PDT_KLOOP_TT_ASM(MAC)                                                                                     \
  asm volatile(MAC : : PDT_ITEM_OPS, [voa0] "v"(voa0), [voa1] "v"(voa1), [vob0] "v"(vob0), [vob1] "v"(vob1),    \
               [rd0] "v"(rd0), [rdx] "v"(rd1) : PDT_KLOOP_CLOBBERS)
// P3: the 3-stage A-ring program (gen_gemm_kloop.py Gen3) also uses v96.. for its third A buffer's read addresses
#define PDT_KLOOP_NT_ASM3(MAC)                                                                                    \
  asm volatile(MAC : : PDT_ITEM_OPS, [voa] "v"(voa0), [vob] "v"(vob0), [rd0] "v"(rd0), [rd1] "v"(rd1)           \
               : PDT_KLOOP_CLOBBERS, "v96", "v97")
#define PDT_KLOOP_TT_ASM3(MAC)                                                                                    \
  asm volatile(MAC : : PDT_ITEM_OPS, [voa0] "v"(voa0), [voa1] "v"(voa1), [vob0] "v"(vob0), [vob1] "v"(vob1),    \
               [rd0] "v"(rd0), [rdx] "v"(rd1)                                                                    \
               : PDT_KLOOP_CLOBBERS, "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103")
// DIAG: the stamped loop (gen_gemm_kloop.py *_STAMPS) hands its 4 phase stamps out as 8 SGPR halves
#define PDT_STAMP_OUTS                                                                                            \
  [st0] "=s"(ph[0]), [st1] "=s"(ph[1]), [st2] "=s"(ph[2]), [st3] "=s"(ph[3]), [st4] "=s"(ph[4]),               \
      [st5] "=s"(ph[5]), [st6] "=s"(ph[6]), [st7] "=s"(ph[7])
#define PDT_KLOOP_NT_ASM_ST(MAC)                                                                                  \
  asm volatile(MAC : PDT_STAMP_OUTS : PDT_ITEM_OPS, [voa] "v"(voa0), [vob] "v"(vob0), [rd0] "v"(rd0),            \
               [rd1] "v"(rd1) : PDT_KLOOP_CLOBBERS, "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99")
#define PDT_KLOOP_TT_ASM_ST(MAC)                                                                                  \
  asm volatile(MAC : PDT_STAMP_OUTS : PDT_ITEM_OPS, [voa0] "v"(voa0), [voa1] "v"(voa1), [vob0] "v"(vob0),         \
               [vob1] "v"(vob1), [rd0] "v"(rd0), [rdx] "v"(rd1)                                                  \
               : PDT_KLOOP_CLOBBERS, "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99")

  // (Workgroups run their items in near lockstep, so their epilogues' stores arrive together; delaying phase groups
  // of them by 6-24 us at start measured 1-4 % SLOWER on c_fc / c_proj, profiles/r5/r5p_gemm_stagger_ab.txt: the
  // lockstep walk is what lets an XCD's workgroups share A / B panels in L2.)
  ItemOps<LAYOUT> cur;
  int item = blockIdx.x;
  cur.init(p, item, ntiles);
  int first = 1;
  while (true) {
    const int next_item = item + (int)gridDim.x;
    const bool has_next = next_item < nall;
    ItemOps<LAYOUT> nxt = cur;
    if (has_next) {
      GemmArgs q = p;                    // tile-walk divisors opaque per item (opaque_s)
      q.M = opaque_s(p.M); q.N = opaque_s(p.N); q.xpr = opaque_s(p.xpr); q.grp = opaque_s(p.grp);
      q.K = opaque_s(p.K); q.k_per_split = opaque_s(p.k_per_split);
      nxt.init(q, next_item, opaque_s(ntiles));
    }
    // the last two K-steps load the next item's first two K-tiles (even K-step counts only: stage parity)
    // integer arithmetic, not a select: a bool-derived operand can be rematerialised as a VGPR v_cndmask
    // (P3, the 3-stage program: no next-item prefetch -- every item runs its own prologue)
    const int hnx = P3 ? 0 : __builtin_amdgcn_readfirstlane((((nall - 1 - next_item) >> 31) + 1) & ~cur.T & 1);
    const int cnt = __builtin_amdgcn_readfirstlane(cur.T);
    first = __builtin_amdgcn_readfirstlane(first);
    // the main loop's own DMA starts at K-tile 2 when the previous item's last K-steps issued tiles 0 and 1
    ItemOps<LAYOUT> lo = cur;
    if (!first) lo.skip2(astep, bstep);
    lo.alo = __builtin_amdgcn_readfirstlane(lo.alo); lo.ahi = __builtin_amdgcn_readfirstlane(lo.ahi);
    lo.blo = __builtin_amdgcn_readfirstlane(lo.blo); lo.bhi = __builtin_amdgcn_readfirstlane(lo.bhi);
    uint64_t st0 = 0, st1 = 0, rt0 = 0;
    if (DIAG) { st0 = stamp(); rt0 = __builtin_amdgcn_s_memrealtime(); }
    const int ltid = item_tid(wv);     // per-item lane terms (lane_ops)
    uint32_t voa0, voa1, vob0, vob1, rd0, rd1;
    lane_ops(ltid, voa0, voa1, vob0, vob1, rd0, rd1);
    // DGELU: this item's round-0 derivative rows into the (idle) staging image under the main loop, round 1 into
    // registers; bias epilogues: the bias columns (preload_*)
    u16x4 pb[8];
    u16x8 pa[8];
    if constexpr (EPI == E_DGELU) {
      stg_dma_round0(p.aux, p.ldc, cur.m0, cur.n0, lds_addr + RING, ltid >> 6, ltid & 63);
      preload_round1(pa, p.aux, p.ldc, cur.m0, cur.n0, stg_voff(p.ldc, ltid >> 6, ltid & 63));
    }
    if constexpr (EPI == E_BIAS || EPI == E_GELU) preload_bias(pb, p.bias, cur.n0, 128 * ((ltid >> 6) & 1) + 4 * ((ltid & 63) >> 4));
    // ---------------------------------------------------------------- main loop
    uint32_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (DIAG) {
      if constexpr (LAYOUT == L_NT) PDT_KLOOP_NT_ASM_ST(PDT_GEMM_KLOOP_NT_STAMPS);
      else PDT_KLOOP_TT_ASM_ST(PDT_GEMM_KLOOP_TT_STAMPS);
    } else if constexpr (P3) {
      if constexpr (LAYOUT == L_NT) PDT_KLOOP_NT_ASM3(PDT_GEMM_KLOOP_NT3);
      else PDT_KLOOP_TT_ASM3(PDT_GEMM_KLOOP_TT3);
    } else {
      if constexpr (LAYOUT == L_NT) PDT_KLOOP_NT_ASM(PDT_GEMM_KLOOP_NT);
      else PDT_KLOOP_TT_ASM(PDT_GEMM_KLOOP_TT);
    }
    if constexpr (EPI == E_DGELU) settle(pa);
    if constexpr (EPI == E_BIAS || EPI == E_GELU) settle(pb);
    if (DIAG) st1 = stamp();
    const int m0 = cur.m0, n0 = cur.n0, tm = cur.tm;

    // The epilogue's lane terms are recomputed every item from an opaque copy of the thread id: hoisted out of the
    // persistent loop they stay live across the main-loop statement (which leaves the compiler 96 VGPRs) and spill
    // to scratch -- the DGELU kernel spilled 46 VGPRs that way, reloaded from scratch in every epilogue.
    const int etid = item_tid(wv);
    {
    const int tid = etid, w = etid >> 6, lane = etid & 63, wr = w >> 1, wc = w & 1;
    const int lrow = 128 * wr + (lane & 15);
    const int lcol = 128 * wc + 4 * (lane >> 4);
    // ---------------------------------------------------------------- epilogue
    // acc tile (i, j): C[m0 + 128 wr + 16 i + (lane & 15)][n0 + 128 wc + 16 j + 4 (lane >> 4) + r]
    if constexpr (EPI == E_F32) {
      float* C = p.ws + (int64_t)cur.split * p.M * p.N;
      sfor<0, 64>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const f32x4 v = acc_tile<k>();
        *reinterpret_cast<f32x4*>(C + (int64_t)(m0 + lrow + 16 * (k >> 3)) * p.N + n0 + lcol + 16 * (k & 7)) = v;
      });
    } else {
      bf16_t* C = reinterpret_cast<bf16_t*>(p.C);
      u16x8 buf[8];
      float bj[8][4];
      if constexpr (EPI == E_BIAS || EPI == E_GELU) {   // loaded before the main loop (preload_bias)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) bj[j][r] = bf2f(pb[j][r]);
      }
      float cs[8][4];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
      // round r: this wave's accumulator tiles i = 2 r, 2 r + 1 -> image rows q = 32 wr + 16 (i & 1) + (lane & 15)
      // DGELU: the derivative rows of round 0 are already in the image (stg_dma_round0 under the main loop); rounds
      // 1-3 are fetched into registers a round ahead of their use
      u16x8 aux[2][8];                       // round r in aux[r & 1]: round 1 loaded before the main loop, 2 and 3
      const uint32_t svo = stg_voff(p.ldc, w, lane), ldc2 = (uint32_t)(p.ldc * 2);   // a round ahead
      const __amdgpu_buffer_rsrc_t rsc = tile_rsrc(C, p.ldc, m0, n0);
      if constexpr (EPI == E_DGELU) {
#pragma unroll
        for (int it = 0; it < 8; ++it) aux[1][it] = pa[it];
      }
      sfor<0, 4>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if constexpr (EPI == E_DGELU && r > 0) {
          __syncthreads();                   // the previous round's image is read
          stg_put(img, aux[r & 1], w, lane);
          if constexpr (r < 3) stg_fetch(aux[(r + 1) & 1], tile_rsrc(p.aux, p.ldc, m0, n0), svo, ldc2, r + 1);
        }
        __syncthreads();
        u16x4 dk[16];                        // GELU: this round's derivatives, written out after the values
        u16x4 hk[8];                         // DGELU: 8 tiles' derivatives read before their first write (a
                                             // read-after-write order would serialise 16 LDS round trips)
        sfor<0, 16>([&](auto kc) {
          constexpr int kk = decltype(kc)::value, k = 16 * r + kk, i = k >> 3, j = k & 7;
          if constexpr (EPI == E_DGELU && (kk & 7) == 0) {
            sfor<0, 8>([&](auto hc) {
              constexpr int k2 = k + decltype(hc)::value, i2 = k2 >> 3, j2 = k2 & 7;
              hk[decltype(hc)::value] = *reinterpret_cast<const u16x4*>(
                  img + stg_off(32 * wr + 16 * (i2 & 1) + (lane & 15), lcol + 16 * j2));
            });
          }
          const f32x4 v = acc_tile<k>();
          const uint32_t at = stg_off(32 * wr + 16 * (i & 1) + (lane & 15), lcol + 16 * j);
          u16x4 o;
          if constexpr (EPI == E_DGELU) {
            const u16x4 hh = hk[kk & 7];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bf16_t gb = f2bf(v[e] * bf2f(hh[e]));
              o[e] = gb;
              cs[j][e] += bf2f(gb);          // the bias gradient sums the gradient as stored
            }
          } else if constexpr (EPI == E_GELU) {
            // value and derivative of the rounded pre-activation, two per packed instruction (gelu.h)
#pragma unroll
            for (int e = 0; e < 4; e += 2) {
              gelu_f32x2 y2, d2;
              gelu_fwd_grad2(gelu_f32x2{bf2f(f2bf(v[e] + bj[j][e])), bf2f(f2bf(v[e + 1] + bj[j][e + 1]))}, y2, d2);
              o[e] = f2bf(y2[0]); o[e + 1] = f2bf(y2[1]);
              dk[kk][e] = f2bf(d2[0]); dk[kk][e + 1] = f2bf(d2[1]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f2bf(EPI == E_BIAS ? v[e] + bj[j][e] : v[e]);
          }
          *reinterpret_cast<u16x4*>(img + at) = o;
        });
        __syncthreads();
        stg_read(img, buf, w, lane);
        stg_write_out(buf, rsc, svo, ldc2, r);
        if constexpr (EPI == E_GELU) {       // then the derivatives, same rows
          __syncthreads();
          sfor<0, 16>([&](auto kc) {
            constexpr int kk = decltype(kc)::value, k = 16 * r + kk, i = k >> 3, j = k & 7;
            const uint32_t at = stg_off(32 * wr + 16 * (i & 1) + (lane & 15), lcol + 16 * j);
            *reinterpret_cast<u16x4*>(img + at) = dk[kk];
          });
          __syncthreads();
          stg_read(img, buf, w, lane);
          stg_write_out(buf, tile_rsrc(p.aux_out, p.ldc, m0, n0), svo, ldc2, r);
        }
      });
      if constexpr (EPI == E_DGELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) cs[j][e] = row16_sum(cs[j][e]);
        __syncthreads();                                   // the last round's image is read
        float* red = reinterpret_cast<float*>(img);        // [2 wave rows][256 columns]
        if ((lane & 15) == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[wr * 256 + lcol + 16 * j + e] = cs[j][e];
        }
        __syncthreads();
        p.ws[(int64_t)tm * p.N + n0 + tid] = red[tid] + red[256 + tid];
      }
      __syncthreads();                       // the staging image is free for the next item's epilogue
    }
    }   // epilogue lane terms
    if (DIAG) {
      const uint64_t st2 = stamp();
      if (tid == 0) {
        uint64_t* d = reinterpret_cast<uint64_t*>(p.ws) + 8 * (int64_t)item;
        d[0] = st0; d[1] = st1; d[2] = st2; d[3] = rt0;
        for (int i = 0; i < 4; ++i) d[4 + i] = ((uint64_t)ph[2 * i + 1] << 32) | ph[2 * i];
      }
    }
    if (!has_next) break;
    item = next_item;
    first = 1 - hnx;
    cur = nxt;
  }
#undef PDT_KLOOP_CLOBBERS
#undef PDT_ITEM_OPS
#undef PDT_KLOOP_NT_ASM3
#undef PDT_KLOOP_TT_ASM3
#undef PDT_KLOOP_NT_ASM_ST
#undef PDT_KLOOP_TT_ASM_ST
#undef PDT_STAMP_OUTS
#undef PDT_KLOOP_NT_ASM
#undef PDT_KLOOP_TT_ASM
}

// one workgroup per CU (all 160 KiB of LDS each) walking its items; a multiple of 8 (tile ids b, b + 8 share an XCD)
static int persist_grid(int nitems) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      n = 256;
    return n;
  }();
  int g = cus < nitems ? cus : nitems;
  return g >= 8 ? g & ~7 : g;
}

// The 3-stage program (two K-steps of DMA lead for A) where it measured faster (profiles/r4/r4_gemm_p3_ab.log, one
// process, interleaved rounds): NT with K >= 8192 per item (c_proj forward shape 1,467 -> 1,589 TFLOP/s, 8192^3
// 1,549 -> 1,619: hipBLASLt parity) and TT with more items than workgroups (qkv weight gradient 1,361 -> 1,422);
// the one-item-per-workgroup TT shapes ran 3-7 % slower with it.  Needs >= 6 K-steps per item; gives up the
// next-item prefetch.  PDT_GEMM_P3=0 / 1 forces it off / on (A/B runs).
bool use_p3(int layout, const GemmArgs& a, int items, int grid) {
  static const int forced = [] { const char* e = getenv("PDT_GEMM_P3"); return e ? atoi(e) : -1; }();
  const int T = a.k_per_split / KB;
  if (T < 6 || forced == 0) return false;
  if (forced == 1) return true;
  // NT: also every product whose XCD block is <= 8 tiles wide (A panels barely reused, i.e. streamed): attention
  // projection 1,338 -> 1,382, the qkv data gradient (K = 6144) 1,298 -> 1,492 (r4_gemm_p3_nt_shapes_ab.log); wide
  // blocks (c_fc, qkv forward: A re-read from L2) keep the 2-stage program and its next-item prefetch
  const int cb = a.xpr > 0 ? (a.N / TN) / (8 / a.xpr) : a.N / TN;
  // TT: only where the token split made the extra items (output below one wave of tiles: the qkv weight
  // gradient); a many-tile output -- the tied LM head's 1,568 tiles x 2 splits -- ran 7 % slower with it
  // (15.3 vs 16.4 ms, profiles/r4/r4_lm_head_wgrad_ab.jsonl)
  return layout == L_TT ? (items > grid && (a.M / TM) * (a.N / TN) < grid) : (a.k_per_split >= 8192 || cb <= 8);
}

template <int LAYOUT>
int launch_asm_layout(int epi, const GemmArgs& a, int splits, hipStream_t s) {
  const int items = (a.M / TM) * (a.N / TN) * splits;
  const dim3 grid(persist_grid(items), 1);
  if (use_p3(LAYOUT, a, items, (int)grid.x) && (epi == E_PLAIN || epi == E_BIAS || epi == E_F32)) {
    switch (epi) {   // (GELU / DGELU epilogues keep the 2-stage program)
      case E_PLAIN: gemm_asm_kernel<LAYOUT, E_PLAIN, 0, true><<<grid, NTH, 0, s>>>(a); break;
      case E_BIAS: gemm_asm_kernel<LAYOUT, E_BIAS, 0, true><<<grid, NTH, 0, s>>>(a); break;
      default: gemm_asm_kernel<LAYOUT, E_F32, 0, true><<<grid, NTH, 0, s>>>(a); break;
    }
    return (int)hipGetLastError();
  }
  switch (epi) {
    case E_PLAIN: gemm_asm_kernel<LAYOUT, E_PLAIN><<<grid, NTH, 0, s>>>(a); break;
    case E_BIAS: gemm_asm_kernel<LAYOUT, E_BIAS><<<grid, NTH, 0, s>>>(a); break;
    case E_GELU: gemm_asm_kernel<LAYOUT, E_GELU><<<grid, NTH, 0, s>>>(a); break;
    case E_DGELU: gemm_asm_kernel<LAYOUT, E_DGELU><<<grid, NTH, 0, s>>>(a); break;
    case E_F32: gemm_asm_kernel<LAYOUT, E_F32><<<grid, NTH, 0, s>>>(a); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
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


// rows per group of tile_of's walk, dividing the block's rows.  Measured on the flagship's NT shapes
// (profiles/r4/r4_gemm_grp_ab.log, PDT_GEMM_GRP forces one): short K (<= 4096: the A panels of an item are
// small) runs best on 8-row groups -- c_fc 1,228 -> 1,446 TFLOP/s, qkv 1,307 -> 1,427, attention projection
// 1,302 -> 1,367 -- long K on 4-row ones (4 x 8 tiles in flight per XCD; 8-row groups lose 2-8 % there)
int xcd_grp(int mt, int nt, int K, int xpr) {
  if (xpr <= 0) return 1;
  const int rb = mt / xpr, cb = nt / (8 / xpr);
  static const int forced = [] { const char* e = getenv("PDT_GEMM_GRP"); return e ? atoi(e) : 0; }();
  if (forced > 0 && rb % forced == 0) return forced;
  const int pref[3] = {K <= 4096 ? 8 : 4, K <= 4096 ? 4 : 8, 2};
  for (int g : pref)
    if (rb % g == 0 && g * cb >= 16) return g;
  return 1;
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
// GELU derivative, dbias = column sums of the result; ws >= (M / 256 + 64) * N floats), 4 is internal.
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
  a.grp = xcd_grp((int)(M / TM), (int)(N / TN), (int)(K / splits), a.xpr);
  const int run_epi = splits > 1 ? E_F32 : epi;
  if (splits > 1) a.ldc = N;
  int err = layout == L_NT ? launch_layout<L_NT>(run_epi, a, splits, s) : launch_layout<L_TT>(run_epi, a, splits, s);
  if (err) return err;
  if (splits > 1) {
    const int64_t n4 = M * N / 4;
    gemm_splitk_reduce_kernel<<<grid_for(n4, 256, 256 * 16), 256, 0, s>>>(ws, (bf16_t*)C, n4, splits, M * N);
    if (ldc != N) return (int)hipErrorInvalidValue;   // slab reduce writes a dense [M, N]
  }
  if (epi == E_DGELU)   // dbias = the R = M / 256 tile partials summed in a fixed two-level order (deterministic);
    // a one-level pass (one thread per column, 32 workgroups at N = 8192) ran 0.15 ms: latency-bound
    red::col_reduce<bf16_t>(ws, (int)(M / TM), (int)N, (bf16_t*)dbias, ws + (M / TM) * N, 0, s);
  return (int)hipGetLastError();
}

// The hand-scheduled main loop (gemm_asm_kernel): same contract as pdt_gemm_bf16, plus K / splits >= 128 and
// ldc % 8 == 0 (16-byte epilogue stores).
PDT_API int pdt_gemm2_bf16(int layout, int epi, const void* A, const void* B, void* C, int64_t M, int64_t N,
                           int64_t K, int64_t lda, int64_t ldb, int64_t ldc, const void* bias, const void* aux,
                           void* aux_out, void* dbias, float* ws, int splits, hipStream_t s) {
  if (!pdt_gemm_ok(layout, M, N, K, lda, ldb, splits) || ldc < N || ldc % 8) return (int)hipErrorInvalidValue;
  if (K / splits < 2 * KB) return (int)hipErrorInvalidValue;
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
  a.grp = xcd_grp((int)(M / TM), (int)(N / TN), (int)(K / splits), a.xpr);
  const int run_epi = splits > 1 ? E_F32 : epi;
  if (splits > 1) a.ldc = N;
  int err = layout == L_NT ? launch_asm_layout<L_NT>(run_epi, a, splits, s)
                           : launch_asm_layout<L_TT>(run_epi, a, splits, s);
  if (err) return err;
  if (splits > 1) {
    if (ldc != N) return (int)hipErrorInvalidValue;
    const int64_t n4 = M * N / 4;
    gemm_splitk_reduce_kernel<<<grid_for(n4, 256, 256 * 16), 256, 0, s>>>(ws, (bf16_t*)C, n4, splits, M * N);
  }
  if (epi == E_DGELU)   // dbias = the R = M / 256 tile partials summed in a fixed two-level order (deterministic);
    // a one-level pass (one thread per column, 32 workgroups at N = 8192) ran 0.15 ms: latency-bound
    red::col_reduce<bf16_t>(ws, (int)(M / TM), (int)N, (bf16_t*)dbias, ws + (M / TM) * N, 0, s);
  return (int)hipGetLastError();
}

PDT_API int pdt_gemm_stamps_epi_bf16(int layout, int epi, const void* A, const void* B, void* C, int64_t M, int64_t N,
                                     int64_t K, int64_t lda, int64_t ldb, const void* bias, void* aux_out,
                                     void* stamps, hipStream_t s);
// Instrumented build (results unchanged): the plain-epilogue kernel with phase stamps (DIAG above) into `stamps`
// (uint64 [items][4]) -- scripts/gemm_stamps.py.
PDT_API int pdt_gemm_stamps_bf16(int layout, const void* A, const void* B, void* C, int64_t M, int64_t N, int64_t K,
                                 int64_t lda, int64_t ldb, void* stamps, hipStream_t s) {
  if (!pdt_gemm_ok(layout, M, N, K, lda, ldb, 1) || K < 2 * KB || !stamps) return (int)hipErrorInvalidValue;
  return pdt_gemm_stamps_epi_bf16(layout, E_PLAIN, A, B, C, M, N, K, lda, ldb, nullptr, nullptr, stamps, s);
}

// The same for the bias / GELU epilogues (NT only): bias [N], aux_out [M, N] (GELU's derivative)
PDT_API int pdt_gemm_stamps_epi_bf16(int layout, int epi, const void* A, const void* B, void* C, int64_t M, int64_t N,
                                     int64_t K, int64_t lda, int64_t ldb, const void* bias, void* aux_out,
                                     void* stamps, hipStream_t s) {
  if (!pdt_gemm_ok(layout, M, N, K, lda, ldb, 1) || K < 2 * KB || !stamps) return (int)hipErrorInvalidValue;
  if (epi != E_PLAIN && (layout != L_NT || !bias || (epi == E_GELU && !aux_out) || (epi != E_BIAS && epi != E_GELU)))
    return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.B = (const bf16_t*)B; a.C = C; a.ws = (float*)stamps;
  a.bias = (const bf16_t*)bias; a.aux_out = (bf16_t*)aux_out;
  a.M = (int)M; a.N = (int)N; a.K = (int)K; a.lda = lda; a.ldb = ldb; a.ldc = N; a.k_per_split = (int)K;
  a.xpr = xcd_cut((int)(M / TM), (int)(N / TN));
  a.grp = xcd_grp((int)(M / TM), (int)(N / TN), (int)K, a.xpr);
  const dim3 grid(persist_grid((int)((M / TM) * (N / TN))), 1);
  if (layout == L_TT) gemm_asm_kernel<L_TT, E_PLAIN, 1><<<grid, NTH, 0, s>>>(a);
  else if (epi == E_BIAS) gemm_asm_kernel<L_NT, E_BIAS, 1><<<grid, NTH, 0, s>>>(a);
  else if (epi == E_GELU) gemm_asm_kernel<L_NT, E_GELU, 1><<<grid, NTH, 0, s>>>(a);
  else gemm_asm_kernel<L_NT, E_PLAIN, 1><<<grid, NTH, 0, s>>>(a);
  return (int)hipGetLastError();
}
