// Causal / full flash attention (forward + backward) for gfx950, bf16 in/out, fp32 softmax state.
// Head dims 64 and 128, GQA (H % Hkv == 0), strided q/k/v so a fused [B, S, 3, H, D] projection
// is consumed in place.
//
// Built on v_mfma_f32_32x32x16_bf16 with the "accumulator as the next MFMA's operand" idiom
// (cdna_hip_programming.md §3): scores are computed transposed (S^T = K Q^T) so that each lane owns
// one query row -- the softmax max/sum are lane-local (+ one xor-32 exchange), and the probability
// registers are reused directly as the B operand of O^T += V^T P^T with no LDS round trip.  The
// key order inside each 16-key MFMA step is the permutation that idiom implies
// (key = 16s + 8(j>>2) + 4h + (j&3)); the A operands that pair with it (V^T, dO^T, Q^T, K^T) are
// staged TRANSPOSED in LDS with a +4-element row pad (136-B stride: conflict-free 8-B reads), and the
// row-major operands (K, V, Q, dO) are staged with a 16-B-chunk XOR swizzle (conflict-free b128 reads).
//
// Forward (v5, default): workgroup = 4 waves x 32 query rows (BM = 128), 64-key tiles DMA'd into an LDS
// ring overlapping the current tile's MFMAs, heavy (diagonal-rich) blocks launched first under the causal
// mask; alternative v7: the same tile on 8 waves x 32 rows (256 rows share each staged K/V tile).
// Backward: FA2-style split into (a) the dQ kernel (workgroup owns 128 / 256 query rows; it also computes
// delta = rowsum(dO*O) for its rows and hands it on), (b) the dK/dV kernel (workgroup owns 128 keys of one
// kv head and sweeps every query head of its GQA group, so dK/dV need no cross-workgroup sum).  No
// atomics: bitwise deterministic.  Selection: ops/attention.py set_kernel_variant.
//
// Used by the GPT-2 / Llama models (BASELINE.json configs 3-5; SURVEY.md K16 "flash attention
// (causal, head_dim 64/128)").
#include "common.h"
#include "reduce.h"
#include <stdlib.h>

using namespace pdt;

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int NT = 256;
constexpr int TILE = 64;          // rows per staged LDS tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma32(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// Accumulate into an AGPR-resident tile.  Used for long-lived accumulators that only MFMAs touch until
// the epilogue (dK/dV, dQ): the file is built with the MFMA VGPR form, which would otherwise put them in
// the 256 arch VGPRs next to the softmax tiles and leave no room for operand prefetch.  Callers must run
// acc_fence() before VALU reads the tile (the hazard recognizer does not see through inline asm).
__device__ __forceinline__ void mfma32_acc(f32x16& acc, const u16x8& a, const u16x8& b) {
  asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void acc_fence() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// accumulator register r of a 32x32 tile, lane half h -> row index inside the tile
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Row-major bf16 tile image [TILE][D] with a 16-byte-chunk XOR swizzle that is conflict-free for BOTH
// access kinds the kernels issue (cdna_hip_programming.md §5.5 T2/T10, layout (b) "one image for row
// reads AND transposed reads"):
//   * ds_read_b128 row reads: 16 consecutive rows, same logical chunk -> 16 distinct slots;
//   * ds_read_b64_tr_b16 transposed reads: 4 aligned rows x 4 chunks per 32-lane half -> distinct slots.
// D=128 (256-B rows): phys = c ^ ((r&3)<<2 | (r>>2)&3).  D=64 (128-B rows, two rows per 256-B bank
// row): phys = c ^ (((r>>1)&1)<<2 | (r>>2)&3).
template <int D>
__device__ __forceinline__ int swz(int r, int c) {
  if constexpr (D == 128) return r * 128 + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 3);
  else return r * 64 + ((c ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))) << 3);
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;


// pack registers 8s..8s+7 of an fp32 accumulator into a bf16 fragment
__device__ __forceinline__ u16x8 pack8(const f32x16& x, int s) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(x[8 * s + j]);
  return r;
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32): the softmax math of two accumulator registers per
// instruction -- an f32x16 tile's registers r, r + 1 (r even) are an aligned VGPR pair, so no moves are needed.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 pair(const f32x16& t, int r) { return f32x2{t[r], t[r + 1]}; }
__device__ __forceinline__ f32x2 bcast(float x) { return f32x2{x, x}; }
__device__ __forceinline__ f32x2 exp2_2(f32x2 x) { return f32x2{fast_exp2(x[0]), fast_exp2(x[1])}; }

struct AttnParams {
  const bf16_t* q; const bf16_t* k; const bf16_t* v;
  bf16_t* o; float* lse;
  const bf16_t* dout; bf16_t* dq; bf16_t* dk; bf16_t* dv; float* delta;
  int64_t q_sb, q_ss, q_sh;   // element strides: batch, seq, head
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t o_sb, o_ss, o_sh;   // also used for dout / dq (same layout as o / q)
  int64_t do_sb, do_ss, do_sh;
  int64_t dq_sb, dq_ss, dq_sh;
  int64_t dk_sb, dk_ss, dk_sh;
  int64_t dv_sb, dv_ss, dv_sh;
  int B, H, Hkv, Sq, Sk;
  float scale;   // softmax scale (natural domain)
  int order;     // workgroup -> block order: 0 heavy-first, 1 XCD-grouped (block_order)
  // backward, nullable: per-workgroup column sums of the stored dQ rows (the q part of the bias gradient of the
  // Linear that produced q, k, v -- GPT-2's c_attn -- without a separate column-sum pass over dqkv):
  // cs_q [B * nqb][H * D] (nqb = query blocks of the dQ kernel).  The k and v parts need no kernel work
  // (pdt_flash_attn_bwd).
  float* cs_q;
  // backward: the dQ kernel computes delta = rowsum(dO * O) and the log2-domain lse for its rows itself (from
  // the dO fragments it holds anyway) and writes them for the dK/dV kernel, which then runs after it -- no
  // separate delta pass re-reading O and dO
  int fuse_delta;
  // A/B switch (PDT_FA_MASK_ALL=1): every backward tile takes the masked path (the pre-dispatch code)
  int mask_all;
  // timing diagnostics only (PDT_FA_DIAG, results WRONG when set): bit 0 dK/dV kernel skips its K / V prologue
  // loads, bit 1 its dK / dV stores; bit 2 the dQ kernel skips its Q / dO / O prologue loads, bit 3 its dQ stores
  int diag;
};

// delta of this lane's query row from its dO fragments (gf, already in registers) and the O row; written with
// the log2-domain lse for the dK/dV kernel by the h == 0 lane.  Returns delta (both halves of the row).
template <int KS>
__device__ __forceinline__ float row_delta(const AttnParams& p, const u16x8 (&gf)[KS], int b, int hq, int qrow,
                                           int h) {
  float acc = 0.f;
  if (qrow < p.Sq) {
    const bf16_t* Op = p.o + b * p.o_sb + hq * p.o_sh + (int64_t)qrow * p.o_ss + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 of = *reinterpret_cast<const u16x8*>(Op + 16 * ks);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += bf2f(of[e]) * bf2f(gf[ks][e]);
    }
  }
  acc += __shfl_xor(acc, 32, 64);
  if (qrow < p.Sq && h == 0) {
    const int64_t idx = ((int64_t)b * p.H + hq) * p.Sq + qrow;
    p.delta[idx] = acc;
    p.delta[(int64_t)p.B * p.H * p.Sq + idx] = -p.lse[idx] * LOG2E;
  }
  return acc;
}


// ------------------------------------------------------------------------------------------------
// LDS-DMA operand staging shared by every kernel below: K/V (Q/dO) tiles arrive by buffer_load ... lds into
// an LDS ring -- no staging registers, ONE barrier per 64-row tile (the barrier's vmcnt wait retires the tile
// this iteration reads; the DMA for the next tile is issued right after it and overlaps this tile's MFMAs).
// The XOR swizzle is applied on the per-lane SOURCE address (the DMA destination is lane-linear,
// cdna_hip_programming.md §5.4 rule 21); rows past Sk are clamped to a real row and masked.
// ------------------------------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ int swz_f(int r) {
  if constexpr (D == 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
}

typedef __attribute__((address_space(3))) void lds_void;

// Barrier that retires this wave's LDS-DMA before other waves read what it wrote.  hipcc treats
// buffer/global_load ... lds as plain VMEM loads: a workgroup-scope fence does not wait for loads, so
// __syncthreads() alone emits NO s_waitcnt vmcnt(0) where the waitcnt pass sees no register dependency
// (the first barrier of a 2x-unrolled ring loop had none: under load, waves read a tile before its DMA
// landed -- wrong rows of O at B*H >= 512 on the GPT-2 1.3B shape).  The explicit wait is mandatory.
__device__ __forceinline__ void dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}


// LDS-DMA of a TILE-row window through a buffer resource (T8): the per-lane byte offset of this lane's
// 16-B chunk (row-major, XOR-swizzled) is computed once per kernel; per tile only the wave-uniform
// descriptor (base = first row of the window, num_records = bytes of the rows that exist) is rebuilt
// in SGPRs, so `buffer_load_dwordx4 ... offen lds` issues with no VALU address math, and rows past the
// end of the tensor come back as zeros from the range check (callers mask them) -- no clamping path.
// LDS-DMA issued from inline asm, hidden from hipcc's waitcnt pass.  For the builtin forms the pass cannot
// tell the ring stage being filled from the stage being read, and in the backward kernels it drained the
// freshly issued prefetch (s_waitcnt vmcnt(0)) before the tile's first ds_read -- the next tile's DMA
// latency exposed on every tile.  Ordering is then entirely the rings' dma_barrier() (explicit vmcnt(0) +
// barrier before a stage is read); hipcc's own counted waits for its loads only over-wait beside these.
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i make_rsrc(const void* base, int num_bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  v4i r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = __builtin_amdgcn_readfirstlane(num_bytes);   // range check: lanes past it read zeros
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void dma16_asm(const v4i& rsrc, uint32_t voff, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)lds_dst);
  // no "memory" clobber: the ring barriers (asm memory clobber + __syncthreads) already order every LDS access
  // of the target stage around the DMA, and leaving the compiler free to move other accesses lowers pressure
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(m0), "v"(voff), "s"(rsrc));   // m0: reserved, never allocated by hipcc
}
// the same with the LDS destination already a wave-uniform byte address
__device__ __forceinline__ void dma16_m0(const v4i& rsrc, uint32_t voff, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(m0), "v"(voff), "s"(rsrc));
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) { return (uint32_t)(uintptr_t)(lds_void*)p; }
// a value every lane holds equally (block coordinates, tile counters): keep it -- and everything derived from it,
// the 64-bit tile addresses included -- in SGPRs / on the scalar ALU instead of the VALU
__device__ __forceinline__ int sgpr(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ void dma4_asm(const v4i& rsrc, uint32_t voff, const void* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void*)lds_dst);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :: "s"(m0), "v"(voff), "s"(rsrc));
}

// Consume registers loaded by plain global loads in a kernel prologue, so hipcc's wait for them lands
// HERE, before the tile loop.  Otherwise its first use sits inside the loop, the waitcnt pass (merging the
// loop entry with the back edge) re-emits the wait every tile, and -- blind to the inline-asm DMA queued
// behind those loads -- as vmcnt(0), which drains the tile prefetch.
template <int N>
__device__ __forceinline__ void retire(const u16x8 (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" :: "v"(x[i]));
}

template <int D, bool ASM = true, int NW = 4>
struct DmaLane {
  // NW waves fill a TILE-row window, RW rows each, RPI rows per 1-KiB wave-instruction
  static constexpr int RW = TILE / NW, RPI = 1024 / (D * 2), NI = RW / RPI, LPR = 64 / RPI;
  static_assert(NI >= 1 && RW % RPI == 0, "tile rows per wave must be whole DMA instructions");
  uint32_t off_[NI];
  uint32_t woff_;   // this wave's byte offset inside a staged tile (wave-uniform: an SGPR)
  __device__ __forceinline__ void init(int64_t row_stride, int w, int lane) {
    woff_ = (uint32_t)sgpr(RW * w * D * 2);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int row = RW * w + RPI * i + lane / LPR;
      const int c = (lane % LPR) ^ swz_f<D>(row);
      off_[i] = (uint32_t)((row * row_stride + c * 8) * 2);
    }
  }
  __device__ __forceinline__ uint32_t off(int i, int) const { return off_[i]; }
  // the same with the stage's LDS byte address given (no generic-pointer round trip)
  __device__ __forceinline__ void issue_at(const bf16_t* base, int64_t row_stride, int row0, int nrows, uint32_t lds,
                                           int w) const {
    static_assert(ASM, "issue_at: inline-asm DMA only");
    const int rows_left = nrows - row0;
    const int bytes = rows_left > 0 ? (int)((int64_t)(rows_left - 1) * row_stride * 2 + D * 2) : 0;
    const v4i rsrc = make_rsrc(base + (int64_t)row0 * row_stride, bytes);
    const uint32_t m0 = lds + woff_;
#pragma unroll
    for (int i = 0; i < NI; ++i) dma16_m0(rsrc, off(i, w), m0 + RPI * i * D * 2);
  }
  __device__ __forceinline__ void issue(const bf16_t* base, int64_t row_stride, int row0, int nrows, bf16_t* lds,
                                        int w) const {
    const int rows_left = nrows - row0;
    const int bytes = rows_left > 0 ? (int)((int64_t)(rows_left - 1) * row_stride * 2 + D * 2) : 0;
    if constexpr (ASM) {
      const v4i rsrc = make_rsrc(base + (int64_t)row0 * row_stride, bytes);
      // m0 = stage base (scalar) + wave offset (SGPR) + piece immediate: no per-issue VALU address math
      const uint32_t m0 = lds_u32(lds) + woff_;
#pragma unroll
      for (int i = 0; i < NI; ++i) dma16_m0(rsrc, off(i, w), m0 + RPI * i * D * 2);
    } else {
#if __HIP_DEVICE_COMPILE__   // the buffer-resource type exists only in the device pass
      const __amdgpu_buffer_rsrc_t rsrc =
          __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)row0 * row_stride), 0, bytes, 0x00020000);
#pragma unroll
      for (int i = 0; i < NI; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + (RW * w + RPI * i) * D), 16, off(i, w), 0,
                                                 0, 0);
#endif
    }
  }
};

// ------------------------------------------------------------------------------------------------
// Forward tile body (the recipe of v5 below): per 64-key tile a wave issues 32 MFMAs (1024 MFMA cycles);
// the first LDS-DMA generation spent ~3x that on VALU (address math, zero-fills, scale, rescale, masks).
// (1) every LDS fragment address is a per-lane base computed ONCE (the swizzle depends only on
// row & 15, which tile/k-block steps never change) plus a compile-time immediate -- the loop is
// unrolled by the 2-deep ring so the buffer offset is an immediate too; (2) the softmax scale is
// folded into one FMA feeding v_exp (max taken on raw scores); (3) the O rescale is skipped when no
// lane's running max moved; (4) the causal mask is one compare+select per element and only on
// diagonal tiles.
// ------------------------------------------------------------------------------------------------
// Causal blocks carry work proportional to their distance from the diagonal.  Workgroups dispatch in
// flattened-id order, so with the natural (tile, head, batch) grid every (head, batch) group ends with its
// light tiles and the heaviest tiles of the LAST groups start last (a long tail: causal ran at 80-86 % of
// the full-attention time, scripts/attn_causal_probe.py).  Decoding the flattened id tile-major instead
// dispatches the heaviest tile of every (head, batch) first (longest-processing-time order).
struct BlockCoord {
  int t, h, b;
};
__device__ __forceinline__ BlockCoord heavy_first(bool heavy_is_high) {
  const int nt = gridDim.x, nh = gridDim.y;
  const int lin = blockIdx.x + nt * (blockIdx.y + nh * blockIdx.z);
  const int hb = nh * gridDim.z;
  const int rank = lin / hb, rem = lin - rank * hb;
  BlockCoord c;
  c.h = rem % nh;
  c.b = rem / nh;
  c.t = heavy_is_high ? nt - 1 - rank : rank;
  return c;
}

// XCD-grouped order (p.order == 1): workgroups are dealt to the 8 XCDs round-robin in flattened-id order
// (lin % 8), each XCD with its own L2.  heavy_first() spreads the blocks that stream the SAME K/V tiles
// (forward, dQ: every query head of one (batch, kv head) unit) or Q/dO tiles (dK/dV) over every XCD and over
// the whole launch, so each re-read comes from HBM.  Here every unit lives on one XCD (unit u -> XCD u % 8)
// and its blocks -- all its query heads', heaviest first -- run back to back there, so the re-reads hit that
// XCD's L2.  grp = query heads per kv head for the query-side grids (1 for dK/dV's kv-head grid).
__device__ __forceinline__ BlockCoord grouped_coord(int lin, int nt, int nh, int grp, bool heavy_is_high) {
  const int per = grp * nt, j = lin >> 3, ui = j / per, r = j - ui * per;
  const int u = ui * 8 + (lin & 7), rank = r / grp, hi = r - rank * grp, nkv = nh / grp;
  BlockCoord c;
  c.b = u / nkv;
  c.h = (u - c.b * nkv) * grp + hi;
  c.t = heavy_is_high ? nt - 1 - rank : rank;
  return c;
}
__device__ __forceinline__ bool grouped_ok(int order, int nh, int nb, int grp) {
  return order == 1 && !(((nh / grp) * nb) & 7);
}
// order 2: the tile index cycles fastest (heaviest first within each cycle): consecutive workgroups get different
// amounts of causal work, so they finish -- and start their HBM-bound prologues -- at different times instead of
// every CU loading its Q / dO (K / V) rows in the same burst (a measured A/B: PDT_FA_CYCLE)
__device__ __forceinline__ BlockCoord cycled(bool heavy_is_high) {
  const int nt = gridDim.x, nh = gridDim.y;
  const int lin = blockIdx.x + nt * (blockIdx.y + nh * blockIdx.z);
  const int tr = lin % nt, rest = lin / nt;
  BlockCoord c;
  c.t = heavy_is_high ? nt - 1 - tr : tr;
  c.h = rest % nh;
  c.b = rest / nh;
  return c;
}
__device__ __forceinline__ BlockCoord block_order(bool heavy_is_high, int order, int grp) {
  if (order == 2) return cycled(heavy_is_high);
  if (!grouped_ok(order, gridDim.y, gridDim.z, grp)) return heavy_first(heavy_is_high);
  return grouped_coord(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), gridDim.x, gridDim.y, grp,
                       heavy_is_high);
}

// ------------------------------------------------------------------------------------------------
// Row-per-lane epilogue with 16-byte stores (cdna_hip_programming.md T21): a lane holds 4 consecutive
// columns per (dt, g) of its row and its xor-32 partner the next 4, so a v_permlane32_swap per dword
// pair hands each lane 8 consecutive columns -- D/16 dwordx4 stores per lane instead of D/8 dwordx2
// (the store-issue-bound tail of MI355X_MICROARCH.md 'attention epilogue store tail').  Every lane must
// run it (EXEC all ones for the swap); `ok` only gates the stores (both partner lanes share one row).
// ------------------------------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void store_row16(bf16_t* row, const f32x16 (&acc)[DT], float scale, int h, bool ok) {
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      unsigned a[2], c[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int g0 = 2 * pr, g1 = 2 * pr + 1;
        a[k] = (unsigned)f2bf(acc[dt][4 * g0 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g0 + 2 * k + 1] * scale) << 16);
        c[k] = (unsigned)f2bf(acc[dt][4 * g1 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g1 + 2 * k + 1] * scale) << 16);
        const auto r = __builtin_amdgcn_permlane32_swap(a[k], c[k], false, false);
        a[k] = r[0];
        c[k] = r[1];
      }
      if (ok) {
        u32x4 v;
        v[0] = a[0]; v[1] = a[1]; v[2] = c[0]; v[3] = c[1];
        *reinterpret_cast<u32x4*>(row + dt * 32 + 16 * pr + 8 * h) = v;
      }
    }
}

// store_row16 that also returns the stored (bf16-rounded, scaled) values as floats, zero for a masked row:
// v[(dt * 2 + pr) * 8 + k] is column dt * 32 + 16 * pr + 8 * h + k of this lane's row
template <int DT>
__device__ __forceinline__ void store_row16_vals(bf16_t* row, const f32x16 (&acc)[DT], float scale, int h, bool ok,
                                                 float (&v)[DT * 16]) {
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      unsigned a[2], c[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int g0 = 2 * pr, g1 = 2 * pr + 1;
        a[k] = (unsigned)f2bf(acc[dt][4 * g0 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g0 + 2 * k + 1] * scale) << 16);
        c[k] = (unsigned)f2bf(acc[dt][4 * g1 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g1 + 2 * k + 1] * scale) << 16);
        const auto r = __builtin_amdgcn_permlane32_swap(a[k], c[k], false, false);
        a[k] = r[0];
        c[k] = r[1];
      }
      u32x4 q;
      q[0] = a[0]; q[1] = a[1]; q[2] = c[0]; q[3] = c[1];
      if (ok) *reinterpret_cast<u32x4*>(row + dt * 32 + 16 * pr + 8 * h) = q;
      const float m = ok ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[(dt * 2 + pr) * 8 + 2 * k] = m * __uint_as_float(q[k] << 16);
        v[(dt * 2 + pr) * 8 + 2 * k + 1] = m * __uint_as_float(q[k] & 0xffff0000u);
      }
    }
}

// Column sums over the 32 rows (lanes c32 = 0..31) of a wave half: a reduce-scatter butterfly (each step halves
// the values a lane keeps, 62 exchanges for 64 values instead of 320 for a full all-reduce).  In: N values per
// lane (index i = the store_row16_vals layout); out: lane c32 holds the sums of indices c32 * (N / 32) + e.
template <int NV, int M, int N>
__device__ __forceinline__ void colsum32_step(float (&v)[N], int c32) {
  // NV live values v[0, NV); exchange with lane ^ M (compile-time indices only: the array stays in registers)
  const bool up = (c32 & M) != 0;   // this lane keeps the upper half
#pragma unroll
  for (int i = 0; i < NV / 2; ++i) {
    const float send = up ? v[i] : v[i + NV / 2];
    const float keep = up ? v[i + NV / 2] : v[i];
    v[i] = keep + __shfl_xor(send, M, 64);
  }
  if constexpr (M > 1) colsum32_step<NV / 2, M / 2, N>(v, c32);
}
template <int N>
__device__ __forceinline__ void colsum32_scatter(float (&v)[N], int c32) {
  static_assert(N == 32 || N == 64, "D 64 or 128");
  colsum32_step<N, 16, N>(v, c32);
}

// one workgroup's partial column sums of its NW waves' stored rows -> out[0, D) (one fp32 row); lds: >= NW * D
// floats of workgroup LDS no longer in use (every wave has passed its last read of it: barrier first)
// Raw barriers (LDS counter only): __syncthreads() would also wait for this wave's just-issued dQ / dK / dV
// row stores to complete (vmcnt(0)) -- measured +0.7 ms per flagship attention backward with it, 4x the
// separate column-sum pass this replaces.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int D, int NW>
__device__ __forceinline__ void wg_colsum_store(float (&v)[D / 2], float* lds, float* out, int w, int lane) {
  constexpr int E = D / 64;             // values left per lane after the butterfly
  const int h = lane >> 5, c32 = lane & 31;
  colsum32_scatter<D / 2>(v, c32);
  lds_barrier();                        // every wave is past its last read of the reused LDS
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = c32 * E + e;
    lds[w * D + (i >> 4) * 32 + ((i >> 3) & 1) * 16 + 8 * h + (i & 7)] = v[e];
  }
  lds_barrier();
  if ((int)threadIdx.x < D) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) t += lds[q * D + threadIdx.x];
    out[threadIdx.x] = t;
  }
}

// ------------------------------------------------------------------------------------------------
// forward v5 (default) = the VALU-lean tile body above + (1) deferred rescale (T13): the running max m used in exp2 moves only when some
// row's tile max exceeds it by more than RESCALE_THR (log2 units), so the 64-register O rescale runs on a
// handful of tiles instead of most of them (probabilities stay <= 2^THR, exact in fp32 / bf16 range);
// (2) the K row fragments stream two MFMA steps ahead of their use and the V transposed fragments one
// step ahead, each step its own scheduling region, so an LDS read's latency hides behind the MFMAs
// instead of stalling every pair; (3) the 16-byte permlane epilogue.
// Measured and NOT adopted (scripts/bench_attn_ab.py, one process, interleaved rounds): an in-wave pipeline
// across tiles (QK(t+1) MFMAs under the softmax VALU of tile t, PV(t) under the row max of t+1, K and V
// on separate rings) ran 555 vs 571 TFLOP/s causal and tied non-causal -- the co-resident wave of the
// other workgroup already fills this wave's softmax gaps; likewise two-step-ahead fragment reads in the
// backward tiles ran 2-5 % slower than the one-step hand pipeline.
// ------------------------------------------------------------------------------------------------
constexpr float RESCALE_THR = 8.0f;

template <int D, bool CAUSAL>
struct FwdV5 {
  static constexpr int KS = D / 16, DT = D / 32, TE = TILE * D;

  __device__ __forceinline__ static u16x8 kfr(const bf16_t* lds, const int (&koff)[KS], int i) {
    // step i: k-step i / 2, key subtile i % 2
    return *reinterpret_cast<const u16x8*>(lds + koff[i >> 1] + (i & 1) * 32 * D);
  }
  __device__ __forceinline__ static u16x8 vfr(const bf16_t* vs, const int (&voff)[DT][2], int j) {
    // step j: dt = j / 4, key block kb = 16 * (j % 4)
    const int dt = j >> 2, kb = 16 * (j & 3);
    const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(vs + voff[dt][0] + kb * D));
    const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(vs + voff[dt][1] + kb * D));
    return __builtin_bit_cast(u16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
  }

  __device__ __forceinline__ static void tile(const bf16_t* __restrict__ lds, const int (&koff)[KS],
                                              const int (&voff)[DT][2], const u16x8 (&qf)[KS], f32x16 (&o)[DT],
                                              float& m, float& l, float sl2, int k0, bool diag, int lim) {
    constexpr int NS = 2 * KS;   // QK^T steps (one MFMA each)
    f32x16 s[2];
    u16x8 kb0 = kfr(lds, koff, 0), kb1 = kfr(lds, koff, 1);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      u16x8 kn;
      if (i + 2 < NS) kn = kfr(lds, koff, i + 2);
      __builtin_amdgcn_sched_barrier(0);   // the read issues BEFORE this step's MFMA (two steps of cover)
      const int ks = i >> 1, st = i & 1;
      s[st] = mfma32(kb0, qf[ks], ks == 0 ? zero16() : s[st]);
      kb0 = kb1;
      kb1 = kn;
      __builtin_amdgcn_sched_barrier(0);
    }
    const bf16_t* vs = lds + TE;
    u16x8 vb0 = vfr(vs, voff, 0), vb1 = vfr(vs, voff, 1);   // first V fragments in flight under the softmax
    if (diag) {   // keys k0 + kt*32 + acc_row(r, h) > lim are masked (future / past Sk)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2);
        s[0][r] = (k0 + rr > lim) ? -INFINITY : s[0][r];
        s[1][r] = (k0 + 32 + rr > lim) ? -INFINITY : s[1][r];
      }
    }
    float mx = fmaxf(s[0][0], s[1][0]);
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, fmaxf(s[0][r], s[1][r]));   // v_max3_f32 chain
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * sl2;
    if (!__all(mx <= m + RESCALE_THR)) {   // some row's max ran past the deferred reference: move it
      const float mn = fmaxf(m, mx);
      const float alpha = (m == -INFINITY) ? 0.f : fast_exp2(m - mn);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      l *= alpha;
      m = mn;
    }
    const float msub = (m == -INFINITY) ? 0.f : m;
    // p = exp2(s * scale * log2e - m), two registers per packed FMA / add (row sums in two partial lanes)
    f32x2 ls2 = bcast(0.f);
    const f32x2 sc2 = bcast(sl2), ms2 = bcast(-msub);
    u16x8 pf[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const f32x2 pv = exp2_2(pk_fma(pair(s[t], r), sc2, ms2));
        s[t][r] = pv[0];
        s[t][r + 1] = pv[1];
        ls2 += pv;
      }
      pf[t][0] = pack8(s[t], 0);
      pf[t][1] = pack8(s[t], 1);
    }
    l += ls2[0] + ls2[1];
    constexpr int NV = 4 * DT;   // PV steps: (dt, kt, ss)
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      u16x8 vn;
      if (j + 2 < NV) vn = vfr(vs, voff, j + 2);
      __builtin_amdgcn_sched_barrier(0);
      const int dt = j >> 2, kt = (j >> 1) & 1, ss = j & 1;
      o[dt] = mfma32(vb0, pf[kt][ss], o[dt]);
      vb0 = vb1;
      vb1 = vn;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
};

template <int D, bool CAUSAL>
__global__ __launch_bounds__(NT, 2) void fa_fwd_v5_kernel(AttnParams p) {
  using K = FwdV5<D, CAUSAL>;
  constexpr int KS = K::KS, DT = K::DT, TE = K::TE;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TE];   // [buf 0/1][K | V]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const BlockCoord bc = block_order(true, p.order, p.H / p.Hkv);
  const bool remap = CAUSAL || p.order != 0;
  const int b = sgpr(remap ? bc.b : (int)blockIdx.z), hq = sgpr(remap ? bc.h : (int)blockIdx.y);
  const int qb = sgpr(remap ? bc.t : (int)blockIdx.x);
  const int hk = sgpr(hq / (p.H / p.Hkv));
  const int off = p.Sk - p.Sq;
  const int q0 = qb * 128, qw = q0 + w * 32, qrow = qw + c32;
  const bf16_t* Qp = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* Kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vp = p.v + b * p.v_sb + hk * p.v_sh;
  const float sl2 = p.scale * LOG2E;

  int kend = p.Sk;
  if (CAUSAL) kend = min(p.Sk, q0 + 128 + off);
  const int ntiles = kend > 0 ? (kend + TILE - 1) / TILE : 0;
  DmaLane<D> lk, lv;
  lk.init(p.k_ss, w, lane);
  lv.init(p.v_ss, w, lane);
  if (ntiles > 0) {
    lk.issue(Kp, p.k_ss, 0, p.Sk, smem, w);
    lv.issue(Vp, p.v_ss, 0, p.Sk, smem + TE, w);
  }

  int koff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) koff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int voff[DT][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int r1 = 4 * (g >> 1) + q;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = 32 * dt + 16 * (g & 1) + 4 * pp;
      voff[dt][0] = r1 * D + (((col >> 3) ^ swz_f<D>(r1)) << 3) + (col & 7);
      voff[dt][1] = (r1 + 8) * D + (((col >> 3) ^ swz_f<D>(r1 + 8)) << 3) + (col & 7);
    }
  }

  u16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (qrow < p.Sq) qf[ks] = *reinterpret_cast<const u16x8*>(Qp + (int64_t)qrow * p.q_ss + 16 * ks + 8 * h);
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) qf[ks][k] = 0;
    }
  }
  retire(qf);
  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = zero16();
  float m = -INFINITY, l = 0.f;
  const int lim = min(p.Sk - 1, CAUSAL ? qrow + off : p.Sk - 1) - 4 * h;

  for (int t = 0; t < ntiles; t += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tt = t + u;
      if (tt < ntiles) {
        dma_barrier();
        if (tt + 1 < ntiles) {
          bf16_t* nb = smem + (1 - u) * 2 * TE;
          lk.issue(Kp, p.k_ss, (tt + 1) * TILE, p.Sk, nb, w);
          lv.issue(Vp, p.v_ss, (tt + 1) * TILE, p.Sk, nb + TE, w);
        }
        const int k0 = tt * TILE;
        if (!(CAUSAL && k0 > qw + 31 + off)) {
          const bool diag = (k0 + TILE > p.Sk) || (CAUSAL && k0 + TILE - 1 > qw + off);
          K::tile(smem + u * 2 * TE, koff, voff, qf, o, m, l, sl2, k0, diag, lim);
        }
      }
    }
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  store_row16<DT>(p.o + b * p.o_sb + hq * p.o_sh + (int64_t)qrow * p.o_ss, o, inv, h, qrow < p.Sq);
  if (qrow < p.Sq && h == 0)
    p.lse[((int64_t)b * p.H + hq) * p.Sq + qrow] = lt > 0.f ? (m + __log2f(lt)) * LN2 : INFINITY;
}

// ------------------------------------------------------------------------------------------------
// forward v7 = v5's per-wave tile on a 512-thread workgroup: 8 waves x 32 query rows = 256 rows share every
// staged K/V tile, twice v5's 128.  Each 64-key tile (32 KB of K and V) then feeds 2 x 128 x 64 x 128 x 2
// FLOPs per 16 KB -- 256 FLOP/B instead of 128 -- which halves the L2 -> LDS tile traffic per FLOP: at
// the GPT-2 1.3B shape v5 streamed ~3.9 TB/s of K/V for 460 TFLOP/s, i.e. it was fed, not computing.
// One workgroup per CU (two waves per SIMD, the same register budget as v5's two 256-thread groups),
// NBUF-deep LDS ring with counted vmcnt: tile t's DMA is waited for while tiles t+1 .. t+NBUF-2 stay in
// flight (NBUF = 3: two tiles of latency cover instead of one).
// ------------------------------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

// top of ring iteration t: this wave's DMA of tile t landed (later tiles may still fly), then the barrier
// publishes every wave's part of tile t and retires all reads of the stage about to be refilled
template <int PER_TILE, int NBUF>
__device__ __forceinline__ void ring_wait(bool later_in_flight) {
  static_assert(NBUF == 2 || NBUF == 3, "ring depth 2 or 3");
  if constexpr (NBUF == 3) {
    if (later_in_flight) vm_wait<PER_TILE>();
    else vm_wait<0>();
  } else {
    vm_wait<0>();
  }
  __syncthreads();
}

constexpr int NT8 = 512;

template <int D, bool CAUSAL, int NBUF>
__global__ __launch_bounds__(NT8, 1) void fa_fwd_v7_kernel(AttnParams p) {
  using K = FwdV5<D, CAUSAL>;
  constexpr int KS = K::KS, DT = K::DT, TE = K::TE, NW = 8, BM = 32 * NW;
  using Dma = DmaLane<D, true, NW>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NBUF * 2 * TE];   // [stage][K | V]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const BlockCoord bc = block_order(true, p.order, p.H / p.Hkv);
  const bool remap = CAUSAL || p.order != 0;
  const int b = sgpr(remap ? bc.b : (int)blockIdx.z), hq = sgpr(remap ? bc.h : (int)blockIdx.y);
  const int qb = sgpr(remap ? bc.t : (int)blockIdx.x);
  const int hk = sgpr(hq / (p.H / p.Hkv));
  const int off = p.Sk - p.Sq;
  const int q0 = qb * BM, qw = q0 + w * 32, qrow = qw + c32;
  const bf16_t* Qp = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* Kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vp = p.v + b * p.v_sb + hk * p.v_sh;
  const float sl2 = p.scale * LOG2E;

  int kend = p.Sk;
  if (CAUSAL) kend = min(p.Sk, q0 + BM + off);
  const int ntiles = kend > 0 ? (kend + TILE - 1) / TILE : 0;
  Dma lk, lv;
  lk.init(p.k_ss, w, lane);
  lv.init(p.v_ss, w, lane);
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < ntiles) {
      lk.issue(Kp, p.k_ss, t * TILE, p.Sk, smem + t * 2 * TE, w);
      lv.issue(Vp, p.v_ss, t * TILE, p.Sk, smem + t * 2 * TE + TE, w);
    }

  int koff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) koff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int voff[DT][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int r1 = 4 * (g >> 1) + q;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = 32 * dt + 16 * (g & 1) + 4 * pp;
      voff[dt][0] = r1 * D + (((col >> 3) ^ swz_f<D>(r1)) << 3) + (col & 7);
      voff[dt][1] = (r1 + 8) * D + (((col >> 3) ^ swz_f<D>(r1 + 8)) << 3) + (col & 7);
    }
  }

  u16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (qrow < p.Sq) qf[ks] = *reinterpret_cast<const u16x8*>(Qp + (int64_t)qrow * p.q_ss + 16 * ks + 8 * h);
    else {
#pragma unroll
      for (int k = 0; k < 8; ++k) qf[ks][k] = 0;
    }
  }
  retire(qf);
  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = zero16();
  float m = -INFINITY, l = 0.f;
  const int lim = min(p.Sk - 1, CAUSAL ? qrow + off : p.Sk - 1) - 4 * h;

  int stage = 0;   // stage of tile t; tile t + NBUF - 1 refills stage (t - 1) % NBUF
  for (int t = 0; t < ntiles; ++t) {
    ring_wait<2 * Dma::NI, NBUF>(t + 1 < ntiles);
    if (t + NBUF - 1 < ntiles) {
      const int ns = stage == 0 ? NBUF - 1 : stage - 1;
      bf16_t* nb = smem + ns * 2 * TE;
      lk.issue(Kp, p.k_ss, (t + NBUF - 1) * TILE, p.Sk, nb, w);
      lv.issue(Vp, p.v_ss, (t + NBUF - 1) * TILE, p.Sk, nb + TE, w);
    }
    const int k0 = t * TILE;
    if (!(CAUSAL && k0 > qw + 31 + off)) {
      const bool diag = (k0 + TILE > p.Sk) || (CAUSAL && k0 + TILE - 1 > qw + off);
      K::tile(smem + stage * 2 * TE, koff, voff, qf, o, m, l, sl2, k0, diag, lim);
    }
    stage = stage + 1 == NBUF ? 0 : stage + 1;
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  store_row16<DT>(p.o + b * p.o_sb + hq * p.o_sh + (int64_t)qrow * p.o_ss, o, inv, h, qrow < p.Sq);
  if (qrow < p.Sq && h == 0)
    p.lse[((int64_t)b * p.H + hq) * p.Sq + qrow] = lt > 0.f ? (m + __log2f(lt)) * LN2 : INFINITY;
}

// ------------------------------------------------------------------------------------------------
// backward (a): delta[b, h, q] = sum_d dO * O
// ------------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(NT) void fa_bwd_delta_kernel(AttnParams p) {
  // delta = rowsum(dO * O) and the log2-domain lse, D/8 lanes per row (16-B coalesced loads)
  constexpr int LPR = D / 8;
  const int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x;
  const int64_t idx = t / LPR;                      // row over B*H*Sq
  const int c = (int)(t % LPR) * 8;
  const int64_t total = (int64_t)p.B * p.H * p.Sq;
  float acc = 0.f;
  if (idx < total) {
    const int q = (int)(idx % p.Sq);
    const int hq = (int)((idx / p.Sq) % p.H);
    const int b = (int)(idx / ((int64_t)p.Sq * p.H));
    float a[8], g[8];
    Vec8<bf16_t>::load(p.o + b * p.o_sb + hq * p.o_sh + (int64_t)q * p.o_ss + c, a);
    Vec8<bf16_t>::load(p.dout + b * p.do_sb + hq * p.do_sh + (int64_t)q * p.do_ss + c, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += a[k] * g[k];
  }
#pragma unroll
  for (int m = LPR / 2; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if (idx < total && c == 0) {
    p.delta[idx] = acc;
    p.delta[total + idx] = -p.lse[idx] * LOG2E;   // log2-domain lse for the v3 dK/dV kernel
  }
}


// ------------------------------------------------------------------------------------------------
// backward operand staging (dK/dV and dQ): same recipe as the forward -- LDS-DMA double-buffered operand tiles
// (one barrier per tile), per-lane LDS bases + immediates (no per-read address math), scale folded
// into an FMA ahead of v_exp, and compare/select masks only on boundary sub-tiles.  LSE and delta
// rows travel by LDS-DMA too (4-byte pieces), so no ordinary global load sits in the loop to force
// a vmcnt(0) drain of the prefetch.
// ------------------------------------------------------------------------------------------------
// one wave: 64 fp32 rows [row0, row0 + 64) of a row vector into LDS (rows past nrows read as 0: they pair with
// the zero Q / dO rows of the ragged tile and contribute nothing)
__device__ __forceinline__ void dma_f32_row(const float* src, int row0, int nrows, float* lds, int lane) {
  const int left = nrows - row0;
  dma4_asm(make_rsrc(src + row0, left > 0 ? left * 4 : 0), (uint32_t)lane * 4, lds);
}

__device__ __forceinline__ void dma_f32_row_at(const float* src, int row0, int nrows, uint32_t lds, int lane) {
  const int left = nrows - row0;
  const v4i rsrc = make_rsrc(src + row0, left > 0 ? left * 4 : 0);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :: "s"(lds), "v"((uint32_t)lane * 4), "s"(rsrc));
}

// transposed-fragment offsets for a [TILE][D] swizzled image (rows kb + 4(g>>1) + q (+8), column
// 32dt + 16(g&1) + 4p); kb must be a multiple of 16 and is added as an immediate by the caller.
template <int D>
__device__ __forceinline__ void tr_offsets(int lane, int (&toff)[D / 32][2]) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int r1 = 4 * (g >> 1) + q;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
    const int col = 32 * dt + 16 * (g & 1) + 4 * pp;
    toff[dt][0] = r1 * D + (((col >> 3) ^ swz_f<D>(r1)) << 3) + (col & 7);
    toff[dt][1] = (r1 + 8) * D + (((col >> 3) ^ swz_f<D>(r1 + 8)) << 3) + (col & 7);
  }
}

__device__ __forceinline__ u16x8 tr_pair(const bf16_t* p0, const bf16_t* p1) {
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)p0);
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)p1);
  return __builtin_bit_cast(u16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// ------------------------------------------------------------------------------------------------
// backward v3: the staging above, re-shaped for intra-wave MFMA/VALU overlap.  Each 64-row tile is
// one straight-line region: BOTH 32-row subtiles' S / dP chains are issued first, then the softmax-
// gradient VALU work of subtile 0 runs under the MFMAs of subtile 1's chains and subtile 0's dK/dV
// (dQ) updates, and so on -- independent work the scheduler can interleave even at one wave per SIMD.
// Masking is resolved per tile (wave-uniform EDGE template switch) instead of per 32-row subtile, so
// the common interior tile has no branches at all.  The file is built with the MFMA VGPR form
// (-mllvm -amdgpu-mfma-vgpr-form): accumulators the VALU post-processes stay in arch VGPRs instead of
// being shuttled through AGPRs with v_accvgpr_read/write.
// ------------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
struct BwdKVTile {
  static constexpr int KS = D / 16, DT = D / 32;
  static constexpr int EA = 16 / KS;        // softmax elements finished per stage-A step
  static constexpr int EB = 16 / (2 * DT);  // ... per stage-B step (== EA since KS == 2 DT)
  static_assert(EA % 2 == 0, "packed softmax pairs");

  // Q / dO row fragment of step i (subtile i / KS, k-step i % KS)
  __device__ __forceinline__ static u16x8 rowf(const bf16_t* base, const int (&roff)[KS], int i) {
    return *reinterpret_cast<const u16x8*>(base + roff[i % KS] + (i / KS) * 32 * D);
  }
  // transposed dO / Q fragment of subtile qs, step j (dt = j / 2, 16-row half j % 2)
  __device__ __forceinline__ static u16x8 trf(const bf16_t* base, const int (&toff)[DT][2], int qs, int j) {
    const int o = (qs * 32 + 16 * (j & 1)) * D;
    return tr_pair(base + toff[j >> 1][0] + o, base + toff[j >> 1][1] + o);
  }
  // softmax-gradient of accumulator registers [e0, e0 + N) of one 32-row subtile (scalar: the packed form
  // produced wrong dK / dV at one wave per SIMD -- an MFMA-result hazard on v_pk_* reads, not chased further):
  //   p = exp2(s * scale*log2e - lse*log2e),  dS = p * (dP - delta)
  // MASK (wave-uniform: the tile crosses the causal diagonal) selects the masked rows; query rows past Sq
  // arrive as zero Q / dO rows (buffer range check), which contribute exactly 0 to dK (dS * q) and dV (p * dO)
  // without masking
  template <int N, bool MASK>
  __device__ __forceinline__ static void smx(f32x16& sv, f32x16& dpv, int e0, const float* nl, const float* dl, float sl2,
                                             int qs, int tmask, int tsq) {
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const int r = e0 + e, rr = (r & 3) + 8 * (r >> 2) + 32 * qs;
      float pv = fast_exp2(fmaf(sv[r], sl2, nl[e]));
      if constexpr (MASK) pv = rr < tmask ? 0.f : pv;
      sv[r] = pv;
      dpv[r] = pv * (dpv[r] - dl[e]);
    }
  }
  template <int N>
  __device__ __forceinline__ static void ldstat(const float* Ls, const float* Ds, int e0, int qs, int h, float (&nl)[N],
                                                float (&dl)[N]) {
    const int r0 = (e0 & 3) + 8 * (e0 >> 2) + 32 * qs + 4 * h;   // N <= 4 consecutive rows
#pragma unroll
    for (int e = 0; e < N; ++e) { nl[e] = Ls[r0 + e]; dl[e] = Ds[r0 + e]; }
  }

  // One 64-query tile against this wave's 32 keys, software-pipelined by hand: every step is its own
  // scheduling region (sched_barrier) holding 2 MFMAs, the LDS reads for the NEXT step and a slice of
  // softmax VALU -- the compiler's own schedule issues each LDS read just before its MFMA, which at one
  // wave per SIMD exposes the full LDS latency on every MFMA.
  //   stage A (2*KS steps): S / dP chains of subtiles 0 and 1; subtile 0's softmax under subtile 1's chain
  //   stage B (2*DT steps): dV/dK += subtile 0;                   subtile 1's softmax under it
  //   stage C (2*DT steps): dV/dK += subtile 1
  // Ls holds -lse*log2(e) rows, Ds delta rows.  MASK: the tile crosses the causal diagonal (selects on its rows).
  template <bool MASK>
  __device__ __forceinline__ static void run(const bf16_t* Qs, const bf16_t* Gs, const float* Ls, const float* Ds,
                                             const u16x8 (&kf)[KS], const u16x8 (&vf)[KS], const int (&roff)[KS],
                                             const int (&toff)[DT][2], f32x16 (&dk)[DT], f32x16 (&dv)[DT], float sl2,
                                             int tmask, int tsq, int h) {
    acc_fence();   // accumulator copies the register allocator placed before this tile have retired
    f32x16 s[2], dp[2];
    u16x8 pf[2][2], df[2][2];
    const f32x16 z = zero16();
    // ---- stage A
    u16x8 qa = rowf(Qs, roff, 0), ga = rowf(Gs, roff, 0);
    float nl[EA], dl[EA];
    ldstat<EA>(Ls, Ds, 0, 0, h, nl, dl);
    u16x8 ta, tb;
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const int qs = i / KS, ks = i % KS;
      u16x8 qn, gn;
      if (i + 1 < 2 * KS) { qn = rowf(Qs, roff, i + 1); gn = rowf(Gs, roff, i + 1); }
      else { ta = trf(Gs, toff, 0, 0); tb = trf(Qs, toff, 0, 0); }
      s[qs] = mfma32(qa, kf[ks], ks == 0 ? z : s[qs]);
      dp[qs] = mfma32(ga, vf[ks], ks == 0 ? z : dp[qs]);
      if (qs == 1) {
        float nn[EA], dd[EA];
        if (ks + 1 < KS) ldstat<EA>(Ls, Ds, (ks + 1) * EA, 0, h, nn, dd);
        else ldstat<EA>(Ls, Ds, 0, 1, h, nn, dd);   // EA == EB: first stage-B slice
        smx<EA, MASK>(s[0], dp[0], ks * EA, nl, dl, sl2, 0, tmask, tsq);
#pragma unroll
        for (int e = 0; e < EA; ++e) { nl[e] = nn[e]; dl[e] = dd[e]; }
      }
      qa = qn; ga = gn;
      __builtin_amdgcn_sched_barrier(0);
    }
    pf[0][0] = pack8(s[0], 0); pf[0][1] = pack8(s[0], 1);
    df[0][0] = pack8(dp[0], 0); df[0][1] = pack8(dp[0], 1);
    // ---- stage B
#pragma unroll
    for (int j = 0; j < 2 * DT; ++j) {
      u16x8 tan, tbn;
      if (j + 1 < 2 * DT) { tan = trf(Gs, toff, 0, j + 1); tbn = trf(Qs, toff, 0, j + 1); }
      else { tan = trf(Gs, toff, 1, 0); tbn = trf(Qs, toff, 1, 0); }
      mfma32_acc(dv[j >> 1], ta, pf[0][j & 1]);
      mfma32_acc(dk[j >> 1], tb, df[0][j & 1]);
      float nn[EB], dd[EB];
      if (j + 1 < 2 * DT) ldstat<EB>(Ls, Ds, (j + 1) * EB, 1, h, nn, dd);
      smx<EB, MASK>(s[1], dp[1], j * EB, nl, dl, sl2, 1, tmask, tsq);
      if (j + 1 < 2 * DT) {
#pragma unroll
        for (int e = 0; e < EB; ++e) { nl[e] = nn[e]; dl[e] = dd[e]; }
      }
      if ((j + 1) * EB == 8) { pf[1][0] = pack8(s[1], 0); df[1][0] = pack8(dp[1], 0); }
      ta = tan; tb = tbn;
      __builtin_amdgcn_sched_barrier(0);
    }
    pf[1][1] = pack8(s[1], 1); df[1][1] = pack8(dp[1], 1);
    // ---- stage C
#pragma unroll
    for (int j = 0; j < 2 * DT; ++j) {
      u16x8 tan, tbn;
      if (j + 1 < 2 * DT) { tan = trf(Gs, toff, 1, j + 1); tbn = trf(Qs, toff, 1, j + 1); }
      mfma32_acc(dv[j >> 1], ta, pf[1][j & 1]);
      mfma32_acc(dk[j >> 1], tb, df[1][j & 1]);
      ta = tan; tb = tbn;
      __builtin_amdgcn_sched_barrier(0);
    }
    acc_fence();   // inline-asm MFMA results are invisible to the hazard recognizer: retire before any copy
  }
};

template <int D, bool CAUSAL, int OCC>
__global__ __launch_bounds__(NT, OCC) void fa_bwd_dkdv_v3_kernel(AttnParams p) {
  constexpr int KS = D / 16, DT = D / 32, TE = TILE * D;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TE];        // [buf][Q | dO]
  __shared__ __attribute__((aligned(16))) float sstat[2][2][TILE];    // [buf][lse | delta]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const BlockCoord bc = block_order(false, p.order, 1);   // causal: low key blocks see the most queries
  const bool remap = CAUSAL || p.order != 0;
  const int b = sgpr(remap ? bc.b : (int)blockIdx.z), hk = sgpr(remap ? bc.h : (int)blockIdx.y);
  const int kb = sgpr(remap ? bc.t : (int)blockIdx.x);
  const int group = p.H / p.Hkv;
  const int off = p.Sk - p.Sq;
  const int kw = kb * 128 + w * 32, key = kw + c32;
  const bf16_t* Kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vp = p.v + b * p.v_sb + hk * p.v_sh;
  const float sl2 = p.scale * LOG2E;

  u16x8 kf[KS], vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (key < p.Sk && !(p.diag & 1)) {
      kf[ks] = *reinterpret_cast<const u16x8*>(Kp + (int64_t)key * p.k_ss + 16 * ks + 8 * h);
      vf[ks] = *reinterpret_cast<const u16x8*>(Vp + (int64_t)key * p.v_ss + 16 * ks + 8 * h);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) { kf[ks][k] = 0; vf[ks][k] = 0; }
    }
  }
  retire(kf);
  retire(vf);
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }

  int roff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int toff[DT][2];
  tr_offsets<D>(lane, toff);

  const int qstart = CAUSAL ? max(0, kb * 128 - off) / TILE * TILE : 0;
  const int qtiles = p.Sq > qstart ? (p.Sq - qstart + TILE - 1) / TILE : 0;
  const int total = qtiles * group;

  DmaLane<D> lq, lg;
  lq.init(p.q_ss, w, lane);
  lg.init(p.do_ss, w, lane);
  // (query head, query tile) of the next tile to stage / of the tile being computed, advanced by counters
  // (wave-uniform: no integer division -- a VALU sequence -- per tile)
  int iss_hi = 0, iss_qi = 0, cur_qi = 0;
  auto issue = [&](int buf) {
    const int q0 = sgpr(qstart + iss_qi * TILE), hq = sgpr(hk * group + iss_hi);
    bf16_t* base = smem + buf * 2 * TE;
    lq.issue(p.q + b * p.q_sb + hq * p.q_sh, p.q_ss, q0, p.Sq, base, w);
    lg.issue(p.dout + b * p.do_sb + hq * p.do_sh, p.do_ss, q0, p.Sq, base + TE, w);
    if (w == 0) dma_f32_row(p.delta + (int64_t)p.B * p.H * p.Sq + ((int64_t)b * p.H + hq) * p.Sq, q0, p.Sq, sstat[buf][0], lane);
    if (w == 1) dma_f32_row(p.delta + ((int64_t)b * p.H + hq) * p.Sq, q0, p.Sq, sstat[buf][1], lane);
    if (++iss_qi == qtiles) { iss_qi = 0; ++iss_hi; }
  };
  if (total > 0) issue(0);

  for (int it = 0; it < total; it += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int cur = it + u;
      if (cur >= total) break;
      dma_barrier();
      if (cur + 1 < total) issue(1 - u);
      const int q0 = sgpr(qstart + cur_qi * TILE);
      if (++cur_qi == qtiles) cur_qi = 0;
      if (CAUSAL && q0 + TILE - 1 + off < kw) continue;         // every query of the tile precedes these keys
      const bf16_t* Qs = smem + u * 2 * TE;
      const float* Ls = sstat[u][0];
      // rows of S = queries q0 + rr (+4h) with rr in [0, 64); masked if rr < tmask or rr >= tsq
      const int tmask = CAUSAL ? key - off - q0 - 4 * h : -1;
      const int tsq = p.Sq - q0 - 4 * h;
      if (CAUSAL && (p.mask_all || kw + 31 - off - q0 > 0))   // some query of the tile precedes some key of this wave
        BwdKVTile<D, CAUSAL>::template run<true>(Qs, Qs + TE, Ls, Ls + TILE, kf, vf, roff, toff, dk, dv, sl2, tmask,
                                                 tsq, h);
      else
        BwdKVTile<D, CAUSAL>::template run<false>(Qs, Qs + TE, Ls, Ls + TILE, kf, vf, roff, toff, dk, dv, sl2, tmask,
                                                  tsq, h);
    }
  }
  acc_fence();
  const bool st = key < p.Sk && !(p.diag & 2);
  store_row16<DT>(p.dk + b * p.dk_sb + hk * p.dk_sh + (int64_t)key * p.dk_ss, dk, p.scale, h, st);
  store_row16<DT>(p.dv + b * p.dv_sb + hk * p.dv_sh + (int64_t)key * p.dv_ss, dv, 1.0f, h, st);
}

// ------------------------------------------------------------------------------------------------
// dK/dV, persistent (default where eligible; v3 above: PDT_FA_DKDV=3).  At the flagship shape a v3 workgroup computes ~9 query
// tiles, and with one workgroup per CU (320 registers per lane) nothing overlaps its prologue (the K / V fragments
// of its 128 keys from HBM, the first Q / dO tile) or its epilogue (the dK / dV stores): measured as a fixed cost
// of 0.46 ms of the kernel's 1.41 ms (S 1024 vs 8192 at equal tokens, profiles/r5/r5h_attn_fixed_cost.txt).  Here
// one workgroup per CU walks a stream of (key block, query tile) pairs across work items:
//   * the tile ring continues across items -- the last tile of item i stages the first Q / dO tile of item i+1;
//   * the next item's K / V fragments are loaded into a second register set during that last tile;
//   * the dK / dV stores are buffer stores with a range-checked resource (rows past Sk dropped, no branch), so
//     their count is fixed and the next item's first barrier waits with vmcnt(#stores) -- for everything issued
//     before them -- instead of draining the stores too.
// Items are dealt heavy-first (low key blocks see the most queries under the causal mask) in snake order.
// ------------------------------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void store_row16_rs(__amdgpu_buffer_rsrc_t rs, uint32_t row_byte, const f32x16 (&acc)[DT],
                                               float scale, int h) {
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      unsigned a[2], c[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int g0 = 2 * pr, g1 = 2 * pr + 1;
        a[k] = (unsigned)f2bf(acc[dt][4 * g0 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g0 + 2 * k + 1] * scale) << 16);
        c[k] = (unsigned)f2bf(acc[dt][4 * g1 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g1 + 2 * k + 1] * scale) << 16);
        const auto r = __builtin_amdgcn_permlane32_swap(a[k], c[k], false, false);
        a[k] = r[0];
        c[k] = r[1];
      }
      u32x4 v;
      v[0] = a[0]; v[1] = a[1]; v[2] = c[0]; v[3] = c[1];
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(row_byte + (uint32_t)(dt * 32 + 16 * pr + 8 * h) * 2u), 0, 0);
    }
}

struct KvItem {
  int b, hk, kb, qstart, qtiles, total;
};

template <int D, bool CAUSAL>
__device__ __forceinline__ KvItem kv_item(const AttnParams& p, int j) {
  const int bh = p.B * p.Hkv, group = p.H / p.Hkv, off = p.Sk - p.Sq;
  KvItem it;
  it.kb = sgpr(j / bh);
  const int rest = j - it.kb * bh;
  it.b = sgpr(rest / p.Hkv);
  it.hk = sgpr(rest - it.b * p.Hkv);
  it.qstart = CAUSAL ? max(0, it.kb * 128 - off) / TILE * TILE : 0;
  it.qtiles = p.Sq > it.qstart ? (p.Sq - it.qstart + TILE - 1) / TILE : 0;
  it.total = it.qtiles * group;
  return it;
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(NT, 1) void fa_bwd_dkdv_p_kernel(AttnParams p, int nitems, int upr) {
  constexpr int KS = D / 16, DT = D / 32, TE = TILE * D, NSTORE = 2 * 2 * DT;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TE];        // [buf][Q | dO]
  __shared__ __attribute__((aligned(16))) bf16_t kvs[2][2 * TE];      // [K | V][128 key rows, two tile images]
  __shared__ __attribute__((aligned(16))) float sstat[2][2][TILE];    // [buf][lse | delta]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int G = gridDim.x, bid = blockIdx.x;
  const int group = p.H / p.Hkv;
  const int off = p.Sk - p.Sq;
  const float sl2 = p.scale * LOG2E;
  // upr == 0: snake over the heavy-first order (item j = kb * B * Hkv + unit).  upr > 0 (unit-local order): the
  // nkb / 2 workgroups of one (batch, kv head) unit sit on one XCD (ids b, b + 8, ... share an XCD) and each runs
  // key blocks kb = i and nkb - 1 - i of it back to back (causal: 16 - 2 i + 2 + 2 i query tiles, every pair the
  // same), so the unit's key blocks stream its Q / dO tiles together out of that XCD's L2 instead of 256 unrelated
  // streams from HBM; upr = units per XCD per round
  const int nkb = (p.Sk + 127) / 128, bh = p.B * p.Hkv;
  auto item_of = [&](int r) {
    if (upr == 0) return r * G + ((r & 1) ? G - 1 - bid : bid);
    const int loc = bid >> 3, pi = loc % (nkb >> 1), slot = loc / (nkb >> 1);
    const int u = ((r >> 1) * upr + slot) * 8 + (bid & 7);
    if (u >= bh) return nitems;
    return ((r & 1) ? nkb - 1 - pi : pi) * bh + u;
  };

  int r = 0;
  const int j0 = item_of(0);
  if (j0 >= nitems) return;
  KvItem cur = kv_item<D, CAUSAL>(p, j0);

  int roff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int toff[DT][2];
  tr_offsets<D>(lane, toff);

  DmaLane<D> lq, lg;
  lq.init(p.q_ss, w, lane);
  lg.init(p.do_ss, w, lane);
  const uint32_t sm0 = lds_u32(smem), ss0 = lds_u32(&sstat[0][0][0]), kv0 = lds_u32(&kvs[0][0]);
  auto issue = [&](const KvItem& it, int hi, int qi, int buf) {
    const int q0 = sgpr(it.qstart + qi * TILE), hq = sgpr(it.hk * group + hi);
    const uint32_t base = sm0 + (uint32_t)(buf * 2 * TE * 2);
    lq.issue_at(p.q + it.b * p.q_sb + hq * p.q_sh, p.q_ss, q0, p.Sq, base, w);
    lg.issue_at(p.dout + it.b * p.do_sb + hq * p.do_sh, p.do_ss, q0, p.Sq, base + TE * 2, w);
    const uint32_t sb = ss0 + (uint32_t)(buf * 2 * TILE * 4);
    if (w == 0)
      dma_f32_row_at(p.delta + (int64_t)p.B * p.H * p.Sq + ((int64_t)it.b * p.H + hq) * p.Sq, q0, p.Sq, sb, lane);
    if (w == 1) dma_f32_row_at(p.delta + ((int64_t)it.b * p.H + hq) * p.Sq, q0, p.Sq, sb + TILE * 4, lane);
  };
  // an item's 128 K and V rows into kvs (two tile images each; rows past Sk read 0 from the range check)
  // (lane offsets computed here, once per item: no registers held for them across the tile loop)
  auto issue_kv = [&](const KvItem& it) {
    DmaLane<D> l;
    const bf16_t* Kp = p.k + it.b * p.k_sb + it.hk * p.k_sh;
    const bf16_t* Vp = p.v + it.b * p.v_sb + it.hk * p.v_sh;
    l.init(p.k_ss, w, lane);
#pragma unroll
    for (int half = 0; half < 2; ++half)
      l.issue_at(Kp, p.k_ss, it.kb * 128 + half * TILE, p.Sk, kv0 + (uint32_t)(half * TE * 2), w);
    l.init(p.v_ss, w, lane);
#pragma unroll
    for (int half = 0; half < 2; ++half)
      l.issue_at(Vp, p.v_ss, it.kb * 128 + half * TILE, p.Sk, kv0 + (uint32_t)((2 * TE + half * TE) * 2), w);
  };
  // this wave's 32 key rows: image w / 2, rows 32 (w % 2) + c32 (swizzle phase = c32's)
  u16x8 kf[KS], vf[KS];
  auto read_kv = [&]() {
    const bf16_t* kb_ = &kvs[0][0] + (w >> 1) * TE + (w & 1) * 32 * D;
    const bf16_t* vb_ = &kvs[1][0] + (w >> 1) * TE + (w & 1) * 32 * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *reinterpret_cast<const u16x8*>(kb_ + roff[ks]);
      vf[ks] = *reinterpret_cast<const u16x8*>(vb_ + roff[ks]);
    }
  };
  auto store_item = [&](const KvItem& it, const f32x16 (&dk_)[DT], const f32x16 (&dv_)[DT]) {
    const int rows = min(128, p.Sk - it.kb * 128);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.dk + it.b * p.dk_sb + it.hk * p.dk_sh + (int64_t)it.kb * 128 * p.dk_ss), (short)0,
        (int)(((int64_t)(rows - 1) * p.dk_ss + D) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.dv + it.b * p.dv_sb + it.hk * p.dv_sh + (int64_t)it.kb * 128 * p.dv_ss), (short)0,
        (int)(((int64_t)(rows - 1) * p.dv_ss + D) * 2), 0x00020000);
    const int row = w * 32 + c32;
    store_row16_rs<DT>(rk, (uint32_t)(row * p.dk_ss * 2), dk_, p.scale, h);
    store_row16_rs<DT>(rv, (uint32_t)(row * p.dv_ss * 2), dv_, 1.0f, h);
  };
  // every item has >= 1 query tile: the host launches this kernel only for Sq, Sk > 0 (causal: the first query
  // tile that sees key block kb starts below Sq for every kb < Sk / 128)

  // prologue: the first item's K / V and first Q / dO tile
  issue_kv(cur);
  issue(cur, 0, 0, 0);
  dma_barrier();
  read_kv();

  // The item loop is the outer loop; the tile loop inside it is v3's, unrolled by the 2-deep ring with the buffer
  // a compile-time constant.  Every item has an EVEN number of query tiles (host condition: Sq, Sk multiples of 128
  // and Sq == Sk under the causal mask), so each item starts on buffer 0 and the last tile (buffer 1) stages the
  // next item's first tile into buffer 0.  The epilogue and the accumulator reset sit outside the tile loop.
  bool first_item = true;
  for (;;) {
    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }
    int iss_hi = 0, iss_qi = 1;        // next tile of this item to stage (tile 0 already is)
    if (iss_qi == cur.qtiles) { iss_qi = 0; ++iss_hi; }
    const int jn = item_of(r + 1);
    const int kw = cur.kb * 128 + w * 32, key = kw + c32;
    int cur_qi = 0;
    for (int ct = 0; ct < cur.total; ct += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 0 && ct == 0) {
          if (!first_item) {
            // everything issued before the previous item's NSTORE dK / dV stores (this tile's DMA, this item's
            // K / V rows) has landed; the stores themselves may still be in flight
            vm_wait<NSTORE>();
            __syncthreads();
            read_kv();
          }
        } else {
          dma_barrier();
        }
        if (ct + u + 1 < cur.total) {
          issue(cur, iss_hi, iss_qi, 1 - u);
          if (++iss_qi == cur.qtiles) { iss_qi = 0; ++iss_hi; }
        } else if (jn < nitems) {
          const KvItem nx = kv_item<D, CAUSAL>(p, jn);
          issue(nx, 0, 0, 1 - u);        // the next item's first tile and K / V rows ride this tile's compute
          issue_kv(nx);
        }
        const int q0 = sgpr(cur.qstart + cur_qi * TILE);
        if (++cur_qi == cur.qtiles) cur_qi = 0;
        if (CAUSAL && q0 + TILE - 1 + off < kw) continue;         // every query of the tile precedes these keys
        const bf16_t* Qs = smem + u * 2 * TE;
        const float* Ls = sstat[u][0];
        const int tmask = CAUSAL ? key - off - q0 - 4 * h : -1;
        const int tsq = p.Sq - q0 - 4 * h;
        if (CAUSAL && (p.mask_all || kw + 31 - off - q0 > 0))
          BwdKVTile<D, CAUSAL>::template run<true>(Qs, Qs + TE, Ls, Ls + TILE, kf, vf, roff, toff, dk, dv, sl2, tmask,
                                                   tsq, h);
        else
          BwdKVTile<D, CAUSAL>::template run<false>(Qs, Qs + TE, Ls, Ls + TILE, kf, vf, roff, toff, dk, dv, sl2,
                                                    tmask, tsq, h);
      }
    }
    acc_fence();
    store_item(cur, dk, dv);
    if (jn >= nitems) return;
    ++r;
    cur = kv_item<D, CAUSAL>(p, jn);
    first_item = false;
  }
}

// dQ kernels: the per-element select inside every tile's softmax steps (1) or the dS post-mask on diagonal tiles
// only (0, default) -- a compile-time A/B switch (-DPDT_FA_DQ_MASK_EVERY_TILE=1)
#ifndef PDT_FA_DQ_MASK_EVERY_TILE
#define PDT_FA_DQ_MASK_EVERY_TILE 0
#endif
constexpr bool kMaskEveryTile = PDT_FA_DQ_MASK_EVERY_TILE != 0;

template <int D, bool CAUSAL>
struct BwdQTile {
  static constexpr int KS = D / 16, DT = D / 32;
  static constexpr int EA = 16 / KS;   // softmax elements per pipeline step (KS == 2 DT)
  // K / V row fragment of step i (subtile i / KS, k-step i % KS)
  __device__ __forceinline__ static u16x8 rowf(const bf16_t* base, const int (&roff)[KS], int i) {
    return *reinterpret_cast<const u16x8*>(base + roff[i % KS] + (i / KS) * 32 * D);
  }
  __device__ __forceinline__ static u16x8 trf(const bf16_t* base, const int (&toff)[DT][2], int kt, int j) {
    const int o = (kt * 32 + 16 * (j & 1)) * D;
    return tr_pair(base + toff[j >> 1][0] + o, base + toff[j >> 1][1] + o);
  }
  // dS^T registers [e0, e0 + EA) of key subtile kt (rows = keys, lanes = queries);
  // MASK (wave-uniform): the tile holds keys past some lane's last valid key (causal diagonal / ragged Sk)
  template <bool MASK>
  __device__ __forceinline__ static void smx(const f32x16& sv, f32x16& dpv, int e0, int kt, float sl2, float nlse2,
                                             float dl, int lim) {
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int r = e0 + e, rr = (r & 3) + 8 * (r >> 2) + 32 * kt;
      float pv = fast_exp2(fmaf(sv[r], sl2, nlse2));
      if constexpr (MASK) pv = rr > lim ? 0.f : pv;
      dpv[r] = pv * (dpv[r] - dl);
    }
  }
  // dS registers [R0, R1) of key subtile kt -> 0 where the key row is past lim.  Only dS feeds an MFMA in this
  // kernel, so masking it after the fact equals masking P (the select discards whatever exp2 made of a masked
  // score, inf / NaN included)
  template <int R0, int R1>
  __device__ __forceinline__ static void mask_ds(f32x16& dpv, int kt, int lim) {
#pragma unroll
    for (int r = R0; r < R1; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + 32 * kt;
      dpv[r] = rr > lim ? 0.f : dpv[r];
    }
  }
  // One 64-key tile, hand-pipelined like BwdKVTile: stage A = S/dP chains of both key subtiles (subtile
  // 0's softmax-gradient under subtile 1's chain), stage B = dQ += dS0 K0 (subtile 1's softmax under it),
  // stage C = dQ += dS1 K1.  MASK: selects against lim (= last valid key row of this lane's query) inside the
  // softmax steps of every tile; otherwise ``diag`` (wave-uniform: the tile crosses the causal diagonal or Sk)
  // masks the finished dS registers in three short branches -- the interior tiles issue no mask VALU at all and
  // the body stays ONE copy (a second unrolled body cost 20 % in instruction-cache misses)
  template <bool MASK>
  __device__ __forceinline__ static void run(const bf16_t* Ks, const bf16_t* Vs, const u16x8 (&qf)[KS],
                                             const u16x8 (&gf)[KS], const int (&roff)[KS], const int (&toff)[DT][2],
                                             f32x16 (&dq)[DT], float sl2, float nlse2, float dl, int lim,
                                             bool diag = false) {
    f32x16 s[2], dp[2];
    u16x8 df[2][2];
    const f32x16 z = zero16();
    u16x8 ka = rowf(Ks, roff, 0), va = rowf(Vs, roff, 0), ta;
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      const int kt = i / KS, ks = i % KS;
      u16x8 kn, vn;
      if (i + 1 < 2 * KS) { kn = rowf(Ks, roff, i + 1); vn = rowf(Vs, roff, i + 1); }
      else ta = trf(Ks, toff, 0, 0);
      s[kt] = mfma32(ka, qf[ks], ks == 0 ? z : s[kt]);
      dp[kt] = mfma32(va, gf[ks], ks == 0 ? z : dp[kt]);
      if (kt == 1) smx<MASK>(s[0], dp[0], ks * EA, 0, sl2, nlse2, dl, lim);
      ka = kn; va = vn;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!MASK && diag) mask_ds<0, 16>(dp[0], 0, lim);
    df[0][0] = pack8(dp[0], 0); df[0][1] = pack8(dp[0], 1);
#pragma unroll
    for (int j = 0; j < 2 * DT; ++j) {
      const u16x8 tn = j + 1 < 2 * DT ? trf(Ks, toff, 0, j + 1) : trf(Ks, toff, 1, 0);
      dq[j >> 1] = mfma32(ta, df[0][j & 1], dq[j >> 1]);
      smx<MASK>(s[1], dp[1], j * EA, 1, sl2, nlse2, dl, lim);
      if ((j + 1) * EA == 8) {
        if (!MASK && diag) mask_ds<0, 8>(dp[1], 1, lim);
        df[1][0] = pack8(dp[1], 0);
      }
      ta = tn;
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!MASK && diag) mask_ds<8, 16>(dp[1], 1, lim);
    df[1][1] = pack8(dp[1], 1);
#pragma unroll
    for (int j = 0; j < 2 * DT; ++j) {
      u16x8 tn;
      if (j + 1 < 2 * DT) tn = trf(Ks, toff, 1, j + 1);
      dq[j >> 1] = mfma32(ta, df[1][j & 1], dq[j >> 1]);
      ta = tn;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
};

template <int D, bool CAUSAL, int OCC = 2>
__global__ __launch_bounds__(NT, OCC) void fa_bwd_dq_v3_kernel(AttnParams p) {
  constexpr int KS = D / 16, DT = D / 32, TE = TILE * D;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TE];   // [buf][K | V]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const BlockCoord bc = block_order(true, p.order, p.H / p.Hkv);
  const bool remap = CAUSAL || p.order != 0;
  const int b = sgpr(remap ? bc.b : (int)blockIdx.z), hq = sgpr(remap ? bc.h : (int)blockIdx.y);
  const int qb = sgpr(remap ? bc.t : (int)blockIdx.x);
  const int hk = sgpr(hq / (p.H / p.Hkv));
  const int off = p.Sk - p.Sq;
  const int q0 = qb * 128, qw = q0 + w * 32, qrow = qw + c32;
  const bf16_t* Qp = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* Gp = p.dout + b * p.do_sb + hq * p.do_sh;
  const bf16_t* Kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vp = p.v + b * p.v_sb + hk * p.v_sh;
  const float sl2 = p.scale * LOG2E;

  int kend = p.Sk;
  if (CAUSAL) kend = min(p.Sk, q0 + 128 + off);
  const int ntiles = kend > 0 ? (kend + TILE - 1) / TILE : 0;
  // OCC 2 (256 VGPRs): the builtin DMA -- the inline-asm form spills 21-27 VGPRs here (scratch reloads with
  // vmcnt(0) before every DMA), even with the per-lane offsets recomputed at each issue
  DmaLane<D, OCC == 1> lk, lv;
  lk.init(p.k_ss, w, lane);
  lv.init(p.v_ss, w, lane);
  if (ntiles > 0) {
    lk.issue(Kp, p.k_ss, 0, p.Sk, smem, w);
    lv.issue(Vp, p.v_ss, 0, p.Sk, smem + TE, w);
  }
  u16x8 qf[KS], gf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (qrow < p.Sq) {
      qf[ks] = *reinterpret_cast<const u16x8*>(Qp + (int64_t)qrow * p.q_ss + 16 * ks + 8 * h);
      gf[ks] = *reinterpret_cast<const u16x8*>(Gp + (int64_t)qrow * p.do_ss + 16 * ks + 8 * h);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) { qf[ks][k] = 0; gf[ks][k] = 0; }
    }
  }
  const float nlse2 = qrow < p.Sq ? -p.lse[((int64_t)b * p.H + hq) * p.Sq + qrow] * LOG2E : -INFINITY;
  const float dl = p.fuse_delta ? row_delta<KS>(p, gf, b, hq, qrow, h)
                                : (qrow < p.Sq ? p.delta[((int64_t)b * p.H + hq) * p.Sq + qrow] : 0.f);
  retire(qf);
  retire(gf);
  asm volatile("" :: "v"(nlse2), "v"(dl));
  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = zero16();
  int roff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int toff[DT][2];
  tr_offsets<D>(lane, toff);
  const int lim0 = min(p.Sk - 1, CAUSAL ? qrow + off : p.Sk - 1) - 4 * h;

  for (int t = 0; t < ntiles; t += 2) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tt = t + u;
      if (tt >= ntiles) break;
      dma_barrier();
      if (tt + 1 < ntiles) {
        bf16_t* nb = smem + (1 - u) * 2 * TE;
        lk.issue(Kp, p.k_ss, (tt + 1) * TILE, p.Sk, nb, w);
        lv.issue(Vp, p.v_ss, (tt + 1) * TILE, p.Sk, nb + TE, w);
      }
      const int k0 = tt * TILE;
      if (CAUSAL && k0 > qw + 31 + off) continue;               // every key of the tile follows these queries
      const bf16_t* Ks = smem + u * 2 * TE;
      const bool diag = (k0 + TILE > p.Sk) || (CAUSAL && k0 + TILE - 1 > qw + off);
      if (kMaskEveryTile)
        BwdQTile<D, CAUSAL>::template run<true>(Ks, Ks + TE, qf, gf, roff, toff, dq, sl2, nlse2, dl, lim0 - k0);
      else
        BwdQTile<D, CAUSAL>::template run<false>(Ks, Ks + TE, qf, gf, roff, toff, dq, sl2, nlse2, dl, lim0 - k0, diag);
    }
  }
  if (p.cs_q == nullptr) {
    store_row16<DT>(p.dq + b * p.dq_sb + hq * p.dq_sh + (int64_t)qrow * p.dq_ss, dq, p.scale, h, qrow < p.Sq);
  } else {
    float vals[DT * 16];
    store_row16_vals<DT>(p.dq + b * p.dq_sb + hq * p.dq_sh + (int64_t)qrow * p.dq_ss, dq, p.scale, h, qrow < p.Sq,
                         vals);
    wg_colsum_store<D, 4>(vals, reinterpret_cast<float*>(smem),
                          p.cs_q + ((int64_t)b * gridDim.x + qb) * p.H * D + hq * D, w, lane);
  }
}


// dQ v4: dQ v3's per-wave tile on a 512-thread workgroup (8 waves x 32 query rows = 256 rows per staged
// K/V tile, 384 instead of 192 FLOP per staged byte) with the NBUF-deep counted-vmcnt ring of forward v7.
template <int D, bool CAUSAL, int NBUF>
__global__ __launch_bounds__(NT8, 1) void fa_bwd_dq_v4_kernel(AttnParams p) {
  constexpr int KS = D / 16, DT = D / 32, TE = TILE * D, NW = 8, BM = 32 * NW;
  using Dma = DmaLane<D, true, NW>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NBUF * 2 * TE];   // [stage][K | V]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const BlockCoord bc = block_order(true, p.order, p.H / p.Hkv);
  const bool remap = CAUSAL || p.order != 0;
  const int b = sgpr(remap ? bc.b : (int)blockIdx.z), hq = sgpr(remap ? bc.h : (int)blockIdx.y);
  const int qb = sgpr(remap ? bc.t : (int)blockIdx.x);
  const int hk = sgpr(hq / (p.H / p.Hkv));
  const int off = p.Sk - p.Sq;
  const int q0 = qb * BM, qw = q0 + w * 32, qrow = qw + c32;
  const bf16_t* Qp = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* Gp = p.dout + b * p.do_sb + hq * p.do_sh;
  const bf16_t* Kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vp = p.v + b * p.v_sb + hk * p.v_sh;
  const float sl2 = p.scale * LOG2E;

  int kend = p.Sk;
  if (CAUSAL) kend = min(p.Sk, q0 + BM + off);
  const int ntiles = kend > 0 ? (kend + TILE - 1) / TILE : 0;
  Dma lk, lv;
  lk.init(p.k_ss, w, lane);
  lv.init(p.v_ss, w, lane);
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < ntiles) {
      lk.issue(Kp, p.k_ss, t * TILE, p.Sk, smem + t * 2 * TE, w);
      lv.issue(Vp, p.v_ss, t * TILE, p.Sk, smem + t * 2 * TE + TE, w);
    }
  u16x8 qf[KS], gf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (qrow < p.Sq && !(p.diag & 4)) {
      qf[ks] = *reinterpret_cast<const u16x8*>(Qp + (int64_t)qrow * p.q_ss + 16 * ks + 8 * h);
      gf[ks] = *reinterpret_cast<const u16x8*>(Gp + (int64_t)qrow * p.do_ss + 16 * ks + 8 * h);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) { qf[ks][k] = 0; gf[ks][k] = 0; }
    }
  }
  const float nlse2 = qrow < p.Sq ? -p.lse[((int64_t)b * p.H + hq) * p.Sq + qrow] * LOG2E : -INFINITY;
  const float dl = (p.diag & 4) ? 0.f : p.fuse_delta ? row_delta<KS>(p, gf, b, hq, qrow, h)
                                : (qrow < p.Sq ? p.delta[((int64_t)b * p.H + hq) * p.Sq + qrow] : 0.f);
  retire(qf);
  retire(gf);
  asm volatile("" :: "v"(nlse2), "v"(dl));
  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = zero16();
  int roff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int toff[DT][2];
  tr_offsets<D>(lane, toff);
  const int lim0 = min(p.Sk - 1, CAUSAL ? qrow + off : p.Sk - 1) - 4 * h;

  int stage = 0;
  for (int t = 0; t < ntiles; ++t) {
    ring_wait<2 * Dma::NI, NBUF>(t + 1 < ntiles);
    if (t + NBUF - 1 < ntiles) {
      const int ns = stage == 0 ? NBUF - 1 : stage - 1;
      bf16_t* nb = smem + ns * 2 * TE;
      lk.issue(Kp, p.k_ss, (t + NBUF - 1) * TILE, p.Sk, nb, w);
      lv.issue(Vp, p.v_ss, (t + NBUF - 1) * TILE, p.Sk, nb + TE, w);
    }
    const int k0 = t * TILE;
    if (!(CAUSAL && k0 > qw + 31 + off)) {
      const bf16_t* Ks = smem + stage * 2 * TE;
      const bool diag = (k0 + TILE > p.Sk) || (CAUSAL && k0 + TILE - 1 > qw + off);
      if (kMaskEveryTile)
        BwdQTile<D, CAUSAL>::template run<true>(Ks, Ks + TE, qf, gf, roff, toff, dq, sl2, nlse2, dl, lim0 - k0);
      else
        BwdQTile<D, CAUSAL>::template run<false>(Ks, Ks + TE, qf, gf, roff, toff, dq, sl2, nlse2, dl, lim0 - k0, diag);
    }
    stage = stage + 1 == NBUF ? 0 : stage + 1;
  }
  if (p.diag & 8) {
  } else if (p.cs_q == nullptr) {
    store_row16<DT>(p.dq + b * p.dq_sb + hq * p.dq_sh + (int64_t)qrow * p.dq_ss, dq, p.scale, h, qrow < p.Sq);
  } else {
    float vals[DT * 16];
    store_row16_vals<DT>(p.dq + b * p.dq_sb + hq * p.dq_sh + (int64_t)qrow * p.dq_ss, dq, p.scale, h, qrow < p.Sq,
                         vals);
    wg_colsum_store<D, NW>(vals, reinterpret_cast<float*>(smem),
                           p.cs_q + ((int64_t)b * gridDim.x + qb) * p.H * D + hq * D, w, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// dQ, persistent (OPT-IN: PDT_FA_DQP=1 or pdt_flash_attn_set_dqp(1); v4 stays the default).  v4's workgroup loads
// the Q / dO rows of its 256 queries (and the O rows for delta) in a prologue nothing overlaps -- 0.37 ms of the
// kernel's 1.01 at the flagship shape (profiles/r5/r5h_attn_fixed_cost.txt).  Here one workgroup per CU walks
// (batch, head, query block) items heavy-first in snake order: the K / V ring continues across items (the last
// tile stages the next item's first tile), the next item's Q / dO rows load under the epilogue and the next ring
// wait, its O rows DMA into LDS beside its first K / V tile (delta fused as in v4), and dQ leaves through
// range-checked buffer stores whose count is fixed, so the next item's first ring wait leaves them in flight.
// Measured at the flagship shape (profiles/r5/r5o_dq_persistent_ab.txt): 0.912 ms + the 0.171 ms delta pass with
// delta unfused, 1.163 ms fused, against v4's 1.04-1.07 ms -- the hidden prologue is paid back in register
// pressure (256 VGPRs, 16-34 spilled) -- so it stays opt-in.  Requires an even tile count per item: Sq a multiple
// of 256 and Sq == Sk under the causal mask (4 (qb + 1) tiles), Sk a multiple of 128 otherwise.
// ------------------------------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void store_row16_vals_rs(__amdgpu_buffer_rsrc_t rs, uint32_t row_byte, const f32x16 (&acc)[DT],
                                                    float scale, int h, bool ok, float (&v)[DT * 16]) {
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      unsigned a[2], c[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int g0 = 2 * pr, g1 = 2 * pr + 1;
        a[k] = (unsigned)f2bf(acc[dt][4 * g0 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g0 + 2 * k + 1] * scale) << 16);
        c[k] = (unsigned)f2bf(acc[dt][4 * g1 + 2 * k] * scale) | ((unsigned)f2bf(acc[dt][4 * g1 + 2 * k + 1] * scale) << 16);
        const auto r = __builtin_amdgcn_permlane32_swap(a[k], c[k], false, false);
        a[k] = r[0];
        c[k] = r[1];
      }
      u32x4 q;
      q[0] = a[0]; q[1] = a[1]; q[2] = c[0]; q[3] = c[1];
      __builtin_amdgcn_raw_buffer_store_b128(q, rs, (int)(row_byte + (uint32_t)(dt * 32 + 16 * pr + 8 * h) * 2u), 0, 0);
      const float m = ok ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[(dt * 2 + pr) * 8 + 2 * k] = m * __uint_as_float(q[k] << 16);
        v[(dt * 2 + pr) * 8 + 2 * k + 1] = m * __uint_as_float(q[k] & 0xffff0000u);
      }
    }
}

struct QItem {
  int b, hq, hk, qb, ntiles;
};

template <bool CAUSAL>
__device__ __forceinline__ QItem q_item(const AttnParams& p, int j, int nqb) {
  const int bh = p.B * p.H, off = p.Sk - p.Sq;
  QItem it;
  const int rank = sgpr(j / bh);
  const int rest = j - rank * bh;
  it.qb = sgpr(nqb - 1 - rank);                       // heavy first: high query blocks see the most keys
  it.b = sgpr(rest / p.H);
  it.hq = sgpr(rest - it.b * p.H);
  it.hk = it.hq / (p.H / p.Hkv);
  const int kend = CAUSAL ? min(p.Sk, it.qb * 256 + 256 + off) : p.Sk;
  it.ntiles = kend > 0 ? (kend + TILE - 1) / TILE : 0;
  return it;
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(NT8, 1) void fa_bwd_dq_p_kernel(AttnParams p, int nitems, int nqb) {
  constexpr int KS = D / 16, DT = D / 32, TE = TILE * D, NW = 8, NSTORE = 2 * DT;
  using Dma = DmaLane<D, true, NW>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * 2 * TE];   // [stage][K | V]
  __shared__ __attribute__((aligned(16))) float csl[NW * D];         // column-sum scratch (the ring stays live)
  __shared__ __attribute__((aligned(16))) bf16_t osm[4 * TE];        // the item's 256 O rows (fused delta)

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int G = gridDim.x, bid = blockIdx.x;
  const int off = p.Sk - p.Sq;
  const float sl2 = p.scale * LOG2E;
  auto item_of = [&](int r) { return r * G + ((r & 1) ? G - 1 - bid : bid); };

  int r = 0;
  const int j0 = item_of(0);
  if (j0 >= nitems) return;
  QItem cur = q_item<CAUSAL>(p, j0, nqb);

  Dma lk, lv;
  lk.init(p.k_ss, w, lane);
  lv.init(p.v_ss, w, lane);
  const uint32_t sm0 = lds_u32(smem);
  auto issue = [&](const QItem& it, int t, int stage) {
    const bf16_t* Kp = p.k + it.b * p.k_sb + it.hk * p.k_sh;
    const bf16_t* Vp = p.v + it.b * p.v_sb + it.hk * p.v_sh;
    const uint32_t base = sm0 + (uint32_t)(stage * 2 * TE * 2);
    lk.issue_at(Kp, p.k_ss, t * TILE, p.Sk, base, w);
    lv.issue_at(Vp, p.v_ss, t * TILE, p.Sk, base + TE * 2, w);
  };
  // the item's O rows -> osm (4 swizzled 64-row tiles, as K / V): issued beside the item's first K / V tile, so
  // the wait that lands that tile lands them too and no register holds them across the previous epilogue
  // (prefetching them into registers there spilled 92)
  const uint32_t os0 = lds_u32(osm);
  Dma lo;   // its lane offsets carry O's row stride (a packed projection's K rows are 3x longer)
  lo.init(p.o_ss, w, lane);
  auto issue_o = [&](const QItem& it) {
    if (!p.fuse_delta) return;
    const bf16_t* Op = p.o + it.b * p.o_sb + it.hq * p.o_sh;
#pragma unroll
    for (int i = 0; i < 4; ++i) lo.issue_at(Op, p.o_ss, it.qb * 256 + i * TILE, p.Sq, os0 + (uint32_t)(i * TE * 2), w);
  };
  u16x8 qf[KS], gf[KS];
  // this lane's query row of item it: Q / dO fragments and, for the fused delta, the natural lse (rows past Sq:
  // zeros / +inf); with the separate delta pass, -lse*log2(e) and delta straight from it
  // (returns {-lse*log2(e), delta or 0}: values, not captured references -- written through the lambdas'
  // references they lived in scratch and every tile reloaded them)
  auto load_rows = [&](const QItem& it) -> float2 {
    const int qrow = it.qb * 256 + w * 32 + c32;
    const bool ok = qrow < p.Sq;
    const bf16_t* Qp = p.q + it.b * p.q_sb + it.hq * p.q_sh;
    const bf16_t* Gp = p.dout + it.b * p.do_sb + it.hq * p.do_sh;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ok) {
        qf[ks] = *reinterpret_cast<const u16x8*>(Qp + (int64_t)qrow * p.q_ss + 16 * ks + 8 * h);
        gf[ks] = *reinterpret_cast<const u16x8*>(Gp + (int64_t)qrow * p.do_ss + 16 * ks + 8 * h);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) { qf[ks][k] = 0; gf[ks][k] = 0; }
      }
    }
    const int64_t ri = ((int64_t)it.b * p.H + it.hq) * p.Sq + qrow;
    if (p.fuse_delta) return make_float2(ok ? -p.lse[ri] * LOG2E : -INFINITY, 0.f);
    // the delta pass stored -lse * log2(e)
    return make_float2(ok ? p.delta[(int64_t)p.B * p.H * p.Sq + ri] : -INFINITY, ok ? p.delta[ri] : 0.f);
  };
  int roff[KS];
  const int F = swz_f<D>(c32);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = c32 * D + (((2 * ks + h) ^ F) << 3);
  int toff[DT][2];
  tr_offsets<D>(lane, toff);

  // fused delta = rowsum(dO * O) once osm has landed (rows past Sq: the DMA range check zero-filled them); the
  // h == 0 lane hands delta and the log2-domain lse to the dK/dV kernel (as the per-item kernel's row_delta does)
  auto finish_rows = [&](const QItem& it, float nlse2, float dl) -> float {
    if (!p.fuse_delta) return dl;
    const int qrow = it.qb * 256 + w * 32 + c32;
    const bf16_t* Os = osm + w * 32 * D;   // this lane's row sits in 64-row tile w / 2, at row (w & 1) * 32 + c32
    float acc = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 o = *reinterpret_cast<const u16x8*>(Os + roff[ks]);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += bf2f(o[e]) * bf2f(gf[ks][e]);
    }
    acc += __shfl_xor(acc, 32, 64);
    if (qrow < p.Sq && h == 0) {
      const int64_t idx = ((int64_t)it.b * p.H + it.hq) * p.Sq + qrow;
      p.delta[idx] = acc;
      p.delta[(int64_t)p.B * p.H * p.Sq + idx] = nlse2;
    }
    return acc;
  };

  issue(cur, 0, 0);
  issue_o(cur);
  float2 rl = load_rows(cur);
  float nlse2 = rl.x, dl = rl.y;
  bool first_item = true;
  for (;;) {
    f32x16 dq[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dq[dt] = zero16();
    const int jn = item_of(r + 1);
    const bool more = jn < nitems;
    const QItem nx = q_item<CAUSAL>(p, more ? jn : j0, nqb);
    const int q0 = cur.qb * 256, qw = q0 + w * 32, qrow = qw + c32;
    const int lim0 = min(p.Sk - 1, CAUSAL ? qrow + off : p.Sk - 1) - 4 * h;
    for (int t = 0; t < cur.ntiles; t += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int tt = t + u;
        if (tt == 0) {
          // everything issued before the previous item's dQ / column-sum stores has landed (this tile's DMA, the
          // O rows, this item's Q / dO rows); the stores may still be in flight.  osm is read here and
          // overwritten at the LAST tile's issue: ntiles >= 2 (Sq % 256 == 0, Sk % 128 == 0), so a barrier of a
          // later tile separates every wave's read from that DMA
          if (first_item) vm_wait<0>();
          else if (w < 2 && p.cs_q != nullptr) vm_wait<NSTORE + 1>();   // + the column-sum partial store
          else vm_wait<NSTORE>();
          __syncthreads();
          dl = finish_rows(cur, nlse2, dl);
        } else {
          vm_wait<0>();
          __syncthreads();
        }
        const bool last = tt + 1 == cur.ntiles;
        if (!last) issue(cur, tt + 1, 1 - u);
        else if (more) { issue(nx, 0, 1 - u); issue_o(nx); }
        const int k0 = tt * TILE;
        if (!(CAUSAL && k0 > qw + 31 + off)) {
          const bf16_t* Ks = smem + u * 2 * TE;
          const bool diag = (k0 + TILE > p.Sk) || (CAUSAL && k0 + TILE - 1 > qw + off);
          BwdQTile<D, CAUSAL>::template run<false>(Ks, Ks + TE, qf, gf, roff, toff, dq, sl2, nlse2, dl, lim0 - k0,
                                                   diag);
        }
      }
    }
    // the next item's Q / dO rows load under the epilogue (loading them right after the last tile's S / dP chains
    // kept them live beside stages B / C: 191 spilled registers)
    if (more) rl = load_rows(nx);
    // epilogue: dQ rows (buffer stores: rows past Sq dropped by the range check) + this item's column sums, one
    // 32-column block (dt) at a time so only 16 values per lane are live beside the prefetched qf / gf
    {
      const int rows = min(256, p.Sq - q0);
      const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.dq + cur.b * p.dq_sb + cur.hq * p.dq_sh + (int64_t)q0 * p.dq_ss), (short)0,
          (int)(((int64_t)(rows - 1) * p.dq_ss + D) * 2), 0x00020000);
      const uint32_t row_byte = (uint32_t)((w * 32 + c32) * p.dq_ss * 2);
      const bool cs = p.cs_q != nullptr;
      const float m = qrow < p.Sq ? 1.f : 0.f;
      if (cs) lds_barrier();              // every wave is past its last read of csl (previous item)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        float v[16];
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          unsigned a[2], c[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int g0 = 2 * pr, g1 = 2 * pr + 1;
            a[k] = (unsigned)f2bf(dq[dt][4 * g0 + 2 * k] * p.scale) |
                   ((unsigned)f2bf(dq[dt][4 * g0 + 2 * k + 1] * p.scale) << 16);
            c[k] = (unsigned)f2bf(dq[dt][4 * g1 + 2 * k] * p.scale) |
                   ((unsigned)f2bf(dq[dt][4 * g1 + 2 * k + 1] * p.scale) << 16);
            const auto rr = __builtin_amdgcn_permlane32_swap(a[k], c[k], false, false);
            a[k] = rr[0];
            c[k] = rr[1];
          }
          u32x4 qv;
          qv[0] = a[0]; qv[1] = a[1]; qv[2] = c[0]; qv[3] = c[1];
          __builtin_amdgcn_raw_buffer_store_b128(qv, rq, (int)(row_byte + (uint32_t)(dt * 32 + 16 * pr + 8 * h) * 2u),
                                                 0, 0);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[pr * 8 + 2 * k] = m * __uint_as_float(qv[k] << 16);
            v[pr * 8 + 2 * k + 1] = m * __uint_as_float(qv[k] & 0xffff0000u);
          }
        }
        if (cs) {
          // sum over the 32 rows of this half-wave: reduce-scatter 16 -> 1 value per lane (masks 16..2), then the
          // xor-1 partner; lane c32 then holds value index c32 >> 1 = column dt*32 + 8h + (i & 7) + 16 (i >> 3)
          colsum32_step<16, 16, 16>(v, c32);
          v[0] += __shfl_xor(v[0], 1, 64);
          if (!(c32 & 1)) {
            const int i = c32 >> 1;
            csl[w * D + dt * 32 + 8 * h + (i & 7) + 16 * (i >> 3)] = v[0];
          }
        }
      }
      if (cs) {
        lds_barrier();
        if ((int)threadIdx.x < D) {
          float t = 0.f;
#pragma unroll
          for (int q = 0; q < NW; ++q) t += csl[q * D + threadIdx.x];
          p.cs_q[((int64_t)cur.b * nqb + cur.qb) * p.H * D + cur.hq * D + threadIdx.x] = t;
        }
      }
    }
    if (!more) return;
    ++r;
    cur = nx;
    nlse2 = rl.x;
    dl = rl.y;
    first_item = false;
  }
}

// kernel-variant selection: PDT_FA_FWD / PDT_FA_BWD env at first use, or pdt_flash_attn_set_variant()
int g_fwd_variant = -1, g_bwd_variant = -1, g_order = -1;
// block order bitmask (bit 0 forward, bit 1 dK/dV, bit 2 dQ): PDT_FA_ORDER / pdt_flash_attn_set_order, else
// per shape -- the forward groups (batch, kv head) units per XCD when the whole K/V no longer fits the 256 MB
// Infinity Cache (so heavy-first re-reads go to HBM) but one unit's K/V (2 x Sk x D bf16) fits an XCD's L2
// share: GPT-2 1.3B B96 (805 MB of K/V) 0.95 -> 0.68 ms; at B32 (268 MB), Llama-3 8B B8, GPT-2 124M B64 and
// S4096 grouping lost 4-10 %.  The backward kernels measured neutral (dK/dV v3) or slower (dQ v4) grouped.
// (profiles/r3_attn_ab*.jsonl; a persistent forward with pipelined block seams ran 5-45 % SLOWER than v5 in
// every shape but one, profiles/r3_attn_ab3_persistent_fwd.jsonl -- removed)
int block_order_mode(int B, int Hkv, int Sk, int D) {
  if (g_order < 0) {
    const char* e = getenv("PDT_FA_ORDER");
    if (e) g_order = atoi(e);
  }
  if (g_order >= 0) return g_order;
  const int64_t unit = (int64_t)Sk * D * 4, total = unit * B * Hkv;
  return (unit <= (1 << 20) && total > ((int64_t)384 << 20)) ? 1 : 0;
}

// dQ kernel: persistent (opt-in, PDT_FA_DQP=1) or the dQ variant below (default)
int g_dqp = -1;
bool dq_persistent(const AttnParams& p, int causal) {
  if (g_dqp < 0) { const char* e = getenv("PDT_FA_DQP"); g_dqp = e ? atoi(e) : 0; }
  if (!g_dqp || p.Sq <= 0 || p.Sq % 256 != 0) return false;
  return causal ? p.Sq == p.Sk : p.Sk % 128 == 0;
}
int dq_items(const AttnParams& p) { return p.B * p.H * (p.Sq / 256); }

// dK/dV kernel: persistent (default where every item has an even tile count; flagship layer 1.41 -> 1.26 ms,
// profiles/r5/r5m_dkdv_persistent_ab.txt) or v3 (PDT_FA_DKDV=3)
int g_dkdv_variant = -1;
int dkdv_items(const AttnParams& p) { return p.B * p.Hkv * ((p.Sk + 127) / 128); }
bool dkdv_persistent(const AttnParams& p) {
  if (g_dkdv_variant < 0) { const char* e = getenv("PDT_FA_DKDV"); g_dkdv_variant = e ? atoi(e) : 0; }
  // every item must have an even number of query tiles (the kernel's ring parity): Sq, Sk multiples of 128, and
  // Sq == Sk (no key / query offset) for the causal mask -- the shapes every model here runs
  return g_dkdv_variant != 3 && p.Sq > 0 && p.Sq % 128 == 0 && p.Sk % 128 == 0 && p.Sq == p.Sk;
}
// unit-local item order of the persistent dK/dV kernel (see fa_bwd_dkdv_p_kernel): units per XCD per round, or 0
// for the snake order -- needs an even key-block count, a grid of whole XCD rows of pairs (G / 8 a multiple of
// nkb / 2) and at least as many units as the grid hosts at once.  PDT_FA_DKDV_ORDER=0 forces the snake order.
int dkdv_upr(const AttnParams& p, int grid) {
  static const int forced = [] { const char* e = getenv("PDT_FA_DKDV_ORDER"); return e ? atoi(e) : -1; }();
  if (forced == 0) return 0;
  const int nkb = (p.Sk + 127) / 128, half = nkb / 2;
  if (nkb < 2 || nkb % 2 || grid % 8 || (grid / 8) % half) return 0;
  const int upr = (grid / 8) / half;
  return p.B * p.Hkv >= 8 * upr ? upr : 0;
}
int dkdv_grid(const AttnParams& p) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      n = 256;
    return n;
  }();
  const int n = dkdv_items(p);
  return n < cus ? n : cus;        // one workgroup per CU (320 registers per lane: one wave per SIMD)
}

int fwd_variant() {
  if (g_fwd_variant < 0) { const char* e = getenv("PDT_FA_FWD"); g_fwd_variant = e ? atoi(e) : 0; }
  return g_fwd_variant > 0 ? g_fwd_variant : 5;
}
// backward default: dQ v4 (variant 9) at head dim 128 (B96 S1024: 2.77 -> 2.58 ms), v3 at 64 where the 8-wave
// dQ measured 1-3 % slower (profiles/r3_attn_ab2_bwd_orders.jsonl)
int bwd_variant(int D = 128) {
  if (g_bwd_variant < 0) { const char* e = getenv("PDT_FA_BWD"); g_bwd_variant = e ? atoi(e) : 0; }
  if (g_bwd_variant > 0) return g_bwd_variant;
  return D == 128 ? 9 : 3;
}

template <int D>
int launch_fwd(const AttnParams& p0, int causal, int variant, hipStream_t st) {
  AttnParams p = p0;                       // p.order bit 0: forward block order
  p.order = p0.order & 1;
  if (variant == 7 || variant == 8) {      // alternative: v5's tile on 8 waves x 32 rows; 7: 3-deep ring, 8: 2-deep
    dim3 g8((p.Sq + 255) / 256, p.H, p.B);
    if (variant == 7) {
      if (causal) fa_fwd_v7_kernel<D, true, 3><<<g8, NT8, 0, st>>>(p);
      else fa_fwd_v7_kernel<D, false, 3><<<g8, NT8, 0, st>>>(p);
    } else {
      if (causal) fa_fwd_v7_kernel<D, true, 2><<<g8, NT8, 0, st>>>(p);
      else fa_fwd_v7_kernel<D, false, 2><<<g8, NT8, 0, st>>>(p);
    }
  } else {                                 // default (5): 4 waves x 32 rows, LDS-DMA ring
    dim3 grid((p.Sq + 127) / 128, p.H, p.B);
    if (causal) fa_fwd_v5_kernel<D, true><<<grid, NT, 0, st>>>(p);
    else fa_fwd_v5_kernel<D, false><<<grid, NT, 0, st>>>(p);
  }
  return (int)hipGetLastError();
}

// Backward: dQ first (it computes delta = rowsum(dO * O) itself unless PDT_FA_FUSE_DELTA=0), then dK/dV v3
// (one wave per SIMD).  dQ kernel: 9 (default at head dim 128) dQ v4, 8 waves x 32 rows, 2-deep ring;
// 8 the same with a 3-deep ring; 3 (default at head dim 64) dQ v3, 4 waves x 32 rows.
template <int D>
int launch_bwd(const AttnParams& p, int causal, hipStream_t st) {
  const int64_t rows = (int64_t)p.B * p.H * p.Sq;
  dim3 gkv((p.Sk + 127) / 128, p.Hkv, p.B);
  dim3 gq((p.Sq + 127) / 128, p.H, p.B);
  dim3 gq8((p.Sq + 255) / 256, p.H, p.B);
  const int variant = bwd_variant(D);
  AttnParams kv = p, qp = p;               // per-kernel block order (p.order bit 1: dK/dV, bit 2: dQ)
  kv.order = (p.order >> 1) & 1;
  qp.order = (p.order >> 2) & 1;
  static const int cyc = [] { const char* e = getenv("PDT_FA_CYCLE"); return e ? atoi(e) : 0; }();
  if (cyc & 2) kv.order = 2;
  if (cyc & 4) qp.order = 2;
  kv.fuse_delta = 0;
  static const int mask_all = [] { const char* e = getenv("PDT_FA_MASK_ALL"); return e && atoi(e) != 0 ? 1 : 0; }();
  kv.mask_all = qp.mask_all = mask_all;
  static const int diag = [] { const char* e = getenv("PDT_FA_DIAG"); return e ? atoi(e) : 0; }();
  kv.diag = qp.diag = diag;
  static const bool fuse = [] { const char* e = getenv("PDT_FA_FUSE_DELTA"); return !e || atoi(e) != 0; }();
  const bool dqp = dq_persistent(p, causal) && bwd_variant(D) == 9;
  qp.fuse_delta = fuse ? 1 : 0;
  if (!qp.fuse_delta) fa_bwd_delta_kernel<D><<<(rows * (D / 8) + NT - 1) / NT, NT, 0, st>>>(p);
  if (dqp) {
    const int n = dq_items(p);
    const int g = n < dkdv_grid(p) ? n : dkdv_grid(p);
    if (causal) fa_bwd_dq_p_kernel<D, true><<<g, NT8, 0, st>>>(qp, n, p.Sq / 256);
    else fa_bwd_dq_p_kernel<D, false><<<g, NT8, 0, st>>>(qp, n, p.Sq / 256);
    if (causal) {
      if (dkdv_persistent(p)) fa_bwd_dkdv_p_kernel<D, true><<<dkdv_grid(p), NT, 0, st>>>(kv, dkdv_items(p), dkdv_upr(kv, dkdv_grid(p)));
      else fa_bwd_dkdv_v3_kernel<D, true, 1><<<gkv, NT, 0, st>>>(kv);
    } else {
      if (dkdv_persistent(p)) fa_bwd_dkdv_p_kernel<D, false><<<dkdv_grid(p), NT, 0, st>>>(kv, dkdv_items(p), dkdv_upr(kv, dkdv_grid(p)));
      else fa_bwd_dkdv_v3_kernel<D, false, 1><<<gkv, NT, 0, st>>>(kv);
    }
    return (int)hipGetLastError();
  }
  if (causal) {
    if (variant == 3) fa_bwd_dq_v3_kernel<D, true><<<gq, NT, 0, st>>>(qp);
    else if (variant == 8) fa_bwd_dq_v4_kernel<D, true, 3><<<gq8, NT8, 0, st>>>(qp);
    else fa_bwd_dq_v4_kernel<D, true, 2><<<gq8, NT8, 0, st>>>(qp);
    if (dkdv_persistent(p)) fa_bwd_dkdv_p_kernel<D, true><<<dkdv_grid(p), NT, 0, st>>>(kv, dkdv_items(p), dkdv_upr(kv, dkdv_grid(p)));
    else fa_bwd_dkdv_v3_kernel<D, true, 1><<<gkv, NT, 0, st>>>(kv);
  } else {
    if (variant == 3) fa_bwd_dq_v3_kernel<D, false><<<gq, NT, 0, st>>>(qp);
    else if (variant == 8) fa_bwd_dq_v4_kernel<D, false, 3><<<gq8, NT8, 0, st>>>(qp);
    else fa_bwd_dq_v4_kernel<D, false, 2><<<gq8, NT8, 0, st>>>(qp);
    if (dkdv_persistent(p)) fa_bwd_dkdv_p_kernel<D, false><<<dkdv_grid(p), NT, 0, st>>>(kv, dkdv_items(p), dkdv_upr(kv, dkdv_grid(p)));
    else fa_bwd_dkdv_v3_kernel<D, false, 1><<<gkv, NT, 0, st>>>(kv);
  }
  return (int)hipGetLastError();
}

}  // namespace

// strides[0..11]: q(b,s,h) k(b,s,h) v(b,s,h) o(b,s,h), in elements; D contiguous everywhere.
PDT_API int pdt_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                               const int64_t* strides, int B, int H, int Hkv, int Sq, int Sk, int D, float scale,
                               int causal, hipStream_t st) {
  if (H % Hkv != 0 || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  AttnParams p{};
  p.q = (const bf16_t*)q; p.k = (const bf16_t*)k; p.v = (const bf16_t*)v; p.o = (bf16_t*)o; p.lse = lse;
  p.q_sb = strides[0]; p.q_ss = strides[1]; p.q_sh = strides[2];
  p.k_sb = strides[3]; p.k_ss = strides[4]; p.k_sh = strides[5];
  p.v_sb = strides[6]; p.v_ss = strides[7]; p.v_sh = strides[8];
  p.o_sb = strides[9]; p.o_ss = strides[10]; p.o_sh = strides[11];
  p.B = B; p.H = H; p.Hkv = Hkv; p.Sq = Sq; p.Sk = Sk; p.scale = scale;
  p.order = block_order_mode(B, Hkv, Sk, D);
  const int variant = fwd_variant();
  return D == 64 ? launch_fwd<64>(p, causal, variant, st) : launch_fwd<128>(p, causal, variant, st);
}

// rows of the backward's dQ column-sum partials (cs_q) for the current kernel variant
static int colsum_rows(int B, int Sq, int D) {
  return bwd_variant(D) == 3 ? B * ((Sq + 127) / 128) : B * ((Sq + 255) / 256);
}

// fp32 workspace floats pdt_flash_attn_bwd needs for the bias-gradient column sums (0: unsupported -- the caller
// sums dqkv itself)
PDT_API int64_t pdt_flash_attn_colsum_ws_floats(int B, int H, int Hkv, int Sq, int Sk, int D) {
  (void)Hkv; (void)Sk;
  if (D != 64 && D != 128) return 0;
  const int64_t hd = (int64_t)H * D;
  return (int64_t)colsum_rows(B, Sq, D) * hd + 64 * hd;
}

namespace {
// dbias_k = 0, dbias_v[hk][d] = sum over the group's query heads of cso[h][d] (see pdt_flash_attn_bwd)
template <typename W>
__global__ void kv_bias_grad_kernel(const float* __restrict__ cso, int Hkv, int group, int D, W* __restrict__ dk,
                                    W* __restrict__ dv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Hkv * D) return;
  const int hk = i / D, d = i - hk * D;
  float s = 0.f;
  for (int g = 0; g < group; ++g) s += cso[(hk * group + g) * D + d];
  dk[i] = from_f<W>(0.f);
  dv[i] = from_f<W>(s);
}
}  // namespace

// strides[0..23]: q k v o dout dq dk dv, each (b, s, h).  delta: fp32 workspace of B*H*Sq.
// dbias (nullable; dtype code dbias_dt: bf16 or fp32): the bias gradient of a packed qkv projection, i.e. the
// column sums of the stored dq | dk | dv rows -> [H*D | Hkv*D | Hkv*D]:
//   q part: per-workgroup partials of the dQ kernel (cs_ws, pdt_flash_attn_colsum_ws_floats) + a deterministic
//           column reduce;
//   k part: exactly 0 -- a key bias adds q . b_k to every score of query row q, which the row softmax cancels
//           (sum_k dS[q, k] = sum_k P (dP - delta) = delta - delta = 0);
//   v part: sum over rows of dO (each P row sums to 1: sum_q sum_k P[q, k] dO[q] = sum_q dO[q]), folded over the
//           query heads of each kv head; dout_colsum = the fp32 [H*D] column sums of dO (required with dbias).
// So the dK/dV kernel carries no column-sum epilogue at all.
PDT_API int pdt_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o, const float* lse,
                               const void* dout, void* dq, void* dk, void* dv, float* delta, const int64_t* strides,
                               int B, int H, int Hkv, int Sq, int Sk, int D, float scale, int causal, float* cs_ws,
                               void* dbias, int dbias_dt, const float* dout_colsum, hipStream_t st) {
  if (H % Hkv != 0 || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  int rq = 0;
  if (dbias) {
    rq = colsum_rows(B, Sq, D);
    if (!cs_ws || !dout_colsum || (dbias_dt != kBF16 && dbias_dt != kF32)) return (int)hipErrorInvalidValue;
  }
  AttnParams p{};
  if (dbias) p.cs_q = cs_ws;
  p.q = (const bf16_t*)q; p.k = (const bf16_t*)k; p.v = (const bf16_t*)v; p.o = (bf16_t*)o;
  p.lse = const_cast<float*>(lse); p.dout = (const bf16_t*)dout;
  p.dq = (bf16_t*)dq; p.dk = (bf16_t*)dk; p.dv = (bf16_t*)dv; p.delta = delta;
  p.q_sb = strides[0]; p.q_ss = strides[1]; p.q_sh = strides[2];
  p.k_sb = strides[3]; p.k_ss = strides[4]; p.k_sh = strides[5];
  p.v_sb = strides[6]; p.v_ss = strides[7]; p.v_sh = strides[8];
  p.o_sb = strides[9]; p.o_ss = strides[10]; p.o_sh = strides[11];
  p.do_sb = strides[12]; p.do_ss = strides[13]; p.do_sh = strides[14];
  p.dq_sb = strides[15]; p.dq_ss = strides[16]; p.dq_sh = strides[17];
  p.dk_sb = strides[18]; p.dk_ss = strides[19]; p.dk_sh = strides[20];
  p.dv_sb = strides[21]; p.dv_ss = strides[22]; p.dv_sh = strides[23];
  p.B = B; p.H = H; p.Hkv = Hkv; p.Sq = Sq; p.Sk = Sk; p.scale = scale;
  p.order = block_order_mode(B, Hkv, Sk, D);
  const int err = D == 64 ? launch_bwd<64>(p, causal, st) : launch_bwd<128>(p, causal, st);
  if (err || !dbias) return err;
  const int hd = H * D, kvd = Hkv * D, group = H / Hkv;
  float* ws2 = p.cs_q + (int64_t)rq * hd;
  const int g = (kvd + 255) / 256;
  if (dbias_dt == kBF16) {
    bf16_t* out = (bf16_t*)dbias;
    red::col_reduce<bf16_t>(p.cs_q, rq, hd, out, ws2, 0, st);
    kv_bias_grad_kernel<bf16_t><<<g, 256, 0, st>>>(dout_colsum, Hkv, group, D, out + hd, out + hd + kvd);
  } else {
    float* out = (float*)dbias;
    red::col_reduce<float>(p.cs_q, rq, hd, out, ws2, 0, st);
    kv_bias_grad_kernel<float><<<g, 256, 0, st>>>(dout_colsum, Hkv, group, D, out + hd, out + hd + kvd);
  }
  return (int)hipGetLastError();
}

// workgroup -> block order bitmask (bit 0 forward, bit 1 dK/dV, bit 2 dQ: 0 heavy-first, 1 XCD-grouped);
// -2 restores the per-shape default, -1 keeps the current setting; returns the setting (-1: per shape)
PDT_API int pdt_flash_attn_set_order(int order) {
  if (order >= 0 || order == -2) g_order = order == -2 ? -1 : order;
  return g_order;
}

// dQ kernel: 1 persistent where eligible, 2 the dQ variant of pdt_flash_attn_set_variant, -1 restores the
// default; returns the setting
PDT_API int pdt_flash_attn_set_dqp(int v) {
  if (g_dqp < 0) { const char* e = getenv("PDT_FA_DQP"); g_dqp = e ? atoi(e) : 0; }
  if (v == 1) g_dqp = 1;
  if (v == 2) g_dqp = 0;
  if (v == -1) { const char* e = getenv("PDT_FA_DQP"); g_dqp = e ? atoi(e) : 0; }
  return g_dqp;
}

// dK/dV kernel: 4 persistent, 3 v3, 0 keeps, -1 restores the default; returns the setting
PDT_API int pdt_flash_attn_set_dkdv(int v) {
  (void)dkdv_items(AttnParams{});
  if (g_dkdv_variant < 0) { const char* e = getenv("PDT_FA_DKDV"); g_dkdv_variant = e ? atoi(e) : 0; }
  if (v > 0) g_dkdv_variant = v;
  if (v == -1) g_dkdv_variant = 0;
  return g_dkdv_variant;
}

// select kernel variants (0 keeps the current choice, -1 restores the default); returns fwd * 32 + bwd of the
// pinned choices (0 = the default: forward v5, backward 9 at head dim 128 / 3 at 64)
PDT_API int pdt_flash_attn_set_variant(int fwd, int bwd) {
  (void)fwd_variant();
  (void)bwd_variant();                       // read the env once before overriding
  if (fwd > 0 || fwd == -1) g_fwd_variant = fwd > 0 ? fwd : 0;
  if (bwd > 0 || bwd == -1) g_bwd_variant = bwd > 0 ? bwd : 0;
  return g_fwd_variant * 32 + g_bwd_variant;
}
