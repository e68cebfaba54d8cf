#!/usr/bin/env python
"""Generates ``gemm_kloop.inc``: the whole MFMA main loop of the 256 x 256 x 64 bf16 GEMM (csrc/kernels/gemm.hip)
as ONE inline-asm statement per operand layout, with every instruction placed by hand.

Why asm: the compiler-scheduled loop of round 3 (same tile, same LDS images, same MFMA count) held the matrix
pipe busy 0.61 of the time against hipBLASLt's 0.78-0.85 at the same 4-wave / one-wave-per-SIMD structure
(profiles/r3_pmc_attention_tt_gemm_hipblaslt.txt).  With one wave per SIMD nobody hides a stall of the wave
that owns the MFMA pipe, so the order of LDS reads, LDS-DMA pieces, waits and barriers between the MFMAs is
the whole game; hipcc neither keeps 256 accumulators in place across a hand-placed schedule nor counts the
inline-asm DMA it cannot see.

Structure (per workgroup: 4 waves as 2 x 2, each wave 128 x 128 = 8 x 8 tiles of v_mfma_f32_16x16x32_bf16,
accumulators a[0:255]; LDS: two 64 KiB stages, A tile then B tile, filled by buffer_load ... lds):

  K-step t reads stage s = t & 1 (tile t); fragments double-buffered: F0 = substep 0 (k 0..31), F1 = substep 1
  Q1  32 MFMA F0.A[0..3] x F0.B        || F1 reads (tile t, stage s)          -> lgkmcnt(0), barrier
  Q2  32 MFMA F0.A[4..7] x F0.B        || DMA of tile t+2, A pieces -> stage s (every wave done reading it)
  Q3  32 MFMA F1.A[0..3] x F1.B        || DMA of tile t+2, B pieces           -> vmcnt(16) (= tile t+1 landed),
                                                                                barrier
  Q4  32 MFMA F1.A[4..7] x F1.B        || F0 reads of tile t+1 (stage s ^ 1)

  Every tile's DMA has a full K-step of MFMAs to land; no MFMA waits for an LDS read issued in its own quarter;
  the only two barriers per K-step sit where an LDS stage changes hands.

Register map inside the statement (clobbered): v[128:255] fragments (F0.A, F0.B, F1.A, F1.B, 8 x 4 VGPRs
each), v[64:95] LDS read addresses, s[80:91] buffer resources / counters, m0.  MFMA operand order is
(B fragment, A fragment), so accumulator tile (i, j) holds C^T: lane l has 4 consecutive columns
n = 16 j + 4 (l >> 4) + r of row m = 16 i + (l & 15) in a[4 (8 i + j) + r].

Hazards handled here (hipcc pads nothing inside asm, cdna_hip_programming.md §5.7): an MFMA separates every
m0 / soffset write from the DMA reading it; fragment registers are overwritten >= 8 MFMAs after their last
MFMA read; the statement ends with s_nop padding so the compiler's v_accvgpr_read of the accumulators sits
behind the last MFMA's result latency.

Run ``python csrc/kernels/gen_gemm_kloop.py`` (the build does it when this file is newer than the .inc).
"""
import os

NT, TT = 0, 1
STB = 65536            # one LDS stage: A tile (32 KiB) then B tile
OPB = 32768
F0A, F0B, F1A, F1B = 128, 160, 192, 224
RD = 64                # read-address registers
S_RA, S_RB, S_CNT, S_OA, S_OB = 80, 84, 88, 89, 90


def frag(base, i):
    return f"v[{base + 4 * i}:{base + 4 * i + 3}]"


def acc(i, j):
    k = 4 * (8 * i + j)
    return f"a[{k}:{k + 3}]"


# Schedule knobs (a variant = one set; VARIANTS[0] is the production schedule and the only one emitted -- the
# others are the measured alternatives, profiles/r4/r4_gemm_variants_v1.jsonl, kept to re-run the A/B):
#   rd1  MFMAs of Q1 over which the F1 reads are spread      dma  MFMAs per quarter over which 8 DMA pieces spread
#   rd0  MFMAs of Q4 over which the F0 reads are spread      bar  Q2 MFMAs issued before Q1's lgkmcnt(0) + barrier
VARIANTS = [
    dict(rd1=16, rd0=16, dma=32, bar=0),     # production: one DMA piece per 4 MFMAs (+2.5-5.6 % over dma=16,
                                             # profiles/r4/r4_gemm_variants_v1.jsonl)
    dict(rd1=16, rd0=16, dma=16, bar=0),     # round-4 first schedule
    dict(rd1=16, rd0=24, dma=32, bar=0),
    dict(rd1=12, rd0=12, dma=32, bar=0),
]


class Gen:
    def __init__(self, layout, sched=None, stamps=False):
        self.layout = layout
        self.stamps = stamps      # diagnostic build: s_memtime at the phase boundaries into s[92:99]
        self.lines = []
        self.sc = dict(VARIANTS[0] if sched is None else sched)

    def emit(self, s):
        self.lines.append(s)

    # ---------------------------------------------------------------- pieces of work
    def rd_reg(self, stage, op, sub_or_blk):
        """NT: one address register per (stage, operand, substep); TT: one per (stage, operand, block).  Stage 2
        (the 3-stage program's third A buffer, in the epilogue staging area) uses v96.. (A only)."""
        if stage == 2:
            assert op == 0
            return f"v{96 + sub_or_blk}"
        if self.layout == NT:
            return f"v{RD + stage * 4 + op * 2 + sub_or_blk}"
        return f"v{RD + stage * 16 + op * 8 + sub_or_blk}"

    def read_ops2(self, sa, sb, sub, which):
        """read_ops with separate A / B stages (3-stage program)."""
        out = []
        for op, blk, dst in which:
            out += self.read_ops(sa if op == 0 else sb, sub, [(op, blk, dst)])
        return out

    def read_ops(self, stage, sub, which):
        """LDS reads of one fragment set: list of instruction strings.  which = [(op, blk, dst_base)]."""
        out = []
        for op, blk, dst in which:
            if self.layout == NT:
                out.append(f"ds_read_b128 {frag(dst, blk)}, {self.rd_reg(stage, op, sub)} offset:{blk * 2048}")
            else:
                r = self.rd_reg(stage, op, blk)
                o = sub * 16384
                out.append(f"ds_read_b64_tr_b16 v[{dst + 4 * blk}:{dst + 4 * blk + 1}], {r} offset:{o}")
                out.append(f"ds_read_b64_tr_b16 v[{dst + 4 * blk + 2}:{dst + 4 * blk + 3}], {r} offset:{o + 2048}")
        return out

    def dma_ops_at(self, off, op):
        """dma_ops into the LDS byte offset `off` (3-stage program: A buffers 0 / STB / 2 STB, B buffers OPB / STB + OPB)."""
        ops, tail = self.dma_ops(0, op)
        ops = [([x.replace(f"%[m0b], {op * OPB + i * 4096}", f"%[m0b], {off + i * 4096}") if x.startswith("s_add_u32 m0")
                 else x for x in setup], load) for i, (setup, load) in enumerate(ops)]
        return ops, tail

    def dma_ops(self, stage, op):
        """8 LDS-DMA pieces of one operand of one tile into `stage` (each piece: SALU set-up, then the load
        one MFMA later), followed by the buffer-resource advance to the next tile."""
        s_rs = S_RA if op == 0 else S_RB
        s_off = S_OA if op == 0 else S_OB
        ops = []
        for i in range(8):
            setup = [f"s_add_u32 m0, %[m0b], {stage * STB + op * OPB + i * 4096}"]
            if i > 0:
                setup.append(f"s_add_u32 s{s_off}, s{s_off}, %[{'rsa' if op == 0 else 'rsb'}]")
            if self.layout == NT:
                voff = "%[voa]" if op == 0 else "%[vob]"
            else:
                voff = (("%[voa1]" if op == 0 else "%[vob1]") if i & 1 else ("%[voa0]" if op == 0 else "%[vob0]"))
            load = f"buffer_load_dwordx4 {voff}, s[{s_rs}:{s_rs + 3}], s{s_off} offen lds"
            ops.append((setup, load))
        tail = [f"s_add_u32 s{s_rs}, s{s_rs}, %[{'asl' if op == 0 else 'bsl'}]",
                f"s_addc_u32 s{s_rs + 1}, s{s_rs + 1}, %[{'ash' if op == 0 else 'bsh'}]",
                f"s_mov_b32 s{s_off}, 0"]
        return ops, tail

    def mfmas(self, fa, fb, rows, zero=False):
        """zero: the accumulator's first MFMA (C = 0: no separate zeroing pass over a[0:255])."""
        return [f"v_mfma_f32_16x16x32_bf16 {acc(i, j)}, {frag(fb, j)}, {frag(fa, i)}, {0 if zero else acc(i, j)}"
                for i in rows for j in range(8)]

    # ---------------------------------------------------------------- schedule helpers
    def interleave_reads(self, mf, reads, span):
        """The reads spread evenly over the first `span` MFMAs of the quarter (at least one MFMA between two
        read slots; several reads per slot when there are more reads than MFMAs in the span)."""
        slots = [[] for _ in mf]
        span = max(1, min(span, len(mf)))
        for k, r in enumerate(reads):
            slots[min(span - 1, (k * span) // len(reads))].append(r)
        for m, sl in zip(mf, slots):
            self.emit(m)
            for r in sl:
                self.emit(r)

    def interleave_dma(self, mf, pieces, tail, span):
        """Piece k: SALU set-up after MFMA p_k, its load after MFMA p_k + 1, with p_k spread evenly over the first
        `span` MFMAs of the quarter (>= 2 apart)."""
        n = len(pieces)
        span = max(2 * n, min(span, len(mf)))
        pos = {(k * span) // n: k for k in range(n)}
        pending = None
        for idx, m in enumerate(mf):
            self.emit(m)
            if pending is not None:
                self.emit(pending)
                pending = None
            if idx in pos:
                setup, load = pieces[pos[idx]]
                for x in setup:
                    self.emit(x)
                pending = load
        if pending is not None:
            self.emit(pending)
        for x in tail:
            self.emit(x)

    # ---------------------------------------------------------------- one K-step
    def step(self, stage, dma, has_next, vm, first=False):
        nxt = stage ^ 1
        self.emit(f"; ---- K-step: stage {stage} dma {dma} next {has_next} first {first}")
        self.emit("s_waitcnt lgkmcnt(0)")
        # Q1: F0.A[0..3] x F0.B, F1 reads of this tile.  Order: A blocks 0-3 (last MFMA read a quarter ago), B
        # blocks, A blocks 4-7 -- each register is rewritten >= 8 MFMAs after the previous K-step's last MFMA
        # that read it (Q4 reads F1.A[4..7] and every F1.B block)
        f1 = self.read_ops(stage, 1, [(0, i, F1A) for i in range(4)] + [(1, j, F1B) for j in range(8)] +
                           [(0, i, F1A) for i in range(4, 8)])
        sc = self.sc
        self.interleave_reads(self.mfmas(F0A, F0B, range(0, 4), first), f1, sc["rd1"])
        # Q2 / Q3: the DMA of tile t+2 into this stage (free once every wave passed the barrier after its F1 reads;
        # the barrier sits `bar` MFMAs into Q2 so the last F1 reads have landed when it is reached)
        q2 = self.mfmas(F0A, F0B, range(4, 8), first)
        for m in q2[:sc["bar"]]:
            self.emit(m)
        self.emit("s_waitcnt lgkmcnt(0)")
        self.emit("s_barrier")
        q2 = q2[sc["bar"]:]
        q3 = self.mfmas(F1A, F1B, range(0, 4))
        if dma:
            pa, ta = self.dma_ops(stage, 0)
            pb, tb = self.dma_ops(stage, 1)
            self.interleave_dma(q2, pa, ta, sc["dma"])
            self.interleave_dma(q3, pb, tb, sc["dma"])
        else:
            for m in q2 + q3:
                self.emit(m)
        if has_next:
            self.emit(f"s_waitcnt vmcnt({vm})")      # tile t+1 (issued a K-step ago) landed in stage s^1
            self.emit("s_barrier")
        # Q4: F1.A[4..7] x F1.B, F0 reads of tile t+1 (A block 0 and every B block first: Q1 order)
        q4 = self.mfmas(F1A, F1B, range(4, 8))
        if has_next:
            f0 = self.read_ops(nxt, 0, [(0, 0, F0A)] + [(1, j, F0B) for j in range(8)] +
                               [(0, i, F0A) for i in range(1, 8)])
            self.interleave_reads(q4, f0, sc["rd0"])
        else:
            for m in q4:
                self.emit(m)

    def next_tail(self, first):
        """The last two K-steps (stages 0, 1) of an item whose K-step count is even.  With %[hnx] set they DMA the
        workgroup's NEXT item's K-tiles 0 and 1 into stages 0 and 1 in their Q2 / Q3 DMA slots (buffer resources
        from %[nalo] .. %[nbhi]), so the next item's first loads are in flight under this item's last MFMAs and
        its epilogue (which stages through the LDS past the ring)."""
        e = self.emit
        e("s_cmp_eq_u32 %[hnx], 0")
        e("s_cbranch_scc1 pdtk%=_tl" + ("f" if first else "0"))
        for base, x in ((S_RA, "na"), (S_RB, "nb")):
            e(f"s_mov_b32 s{base}, %[{x}lo]")
            e(f"s_mov_b32 s{base + 1}, %[{x}hi]")
        e(f"s_mov_b32 s{S_OA}, 0")
        e(f"s_mov_b32 s{S_OB}, 0")
        self.step(0, True, True, 16, first=first)
        self.step(1, True, False, 0)
        e("s_branch pdtk%=_done")
        e("pdtk%=_tl" + ("f" if first else "0") + ":")
        self.step(0, False, True, 0, first=first)
        self.step(1, False, False, 0)
        e("s_branch pdtk%=_done")

    def tile_dma(self, stage):
        for op in (0, 1):
            pieces, tail = self.dma_ops(stage, op)
            for setup, load in pieces:
                for s in setup:
                    self.emit(s)
                self.emit("s_nop 0")
                self.emit(load)
            for s in tail:
                self.emit(s)

    def stamp(self, i):
        """Diagnostic builds: s_memtime into s[92 + 2i : 93 + 2i] (i = 0 start, 1 prologue wait done, 2 first
        K-step done, 3 tail entry); read back after the loop's final lgkmcnt(0)."""
        if self.stamps:
            self.emit(f"s_memtime s[{92 + 2 * i}:{93 + 2 * i}]")

    def first_step(self, vm):
        """Barrier on tile 0, its substep-0 fragments, then K-step 0 (or the whole of a <= 2-step item)."""
        e = self.emit
        e("s_barrier")
        for r in self.read_ops(0, 0, [(0, 0, F0A)] + [(1, j, F0B) for j in range(8)] +
                               [(0, i, F0A) for i in range(1, 8)]):
            e(r)
        e(f"s_cmp_le_u32 s{S_CNT}, 2")
        e("s_cbranch_scc1 pdtk%=_first_tail")
        self.step(0, True, True, vm, first=True)

    def program(self):
        L = self.layout
        e = self.emit
        e("; pdt gemm main loop (generated by gen_gemm_kloop.py)")
        for base, x in ((S_RA, "a"), (S_RB, "b")):     # {base lo, base hi | stride 0, num_records, dword3}
            e(f"s_mov_b32 s{base}, %[{x}lo]")
            e(f"s_mov_b32 s{base + 1}, %[{x}hi]")
            e(f"s_mov_b32 s{base + 2}, %[{x}nr]")
            e(f"s_mov_b32 s{base + 3}, 0x20000")
        e(f"s_mov_b32 s{S_CNT}, %[cnt]")
        e(f"s_mov_b32 s{S_OA}, 0")
        e(f"s_mov_b32 s{S_OB}, 0")
        # LDS read addresses
        if L == NT:
            # %[ra0] / %[ra1]: A fragment address for substep 0 / 1 (stage 0, block 0); B = A + %[db]
            for stage in (0, 1):
                for op in (0, 1):
                    for sub in (0, 1):
                        dst = self.rd_reg(stage, op, sub)
                        src = "%[rd0]" if sub == 0 else "%[rd1]"
                        off = stage * STB
                        if op == 0:
                            e(f"v_add_u32 {dst}, {off}, {src}")
                        else:
                            e(f"v_add_u32 {dst}, %[db], {src}")
                            if off:
                                e(f"v_add_u32 {dst}, {off}, {dst}")
        else:
            # block i address: %[rd0] + 16 * ((2 i) ^ %[rdx]);  B = A + %[db]
            for i in range(8):
                a0 = self.rd_reg(0, 0, i)
                e(f"v_xor_b32 {a0}, {2 * i}, %[rdx]")
                e(f"v_lshl_add_u32 {a0}, {a0}, 4, %[rd0]")
                e(f"v_add_u32 {self.rd_reg(0, 1, i)}, %[db], {a0}")
                e(f"v_add_u32 {self.rd_reg(1, 0, i)}, {STB}, {a0}")
                e(f"v_add_u32 {self.rd_reg(1, 1, i)}, {STB}, {self.rd_reg(0, 1, i)}")
        # prologue: tiles 0 and 1 in flight, tile 0 landed, its substep-0 fragments read.  A persistent
        # workgroup's later items (%[first] = 0) find tiles 0 / 1 already issued by the previous item's last two
        # K-steps (next_tail): then only the wait, counted past the previous epilogue's global stores (%[wnx])
        # K-step 0 is peeled (its substep-0 MFMAs start every accumulator from C = 0) and emitted twice: for a
        # later item its end-of-step wait for tile 1 also counts the previous epilogue's stores as older than
        # tile 2's DMA (vmcnt(%[wnx]) = 16 + stores), so they drain under the K-step instead of stalling it
        self.stamp(0)
        e("s_cmp_eq_u32 %[first], 0")
        e("s_cbranch_scc1 pdtk%=_issued")
        self.tile_dma(0)
        self.tile_dma(1)
        e("s_waitcnt vmcnt(16)")
        self.stamp(1)
        self.first_step(16)
        e("s_branch pdtk%=_stepped")
        e("pdtk%=_issued:")
        e("s_waitcnt vmcnt(%[wnx])")
        self.stamp(1)
        self.first_step("%[wnx]")
        e("pdtk%=_stepped:")
        self.stamp(2)
        # then two K-steps per iteration (stage 1, stage 0); s88 = K-steps left including the current one
        e(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
        e(f"s_cmp_le_u32 s{S_CNT}, 2")
        e("s_cbranch_scc1 pdtk%=_tail1")
        e("pdtk%=_loop:")
        self.step(1, True, True, 16)
        e(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
        e(f"s_cmp_le_u32 s{S_CNT}, 2")
        e("s_cbranch_scc1 pdtk%=_tail0")
        self.step(0, True, True, 16)
        e(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
        e(f"s_cmp_le_u32 s{S_CNT}, 2")
        e("s_cbranch_scc0 pdtk%=_loop")
        e("s_branch pdtk%=_tail1")
        e("pdtk%=_tail0:")                      # 2 K-steps left, stage 0 (T even)
        self.stamp(3)
        self.next_tail(False)
        e("pdtk%=_tail1:")                      # 2 K-steps left, stage 1 (T odd: the next item loads itself)
        self.stamp(3)
        self.step(1, False, True, 0)
        self.step(0, False, False, 0)
        e("s_branch pdtk%=_done")
        e("pdtk%=_first_tail:")                 # K = 128: both K-steps, the first from C = 0
        self.next_tail(True)
        e("pdtk%=_done:")
        if self.stamps:
            e("s_waitcnt lgkmcnt(0)")
            for i in range(8):
                e(f"s_mov_b32 %[st{i}], s{92 + i}")
        e("s_nop 15")
        e("s_nop 15")
        return self.lines


class Gen3(Gen):
    """3-stage program for long-K items: the A operand gets a third LDS buffer (the epilogue's 32 KiB staging area,
    idle during the loop), so A's K-tile t+3 is DMA'd in K-step t -- two K-steps of lead instead of one: an A
    operand streamed from HBM (every weight-gradient shape) no longer waits on HBM latency at the step boundary
    (2,350 vs 2,240 cycles per K-step, profiles/r4/r4_gemm_stamps_cached_vs_streamed.jsonl).  B keeps 2 buffers
    (DMA'd one K-step ahead, in Q2, before A's pieces in Q3, so a wait for B never forces a younger A tile).  No
    next-item prefetch; items need T >= 6 K-steps (the host's choice).  Unrolled by 6 = lcm(3, 2)."""

    A_OFF = (0, STB, 2 * STB)
    B_OFF = (OPB, STB + OPB)

    def step3(self, p, dma_a, dma_b, has_next, vm, first=False):
        sa, sb = p % 3, p % 2
        nxa, nxb = (p + 1) % 3, (p + 1) % 2
        e = self.emit
        e(f"; ---- K-step (3-stage): A {sa} B {sb} dma A {dma_a} B {dma_b} next {has_next} first {first}")
        e("s_waitcnt lgkmcnt(0)")
        f1 = self.read_ops2(sa, sb, 1, [(0, i, F1A) for i in range(4)] + [(1, j, F1B) for j in range(8)] +
                            [(0, i, F1A) for i in range(4, 8)])
        sc = self.sc
        self.interleave_reads(self.mfmas(F0A, F0B, range(0, 4), first), f1, sc["rd1"])
        q2 = self.mfmas(F0A, F0B, range(4, 8), first)
        e("s_waitcnt lgkmcnt(0)")
        e("s_barrier")
        q3 = self.mfmas(F1A, F1B, range(0, 4))
        if dma_b:
            pb, tb = self.dma_ops_at(self.B_OFF[sb], 1)
            self.interleave_dma(q2, pb, tb, sc["dma"])
        else:
            for m in q2:
                e(m)
        if dma_a:
            pa, ta = self.dma_ops_at(self.A_OFF[sa], 0)
            self.interleave_dma(q3, pa, ta, sc["dma"])
        else:
            for m in q3:
                e(m)
        if has_next:
            e(f"s_waitcnt vmcnt({vm})")
            e("s_barrier")
        q4 = self.mfmas(F1A, F1B, range(4, 8))
        if has_next:
            f0 = self.read_ops2(nxa, nxb, 0, [(0, 0, F0A)] + [(1, j, F0B) for j in range(8)] +
                                [(0, i, F0A) for i in range(1, 8)])
            self.interleave_reads(q4, f0, sc["rd0"])
        else:
            for m in q4:
                e(m)

    def tile_dma_at(self, off, op):
        pieces, tail = self.dma_ops_at(off, op)
        for setup, load in pieces:
            for x in setup:
                self.emit(x)
            self.emit("s_nop 0")
            self.emit(load)
        for x in tail:
            self.emit(x)

    def program(self):
        L = self.layout
        e = self.emit
        e("; pdt gemm main loop, 3-stage A (generated by gen_gemm_kloop.py)")
        for base, x in ((S_RA, "a"), (S_RB, "b")):
            e(f"s_mov_b32 s{base}, %[{x}lo]")
            e(f"s_mov_b32 s{base + 1}, %[{x}hi]")
            e(f"s_mov_b32 s{base + 2}, %[{x}nr]")
            e(f"s_mov_b32 s{base + 3}, 0x20000")
        e(f"s_mov_b32 s{S_CNT}, %[cnt]")
        e(f"s_mov_b32 s{S_OA}, 0")
        e(f"s_mov_b32 s{S_OB}, 0")
        if L == NT:
            for stage in (0, 1):
                for op in (0, 1):
                    for sub in (0, 1):
                        dst = self.rd_reg(stage, op, sub)
                        src = "%[rd0]" if sub == 0 else "%[rd1]"
                        if op == 0:
                            e(f"v_add_u32 {dst}, {stage * STB}, {src}")
                        else:
                            e(f"v_add_u32 {dst}, %[db], {src}")
                            if stage:
                                e(f"v_add_u32 {dst}, {STB}, {dst}")
            for sub in (0, 1):
                e(f"v_add_u32 {self.rd_reg(2, 0, sub)}, {2 * STB}, {'%[rd0]' if sub == 0 else '%[rd1]'}")
        else:
            for i in range(8):
                a0 = self.rd_reg(0, 0, i)
                e(f"v_xor_b32 {a0}, {2 * i}, %[rdx]")
                e(f"v_lshl_add_u32 {a0}, {a0}, 4, %[rd0]")
                e(f"v_add_u32 {self.rd_reg(0, 1, i)}, %[db], {a0}")
                e(f"v_add_u32 {self.rd_reg(1, 0, i)}, {STB}, {a0}")
                e(f"v_add_u32 {self.rd_reg(1, 1, i)}, {STB}, {self.rd_reg(0, 1, i)}")
                e(f"v_add_u32 {self.rd_reg(2, 0, i)}, {2 * STB}, {a0}")
        # prologue: A0 B0 A1 B1 A2 in flight; tile 0 (A0, B0) landed: A1 B1 A2 (24 pieces) may still fly
        self.tile_dma_at(self.A_OFF[0], 0)
        self.tile_dma_at(self.B_OFF[0], 1)
        self.tile_dma_at(self.A_OFF[1], 0)
        self.tile_dma_at(self.B_OFF[1], 1)
        self.tile_dma_at(self.A_OFF[2], 0)
        e("s_waitcnt vmcnt(24)")
        e("s_barrier")
        for r in self.read_ops2(0, 0, 0, [(0, 0, F0A)] + [(1, j, F0B) for j in range(8)] +
                                [(0, i, F0A) for i in range(1, 8)]):
            e(r)
        # K-step 0 (accumulators from C = 0); then steady steps while t + 3 < T (s88 = T - t > 3): B tile t + 2 and
        # A tile t + 3 in flight, the wait for tile t + 1 leaves A(t+2), B(t+2), A(t+3) (24 pieces) flying
        self.step3(0, True, True, True, 24, first=True)
        e(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
        e("pdtk%=_loop3:")
        for p in (1, 2, 3, 4, 5, 0):
            e(f"s_cmp_le_u32 s{S_CNT}, 3")
            e(f"s_cbranch_scc1 pdtk%=_t3_{p}")
            self.step3(p, True, True, True, 24)
            e(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
        e("s_branch pdtk%=_loop3")
        # the last three K-steps, entered at phase p: t = T-3 issues B(T-1) only (its wait for tile T-2 leaves A(T-1)
        # and B(T-1) flying), t = T-2 drains, t = T-1 has no next tile
        for p in range(6):
            e(f"pdtk%=_t3_{p}:")
            self.step3(p, False, True, True, 16)
            self.step3((p + 1) % 6, False, False, True, 0)
            self.step3((p + 2) % 6, False, False, False, 0)
            e("s_branch pdtk%=_done3")
        e("pdtk%=_done3:")
        e("s_nop 15")
        e("s_nop 15")
        return self.lines


def render(name, lines):
    return f"#define {name} \\\n" + " \\\n".join(f'  "{ln}\\n"' for ln in lines) + "\n"


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    out = ["// GENERATED by gen_gemm_kloop.py -- do not edit.  The hand-scheduled main loops of gemm.hip.",
           "#pragma once", ""]
    for L, name in ((NT, "PDT_GEMM_KLOOP_NT"), (TT, "PDT_GEMM_KLOOP_TT")):
        sched = VARIANTS[int(os.environ.get("PDT_GEMM_SCHEDULE", "0"))]
        lines = Gen(L, sched).program()
        n_mfma = sum(1 for ln in lines if ln.startswith("v_mfma"))
        out.append(f"// {name} {sched}: {len(lines)} lines, {n_mfma} MFMAs")
        out.append(render(name, lines))
        out.append(f"// {name}_STAMPS: the same loop with s_memtime phase stamps (gemm.hip DIAG builds)")
        out.append(render(name + "_STAMPS", Gen(L, sched, stamps=True).program()))
        lines3 = Gen3(L, sched).program()
        out.append(f"// {name}3: 3-stage A ring for long-K items, {len(lines3)} lines")
        out.append(render(name + "3", lines3))
    out.append("#define PDT_AGPR_CLOBBERS " + ", ".join(f'"a{i}"' for i in range(256)))
    out.append("")
    with open(os.path.join(here, "gemm_kloop.inc"), "w") as f:
        f.write("\n".join(out))


if __name__ == "__main__":
    main()
