#!/usr/bin/env python3
"""Generates metal-flash-attention-plus_amd/csrc/fwd_pipe_asm.h: the hand-placed steady-state
blocks of the software-pipelined 16-bit forward (attention_fwd_pipe.hip), fp16, D = 128,
64-key tiles, one wave = 32 query rows.

Why a generator: the loop step is ~130 instructions whose placement is the point (MFMA gaps,
counted LDS waits, hazard distances), and hipcc schedules the equivalent HIP in bursts (all
exponentials after the QK^T chain).  Every block names its registers
explicitly; the kernel pins its state to the same registers with "{v[a:b]}" asm constraints,
so the compiler keeps it there between blocks (no copies).

Per step t of a wave (tile t's PV, tile t+1's QK^T):
  X block: S(t+1) = K(t+1)·Q^T (16 MFMAs, K fragments read 4 ahead) with, in the MFMA gaps,
           P(t) = exp2(S'(t)) (S' = S·c − m straight from the MFMA), its row-sum partials and
           the fp16 packing of P(t) in place (the PV B operand), then the first V(t) reads.
  Y block: O^T += V(t)^T·P(t)^T (16 MFMAs, V fragments read 3 ahead) with, in the gaps, the
           row max of S(t+1) (v_max3 chains), once the QK^T results are ready.
The rescale decision, the masks of edge / causal tiles, the LDS-DMA of later tiles and the
barrier stay in HIP between the blocks.

Register map (per lane, 256 = two waves per SIMD):
  v[192:255] O^T accumulators o[dt], dt = 0..3      v[160:191] Q fragments q[ds], ds = 0..7
  v[144:159] −m tile (QK^T chain start)            v[112:143] S buffer B (s[0], s[1])
  v[80:111]  S buffer A                            v[64:79]   K fragment ring (4)
  v[52:63]   V fragment ring (3)                   v[48:51]   row-sum partials
  v0..v47    the compiler's (addresses, loop state, DMA offsets).
Parity par = t & 1: K(t+1) in K slot par ^ 1, V(t) in V slot par, S(t) in buffer (par ? B : A),
S(t+1) in the other.  The prologue (QK^T of the first tile) is the par = 1 X block without
exponentials followed by the par = 1 Y block without PV.

Hazards handled here (cdna_hip_programming.md §5.7 item 2): a transcendental's result is read
no earlier than one instruction later; a VALU never reads an MFMA result sooner than MIN_DIST
instructions after the MFMA (s_nop otherwise); LDS fragment reads are waited for with counted
lgkmcnt (LDS returns in order; SMEM the compiler leaves in flight only makes a wait longer).
"""
import os

TILEB = 64 * 128 * 2          # one K or V tile (bytes)
KRING = 0                     # K slots at +0, +TILEB
VRING = 2 * TILEB             # V slots at +2*TILEB, +3*TILEB
RB = 16 * 128                 # TileA: bytes per 8-row block at DP = 128
MIN_DIST = 14                 # instructions between an MFMA and a VALU reading its result

O = [192 + 16 * i for i in range(4)]
Q = [160 + 4 * i for i in range(8)]
NEGM = 144
SBUF = {0: [80, 96], 1: [112, 128]}     # buffer A (0), buffer B (1): s[0], s[1]
KR = [64 + 4 * i for i in range(4)]
VR = [52 + 4 * i for i in range(3)]
RS = 48


def r(a, b=None):
    return f"v{a}" if b is None else f"v[{a}:{b}]"


# Ablation switches (timing-only diagnostic builds, tools/diag/pipe_abl.hip): drop every LDS
# fragment read and its waits (NOLDS) or the exp / row-sum / pack work (NOEXP).
ABL = {"nolds": False, "noexp": False}


class Block:
    """Instruction list with LDS-wait and MFMA-hazard bookkeeping."""

    def __init__(self):
        self.ins = []          # (text, kind)
        self.lds = []          # tags of issued LDS reads, in order
        self.mfma_dst = {}     # register -> wait-state count at the MFMA that wrote it
        self.states = 0        # wait states elapsed (an instruction 1, s_nop N N + 1)

    def emit(self, text, kind="salu"):
        self.ins.append((text, kind))
        if kind == "nop":
            self.states += sum(int(t.split()[1]) + 1 for t in text.split("\\n\\t"))
        else:
            self.states += 1

    def lds_read(self, text, tag):
        if ABL["nolds"]:
            return
        self.emit(text, "lds")
        self.lds.append(tag)

    def wait_lds(self, tag):
        if ABL["nolds"]:
            return
        # Wait until the read `tag` has returned: the reads issued after it may stay in flight.
        n = len(self.lds) - 1 - self.lds.index(tag)
        self.emit(f"s_waitcnt lgkmcnt({min(n, 15)})", "wait")

    def mfma(self, dst, a, b, c):
        self.emit(f"v_mfma_f32_32x32x16_f16 {r(dst, dst + 15)}, {r(a, a + 3)}, {r(b, b + 3)}, "
                  f"{r(c, c + 15)}", "mfma")
        for k in range(16):
            self.mfma_dst[dst + k] = self.states

    def valu(self, text, reads=()):
        # Pad so that no source register is read within MIN_DIST wait states of the MFMA that
        # wrote it.
        for reg in reads:
            if reg in self.mfma_dst:
                d = self.states - self.mfma_dst[reg]
                if d < MIN_DIST:
                    self.emit(f"s_nop {min(MIN_DIST - d - 1, 15)}", "nop")
                del self.mfma_dst[reg]
        self.emit(text, "valu")

    def text(self):
        return "\\n\\t".join(t for t, _ in self.ins)


def exp_work(cur):
    """P(t) = exp2(S'(t)) in place, row-sum partials rs[i & 3] in the order of fwd2_exp
    (attention_fwd2.h), and the fp16 pack: registers 8ks..8ks+7 of s[j] become P[2j+ks] in
    registers 8ks..8ks+3.  A list of (text, reads, cost)."""
    w = []
    first = [True] * 4
    for j in range(2):
        base = SBUF[cur][j]
        for ks in range(2):
            g = base + 8 * ks
            for pr in range(4):
                a, b = g + 2 * pr, g + 2 * pr + 1
                w.append((f"v_exp_f32 {r(a)}, {r(a)}", (a,), 2))
                w.append((f"v_exp_f32 {r(b)}, {r(b)}", (b,), 2))
                for x in (a, b):
                    i = x - base
                    ra = RS + (i & 3)
                    if first[i & 3]:
                        w.append((f"v_add_f32 {r(ra)}, 0, {r(x)}", (), 1))
                        first[i & 3] = False
                    else:
                        w.append((f"v_add_f32 {r(ra)}, {r(ra)}, {r(x)}", (), 1))
                w.append((f"v_cvt_pk_f16_f32 {r(g + pr)}, {r(a)}, {r(b)}", (), 1))
    return w


# Balanced schedule (BAL): the exponentials of a tile are split between the two blocks.  The Y
# block of step t computes P = exp2(S'(t+1)) for s[0] of tile t+1 out of place, into the K
# fragment ring (free during Y), beside the row max — speculatively, against the current
# offset, since the rescale decision follows the block (a rescale recomputes them from the
# shifted S').  The X block of step t+1 packs those first (before its K reads reuse the ring),
# then exponentiates s[1] in place.  The row-sum partials run in fwd2_exp's order across the
# two blocks, so the results are bit-identical to the compiler-scheduled kernels.
BAL = True


def exp_y_work(nxt):
    """Y block: P of s[0] of S(t+1) into KR (v64..v79) and its row-sum partials (started)."""
    w = []
    base = SBUF[nxt][0]
    for pr in range(8):
        a, b = 2 * pr, 2 * pr + 1
        w.append((f"v_exp_f32 {r(KR[0] + a)}, {r(base + a)}", (base + a,), 2))
        w.append((f"v_exp_f32 {r(KR[0] + b)}, {r(base + b)}", (base + b,), 2))
        for i in (a, b):
            ra = RS + (i & 3)
            src = "0" if i < 4 else r(ra)
            w.append((f"v_add_f32 {r(ra)}, {src}, {r(KR[0] + i)}", (), 1))
    return w


def pack_s0_work(cur):
    """X block prelude: P[0], P[1] of tile t (s[0], computed by the previous Y block into KR)
    packed to fp16 into s[0]'s registers 0..3 and 8..11."""
    base = SBUF[cur][0]
    w = []
    for ks in range(2):
        for pr in range(4):
            a = KR[0] + 8 * ks + 2 * pr
            w.append((f"v_cvt_pk_f16_f32 {r(base + 8 * ks + pr)}, {r(a)}, {r(a + 1)}", (), 1))
    return w


def exp_x_work(cur):
    """X block: exp2 of s[1] of tile t in place, row-sum partials continued, fp16 pack."""
    w = []
    base = SBUF[cur][1]
    for ks in range(2):
        g = base + 8 * ks
        for pr in range(4):
            a, b = g + 2 * pr, g + 2 * pr + 1
            w.append((f"v_exp_f32 {r(a)}, {r(a)}", (a,), 2))
            w.append((f"v_exp_f32 {r(b)}, {r(b)}", (b,), 2))
            for x in (a, b):
                ra = RS + ((x - base) & 3)
                w.append((f"v_add_f32 {r(ra)}, {r(ra)}, {r(x)}", (), 1))
            w.append((f"v_cvt_pk_f16_f32 {r(g + pr)}, {r(a)}, {r(b)}", (), 1))
    return w


def max_work(nxt):
    """Row max of S(t+1): two v_max3 chains (s[0] into mx, s[1] into mt), interleaved so the
    two dependency chains run side by side; the caller ends with max(mx, mt).  A list of
    (text, reads, cost)."""
    chains = []
    for j in range(2):
        base = SBUF[nxt][j]
        acc = "%[mx]" if j == 0 else "%[mt]"
        c = [(f"v_max3_f32 {acc}, {r(base)}, {r(base + 1)}, {r(base + 2)}",
              (base, base + 1, base + 2), 1)]
        k = 3
        while k < 16:
            if k + 1 < 16:
                c.append((f"v_max3_f32 {acc}, {acc}, {r(base + k)}, {r(base + k + 1)}",
                          (base + k, base + k + 1), 1))
                k += 2
            else:
                c.append((f"v_max_f32 {acc}, {acc}, {r(base + k)}", (base + k,), 1))
                k += 1
        chains.append(c)
    out = []
    for i in range(max(len(chains[0]), len(chains[1]))):
        for c in chains:
            if i < len(c):
                out.append(c[i])
    return out


def k_frag(i, kslot):
    """QK^T MFMA i: (j, ds) = (i % 2, i // 2); its K fragment read."""
    j, ds = i % 2, i // 2
    off = KRING + kslot * TILEB + RB * 4 * j + 512 * (ds >> 1)
    reg = KR[i % 4]
    return f"ds_read_b128 {r(reg, reg + 3)}, %[ka{ds & 1}] offset:{off}", reg


def v_frag(i, vslot):
    """PV MFMA i: (jk, dt) = (i // 4, i % 4); its two transposed V reads (TileA read_tr_a)."""
    jk, dt = i // 4, i % 4
    o = RB * (4 * (jk >> 1) + 2 * (jk & 1)) + 512 * dt + VRING + vslot * TILEB
    reg = VR[i % 3]
    return (f"ds_read_b64_tr_b16 {r(reg, reg + 1)}, %[va0] offset:{o}",
            f"ds_read_b64_tr_b16 {r(reg + 2, reg + 3)}, %[va1] offset:{o + RB}", reg)


# MFMA gaps of the X block that issue the step's four LDS-DMA pieces (dma variant): K(t+2)
# pieces 0/1 and V(t+1) pieces 0/1 of this wave (DmaA<128, 64, 512>: two pieces per operand).
DMA_GAPS = {1: ("kd", "ko0", "kl0"), 4: ("kd", "ko1", "kl1"), 7: ("vd", "vo0", "vl0"),
            10: ("vd", "vo1", "vl1")}


def gen_x(par, qk, ex, dma=False):
    """X block of step parity par: QK^T(t+1) (qk) with exp/pack of S(t) (ex); ends with the
    first three V(t) fragment reads when ex (the PV of this step follows).  dma: the step's
    LDS-DMA pieces ride in the MFMA gaps (DMA_GAPS) instead of being issued before the block."""
    kslot, vslot = par ^ 1, par
    cur, nxt = (1, 0) if par else (0, 1)
    b = Block()
    if BAL:
        work = exp_x_work(cur) if ex and not ABL["noexp"] else []
        if ex:
            # P[0], P[1] out of the K ring before the K reads reuse it.
            for t, rd, _ in pack_s0_work(cur):
                b.valu(t, rd)
    else:
        work = exp_work(cur) if ex and not ABL["noexp"] else []
    wi = 0
    if qk:
        for i in range(4):
            t, _ = k_frag(i, kslot)
            b.lds_read(t, ("k", i))
        # Exponentials first while the first K fragments land.
        pre = min(10, len(work))
        for _ in range(pre):
            t, rd, _ = work[wi]
            b.valu(t, rd)
            wi += 1
        per = (len(work) - wi) / 16.0
        acc = 0.0
        for i in range(16):
            j, ds = i % 2, i // 2
            b.wait_lds(("k", i))
            c = NEGM if ds == 0 else SBUF[nxt][j]
            b.mfma(SBUF[nxt][j], KR[i % 4], Q[ds], c)
            if i + 4 < 16:
                t, _ = k_frag(i + 4, kslot)
                b.lds_read(t, ("k", i + 4))
            if dma and i in DMA_GAPS:
                d, o, l = DMA_GAPS[i]
                b.emit(f"s_mov_b32 m0, %[{l}]", "salu")
                b.emit("s_nop 0", "nop")
                b.emit(f"buffer_load_dwordx4 %[{o}], %[{d}], 0 offen lds", "vmem")
            acc += per
            while wi < len(work) and wi < round(acc) + pre:
                t, rd, _ = work[wi]
                b.valu(t, rd)
                wi += 1
            if ex and i >= 13:
                ta, tb, _ = v_frag(i - 13, vslot)
                b.lds_read(ta, ("v", i - 13, 0))
                b.lds_read(tb, ("v", i - 13, 1))
    while wi < len(work):
        t, rd, _ = work[wi]
        b.valu(t, rd)
        wi += 1
    if ex and not qk:
        for i in range(3):
            ta, tb, _ = v_frag(i, vslot)
            b.lds_read(ta, ("v", i, 0))
            b.lds_read(tb, ("v", i, 1))
    return b


def trailing(b, regs):
    """Wait states of block b after its last MFMA writing any of `regs`."""
    last = max(b.mfma_dst.get(x, -1) for x in regs)
    return b.states - last


def gen_y(par, pv, mx, trail=(0, 0)):
    """Y block: PV(t) (pv) with the row max of S(t+1) (mx) in the gaps.  trail: instructions
    the X blocks that precede it (either variant) place after their last MFMA into s[0] / s[1]
    of S(t+1)."""
    vslot = par
    cur, nxt = (1, 0) if par else (0, 1)
    b = Block()
    work = max_work(nxt) if mx else []
    if mx and BAL and not ABL["noexp"]:
        # Max chains and the speculative exponentials of s[0] side by side (independent: the
        # exponentials go out of place).
        ew = exp_y_work(nxt)
        merged = []
        mi = ei = 0
        while mi < len(work) or ei < len(ew):
            if mi < len(work):
                merged.append(work[mi])
                mi += 1
            for _ in range(2):
                if ei < len(ew):
                    merged.append(ew[ei])
                    ei += 1
        work = merged
    if mx:
        # The QK^T results were written by the X block's last MFMAs: the reads below are
        # padded by their distance from those MFMAs (code between the blocks only adds).
        for jj in range(2):
            for k in range(16):
                b.mfma_dst[SBUF[nxt][jj] + k] = -trail[jj]
    wi = 0
    if pv:
        # Fragments 0..2 were issued by the X block (tags continue from there).
        for i in range(3 if not ABL["nolds"] else 0):
            b.lds.append(("v", i, 0))
            b.lds.append(("v", i, 1))
        for i in range(16):
            jk, dt = i // 4, i % 4
            b.wait_lds(("v", i, 1))
            preg = SBUF[cur][jk >> 1] + 8 * (jk & 1)
            b.mfma(O[dt], VR[i % 3], preg, O[dt])
            if i + 3 < 16:
                ta, tb, _ = v_frag(i + 3, vslot)
                b.lds_read(ta, ("v", i + 3, 0))
                b.lds_read(tb, ("v", i + 3, 1))
            # From gap 1 on, an even share of the max / exp work per gap.
            if i >= 1:
                quota = -(-len(work) * i // 15)
                while wi < len(work) and wi < quota:
                    t, rd, _ = work[wi]
                    b.valu(t, rd)
                    wi += 1
    while wi < len(work):
        t, rd, _ = work[wi]
        b.valu(t, rd)
        wi += 1
    if mx:
        b.valu("v_max_f32 %[mx], %[mx], %[mt]")
    return b


# Every block names the whole pinned range as clobbered: the kernel limits the compiler to
# v0..v47 (amdgpu_num_vgpr), so v48..v255 are reserved registers that only these blocks touch;
# listing them makes the kernel descriptor allocate all 256.
CLOBBER_MACRO = "MFA_PIPE_CLOBBERS"


def func(name, block, args, outs=(), inouts=(), extra_clobbers=()):
    ops_out = ", ".join([f'[{o}] "=&v"({o})' for o in outs] + [f'[{o}] "+v"({o})' for o in inouts])
    ops_in = ", ".join(f'[{a}] "v"({a})' for a in args)
    params = "".join(f", int {a}" if a in ("ka0", "ka1", "va0", "va1", "hi") else f", float {a}"
                     for a in args)
    params += "".join(f", float& {o}" for o in list(outs) + list(inouts))
    params = params[2:]
    decl = "".join(f"  float {o};\n" for o in ("mt",) if o in outs and o != "mx")
    clob = CLOBBER_MACRO + "".join(f', "{c}"' for c in extra_clobbers)
    return (f"__device__ __forceinline__ void {name}({params}) {{\n"
            + f"  asm volatile(\"{block.text()}\"\n"
            + f"               : {ops_out}\n"
            + f"               : {ops_in}\n"
            + f"               : {clob});\n}}\n")


def func_dma(name, block):
    """The X block with the step's LDS-DMA pieces: two buffer descriptors (K(t+2), V(t+1)),
    the wave's per-lane offsets and LDS destinations of its two pieces of each."""
    return (f"__device__ __forceinline__ void {name}(int ka0, int ka1, int va0, int va1, float& lh,\n"
            "    const DmaPieces& dp) {\n"
            + f"  asm volatile(\"{block.text()}\"\n"
            + "               : [lh] \"+v\"(lh)\n"
            + "               : [ka0] \"v\"(ka0), [ka1] \"v\"(ka1), [va0] \"v\"(va0), [va1] \"v\"(va1),\n"
            + "                 [kd] \"s\"(dp.kd), [vd] \"s\"(dp.vd), [ko0] \"v\"(dp.ko0), [ko1] \"v\"(dp.ko1),\n"
            + "                 [vo0] \"v\"(dp.vo0), [vo1] \"v\"(dp.vo1), [kl0] \"s\"(dp.kl0), [kl1] \"s\"(dp.kl1),\n"
            + "                 [vl0] \"s\"(dp.vl0), [vl1] \"s\"(dp.vl1)\n"
            + f"               : {CLOBBER_MACRO}, \"m0\", \"memory\");\n}}\n")


def lh_fold(b):
    """lh += (rs0 + rs1) + (rs2 + rs3), fwd2_exp's order."""
    b.emit(f"v_add_f32 {r(RS)}, {r(RS)}, {r(RS + 1)}", "valu")
    b.emit(f"v_add_f32 {r(RS + 2)}, {r(RS + 2)}, {r(RS + 3)}", "valu")
    b.emit(f"v_add_f32 {r(RS)}, {r(RS)}, {r(RS + 2)}", "valu")
    b.emit(f"v_add_f32 %[lh], %[lh], {r(RS)}", "valu")


def gen_rescale(par):
    """The lazy rescale's rare branch (fwd2_max): O *= corr, S(t+1) -= shift, −m tile =
    negm.  Opens with the MFMA-result wait (the PV MFMAs of the Y block write O)."""
    cur, nxt = (1, 0) if par else (0, 1)
    b = Block()
    b.emit("s_nop 7\\n\\ts_nop 7", "nop")
    for o in O:
        for k in range(16):
            b.emit(f"v_mul_f32 {r(o + k)}, {r(o + k)}, %[corr]", "valu")
    for base in SBUF[nxt]:
        for k in range(16):
            b.emit(f"v_sub_f32 {r(base + k)}, {r(base + k)}, %[shift]", "valu")
    for k in range(16):
        b.emit(f"v_mov_b32 {r(NEGM + k)}, %[negm]", "valu")
    if BAL:
        # The Y block's speculative P of s[0] (and its row-sum partials) from the shifted S'.
        for t, rd, _ in exp_y_work(nxt):
            b.emit(t, "valu")
    return b


def gen_mask(par):
    """Edge / causal mask of S(t+1) (mask_outside<2> with lo unbounded): element (j, i) sits at
    key offset kk = 32j + (i & 3) + 8(i >> 2) from the lane's base and becomes −inf when
    kk > hi.  Opens with the MFMA-result wait (the X block's QK^T MFMAs write S(t+1))."""
    nxt = 0 if par else 1
    b = Block()
    b.emit("s_nop 7\\n\\ts_nop 7", "nop")
    for j, base in enumerate(SBUF[nxt]):
        for i in range(16):
            kk = 32 * j + (i & 3) + 8 * (i >> 2)
            b.emit(f"v_cmp_lt_i32 vcc, %[hi], {kk}", "valu")
            b.emit("s_nop 1", "nop")
            b.emit(f"v_cndmask_b32 {r(base + i)}, {r(base + i)}, %[ninf], vcc", "valu")
    return b


def main():
    out = ["// Generated by tools/gen_fwd_pipe.py — do not edit by hand.  The hand-placed blocks of",
           "// the software-pipelined fp16 D = 128 forward (attention_fwd_pipe.hip); the generator's",
           "// docstring describes the schedule, the register map and the hazards it pads.",
           "#pragma once",
           '#include "mfa_device.h"',
           "",
           "// v48..v255: reserved for the pipelined kernel's state (it limits the compiler to v0..v47).",
           "#define MFA_PIPE_CLOBBERS " + ", ".join(f'"v{k}"' for k in range(48, 256)),
           "",
           "namespace mfa {",
           "",
           "typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));",
           "// The LDS-DMA operands of one step (pipe_x_qk_exp_dma_*): buffer descriptors of K(t+2) and",
           "// V(t+1), this wave's per-lane offsets and LDS destinations of its two pieces of each.",
           "struct DmaPieces {",
           "  u32x4_t kd, vd;",
           "  int ko0, ko1, vo0, vo1;",
           "  unsigned kl0, kl1, vl0, vl1;",
           "};",
           ""]
    for par in (0, 1):
        for qk, ex, tag in ((1, 1, "qk_exp"), (1, 0, "qk"), (0, 1, "exp")):
            b = gen_x(par, qk, ex)
            if ex:
                lh_fold(b)
            args = (["ka0", "ka1"] if qk else []) + (["va0", "va1"] if ex else [])
            out.append(func(f"pipe_x_{tag}_{par}", b, args, inouts=["lh"] if ex else []))
        b = gen_x(par, 1, 1, dma=True)
        lh_fold(b)
        out.append(func_dma(f"pipe_x_qk_exp_dma_{par}", b))
        nxt = 0 if par else 1
        xqe, xq = gen_x(par, 1, 1), gen_x(par, 1, 0)
        lh_fold(xqe)
        tr = {k: tuple(trailing(xb, range(SBUF[nxt][jj], SBUF[nxt][jj] + 16)) for jj in range(2))
              for k, xb in (("pv_max", xqe), ("max", xq), ("pv", xq))}
        for pv, mx, tag in ((1, 1, "pv_max"), (0, 1, "max"), (1, 0, "pv")):
            # pv_max follows the qk_exp X block, max the qk one (prologue).
            b = gen_y(par, pv, mx, tr[tag])
            args = ["va0", "va1"] if pv else []
            if mx:
                text = func(f"pipe_y_{tag}_{par}", b, args, outs=["mx", "mt"])
                # mt is a block-local temporary: declare it inside, not as a parameter.
                text = text.replace(", float& mt)", ")").replace(
                    " {\n  asm volatile", " {\n  float mt;\n  asm volatile", 1)
                out.append(text)
            else:
                out.append(func(f"pipe_y_{tag}_{par}", b, args))
        out.append(func(f"pipe_rescale_{par}", gen_rescale(par), ["corr", "shift", "negm"]))
        out.append(func(f"pipe_mask_{par}", gen_mask(par), ["hi", "ninf"],
                        extra_clobbers=["vcc"]))
    init = Block()
    for o in O:
        for k in range(16):
            init.emit(f"v_mov_b32 {r(o + k)}, 0", "valu")
    for k in range(16):
        init.emit(f"v_mov_b32 {r(NEGM + k)}, 0", "valu")
    out.append(func("pipe_init", init, []).replace("(, ", "(").replace("void pipe_init()", "void pipe_init()"))
    out.append("}  // namespace mfa")
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                       "metal-flash-attention-plus_amd", "csrc", "fwd_pipe_asm.h")
    open(dst, "w").write("\n".join(out) + "\n")
    print("wrote", os.path.normpath(dst))
    # Ablation variants of the two steady-state blocks for the diagnostic build.
    abl = ["// Generated by tools/gen_fwd_pipe.py: timing-only ablations of the steady blocks",
           "// (tools/diag/pipe_abl.hip).  Wrong results by construction.", "#pragma once",
           '#include "../../metal-flash-attention-plus_amd/csrc/fwd_pipe_asm.h"', "",
           "namespace mfa {", ""]
    for code, flags in ((4, dict(noexp=True)), (8, dict(nolds=True)),
                        (12, dict(noexp=True, nolds=True))):
        ABL.update(nolds=False, noexp=False)
        ABL.update(flags)
        for par in (0, 1):
            b = gen_x(par, 1, 1)
            lh_fold(b)
            abl.append(func(f"pipe_x_qk_exp_{par}_a{code}", b, ["ka0", "ka1", "va0", "va1"],
                            inouts=["lh"]))
            b = gen_y(par, 1, 1, (16, 16))
            text = func(f"pipe_y_pv_max_{par}_a{code}", b, ["va0", "va1"], outs=["mx", "mt"])
            text = text.replace(", float& mt)", ")").replace(
                " {\n  asm volatile", " {\n  float mt;\n  asm volatile", 1)
            abl.append(text)
    ABL.update(nolds=False, noexp=False)
    for par in (0, 1):
        for nm, sig, call in ((f"pipe_x_qk_exp_{par}", "int ka0, int ka1, int va0, int va1, float& lh",
                               "ka0, ka1, va0, va1, lh"),
                              (f"pipe_y_pv_max_{par}", "int va0, int va1, float& mx", "va0, va1, mx")):
            abl.append(f"template <int A> __device__ __forceinline__ void {nm}_a({sig}) {{")
            for code in (4, 8, 12):
                abl.append(f"  if constexpr (A == {code}) {nm}_a{code}({call});")
            abl.append("}")
    abl.append("}  // namespace mfa")
    dst2 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag", "fwd_pipe_asm_abl.h")
    open(dst2, "w").write("\n".join(abl) + "\n")
    print("wrote", os.path.normpath(dst2))


if __name__ == "__main__":
    main()
