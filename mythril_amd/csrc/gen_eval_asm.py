#!/usr/bin/env python3
"""Generator of mgp_eval_gfx950 — the hand-written gfx950 interpreter of the uop encoding.

    python3 gen_eval_asm.py <out.s> <out_header.h>

Design: one 64-lane wave per (state, 64-candidate chunk); the
uop stream is wave-uniform and is read through the scalar cache one uop ahead;
every uop is dispatched through a jump table (s_setpc_b64 into a table of
s_branch stubs), so the kernel has no decode chain and no divergent branch.
Handlers are straight-line gfx950 code on fixed registers:

  VGPR  v0 lane, v1 lane*16 (LDS lane base), v2/v3 candidate byte offsets of
        the two 16-B halves, v4-v7 scratch, vA=v[8:15], vB=v[16:23],
        vC=v[24:31], T=v[32:41] (product / division temporaries), v[42:121]
        register bank (10 positions), v[122:126] uop page, v127 loop state
  SGPR  s[4:5] uop pointer, s[6:7] candidate base of the state, s8 bytes per
        variable, s9 n_vars-1, s[10:11] jump table, s[14:15] constant pool,
        s16 w1 of the next uop, s[17:19] w1-w3 of the current uop, s[24:31] constant
        operand, s[32:39] sign constant H, s[40:47] mask constant M,
        s[48:55] temporaries, s[56:57] valid-lane mask, s[58:59] partial
        result address, s60 first candidate of the chunk, s[62:63] 2^32 (f64),
        s[64:101] 19 Bool slots as 64-bit lane masks (M0-relative s_movrels)

Every handler writes 256-bit values in 8 x u32 limbs; carries go through VCC
(v_add_co / v_addc_co), products through v_mad_u64_u32 (Comba columns),
funnel shifts through v_alignbit_b32, division is Knuth's algorithm D with
32-bit digits and a double-precision quotient estimate.  No MFMA: nothing
here is a contraction.  No scalar memory writes anywhere (vector stores only).
"""
from __future__ import annotations

import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mythril_amd import uop_spec as U  # noqa: E402

KNAME = "mgp_eval_gfx950"
# The division keeps its 16-limb dividend in vA:vC and normalises the divisor in vB, so the
# temporaries fit the 10 registers of T; that leaves 80 VGPRs for the register bank: 10
# positions, 6 for preloaded variables and register slots, 4 for register slots only
VA, VB, VC, VT = 8, 16, 24, 32
NT = 10          # T = v[32:41]: products / compare scratch; in DIV the f64 and digit registers
RV = 42          # v[42:121]: register bank, U.REG_POS positions of 8 (variables 0..5 preloaded)
PG = RV + 8 * U.REG_POS   # v[122:126]: the current 64-uop page, uop k in lane k (v_readlane):
                 #   PG first-handler address (low 32 bits), PG+1 op-handler address, PG+2..4 w1-w3
VD = PG + 5      # v127: descriptor / loop state / diagnostic lanes (SGPRs above s63 are Bools)
NVGPR = (VD + 1 + 7) // 8 * 8   # 128 with the 10-position bank (4 waves/SIMD); 96 with 6 (5 waves)
# 64-B pool lines of the state's constants pulled into the scalar cache by each wave, hidden
# behind the variable loads (4 measured 0.8 % faster than none and than 8; MGP_POOL_PF A/B)
POOL_PREFETCH_LINES = int(os.environ.get("MGP_POOL_PF", "4"))
POOL_PREFETCH_CHUNK = bool(int(os.environ.get("MGP_POOL_PF_CHUNK", "0")))   # again at each chunk
HALIGN = int(os.environ.get("MGP_HALIGN", "2"))   # log2 byte alignment of handler entries
# diagnostic builds only (A/B of the VALU cost of the dispatch reads): extra v_readlane per uop
# dispatch into the dead temporary s48; 0 in every shipped build
EXTRA_READLANES = int(os.environ.get("MGP_EXTRA_RL", "0"))
# division registers inside T
D_FA, D_FB = 32, 34          # f64 pairs: dividend / reciprocal, divisor / estimate
D_M = 36                     # v36 carry into the next product, v37 = 0 (64-bit mad addend)
D_Q, D_T = 38, 39            # qhat, scratch
D_K, D_D = 40, 41            # per-lane limb shift k, top-limb difference d
D_SA, D_SB = "s[32:33]", "s[34:35]"   # operand sign lane masks (SDIV/SREM/SMOD)
# A v_readlane costs a wave64 ~8.7 SIMD-cycles of VALU issue at 4 waves/SIMD
# (profiles/contention_probe.hip, contention_r2.json), so a handler reads only the uop
# fields it uses, and pool constants come through the scalar cache (one s_load_dwordx8
# instead of 8 readlanes).  The uop stream itself stays in VGPR lanes: read through the
# scalar cache, every 4th uop missed it (SQC_DCACHE_MISSES) and the step got slower.
S_KB, S_KH, S_KM = 24, 32, 40


def v(i):
    return f"v{i}"


def vr(i, n):
    return f"v[{i}:{i + n - 1}]"


def s(i):
    return f"s{i}"


def sr(i, n=2):
    return f"s[{i}:{i + n - 1}]"


class Asm:
    def __init__(self):
        self.lines = []
        self.n = 0
        self.ool = []   # out-of-line blocks of the current handler (rare paths), emitted after it

    def __call__(self, *ins):
        for x in ins:
            self.lines.append("  " + x)

    def label(self, name):
        self.lines.append(f"{name}:")

    def fresh(self, stem):
        self.n += 1
        return f".L{stem}_{self.n}"

    def comment(self, text):
        self.lines.append(f"  // {text}")

    def out_of_line(self, label, body):
        """Emit `body` (a callable) as a block after the handler; the common path falls through."""
        self.ool.append((label, body))

    def flush_ool(self):
        while self.ool:
            label, body = self.ool.pop(0)
            self.lines.append(f"{label}:")
            body()


A = Asm()

# ---------------------------------------------------------------- helpers


def prefetch_next():
    """At handler entry: the first-handler address of the next uop (lane s21 + 1 of the
    page, computed lane-parallel when the page was loaded) straight into s0 (s1 is the
    constant high half of the code address) and its w1 into s16, which the tail moves to
    s17: a handler finds its w1 in place instead of waiting on a v_readlane at its top.
    s21 = lane of the current uop."""
    A("s_add_u32 s3, s21, 1",
      f"v_readlane_b32 s0, {v(PG)}, s3",
      f"v_readlane_b32 s16, {v(PG + 2)}, s3")


def read_fields(used):
    """The uop fields a handler uses (w2, w3 -> s18, s19), read from lane s21 of the page
    (w1 is in s17 already: the previous uop's prefetch_next and tail)."""
    for f in (18, 19):
        if f in used:
            A(f"v_readlane_b32 s{f}, v{PG + f - 15}, s21")


def page_decode():
    """v[PG:PG+3] raw uop words w0-w3 -> PG / PG+1 absolute handler addresses (low 32 bits;
    the prologue checked that the kernel code does not cross a 4 GiB boundary), PG+2..4 w1-w3."""
    A(f"v_mov_b32 {v(PG + 4)}, {v(PG + 3)}",
      f"v_mov_b32 {v(PG + 3)}, {v(PG + 2)}",
      f"v_mov_b32 {v(PG + 2)}, {v(PG + 1)}",
      f"v_lshrrev_b32 {v(PG + 1)}, 16, {v(PG)}",
      f"v_lshl_add_u32 {v(PG + 1)}, {v(PG + 1)}, 2, s10",
      f"v_and_b32 {v(PG)}, 0xffff, {v(PG)}",
      f"v_lshl_add_u32 {v(PG)}, {v(PG)}, 2, s10",
      "s_nop 1")   # VALU write -> v_readlane of the same VGPR


def tail_wait():
    pass


def tail_jump():
    tail()


def first_fields():
    """s16 <- w1 of the uop at lane s3 (a new page, a chunk restart, the first dispatch)."""
    A(f"v_readlane_b32 s16, {v(PG + 2)}, s3")


def tail():
    """Make the prefetched uop current (s21 = its lane, s17 = its w1) and jump to its first
    handler."""
    for _ in range(EXTRA_READLANES):
        A(f"v_readlane_b32 s48, {v(PG + 2)}, s3")
    A("s_mov_b32 s21, s3",
      "s_mov_b32 s17, s16",
      "s_setpc_b64 s[0:1]")


def op_target():
    """s[12:13] <- address of the op handler of the current uop (s13 = code high half)."""
    A(f"v_readlane_b32 s12, {v(PG + 1)}, s21")


def op_dispatch():
    A("s_setpc_b64 s[12:13]")


def bool_read(field_sreg, shift, dst_pair):
    """dst_pair <- Bool slot whose (index*2) is the 16-bit field of field_sreg at shift."""
    if shift == 0:
        A(f"s_and_b32 s48, {field_sreg}, 0xffff")
    else:
        A(f"s_lshr_b32 s48, {field_sreg}, 16")
    A("s_mov_b32 m0, s48", "s_nop 0", f"s_movrels_b64 {sr(dst_pair)}, s[64:65]")


def bool_write(src_pair):
    A("s_lshr_b32 s48, s19, 16", "s_mov_b32 m0, s48", "s_nop 0", f"s_movreld_b64 s[64:65], {src_pair}")


def copy8(dst, src):
    for i in range(8):
        A(f"v_mov_b32 {v(dst + i)}, {v(src + i)}")


def sext_inplace(base):
    """x = (x ^ H) - H, H = 2^(w-1) in s[32:39] (load_kh first): sign-extends a zero-extended w-bit value.
    (gfx950 VOP2 carry ops read VCC over the constant bus, so H is copied to T first.)"""
    sext_to(base, base)


def sext_to(dst, src):
    for i in range(8):
        A(f"v_mov_b32 {v(VT + i)}, {s(S_KH + i)}")
    for i in range(8):
        A(f"v_xor_b32 {v(dst + i)}, {v(VT + i)}, {v(src + i)}")
    A(f"v_sub_co_u32 {v(dst)}, vcc, {v(dst)}, {v(VT)}")
    for i in range(1, 8):
        A(f"v_subb_co_u32 {v(dst + i)}, vcc, {v(dst + i)}, {v(VT + i)}, vcc")


def cneg(base, smask):
    """x = m ? -x : x with m a lane mask in an SGPR pair (v4, v5 scratch)."""
    A(f"v_cndmask_b32_e64 v4, 0, -1, {smask}")
    for i in range(8):
        A(f"v_xor_b32 {v(base + i)}, {v(base + i)}, v4")
    A("v_lshrrev_b32 v5, 31, v4",
      f"v_add_co_u32 {v(base)}, vcc, v5, {v(base)}")
    for i in range(1, 8):
        A(f"v_addc_co_u32 {v(base + i)}, vcc, 0, {v(base + i)}, vcc")


def or_reduce(dst, regs):
    """dst = OR of the regs (dst may be one of them)."""
    regs = list(regs)
    cur = regs[0]
    rest = regs[1:]
    while rest:
        if len(rest) >= 2:
            A(f"v_or3_b32 {v(dst)}, {v(cur)}, {v(rest[0])}, {v(rest[1])}")
            rest = rest[2:]
        else:
            A(f"v_or_b32 {v(dst)}, {v(cur)}, {v(rest[0])}")
            rest = []
        cur = dst


def shift_setup(vs, left):
    """Per-lane shift amount vs (0..255) -> k masks s[48:49] (4), s[50:51] (2), s[52:53] (1),
    v5 = bit shift b, v6 = 32-b, s[54:55] = (b == 0).  Uses v4, v7."""
    A(f"v_lshrrev_b32 v4, 5, {v(vs)}",
      f"v_and_b32 v5, 31, {v(vs)}",
      "v_and_b32 v7, 4, v4", "v_cmp_ne_u32_e64 s[48:49], 0, v7",
      "v_and_b32 v7, 2, v4", "v_cmp_ne_u32_e64 s[50:51], 0, v7",
      "v_and_b32 v7, 1, v4", "v_cmp_ne_u32_e64 s[52:53], 0, v7")
    if left:
        A("v_sub_u32 v6, 32, v5", "v_cmp_eq_u32_e64 s[54:55], 0, v5")


def shl_var(regs, nz):
    """In-place per-lane left shift of the limb list `regs` (low first) after shift_setup(left).
    nz = number of low limbs that may be non-zero on entry (the rest are zero)."""
    n = len(regs)
    for L, m in ((4, "s[48:49]"), (2, "s[50:51]"), (1, "s[52:53]")):
        new_nz = min(n, nz + L)
        for i in range(new_nz - 1, -1, -1):
            src = i - L
            if i >= nz:
                if src >= 0:
                    A(f"v_cndmask_b32_e64 {v(regs[i])}, 0, {v(regs[src])}, {m}")
            elif src < 0:
                A(f"v_cndmask_b32_e64 {v(regs[i])}, {v(regs[i])}, 0, {m}")
            else:
                A(f"v_cndmask_b32_e64 {v(regs[i])}, {v(regs[i])}, {v(regs[src])}, {m}")
        nz = new_nz
    top = min(n - 1, nz)
    for i in range(top, 0, -1):
        A(f"v_alignbit_b32 v7, {v(regs[i])}, {v(regs[i - 1])}, v6",
          f"v_cndmask_b32_e64 {v(regs[i])}, v7, {v(regs[i])}, s[54:55]")
    A(f"v_lshlrev_b32 {v(regs[0])}, v5, {v(regs[0])}")


def shr_var(regs, fill):
    """In-place per-lane right shift after shift_setup(left=False); fill = '0' or a VGPR name."""
    n = len(regs)
    for L, m in ((4, "s[48:49]"), (2, "s[50:51]"), (1, "s[52:53]")):
        for i in range(n):
            src = regs[i + L] if i + L < n else None
            val = v(src) if src is not None else fill
            A(f"v_cndmask_b32_e64 {v(regs[i])}, {v(regs[i])}, {val}, {m}")
    for i in range(n):
        hi = v(regs[i + 1]) if i + 1 < n else fill
        A(f"v_alignbit_b32 {v(regs[i])}, {hi}, {v(regs[i])}, v5")


def amount_from_vB():
    """v4 <- per-lane shift amount from vB clamped to 0..255, v6 <- all-ones where it is >= 256."""
    A(f"v_lshrrev_b32 v7, 8, {v(VB)}")
    or_reduce(4, [7, VB + 1, VB + 2, VB + 3, VB + 4, VB + 5, VB + 6, VB + 7])
    A("v_cmp_ne_u32_e64 s[48:49], 0, v4",
      "v_cndmask_b32_e64 v6, 0, -1, s[48:49]",
      f"v_and_b32 v4, 0xff, {v(VB)}")


def top_limb(base, out):
    """out = index of the top non-zero limb of the 256-bit value at base (0 when zero)."""
    A(f"v_mov_b32 {v(out)}, 0")
    for i in range(1, 8):
        A(f"v_cmp_ne_u32 vcc, 0, {v(base + i)}", f"v_cndmask_b32_e64 {v(out)}, {v(out)}, {i}, vcc")


def limb_masks(vk):
    """Per-lane limb count vk (0..7) -> stage masks s[48:49] (4), s[50:51] (2), s[52:53] (1)."""
    A(f"v_and_b32 v7, 4, {v(vk)}", "v_cmp_ne_u32_e64 s[48:49], 0, v7",
      f"v_and_b32 v7, 2, {v(vk)}", "v_cmp_ne_u32_e64 s[50:51], 0, v7",
      f"v_and_b32 v7, 1, {v(vk)}", "v_cmp_ne_u32_e64 s[52:53], 0, v7")


def shl_limbs(regs, nz):
    """In-place per-lane left shift by whole limbs after limb_masks; nz = number of low
    limbs that may be non-zero on entry."""
    n = len(regs)
    for L, m in ((4, "s[48:49]"), (2, "s[50:51]"), (1, "s[52:53]")):
        new_nz = min(n, nz + L)
        for i in range(new_nz - 1, -1, -1):
            src = i - L
            if i >= nz:
                if src >= 0:
                    A(f"v_cndmask_b32_e64 {v(regs[i])}, 0, {v(regs[src])}, {m}")
            elif src < 0:
                A(f"v_cndmask_b32_e64 {v(regs[i])}, {v(regs[i])}, 0, {m}")
            else:
                A(f"v_cndmask_b32_e64 {v(regs[i])}, {v(regs[i])}, {v(regs[src])}, {m}")
        nz = new_nz


def shr_limbs(regs):
    """In-place per-lane right shift by whole limbs after limb_masks (zero fill)."""
    n = len(regs)
    for L, m in ((4, "s[48:49]"), (2, "s[50:51]"), (1, "s[52:53]")):
        for i in range(n):
            val = v(regs[i + L]) if i + L < n else "0"
            A(f"v_cndmask_b32_e64 {v(regs[i])}, {v(regs[i])}, {val}, {m}")


# ---------------------------------------------------------------- handlers

HBODY = {}


def handler(name):
    def deco(fn):
        HBODY[name] = fn
        return fn
    return deco


def wait_operands():
    """Operands of the op: LDS slot and pool-constant reads (a fetch handler with an HBM
    variable operand waits for its own vector loads before it dispatches, so outstanding
    spill stores do not hold up the op handlers)."""
    A("s_waitcnt lgkmcnt(0)")


# uop flag bits (w2 = s18, w3 = s19; see uop_spec)
B_STORE, B_MASK, B_SEXT, B_INVERT, B_REGST = 22, 23, 24, 25, 29
B_BCOMB, B_BCOMB_OR = U.F_BCOMB.bit_length() - 1, U.F_BCOMB_OR.bit_length() - 1


def load_pool(dst, idx_sreg):
    """s[dst:dst+7] <- pool entry idx (32 B per entry at s[14:15])."""
    A(f"s_lshl_b32 {idx_sreg}, {idx_sreg}, 5",
      f"s_load_dwordx8 {sr(dst, 8)}, s[14:15], {idx_sreg}",
      "s_waitcnt lgkmcnt(0)")


def load_km():
    """s[40:47] <- pool[mask index w2[21:16]] (2^w - 1)."""
    A(f"s_bfe_u32 s48, s18, {(6 << 16) | 16:#x}")
    load_pool(S_KM, "s48")


def load_kh():
    """s[32:39] <- pool[sign index w3[5:0]] (2^(w-1))."""
    A("s_and_b32 s49, s19, 0x3f")
    load_pool(S_KH, "s49")


def store_slot():
    A("s_and_b32 s48, s18, 0xffff",
      "v_add_u32 v4, s48, v1",
      f"ds_write_b128 v4, {vr(VA, 4)}",
      f"ds_write_b128 v4, {vr(VA + 4, 4)} offset:1024")


def store_reg():
    """vA -> register-bank position p (w2[15:0] = 8p): GPR-index mode offsets the
    destination of the moves into the bank."""
    A("s_and_b32 s48, s18, 0xffff",
      "s_set_gpr_idx_on s48, gpr_idx(DST)")
    for i in range(8):
        A(f"v_mov_b32 {v(RV + i)}, {v(VA + i)}")
    A("s_set_gpr_idx_off")


EPI_MODE = [None]   # None: test the STORE/MASK flags at run time; else the variant's fixed epilogue


def bv_epilogue():
    """[mask] [store] then dispatch; unmasked results fall straight through to the tail."""
    mode = EPI_MODE[0]
    if mode is not None:
        if "M" in mode:
            load_km()
            for i in range(8):
                A(f"v_and_b32 {v(VA + i)}, {s(S_KM + i)}, {v(VA + i)}")
        if "S" in mode:
            tail_wait()
            store_slot()
            tail_jump()
            return
        if "R" in mode:
            store_reg()
        tail()
        return
    lm, ls = A.fresh("mask"), A.fresh("store")
    A(f"s_bitcmp1_b32 s18, {B_MASK}", f"s_cbranch_scc1 {lm}",
      f"s_bitcmp1_b32 s18, {B_STORE}", f"s_cbranch_scc1 {ls}")
    tail()

    def masked():
        load_km()
        for i in range(8):
            A(f"v_and_b32 {v(VA + i)}, {s(S_KM + i)}, {v(VA + i)}")
        A(f"s_bitcmp1_b32 s18, {B_STORE}", f"s_cbranch_scc1 {ls}")
        tail()

    def stored():
        lr = A.fresh("regst")
        A(f"s_bitcmp1_b32 s18, {B_REGST}", f"s_cbranch_scc1 {lr}")
        tail_wait()
        store_slot()
        tail_jump()

        def reg():
            store_reg()
            tail()
        A.out_of_line(lr, reg)
    A.out_of_line(lm, masked)
    A.out_of_line(ls, stored)


def cmp_epilogue():
    """vcc -> Bool slot w3[31:16].  Out of line: INVERT negates it; BCOMB combines it with
    the Bool slot w3[15:8] (AND, or OR with BCOMB_OR) first: a compare whose result only
    feeds the next BAND / BOR, folded by the translator (one dispatch instead of two)."""
    li = A.fresh("inv")
    A(f"s_and_b32 s48, s18, {(1 << B_INVERT) | (1 << B_BCOMB):#x}", f"s_cbranch_scc1 {li}")
    bool_write("vcc")
    tail()

    def special():
        lni, lw, lor = A.fresh("noinv"), A.fresh("cwrite"), A.fresh("cor")
        A(f"s_bitcmp1_b32 s18, {B_INVERT}", f"s_cbranch_scc0 {lni}",
          "s_not_b64 vcc, vcc")
        A.label(lni)
        A(f"s_bitcmp1_b32 s18, {B_BCOMB}", f"s_cbranch_scc0 {lw}",
          f"s_bfe_u32 s48, s19, {(8 << 16) | U.BCOMB_POS:#x}",
          "s_mov_b32 m0, s48", "s_nop 0", "s_movrels_b64 s[50:51], s[64:65]",
          f"s_bitcmp1_b32 s18, {B_BCOMB_OR}", f"s_cbranch_scc1 {lor}",
          "s_and_b64 vcc, vcc, s[50:51]", f"s_branch {lw}")
        A.label(lor)
        A("s_or_b64 vcc, vcc, s[50:51]")
        A.label(lw)
        bool_write("vcc")
        tail()
    A.out_of_line(li, special)


def write_partial_and_end(value_sreg):
    A("s_mov_b64 exec, 1",
      f"v_mov_b32 v4, {value_sreg}",
      "v_mov_b32 v5, 0",
      "global_store_dword v5, v4, s[58:59]",
      "s_endpgm")


@handler("INVALID")
def h_invalid():
    A("s_waitcnt vmcnt(0) lgkmcnt(0)", "s_mov_b32 s48, -2")
    write_partial_and_end("s48")


def fetch_one(kind, dst, which):
    """Issue the fetch of operand A (which='A', w1[15:0]) or B (w1[31:16]) into dst."""
    sp = "s51" if which == "A" else "s50"
    pr = "s[54:55]" if which == "A" else "s[52:53]"
    vaddr = "v5" if which == "A" else "v4"
    get = (f"s_and_b32 {sp}, s17, 0xffff" if which == "A" else f"s_lshr_b32 {sp}, s17, 16")
    if kind == "acc":
        if which == "B":
            copy8(dst, VA)
        return
    A(get)
    if kind == "rvar":
        # v[dst+i] = v[RV + 8*p + i]: GPR-index mode (gfx950 has no v_movrels) offsets
        # SRC0 of the moves by 8*var into the preloaded variable bank
        A(f"s_set_gpr_idx_on {sp}, gpr_idx(SRC0)")
        for i in range(8):
            A(f"v_mov_b32 {v(dst + i)}, {v(RV + i)}")
        A("s_set_gpr_idx_off")
        return
    if kind == "slot":
        A(f"v_add_u32 {vaddr}, {sp}, v1",
          f"ds_read_b128 {vr(dst, 4)}, {vaddr}",
          f"ds_read_b128 {vr(dst + 4, 4)}, {vaddr} offset:1024")
    elif kind == "var":
        lo = 54 if which == "A" else 52
        A(f"s_min_u32 {sp}, {sp}, s9",
          f"s_mul_i32 {sp}, {sp}, s8",
          f"s_add_u32 s{lo}, s6, {sp}",
          f"s_addc_u32 s{lo + 1}, s7, 0",
          f"global_load_dwordx4 {vr(dst, 4)}, v2, {pr}",
          f"global_load_dwordx4 {vr(dst + 4, 4)}, v3, {pr}")
    else:  # const: pool entry `idx` through the scalar cache (make_fetch issues it first)
        const_issue(which)
        const_finish(dst, which)


def const_issue(which):
    """Issue the scalar load of a pool-constant operand (A: w1[15:0] -> s[32:39], B:
    w1[31:16] -> s[24:31]; 32 B per pool entry at s[14:15]); VGPR pool: the readlanes."""
    sp = "s51" if which == "A" else "s50"
    ks = S_KB if which == "B" else S_KH
    A(f"s_and_b32 {sp}, s17, 0xffff" if which == "A" else f"s_lshr_b32 {sp}, s17, 16")
    A(f"s_lshl_b32 {sp}, {sp}, 5",
      f"s_load_dwordx8 {sr(ks, 8)}, s[14:15], {sp}")


def const_finish(dst, which):
    ks = S_KB if which == "B" else S_KH
    A("s_waitcnt lgkmcnt(0)")
    for i in range(8):
        A(f"v_mov_b32 {v(dst + i)}, {s(ks + i)}")


def make_fetch(name):
    _, ka, kb, tgt = name.split("_")

    def body():
        # pool constants first: their scalar loads overlap the other operand's fetch
        for kind, which in ((kb, "B"), (ka, "A")):
            if kind == "const":
                const_issue(which)
        op_target()
        if kb not in ("none", "const"):
            fetch_one(kb, VB, "B")
        if ka != "const":
            fetch_one(ka, VA if tgt == "A" else VC, "A")
        if kb == "const":
            const_finish(VB, "B")
        if ka == "const":
            const_finish(VA if tgt == "A" else VC, "A")
        if "var" in (ka, kb):
            A("s_waitcnt vmcnt(0)")
        op_dispatch()
    return body


for _f in U.FETCH:
    HBODY[_f] = make_fetch(_f)


# ---- program paging
@handler("PAGE")
def h_page():
    # next 64 uops: lane k loads uop min(k, remaining) of the next page into v[PG:PG+3]
    # (s2 = uops left from the page start; index `remaining` is the INVALID pad)
    A("s_add_u32 s4, s4, 0x400", "s_addc_u32 s5, s5, 0",
      "s_sub_u32 s2, s2, 64",
      "v_min_u32 v4, s2, v0",
      "v_lshlrev_b32 v4, 4, v4",
      "s_waitcnt vmcnt(0)",
      f"global_load_dwordx4 {vr(PG, 4)}, v4, s[4:5]",
      "s_waitcnt vmcnt(0)",
      "s_mov_b32 s3, 0")
    page_decode()
    A(f"v_readlane_b32 s0, {v(PG)}, s3")
    first_fields()
    tail()


# ---- spill rows
@handler("VST")
def h_vst():
    """vA -> this lane's candidate row w2[15:0]: a BV slot past the LDS slots (spill,
    include/mgp_ir.h).  Later uops read the row back as a VAR operand; a wave's vector
    memory accesses to one address stay in order, so the load sees this store."""
    A("s_and_b32 s48, s18, 0xffff",
      "s_mul_i32 s48, s48, s8",
      "s_add_u32 s52, s6, s48",
      "s_addc_u32 s53, s7, 0",
      f"global_store_dwordx4 v2, {vr(VA, 4)}, s[52:53]",
      f"global_store_dwordx4 v3, {vr(VA + 4, 4)}, s[52:53]")
    tail()


# ---- Bool ops
def diag_stamp():
    """Diagnostic build-in (kernarg diag != 0): diag[item] = {descriptor landed - entry,
    page/pool/variables landed - descriptor, first dispatch - loads, RET - first
    dispatch} in shader clocks (32-bit differences)."""
    ln = A.fresh("nodiag")
    A("s_cmp_eq_u32 s20, 0", f"s_cbranch_scc1 {ln}",
      f"v_readlane_b32 s24, {v(VD)}, 0", f"v_readlane_b32 s25, {v(VD)}, 1",
      "s_memtime s[54:55]",
      f"v_readlane_b32 s26, {v(VD)}, 2", f"v_readlane_b32 s27, {v(VD)}, 7",
      f"v_readlane_b32 s28, {v(VD)}, 8", f"v_readlane_b32 s29, {v(VD)}, 4",
      f"v_readlane_b32 s30, {v(VD)}, 6",
      "s_lshl_b32 s30, s30, 4", "s_add_u32 s24, s24, s30", "s_addc_u32 s25, s25, 0",
      "s_sub_u32 s26, s27, s26", "s_sub_u32 s27, s28, s27", "s_sub_u32 s28, s29, s28",
      "s_waitcnt lgkmcnt(0)",
      "s_sub_u32 s29, s54, s29",
      "s_mov_b64 exec, 1",
      "v_mov_b32 v4, s26", "v_mov_b32 v5, s27", "v_mov_b32 v6, s28", "v_mov_b32 v7, s29",
      "v_mov_b32 v8, 0",
      "global_store_dwordx4 v8, v[4:7], s[24:25]")
    A.label(ln)


@handler("RET")
def h_ret():
    A("s_waitcnt vmcnt(0)")
    bool_read("s17", 0, 50)
    A("s_and_b64 s[50:51], s[50:51], s[56:57]",
      "s_ff1_i32_b64 s52, s[50:51]",
      "s_add_u32 s53, s60, s52",
      "s_cmp_lt_i32 s52, 0",
      "s_cselect_b32 s53, 0x7fffffff, s53")
    diag_stamp()
    A("s_mov_b64 exec, 1",
      "v_mov_b32 v4, s53",
      "v_mov_b32 v5, 0",
      "global_store_dword v5, v4, s[58:59]",
      "s_mov_b64 exec, -1",
      "s_add_u32 s22, s22, 1",
      "s_cmp_lt_u32 s22, s23",
      "s_cbranch_scc1 .Lnext_chunk",
      "s_endpgm")
    next_chunk()


def next_chunk():
    """RET of a wave with chunks left: the same program on the next 64 candidates of
    the state.  Partial entry, first candidate, valid lanes and candidate offsets
    advance; page 0 is reloaded when the program had more than one page; the
    variables are preloaded again; Bool slots 0/1 and the f64 constant are restored."""
    A.label(".Lnext_chunk")
    A("s_add_u32 s58, s58, 4",
      "s_addc_u32 s59, s59, 0",
      "s_add_u32 s60, s60, 64",
      f"v_readlane_b32 s49, {v(VD)}, 15",
      f"v_readlane_b32 s2, {v(VD)}, 13",
      f"v_readlane_b32 s4, {v(VD)}, 11",
      f"v_readlane_b32 s5, {v(VD)}, 12",
      f"v_readlane_b32 s91, {v(VD)}, 14",
      "s_sub_u32 s50, s49, 1",
      "s_lshl_b32 s51, s49, 4",
      # VALU-written SGPRs feed VALU operands and a VMEM base below
      "s_nop 4",
      "v_add_u32 v5, s60, v0",
      "v_cmp_gt_u32_e64 s[56:57], s49, v5",
      "v_min_u32 v5, s50, v5",
      "v_lshlrev_b32 v2, 4, v5",
      "v_add_u32 v3, s51, v2",
      "s_cmp_lt_u32 s2, 64",
      "s_cbranch_scc1 .Lpage0_kept",
      "v_min_u32 v4, s2, v0",
      "v_lshlrev_b32 v4, 4, v4",
      f"global_load_dwordx4 {vr(PG, 4)}, v4, s[4:5]")
    if POOL_PREFETCH_CHUNK:
        A.lines.extend(pool_prefetch("r"))
    A.lines.append(var_preload("r").rstrip("\n"))
    page_decode()
    A("s_branch .Lrestart")
    A.label(".Lpage0_kept")
    if POOL_PREFETCH_CHUNK:
        A.lines.extend(pool_prefetch("k"))
    A.lines.append(var_preload("k").rstrip("\n"))
    A.label(".Lrestart")
    A("s_mov_b64 s[64:65], 0",
      "s_mov_b64 s[66:67], -1",
      "s_mov_b32 s62, 0",
      "s_mov_b32 s63, 0x41f00000",
      "s_mov_b32 s3, 0",
      f"v_readlane_b32 s0, {v(PG)}, s3")
    first_fields()
    tail()


def bool_binop(name, instr):
    @handler(name)
    def _():
        # the S_MOVREL-after-M0-write wait state is filled with the next operand's field extract
        A("s_and_b32 s48, s17, 0xffff", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s17, 16",
          "s_movrels_b64 s[50:51], s[64:65]", "s_mov_b32 m0, s49", "s_lshr_b32 s48, s19, 16",
          "s_movrels_b64 s[52:53], s[64:65]", "s_mov_b32 m0, s48",
          f"{instr} s[50:51], s[50:51], s[52:53]", "s_movreld_b64 s[64:65], s[50:51]")
        tail()


bool_binop("BAND", "s_and_b64")
bool_binop("BOR", "s_or_b64")
bool_binop("BXOR", "s_xor_b64")
bool_binop("BEQ", "s_xnor_b64")


@handler("BAND4")
def h_band4():
    # dst = a & b & c & d: a, b in w1 (s17), c, d in w2 (s18); each M0 write's wait state is
    # filled with the next field extract or AND
    A("s_and_b32 s48, s17, 0xffff", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s17, 16",
      "s_movrels_b64 s[50:51], s[64:65]", "s_mov_b32 m0, s49", "s_and_b32 s48, s18, 0xffff",
      "s_movrels_b64 s[52:53], s[64:65]", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s18, 16",
      "s_movrels_b64 s[54:55], s[64:65]", "s_mov_b32 m0, s49", "s_and_b64 s[50:51], s[50:51], s[52:53]",
      "s_movrels_b64 s[52:53], s[64:65]", "s_lshr_b32 s48, s19, 16",
      "s_and_b64 s[50:51], s[50:51], s[54:55]", "s_mov_b32 m0, s48",
      "s_and_b64 s[50:51], s[50:51], s[52:53]", "s_movreld_b64 s[64:65], s[50:51]")
    tail()


def make_band4n(m):
    """BAND4N<m>: dst = a' & b' & c' & d' where x' = ~x for the operands in mask m (bit 0 =
    a), same schedule as BAND4 (each M0 write's wait state filled)."""
    def comb(r, x, neg):
        A(f"s_andn2_b64 {r}, {r}, {x}" if neg else f"s_and_b64 {r}, {r}, {x}")

    def first():   # s[50:51] = a' & b'
        na, nb = m & 1, m >> 1 & 1
        if na and nb:
            A("s_nor_b64 s[50:51], s[50:51], s[52:53]")
        elif na:
            A("s_andn2_b64 s[50:51], s[52:53], s[50:51]")
        else:
            comb("s[50:51]", "s[52:53]", nb)

    def _():
        A("s_and_b32 s48, s17, 0xffff", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s17, 16",
          "s_movrels_b64 s[50:51], s[64:65]", "s_mov_b32 m0, s49", "s_and_b32 s48, s18, 0xffff",
          "s_movrels_b64 s[52:53], s[64:65]", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s18, 16",
          "s_movrels_b64 s[54:55], s[64:65]", "s_mov_b32 m0, s49")
        first()
        A("s_movrels_b64 s[52:53], s[64:65]", "s_lshr_b32 s48, s19, 16")
        comb("s[50:51]", "s[54:55]", m >> 2 & 1)
        A("s_mov_b32 m0, s48")
        comb("s[50:51]", "s[52:53]", m >> 3 & 1)
        A("s_movreld_b64 s[64:65], s[50:51]")
        tail()
    return _


for _m in range(1, 16):
    HBODY[f"BAND4N{_m}"] = make_band4n(_m)


@handler("BANDN")
def h_bandn():
    # dst = a & ~b (a BNOT whose result only feeds the next BAND, folded by the translator)
    A("s_and_b32 s48, s17, 0xffff", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s17, 16",
      "s_movrels_b64 s[50:51], s[64:65]", "s_mov_b32 m0, s49", "s_lshr_b32 s48, s19, 16",
      "s_movrels_b64 s[52:53], s[64:65]", "s_mov_b32 m0, s48",
      "s_andn2_b64 s[50:51], s[50:51], s[52:53]", "s_movreld_b64 s[64:65], s[50:51]")
    tail()


@handler("BNOT")
def h_bnot():
    A("s_and_b32 s48, s17, 0xffff", "s_mov_b32 m0, s48", "s_lshr_b32 s49, s19, 16",
      "s_movrels_b64 s[50:51], s[64:65]", "s_mov_b32 m0, s49", "s_not_b64 s[50:51], s[50:51]",
      "s_movreld_b64 s[64:65], s[50:51]")
    tail()


@handler("BITE")
def h_bite():
    bool_read("s17", 0, 50)
    bool_read("s17", 16, 52)
    bool_read("s18", 0, 54)
    A("s_and_b64 s[52:53], s[50:51], s[52:53]",
      "s_andn2_b64 s[54:55], s[54:55], s[50:51]",
      "s_or_b64 s[50:51], s[52:53], s[54:55]")
    bool_write("s[50:51]")
    tail()


# ---- BV binary
def bin_limbs(name, first, rest):
    @handler(name)
    def _():
        wait_operands()
        A(first.format(d=v(VA), a=v(VA), b=v(VB)))
        for i in range(1, 8):
            A(rest.format(d=v(VA + i), a=v(VA + i), b=v(VB + i)))
        bv_epilogue()


BIN_LIMBS = {
    "ADD": ("v_add_co_u32 {d}, vcc, {a}, {b}", "v_addc_co_u32 {d}, vcc, {a}, {b}, vcc"),
    "SUB": ("v_sub_co_u32 {d}, vcc, {a}, {b}", "v_subb_co_u32 {d}, vcc, {a}, {b}, vcc"),
    "AND": ("v_and_b32 {d}, {a}, {b}", "v_and_b32 {d}, {a}, {b}"),
    "OR": ("v_or_b32 {d}, {a}, {b}", "v_or_b32 {d}, {a}, {b}"),
    "XOR": ("v_xor_b32 {d}, {a}, {b}", "v_xor_b32 {d}, {a}, {b}"),
}
for _n, (_f, _r) in BIN_LIMBS.items():
    bin_limbs(_n, _f, _r)


def make_xr(name):
    """XR_<op>[_<epilogue>]: vA = vA op bank[B].  Operand B (w1[31:16] = 8p) is read as
    the indexed SRC1 of the limb ops themselves (GPR-index mode), so the uop needs no
    fetch handler, no moves and no operand wait (vA and the bank are both resident)."""
    base = name[3:]
    if base in ("EQ_RA", "ULT_RA", "UGT_RA"):
        return make_xr_cmp(base[:-3])
    op, mode = (base.split("_", 1) + [""])[:2]
    first, rest = BIN_LIMBS[op]

    def body():
        A("s_lshr_b32 s50, s17, 16",
          "s_set_gpr_idx_on s50, gpr_idx(SRC1)",
          first.format(d=v(VA), a=v(VA), b=v(RV)))
        for i in range(1, 8):
            A(rest.format(d=v(VA + i), a=v(VA + i), b=v(RV + i)))
        A("s_set_gpr_idx_off")
        EPI_MODE[0] = mode
        try:
            bv_epilogue()
        finally:
            EPI_MODE[0] = None
    return body


def make_xr_cmp(base, X=VA):
    """XR_<cmp>_RA: Bool = X cmp bank[B] (X = vA; vC for the XV C-target forms), B read in
    GPR-index mode as SRC1 (EQ, ULT) or, for UGT (computed as B < X), as SRC0 of the borrow
    chain."""
    def body():
        A("s_lshr_b32 s50, s17, 16")
        if base == "EQ":
            A("s_set_gpr_idx_on s50, gpr_idx(SRC1)")
            for i in range(8):
                A(f"v_xor_b32 {v(VT + i)}, {v(X + i)}, {v(RV + i)}")
            A("s_set_gpr_idx_off")
            or_reduce(VT, range(VT, VT + 8))
            A(f"v_cmp_eq_u32 vcc, 0, {v(VT)}")
        elif base == "ULT":
            A("s_set_gpr_idx_on s50, gpr_idx(SRC1)")
            ult_chain(X, RV)
            A("s_set_gpr_idx_off")
        else:
            A("s_set_gpr_idx_on s50, gpr_idx(SRC0)")
            ult_chain(RV, X)
            A("s_set_gpr_idx_off")
        cmp_epilogue()
    return body


for _x in U.XR_OPS:
    HBODY[_x] = make_xr(_x)


def make_xs(name):
    """XS_<op>: the B slot read of F_acc_slot_A at the top of the op handler itself,
    issued before the next uop's readlanes so that they overlap its latency."""
    def body():
        fetch_one("slot", VB, "B")
        prefetch_next()
        HBODY[name[3:]]()
    return body


def make_xc(name):
    """XC_<op>: the pool-constant fetch of F_acc_const_A at the top of the op handler itself
    (scalar load issued before the next uop's readlane, so that the readlane overlaps it)."""
    def body():
        const_issue("B")
        prefetch_next()
        const_finish(VB, "B")
        HBODY[name[3:]]()
    return body


def with_epi(mode):
    """bv_epilogue() with a fixed epilogue variant ("" / "S" / "R" ...)."""
    EPI_MODE[0] = mode
    try:
        bv_epilogue()
    finally:
        EPI_MODE[0] = None


def idx_on(field, mode):
    """GPR-index mode on the bank offset of operand A (field "A": w1[15:0]) or B (w1[31:16])."""
    A("s_and_b32 s51, s17, 0xffff" if field == "A" else "s_lshr_b32 s51, s17, 16",
      f"s_set_gpr_idx_on s51, gpr_idx({mode})")


def xv_ite(field, then_bank):
    """vA = c ? then : else with one of the two read straight from the bank (GPR-index mode
    on the VOP2 cndmask: the else value is SRC0, the then value SRC1; c moved to vcc)."""
    bool_read("s19", 16, 50)
    A("s_mov_b64 vcc, s[50:51]")
    idx_on(field, "SRC1" if then_bank else "SRC0")
    for i in range(8):
        if then_bank:
            A(f"v_cndmask_b32 {v(VA + i)}, {v(VA + i)}, {v(RV + i)}, vcc")
        else:
            A(f"v_cndmask_b32 {v(VA + i)}, {v(RV + i)}, {v(VA + i)}, vcc")
    A("s_set_gpr_idx_off")


def make_xv(name):
    """XV_<ka>_<kb>_<tgt>_<op>: a register-only fetch and its op in one handler.  Where the
    op body reads a bank operand through one operand position, that position is read in
    GPR-index mode (no moves); otherwise the operands are moved (accumulator / bank) and
    the op body follows."""
    _, ka, kb, tgt, op = name.split("_", 4)
    base, mode = (op.split("_", 1) + [""])[:2]

    def generic():
        if kb != "none":
            fetch_one(kb, VB, "B")
        if ka != "acc":
            fetch_one(ka, VA if tgt == "A" else VC, "A")
        prefetch_next()
        HBODY[op]()

    def body():
        if kb == "rvar" and ka in ("acc", "rvar") and tgt == "A" and op in U.XR_BASE:
            # vA = A op bank[B]: A moved when it is a bank value, B indexed (the XR body)
            if ka == "rvar":
                fetch_one("rvar", VA, "A")
            prefetch_next()
            HBODY["XR_" + op]()
        elif kb == "rvar" and ka == "rvar" and tgt == "C" and base in ("EQ", "ULT", "UGT") and mode == "RC":
            fetch_one("rvar", VC, "A")
            prefetch_next()
            make_xr_cmp(base, VC)()
        elif kb == "rvar" and tgt == "A" and base == "ITE" and mode in ("", "R"):
            if ka == "rvar":
                fetch_one("rvar", VA, "A")
            prefetch_next()
            xv_ite("B", then_bank=False)
            with_epi(mode)
        elif kb == "acc" and ka == "rvar" and base == "ITE" and mode in ("", "R"):
            prefetch_next()
            xv_ite("A", then_bank=True)
            with_epi(mode)
        elif kb == "acc" and ka == "rvar" and base == "SUB" and mode in ("", "R"):
            # vA = bank[A] - vA: the minuend indexed as SRC0
            prefetch_next()
            idx_on("A", "SRC0")
            A(f"v_sub_co_u32 {v(VA)}, vcc, {v(RV)}, {v(VA)}")
            for i in range(1, 8):
                A(f"v_subb_co_u32 {v(VA + i)}, vcc, {v(RV + i)}, {v(VA + i)}, vcc")
            A("s_set_gpr_idx_off")
            with_epi(mode)
        elif kb == "none" and ka == "rvar" and base == "NOT" and mode in ("", "R"):
            prefetch_next()
            idx_on("A", "SRC0")
            for i in range(8):
                A(f"v_not_b32 {v(VA + i)}, {v(RV + i)}")
            A("s_set_gpr_idx_off")
            with_epi(mode)
        elif kb == "none" and ka == "rvar" and re.fullmatch(r"LSHRI[0-7]", op):
            # vA = bank[A] >> (32k + b): both funnel sources from the bank (SRC0 | SRC1)
            k = int(op[-1])
            prefetch_next()
            uniform_b()
            idx_on("A", "SRC0,SRC1")
            shri_body(k, "0", src=RV)
            A("s_set_gpr_idx_off")
            bv_epilogue()          # MASK / STORE tested at run time, as in LSHRI<k>
        elif kb == "rvar" and ka in ("acc", "rvar") and tgt == "A" and op == "MUL":
            # the multiplier's limbs are SRC1 of every v_mad_u64_u32: indexed
            if ka == "rvar":
                fetch_one("rvar", VA, "A")
            prefetch_next()
            A("s_lshr_b32 s52, s17, 16", "s_set_gpr_idx_on s52, gpr_idx(SRC1)")
            mul_low(VA, RV, VT)
            A("s_set_gpr_idx_off")
            copy8(VA, VT)
            bv_epilogue()          # MASK / STORE tested at run time, as in MUL
        else:
            generic()
    return body


def mul_low(xa, yb, out):
    """out[0..7] = low 256 bits of X*Y (Comba columns, v[4:5] + v6 accumulator; the first
    carry of a column sets v6 instead of adding to a zeroed one)."""
    for k in range(8):
        pairs = [(i, k - i) for i in range(k + 1)]
        for n, (i, j) in enumerate(pairs):
            src2 = "0" if (k == 0 and n == 0) else "v[4:5]"
            A(f"v_mad_u64_u32 v[4:5], s[48:49], {v(xa + i)}, {v(yb + j)}, {src2}")
            if k < 7 and not (k == 0 and n == 0):
                A("v_addc_co_u32 v6, s[50:51], 0, 0, s[48:49]" if n == 0 else
                  "v_addc_co_u32 v6, s[50:51], v6, 0, s[48:49]")
        A(f"v_mov_b32 {v(out + k)}, v4")
        if k < 7:
            # column 0 has one product and no carry word
            A("v_mov_b32 v4, v5", "v_mov_b32 v5, 0" if k == 0 else "v_mov_b32 v5, v6")


def mul_full(xa, yb, out, hi_or):
    """out[0..7] = low 256 bits of X*Y, hi_or = OR of the high 256 bits' limbs (!= 0 iff
    the 512-bit product overflows 256 bits)."""
    A("v_mov_b32 v4, 0", "v_mov_b32 v5, 0", "v_mov_b32 v6, 0")
    for k in range(15):
        for i in range(max(0, k - 7), min(k, 7) + 1):
            j = k - i
            A(f"v_mad_u64_u32 v[4:5], s[48:49], {v(xa + i)}, {v(yb + j)}, v[4:5]",
              "v_addc_co_u32 v6, s[50:51], v6, 0, s[48:49]")
        if k < 8:
            A(f"v_mov_b32 {v(out + k)}, v4")
        elif k == 8:
            A(f"v_mov_b32 {v(hi_or)}, v4")
        else:
            A(f"v_or_b32 {v(hi_or)}, {v(hi_or)}, v4")
        A("v_mov_b32 v4, v5", "v_mov_b32 v5, v6", "v_mov_b32 v6, 0")
    A(f"v_or_b32 {v(hi_or)}, {v(hi_or)}, v4")


@handler("MUL")
def h_mul():
    wait_operands()
    mul_low(VA, VB, VT)
    copy8(VA, VT)
    bv_epilogue()


@handler("NOT")
def h_not():
    wait_operands()
    for i in range(8):
        A(f"v_not_b32 {v(VA + i)}, {v(VA + i)}")
    bv_epilogue()


@handler("NEG")
def h_neg():
    wait_operands()
    A(f"v_sub_co_u32 {v(VA)}, vcc, 0, {v(VA)}")
    for i in range(1, 8):
        A(f"v_subb_co_u32 {v(VA + i)}, vcc, 0, {v(VA + i)}, vcc")
    bv_epilogue()


@handler("MOV")
def h_mov():
    wait_operands()
    bv_epilogue()


@handler("SEXT")
def h_sext():
    wait_operands()
    load_kh()
    sext_inplace(VA)
    bv_epilogue()


def maybe_sext_A():
    l = A.fresh("nosx")
    A(f"s_bitcmp1_b32 s18, {B_SEXT}", f"s_cbranch_scc0 {l}")
    load_kh()
    sext_inplace(VA)
    A.label(l)


@handler("SHL")
def h_shl():
    wait_operands()
    amount_from_vB()
    A("v_mov_b32 v26, v6", "v_mov_b32 v27, v4")   # vC is free in BV handlers
    shift_setup(27, left=True)
    shl_var(list(range(VA, VA + 8)), 8)
    A("v_cmp_ne_u32_e64 s[48:49], 0, v26")
    for i in range(8):
        A(f"v_cndmask_b32_e64 {v(VA + i)}, {v(VA + i)}, 0, s[48:49]")
    bv_epilogue()


def h_shr(arith):
    def _():
        wait_operands()
        if arith:
            maybe_sext_A()
        amount_from_vB()
        A("v_mov_b32 v26, v6", "v_mov_b32 v27, v4")
        if arith:
            A(f"v_ashrrev_i32 v28, 31, {v(VA + 7)}")
            fill = "v28"
        else:
            fill = "0"
        shift_setup(27, left=False)
        shr_var(list(range(VA, VA + 8)), fill)
        A("v_cmp_ne_u32_e64 s[48:49], 0, v26")
        for i in range(8):
            A(f"v_cndmask_b32_e64 {v(VA + i)}, {v(VA + i)}, {fill}, s[48:49]")
        bv_epilogue()
    return _


HBODY["LSHR"] = h_shr(False)
HBODY["ASHR"] = h_shr(True)


def uniform_b():
    A(f"s_bfe_u32 s48, s19, {(5 << 16) | U.SHIFT_B_POS:#x}")


def shli_body(k, regs_base=VA):
    """vA <<= 32k + b (b in s48, uniform)."""
    if k >= 8:
        for i in range(8):
            A(f"v_mov_b32 {v(regs_base + i)}, 0")
        return
    lb0, ldone = A.fresh("b0"), A.fresh("shldone")
    A("s_cmp_eq_u32 s48, 0", f"s_cbranch_scc1 {lb0}", "s_sub_u32 s49, 32, s48")
    for i in range(7, -1, -1):
        src = i - k
        if src < 0:
            A(f"v_mov_b32 {v(regs_base + i)}, 0")
        elif src == 0:
            A(f"v_alignbit_b32 {v(regs_base + i)}, {v(regs_base + src)}, 0, s49")
        else:
            A(f"v_alignbit_b32 {v(regs_base + i)}, {v(regs_base + src)}, {v(regs_base + src - 1)}, s49")
    A(f"s_branch {ldone}")
    A.label(lb0)
    for i in range(7, -1, -1):
        src = i - k
        if src < 0:
            A(f"v_mov_b32 {v(regs_base + i)}, 0")
        elif k:
            A(f"v_mov_b32 {v(regs_base + i)}, {v(regs_base + src)}")
    A.label(ldone)


def shri_body(k, fill, src=VA):
    """vA = src >> (32k + b), b in s48 (src = vA, or the bank in GPR-index mode)."""
    for i in range(8):
        lo, hi = i + k, i + k + 1
        if lo >= 8:
            A(f"v_mov_b32 {v(VA + i)}, {fill}")
        else:
            hv = v(src + hi) if hi < 8 else fill
            A(f"v_alignbit_b32 {v(VA + i)}, {hv}, {v(src + lo)}, s48")


def make_shli(k):
    def _():
        wait_operands()
        uniform_b()
        shli_body(k)
        bv_epilogue()
    return _


def make_lshri(k):
    def _():
        wait_operands()
        uniform_b()
        shri_body(k, "0")
        bv_epilogue()
    return _


def make_ashri(k):
    def _():
        wait_operands()
        maybe_sext_A()
        uniform_b()
        A(f"v_ashrrev_i32 v4, 31, {v(VA + 7)}")
        shri_body(k, "v4")
        bv_epilogue()
    return _


def make_concat(k):
    def _():
        wait_operands()
        uniform_b()
        shli_body(k)
        for i in range(8):
            A(f"v_or_b32 {v(VA + i)}, {v(VA + i)}, {v(VB + i)}")
        bv_epilogue()
    return _


for _k in range(9):
    HBODY[f"SHLI{_k}"] = make_shli(_k)
    HBODY[f"LSHRI{_k}"] = make_lshri(_k)
    HBODY[f"ASHRI{_k}"] = make_ashri(_k)
for _k in range(8):
    HBODY[f"CONCAT{_k}"] = make_concat(_k)


@handler("ITE")
def h_ite():
    bool_read("s19", 16, 50)      # SALU only: overlaps the operand wait
    wait_operands()
    for i in range(8):
        A(f"v_cndmask_b32_e64 {v(VA + i)}, {v(VB + i)}, {v(VA + i)}, s[50:51]")
    bv_epilogue()


# ---- compares (result -> vcc -> Bool slot)
def ult_chain(x, y, tmp=VT):
    A(f"v_sub_co_u32 {v(tmp)}, vcc, {v(x)}, {v(y)}")
    for i in range(1, 8):
        A(f"v_subb_co_u32 {v(tmp)}, vcc, {v(x + i)}, {v(y + i)}, vcc")


def slt_chain(x, y):
    A(f"v_xor_b32 v4, 0x80000000, {v(x + 7)}", f"v_xor_b32 v5, 0x80000000, {v(y + 7)}")
    A(f"v_sub_co_u32 {v(VT)}, vcc, {v(x)}, {v(y)}")
    for i in range(1, 7):
        A(f"v_subb_co_u32 {v(VT)}, vcc, {v(x + i)}, {v(y + i)}, vcc")
    A(f"v_subb_co_u32 {v(VT)}, vcc, v4, v5, vcc")


def make_cmp(base, xreg):
    def _():
        wait_operands()
        X, Y = xreg, VB
        if base == "EQ":
            for i in range(8):
                A(f"v_xor_b32 {v(VT + i)}, {v(X + i)}, {v(Y + i)}")
            or_reduce(VT, range(VT, VT + 8))
            A(f"v_cmp_eq_u32 vcc, 0, {v(VT)}")
        elif base in ("ULT", "UGT"):
            x, y = (X, Y) if base == "ULT" else (Y, X)
            ult_chain(x, y)
        elif base in ("SLT", "SGT"):
            lsx, ldone = A.fresh("sx"), A.fresh("cmpdone")
            A(f"s_bitcmp1_b32 s18, {B_SEXT}", f"s_cbranch_scc1 {lsx}")
            x, y = (X, Y) if base == "SLT" else (Y, X)
            slt_chain(x, y)
            A(f"s_branch {ldone}")
            A.label(lsx)
            # X (vA or vC) sign-extended into vC (vA stays the accumulator), Y in place
            load_kh()
            sext_to(VC, X)
            sext_to(VB, Y)
            x, y = (VC, VB) if base == "SLT" else (VB, VC)
            slt_chain(x, y)
            A.label(ldone)
        elif base == "UADDNO256":
            A(f"v_add_co_u32 {v(VT)}, vcc, {v(X)}, {v(Y)}")
            for i in range(1, 8):
                A(f"v_addc_co_u32 {v(VT)}, vcc, {v(X + i)}, {v(Y + i)}, vcc")
        elif base == "UADDNOW":
            load_km()
            A(f"v_add_co_u32 {v(VT)}, vcc, {v(X)}, {v(Y)}")
            for i in range(1, 8):
                A(f"v_addc_co_u32 {v(VT + i)}, vcc, {v(X + i)}, {v(Y + i)}, vcc")
            # raw = M < sum (M copied into vB: operand B is dead once the sum is formed)
            for i in range(8):
                A(f"v_mov_b32 {v(VB + i)}, {s(S_KM + i)}")
            A(f"v_sub_co_u32 v4, vcc, {v(VB)}, {v(VT)}")
            for i in range(1, 8):
                A(f"v_subb_co_u32 v4, vcc, {v(VB + i)}, {v(VT + i)}, vcc")
        elif base in ("UMULNO256", "UMULNOW"):
            if base == "UMULNOW":
                load_km()
            mul_full(X, Y, VT, 7)
            A("v_cmp_ne_u32 vcc, 0, v7")
            if base == "UMULNOW":
                A("s_mov_b64 s[52:53], vcc")
                for i in range(8):
                    A(f"v_mov_b32 {v(VB + i)}, {s(S_KM + i)}")
                A(f"v_sub_co_u32 v4, vcc, {v(VB)}, {v(VT)}")
                for i in range(1, 8):
                    A(f"v_subb_co_u32 v4, vcc, {v(VB + i)}, {v(VT + i)}, vcc")
                A("s_or_b64 vcc, vcc, s[52:53]")
        cmp_epilogue()
    return _


for _c in U.CMPS:
    HBODY[f"{_c}_RA"] = make_cmp(_c, VA)
    HBODY[f"{_c}_RC"] = make_cmp(_c, VC)


def make_eqsel(zk):
    """EQSEL_<zk>: vA = (vC == vB) ? Z : vA, one select-chain step (uop_spec.EQSEL_OPS).  The
    fetch handler brought the compared operands into vC / vB; Z's read (parameter w3[31:16],
    moved to where fetch_one reads operand B) is issued first and lands while the compare
    runs; the selection is one VOP2 cndmask per limb on vcc (a bank operand indexed as
    SRC1, no moves)."""
    def body():
        wait_operands()
        A("s_mov_b32 s17, s19")
        if zk in ("slot", "var"):
            fetch_one(zk, VT, "B")
        elif zk == "const":
            const_issue("B")
        for i in range(8):
            A(f"v_xor_b32 {v(VC + i)}, {v(VC + i)}, {v(VB + i)}")
        or_reduce(VC, range(VC, VC + 8))
        A(f"v_cmp_eq_u32 vcc, 0, {v(VC)}")
        if zk == "slot":
            A("s_waitcnt lgkmcnt(0)")
        elif zk == "var":
            A("s_waitcnt vmcnt(0)")
        elif zk == "const":
            const_finish(VT, "B")
        if zk == "rvar":
            idx_on("B", "SRC1")
            for i in range(8):
                A(f"v_cndmask_b32 {v(VA + i)}, {v(VA + i)}, {v(RV + i)}, vcc")
            A("s_set_gpr_idx_off")
        else:
            for i in range(8):
                A(f"v_cndmask_b32 {v(VA + i)}, {v(VA + i)}, {v(VT + i)}, vcc")
        bv_epilogue()
    return body


for _x in U.EQSEL_OPS:
    HBODY[_x] = make_eqsel(_x[6:])


@handler("TSEL")
def h_tsel():
    """vA = z_i where q == k_i over the uop's table of (k_i, z_i) u32 pairs (uop_spec TSEL;
    keys distinct, so at most one entry matches a lane).  q (vC) matches only where its
    limbs 1-7 are zero (s[50:51]); 8 entries per s_load_dwordx16; an entry's two row loads
    are issued under exec = the lanes whose q equals its key (skipped when none does), so
    the loads of a chain overlap instead of running one per uop."""
    wait_operands()
    lp, ld = A.fresh("tsel"), A.fresh("tseld")
    A("s_and_b32 s55, s19, 0xffff",
      "s_lshr_b32 s54, s19, 16",
      "s_lshl_b32 s54, s54, 3",
      "s_mov_b64 s[48:49], exec")
    or_reduce(4, range(VC + 1, VC + 8))
    A("v_cmp_eq_u32 s[50:51], 0, v4",
      "s_and_b64 s[50:51], s[50:51], exec")
    A.label(lp)
    A("s_load_dwordx16 s[24:39], s[14:15], s54",
      "s_waitcnt lgkmcnt(0)")
    for e in range(8):
        skip = A.fresh("tskip")
        if e:
            A(f"s_cmp_le_u32 s55, {e}", f"s_cbranch_scc1 {ld}")
        A(f"v_cmp_eq_u32 vcc, s{24 + 2 * e}, {v(VC)}",
          "s_and_b64 exec, vcc, s[50:51]",
          f"s_cbranch_execz {skip}")
        tsel_row_load(e)
        A.label(skip)
        A("s_mov_b64 exec, s[48:49]")
    A("s_add_u32 s54, s54, 64",
      "s_sub_u32 s55, s55, 8",
      "s_cmp_gt_i32 s55, 0",
      f"s_cbranch_scc1 {lp}")
    A.label(ld)
    A("s_mov_b64 exec, s[48:49]",
      "s_waitcnt vmcnt(0)")
    bv_epilogue()


def tsel_row_load(e):
    """Entry e's z row (variable index s[25+2e], clamped like fetch_one) into vA under exec."""
    A(f"s_min_u32 s53, s{25 + 2 * e}, s9",
      "s_mul_i32 s53, s53, s8",
      "s_add_u32 s52, s6, s53",
      "s_addc_u32 s53, s7, 0",
      f"global_load_dwordx4 {vr(VA, 4)}, v2, s[52:53]",
      f"global_load_dwordx4 {vr(VA + 4, 4)}, v3, s[52:53]")


@handler("TSELS")
def h_tsels():
    """TSEL with keys in slots (entries (key word, z_i), chain order): q (vC) is compared
    with all 256 bits of each key.  The key of entry e+1 is fetched into the other of two
    buffers (T, vB) while entry e is compared: an LDS key by two ds_reads, a candidate-row
    key (an HBM variable or a spill row, word bit 30) by its two row loads; a bank key is
    read in place when compared.  The waits follow the kinds of the two entries: an LDS key
    waits for lgkmcnt(2) when the next key's reads are behind it, else lgkmcnt(0); a
    candidate-row key waits for vmcnt(2) when the next key's two loads are behind it (the
    row loads of entry e-1, issued before them, land first: loads return in order), else
    vmcnt(0).  Overlapping matches resolve as in the chain: one wave's row loads return in
    issue order, so a lane's last match lands last."""
    wait_operands()
    lp, ld = A.fresh("tsels"), A.fresh("tselsd")
    A("s_and_b32 s55, s19, 0xffff",
      "s_lshr_b32 s54, s19, 16",
      "s_lshl_b32 s54, s54, 3",
      "s_mov_b64 s[48:49], exec")
    A.label(lp)
    A("s_load_dwordx16 s[24:39], s[14:15], s54",
      "s_waitcnt lgkmcnt(0)")
    bufs = (VT, VB)

    def issue(e):
        # a bank key's word has no LDS offset in [15:0]: its read is of slot 0, unused
        lrow, ldone = A.fresh("tsirow"), A.fresh("tsidone")
        A(f"s_bitcmp1_b32 s{24 + 2 * e}, 30", f"s_cbranch_scc1 {lrow}",
          f"s_and_b32 s53, s{24 + 2 * e}, 0xffff",
          "v_add_u32 v4, s53, v1",
          f"ds_read_b128 {vr(bufs[e % 2], 4)}, v4",
          f"ds_read_b128 {vr(bufs[e % 2] + 4, 4)}, v4 offset:1024",
          f"s_branch {ldone}")
        A.label(lrow)
        # candidate-row key: variable w[29:16] (clamped like fetch_one) of this lane's row
        A(f"s_bfe_u32 s53, s{24 + 2 * e}, {(14 << 16) | 16:#x}",
          "s_min_u32 s53, s53, s9",
          "s_mul_i32 s53, s53, s8",
          "s_add_u32 s52, s6, s53",
          "s_addc_u32 s53, s7, 0",
          f"global_load_dwordx4 {vr(bufs[e % 2], 4)}, v2, s[52:53]",
          f"global_load_dwordx4 {vr(bufs[e % 2] + 4, 4)}, v3, s[52:53]")
        A.label(ldone)

    issue(0)
    for e in range(8):
        buf, skip = bufs[e % 2], A.fresh("tsskip")
        lbank, lcmp, lwait = A.fresh("tsbank"), A.fresh("tscmp"), A.fresh("tswait")
        if e:
            A(f"s_cmp_le_u32 s55, {e}", f"s_cbranch_scc1 {ld}")
        if e < 7:
            lnext = A.fresh("tsnrow")
            issue(e + 1)
            A(f"s_bitcmp1_b32 s{24 + 2 * (e + 1)}, 30", f"s_cbranch_scc1 {lnext}",
              "s_waitcnt lgkmcnt(2)",
              f"s_bitcmp1_b32 s{24 + 2 * e}, 30", f"s_cbranch_scc0 {lwait}",
              "s_waitcnt vmcnt(0)",
              f"s_branch {lwait}")
            A.label(lnext)
            A("s_waitcnt lgkmcnt(0)",
              f"s_bitcmp1_b32 s{24 + 2 * e}, 30", f"s_cbranch_scc0 {lwait}",
              "s_waitcnt vmcnt(2)")
            A.label(lwait)
        else:
            A("s_waitcnt vmcnt(0) lgkmcnt(0)")
        A(f"s_bitcmp1_b32 s{24 + 2 * e}, 31", f"s_cbranch_scc1 {lbank}")
        for i in range(8):
            A(f"v_xor_b32 {v(buf + i)}, {v(buf + i)}, {v(VC + i)}")
        A(f"s_branch {lcmp}")
        A.label(lbank)
        # key in register-bank position w[23:16]/8: read as the indexed SRC0
        A(f"s_bfe_u32 s53, s{24 + 2 * e}, {(8 << 16) | 16:#x}",
          "s_set_gpr_idx_on s53, gpr_idx(SRC0)")
        for i in range(8):
            A(f"v_xor_b32 {v(buf + i)}, {v(RV + i)}, {v(VC + i)}")
        A("s_set_gpr_idx_off")
        A.label(lcmp)
        or_reduce(buf, range(buf, buf + 8))
        A(f"v_cmp_eq_u32 vcc, 0, {v(buf)}",
          "s_and_b64 exec, vcc, s[48:49]",
          f"s_cbranch_execz {skip}")
        tsel_row_load(e)
        A.label(skip)
        A("s_mov_b64 exec, s[48:49]")
    A("s_add_u32 s54, s54, 64",
      "s_sub_u32 s55, s55, 8",
      "s_cmp_gt_i32 s55, 0",
      f"s_cbranch_scc1 {lp}")
    A.label(ld)
    A("s_mov_b64 exec, s[48:49]",
      "s_waitcnt vmcnt(0) lgkmcnt(0)")
    bv_epilogue()


# ---- division (Knuth D, 32-bit digits)
# The 16-limb working dividend u is vA (u[0..7]) : vC (u[8..15]); quotient digit J is stored
# into u[J+8].  The normalised divisor is formed in place in vB (the single-digit path keeps
# vB as it is).  f64, qhat and the digit bookkeeping live in T (D_* registers).


def u(i):
    return v(VA + i) if i < 8 else v(VC + i - 8)


def vn(i):
    return v(VB + i)


def knuth_digit(J):
    """One quotient digit of Knuth's algorithm D at window u[J..J+8] (vn normalised).

    qhat = floor(2^32 U3/V3 + 2^-12) in double precision, U3 = u[J+8..J+6] (96 bits),
    V3 = vn7:vn6:vn5 (96 bits, vn7 != 0 after the limb normalisation, so V3 >= 2^64).
    Truncating U and V to those limbs moves U/V by at most 2^32/V3 <= 2^-32, and the
    double evaluation is within 2^-18 of 2^32 U3/V3 (2^32/V3 from v_rcp_f64 + two Newton
    steps), so with the 2^-12 bias qhat is the true digit q or q+1 — never below it.  q+1
    makes the multiply-subtract go negative: one add-back, taken by a wave only when one
    of its lanes sits within 2^-12 of the next integer.
    """
    E, R = vr(D_FB, 2), vr(D_FA, 2)
    A(f"v_cvt_f64_u32 {E}, {u(J + 8)}",
      f"v_cvt_f64_u32 v[4:5], {u(J + 7)}",
      f"v_cvt_f64_u32 v[6:7], {u(J + 6)}",
      f"v_fma_f64 {E}, {E}, s[62:63], v[4:5]",
      f"v_fma_f64 {E}, {E}, s[62:63], v[6:7]",
      f"v_fma_f64 {E}, {E}, {R}, s[28:29]",
      f"v_cvt_u32_f64 {v(D_Q)}, {E}",
      # lanes whose digit J is zero (J > d = top limb(a) - top limb(b), or not dividing;
      # vcc from the caller's skip test) take qhat = 0.  Every lane left has
      # top limb(b) <= 7 - J, so its normalised divisor has vn[i] = 0 for i < J: the
      # products and the subtraction only involve vn[J..7] and u[2J..J+8]
      f"v_cndmask_b32 {v(D_Q)}, 0, {v(D_Q)}, vcc")
    msub_digit(J, VB)


def msub_digit(J, dv):
    """u[2J..J+8] -= qhat (D_Q) * d[J..7] (d = v[dv:dv+8]); one add-back when it goes
    negative (qhat = q + 1), then u[J+8] <- the digit."""
    # u[2J..J+8] -= qhat * vn[J..7]: one multiply-accumulate chain, the high half of each
    # product (+ carry) entering the next as its 64-bit addend (qhat * vn[i] + c < 2^64),
    # interleaved with the borrow chain of the subtraction (VCC).  Per limb: mad + mov +
    # subb, against mad + add + subb with independent products (carry ops issue at half
    # the rate of a mov)
    q, t, m = v(D_Q), v(D_T), vr(D_M, 2)
    A(f"v_mov_b32 {v(D_M + 1)}, 0",
      f"v_mad_u64_u32 v[4:5], s[50:51], {q}, {v(dv + J)}, 0",
      f"v_sub_co_u32 {u(2 * J)}, vcc, {u(2 * J)}, v4")
    for i in range(J + 1, 8):
        A(f"v_mov_b32 {v(D_M)}, v5",
          f"v_mad_u64_u32 v[4:5], s[50:51], {q}, {v(dv + i)}, {m}",
          f"v_subb_co_u32 {u(J + i)}, vcc, {u(J + i)}, v4, vcc")
    A(f"v_subb_co_u32 {u(J + 8)}, vcc, {u(J + 8)}, v5, vcc")
    lno = A.fresh("noaddback")
    A("s_cmp_eq_u64 vcc, 0", f"s_cbranch_scc1 {lno}",
      "s_mov_b64 s[50:51], vcc",
      f"v_subb_co_u32 {q}, s[48:49], {q}, 0, s[50:51]")
    for i in range(J, 8):
        A(f"v_cndmask_b32_e64 {t}, 0, {v(dv + i)}, s[50:51]")
        if i == J:
            A(f"v_add_co_u32 {u(J + i)}, vcc, {t}, {u(J + i)}")
        else:
            A(f"v_addc_co_u32 {u(J + i)}, vcc, {t}, {u(J + i)}, vcc")
    A(f"v_addc_co_u32 {u(J + 8)}, vcc, 0, {u(J + 8)}, vcc")
    A.label(lno)
    A(f"v_mov_b32 {u(J + 8)}, {q}")


def single_digit():
    """Quotient of a wave whose dividing lanes all have q = floor(a / b) < 2^32: one digit
    against the unnormalised divisor.

    qhat = trunc(a_f * (1 / b_f) + 2^-12).  a_f, b_f are the 256-bit values in double
    precision by a Horner chain over the limbs (one rounding per step, each relative error
    below 8 * 2^-53); 1 / b_f from v_rcp_f64 + two Newton steps; the product one more
    rounding.  So a_f / b_f is within 2^-48 relative, 2^-16 absolute (q < 2^32), of a / b,
    and with the 2^-12 bias qhat is q or q + 1 (v_cvt_u32_f64 clamps 2^32 to q): at most
    one add-back in msub_digit.  Non-dividing lanes take qhat = 0 (u[0..8] stays a, 0)."""
    FA, FB = vr(D_FA, 2), vr(D_FB, 2)
    A("s_mov_b32 s62, 0", "s_mov_b32 s63, 0x41f00000",      # 2^32
      "s_mov_b32 s28, 0", "s_mov_b32 s29, 0x3f300000",      # 2^-12 (qhat bias)
      f"v_cvt_f64_u32 {FA}, {u(7)}",
      f"v_cvt_f64_u32 {FB}, {v(VB + 7)}")
    for i in range(6, -1, -1):
        A(f"v_cvt_f64_u32 v[4:5], {u(i)}",
          f"v_cvt_f64_u32 v[6:7], {v(VB + i)}",
          f"v_fma_f64 {FA}, {FA}, s[62:63], v[4:5]",
          f"v_fma_f64 {FB}, {FB}, s[62:63], v[6:7]")
    A(f"v_rcp_f64 v[6:7], {FB}",
      "s_nop 1",
      f"v_fma_f64 v[4:5], -{FB}, v[6:7], 1.0",
      "v_fma_f64 v[6:7], v[6:7], v[4:5], v[6:7]",
      f"v_fma_f64 v[4:5], -{FB}, v[6:7], 1.0",
      "v_fma_f64 v[6:7], v[6:7], v[4:5], v[6:7]",
      f"v_fma_f64 v[4:5], {FA}, v[6:7], s[28:29]",
      f"v_cvt_u32_f64 {v(D_Q)}, v[4:5]",
      f"v_cndmask_b32_e64 {v(D_Q)}, 0, {v(D_Q)}, s[24:25]")
    msub_digit(0, VB)


@handler("DIV")
def h_div():
    wait_operands()
    maybe_sext_op = A.fresh("nosxd")
    A(f"s_bitcmp1_b32 s18, {B_SEXT}", f"s_cbranch_scc0 {maybe_sext_op}")
    load_kh()
    sext_inplace(VA)
    sext_inplace(VB)
    A.label(maybe_sext_op)
    lus, lsd = A.fresh("udiv"), A.fresh("sdone")
    # operand signs as lane masks D_SA / D_SB (s[32:35]: the sign constant is no longer needed)
    A(f"s_bfe_u32 s61, s18, {(3 << 16) | U.DIVOP_POS:#x}",
      "s_cmp_lt_u32 s61, 2", f"s_cbranch_scc1 {lus}",
      f"v_cmp_gt_i32_e64 {D_SA}, 0, {v(VA + 7)}",
      f"v_cmp_gt_i32_e64 {D_SB}, 0, {v(VB + 7)}")
    cneg(VA, D_SA)
    cneg(VB, D_SB)
    A(f"s_branch {lsd}")
    A.label(lus)
    A(f"s_mov_b64 {D_SA}, 0", f"s_mov_b64 {D_SB}, 0")
    A.label(lsd)
    # divides = b != 0 && a >= b, first: a wave where no lane divides skips everything else
    or_reduce(D_T, range(VB, VB + 8))
    A(f"v_cmp_ne_u32_e64 s[26:27], 0, {v(D_T)}")       # bnz
    ult_chain(VA, VB, tmp=D_T)
    A("s_andn2_b64 s[24:25], s[26:27], vcc")
    lpost = A.fresh("divpost")
    # u[0..7] = vA = a: the remainder of a lane that does not divide (its shift is 0 and
    # every digit of it is forced to 0, so u[0..7] stays a)
    A("s_cmp_eq_u64 s[24:25], 0", f"s_cbranch_scc1 {lpost}")
    for i in range(8, 16):
        A(f"v_mov_b32 {u(i)}, 0")
    # single-digit waves: q < 2^32, i.e. (a >> 32) < b, on every dividing lane (one borrow
    # chain; the top-limb bookkeeping of the general path is skipped).  Covers every wave
    # whose dividing lanes have top limb(a) = top limb(b) (47 % of the executed DIVs on the
    # synthetic batch) and more
    lmulti, lnorem = A.fresh("multidig"), A.fresh("norem")
    A(f"v_sub_co_u32 {v(D_T)}, vcc, {v(VA + 1)}, {v(VB)}")
    for i in range(1, 7):
        A(f"v_subb_co_u32 {v(D_T)}, vcc, {v(VA + i + 1)}, {v(VB + i)}, vcc")
    A(f"v_subb_co_u32 {v(D_T)}, vcc, 0, {v(VB + 7)}, vcc",
      "s_andn2_b64 s[48:49], s[24:25], vcc", "s_cmp_eq_u64 s[48:49], 0", f"s_cbranch_scc0 {lmulti}")
    single_digit()
    A(f"s_branch {lnorem}")
    A.label(lmulti)
    # d = top limb(a) - top limb(b) (-1 when not dividing): digits J > d are zero
    K, D = v(D_K), v(D_D)
    top_limb(VB, D_K)
    top_limb(VA, D_D)
    A(f"v_sub_u32 {D}, {D}, {K}",
      f"v_cndmask_b32_e64 {D}, -1, {D}, s[24:25]",
      f"v_sub_u32 {K}, 7, {K}",                        # k = 7 - top limb(b) limbs
      f"v_cndmask_b32_e64 {K}, 0, {K}, s[24:25]")
    # limb normalisation in place: vn = b << 32k, u = a << 32k (vn7 != 0 on dividing lanes;
    # no bit shift is needed because qhat is estimated from the top three limbs of vn)
    limb_masks(D_K)
    shl_limbs(list(range(VB, VB + 8)), 8)
    shl_limbs([VA + i for i in range(8)] + [VC + i for i in range(8)], 8)
    # 2^32 / V3, V3 = vn7*2^64 + vn6*2^32 + vn5, in double precision (rcp + two Newton steps)
    E, R = vr(D_FB, 2), vr(D_FA, 2)
    A("s_mov_b32 s62, 0", "s_mov_b32 s63, 0x41f00000",      # 2^32
      "s_mov_b32 s28, 0", "s_mov_b32 s29, 0x3f300000",      # 2^-12 (qhat bias)
      f"v_cvt_f64_u32 {E}, {vn(7)}",
      f"v_cvt_f64_u32 v[4:5], {vn(6)}",
      f"v_cvt_f64_u32 v[6:7], {vn(5)}",
      f"v_fma_f64 {E}, {E}, s[62:63], v[4:5]",
      "v_mov_b32 v4, 0", "v_mov_b32 v5, 0x3df00000",         # 2^-32
      f"v_fma_f64 {E}, v[6:7], v[4:5], {E}",               # V3 / 2^32
      f"v_rcp_f64 {R}, {E}",
      "s_nop 1",
      f"v_fma_f64 v[4:5], -{E}, {R}, 1.0",
      f"v_fma_f64 {R}, {R}, v[4:5], {R}",
      f"v_fma_f64 v[4:5], -{E}, {R}, 1.0",
      f"v_fma_f64 {R}, {R}, v[4:5], {R}")
    for J in range(7, -1, -1):
        lskip = A.fresh(f"skipdig{J}")
        A(f"v_cmp_le_i32 vcc, {J}, {D}",
          "s_cmp_eq_u64 vcc, 0", f"s_cbranch_scc1 {lskip}")
        knuth_digit(J)
        A.label(lskip)
    # remainder = u[0..7] >> 32k (only UREM/SREM/SMOD need it); SMOD also needs |b| back
    # from the normalised divisor
    lnob = A.fresh("nob")
    A("s_cmp_eq_u32 s61, 0", f"s_cbranch_scc1 {lnorem}",
      "s_cmp_eq_u32 s61, 2", f"s_cbranch_scc1 {lnorem}")
    limb_masks(D_K)
    shr_limbs(list(range(VA, VA + 8)))
    A("s_cmp_lg_u32 s61, 4", f"s_cbranch_scc1 {lnob}")
    shr_limbs(list(range(VB, VB + 8)))
    A.label(lnob)
    A.label(lnorem)
    A.label(lpost)
    # per lane: dividing -> (q = u[8..15], r = u[0..7]); else q = (b == 0 ? ~0 : 0), r = u[0..7] = a
    A(f"v_cndmask_b32_e64 {v(D_T)}, -1, 0, s[26:27]")
    for i in range(8):
        A(f"v_cndmask_b32_e64 {u(8 + i)}, {v(D_T)}, {u(8 + i)}, s[24:25]")
    # result by variant: 0 UDIV, 1 UREM, 2 SDIV, 3 SREM, 4 SMOD (the remainder is vA already)
    l_sd, l_sr, l_end = A.fresh("sdiv"), A.fresh("srem"), A.fresh("divend")
    A("s_cmp_eq_u32 s61, 1", f"s_cbranch_scc1 {l_end}",
      "s_cmp_eq_u32 s61, 2", f"s_cbranch_scc1 {l_sd}",
      "s_cmp_eq_u32 s61, 3", f"s_cbranch_scc1 {l_sr}",
      "s_cmp_eq_u32 s61, 4", f"s_cbranch_scc1 {l_end}_smod")
    copy8(VA, VC)                                     # UDIV
    A(f"s_branch {l_end}")
    A.label(l_sd)
    copy8(VA, VC)
    A(f"s_xor_b64 {D_SA}, {D_SA}, {D_SB}")
    cneg(VA, D_SA)
    A(f"s_branch {l_end}")
    A.label(l_sr)
    cneg(VA, D_SA)
    A(f"s_branch {l_end}")
    A.label(f"{l_end}_smod")
    # r = |a| mod |b| in vA, |b| in vB; the sign follows the divisor (candidates in vC)
    or_reduce(D_T, range(VA, VA + 8))
    A(f"v_cmp_ne_u32_e64 s[48:49], 0, {v(D_T)}",       # r != 0
      f"s_and_b64 s[50:51], {D_SA}, s[48:49]",         # sa
      f"s_and_b64 s[52:53], {D_SB}, s[48:49]",         # sb
      "s_andn2_b64 s[54:55], s[50:51], s[52:53]",       # sa & !sb & r != 0 -> |b| - r
      "s_andn2_b64 s[48:49], s[52:53], s[50:51]",       # !sa & sb & r != 0 -> r - |b|
      "s_and_b64 s[50:51], s[50:51], s[52:53]")         # sa & sb & r != 0 -> -r
    A(f"v_sub_co_u32 {v(VC)}, vcc, {v(VB)}, {v(VA)}")
    for i in range(1, 8):
        A(f"v_subb_co_u32 {v(VC + i)}, vcc, {v(VB + i)}, {v(VA + i)}, vcc")
    A(f"v_sub_co_u32 {v(VT)}, vcc, {v(VA)}, {v(VB)}")
    for i in range(1, 8):
        A(f"v_subb_co_u32 {v(VT + i)}, vcc, {v(VA + i)}, {v(VB + i)}, vcc")
    A(f"v_sub_co_u32 {v(VB)}, vcc, 0, {v(VA)}")       # -r (|b| is no longer needed)
    for i in range(1, 8):
        A(f"v_subb_co_u32 {v(VB + i)}, vcc, 0, {v(VA + i)}, vcc")
    for i in range(8):
        A(f"v_cndmask_b32_e64 {v(VA + i)}, {v(VA + i)}, {v(VC + i)}, s[54:55]",
          f"v_cndmask_b32_e64 {v(VA + i)}, {v(VA + i)}, {v(VT + i)}, s[48:49]",
          f"v_cndmask_b32_e64 {v(VA + i)}, {v(VA + i)}, {v(VB + i)}, s[50:51]")
    A.label(l_end)
    bv_epilogue()


def make_epi_variant(body, mode):
    def _():
        EPI_MODE[0] = mode
        try:
            body()
        finally:
            EPI_MODE[0] = None
    return _


_EPI_BASE = {_op: HBODY[_op] for _op in U.EPI_OPS}
for _name in U.EPI_VARIANTS:
    _op, _mode = _name.rsplit("_", 1)
    HBODY[_name] = make_epi_variant(_EPI_BASE[_op], _mode)
# the translator only names the base handler of these ops when neither flag is set
for _op in U.EPI_OPS:
    HBODY[_op] = make_epi_variant(_EPI_BASE[_op], "")
for _x in U.XS_OPS:
    HBODY[_x] = make_xs(_x)
for _x in U.XC_OPS:
    HBODY[_x] = make_xc(_x)
for _x in U.XV_OPS:
    HBODY[_x] = make_xv(_x)


# ---------------------------------------------------------------- kernel

PROLOGUE = """\
  s_memtime s[96:97]
  s_load_dwordx8 s[64:71], s[0:1], 0x0
  s_load_dwordx8 s[72:79], s[0:1], 0x20
  s_waitcnt lgkmcnt(0)
  // s[64:65] desc  s[66:67] cands  s[68:69] partial  s[70:71] diag
  // s72 n_states  s73 n_cand  s74 n_vars  s75 n_chunks  s76 n_slots  s77 position base  s78 grid x
  // s79 chunks per wave: this wave runs chunks [s3, s80) of its state one after the other
  // (RET restarts the program on the next chunk), s3 = workgroup y * chunks per wave
  s_max_u32 s79, s79, 1
  s_mul_i32 s3, s3, s79
  s_add_u32 s80, s3, s79
  s_min_u32 s80, s80, s75
  // diagnostic stamps (diag != 0): v126 lanes 0-1 diag, 2-3 entry time, 4-5 first
  // dispatch time, 6 item index; written at RET as 16 B per (state, chunk) item
  v_writelane_b32 v126, s70, 0
  v_writelane_b32 v126, s71, 1
  v_writelane_b32 v126, s96, 2
  v_writelane_b32 v126, s97, 3
  // XCD-aware bijective remap of workgroup x (cdna_hip_programming.md §5 T1)
  s_and_b32 s82, s2, 7
  s_lshr_b32 s83, s78, 3
  s_and_b32 s84, s78, 7
  s_add_u32 s85, s83, 1
  s_mul_i32 s86, s82, s85
  s_mul_i32 s87, s84, s85
  s_sub_u32 s88, s82, s84
  s_mul_i32 s88, s88, s83
  s_add_u32 s87, s87, s88
  s_cmp_lt_u32 s82, s84
  s_cselect_b32 s86, s86, s87
  s_lshr_b32 s81, s2, 3
  s_add_u32 s81, s81, s86
  s_add_u32 s81, s81, s77
  s_cmp_ge_u32 s81, s72
  s_cbranch_scc1 .Lexit
  // launch descriptor of this position (mgp_desc_kernel): 32 B.  glc: the descriptors
  // were written by the kernel just before this one on the stream, into a buffer that a
  // previous launch may have read at the same address, and the scalar cache is not
  // guaranteed to be invalidated between two kernels of one stream - read them from L2
  s_lshl_b32 s82, s81, 5
  s_lshr_b32 s83, s81, 27
  s_add_u32 s82, s64, s82
  s_addc_u32 s83, s65, s83
  s_load_dwordx8 s[84:91], s[82:83], 0x0 glc
  s_waitcnt lgkmcnt(0)
  s_cmp_eq_u64 s[70:71], 0
  s_cbranch_scc1 .Lnostampd
  s_memtime s[96:97]
  s_waitcnt lgkmcnt(0)
  v_writelane_b32 v126, s96, 7
.Lnostampd:
  // s84 state  s85 undecided  s86 slots  s87 n_uops  s[88:89] page 0  s90 pool offset from
  // page 0  s91 n_pool | register-variable mask << 8
  // partial entry: partial + (state * n_chunks + chunk) * 4
  s_mul_i32 s82, s84, s75
  s_add_u32 s82, s82, s3
  v_writelane_b32 v126, s82, 6
  s_mul_hi_u32 s83, s82, 4
  s_lshl_b32 s82, s82, 2
  s_add_u32 s58, s68, s82
  s_addc_u32 s59, s69, s83
  // loop state for RET: s22 chunk, s23 end chunk, s20 diag != 0; the SGPRs above s63
  // become Bool slots, so v126 keeps lanes 11-12 page 0, 13 n_uops, 14 n_pool |
  // variable mask << 8, 15 n_cand
  s_mov_b32 s22, s3
  s_mov_b32 s23, s80
  s_or_b32 s20, s70, s71
  v_writelane_b32 v126, s88, 11
  v_writelane_b32 v126, s89, 12
  v_writelane_b32 v126, s87, 13
  v_writelane_b32 v126, s91, 14
  v_writelane_b32 v126, s73, 15
  s_cmp_lg_u32 s85, 0
  s_cbranch_scc1 .Lundec
  s_cmp_gt_u32 s86, s76
  s_cbranch_scc1 .Lundec
  s_mov_b64 s[4:5], s[88:89]
  s_add_u32 s14, s88, s90
  s_addc_u32 s15, s89, 0
  s_mov_b32 s2, s87
{POOL_PREFETCH}  // candidates of this state: cands + state * n_vars * n_cand * 32, layout [var][half][cand] x 16 B
  s_lshl_b32 s8, s73, 5
  s_mul_i32 s92, s74, s8
  s_mul_i32 s6, s84, s92
  s_mul_hi_u32 s7, s84, s92
  s_add_u32 s6, s66, s6
  s_addc_u32 s7, s67, s7
  s_sub_u32 s9, s74, 1
  // lanes: candidate = chunk*64 + lane (clamped; lanes past n_cand are masked out of the result)
  s_lshl_b32 s60, s3, 6
  v_add_u32 v5, s60, v0
  v_cmp_gt_u32_e64 s[56:57], s73, v5
  s_sub_u32 s92, s73, 1
  v_min_u32 v5, s92, v5
  v_lshlrev_b32 v2, 4, v5
  s_lshl_b32 s92, s73, 4
  v_add_u32 v3, s92, v2
  v_lshlrev_b32 v1, 4, v0
  // uop page 0 -> v[112:115] (lane k = uop min(k, n_uops): lanes past the end hold the INVALID pad)
  v_min_u32 v4, s2, v0
  v_lshlrev_b32 v4, 4, v4
  global_load_dwordx4 v[112:115], v4, s[4:5]
  // preload variables 0..min(n_vars, 6)-1 of this lane's candidate into the register bank
  // s[10:11] = kernel entry address: uops hold handler offsets / 4 from it.  Handler
  // addresses are formed as 32-bit sums: a code object crossing a 4 GiB boundary (never
  // seen; would need the loader to place it there) makes every wave report undecided.
  s_getpc_b64 s[10:11]
.Lpc_base:
  s_sub_u32 s10, s10, .Lpc_base-mgp_eval_gfx950
  s_subb_u32 s11, s11, 0
  s_add_u32 s92, s10, .Lfunc_end-mgp_eval_gfx950
  s_cbranch_scc1 .Lundec
  s_mov_b32 s1, s11
  s_mov_b32 s13, s11
{VAR_PRELOAD}  s_cmp_eq_u64 s[70:71], 0
  s_cbranch_scc1 .Lnostampl
  s_memtime s[96:97]
  s_waitcnt lgkmcnt(0)
  v_writelane_b32 v126, s96, 8
.Lnostampl:
{PAGE_DECODE}  s_cmp_eq_u64 s[70:71], 0
  s_cbranch_scc1 .Lnostampx
  s_memtime s[96:97]
  s_waitcnt lgkmcnt(0)
  v_writelane_b32 v126, s96, 4
.Lnostampx:
  s_mov_b64 s[64:65], 0
  s_mov_b64 s[66:67], -1
  s_mov_b32 s62, 0
  s_mov_b32 s63, 0x41f00000
  s_mov_b32 s3, 0
{FIRST_DISPATCH}
.Lundec:
  // -2 into the partial entries of chunks [s3, s80): lane i writes chunk s3 + i
  s_sub_u32 s48, s80, s3
  v_cmp_gt_u32_e64 vcc, s48, v0
  s_mov_b64 exec, vcc
  v_mov_b32 v4, -2
  v_lshlrev_b32 v5, 2, v0
  global_store_dword v5, v4, s[58:59]
.Lexit:
  s_endpgm
"""

KARGS = [("desc", 8, "global_buffer"), ("cands", 8, "global_buffer"), ("partial", 8, "global_buffer"),
         ("diag", 8, "global_buffer"), ("n_states", 4, "by_value"), ("n_cand", 4, "by_value"),
         ("n_vars", 4, "by_value"), ("n_chunks", 4, "by_value"), ("n_slots", 4, "by_value"),
         ("pos_base", 4, "by_value"), ("grid_x", 4, "by_value"), ("chunks_per_wave", 4, "by_value")]


def metadata():
    out = ["amdhsa.kernels:"]
    for kname, nv in ((KNAME, NVGPR),):
        out.append("  - .args:")
        off = 0
        for name, size, kind in KARGS:
            out.append(f"      - .name: {name}")
            if kind == "global_buffer":
                out.append("        .address_space: global")
            out += [f"        .offset: {off}", f"        .size: {size}", f"        .value_kind: {kind}"]
            off += size
        ksize = (off + 7) // 8 * 8
        out += [
            "    .group_segment_fixed_size: 0",
            "    .kernarg_segment_align: 8",
            f"    .kernarg_segment_size: {ksize}",
            "    .max_flat_workgroup_size: 64",
            f"    .name: {kname}",
            "    .private_segment_fixed_size: 0",
            "    .sgpr_count: 104",
            f"    .symbol: {kname}.kd",
            f"    .vgpr_count: {nv}",
            "    .wavefront_size: 64",
        ]
    out += ["amdhsa.target: amdgcn-amd-amdhsa--gfx950", "amdhsa.version:", "  - 1", "  - 2"]
    return "\n".join(out), ksize


def pool_prefetch(tag: str) -> list:
    """The first POOL_PREFETCH_LINES 64-B lines of the pool (within n_pool = s91 & 0xff) into
    the scalar cache: s_load_dwordx16 into s[24:39], results discarded (those SGPRs are free
    until the first uop); var_preload's wait includes them."""
    if not POOL_PREFETCH_LINES:
        return []
    pf = ["  s_and_b32 s93, s91, 0xff"]
    for i in range(POOL_PREFETCH_LINES):
        pf += [f"  s_cmp_le_u32 s93, {2 * i}", f"  s_cbranch_scc1 .Lpoolpf_end{tag}",
               f"  s_load_dwordx16 s[24:39], s[14:15], {64 * i:#x}"]
    pf.append(f".Lpoolpf_end{tag}:")
    return pf


def var_preload(tag: str = "") -> str:
    """Variables v < REG_VARS the program reads (mask bit 8+v of s91) -> v[64+8v : 72+8v]
    (index clamped to n_vars-1); the others are never read and not loaded."""
    out = []
    for i in range(U.REG_VARS):
        r = RV + 8 * i
        out += [f"  s_bitcmp1_b32 s91, {8 + i}", f"  s_cbranch_scc0 .Lnovar{tag}{i}",
                f"  s_min_u32 s94, s9, {i}", "  s_mul_i32 s94, s94, s8",
                "  s_add_u32 s92, s6, s94", "  s_addc_u32 s93, s7, 0",
                f"  global_load_dwordx4 v[{r}:{r + 3}], v2, s[92:93]",
                f"  global_load_dwordx4 v[{r + 4}:{r + 7}], v3, s[92:93]",
                f".Lnovar{tag}{i}:"]
    # page, pool and variables all present before the first uop (the variable loads were
    # issued right behind the page and pool, so this adds little over waiting for those);
    # in the prologue also the pool prefetch (scalar loads)
    pf = POOL_PREFETCH_LINES and (tag == "" or POOL_PREFETCH_CHUNK)
    out.append("  s_waitcnt vmcnt(0)" + (" lgkmcnt(0)" if pf else ""))
    return "\n".join(out) + "\n"


def generate() -> str:
    body = Asm()
    global A
    A = body
    first = Asm()
    global_A = A
    globals()["A"] = first
    A(f"v_readlane_b32 s0, {v(PG)}, s3")
    first_fields()
    tail()
    globals()["A"] = global_A
    dec = Asm()
    globals()["A"] = dec
    page_decode()
    globals()["A"] = global_A
    pf = pool_prefetch("")
    pro = (PROLOGUE.replace("{POOL_PREFETCH}", "\n".join(pf) + ("\n" if pf else "")).replace("v126", v(VD)).replace("v[112:115]", vr(PG, 4))
           .replace("{VAR_PRELOAD}", var_preload()).replace("{FIRST_DISPATCH}", "\n".join(first.lines))
           .replace("{PAGE_DECODE}", "\n".join(dec.lines) + "\n"))
    A.lines.append(pro)
    no_prefetch = set(U.FETCH) | set(U.XS_OPS) | set(U.XC_OPS) | set(U.XV_OPS) | {"INVALID", "RET", "PAGE"}
    wait = "  s_waitcnt lgkmcnt(0)"
    for name in U.HANDLERS:
        # two entries per handler: mgp_h_<name> (reached from a fetch handler, whose
        # operand loads are still in flight) and mgp_hd_<name> (dispatched directly: its
        # operands are resident, so the leading operand wait is skipped).  An op handler
        # that waits for operands is laid out [wait][prefetch][body]: the direct entry
        # sits right behind the wait, 4 bytes in.
        body = Asm()
        body.n = A.n
        globals()["A"] = body
        HBODY[name]()
        body.flush_ool()
        globals()["A"] = global_A
        A.n = body.n
        lines = body.lines
        used = {f for f in (18, 19) if any(re.search(rf"\bs{f}\b|\bs\[{f}:|\bs\[\d+:{f}\]", l) for l in lines)}
        A.lines.append(f".p2align {HALIGN}\nmgp_h_{name}:")
        if name not in no_prefetch and lines and lines[0] == wait:
            A.lines.append(wait)
            lines = lines[1:]
        A.lines.append(f"mgp_hd_{name}:")
        read_fields(used)
        if name not in no_prefetch:
            prefetch_next()
        A.lines.extend(lines)
    md, ksize = metadata()
    head = [
        '.amdgcn_target "amdgcn-amd-amdhsa--gfx950"',
        ".text",
        f".globl {KNAME}",
        ".p2align 8",
        f".type {KNAME},@function",
        f"{KNAME}:",
    ]
    def kd(kname, nv):
        return [
            ".rodata",
            ".p2align 6",
            f".amdhsa_kernel {kname}",
            "  .amdhsa_group_segment_fixed_size 0",
            "  .amdhsa_private_segment_fixed_size 0",
            f"  .amdhsa_kernarg_size {ksize}",
            "  .amdhsa_user_sgpr_count 2",
            "  .amdhsa_user_sgpr_kernarg_segment_ptr 1",
            "  .amdhsa_system_sgpr_workgroup_id_x 1",
            "  .amdhsa_system_sgpr_workgroup_id_y 1",
            "  .amdhsa_system_vgpr_workitem_id 0",
            f"  .amdhsa_next_free_vgpr {nv}",
            "  .amdhsa_next_free_sgpr 102",
            f"  .amdhsa_accum_offset {nv}",
            "  .amdhsa_reserve_vcc 1",
            "  .amdhsa_float_denorm_mode_32 3",
            "  .amdhsa_float_denorm_mode_16_64 3",
            ".end_amdhsa_kernel",
            "",
        ]
    tail_ = [
        ".Lfunc_end:",
        f".size {KNAME}, .Lfunc_end-{KNAME}",
        "",
    ] + kd(KNAME, NVGPR) + [
        ".amdgpu_metadata",
        "---",
        md,
        "...",
        ".end_amdgpu_metadata",
    ]
    return "\n".join(head + A.lines + tail_) + "\n"


def main():
    out_s, out_h = sys.argv[1], sys.argv[2]
    src = generate()
    with open(out_s, "w") as f:
        f.write(f"// generated by gen_eval_asm.py — do not edit\n{src}")
    with open(out_h, "w") as f:
        f.write(U.c_header())


if __name__ == "__main__":
    main()
