"""Micro-op ("uop") encoding of the gfx950 assembly interpreter — single source of truth.

The host translator (csrc/mgp_uop.cpp, via the generated header mgp_uop.h), the
assembly generator (csrc/gen_eval_asm.py) and the CPU reference interpreter of
the encoding (oracle/uop_ref.py, test infrastructure) all read this table.

Program layout (per state, appended after the v1 bytecode of include/mgp_ir.h,
at word offset align4(4 + 4*n_ins + 8*n_consts) + 4 from the program start):

  header   4 words: n_uops, status (0 = runnable), pool byte offset (from the
           uop header), n_pool | register-variable mask << 8 (bit v: the program
           reads variable v < REG_VARS, which the kernel preloads into VGPRs)
           | LDS slots << 16 (BV slots left in LDS after register slots)
  uops     n_uops x 4 words in pages of 64: uop 63 of every full page is PAGE
           (the kernel holds one page in 4 VGPRs, uop k in lane k, and reads
           the current uop with v_readlane; PAGE loads the next page), then one
           all-zero uop
  pool     n_pool <= 255 constants, 8 little-endian u32 limbs each: the width masks
           2^w-1 and sign constants 2^(w-1) the uops use first (their index fields
           are 6 bits), then the v1 pool; handlers read an entry with one scalar load
  tables   the TSEL tables: (key, variable index) u32 pairs, 8-entry blocks (scalar
           loads of 64 B), identical tables stored once

uop words:
  w0 [15:0]  entry offset / 4 (from the kernel entry) of the FIRST handler: a fetch
             handler for BV/compare uops, the op handler otherwise
     [31:16] entry offset / 4 of the op handler (fetch handlers jump to it)
             (offsets come from the assembled kernel's symbol table, gen_offsets.py)
  w1 [15:0] operand A parameter, [31:16] operand B parameter
            SLOT: LDS byte offset (slot*2048), VAR: variable index (a spilled
            BV slot is the VAR row the state's VST uops write, mgp_ir.h), RVAR:
            8 x register-bank position p (v[42+8p]: a preloaded variable, or a
            register slot),
            CONST: pool index; Bool operands: bool slot * 2
  w2 [15:0] store slot byte offset, or 8 x bank position with REGST /
            third Bool operand * 2;  BAND4: [31:16] fourth Bool operand * 2
     [21:16] mask pool index
     [22] STORE   result -> LDS slot
     [23] MASK    result &= pool[mask] (2^w - 1); compares: M for the overflow tests
     [24] SEXT    operands sign-extended from width w with H = pool[w3[5:0]]
     [25] INVERT  compare result negated
     [28:26]      division variant (DIV_*)
     [29] REGST   the STORE goes to register-bank position w2[15:0]/8 (v[42+8p]),
                  not to LDS: the translator maps a state's highest BV slots onto
                  bank positions no variable of that state uses
     [30] BCOMB   compares: the (possibly inverted) result is combined with Bool slot
                  w3[15:8]/2 before it is written: AND, or OR with [31] BCOMB_OR
  BANDN: dst = a & ~b (a = w1[15:0], b = w1[31:16])
  VST: w2 [15:0] candidate variable row the lane's vA is stored to (a spill slot)
  w3 [5:0]  sign-constant pool index, [12:8] uniform shift bits (SHLI/LSHRI/ASHRI/CONCAT),
     [15:8] compares with BCOMB: the other Bool operand * 2,
     [31:16] Bool destination * 2 (compares, Bool ops) or ITE condition * 2, or the
             EQSEL_<kind> select operand's parameter

Registers of the interpreter: vA (accumulator / operand A), vB (operand B),
vC (operand A of a compare that is not the accumulator); Bool slots are
64-bit lane masks in SGPRs: slot 0 = false, slot 1 = true, 2.. allocatable.
"""
import os


# operand kinds: acc = the accumulator vA, slot = per-lane LDS slot, var = candidate
# variable loaded from HBM, const = constant pool (scalar load), rvar = candidate
# variable 0..REG_VARS-1 preloaded into the register bank at wave start (GPR-index moves);
# the bank has REG_POS positions of 8 VGPRs (v[42+8p]): positions no preloaded variable uses
# hold BV slots (register slots), so a program needs fewer LDS slots
KINDS = ("acc", "slot", "var", "const", "rvar")
REG_VARS = 6
REG_POS = int(os.environ.get("MGP_REG_POS", "10"))   # build-time knob (A/B of bank size vs occupancy)
B_KINDS = ("none",) + KINDS

# fetch handlers: F_<kindA>_<kindB>_<target of A>; A = acc with target C never occurs
FETCH = [f"F_{ka}_{kb}_A" for ka in KINDS for kb in B_KINDS] + \
        [f"F_{ka}_{kb}_C" for ka in KINDS[1:] for kb in B_KINDS]

# BAND4N<m>: BAND4 with the operands of mask m (bit 0 = first .. bit 3 = fourth) negated (a
# BNOT whose result only one AND chain reads, folded by the translator)
BAND4N = [f"BAND4N{m}" for m in range(1, 16)]
BOOL_OPS = ["PAGE", "RET", "BAND", "BOR", "BXOR", "BNOT", "BITE", "BEQ", "BAND4", "BANDN"] + BAND4N
# vA -> the lane's candidate row w2[15:0] (a spilled BV slot; read back as a VAR operand)
MEM_OPS = ["VST"]
BV_BIN = ["ADD", "SUB", "MUL", "AND", "OR", "XOR", "SHL", "LSHR", "ASHR", "DIV"]
BV_UN = ["NOT", "NEG", "MOV", "SEXT"]
SHIFT_I = [f"SHLI{k}" for k in range(9)] + [f"LSHRI{k}" for k in range(9)] + [f"ASHRI{k}" for k in range(9)]
CONCAT = [f"CONCAT{k}" for k in range(8)]
CMPS = ["EQ", "ULT", "UGT", "SLT", "SGT", "UADDNO256", "UADDNOW", "UMULNO256", "UMULNOW"]
CMP_VARIANTS = [f"{c}_{r}" for c in CMPS for r in ("RA", "RC")]

# epilogue-specialised variants of the cheap BV ops: _S store, _M mask, _MS both (the
# translator picks one from the STORE/MASK flags, so these handlers test no flags)
EPI_OPS = ["ADD", "SUB", "AND", "OR", "XOR", "NOT", "NEG", "MOV", "ITE"]
EPI_VARIANTS = [f"{o}_{v}" for o in EPI_OPS for v in ("S", "M", "MS", "R", "MR")]

# fused handlers "vA = vA op bank[B]" (F_acc_rvar_A + op in one handler: B is read in
# GPR-index mode straight from the register bank, no moves, no second dispatch)
XR_BASE = [f"{o}{v}" for o in ("ADD", "SUB", "AND", "OR", "XOR") for v in ("", "_S", "_R")] + \
          ["EQ_RA", "ULT_RA", "UGT_RA"]   # compares "vA cmp bank[B]" (Bool result)
XR_OPS = [f"XR_{o}" for o in XR_BASE]

# fused handlers "vA = vA op lds[B]" (F_acc_slot_A + op in one handler: the B slot read
# is issued at the top of the op, one dispatch instead of two)
# (the masked variants and DIV stay two-dispatch: rare, or a long body not worth a copy)
XS_BASE = [f"{c}_RA" for c in ("EQ", "ULT", "UGT", "SLT", "SGT")] + ["MUL"] + \
          [f"{o}{v}" for o in ("ADD", "SUB", "AND", "OR", "XOR", "ITE") for v in ("", "_S", "_R")]
XS_OPS = [f"XS_{o}" for o in XS_BASE]

# fused handlers "vA = vA op pool[B]" (F_acc_const_A + op in one handler: the scalar load
# of the constant is issued at the top, the next uop's readlane overlaps it)
XC_BASE = list(XS_BASE)
XC_OPS = [f"XC_{o}" for o in XC_BASE]

# fused handlers "register operands + op": a fetch whose operands are all registers (the
# accumulator or register-bank positions) and its op in one handler (the bank moves, then
# the op body: no second dispatch).  XV_<kindA>_<kindB>_<target>_<op>; the pairs most
# frequent on the synthetic batch (profiles/uop_mix.py), DIV excluded (a long body)
XV_LIST = [("acc", "rvar", "A", o) for o in ("MUL", "ITE", "ITE_R", "SLT_RA")] + \
          [("rvar", "rvar", "C", o) for o in ("EQ_RC", "ULT_RC", "UGT_RC", "SLT_RC")] + \
          [("rvar", "rvar", "A", o) for o in ("ITE", "ITE_R", "MUL", "ADD", "ADD_R", "SUB", "SUB_R", "AND", "AND_R",
                                              "OR", "OR_R", "XOR", "XOR_R")] + \
          [("acc", "acc", "A", o) for o in ("EQ_RA", "ULT_RA")] + \
          [("rvar", "acc", "A", o) for o in ("SUB", "SUB_R", "ITE", "ITE_R")] + \
          [("rvar", "none", "A", o) for o in ("NOT", "NOT_R") + tuple(f"LSHRI{k}" for k in range(8))]
XV_OPS = [f"XV_{ka}_{kb}_{t}_{o}" for ka, kb, t, o in XV_LIST]

# one step of a select chain (Select over a Store chain, calldata byte tables, lowered as
# `EQ key k_i` + `ITE(that, v_i, acc)`): vA = (vC == vB) ? Z : vA, with the compared
# operands fetched by F_<kx>_<ky>_C and Z (operand kind <zk>, parameter w3[31:16]) read by
# the op handler while the compare runs.  The translator fuses an EQ whose Bool result only
# the next ITE reads (as its condition, the else operand being the accumulator).
EQSEL_OPS = [f"EQSEL_{k}" for k in KINDS[1:]]

# a run of select-chain steps over one key q (fetched into vC by F_<kq>_none_C) against
# 32-bit constants k_i, selecting HBM variables z_i: one TSEL uop over a table of (k_i, z_i)
# u32 pairs behind the pool (w3[15:0] entries, w3[31:16] = the table's byte offset from the
# pool / 8, keys distinct, padded to 8 entries).  vA = z_i where q == k_i (the last i in
# chain order), else vA unchanged; the handler compares q against 8 keys per scalar load
# and issues each z_i row load under the lanes that match it.  TSELS: the same with keys in
# slots (pairs (key word, z_i), chain order kept: a lane's last match wins, as the row loads
# of one wave return in issue order) -- a Store chain at symbolic indices read at one index.
# Key word: an LDS slot's byte offset; bit 31 | 8p << 16: register-bank position p;
# bit 30 | v << 16: candidate-row variable v (an HBM variable or a spill row, loaded by the
# handler) -- WalletLibrary's long-lived symbolic offsets are mostly spilled.
TSELS_KEY_BANK = 1 << 31
TSELS_KEY_ROW = 1 << 30
TSEL_MIN = 3     # shorter runs stay EQSEL uops

OPS = BOOL_OPS + MEM_OPS + BV_BIN + BV_UN + SHIFT_I + CONCAT + ["ITE"] + CMP_VARIANTS + EPI_VARIANTS + XR_OPS + \
    XS_OPS + XC_OPS + XV_OPS + EQSEL_OPS + ["TSEL", "TSELS"]
# handler 0 stops the wave with MGP_UNDECIDED: an all-zero uop (the prefetch pad) or any
# id past the table ends the program instead of running off into memory
HANDLERS = ["INVALID"] + FETCH + OPS
ID = {name: i for i, name in enumerate(HANDLERS)}
assert len(HANDLERS) < 1024   # ids are host-side table indices (uops carry offsets)

DIV_VARIANTS = {"UDIV": 0, "UREM": 1, "SDIV": 2, "SREM": 3, "SMOD": 4}

F_STORE, F_MASK, F_SEXT, F_INVERT = 1 << 22, 1 << 23, 1 << 24, 1 << 25   # in w2
F_REGST = 1 << 29                                                         # in w2
F_BCOMB, F_BCOMB_OR = 1 << 30, 1 << 31                                    # in w2
BCOMB_POS = 8       # in w3
SHIFT_B_POS = 8     # in w3
DIVOP_POS = 26      # in w2

BOOL_SLOTS = 19          # 0 false, 1 true, 2..18 allocatable
MAX_LDS_SLOTS = 31       # LDS slots per wave (62 KiB); more BV slots spill to candidate rows
SLOT_BYTES = 2048        # 64 lanes x 32 B
HDR_WORDS = 4
UOP_WORDS = 4
PAGE_UOPS = 64           # uops per VGPR page (one per lane); the last one is PAGE
MAX_POOL = 255           # constants per state (header byte; scalar loads, no lane limit)
MAX_MS = 64              # mask / sign constants (6-bit index fields)


def c_header() -> str:
    """The C view of this table (written to build/mgp/mgp_uop.h by the generator)."""
    lines = ["/* generated from mythril_amd/uop_spec.py — do not edit */", "#pragma once"]
    for name, i in ID.items():
        lines.append(f"#define MGP_U_{name} {i}")
    for name, v in DIV_VARIANTS.items():
        lines.append(f"#define MGP_DIV_{name} {v}")
    lines += [
        f"#define MGP_UF_STORE {F_STORE}u", f"#define MGP_UF_MASK {F_MASK}u",
        f"#define MGP_UF_SEXT {F_SEXT}u", f"#define MGP_UF_INVERT {F_INVERT}u",
        f"#define MGP_UF_REGST {F_REGST}u", f"#define MGP_UF_BCOMB {F_BCOMB}u",
        f"#define MGP_UF_BCOMB_OR {F_BCOMB_OR}u", f"#define MGP_U_BCOMB_POS {BCOMB_POS}",
        f"#define MGP_U_SHIFT_B_POS {SHIFT_B_POS}", f"#define MGP_U_DIVOP_POS {DIVOP_POS}",
        f"#define MGP_U_BOOL_SLOTS {BOOL_SLOTS}", f"#define MGP_U_MAX_LDS_SLOTS {MAX_LDS_SLOTS}",
        f"#define MGP_U_SLOT_BYTES {SLOT_BYTES}", f"#define MGP_U_HDR_WORDS {HDR_WORDS}",
        f"#define MGP_U_UOP_WORDS {UOP_WORDS}", f"#define MGP_U_REG_VARS {REG_VARS}", f"#define MGP_U_REG_POS {REG_POS}",
        f"#define MGP_U_N_KINDS {len(KINDS)}", f"#define MGP_U_PAGE_UOPS {PAGE_UOPS}",
        f"#define MGP_U_MAX_POOL {MAX_POOL}", f"#define MGP_U_MAX_MS {MAX_MS}", f"#define MGP_U_XR_FIRST {ID[XR_OPS[0]]}",
    ]
    lines.append("static const unsigned short kXrBase[%d] = {%s};" % (len(XR_BASE), ", ".join(
        f"MGP_U_{o}" for o in XR_BASE)))
    lines.append(f"#define MGP_U_BAND4N_FIRST {ID[BAND4N[0]]}")
    lines.append(f"#define MGP_U_XV_FIRST {ID[XV_OPS[0]]}")
    lines.append("static const short kXv[%d][4] = {%s};" % (len(XV_LIST), ", ".join(
        "{%d, %d, %d, MGP_U_%s}" % (KINDS.index(ka), B_KINDS.index(kb) - 1, t == "C", o) for ka, kb, t, o in XV_LIST)))
    lines.append(f"#define MGP_U_XS_FIRST {ID[XS_OPS[0]]}")
    lines.append("static const unsigned short kXsBase[%d] = {%s};" % (len(XS_BASE), ", ".join(
        f"MGP_U_{o}" for o in XS_BASE)))
    lines.append(f"#define MGP_U_EQSEL_FIRST {ID[EQSEL_OPS[0]]}")
    lines.append(f"#define MGP_U_TSEL_MIN {TSEL_MIN}")
    lines.append(f"#define MGP_U_XC_FIRST {ID[XC_OPS[0]]}")
    lines.append("static const unsigned short kXcBase[%d] = {%s};" % (len(XC_BASE), ", ".join(
        f"MGP_U_{o}" for o in XC_BASE)))
    return "\n".join(lines) + "\n"
