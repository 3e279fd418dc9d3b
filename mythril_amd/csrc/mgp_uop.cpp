// mgp_uop.cpp — v1 bytecode -> micro-ops of the gfx950 assembly interpreter.
//
// mgp_lower produces, per state, the v1 program of include/mgp_ir.h (the
// schedule, slot/Bool allocation and accumulator forwarding live there).  This
// pass re-encodes it for mgp_eval_gfx950 (gen_eval_asm.py): one uop per v1
// instruction, with everything the kernel would otherwise decode at run time
// resolved here —
//   * the operand kinds select a fetch handler (F_<kindA>_<kindB>_<target>),
//     so the kernel never branches on operand kinds;
//   * commutative ops / compares are swapped so the accumulator is operand A
//     (a compare never overwrites the accumulator: a non-accumulator A goes to
//     vC);
//   * shifts by a constant become uniform-shift handlers (limb move + one
//     v_alignbit per limb), EXTRACT is LSHRI + mask, CONCAT a fused
//     shift-or;
//   * narrow widths carry explicit MASK / SEXT flags whose constants
//     (2^w - 1, 2^(w-1)) are appended to the state's constant pool;
//   * LDS slot / pool / Bool operands are pre-scaled byte offsets.
// Encoding: mythril_amd/uop_spec.py (mgp_uop.h is generated from it).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>

#include "../../include/mgp_ir.h"
#include "mgp_uop.h"
#include "mgp_uop_off.h"

// handler entry offsets (/4, from the kernel entry) by handler id; exported for the
// CPU reference interpreter of the encoding (oracle/uop_ref.py)
extern "C" const uint16_t *mgp_uop_handler_offsets(uint32_t *n) {
  if (n) *n = MGP_U_N_HANDLERS;
  return kUopHandlerOffset;
}

// the direct-dispatch entries (a uop whose first handler is its op handler)
extern "C" const uint16_t *mgp_uop_direct_offsets(uint32_t *n) {
  if (n) *n = MGP_U_N_HANDLERS;
  return kUopDirectOffset;
}

namespace {

struct Opnd {
  int kind;       // 0 acc, 1 slot, 2 var (HBM), 3 const, 4 rvar (register-resident var), -1 none
  uint32_t param;
};

constexpr int KACC = 0, KSLOT = 1, KVAR = 2, KCONST = 3, KRVAR = 4, KNONE = -1;

// fetch handler ids, in uop_spec.FETCH order: A-target block (K x (K+1)), then
// C-target ((K-1) x (K+1)), K = MGP_U_N_KINDS, B kind "none" first
inline uint32_t fetch_id(int ka, int kb, bool to_c) {
  const int kbi = kb + 1;
  if (!to_c) return (uint32_t)(MGP_U_F_acc_none_A + ka * (MGP_U_N_KINDS + 1) + kbi);
  return (uint32_t)(MGP_U_F_slot_none_C + (ka - 1) * (MGP_U_N_KINDS + 1) + kbi);
}

struct Translator {
  const uint32_t *v1;
  uint32_t n_ins, n_c;
  std::vector<uint32_t> v1pool;      // the v1 constants, 8 words each (by v1 index)
  std::vector<uint32_t> ms;          // mask / sign constants: pool entries 0.. (6-bit index fields)
  uint32_t ms_base = 0;              // pool index of v1 constant 0 (pass 2: the mask/sign count)
  uint32_t var_mask = 0;             // register variables the program reads (preloaded)
  // BV slot map (pass 2): v1 slot -> LDS slot, register-bank position or spill row (KVAR)
  std::vector<Opnd> slot_map;
  uint32_t n_lds = 0;                // LDS slots the program uses
  std::map<uint32_t, uint32_t> mask_c, sign_c;  // width -> pool index
  std::vector<uint32_t> tables;                 // TSEL tables (behind the pool)
  std::map<std::vector<uint32_t>, uint32_t> table_at;  // table -> word offset in `tables`
  bool bad = false;

  // v1 constant operand o with zero limbs above the first: its low limb
  bool small_const(uint32_t o, uint32_t *lo) const {
    const uint32_t *c = &v1pool[(size_t)(o & 0x3FFFu) * 8];
    for (int l = 1; l < 8; ++l)
      if (c[l]) return false;
    *lo = c[0];
    return true;
  }
  // a TSEL / TSELS table, padded to 8-entry blocks; returns its word offset, stored once
  // per distinct table.  Constant keys are made distinct (a key's last entry wins, as in
  // the chain); slot keys are per-lane values and stay in chain order.
  uint32_t add_table(const std::vector<std::pair<uint32_t, uint32_t>> &ent, bool dedupe, uint32_t *n_out) {
    std::vector<uint32_t> t;
    for (size_t i = 0; i < ent.size(); ++i) {
      bool later = false;
      for (size_t j = i + 1; dedupe && j < ent.size() && !later; ++j) later = ent[j].first == ent[i].first;
      if (!later) { t.push_back(ent[i].first); t.push_back(ent[i].second); }
    }
    *n_out = (uint32_t)(t.size() / 2);
    while (t.size() % 16) t.push_back(0u);
    auto it = table_at.find(t);
    if (it != table_at.end()) return it->second;
    const uint32_t off = (uint32_t)tables.size();
    tables.insert(tables.end(), t.begin(), t.end());
    table_at.emplace(std::move(t), off);
    return off;
  }

  uint32_t add_ms(const uint32_t w[8]) {
    const uint32_t idx = (uint32_t)(ms.size() / 8);
    if (idx >= MGP_U_MAX_MS) bad = true;
    ms.insert(ms.end(), w, w + 8);
    return idx;
  }
  uint32_t mask_off(uint32_t width) {
    auto it = mask_c.find(width);
    if (it == mask_c.end()) {
      uint32_t w[8];
      for (int l = 0; l < 8; ++l) {
        const int lo = 32 * l;
        w[l] = (int)width >= lo + 32 ? 0xFFFFFFFFu : ((int)width <= lo ? 0u : ((1u << (width - lo)) - 1u));
      }
      it = mask_c.emplace(width, add_ms(w)).first;
    }
    return it->second;
  }
  uint32_t sign_off(uint32_t width) {
    auto it = sign_c.find(width);
    if (it == sign_c.end()) {
      uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      w[(width - 1) >> 5] = 1u << ((width - 1) & 31);
      it = sign_c.emplace(width, add_ms(w)).first;
    }
    return it->second;
  }
  // pool index of v1 constant idx (the kernel reads entry idx with one scalar load)
  uint32_t pool_idx(uint32_t idx) {
    if (idx + ms_base >= MGP_U_MAX_POOL) bad = true;
    return idx + ms_base;
  }
  Opnd bv(uint32_t o) {
    const uint32_t kind = o >> 14, idx = o & 0x3FFFu;
    switch (kind) {
      case MGP_K_ACC: return {KACC, 0};
      case MGP_K_SLOT:
        if (idx < slot_map.size()) return slot_map[idx];
        return {KSLOT, 0};  // pass 1: only the variable mask and the mask/sign set matter
      case MGP_K_CONST: return {KCONST, pool_idx(idx)};
      default:
        if (idx < MGP_U_REG_VARS) {
          var_mask |= 1u << idx;
          return {KRVAR, idx * 8u};  // RVAR parameter: VGPR offset 8p into the bank
        }
        return {KVAR, idx};
    }
  }
  uint32_t boolslot(uint32_t b) {
    if (b == MGP_BOOL_FALSE) return 0;
    if (b == MGP_BOOL_TRUE) return 2;
    const uint32_t s = b + 2;
    if (s >= MGP_U_BOOL_SLOTS) bad = true;
    return s * 2;
  }
  // value of a v1 constant operand (v1 pool index), low limb + "any high bits"
  void const_value(uint32_t o, uint32_t *lo, bool *big) {
    const uint32_t idx = o & 0x3FFFu;
    const uint32_t *c = &v1pool[(size_t)idx * 8];
    *lo = c[0];
    bool hi = false;
    for (int l = 1; l < 8; ++l) hi |= c[l] != 0;
    *big = hi || c[0] >= 256u;
  }
  // pass 2: where each v1 BV slot lives.  A program within MGP_LDS_SLOTS keeps its highest
  // slots in the register-bank positions no variable uses (register slots) and the rest in
  // LDS; a spilling program (slots numbered by access count, mgp_lower) gives the register
  // positions to its lowest slots, then LDS, then spill rows MGP_SPILL_BASE(max_var) + j.
  void map_slots(uint32_t n_slots, uint32_t max_var) {
    uint32_t free_pos[MGP_U_REG_POS], n_free = 0;
    for (uint32_t p = 0; p < MGP_U_REG_POS; ++p)
      if (p >= MGP_U_REG_VARS || !(var_mask & (1u << p))) free_pos[n_free++] = p;
    const uint32_t k = n_free < n_slots ? n_free : n_slots;
    const uint32_t spill0 = MGP_SPILL_BASE(max_var);
    slot_map.assign(n_slots, Opnd{KSLOT, 0});
    uint32_t n_spill = 0;
    n_lds = 0;
    auto lds_or_spill = [&](uint32_t s, uint32_t l) {
      if (l < MGP_U_MAX_LDS_SLOTS) {
        slot_map[s] = {KSLOT, l * MGP_U_SLOT_BYTES};
        n_lds = std::max(n_lds, l + 1);
      } else {
        slot_map[s] = {KVAR, spill0 + n_spill++};
      }
    };
    if (n_slots <= MGP_LDS_SLOTS) {
      const uint32_t nl = n_slots - k;
      for (uint32_t s = 0; s < nl; ++s) lds_or_spill(s, s);
      for (uint32_t s = nl; s < n_slots; ++s) slot_map[s] = {KRVAR, free_pos[s - nl] * 8u};
    } else {
      for (uint32_t s = 0; s < k; ++s) slot_map[s] = {KRVAR, free_pos[s] * 8u};
      for (uint32_t s = k; s < n_slots; ++s) lds_or_spill(s, s - k);
    }
  }
};

// w0 = entry offsets of the first handler and of the op handler (fetch handlers jump to it)
// cheap BV ops have handler variants with a fixed epilogue (no flag tests at run time)
inline uint32_t epi_variant(uint32_t op, bool store, bool mask, bool reg) {
  if (!store && !mask) return op;
#define MGP_EPI_ROW(o) {MGP_U_##o, MGP_U_##o##_S, MGP_U_##o##_M, MGP_U_##o##_MS, MGP_U_##o##_R, MGP_U_##o##_MR}
  static const uint32_t T[][6] = {MGP_EPI_ROW(ADD), MGP_EPI_ROW(SUB), MGP_EPI_ROW(AND), MGP_EPI_ROW(OR),
                                  MGP_EPI_ROW(XOR), MGP_EPI_ROW(NOT), MGP_EPI_ROW(NEG), MGP_EPI_ROW(MOV),
                                  MGP_EPI_ROW(ITE)};
#undef MGP_EPI_ROW
  for (const auto &e : T)
    if (e[0] == op) {
      if (!store) return e[2];
      if (reg) return mask ? e[5] : e[4];
      return mask ? e[3] : e[1];
    }
  return op;
}

// fused "vA op= bank[B]" handler of an op (uop_spec.XR_OPS), or -1
inline int xr_handler(uint32_t op) {
  for (uint32_t i = 0; i < sizeof(kXrBase) / sizeof(kXrBase[0]); ++i)
    if (kXrBase[i] == op) return (int)(MGP_U_XR_FIRST + i);
  return -1;
}

// fused "vA op= lds[B]" handler of an op (uop_spec.XS_OPS), or -1
inline int xs_handler(uint32_t op) {
  for (uint32_t i = 0; i < sizeof(kXsBase) / sizeof(kXsBase[0]); ++i)
    if (kXsBase[i] == op) return (int)(MGP_U_XS_FIRST + i);
  return -1;
}

// fused "vA op= pool[B]" handler of an op (uop_spec.XC_OPS), or -1
inline int xc_handler(uint32_t op) {
  for (uint32_t i = 0; i < sizeof(kXcBase) / sizeof(kXcBase[0]); ++i)
    if (kXcBase[i] == op) return (int)(MGP_U_XC_FIRST + i);
  return -1;
}

// fused "register operands + op" handler (uop_spec.XV_LIST) of a fetch pattern and op, or -1
inline int xv_handler(int ka, int kb, bool to_c, uint32_t op) {
  for (uint32_t i = 0; i < sizeof(kXv) / sizeof(kXv[0]); ++i)
    if (kXv[i][0] == ka && kXv[i][1] == kb && (kXv[i][2] != 0) == to_c && (uint32_t)kXv[i][3] == op)
      return (int)(MGP_U_XV_FIRST + i);
  return -1;
}
inline bool reg_kind(int k) { return k == KACC || k == KRVAR; }

// ---- Bool peepholes on the v1 instruction list (asm engine only; the v1 program is untouched)
//   * a compare immediately followed by a BNOT of its result: the compare is emitted with
//     its INVERT flag toggled and the BNOT's destination (one dispatch instead of two);
//   * chains of adjacent BANDs whose intermediate result has no other reader: one BAND4
//     (AND of up to four Bool slots).
inline uint32_t v1_op(const uint32_t *I) { return I[0] & 0xFFu; }
inline bool v1_writes_bool(const uint32_t *I, uint32_t bit) {
  const uint32_t op = v1_op(I);
  const bool boolres = (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) || (op >= MGP_OP_BAND && op <= MGP_OP_BEQ);
  return boolres && ((I[0] >> 16) & 0xFFu) == bit;
}
inline bool v1_reads_bool(const uint32_t *I, uint32_t bit) {
  const uint32_t op = v1_op(I), oa = I[1] & 0xFFFFu, ob = I[1] >> 16, oc = I[2] & 0xFFFFu;
  switch (op) {
    case MGP_OP_BAND: case MGP_OP_BOR: case MGP_OP_BXOR: case MGP_OP_BEQ: return oa == bit || ob == bit;
    case MGP_OP_BNOT: case MGP_OP_ITE: case MGP_OP_RET: return oa == bit;
    case MGP_OP_BITE: return oa == bit || ob == bit || oc == bit;
    default: return false;
  }
}
// is Bool bit `bit` read at or after instruction `from` before being redefined?
inline bool v1_live_after(const uint32_t *ins, uint32_t n, uint32_t from, uint32_t bit) {
  if (bit == MGP_BOOL_TRUE || bit == MGP_BOOL_FALSE) return true;
  for (uint32_t k = from; k < n; ++k) {
    const uint32_t *I = ins + (size_t)k * MGP_INS_WORDS;
    if (v1_reads_bool(I, bit)) return true;
    if (v1_writes_bool(I, bit)) return false;
  }
  return false;
}

// Per Bool bit, the positions of the v1 instructions that read it and that write it
// (ascending): v1_live_after and the writer / reader queries of the BAND4N fold as binary
// searches instead of scans (WalletLibrary's programs run to 12 k instructions).
struct BitIndex {
  std::vector<std::vector<uint32_t>> rd, wr;
  void build(const uint32_t *ins, uint32_t n) {
    // Bool bits are 8-bit destinations; a read field past 255 names no Bool
    rd.assign(256, {});
    wr.assign(256, {});
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t *I = ins + (size_t)k * MGP_INS_WORDS;
      const uint32_t cand[3] = {I[1] & 0xFFFFu, I[1] >> 16, I[2] & 0xFFFFu};
      for (int c = 0; c < 3; ++c) {
        const uint32_t b = cand[c];
        if (b < 256u && (c == 0 || cand[0] != b) && (c < 2 || cand[1] != b) && v1_reads_bool(I, b)) rd[b].push_back(k);
      }
      const uint32_t d = (I[0] >> 16) & 0xFFu;
      if (v1_writes_bool(I, d)) wr[d].push_back(k);
    }
  }
  static uint32_t first_at_or_after(const std::vector<uint32_t> &v, uint32_t k) {
    const auto it = std::lower_bound(v.begin(), v.end(), k);
    return it == v.end() ? 0xFFFFFFFFu : *it;
  }
  // v1_live_after: read at or after `from` before a (static) write; a read and a write in one
  // instruction count as a read
  bool live_after(uint32_t from, uint32_t bit) const {
    if (bit == MGP_BOOL_TRUE || bit == MGP_BOOL_FALSE) return true;
    if (bit >= rd.size()) return false;
    const uint32_t r = first_at_or_after(rd[bit], from);
    return r != 0xFFFFFFFFu && r <= first_at_or_after(wr[bit], from);
  }
  // instructions in [a, b) reading bit
  uint32_t reads_in(uint32_t bit, uint32_t a, uint32_t b) const {
    if (bit >= rd.size() || a >= b) return 0;
    return (uint32_t)(std::lower_bound(rd[bit].begin(), rd[bit].end(), b) - std::lower_bound(rd[bit].begin(), rd[bit].end(), a));
  }
  // the last static writer of bit before q (-1: none)
  int64_t last_write_before(uint32_t bit, uint32_t q) const {
    if (bit >= wr.size()) return -1;
    const auto it = std::lower_bound(wr[bit].begin(), wr[bit].end(), q);
    return it == wr[bit].begin() ? -1 : (int64_t)*(it - 1);
  }
  bool writes_in(uint32_t bit, uint32_t a, uint32_t b) const {
    if (bit >= wr.size() || a >= b) return false;
    const uint32_t w = first_at_or_after(wr[bit], a);
    return w != 0xFFFFFFFFu && w < b;
  }
};

struct BoolPlan {
  std::vector<uint8_t> dead;                  // instruction folded into a neighbour
  std::vector<uint8_t> inv;                   // compare: toggle INVERT
  std::vector<uint32_t> dst;                  // compare / BAND: destination bit override
  std::vector<std::vector<uint32_t>> andops;  // BAND: operand bits (2..4)
  std::vector<uint32_t> comb;                 // compare: 1 + other bit | OR << 16 (folded BAND / BOR)
  std::vector<uint32_t> andn;                 // BAND: 1 + negated bit (folded BNOT), andops[0] the other
  std::vector<uint8_t> merged;                // BAND merged into the next BAND of its AND chain
  std::vector<uint8_t> neg;                   // BAND: andops negated (bit j = andops[j]; BAND4N)
  std::vector<uint8_t> eqsel;                 // ITE: condition from the folded EQ just before it
};

void plan_bools(const uint32_t *ins, uint32_t n, BoolPlan &P) {
  P.dead.assign(n, 0);
  P.inv.assign(n, 0);
  P.dst.assign(n, 0xFFFFFFFFu);
  P.andops.assign(n, {});
  P.comb.assign(n, 0);
  P.andn.assign(n, 0);
  P.merged.assign(n, 0);
  P.neg.assign(n, 0);
  static thread_local BitIndex X;  // build() re-assigns it, keeping the per-bit lists' capacity
  X.build(ins, n);
  for (uint32_t pc = 0; pc + 1 < n; ++pc) {
    const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS, *J = I + MGP_INS_WORDS;
    const uint32_t op = v1_op(I), d = (I[0] >> 16) & 0xFFu;
    if (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF && v1_op(J) == MGP_OP_BNOT && (J[1] & 0xFFFFu) == d) {
      const uint32_t e = (J[0] >> 16) & 0xFFu;
      if (e == d || !X.live_after(pc + 2, d)) {
        P.inv[pc] = 1;
        P.dst[pc] = e;
        P.dead[pc + 1] = 1;
        ++pc;
      }
    }
  }
  for (uint32_t pc = 0; pc < n; ++pc) {
    const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS;
    if (!P.dead[pc] && v1_op(I) == MGP_OP_BAND) P.andops[pc] = {I[1] & 0xFFFFu, I[1] >> 16};
  }
  for (uint32_t pc = 0; pc + 1 < n; ++pc) {
    const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS, *J = I + MGP_INS_WORDS;
    if (P.dead[pc] || P.dead[pc + 1] || v1_op(I) != MGP_OP_BAND || v1_op(J) != MGP_OP_BAND) continue;
    const uint32_t t = (I[0] >> 16) & 0xFFu, ja = J[1] & 0xFFFFu, jb = J[1] >> 16;
    if ((ja == t) == (jb == t)) continue;  // J must read t exactly once
    const bool j_redefines_t = ((J[0] >> 16) & 0xFFu) == t;
    if (P.andops[pc].size() + 1 > 4 || (!j_redefines_t && X.live_after(pc + 2, t))) continue;
    std::vector<uint32_t> ops = P.andops[pc];
    ops.push_back(ja == t ? jb : ja);
    P.andops[pc + 1] = ops;
    P.dead[pc] = 1;
    P.merged[pc] = 1;
  }
  // the next instruction left after pc
  auto next_live = [&](uint32_t pc) {
    uint32_t q = pc + 1;
    while (q < n && P.dead[q]) ++q;
    return q;
  };
  // a plain two-operand BAND / BOR at q that reads bit t exactly once and is t's last
  // reader (or redefines it): the other operand, else 0xFFFFFFFF
  auto sole_reader = [&](uint32_t q, uint32_t t, bool allow_or) -> uint32_t {
    if (q >= n || P.dead[q]) return 0xFFFFFFFFu;
    const uint32_t *J = ins + (size_t)q * MGP_INS_WORDS;
    const uint32_t jop = v1_op(J);
    if (!(jop == MGP_OP_BAND && P.andops[q].size() == 2) && !(allow_or && jop == MGP_OP_BOR)) return 0xFFFFFFFFu;
    const uint32_t ja = J[1] & 0xFFFFu, jb = J[1] >> 16;
    if ((ja == t) == (jb == t)) return 0xFFFFFFFFu;
    if (t == MGP_BOOL_TRUE || t == MGP_BOOL_FALSE) return 0xFFFFFFFFu;
    const bool redefines = ((J[0] >> 16) & 0xFFu) == t;
    if (!redefines && X.live_after(q + 1, t)) return 0xFFFFFFFFu;
    return ja == t ? jb : ja;
  };
  // a compare whose result only feeds the next BAND / BOR: the compare combines it (BCOMB)
  for (uint32_t pc = 0; pc < n; ++pc) {
    const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS;
    const uint32_t op = v1_op(I);
    if (P.dead[pc] || !(op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF)) continue;
    const uint32_t t = P.dst[pc] != 0xFFFFFFFFu ? P.dst[pc] : (I[0] >> 16) & 0xFFu;
    const uint32_t q = next_live(pc);
    const uint32_t x = sole_reader(q, t, true);
    if (x == 0xFFFFFFFFu) continue;
    const uint32_t *J = ins + (size_t)q * MGP_INS_WORDS;
    P.comb[pc] = (1u + x) | (v1_op(J) == MGP_OP_BOR ? 1u << 16 : 0u);
    P.dst[pc] = (J[0] >> 16) & 0xFFu;
    P.dead[q] = 1;
  }
  // a BNOT whose result only feeds the next BAND: BANDN
  for (uint32_t pc = 0; pc < n; ++pc) {
    const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS;
    if (P.dead[pc] || v1_op(I) != MGP_OP_BNOT) continue;
    const uint32_t t = (I[0] >> 16) & 0xFFu, x = I[1] & 0xFFFFu;
    if (x == t) continue;
    const uint32_t q = next_live(pc);
    const uint32_t y = sole_reader(q, t, false);
    if (y == 0xFFFFFFFFu) continue;
    P.andn[q] = 1u + x;
    P.andops[q] = {y, x};
    P.dead[pc] = 1;
  }
  // a BNOT whose result only one AND chain reads, anywhere before it: the chain's last BAND
  // reads the BNOT's source with a negate flag (BAND4N) and the BNOT goes.  Checked on the v1
  // stream with folded instructions included, so every reader counts: x (the BNOT's result)
  // is read exactly once before q, inside the chain, and is not live after q; s (its
  // source) is not written between the BNOT and q.
  // destination overrides of the earlier folds (compare -> BNOT, BCOMB), per bit: with the
  // static writers they are every instruction that writes a bit
  std::vector<std::vector<uint32_t>> dpos(X.wr.size());
  for (uint32_t r = 0; r < n; ++r)
    if (P.dst[r] != 0xFFFFFFFFu) {
      if (P.dst[r] >= dpos.size()) dpos.resize(P.dst[r] + 1);
      dpos[P.dst[r]].push_back(r);
    }
  auto last_writer = [&](uint32_t bit, uint32_t q) -> int64_t {  // the last r < q writing bit
    int64_t p = X.last_write_before(bit, q);
    if (bit < dpos.size()) {
      const auto &v = dpos[bit];
      for (auto it = std::lower_bound(v.begin(), v.end(), q); it != v.begin();) {
        --it;
        if ((int64_t)*it <= p) break;
        if (!P.dead[*it]) { p = *it; break; }
      }
    }
    return p;
  };
  auto written_in = [&](uint32_t bit, uint32_t a, uint32_t b) {  // some r in [a, b) writes bit
    if (X.writes_in(bit, a, b)) return true;
    if (bit >= dpos.size()) return false;
    for (auto it = std::lower_bound(dpos[bit].begin(), dpos[bit].end(), a); it != dpos[bit].end() && *it < b; ++it)
      if (!P.dead[*it]) return true;
    return false;
  };
  for (uint32_t q = 0; q < n; ++q) {
    if (P.dead[q] || v1_op(ins + (size_t)q * MGP_INS_WORDS) != MGP_OP_BAND || P.andn[q]) continue;
    uint32_t lo = q;  // the AND chain ending at q
    while (lo > 0 && P.merged[lo - 1]) --lo;
    std::vector<uint32_t> &ops = P.andops[q];
    for (size_t j = 0; j < ops.size(); ++j) {
      const uint32_t x = ops[j];
      if (x == MGP_BOOL_TRUE || x == MGP_BOOL_FALSE || std::count(ops.begin(), ops.end(), x) != 1) continue;
      const int64_t p = last_writer(x, q);
      if (p < 0 || (uint32_t)p >= lo || P.dead[p]) continue;
      const uint32_t *B = ins + (size_t)p * MGP_INS_WORDS;
      const uint32_t sx = B[1] & 0xFFFFu;
      if (v1_op(B) != MGP_OP_BNOT || P.dst[p] != 0xFFFFFFFFu) continue;  // in place (sx == x) too
      const uint32_t reads = X.reads_in(x, (uint32_t)p + 1, q + 1);
      const uint32_t reads_in_chain = X.reads_in(x, std::max((uint32_t)p + 1, lo), q + 1);
      const bool s_written = written_in(sx, (uint32_t)p + 1, q);
      const bool q_redefines = v1_writes_bool(ins + (size_t)q * MGP_INS_WORDS, x);
      if (reads != 1 || reads_in_chain != 1 || s_written || (!q_redefines && X.live_after(q + 1, x)))
        continue;
      ops[j] = sx;
      P.neg[q] |= (uint8_t)(1u << j);
      P.dead[p] = 1;
    }
  }
  // select chains (a Select over a Store chain, a calldata byte table): `EQ x y -> t` then
  // `ITE(t, z, acc)` with t read nowhere else -> one EQSEL uop.  The compared operands and
  // z must not be the accumulator (it holds the chain's running value).
  P.eqsel.assign(n, 0);
  auto not_acc = [](uint32_t o) { return (o >> 14) != MGP_K_ACC; };
  for (uint32_t pc = 0; pc + 1 < n; ++pc) {
    const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS, *J = I + MGP_INS_WORDS;
    if (P.dead[pc] || P.dead[pc + 1] || v1_op(I) != MGP_OP_EQ || v1_op(J) != MGP_OP_ITE) continue;
    if (P.inv[pc] || P.comb[pc] || P.dst[pc] != 0xFFFFFFFFu) continue;
    const uint32_t t = (I[0] >> 16) & 0xFFu;
    if (t == MGP_BOOL_TRUE || t == MGP_BOOL_FALSE || (J[1] & 0xFFFFu) != t) continue;
    if (!not_acc(I[1] & 0xFFFFu) || !not_acc(I[1] >> 16) || !not_acc(J[1] >> 16) || not_acc(J[2] & 0xFFFFu))
      continue;
    if (X.live_after(pc + 2, t)) continue;
    P.dead[pc] = 1;
    P.eqsel[pc + 1] = 1;
    ++pc;
  }
}

// w0 = first-handler offset | op-handler offset << 16.  A uop dispatched straight to its
// op handler enters past the handler's operand wait (its operands are resident); the op
// field keeps the fetch-path entry that a fetch handler jumps to.
inline uint32_t w0_of(uint32_t first, uint32_t op) {
  const uint32_t f = first == op ? kUopDirectOffset[first] : kUopHandlerOffset[first];
  return f | ((uint32_t)kUopHandlerOffset[op] << 16);
}

}  // namespace

// Appends the uop program of one v1 program to `out`.  Returns 0, or 1 when the
// state does not fit the interpreter's limits (it is then marked undecided).
int mgp_uop_translate(const uint32_t *v1, std::vector<uint32_t> &out) {
  const size_t base = out.size();
  out.resize(base + MGP_U_HDR_WORDS, 0u);
  Translator T;
  T.v1 = v1;
  T.n_ins = v1[0];
  T.n_c = v1[1];
  const bool v1_ok = (v1[3] & 0xFFu) == MGP_ST_OK;
  const uint32_t *ins = v1 + MGP_HDR_WORDS;
  if (v1_ok) T.v1pool.assign(ins + (size_t)T.n_ins * MGP_INS_WORDS, ins + (size_t)T.n_ins * MGP_INS_WORDS + (size_t)T.n_c * 8);
  // per-thread scratch reused across calls (a WalletLibrary program reserves ~120 KB here;
  // fresh memory per call is page faults that a batch's threads take in turn)
  static thread_local std::vector<uint32_t> uops;
  uops.clear();
  uops.reserve((size_t)T.n_ins * MGP_U_UOP_WORDS + 64u);
  // pass 1 only collects the register variables and the mask / sign constants: it emits
  // nothing and looks for no TSEL runs (a run reads the operands its steps would)
  bool pass2 = false;
  auto emit = [&](uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    if (!pass2) return;
    uops.push_back(w0); uops.push_back(w1); uops.push_back(w2); uops.push_back(w3);
  };

  static thread_local BoolPlan BP;  // every field is re-assigned by plan_bools (read only when v1_ok)
  if (v1_ok) plan_bools(ins, T.n_ins, BP);
  auto translate = [&]() {
    for (uint32_t pc = 0; v1_ok && pc < T.n_ins && !T.bad; ++pc) {
      if (BP.dead[pc]) continue;
      const uint32_t *I = ins + (size_t)pc * MGP_INS_WORDS;
      const uint32_t op = I[0] & 0xFFu, width = ((I[0] >> 8) & 0xFFu) + 1u;
      const uint32_t dst = BP.dst[pc] != 0xFFFFFFFFu ? BP.dst[pc] : ((I[0] >> 16) & 0xFFu) | ((I[3] & 0xFFu) << 8);
      const bool store = ((I[0] >> 24) & MGP_INS_STORE) != 0;
      const uint32_t oa = I[1] & 0xFFFFu, ob = I[1] >> 16, oc = I[2] & 0xFFFFu, imm = I[2] >> 16;
      const bool narrow = width < 256u;

      if (op == MGP_OP_RET) {
        emit(w0_of(MGP_U_RET, MGP_U_RET), T.boolslot(oa), 0, 0);
        break;
      }
      if (op == MGP_OP_BAND && BP.andn[pc]) {  // a & ~b
        emit(w0_of(MGP_U_BANDN, MGP_U_BANDN), T.boolslot(BP.andops[pc][0]) | (T.boolslot(BP.andops[pc][1]) << 16),
             0u, T.boolslot(dst) << 16);
        continue;
      }
      if (op == MGP_OP_BAND && BP.neg[pc]) {  // AND chain with negated operands
        const std::vector<uint32_t> &q = BP.andops[pc];
        const uint32_t c = q.size() > 2 ? T.boolslot(q[2]) : T.boolslot(MGP_BOOL_TRUE);
        const uint32_t d = q.size() > 3 ? T.boolslot(q[3]) : T.boolslot(MGP_BOOL_TRUE);
        const uint32_t id = MGP_U_BAND4N_FIRST + BP.neg[pc] - 1u;
        emit(w0_of(id, id), T.boolslot(q[0]) | (T.boolslot(q[1]) << 16), c | (d << 16), T.boolslot(dst) << 16);
        continue;
      }
      if (op == MGP_OP_BAND && BP.andops[pc].size() > 2) {
        const std::vector<uint32_t> &q = BP.andops[pc];
        const uint32_t c = T.boolslot(q[2]), d = q.size() > 3 ? T.boolslot(q[3]) : T.boolslot(MGP_BOOL_TRUE);
        emit(w0_of(MGP_U_BAND4, MGP_U_BAND4), T.boolslot(q[0]) | (T.boolslot(q[1]) << 16), c | (d << 16),
             T.boolslot(dst) << 16);
        continue;
      }
      if (op >= MGP_OP_BAND && op <= MGP_OP_BEQ) {
        static const uint32_t ids[] = {MGP_U_BAND, MGP_U_BOR, MGP_U_BXOR, MGP_U_BNOT, MGP_U_BITE, MGP_U_BEQ};
        const uint32_t id = ids[op - MGP_OP_BAND];
        emit(w0_of(id, id), T.boolslot(oa) | (T.boolslot(ob) << 16), T.boolslot(oc), T.boolslot(dst) << 16);
        continue;
      }
      if (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) {
        Opnd a = T.bv(oa), b = T.bv(ob);
        // base compare, invert, commutes-with-swap partner
        uint32_t base;
        bool inv = false;
        switch (op) {
          case MGP_OP_EQ: base = MGP_U_EQ_RA; break;
          case MGP_OP_ULT: base = MGP_U_ULT_RA; break;
          case MGP_OP_UGE: base = MGP_U_ULT_RA; inv = true; break;
          case MGP_OP_UGT: base = MGP_U_UGT_RA; break;
          case MGP_OP_ULE: base = MGP_U_UGT_RA; inv = true; break;
          case MGP_OP_SLT: base = MGP_U_SLT_RA; break;
          case MGP_OP_SGE: base = MGP_U_SLT_RA; inv = true; break;
          case MGP_OP_SGT: base = MGP_U_SGT_RA; break;
          case MGP_OP_SLE: base = MGP_U_SGT_RA; inv = true; break;
          case MGP_OP_UADD_NOOVF: base = narrow ? MGP_U_UADDNOW_RA : MGP_U_UADDNO256_RA; inv = true; break;
          case MGP_OP_UMUL_NOOVF: base = narrow ? MGP_U_UMULNOW_RA : MGP_U_UMULNO256_RA; inv = true; break;
          default: base = MGP_U_ULT_RA; inv = true; break;  // USUB_NOUDF(a,b) = !(a < b)
        }
        if (b.kind == KACC && a.kind != KACC) {
          std::swap(a, b);
          if (base == MGP_U_ULT_RA) base = MGP_U_UGT_RA;
          else if (base == MGP_U_UGT_RA) base = MGP_U_ULT_RA;
          else if (base == MGP_U_SLT_RA) base = MGP_U_SGT_RA;
          else if (base == MGP_U_SGT_RA) base = MGP_U_SLT_RA;
        }
        if (BP.inv[pc]) inv = !inv;  // a folded BNOT of this compare's result
        uint32_t flags = inv ? MGP_UF_INVERT : 0u, w2 = 0, w3 = T.boolslot(dst) << 16;
        if (BP.comb[pc]) {  // a folded BAND / BOR of this compare's result
          flags |= MGP_UF_BCOMB | ((BP.comb[pc] >> 16) ? MGP_UF_BCOMB_OR : 0u);
          w3 |= T.boolslot((BP.comb[pc] & 0xFFFFu) - 1u) << MGP_U_BCOMB_POS;
        }
        if (narrow && (base == MGP_U_SLT_RA || base == MGP_U_SGT_RA)) {
          flags |= MGP_UF_SEXT;
          w3 |= T.sign_off(width);
        }
        if (base == MGP_U_UADDNOW_RA || base == MGP_U_UMULNOW_RA) {
          flags |= MGP_UF_MASK;
          w2 |= T.mask_off(width) << 16;
        }
        const bool ra = a.kind == KACC;
        uint32_t opid = ra ? base : base + 1u;  // _RC follows _RA
        uint32_t first = fetch_id(a.kind, b.kind, !ra);
      if (ra && b.kind == KSLOT) {
        const int xs = xs_handler(opid);
        if (xs >= 0) opid = first = (uint32_t)xs;
      } else if (ra && b.kind == KCONST) {
        const int xc = xc_handler(opid);
        if (xc >= 0) opid = first = (uint32_t)xc;
      } else if (ra && b.kind == KRVAR && !(flags & (MGP_UF_SEXT | MGP_UF_MASK)) && xr_handler(opid) >= 0) {
        opid = first = (uint32_t)xr_handler(opid);  // EQ / ULT / UGT against a register-bank operand
      } else if (reg_kind(a.kind) && (reg_kind(b.kind) || b.kind == KNONE)) {
        const int xv = xv_handler(a.kind, b.kind, !ra, opid);
        if (xv >= 0) opid = first = (uint32_t)xv;
      }
        emit(w0_of(first, opid), (ra ? 0u : a.param) | (b.param << 16), w2 | flags, w3);
        continue;
      }
      // the slot a BV result is stored to: a register slot, an LDS slot, or a spill row (the
      // op keeps its result in vA; a VST uop behind it writes the row)
      auto store_to = [&](uint32_t d_slot, uint32_t &flags, uint32_t &w2, int32_t &vst_row) {
        const Opnd d = T.bv(MGP_OPND(MGP_K_SLOT, d_slot));
        if (d.kind == KRVAR) {
          flags |= MGP_UF_STORE | MGP_UF_REGST;
          w2 |= d.param;
        } else if (d.kind == KVAR) {
          vst_row = (int32_t)d.param;
        } else {
          flags |= MGP_UF_STORE;
          w2 |= d.param;
        }
      };
      // select-chain steps: a v1 EQSEL, or an ITE whose condition is the folded EQ before it
      // (BoolPlan::eqsel); each compares x with y and selects z over the accumulator
      auto is_step = [&](uint32_t p) {
        return p < T.n_ins && (v1_op(ins + (size_t)p * MGP_INS_WORDS) == MGP_OP_EQSEL || BP.eqsel[p]);
      };
      auto step_ops = [&](uint32_t p, uint32_t *x, uint32_t *y, uint32_t *z) {
        const uint32_t *J = ins + (size_t)p * MGP_INS_WORDS;
        const uint32_t *E = v1_op(J) == MGP_OP_EQSEL ? J : J - MGP_INS_WORDS;
        *x = E[1] & 0xFFFFu;
        *y = E[1] >> 16;
        *z = v1_op(J) == MGP_OP_EQSEL ? J[2] & 0xFFFFu : J[1] >> 16;
      };
      // the step right after the step at p (0xFFFFFFFF: none)
      auto next_step = [&](uint32_t p) -> uint32_t {
        if (p + 1 < T.n_ins && v1_op(ins + (size_t)(p + 1) * MGP_INS_WORDS) == MGP_OP_EQSEL) return p + 1;
        if (p + 2 < T.n_ins && BP.eqsel[p + 2]) return p + 2;
        return 0xFFFFFFFFu;
      };
      if (pass2 && is_step(pc) && next_step(pc) != 0xFFFFFFFFu) {
        // a run of select steps comparing one operand q against keys that are all 32-bit
        // constants (TSEL) or all values in LDS / bank / candidate rows (TSELS), each selecting an HBM variable
        // (a calldata / memory byte table): one uop over a table behind the pool
        struct Run {
          uint32_t n = 0;
          int cls = 0;  // 1: constant keys (TSEL), 2: value keys: LDS, bank or candidate row (TSELS)
          uint32_t end = 0;
        };
        // the steps from pc on that compare qraw with a key of one class and select a
        // variable; with `ent`, their (key word, variable) table entries (no allocation
        // while runs are only measured: this runs at every step of every chain)
        auto collect = [&](uint32_t qraw, std::vector<std::pair<uint32_t, uint32_t>> *ent) {
          Run r;
          r.end = pc;
          for (uint32_t p = pc; p != 0xFFFFFFFFu; p = next_step(p)) {
            const uint32_t *J = ins + (size_t)p * MGP_INS_WORDS;
            uint32_t x, y, zo;
            step_ops(p, &x, &y, &zo);
            if (x != qraw && y != qraw) break;
            const uint32_t key = x == qraw ? y : x;
            uint32_t kv = 0;
            int c = 0;
            if ((key >> 14) == MGP_K_CONST) {
              if (T.small_const(key, &kv)) c = 1;
            } else if ((key >> 14) != MGP_K_ACC) {
              const Opnd k = T.bv(key);
              // TSELS key word: LDS byte offset, bit 31 + bank offset 8p in [23:16], or
              // bit 30 + candidate-row variable in [29:16] (an HBM variable or a spill row)
              if (k.kind == KSLOT) { c = 2; kv = k.param; }
              else if (k.kind == KRVAR) { c = 2; kv = 0x80000000u | (k.param << 16); }
              else if (k.kind == KVAR && k.param < 0x4000u) { c = 2; kv = 0x40000000u | (k.param << 16); }
            }
            const Opnd z = T.bv(zo);
            if (!c || (r.cls && c != r.cls) || z.kind != KVAR || ((J[0] >> 8) & 0xFFu) != ((I[0] >> 8) & 0xFFu)) break;
            r.cls = c;
            ++r.n;
            if (ent) ent->emplace_back(kv, z.param);
            r.end = p;
            if ((J[0] >> 24) & MGP_INS_STORE) break;  // a stored step ends the run
          }
          return r;
        };
        uint32_t a0, b0, z0;
        step_ops(pc, &a0, &b0, &z0);
        // an operand that the next MGP_U_TSEL_MIN - 1 steps all compare (raw operand
        // fields, no kind lookups): most steps start no run, and this rejects them cheaply
        auto shared = [&](uint32_t q) {
          uint32_t p = pc;
          for (uint32_t k = 1; k < MGP_U_TSEL_MIN; ++k) {
            p = next_step(p);
            if (p == 0xFFFFFFFFu) return false;
            uint32_t x, y, z;
            step_ops(p, &x, &y, &z);
            if (x != q && y != q) return false;
          }
          return true;
        };
        const bool sa = shared(a0), sb = a0 != b0 && shared(b0);
        const Run ra = sa ? collect(a0, nullptr) : Run(), rb = sb ? collect(b0, nullptr) : Run();
        const bool use_a = ra.n >= rb.n;
        const uint32_t qraw = use_a ? a0 : b0;
        const Run &run = use_a ? ra : rb;
        const int cls = run.cls;
        const uint32_t end = run.end;
        const uint32_t n_pool = (uint32_t)((T.ms.size() + T.v1pool.size()) / 8);
        const uint32_t tpos = n_pool * 4u + (uint32_t)(T.tables.size() / 2);  // (pool bytes + table bytes) / 8
        const Opnd q = T.bv(qraw);
        if (run.n >= MGP_U_TSEL_MIN && tpos + run.n + 8 < 0xFFFFu && q.kind != KACC &&
            !(cls == 1 && q.kind == KCONST)) {
          std::vector<std::pair<uint32_t, uint32_t>> ent;
          ent.reserve(run.n);
          collect(qraw, &ent);
          uint32_t n_ent;
          const uint32_t toff = T.add_table(ent, cls == 1, &n_ent);
          const uint32_t *J = ins + (size_t)end * MGP_INS_WORDS;
          uint32_t flags = 0, w2 = 0;
          int32_t vst_row = -1;
          if (narrow && op == MGP_OP_EQSEL) {  // the selected variables are read unmasked (v1 EQSEL; pass 1 found its mask)
            flags |= MGP_UF_MASK;
            w2 |= T.mask_off(width) << 16;
          }
          if ((J[0] >> 24) & MGP_INS_STORE) store_to(((J[0] >> 16) & 0xFFu) | ((J[3] & 0xFFu) << 8), flags, w2, vst_row);
          emit(w0_of(fetch_id(q.kind, KNONE, true), cls == 1 ? MGP_U_TSEL : MGP_U_TSELS), q.param, w2 | flags,
               n_ent | ((n_pool * 4u + toff / 2u) << 16));
          if (vst_row >= 0) emit(w0_of(MGP_U_VST, MGP_U_VST), 0u, (uint32_t)vst_row, 0u);
          pc = end;
          continue;
        }
      }
      // ---- BV-producing
      uint32_t flags = 0, w2 = 0, w3 = 0, opid = 0;
      Opnd a = {KNONE, 0}, b = {KNONE, 0};
      bool need_mask = false;
      switch (op) {
        case MGP_OP_ADD: case MGP_OP_MUL: case MGP_OP_AND: case MGP_OP_OR: case MGP_OP_XOR: {
          a = T.bv(oa); b = T.bv(ob);
          if (b.kind == KACC && a.kind != KACC) std::swap(a, b);
          opid = op == MGP_OP_ADD ? MGP_U_ADD : op == MGP_OP_MUL ? MGP_U_MUL : op == MGP_OP_AND ? MGP_U_AND
               : op == MGP_OP_OR ? MGP_U_OR : MGP_U_XOR;
          need_mask = narrow && (op == MGP_OP_ADD || op == MGP_OP_MUL);
          break;
        }
        case MGP_OP_SUB:
          a = T.bv(oa); b = T.bv(ob); opid = MGP_U_SUB; need_mask = narrow;
          break;
        case MGP_OP_SHL: case MGP_OP_LSHR: case MGP_OP_ASHR: {
          a = T.bv(oa);
          if ((ob >> 14) == MGP_K_CONST) {
            uint32_t lo;
            bool big;
            T.const_value(ob, &lo, &big);
            const uint32_t k = big ? 8u : lo >> 5, sb = big ? 0u : lo & 31u;
            opid = (op == MGP_OP_SHL ? MGP_U_SHLI0 : op == MGP_OP_LSHR ? MGP_U_LSHRI0 : MGP_U_ASHRI0) + k;
            w3 |= sb << MGP_U_SHIFT_B_POS;
          } else {
            b = T.bv(ob);
            opid = op == MGP_OP_SHL ? MGP_U_SHL : op == MGP_OP_LSHR ? MGP_U_LSHR : MGP_U_ASHR;
          }
          if (op == MGP_OP_ASHR && narrow) {
            flags |= MGP_UF_SEXT;
            w3 |= T.sign_off(width);
          }
          need_mask = narrow && op != MGP_OP_LSHR;
          break;
        }
        case MGP_OP_UDIV: case MGP_OP_UREM: case MGP_OP_SDIV: case MGP_OP_SREM: case MGP_OP_SMOD: {
          a = T.bv(oa); b = T.bv(ob); opid = MGP_U_DIV;
          static const uint32_t dv[] = {MGP_DIV_UDIV, MGP_DIV_UREM, MGP_DIV_SDIV, MGP_DIV_SREM, MGP_DIV_SMOD};
          flags |= dv[op - MGP_OP_UDIV] << MGP_U_DIVOP_POS;
          if (narrow && op >= MGP_OP_SDIV) {
            flags |= MGP_UF_SEXT;
            w3 |= T.sign_off(width);
          }
          need_mask = narrow && op != MGP_OP_UREM;
          break;
        }
        case MGP_OP_NOT: case MGP_OP_NEG:
          a = T.bv(oa); opid = op == MGP_OP_NOT ? MGP_U_NOT : MGP_U_NEG; need_mask = narrow;
          break;
        case MGP_OP_MOV: case MGP_OP_ZEXT:
          a = T.bv(oa); opid = MGP_U_MOV; need_mask = narrow;
          break;
        case MGP_OP_EXTRACT:
          a = T.bv(oa);
          if (imm == 0) {
            opid = MGP_U_MOV;
          } else {
            opid = MGP_U_LSHRI0 + (imm >> 5);
            w3 |= (imm & 31u) << MGP_U_SHIFT_B_POS;
          }
          need_mask = narrow;
          break;
        case MGP_OP_SEXT:
          a = T.bv(oa); opid = MGP_U_SEXT; w3 |= T.sign_off(imm); need_mask = narrow;
          break;
        case MGP_OP_CONCAT:
          a = T.bv(oa); b = T.bv(ob);
          if (imm == 0 || imm >= 256u) { T.bad = true; break; }
          opid = MGP_U_CONCAT0 + (imm >> 5);
          w3 |= (imm & 31u) << MGP_U_SHIFT_B_POS;
          break;
        case MGP_OP_EQSEL:
        case MGP_OP_ITE:
          if (op == MGP_OP_EQSEL || BP.eqsel[pc]) {  // the compared operands are fetched (x -> vC, y -> vB)
            uint32_t x, y, zo;
            step_ops(pc, &x, &y, &zo);
            const Opnd z = T.bv(zo);
            a = T.bv(x); b = T.bv(y);
            if (a.kind == KACC || b.kind == KACC || z.kind == KACC) { T.bad = true; break; }
            opid = MGP_U_EQSEL_FIRST + (uint32_t)(z.kind - KSLOT);
            w3 |= z.param << 16;
            need_mask = narrow && op == MGP_OP_EQSEL;  // a v1 EQSEL may select an unmasked variable
            break;
          }
          a = T.bv(ob); b = T.bv(oc); opid = MGP_U_ITE;
          w3 |= T.boolslot(oa) << 16;
          break;
        default:
          T.bad = true;
      }
      if (T.bad) break;
      if (need_mask) {
        flags |= MGP_UF_MASK;
        w2 |= T.mask_off(width) << 16;
      }
      int32_t vst_row = -1;
      if (store) store_to(dst, flags, w2, vst_row);
      if (op == MGP_OP_EQSEL || (op == MGP_OP_ITE && BP.eqsel[pc])) {
        emit(w0_of(fetch_id(a.kind, b.kind, true), opid), a.param | (b.param << 16), w2 | flags, w3);
        if (vst_row >= 0) emit(w0_of(MGP_U_VST, MGP_U_VST), 0u, (uint32_t)vst_row, 0u);
        continue;
      }
      opid = epi_variant(opid, (flags & MGP_UF_STORE) != 0, (flags & MGP_UF_MASK) != 0,
                         (flags & MGP_UF_REGST) != 0);
      // an operand in vA and no operand B: nothing to fetch, dispatch straight to the op
      uint32_t first = (a.kind == KACC && b.kind == KNONE) ? opid : fetch_id(a.kind, b.kind, false);
      // vA op bank-register: one fused handler reads B straight from the bank
      if (a.kind == KACC && b.kind == KRVAR) {
        const int xr = xr_handler(opid);
        if (xr >= 0) opid = first = (uint32_t)xr;
      } else if (a.kind == KACC && b.kind == KSLOT) {
        const int xs = xs_handler(opid);
        if (xs >= 0) opid = first = (uint32_t)xs;
      } else if (a.kind == KACC && b.kind == KCONST) {
        const int xc = xc_handler(opid);
        if (xc >= 0) opid = first = (uint32_t)xc;
      }
      if (first != opid && reg_kind(a.kind) && (reg_kind(b.kind) || b.kind == KNONE)) {
        const int xv = xv_handler(a.kind, b.kind, false, opid);  // register operands + op
        if (xv >= 0) opid = first = (uint32_t)xv;
      }
      emit(w0_of(first, opid), a.param | (b.param << 16), w2 | flags, w3);
      if (vst_row >= 0) emit(w0_of(MGP_U_VST, MGP_U_VST), 0u, (uint32_t)vst_row, 0u);
    }
  };
  // pass 1 finds the register variables the program reads and the mask / sign constants;
  // pass 2 places the BV slots (map_slots) and puts the v1 pool behind the mask / sign
  // entries (their index fields are 6 bits, the operand fields 16)
  translate();
  const uint32_t n_slots = v1_ok ? v1[2] : 0u;
  if (v1_ok && !T.bad) {
    T.map_slots(n_slots, v1[3] >> 8);
    T.ms_base = (uint32_t)(T.ms.size() / 8);
    const size_t n_ms = T.ms.size();
    uops.clear();
    T.tables.clear();
    T.table_at.clear();
    pass2 = true;
    translate();
    if (T.ms.size() != n_ms) T.bad = true;  // pass 2 found a constant pass 1 did not
  }
  const size_t n_pool = (T.ms.size() + T.v1pool.size()) / 8;
  static const bool why = getenv("MGP_LOWER_WHY") != nullptr;
  if (why && (!v1_ok || T.bad || uops.empty() || n_pool > MGP_U_MAX_POOL))
    fprintf(stderr, "[mgp_uop] not runnable: v1_ok %d bad %d uops %zu pool %zu\n", (int)v1_ok, (int)T.bad,
            uops.size(), n_pool);
  if (!v1_ok || T.bad || uops.empty() || n_pool > MGP_U_MAX_POOL) {
    out[base + 0] = 0;
    out[base + 1] = 1;  // not runnable: the kernel reports MGP_UNDECIDED
    out[base + 2] = MGP_U_HDR_WORDS * 4u;
    for (int k = 0; k < MGP_U_UOP_WORDS; ++k) out.push_back(0u);
    return v1_ok ? 1 : 0;
  }
  // pages of 64 uops: the last uop of every full page is PAGE (load the next page)
  const uint32_t n_real = (uint32_t)(uops.size() / MGP_U_UOP_WORDS);
  out.reserve(out.size() + ((size_t)n_real + n_real / (MGP_U_PAGE_UOPS - 1) + 2u) * MGP_U_UOP_WORDS + T.ms.size() +
              T.v1pool.size() + T.tables.size());
  uint32_t n_uops = 0;
  for (uint32_t i = 0; i < n_real; ++i) {
    if (n_uops % MGP_U_PAGE_UOPS == MGP_U_PAGE_UOPS - 1) {
      const uint32_t page[4] = {w0_of(MGP_U_PAGE, MGP_U_PAGE), 0, 0, 0};
      out.insert(out.end(), page, page + 4);
      ++n_uops;
    }
    out.insert(out.end(), uops.begin() + (size_t)i * 4, uops.begin() + (size_t)i * 4 + 4);
    ++n_uops;
  }
  const uint32_t pad[4] = {w0_of(MGP_U_INVALID, MGP_U_INVALID), 0, 0, 0};  // ends a runaway program
  out.insert(out.end(), pad, pad + 4);
  out[base + 0] = n_uops;
  out[base + 1] = 0;
  out[base + 2] = (uint32_t)((MGP_U_HDR_WORDS + (n_uops + 1) * MGP_U_UOP_WORDS) * 4u);
  out[base + 3] = (uint32_t)n_pool | (T.var_mask << 8) | (T.n_lds << 16);
  out.insert(out.end(), T.ms.begin(), T.ms.end());
  out.insert(out.end(), T.v1pool.begin(), T.v1pool.end());
  out.insert(out.end(), T.tables.begin(), T.tables.end());
  return 0;
}
