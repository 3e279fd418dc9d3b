// mgp_domain.h — the abstract domain of the UNSAT pre-check and the decision rows
// (host code, mgp_refute.cpp).
//
// Known bits x unsigned interval per BV node, truth sets per Bool node, operand-pair
// orderings and UF congruence (DESIGN.md §4 "mgp_refute").  Everything the propagation
// touches is reached through `Dom`, a view of plain pointers: the host builds a state
// with std::vector storage (mgp_refute.cpp State::setup / build_atoms / build_graph) and
// views it; a decision row works on its own copy of the mutable arrays (node values,
// truth sets, variable values, pair orderings) with a bounded undo log and work list
// (`Stack`).  (Round 5: the device build of this code, one lane per (state, row), ran
// 7x slower than 16 host threads and was removed)
#pragma once
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/mgp.h"
#include "mgp_bv.h"
#include "mgp_fe_sample.h"

#define MGP_RD inline

namespace mgpd {

// Study builds only (make EXTRA=-DMGPD_TRACE_ON OUT=... OBJDIR=..., loaded through
// MGP_LIB_PATH): MGP_DECIDE_TRACE=1 makes decision rows print their steps to stderr
#ifdef MGPD_TRACE_ON
inline bool trace_on() {
  static const int t = [] { const char *e = getenv("MGP_DECIDE_TRACE"); return e ? atoi(e) : 0; }();
  return t != 0;
}
#define MGPD_TRACE(...) do { if (trace_on()) fprintf(stderr, __VA_ARGS__); } while (0)
// MGP_DECIDE_TRACE=2 also prints every narrowing of a node in [MGP_TRACE_LO, MGP_TRACE_HI]
inline bool trace_node(int32_t i) {
  static const int lvl = [] { const char *e = getenv("MGP_DECIDE_TRACE"); return e ? atoi(e) : 0; }();
  static const int lo = [] { const char *e = getenv("MGP_TRACE_LO"); return e ? atoi(e) : 0; }();
  static const int hi = [] { const char *e = getenv("MGP_TRACE_HI"); return e ? atoi(e) : -1; }();
  return lvl >= 2 && i >= lo && i <= hi;
}
#else
inline bool trace_node(int32_t) { return false; }
inline bool trace_on() { return false; }
#define MGPD_TRACE(...) do { } while (0)
#endif

using V = U256;

// 2^w - 1 for w = 0..256: from a table on the host (the transfer functions build masks
// constantly), computed on the device
struct MaskTable {
  V m[257];
  MaskTable() {
    for (uint32_t w = 0; w <= 256; ++w) m[w] = bv_mask(bv_ones(), w);
  }
};
MGP_RD V M(uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return bv_mask(bv_ones(), w < 256u ? w : 256u);
#else
  static const MaskTable t;
  return t.m[w < 256u ? w : 256u];
#endif
}
MGP_RD bool Z(const V &a) { return bv_is_zero(a); }
MGP_RD bool EQV(const V &a, const V &b) { return bv_eq(a, b); }
MGP_RD bool LT(const V &a, const V &b) { return bv_ult(a, b); }
MGP_RD V AND(const V &a, const V &b) { return bv_and(a, b); }
MGP_RD V OR(const V &a, const V &b) { return bv_or(a, b); }
MGP_RD V XOR(const V &a, const V &b) { return bv_xor(a, b); }
MGP_RD V NOT(const V &a) { return bv_not(a); }
MGP_RD V MIN(const V &a, const V &b) { return LT(a, b) ? a : b; }
MGP_RD V MAX(const V &a, const V &b) { return LT(a, b) ? b : a; }
MGP_RD V SHL(const V &a, uint32_t s) { return s >= 256u ? bv_zero() : bv_shl(a, s); }
MGP_RD V SHR(const V &a, uint32_t s) { return s >= 256u ? bv_zero() : bv_lshr(a, s); }
MGP_RD V BIT(uint32_t i) { return SHL(bv_small(1u), i); }
MGP_RD V ADDV(const V &a, const V &b) { return bv_add(a, b, nullptr); }
MGP_RD V SUBV(const V &a, const V &b) { return bv_sub(a, b, nullptr); }
MGP_RD V ONE() { return bv_small(1u); }

// number of trailing one bits (a known-zero mask's run of low zeros)
MGP_RD uint32_t ctz_ones(const V &z) {
  uint32_t n = 0;
  for (int i = 0; i < 8; ++i) {
    if (z.w[i] == 0xFFFFFFFFu) { n += 32; continue; }
    return n + (uint32_t)__builtin_ctz(~z.w[i]);
  }
  return n;
}

struct AV {
  V z, o, lo, hi;
};
MGP_RD bool same(const AV &a, const AV &b) {
  return EQV(a.z, b.z) && EQV(a.o, b.o) && EQV(a.lo, b.lo) && EQV(a.hi, b.hi);
}

MGP_RD AV top(uint32_t w) {
  AV a;
  a.z = NOT(M(w));
  a.o = bv_zero();
  a.lo = bv_zero();
  a.hi = M(w);
  return a;
}
MGP_RD AV exact(V v, uint32_t w) {
  v = bv_mask(v, w);
  AV a;
  a.z = NOT(v);
  a.o = v;
  a.lo = v;
  a.hi = v;
  return a;
}
MGP_RD bool is_exact(const AV &a) { return EQV(a.lo, a.hi); }
// no bit known and the full interval: a backward transfer from it narrows nothing
MGP_RD bool is_top(const AV &a, uint32_t w) {
  const uint32_t li = w ? (w - 1u) >> 5 : 0u;
  for (uint32_t i = 0; i <= li && i < 8; ++i) {
    const uint32_t m = bv_limb_mask(w, (int)i);
    if ((a.z.w[i] & m) || (a.o.w[i] & m) || a.lo.w[i] || a.hi.w[i] != m) return false;
  }
  return true;
}

// Re-establish the invariants (bits above w known zero, interval within the
// bits' range, common high prefix of lo/hi as known bits).  false = empty.
MGP_RD bool normalize(AV &a, uint32_t w) {
  const V m = M(w);
  a.z = OR(a.z, NOT(m));
  a.o = AND(a.o, m);  // values are taken mod 2^w
  for (int it = 0; it < 3; ++it) {
    if (!Z(AND(a.o, a.z))) return false;
    const V maxb = AND(NOT(a.z), m);
    if (LT(a.lo, a.o)) a.lo = a.o;
    if (LT(maxb, a.hi)) a.hi = maxb;
    if (LT(a.hi, a.lo)) return false;
    const uint32_t k = bv_bitlen(XOR(a.lo, a.hi));
    const V pm = AND(NOT(M(k)), m);
    const V nz = OR(a.z, AND(NOT(a.lo), pm)), no = OR(a.o, AND(a.lo, pm));
    if (EQV(nz, a.z) && EQV(no, a.o)) break;
    a.z = nz;
    a.o = no;
  }
  return Z(AND(a.o, a.z));
}

// ------------------------------------------------------ transfer functions
// LLVM-style known bits of a + b + carry (carry-in 0 or 1, known)
MGP_RD void kb_add(const AV &a, const AV &b, uint32_t cin, uint32_t w, V &rz, V &ro) {
  const V m = M(w);
  const V c = bv_small(cin);
  const V psz = AND(ADDV(ADDV(AND(NOT(a.z), m), AND(NOT(b.z), m)), c), m);
  const V pso = AND(ADDV(ADDV(a.o, b.o), c), m);
  const V ckz = NOT(XOR(XOR(psz, a.z), b.z));
  const V cko = XOR(XOR(pso, a.o), b.o);
  const V known = AND(AND(AND(OR(a.z, a.o), OR(b.z, b.o)), OR(ckz, cko)), m);
  rz = OR(AND(NOT(psz), known), NOT(m));
  ro = AND(pso, known);
}

// (x + y) mod 2^w and whether x + y >= 2^w (x, y < 2^w)
MGP_RD V add_w(const V &x, const V &y, uint32_t w, bool &ovf) {
  uint32_t c = 0;
  V s = bv_add(x, y, &c);
  if (w == 256u) {
    ovf = c != 0u;
    return s;
  }
  ovf = !Z(AND(s, NOT(M(w))));
  return bv_mask(s, w);
}

MGP_RD AV av_not(const AV &a, uint32_t w) {
  const V m = M(w);
  AV r;
  r.z = OR(a.o, NOT(m));
  r.o = AND(a.z, m);
  r.lo = SUBV(m, a.hi);
  r.hi = SUBV(m, a.lo);
  return r;
}

MGP_RD AV av_add(const AV &a, const AV &b, uint32_t w) {
  AV r;
  kb_add(a, b, 0u, w, r.z, r.o);
  bool o1, o2;
  const V s1 = add_w(a.lo, b.lo, w, o1), s2 = add_w(a.hi, b.hi, w, o2);
  if (o1 == o2) {
    r.lo = s1;
    r.hi = s2;
  } else {
    r.lo = bv_zero();
    r.hi = M(w);
  }
  return r;
}

MGP_RD AV av_sub(const AV &a, const AV &b, uint32_t w) {
  // a - b = a + ~b + 1
  const AV nb = av_not(b, w);
  AV r;
  kb_add(a, nb, 1u, w, r.z, r.o);
  const bool u1 = LT(a.lo, b.hi), u2 = LT(a.hi, b.lo);
  if (u1 == u2) {
    r.lo = bv_mask(SUBV(a.lo, b.hi), w);
    r.hi = bv_mask(SUBV(a.hi, b.lo), w);
  } else {
    r.lo = bv_zero();
    r.hi = M(w);
  }
  return r;
}

MGP_RD AV av_and(const AV &a, const AV &b, uint32_t w) {
  AV r = top(w);
  r.z = OR(a.z, b.z);
  r.o = AND(a.o, b.o);
  r.hi = MIN(a.hi, b.hi);
  return r;
}
MGP_RD AV av_or(const AV &a, const AV &b, uint32_t w) {
  AV r = top(w);
  r.z = AND(a.z, b.z);
  r.o = OR(a.o, b.o);
  r.lo = MAX(a.lo, b.lo);
  return r;
}
MGP_RD AV av_xor(const AV &a, const AV &b, uint32_t w) {
  AV r = top(w);
  r.z = OR(AND(a.z, b.z), AND(a.o, b.o));
  r.o = OR(AND(a.z, b.o), AND(a.o, b.z));
  (void)w;
  return r;
}

// x >> w of the 512-bit value (hi, lo), as (high part, low part)
MGP_RD void shr512(const V &hi, const V &lo, uint32_t w, V *qh, V *ql) {
  if (w >= 256u) {
    *qh = bv_zero();
    *ql = SHR(hi, w - 256u);
    return;
  }
  *qh = SHR(hi, w);
  *ql = w ? OR(SHR(lo, w), SHL(hi, 256u - w)) : lo;
}

// c * [lo, hi] for every c of a small range [c0, c1] (a loop count, a batch size): each
// product interval that stays inside one multiple of 2^w is exact mod 2^w, and the result
// is their hull -- a product that wraps for every c of the range still gets a bound
// (cnt * value with value near 2^w is near 2^w, never small).  false: some c's products
// straddle a multiple of 2^w.
MGP_RD bool mul_small_range(const V &c0, uint32_t n_c, const V &lo, const V &hi, uint32_t w, V *rlo, V *rhi) {
  bool any = false;
  V c = c0;
  for (uint32_t k = 0; k < n_c; ++k, c = ADDV(c, ONE())) {
    V pl, ph, ql1, qh1, ql2, qh2;
    const V hl = bv_mul_full(c, lo, &pl), hh = bv_mul_full(c, hi, &ph);
    shr512(hl, pl, w, &qh1, &ql1);
    shr512(hh, ph, w, &qh2, &ql2);
    if (!EQV(qh1, qh2) || !EQV(ql1, ql2)) return false;
    const V a = AND(pl, M(w)), b = AND(ph, M(w));
    *rlo = any ? MIN(*rlo, a) : a;
    *rhi = any ? MAX(*rhi, b) : b;
    any = true;
  }
  return any;
}

MGP_RD AV av_mul(const AV &a, const AV &b, uint32_t w) {
  AV r = top(w);
  const uint32_t tz = ctz_ones(a.z) + ctz_ones(b.z);
  r.z = OR(r.z, M(tz < w ? tz : w));
  V lo;
  const V hi = bv_mul_full(a.hi, b.hi, &lo);
  if (Z(hi) && (w == 256u || Z(AND(lo, NOT(M(w)))))) {
    r.hi = lo;
    r.lo = bv_mul(a.lo, b.lo);
    return r;
  }
  // the product may wrap: an operand of at most 32 values bounds it per value
  constexpr uint32_t kSmallRange = 32u;
  for (int k = 0; k < 2; ++k) {
    const AV &s = k ? b : a, &o = k ? a : b;
    const V span = SUBV(s.hi, s.lo);
    if (!LT(span, bv_small(kSmallRange))) continue;
    V rl, rh;
    if (mul_small_range(s.lo, span.w[0] + 1u, o.lo, o.hi, w, &rl, &rh)) {
      r.lo = rl;
      r.hi = rh;
      break;
    }
  }
  return r;
}

// concrete value of a BV op on exact operands (semantics: include/mgp_ir.h)
MGP_RD V fold_bv(uint8_t op, uint32_t w, const V &x, const V &y, uint32_t wa) {
  switch (op) {
    case MGP_OP_MUL: return bv_mul(x, y);
    case MGP_OP_UDIV: { V q, r; bv_udivrem(x, y, &q, &r); return Z(y) ? M(w) : q; }
    case MGP_OP_UREM: { V q, r; bv_udivrem(x, y, &q, &r); return Z(y) ? x : r; }
    case MGP_OP_SDIV: return bv_sdiv(bv_sext(x, w), bv_sext(y, w));
    case MGP_OP_SREM: return bv_srem(bv_sext(x, w), bv_sext(y, w));
    case MGP_OP_SMOD: return bv_smod(bv_sext(x, w), bv_sext(y, w));
    case MGP_OP_SHL: { const uint32_t s = bv_shift_amount(y); return s >= w ? bv_zero() : SHL(x, s); }
    case MGP_OP_LSHR: { const uint32_t s = bv_shift_amount(y); return s >= w ? bv_zero() : SHR(x, s); }
    case MGP_OP_ASHR: {
      const uint32_t s = bv_shift_amount(y);
      return bv_ashr(bv_sext(x, w), s >= w ? w : s);
    }
    case MGP_OP_SEXT: return bv_sext(x, wa);
    default: return bv_zero();
  }
}

// truth sets: bit0 = may be false, bit1 = may be true
enum : uint8_t { BF = 1, BT = 2, BB = 3 };

MGP_RD uint8_t dec_ult(const AV &a, const AV &b) {  // a <u b
  if (LT(a.hi, b.lo)) return BT;
  if (!LT(a.lo, b.hi)) return BF;
  return BB;
}
MGP_RD uint8_t dec_ule(const AV &a, const AV &b) {  // a <=u b
  if (!LT(b.lo, a.hi)) return BT;
  if (LT(b.hi, a.lo)) return BF;
  return BB;
}
MGP_RD uint8_t dec_eq(const AV &a, const AV &b) {
  if (!Z(OR(AND(a.o, b.z), AND(a.z, b.o))) || LT(a.hi, b.lo) || LT(b.hi, a.lo)) return BF;
  if (is_exact(a) && is_exact(b)) return BT;  // (and equal, else the test above fired)
  return BB;
}

// signed order = unsigned order after flipping the sign bit
MGP_RD AV flip(const AV &a, uint32_t w) {
  // the sign bit sits in one limb: swap it between the known-zero and known-one masks and
  // toggle it in the bounds there (limb-wise; the decision rows call this per signed
  // compare, e.g. every calldata byte guard)
  const uint32_t li = (w - 1u) >> 5, sb = 1u << ((w - 1u) & 31u);
  AV r;
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t m = bv_limb_mask(w, (int)i);
    uint32_t z = a.z.w[i], o = a.o.w[i];
    if (i == li) {
      const uint32_t zb = z & sb, ob = o & sb;
      z = (z & ~sb) | ob;
      o = (o & ~sb) | zb;
    }
    r.z.w[i] = z | ~m;
    r.o.w[i] = o & m;
  }
  if ((a.lo.w[li] & sb) == (a.hi.w[li] & sb)) {
    r.lo = a.lo;
    r.hi = a.hi;
    r.lo.w[li] ^= sb;
    r.hi.w[li] ^= sb;
  } else {
    r.lo = bv_zero();
    r.hi = M(w);
  }
  return r;
}

// orderings of an operand pair (x vs y)
enum : uint8_t { OLT = 1, OEQ = 2, OGT = 4, OALL = 7 };
constexpr uint32_t kVarBit = 0x80000000u;  // a work-list entry naming a variable-table entry
constexpr uint32_t kUfGroup = 48;          // UF congruence: functions with at most this many applications
constexpr int kCongDepth = 4;    // structural congruence: operator levels arg_equal looks through
constexpr int kChainBudget = 256;  // rel_under steps per pair (Dom::chain_orders)
constexpr int kChainTotal = 1 << 16;  // rel_under steps per chain_orders call, all pairs

struct Pair { int32_t x, y; uint8_t u, s; };
struct UfApp { int32_t node, arg; uint32_t fn; uint8_t op; };
// r = a + b (op ADD; flag = a BVAddNoOverflow(a, b) node or -1) or r = a - b (op SUB)
struct ArithRel { int32_t r, a, b, flag; uint8_t op; };
// Disjunctive hull: a BOR tree (root) of disjuncts [d0, d1), each an AND tree of atoms
// [a0, a1) (an atom: a compare of a node with a constant, or a BOR of two such compares on
// one node, e.g. ULE's Or(ULT, ==) expansion); targets [t0, t1): the nodes every disjunct
// bounds.  See Dom::or_hull.
struct OrGroup { int32_t root; uint32_t d0, d1, t0, t1; };
// an application u = f(arg) whose inverse is asserted: eq is the node inv(u) == arg
struct InjApp { int32_t u, arg, eq; uint32_t fn; };
struct OrDis { int32_t node; uint32_t a0, a1; };
struct UndoRec {
  uint8_t kind;  // 0 av, 1 bs, 2 pair, 3 var entry
  uint32_t idx;
  AV av;
  uint8_t b, pu, ps;
};

// a bounded stack over caller storage (the same bound on host and device: a push past
// `cap` is dropped and sets `over`, which a decision row treats as the end of the row)
template <typename T>
struct Stack {
  T *p = nullptr;
  uint32_t n = 0, cap = 0;
  bool over = false;
  MGP_RD void push_back(const T &v) {
    if (n < cap) p[n++] = v;
    else over = true;
  }
  MGP_RD uint32_t size() const { return n; }
  MGP_RD void clear() { n = 0; }
  MGP_RD T &back() { return p[n - 1]; }
  MGP_RD void pop_back() { --n; }
  MGP_RD T &operator[](uint32_t i) { return p[i]; }
};

// Undo-log / work-list bounds of one decision row (a decision's propagation is limited
// to 4n + 64 transfer-function evaluations, each changing at most three values, plus the
// pair and congruence ties of up to three rounds)
MGP_RD uint32_t undo_cap(uint32_t n, uint32_t n_pairs, uint32_t n_ufs) { return 16u * n + 4u * (n_pairs + n_ufs) + 4096u; }
MGP_RD uint32_t work_cap(uint32_t n, uint32_t n_pairs, uint32_t n_ufs) { return 16u * n + 4u * (n_pairs + n_ufs) + 4096u; }

// The propagation state of one DAG (a view; see the header comment)
struct Dom {
  const mgp_node *nd = nullptr;    // the DAG the domain runs on (wide values relaxed)
  const mgp_node *orig = nullptr;  // the DAG before relax_wide (UF arguments, congruence)
  uint32_t n = 0;
  const uint32_t *consts = nullptr;
  uint64_t n_consts = 0;
  AV *av = nullptr;            // value of every BV node
  uint8_t *bs = nullptr;       // truth set of every Bool node
  const uint8_t *isb = nullptr;    // node is Bool-typed
  const int32_t *vtie = nullptr;   // VAR node -> variable-table entry
  AV *vars = nullptr;          // variable table (every VAR node of one variable shares it)
  // Orderings of operand pairs: every compare node on the same two operand nodes reads
  // one set of possible unsigned orderings {<, =, >} and one of signed orderings (the "="
  // bit is shared).  ULT(a,b), ULE(a,b), UGE(b,a), BVSubNoUnderflow(b,a), the Or(ULT, ==)
  // expansions and EQ all constrain the same set, so `amount <= bal` and
  // `Not(BVSubNoUnderflow(bal, amount))` contradict each other although neither operand
  // has a useful range.
  Pair *pairs = nullptr;
  uint32_t n_pairs = 0;
  const int32_t *cmp_pair = nullptr;  // compare node -> pair index, -1 = none
  const uint8_t *cmp_dom = nullptr;   // 0 unsigned, 1 signed, 2 both (EQ)
  const uint8_t *cmp_t = nullptr;     // orderings (x vs y) under which the node is true
  const uint64_t *pair_keys = nullptr;  // (x << 32 | y), x < y, sorted ...
  const int32_t *pair_idx = nullptr;    // ... -> pairs index
  // UF congruence (f(a) = f(b) when a = b is known, the Ackermann axiom the lowering's
  // ITE chains implement, include/mgp_ir.h): the applications of each function with at
  // most kUfGroup of them, sorted by (op, function); arguments compared on the original
  // DAG, so a keccak256_512 application whose 512-bit argument was relaxed still meets
  // the value of an application of the same key (WalletLibrary's m_ownerIndex[sender]
  // read in tx 2 against the write in tx 1 when both senders are equal)
  const UfApp *ufs = nullptr;
  uint32_t n_ufs = 0;
  // what tie() visits, fixed per state (mgp_refute.cpp build_atoms): the compare nodes with
  // a pair, then the BOR nodes whose operands are compares of one pair (tien, n_cmpn +
  // n_borp entries), and the pairs (i, j) of ufs entries of one function whose arguments
  // can be equal (ufp, 2 * n_ufp entries: two constants that differ never are)
  const int32_t *tien = nullptr;
  uint32_t n_cmpn = 0, n_borp = 0;
  const uint32_t *ufp = nullptr;
  uint32_t n_ufp = 0;
  // Structural congruence (round 4): pairs whose two operand nodes apply the same
  // operator with the same parameters (on the original DAG).  Once arg_equal proves their
  // operands equal -- a pair known equal, equal exact values, recursively -- the pair is
  // {=}: f(a, b) = f(a', b') for any operator f.  This is what makes
  // `calldata[i] != calldata[j] ∧ i == j` UNSAT (tests/laser/state/calldata_test.py:79-91):
  // both loads are If(i < size, Select(cd, i), 0) with i, j known equal.
  const int32_t *cong = nullptr;
  uint32_t n_cong = 0;
  // Wrap orderings (round 4): r = a + b does not wrap iff r >=u a (and then r >=u b); it
  // wraps iff r <u a.  r = a - b does not underflow iff r <=u a; it underflows iff r >u a.
  // A known wrap status (a BVAddNoOverflow node's truth, b <= a as a pair ordering, or the
  // operands' intervals) orders (r, a) and (r, b) for the compares that read those pairs,
  // and a known ordering of (r, a) decides the BVAddNoOverflow node.  So SafeMath.add's
  // assert(c >= a) contradicts the integer module's Not(BVAddNoOverflow(a, b))
  // (BECToken.sol:25-29, integer.py:141-147).
  const ArithRel *arel = nullptr;
  uint32_t n_arel = 0;
  // Disjunctive hull (round 4): when a BOR tree is true, one of its disjuncts holds, so a
  // node that every disjunct bounds by constants lies in the hull of those bounds.  The
  // keccak manager's `Or(lo <= f(x) < hi ∧ f(x) % 64 == 0, f(x) == H_1 ∧ x == k_1, ...)`
  // (keccak_function_manager.py:118-146) then keeps f(x) away from every small storage slot,
  // so a read of mapping[x] over a Store chain that also wrote slots 0..n sees those keys as
  // different.  A disjunct whose bounds are empty is false.
  const OrGroup *og = nullptr;
  uint32_t n_og = 0;
  const OrDis *odis = nullptr;
  const int32_t *oatom = nullptr;
  const int32_t *otgt = nullptr;
  // Injectivity (round 4): the keccak manager asserts inv(f(x)) == x for every
  // application (keccak_function_manager.py:118-146), so two applications with equal
  // values have equal arguments.  When both inverse equalities are required and the
  // values are known equal, the arguments are equated -- a wide Concat(key, slot) argument
  // piecewise, on the original DAG -- so a Store chain read m[owner] that must meet the
  // write m[sender] forces owner == sender (WalletLibrary's ownerIndex reads).
  const InjApp *inj = nullptr;
  uint32_t n_inj = 0;
  // decision rows: users of each node, VAR nodes of each variable entry, nodes tie() reads
  const uint32_t *uoff = nullptr, *ulist = nullptr, *voff = nullptr, *vlist = nullptr;
  const uint8_t *tie_rel = nullptr;
  // Equality substitution (round 5): once a pair is known equal, x == y, every ordering known
  // between x and a third node z also holds between y and z (when a compare reads (y, z)).
  // `h_to == h_r1` next to `h_to != h_s2` then decides `h_s2 == h_r1` false: three keccak
  // values of one Store chain that no interval separates (pairs incident to each node: CSR)
  const uint32_t *pinc_off = nullptr, *pinc = nullptr;
  bool changed = false;
  // decision mode (decision rows only, never a refutation): backward rules may also
  // narrow to the PREFERRED part of a solution set -- e.g. the non-wrapping preimages of
  // a product -- because a decision row is only a candidate that the GPU evaluation
  // checks.  Such narrowing is unsound for a proof, so run()/refute_one never enable it.
  bool heur = false;
  // decision mode, wrap rows only: a product narrowed from above prefers its preimages
  // that wrap once (c * a = 2^w + r) over the non-wrapping ones
  bool wrap_pref = false;
  // decision rows: every change can go to an undo log (a failed draw rolls back instead
  // of copying the state) and the changed nodes to a work list (a decision propagates
  // from the decided node, run_from); variable entries are listed as kVarBit | entry
  Stack<UndoRec> *undo = nullptr;
  Stack<uint32_t> *touched = nullptr;

  MGP_RD uint32_t W(int32_t i) const { return nd[i].width; }
  MGP_RD int32_t pair_find(uint64_t key) const {
    uint32_t lo = 0, hi = n_pairs;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pair_keys[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    return (lo < n_pairs && pair_keys[lo] == key) ? pair_idx[lo] : -1;
  }

  MGP_RD bool meet(int32_t i, const AV &s) {
    const uint32_t w = nd[i].width;
    AV t = av[i];
    t.z = OR(t.z, s.z);
    t.o = OR(t.o, s.o);
    t.lo = MAX(t.lo, s.lo);
    t.hi = MIN(t.hi, s.hi);
    if (same(t, av[i])) return true;  // s adds nothing (stored values are normalised)
    if (!normalize(t, w)) {
      MGPD_TRACE("  empty: node %d (op %u)\n", i, nd[i].op);
      return false;
    }
    if (!same(t, av[i])) {
      if (trace_node(i))
        fprintf(stderr, "  node %d (op %u) -> [%08x..%08x, %08x..%08x]\n", i, nd[i].op, t.lo.w[7], t.lo.w[0], t.hi.w[7],
                t.hi.w[0]);
      if (undo) undo->push_back(UndoRec{0, (uint32_t)i, av[i], 0, 0, 0});
      if (touched) touched->push_back((uint32_t)i);
      av[i] = t;
      changed = true;
    }
    return true;
  }
  MGP_RD bool meetb(int32_t i, uint8_t s) {
    const uint8_t t = bs[i] & s;
    if (!t) {
      MGPD_TRACE("  empty: bool node %d (op %u)\n", i, nd[i].op);
      return false;
    }
    if (t != bs[i]) {
      if (trace_node(i)) fprintf(stderr, "  bool %d (op %u) -> %u\n", i, nd[i].op, t);
      if (undo) undo->push_back(UndoRec{1, (uint32_t)i, AV(), bs[i], 0, 0});
      if (touched) touched->push_back((uint32_t)i);
      bs[i] = t;
      changed = true;
    }
    return true;
  }
  // would meeting s into node i leave it non-empty?
  // ITE node i is narrowed past the hull of its branches (a requirement from above that
  // one branch may not meet): some value either branch could take is excluded
  // and the chain's fall-through (the else-branches followed past conditions not known
  // true, to the first non-ITE) cannot supply it: a draw alone cannot meet the requirement
  MGP_RD bool ite_required(uint32_t i) const {
    const AV &r = av[i], &b = av[nd[i].b], &e = av[nd[i].c];
    const V hz = AND(b.z, e.z), ho = AND(b.o, e.o), hlo = MIN(b.lo, e.lo), hhi = MAX(b.hi, e.hi);
    if (EQV(AND(r.z, hz), r.z) && EQV(AND(r.o, ho), r.o) && !LT(hlo, r.lo) && !LT(r.hi, hhi)) return false;
    int32_t j = (int32_t)i;
    for (uint32_t hop = 0; hop < n && nd[j].op == MGP_OP_ITE && nd[j].a >= 0 && bs[nd[j].a] != BT; ++hop) j = nd[j].c;
    return nd[j].op == MGP_OP_ITE ? false : !compatible(j, r);
  }

  MGP_RD bool compatible(int32_t i, const AV &s) const {
    AV t = av[i];
    t.z = OR(t.z, s.z);
    t.o = OR(t.o, s.o);
    t.lo = MAX(t.lo, s.lo);
    t.hi = MIN(t.hi, s.hi);
    return same(t, av[i]) || normalize(t, nd[i].width);
  }

  // x and y (nodes of the original DAG) are known to have equal values: the same node,
  // equal exact values, a pair known equal, or the same operator over operands known
  // equal (depth-limited)
  MGP_RD bool arg_equal(int32_t x0, int32_t y0, int depth0) const {
    // the conjunction over operand pairs, on an explicit stack (no recursion: the device
    // kernel then needs no dynamic stack); each level pops one entry and pushes at most
    // three, so depth <= 4 stays within 2 x depth + 1 <= 9 live entries (bounded below anyway)
    struct Q { int32_t x, y, d; } q[16];
    int nq = 0;
    q[nq++] = Q{x0, y0, depth0};
    while (nq) {
      const Q e = q[--nq];
      const int32_t x = e.x, y = e.y;
      if (x == y) continue;
      if (x < 0 || y < 0) return false;
      const mgp_node *o = orig ? orig : nd;
      const mgp_node &a = o[x], &b = o[y];
      if (a.width != b.width) return false;
      if (isb[x] && isb[y] && (bs[x] == BT || bs[x] == BF) && bs[x] == bs[y]) continue;  // one known truth value
      if (a.width <= MGP_MAX_WIDTH && !isb[x] && !isb[y]) {
        if (is_exact(av[x]) && is_exact(av[y]) && EQV(av[x].lo, av[y].lo)) continue;
        const uint64_t pk = x < y ? ((uint64_t)(uint32_t)x << 32) | (uint32_t)y : ((uint64_t)(uint32_t)y << 32) | (uint32_t)x;
        const int32_t pi = pair_find(pk);
        if (pi >= 0 && pairs[pi].u == OEQ) continue;
      }
      // (a UF application's p1 is its own fresh-value slot: applications of one function
      // are congruent whatever their slots)
      const bool uf = a.op == MGP_OP_UFAPP || a.op == MGP_OP_UFINV;
      if (e.d == 0 || a.op != b.op || a.p0 != b.p0 || (a.p1 != b.p1 && !uf)) return false;
      if (a.op == MGP_OP_VAR || a.op == MGP_OP_TRUE || a.op == MGP_OP_FALSE) continue;  // same variable / constant
      if (a.op == MGP_OP_CONST) return false;  // different pool entries (narrow ones compared above)
      if (nq + 3 > 16) return false;
      if (a.c >= 0) q[nq++] = Q{a.c, b.c, e.d - 1};
      if (a.b >= 0) q[nq++] = Q{a.b, b.b, e.d - 1};
      if (a.a >= 0) q[nq++] = Q{a.a, b.a, e.d - 1};
    }
    return true;
  }

  MGP_RD bool set_order(Pair &p, uint8_t dom, uint8_t m) {
    uint8_t u = p.u, s = p.s;
    if (dom != 1) u &= m;
    if (dom != 0) s &= m;
    const uint8_t eq = (uint8_t)(u & s & OEQ);  // a == b is one fact in both orders
    u = (uint8_t)((u & ~OEQ) | eq);
    s = (uint8_t)((s & ~OEQ) | eq);
    if (u == OEQ) s = OEQ;
    if (s == OEQ) u = OEQ;
    if (!u || !s) return false;
    if (u != p.u || s != p.s) {
      if (undo) undo->push_back(UndoRec{2, (uint32_t)(&p - pairs), AV(), 0, p.u, p.s});
      p.u = u;
      p.s = s;
      changed = true;
    }
    return true;
  }
  // the unsigned orderings of node i vs node j that a compare pair on them allows (OALL
  // when no compare reads the pair)
  MGP_RD uint8_t known_order(int32_t i, int32_t j) const {
    if (i == j) return OEQ;
    const bool sw = i > j;
    const int32_t x = sw ? j : i, y = sw ? i : j;
    const int32_t pi = pair_find(((uint64_t)(uint32_t)x << 32) | (uint32_t)y);
    if (pi < 0) return OALL;
    const uint8_t m = pairs[pi].u;
    return sw ? (uint8_t)((m & OEQ) | ((m & OLT) ? OGT : 0) | ((m & OGT) ? OLT : 0)) : m;
  }
  // restrict the unsigned orderings of node i vs node j to m (no-op without a pair)
  MGP_RD bool order(int32_t i, int32_t j, uint8_t m) {
    if (i == j) return (m & OEQ) != 0;
    const bool sw = i > j;
    const int32_t x = sw ? j : i, y = sw ? i : j;
    const int32_t pi = pair_find(((uint64_t)(uint32_t)x << 32) | (uint32_t)y);
    if (pi < 0) return true;
    if (sw) m = (uint8_t)((m & OEQ) | ((m & OLT) ? OGT : 0) | ((m & OGT) ? OLT : 0));
    return set_order(pairs[pi], 0, m);
  }
  MGP_RD bool arith_rel(const ArithRel &e) {
    const uint32_t w = nd[e.r].width;
    if (e.op == MGP_OP_ADD) {
      int wrap = -1;
      if (e.flag >= 0) wrap = bs[e.flag] == BT ? 0 : (bs[e.flag] == BF ? 1 : -1);
      if (wrap < 0) {
        bool o1 = false, o2 = false;
        add_w(av[e.a].hi, av[e.b].hi, w, o1);
        if (!o1) {
          wrap = 0;
        } else {
          add_w(av[e.a].lo, av[e.b].lo, w, o2);
          if (o2) wrap = 1;
        }
      }
      if (wrap < 0) {  // the ordering of (r, a) or (r, b) decides the wrap
        const uint8_t ra = known_order(e.r, e.a), rb = known_order(e.r, e.b);
        if (ra == OLT || rb == OLT) wrap = 1;
        else if (!(ra & OLT) || !(rb & OLT)) wrap = 0;
      }
      if (wrap < 0) return true;
      if (e.flag >= 0 && !meetb(e.flag, wrap ? BF : BT)) return false;
      const uint8_t m = wrap ? (uint8_t)OLT : (uint8_t)(OGT | OEQ);
      if (!order(e.r, e.a, m) || !order(e.r, e.b, m)) return false;
      return sum_bounds(e, wrap == 1);
    }
    int udf = -1;  // r = a - b underflows iff b >u a
    const uint8_t ab = known_order(e.a, e.b);
    if (!(ab & OLT)) udf = 0;
    else if (ab == OLT) udf = 1;
    if (udf < 0) {
      if (!LT(av[e.a].lo, av[e.b].hi)) udf = 0;
      else if (LT(av[e.a].hi, av[e.b].lo)) udf = 1;
    }
    if (udf < 0) {
      const uint8_t ra = known_order(e.r, e.a);
      if (ra == OGT) udf = 1;
      else if (!(ra & OGT)) udf = 0;
    }
    if (udf < 0) return true;
    if (!order(e.a, e.b, udf ? (uint8_t)OLT : (uint8_t)(OGT | OEQ))) return false;
    if (!order(e.r, e.a, udf ? (uint8_t)OGT : (uint8_t)(OLT | OEQ))) return false;
    return sum_bounds(e, udf == 1);
  }
  // The interval of r = a + b (a - b) once its wrap status is known (round 5): without a wrap
  // r lies in [a.lo + b.lo, a.hi + b.hi] ([a.lo - b.hi, a.hi - b.lo]), with one it is that
  // range shifted by 2^w, where av_add / av_sub give up as soon as the operand ranges straddle
  // the wrap.  SafeMath's asserts (BECToken.sol:20-29) fix the status, so a balance that went
  // through `sub` and `add` keeps a bound and a later overflow test against it is decided.
  MGP_RD bool sum_bounds(const ArithRel &e, bool wrapped) {
    const uint32_t w = nd[e.r].width;
    const AV &A = av[e.a], &B = av[e.b];
    const V m = M(w);
    V lo, hi;
    if (e.op == MGP_OP_ADD) {
      uint32_t c1 = 0, c2 = 0;
      lo = bv_add(A.lo, B.lo, &c1);
      hi = bv_add(A.hi, B.hi, &c2);
      if (w < 256u) {  // carries out of bit w-1
        c1 = !Z(AND(lo, NOT(m)));
        c2 = !Z(AND(hi, NOT(m)));
      }
      if (!wrapped) {
        if (c1) return false;             // even the smallest sum wraps
        if (c2) hi = m;                   // the largest would: cap at 2^w - 1
      } else {
        if (!c2) return false;            // even the largest sum does not wrap
        if (!c1) lo = bv_zero();          // the smallest would not: from 0
      }
    } else {
      const bool b1 = LT(A.lo, B.hi), b2 = LT(A.hi, B.lo);  // borrows of lo - hi, hi - lo
      lo = SUBV(A.lo, B.hi);
      hi = SUBV(A.hi, B.lo);
      if (!wrapped) {
        if (b2) return false;
        if (b1) lo = bv_zero();
      } else {
        if (!b1) return false;
        if (!b2) hi = m;
      }
    }
    AV t = top(w);
    t.lo = bv_mask(lo, w);
    t.hi = bv_mask(hi, w);
    if (!LT(t.hi, t.lo) && !meet(e.r, t)) return false;  // (a capped bound masked past: other rules)
    return e.op == MGP_OP_ADD ? addend_bounds(e.a, e.b, e.r, wrapped) && addend_bounds(e.b, e.a, e.r, wrapped)
                              : true;
  }
  // An addend y of r = x + y once the wrap status is known: y = r - x (+ 2^w if wrapped),
  // so y lies in [r.lo - x.hi, r.hi - x.lo] (+ 2^w).  An overflow test that fails
  // (SafeMath.add's assert, BECToken.sol:25-29) bounds the addend from below: y >= 2^w - x.hi.
  MGP_RD bool addend_bounds(int32_t y, int32_t x, int32_t r, bool wrapped) {
    const uint32_t w = nd[r].width;
    const AV &X = av[x], &R = av[r];
    AV t = top(w);
    if (wrapped) {
      // r = x + y - 2^w < x: r.lo < x.hi, y >= 2^w - (x.hi - r.lo); y <= 2^w - (x.lo - r.hi)
      if (!LT(R.lo, X.hi)) return false;
      t.lo = bv_mask(SUBV(bv_zero(), SUBV(X.hi, R.lo)), w);
      if (LT(R.hi, X.lo)) t.hi = bv_mask(SUBV(bv_zero(), SUBV(X.lo, R.hi)), w);
    } else {
      // r = x + y >= x: y in [r.lo - x.hi, r.hi - x.lo]
      if (LT(R.hi, X.lo)) return false;
      t.hi = SUBV(R.hi, X.lo);
      if (LT(X.hi, R.lo)) t.lo = SUBV(R.lo, X.hi);
    }
    if (LT(t.hi, t.lo)) return false;
    return meet(y, t);
  }

  // narrow [lo, hi] of node t by compare atom k (a compare of t with an exact node);
  // false = the atom cannot hold within [lo, hi]
  MGP_RD bool atom_bound(int32_t k, int32_t t, V &lo, V &hi) const {
    const mgp_node &x = nd[k];
    const bool left = x.a == t;
    const int32_t c = left ? x.b : x.a;
    if ((!left && x.b != t) || !is_exact(av[c])) return true;
    const V v = av[c].lo, mw = M(nd[t].width);
    uint8_t op = x.op;  // normalise to "t op v"
    if (!left) op = op == MGP_OP_ULT ? MGP_OP_UGT : op == MGP_OP_UGT ? MGP_OP_ULT :
                     op == MGP_OP_ULE ? MGP_OP_UGE : op == MGP_OP_UGE ? MGP_OP_ULE : op;
    switch (op) {
      case MGP_OP_EQ: lo = MAX(lo, v); hi = MIN(hi, v); break;
      case MGP_OP_ULT: if (Z(v)) return false; hi = MIN(hi, SUBV(v, ONE())); break;
      case MGP_OP_ULE: hi = MIN(hi, v); break;
      case MGP_OP_UGT: if (EQV(v, mw)) return false; lo = MAX(lo, ADDV(v, ONE())); break;
      case MGP_OP_UGE: lo = MAX(lo, v); break;
      default: break;
    }
    return !LT(hi, lo);
  }
  MGP_RD bool or_hull(const OrGroup &g) {
    if (bs[g.root] != BT) return true;
    for (uint32_t ti = g.t0; ti < g.t1; ++ti) {
      const int32_t t = otgt[ti];
      V hlo = M(256), hhi = bv_zero();
      bool any = false;
      for (uint32_t di = g.d0; di < g.d1; ++di) {
        const OrDis &d = odis[di];
        if (bs[d.node] == BF) continue;
        V lo = av[t].lo, hi = av[t].hi;
        bool ok = true;
        for (uint32_t ai = d.a0; ai < d.a1 && ok; ++ai) {
          const int32_t k = oatom[ai];
          if (nd[k].op != MGP_OP_BOR) {
            ok = atom_bound(k, t, lo, hi);
            continue;
          }
          // BOR of two atoms on t: the hull of both (an atom that cannot hold drops out)
          V l1 = lo, h1 = hi, l2 = lo, h2 = hi;
          const bool o1 = atom_bound(nd[k].a, t, l1, h1), o2 = atom_bound(nd[k].b, t, l2, h2);
          if (o1 && o2) { lo = MIN(l1, l2); hi = MAX(h1, h2); }
          else if (o1) { lo = l1; hi = h1; }
          else if (o2) { lo = l2; hi = h2; }
          else ok = false;
        }
        if (!ok) {  // this disjunct cannot hold
          if (!meetb(d.node, BF)) return false;
          continue;
        }
        hlo = MIN(hlo, lo);
        hhi = MAX(hhi, hi);
        any = true;
      }
      if (!any) return false;
      AV a = top(nd[t].width);
      a.lo = hlo;
      a.hi = hhi;
      if (!meet(t, a)) return false;
    }
    return true;
  }

  // x and y (nodes) have equal values: narrow nodes meet each other and their pair (if any)
  // becomes {=}; wide Concat trees of matching shape are equated piecewise
  MGP_RD bool equate(int32_t x0, int32_t y0) {
    const mgp_node *o = orig ? orig : nd;
    int32_t st[16];
    int ns = 0;
    st[ns++] = x0;
    st[ns++] = y0;
    while (ns >= 2) {
      const int32_t y = st[--ns], x = st[--ns];
      if (x == y || x < 0 || y < 0) continue;
      const uint32_t w = o[x].width;
      if (w != o[y].width || isb[x] || isb[y]) continue;
      if (w <= MGP_MAX_WIDTH && nd[x].width == w && nd[y].width == w) {
        const AV ax = av[x], ay = av[y];
        if (!meet(x, ay) || !meet(y, ax)) return false;
        const int32_t pi = pair_find(((uint64_t)(uint32_t)(x < y ? x : y) << 32) | (uint32_t)(x < y ? y : x));
        if (pi >= 0 && !set_order(pairs[pi], 2, OEQ)) return false;
        continue;
      }
      if (o[x].op == MGP_OP_CONCAT && o[y].op == MGP_OP_CONCAT && o[o[x].b].width == o[o[y].b].width &&
          ns + 4 <= 16) {
        st[ns++] = o[x].a;
        st[ns++] = o[y].a;
        st[ns++] = o[x].b;
        st[ns++] = o[y].b;
      }
    }
    return true;
  }
  // the node whose value x is known to equal: through BV ITEs whose condition is decided
  // and through x + 0, x - 0, x | 0, x ^ 0 (LASER's balance updates by a zero call value)
  MGP_RD bool zero_exact(int32_t i) const { return i >= 0 && is_exact(av[i]) && Z(av[i].lo); }
  MGP_RD int32_t resolve(int32_t x) const {
    for (int hop = 0; hop < 64 && x >= 0; ++hop) {
      const mgp_node &t = nd[x];
      if (t.op == MGP_OP_ITE && t.a >= 0) {
        if (bs[t.a] == BT) { x = t.b; continue; }
        if (bs[t.a] == BF) { x = t.c; continue; }
      } else if ((t.op == MGP_OP_ADD || t.op == MGP_OP_OR || t.op == MGP_OP_XOR) && t.a >= 0 && t.b >= 0) {
        if (zero_exact(t.b)) { x = t.a; continue; }
        if (zero_exact(t.a)) { x = t.b; continue; }
      } else if (t.op == MGP_OP_SUB && t.b >= 0 && zero_exact(t.b)) {
        x = t.a;
        continue;
      }
      break;
    }
    return x;
  }
  // x and y have one value in every model the analysis admits: they resolve to one node,
  // to one function's applications on arguments known equal (after resolving them too),
  // or to operators arg_equal matches
  MGP_RD bool same_value(int32_t x, int32_t y) const {
    const int32_t rx = resolve(x), ry = resolve(y);
    if (rx == ry) return true;
    if (rx < 0 || ry < 0) return false;
    const mgp_node *o = orig ? orig : nd;
    const mgp_node &a = o[rx], &b = o[ry];
    if (a.op == MGP_OP_UFAPP && b.op == MGP_OP_UFAPP && a.p0 == b.p0 && a.width == b.width) {
      const int32_t ax = a.a >= 0 && o[a.a].width <= MGP_MAX_WIDTH ? resolve(a.a) : a.a;
      const int32_t bx = b.a >= 0 && o[b.a].width <= MGP_MAX_WIDTH ? resolve(b.a) : b.a;
      return arg_equal(ax, bx, kCongDepth);
    }
    return rx != x || ry != y ? arg_equal(rx, ry, kCongDepth) : false;
  }

  // ---------------------------------------------------------- select-chain relation
  // Path-sensitive ordering of x against z (round 5): the unsigned orderings {<, =, >} of x
  // vs z that any model can give, following BV ITEs down both branches under the assumption
  // their condition makes (an `a == b` condition: a and b equal on the then-path, different
  // on the else-path), through x + 0, x - 0, x | 0, x ^ 0 and one function's applications
  // on arguments equal under those assumptions.  A Store chain read of balances[ATTACKER]
  // after zero-value transfers is then `=` to the starting balance on every path, which
  // refutes ether_thief's `balance > starting` (ether_thief.py:55-95) however many
  // transfers the chain holds -- the case split (refute_split) runs out of levels first.
  struct Asm { int32_t p, q; uint8_t eq; };
  static constexpr int kMaxAsm = 24;
  // x's exact value, directly or through an assumed equality with an exact node
  // the nodes assumed equal to x (x first), transitively over the equality assumptions
  MGP_RD int eq_class(int32_t x, const Asm *as, int na, int32_t *cl) const {
    int nc = 0;
    cl[nc++] = x;
    for (bool grew = true; grew;) {
      grew = false;
      for (int k = 0; k < na; ++k) {
        if (!as[k].eq) continue;
        bool hp = false, hq = false;
        for (int j = 0; j < nc; ++j) {
          hp |= cl[j] == as[k].p;
          hq |= cl[j] == as[k].q;
        }
        if (hp != hq && nc < kMaxAsm + 1) {
          cl[nc++] = hp ? as[k].q : as[k].p;
          grew = true;
        }
      }
    }
    return nc;
  }
  MGP_RD bool value_under(int32_t x, const Asm *as, int na, V &v) const {
    if (is_exact(av[x])) { v = av[x].lo; return true; }
    int32_t cl[kMaxAsm + 1];
    const int nc = eq_class(x, as, na, cl);
    for (int j = 1; j < nc; ++j)
      if (is_exact(av[cl[j]])) { v = av[cl[j]].lo; return true; }
    return false;
  }
  // truth of p == q under the assumptions: BT, BF or BB
  MGP_RD uint8_t eq_under(int32_t p, int32_t q, const Asm *as, int na, int depth) const {
    if (p == q) return BT;
    if (na) {
      int32_t cp[kMaxAsm + 1], cq[kMaxAsm + 1];
      const int np = eq_class(p, as, na, cp), nq = eq_class(q, as, na, cq);
      for (int j = 1; j < np; ++j)
        if (cp[j] == q) return BT;
      for (int k = 0; k < na; ++k) {  // a disequality between the two classes
        if (as[k].eq) continue;
        bool ap = false, aq = false, bp = false, bq = false;
        for (int j = 0; j < np; ++j) { ap |= cp[j] == as[k].p; bp |= cp[j] == as[k].q; }
        for (int j = 0; j < nq; ++j) { aq |= cq[j] == as[k].p; bq |= cq[j] == as[k].q; }
        if ((ap && bq) || (bp && aq)) return BF;
      }
    }
    if (nd[p].width != nd[q].width || isb[p] || isb[q]) return BB;
    V vp, vq;
    const bool kp = value_under(p, as, na, vp), kq = value_under(q, as, na, vq);
    if (kp && kq) return EQV(vp, vq) ? BT : BF;
    if (kp && !inside_dom(av[q], vp)) return BF;
    if (kq && !inside_dom(av[p], vq)) return BF;
    const uint8_t o = known_order(p, q);
    if (o == OEQ) return BT;
    if (!(o & OEQ)) return BF;
    if (depth > 0) {  // one function's applications on arguments equal under the assumptions
      const mgp_node *og = orig ? orig : nd;
      const mgp_node &a = og[p], &b = og[q];
      if (a.op == MGP_OP_UFAPP && b.op == MGP_OP_UFAPP && a.p0 == b.p0 && a.a >= 0 && b.a >= 0 &&
          og[a.a].width <= MGP_MAX_WIDTH && og[a.a].width == og[b.a].width &&
          eq_under(a.a, b.a, as, na, depth - 1) == BT)
        return BT;
    }
    return dec_eq(av[p], av[q]);
  }
  MGP_RD static bool inside_dom(const AV &a, const V &v) {
    return !LT(v, a.lo) && !LT(a.hi, v) && Z(AND(v, a.z)) && EQV(AND(v, a.o), a.o);
  }
  MGP_RD uint8_t cond_under(int32_t c, const Asm *as, int na) const {
    if (bs[c] == BT || bs[c] == BF) return bs[c];
    if (nd[c].op == MGP_OP_EQ && !isb[nd[c].a]) {
      const uint8_t r = eq_under(nd[c].a, nd[c].b, as, na, 2);
      MGPD_TRACE("  cond %d = EQ(%d, %d) under %d assumptions: %u (exact %d %d)\n", c, nd[c].a, nd[c].b, na, r,
                 (int)is_exact(av[nd[c].a]), (int)is_exact(av[nd[c].b]));
      return r;
    }
    return BB;
  }
  MGP_RD bool zero_under(int32_t x, const Asm *as, int na) const {
    V v;
    return value_under(x, as, na, v) && Z(v);
  }
  MGP_RD uint8_t rel_under(int32_t x, int32_t z, Asm *as, int na, int &budget) const {
    if (--budget < 0) return OALL;
    for (int hop = 0; hop < 64; ++hop) {
      if (x == z) return OEQ;
      const mgp_node &t = nd[x];
      if (t.op == MGP_OP_ITE && t.a >= 0) {
        const uint8_t c = cond_under(t.a, as, na);
        if (c == BT) { x = t.b; continue; }
        if (c == BF) { x = t.c; continue; }
        const bool eqc = nd[t.a].op == MGP_OP_EQ && !isb[nd[t.a].a] && na < kMaxAsm;
        uint8_t r = 0;
        for (int side = 0; side < 2; ++side) {
          int m = na;
          if (eqc) as[m++] = Asm{nd[t.a].a, nd[t.a].b, (uint8_t)(side == 0)};
          r |= rel_under(side == 0 ? t.b : t.c, z, as, m, budget);
          if (r == OALL) return OALL;
        }
        return r;
      }
      if ((t.op == MGP_OP_ADD || t.op == MGP_OP_OR || t.op == MGP_OP_XOR) && t.a >= 0 && t.b >= 0) {
        if (zero_under(t.b, as, na)) { x = t.a; continue; }
        if (zero_under(t.a, as, na)) { x = t.b; continue; }
      } else if (t.op == MGP_OP_SUB && t.b >= 0 && zero_under(t.b, as, na)) {
        x = t.a;
        continue;
      }
      break;
    }
    if (x == z) return OEQ;
    // a leaf: equal under the assumptions (a value, one function on equal arguments), else
    // what the pair orderings and the intervals allow
    const uint8_t e = nd[x].width == nd[z].width && !isb[x] && !isb[z] ? eq_under(x, z, as, na, 2) : BB;
    if (e == BT) return OEQ;
    uint8_t r = known_order(x, z);
    if (e == BF) r &= (uint8_t)~OEQ;
    const AV &X = av[x], &Zv = av[z];
    if (!LT(X.lo, Zv.hi)) r &= (uint8_t)~OLT;  // x < z needs x.lo < z.hi
    if (!LT(Zv.lo, X.hi)) r &= (uint8_t)~OGT;
    if (LT(X.hi, Zv.lo) || LT(Zv.hi, X.lo)) r &= (uint8_t)~OEQ;
    MGPD_TRACE("  rel leaf %d (op %u) vs %d: eq %u -> %u (assumptions %d)\n", x, nd[x].op, z, e, r, na);
    return r;
  }
  // the pairs whose operand is an open select chain: their orderings from rel_under
  // (every call also has a total of kChainTotal steps over all its pairs, so a
  // state with thousands of chain pairs cannot make one tie() unbounded; the corpus never
  // reaches it -- the suite's refutations are unchanged -- and stopping early only leaves
  // orderings unknown, which is sound)
  MGP_RD bool chain_orders() {
    int total = kChainTotal;
    for (uint32_t pj = 0; pj < n_pairs && total > 0; ++pj) {
      Pair &p = pairs[pj];
      const bool cx = nd[p.x].op == MGP_OP_ITE && bs[nd[p.x].a] == BB;
      const bool cy = nd[p.y].op == MGP_OP_ITE && bs[nd[p.y].a] == BB;
      if (!cx && !cy) continue;
      Asm as[kMaxAsm];
      int budget = kChainBudget;
      uint8_t r = OALL;  // each side that is a chain, walked against the other (both sound)
      if (cx) r &= rel_under(p.x, p.y, as, 0, budget);
      total -= kChainBudget - budget;
      if (cy) {
        budget = kChainBudget;
        r &= mirror_order(rel_under(p.y, p.x, as, 0, budget));
        total -= kChainBudget - budget;
      }
      MGPD_TRACE("chain pair %d %d: u %u -> rel %u (budget left %d)\n", p.x, p.y, p.u, r, budget);
      if (r != OALL && !set_order(p, 0, r)) return false;
    }
    return true;
  }

  MGP_RD bool injective() {
    for (uint32_t i = 0; i < n_inj; ++i) {
      if (bs[inj[i].eq] != BT) continue;
      for (uint32_t j = i + 1; j < n_inj && inj[j].fn == inj[i].fn; ++j) {
        if (bs[inj[j].eq] != BT) continue;
        const int32_t x = inj[i].u, y = inj[j].u;
        bool same = is_exact(av[x]) && is_exact(av[y]) && EQV(av[x].lo, av[y].lo);
        if (!same) {
          const int32_t pi = pair_find(((uint64_t)(uint32_t)(x < y ? x : y) << 32) | (uint32_t)(x < y ? y : x));
          same = pi >= 0 && pairs[pi].u == OEQ;
        }
        if (same && !equate(inj[i].arg, inj[j].arg)) return false;
      }
    }
    return true;
  }

  MGP_RD static uint8_t mirror_order(uint8_t m) {
    return (uint8_t)((m & OEQ) | ((m & OLT) ? OGT : 0) | ((m & OGT) ? OLT : 0));
  }
  MGP_RD bool substitute() {
    for (uint32_t pj = 0; pj < n_pairs; ++pj) {
      if (pairs[pj].u != OEQ) continue;
      for (int side = 0; side < 2; ++side) {
        const int32_t a = side ? pairs[pj].y : pairs[pj].x, b = side ? pairs[pj].x : pairs[pj].y;
        for (uint32_t k = pinc_off[a]; k < pinc_off[a + 1]; ++k) {
          const uint32_t qk = pinc[k];
          if (qk == pj) continue;
          const Pair &q = pairs[qk];
          const int32_t z = q.x == a ? q.y : q.x;
          if (z == b) continue;
          // orderings of a vs z (the pair stores x vs y)
          const uint8_t mu = q.x == a ? q.u : mirror_order(q.u), ms = q.x == a ? q.s : mirror_order(q.s);
          if (mu == OALL && ms == OALL) continue;
          const int32_t lo = b < z ? b : z, hi = b < z ? z : b;
          const int32_t pi = pair_find(((uint64_t)(uint32_t)lo << 32) | (uint32_t)hi);
          if (pi < 0) continue;
          Pair &t = pairs[pi];  // b vs z when t.x == b
          const bool fw = t.x == b;
          if (!set_order(t, 0, fw ? mu : mirror_order(mu)) || !set_order(t, 1, fw ? ms : mirror_order(ms)))
            return false;
        }
      }
    }
    return true;
  }

  MGP_RD bool tie() {
    for (uint32_t k = 0; k < n_og; ++k)
      if (!or_hull(og[k])) return false;
    if (n_inj && !injective()) return false;
    if (n_pairs == 0 && n_ufs == 0 && n_arel == 0) return true;
    for (int sweep = 0; sweep < 2; ++sweep)
      for (uint32_t q = 0; q < n_cmpn; ++q) {
        const uint32_t i = (uint32_t)tien[q];
        const int32_t pi = cmp_pair[i];
        Pair &p = pairs[pi];
        const uint8_t t = cmp_t[i], f = (uint8_t)(OALL & ~t);
        if (bs[i] == BT && !set_order(p, cmp_dom[i], t)) return false;
        if (bs[i] == BF && !set_order(p, cmp_dom[i], f)) return false;
        const uint8_t cur = cmp_dom[i] == 1 ? p.s : p.u;
        if (!meetb((int32_t)i, (uint8_t)(((cur & t) ? BT : 0) | ((cur & f) ? BF : 0)))) return false;
      }
    // a true Or of two compares on one operand pair (the Or(ULT, ==) expansion of ULE /
    // UGE, bitvec_helper.py:53-80) allows only the union of their orderings
    for (uint32_t q = n_cmpn; q < n_cmpn + n_borp; ++q) {
      const int32_t i = tien[q];
      if (bs[i] != BT) continue;
      const int32_t a = nd[i].a, b = nd[i].b;
      const int32_t pa = cmp_pair[a];
      const uint8_t da = cmp_dom[a], db = cmp_dom[b];
      if (da != db && da != 2 && db != 2) continue;  // signed with unsigned: no common set
      const uint8_t dom = da == 2 ? db : da;
      if (!set_order(pairs[pa], dom, (uint8_t)(cmp_t[a] | cmp_t[b]))) return false;
    }
    for (uint32_t k = 0; k < n_cong; ++k) {
      Pair &p = pairs[cong[k]];
      if (p.u != OEQ && arg_equal(p.x, p.y, kCongDepth) && !set_order(p, 2, OEQ)) return false;
    }
    // value aliases (refutation only: the decision rows keep their propagation cost):
    // a compare of a balance read through zero-value transfers and decided ITEs against
    // the starting balance of the same account compares one value with itself
    if (!heur) {
      for (uint32_t pj = 0; pj < n_pairs; ++pj) {
        Pair &p = pairs[pj];
        if (p.u != OEQ && same_value(p.x, p.y) && !set_order(p, 2, OEQ)) return false;
      }
      if (!chain_orders()) return false;
    }
    for (uint32_t k = 0; k < n_arel; ++k)
      if (!arith_rel(arel[k])) return false;
    for (uint32_t pj = 0; pj < n_pairs; ++pj) {
      const Pair &p = pairs[pj];
      if (p.u == OEQ) {  // known equal: the operands share one value
        const AV ax = av[p.x], ay = av[p.y];
        if (!meet(p.x, ay) || !meet(p.y, ax)) return false;
        continue;
      }
      // known unsigned order: x <= y (or x < y) bounds x from above by y.hi and y from
      // below by x.lo (ULE / UGE arrive as Or(ULT, ==), bitvec_helper.py:53-80, whose
      // operands the per-node backward pass cannot narrow)
      const bool le = !(p.u & OGT), ge = !(p.u & OLT);
      if (le == ge) continue;
      const int32_t lo_n = le ? p.x : p.y, hi_n = le ? p.y : p.x;  // lo_n <= hi_n
      const bool strict = (p.u & OEQ) == 0;
      const uint32_t w = nd[lo_n].width;
      if (w == 0u || w != nd[hi_n].width) continue;
      AV a = top(w), b = top(w);
      a.hi = av[hi_n].hi;
      b.lo = av[lo_n].lo;
      if (strict) {
        if (Z(a.hi) || EQV(b.lo, M(w))) return false;
        a.hi = SUBV(a.hi, ONE());
        b.lo = ADDV(b.lo, ONE());
      }
      if (!meet(lo_n, a) || !meet(hi_n, b)) return false;
    }
    if (pinc_off && !substitute()) return false;
    for (uint32_t q = 0; q < n_ufp; ++q) {
      const uint32_t i = ufp[2 * q], j = ufp[2 * q + 1];
      if (!arg_equal(ufs[i].arg, ufs[j].arg, 3)) continue;
      const int32_t x = ufs[i].node, y = ufs[j].node;
      const AV ax = av[x], ay = av[y];
      if (!meet(x, ay) || !meet(y, ax)) return false;
      const int32_t pi = pair_find(((uint64_t)(uint32_t)(x < y ? x : y) << 32) | (uint32_t)(x < y ? y : x));
      if (pi >= 0 && !set_order(pairs[pi], 2, OEQ)) return false;
    }
    // the pairs this call made equal (two keccak values required equal by a decided read)
    // change no value when both are intervals, so no later round would revisit them:
    // equate their preimages now
    if (n_inj && !injective()) return false;
    return true;
  }


  // --------------------------------------------------------------- forward
  MGP_RD bool forward(uint32_t i) {
    const mgp_node &x = nd[i];
    const uint32_t w = x.width;
    if (isb[i]) {
      uint8_t r = BB;
      switch (x.op) {
        case MGP_OP_TRUE: r = BT; break;
        case MGP_OP_FALSE: r = BF; break;
        case MGP_OP_BNOT: r = (uint8_t)(((bs[x.a] & BF) ? BT : 0) | ((bs[x.a] & BT) ? BF : 0)); break;
        case MGP_OP_BAND: {
          const uint8_t a = bs[x.a], b = bs[x.b];
          r = (uint8_t)((((a & BT) && (b & BT)) ? BT : 0) | (((a & BF) || (b & BF)) ? BF : 0));
          break;
        }
        case MGP_OP_BOR: {
          const uint8_t a = bs[x.a], b = bs[x.b];
          r = (uint8_t)((((a & BT) || (b & BT)) ? BT : 0) | (((a & BF) && (b & BF)) ? BF : 0));
          break;
        }
        case MGP_OP_BXOR: case MGP_OP_BEQ: case MGP_OP_EQ:
          if (x.op == MGP_OP_EQ && !isb[x.a]) {
            r = dec_eq(av[x.a], av[x.b]);
          } else {
            const uint8_t a = bs[x.a], b = bs[x.b];
            const bool diff = ((a & BT) && (b & BF)) || ((a & BF) && (b & BT));
            const bool eqp = ((a & BT) && (b & BT)) || ((a & BF) && (b & BF));
            r = (uint8_t)(x.op == MGP_OP_BXOR ? ((diff ? BT : 0) | (eqp ? BF : 0))
                                              : ((eqp ? BT : 0) | (diff ? BF : 0)));
          }
          break;
        case MGP_OP_BITE: case MGP_OP_ITE: {
          const uint8_t c = bs[x.a];
          r = (uint8_t)(((c & BT) ? bs[x.b] : 0) | ((c & BF) ? bs[x.c] : 0));
          break;
        }
        case MGP_OP_ULT: r = dec_ult(av[x.a], av[x.b]); break;
        case MGP_OP_ULE: r = dec_ule(av[x.a], av[x.b]); break;
        case MGP_OP_UGT: r = dec_ult(av[x.b], av[x.a]); break;
        case MGP_OP_UGE: r = dec_ule(av[x.b], av[x.a]); break;
        case MGP_OP_SLT: case MGP_OP_SLE: case MGP_OP_SGT: case MGP_OP_SGE: {
          const uint32_t ow = W(x.a);
          const AV fa = flip(av[x.a], ow), fb = flip(av[x.b], ow);
          r = x.op == MGP_OP_SLT ? dec_ult(fa, fb) : x.op == MGP_OP_SLE ? dec_ule(fa, fb)
            : x.op == MGP_OP_SGT ? dec_ult(fb, fa) : dec_ule(fb, fa);
          break;
        }
        case MGP_OP_UADD_NOOVF: {
          const uint32_t ow = W(x.a);
          bool oh, ol;
          add_w(av[x.a].hi, av[x.b].hi, ow, oh);
          add_w(av[x.a].lo, av[x.b].lo, ow, ol);
          r = !oh ? BT : ol ? BF : BB;
          break;
        }
        case MGP_OP_UMUL_NOOVF: {
          const uint32_t ow = W(x.a);
          auto ovf = [&](const V &p, const V &q) {
            V lo;
            const V hi = bv_mul_full(p, q, &lo);
            return !Z(hi) || (ow < 256u && !Z(AND(lo, NOT(M(ow)))));
          };
          r = !ovf(av[x.a].hi, av[x.b].hi) ? BT : ovf(av[x.a].lo, av[x.b].lo) ? BF : BB;
          break;
        }
        case MGP_OP_USUB_NOUDF: r = dec_ule(av[x.b], av[x.a]); break;
        default: r = BB;
      }
      return meetb((int32_t)i, r);
    }
    AV r = top(w);
    const AV *A = x.a >= 0 ? &av[x.a] : nullptr;
    const AV *B = x.b >= 0 ? &av[x.b] : nullptr;
    switch (x.op) {
      case MGP_OP_VAR: r = vars[vtie[i]]; break;
      case MGP_OP_CONST: {
        V c;
        for (int k = 0; k < 8; ++k) c.w[k] = consts[8ull * x.p0 + k];
        r = exact(c, w);
        break;
      }
      case MGP_OP_ADD: r = av_add(*A, *B, w); break;
      case MGP_OP_SUB:
        // x - x = 0, also when the operands resolve to one node through decided selects (a
        // balance minus the amount read from the same slot: `this.balance` sent in full)
        r = (x.a == x.b || resolve(x.a) == resolve(x.b) || known_order(x.a, x.b) == OEQ) ? exact(bv_zero(), w)
                                                                                          : av_sub(*A, *B, w);
        break;
      case MGP_OP_NEG: r = av_sub(exact(bv_zero(), w), *A, w); break;
      case MGP_OP_MUL: r = av_mul(*A, *B, w); break;
      case MGP_OP_AND: r = av_and(*A, *B, w); break;
      case MGP_OP_OR: r = av_or(*A, *B, w); break;
      case MGP_OP_XOR: r = av_xor(*A, *B, w); break;
      case MGP_OP_NOT: r = av_not(*A, w); break;
      case MGP_OP_UDIV:
        if (!Z(B->lo)) {  // divisor never 0: quotient monotone in both operands
          V q1, q2, rr;
          bv_udivrem(A->lo, B->hi, &q1, &rr);
          bv_udivrem(A->hi, B->lo, &q2, &rr);
          r.lo = q1;
          r.hi = q2;
        }
        break;
      case MGP_OP_UREM:
        r.hi = A->hi;  // x % y <= x, and x % 0 = x
        if (!Z(B->lo)) r.hi = MIN(r.hi, SUBV(B->hi, ONE()));
        if (LT(A->hi, B->lo)) r = *A;  // x < y: x % y = x
        break;
      case MGP_OP_SHL: case MGP_OP_LSHR: case MGP_OP_ASHR: {
        if (is_exact(*B)) {
          const uint32_t s = bv_shift_amount(B->lo);
          if (x.op == MGP_OP_SHL) {
            if (s >= w) { r = exact(bv_zero(), w); break; }
            r.z = OR(SHL(A->z, s), M(s));
            r.o = SHL(A->o, s);
            bool ovf;
            V t, lo2;
            t = bv_mul_full(A->hi, BIT(s), &lo2);
            ovf = !Z(t) || (w < 256u && !Z(AND(lo2, NOT(M(w)))));
            if (!ovf) {
              r.lo = SHL(A->lo, s);
              r.hi = lo2;
            }
          } else if (x.op == MGP_OP_LSHR) {
            if (s >= w) { r = exact(bv_zero(), w); break; }
            r.z = OR(SHR(AND(A->z, M(w)), s), NOT(M(w - s)));
            r.o = SHR(A->o, s);
            r.lo = SHR(A->lo, s);
            r.hi = SHR(A->hi, s);
          } else {
            const uint32_t ss = s >= w ? w - 1u : s;  // shifting by >= w-1 leaves only sign copies
            const V sb = BIT(w - 1u), m = M(w);
            const bool s0 = !Z(AND(A->z, sb)), s1 = !Z(AND(A->o, sb));
            const V zs = OR(AND(A->z, m), s0 ? NOT(m) : bv_zero());
            const V os = OR(AND(A->o, m), s1 ? NOT(m) : bv_zero());
            r.z = OR(bv_shr_fill(zs, ss, s0 ? 0xFFFFFFFFu : 0u), NOT(m));
            r.o = AND(bv_shr_fill(os, ss, s1 ? 0xFFFFFFFFu : 0u), m);
          }
        } else if (x.op != MGP_OP_ASHR) {
          const uint32_t slo = bv_shift_amount(B->lo);
          if (slo >= w) {
            r = exact(bv_zero(), w);
          } else if (x.op == MGP_OP_LSHR) {  // monotone: up in x, down in s
            const uint32_t shi = bv_shift_amount(B->hi);
            r.hi = SHR(A->hi, slo);
            r.lo = shi >= w ? bv_zero() : SHR(A->lo, shi);
          } else {  // shl: at least min(s) low zero bits
            r.z = OR(r.z, M(slo));
          }
        }
        break;
      }
      case MGP_OP_EXTRACT: {
        const uint32_t lo = x.p1, hiw = lo + w;
        r.z = OR(SHR(A->z, lo), NOT(M(w)));
        r.o = AND(SHR(A->o, lo), M(w));
        if (EQV(SHR(A->lo, hiw), SHR(A->hi, hiw))) {  // same prefix above the field: monotone
          r.lo = AND(SHR(A->lo, lo), M(w));
          r.hi = AND(SHR(A->hi, lo), M(w));
        }
        break;
      }
      case MGP_OP_CONCAT: {
        const uint32_t wb = W(x.b);
        r.z = OR(SHL(A->z, wb), AND(B->z, M(wb)));
        r.o = OR(SHL(A->o, wb), B->o);
        r.lo = OR(SHL(A->lo, wb), B->lo);
        r.hi = OR(SHL(A->hi, wb), B->hi);
        break;
      }
      case MGP_OP_ZEXT: r.z = OR(A->z, NOT(M(W(x.a)))); r.o = A->o; r.lo = A->lo; r.hi = A->hi; break;
      case MGP_OP_SEXT: {
        const uint32_t wa = W(x.a);
        const V sb = BIT(wa - 1u), ext = AND(NOT(M(wa)), M(w));
        const bool s0 = !Z(AND(A->z, sb)), s1 = !Z(AND(A->o, sb));
        r.z = OR(AND(A->z, M(wa)), s0 ? NOT(M(wa)) : NOT(M(w)));
        r.o = OR(A->o, s1 ? ext : bv_zero());
        if (s0) { r.lo = A->lo; r.hi = A->hi; }
        if (s1) { r.lo = OR(A->lo, ext); r.hi = OR(A->hi, ext); }
        break;
      }
      case MGP_OP_ITE: {
        const uint8_t c = bs[x.a];
        const AV &b = av[x.b], &e = av[x.c];
        if (c == BT) r = b;
        else if (c == BF) r = e;
        else {
          r.z = AND(b.z, e.z);
          r.o = AND(b.o, e.o);
          r.lo = MIN(b.lo, e.lo);
          r.hi = MAX(b.hi, e.hi);
        }
        break;
      }
      default: break;  // UFAPP / UFINV / SDIV / SREM / SMOD: unconstrained unless folded
    }
    // exact operands: fold the ops whose transfer above is coarse
    const bool two = x.op >= MGP_OP_MUL && x.op <= MGP_OP_ASHR && x.op != MGP_OP_AND && x.op != MGP_OP_OR &&
                     x.op != MGP_OP_XOR && x.op != MGP_OP_NOT && x.op != MGP_OP_NEG;
    if (two && is_exact(*A) && is_exact(*B)) r = exact(fold_bv(x.op, w, A->lo, B->lo, 0), w);
    if (x.op == MGP_OP_SEXT && is_exact(*A)) r = exact(fold_bv(x.op, w, A->lo, bv_zero(), W(x.a)), w);
    return meet((int32_t)i, r);
  }

  // -------------------------------------------------------------- backward
  MGP_RD bool narrow_ult(int32_t a, int32_t b, bool strict) {  // require a < b (strict) or a <= b
    const AV &A = av[a], &B = av[b];
    if (strict ? LT(A.hi, B.lo) : !LT(B.lo, A.hi)) return true;  // holds already: nothing narrows
    AV ta = top(W(a)), tb = top(W(b));
    if (strict) {
      if (Z(B.hi) || EQV(A.lo, M(W(a)))) return false;
      ta.hi = SUBV(B.hi, ONE());
      tb.lo = ADDV(A.lo, ONE());
    } else {
      ta.hi = B.hi;
      tb.lo = A.lo;
    }
    return meet(a, ta) && meet(b, tb);
  }
  // signed: the same on flipped images, mapped back
  MGP_RD bool narrow_slt(int32_t a, int32_t b, bool strict) {
    const uint32_t w = W(a);
    AV fa = flip(av[a], w), fb = flip(av[b], w);
    if (strict ? LT(fa.hi, fb.lo) : !LT(fb.lo, fa.hi)) return true;  // holds already
    if (strict) {
      if (Z(fb.hi) || EQV(fa.lo, M(w))) return false;
      fa.hi = MIN(fa.hi, SUBV(fb.hi, ONE()));
      fb.lo = MAX(fb.lo, ADDV(fa.lo, ONE()));
    } else {
      fa.hi = MIN(fa.hi, fb.hi);
      fb.lo = MAX(fb.lo, fa.lo);
    }
    if (!normalize(fa, w) || !normalize(fb, w)) return false;
    return meet(a, flip(fa, w)) && meet(b, flip(fb, w));
  }

  MGP_RD bool backward(uint32_t i) {
    const mgp_node &x = nd[i];
    if (isb[i]) {
      const uint8_t r = bs[i];
      switch (x.op) {
        case MGP_OP_BNOT: return meetb(x.a, (uint8_t)(((r & BF) ? BT : 0) | ((r & BT) ? BF : 0)));
        case MGP_OP_BAND:
          if (r == BT) return meetb(x.a, BT) && meetb(x.b, BT);
          if (r == BF) {
            if (bs[x.a] == BT && !meetb(x.b, BF)) return false;
            if (bs[x.b] == BT && !meetb(x.a, BF)) return false;
          }
          return true;
        case MGP_OP_BOR:
          if (r == BF) return meetb(x.a, BF) && meetb(x.b, BF);
          if (r == BT) {
            if (bs[x.a] == BF && !meetb(x.b, BT)) return false;
            if (bs[x.b] == BF && !meetb(x.a, BT)) return false;
          }
          return true;
        case MGP_OP_BITE: case MGP_OP_ITE:
          if (bs[x.a] == BT) return meetb(x.b, r);
          if (bs[x.a] == BF) return meetb(x.c, r);
          if (!(bs[x.b] & r) && !meetb(x.a, BF)) return false;
          if (!(bs[x.c] & r) && !meetb(x.a, BT)) return false;
          return true;
        default: break;
      }
      if (r == BB) return true;
      const bool T = r == BT;
      if ((x.op == MGP_OP_EQ && isb[x.a]) || x.op == MGP_OP_BEQ || x.op == MGP_OP_BXOR) {
        const bool same_req = (x.op == MGP_OP_BXOR) ? !T : T;
        auto other = [&](uint8_t v) -> uint8_t {
          return same_req ? v : (uint8_t)(((v & BF) ? BT : 0) | ((v & BT) ? BF : 0));
        };
        if ((bs[x.a] == BT || bs[x.a] == BF) && !meetb(x.b, other(bs[x.a]))) return false;
        if ((bs[x.b] == BT || bs[x.b] == BF) && !meetb(x.a, other(bs[x.b]))) return false;
        return true;
      }
      switch (x.op) {
        case MGP_OP_EQ:
          if (T) {
            const AV A = av[x.a], B = av[x.b];
            return meet(x.a, B) && meet(x.b, A);
          } else {  // a != b: an exact side trims the other's interval ends
            for (int k = 0; k < 2; ++k) {
              const int32_t p = k ? x.b : x.a, q = k ? x.a : x.b;
              if (!is_exact(av[q])) continue;
              AV t = av[p];
              if (EQV(t.lo, av[q].lo)) {
                if (is_exact(t)) return false;
                t.lo = ADDV(t.lo, ONE());
              }
              if (EQV(t.hi, av[q].lo)) t.hi = SUBV(t.hi, ONE());
              if (!meet(p, t)) return false;
            }
            return true;
          }
        case MGP_OP_ULT: return T ? narrow_ult(x.a, x.b, true) : narrow_ult(x.b, x.a, false);
        case MGP_OP_ULE: return T ? narrow_ult(x.a, x.b, false) : narrow_ult(x.b, x.a, true);
        case MGP_OP_UGT: return T ? narrow_ult(x.b, x.a, true) : narrow_ult(x.a, x.b, false);
        case MGP_OP_UGE: return T ? narrow_ult(x.b, x.a, false) : narrow_ult(x.a, x.b, true);
        case MGP_OP_SLT: return T ? narrow_slt(x.a, x.b, true) : narrow_slt(x.b, x.a, false);
        case MGP_OP_SLE: return T ? narrow_slt(x.a, x.b, false) : narrow_slt(x.b, x.a, true);
        case MGP_OP_SGT: return T ? narrow_slt(x.b, x.a, true) : narrow_slt(x.a, x.b, false);
        case MGP_OP_SGE: return T ? narrow_slt(x.b, x.a, false) : narrow_slt(x.a, x.b, true);
        case MGP_OP_USUB_NOUDF: return T ? narrow_ult(x.b, x.a, false) : narrow_ult(x.a, x.b, true);
        case MGP_OP_UADD_NOOVF: {
          const uint32_t ow = W(x.a);
          const V m = M(ow);
          const AV A = av[x.a], B = av[x.b];
          AV ta = top(ow), tb = top(ow);
          if (T) {  // a + b < 2^w
            ta.hi = SUBV(m, B.lo);
            tb.hi = SUBV(m, A.lo);
          } else {  // a + b >= 2^w
            if (Z(A.hi) || Z(B.hi)) return false;
            ta.lo = bv_mask(ADDV(SUBV(m, B.hi), ONE()), ow);
            tb.lo = bv_mask(ADDV(SUBV(m, A.hi), ONE()), ow);
          }
          return meet(x.a, ta) && meet(x.b, tb);
        }
        case MGP_OP_UMUL_NOOVF:
          if (!T) {  // a * b >= 2^w: a >= ceil(2^w / b.hi) and b >= ceil(2^w / a.hi)
            const uint32_t ow = W(x.a);
            const V m = M(ow);
            const AV A = av[x.a], B = av[x.b];
            if (Z(A.hi) || Z(B.hi)) return false;
            V q, rr;
            for (int k = 0; k < 2; ++k) {
              bv_udivrem(m, k ? A.hi : B.hi, &q, &rr);  // floor((2^w - 1) / h) + 1 = ceil(2^w / h)
              if (EQV(q, m)) return false;            // h = 1: the other operand would need 2^w
              AV t = top(ow);
              t.lo = ADDV(q, ONE());
              if (!meet(k ? x.b : x.a, t)) return false;
            }
            return true;
          }
          if (T) {
            const uint32_t ow = W(x.a);
            const AV A = av[x.a], B = av[x.b];
            V q, rr;
            if (!Z(B.lo)) {
              AV ta = top(ow);
              bv_udivrem(M(ow), B.lo, &q, &rr);
              ta.hi = q;
              if (!meet(x.a, ta)) return false;
            }
            if (!Z(A.lo)) {
              AV tb = top(ow);
              bv_udivrem(M(ow), A.lo, &q, &rr);
              tb.hi = q;
              if (!meet(x.b, tb)) return false;
            }
          }
          return true;
        default: return true;
      }
    }
    // BV node: the result's narrowed value constrains its operands
    const uint32_t w = x.width;
    const AV R = av[i];
    switch (x.op) {
      case MGP_OP_VAR: {  // every VAR node of one (index, width) shares the variable's value
        AV &v = vars[vtie[i]];
        AV t = v;
        t.z = OR(t.z, R.z); t.o = OR(t.o, R.o); t.lo = MAX(t.lo, R.lo); t.hi = MIN(t.hi, R.hi);
        if (!normalize(t, w)) return false;
        if (!same(t, v)) {
          if (undo) undo->push_back(UndoRec{3, (uint32_t)vtie[i], v, 0, 0, 0});
          if (touched) touched->push_back(kVarBit | (uint32_t)vtie[i]);
          v = t;
          changed = true;
        }
        return true;
      }
      case MGP_OP_ADD: {
        const AV A = av[x.a], B = av[x.b];
        if ((is_exact(A) && is_exact(B)) || is_top(R, w)) return true;  // nothing to narrow
        return meet(x.a, av_sub(R, B, w)) && meet(x.b, av_sub(R, A, w));
      }
      case MGP_OP_SUB: {
        const AV A = av[x.a], B = av[x.b];
        if ((is_exact(A) && is_exact(B)) || is_top(R, w)) return true;
        return meet(x.a, av_add(R, B, w)) && meet(x.b, av_sub(A, R, w));
      }
      case MGP_OP_XOR: {
        const AV A = av[x.a], B = av[x.b];
        return meet(x.a, av_xor(R, B, w)) && meet(x.b, av_xor(R, A, w));
      }
      case MGP_OP_MUL: {
        // a * b = R (mod 2^w) with b exact, b = d * 2^s, d odd: a * b = ((a * d) mod 2^(w-s))
        // << s, and d is invertible mod 2^k, so the k known bits of R from bit s up fix the k
        // low bits of a = (R >> s) * d^-1 (x * 5 == 1 pins x; cnt * 2^255 below 2^255 makes
        // cnt even)
        for (int k = 0; k < 2; ++k) {
          const int32_t p = k ? x.b : x.a, q = k ? x.a : x.b;
          const AV B = av[q];
          if (!is_exact(B) || Z(B.lo)) continue;
          if (EQV(B.lo, ONE())) {  // a * 1 = a (a loop count narrowed to one transfer)
            if (!meet(p, R)) return false;
            continue;
          }
          const uint32_t s = ctz_ones(NOT(B.lo));
          if (s >= w) continue;
          const V d = SHR(B.lo, s);
          uint32_t kn = ctz_ones(SHR(OR(R.z, R.o), s));
          if (kn > w - s) kn = w - s;
          if (kn == 0) continue;
          V inv = d;  // Newton: d * d = 1 (mod 8), each step doubles the correct bits
          for (int it = 0; it < 7; ++it) inv = bv_mul(inv, SUBV(bv_small(2u), bv_mul(d, inv)));
          const V lowm = M(kn);
          const V al = AND(bv_mul(AND(SHR(R.o, s), lowm), inv), lowm);
          AV t = top(w);
          t.z = OR(t.z, AND(NOT(al), lowm));
          t.o = al;
          if (!meet(p, t)) return false;
        }
        if (heur) {  // decision mode: a * c in [R.lo, R.hi] without wrapping, when that is possible
          for (int k = 0; k < 2; ++k) {
            const int32_t p = k ? x.b : x.a, q = k ? x.a : x.b;
            const AV B = av[q];
            if (!is_exact(B) || Z(B.lo) || is_exact(av[p])) continue;
            V lo, hi, rl, rh;
            if (wrap_pref && LT(ONE(), B.lo) && LT(av[i].hi, SUBV(M(w), B.lo))) {
              // a wrap row: the preimages that wrap once, c * a = 2^w + r (r in [R.lo, R.hi]),
              // a = q0 + (r0 + 1 + r) / c with 2^w - 1 = q0 * c + r0
              V q0, r0;
              bv_udivrem(M(w), B.lo, &q0, &r0);
              bv_udivrem(ADDV(ADDV(r0, ONE()), av[i].lo), B.lo, &lo, &rl);
              if (!Z(rl)) lo = ADDV(lo, ONE());
              bv_udivrem(ADDV(ADDV(r0, ONE()), av[i].hi), B.lo, &hi, &rh);
              lo = ADDV(q0, lo);
              hi = ADDV(q0, hi);
              if (!LT(hi, lo) && !LT(M(w), hi)) {
                AV t = top(w);
                t.lo = lo;
                t.hi = hi;
                if (compatible(p, t)) {
                  if (!meet(p, t)) return false;
                  continue;
                }
              }
            }
            bv_udivrem(av[i].lo, B.lo, &lo, &rl);
            if (!Z(rl)) lo = ADDV(lo, ONE());
            bv_udivrem(av[i].hi, B.lo, &hi, &rh);
            if (LT(hi, lo)) continue;
            AV t = top(w);
            t.lo = lo;
            t.hi = hi;
            if (compatible(p, t) && !meet(p, t)) return false;
          }
        }
        return true;
      }
      case MGP_OP_NOT: return meet(x.a, av_not(R, w));
      case MGP_OP_NEG: return meet(x.a, av_sub(exact(bv_zero(), w), R, w));
      case MGP_OP_UREM: {
        // x % 2^k (k < w) is x's low k bits: the result's known bits below 2^k are x's
        // (URem(hash, 64) == 0, keccak_function_manager.py:139)
        const AV B = av[x.b];
        if (!is_exact(B) || Z(B.lo)) return true;
        const V m1 = SUBV(B.lo, ONE());
        if (!Z(AND(B.lo, m1))) return true;  // not a power of two
        AV ta = top(w);
        ta.z = OR(ta.z, AND(R.z, m1));
        ta.o = AND(R.o, m1);
        return meet(x.a, ta);
      }
      case MGP_OP_AND: {
        const AV A = av[x.a], B = av[x.b];
        AV ta = top(w), tb = top(w);
        ta.o = R.o; tb.o = R.o;
        ta.z = OR(ta.z, AND(R.z, B.o));
        tb.z = OR(tb.z, AND(R.z, A.o));
        ta.lo = R.lo; tb.lo = R.lo;  // a & b <= a
        return meet(x.a, ta) && meet(x.b, tb);
      }
      case MGP_OP_OR: {
        const AV A = av[x.a], B = av[x.b];
        AV ta = top(w), tb = top(w);
        ta.z = OR(ta.z, R.z); tb.z = OR(tb.z, R.z);
        ta.o = AND(R.o, AND(B.z, M(w)));
        tb.o = AND(R.o, AND(A.z, M(w)));
        ta.hi = R.hi; tb.hi = R.hi;  // a | b >= a
        return meet(x.a, ta) && meet(x.b, tb);
      }
      case MGP_OP_ZEXT: {
        const uint32_t wa = W(x.a);
        AV t = top(wa);
        t.z = OR(t.z, R.z);
        t.o = AND(R.o, M(wa));
        if (!Z(AND(R.lo, NOT(M(wa))))) return false;
        t.lo = R.lo;
        t.hi = MIN(R.hi, M(wa));
        return meet(x.a, t);
      }
      case MGP_OP_SEXT: {
        const uint32_t wa = W(x.a);
        AV t = top(wa);
        t.z = OR(t.z, AND(R.z, M(wa)));
        t.o = AND(R.o, M(wa));
        return meet(x.a, t);
      }
      case MGP_OP_EXTRACT: {
        const uint32_t wa = W(x.a), lo = x.p1;
        AV t = top(wa);
        t.z = OR(t.z, SHL(AND(R.z, M(w)), lo));
        t.o = SHL(R.o, lo);
        return meet(x.a, t);
      }
      case MGP_OP_CONCAT: {
        const uint32_t wa = W(x.a), wb = W(x.b);
        if ((is_exact(av[x.a]) && is_exact(av[x.b])) || is_top(R, w)) return true;
        AV ta = top(wa), tb = top(wb);
        ta.z = OR(ta.z, SHR(AND(R.z, M(w)), wb));
        ta.o = SHR(R.o, wb);
        ta.lo = SHR(R.lo, wb);
        ta.hi = SHR(R.hi, wb);
        tb.z = OR(tb.z, AND(R.z, M(wb)));
        tb.o = AND(R.o, M(wb));
        if (EQV(SHR(R.lo, wb), SHR(R.hi, wb))) {
          tb.lo = AND(R.lo, M(wb));
          tb.hi = AND(R.hi, M(wb));
        }
        return meet(x.a, ta) && meet(x.b, tb);
      }
      case MGP_OP_SHL: case MGP_OP_LSHR: {
        if (!is_exact(av[x.b])) return true;
        const uint32_t s = bv_shift_amount(av[x.b].lo);
        if (s >= w) return true;
        AV t = top(w);
        if (x.op == MGP_OP_SHL) {  // r[w-1..s] = a[w-1-s..0]
          t.z = OR(t.z, AND(SHR(AND(R.z, M(w)), s), M(w - s)));
          t.o = SHR(R.o, s);
        } else {  // r[w-1-s..0] = a[w-1..s]
          t.z = OR(t.z, SHL(AND(R.z, M(w - s)), s));
          t.o = SHL(AND(R.o, M(w - s)), s);
          t.lo = SHL(R.lo, s);
          t.hi = AND(OR(SHL(R.hi, s), M(s)), M(w));
        }
        return meet(x.a, t);
      }
      case MGP_OP_ITE: {
        const uint8_t c = bs[x.a];
        if (c == BT) return meet(x.b, R);
        if (c == BF) return meet(x.c, R);
        if (!compatible(x.b, R) && !meetb(x.a, BF)) return false;
        if (!compatible(x.c, R) && !meetb(x.a, BT)) return false;
        return true;
      }
      default: return true;
    }
  }

  MGP_RD void rollback(size_t mark) {
    while (undo->size() > mark) {
      const UndoRec &u = undo->back();
      if (u.kind == 0) av[u.idx] = u.av;
      else if (u.kind == 1) bs[u.idx] = u.b;
      else if (u.kind == 2) pairs[u.idx].u = u.pu, pairs[u.idx].s = u.ps;
      else vars[u.idx] = u.av;
      undo->pop_back();
    }
  }
  // Propagation from one changed node (a decision): backward into its operands, forward
  // and backward through its users, transitively over the nodes that change, then the
  // pair orderings when a node they read changed; at most `budget` transfer-function
  // evaluations (a node with many users, e.g. calldatasize under every byte guard, counts
  // each of them).  1 = the decision empties a domain.  Only decision rows use it
  // (candidates, checked on the GPU); refutations run().
  MGP_RD int run_from(uint32_t seed, uint32_t budget, int rounds = 3) {
    Stack<uint32_t> &T = *touched;
    T.clear();
    T.push_back(seed);
    size_t head = 0;
    uint32_t work = 0;
    bool need_tie = false;
    for (int round = 0; round < rounds; ++round) {
      while (head < T.size()) {
        const uint32_t t = T[head++];
        if (t & kVarBit) {  // a variable's shared value changed: every VAR node of it
          const uint32_t j = t & ~kVarBit;
          if ((work += voff[j + 1] - voff[j] + 1) > budget) return 0;
          for (uint32_t k = voff[j]; k < voff[j + 1]; ++k)
            if (!forward(vlist[k])) return 1;
          continue;
        }
        need_tie |= tie_rel[t] != 0;
        if ((work += 2u * (uoff[t + 1] - uoff[t]) + 1u) > budget) return 0;
        if (!backward(t)) return 1;
        // a user whose value the forward step changed is on the work list now, and its
        // backward step runs when it is reached: only the unchanged ones need it here
        for (uint32_t k = uoff[t]; k < uoff[t + 1]; ++k) {
          const size_t before = T.size();
          if (!forward(ulist[k])) return 1;
          if (T.size() == before && !backward(ulist[k])) return 1;
        }
      }
      const size_t before = T.size();
      if (!meetb((int32_t)n - 1, BT)) return 1;
      if (need_tie) {  // tie() is at its fixpoint unless a node it reads changed
        need_tie = false;
        if (!tie()) return 1;
      }
      if (T.size() == before) break;
    }
    return 0;
  }

  // 1 = refuted (UNSAT), 0 = not refuted
  // the nodes required true: the root, or (core trials, mgp_refute_cores) a chosen subset of
  // the root conjuncts plus the piece-expansion ties
  const int32_t *req = nullptr;
  uint32_t n_req = 0;
  MGP_RD bool require_root() {
    if (!req) return meetb((int32_t)n - 1, BT);
    for (uint32_t k = 0; k < n_req; ++k)
      if (!meetb(req[k], BT)) return false;
    return true;
  }
  MGP_RD int run(uint32_t max_passes) {
    if (!require_root()) return 1;
    for (uint32_t pass = 0; pass < max_passes; ++pass) {
      changed = false;
      for (uint32_t i = 0; i < n; ++i)
        if (!forward(i)) return 1;
      if (!require_root() || !tie()) return 1;
      for (uint32_t i = n; i-- > 0;)
        if (!backward(i)) return 1;
      if (!tie()) return 1;
      if (!changed) break;
    }
    return 0;
  }
};

// ------------------------------------------------------------ decision rows
// One prepared state (mgp_refute.cpp prep_state): its variable slots (VAR nodes and the
// fresh value of UF applications) and, per slot, the constants it is compared equal to.
struct PrepView {
  uint32_t n_slot = 0;
  const uint32_t *slot = nullptr, *width = nullptr;
  const int32_t *node = nullptr;
  const uint32_t *eqh_off = nullptr;  // n_slot + 1
  const V *eqh = nullptr;
};

MGP_RD bool inside_av(const AV &a, const V &v) {
  return !LT(v, a.lo) && !LT(a.hi, v) && Z(AND(v, a.z)) && EQV(AND(v, a.o), a.o);
}

// rows whose decisions start with the Or case split and the ITE branch split (bit r: row r)
constexpr uint32_t kOrRowsDefault = 0xAu;
// the split row whose ITE branch split always tries the then-branch first
constexpr uint32_t kIteGreedyRow = 1u;

// rows that start with the wrap decisions (bit r: row r)
#ifndef MGP_WRAP_ROWS
#define MGP_WRAP_ROWS 0xCu
#endif
constexpr uint32_t kWrapRows = MGP_WRAP_ROWS;
constexpr int kSplitRounds = 8;
#ifndef SPLIT_BUDGET_X
#define SPLIT_BUDGET_X 16u
#endif

// Decision row `row` of a prepared state on `d`, a private copy of the state's base
// analysis (heur set, undo log and work list attached): each variable slot in turn is
// fixed to a draw from its current abstract value and the analysis re-propagated from
// the decided node (Dom::run_from: backward into its operands, through its users,
// transitively, then the pair orderings), so later variables are drawn from values
// narrowed by the earlier choices (x + y == c, a mapping key fixed by an equality, ...).
// A draw that empties a domain is rolled back through the undo log and replaced (up to
// kTries draws).  Writes the value of slot k through put(slot[k], value); stops early
// (remaining slots unwritten) if the undo log overflows.  Stream key per slot:
// (seed, tag, c, slot).
//
// Seeded rows (round 4): with `sv` / `sm` (a value and a flag per variable slot: the parent
// state's witness, matched by slot key) and bit `row` of `seed_rows` set, every seeded slot
// is first fixed to its parent value and propagated (a value the child's constraints reject
// is rolled back and left to the draws), before the Or case split and the draws.  A child
// state extends its parent by one constraint (svm.py:251-255), so the parent's values fix
// most of the row and the draws only decide what the new constraint brought in (a new
// keccak application, a new calldata word).
template <typename Put>
MGP_RD void decision_row(const PrepView &P, Dom &d, uint32_t row, uint32_t c, uint64_t seed, uint64_t tag,
                         uint32_t or_rows, Put &put, const uint32_t *sv = nullptr, const uint8_t *sm = nullptr,
                         uint32_t seed_rows = 0) {
  constexpr uint32_t kTries = 4;
  MGPD_TRACE("=== row %u\n", row);
  Stack<UndoRec> &undo_log = *d.undo;
  Stack<uint32_t> &work = *d.touched;
  const uint32_t budget = 4u * d.n + 64u;
  // the case splits (wrap pairs, Or and ITE branches) are few and steer the whole row: a
  // split whose consequences are cut short by the budget leaves a contradiction that every
  // later draw runs into, so they propagate further
  const uint32_t split_budget = SPLIT_BUDGET_X * d.n + 64u;
  if (sv && sm && row < 32u && ((seed_rows >> row) & 1u)) {
    for (uint32_t k = 0; k < P.n_slot; ++k) {
      if (!sm[P.slot[k]]) continue;
      V v;
      for (int l = 0; l < 8; ++l) v.w[l] = sv[P.slot[k] * 8u + l];
      v = bv_mask(v, P.width[k]);
      const int32_t nk = P.node[k];
      const uint32_t mark = undo_log.size();
      work.clear();
      if (d.meet(nk, exact(v, P.width[k])) && d.run_from((uint32_t)nk, budget) == 0 && !undo_log.over) {
        undo_log.clear();
        continue;
      }
      if (undo_log.over) return;
      d.rollback(mark);
    }
  }
  // the draw schedule of decision row `row`: the first eight rows decide in node
  // order (schedules 0, 4, 6, 8, 2, 10, 12, 14: the lo/hi schedule 0 that BECToken's
  // mapping witness needs and three random-draw schedules first, so a state given
  // four rows keeps most of its yield), later ones add the reverse-order schedules
  // (odd) and then the rest, so any n_decide = 16 + k covers schedules 0..15+k.
  // Node order is what contract states need (WalletLibrary's loop and mapping
  // queries: 60 against 57 states of the mixed corpus at eight rows, at a third
  // of the host time)
  const uint8_t kFirst8[8] = {0, 4, 6, 8, 2, 10, 12, 14};
  const uint32_t drow = row < 8u ? kFirst8[row] : row < 16u ? 2u * (row - 8u) + 1u : row;
  // Wrap decisions (round 5).  A required wrap -- Not(BVAddNoOverflow(a, b)) or
  // Not(BVMulNoOverflow(a, b)) (integer.py:141-160), or r = a + b ordered below an operand
  // (SafeMath.add's assert(c >= a) failing, BECToken.sol:25-29) -- is met first by a wrapping
  // pair of operand values: a + b = 2^w by (2^(w-1), 2^(w-1)) or by an operand's upper bound and
  // its complement, a * b >= 2^w by (2, 2^(w-1)).  The choice propagates back through whatever
  // supplies the operands: an exact 2^255 balance read excludes every store of a small constant
  // from its Store chain, so the row aims at the state in which an earlier transaction's
  // product wrapped (CVE-2018-10299: batchTransfer with cnt = 2, value = 2^255).  Random draws
  // almost never produce such pairs.  A pair that empties a domain is rolled back.
  if (row < 32u && ((kWrapRows >> row) & 1u)) {
    bool over = false;
    auto try_pair = [&](int32_t a, int32_t b, const V &va, const V &vb) -> bool {
      const uint32_t w = d.W(a);
      if (!inside_av(d.av[a], va) || !inside_av(d.av[b], vb)) return false;
      const uint32_t mark = undo_log.size();
      work.clear();
      bool ok = d.meet(a, exact(va, w)) && d.run_from((uint32_t)a, split_budget, kSplitRounds) == 0 && !undo_log.over;
      if (ok) {
        work.clear();
        ok = d.meet(b, exact(vb, w)) && d.run_from((uint32_t)b, split_budget, kSplitRounds) == 0 && !undo_log.over;
      }
      MGPD_TRACE("row %u wrap pair nodes %d %d (w %u): %s\n", row, a, b, w, ok ? "kept" : "rolled back");
      if (ok) {
        undo_log.clear();
        d.wrap_pref = true;  // the row now aims at a wrapped state: products prefer wrapping
        return true;
      }
      over = undo_log.over;
      if (!over) d.rollback(mark);
      return false;
    };
    auto wrap = [&](int32_t a, int32_t b, bool mul) {
      if (a < 0 || b < 0 || is_exact(d.av[a]) || is_exact(d.av[b])) return;
      const uint32_t w = d.W(a);
      if (w < 2u || w != d.W(b)) return;
      const V h = BIT(w - 1u), m = M(w);
      if (mul) {
        const V two = bv_small(2u);
        if (try_pair(a, b, two, h) || over || try_pair(a, b, h, two)) return;
        return;
      }
      if (try_pair(a, b, h, h) || over) return;
      const V ah = d.av[a].hi, bh = d.av[b].hi;
      if (!Z(ah) && (try_pair(a, b, ah, bv_mask(ADDV(SUBV(m, ah), ONE()), w)) || over)) return;
      if (!Z(bh)) try_pair(a, b, bv_mask(ADDV(SUBV(m, bh), ONE()), w), bh);
    };
    for (uint32_t i = d.n; i-- > 0 && !over;) {
      const mgp_node &x = d.nd[i];
      if ((x.op == MGP_OP_UADD_NOOVF || x.op == MGP_OP_UMUL_NOOVF) && d.bs[i] == BF && !d.isb[x.a])
        wrap(x.a, x.b, x.op == MGP_OP_UMUL_NOOVF);
    }
    for (uint32_t k = 0; k < d.n_arel && !over; ++k) {
      const ArithRel &e = d.arel[k];
      if (e.op == MGP_OP_ADD && (d.known_order(e.r, e.a) == OLT || d.known_order(e.r, e.b) == OLT))
        wrap(e.a, e.b, false);
    }
    if (over) return;
  }
  if (row < 32u && ((or_rows >> row) & 1u)) {
    // case split on the disjunctions the root requires: from the root down, a required Or
    // with both operands open takes its first operand (else its second) before any
    // variable is drawn, so its domain narrows as if that disjunct were a plain conjunct
    // (keccak_function_manager.py:158-168: Or(interval condition, concrete-hash matches))
    for (uint32_t i = d.n; i-- > 0;) {
      if (d.nd[i].op != MGP_OP_BOR || d.bs[i] != BT) continue;
      const int32_t a = d.nd[i].a, b = d.nd[i].b;
      if (a < 0 || b < 0 || d.bs[a] != BB || d.bs[b] != BB) continue;
      // a row aiming at a wrapped state leaves a ULE / UGE (Or(ULT, ==) on one operand pair,
      // bitvec_helper.py:53-80) whole: splitting it would drop the boundary value (a transfer
      // of a whole balance, value == bal, as the overflow witness needs); other rows split it
      // too, and the strict side first bounds a balance read away from its zero default
      if (d.wrap_pref && d.cmp_pair[a] >= 0 && d.cmp_pair[a] == d.cmp_pair[b]) continue;
      for (int side = 0; side < 2; ++side) {
        const int32_t pick = side ? b : a;
        const uint32_t mark = undo_log.size();
        work.clear();
        if (d.meetb(pick, BT) && d.run_from((uint32_t)pick, split_budget, kSplitRounds) == 0 && !undo_log.over) {
          MGPD_TRACE("row %u or node %u takes side %d\n", row, i, side);
          undo_log.clear();
          break;
        }
        if (undo_log.over) return;
        d.rollback(mark);
      }
    }
  }
  // Branch split of required selects (round 4): an ITE whose value the analysis has
  // narrowed past the hull of its two branches (a storage read required non-zero, a
  // balance read required >= a bound) with its condition open is a disjunction over the
  // branches that can supply the value.  From the root down, such an ITE takes its
  // then-branch (condition true: the read address equals that store's address, so the
  // keys are equated and, through the keccak inverse, their preimages) or its else-branch;
  // row kIteGreedyRow takes the first then-branch that propagates, the other split rows
  // choose per node by the row's stream, and either way a choice that empties a domain
  // is rolled back and the other side taken.  Without it a read of m_ownerIndex[k] after
  // m_ownerIndex[sender] = 1 needs k == sender, which no independent draw of k gives.
  const bool wrap_row = row < 32u && ((kWrapRows >> row) & 1u);
  if (row < 32u && (((or_rows >> row) & 1u) || wrap_row)) {
    for (uint32_t i = d.n; i-- > 0;) {
      const mgp_node &x = d.nd[i];
      if (x.op == MGP_OP_ITE && x.a >= 0 && d.bs[x.a] == BB && trace_on() && !d.ite_required(i) && !is_top(d.av[i], x.width))
        MGPD_TRACE("row %u ite node %u open, narrowed, not required (then %d else %d)\n", row, i, x.b, x.c);
      if (x.op != MGP_OP_ITE || x.a < 0 || d.bs[x.a] != BB || !d.ite_required(i)) continue;
      // (a wrap row takes the latest store first: a value required past the old state comes
      // from the writes of the transactions before, not from the initial storage)
      const bool then_first = row == kIteGreedyRow || wrap_row ||
                              ((fe_mix64(seed ^ fe_mix64(tag ^ i ^ ((uint64_t)row << 40))) >> 17) & 1u);
      for (int side = 0; side < 2; ++side) {
        const uint8_t want = (side == 0) == then_first ? BT : BF;
        const uint32_t mark = undo_log.size();
        work.clear();
        if (d.meetb(x.a, want) && d.run_from((uint32_t)x.a, split_budget, kSplitRounds) == 0 && !undo_log.over) {
          MGPD_TRACE("row %u ite node %u takes %s\n", row, i, want == BT ? "then" : "else");
          undo_log.clear();
          break;
        }
        MGPD_TRACE("row %u ite node %u: %s fails\n", row, i, want == BT ? "then" : "else");
        if (undo_log.over) return;
        d.rollback(mark);
      }
    }
  }
  // Fresh values of one injective function's applications are drawn pairwise distinct
  // (round 4). keccak is injective on the formula's models (inv(f(x)) == x,
  // keccak_function_manager.py:118-146), so two applications with different arguments need
  // different values (other functions -- calldata bytes, balances -- are not injective and
  // draw freely: two calldata bytes are often both 0); the lo / hi schedules used to give every application of a keccak
  // interval the same bound, and the inverse then read the first application's argument
  // (WalletLibrary's m_ownerIndex[owner] next to m_ownerIndex[sender]).  Applications with
  // equal arguments lose nothing: the evaluation gives a later one the earlier one's value.
  constexpr uint32_t kSeenUf = 64;
  uint32_t seen_fn[kSeenUf];
  V seen_v[kSeenUf];
  uint32_t n_seen = 0;
  auto taken = [&](uint32_t fn, const V &v) {
    for (uint32_t j = 0; j < n_seen; ++j)
      if (seen_fn[j] == fn && EQV(seen_v[j], v)) return true;
    return false;
  };
  for (uint32_t kk = 0; kk < P.n_slot; ++kk) {
    const uint32_t k = (drow & 1) ? P.n_slot - 1 - kk : kk;  // odd rows decide in reverse order
    const uint64_t key = fe_mix64(seed ^ fe_mix64(tag ^ ((uint64_t)c << 12) ^ P.slot[k]));
    const int32_t nk = P.node[k];
    // (on the original DAG: an application with a wide argument is a fresh variable in the
    // relaxed one the domain runs on)
    const mgp_node &on = (d.orig ? d.orig : d.nd)[nk];
    const uint32_t fn = on.p0;
    bool ufapp = false;  // an application of a function with an asserted inverse
    if (on.op == MGP_OP_UFAPP)
      for (uint32_t j = 0; j < d.n_inj && !ufapp; ++j) ufapp = d.inj[j].fn == fn;
    if (EQV(d.av[nk].lo, d.av[nk].hi)) {  // already one value: nothing to decide
      put(P.slot[k], d.av[nk].lo);
      if (ufapp && n_seen < kSeenUf) {
        seen_fn[n_seen] = fn;
        seen_v[n_seen++] = d.av[nk].lo;
      }
      continue;
    }
    V v = bv_zero();
    const uint32_t h0 = P.eqh_off[k], nh = P.eqh_off[k + 1] - h0;
    MGPD_TRACE("row %u draw slot %u (node %d)\n", row, P.slot[k], nk);
    for (uint32_t t = 0; t < kTries + nh; ++t) {
      if (t < nh) {
        v = P.eqh[h0 + (t + drow + (drow < 8u ? 0u : (uint32_t)(key >> 40))) % nh];
        if (!inside_av(d.av[nk], v)) continue;
      } else {
        const AV &a = d.av[nk];
        v = fe_sample_domain(a.z, a.o, a.lo, a.hi, P.width[k],
                             t > nh ? 3u + drow + t
                                    : (drow < 4 ? drow / 2
                                                : (uint32_t)(key % 3u) * 3u / 2u + (key % 3u == 2u ? 1u + drow : 0u)),
                             fe_mix64(key + t));
      }
      if (ufapp && taken(fn, v)) {  // step past the taken values along the domain's alignment
        const uint32_t al = ctz_ones(d.av[nk].z);
        const V step = SHL(ONE(), al < P.width[k] ? al : 0u);
        bool free = false;
        for (uint32_t r = 0; r < 4u && !free; ++r) {
          v = bv_mask(ADDV(v, step), P.width[k]);
          if (!inside_av(d.av[nk], v)) break;
          free = !taken(fn, v);
        }
        if (!free) continue;
      }
      const uint32_t mark = undo_log.size();
      work.clear();
      if (d.meet(nk, exact(v, P.width[k])) && d.run_from((uint32_t)nk, budget) == 0 && !undo_log.over) {
        undo_log.clear();
        if (ufapp && n_seen < kSeenUf) {
          seen_fn[n_seen] = fn;
          seen_v[n_seen++] = v;
        }
        break;
      }
      if (undo_log.over) return;
      d.rollback(mark);
    }
    put(P.slot[k], v);
  }
}

}  // namespace mgpd
