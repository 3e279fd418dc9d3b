/*
 * oracle.c — CPU restatement of the pre-filter semantics in plain C.
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY: linked by tests/, smoke() and
 * bench.py's cpu_baseline leg, never by the product library.
 *
 * Restates (independently of the HIP kernel, with 4 x 64-bit limbs and
 * unsigned __int128 arithmetic) what z3 computes for the laser.smt vocabulary:
 *   bvadd/bvsub/bvmul            mythril/laser/smt/bitvec.py:63-94
 *   bvudiv/bvurem/bvsrem         mythril/laser/smt/bitvec_helper.py:125-152
 *   bvsdiv (__truediv__)         mythril/laser/smt/bitvec.py:96-103
 *   shifts                       mythril/laser/smt/bitvec.py:232-246, bitvec_helper.py:21-22
 *   signed / unsigned compares   mythril/laser/smt/bitvec.py:138-180, bitvec_helper.py:43-80
 *   If / Concat / Extract        mythril/laser/smt/bitvec_helper.py:25-40, 93-122
 *   no-overflow predicates       mythril/laser/smt/bitvec_helper.py:168-214
 *   Bool connectives             mythril/laser/smt/bool.py:87-123
 *   UF apps (keccak pairs)       mythril/laser/ethereum/keccak_function_manager.py:56-69
 * at the DAG level (include/mgp_ir.h node lists — NOT the bytecode), plus
 * Keccak-256 (Keccak-f[1600], 0x01 padding) for keccak_function_manager.py:40-54.
 * SMT-LIB definitions for bvsdiv/bvsrem/bvsmod (msb case split).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mgp_ir.h"

typedef unsigned __int128 u128;
typedef struct { uint64_t l[4]; } w256;

static w256 z256(void) { w256 r = {{0, 0, 0, 0}}; return r; }
static w256 mask256(unsigned w) {
  w256 r;
  for (int i = 0; i < 4; ++i) {
    int lo = 64 * i;
    if ((int)w >= lo + 64) r.l[i] = ~0ull;
    else if ((int)w <= lo) r.l[i] = 0;
    else r.l[i] = (1ull << (w - lo)) - 1ull;
  }
  return r;
}
static w256 and256(w256 a, w256 b) { for (int i = 0; i < 4; ++i) a.l[i] &= b.l[i]; return a; }
static w256 or256(w256 a, w256 b) { for (int i = 0; i < 4; ++i) a.l[i] |= b.l[i]; return a; }
static w256 xor256(w256 a, w256 b) { for (int i = 0; i < 4; ++i) a.l[i] ^= b.l[i]; return a; }
static w256 not256(w256 a) { for (int i = 0; i < 4; ++i) a.l[i] = ~a.l[i]; return a; }
static int eq256(w256 a, w256 b) { return !((a.l[0] ^ b.l[0]) | (a.l[1] ^ b.l[1]) | (a.l[2] ^ b.l[2]) | (a.l[3] ^ b.l[3])); }
static int iszero256(w256 a) { return !(a.l[0] | a.l[1] | a.l[2] | a.l[3]); }
static int cmp256(w256 a, w256 b) {
  for (int i = 3; i >= 0; --i) {
    if (a.l[i] < b.l[i]) return -1;
    if (a.l[i] > b.l[i]) return 1;
  }
  return 0;
}
static w256 add256(w256 a, w256 b, int *carry) {
  w256 r;
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a.l[i] + b.l[i];
    r.l[i] = (uint64_t)c;
    c >>= 64;
  }
  if (carry) *carry = (int)c;
  return r;
}
static w256 sub256(w256 a, w256 b) { return add256(a, add256(not256(b), (w256){{1, 0, 0, 0}}, NULL), NULL); }
static w256 neg256(w256 a) { return sub256(z256(), a); }
/* full 512-bit product as two halves */
static void mul512(w256 a, w256 b, w256 *lo, w256 *hi) {
  uint64_t r[8] = {0};
  for (int i = 0; i < 4; ++i) {
    u128 c = 0;
    for (int j = 0; j < 4; ++j) {
      c += (u128)a.l[i] * b.l[j] + r[i + j];
      r[i + j] = (uint64_t)c;
      c >>= 64;
    }
    r[i + 4] = (uint64_t)c;
  }
  for (int i = 0; i < 4; ++i) {
    if (lo) lo->l[i] = r[i];
    if (hi) hi->l[i] = r[i + 4];
  }
}
static int bit256(w256 a, unsigned k) { return (int)((a.l[k >> 6] >> (k & 63)) & 1ull); }
static w256 shl256(w256 a, unsigned s) {
  w256 r = z256();
  if (s >= 256) return r;
  unsigned q = s >> 6, b = s & 63;
  for (int i = 3; i >= (int)q; --i) {
    uint64_t v = a.l[i - q] << b;
    if (b && i - (int)q - 1 >= 0) v |= a.l[i - q - 1] >> (64 - b);
    r.l[i] = v;
  }
  return r;
}
static w256 lshr256(w256 a, unsigned s) {
  w256 r = z256();
  if (s >= 256) return r;
  unsigned q = s >> 6, b = s & 63;
  for (int i = 0; i + (int)q < 4; ++i) {
    uint64_t v = a.l[i + q] >> b;
    if (b && i + q + 1 < 4) v |= a.l[i + q + 1] << (64 - b);
    r.l[i] = v;
  }
  return r;
}
static unsigned bitlen256(w256 a) {
  for (int i = 3; i >= 0; --i)
    if (a.l[i]) return 64u * (unsigned)i + 64u - (unsigned)__builtin_clzll(a.l[i]);
  return 0;
}
/* restoring binary long division over the significant bits */
static void udivrem256(w256 a, w256 b, w256 *q, w256 *r) {
  if (iszero256(b)) { *q = not256(z256()); *r = a; return; }
  w256 Q = z256(), R = z256();
  unsigned n = bitlen256(a);
  for (int k = (int)n - 1; k >= 0; --k) {
    R = shl256(R, 1);
    R.l[0] |= (uint64_t)bit256(a, (unsigned)k);
    if (cmp256(R, b) >= 0) {
      R = sub256(R, b);
      Q.l[k >> 6] |= 1ull << (k & 63);
    }
  }
  *q = Q;
  *r = R;
}

/* values are kept zero-extended at their width */
static w256 trunc_w(w256 a, unsigned w) { return and256(a, mask256(w)); }
static int msb_w(w256 a, unsigned w) { return bit256(a, w - 1); }
static w256 neg_w(w256 a, unsigned w) { return trunc_w(neg256(a), w); }
static w256 udiv_w(w256 s, w256 t, unsigned w) { w256 q, r; udivrem256(s, t, &q, &r); return trunc_w(q, w); }
static w256 urem_w(w256 s, w256 t, unsigned w) { w256 q, r; (void)w; udivrem256(s, t, &q, &r); return r; }
static w256 sdiv_w(w256 s, w256 t, unsigned w) {
  int ms = msb_w(s, w), mt = msb_w(t, w);
  if (!ms && !mt) return udiv_w(s, t, w);
  if (ms && !mt) return neg_w(udiv_w(neg_w(s, w), t, w), w);
  if (!ms && mt) return neg_w(udiv_w(s, neg_w(t, w), w), w);
  return udiv_w(neg_w(s, w), neg_w(t, w), w);
}
static w256 srem_w(w256 s, w256 t, unsigned w) {
  int ms = msb_w(s, w), mt = msb_w(t, w);
  if (!ms && !mt) return urem_w(s, t, w);
  if (ms && !mt) return neg_w(urem_w(neg_w(s, w), t, w), w);
  if (!ms && mt) return urem_w(s, neg_w(t, w), w);
  return neg_w(urem_w(neg_w(s, w), neg_w(t, w), w), w);
}
static w256 smod_w(w256 s, w256 t, unsigned w) {
  int ms = msb_w(s, w), mt = msb_w(t, w);
  w256 as = ms ? neg_w(s, w) : s, at = mt ? neg_w(t, w) : t;
  w256 u = urem_w(as, at, w);
  if (iszero256(u) || (!ms && !mt)) return u;
  if (ms && !mt) return trunc_w(add256(neg_w(u, w), t, NULL), w);
  if (!ms && mt) return trunc_w(add256(u, t, NULL), w);
  return neg_w(u, w);
}
static unsigned shamt(w256 s) {
  if (s.l[1] | s.l[2] | s.l[3] || s.l[0] >= 256) return 256;
  return (unsigned)s.l[0];
}
static w256 ashr_w(w256 a, w256 s, unsigned w) {
  unsigned k = shamt(s);
  int neg = msb_w(a, w);
  if (k >= w) return neg ? mask256(w) : z256();
  w256 r = lshr256(a, k);
  if (neg) r = or256(r, and256(mask256(w), not256(mask256(w - k))));
  return r;
}
static w256 sext_w(w256 a, unsigned from, unsigned to) {
  if (msb_w(a, from)) a = or256(a, and256(mask256(to), not256(mask256(from))));
  return a;
}
static int slt_w(w256 a, w256 b, unsigned w) {
  int ma = msb_w(a, w), mb = msb_w(b, w);
  if (ma != mb) return ma > mb;
  return cmp256(a, b) < 0;
}

static w256 from_u32(const uint32_t *p) {
  w256 r;
  for (int i = 0; i < 4; ++i) r.l[i] = (uint64_t)p[2 * i] | ((uint64_t)p[2 * i + 1] << 32);
  return r;
}

/* evaluate node i of a DAG (operands already evaluated); 0, or -2 when not evaluable */
static int eval_node(const mgp_node *nd, uint64_t i, const uint32_t *consts, uint64_t nc,
                     const uint32_t *xs /* n_vars*8 */, uint32_t n_vars, w256 *v, unsigned char *b,
                     uint16_t *wd) {
  {
    const mgp_node *x = &nd[i];
    unsigned w = x->width;
    w256 r = z256();
    int isbool = 0, bv = 0;
    switch (x->op) {
      case MGP_OP_VAR:
        if (x->p0 >= n_vars) return -2;
        r = trunc_w(from_u32(xs + 8u * x->p0), w); break;
      case MGP_OP_CONST:
        if (x->p0 >= nc) return -2;
        r = trunc_w(from_u32(consts + 8u * x->p0), w); break;
      case MGP_OP_TRUE: isbool = 1; bv = 1; break;
      case MGP_OP_FALSE: isbool = 1; bv = 0; break;
      case MGP_OP_ADD: r = trunc_w(add256(v[x->a], v[x->b], NULL), w); break;
      case MGP_OP_SUB: r = trunc_w(sub256(v[x->a], v[x->b]), w); break;
      case MGP_OP_MUL: mul512(v[x->a], v[x->b], &r, NULL); r = trunc_w(r, w); break;
      case MGP_OP_UDIV: r = udiv_w(v[x->a], v[x->b], w); break;
      case MGP_OP_UREM: r = urem_w(v[x->a], v[x->b], w); break;
      case MGP_OP_SDIV: r = sdiv_w(v[x->a], v[x->b], w); break;
      case MGP_OP_SREM: r = srem_w(v[x->a], v[x->b], w); break;
      case MGP_OP_SMOD: r = smod_w(v[x->a], v[x->b], w); break;
      case MGP_OP_AND: r = and256(v[x->a], v[x->b]); break;
      case MGP_OP_OR: r = or256(v[x->a], v[x->b]); break;
      case MGP_OP_XOR: r = xor256(v[x->a], v[x->b]); break;
      case MGP_OP_NOT: r = trunc_w(not256(v[x->a]), w); break;
      case MGP_OP_NEG: r = neg_w(v[x->a], w); break;
      case MGP_OP_SHL: { unsigned k = shamt(v[x->b]); r = k >= w ? z256() : trunc_w(shl256(v[x->a], k), w); break; }
      case MGP_OP_LSHR: { unsigned k = shamt(v[x->b]); r = k >= w ? z256() : lshr256(v[x->a], k); break; }
      case MGP_OP_ASHR: r = ashr_w(v[x->a], v[x->b], w); break;
      case MGP_OP_EXTRACT: r = trunc_w(lshr256(v[x->a], x->p1), x->p0 - x->p1 + 1); w = x->p0 - x->p1 + 1; break;
      case MGP_OP_CONCAT: r = or256(shl256(v[x->a], wd[x->b]), v[x->b]); break;
      case MGP_OP_ZEXT: r = v[x->a]; break;
      case MGP_OP_SEXT: r = sext_w(v[x->a], wd[x->a], w); break;
      case MGP_OP_ITE:
        if (b[x->b] != 2) { isbool = 1; bv = b[x->a] ? b[x->b] : b[x->c]; }
        else r = b[x->a] ? v[x->b] : v[x->c];
        break;
      case MGP_OP_EQ:
        isbool = 1;
        if (b[x->a] != 2) bv = b[x->a] == b[x->b];
        else bv = eq256(v[x->a], v[x->b]);
        break;
      case MGP_OP_ULT: isbool = 1; bv = cmp256(v[x->a], v[x->b]) < 0; break;
      case MGP_OP_ULE: isbool = 1; bv = cmp256(v[x->a], v[x->b]) <= 0; break;
      case MGP_OP_UGT: isbool = 1; bv = cmp256(v[x->a], v[x->b]) > 0; break;
      case MGP_OP_UGE: isbool = 1; bv = cmp256(v[x->a], v[x->b]) >= 0; break;
      case MGP_OP_SLT: isbool = 1; bv = slt_w(v[x->a], v[x->b], wd[x->a]); break;
      case MGP_OP_SLE: isbool = 1; bv = !slt_w(v[x->b], v[x->a], wd[x->a]); break;
      case MGP_OP_SGT: isbool = 1; bv = slt_w(v[x->b], v[x->a], wd[x->a]); break;
      case MGP_OP_SGE: isbool = 1; bv = !slt_w(v[x->a], v[x->b], wd[x->a]); break;
      case MGP_OP_UADD_NOOVF: {
        int c;
        w256 s = add256(v[x->a], v[x->b], &c);
        isbool = 1;
        bv = !c && eq256(s, trunc_w(s, wd[x->a]));
        break;
      }
      case MGP_OP_UMUL_NOOVF: {
        w256 lo, hi;
        mul512(v[x->a], v[x->b], &lo, &hi);
        isbool = 1;
        bv = iszero256(hi) && eq256(lo, trunc_w(lo, wd[x->a]));
        break;
      }
      case MGP_OP_USUB_NOUDF: isbool = 1; bv = cmp256(v[x->b], v[x->a]) <= 0; break;
      case MGP_OP_BAND: isbool = 1; bv = b[x->a] && b[x->b]; break;
      case MGP_OP_BOR: isbool = 1; bv = b[x->a] || b[x->b]; break;
      case MGP_OP_BXOR: isbool = 1; bv = b[x->a] != b[x->b]; break;
      case MGP_OP_BNOT: isbool = 1; bv = !b[x->a]; break;
      case MGP_OP_BITE: isbool = 1; bv = b[x->a] ? b[x->b] : b[x->c]; break;
      case MGP_OP_BEQ: isbool = 1; bv = b[x->a] == b[x->b]; break;
      case MGP_OP_UFAPP: {
        if (x->p1 >= n_vars) return -2;
        r = trunc_w(from_u32(xs + 8u * x->p1), w);
        for (uint64_t j = 0; j < i; ++j)
          if (nd[j].op == MGP_OP_UFAPP && nd[j].p0 == x->p0 && eq256(v[nd[j].a], v[x->a])) { r = v[j]; break; }
        break;
      }
      case MGP_OP_UFINV: {
        int found = 0;
        if (x->p1 >= n_vars) return -2;
        for (uint64_t j = 0; j < i && !found; ++j)
          if (nd[j].op == MGP_OP_UFINV && nd[j].p0 == x->p0 && eq256(v[nd[j].a], v[x->a])) { r = v[j]; found = 1; }
        for (uint64_t j = 0; j < i && !found; ++j)
          if (nd[j].op == MGP_OP_UFAPP && nd[j].p0 == x->p0 && eq256(v[j], v[x->a])) { r = v[nd[j].a]; found = 1; }
        if (!found) r = trunc_w(from_u32(xs + 8u * x->p1), w);
        break;
      }
      default:
        return -2;
    }
    if (isbool) { b[i] = (unsigned char)(bv ? 1 : 0); wd[i] = 1; v[i] = z256(); }
    else { b[i] = 2; wd[i] = (uint16_t)w; v[i] = r; }
  }
  return 0;
}

/* evaluate one state's DAG (values <= 256 bits) for one candidate; root (0/1) or -2 */
static int eval_state(const mgp_node *nd, uint64_t n, const uint32_t *consts, uint64_t nc,
                      const uint32_t *xs /* n_vars*8 */, uint32_t n_vars, w256 *v, unsigned char *b,
                      uint16_t *wd) {
  for (uint64_t i = 0; i < n; ++i)
    if (eval_node(nd, i, consts, nc, xs, n_vars, v, b, wd) != 0) return -2;
  return n ? (b[n - 1] == 1) : -2;
}

static int eval_one(const mgp_node *nd, uint64_t i, w256 *v, unsigned char *b, uint16_t *wd) {
  return eval_node(nd, i, NULL, 0, NULL, 0, v, b, wd);
}

/* ---------------------------------------------------------- wide values
 * A state with a value wider than 256 bits (512-bit mapping preimages Concat(key, slot),
 * keccak256_512 and its inverse, 257-bit overflow sums; include/mgp_ir.h "wide values")
 * is evaluated with MGP_MAX_WIDE-bit values: a w-bit VAR / CONST / fresh UF value is
 * ceil(w/256) consecutive 256-bit entries, low bits first.  Ops on values <= 256 bits
 * reuse the w256 helpers above; the ops the node format allows on wide values
 * (structural ops, EQ / unsigned compares, ADD / SUB / MUL, bitwise ops, UF arguments
 * and results) act on all limbs. */
#define WL (MGP_MAX_WIDE / 64)
typedef struct { uint64_t l[WL]; } wbig;

static wbig bz(void) { wbig r; memset(&r, 0, sizeof(r)); return r; }
static wbig b_trunc(wbig a, unsigned w) {
  for (unsigned i = 0; i < WL; ++i) {
    const unsigned lo = 64u * i;
    if (w <= lo) a.l[i] = 0;
    else if (w < lo + 64) a.l[i] &= (1ull << (w - lo)) - 1ull;
  }
  return a;
}
static wbig b_from256(w256 a) { wbig r = bz(); memcpy(r.l, a.l, sizeof(a.l)); return r; }
static w256 b_to256(wbig a) { w256 r; memcpy(r.l, a.l, sizeof(r.l)); return r; }
static wbig b_shl(wbig a, unsigned s) {
  wbig r = bz();
  if (s >= MGP_MAX_WIDE) return r;
  const unsigned q = s >> 6, b = s & 63;
  for (int i = WL - 1; i >= (int)q; --i) {
    uint64_t v = a.l[i - q] << b;
    if (b && i - (int)q - 1 >= 0) v |= a.l[i - q - 1] >> (64 - b);
    r.l[i] = v;
  }
  return r;
}
static wbig b_lshr(wbig a, unsigned s) {
  wbig r = bz();
  if (s >= MGP_MAX_WIDE) return r;
  const unsigned q = s >> 6, b = s & 63;
  for (unsigned i = 0; i + q < WL; ++i) {
    uint64_t v = a.l[i + q] >> b;
    if (b && i + q + 1 < WL) v |= a.l[i + q + 1] << (64 - b);
    r.l[i] = v;
  }
  return r;
}
static int b_cmp(wbig a, wbig b) {
  for (int i = WL - 1; i >= 0; --i) {
    if (a.l[i] < b.l[i]) return -1;
    if (a.l[i] > b.l[i]) return 1;
  }
  return 0;
}
static wbig b_add(wbig a, wbig b) {
  u128 c = 0;
  for (unsigned i = 0; i < WL; ++i) {
    c += (u128)a.l[i] + b.l[i];
    a.l[i] = (uint64_t)c;
    c >>= 64;
  }
  return a;
}
static wbig b_not(wbig a) { for (unsigned i = 0; i < WL; ++i) a.l[i] = ~a.l[i]; return a; }
static wbig b_sub(wbig a, wbig b) { wbig one = bz(); one.l[0] = 1; return b_add(a, b_add(b_not(b), one)); }
static wbig b_mul(wbig a, wbig b) {
  wbig r = bz();
  for (unsigned i = 0; i < WL; ++i) {
    if (!a.l[i]) continue;
    u128 c = 0;
    for (unsigned j = 0; i + j < WL; ++j) {
      c += (u128)a.l[i] * b.l[j] + r.l[i + j];
      r.l[i + j] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}
/* ceil(w/256) consecutive 256-bit entries starting at base[idx], low first */
static int b_entries(const uint32_t *base, uint64_t n_entries, uint64_t idx, unsigned w, wbig *out) {
  const unsigned k = (w + 255u) / 256u;
  if (idx + k > n_entries) return 0;
  wbig r = bz();
  for (unsigned j = 0; j < k; ++j) {
    w256 e = from_u32(base + 8u * (idx + j));
    for (int i = 0; i < 4 && 4 * j + i < WL; ++i) r.l[4 * j + i] = e.l[i];
  }
  *out = b_trunc(r, w);
  return 1;
}

static int eval_state_wide(const mgp_node *nd, uint64_t n, const uint32_t *consts, uint64_t nc,
                           const uint32_t *xs, uint32_t n_vars, wbig *v, unsigned char *b, uint16_t *wd) {
  for (uint64_t i = 0; i < n; ++i) {
    const mgp_node *x = &nd[i];
    unsigned w = x->width;
    wbig r = bz();
    int isbool = 0, bv = 0;
    const int wide_in = (x->a >= 0 && wd[x->a] > 256) || (x->b >= 0 && wd[x->b] > 256);
    switch (x->op) {
      case MGP_OP_VAR:
        if (!b_entries(xs, n_vars, x->p0, w, &r)) return -2;
        break;
      case MGP_OP_CONST:
        if (!b_entries(consts, nc, x->p0, w, &r)) return -2;
        break;
      case MGP_OP_TRUE: isbool = 1; bv = 1; break;
      case MGP_OP_FALSE: isbool = 1; bv = 0; break;
      case MGP_OP_ADD: r = b_trunc(b_add(v[x->a], v[x->b]), w); break;
      case MGP_OP_SUB: r = b_trunc(b_sub(v[x->a], v[x->b]), w); break;
      case MGP_OP_MUL: r = b_trunc(b_mul(v[x->a], v[x->b]), w); break;
      case MGP_OP_AND: for (unsigned k = 0; k < WL; ++k) r.l[k] = v[x->a].l[k] & v[x->b].l[k]; break;
      case MGP_OP_OR: for (unsigned k = 0; k < WL; ++k) r.l[k] = v[x->a].l[k] | v[x->b].l[k]; break;
      case MGP_OP_XOR: for (unsigned k = 0; k < WL; ++k) r.l[k] = v[x->a].l[k] ^ v[x->b].l[k]; break;
      case MGP_OP_NOT: r = b_trunc(b_not(v[x->a]), w); break;
      case MGP_OP_EXTRACT: w = x->p0 - x->p1 + 1; r = b_trunc(b_lshr(v[x->a], x->p1), w); break;
      case MGP_OP_CONCAT: r = b_trunc(b_add(b_shl(v[x->a], wd[x->b]), v[x->b]), w); break;
      case MGP_OP_ZEXT: r = v[x->a]; break;
      case MGP_OP_ITE:
        if (b[x->b] != 2) { isbool = 1; bv = b[x->a] ? b[x->b] : b[x->c]; }
        else r = b[x->a] ? v[x->b] : v[x->c];
        break;
      case MGP_OP_EQ:
        isbool = 1;
        if (b[x->a] != 2) bv = b[x->a] == b[x->b];
        else bv = b_cmp(v[x->a], v[x->b]) == 0;
        break;
      case MGP_OP_ULT: isbool = 1; bv = b_cmp(v[x->a], v[x->b]) < 0; break;
      case MGP_OP_ULE: isbool = 1; bv = b_cmp(v[x->a], v[x->b]) <= 0; break;
      case MGP_OP_UGT: isbool = 1; bv = b_cmp(v[x->a], v[x->b]) > 0; break;
      case MGP_OP_UGE: isbool = 1; bv = b_cmp(v[x->a], v[x->b]) >= 0; break;
      case MGP_OP_BAND: isbool = 1; bv = b[x->a] && b[x->b]; break;
      case MGP_OP_BOR: isbool = 1; bv = b[x->a] || b[x->b]; break;
      case MGP_OP_BXOR: isbool = 1; bv = b[x->a] != b[x->b]; break;
      case MGP_OP_BNOT: isbool = 1; bv = !b[x->a]; break;
      case MGP_OP_BITE: isbool = 1; bv = b[x->a] ? b[x->b] : b[x->c]; break;
      case MGP_OP_BEQ: isbool = 1; bv = b[x->a] == b[x->b]; break;
      case MGP_OP_UFAPP: {
        if (!b_entries(xs, n_vars, x->p1, w, &r)) return -2;
        for (uint64_t j = 0; j < i; ++j)
          if (nd[j].op == MGP_OP_UFAPP && nd[j].p0 == x->p0 && b_cmp(v[nd[j].a], v[x->a]) == 0) { r = v[j]; break; }
        break;
      }
      case MGP_OP_UFINV: {
        int found = 0;
        for (uint64_t j = 0; j < i && !found; ++j)
          if (nd[j].op == MGP_OP_UFINV && nd[j].p0 == x->p0 && b_cmp(v[nd[j].a], v[x->a]) == 0) { r = v[j]; found = 1; }
        for (uint64_t j = 0; j < i && !found; ++j)
          if (nd[j].op == MGP_OP_UFAPP && nd[j].p0 == x->p0 && b_cmp(v[j], v[x->a]) == 0) { r = v[nd[j].a]; found = 1; }
        if (!found && !b_entries(xs, n_vars, x->p1, w, &r)) return -2;
        break;
      }
      default: {
        /* every other op acts on values <= 256 bits: the w256 evaluator's rules */
        if (wide_in || w > 256) return -2;
        const mgp_node y = {x->op, 0, (uint16_t)w, x->a >= 0 ? 0 : -1, x->b >= 0 ? 1 : -1, x->c >= 0 ? 2 : -1,
                            x->p0, x->p1};
        mgp_node tmp[4];
        w256 tv[4];
        unsigned char tb[4];
        uint16_t tw[4];
        const int32_t ops[3] = {x->a, x->b, x->c};
        for (int k = 0; k < 3; ++k) {
          tmp[k].op = MGP_OP_FALSE;  /* placeholders; their values are set directly */
          if (ops[k] >= 0) { tv[k] = b_to256(v[ops[k]]); tb[k] = b[ops[k]]; tw[k] = wd[ops[k]]; }
          else { tv[k] = z256(); tb[k] = 0; tw[k] = 1; }
        }
        tmp[3] = y;
        if (eval_one(tmp, 3, tv, tb, tw) != 0) return -2;
        if (tb[3] != 2) { isbool = 1; bv = tb[3]; }
        else { r = b_from256(tv[3]); w = tw[3]; }
        break;
      }
    }
    if (isbool) { b[i] = (unsigned char)(bv ? 1 : 0); wd[i] = 1; v[i] = bz(); }
    else { b[i] = 2; wd[i] = (uint16_t)w; v[i] = r; }
  }
  return n ? (b[n - 1] == 1) : -2;
}

static int state_is_wide(const mgp_node *nd, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i)
    if (nd[i].width > 256) return 1;
  return 0;
}

/* first satisfying candidate per state; cands AoS [state][cand][var][8] */
int oracle_first_sat(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                     const uint32_t *consts, const uint64_t *const_offsets, const uint32_t *cands,
                     uint32_t n_cand, uint32_t n_vars, int32_t *out, int full /* evaluate every candidate */) {
  int rc = 0;
#pragma omp parallel
  {
    uint64_t cap = 0, wcap = 0;
    w256 *v = NULL;
    wbig *vw = NULL;
    unsigned char *b = NULL;
    uint16_t *wd = NULL;
#pragma omp for schedule(dynamic, 16)
    for (int64_t s = 0; s < (int64_t)n_states; ++s) {
      const uint64_t n0 = node_offsets[s], n = node_offsets[s + 1] - n0;
      if (n > cap) {
        free(v); free(b); free(wd);
        cap = n;
        v = (w256 *)malloc(cap * sizeof(w256));
        b = (unsigned char *)malloc(cap);
        wd = (uint16_t *)malloc(cap * sizeof(uint16_t));
      }
      const int wide = state_is_wide(nodes + n0, n);
      if (wide && n > wcap) {
        free(vw);
        wcap = n;
        vw = (wbig *)malloc(wcap * sizeof(wbig));
      }
      int32_t res = -1;
      for (uint32_t c = 0; c < n_cand; ++c) {
        const uint32_t *xs = cands + ((uint64_t)s * n_cand + c) * n_vars * 8u;
        const uint32_t *cs = consts + const_offsets[s] * 8u;
        const uint64_t nc = const_offsets[s + 1] - const_offsets[s];
        int r = wide ? eval_state_wide(nodes + n0, n, cs, nc, xs, n_vars, vw, b, wd)
                     : eval_state(nodes + n0, n, cs, nc, xs, n_vars, v, b, wd);
        if (r == -2) { res = -2; break; }
        if (r == 1 && res < 0) { res = (int32_t)c; if (!full) break; }
      }
      out[s] = res;
    }
    free(v); free(vw); free(b); free(wd);
  }
  return rc;
}

/* ------------------------------------------------------------- Keccak */
static const uint64_t RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
static uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }
static void keccakf(uint64_t A[25]) {
  for (int r = 0; r < 24; ++r) {
    uint64_t C[5], D[5], B[25];
    for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rol(A[x + 5 * y], RHO[x + 5 * y]);
    for (int y = 0; y < 5; ++y)
      for (int x = 0; x < 5; ++x) A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    A[0] ^= RC[r];
  }
}
static void keccak256_one(const uint8_t *p, uint32_t len, uint8_t *out) {
  uint64_t A[25];
  uint8_t blk[136];
  memset(A, 0, sizeof(A));
  uint32_t off = 0;
  for (;;) {
    uint32_t take = len - off >= 136 ? 136 : len - off;
    memset(blk, 0, sizeof(blk));
    memcpy(blk, p + off, take);
    int last = take < 136;
    if (last) { blk[take] ^= 0x01; blk[135] ^= 0x80; }
    for (int k = 0; k < 17; ++k) {
      uint64_t v = 0;
      for (int b = 7; b >= 0; --b) v = (v << 8) | blk[8 * k + b];
      A[k] ^= v;
    }
    keccakf(A);
    off += take;
    if (last) break;
  }
  for (int k = 0; k < 4; ++k)
    for (int b = 0; b < 8; ++b) out[8 * k + b] = (uint8_t)(A[k] >> (8 * b));
}
int oracle_keccak256(const uint8_t *in, uint64_t n, uint32_t len, uint32_t stride, uint8_t *out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) keccak256_one(in + (uint64_t)i * stride, len, out + 32u * (uint64_t)i);
  return 0;
}
/* benchmark preimages, same definition as mgp_fill_mapping_preimages_dev */
static uint64_t sm64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
int oracle_mapping_preimages(uint8_t *out, uint64_t first, uint64_t n, uint64_t seed) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    uint8_t *b = out + 64u * (uint64_t)i;
    uint64_t g = first + (uint64_t)i;
    uint64_t x0 = sm64(seed + g), x1 = sm64(x0), x2 = sm64(x1);
    memset(b, 0, 64);
    for (int k = 0; k < 8; ++k) b[31 - k] = (uint8_t)(x0 >> (8 * k));
    for (int k = 0; k < 8; ++k) b[23 - k] = (uint8_t)(x1 >> (8 * k));
    for (int k = 0; k < 4; ++k) b[15 - k] = (uint8_t)(x2 >> (8 * k));
    b[63] = (uint8_t)(g & 7u);
  }
  return 0;
}
