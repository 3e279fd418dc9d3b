// mgp_bv.h — 256-bit bit-vector arithmetic on 8 x u32 little-endian limbs.
//
// One candidate model per lane: every value lives in 8 VGPRs, every helper is
// straight-line code with constant limb indices (no runtime-indexed register
// arrays, which hipcc would demote to scratch), carries go through
// v_add_co/v_addc_co (__builtin_addc/__builtin_subc) and funnel shifts through
// v_alignbit_b32.  The same code compiles for the host (the synthetic
// generator uses it to plant witnesses); the independent checker lives in
// oracle/, not here.
//
// Semantics are z3 / SMT-LIB bit-vector semantics at width 256; narrower
// widths are handled by the caller (zero-extended storage, sign-extend before
// signed ops, mask after) — see mgp_kernels.hip.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MGP_HD __host__ __device__ __forceinline__
#else
#define MGP_HD static inline
#endif

struct U256 {
  uint32_t w[8];
};

MGP_HD uint32_t mgp_funnel_r(uint32_t hi, uint32_t lo, uint32_t s) {
  // low 32 bits of ({hi,lo} >> (s & 31))
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (s & 31));
#endif
}

#if defined(__clang__)
MGP_HD uint32_t mgp_addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t *cout) {
  return __builtin_addc(a, b, cin, cout);
}
MGP_HD uint32_t mgp_subc(uint32_t a, uint32_t b, uint32_t bin, uint32_t *bout) {
  return __builtin_subc(a, b, bin, bout);
}
#else
MGP_HD uint32_t mgp_addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t *cout) {
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
MGP_HD uint32_t mgp_subc(uint32_t a, uint32_t b, uint32_t bin, uint32_t *bout) {
  uint64_t s = (uint64_t)a - b - bin;
  *bout = (uint32_t)(s >> 63);
  return (uint32_t)s;
}
#endif

MGP_HD U256 bv_zero() {
  U256 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = 0u;
  return r;
}
MGP_HD U256 bv_ones() {
  U256 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = 0xFFFFFFFFu;
  return r;
}
MGP_HD U256 bv_small(uint32_t v) {
  U256 r = bv_zero();
  r.w[0] = v;
  return r;
}

// limb mask for width w (1..256)
MGP_HD uint32_t bv_limb_mask(uint32_t w, int l) {
  int lo = 32 * l;
  if ((int)w >= lo + 32) return 0xFFFFFFFFu;
  if ((int)w <= lo) return 0u;
  return (1u << (w - lo)) - 1u;
}
MGP_HD U256 bv_mask(U256 a, uint32_t w) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] &= bv_limb_mask(w, i);
  return a;
}

MGP_HD U256 bv_add(const U256 &a, const U256 &b, uint32_t *carry_out) {
  U256 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = mgp_addc(a.w[i], b.w[i], c, &c);
  if (carry_out) *carry_out = c;
  return r;
}
MGP_HD U256 bv_sub(const U256 &a, const U256 &b, uint32_t *borrow_out) {
  U256 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = mgp_subc(a.w[i], b.w[i], c, &c);
  if (borrow_out) *borrow_out = c;
  return r;
}
MGP_HD U256 bv_neg(const U256 &a) { return bv_sub(bv_zero(), a, nullptr); }
MGP_HD U256 bv_not(U256 a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] = ~a.w[i];
  return a;
}
MGP_HD U256 bv_and(U256 a, const U256 &b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] &= b.w[i];
  return a;
}
MGP_HD U256 bv_or(U256 a, const U256 &b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] |= b.w[i];
  return a;
}
MGP_HD U256 bv_xor(U256 a, const U256 &b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] ^= b.w[i];
  return a;
}
MGP_HD U256 bv_sel(bool c, const U256 &a, const U256 &b) {
  U256 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = c ? a.w[i] : b.w[i];
  return r;
}

MGP_HD bool bv_is_zero(const U256 &a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.w[i];
  return o == 0u;
}
MGP_HD bool bv_eq(const U256 &a, const U256 &b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.w[i] ^ b.w[i];
  return o == 0u;
}
MGP_HD bool bv_ult(const U256 &a, const U256 &b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) (void)mgp_subc(a.w[i], b.w[i], c, &c);
  return c != 0u;
}
MGP_HD bool bv_slt(U256 a, U256 b) {
  a.w[7] ^= 0x80000000u;
  b.w[7] ^= 0x80000000u;
  return bv_ult(a, b);
}
MGP_HD bool bv_sign(const U256 &a) { return (a.w[7] >> 31) != 0u; }

// shift amount of a 256-bit shift operand, saturated at 256
MGP_HD uint32_t bv_shift_amount(const U256 &s) {
  uint32_t hi = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i) hi |= s.w[i];
  return (hi != 0u || s.w[0] >= 256u) ? 256u : s.w[0];
}

// Variable shifts are branch-free: three limb-granular select stages
// (v_cndmask) and one funnel stage (v_alignbit), so a per-lane shift amount
// costs no exec-mask manipulation and no scalar work.
// logical / arithmetic right shift by s (0..256); fill = 0 or 0xFFFFFFFF
MGP_HD U256 bv_shr_fill(U256 a, uint32_t s, uint32_t fill) {
  const bool all = s >= 256u;
  const uint32_t k = s >> 5, b = s & 31u;
  const bool k4 = (k & 4u) != 0u, k2 = (k & 2u) != 0u, k1 = (k & 1u) != 0u;
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] = k4 ? ((i + 4 < 8) ? a.w[i + 4] : fill) : a.w[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] = k2 ? ((i + 2 < 8) ? a.w[i + 2] : fill) : a.w[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] = k1 ? ((i + 1 < 8) ? a.w[i + 1] : fill) : a.w[i];
  U256 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t v = mgp_funnel_r((i + 1 < 8) ? a.w[i + 1] : fill, a.w[i], b);
    r.w[i] = all ? fill : v;
  }
  return r;
}
MGP_HD U256 bv_lshr(const U256 &a, uint32_t s) { return bv_shr_fill(a, s, 0u); }
MGP_HD U256 bv_ashr(const U256 &a, uint32_t s) {
  return bv_shr_fill(a, s, bv_sign(a) ? 0xFFFFFFFFu : 0u);
}
MGP_HD U256 bv_shl(U256 a, uint32_t s) {
  const bool all = s >= 256u;
  const uint32_t k = s >> 5, b = s & 31u;
  const bool k4 = (k & 4u) != 0u, k2 = (k & 2u) != 0u, k1 = (k & 1u) != 0u;
#pragma unroll
  for (int i = 7; i >= 0; --i) a.w[i] = k4 ? ((i >= 4) ? a.w[i - 4] : 0u) : a.w[i];
#pragma unroll
  for (int i = 7; i >= 0; --i) a.w[i] = k2 ? ((i >= 2) ? a.w[i - 2] : 0u) : a.w[i];
#pragma unroll
  for (int i = 7; i >= 0; --i) a.w[i] = k1 ? ((i >= 1) ? a.w[i - 1] : 0u) : a.w[i];
  U256 r;
  const uint32_t rb = (32u - b) & 31u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t v = mgp_funnel_r(a.w[i], (i >= 1) ? a.w[i - 1] : 0u, rb);
    r.w[i] = all ? 0u : (b == 0u ? a.w[i] : v);
  }
  return r;
}
// shift left by one, shifting in bit `in`
MGP_HD U256 bv_shl1(const U256 &a, uint32_t in) {
  U256 r;
#pragma unroll
  for (int i = 7; i >= 1; --i) r.w[i] = mgp_funnel_r(a.w[i], a.w[i - 1], 31u);
  r.w[0] = (a.w[0] << 1) | in;
  return r;
}
MGP_HD U256 bv_shr1(const U256 &a) {
  U256 r;
#pragma unroll
  for (int i = 0; i < 7; ++i) r.w[i] = mgp_funnel_r(a.w[i + 1], a.w[i], 1u);
  r.w[7] = a.w[7] >> 1;
  return r;
}

MGP_HD uint32_t bv_clz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return x ? (uint32_t)__builtin_clz(x) : 32u;
#else
  return x ? (uint32_t)__builtin_clz(x) : 32u;
#endif
}
// number of significant bits (0 for zero)
MGP_HD uint32_t bv_bitlen(const U256 &a) {
  uint32_t n = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (a.w[i] != 0u) n = 32u * (uint32_t)i + 32u - bv_clz32(a.w[i]);
  return n;
}

// low 256 bits of a*b (schoolbook, 36 limb products)
MGP_HD U256 bv_mul(const U256 &a, const U256 &b) {
  U256 r = bv_zero();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; i + j < 8; ++j) {
      uint64_t t = (uint64_t)a.w[i] * b.w[j] + r.w[i + j] + carry;
      r.w[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
  }
  return r;
}
// full 512-bit product; returns the high 256 bits, low bits in *lo
MGP_HD U256 bv_mul_full(const U256 &a, const U256 &b, U256 *lo) {
  uint32_t r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = 0u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t t = (uint64_t)a.w[i] * b.w[j] + r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + 8] = (uint32_t)carry;
  }
  U256 hi;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (lo) lo->w[i] = r[i];
    hi.w[i] = r[i + 8];
  }
  return hi;
}

#if defined(__HIP_DEVICE_COMPILE__)
MGP_HD bool mgp_wave_any(bool p) { return __ballot(p) != 0ull; }
#else
MGP_HD bool mgp_wave_any(bool p) { return p; }
#endif

// One quotient digit of Knuth's algorithm D (TAOCP 4.3.1) at a compile-time
// digit position J over the normalised 16-limb dividend u and 8-limb divisor v
// (v.w[7] has its top bit set).  qhat comes from a double-precision estimate
// of (u[J+8]:u[J+7]) / v7 (exact to +-1, fixed with one integer correction
// each way), refined with v6, then multiply-subtract with a rare add-back.
template <int J>
MGP_HD uint32_t bv_knuth_digit(uint32_t (&u)[16], const U256 &v, double inv_v7) {
  const uint32_t v7 = v.w[7], v6 = v.w[6];
  const uint64_t num = ((uint64_t)u[J + 8] << 32) | u[J + 7];
  // qhat = min(floor(num / v7), B - 1): double estimate, one integer fix each way
  const double dn = (double)u[J + 8] * 4294967296.0 + (double)u[J + 7];
  uint64_t qhat = (uint64_t)(dn * inv_v7);
  qhat = qhat > 0xFFFFFFFFull ? 0xFFFFFFFFull : qhat;
  {
    const int64_t r0 = (int64_t)(num - qhat * v7);
    qhat = r0 < 0 ? qhat - 1u : (r0 >= (int64_t)v7 && qhat < 0xFFFFFFFFull ? qhat + 1u : qhat);
  }
  uint64_t rhat = num - qhat * v7;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const bool dec = rhat < 0x100000000ull && qhat * v6 > ((rhat << 32) | u[J + 6]);
    qhat = dec ? qhat - 1u : qhat;
    rhat = dec ? rhat + v7 : rhat;
  }
  // u[J .. J+8] -= qhat * v
  uint32_t borrow = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t p = qhat * v.w[i] + hi;
    hi = (uint32_t)(p >> 32);
    u[J + i] = mgp_subc(u[J + i], (uint32_t)p, borrow, &borrow);
  }
  u[J + 8] = mgp_subc(u[J + 8], hi, borrow, &borrow);
  if (borrow) {  // qhat was one too large (probability ~2^-31): add v back
    --qhat;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) u[J + i] = mgp_addc(u[J + i], v.w[i], c, &c);
    u[J + 8] += c;
  }
  return (uint32_t)qhat;
}

template <int J>
MGP_HD void bv_knuth_step(uint32_t (&u)[16], const U256 &v, double inv_v7, uint32_t ndig, U256 &q) {
  // digit J of every lane is zero unless 32*J <= bitlen(a) - bitlen(b); skip it
  // when that holds for no lane of the wave (uniform branch)
  if (mgp_wave_any((uint32_t)J < ndig)) q.w[J] = bv_knuth_digit<J>(u, v, inv_v7);
}

// unsigned division with remainder; b == 0 -> q = 2^256-1, r = a (z3 bvudiv/bvurem)
// Knuth D with 32-bit digits over the fixed 512/256-bit shapes: every limb
// index is a compile-time constant, so all of u, v and q stay in VGPRs.
MGP_HD void bv_udivrem(const U256 &a, const U256 &b, U256 *q_out, U256 *r_out) {
  const uint32_t la = bv_bitlen(a), lb = bv_bitlen(b);
  U256 q = bv_zero(), r = a;
  const bool divides = lb != 0u && la >= lb;
  if (mgp_wave_any(divides)) {
    const uint32_t s = divides ? 256u - lb : 0u;  // normalisation shift
    const U256 v = bv_shl(divides ? b : bv_ones(), s);
    const U256 ulo = bv_shl(a, s);
    const U256 uhi = s ? bv_lshr(a, 256u - s) : bv_zero();
    uint32_t u[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      u[i] = ulo.w[i];
      u[i + 8] = uhi.w[i];
    }
    const double inv_v7 = 1.0 / (double)v.w[7];
    const uint32_t ndig = divides ? ((la - lb) >> 5) + 1u : 0u;
    bv_knuth_step<7>(u, v, inv_v7, ndig, q);
    bv_knuth_step<6>(u, v, inv_v7, ndig, q);
    bv_knuth_step<5>(u, v, inv_v7, ndig, q);
    bv_knuth_step<4>(u, v, inv_v7, ndig, q);
    bv_knuth_step<3>(u, v, inv_v7, ndig, q);
    bv_knuth_step<2>(u, v, inv_v7, ndig, q);
    bv_knuth_step<1>(u, v, inv_v7, ndig, q);
    bv_knuth_step<0>(u, v, inv_v7, ndig, q);
    U256 rn;
#pragma unroll
    for (int i = 0; i < 8; ++i) rn.w[i] = u[i];
    if (divides) r = bv_lshr(rn, s);
    if (!divides) q = bv_zero();
  }
  if (lb == 0u) q = bv_ones();
  *q_out = q;
  *r_out = r;
}

MGP_HD U256 bv_abs(const U256 &a) { return bv_sign(a) ? bv_neg(a) : a; }

// signed ops on 256-bit two's complement (SMT-LIB definitions)
MGP_HD U256 bv_sdiv(const U256 &a, const U256 &b) {
  bool sa = bv_sign(a), sb = bv_sign(b);
  U256 q, r;
  bv_udivrem(bv_abs(a), bv_abs(b), &q, &r);
  return (sa != sb) ? bv_neg(q) : q;
}
MGP_HD U256 bv_srem(const U256 &a, const U256 &b) {
  bool sa = bv_sign(a);
  U256 q, r;
  bv_udivrem(bv_abs(a), bv_abs(b), &q, &r);
  return sa ? bv_neg(r) : r;
}
MGP_HD U256 bv_smod(const U256 &a, const U256 &b) {
  bool sa = bv_sign(a), sb = bv_sign(b);
  U256 q, u;
  bv_udivrem(bv_abs(a), bv_abs(b), &q, &u);
  if (bv_is_zero(u) || (!sa && !sb)) return u;
  if (sa && !sb) return bv_add(bv_neg(u), b, nullptr);
  if (!sa && sb) return bv_add(u, b, nullptr);
  return bv_neg(u);
}

// sign-extend a value of width w (stored zero-extended) to 256 bits
MGP_HD U256 bv_sext(U256 a, uint32_t w) {
  if (w >= 256u) return a;
  uint32_t bit = 0u, li = (w - 1u) >> 5, bi = (w - 1u) & 31u;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if ((uint32_t)i == li) bit = (a.w[i] >> bi) & 1u;  // constant limb index
  if (bit) {
#pragma unroll
    for (int i = 0; i < 8; ++i) a.w[i] |= ~bv_limb_mask(w, i);
  }
  return a;
}
