// mgp_fe_sample.h — drawing candidate values from a refined abstract value, shared by
// the host (guided candidates, mgp_refute.cpp; the host candidate generator,
// mgp_cands.cpp) and the device candidate generator (mgp_fe_cands_kernel), so the two
// generators stay bit-identical.
//
// An abstract value is known bits (z = known-zero mask, o = known-one mask) x an
// unsigned interval [lo, hi] (mgp_refute.cpp).  Row 0 takes lo, row 1 hi, row 2 lo + 1;
// later rows a draw inside the interval (for a span of more than 64 bits: a full-width
// draw when the interval covers half the values or more, else lo plus a draw below the
// span) with the known bits forced when that stays inside.
#pragma once
#include <stdint.h>

#include "mgp_bv.h"

MGP_HD uint64_t fe_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

MGP_HD U256 fe_sample_domain(const U256 &z, const U256 &o, const U256 &lo, const U256 &hi, uint32_t w,
                             uint32_t row, uint64_t r0) {
  U256 v;
  uint64_t r = r0;
  for (int l = 0; l < 8; ++l) {
    if ((l & 1) == 0) r = fe_mix64(r);
    v.w[l] = (uint32_t)(r >> (32 * (l & 1)));
  }
  v = bv_mask(v, w);
  const U256 span = bv_sub(hi, lo, nullptr);
  if (row == 0) return lo;
  if (row == 1) return hi;
  U256 x;
  bool small = true;
  for (int l = 2; l < 8; ++l) small = small && span.w[l] == 0u;
  if (small) {
    const uint64_t sp = ((uint64_t)span.w[1] << 32) | span.w[0];
    const uint64_t h = fe_mix64(r0 ^ 0x5851F42D4C957F2Dull);
    const uint64_t k = (row == 2) ? 1u : (sp == ~0ull ? h : h % (sp + 1u));
    U256 kk = bv_zero();
    kk.w[0] = (uint32_t)k;
    kk.w[1] = (uint32_t)(k >> 32);
    x = bv_add(lo, kk, nullptr);
    if (bv_ult(hi, x)) x = hi;
  } else {
    // wide interval: a full-width draw when the interval covers at least half the width's
    // values; else lo + a draw below the span (round 4: a narrow interval high in the range,
    // e.g. a keccak manager interval of 2^123 values near 2^256, used to get lo or hi here,
    // neither of which keeps the interval's alignment)
    const uint32_t bl = bv_bitlen(span);
    if (bl >= w) {
      x = v;
    } else {
      U256 d = bv_mask(v, bl);
      if (bv_ult(span, d)) d = bv_mask(v, bl - 1u);
      x = bv_add(lo, d, nullptr);
    }
  }
  U256 yw = bv_mask(bv_or(bv_and(x, bv_not(z)), o), w);
  if (!bv_ult(yw, lo) && !bv_ult(hi, yw)) return yw;
  if (!small && bv_ult(yw, lo)) {
    // forcing known-zero low bits (an alignment) dropped below lo: one alignment step up
    uint32_t a = 0;
    while (a < w && ((z.w[a >> 5] >> (a & 31)) & 1u)) ++a;
    if (a > 0 && a < w) {
      const U256 up = bv_mask(bv_or(bv_and(bv_add(yw, bv_shl(bv_small(1u), a), nullptr), bv_not(z)), o), w);
      if (!bv_ult(up, lo) && !bv_ult(hi, up)) return up;
    }
  }
  return (small || (!bv_ult(x, lo) && !bv_ult(hi, x))) ? x : ((row & 1) ? hi : lo);
}

// v inside the abstract value (interval and known bits)
MGP_HD bool fe_inside(const U256 &z, const U256 &o, const U256 &lo, const U256 &hi, const U256 &v) {
  return !bv_ult(v, lo) && !bv_ult(hi, v) && bv_is_zero(bv_and(v, z)) && bv_eq(bv_and(v, o), o);
}
