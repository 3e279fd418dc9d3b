// mgp_cands.cpp — candidate assignments for the GPU witness search (host side).
//
// The candidates one state is evaluated on (mythril_amd/dag.py make_candidates):
// row 0 is left for the parent state's witness when there is one (a successor only
// adds constraints to its parent, svm.py:251-255), then the first harvested hint of
// every variable, the same row with the x == y aliases applied, then a seeded
// mixture per variable: 35 % harvested hint, 25 % pool (state constants and their
// neighbours +-1, LASER's actor addresses and boundary values), 15 % alias (an x == y
// partner, else the next equal-width variable from a random start), 25 % uniform.  Every value is masked to its slot width.
// A pinned-constant slot (var_kind 2, mgp_front.cpp) holds its hint 0 in every row.
// With domains (mgp_refute_domains), every other mixture row draws the variables that
// have a refined abstract value from it (mgp_fe_sample.h).
// States are independent (OpenMP); the stream is splitmix64 keyed by (seed, state tag,
// row, variable), so the result does not depend on the thread count; with state_keys the
// tag is the state's content key, so it does not depend on the batch either.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/mgp.h"
#include "mgp_fe_sample.h"

namespace {
inline uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void add_small(const uint32_t *a, int64_t d, uint32_t *r) {  // r = a + d mod 2^256, d = +-1
  uint64_t carry = d > 0 ? 1u : 0u;
  const uint32_t ext = d < 0 ? 0xFFFFFFFFu : 0u;  // -1 = all ones
  for (int l = 0; l < 8; ++l) {
    const uint64_t s = (uint64_t)a[l] + ext + carry;
    r[l] = (uint32_t)s;
    carry = s >> 32;
  }
}

void mask_to(uint32_t *v, uint32_t w) {
  for (int l = 0; l < 8; ++l) {
    const int lo = 32 * l;
    const uint32_t m = (int)w >= lo + 32 ? 0xFFFFFFFFu : ((int)w <= lo ? 0u : ((1u << (w - lo)) - 1u));
    v[l] &= m;
  }
}
}  // namespace

extern "C" int mgp_make_candidates(uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                                   const uint64_t *var_off, const uint32_t *var_width, const uint8_t *var_kind,
                                   const uint64_t *hint_off, const uint32_t *hints,
                                   const uint64_t *alias_off, const uint32_t *aliases,
                                   const uint64_t *const_off, const uint32_t *consts,
                                   const uint32_t *fixed_pool, uint32_t n_fixed,
                                   const uint8_t *has_parent, const uint32_t *dom, const uint64_t *state_keys,
                                   uint32_t *out) {
  if (!var_off || !hint_off || !alias_off || !const_off || !out || (n_states && !has_parent)) return MGP_E_ARG;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const uint64_t v0 = var_off[s], V = var_off[s + 1] - v0;
    // the state's stream tag: its content key (MGP_FE_STATE_KEY) when given, so the rows do
    // not depend on the state's position in the batch; else its index
    const uint64_t tag = state_keys ? state_keys[s] : (uint64_t)s << 40;
    uint32_t *o = out + (uint64_t)s * n_cand * n_vars * 8u;
    // uniform everywhere first (also the padding variables of narrower states)
    for (uint32_t c = 0; c < n_cand; ++c)
      for (uint32_t v = 0; v < n_vars; ++v) {
        uint32_t *d = o + ((uint64_t)c * n_vars + v) * 8u;
        uint64_t k = mix(seed ^ mix(tag ^ ((uint64_t)c << 16) ^ v));
        for (int l = 0; l < 8; l += 2) {
          k = mix(k);
          d[l] = (uint32_t)k;
          d[l + 1] = (uint32_t)(k >> 32);
        }
      }
    if (V == 0 || V > n_vars) continue;
    // pool: constants, +1, -1, fixed values
    const uint64_t c0 = const_off[s], nc = const_off[s + 1] - c0;
    std::vector<uint32_t> pool((3 * nc + n_fixed) * 8u);
    for (uint64_t i = 0; i < nc; ++i) {
      memcpy(&pool[i * 8u], consts + (c0 + i) * 8u, 32);
      add_small(consts + (c0 + i) * 8u, 1, &pool[(nc + i) * 8u]);
      add_small(consts + (c0 + i) * 8u, -1, &pool[(2 * nc + i) * 8u]);
    }
    if (n_fixed) memcpy(&pool[3 * nc * 8u], fixed_pool, (size_t)n_fixed * 32u);
    const uint64_t n_pool = 3 * nc + n_fixed;
    const uint64_t a0 = alias_off[s], na = alias_off[s + 1] - a0;
    auto cell = [&](uint32_t c, uint64_t v) { return o + ((uint64_t)c * n_vars + v) * 8u; };
    auto n_hint = [&](uint64_t v) { return hint_off[v0 + v + 1] - hint_off[v0 + v]; };
    auto hint = [&](uint64_t v, uint64_t j) { return hints + (hint_off[v0 + v] + j) * 8u; };
    uint32_t row = has_parent[s] ? 1u : 0u;
    for (int structured = 0; structured < 2 && row < n_cand; ++structured, ++row) {
      for (uint64_t v = 0; v < V; ++v)
        if (n_hint(v)) memcpy(cell(row, v), hint(v, 0), 32);
      if (structured)
        for (uint64_t a = 0; a < na; ++a) {
          const uint32_t dst = aliases[2 * (a0 + a)], src = aliases[2 * (a0 + a) + 1];
          if (dst < V && src < V && var_width[v0 + dst] == var_width[v0 + src] && n_hint(src) && !n_hint(dst))
            memcpy(cell(row, dst), cell(row, src), 32);
        }
    }
    std::vector<uint32_t> srcs;
    std::vector<uint8_t> pend(V);
    const uint32_t mix0 = row;  // first mixture row
    for (uint32_t c = row; c < n_cand; ++c) {
      for (uint64_t v = 0; v < V; ++v) {
        const uint64_t k = mix(seed ^ 0xA5A5A5A5ull ^ mix(tag ^ ((uint64_t)c << 16) ^ v));
        const double r = (double)(k >> 11) * (1.0 / 9007199254740992.0);
        const uint64_t pick = mix(k);
        pend[v] = 0;
        if (r < 0.35 && n_hint(v)) memcpy(cell(c, v), hint(v, pick % n_hint(v)), 32);
        else if (r < 0.60 && n_pool) memcpy(cell(c, v), &pool[(pick % n_pool) * 8u], 32);
        else if (r < 0.75) pend[v] = 1;
      }
      for (uint64_t v = 0; v < V; ++v) {  // after the others, so an alias can copy any var
        if (!pend[v]) continue;
        srcs.clear();
        for (uint64_t a = 0; a < na; ++a)
          if (aliases[2 * (a0 + a)] == v && aliases[2 * (a0 + a) + 1] < V) srcs.push_back(aliases[2 * (a0 + a) + 1]);
        const uint64_t k = mix(seed ^ 0x5A5A5A5Aull ^ mix(tag ^ ((uint64_t)c << 16) ^ v));
        if (!srcs.empty()) {
          memcpy(cell(c, v), cell(c, srcs[k % srcs.size()]), 32);
          continue;
        }
        // no x == y alias: the next equal-width variable from a random start (O(1) when
        // widths repeat, instead of collecting all of them: states hold hundreds of slots)
        for (uint64_t t = 0, st0 = k % V; t < V; ++t) {
          const uint64_t u = (st0 + t) % V;
          if (u != v && var_width[v0 + u] == var_width[v0 + v]) {
            memcpy(cell(c, v), cell(c, u), 32);
            break;
          }
        }
      }
      // domain rows (every other mixture row): variables with a refined abstract value
      // (mgp_refute_domains) are drawn from it, an inside hint half of the time
      const uint32_t kk = c - mix0;
      if (dom && (kk & 1u) == 0u)
        for (uint64_t v = 0; v < V; ++v) {
          const uint32_t *d = dom + (v0 + v) * 33u;
          if (!d[32]) continue;
          U256 z, o, lo, hi;
          memcpy(z.w, d, 32);
          memcpy(o.w, d + 8, 32);
          memcpy(lo.w, d + 16, 32);
          memcpy(hi.w, d + 24, 32);
          const uint64_t key = fe_mix64(seed ^ 0xD0D0D0D0ull ^ fe_mix64(tag ^ ((uint64_t)c << 16) ^ v));
          U256 x = fe_sample_domain(z, o, lo, hi, var_width[v0 + v], kk / 2u, key);
          if (n_hint(v) && (fe_mix64(key ^ 0x9E37ull) & 1u)) {
            U256 h;
            memcpy(h.w, hint(v, fe_mix64(key ^ 0x7F4Aull) % n_hint(v)), 32);
            h = bv_mask(h, var_width[v0 + v]);
            if (fe_inside(z, o, lo, hi, h)) x = h;
          }
          memcpy(cell(c, v), x.w, 32);
        }
    }
    for (uint32_t c = 0; c < n_cand; ++c)
      for (uint64_t v = 0; v < V; ++v) {
        if (var_kind && var_kind[v0 + v] == 2 && n_hint(v)) memcpy(cell(c, v), hint(v, 0), 32);  // pinned constant
        mask_to(cell(c, v), var_width[v0 + v]);
      }
  }
  return 0;
}
