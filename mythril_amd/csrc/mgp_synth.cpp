// mgp_synth.cpp — seeded synthetic constraint DAGs
// and the nominal-op accounting the roofline fraction is priced on.
//
// Each state: 4 free 256-bit vars (x0..x3), up to 2 keccak-UF applications
// whose fresh values are vars 4 and 5 (Ackermannised), a <=16-entry constant
// pool, n_nodes op-nodes drawn from the fixed op mix below, root = conjunction
// of the last 4 Bool nodes.  Operands prefer recent nodes (constraint DAGs
// built by LASER are mostly tree-shaped: JUMPI conditions over fresh
// arithmetic), which also keeps the live-value count inside the per-lane LDS
// slot budget.
//
// Planting (50 % of states): a random assignment x* is drawn and every root
// term that is false at x* is negated, so x* satisfies the root; x* is placed
// at a random candidate index by mgp_plant_candidates_dev.  Evaluating at x*
// uses the same 256-bit helpers as the kernel (mgp_bv.h) — this is workload
// construction, not verification; parity is checked against oracle/.
#include <atomic>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/mgp.h"
#include "mgp_bv.h"

namespace {
std::atomic<int> g_ablate{-1};
int synth_ablate_mode() {
  int m = g_ablate.load(std::memory_order_relaxed);
  if (m >= 0) return m;
  const char *e = getenv("MGP_SYNTH_ABLATE");
  m = !e ? 0 : !strcmp(e, "nodiv") ? 1 : !strcmp(e, "nomul") ? 2 : !strcmp(e, "nodivmul") ? 3 : 0;
  g_ablate.store(m, std::memory_order_relaxed);
  return m;
}

constexpr uint32_t kSynthVars = 6;
constexpr uint32_t kFreeVars = 4;
constexpr uint32_t kMaxUF = 2;

inline uint64_t splitmix64(uint64_t &z) {
  uint64_t r = (z += 0x9E3779B97F4A7C15ull);
  r = (r ^ (r >> 30)) * 0xBF58476D1CE4E5B9ull;
  r = (r ^ (r >> 27)) * 0x94D049BB133111EBull;
  return r ^ (r >> 31);
}

struct Rng {  // xoshiro256**
  uint64_t s[4];
  Rng(uint64_t seed, uint64_t stream) {
    uint64_t z = seed ^ (stream * 0xD1B54A32D192ED03ull) ^ 0x4D595448ull;
    for (int i = 0; i < 4; ++i) s[i] = splitmix64(z);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  bool chance(uint32_t pct) { return below(100) < pct; }
  U256 u256() {
    U256 v;
    for (int i = 0; i < 4; ++i) {
      uint64_t x = next();
      v.w[2 * i] = (uint32_t)x;
      v.w[2 * i + 1] = (uint32_t)(x >> 32);
    }
    return v;
  }
};

// op mix per 100 op-nodes
struct MixEntry { uint8_t op; uint8_t weight; };
constexpr MixEntry kMix[] = {
    {MGP_OP_ADD, 12}, {MGP_OP_SUB, 8},  {MGP_OP_MUL, 4},  {MGP_OP_UDIV, 1}, {MGP_OP_UREM, 1},
    {MGP_OP_SDIV, 1}, {MGP_OP_SREM, 1}, {MGP_OP_AND, 6},  {MGP_OP_OR, 6},   {MGP_OP_XOR, 3},
    {MGP_OP_NOT, 3},  {MGP_OP_SHL, 2},  {MGP_OP_LSHR, 3}, {MGP_OP_ASHR, 1}, {MGP_OP_EQ, 10},
    {MGP_OP_ULT, 6},  {MGP_OP_ULE, 2},  {MGP_OP_SLT, 2},  {MGP_OP_ITE, 8},  {MGP_OP_EXTRACT, 6},
    {MGP_OP_CONCAT, 4}, {MGP_OP_ZEXT, 2}, {MGP_OP_BAND, 3}, {MGP_OP_BOR, 2}, {MGP_OP_BNOT, 1},
    {MGP_OP_UFAPP, 2}};

// ----------------------------------------------------------- host eval
// (planting only; semantics per mgp_ir.h)
struct HostEval {
  const std::vector<mgp_node> &nodes;
  const std::vector<U256> &consts;
  const U256 *vars;
  std::vector<U256> v;
  std::vector<uint8_t> b;

  HostEval(const std::vector<mgp_node> &n, const std::vector<U256> &c, const U256 *x)
      : nodes(n), consts(c), vars(x), v(n.size()), b(n.size()) {}

  void run() {
    struct App { uint32_t node; };
    std::vector<std::vector<uint32_t>> fapps(4);
    for (size_t i = 0; i < nodes.size(); ++i) {
      const mgp_node &nd = nodes[i];
      const uint32_t w = nd.width;
      U256 r = bv_zero();
      auto A = [&]() -> const U256 & { return v[nd.a]; };
      auto B = [&]() -> const U256 & { return v[nd.b]; };
      switch (nd.op) {
        case MGP_OP_VAR: r = bv_mask(vars[nd.p0], w); break;
        case MGP_OP_CONST: r = bv_mask(consts[nd.p0], w); break;
        case MGP_OP_ADD: r = bv_add(A(), B(), nullptr); break;
        case MGP_OP_SUB: r = bv_sub(A(), B(), nullptr); break;
        case MGP_OP_MUL: r = bv_mul(A(), B()); break;
        case MGP_OP_UDIV: { U256 q, m; bv_udivrem(A(), B(), &q, &m); r = q; break; }
        case MGP_OP_UREM: { U256 q, m; bv_udivrem(A(), B(), &q, &m); r = m; break; }
        case MGP_OP_SDIV: r = bv_sdiv(bv_sext(A(), w), bv_sext(B(), w)); break;
        case MGP_OP_SREM: r = bv_srem(bv_sext(A(), w), bv_sext(B(), w)); break;
        case MGP_OP_AND: r = bv_and(A(), B()); break;
        case MGP_OP_OR: r = bv_or(A(), B()); break;
        case MGP_OP_XOR: r = bv_xor(A(), B()); break;
        case MGP_OP_NOT: r = bv_not(A()); break;
        case MGP_OP_SHL: r = bv_shl(A(), bv_shift_amount(B())); break;
        case MGP_OP_LSHR: r = bv_lshr(A(), bv_shift_amount(B())); break;
        case MGP_OP_ASHR: r = bv_ashr(bv_sext(A(), w), bv_shift_amount(B())); break;
        case MGP_OP_EXTRACT: r = bv_lshr(A(), nd.p1); break;
        case MGP_OP_CONCAT: r = bv_or(bv_shl(A(), nodes[nd.b].width), B()); break;
        case MGP_OP_ZEXT: r = A(); break;
        case MGP_OP_ITE: r = b[nd.a] ? B() : v[nd.c]; break;
        case MGP_OP_EQ: b[i] = bv_eq(A(), B()); break;
        case MGP_OP_ULT: b[i] = bv_ult(A(), B()); break;
        case MGP_OP_ULE: b[i] = !bv_ult(B(), A()); break;
        case MGP_OP_SLT: {
          const uint32_t ow = nodes[nd.a].width;
          b[i] = bv_slt(bv_sext(A(), ow), bv_sext(B(), ow));
          break;
        }
        case MGP_OP_BAND: b[i] = b[nd.a] && b[nd.b]; break;
        case MGP_OP_BOR: b[i] = b[nd.a] || b[nd.b]; break;
        case MGP_OP_BNOT: b[i] = !b[nd.a]; break;
        case MGP_OP_UFAPP: {
          r = bv_mask(vars[nd.p1], w);
          for (uint32_t j : fapps[nd.p0 & 3u])
            if (bv_eq(v[nodes[j].a], A())) { r = v[j]; break; }
          fapps[nd.p0 & 3u].push_back((uint32_t)i);
          break;
        }
        default: break;
      }
      if (!(nd.op >= MGP_OP_EQ && nd.op <= MGP_OP_BEQ)) v[i] = bv_mask(r, w ? w : 1);
    }
  }
};

struct Gen {
  Rng rng;
  std::vector<mgp_node> nodes;
  std::vector<U256> consts;
  std::vector<uint32_t> wide, narrow, bools, shiftc;
  uint32_t n_uf = 0;

  Gen(uint64_t seed, uint64_t state) : rng(seed, state) {}

  int32_t push(uint8_t op, uint16_t width, int32_t a = -1, int32_t b = -1, int32_t c = -1, uint32_t p0 = 0,
               uint32_t p1 = 0) {
    mgp_node n;
    memset(&n, 0, sizeof(n));
    n.op = op;
    n.width = width;
    n.a = a; n.b = b; n.c = c;
    n.p0 = p0; n.p1 = p1;
    nodes.push_back(n);
    return (int32_t)nodes.size() - 1;
  }
  std::vector<uint8_t> used;
  uint32_t mark(uint32_t n) {
    if (n >= used.size()) used.resize(n + 1, 0);
    used[n] = 1;
    return n;
  }
  uint32_t pick(const std::vector<uint32_t> &pool) { return mark(pick_raw(pool)); }
  uint32_t pick_raw(const std::vector<uint32_t> &pool) {
    const uint32_t n = (uint32_t)pool.size();
    if (rng.chance(70)) {  // keep the DAG connected: prefer a recent unused value
      const uint32_t lim = n < 16 ? n : 16;
      for (uint32_t k = 0; k < lim; ++k) {
        const uint32_t cand = pool[n - 1 - k];
        if ((cand >= used.size() || !used[cand]) && nodes[cand].op != MGP_OP_CONST) return cand;
      }
    }
    if (rng.chance(65)) {
      const uint32_t k = n < 6 ? n : 6;
      return pool[n - 1 - rng.below(k)];
    }
    return pool[rng.below(n)];
  }
  uint32_t pick_wide() {
    if (rng.chance(12)) return mark((uint32_t)rng.below(kFreeVars));  // nodes 0..3 are x0..x3
    return pick(wide);
  }

  void make_consts() {
    const uint32_t nc = 8 + rng.below(9);
    const uint32_t shifts[8] = {224, 160, 96, 8, 32, 64, 128, 248};
    for (uint32_t k = 0; k < nc; ++k) {
      U256 c = bv_zero();
      if (k < 3) {
        c.w[0] = shifts[rng.below(8)];
      } else {
        switch (rng.below(8)) {
          case 0: c.w[0] = rng.below(256); break;
          case 1: for (int l = 0; l < 5; ++l) c.w[l] = 0xFFFFFFFFu; break;  // 2^160-1
          case 2: for (int l = 0; l < 5; ++l) c.w[l] = 0xDEADBEEFu; break;  // ATTACKER
          case 3: for (int l = 0; l < 5; ++l) c.w[l] = 0xAFFEAFFEu; break;  // CREATOR
          case 4: c = bv_ones(); break;
          case 5: c.w[rng.below(8)] = 1u << rng.below(32); break;
          case 6: c.w[0] = (uint32_t)rng.next(); c.w[1] = (uint32_t)rng.next(); break;
          default: c = rng.u256(); break;
        }
      }
      consts.push_back(c);
    }
  }

  uint8_t draw_op() {
    uint32_t r = rng.below(100), acc = 0;
    for (const MixEntry &m : kMix) {
      acc += m.weight;
      if (r < acc) return ablate(m.op);
    }
    return MGP_OP_ADD;
  }
  // ablation knob for kernel studies: MGP_SYNTH_ABLATE=nodiv|nomul|nodivmul (or
  // mgp_synth_set_ablate 1 / 2 / 3) replaces those ops by ADD.  The same random stream
  // draws the same DAGs otherwise, so the benchmark's division split (bench.py
  // roofline.div_share) times the same states with every division turned into an ADD.
  static uint8_t ablate(uint8_t op) {
    const int mode = synth_ablate_mode();
    const bool div = op >= MGP_OP_UDIV && op <= MGP_OP_SMOD;
    if (((mode & 1) && div) || ((mode & 2) && op == MGP_OP_MUL)) return MGP_OP_ADD;
    return op;
  }

  void bin_wide(uint8_t op) {
    const uint32_t a = pick_wide(), b = pick_wide();
    wide.push_back((uint32_t)push(op, 256, (int32_t)a, (int32_t)b));
  }

  void op_node() {
    uint8_t op = draw_op();
    switch (op) {
      case MGP_OP_ADD: case MGP_OP_SUB: case MGP_OP_MUL: case MGP_OP_UDIV: case MGP_OP_UREM:
      case MGP_OP_SDIV: case MGP_OP_SREM: case MGP_OP_AND: case MGP_OP_OR: case MGP_OP_XOR:
        bin_wide(op);
        break;
      case MGP_OP_NOT:
        wide.push_back((uint32_t)push(op, 256, (int32_t)pick_wide()));
        break;
      case MGP_OP_SHL: case MGP_OP_LSHR: case MGP_OP_ASHR: {
        const uint32_t a = pick_wide();
        const uint32_t s = rng.chance(75) ? mark(shiftc[rng.below((uint32_t)shiftc.size())]) : pick_wide();
        wide.push_back((uint32_t)push(op, 256, (int32_t)a, (int32_t)s));
        break;
      }
      case MGP_OP_EQ: case MGP_OP_ULT: case MGP_OP_ULE: case MGP_OP_SLT: {
        if (narrow.size() >= 2 && rng.chance(25)) {
          const uint32_t a = pick(narrow);
          for (int tries = 0; tries < 6; ++tries) {
            const uint32_t b = narrow[rng.below((uint32_t)narrow.size())];
            if (nodes[b].width == nodes[a].width) {
              mark(b);
              bools.push_back((uint32_t)push(op, 1, (int32_t)a, (int32_t)b));
              return;
            }
          }
        }
        const uint32_t a = pick_wide(), b = pick_wide();
        bools.push_back((uint32_t)push(op, 1, (int32_t)a, (int32_t)b));
        break;
      }
      case MGP_OP_ITE: {
        if (bools.empty()) { bin_wide(MGP_OP_ADD); break; }
        const uint32_t c = pick(bools), a = pick_wide(), b = pick_wide();
        wide.push_back((uint32_t)push(op, 256, (int32_t)c, (int32_t)a, (int32_t)b));
        break;
      }
      case MGP_OP_EXTRACT: {
        extract_node();
        break;
      }
      case MGP_OP_CONCAT: {
        if (narrow.size() >= 2) {
          const uint32_t a = pick(narrow);
          for (int tries = 0; tries < 6; ++tries) {
            const uint32_t b = narrow[rng.below((uint32_t)narrow.size())];
            const uint32_t w = nodes[a].width + nodes[b].width;
            if (w <= 256) {
              mark(b);
              const uint32_t n = (uint32_t)push(op, (uint16_t)w, (int32_t)a, (int32_t)b);
              (w == 256 ? wide : narrow).push_back(n);
              return;
            }
          }
        }
        extract_node();
        break;
      }
      case MGP_OP_ZEXT: {
        if (narrow.empty()) { extract_node(); break; }
        wide.push_back((uint32_t)push(op, 256, (int32_t)pick(narrow)));
        break;
      }
      case MGP_OP_BAND: case MGP_OP_BOR: {
        if (bools.size() < 2) { cmp_fallback(); break; }
        const uint32_t a = pick(bools), b = pick(bools);
        bools.push_back((uint32_t)push(op, 1, (int32_t)a, (int32_t)b));
        break;
      }
      case MGP_OP_BNOT: {
        if (bools.empty()) { cmp_fallback(); break; }
        bools.push_back((uint32_t)push(op, 1, (int32_t)pick(bools)));
        break;
      }
      case MGP_OP_UFAPP: {
        if (n_uf >= kMaxUF) { bin_wide(MGP_OP_ADD); break; }
        const uint32_t a = pick_wide();
        wide.push_back((uint32_t)push(op, 256, (int32_t)a, -1, -1, 0, kFreeVars + n_uf));
        ++n_uf;
        break;
      }
      default:
        bin_wide(MGP_OP_ADD);
        break;
    }
  }
  void extract_node() {
    const uint32_t widths[5] = {8, 32, 64, 128, 160};
    const uint32_t w = widths[rng.below(5)];
    const uint32_t lo = 8 * rng.below((256 - w) / 8 + 1);
    narrow.push_back((uint32_t)push(MGP_OP_EXTRACT, (uint16_t)w, (int32_t)pick_wide(), -1, -1, lo + w - 1, lo));
  }
  void cmp_fallback() {
    const uint32_t a = pick_wide(), b = pick_wide();
    bools.push_back((uint32_t)push(MGP_OP_ULT, 1, (int32_t)a, (int32_t)b));
  }

  void vars_star(U256 *x) {
    for (uint32_t k = 0; k < kSynthVars; ++k) {
      if (k < kFreeVars && rng.chance(30)) {
        U256 c = consts[rng.below((uint32_t)consts.size())];
        const uint32_t d = rng.below(3);
        if (d == 0) c = bv_sub(c, bv_small(1), nullptr);
        if (d == 2) c = bv_add(c, bv_small(1), nullptr);
        x[k] = c;
      } else {
        x[k] = rng.u256();
      }
    }
  }

  // returns the planted flag
  bool generate(uint32_t n_nodes, uint32_t n_cand, uint32_t *plant_idx, uint32_t *plant_words) {
    make_consts();
    for (uint32_t k = 0; k < kFreeVars; ++k) wide.push_back((uint32_t)push(MGP_OP_VAR, 256, -1, -1, -1, k));
    for (uint32_t k = 0; k < consts.size(); ++k) {
      const uint32_t n = (uint32_t)push(MGP_OP_CONST, 256, -1, -1, -1, k);
      wide.push_back(n);
      if (k < 3) shiftc.push_back(n);
    }
    for (uint32_t k = 0; k < n_nodes; ++k) op_node();
    while (bools.size() < 4) cmp_fallback();
    const bool planted = rng.chance(50);
    uint32_t terms[4];
    for (int t = 0; t < 4; ++t) terms[t] = bools[bools.size() - 4 + t];
    if (planted) {
      U256 x[kSynthVars];
      vars_star(x);
      HostEval ev(nodes, consts, x);
      ev.run();
      for (int t = 0; t < 4; ++t)
        if (!ev.b[terms[t]]) terms[t] = (uint32_t)push(MGP_OP_BNOT, 1, (int32_t)terms[t]);
      *plant_idx = rng.below(n_cand);
      for (uint32_t k = 0; k < kSynthVars; ++k)
        for (int l = 0; l < 8; ++l) plant_words[k * 8 + l] = x[k].w[l];
    }
    int32_t r = push(MGP_OP_BAND, 1, (int32_t)terms[0], (int32_t)terms[1]);
    r = push(MGP_OP_BAND, 1, r, (int32_t)terms[2]);
    push(MGP_OP_BAND, 1, r, (int32_t)terms[3]);
    return planted;
  }
};

uint64_t nominal_op_cost(uint8_t op) {
  switch (op) {
    case MGP_OP_ADD: case MGP_OP_SUB: case MGP_OP_NEG: return 16;
    case MGP_OP_MUL: return 108;
    case MGP_OP_UDIV: case MGP_OP_UREM: case MGP_OP_SDIV: case MGP_OP_SREM: case MGP_OP_SMOD: return 1024;
    case MGP_OP_AND: case MGP_OP_OR: case MGP_OP_XOR: case MGP_OP_NOT: return 8;
    case MGP_OP_SHL: case MGP_OP_LSHR: case MGP_OP_ASHR: return 32;
    case MGP_OP_EQ: case MGP_OP_ULT: case MGP_OP_ULE: case MGP_OP_UGT: case MGP_OP_UGE:
    case MGP_OP_SLT: case MGP_OP_SLE: case MGP_OP_SGT: case MGP_OP_SGE:
    case MGP_OP_UADD_NOOVF: case MGP_OP_USUB_NOUDF: return 16;
    case MGP_OP_UMUL_NOOVF: return 108;
    case MGP_OP_ITE: return 8;
    case MGP_OP_EXTRACT: case MGP_OP_CONCAT: case MGP_OP_ZEXT: case MGP_OP_SEXT: return 8;
    case MGP_OP_BAND: case MGP_OP_BOR: case MGP_OP_BXOR: case MGP_OP_BNOT: case MGP_OP_BITE:
    case MGP_OP_BEQ: return 1;
    case MGP_OP_UFAPP: case MGP_OP_UFINV: return 16;
    default: return 0;  // leaves
  }
}

}  // namespace

extern "C" int mgp_synth_generate(uint64_t seed, uint64_t state_base, uint32_t n_states, uint32_t n_nodes,
                                  uint32_t n_cand, mgp_node *nodes_out, uint64_t *node_offsets,
                                  uint32_t *consts_out, uint64_t *const_offsets, uint8_t *planted,
                                  uint32_t *plant_idx, uint32_t *plant_words) {
  if (!nodes_out || !node_offsets || !consts_out || !const_offsets || n_cand == 0) return MGP_E_ARG;
  const uint64_t node_stride = (uint64_t)n_nodes + 32u;  // leaves (<=20) + root terms
  std::vector<uint32_t> n_used(n_states), c_used(n_states);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    Gen g(seed, state_base + (uint64_t)s);
    uint32_t pidx = 0;
    uint32_t pw[kSynthVars * 8];
    memset(pw, 0, sizeof(pw));
    const bool p = g.generate(n_nodes, n_cand, &pidx, pw);
    const uint32_t nn = (uint32_t)std::min<uint64_t>(g.nodes.size(), node_stride);
    memcpy(nodes_out + (uint64_t)s * node_stride, g.nodes.data(), nn * sizeof(mgp_node));
    n_used[s] = (g.nodes.size() <= node_stride) ? nn : 0u;
    c_used[s] = (uint32_t)g.consts.size();
    for (size_t k = 0; k < g.consts.size(); ++k)
      memcpy(consts_out + ((uint64_t)s * 16u + k) * 8u, g.consts[k].w, 32);
    if (planted) planted[s] = p ? 1 : 0;
    if (plant_idx) plant_idx[s] = pidx;
    if (plant_words) memcpy(plant_words + (uint64_t)s * kSynthVars * 8u, pw, sizeof(pw));
  }
  // compact in place (offsets are prefix sums; stride layout -> packed)
  uint64_t no = 0, co = 0;
  for (uint32_t s = 0; s < n_states; ++s) {
    if (n_used[s] == 0) return MGP_E_CAPACITY;
    if (no != (uint64_t)s * node_stride)
      memmove(nodes_out + no, nodes_out + (uint64_t)s * node_stride, n_used[s] * sizeof(mgp_node));
    if (co != (uint64_t)s * 16u)
      memmove(consts_out + co * 8u, consts_out + (uint64_t)s * 16u * 8u, c_used[s] * 32u);
    node_offsets[s] = no;
    const_offsets[s] = co;
    no += n_used[s];
    co += c_used[s];
  }
  node_offsets[n_states] = no;
  const_offsets[n_states] = co;
  return MGP_OK;
}

extern "C" int mgp_nominal_ops(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                               uint64_t *out_ops) {
  if (!nodes || !node_offsets || !out_ops) return MGP_E_ARG;
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    // only nodes in the root's cone are work: everything else cannot change
    // satisfiability (and the lowering drops it)
    const uint64_t n0 = node_offsets[s], n = node_offsets[s + 1] - n0;
    std::vector<uint8_t> live(n, 0);
    if (n) live[n - 1] = 1;
    uint64_t t = 0;
    for (int64_t i = (int64_t)n - 1; i >= 0; --i) {
      if (!live[i]) continue;
      const mgp_node &nd = nodes[n0 + i];
      t += nominal_op_cost(nd.op);
      for (int32_t j : {nd.a, nd.b, nd.c})
        if (j >= 0 && j < i) live[j] = 1;
    }
    out_ops[s] = t;
  }
  return MGP_OK;
}

extern "C" int mgp_synth_set_ablate(int mode) {
  if (mode < 0 || mode > 3) return MGP_E_ARG;
  g_ablate.store(mode, std::memory_order_relaxed);
  return MGP_OK;
}
