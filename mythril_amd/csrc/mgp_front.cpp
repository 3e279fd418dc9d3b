// mgp_front.cpp — native front end of the pre-filter: term arena -> per-state
// constraint DAGs (include/mgp_ir.h node lists), variable tables, candidate hints.
//
// The reference checks one state at a time: Constraints.is_possible re-adds every
// constraint of the state to a fresh z3 Solver (mythril/laser/ethereum/state/
// constraints.py:34-51), and analysis.solver.get_model does the same with Optimize
// (mythril/analysis/solver.py:27-61).  Here a whole batch of states is flattened at
// once from the term arena (mythril_amd/smt.py: _Arena, one row per hash-consed term;
// the z3 walker mythril_amd/z3_lower.py fills the same arena from z3 ASTs), OpenMP
// over states.  The result is exactly what mythril_amd/dag.py build_state +
// pack_states + make_candidates' table flattening produce in Python (the tests pin
// the two against each other node for node), so every downstream stage — lowering
// (mgp_lower.cpp), UNSAT pre-check (mgp_refute.cpp), candidate generation, the HIP
// evaluation — consumes it unchanged.
//
// Per state:
//   * nodes in DFS post-order over the roots (children a, b, c first), memoised per
//     term; the roots are AND-chained into a final Bool node (TRUE if none);
//   * constants pooled per (value, 256-bit pieces); variables per (name, width), a
//     value wider than 256 bits spread over ceil(w/256) slots (low piece first);
//     each uninterpreted-function application gets a fresh variable (Ackermann);
//   * candidate hints x == c -> c, x <op> c -> c, c +- 1, 64-aligned neighbours, and
//     x == y alias pairs;
//   * padded key equalities: `key == x` with a constant key narrower than x reaches
//     z3 as x == Concat(0, key) (bitvec.py:16-22; keccak_function_manager.py:141-145
//     builds one per concrete hash seen for every symbolic hash input).  Whether z3
//     sees such a disjunct at all depends on the manager's dict of concrete hashes,
//     keyed by z3 AST hashes (tests/laser/keccak_tests.py expects `unsat` for
//     keccak(100_8) == keccak(N1_256), which the formula as written satisfies).  The
//     GPU program therefore replaces every such equality by the constant that makes
//     the formula STRONGER — false where it occurs positively, true where it occurs
//     negatively — so a GPU witness never rests on one: it is a model of the
//     formula with or without those disjuncts.  A state where one occurs with both
//     polarities gets no GPU SAT answer (flag FE_SAT_UNSAFE).  The UNSAT pre-check
//     reads the original nodes (refuting the weaker formula is the sound direction).
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/mgp.h"
#include "mgp_buf.h"
#include "mgp_bv.h"

namespace {

struct StateOut {
  std::vector<mgp_node> nodes;
  std::vector<uint32_t> gpu_ops;           // (node index, op) pairs: padded equalities replaced
  std::vector<mgp_node> gpu_nodes;         // the GPU program when it differs from `nodes` (else empty)
  std::vector<uint32_t> consts;            // 8 limbs per pool entry
  std::vector<uint32_t> var_width, var_full, var_name, var_aux;  // per slot
  std::vector<uint8_t> var_kind;
  std::vector<uint64_t> var_key;
  std::vector<int32_t> var_tid;            // per slot: the VAR / UF term it stands for (-1 pinned)
  std::vector<std::vector<uint32_t>> hints;  // per slot: 8 limbs per hint
  std::vector<uint32_t> aliases;           // (dst, src) pairs
  uint8_t flags = 0;
  bool bad = false;
};

struct Arena {
  const uint8_t *op;
  const uint32_t *width;
  const int32_t *args;
  const uint32_t *p;
  const uint32_t *limbs;
  uint64_t n_terms, n_limbs;
};

inline uint64_t hash_limbs(const uint32_t *l, uint32_t n, uint32_t k) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ k;
  for (uint32_t i = 0; i < n; ++i) {
    h ^= l[i];
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
  }
  return h;
}

inline void mask_limbs(uint32_t *v, uint32_t w) {
  for (int l = 0; l < 8; ++l) {
    const int lo = 32 * l;
    v[l] &= (int)w >= lo + 32 ? 0xFFFFFFFFu : ((int)w <= lo ? 0u : ((1u << (w - lo)) - 1u));
  }
}

inline void add_u64(const uint32_t *a, uint64_t d, bool sub, uint32_t *r) {  // r = a +- d mod 2^256
  uint64_t carry = 0;
  for (int l = 0; l < 8; ++l) {
    const uint64_t dl = l == 0 ? (uint32_t)d : (l == 1 ? (uint32_t)(d >> 32) : 0u);
    if (!sub) {
      const uint64_t s = (uint64_t)a[l] + dl + carry;
      r[l] = (uint32_t)s;
      carry = s >> 32;
    } else {
      const uint64_t s = (uint64_t)a[l] - dl - carry;
      r[l] = (uint32_t)s;
      carry = (s >> 63) & 1u;
    }
  }
}

// Open-addressing map uint64 -> uint32 (linear probing), reused across the states one
// thread builds: clear() resets only the slots that were used (no per-node allocation).
struct FlatMap {
  std::vector<uint64_t> keys;
  std::vector<uint32_t> vals;
  std::vector<uint32_t> used;
  uint64_t mask = 0;
  static constexpr uint64_t kEmpty = ~0ull;
  void reset(uint64_t expect) {
    uint64_t cap = 64;
    while (cap < 2 * expect) cap <<= 1;
    if (cap > keys.size()) {
      keys.assign(cap, kEmpty);
      vals.assign(cap, 0);
      used.clear();
      mask = cap - 1;
      return;
    }
    for (uint32_t u : used) keys[u] = kEmpty;
    used.clear();
  }
  uint64_t slot(uint64_t k) const {
    uint64_t h = k * 0x9E3779B97F4A7C15ull;
    return (h ^ (h >> 32)) & mask;
  }
  // value of k or nullptr
  uint32_t *find(uint64_t k) {
    for (uint64_t i = slot(k);; i = (i + 1) & mask) {
      if (keys[i] == k) return &vals[i];
      if (keys[i] == kEmpty) return nullptr;
    }
  }
  void put(uint64_t k, uint32_t v) {
    if (2 * (used.size() + 1) > keys.size()) grow();
    uint64_t i = slot(k);
    while (keys[i] != kEmpty && keys[i] != k) i = (i + 1) & mask;
    if (keys[i] == kEmpty) used.push_back((uint32_t)i);
    keys[i] = k;
    vals[i] = v;
  }
  void grow() {
    std::vector<uint64_t> ok;
    std::vector<uint32_t> ov;
    for (uint32_t u : used) {
      ok.push_back(keys[u]);
      ov.push_back(vals[u]);
    }
    keys.assign(keys.size() * 2, kEmpty);
    vals.assign(keys.size(), 0);
    mask = keys.size() - 1;
    used.clear();
    for (size_t i = 0; i < ok.size(); ++i) put(ok[i], ov[i]);
  }
};

struct Scratch {
  FlatMap memo, var_idx, const_idx;
  struct CEnt {
    uint32_t pool, term, k;
  };
  std::vector<CEnt> cents;
  std::vector<std::pair<int32_t, bool>> stack;
};

// slot key: which variable (name, kind, UF node) and which 256-bit piece -- a parent
// witness is matched to a child's slots by it (mgp_check_batch)
inline uint64_t slot_key(uint32_t name, uint8_t kind, uint32_t aux, uint32_t j) {
  if (kind == 2) return ~0ull;  // pinned constant: never matched to a parent
  return kind ? (1ull << 63) | ((uint64_t)(name & 0x7FFFFFFFu) << 32) | ((uint64_t)(aux & 0xFFFFFFu) << 8) | (j & 0xFFu)
              : ((uint64_t)(name & 0x7FFFFFFFu) << 32) | (j & 0xFFFFFFFFu);
}

inline uint64_t uf_slot_key(uint32_t name, uint32_t tid, uint32_t j) {
  uint64_t z = ((uint64_t)name << 40) ^ ((uint64_t)tid << 8) ^ j ^ 0x5546A7E1ull;  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (1ull << 63) | ((z ^ (z >> 31)) >> 1);
}

template <typename IsPadded>
void strengthen_padded(StateOut &S, IsPadded is_padded_eq);
void pin_constants(StateOut &S);

void build_one(const Arena &A, const int32_t *roots, uint64_t n_roots, StateOut &S, Scratch &X) {
  FlatMap &memo = X.memo, &var_idx = X.var_idx, &const_idx = X.const_idx;
  memo.reset(512);
  var_idx.reset(64);
  const_idx.reset(64);
  X.cents.clear();
  using CEnt = Scratch::CEnt;
  auto new_slots = [&](uint32_t name, uint32_t width, uint8_t kind, uint32_t aux, int32_t tid) -> uint32_t {
    const uint32_t first = (uint32_t)S.var_width.size();
    for (uint32_t off = 0, j = 0; off < width; off += 256, ++j) {
      S.var_tid.push_back(tid);
      S.var_width.push_back(std::min<uint32_t>(256, width - off));
      S.var_full.push_back(j == 0 ? width : 0u);
      S.var_name.push_back(name);
      S.var_aux.push_back(kind == 0 ? j : aux);
      S.var_kind.push_back(kind);
      // a UF application's slot is keyed by its term (the arena hash-conses terms, so a
      // child's constraint list names its parent's applications by the same ids): keying it
      // by DAG position matched a parent's keccak256_512(sender, slot) value to the child's
      // keccak256_512(to, slot) whenever the child's DAG ordered its applications differently
      S.var_key.push_back(kind == 1 && tid >= 0 ? uf_slot_key(name, (uint32_t)tid, j) : slot_key(name, kind, aux, j));
    }
    return first;
  };
  auto emit = [&](int32_t t) -> int32_t {
    mgp_node nd;
    memset(&nd, 0, sizeof nd);
    const uint8_t op = A.op[t];
    const uint32_t w = A.width[t] == 0 ? 1u : A.width[t];
    int32_t ch[3] = {-1, -1, -1};
    for (int i = 0; i < 3; ++i) {
      const int32_t a = A.args[3 * (uint64_t)t + i];
      if (a >= 0) ch[i] = (int32_t)*memo.find((uint64_t)a);
    }
    nd.op = op;
    nd.width = (uint16_t)w;
    nd.a = ch[0];
    nd.b = ch[1];
    nd.c = ch[2];
    const uint32_t p0 = A.p[2 * (uint64_t)t], p1 = A.p[2 * (uint64_t)t + 1];
    if (w > 0xFFFFu) S.bad = true;
    if (op == MGP_OP_VAR) {
      const uint64_t key = ((uint64_t)p0 << 32) | w;
      const uint32_t *it = var_idx.find(key);
      if (it) {
        nd.p0 = *it;
      } else {
        nd.p0 = new_slots(p0, w, 0, 0, t);
        var_idx.put(key, nd.p0);
      }
    } else if (op == MGP_OP_CONST) {
      const uint32_t k = (w + 255) / 256;
      const uint32_t *l = A.limbs + p0;
      uint32_t n = p1;
      if ((uint64_t)p0 + p1 > A.n_limbs) {
        S.bad = true;
        n = 0;
      }
      while (n && l[n - 1] == 0) --n;  // the value, not its storage width, is the key
      // hash -> entry; a genuine collision probes the next hash value
      uint64_t h = hash_limbs(l, n, k) & ~(1ull << 63);
      int64_t found = -1;
      for (;; h = (h + 1) & ~(1ull << 63)) {
        const uint32_t *ei = const_idx.find(h);
        if (!ei) break;
        const CEnt &e = X.cents[*ei];
        const uint32_t *ul = A.limbs + A.p[2 * (uint64_t)e.term];
        uint32_t un = A.p[2 * (uint64_t)e.term + 1];
        while (un && ul[un - 1] == 0) --un;
        if (e.k == k && un == n && (n == 0 || memcmp(ul, l, 4u * n) == 0)) {
          found = e.pool;
          break;
        }
      }
      if (found < 0) {
        found = (int64_t)(S.consts.size() / 8);
        const_idx.put(h, (uint32_t)X.cents.size());
        X.cents.push_back(CEnt{(uint32_t)found, (uint32_t)t, k});
        for (uint32_t j = 0; j < k; ++j)
          for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t li = 8 * j + q;
            S.consts.push_back(li < n ? l[li] : 0u);
          }
      }
      nd.p0 = (uint32_t)found;
    } else if (op == MGP_OP_EXTRACT) {
      nd.p0 = p0;
      nd.p1 = p1;
    } else if (op == MGP_OP_UFAPP || op == MGP_OP_UFINV) {
      nd.p0 = p0;
      nd.p1 = new_slots(p1, w, 1, (uint32_t)S.nodes.size(), t);
    }
    S.nodes.push_back(nd);
    return (int32_t)S.nodes.size() - 1;
  };

  std::vector<int32_t> root_nodes;
  auto &stack = X.stack;
  for (uint64_t r = 0; r < n_roots; ++r) {
    const int32_t root = roots[r];
    if (root < 0 || (uint64_t)root >= A.n_terms) {
      S.bad = true;
      return;
    }
    stack.clear();
    stack.emplace_back(root, false);
    // Rows of dead terms are reused (smt._Arena.release), so an argument's row may come
    // after its user's; a term being expanded is marked kOpen, and meeting an open term
    // again below itself is a cycle (malformed input), never a DAG.
    constexpr uint32_t kOpen = 0xFFFFFFFFu;
    while (!stack.empty()) {
      const auto [t, done] = stack.back();
      stack.pop_back();
      if (done) {
        const int32_t idx = emit(t);
        memo.put((uint64_t)t, (uint32_t)idx);
        continue;
      }
      if (const uint32_t *m = memo.find((uint64_t)t)) {
        if (*m == kOpen) {
          S.bad = true;
          return;
        }
        continue;
      }
      memo.put((uint64_t)t, kOpen);
      stack.emplace_back(t, true);
      for (int i = 2; i >= 0; --i) {
        const int32_t a = A.args[3 * (uint64_t)t + i];
        if (a < 0) continue;
        if ((uint64_t)a >= A.n_terms || a == t) {
          S.bad = true;
          return;
        }
        const uint32_t *m = memo.find((uint64_t)a);
        if (m && *m == kOpen) {
          S.bad = true;
          return;
        }
        if (!m) stack.emplace_back(a, false);
      }
    }
    root_nodes.push_back((int32_t)*memo.find((uint64_t)root));
  }
  auto push_bool = [&](uint8_t op, int32_t a, int32_t b) {
    mgp_node nd;
    memset(&nd, 0, sizeof nd);
    nd.op = op;
    nd.width = 1;
    nd.a = a;
    nd.b = b;
    nd.c = -1;
    S.nodes.push_back(nd);
  };
  if (root_nodes.empty()) {
    push_bool(MGP_OP_TRUE, -1, -1);
  } else {
    int32_t r = root_nodes[0];
    for (size_t i = 1; i < root_nodes.size(); ++i) {
      push_bool(MGP_OP_BAND, r, root_nodes[i]);
      r = (int32_t)S.nodes.size() - 1;
    }
    if (r != (int32_t)S.nodes.size() - 1) push_bool(MGP_OP_BAND, r, r);
  }

  // ---- hints and aliases (dag.py _harvest_hints)
  const uint32_t n_slots = (uint32_t)S.var_width.size();
  S.hints.assign(n_slots, {});
  auto var_of = [&](int32_t x) -> int64_t {
    const mgp_node &n = S.nodes[x];
    if (n.op == MGP_OP_VAR) return n.p0;
    if (n.op == MGP_OP_UFAPP || n.op == MGP_OP_UFINV) return n.p1;
    return -1;
  };
  // wrap hints: x * c (and BVMulNoOverflow(x, c)) with a constant c >= 2 -> the largest x
  // that does not wrap and the smallest that does, floor((2^w-1)/c) and +1.  Paths whose
  // feasibility rests on an overflowing product (rubixi's payout = value * multiplier / 100
  // against the balance share, the integer module's Not(BVMulNoOverflow)) have their
  // witnesses right past that boundary, where neither uniform nor small values land.
  auto wrap_hints = [&](int64_t vi, int32_t cnode, uint32_t w) {
    if (vi < 0 || S.nodes[cnode].op != MGP_OP_CONST || w > 256 || w < 2) return;
    U256 c, q, r;
    memcpy(c.w, &S.consts[8u * S.nodes[cnode].p0], 32);
    c = bv_mask(c, w);
    if (bv_ult(c, bv_small(2))) return;
    bv_udivrem(bv_mask(bv_ones(), w), c, &q, &r);
    U256 q1 = bv_mask(bv_add(q, bv_small(1), nullptr), w);
    auto &H = S.hints[vi];
    H.insert(H.end(), q.w, q.w + 8);
    H.insert(H.end(), q1.w, q1.w + 8);
  };
  for (const mgp_node &n : S.nodes) {
    if (n.a < 0 || n.b < 0) continue;
    if (n.op == MGP_OP_MUL || n.op == MGP_OP_UMUL_NOOVF) {
      const uint32_t w = S.nodes[n.a].width;
      wrap_hints(var_of(n.a), n.b, w);
      wrap_hints(var_of(n.b), n.a, w);
    }
    if (n.op < MGP_OP_EQ || n.op > MGP_OP_USUB_NOUDF) continue;
    const int64_t va = var_of(n.a), vb = var_of(n.b);
    if (n.op == MGP_OP_EQ && va >= 0 && vb >= 0 && va != vb) {
      S.aliases.push_back((uint32_t)va);
      S.aliases.push_back((uint32_t)vb);
      S.aliases.push_back((uint32_t)vb);
      S.aliases.push_back((uint32_t)va);
    }
    const uint32_t wa = S.nodes[n.a].width;
    const std::pair<int64_t, int32_t> pairs[2] = {{va, n.b}, {vb, n.a}};
    for (const auto &pr : pairs) {
      if (pr.first < 0 || S.nodes[pr.second].op != MGP_OP_CONST || wa > 256) continue;
      const uint32_t *cv = &S.consts[8u * S.nodes[pr.second].p0];
      auto &H = S.hints[pr.first];
      if (n.op == MGP_OP_EQ) {
        uint32_t v[8];
        memcpy(v, cv, 32);
        mask_limbs(v, wa);  // the pool entry is the value's low 256 bits; w <= 256 here
        H.insert(H.end(), v, v + 8);
      } else {
        uint32_t up[8], up64[8], c0[8], cm[8], cp[8];
        add_u64(cv, 63, false, up);
        up[0] &= ~63u;
        mask_limbs(up, wa);
        add_u64(up, 64, false, up64);
        mask_limbs(up64, wa);
        memcpy(c0, cv, 32);
        mask_limbs(c0, wa);
        add_u64(cv, 1, true, cm);
        mask_limbs(cm, wa);
        add_u64(cv, 1, false, cp);
        mask_limbs(cp, wa);
        for (const uint32_t *v : {up, up64, c0, cm, cp}) H.insert(H.end(), v, v + 8);
      }
    }
  }

  // ---- padded key equalities: polarity from the root, strengthened for the GPU
  auto is_padded_eq = [&](const mgp_node &n) {
    if (n.op != MGP_OP_EQ || n.a < 0 || n.b < 0) return false;
    auto zc = [&](int32_t x) {
      const mgp_node &z = S.nodes[x];
      return z.op == MGP_OP_ZEXT && z.a >= 0 && S.nodes[z.a].op == MGP_OP_CONST;
    };
    const bool za = zc(n.a), zb = zc(n.b);
    return (za && S.nodes[n.b].op != MGP_OP_CONST) || (zb && S.nodes[n.a].op != MGP_OP_CONST);
  };
  bool any = false;
  for (const mgp_node &n : S.nodes) any |= is_padded_eq(n);
  if (any) strengthen_padded(S, is_padded_eq);
  pin_constants(S);
  if (!S.gpu_ops.empty() && S.gpu_nodes.empty()) S.gpu_nodes = S.nodes;
  const uint32_t shift = S.gpu_nodes.size() - S.nodes.size();  // front VAR nodes of pinned constants
  for (size_t k = 0; k < S.gpu_ops.size(); k += 2) {
    mgp_node &nd = S.gpu_nodes[shift + S.gpu_ops[k]];
    nd.op = (uint8_t)S.gpu_ops[k + 1];
    nd.width = 1;
    nd.a = nd.b = nd.c = -1;
    nd.p0 = nd.p1 = 0;
  }
}

// Polarity of every padded key equality from the root (bit 0 positive, bit 1 negative).
template <typename IsPadded>
void strengthen_padded(StateOut &S, IsPadded is_padded_eq) {
  const int32_t N = (int32_t)S.nodes.size();
  std::vector<uint8_t> pol(N, 0);
  pol[N - 1] = 1;
  for (int32_t i = N - 1; i >= 0; --i) {
    const uint8_t p = pol[i];
    if (!p) continue;
    const mgp_node &n = S.nodes[i];
    const uint8_t flip = (uint8_t)(((p & 1) << 1) | ((p >> 1) & 1));
    switch (n.op) {
      case MGP_OP_BAND: case MGP_OP_BOR:
        if (n.a >= 0) pol[n.a] |= p;
        if (n.b >= 0) pol[n.b] |= p;
        break;
      case MGP_OP_BNOT:
        if (n.a >= 0) pol[n.a] |= flip;
        break;
      case MGP_OP_BXOR: case MGP_OP_BEQ:
        if (n.a >= 0) pol[n.a] |= 3;
        if (n.b >= 0) pol[n.b] |= 3;
        break;
      case MGP_OP_BITE:
        if (n.a >= 0) pol[n.a] |= 3;
        if (n.b >= 0) pol[n.b] |= p;
        if (n.c >= 0) pol[n.c] |= p;
        break;
      default:
        // a node the pass does not model (a compare, a BV ITE, a BV operator, a UF
        // application): its operands -- a padded equality under If(eq, 1, 0) == 1, the
        // shape LASER's EQ / ISZERO build -- are reached with both polarities, which flags
        // the state SAT-unsafe instead of leaving the equality unstrengthened
        if (n.a >= 0) pol[n.a] |= 3;
        if (n.b >= 0) pol[n.b] |= 3;
        if (n.c >= 0) pol[n.c] |= 3;
        break;
    }
  }
  for (int32_t i = 0; i < N; ++i) {
    if (!pol[i] || !is_padded_eq(S.nodes[i])) continue;
    if (pol[i] == 3) {
      S.flags |= MGP_FE_SAT_UNSAFE;
      continue;
    }
    S.gpu_ops.push_back((uint32_t)i);
    S.gpu_ops.push_back(pol[i] == 1 ? (uint32_t)MGP_OP_FALSE : (uint32_t)MGP_OP_TRUE);
    S.flags |= MGP_FE_STRENGTHENED;
  }
}

// Constant-pool budget of the GPU program.  The gfx950 interpreter holds a state's
// constants in VGPR lanes (<= 64 entries, width masks and sign constants included,
// mgp_uop.cpp); LASER's calldata words alone bring 32 byte indices each
// (calldata.py:219-232), so two or three words overflow it.  A CONST node whose pool
// entry lies at or past MGP_FE_POOL_KEEP is PINNED in the GPU program: its operand uses
// read a new VAR node (placed in front of the program, so every index shifts by the
// number of such nodes) of a pinned variable slot (kind 2), which every candidate row
// fills with the constant (hint 0 of the slot, written last by the generators).  Uses
// as an uninterpreted-function argument keep the CONST node: the lowering compares
// known arguments at lowering time and needs no pool entry for them (a calldata byte
// index is both a select argument and a bound in If(i < calldatasize, ...)).  The
// UNSAT pre-check and the hints keep the original nodes.
void pin_constants(StateOut &S) {
  const uint32_t n_pool = (uint32_t)(S.consts.size() / 8);
  if (n_pool <= MGP_FE_POOL_KEEP) return;
  const uint32_t N = (uint32_t)S.nodes.size();
  std::vector<uint8_t> pinned(N, 0), other_use(N, 0);
  bool any = false;
  for (uint32_t i = 0; i < N; ++i) {
    const mgp_node &n = S.nodes[i];
    if (n.op == MGP_OP_CONST && n.p0 + (n.width + 255u) / 256u > MGP_FE_POOL_KEEP) pinned[i] = 1, any = true;
  }
  if (!any) return;
  for (uint32_t i = 0; i < N; ++i) {
    const mgp_node &n = S.nodes[i];
    const int32_t ops[3] = {n.a, n.b, n.c};
    for (int k = 0; k < 3; ++k) {
      const int32_t x = ops[k];
      if (x < 0 || !pinned[x]) continue;
      if (k == 0 && (n.op == MGP_OP_UFAPP || n.op == MGP_OP_UFINV)) continue;  // UF argument
      other_use[x] = 1;
    }
  }
  std::vector<int64_t> slot_of(n_pool, -1);
  std::vector<int32_t> front(N, -1);
  std::vector<mgp_node> pre;
  for (uint32_t i = 0; i < N; ++i) {
    if (!other_use[i]) continue;
    const mgp_node &n = S.nodes[i];
    const uint32_t k = (n.width + 255u) / 256u;
    if (slot_of[n.p0] < 0) {
      slot_of[n.p0] = (int64_t)S.var_width.size();
      for (uint32_t j = 0; j < k; ++j) {
        S.var_width.push_back(std::min<uint32_t>(256, n.width - 256 * j));
        S.var_full.push_back(j == 0 ? n.width : 0u);
        S.var_name.push_back(0u);
        S.var_aux.push_back(n.p0);
        S.var_kind.push_back(2u);
        S.var_key.push_back(slot_key(0, 2, n.p0, j));
        S.var_tid.push_back(-1);
        S.hints.emplace_back(S.consts.begin() + 8ull * (n.p0 + j), S.consts.begin() + 8ull * (n.p0 + j) + 8);
      }
    }
    mgp_node v;
    memset(&v, 0, sizeof v);
    v.op = MGP_OP_VAR;
    v.width = n.width;
    v.a = v.b = v.c = -1;
    v.p0 = (uint32_t)slot_of[n.p0];
    front[i] = (int32_t)pre.size();
    pre.push_back(v);
  }
  if (pre.empty()) return;
  const int32_t P = (int32_t)pre.size();
  S.gpu_nodes = pre;
  S.gpu_nodes.reserve(P + N);
  for (uint32_t i = 0; i < N; ++i) {
    mgp_node n = S.nodes[i];
    int32_t *ops[3] = {&n.a, &n.b, &n.c};
    for (int k = 0; k < 3; ++k) {
      const int32_t x = *ops[k];
      if (x < 0) continue;
      const bool uf_arg = k == 0 && (n.op == MGP_OP_UFAPP || n.op == MGP_OP_UFINV);
      *ops[k] = (front[x] >= 0 && !uf_arg) ? front[x] : x + P;
    }
    S.gpu_nodes.push_back(n);
  }
  S.flags |= MGP_FE_PINNED;
}

}  // namespace

// The flat arrays are sized and then written in full by the per-state copy (in parallel):
// no zero fill first (a 1 024-state batch is tens of MB of nodes, and a serial fill of them
// cost more than building the states)
template <typename T>
using FeVec = std::vector<T, NoInitAlloc<T>>;
struct mgp_fe_batch {
  uint32_t n_states = 0;
  FeVec<mgp_node> nodes, gpu_nodes, dec_nodes;
  std::vector<uint64_t> node_off, gpu_node_off, const_off, var_off, hint_off, alias_off;
  FeVec<uint32_t> consts, var_width, var_full, var_name, var_aux, hints, aliases;
  FeVec<uint8_t> var_kind;
  std::vector<uint8_t> flags;
  FeVec<uint64_t> var_key;
  FeVec<int32_t> var_tid;
  std::vector<uint64_t> state_key;
};

namespace {
// Released batches, kept for the next mgp_build_states (their arrays keep their capacity):
// a 1 024-state batch is ~50 MB, and returning it to the system on every call cost several
// ms in the caller's result stage.  At most two are kept.
std::mutex &fe_pool_mu() {
  static std::mutex m;
  return m;
}
std::vector<mgp_fe_batch *> &fe_pool() {
  static std::vector<mgp_fe_batch *> p;
  return p;
}
mgp_fe_batch *fe_take() {
  {
    std::lock_guard<std::mutex> lk(fe_pool_mu());
    if (!fe_pool().empty()) {
      mgp_fe_batch *B = fe_pool().back();
      fe_pool().pop_back();
      // the arrays a build may leave unset
      B->gpu_nodes.clear();
      B->dec_nodes.clear();
      B->gpu_node_off.clear();
      return B;
    }
  }
  return new (std::nothrow) mgp_fe_batch();
}

inline uint64_t key_mix(uint64_t h, uint64_t x) {
  h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h *= 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 31);
}
// Content key of one built state: its node list with every name replaced by a stable hash
// of the name's text (the arena's name ids depend on the order names were first seen),
// its GPU program, constants and variable table.  Candidate generators key their streams
// by it instead of the state's position in the batch, so a state gets the same candidates
// -- and the same answer -- whatever batch it arrives in and in whatever order.
uint64_t state_key_of(const StateOut &S, const uint64_t *name_hash, uint64_t n_names) {
  auto nh = [&](uint32_t id) -> uint64_t { return (name_hash && id < n_names) ? name_hash[id] : 0xA11CEull ^ id; };
  uint64_t h = 0x4D595448ull;
  auto node = [&](const mgp_node &n) {
    h = key_mix(h, (uint64_t)n.op | ((uint64_t)n.flags << 8) | ((uint64_t)n.width << 16));
    h = key_mix(h, ((uint64_t)(uint32_t)n.a << 32) | (uint32_t)n.b);
    const bool uf = n.op == MGP_OP_UFAPP || n.op == MGP_OP_UFINV;
    const uint64_t p0 = uf && n.p1 < S.var_name.size() ? nh(S.var_name[n.p1]) : n.p0;
    h = key_mix(h, ((uint64_t)(uint32_t)n.c << 32) ^ p0);
    h = key_mix(h, n.p1);
  };
  for (const mgp_node &n : S.nodes) node(n);
  h = key_mix(h, S.gpu_nodes.size());
  for (const mgp_node &n : S.gpu_nodes) node(n);
  for (uint32_t c : S.consts) h = key_mix(h, c);
  for (size_t v = 0; v < S.var_width.size(); ++v) {
    // (a pinned constant's slot has no name -- var_name 0 is whatever name the arena interned
    // first in this process, so hashing it made the key depend on the process' history)
    h = key_mix(h, S.var_kind[v] == 2u ? 0x50494E4E4544ull : nh(S.var_name[v]));
    h = key_mix(h, ((uint64_t)S.var_width[v] << 40) ^ ((uint64_t)S.var_kind[v] << 32) ^ S.var_aux[v]);
    h = key_mix(h, S.var_full[v]);
  }
  return key_mix(h, S.flags);
}
}  // namespace

extern "C" {

int mgp_build_states(const uint8_t *t_op, const uint32_t *t_width, const int32_t *t_args, const uint32_t *t_p,
                     uint64_t n_terms, const uint32_t *limbs, uint64_t n_limbs, const int32_t *roots,
                     const uint64_t *root_off, uint32_t n_states, const uint64_t *name_hash, uint64_t n_names,
                     mgp_fe_batch **out) {
  if (!out || !root_off || (n_terms && (!t_op || !t_width || !t_args || !t_p)) || (n_states && !roots && root_off[n_states]))
    return MGP_E_ARG;
  *out = nullptr;
  const Arena A{t_op, t_width, t_args, t_p, limbs, n_terms, n_limbs};
  const double t_start = omp_get_wtime();
  std::vector<StateOut> res(n_states);
  int bad = 0;
#pragma omp parallel
  {
    Scratch X;
#pragma omp for schedule(dynamic, 4)
    for (int64_t s = 0; s < (int64_t)n_states; ++s) {
      const uint64_t r0 = root_off[s], r1 = root_off[s + 1];
      if (r1 < r0) {
#pragma omp atomic write
        bad = 1;
        continue;
      }
      build_one(A, roots + r0, r1 - r0, res[s], X);
      if (res[s].bad) {
#pragma omp atomic write
        bad = 1;
      }
    }
  }
  if (getenv("MGP_FE_TIMING")) fprintf(stderr, "[fe] build %.3f ms\n", 1e3 * omp_get_wtime() - 1e3 * t_start);
  if (bad) return MGP_E_ARG;
  mgp_fe_batch *B = fe_take();
  if (!B) return MGP_E_NOMEM;
  B->n_states = n_states;
  B->node_off.assign(n_states + 1, 0);
  B->const_off.assign(n_states + 1, 0);
  B->var_off.assign(n_states + 1, 0);
  B->alias_off.assign(n_states + 1, 0);
  B->flags.assign(n_states, 0);
  for (uint32_t s = 0; s < n_states; ++s) {
    B->node_off[s + 1] = B->node_off[s] + res[s].nodes.size();
    B->const_off[s + 1] = B->const_off[s] + res[s].consts.size() / 8;
    B->var_off[s + 1] = B->var_off[s] + res[s].var_width.size();
    B->alias_off[s + 1] = B->alias_off[s] + res[s].aliases.size() / 2;
    B->flags[s] = res[s].flags;
  }
  const uint64_t nn = B->node_off[n_states], nv = B->var_off[n_states];
  B->nodes.resize(nn);
  B->consts.resize(B->const_off[n_states] * 8);
  B->var_width.resize(nv);
  B->var_full.resize(nv);
  B->var_name.resize(nv);
  B->var_aux.resize(nv);
  B->var_kind.resize(nv);
  B->var_key.resize(nv);
  B->var_tid.resize(nv);
  B->aliases.resize(B->alias_off[n_states] * 2);
  B->state_key.resize(n_states);
  B->hint_off.assign(nv + 1, 0);
  bool strengthened = false;
  for (uint32_t s = 0; s < n_states; ++s) {
    const uint64_t v0 = B->var_off[s];
    for (size_t v = 0; v < res[s].hints.size(); ++v) B->hint_off[v0 + v + 1] = res[s].hints[v].size() / 8;
    strengthened |= !res[s].gpu_nodes.empty();
  }
  for (uint64_t v = 0; v < nv; ++v) B->hint_off[v + 1] += B->hint_off[v];
  B->hints.resize(B->hint_off[nv] * 8);
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const StateOut &S = res[s];
    std::copy(S.nodes.begin(), S.nodes.end(), B->nodes.begin() + B->node_off[s]);
    std::copy(S.consts.begin(), S.consts.end(), B->consts.begin() + B->const_off[s] * 8);
    const uint64_t v0 = B->var_off[s];
    std::copy(S.var_width.begin(), S.var_width.end(), B->var_width.begin() + v0);
    std::copy(S.var_full.begin(), S.var_full.end(), B->var_full.begin() + v0);
    std::copy(S.var_name.begin(), S.var_name.end(), B->var_name.begin() + v0);
    std::copy(S.var_aux.begin(), S.var_aux.end(), B->var_aux.begin() + v0);
    std::copy(S.var_kind.begin(), S.var_kind.end(), B->var_kind.begin() + v0);
    std::copy(S.var_key.begin(), S.var_key.end(), B->var_key.begin() + v0);
    std::copy(S.var_tid.begin(), S.var_tid.end(), B->var_tid.begin() + v0);
    std::copy(S.aliases.begin(), S.aliases.end(), B->aliases.begin() + B->alias_off[s] * 2);
    for (size_t v = 0; v < S.hints.size(); ++v)
      std::copy(S.hints[v].begin(), S.hints[v].end(), B->hints.begin() + B->hint_off[v0 + v] * 8);
    B->state_key[s] = state_key_of(S, name_hash, n_names);
  }
  bool any_ops = false;
  for (uint32_t s = 0; s < n_states; ++s) any_ops |= !res[s].gpu_ops.empty();
  if (any_ops) {  // the strengthened formula on the original node indices (decision rows)
    B->dec_nodes.resize(nn);
#pragma omp parallel for schedule(static)
    for (int64_t s = 0; s < (int64_t)n_states; ++s) {
      std::copy(res[s].nodes.begin(), res[s].nodes.end(), B->dec_nodes.begin() + B->node_off[s]);
      const auto &ops = res[s].gpu_ops;
      for (size_t k = 0; k < ops.size(); k += 2) {
        mgp_node &nd = B->dec_nodes[B->node_off[s] + ops[k]];
        nd.op = (uint8_t)ops[k + 1];
        nd.width = 1;
        nd.a = nd.b = nd.c = -1;
        nd.p0 = nd.p1 = 0;
      }
    }
  }
  if (strengthened) {  // some state's GPU program differs: a separate node list and offsets
    B->gpu_node_off.assign(n_states + 1, 0);
    for (uint32_t s = 0; s < n_states; ++s)
      B->gpu_node_off[s + 1] = B->gpu_node_off[s] +
                               (res[s].gpu_nodes.empty() ? res[s].nodes.size() : res[s].gpu_nodes.size());
    B->gpu_nodes.resize(B->gpu_node_off[n_states]);
#pragma omp parallel for schedule(static)
    for (int64_t s = 0; s < (int64_t)n_states; ++s) {
      const auto &g = res[s].gpu_nodes.empty() ? res[s].nodes : res[s].gpu_nodes;
      std::copy(g.begin(), g.end(), B->gpu_nodes.begin() + B->gpu_node_off[s]);
    }
  }
  // the per-state results released in parallel: a 1 024-state batch is tens of thousands of
  // small vectors, and their serial release at the return cost as much as the copy above
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) res[s] = StateOut();
  if (getenv("MGP_FE_TIMING")) fprintf(stderr, "[fe] total %.3f ms\n", 1e3 * omp_get_wtime() - 1e3 * t_start);
  *out = B;
  return MGP_OK;
}

int mgp_fe_get(const mgp_fe_batch *B, int field, const void **ptr, uint64_t *count) {
  if (!B || !ptr || !count) return MGP_E_ARG;
  auto set = [&](const auto &v) {
    *ptr = v.empty() ? nullptr : (const void *)v.data();
    *count = v.size();
    return MGP_OK;
  };
  switch (field) {
    case MGP_FE_NODES: return set(B->nodes);
    case MGP_FE_GPU_NODES: return set(B->gpu_nodes.empty() ? B->nodes : B->gpu_nodes);
    case MGP_FE_NODE_OFF: return set(B->node_off);
    case MGP_FE_CONSTS: return set(B->consts);
    case MGP_FE_CONST_OFF: return set(B->const_off);
    case MGP_FE_VAR_OFF: return set(B->var_off);
    case MGP_FE_VAR_WIDTH: return set(B->var_width);
    case MGP_FE_VAR_FULL: return set(B->var_full);
    case MGP_FE_VAR_NAME: return set(B->var_name);
    case MGP_FE_VAR_AUX: return set(B->var_aux);
    case MGP_FE_VAR_KIND: return set(B->var_kind);
    case MGP_FE_HINT_OFF: return set(B->hint_off);
    case MGP_FE_HINTS: return set(B->hints);
    case MGP_FE_ALIAS_OFF: return set(B->alias_off);
    case MGP_FE_ALIASES: return set(B->aliases);
    case MGP_FE_FLAGS: return set(B->flags);
    case MGP_FE_VAR_KEY: return set(B->var_key);
    case MGP_FE_VAR_TID: return set(B->var_tid);
    case MGP_FE_STATE_KEY: return set(B->state_key);
    case MGP_FE_GPU_NODE_OFF: return set(B->gpu_nodes.empty() ? B->node_off : B->gpu_node_off);
    case MGP_FE_DEC_NODES: return set(B->dec_nodes.empty() ? B->nodes : B->dec_nodes);
    default: return MGP_E_ARG;
  }
}

// The states idx[0..n) of a built batch as a batch of their own, in that order: every
// per-state array sliced and concatenated (node, constant, slot and alias references are
// local to their state, so slices need no renumbering).  The same arrays a build of those
// states' roots would give, without walking the term arena again (solver.Prefilter splits a
// batch into candidate-memory groups and retry rounds this way).
int mgp_fe_select(const mgp_fe_batch *B, const uint32_t *idx, uint32_t n, mgp_fe_batch **out) {
  if (!B || !out || (n && !idx)) return MGP_E_ARG;
  *out = nullptr;
  for (uint32_t k = 0; k < n; ++k)
    if (idx[k] >= B->n_states) return MGP_E_ARG;
  mgp_fe_batch *S = fe_take();
  if (!S) return MGP_E_NOMEM;
  S->n_states = n;
  const bool gpu = !B->gpu_nodes.empty(), dec = !B->dec_nodes.empty();
  auto offsets = [&](const std::vector<uint64_t> &src, std::vector<uint64_t> &dst) {
    dst.assign((size_t)n + 1, 0);
    for (uint32_t k = 0; k < n; ++k) dst[k + 1] = dst[k] + (src[idx[k] + 1] - src[idx[k]]);
  };
  offsets(B->node_off, S->node_off);
  offsets(B->const_off, S->const_off);
  offsets(B->var_off, S->var_off);
  offsets(B->alias_off, S->alias_off);
  if (gpu) offsets(B->gpu_node_off, S->gpu_node_off);
  const uint64_t nv = S->var_off[n];
  S->hint_off.assign(nv + 1, 0);
  for (uint32_t k = 0; k < n; ++k) {
    const uint64_t v0 = B->var_off[idx[k]], d0 = S->var_off[k], V = S->var_off[k + 1] - d0;
    for (uint64_t v = 0; v < V; ++v) S->hint_off[d0 + v + 1] = B->hint_off[v0 + v + 1] - B->hint_off[v0 + v];
  }
  for (uint64_t v = 0; v < nv; ++v) S->hint_off[v + 1] += S->hint_off[v];
  S->nodes.resize(S->node_off[n]);
  if (dec) S->dec_nodes.resize(S->node_off[n]);
  if (gpu) S->gpu_nodes.resize(S->gpu_node_off[n]);
  S->consts.resize(S->const_off[n] * 8);
  S->var_width.resize(nv);
  S->var_full.resize(nv);
  S->var_name.resize(nv);
  S->var_aux.resize(nv);
  S->var_kind.resize(nv);
  S->var_key.resize(nv);
  S->var_tid.resize(nv);
  S->hints.resize(S->hint_off[nv] * 8);
  S->aliases.resize(S->alias_off[n] * 2);
  S->flags.assign(n, 0);
  S->state_key.assign(n, 0);
#pragma omp parallel for schedule(static) if (n > 64)
  for (int64_t k = 0; k < (int64_t)n; ++k) {
    const uint32_t s = idx[k];
    auto slice = [&](const auto &src, auto &dst, uint64_t from, uint64_t to, uint64_t at) {
      std::copy(src.begin() + from, src.begin() + to, dst.begin() + at);
    };
    slice(B->nodes, S->nodes, B->node_off[s], B->node_off[s + 1], S->node_off[k]);
    if (dec) slice(B->dec_nodes, S->dec_nodes, B->node_off[s], B->node_off[s + 1], S->node_off[k]);
    if (gpu) slice(B->gpu_nodes, S->gpu_nodes, B->gpu_node_off[s], B->gpu_node_off[s + 1], S->gpu_node_off[k]);
    slice(B->consts, S->consts, B->const_off[s] * 8, B->const_off[s + 1] * 8, S->const_off[k] * 8);
    const uint64_t v0 = B->var_off[s], v1 = B->var_off[s + 1], d0 = S->var_off[k];
    slice(B->var_width, S->var_width, v0, v1, d0);
    slice(B->var_full, S->var_full, v0, v1, d0);
    slice(B->var_name, S->var_name, v0, v1, d0);
    slice(B->var_aux, S->var_aux, v0, v1, d0);
    slice(B->var_kind, S->var_kind, v0, v1, d0);
    slice(B->var_key, S->var_key, v0, v1, d0);
    slice(B->var_tid, S->var_tid, v0, v1, d0);
    slice(B->hints, S->hints, B->hint_off[v0] * 8, B->hint_off[v1] * 8, S->hint_off[d0] * 8);
    slice(B->aliases, S->aliases, B->alias_off[s] * 2, B->alias_off[s + 1] * 2, S->alias_off[k] * 2);
    S->flags[k] = B->flags[s];
    S->state_key[k] = B->state_key[s];
  }
  *out = S;
  return MGP_OK;
}

void mgp_fe_free(mgp_fe_batch *B) {
  if (!B) return;
  {
    std::lock_guard<std::mutex> lk(fe_pool_mu());
    if (fe_pool().size() < 2) {
      fe_pool().push_back(B);
      return;
    }
  }
  delete B;
}

}  // extern "C"
