// mgp_lower.cpp — constraint DAG -> flat bytecode (host side).
//
// Per state:
//   1. validate the topologically ordered node list (operand indices point
//      backwards, root is Bool); values wider than 256 bits are split into
//      <= 256-bit pieces that only structural ops touch (mgp_ir.h);
//   2. expand uninterpreted-function applications (keccak256_<n> and its
//      inverse, keccak_function_manager.py:56-69, and base-array Selects) into
//      EQ/ITE chains: Ackermann expansion with a lazily built interpretation
//      (mgp_ir.h, MGP_OP_UFAPP / MGP_OP_UFINV);
//   3. re-pool constants (masked to the using node's width, de-duplicated);
//   4. liveness-based allocation of BV slots (per-lane LDS) and Bool bits,
//      with accumulator forwarding: an operand produced by the immediately
//      preceding BV instruction is read from registers (ACC) and only values
//      with a later use are stored;
//   5. emit header + instructions + constant pool;
//   6. append the micro-op re-encoding for the gfx950 assembly interpreter
//      (mgp_uop.cpp; layout in mythril_amd/uop_spec.py).
// States are independent; the batch is lowered in parallel with OpenMP.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "../../include/mgp.h"
#include "mgp_buf.h"

int mgp_uop_translate(const uint32_t *v1, std::vector<uint32_t> &out);  // mgp_uop.cpp

namespace {

// value reference during lowering
enum RefKind : uint8_t { R_NONE = 0, R_VAR, R_CONST, R_INS, R_BOOLC };

struct Ref {
  RefKind k = R_NONE;
  uint32_t idx = 0;  // var index / const pool index / vinstr index / bool const (0,1)
  bool operator==(const Ref &o) const { return k == o.k && idx == o.idx; }
};

struct VIns {
  uint8_t op;
  uint16_t width;   // result width (BV) or operand width (compare)
  bool is_bool;     // produces a Bool
  Ref a, b, c;
  uint32_t imm;
  Ref d;            // EQSEL: the else value (emitted as the accumulator)
};

inline bool op_is_bool_result(uint8_t op) {
  return (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) || (op >= MGP_OP_BAND && op <= MGP_OP_BEQ) ||
         op == MGP_OP_TRUE || op == MGP_OP_FALSE;
}
inline bool op_takes_bools(uint8_t op) { return op >= MGP_OP_BAND && op <= MGP_OP_BEQ; }

struct ConstKey {
  uint32_t w[8];
  bool operator==(const ConstKey &o) const { return memcmp(w, o.w, sizeof(w)) == 0; }
};
struct ConstHash {
  size_t operator()(const ConstKey &k) const {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 8; ++i) h = (h ^ k.w[i]) * 1099511628211ull;
    return (size_t)h;
  }
};

inline uint32_t limb_mask(uint32_t w, int l) {
  int lo = 32 * l;
  if ((int)w >= lo + 32) return 0xFFFFFFFFu;
  if ((int)w <= lo) return 0u;
  return (1u << (w - lo)) - 1u;
}

struct Lowered {
  std::vector<uint32_t> words;  // the v1 program
  std::vector<uint32_t> uops;   // the gfx950 interpreter's translation, stored right behind it
  uint8_t status = MGP_ST_OK;
};

struct LowerState {
  std::vector<VIns> ins;
  std::vector<ConstKey> pool;
  std::unordered_map<ConstKey, uint32_t, ConstHash> pool_map;
  uint32_t max_var = 0;  // 1 + highest var index used

  Ref add(uint8_t op, uint16_t width, bool is_bool, Ref a, Ref b = Ref(), Ref c = Ref(), uint32_t imm = 0,
          Ref d = Ref()) {
    ins.push_back(VIns{op, width, is_bool, a, b, c, imm, d});
    Ref r;
    r.k = R_INS;
    r.idx = (uint32_t)ins.size() - 1;
    return r;
  }
  Ref constant(const uint32_t *limbs, uint32_t width) {
    ConstKey k;
    for (int l = 0; l < 8; ++l) k.w[l] = limbs[l] & limb_mask(width, l);
    auto it = pool_map.find(k);
    Ref r;
    r.k = R_CONST;
    if (it != pool_map.end()) {
      r.idx = it->second;
    } else {
      r.idx = (uint32_t)pool.size();
      pool.push_back(k);
      pool_map.emplace(k, r.idx);
    }
    return r;
  }
};

// Instruction lists of finished lowerings, one per thread, reused by the next state on that
// thread: a WalletLibrary state's list is ~350 KB, and fresh memory per state is page faults,
// which the threads of a large batch take in turn (1 024-state corpus on a GPU box's host, 16
// threads: 25.3 -> 21.5 ms, page faults 28 -> 16 per state; one thread: 301 -> 290 ms).  A
// list past 8 MB is not kept.
thread_local std::vector<VIns> g_ins_pool;
// the same for the v1 program and the uop program of a state (recycled once copied out)
thread_local std::vector<uint32_t> g_words_pool, g_uops_pool;
template <typename T>
inline void recycle(std::vector<T> &v, std::vector<T> &pool) {
  if (v.capacity() > pool.capacity() && v.capacity() * sizeof(T) <= (8u << 20)) {
    v.clear();
    pool.swap(v);
  }
}
inline void ins_recycle(std::vector<VIns> &v) { recycle(v, g_ins_pool); }

// A value wider than one 256-bit slot (512-bit mapping preimages
// Concat(key, slot), keccak256_512 / its inverse, 257-bit overflow sums) is a
// list of <= 256-bit pieces, low bits first.  Only the structural ops act on
// such lists (mgp_ir.h, "wide values"); every piece is an ordinary narrow value.
struct Piece {
  Ref r;
  uint32_t w;
};
typedef std::vector<Piece> Pieces;

// a piece of an argument as base term + constant offset (sum_form in lower_one)
struct SumForm {
  Ref r, base;
  uint32_t w;
  uint32_t off[8];
};

struct UFApp {
  Pieces arg, val, fresh;  // argument, value, the application's own fresh variable(s)
  std::vector<SumForm> form;  // of arg, piece by piece (f applications only)
  Ref raw;  // one-piece value: its fresh variable unmasked (EQSEL masks what it selects)
};

// MGP_LOWER_WHY=1: name the source line of every "unsupported" verdict (diagnostics)
Lowered unsupported_at(int line) {
  static const bool why = getenv("MGP_LOWER_WHY") != nullptr;
  if (why) fprintf(stderr, "[mgp_lower] unsupported at mgp_lower.cpp:%d\n", line);
  Lowered L;
  L.status = MGP_ST_UNSUPPORTED;
  L.words = {0u, 0u, 0u, (uint32_t)MGP_ST_UNSUPPORTED, 0u, 0u, 0u, 0u};
  return L;
}

#define unsupported() unsupported_at(__LINE__)

// Lists of u32 per key (CSR) from (key, value) pairs in emission order: one allocation
// instead of one vector per instruction (20 000-instruction programs)
struct Lists {
  std::vector<uint32_t> off, val;
  const uint32_t *begin(uint32_t k) const { return val.data() + off[k]; }
  const uint32_t *end(uint32_t k) const { return val.data() + off[k + 1]; }
};
Lists make_lists(uint32_t n_keys, const std::vector<std::pair<uint32_t, uint32_t>> &kv) {
  Lists L;
  L.off.assign((size_t)n_keys + 1, 0u);
  for (const auto &p : kv) L.off[p.first + 1]++;
  for (uint32_t k = 0; k < n_keys; ++k) L.off[k + 1] += L.off[k];
  L.val.resize(kv.size());
  std::vector<uint32_t> pos(L.off.begin(), L.off.end() - 1);
  for (const auto &p : kv) L.val[pos[p.first]++] = p.second;
  return L;
}

// Scheduling, Bool demotion, liveness, slot allocation and emission of one prepared
// state (lower_one runs it once per schedule it tries on a copy of the prepared state).
Lowered finish_one(LowerState S, Ref root, uint32_t max_slots, int sched) {
  // ------------------------------------------- register-pressure scheduling
  // sched 1: depth-first post-order from the root, operand with the larger
  //          Sethi-Ullman need first (trees need O(log n) live values and a
  //          parent usually follows its last operand: accumulator forwarding);
  // sched 2: greedy list scheduling — among ready instructions take the one
  //          that frees the most BV values (last use) minus the one it creates,
  //          ties to the one reading the most recent result.
  // The caller keeps whichever schedule needs the fewest LDS slots.
  if (sched != 0) {
    const uint32_t n0 = (uint32_t)S.ins.size();
    auto kids = [&](uint32_t t, uint32_t out[4]) -> int {
      int k = 0;
      const VIns &I = S.ins[t];
      for (const Ref *r : {&I.a, &I.b, &I.c, &I.d})
        if (r->k == R_INS) {
          bool dup = false;
          for (int j = 0; j < k; ++j) dup |= out[j] == r->idx;
          if (!dup) out[k++] = r->idx;
        }
      return k;
    };
    std::vector<uint32_t> order;
    order.reserve(n0);
    if (sched == 1) {
      std::vector<uint32_t> need(n0, 1);
      for (uint32_t t = 0; t < n0; ++t) {
        uint32_t ch[4];
        const int k = kids(t, ch);
        uint32_t nd[4] = {0, 0, 0, 0};
        for (int i = 0; i < k; ++i) nd[i] = need[ch[i]];
        std::sort(nd, nd + k, [](uint32_t x, uint32_t y) { return x > y; });
        uint32_t m = 1;
        for (int i = 0; i < k; ++i) m = std::max(m, nd[i] + (uint32_t)i);
        need[t] = m;
      }
      std::vector<uint8_t> state(n0, 0);  // 0 new, 1 expanded, 2 emitted
      std::vector<uint32_t> stack;
      if (root.k == R_INS) stack.push_back(root.idx);
      while (!stack.empty()) {
        const uint32_t t = stack.back();
        if (state[t] == 2) { stack.pop_back(); continue; }
        if (state[t] == 1) { state[t] = 2; order.push_back(t); stack.pop_back(); continue; }
        state[t] = 1;
        uint32_t ch[4];
        const int k = kids(t, ch);
        std::sort(ch, ch + k, [&](uint32_t x, uint32_t y) { return need[x] < need[y]; });
        for (int i = 0; i < k; ++i)
          if (state[ch[i]] == 0) stack.push_back(ch[i]);
      }
    } else {
      // the greedy list scheduler rescans the ready list per step (quadratic): not worth it
      // for very long programs, whose other schedules are kept instead
      if (n0 > 1536) return unsupported();
      std::vector<uint32_t> uses(n0, 0), pending(n0, 0);
      std::vector<std::vector<uint32_t>> users(n0);
      for (uint32_t t = 0; t < n0; ++t) {
        uint32_t ch[4];
        const int k = kids(t, ch);
        pending[t] = (uint32_t)k;
        for (int i = 0; i < k; ++i) {
          uses[ch[i]]++;
          users[ch[i]].push_back(t);
        }
      }
      std::vector<uint32_t> ready;
      for (uint32_t t = 0; t < n0; ++t)
        if (pending[t] == 0) ready.push_back(t);
      int64_t last = -1;
      while (!ready.empty()) {
        size_t best = 0;
        int best_score = -1000, best_recent = -1;
        for (size_t r = 0; r < ready.size(); ++r) {
          const uint32_t t = ready[r];
          uint32_t ch[4];
          const int k = kids(t, ch);
          int score = 0, recent = 0;
          for (int i = 0; i < k; ++i) {
            if (!S.ins[ch[i]].is_bool && uses[ch[i]] == 1) score += 1;
            if ((int64_t)ch[i] == last) recent = 1;
          }
          if (!S.ins[t].is_bool && !users[t].empty()) score -= 1;
          if (score > best_score || (score == best_score && recent > best_recent)) {
            best = r, best_score = score, best_recent = recent;
          }
        }
        const uint32_t t = ready[best];
        ready.erase(ready.begin() + (ptrdiff_t)best);
        order.push_back(t);
        last = t;
        uint32_t ch[4];
        const int k = kids(t, ch);
        for (int i = 0; i < k; ++i) uses[ch[i]]--;
        for (uint32_t u : users[t])
          if (--pending[u] == 0) ready.push_back(u);
      }
    }
    if (order.size() == n0) {
      std::vector<uint32_t> remap(n0);
      for (uint32_t i = 0; i < n0; ++i) remap[order[i]] = i;
      std::vector<VIns> re(n0);
      for (uint32_t i = 0; i < n0; ++i) {
        VIns I = S.ins[order[i]];
        for (Ref *r : {&I.a, &I.b, &I.c, &I.d})
          if (r->k == R_INS) r->idx = remap[r->idx];
        re[i] = I;
      }
      S.ins.swap(re);
      if (root.k == R_INS) root.idx = remap[root.idx];
    }
  }

  // ------------------------------------------------ Bool pressure: demotion
  // At most MGP_BOOL_LIVE Bool values are live at once (the gfx950 interpreter's Bool
  // registers).  While the schedule needs more, the live Bool whose next read is
  // farthest becomes a 1-bit BV value: D = ITE(b, 1, 0) right after its definition and
  // EQ(D, 1) right before each reader.  BV values can spill, Bools cannot.
  {
    auto const_ref = [&](uint32_t v) {
      ConstKey k;
      memset(k.w, 0, sizeof(k.w));
      k.w[0] = v;
      Ref r;
      r.k = R_CONST;
      for (uint32_t i = 0; i < S.pool.size(); ++i)
        if (S.pool[i] == k) {
          r.idx = i;
          return r;
        }
      r.idx = (uint32_t)S.pool.size();
      S.pool.push_back(k);
      return r;
    };
    // the Bool operand positions of an instruction (ITE: the condition only)
    auto bool_refs = [](VIns &I, Ref *out[3]) -> int {
      if (op_takes_bools(I.op)) {
        out[0] = &I.a, out[1] = &I.b, out[2] = &I.c;
        return 3;
      }
      if (I.op == MGP_OP_ITE) {
        out[0] = &I.a;
        return 1;
      }
      return 0;
    };
    // one pass over the schedule plans every demotion (victim: the live Bool read farthest
    // in the future; a demoted Bool's readers need one short-lived EQ bit each, right
    // before them), then one rewrite applies them
    const uint32_t n0 = (uint32_t)S.ins.size();
    std::vector<int64_t> lu(n0, -1);
    std::vector<std::pair<uint32_t, uint32_t>> kv;
    std::vector<int64_t> last_t(n0, -1);
    for (uint32_t t = 0; t < n0; ++t) {
      Ref *br[3];
      const int k = bool_refs(S.ins[t], br);
      for (int i = 0; i < k; ++i)
        if (br[i]->k == R_INS) {
          lu[br[i]->idx] = std::max<int64_t>(lu[br[i]->idx], t);
          if (last_t[br[i]->idx] != (int64_t)t) kv.push_back({br[i]->idx, t}), last_t[br[i]->idx] = t;
        }
    }
    const Lists readers = make_lists(n0, kv);  // readers of each Bool, ascending
    if (root.k == R_INS) lu[root.idx] = std::max<int64_t>(lu[root.idx], n0);
    kv.clear();
    for (uint32_t t = 0; t < n0; ++t)
      if (S.ins[t].is_bool && lu[t] > (int64_t)t && lu[t] <= (int64_t)n0) kv.push_back({(uint32_t)lu[t], t});
    const Lists expire_at = make_lists(n0 + 1, kv);
    std::vector<uint8_t> demoted(n0, 0);
    bool any = false;
    std::vector<uint32_t> cur;  // live Bools holding a bit
    auto next_read = [&](uint32_t v, uint32_t t) -> int64_t {
      const uint32_t *it = std::lower_bound(readers.begin(v), readers.end(v), t);
      return it == readers.end(v) ? (int64_t)n0 : (int64_t)*it;
    };
    // demote the member of cur read farthest after t (not one t itself reads)
    auto demote_one = [&](uint32_t t, const uint32_t *keep, int n_keep) -> bool {
      int64_t best = -1;
      size_t at = 0;
      for (size_t j = 0; j < cur.size(); ++j) {
        bool kept = false;
        for (int q = 0; q < n_keep; ++q) kept |= keep[q] == cur[j];
        if (kept) continue;
        const int64_t nx = next_read(cur[j], t);
        if (nx > best) best = nx, at = j;
      }
      if (best < 0) return false;
      demoted[cur[at]] = 1;
      any = true;
      cur.erase(cur.begin() + (ptrdiff_t)at);
      return true;
    };
    for (uint32_t t = 0; t < n0; ++t) {
      Ref *br[3];
      const int k = bool_refs(S.ins[t], br);
      uint32_t rd[3];
      int n_rd = 0, transients = 0;
      for (int i = 0; i < k; ++i)
        if (br[i]->k == R_INS) {
          bool dup = false;
          for (int q = 0; q < n_rd; ++q) dup |= rd[q] == br[i]->idx;
          if (dup) continue;
          rd[n_rd++] = br[i]->idx;
          transients += demoted[br[i]->idx];
        }
      while (cur.size() + (size_t)transients > MGP_BOOL_LIVE)
        if (!demote_one(t, rd, n_rd)) return unsupported();
      for (const uint32_t *pv = expire_at.begin(t); pv != expire_at.end(t); ++pv) {
        const uint32_t v = *pv;
        auto it = std::find(cur.begin(), cur.end(), v);
        if (it != cur.end()) cur.erase(it);
      }
      if (S.ins[t].is_bool && lu[t] > (int64_t)t) {
        if (cur.size() >= MGP_BOOL_LIVE && !demote_one(t, nullptr, 0)) return unsupported();
        cur.push_back(t);
      }
    }
    if (any) {
      const Ref one = const_ref(1u), zero = const_ref(0u);
      std::vector<VIns> re;
      re.reserve(n0 + n0 / 4 + 8);
      std::vector<uint32_t> remap(n0, 0);
      std::vector<Ref> dref(n0);  // the 1-bit value of a demoted Bool
      for (uint32_t t = 0; t < n0; ++t) {
        VIns I = S.ins[t];
        for (Ref *r : {&I.a, &I.b, &I.c, &I.d})
          if (r->k == R_INS) r->idx = remap[r->idx];
        Ref *br[3], *nr[3];
        const int k = bool_refs(S.ins[t], br);
        bool_refs(I, nr);
        for (int i = 0; i < k; ++i) {
          if (br[i]->k != R_INS || !demoted[br[i]->idx]) continue;
          const uint32_t v = br[i]->idx;
          // one EQ per distinct demoted operand (BITE / BAND may read one Bool twice)
          Ref e;
          e.k = R_INS;
          e.idx = 0xFFFFFFFFu;
          for (int j = 0; j < i; ++j)
            if (br[j]->k == R_INS && br[j]->idx == v) e = *nr[j];
          if (e.idx == 0xFFFFFFFFu) {
            re.push_back(VIns{MGP_OP_EQ, 1, true, dref[v], one, Ref(), 0});
            e.idx = (uint32_t)re.size() - 1;
          }
          *nr[i] = e;
        }
        remap[t] = (uint32_t)re.size();
        re.push_back(I);
        if (demoted[t]) {
          Ref b;
          b.k = R_INS;
          b.idx = remap[t];
          re.push_back(VIns{MGP_OP_ITE, 1, false, b, one, zero, 0});
          dref[t].k = R_INS;
          dref[t].idx = (uint32_t)re.size() - 1;
        }
      }
      if (root.k == R_INS) {
        if (demoted[root.idx]) {
          re.push_back(VIns{MGP_OP_EQ, 1, true, dref[root.idx], one, Ref(), 0});
          root.idx = (uint32_t)re.size() - 1;
        } else {
          root.idx = remap[root.idx];
        }
      }
      S.ins.swap(re);
    }
  }

  // ---------------------------------------------------------- liveness
  const uint32_t n = (uint32_t)S.ins.size();
  std::vector<int64_t> last_use(n, -1);       // last instruction reading the value
  std::vector<uint8_t> needs_slot(n, 0);      // some use cannot be served from ACC
  std::vector<int64_t> prev_bv(n + 1, -1);    // last BV-producing instruction before t
  {
    int64_t last = -1;
    for (uint32_t t = 0; t < n; ++t) {
      prev_bv[t] = last;
      if (!S.ins[t].is_bool) last = t;
    }
    prev_bv[n] = last;
  }
  auto use = [&](const Ref &r, uint32_t t, bool bool_opnd) {
    if (r.k != R_INS) return;
    last_use[r.idx] = std::max<int64_t>(last_use[r.idx], t);
    if (!bool_opnd && prev_bv[t] != (int64_t)r.idx) needs_slot[r.idx] = 1;
  };
  for (uint32_t t = 0; t < n; ++t) {
    const VIns &I = S.ins[t];
    if (op_takes_bools(I.op)) {
      use(I.a, t, true); use(I.b, t, true); use(I.c, t, true);
    } else if (I.op == MGP_OP_ITE) {
      use(I.a, t, true); use(I.b, t, false); use(I.c, t, false);
    } else if (I.op == MGP_OP_EQSEL) {
      // a, b, c are read from slots (the accumulator holds the else value d; a d that
      // is not the previous BV result is moved into it first, from its slot)
      for (const Ref *r : {&I.a, &I.b, &I.c}) {
        use(*r, t, false);
        if (r->k == R_INS) needs_slot[r->idx] = 1;
      }
      use(I.d, t, false);
    } else {
      use(I.a, t, false); use(I.b, t, false); use(I.c, t, false);
    }
  }
  if (root.k == R_INS) last_use[root.idx] = std::max<int64_t>(last_use[root.idx], n);

  // ---------------------------------------------------------- allocation
  // LDS slots first (max_slots < MGP_LDS_SLOTS is a test knob that spills earlier), then
  // spill slots MGP_LDS_SLOTS.. (include/mgp_ir.h), up to MGP_MAX_SLOTS in all
  const uint32_t slot_cap = std::min<uint32_t>(max_slots ? max_slots : MGP_LDS_SLOTS, MGP_LDS_SLOTS);
  std::vector<int32_t> loc(n, -1);
  std::vector<uint32_t> free_slots, free_bools, free_spill;
  uint32_t next_spill = MGP_LDS_SLOTS;
  for (int32_t s = (int32_t)slot_cap - 1; s >= 0; --s) free_slots.push_back((uint32_t)s);
  for (int32_t b = MGP_BOOL_LIVE - 1; b >= 0; --b) free_bools.push_back((uint32_t)b);
  // fields naming a BV slot, for the access-count renumbering of spilling programs:
  // (word index, bit shift) of an operand (14-bit index) or of a STORE destination
  std::vector<std::pair<uint32_t, uint32_t>> slot_fields;
  std::vector<std::pair<uint32_t, uint32_t>> ekv;
  for (uint32_t t = 0; t < n; ++t)
    if (last_use[t] >= 0 && last_use[t] <= (int64_t)n) ekv.push_back({(uint32_t)last_use[t], t});
  const Lists expire = make_lists(n + 1, ekv);
  uint32_t slots_used = 0;

  std::vector<uint32_t> out;
  out.swap(g_words_pool);
  out.clear();
  out.reserve(4 + 4 * n + 8 * S.pool.size() + 4);
  out.resize(4, 0u);

  auto bv_opnd = [&](const Ref &r, uint32_t t) -> uint32_t {
    switch (r.k) {
      case R_VAR: return MGP_OPND(MGP_K_VAR, r.idx);
      case R_CONST: return MGP_OPND(MGP_K_CONST, r.idx);
      case R_INS:
        if (prev_bv[t] == (int64_t)r.idx) return MGP_OPND(MGP_K_ACC, 0);
        return MGP_OPND(MGP_K_SLOT, (uint32_t)loc[r.idx]);
      default: return 0;
    }
  };
  auto bool_opnd = [&](const Ref &r) -> uint32_t {
    if (r.k == R_BOOLC) return r.idx ? MGP_BOOL_TRUE : MGP_BOOL_FALSE;
    if (r.k == R_INS) return (uint32_t)loc[r.idx];
    return MGP_BOOL_FALSE;
  };

  auto in_slot = [&](const Ref &r, uint32_t t) { return r.k == R_INS && prev_bv[t] != (int64_t)r.idx; };
  uint32_t n_emit = 0;
  for (uint32_t t = 0; t < n; ++t) {
    const VIns &I = S.ins[t];
    uint32_t oa, ob = 0, oc = 0;
    uint32_t base = (uint32_t)out.size();
    if (op_takes_bools(I.op)) {
      oa = bool_opnd(I.a); ob = bool_opnd(I.b); oc = bool_opnd(I.c);
    } else if (I.op == MGP_OP_EQSEL) {
      if (!(I.d.k == R_INS && prev_bv[t] == (int64_t)I.d.idx)) {
        // the else value into the accumulator: MOV d (a variable, constant or slot)
        out.push_back((uint32_t)MGP_OP_MOV | (((uint32_t)(I.width - 1) & 0xFFu) << 8));
        out.push_back(bv_opnd(I.d, t) & 0xFFFFu);
        out.push_back(0u);
        out.push_back(0u);
        if (in_slot(I.d, t)) slot_fields.push_back({base + 1, 0});
        ++n_emit;
      }
      base = (uint32_t)out.size();  // this instruction's first word
      auto no_acc = [&](const Ref &r) {
        return r.k == R_INS ? MGP_OPND(MGP_K_SLOT, (uint32_t)loc[r.idx]) : bv_opnd(r, t);
      };
      oa = no_acc(I.a); ob = no_acc(I.b); oc = no_acc(I.c);
      if (I.a.k == R_INS) slot_fields.push_back({base + 1, 0});
      if (I.b.k == R_INS) slot_fields.push_back({base + 1, 16});
      if (I.c.k == R_INS) slot_fields.push_back({base + 2, 0});
    } else if (I.op == MGP_OP_ITE) {
      oa = bool_opnd(I.a); ob = bv_opnd(I.b, t); oc = bv_opnd(I.c, t);
      if (in_slot(I.b, t)) slot_fields.push_back({base + 1, 16});
      if (in_slot(I.c, t)) slot_fields.push_back({base + 2, 0});
    } else {
      oa = bv_opnd(I.a, t);
      ob = I.b.k != R_NONE ? bv_opnd(I.b, t) : 0u;
      oc = I.c.k != R_NONE ? bv_opnd(I.c, t) : 0u;
      if (in_slot(I.a, t)) slot_fields.push_back({base + 1, 0});
      if (I.b.k != R_NONE && in_slot(I.b, t)) slot_fields.push_back({base + 1, 16});
      if (I.c.k != R_NONE && in_slot(I.c, t)) slot_fields.push_back({base + 2, 0});
    }
    // operands read first: free values whose last use is this instruction
    for (const uint32_t *pv = expire.begin(t); pv != expire.end(t); ++pv) {
      const uint32_t v = *pv;
      if (loc[v] < 0) continue;
      if (S.ins[v].is_bool) free_bools.push_back((uint32_t)loc[v]);
      else if ((uint32_t)loc[v] >= MGP_LDS_SLOTS) free_spill.push_back((uint32_t)loc[v]);
      else free_slots.push_back((uint32_t)loc[v]);
    }
    uint32_t dst = 0, flags = 0;
    const bool live = last_use[t] > (int64_t)t;
    if (I.is_bool) {
      if (live) {
        if (free_bools.empty()) return unsupported();
        dst = free_bools.back();
        free_bools.pop_back();
        loc[t] = (int32_t)dst;
      } else {
        return unsupported();  // unreachable after DCE
      }
    } else if (live && needs_slot[t]) {
      if (!free_slots.empty()) {
        dst = free_slots.back();
        free_slots.pop_back();
      } else if (!free_spill.empty()) {
        dst = free_spill.back();
        free_spill.pop_back();
      } else {
        if (next_spill >= MGP_MAX_SLOTS) return unsupported();
        dst = next_spill++;
      }
      loc[t] = (int32_t)dst;
      slots_used = std::max(slots_used, dst + 1);
      flags = MGP_INS_STORE;
      slot_fields.push_back({base, 16});
    }
    const uint32_t width_field = (uint32_t)(I.width ? I.width - 1 : 0) & 0xFFu;
    out.push_back((uint32_t)I.op | (width_field << 8) | (dst << 16) | (flags << 24));
    out.push_back((oa & 0xFFFFu) | (ob << 16));
    out.push_back((oc & 0xFFFFu) | ((I.imm & 0xFFFFu) << 16));
    out.push_back(dst >> 8);  // a BV destination past slot 255 (WalletLibrary's input-order programs)
    ++n_emit;
  }
  // RET
  out.push_back((uint32_t)MGP_OP_RET);
  out.push_back(bool_opnd(root));
  out.push_back(0u);
  out.push_back(0u);
  ++n_emit;

  // a spilling program: slot numbers by access count (reads + stores), most used first,
  // so that the LDS slots (and the gfx950 interpreter's register slots) hold the hot values
  static const bool norenum_dbg = getenv("MGP_LOWER_NORENUM") != nullptr;
  if (slots_used > MGP_LDS_SLOTS && slot_cap == MGP_LDS_SLOTS && !norenum_dbg) {
    auto field = [&](const std::pair<uint32_t, uint32_t> &f) -> uint32_t {
      return f.first % 4u == 0u ? ((out[f.first] >> 16) & 0xFFu) | ((out[f.first + 3] & 0xFFu) << 8)
                                : (out[f.first] >> f.second) & 0x3FFFu;
    };
    std::vector<uint32_t> cnt(slots_used, 0), by(slots_used), rank(slots_used);
    for (const auto &f : slot_fields) cnt[field(f)]++;
    for (uint32_t s = 0; s < slots_used; ++s) by[s] = s;
    std::stable_sort(by.begin(), by.end(), [&](uint32_t x, uint32_t y) { return cnt[x] > cnt[y]; });
    for (uint32_t r = 0; r < slots_used; ++r) rank[by[r]] = r;
    for (const auto &f : slot_fields) {
      const uint32_t nw = rank[field(f)];
      if (f.first % 4u == 0u) {
        out[f.first] = (out[f.first] & ~(0xFFu << 16)) | ((nw & 0xFFu) << 16);
        out[f.first + 3] = nw >> 8;
      } else out[f.first] = (out[f.first] & ~(0x3FFFu << f.second)) | (nw << f.second);
    }
  }

  out[0] = n_emit;
  out[1] = (uint32_t)S.pool.size();
  out[2] = slots_used;
  out[3] = (uint32_t)MGP_ST_OK | (S.max_var << 8);
  for (const ConstKey &k : S.pool)
    for (int l = 0; l < 8; ++l) out.push_back(k.w[l]);
  while (out.size() % 4) out.push_back(0u);
  for (int k = 0; k < 4; ++k) out.push_back(0u);  // the kernel prefetches one instruction past RET
  ins_recycle(S.ins);
  Lowered L;
  L.words.swap(out);
  return L;
}


Lowered lower_one(const mgp_node *nodes, uint64_t n_nodes, const uint32_t *consts, uint64_t n_consts,
                  uint32_t max_slots, const int *scheds, int n_scheds, std::vector<uint32_t> *uops,
                  bool par_scheds = false) {
  if (n_nodes == 0) return unsupported();
  LowerState S;
  S.ins.swap(g_ins_pool);
  S.ins.clear();
  S.ins.reserve((size_t)n_nodes * 4u + 64u);  // UF chains and wide pieces expand nodes; fewer regrowths
  std::vector<Ref> val(n_nodes);
  std::vector<uint16_t> wid(n_nodes);
  std::vector<uint8_t> isb(n_nodes);
  std::vector<Pieces> wide(n_nodes);  // non-empty iff wid > MGP_MAX_WIDTH
  std::unordered_map<uint32_t, std::vector<UFApp>> fapps, iapps;

  // ------------------------------------------------ wide-value helpers
  auto pieces_of = [&](int32_t j) -> Pieces {
    if (wid[j] > MGP_MAX_WIDTH) return wide[j];
    return Pieces{Piece{val[j], wid[j]}};
  };
  // bits [lo, lo + n) of a piece list, as a piece list
  auto slice = [&](const Pieces &p, uint32_t lo, uint32_t n) -> Pieces {
    Pieces out;
    uint32_t off = 0;
    for (const Piece &q : p) {
      const uint32_t a = std::max(lo, off), b = std::min(lo + n, off + q.w);
      if (a < b) {
        if (a == off && b - a == q.w) out.push_back(q);
        else out.push_back(Piece{S.add(MGP_OP_EXTRACT, (uint16_t)(b - a), false, q.r, Ref(), Ref(), a - off), b - a});
      }
      off += q.w;
    }
    return out;
  };
  // cut two equal-width piece lists at the union of their boundaries
  auto align = [&](const Pieces &p, const Pieces &q, Pieces &pa, Pieces &qa) {
    std::vector<uint32_t> cuts;
    uint32_t o = 0;
    for (const Piece &x : p) cuts.push_back(o += x.w);
    o = 0;
    for (const Piece &x : q) cuts.push_back(o += x.w);
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    uint32_t lo = 0;
    for (uint32_t c : cuts) {
      Pieces a = slice(p, lo, c - lo), b = slice(q, lo, c - lo);
      pa.push_back(a[0]);
      qa.push_back(b[0]);
      lo = c;
    }
  };
  auto eq_pieces = [&](const Pieces &p, const Pieces &q) -> Ref {
    if (p.size() == 1 && q.size() == 1) return S.add(MGP_OP_EQ, (uint16_t)p[0].w, true, p[0].r, q[0].r);
    Pieces pa, qa;
    align(p, q, pa, qa);
    Ref e;
    for (size_t k = 0; k < pa.size(); ++k) {
      Ref ek = S.add(MGP_OP_EQ, (uint16_t)pa[k].w, true, pa[k].r, qa[k].r);
      e = (k == 0) ? ek : S.add(MGP_OP_BAND, 1, true, e, ek);
    }
    return e;
  };
  // equality of two UF arguments known at lowering time: 1 equal, 0 different, -1 unknown.
  // Constants are pooled by value, so two constant pieces are equal iff their pool
  // indices are.  Concrete arguments (calldata / storage indices) are the common case,
  // and folding them keeps the Ackermann chain from holding every earlier value live.
  // A piece that is a sum of one symbolic term and constants (calldata indices
  // 4 + offset + i, calldata.py:219-232 with a symbolic ABI offset) is compared by its
  // base term and its constant offset (mod 2^w): two such indices of one base are equal
  // iff their offsets are, so the selects of one symbolic word never test each other.
  auto sum_form = [&](Ref r, uint32_t w, Ref *base, uint32_t off[8]) {
    memset(off, 0, 8 * sizeof(uint32_t));
    auto addc = [&](const ConstKey &c) {
      uint64_t cy = 0;
      for (int l = 0; l < 8; ++l) {
        cy += (uint64_t)off[l] + c.w[l];
        off[l] = (uint32_t)cy;
        cy >>= 32;
      }
    };
    for (int depth = 0; depth < 64 && r.k == R_INS; ++depth) {
      const VIns &I = S.ins[r.idx];
      if (I.op != MGP_OP_ADD || I.width != w) break;
      if (I.b.k == R_CONST) addc(S.pool[I.b.idx]), r = I.a;
      else if (I.a.k == R_CONST) addc(S.pool[I.a.idx]), r = I.b;
      else break;
    }
    if (r.k == R_CONST) {  // a constant: base none, offset = its value
      addc(S.pool[r.idx]);
      r = Ref();
    }
    for (int l = 0; l < 8; ++l) off[l] &= limb_mask(w, l);
    *base = r;
  };
  auto known_eq = [&](const Pieces &p, const Pieces &q) -> int {
    if (p.size() != q.size()) return -1;
    bool all = true;
    for (size_t k = 0; k < p.size(); ++k) {
      if (p[k].w != q[k].w) return -1;
      if (p[k].r == q[k].r) continue;
      if (p[k].r.k == R_CONST && q[k].r.k == R_CONST) return 0;
      Ref bp, bq;
      uint32_t op_[8], oq[8];
      sum_form(p[k].r, p[k].w, &bp, op_);
      sum_form(q[k].r, q[k].w, &bq, oq);
      if (bp == bq) {
        if (memcmp(op_, oq, sizeof(op_)) != 0) return 0;
        continue;
      }
      all = false;
    }
    return all ? 1 : -1;
  };
  // known_eq on sum forms computed once per application: the f-application chains compare
  // every new argument with every earlier one (WalletLibrary's states: ~6 500 comparisons)
  auto forms_of = [&](const Pieces &p) {
    std::vector<SumForm> f(p.size());
    for (size_t k = 0; k < p.size(); ++k) {
      f[k].r = p[k].r;
      f[k].w = p[k].w;
      sum_form(p[k].r, p[k].w, &f[k].base, f[k].off);
    }
    return f;
  };
  auto known_eq_forms = [](const std::vector<SumForm> &p, const std::vector<SumForm> &q) -> int {
    if (p.size() != q.size()) return -1;
    bool all = true;
    for (size_t k = 0; k < p.size(); ++k) {
      if (p[k].w != q[k].w) return -1;
      if (p[k].r == q[k].r) continue;
      if (p[k].r.k == R_CONST && q[k].r.k == R_CONST) return 0;
      if (p[k].base == q[k].base) {
        if (memcmp(p[k].off, q[k].off, sizeof(p[k].off)) != 0) return 0;
        continue;
      }
      all = false;
    }
    return all ? 1 : -1;
  };
  auto ite_pieces = [&](Ref c, const Pieces &p, const Pieces &q) -> Pieces {
    if (p.size() == 1 && q.size() == 1) return Pieces{Piece{S.add(MGP_OP_ITE, (uint16_t)p[0].w, false, c, p[0].r, q[0].r), p[0].w}};
    Pieces pa, qa, out;
    align(p, q, pa, qa);
    for (size_t k = 0; k < pa.size(); ++k)
      out.push_back(Piece{S.add(MGP_OP_ITE, (uint16_t)pa[k].w, false, c, pa[k].r, qa[k].r), pa[k].w});
    return out;
  };
  auto const_small = [&](uint32_t v, uint32_t w) -> Ref {
    uint32_t l[8] = {v, 0, 0, 0, 0, 0, 0, 0};
    return S.constant(l, w);
  };
  auto const_ones = [&](uint32_t w) -> Ref {
    static const uint32_t ones[8] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
    return S.constant(ones, w);
  };
  // piecewise bitwise ops; ADD / SUB with a carry (borrow) chain between pieces:
  //   carry_out = NOT BVAddNoOverflow(a_k, b_k) OR (carry_in AND a_k + b_k == ~0)
  //   borrow_out = a_k <u b_k OR (borrow_in AND a_k == b_k)
  auto arith_pieces = [&](uint8_t op, const Pieces &p, const Pieces &q) -> Pieces {
    Pieces pa, qa, out;
    align(p, q, pa, qa);
    Ref cy;
    bool have_cy = false;
    for (size_t k = 0; k < pa.size(); ++k) {
      const uint16_t pw = (uint16_t)pa[k].w;
      Ref r = S.add(op, pw, false, pa[k].r, qa[k].r);
      Ref part = r;
      if (have_cy) r = S.add(op, pw, false, r, S.add(MGP_OP_ITE, pw, false, cy, const_small(1, pw), const_small(0, pw)));
      if ((op == MGP_OP_ADD || op == MGP_OP_SUB) && k + 1 < pa.size()) {
        Ref c1 = (op == MGP_OP_ADD) ? S.add(MGP_OP_BNOT, 1, true, S.add(MGP_OP_UADD_NOOVF, pw, true, pa[k].r, qa[k].r))
                                    : S.add(MGP_OP_ULT, pw, true, pa[k].r, qa[k].r);
        if (have_cy) {
          Ref c2 = (op == MGP_OP_ADD) ? S.add(MGP_OP_EQ, pw, true, part, const_ones(pw))
                                      : S.add(MGP_OP_EQ, pw, true, pa[k].r, qa[k].r);
          c1 = S.add(MGP_OP_BOR, 1, true, c1, S.add(MGP_OP_BAND, 1, true, cy, c2));
        }
        cy = c1;
        have_cy = true;
      }
      out.push_back(Piece{r, pw});
    }
    return out;
  };
  // a <u b over pieces: lt_k = a_k <u b_k OR (a_k == b_k AND lt_{k-1})
  auto ult_pieces = [&](const Pieces &p, const Pieces &q) -> Ref {
    Pieces pa, qa;
    align(p, q, pa, qa);
    Ref lt;
    for (size_t k = 0; k < pa.size(); ++k) {
      const uint16_t pw = (uint16_t)pa[k].w;
      Ref l = S.add(MGP_OP_ULT, pw, true, pa[k].r, qa[k].r);
      if (k) l = S.add(MGP_OP_BOR, 1, true, l, S.add(MGP_OP_BAND, 1, true, S.add(MGP_OP_EQ, pw, true, pa[k].r, qa[k].r), lt));
      lt = l;
    }
    return lt;
  };
  // concatenation of narrow pieces (total <= 256) into one value
  auto join = [&](const Pieces &p) -> Ref {
    Ref r = p[0].r;
    uint32_t w = p[0].w;
    for (size_t k = 1; k < p.size(); ++k) {
      r = S.add(MGP_OP_CONCAT, (uint16_t)(w + p[k].w), false, p[k].r, r, Ref(), w);
      w += p[k].w;
    }
    return r;
  };
  // a * b mod 2^w over 128-bit limbs: every limb product is exact in one 256-bit MUL
  // (limbs are stored zero-extended); column k sums the low halves of the products
  // a_i b_j with i + j = k, the high halves of those with i + j = k - 1 and the carry
  // out of column k - 1 (each term < 2^128, so a column never wraps 256 bits)
  auto mul_pieces = [&](const Pieces &p, const Pieces &q, uint32_t w) -> Pieces {
    const uint32_t n = (w + 127) / 128;
    std::vector<Ref> a(n), b(n), lo, hi;
    for (uint32_t j = 0; j < n; ++j) {
      const uint32_t lw = std::min<uint32_t>(128, w - 128 * j);
      a[j] = join(slice(p, 128 * j, lw));
      b[j] = join(slice(q, 128 * j, lw));
    }
    std::vector<std::vector<Ref>> col(n + 1);
    for (uint32_t i = 0; i < n; ++i)
      for (uint32_t j = 0; i + j < n; ++j) {
        Ref pr = S.add(MGP_OP_MUL, 256, false, a[i], b[j]);
        col[i + j].push_back(S.add(MGP_OP_EXTRACT, 128, false, pr, Ref(), Ref(), 0));
        if (i + j + 1 < n) col[i + j + 1].push_back(S.add(MGP_OP_EXTRACT, 128, false, pr, Ref(), Ref(), 128));
      }
    Pieces limbs;
    Ref carry;
    bool have_carry = false;
    for (uint32_t k = 0; k < n; ++k) {
      Ref acc = col[k][0];
      for (size_t t = 1; t < col[k].size(); ++t) acc = S.add(MGP_OP_ADD, 256, false, acc, col[k][t]);
      if (have_carry) acc = S.add(MGP_OP_ADD, 256, false, acc, carry);
      const uint32_t lw = std::min<uint32_t>(128, w - 128 * k);
      limbs.push_back(Piece{S.add(MGP_OP_EXTRACT, (uint16_t)lw, false, acc, Ref(), Ref(), 0), lw});
      if (k + 1 < n) {
        carry = S.add(MGP_OP_EXTRACT, 128, false, acc, Ref(), Ref(), 128);
        have_carry = true;
      }
    }
    Pieces out;  // pairs of limbs -> 256-bit pieces
    for (size_t k = 0; k < limbs.size(); k += 2) {
      if (k + 1 < limbs.size()) out.push_back(Piece{join(Pieces{limbs[k], limbs[k + 1]}), limbs[k].w + limbs[k + 1].w});
      else out.push_back(limbs[k]);
    }
    return out;
  };
  // a w-bit value held in consecutive variables first, first+1, ... (low first)
  auto var_pieces = [&](uint32_t first, uint32_t w) -> Pieces {
    Pieces out;
    for (uint32_t off = 0, k = 0; off < w; off += MGP_MAX_WIDTH, ++k) {
      const uint32_t pw = std::min<uint32_t>(MGP_MAX_WIDTH, w - off);
      Ref v;
      v.k = R_VAR;
      v.idx = first + k;
      out.push_back(Piece{pw < 256u ? S.add(MGP_OP_MOV, (uint16_t)pw, false, v) : v, pw});
    }
    S.max_var = std::max(S.max_var, first + (w + MGP_MAX_WIDTH - 1) / MGP_MAX_WIDTH);
    return out;
  };
  auto wid_of = [](const Pieces &p) -> uint32_t {
    uint32_t w = 0;
    for (const Piece &q : p) w += q.w;
    return w;
  };
  auto set_val = [&](uint64_t i, const Pieces &p) {
    if (wid[i] > MGP_MAX_WIDTH) wide[i] = p;
    else val[i] = p.size() == 1 ? p[0].r : join(p);
  };

  // (round 6) bits 256.. of a piece list are constant zero: a zero-extended narrow value, a
  // Concat under zero constant pieces.  Division, right shifts and signed compares of such
  // values are the 256-bit ops on their low pieces (a zero sign bit makes ASHR a LSHR and a
  // signed compare an unsigned one); any other wide operand of them stays unsupported.
  auto high_zero = [&](const Pieces &p) -> bool {
    uint32_t off = 0;
    for (const Piece &q : p) {
      const uint32_t end = off + q.w;
      if (end > MGP_MAX_WIDTH) {
        if (q.r.k != R_CONST) return false;
        const ConstKey &c = S.pool[q.r.idx];
        for (uint32_t b = off >= MGP_MAX_WIDTH ? 0u : MGP_MAX_WIDTH - off; b < q.w; ++b)
          if ((c.w[b >> 5] >> (b & 31u)) & 1u) return false;
      }
      off = end;
    }
    return true;
  };
  for (uint64_t i = 0; i < n_nodes; ++i) {
    const mgp_node &nd = nodes[i];
    const uint8_t op = nd.op;
    const bool rb = op_is_bool_result(op);
    uint32_t w = rb ? 1u : nd.width;
    if (!rb && (w == 0 || w > MGP_MAX_WIDE)) return unsupported();
    auto opnd = [&](int32_t j) -> bool { return j >= 0 && (uint64_t)j < i; };
    auto is_wide = [&](int32_t j) -> bool { return opnd(j) && wid[j] > MGP_MAX_WIDTH; };
    wid[i] = (uint16_t)w;
    isb[i] = rb;
    if (!rb && w > MGP_MAX_WIDTH) {
      // ---------------------------------------- wide results: structural ops only
      const uint32_t k = (w + MGP_MAX_WIDTH - 1) / MGP_MAX_WIDTH;
      switch (op) {
        case MGP_OP_VAR:
          if (nd.p0 + k > 0x3FFFu) return unsupported();
          wide[i] = var_pieces(nd.p0, w);
          break;
        case MGP_OP_CONST: {
          if ((uint64_t)nd.p0 + k > n_consts) return unsupported();
          for (uint32_t j = 0; j < k; ++j) {
            const uint32_t pw = std::min<uint32_t>(MGP_MAX_WIDTH, w - j * MGP_MAX_WIDTH);
            wide[i].push_back(Piece{S.constant(consts + (size_t)(nd.p0 + j) * 8u, pw), pw});
          }
          break;
        }
        case MGP_OP_CONCAT: {
          if (!opnd(nd.a) || !opnd(nd.b) || isb[nd.a] || isb[nd.b]) return unsupported();
          if ((uint32_t)wid[nd.a] + wid[nd.b] != w) return unsupported();
          wide[i] = pieces_of(nd.b);
          for (const Piece &q : pieces_of(nd.a)) wide[i].push_back(q);
          break;
        }
        case MGP_OP_EXTRACT: {
          if (!opnd(nd.a) || isb[nd.a] || nd.p0 < nd.p1 || nd.p0 >= wid[nd.a] || nd.p0 - nd.p1 + 1 != w)
            return unsupported();
          wide[i] = slice(pieces_of(nd.a), nd.p1, w);
          break;
        }
        case MGP_OP_ZEXT: {
          if (!opnd(nd.a) || isb[nd.a] || wid[nd.a] > w) return unsupported();
          wide[i] = pieces_of(nd.a);
          static const uint32_t zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          for (uint32_t off = wid[nd.a]; off < w;) {
            const uint32_t pw = std::min<uint32_t>(MGP_MAX_WIDTH, w - off);
            wide[i].push_back(Piece{S.constant(zero, pw), pw});
            off += pw;
          }
          break;
        }
        case MGP_OP_ITE: {
          if (!opnd(nd.a) || !opnd(nd.b) || !opnd(nd.c) || !isb[nd.a] || isb[nd.b] || isb[nd.c]) return unsupported();
          if (wid[nd.b] != w || wid[nd.c] != w) return unsupported();
          wide[i] = ite_pieces(val[nd.a], pieces_of(nd.b), pieces_of(nd.c));
          break;
        }
        case MGP_OP_ADD: case MGP_OP_SUB: case MGP_OP_AND: case MGP_OP_OR: case MGP_OP_XOR: {
          if (!opnd(nd.a) || !opnd(nd.b) || isb[nd.a] || isb[nd.b] || wid[nd.a] != w || wid[nd.b] != w)
            return unsupported();
          wide[i] = arith_pieces(op, wide[nd.a], wide[nd.b]);
          break;
        }
        case MGP_OP_MUL: {
          if (!opnd(nd.a) || !opnd(nd.b) || isb[nd.a] || isb[nd.b] || wid[nd.a] != w || wid[nd.b] != w)
            return unsupported();
          wide[i] = mul_pieces(wide[nd.a], wide[nd.b], w);
          break;
        }
        case MGP_OP_NOT: {
          if (!opnd(nd.a) || isb[nd.a] || wid[nd.a] != w) return unsupported();
          for (const Piece &q : wide[nd.a]) wide[i].push_back(Piece{S.add(MGP_OP_NOT, (uint16_t)q.w, false, q.r), q.w});
          break;
        }
        case MGP_OP_UDIV: case MGP_OP_UREM: case MGP_OP_LSHR: case MGP_OP_ASHR: {
          if (!opnd(nd.a) || !opnd(nd.b) || isb[nd.a] || isb[nd.b] || wid[nd.a] != w || wid[nd.b] != w)
            return unsupported();
          const Pieces &pa = wide[nd.a], &pb = wide[nd.b];
          if (!high_zero(pa) || !high_zero(pb)) return unsupported();
          const Ref la = join(slice(pa, 0, MGP_MAX_WIDTH)), lb = join(slice(pb, 0, MGP_MAX_WIDTH));
          wide[i].push_back(Piece{S.add(op == MGP_OP_ASHR ? MGP_OP_LSHR : op, MGP_MAX_WIDTH, false, la, lb),
                                  MGP_MAX_WIDTH});
          // a w-bit x / 0 is 2^w - 1 (z3 bvudiv): the high pieces are ones then, else zero
          Ref by0;
          if (op == MGP_OP_UDIV) by0 = S.add(MGP_OP_EQ, MGP_MAX_WIDTH, true, lb, const_small(0, MGP_MAX_WIDTH));
          for (uint32_t off = MGP_MAX_WIDTH; off < w;) {
            const uint32_t pw = std::min<uint32_t>(MGP_MAX_WIDTH, w - off);
            const Ref z = const_small(0, pw);
            wide[i].push_back(Piece{op == MGP_OP_UDIV ? S.add(MGP_OP_ITE, (uint16_t)pw, false, by0, const_ones(pw), z) : z,
                                    pw});
            off += pw;
          }
          break;
        }
        case MGP_OP_UFAPP:
        case MGP_OP_UFINV:
          break;  // below, shared with narrow results
        default:
          return unsupported();
      }
      if (op != MGP_OP_UFAPP && op != MGP_OP_UFINV) continue;
    }
    // narrow results: a wide operand is only legal where the case below says so
    if (is_wide(nd.a) || is_wide(nd.b) || is_wide(nd.c)) {
      const bool sgn = op == MGP_OP_SLT || op == MGP_OP_SLE || op == MGP_OP_SGT || op == MGP_OP_SGE;
      const bool ok = op == MGP_OP_EXTRACT || op == MGP_OP_UFAPP || op == MGP_OP_UFINV ||
                      ((op == MGP_OP_EQ || op == MGP_OP_ULT || op == MGP_OP_ULE || op == MGP_OP_UGT ||
                        op == MGP_OP_UGE) && !isb[nd.a] && !isb[nd.b]) ||
                      (sgn && opnd(nd.a) && opnd(nd.b) && !isb[nd.a] && !isb[nd.b] && wid[nd.a] == wid[nd.b] &&
                       high_zero(wide[nd.a]) && high_zero(wide[nd.b]));
      if (!ok) return unsupported();
    }
    switch (op) {
      case MGP_OP_VAR: {
        if (nd.p0 >= 0x3FFFu) return unsupported();
        S.max_var = std::max(S.max_var, nd.p0 + 1);
        Ref v;
        v.k = R_VAR;
        v.idx = nd.p0;
        val[i] = (w < 256u) ? S.add(MGP_OP_MOV, (uint16_t)w, false, v) : v;
        break;
      }
      case MGP_OP_CONST: {
        if (nd.p0 >= n_consts) return unsupported();
        val[i] = S.constant(consts + (size_t)nd.p0 * 8u, w);
        break;
      }
      case MGP_OP_TRUE:
      case MGP_OP_FALSE: {
        Ref r;
        r.k = R_BOOLC;
        r.idx = (op == MGP_OP_TRUE) ? 1u : 0u;
        val[i] = r;
        break;
      }
      case MGP_OP_ADD: case MGP_OP_SUB: case MGP_OP_MUL: case MGP_OP_UDIV: case MGP_OP_UREM:
      case MGP_OP_SDIV: case MGP_OP_SREM: case MGP_OP_SMOD: case MGP_OP_AND: case MGP_OP_OR:
      case MGP_OP_XOR: case MGP_OP_SHL: case MGP_OP_LSHR: case MGP_OP_ASHR: {
        if (!opnd(nd.a) || !opnd(nd.b)) return unsupported();
        if (isb[nd.a] || isb[nd.b] || wid[nd.a] != w || wid[nd.b] != w) return unsupported();
        val[i] = S.add(op, (uint16_t)w, false, val[nd.a], val[nd.b]);
        break;
      }
      case MGP_OP_NOT: case MGP_OP_NEG: {
        if (!opnd(nd.a) || isb[nd.a] || wid[nd.a] != w) return unsupported();
        val[i] = S.add(op, (uint16_t)w, false, val[nd.a]);
        break;
      }
      case MGP_OP_EXTRACT: {
        if (!opnd(nd.a) || isb[nd.a]) return unsupported();
        const uint32_t hi = nd.p0, lo = nd.p1;
        if (hi < lo || hi >= wid[nd.a] || hi - lo + 1 != w) return unsupported();
        if (wid[nd.a] > MGP_MAX_WIDTH) { val[i] = join(slice(wide[nd.a], lo, w)); break; }
        if (lo == 0 && w == wid[nd.a]) { val[i] = val[nd.a]; break; }
        val[i] = S.add(MGP_OP_EXTRACT, (uint16_t)w, false, val[nd.a], Ref(), Ref(), lo);
        break;
      }
      case MGP_OP_CONCAT: {
        if (!opnd(nd.a) || !opnd(nd.b) || isb[nd.a] || isb[nd.b]) return unsupported();
        if ((uint32_t)wid[nd.a] + wid[nd.b] != w) return unsupported();
        val[i] = S.add(MGP_OP_CONCAT, (uint16_t)w, false, val[nd.a], val[nd.b], Ref(), wid[nd.b]);
        break;
      }
      case MGP_OP_ZEXT: {
        if (!opnd(nd.a) || isb[nd.a] || wid[nd.a] > w) return unsupported();
        val[i] = val[nd.a];  // storage is zero-extended already
        break;
      }
      case MGP_OP_SEXT: {
        if (!opnd(nd.a) || isb[nd.a] || wid[nd.a] > w) return unsupported();
        if (wid[nd.a] == w) { val[i] = val[nd.a]; break; }
        val[i] = S.add(MGP_OP_SEXT, (uint16_t)w, false, val[nd.a], Ref(), Ref(), wid[nd.a]);
        break;
      }
      case MGP_OP_ITE: {
        if (!opnd(nd.a) || !opnd(nd.b) || !opnd(nd.c) || !isb[nd.a]) return unsupported();
        if (isb[nd.b] && isb[nd.c]) {  // Bool-valued ite
          wid[i] = 1;
          isb[i] = 1;
          val[i] = S.add(MGP_OP_BITE, 1, true, val[nd.a], val[nd.b], val[nd.c]);
          break;
        }
        if (isb[nd.b] || isb[nd.c] || wid[nd.b] != w || wid[nd.c] != w) return unsupported();
        val[i] = S.add(MGP_OP_ITE, (uint16_t)w, false, val[nd.a], val[nd.b], val[nd.c]);
        break;
      }
      case MGP_OP_EQ: case MGP_OP_ULT: case MGP_OP_ULE: case MGP_OP_UGT: case MGP_OP_UGE:
      case MGP_OP_SLT: case MGP_OP_SLE: case MGP_OP_SGT: case MGP_OP_SGE:
      case MGP_OP_UADD_NOOVF: case MGP_OP_UMUL_NOOVF: case MGP_OP_USUB_NOUDF: {
        if (!opnd(nd.a) || !opnd(nd.b)) return unsupported();
        if (op == MGP_OP_EQ && isb[nd.a] && isb[nd.b]) {
          val[i] = S.add(MGP_OP_BEQ, 1, true, val[nd.a], val[nd.b]);
          break;
        }
        if (isb[nd.a] || isb[nd.b] || wid[nd.a] != wid[nd.b]) return unsupported();
        if (wid[nd.a] > MGP_MAX_WIDTH) {
          const Pieces &x = wide[nd.a], &y = wide[nd.b];
          switch (op) {
            case MGP_OP_EQ: val[i] = eq_pieces(x, y); break;
            case MGP_OP_ULT: val[i] = ult_pieces(x, y); break;
            case MGP_OP_UGT: val[i] = ult_pieces(y, x); break;
            case MGP_OP_ULE: val[i] = S.add(MGP_OP_BNOT, 1, true, ult_pieces(y, x)); break;
            case MGP_OP_UGE: val[i] = S.add(MGP_OP_BNOT, 1, true, ult_pieces(x, y)); break;
            // signed compares of zero-extended values (checked above): the unsigned ones
            case MGP_OP_SLT: val[i] = ult_pieces(x, y); break;
            case MGP_OP_SGT: val[i] = ult_pieces(y, x); break;
            case MGP_OP_SLE: val[i] = S.add(MGP_OP_BNOT, 1, true, ult_pieces(y, x)); break;
            case MGP_OP_SGE: val[i] = S.add(MGP_OP_BNOT, 1, true, ult_pieces(x, y)); break;
            default: return unsupported();
          }
          break;
        }
        val[i] = S.add(op, wid[nd.a], true, val[nd.a], val[nd.b]);
        break;
      }
      case MGP_OP_BAND: case MGP_OP_BOR: case MGP_OP_BXOR: case MGP_OP_BEQ: {
        if (!opnd(nd.a) || !opnd(nd.b) || !isb[nd.a] || !isb[nd.b]) return unsupported();
        val[i] = S.add(op, 1, true, val[nd.a], val[nd.b]);
        break;
      }
      case MGP_OP_BNOT: {
        if (!opnd(nd.a) || !isb[nd.a]) return unsupported();
        val[i] = S.add(op, 1, true, val[nd.a]);
        break;
      }
      case MGP_OP_BITE: {
        if (!opnd(nd.a) || !opnd(nd.b) || !opnd(nd.c) || !isb[nd.a] || !isb[nd.b] || !isb[nd.c])
          return unsupported();
        val[i] = S.add(op, 1, true, val[nd.a], val[nd.b], val[nd.c]);
        break;
      }
      case MGP_OP_UFAPP: {
        // f(arg): first earlier f-app with equal argument, else fresh var(s) p1..
        const uint32_t k = (w + MGP_MAX_WIDTH - 1) / MGP_MAX_WIDTH;
        if (!opnd(nd.a) || isb[nd.a] || nd.p1 + k > 0x3FFFu) return unsupported();
        // The chain selects the OLDEST earlier application with an equal argument; that
        // one has no older equal application, so its value is its own fresh variable:
        // chaining on fresh variables (free reads) instead of earlier chain results keeps
        // no earlier value live (calldata words are 32 selects of one array each).
        const Pieces arg = pieces_of(nd.a);
        std::vector<SumForm> form = forms_of(arg);
        const Pieces fresh = var_pieces(nd.p1, w);
        Pieces v = fresh;
        // a one-piece value's fresh variable read as it is: an EQSEL step masks the value it
        // selects to its width, so a narrow fresh value (a calldata byte) needs no masked
        // copy held in a slot for every later chain that selects it
        Ref raw;
        if (w <= MGP_MAX_WIDTH) {
          raw.k = R_VAR;
          raw.idx = nd.p1;
        }
        Ref vraw = raw;  // v as an unmasked variable while v is one application's fresh value
        std::vector<UFApp> &fl = fapps[nd.p0];
        for (auto it = fl.rbegin(); it != fl.rend(); ++it) {
          if (wid_of(it->arg) != wid[nd.a] || wid_of(it->val) != w) return unsupported();
          const int ke = known_eq_forms(form, it->form);
          if (ke == 0) continue;
          if (ke == -1 && arg.size() == 1 && it->arg.size() == 1 && v.size() == 1 && it->fresh.size() == 1) {
            // the one-piece case of the line below as one EQSEL step (no Bool, one
            // instruction instead of EQ + ITE)
            const Ref z = it->raw.k == R_VAR ? it->raw : it->fresh[0].r;
            const Ref d = vraw.k == R_VAR ? vraw : v[0].r;
            v[0].r = S.add(MGP_OP_EQSEL, (uint16_t)v[0].w, false, arg[0].r, it->arg[0].r, z, 0, d);
            vraw = Ref();
            continue;
          }
          if (ke == 1) {
            v = it->fresh;
            vraw = it->raw;
          } else {
            v = ite_pieces(eq_pieces(arg, it->arg), it->fresh, v);
            vraw = Ref();
          }
        }
        fl.push_back(UFApp{arg, v, fresh, std::move(form), raw});
        set_val(i, v);
        break;
      }
      case MGP_OP_UFINV: {
        // f^-1(arg): first earlier inverse app with equal argument, else the
        // argument of the first earlier f-app whose value equals arg, else p1..
        const uint32_t k = (w + MGP_MAX_WIDTH - 1) / MGP_MAX_WIDTH;
        if (!opnd(nd.a) || isb[nd.a] || nd.p1 + k > 0x3FFFu) return unsupported();
        const Pieces arg = pieces_of(nd.a);
        Pieces v = var_pieces(nd.p1, w);
        std::vector<UFApp> &fl = fapps[nd.p0];
        for (auto it = fl.rbegin(); it != fl.rend(); ++it) {
          if (wid_of(it->val) != wid[nd.a] || wid_of(it->arg) != w) return unsupported();
          const int ke = known_eq(arg, it->val);
          if (ke == 0) continue;
          v = (ke == 1) ? it->arg : ite_pieces(eq_pieces(arg, it->val), it->arg, v);
        }
        std::vector<UFApp> &il = iapps[nd.p0];
        for (auto it = il.rbegin(); it != il.rend(); ++it) {
          if (wid_of(it->arg) != wid[nd.a] || wid_of(it->val) != w) return unsupported();
          const int ke = known_eq(arg, it->arg);
          if (ke == 0) continue;
          v = (ke == 1) ? it->val : ite_pieces(eq_pieces(arg, it->arg), it->val, v);
        }
        il.push_back(UFApp{arg, v, var_pieces(nd.p1, w), {}, Ref()});
        set_val(i, v);
        break;
      }
      default:
        return unsupported();
    }
  }
  if (!isb[n_nodes - 1]) return unsupported();
  Ref root = val[n_nodes - 1];

  // ---------------------------------------------- dead-code elimination
  {
    const uint32_t n0 = (uint32_t)S.ins.size();
    std::vector<uint8_t> live(n0, 0);
    if (root.k == R_INS) live[root.idx] = 1;
    for (int64_t t = (int64_t)n0 - 1; t >= 0; --t) {
      if (!live[t]) continue;
      const VIns &I = S.ins[t];
      for (const Ref *r : {&I.a, &I.b, &I.c, &I.d})
        if (r->k == R_INS) live[r->idx] = 1;
    }
    // compacted in place (an instruction only moves down, its operands before it): a fresh
    // copy of a WalletLibrary program is ~350 KB of newly faulted pages per state
    std::vector<uint32_t> remap(n0, 0);
    uint32_t kept = 0;
    for (uint32_t t = 0; t < n0; ++t) {
      if (!live[t]) continue;
      remap[t] = kept;
      VIns I = S.ins[t];
      for (Ref *r : {&I.a, &I.b, &I.c, &I.d})
        if (r->k == R_INS) r->idx = remap[r->idx];
      S.ins[kept++] = I;
    }
    S.ins.resize(kept);
    if (root.k == R_INS) root.idx = remap[root.idx];
  }
  // pool compaction: constants only read at lowering time (uninterpreted-function
  // arguments compared here, dead code) take no pool entry in the program
  {
    std::vector<int64_t> cmap(S.pool.size(), -1);
    std::vector<ConstKey> used;
    for (VIns &I : S.ins)
      for (Ref *r : {&I.a, &I.b, &I.c, &I.d})
        if (r->k == R_CONST) {
          if (cmap[r->idx] < 0) {
            cmap[r->idx] = (int64_t)used.size();
            used.push_back(S.pool[r->idx]);
          }
          r->idx = (uint32_t)cmap[r->idx];
        }
    S.pool.swap(used);
    S.pool_map.clear();
  }

  // ---------------------------------------------- schedules
  // The prepared state (expansion, DCE, pool) is shared by every schedule tried; a
  // schedule only counts if the gfx950 interpreter can run it (uop translation).
  // Fewer slots wins (occupancy); between spilling programs, fewer instructions (a
  // spill is a memory access either way, an instruction is issue time).
  // very long programs (WalletLibrary's 8-30 k instructions) keep input order alone: the
  // greedy scheduler is quadratic there, and Sethi-Ullman DFS fails on a third of them (Bool
  // budget) and saves < 0.2 % of the instructions on the rest, for twice the lowering time
  static const int kInputOrder[1] = {0};
  if (n_scheds > 1 && S.ins.size() > 1536) {
    bool has0 = false;
    for (int k = 0; k < n_scheds; ++k) has0 |= scheds[k] == 0;
    if (has0) {
      scheds = kInputOrder;
      n_scheds = 1;
    }
  }
  // the schedules are independent: in parallel when the caller runs few states
  std::vector<Lowered> tried(n_scheds);
  if (n_scheds == 1) {
    tried[0] = finish_one(std::move(S), root, max_slots, scheds[0]);  // S is not read again
  } else {
#pragma omp parallel for schedule(dynamic, 1) if (par_scheds)
    for (int k = 0; k < n_scheds; ++k) tried[k] = finish_one(S, root, max_slots, scheds[k]);
  }
  Lowered best;
  bool have = false;
  for (int k = 0; k < n_scheds; ++k) {
    Lowered &b = tried[k];
    if (b.status != MGP_ST_OK) continue;
    if (have) {
      const bool spill = best.words[2] > MGP_LDS_SLOTS || b.words[2] > MGP_LDS_SLOTS;
      if (spill ? b.words[0] >= best.words[0] : b.words[2] >= best.words[2]) continue;
    }
    std::vector<uint32_t> bu;
    bu.swap(g_uops_pool);
    bu.clear();
    if (mgp_uop_translate(b.words.data(), bu) != 0) {
      recycle(bu, g_uops_pool);
      continue;
    }
    best = std::move(b);
    uops->swap(bu);
    have = true;
  }
  if (!have) uops->clear();
  return have ? best : unsupported();
}

}  // namespace

// Lower every state into res[s] (OpenMP over states); MGP_OK or MGP_E_ARG.
static int lower_all(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                     const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_slots,
                     std::vector<Lowered> &res) {
  res.assign(n_states, Lowered());
  int bad = 0;
  // MGP_LOWER_SCHED (A/B studies): 0 input order, 2 DFS only, 3 greedy only;
  // default 1 = the fewest-slot schedule of the three
  static const int sched_mode = [] {
    const char *e = getenv("MGP_LOWER_SCHED");
    return (e && e[0] >= '0' && e[0] <= '3' && e[1] == 0) ? e[0] - '0' : 1;
  }();
  // few states (LASER's JUMPI forks): states in turn, each state's schedules in parallel --
  // unless every state is large (WalletLibrary's: more than kBigNodes nodes), whose programs
  // keep input order alone (lower_one), so the states themselves run in parallel
  const bool few = (int64_t)n_states * 2 < (int64_t)omp_get_max_threads();
  constexpr uint64_t kBigNodes = 600;
  bool all_big = n_states > 1;
  for (uint32_t s = 0; s < n_states && all_big; ++s) all_big = node_offsets[s + 1] - node_offsets[s] > kBigNodes;
#pragma omp parallel for schedule(dynamic, 1) if (!few || all_big)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const uint64_t n0 = node_offsets[s], n1 = node_offsets[s + 1];
    const uint64_t c0 = const_offsets[s], c1 = const_offsets[s + 1];
    if (n1 < n0 || c1 < c0) {
#pragma omp atomic write
      bad = 1;
      continue;
    }
    // Three schedules (input order, Sethi-Ullman DFS, greedy list) over one prepared
    // state; lower_one keeps the best one the gfx950 interpreter can run.
    const uint32_t *cp = consts ? consts + c0 * 8u : nullptr;
    static const int all3[3] = {0, 1, 2};
    const int one = sched_mode == 0 ? 0 : sched_mode - 1;
    std::vector<uint32_t> uops;
    Lowered a = sched_mode == 1 ? lower_one(nodes + n0, n1 - n0, cp, c1 - c0, max_slots, all3, 3, &uops, few)
                                : lower_one(nodes + n0, n1 - n0, cp, c1 - c0, max_slots, &one, 1, &uops, few);
    // append the uop program of the gfx950 interpreter; a state it cannot run
    // is made unsupported in both encodings so that both engines agree
    if (a.status != MGP_ST_OK) {
      a = unsupported();
      uops.clear();
      mgp_uop_translate(a.words.data(), uops);
    }
    a.uops.swap(uops);
    res[s] = std::move(a);
  }
  return bad ? MGP_E_ARG : MGP_OK;
}

// In-library entry point (mgp_pipeline.cpp): the lowered programs as one vector.
int mgp_lower_vec(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states, const uint32_t *consts,
                  const uint64_t *const_offsets, uint32_t max_slots, U32Buf &words,
                  std::vector<uint64_t> &offs, std::vector<uint8_t> &status) {
  std::vector<Lowered> res;
  const int rc = lower_all(nodes, node_offsets, n_states, consts, const_offsets, max_slots, res);
  if (rc != MGP_OK) return rc;
  offs.assign((size_t)n_states + 1, 0);
  for (uint32_t s = 0; s < n_states; ++s) offs[s + 1] = offs[s] + res[s].words.size() + res[s].uops.size();
  words.resize(offs[n_states]);
  status.resize(n_states);
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    memcpy(words.data() + offs[s], res[s].words.data(), res[s].words.size() * 4u);
    memcpy(words.data() + offs[s] + res[s].words.size(), res[s].uops.data(), res[s].uops.size() * 4u);
    status[s] = res[s].status;
    recycle(res[s].words, g_words_pool);
    recycle(res[s].uops, g_uops_pool);
  }
  return MGP_OK;
}

extern "C" int mgp_lower(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                         const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_slots,
                         uint32_t *out_words, uint64_t out_cap, uint64_t *out_prog_offsets,
                         uint8_t *out_status, uint64_t *out_words_used) {
  if (!node_offsets || !out_prog_offsets || (n_states && (!nodes || !const_offsets))) return MGP_E_ARG;
  std::vector<Lowered> res;
  if (lower_all(nodes, node_offsets, n_states, consts, const_offsets, max_slots, res) != MGP_OK) return MGP_E_ARG;
  uint64_t total = 0;
  for (uint32_t s = 0; s < n_states; ++s) {
    out_prog_offsets[s] = total;
    total += res[s].words.size() + res[s].uops.size();
  }
  out_prog_offsets[n_states] = total;
  if (out_words_used) *out_words_used = total;
  if (!out_words || total > out_cap) return MGP_E_CAPACITY;
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    memcpy(out_words + out_prog_offsets[s], res[s].words.data(), res[s].words.size() * 4u);
    memcpy(out_words + out_prog_offsets[s] + res[s].words.size(), res[s].uops.data(), res[s].uops.size() * 4u);
    if (out_status) out_status[s] = res[s].status;
    recycle(res[s].words, g_words_pool);
    recycle(res[s].uops, g_uops_pool);
  }
  return MGP_OK;
}

extern "C" int mgp_plan_buckets(const uint32_t *prog_words, const uint64_t *prog_offsets, uint32_t n_states,
                                uint32_t *order_out, uint32_t *bounds_out, uint32_t *slots_out,
                                uint32_t max_buckets) {
  // counting sort of the states by BV-slot count (header word 2); one bucket
  // per distinct count, merged upward when there are more than max_buckets
  if (!prog_words || !prog_offsets || !order_out || !bounds_out || !slots_out || max_buckets == 0) return MGP_E_ARG;
  std::vector<uint32_t> cnt(257, 0);
  std::vector<uint16_t> sl(n_states);
  // the gfx950 interpreter keeps some BV slots in registers: it allocates the LDS slot
  // count of the uop header (word 3 bits 16..23) instead of the v1 count
  const bool asm_engine = mgp_set_eval_engine(0) == MGP_ENGINE_ASM;
  for (uint32_t s = 0; s < n_states; ++s) {
    const uint32_t *w = prog_words + prog_offsets[s];
    uint32_t v = std::min<uint32_t>(w[2], MGP_LDS_SLOTS);  // spill slots take no LDS
    if (asm_engine && (w[3] & 0xFFu) == MGP_ST_OK) {
      const uint32_t v1 = 4u + 4u * w[0] + 8u * w[1];
      const uint32_t *u = w + ((v1 + 3u) & ~3u) + 4u;
      if (u[1] == 0u) v = (u[3] >> 16) & 0xFFu;
    }
    v = std::min<uint32_t>(v, 256u);
    sl[s] = (uint16_t)v;
    cnt[v]++;
  }
  std::vector<uint32_t> distinct;
  // a class with few states costs a whole launch (≈ one wave lifetime of ramp-down) for
  // little work: it joins the next larger slot count (its states then run with more LDS
  // than they need, which is harmless), scanning upward so a run of small top classes
  // ends in one launch
  const uint32_t min_states = std::max<uint32_t>(256u, n_states / 128u);
  uint32_t carried = 0;
  for (uint32_t v = 0; v <= 256; ++v) {
    if (!cnt[v]) continue;
    carried += cnt[v];
    bool last = true;
    for (uint32_t w = v + 1; w <= 256; ++w)
      if (cnt[w]) { last = false; break; }
    if (carried >= min_states || last) {
      distinct.push_back(v);
      carried = 0;
    }
  }
  // merge the smallest classes into their upper neighbour until the plan fits
  while (distinct.size() > max_buckets) distinct.erase(distinct.begin());
  std::vector<uint32_t> bucket_of(257, 0);
  uint32_t b = 0;
  for (uint32_t v = 0; v <= 256; ++v) {
    while (b < distinct.size() && distinct[b] < v) ++b;
    bucket_of[v] = std::min<uint32_t>(b, (uint32_t)distinct.size() - 1);
  }
  const uint32_t nb = (uint32_t)distinct.size();
  std::vector<uint32_t> fill(nb + 1, 0);
  for (uint32_t s = 0; s < n_states; ++s) fill[bucket_of[sl[s]] + 1]++;
  for (uint32_t k = 0; k < nb; ++k) fill[k + 1] += fill[k];
  for (uint32_t k = 0; k <= nb; ++k) bounds_out[k] = fill[k];
  for (uint32_t k = 0; k < nb; ++k) slots_out[k] = distinct[k];
  for (uint32_t s = 0; s < n_states; ++s) order_out[fill[bucket_of[sl[s]]]++] = s;
  return (int)nb;
}
