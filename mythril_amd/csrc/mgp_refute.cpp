// mgp_refute.cpp — sound UNSAT pre-check of constraint DAGs (host side, OpenMP).
//
// The GPU evaluator proves SAT (a witness); every state it cannot prove goes
// to z3 in the reference (Constraints.is_possible, constraints.py:34-51;
// get_model, analysis/solver.py:27-61).  Many of those are infeasible for a
// shallow reason: a jump condition contradicting an earlier one
// (instructions.py:1556-1562 adds `cond` to one successor and `Not(cond)` to
// the other, so a later branch on a related value is often decided by ranges
// and bits), a calldata size bound against a byte index
// (calldata.py:219-232), an overflow predicate whose operands are pinned
// (integer.py:141-160).  This pass proves those UNSAT without a solver call.
//
// Abstract domain per BV node of width w <= 256: known bits (z = known-zero
// mask, o = known-one mask) x unsigned interval [lo, hi]; per Bool node the set
// of possible truth values.  Each pass runs forward transfer functions over the
// topological node list, then backward narrowing from "root = true" (a
// conjunct that must hold narrows its operands: x <u c bounds x, x == c pins
// its bits, ...), until nothing changes or the pass limit is hit.  An empty
// abstract value proves that no assignment of the free variables satisfies the
// root: the state is UNSAT.  Every transfer function over-approximates its
// operator under the z3 / SMT-LIB semantics of include/mgp_ir.h, so the claim
// is sound; uninterpreted-function applications are left unconstrained (a
// relaxation of the UF formula, still sound for UNSAT).  tests/test_refute.py
// checks soundness against the oracle: node by node (every concrete evaluation
// lies inside its node's abstract value) and state by state (no refuted state
// has a model, exhaustively at small widths).
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <iterator>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/mgp.h"
#include "mgp_bv.h"
#include "mgp_domain.h"
#include "mgp_fe_sample.h"


namespace {

using namespace mgpd;

// A state's DAG with std::vector storage: validated and set up here (host only), then
// analysed through a view (mgpd::Dom) whose mutable arrays are this state's own.
struct State {
  const mgp_node *nd;
  std::vector<mgp_node> relaxed;  // nd when the DAG holds wide values (relax_wide)
  const mgp_node *orig = nullptr;  // the DAG before relax_wide (UF arguments, congruence)
  std::vector<mgp_node> origx;     // orig + the piece-expansion nodes relax_wide appended
  std::vector<uint32_t> xconsts;   // the constant pool + the pieces' zero (when one is needed)
  std::vector<int32_t> ties;       // the piece-expansion ties (required with the root)
  uint32_t n;
  const uint32_t *consts;
  uint64_t n_consts;
  std::vector<AV> av;
  std::vector<uint8_t> bs;     // truth set of Bool nodes
  std::vector<uint8_t> isb;    // node is Bool-typed
  std::vector<int32_t> vtie;   // VAR node -> var table entry
  std::vector<AV> vars;
  std::vector<uint32_t> vkey;  // (index << 9) | width
  std::vector<Pair> pairs;
  std::vector<int32_t> cmp_pair;  // compare node -> pair index, -1 = none
  std::vector<uint8_t> cmp_dom;   // 0 unsigned, 1 signed, 2 both (EQ)
  std::vector<uint8_t> cmp_t;     // orderings (x vs y) under which the node is true
  std::vector<UfApp> ufs;
  std::vector<int32_t> tien;  // compare nodes with a pair, then BORs of one pair (Dom::tien)
  uint32_t n_cmpn = 0, n_borp = 0;
  std::vector<uint32_t> ufp;  // ufs index pairs whose arguments can be equal (Dom::ufp)
  std::vector<int32_t> cong;  // pairs of structurally matching operand nodes (Dom::cong)
  std::vector<ArithRel> arel;  // ADD / SUB nodes whose wrap status orders a compare pair (Dom::arel)
  std::vector<InjApp> inj;     // applications with an asserted inverse (Dom::injective)
  std::vector<OrGroup> og;     // disjunctive hulls (Dom::or_hull)
  std::vector<OrDis> odis;
  std::vector<int32_t> oatom, otgt;
  std::unordered_map<uint64_t, int32_t> pair_of;  // (x << 32 | y), x < y -> pairs index
  std::vector<uint64_t> pair_keys;                // the same map, sorted (Dom::pair_find)
  std::vector<int32_t> pair_idx;
  std::vector<uint32_t> uoff, ulist, voff, vlist;  // users of each node; VAR nodes of each entry
  std::vector<uint8_t> tie_rel;  // nodes tie() reads: compares with a pair, BOR, pair operands
  std::vector<uint32_t> pinc_off, pinc;  // pairs incident to each node (Dom::substitute)

  uint32_t W(int32_t i) const { return nd[i].width; }

  Dom view() {
    Dom d;
    d.nd = nd;
    d.orig = orig;
    d.n = n;
    d.consts = consts;
    d.n_consts = n_consts;
    d.av = av.data();
    d.bs = bs.data();
    d.isb = isb.data();
    d.vtie = vtie.data();
    d.vars = vars.data();
    d.pairs = pairs.data();
    d.n_pairs = (uint32_t)pairs.size();
    d.cmp_pair = cmp_pair.data();
    d.cmp_dom = cmp_dom.data();
    d.cmp_t = cmp_t.data();
    d.pair_keys = pair_keys.data();
    d.pair_idx = pair_idx.data();
    d.ufs = ufs.data();
    d.n_ufs = (uint32_t)ufs.size();
    d.tien = tien.data();
    d.n_cmpn = n_cmpn;
    d.n_borp = n_borp;
    d.ufp = ufp.data();
    d.n_ufp = (uint32_t)(ufp.size() / 2);
    d.cong = cong.data();
    d.n_cong = (uint32_t)cong.size();
    d.arel = arel.data();
    d.n_arel = (uint32_t)arel.size();
    d.inj = inj.data();
    d.n_inj = (uint32_t)inj.size();
    d.og = og.data();
    d.n_og = (uint32_t)og.size();
    d.odis = odis.data();
    d.oatom = oatom.data();
    d.otgt = otgt.data();
    d.uoff = uoff.data();
    d.ulist = ulist.data();
    d.voff = voff.data();
    d.vlist = vlist.data();
    d.tie_rel = tie_rel.data();
    d.pinc_off = pinc_off.data();
    d.pinc = pinc.data();
    return d;
  }

  // ------------------------------------------------------------ validate
  bool setup() {
    av.assign(n, AV());
    bs.assign(n, BB);
    isb.assign(n, 0);
    vtie.assign(n, -1);
    for (uint32_t i = 0; i < n; ++i) {
      const mgp_node &x = nd[i];
      const uint8_t op = x.op;
      auto opnd = [&](int32_t k) { return k >= 0 && (uint32_t)k < i; };
      const bool boolres = (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) ||
                           (op >= MGP_OP_BAND && op <= MGP_OP_BEQ) || op == MGP_OP_TRUE || op == MGP_OP_FALSE;
      uint32_t nop = 0;
      switch (op) {
        case MGP_OP_VAR: case MGP_OP_CONST: case MGP_OP_TRUE: case MGP_OP_FALSE: nop = 0; break;
        case MGP_OP_NOT: case MGP_OP_NEG: case MGP_OP_EXTRACT: case MGP_OP_ZEXT: case MGP_OP_SEXT:
        case MGP_OP_BNOT: case MGP_OP_UFAPP: case MGP_OP_UFINV: nop = 1; break;
        case MGP_OP_ITE: case MGP_OP_BITE: nop = 3; break;
        default:
          if ((op >= MGP_OP_ADD && op <= MGP_OP_ASHR) || op == MGP_OP_CONCAT || boolres) nop = 2;
          else return false;  // unknown op
      }
      if (nop >= 1 && !opnd(x.a)) return false;
      if (nop >= 2 && !opnd(x.b)) return false;
      if (nop >= 3 && !opnd(x.c)) return false;
      if (op == MGP_OP_ITE) {
        isb[i] = isb[x.b];
        if (isb[x.b] != isb[x.c] || !isb[x.a]) return false;
      } else {
        isb[i] = boolres;
      }
      if (!isb[i]) {
        const uint32_t w = x.width;
        if (w == 0u || w > MGP_MAX_WIDTH) return false;
        av[i] = top(w);
        if (op == MGP_OP_EXTRACT && (x.p0 < x.p1 || x.p0 - x.p1 + 1u != w || x.p0 >= W(x.a))) return false;
        if (op == MGP_OP_CONCAT && W(x.a) + W(x.b) != w) return false;
        if ((op == MGP_OP_ZEXT || op == MGP_OP_SEXT) && W(x.a) > w) return false;
        if (op == MGP_OP_CONST && x.p0 >= n_consts) return false;
        if (((op >= MGP_OP_ADD && op <= MGP_OP_ASHR) && op != MGP_OP_NOT && op != MGP_OP_NEG) &&
            (W(x.a) != w || W(x.b) != w || isb[x.a] || isb[x.b]))
          return false;
        if ((op == MGP_OP_NOT || op == MGP_OP_NEG) && (W(x.a) != w || isb[x.a])) return false;
        if (op == MGP_OP_ITE && (W(x.b) != w || W(x.c) != w)) return false;
        if (op == MGP_OP_VAR) {
          const uint32_t key = (x.p0 << 9) | w;
          int32_t t = -1;
          for (size_t k = 0; k < vkey.size(); ++k)
            if (vkey[k] == key) t = (int32_t)k;
          if (t < 0) {
            t = (int32_t)vkey.size();
            vkey.push_back(key);
            vars.push_back(top(w));
          }
          vtie[i] = t;
        }
      } else if (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) {
        if (isb[x.a] != isb[x.b]) return false;
        if (isb[x.a] && op != MGP_OP_EQ) return false;
        if (!isb[x.a] && W(x.a) != W(x.b)) return false;
      } else if (op >= MGP_OP_BAND && op <= MGP_OP_BEQ) {
        if (!isb[x.a] || (nop >= 2 && !isb[x.b]) || (nop >= 3 && !isb[x.c])) return false;
      }
    }
    if (n == 0 || !isb[n - 1]) return false;
    build_atoms();
    return true;
  }

  void build_atoms() {
    cmp_pair.assign(n, -1);
    cmp_dom.assign(n, 0);
    cmp_t.assign(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
      const mgp_node &x = nd[i];
      if (!(x.op >= MGP_OP_EQ && x.op <= MGP_OP_USUB_NOUDF) || isb[x.a] || x.a == x.b) continue;
      uint8_t t, dom = 0;  // truth set for "a op b"
      switch (x.op) {
        case MGP_OP_EQ: t = OEQ; dom = 2; break;
        case MGP_OP_ULT: t = OLT; break;
        case MGP_OP_ULE: t = OLT | OEQ; break;
        case MGP_OP_UGT: t = OGT; break;
        case MGP_OP_UGE: case MGP_OP_USUB_NOUDF: t = OGT | OEQ; break;  // b <= a
        case MGP_OP_SLT: t = OLT; dom = 1; break;
        case MGP_OP_SLE: t = OLT | OEQ; dom = 1; break;
        case MGP_OP_SGT: t = OGT; dom = 1; break;
        case MGP_OP_SGE: t = OGT | OEQ; dom = 1; break;
        default: continue;  // overflow predicates: not an ordering
      }
      int32_t px = x.a, py = x.b;
      if (px > py) {  // orient as (smaller node id, larger): mirror < and >
        px = x.b;
        py = x.a;
        t = (uint8_t)((t & OEQ) | ((t & OLT) ? OGT : 0) | ((t & OGT) ? OLT : 0));
      }
      const uint64_t pk = ((uint64_t)(uint32_t)px << 32) | (uint32_t)py;
      auto pit = pair_of.find(pk);
      int32_t pi = pit == pair_of.end() ? -1 : pit->second;
      if (pi < 0) {
        pi = (int32_t)pairs.size();
        pairs.push_back({px, py, OALL, OALL});
        pair_of.emplace(pk, pi);
      }
      cmp_pair[i] = pi;
      cmp_dom[i] = dom;
      cmp_t[i] = t;
    }
    ufs.clear();
    const mgp_node *o = orig ? orig : nd;
    for (uint32_t i = 0; i < n; ++i)
      if ((o[i].op == MGP_OP_UFAPP || o[i].op == MGP_OP_UFINV) && !isb[i] && o[i].width == nd[i].width)
        ufs.push_back({(int32_t)i, o[i].a, o[i].p0, o[i].op});
    std::stable_sort(ufs.begin(), ufs.end(), [](const UfApp &x, const UfApp &y) {
      return x.op != y.op ? x.op < y.op : x.fn < y.fn;
    });
    std::vector<UfApp> keep;
    for (size_t i = 0; i < ufs.size();) {
      size_t j = i;
      while (j < ufs.size() && ufs[j].op == ufs[i].op && ufs[j].fn == ufs[i].fn) ++j;
      if (j - i >= 2 && j - i <= kUfGroup) keep.insert(keep.end(), ufs.begin() + i, ufs.begin() + j);
      i = j;
    }
    ufs.swap(keep);
    tien.clear();
    for (uint32_t i = 0; i < n; ++i)
      if (cmp_pair[i] >= 0) tien.push_back((int32_t)i);
    n_cmpn = (uint32_t)tien.size();
    for (uint32_t i = 0; i < n; ++i) {
      if (nd[i].op != MGP_OP_BOR || nd[i].a < 0 || nd[i].b < 0) continue;
      const int32_t pa = cmp_pair[nd[i].a];
      if (pa >= 0 && pa == cmp_pair[nd[i].b]) tien.push_back((int32_t)i);
    }
    n_borp = (uint32_t)tien.size() - n_cmpn;
    // UF application pairs tie() compares: one function and operator; arguments that are
    // two different constants never become equal (calldata bytes at fixed offsets)
    ufp.clear();
    auto const_arg = [&](int32_t a, const uint32_t *&c) {
      if (a < 0 || o[a].op != MGP_OP_CONST || o[a].width > MGP_MAX_WIDTH) return false;
      c = consts + 8u * (size_t)o[a].p0;
      return true;
    };
    for (uint32_t i = 0; i < ufs.size(); ++i)
      for (uint32_t j = i + 1; j < ufs.size() && ufs[j].fn == ufs[i].fn && ufs[j].op == ufs[i].op; ++j) {
        const uint32_t *ci, *cj;
        if (const_arg(ufs[i].arg, ci) && const_arg(ufs[j].arg, cj) && o[ufs[i].arg].width == o[ufs[j].arg].width &&
            memcmp(ci, cj, 32) != 0)
          continue;
        ufp.push_back(i);
        ufp.push_back(j);
      }
    // structural congruence candidates: both operands of the pair apply one operator with
    // the same parameters and width (leaves excluded: one variable is one node's value
    // already, two constants are compared exactly)
    cong.clear();
    for (size_t k = 0; k < pairs.size(); ++k) {
      const mgp_node &a = o[pairs[k].x], &b = o[pairs[k].y];
      const bool uf = a.op == MGP_OP_UFAPP || a.op == MGP_OP_UFINV;  // p1: the application's own slot
      if (a.op != b.op || a.p0 != b.p0 || (a.p1 != b.p1 && !uf) || a.width != b.width) continue;
      if (a.op == MGP_OP_VAR || a.op == MGP_OP_CONST || a.op == MGP_OP_TRUE || a.op == MGP_OP_FALSE) continue;
      cong.push_back((int32_t)k);
    }
    // wrap orderings: ADD / SUB nodes on narrow values where a compare reads (r, a), (r, b)
    // or (a, b), or a BVAddNoOverflow node reads the same operands
    arel.clear();
    {
      std::unordered_map<uint64_t, int32_t> noovf;  // operand pair -> BVAddNoOverflow node
      auto okey = [](int32_t x, int32_t y) {
        return x < y ? ((uint64_t)(uint32_t)x << 32) | (uint32_t)y : ((uint64_t)(uint32_t)y << 32) | (uint32_t)x;
      };
      for (uint32_t i = 0; i < n; ++i)
        if (nd[i].op == MGP_OP_UADD_NOOVF && !isb[nd[i].a]) noovf.emplace(okey(nd[i].a, nd[i].b), (int32_t)i);
      auto has_pair = [&](int32_t x, int32_t y) { return x != y && pair_of.count(okey(x, y)) != 0; };
      for (uint32_t i = 0; i < n; ++i) {
        const mgp_node &x = nd[i];
        if ((x.op != MGP_OP_ADD && x.op != MGP_OP_SUB) || isb[i] || x.width == 0u || x.width > MGP_MAX_WIDTH) continue;
        int32_t flag = -1;
        if (x.op == MGP_OP_ADD) {
          auto it = noovf.find(okey(x.a, x.b));
          if (it != noovf.end()) flag = it->second;
        }
        const int32_t r = (int32_t)i;
        if (flag < 0 && !has_pair(r, x.a) && !(x.op == MGP_OP_ADD && has_pair(r, x.b)) &&
            !(x.op == MGP_OP_SUB && has_pair(x.a, x.b)))
          continue;
        arel.push_back(ArithRel{r, x.a, x.b, flag, x.op});
      }
    }
    build_or_groups();
    // injectivity: EQ(UFINV(u), arg) with u = UFAPP(arg), on the original DAG
    inj.clear();
    for (uint32_t e = 0; e < n; ++e) {
      if (o[e].op != MGP_OP_EQ) continue;
      for (int side = 0; side < 2; ++side) {
        const int32_t iv = side ? o[e].b : o[e].a, other = side ? o[e].a : o[e].b;
        if (iv < 0 || o[iv].op != MGP_OP_UFINV) continue;
        const int32_t u = o[iv].a;
        if (u < 0 || o[u].op != MGP_OP_UFAPP || o[u].a != other || o[u].p0 != o[iv].p0) continue;
        if (o[u].width > MGP_MAX_WIDTH || nd[u].width != o[u].width) continue;
        inj.push_back(InjApp{u, other, (int32_t)e, o[u].p0});
        break;
      }
    }
    std::stable_sort(inj.begin(), inj.end(), [](const InjApp &x, const InjApp &y) { return x.fn < y.fn; });
    if (inj.size() > 4u * kUfGroup) inj.resize(4u * kUfGroup);
    // the pair lookup as a sorted array (the view's binary search, host and device)
    pair_keys.clear();
    pair_idx.clear();
    std::vector<std::pair<uint64_t, int32_t>> kv(pair_of.begin(), pair_of.end());
    std::sort(kv.begin(), kv.end());
    for (const auto &e : kv) {
      pair_keys.push_back(e.first);
      pair_idx.push_back(e.second);
    }
    // pairs incident to each node, for equality substitution
    pinc_off.assign(n + 1, 0u);
    for (const Pair &p : pairs) {
      pinc_off[p.x + 1]++;
      pinc_off[p.y + 1]++;
    }
    for (uint32_t i = 0; i < n; ++i) pinc_off[i + 1] += pinc_off[i];
    pinc.assign(pinc_off[n], 0u);
    {
      std::vector<uint32_t> at(pinc_off.begin(), pinc_off.end() - 1);
      for (uint32_t k = 0; k < pairs.size(); ++k) {
        pinc[at[pairs[k].x]++] = k;
        pinc[at[pairs[k].y]++] = k;
      }
    }
  }

  // The BOR trees for Dom::or_hull: maximal BOR trees (a BOR that is no operand of another
  // BOR), at most kMaxDis disjuncts of at most kMaxAtoms conjuncts each; a conjunct is a
  // compare of a node with a constant, or a BOR of two of those on one node.
  void build_or_groups() {
    constexpr size_t kMaxDis = 16, kMaxAtoms = 24;
    og.clear();
    odis.clear();
    oatom.clear();
    otgt.clear();
    std::vector<uint8_t> under_or(n, 0);
    for (uint32_t i = 0; i < n; ++i)
      if (nd[i].op == MGP_OP_BOR) under_or[nd[i].a] = under_or[nd[i].b] = 1;
    auto cmp_const = [&](int32_t k, int32_t *target) {
      const mgp_node &x = nd[k];
      if (!(x.op == MGP_OP_EQ || (x.op >= MGP_OP_ULT && x.op <= MGP_OP_UGE)) || isb[x.a]) return false;
      const bool ca = nd[x.a].op == MGP_OP_CONST, cb = nd[x.b].op == MGP_OP_CONST;
      if (ca == cb) return false;
      *target = ca ? x.b : x.a;
      return true;
    };
    std::vector<int32_t> st, dis, conj;
    for (uint32_t r = 0; r < n; ++r) {
      if (nd[r].op != MGP_OP_BOR || under_or[r]) continue;
      dis.clear();
      st.assign(1, (int32_t)r);
      while (!st.empty() && dis.size() <= kMaxDis) {
        const int32_t k = st.back();
        st.pop_back();
        if (nd[k].op == MGP_OP_BOR) { st.push_back(nd[k].b); st.push_back(nd[k].a); }
        else dis.push_back(k);
      }
      if (dis.size() < 2 || dis.size() > kMaxDis || !st.empty()) continue;
      const uint32_t d0 = (uint32_t)odis.size();
      std::vector<std::vector<int32_t>> tg;  // per disjunct: nodes it bounds
      bool good = true;
      for (int32_t d : dis) {
        const uint32_t a0 = (uint32_t)oatom.size();
        std::vector<int32_t> bound;
        conj.clear();
        st.assign(1, d);
        while (!st.empty() && conj.size() <= kMaxAtoms) {
          const int32_t k = st.back();
          st.pop_back();
          if (nd[k].op == MGP_OP_BAND) { st.push_back(nd[k].b); st.push_back(nd[k].a); }
          else conj.push_back(k);
        }
        if (!st.empty()) { good = false; break; }
        for (int32_t k : conj) {
          int32_t t = -1, t2 = -1;
          if (cmp_const(k, &t)) {
            oatom.push_back(k);
            bound.push_back(t);
          } else if (nd[k].op == MGP_OP_BOR && cmp_const(nd[k].a, &t) && cmp_const(nd[k].b, &t2) && t == t2) {
            oatom.push_back(k);
            bound.push_back(t);
          } else if (nd[k].op == MGP_OP_FALSE) {
            oatom.push_back(k);  // never bounds anything; the disjunct is false anyway (forward)
          }
        }
        odis.push_back(OrDis{d, a0, (uint32_t)oatom.size()});
        std::sort(bound.begin(), bound.end());
        bound.erase(std::unique(bound.begin(), bound.end()), bound.end());
        tg.push_back(bound);
      }
      if (!good) {
        odis.resize(d0);
        continue;
      }
      // targets: bounded in every disjunct
      std::vector<int32_t> common = tg[0];
      for (size_t j = 1; j < tg.size(); ++j) {
        std::vector<int32_t> keep;
        std::set_intersection(common.begin(), common.end(), tg[j].begin(), tg[j].end(), std::back_inserter(keep));
        common.swap(keep);
      }
      if (common.empty()) {
        odis.resize(d0);
        continue;
      }
      const uint32_t t0 = (uint32_t)otgt.size();
      otgt.insert(otgt.end(), common.begin(), common.end());
      og.push_back(OrGroup{(int32_t)r, d0, (uint32_t)odis.size(), t0, (uint32_t)otgt.size()});
    }
    if (og.empty()) {
      odis.clear();
      oatom.clear();
    }
  }

  // ---------------------------------------------------- decision support
  void build_graph() {
    uoff.assign(n + 1, 0u);
    for (uint32_t i = 0; i < n; ++i)
      for (int32_t o : {nd[i].a, nd[i].b, nd[i].c})
        if (o >= 0 && (uint32_t)o < i) uoff[o + 1]++;
    for (uint32_t i = 0; i < n; ++i) uoff[i + 1] += uoff[i];
    ulist.assign(uoff[n], 0u);
    std::vector<uint32_t> pos(uoff.begin(), uoff.end() - 1);
    for (uint32_t i = 0; i < n; ++i)
      for (int32_t o : {nd[i].a, nd[i].b, nd[i].c})
        if (o >= 0 && (uint32_t)o < i) ulist[pos[o]++] = i;
    voff.assign(vars.size() + 1, 0u);
    for (uint32_t i = 0; i < n; ++i)
      if (nd[i].op == MGP_OP_VAR && vtie[i] >= 0) voff[vtie[i] + 1]++;
    for (size_t j = 0; j < vars.size(); ++j) voff[j + 1] += voff[j];
    vlist.assign(voff[vars.size()], 0u);
    std::vector<uint32_t> vp(voff.begin(), voff.end() - 1);
    for (uint32_t i = 0; i < n; ++i)
      if (nd[i].op == MGP_OP_VAR && vtie[i] >= 0) vlist[vp[vtie[i]]++] = i;
    tie_rel.assign(n, 0);
    for (uint32_t i = 0; i < n; ++i)
      if (cmp_pair[i] >= 0 || nd[i].op == MGP_OP_BOR) tie_rel[i] = 1;
    for (const Pair &p : pairs) tie_rel[p.x] = tie_rel[p.y] = 1;
    for (const UfApp &u : ufs) tie_rel[u.node] = 1;
    for (const ArithRel &e : arel) {
      tie_rel[e.r] = tie_rel[e.a] = tie_rel[e.b] = 1;
      if (e.flag >= 0) tie_rel[e.flag] = 1;
    }
    for (const InjApp &a : inj) tie_rel[a.u] = tie_rel[a.eq] = 1;
    for (const OrGroup &g : og) {
      tie_rel[g.root] = 1;
      for (uint32_t k = g.d0; k < g.d1; ++k) tie_rel[odis[k].node] = 1;
      for (uint32_t k = g.t0; k < g.t1; ++k) tie_rel[otgt[k]] = 1;
    }
  }
};

// Values wider than 256 bits (mgp_ir.h "wide values": 512-bit mapping preimages and
// keccak inverses) are outside the abstract domain.  They are relaxed: every node that
// produces or reads a wide value becomes a fresh unconstrained variable of its own width
// (a Bool reader: EQ of two fresh 8-bit variables).  Replacing subterms by fresh
// variables only enlarges the solution set, so a refutation of the relaxed DAG refutes
// the original; the narrow constraints around the mapping stay exact.
inline bool op_bool_result(uint8_t op) {
  return (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) || (op >= MGP_OP_BAND && op <= MGP_OP_BEQ) ||
         op == MGP_OP_TRUE || op == MGP_OP_FALSE;
}

// Piece expansion (round 5).  The relaxation above loses every constraint that passes
// through a wide value -- in particular the keccak manager's `key == func_input` between a
// mapping access's 512-bit Concat(key, slot) and a concrete key (keccak_function_manager.py:
// 146), so neither the refuter nor the decision rows could use a mapping key's equality
// with a known key.  A wide value built from narrow parts (CONCAT, EXTRACT, ZEXT, ITE, a
// wide constant's pool entries, a wide variable's or UF value's consecutive slots) is a
// list of narrow pieces, low bits first; nodes appended after the original ones hold them:
//   * a wide EQ e becomes BEQ(e, AND of the piece EQs), cut at the union of both sides'
//     piece boundaries (EXTRACTs where a piece is split);
//   * a narrow node that reads a wide value (an EXTRACT out of a Concat) becomes
//     EQ(node, its value rebuilt from pieces);
// and the root becomes the conjunction of the old root with these ties.  Each tie states
// the node's exact meaning in the original DAG, so the expanded DAG is still a relaxation
// of the original formula (UF values stay free): refutations stay sound.  The original
// node indices are unchanged (the decision slots, the UF and injectivity tables and the
// refuter's domain export read them); `orig` is extended by the appended nodes.
namespace {
struct Piece {
  int32_t node;   // a narrow node (original or appended)
  uint16_t lo, w; // bits [lo, lo + w) of that node
};

struct Expander {
  const mgp_node *nd;
  uint64_t n;
  std::vector<mgp_node> &out;
  std::vector<uint32_t> &xc;      // extended constant pool (limbs); empty = the original pool
  const uint32_t *consts;
  uint64_t n_consts;
  std::vector<int8_t> state;      // per original node: 0 unknown, 1 expandable, -1 not
  std::vector<std::vector<Piece>> memo;
  int32_t zero_pool = -1;
  std::unordered_map<uint64_t, int32_t> made;  // (op, a, params) of appended leaf / extract nodes
  static constexpr size_t kMaxPieces = 64;

  bool is_wide(int32_t j) const { return nd[j].width > MGP_MAX_WIDTH && !op_bool_result(nd[j].op); }

  int32_t append(const mgp_node &x) {
    out.push_back(x);
    return (int32_t)out.size() - 1;
  }
  int32_t leaf(uint8_t op, uint16_t w, uint32_t p0) {
    const uint64_t key = ((uint64_t)op << 56) ^ ((uint64_t)w << 40) ^ p0;
    auto it = made.find(key);
    if (it != made.end()) return it->second;
    mgp_node x{};
    x.op = op;
    x.width = w;
    x.a = x.b = x.c = -1;
    x.p0 = p0;
    return made[key] = append(x);
  }
  int32_t zero(uint16_t w) {
    if (zero_pool < 0) {
      if (xc.empty()) xc.assign(consts, consts + 8ull * n_consts);
      zero_pool = (int32_t)(xc.size() / 8);
      xc.insert(xc.end(), 8, 0u);
    }
    return leaf(MGP_OP_CONST, w, (uint32_t)zero_pool);
  }
  // the node holding piece p exactly (an EXTRACT when p is part of its node)
  int32_t mat(const Piece &p) {
    if (p.lo == 0 && p.w == out[p.node].width) return p.node;
    const uint64_t key = (1ull << 63) ^ ((uint64_t)p.node << 24) ^ ((uint64_t)p.lo << 12) ^ p.w;
    auto it = made.find(key);
    if (it != made.end()) return it->second;
    mgp_node x{};
    x.op = MGP_OP_EXTRACT;
    x.width = p.w;
    x.a = p.node;
    x.b = x.c = -1;
    x.p0 = (uint32_t)(p.lo + p.w - 1u);
    x.p1 = p.lo;
    return made[key] = append(x);
  }
  // bits [lo, lo + w) of a piece list
  static bool slice(const std::vector<Piece> &s, uint32_t lo, uint32_t w, std::vector<Piece> &r) {
    uint32_t at = 0;
    for (const Piece &p : s) {
      const uint32_t a = std::max(at, lo), b = std::min(at + p.w, lo + w);
      if (a < b) r.push_back(Piece{p.node, (uint16_t)(p.lo + (a - at)), (uint16_t)(b - a)});
      at += p.w;
    }
    return r.size() <= kMaxPieces;
  }
  // two piece lists of one total width cut at the union of their boundaries
  static void align(const std::vector<Piece> &x, const std::vector<Piece> &y, std::vector<Piece> &ax,
                    std::vector<Piece> &ay) {
    size_t i = 0, j = 0;
    uint32_t ox = 0, oy = 0;  // offsets consumed within x[i], y[j]
    while (i < x.size() && j < y.size()) {
      const uint32_t w = std::min<uint32_t>(x[i].w - ox, y[j].w - oy);
      ax.push_back(Piece{x[i].node, (uint16_t)(x[i].lo + ox), (uint16_t)w});
      ay.push_back(Piece{y[j].node, (uint16_t)(y[j].lo + oy), (uint16_t)w});
      ox += w;
      oy += w;
      if (ox == x[i].w) { ++i; ox = 0; }
      if (oy == y[j].w) { ++j; oy = 0; }
    }
  }
  // the pieces of original node j (low bits first); false = not built from narrow parts
  bool pieces(int32_t j, std::vector<Piece> &r) {
    if (j < 0 || (uint64_t)j >= n) return false;
    if (state[j] == -1) return false;
    if (state[j] == 1) {
      r = memo[j];
      return true;
    }
    state[j] = -1;
    std::vector<Piece> s;
    const mgp_node &x = nd[j];
    bool ok = false;
    if (!is_wide(j)) {
      // a narrow node: itself, unless it reads a wide value (then relaxed in `out`; rebuilt)
      const bool reads_wide = (x.a >= 0 && is_wide(x.a)) || (x.b >= 0 && is_wide(x.b)) || (x.c >= 0 && is_wide(x.c));
      if (!reads_wide || x.op == MGP_OP_UFAPP || x.op == MGP_OP_UFINV) {
        // (a narrow UF value read through a wide argument is its relaxed fresh value)
        s.push_back(Piece{j, 0, x.width});
        ok = true;
      } else if (x.op == MGP_OP_EXTRACT) {
        std::vector<Piece> a;
        ok = pieces(x.a, a) && slice(a, x.p1, x.width, s);
      }
    } else {
      const uint32_t w = x.width;
      switch (x.op) {
        case MGP_OP_CONCAT: {
          std::vector<Piece> a, b;
          ok = pieces(x.b, b) && pieces(x.a, a);
          if (ok) {
            s = b;
            s.insert(s.end(), a.begin(), a.end());
          }
          break;
        }
        case MGP_OP_EXTRACT: {
          std::vector<Piece> a;
          ok = pieces(x.a, a) && slice(a, x.p1, w, s);
          break;
        }
        case MGP_OP_ZEXT: {
          ok = pieces(x.a, s);
          for (uint32_t at = nd[x.a].width; ok && at < w; at += MGP_MAX_WIDTH)
            s.push_back(Piece{zero((uint16_t)std::min<uint32_t>(MGP_MAX_WIDTH, w - at)), 0,
                              (uint16_t)std::min<uint32_t>(MGP_MAX_WIDTH, w - at)});
          break;
        }
        case MGP_OP_CONST:
          if (x.p0 + (w + 255u) / 256u <= n_consts) {
            for (uint32_t k = 0; k * 256u < w; ++k) {
              const uint16_t pw = (uint16_t)std::min<uint32_t>(256u, w - 256u * k);
              s.push_back(Piece{leaf(MGP_OP_CONST, pw, x.p0 + k), 0, pw});
            }
            ok = true;
          }
          break;
        case MGP_OP_VAR: case MGP_OP_UFINV: case MGP_OP_UFAPP: {
          // a wide variable or fresh UF value: consecutive slots from p0 (VAR) / p1 (UF)
          const uint32_t base = x.op == MGP_OP_VAR ? x.p0 : x.p1;
          for (uint32_t k = 0; k * 256u < w; ++k) {
            const uint16_t pw = (uint16_t)std::min<uint32_t>(256u, w - 256u * k);
            s.push_back(Piece{leaf(MGP_OP_VAR, pw, base + k), 0, pw});
          }
          ok = true;
          break;
        }
        case MGP_OP_ITE: {
          std::vector<Piece> b, c, ab, ac;
          if (!(pieces(x.b, b) && pieces(x.c, c))) break;
          align(b, c, ab, ac);
          if (ab.size() > kMaxPieces) break;
          for (size_t k = 0; k < ab.size(); ++k) {
            mgp_node t{};
            t.op = MGP_OP_ITE;
            t.width = ab[k].w;
            t.a = x.a;  // a narrow Bool condition (relaxed DAG: unchanged)
            t.b = mat(ab[k]);
            t.c = mat(ac[k]);
            s.push_back(Piece{append(t), 0, ab[k].w});
          }
          ok = true;
          break;
        }
        default: break;  // wide arithmetic: stays relaxed
      }
    }
    if (!ok || s.size() > kMaxPieces) return false;
    state[j] = 1;
    memo[j] = s;
    r = s;
    return true;
  }
};
}  // namespace

bool relax_wide(const mgp_node *nd, uint64_t n, std::vector<mgp_node> &out, const uint32_t *consts = nullptr,
                uint64_t n_consts = 0, std::vector<mgp_node> *orig_out = nullptr,
                std::vector<uint32_t> *xconsts = nullptr, std::vector<int32_t> *ties_out = nullptr);

bool relax_wide_narrow(const mgp_node *nd, uint64_t n, std::vector<mgp_node> &out);

bool relax_wide(const mgp_node *nd, uint64_t n, std::vector<mgp_node> &out, const uint32_t *consts,
                uint64_t n_consts, std::vector<mgp_node> *orig_out, std::vector<uint32_t> *xconsts,
                std::vector<int32_t> *ties_out) {
  if (!relax_wide_narrow(nd, n, out)) return false;
  if (!orig_out || !xconsts) return true;
  // piece expansion: ties appended after the relaxed DAG (see above)
  std::vector<uint32_t> &xc = *xconsts;
  xc.clear();
  Expander E{nd, n, out, xc, consts, n_consts, std::vector<int8_t>(n, 0), std::vector<std::vector<Piece>>(n), -1, {}};
  std::vector<int32_t> ties;
  for (uint64_t i = 0; i < n; ++i) {
    const mgp_node &x = nd[i];
    const bool wa = x.a >= 0 && E.is_wide(x.a), wb = x.b >= 0 && E.is_wide(x.b);
    if (x.op == MGP_OP_EQ && wa && wb && nd[x.a].width == nd[x.b].width) {
      std::vector<Piece> pa, pb, aa, ab;
      if (!E.pieces(x.a, pa) || !E.pieces(x.b, pb)) continue;
      Expander::align(pa, pb, aa, ab);
      if (aa.empty() || aa.size() > Expander::kMaxPieces) continue;
      int32_t conj = -1;
      for (size_t k = 0; k < aa.size(); ++k) {
        const int32_t l = E.mat(aa[k]), r = E.mat(ab[k]);
        mgp_node q{};
        q.op = MGP_OP_EQ;
        q.width = 1;
        q.a = l;
        q.b = r;
        q.c = -1;
        int32_t e = E.append(q);
        if (conj >= 0) {
          mgp_node t{};
          t.op = MGP_OP_BAND;
          t.width = 1;
          t.a = conj;
          t.b = e;
          t.c = -1;
          e = E.append(t);
        }
        conj = e;
      }
      mgp_node t{};
      t.op = MGP_OP_BEQ;
      t.width = 1;
      t.a = (int32_t)i;
      t.b = conj;
      t.c = -1;
      ties.push_back(E.append(t));
    } else if (!E.is_wide((int32_t)i) && !op_bool_result(x.op) && x.op == MGP_OP_EXTRACT && wa) {
      std::vector<Piece> p;
      if (!E.pieces((int32_t)i, p) || p.empty() || p.size() > Expander::kMaxPieces) continue;
      // rebuild the value: CONCAT of the pieces, high piece first
      int32_t v = E.mat(p[0]);
      uint32_t vw = p[0].w;
      for (size_t k = 1; k < p.size(); ++k) {
        mgp_node t{};
        t.op = MGP_OP_CONCAT;
        t.width = (uint16_t)(vw + p[k].w);
        t.a = E.mat(p[k]);
        t.b = v;
        t.c = -1;
        v = E.append(t);
        vw += p[k].w;
      }
      mgp_node q{};
      q.op = MGP_OP_EQ;
      q.width = 1;
      q.a = (int32_t)i;
      q.b = v;
      q.c = -1;
      ties.push_back(E.append(q));
    }
  }
  if (ties.empty()) {
    out.resize(n);
    xc.clear();
    return true;
  }
  int32_t root = (int32_t)n - 1;
  for (int32_t t : ties) {
    mgp_node b{};
    b.op = MGP_OP_BAND;
    b.width = 1;
    b.a = root;
    b.b = t;
    b.c = -1;
    root = E.append(b);
  }
  orig_out->assign(nd, nd + n);
  orig_out->insert(orig_out->end(), out.begin() + (int64_t)n, out.end());
  if (ties_out) *ties_out = ties;
  return true;
}

bool relax_wide_narrow(const mgp_node *nd, uint64_t n, std::vector<mgp_node> &out) {
  auto wide = [&](int32_t j) { return j >= 0 && (uint64_t)j < n && nd[j].width > MGP_MAX_WIDTH &&
                                      !op_bool_result(nd[j].op); };
  bool any = false;
  for (uint64_t i = 0; i < n && !any; ++i) any = wide((int32_t)i);
  if (!any) return false;
  out.assign(nd, nd + n);
  uint32_t fresh = 1u << 22;  // beyond every variable index of a real DAG (< 0x3FFF)
  auto fresh_var = [&](mgp_node &x, uint16_t w) {
    x.op = MGP_OP_VAR;
    x.width = w;
    x.a = x.b = x.c = -1;
    x.p0 = fresh++;
    x.p1 = 0;
  };
  for (uint64_t i = 0; i < n; ++i) {
    mgp_node &x = out[i];
    if (wide((int32_t)i)) { fresh_var(x, 8); continue; }
    if (!(wide(nd[i].a) || wide(nd[i].b) || wide(nd[i].c))) continue;
    if ((nd[i].op == MGP_OP_UFAPP || nd[i].op == MGP_OP_UFINV) && nd[i].width <= MGP_MAX_WIDTH) {
      // a narrow UF value read through a wide argument: relaxed to its own fresh-value
      // variable p1 (used by no other node, so still unconstrained), which keeps the
      // constraints on the value attached to the slot the kernel reads it from
      x.op = MGP_OP_VAR;
      x.a = x.b = x.c = -1;
      x.p0 = nd[i].p1;
      x.p1 = 0;
    } else if (op_bool_result(nd[i].op)) {
      // operands are relaxed placeholders (8-bit fresh variables, distinct unless a == b)
      x.op = MGP_OP_EQ;
      x.width = 1;
      x.c = -1;
      if (!wide(x.a) || !wide(x.b)) return false;  // malformed; let setup reject it
    } else {
      fresh_var(x, nd[i].width);
    }
  }
  return true;
}

int refute_one(const mgp_node *nd, uint64_t n, const uint32_t *consts, uint64_t n_consts, uint32_t max_passes,
               State *keep) {
  if (n == 0 || n > (1u << 20)) return -1;
  State st;
  State &s = keep ? *keep : st;
  s.orig = nd;
  if (relax_wide(nd, n, s.relaxed, consts, n_consts, &s.origx, &s.xconsts, &s.ties)) {
    nd = s.relaxed.data();
    n = s.relaxed.size();
    if (!s.origx.empty()) s.orig = s.origx.data();
    if (!s.xconsts.empty()) {
      consts = s.xconsts.data();
      n_consts = s.xconsts.size() / 8u;
    }
  }
  s.nd = nd;
  s.n = (uint32_t)n;
  s.consts = consts;
  s.n_consts = n_consts;
  if (!s.setup()) return -1;
  Dom d = s.view();
  return d.run(max_passes ? max_passes : 16u);
}

// Linear forms (round 6).  Under the analysis' decided select conditions and exact values,
// every BV node of width <= 256 gets a linear form sum(coef * atom) + k mod 2^w over atoms:
// variables, UF applications keyed by (function, exact argument) -- congruent applications
// share one atom -- and any other node as itself.  A required compare whose two operands'
// forms differ by a constant k (a = b + k) is then a condition on b alone: a >u b iff
// k != 0 and b + k does not wrap (b <= 2^w-1-k); a == b iff k == 0.  Balance arithmetic
// across a transfer is such a case: ether_thief.py:55-95 compares the attacker's balance
// after (start - value) + refund with start, and refund = value - price cancels value
// (weak_random.sol:18-35), which intervals cannot see.  Each derived condition is an
// equivalence, so meeting it is sound.  true = refuted.
namespace lin {
constexpr uint32_t kMax = 6;
// atoms are exact identities, never hashes: a variable (slot, width), or a node index -- the
// node itself, or for a UF application the first node applying the same function to the
// same exact argument value
constexpr uint64_t kVarAtom = 1ull << 62, kNodeAtom = 2ull << 62;
struct Form {
  uint8_t n = 0;
  uint64_t atom[kMax];
  V coef[kMax];
  V k;
};
inline Form of_const(const V &k) {
  Form f;
  f.k = k;
  return f;
}
inline Form of_atom(uint64_t a) {
  Form f;
  f.k = bv_zero();
  f.n = 1;
  f.atom[0] = a;
  f.coef[0] = bv_small(1u);
  return f;
}
// r = x + s * y (mod 2^w); false if the atoms do not fit
inline bool axpy(Form &r, const Form &x, const V &sc, const Form &y, uint32_t w) {
  r = x;
  r.k = bv_mask(ADDV(x.k, bv_mul(sc, y.k)), w);
  for (uint32_t j = 0; j < y.n; ++j) {
    const V c = bv_mask(bv_mul(sc, y.coef[j]), w);
    uint32_t t = 0;
    while (t < r.n && r.atom[t] != y.atom[j]) ++t;
    if (t == r.n) {
      if (r.n == kMax) return false;
      r.atom[r.n] = y.atom[j];
      r.coef[r.n++] = c;
    } else {
      r.coef[t] = bv_mask(ADDV(r.coef[t], c), w);
    }
  }
  uint32_t o = 0;  // drop cancelled atoms
  for (uint32_t t = 0; t < r.n; ++t)
    if (!Z(r.coef[t])) {
      r.atom[o] = r.atom[t];
      r.coef[o++] = r.coef[t];
    }
  r.n = (uint8_t)o;
  return true;
}
}  // namespace lin

bool linear_refute(State &s, Dom &d, uint32_t passes) {
  using lin::Form;
  const uint32_t n = s.n;
  std::vector<Form> F(n);
  const V minus1 = bv_ones();
  struct UfRep {
    uint8_t op;
    uint32_t fn, w;
    V arg;
    uint32_t node;
  };
  std::vector<UfRep> reps;
  for (int round = 0; round < 3; ++round) {
    reps.clear();
    for (uint32_t i = 0; i < n; ++i) {
      const mgp_node &x = s.nd[i];
      const uint32_t w = x.width;
      Form &f = F[i];
      f = Form();
      if (s.isb[i] || w == 0u || w > 256u) continue;
      const AV &a = s.av[i];
      if (is_exact(a)) {
        f = lin::of_const(a.lo);
        continue;
      }
      const uint64_t self = lin::kNodeAtom | i;
      auto ok_bv = [&](int32_t j) { return j >= 0 && !s.isb[j] && s.nd[j].width == w; };
      bool done = false;
      switch (x.op) {
        case MGP_OP_VAR:
          f = lin::of_atom(lin::kVarAtom | ((uint64_t)x.p0 << 16) | w);
          done = true;
          break;
        case MGP_OP_UFAPP: case MGP_OP_UFINV:
          if (x.a >= 0 && s.nd[x.a].width <= 256u && is_exact(s.av[x.a])) {
            const V &arg = s.av[x.a].lo;
            uint32_t rep = i;
            for (const UfRep &r : reps)
              if (r.op == x.op && r.fn == x.p0 && r.w == w && EQV(r.arg, arg)) {
                rep = r.node;
                break;
              }
            if (rep == i) reps.push_back(UfRep{x.op, x.p0, w, arg, i});
            f = lin::of_atom(lin::kNodeAtom | rep);
            done = true;
          }
          break;
        case MGP_OP_ADD: case MGP_OP_SUB:
          if (ok_bv(x.a) && ok_bv(x.b))
            done = lin::axpy(f, F[x.a], x.op == MGP_OP_ADD ? bv_small(1u) : minus1, F[x.b], w);
          break;
        case MGP_OP_NEG:
          if (ok_bv(x.a)) done = lin::axpy(f, lin::of_const(bv_zero()), minus1, F[x.a], w);
          break;
        case MGP_OP_MUL:
          if (ok_bv(x.a) && ok_bv(x.b)) {
            if (is_exact(s.av[x.a])) done = lin::axpy(f, lin::of_const(bv_zero()), s.av[x.a].lo, F[x.b], w);
            else if (is_exact(s.av[x.b])) done = lin::axpy(f, lin::of_const(bv_zero()), s.av[x.b].lo, F[x.a], w);
          }
          break;
        case MGP_OP_ITE:
          if (x.a >= 0 && s.bs[x.a] != BB) {
            const int32_t br = s.bs[x.a] == BT ? x.b : x.c;
            if (ok_bv(br)) {
              f = F[br];
              done = true;
            }
          }
          break;
        default:
          break;
      }
      if (!done) f = lin::of_atom(self);
    }
    // the required compares whose operands differ by a constant
    bool narrowed = false;
    for (uint32_t i = 0; i < n; ++i) {
      const mgp_node &x = s.nd[i];
      if (x.op != MGP_OP_EQ && x.op != MGP_OP_ULT && x.op != MGP_OP_ULE && x.op != MGP_OP_UGT && x.op != MGP_OP_UGE)
        continue;
      if (s.bs[i] == BB || x.a < 0 || x.b < 0 || s.isb[x.a]) continue;
      const uint32_t w = s.nd[x.a].width;
      if (w == 0u || w > 256u || s.nd[x.b].width != w) continue;
      Form dlt;
      if (!lin::axpy(dlt, F[x.a], minus1, F[x.b], w) || dlt.n != 0) continue;
      const V k = bv_mask(dlt.k, w);  // a = b + k
      bool truth = s.bs[i] == BT;
      if (x.op == MGP_OP_EQ) {
        if (Z(k) != truth) return true;
        continue;
      }
      // normalise to "a >u b" (UGT) or "a >=u b" (UGE) with the required truth
      bool strict = x.op == MGP_OP_UGT || x.op == MGP_OP_ULE;
      if (x.op == MGP_OP_ULT || x.op == MGP_OP_ULE) truth = !truth;  // ULT = !UGE, ULE = !UGT
      if (Z(k)) {  // a == b: UGT false, UGE true
        if (truth == strict) return true;
        continue;
      }
      // k != 0: a >u b and a >=u b both hold iff b <= 2^w-1-k
      const V lim = SUBV(M(w), k);
      AV t = top(w);
      if (truth) t.hi = lim;
      else t.lo = ADDV(lim, ONE());
      // on b and on every node whose form is exactly b's (a congruent UF application)
      for (uint32_t j = 0; j < n; ++j) {
        if (j != (uint32_t)x.b) {
          const Form &g = F[j], &h = F[x.b];
          if (s.isb[j] || s.nd[j].width != w || g.n != h.n || !EQV(g.k, h.k)) continue;
          bool same = true;
          for (uint32_t q = 0; q < g.n && same; ++q) same = g.atom[q] == h.atom[q] && EQV(g.coef[q], h.coef[q]);
          if (!same) continue;
        }
        const AV before = s.av[j];
        if (!d.meet((int32_t)j, t)) return true;
        narrowed |= !(EQV(before.lo, s.av[j].lo) && EQV(before.hi, s.av[j].hi));
      }
    }
    if (!narrowed) return false;
    if (d.run(passes) == 1) return true;
  }
  return false;
}

// refute_one, then case splitting (failed-literal probing, nested): each open condition of
// a select (BV ITE / BITE), nearest the root first, at most max_splits of them, is assumed
// true and false in turn on a copy of the analysis, and each branch is probed again on the
// others down to `depth` levels; both branches refuted -> refuted; one refuted -> the other
// polarity holds and is kept for the next probes at that level.  Sound: the two assumptions
// cover every model of the state they split.
int refute_split_one(const mgp_node *nd, uint64_t n, const uint32_t *consts, uint64_t n_consts, uint32_t max_passes,
                     uint32_t max_splits) {
  // max_splits: atoms per level in bits 0..15, levels in bits 16..19 (0 = 1), bit 20 set =
  // no linear forms and no interval bisection (the round-6 stages)
  const uint32_t n_atoms = max_splits & 0xFFFFu, depth = std::max<uint32_t>(1u, (max_splits >> 16) & 0xFu);
  const bool bisection = ((max_splits >> 20) & 1u) == 0u;
  State s;
  const int r = refute_one(nd, n, consts, n_consts, max_passes, &s);
  if (r != 0 || n_atoms == 0) return r;
  Dom d = s.view();
  const uint32_t passes = max_passes ? max_passes : 16u;
  std::vector<int32_t> atoms;
  std::vector<uint8_t> seen(s.n, 0);
  for (uint32_t i = s.n; i-- > 0 && atoms.size() < n_atoms;) {
    const mgp_node &x = s.nd[i];
    if ((x.op != MGP_OP_ITE && x.op != MGP_OP_BITE) || x.a < 0 || seen[x.a] || s.bs[x.a] != BB) continue;
    seen[x.a] = 1;
    atoms.push_back(x.a);
  }
  struct Snap {
    std::vector<AV> av, vars;
    std::vector<uint8_t> bs;
    std::vector<Pair> pairs;
  };
  auto take = [&](Snap &c) { c.av = s.av; c.vars = s.vars; c.bs = s.bs; c.pairs = s.pairs; };
  auto put = [&](const Snap &c) {
    std::copy(c.av.begin(), c.av.end(), s.av.begin());
    std::copy(c.vars.begin(), c.vars.end(), s.vars.begin());
    std::copy(c.bs.begin(), c.bs.end(), s.bs.begin());
    std::copy(c.pairs.begin(), c.pairs.end(), s.pairs.begin());
  };
  std::vector<Snap> snaps(depth);
  // work cap: at most kSplitWork node evaluations of propagation per state, so a
  // WalletLibrary-size state (600-1 500 nodes) cannot spend a second in nested probes before
  // the fallback; when it runs out the probes stop and the state is "not refuted" (sound)
  constexpr uint64_t kSplitWork = 1ull << 23;
  int64_t runs_left = (int64_t)std::max<uint64_t>(32u, kSplitWork / ((uint64_t)s.n * passes + 1u));
  auto run_capped = [&]() -> int {
    if (--runs_left < 0) return 0;
    return d.run(passes);
  };
  // true = the analysis as it stands (propagated) is refuted by splits `level` deep
  std::function<bool(uint32_t)> probe = [&](uint32_t level) -> bool {
    if (level == 0 || runs_left <= 0) return false;
    Snap &c = snaps[level - 1];
    for (int32_t a : atoms) {
      if (s.bs[a] != BB) continue;
      if (runs_left <= 0) return false;
      take(c);
      // (each branch also gets the linear-form pass: a select condition decided by the
      // branch -- sender == ATTACKER in an earlier transaction -- resolves the balance
      // selects whose forms then cancel)
      const bool rt = !d.meetb(a, BT) || run_capped() == 1 || (bisection && linear_refute(s, d, passes)) ||
                      probe(level - 1);
      put(c);
      const bool rf = !d.meetb(a, BF) || run_capped() == 1 || (bisection && linear_refute(s, d, passes)) ||
                      probe(level - 1);
      put(c);
      if (rt && rf) return true;
      if (rt || rf) {  // the other polarity holds in every model of this branch
        if (!d.meetb(a, rt ? BF : BT) || d.run(passes) == 1) return true;
      }
    }
    return false;
  };
  if (probe(depth)) return 1;
  if (!bisection) return 0;
  if (linear_refute(s, d, passes)) return 1;
  // Interval bisection (round 6): a variable whose interval the analysis bounded (a call
  // value between two require()s, a balance below a cap) is split in two halves, each
  // half propagated and split again, kBisectDepth levels; every leaf refuted -> refuted.
  // Intervals lose the relation between two terms computed from one variable (rubixi.sol
  // addPayout: value * 90 / 100 > value * 300 / 100 for 1 ether <= value < 50 ether holds
  // for no value, yet the two quotients' intervals overlap); on a narrow enough piece of the
  // variable's range they no longer do.  Sound: the halves cover the interval.  Split points
  // follow the bit lengths first (a ratio test needs pieces within a constant factor), then
  // the arithmetic midpoint.
  constexpr uint32_t kBisectVars = 6, kBisectDepth = 8;
  std::vector<int32_t> bvars;
  for (uint32_t i = s.n; i-- > 0 && bvars.size() < kBisectVars;) {
    const mgp_node &x = s.nd[i];
    if (x.op != MGP_OP_VAR && x.op != MGP_OP_UFAPP && x.op != MGP_OP_UFINV) continue;
    if (x.width < 2u || x.width > 256u) continue;
    const AV &a = s.av[i];
    if (is_exact(a) || (Z(a.lo) && EQV(a.hi, M(x.width)))) continue;  // one value, or unbounded
    bvars.push_back((int32_t)i);
  }
  std::vector<Snap> bsnaps(kBisectDepth);
  std::function<bool(int32_t, uint32_t)> bisect = [&](int32_t v, uint32_t level) -> bool {
    if (level == 0 || runs_left <= 0) return false;
    const AV a = s.av[v];
    if (is_exact(a)) return false;
    const uint32_t w = s.nd[v].width, lb = bv_bitlen(a.lo), hb = bv_bitlen(a.hi);
    V mid = hb > lb + 1u ? SUBV(SHL(ONE(), (lb + hb) / 2u), ONE())
                         : ADDV(a.lo, SHR(SUBV(a.hi, a.lo), 1u));
    if (LT(mid, a.lo) || !LT(mid, a.hi)) mid = ADDV(a.lo, SHR(SUBV(a.hi, a.lo), 1u));
    Snap &c = bsnaps[level - 1];
    take(c);
    for (int side = 0; side < 2; ++side) {
      AV t = top(w);
      t.lo = side ? ADDV(mid, ONE()) : a.lo;
      t.hi = side ? a.hi : mid;
      const bool r = !d.meet(v, t) || run_capped() == 1 || bisect(v, level - 1);
      put(c);
      if (!r) return false;
    }
    return true;
  };
  for (int32_t v : bvars)
    if (bisect(v, kBisectDepth)) return 1;
  return 0;
}

}  // namespace

extern "C" int mgp_refute_split(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                uint32_t max_splits, int8_t *out) {
  if (!node_offsets || !out || (n_states && (!nodes || !const_offsets))) return MGP_E_ARG;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const uint64_t n0 = node_offsets[s], n1 = node_offsets[s + 1];
    const uint64_t c0 = const_offsets[s], c1 = const_offsets[s + 1];
    if (n1 < n0 || c1 < c0) {
      out[s] = -1;
      continue;
    }
    out[s] = (int8_t)refute_split_one(nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0, max_passes,
                                      max_splits);
  }
  return MGP_OK;
}

namespace {
// The root conjuncts of a DAG built by mgp_build_states from k constraints: the roots are
// AND-chained into the last k - 1 nodes (mgp_front.cpp build_one); k = 1 is the last node
// (or BAND(r, r) after it).  false = the tail is not such a chain.
bool chain_roots(const mgp_node *nd, uint64_t n, uint32_t k, std::vector<int32_t> &roots) {
  roots.clear();
  if (k == 0 || n == 0) return false;
  if (k == 1) {
    const mgp_node &t = nd[n - 1];
    roots.push_back(t.op == MGP_OP_BAND && t.a == t.b ? t.a : (int32_t)(n - 1));
    return true;
  }
  if (n < k) return false;
  const uint64_t c1 = n - (k - 1);  // first chain node: BAND(r0, r1)
  roots.assign(k, -1);
  for (uint32_t i = 1; i < k; ++i) {
    const mgp_node &t = nd[c1 + i - 1];
    if (t.op != MGP_OP_BAND || (i > 1 && t.a != (int32_t)(c1 + i - 2))) return false;
    roots[i] = t.b;
    if (i == 1) roots[0] = t.a;
  }
  return true;
}

// One refuted constraint list's core: the fewest root conjuncts (a minimal set under the
// refuter, not a minimum) found by halving rounds and then greedy single deletions, every
// trial re-running the analysis from the state's set-up values with only the kept conjuncts
// (and the piece ties) required -- one DAG and one set-up per list, no rebuilding per trial.
int core_one(const mgp_node *nd, uint64_t n, const uint32_t *consts, uint64_t n_consts, uint32_t k,
             uint32_t max_passes, uint32_t halvings, uint32_t max_single, uint8_t *keep) {
  std::vector<int32_t> roots;
  for (uint32_t i = 0; i < k; ++i) keep[i] = 1;
  if (!chain_roots(nd, n, k, roots)) return -1;
  State s;
  s.orig = nd;
  const mgp_node *d0 = nd;
  uint64_t nn = n;
  if (relax_wide(nd, n, s.relaxed, consts, n_consts, &s.origx, &s.xconsts, &s.ties)) {
    d0 = s.relaxed.data();
    nn = s.relaxed.size();
    if (!s.origx.empty()) s.orig = s.origx.data();
    if (!s.xconsts.empty()) {
      consts = s.xconsts.data();
      n_consts = s.xconsts.size() / 8u;
    }
  }
  s.nd = d0;
  s.n = (uint32_t)nn;
  s.consts = consts;
  s.n_consts = n_consts;
  if (!s.setup()) return -1;
  const std::vector<AV> av0 = s.av, vars0 = s.vars;
  const std::vector<uint8_t> bs0 = s.bs;
  const std::vector<Pair> pairs0 = s.pairs;
  const uint32_t passes = max_passes ? max_passes : 16u;
  std::vector<int32_t> req;
  auto refuted = [&](const std::vector<uint32_t> &sel) {
    std::copy(av0.begin(), av0.end(), s.av.begin());
    std::copy(vars0.begin(), vars0.end(), s.vars.begin());
    std::copy(bs0.begin(), bs0.end(), s.bs.begin());
    std::copy(pairs0.begin(), pairs0.end(), s.pairs.begin());
    req.assign(s.ties.begin(), s.ties.end());
    for (uint32_t i : sel) req.push_back(roots[i]);
    Dom d = s.view();
    d.req = req.data();
    d.n_req = (uint32_t)req.size();
    return d.run(passes) == 1;
  };
  std::vector<uint32_t> cur(k);
  for (uint32_t i = 0; i < k; ++i) cur[i] = i;
  // The lists come from refutations, so the whole list is not tested first: a refuted
  // subset (the analysis is monotone in the required conjuncts) shows it, and only a list
  // none of whose trials is refuted pays the whole-list test.  The newer half goes first: a
  // path's older constraints are its parent's, which were satisfiable.
  bool shown = false;
  for (uint32_t h = 0; h < halvings && cur.size() >= 8; ++h) {
    const size_t m = cur.size() / 2;
    std::vector<uint32_t> lo(cur.begin(), cur.begin() + (int64_t)m), hi(cur.begin() + (int64_t)m, cur.end());
    if (refuted(hi)) cur.swap(hi);
    else if (refuted(lo)) cur.swap(lo);
    else break;
    shown = true;
  }
  if (cur.size() >= 2 && cur.size() <= max_single) {
    for (size_t i = 0; i < cur.size() && cur.size() > 1;) {
      std::vector<uint32_t> t(cur);
      t.erase(t.begin() + (int64_t)i);
      if (refuted(t)) {  // conjunct i is not needed: drop it for good
        cur.swap(t);
        shown = true;
      } else {
        ++i;
      }
    }
  }
  if (!shown && !refuted(cur)) {  // not refuted as a whole: keep everything
    for (uint32_t i = 0; i < k; ++i) keep[i] = 1;
    return 0;
  }
  for (uint32_t i = 0; i < k; ++i) keep[i] = 0;
  for (uint32_t i : cur) keep[i] = 1;
  return 1;
}
}  // namespace

// UNSAT cores of refuted constraint lists (solver.UnsatCores.shrink_many, round 5): per
// state, its DAG as mgp_build_states builds it from the list's `n_roots[s]` constraints;
// keep (one byte per constraint, states concatenated) gets 1 for the constraints of the
// core.  out[s]: 1 = core found (refuted), 0 = the whole list is not refuted (all kept),
// -1 = not a root chain / malformed (all kept).
extern "C" int mgp_refute_cores(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                const uint32_t *consts, const uint64_t *const_offsets, const uint32_t *n_roots,
                                uint32_t max_passes, uint32_t halvings, uint32_t max_single, uint8_t *keep,
                                int8_t *out) {
  if (!node_offsets || !out || !n_roots || (n_states && (!nodes || !const_offsets || !keep))) return MGP_E_ARG;
  std::vector<uint64_t> koff(n_states + 1, 0);
  for (uint32_t s = 0; s < n_states; ++s) koff[s + 1] = koff[s] + n_roots[s];
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const uint64_t n0 = node_offsets[s], n1 = node_offsets[s + 1];
    const uint64_t c0 = const_offsets[s], c1 = const_offsets[s + 1];
    if (n1 < n0 || c1 < c0) {
      out[s] = -1;
      for (uint32_t i = 0; i < n_roots[s]; ++i) keep[koff[s] + i] = 1;
      continue;
    }
    out[s] = (int8_t)core_one(nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0, n_roots[s],
                              max_passes, halvings, max_single, keep + koff[s]);
  }
  return MGP_OK;
}

extern "C" int mgp_refute(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                          const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                          int8_t *out) {
  if (!node_offsets || !out || (n_states && (!nodes || !const_offsets))) return MGP_E_ARG;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const uint64_t n0 = node_offsets[s], n1 = node_offsets[s + 1];
    const uint64_t c0 = const_offsets[s], c1 = const_offsets[s + 1];
    if (n1 < n0 || c1 < c0) {
      out[s] = -1;
      continue;
    }
    out[s] = (int8_t)refute_one(nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0,
                                max_passes, nullptr);
  }
  return MGP_OK;
}

// mgp_refute plus, for every variable slot of a state it does not refute, the slot's
// refined abstract value: 33 u32 per slot of var_off (z, o, lo, hi as 8 limbs each,
// then 1 if the slot has a domain).  The device candidate generator draws every other
// first-round row from these domains (mgp_check_batch).
extern "C" int mgp_refute_domains(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                  const uint32_t *consts, const uint64_t *const_offsets, const uint64_t *var_off,
                                  uint32_t max_passes, int8_t *out, uint32_t *out_dom) {
  // out_dom may be null when the batch has no variable at all (e.g. a state that is one
  // literal False, tests/laser/state/calldata_test.py:41-55 after folding)
  if (!node_offsets || !out || !var_off || (n_states && (!nodes || !const_offsets))) return MGP_E_ARG;
  if (!out_dom && var_off[n_states] > 0) return MGP_E_ARG;
  // zeroed per state by the threads (a 1 024-state batch's domains are ~20 MB)
  if (out_dom && var_off[0]) memset(out_dom, 0, (size_t)var_off[0] * 33u * 4u);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t st = 0; st < (int64_t)n_states; ++st) {
    if (out_dom && var_off[st + 1] > var_off[st])
      memset(out_dom + var_off[st] * 33u, 0, (size_t)(var_off[st + 1] - var_off[st]) * 33u * 4u);
    const uint64_t n0 = node_offsets[st], n1 = node_offsets[st + 1];
    const uint64_t c0 = const_offsets[st], c1 = const_offsets[st + 1];
    if (n1 < n0 || c1 < c0) {
      out[st] = -1;
      continue;
    }
    State s;
    const int r = refute_one(nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0, max_passes, &s);
    out[st] = (int8_t)r;
    if (r != 0) continue;
    const uint64_t nv = var_off[st + 1] - var_off[st];
    for (uint32_t i = 0; i < s.n; ++i) {
      const mgp_node &x = s.nd[i];
      uint32_t v;
      if (x.op == MGP_OP_VAR) v = x.p0;
      else if (x.op == MGP_OP_UFAPP || x.op == MGP_OP_UFINV) v = x.p1;
      else continue;
      if (v >= nv || x.width == 0u || x.width > MGP_MAX_WIDTH) continue;
      uint32_t *d = out_dom + (var_off[st] + v) * 33u;
      const AV &a = s.av[i];
      memcpy(d, a.z.w, 32);
      memcpy(d + 8, a.o.w, 32);
      memcpy(d + 16, a.lo.w, 32);
      memcpy(d + 24, a.hi.w, 32);
      d[32] = 1u;
    }
  }
  return MGP_OK;
}

extern "C" int mgp_refute_trace(const mgp_node *nodes, uint64_t n_nodes, const uint32_t *consts,
                                uint64_t n_consts, uint32_t max_passes, uint32_t *out_av) {
  if (!nodes || !out_av) return MGP_E_ARG;
  State s;
  const int r = refute_one(nodes, n_nodes, consts, n_consts, max_passes, &s);
  if (r < 0) return r;
  for (uint64_t i = 0; i < n_nodes; ++i) {
    uint32_t *o = out_av + 33ull * i;
    memcpy(o, s.av[i].z.w, 32);
    memcpy(o + 8, s.av[i].o.w, 32);
    memcpy(o + 16, s.av[i].lo.w, 32);
    memcpy(o + 24, s.av[i].hi.w, 32);
    o[32] = s.bs[i];
  }
  return r;
}

namespace {
// One value of width w inside the abstract value a (mgp_fe_sample.h, shared with the
// candidate generators).
V sample_av(const AV &a, uint32_t w, uint32_t row, uint64_t r0) {
  return fe_sample_domain(a.z, a.o, a.lo, a.hi, w, row, r0);
}

// One state prepared for decision rows: its base analysis (refute_one) with the
// propagation graph built, the variable slots the decisions fix (VAR nodes and the fresh
// value of UF applications) and, per slot, the constants it is compared equal to.
struct Prep {
  State s;
  int r = -1;
  std::vector<uint32_t> slot, width;
  std::vector<int32_t> node;
  std::vector<uint32_t> eqh_off;  // per slot, into eqh
  std::vector<V> eqh;
  PrepView view() const {
    PrepView p;
    p.n_slot = (uint32_t)slot.size();
    p.slot = slot.data();
    p.width = width.data();
    p.node = node.data();
    p.eqh_off = eqh_off.data();
    p.eqh = eqh.data();
    return p;
  }
};

void prep_state(Prep &P, const mgp_node *nodes, uint64_t n, const uint32_t *consts, uint64_t n_consts,
                uint32_t max_passes, uint32_t n_vars) {
  P.r = refute_one(nodes, n, consts, n_consts, max_passes, &P.s);
  if (P.r != 0) return;
  State &s = P.s;
  s.build_graph();
  // (var slot, width, abstract value): VAR nodes and the fresh value of UF applications
  std::vector<int32_t> kof(s.n, -1);
  for (uint32_t i = 0; i < s.n; ++i) {
    const mgp_node &x = s.nd[i];
    uint32_t v;
    if (x.op == MGP_OP_VAR) v = x.p0;
    else if (x.op == MGP_OP_UFAPP || x.op == MGP_OP_UFINV) v = x.p1;
    else continue;
    if (v >= n_vars || x.width == 0u || x.width > MGP_MAX_WIDTH) continue;
    kof[i] = (int32_t)P.slot.size();
    P.slot.push_back(v);
    P.width.push_back(x.width);
    P.node.push_back((int32_t)i);
  }
  // Values each variable is compared equal to (x == c anywhere in the DAG, e.g. the
  // sender against every ACTORS address, transaction/symbolic.py:165-167): an interval
  // cannot hold such a value set, so decisions try them first and plain domain rows
  // draw one half of the time when it lies inside the refined domain.  In node order
  // per variable, at most 16.
  std::vector<std::vector<V>> eqh(P.slot.size());
  for (uint32_t i = 0; i < s.n; ++i) {
    const mgp_node &x = s.nd[i];
    if (x.op != MGP_OP_EQ || x.a < 0 || x.b < 0) continue;
    for (int side = 0; side < 2; ++side) {
      const int32_t me = side ? x.b : x.a, other = side ? x.a : x.b;
      const int32_t k = kof[me];
      if (k < 0 || (side && x.a == x.b)) continue;
      if (s.nd[other].op != MGP_OP_CONST || s.nd[other].width > MGP_MAX_WIDTH) continue;
      if (s.nd[other].p0 >= s.n_consts || eqh[k].size() >= 16) continue;
      V c;
      memcpy(c.w, s.consts + 8ull * s.nd[other].p0, 32);
      eqh[k].push_back(bv_mask(c, P.width[k]));
    }
  }
  // ... then the smallest value whose product with a constant c >= 2 wraps,
  // floor((2^w-1)/c) + 1 (x * c and BVMulNoOverflow(x, c)): an interval holding the
  // variable's bounds says nothing about where x * c wraps, so a draw from it almost never
  // lands past that boundary (rubixi.sol:130-151: payout = value * multiplier / 100 above
  // the balance share only once value * multiplier wraps)
  for (uint32_t i = 0; i < s.n; ++i) {
    const mgp_node &x = s.nd[i];
    if ((x.op != MGP_OP_MUL && x.op != MGP_OP_UMUL_NOOVF) || x.a < 0 || x.b < 0) continue;
    for (int side = 0; side < 2; ++side) {
      const int32_t me = side ? x.b : x.a, other = side ? x.a : x.b;
      const int32_t k = kof[me];
      if (k < 0 || s.nd[other].op != MGP_OP_CONST || s.nd[other].p0 >= s.n_consts) continue;
      const uint32_t w = P.width[k];
      if (w < 2u || w > 256u || eqh[k].size() >= 16) continue;
      V c, q, r;
      memcpy(c.w, s.consts + 8ull * s.nd[other].p0, 32);
      c = bv_mask(c, w);
      if (bv_ult(c, bv_small(2u))) continue;
      bv_udivrem(bv_mask(bv_ones(), w), c, &q, &r);
      const V b = bv_mask(bv_add(q, bv_small(1u), nullptr), w);
      bool dup = false;
      for (const V &e : eqh[k]) dup |= bv_eq(e, b);
      if (!dup) eqh[k].push_back(b);
    }
  }
  P.eqh_off.assign(1, 0u);
  for (const auto &e : eqh) {
    P.eqh.insert(P.eqh.end(), e.begin(), e.end());
    P.eqh_off.push_back((uint32_t)P.eqh.size());
  }
}

// MGP_DECIDE_OR=mask: the rows that start with the Or case split (A/B)
uint32_t or_rows_mask() {
  static const uint32_t m = [] {
    const char *e = getenv("MGP_DECIDE_OR");
    return e ? (uint32_t)strtoul(e, nullptr, 0) : kOrRowsDefault;
  }();
  return m;
}

// A per-thread scratch array: grows on demand without value-initialising its entries,
// and trim() frees it once it holds more than kKeepBytes.
template <typename T>
struct RowBuf {
  static constexpr size_t kKeepBytes = 8u << 20;
  std::unique_ptr<T[]> p;
  size_t cap = 0;
  T *ensure(size_t n) {
    if (n > cap) {
      p.reset(new T[n]);
      cap = n;
    }
    return p.get();
  }
  void trim() {
    if (cap * sizeof(T) > kKeepBytes) {
      p.reset();
      cap = 0;
    }
  }
};

// A state given zero decision rows (rows_per_state; the first round's rows go to large
// states only) is not analysed at all: its status is 0 and it takes no task.
inline bool skip_prep(const uint8_t *rows_per_state, uint32_t n_decide, uint32_t st) {
  return rows_per_state && n_decide && rows_per_state[st] == 0;
}

// Host run of mgpd::decision_row on a private copy of P's base analysis.
template <typename Put>
void decision_row(const Prep &P, uint32_t row, uint32_t c, uint64_t seed, uint64_t tag, Put &put,
                  const uint32_t *sv = nullptr, const uint8_t *sm = nullptr, uint32_t seed_rows = 0) {
  const State &s = P.s;
  // the row's private copy of the base analysis, in per-thread vectors that keep their
  // capacity across rows (fresh ~150 KB copies per row were page faults the threads of a
  // large batch take in turn)
  static thread_local std::vector<AV> av, vars;
  static thread_local std::vector<uint8_t> bs;
  static thread_local std::vector<Pair> pairs;
  av.assign(s.av.begin(), s.av.end());
  vars.assign(s.vars.begin(), s.vars.end());
  bs.assign(s.bs.begin(), s.bs.end());
  pairs.assign(s.pairs.begin(), s.pairs.end());
  // the undo log and work list live in per-thread buffers reused across rows (only the
  // first `cap` entries of each are addressable, as on the device); allocated without a
  // zero fill, and released after a row of a large state so that one big state does not
  // pin hundreds of MB per OpenMP thread for the rest of the process
  static thread_local RowBuf<UndoRec> undo_buf;
  static thread_local RowBuf<uint32_t> work_buf;
  const uint32_t ucap = undo_cap(s.n, (uint32_t)s.pairs.size(), (uint32_t)s.ufs.size());
  const uint32_t wcap = work_cap(s.n, (uint32_t)s.pairs.size(), (uint32_t)s.ufs.size());
  Stack<UndoRec> undo;
  undo.p = undo_buf.ensure(ucap);
  undo.cap = ucap;
  Stack<uint32_t> work;
  work.p = work_buf.ensure(wcap);
  work.cap = wcap;
  Dom d = const_cast<State &>(s).view();
  d.av = av.data();
  d.bs = bs.data();
  d.vars = vars.data();
  d.pairs = pairs.data();
  d.undo = &undo;
  d.touched = &work;
  d.heur = true;
  const PrepView pv = P.view();
  mgpd::decision_row(pv, d, row, c, seed, tag, or_rows_mask(), put, sv, sm, seed_rows);
  undo_buf.trim();
  work_buf.trim();
  if (av.capacity() * sizeof(AV) > RowBuf<AV>::kKeepBytes) {  // (as the undo log: no big state pinned)
    std::vector<AV>().swap(av);
    std::vector<AV>().swap(vars);
    std::vector<Pair>().swap(pairs);
  }
}
}  // namespace

extern "C" int mgp_guided_candidates_rows(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                          const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                          uint32_t n_cand, uint32_t n_vars, uint64_t seed, uint32_t every,
                                          uint32_t n_decide, const uint8_t *rows_per_state, uint32_t *cands,
                                          int8_t *out) {
  if (!node_offsets || !out || (n_states && (!nodes || !const_offsets || !cands)) || every == 0u)
    return MGP_E_ARG;
  // Per chunk of states: the base analysis, the variable slots and their compared
  // constants once per state (in parallel), then one task per (state, decision row) and
  // one per state for its plain rows, so that a small batch (LASER forks two states per
  // JUMPI, svm.py:251-255) spreads its decision rows over the host threads.
  uint32_t n_dec_rows = 0;
  for (uint32_t c = 0, row = 0; c < n_cand && row < n_decide; c += every, ++row) ++n_dec_rows;
  const int64_t per_state = (int64_t)n_dec_rows + 1;
  constexpr uint32_t kChunk = 256;
  for (uint32_t cs = 0; cs < n_states; cs += kChunk) {
    const uint32_t ce = std::min<uint32_t>(n_states, cs + kChunk);
    std::vector<Prep> prep(ce - cs);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t st = cs; st < (int64_t)ce; ++st) {
      Prep &P = prep[st - cs];
      const uint64_t n0 = node_offsets[st], n1 = node_offsets[st + 1];
      const uint64_t c0 = const_offsets[st], c1 = const_offsets[st + 1];
      prep_state(P, nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0, max_passes, n_vars);
      out[st] = (int8_t)P.r;
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t task = (int64_t)cs * per_state; task < (int64_t)ce * per_state; ++task) {
      const int64_t st = task / per_state;
      const uint32_t task_row = (uint32_t)(task % per_state);  // < n_dec_rows: that decision row
      const Prep &P = prep[st - cs];
      if (P.r != 0) continue;
      // decision rows of this state (the rest of its guided rows are plain domain draws)
      const uint32_t rs = rows_per_state ? std::min<uint32_t>(rows_per_state[st], n_dec_rows) : n_dec_rows;
      if (task_row < n_dec_rows && task_row >= rs) continue;
      const State &s = P.s;
      for (uint32_t c = 0, row = 0; c < n_cand; c += every, ++row) {
        uint32_t *dst = cands + ((uint64_t)st * n_cand + c) * n_vars * 8ull;
        if (task_row < n_dec_rows ? row != task_row : row < rs) continue;
        if (row < rs) {
          auto put = [&](uint32_t sl, const V &v) { memcpy(dst + sl * 8ull, v.w, 32); };
          decision_row(P, row, c, seed, (uint64_t)st << 32, put);
          continue;
        }
        for (size_t k = 0; k < P.slot.size(); ++k) {
          const uint64_t key = fe_mix64(seed ^ fe_mix64(((uint64_t)st << 32) ^ ((uint64_t)c << 12) ^ P.slot[k]));
          V v = sample_av(s.av[P.node[k]], P.width[k], row, key);
          const uint32_t h0 = P.eqh_off[k], nh = P.eqh_off[k + 1] - h0;
          if (nh && (fe_mix64(key ^ 0x9E37ull) & 1u)) {
            const V h = P.eqh[h0 + fe_mix64(key ^ 0x7F4Aull) % nh];
            if (inside_av(s.av[P.node[k]], h)) v = h;
          }
          memcpy(dst + P.slot[k] * 8ull, v.w, 32);
        }
      }
    }
  }
  return 0;
}

extern "C" int mgp_decision_rows_seeded(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                        const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                        uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t n_decide,
                                        const uint8_t *rows_per_state, const uint32_t *seed_vals,
                                        const uint8_t *seed_mask, uint32_t seed_rows, uint32_t *out_rows,
                                        uint8_t *out_mask, int8_t *out);

extern "C" int mgp_decision_rows(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                 const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                 uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t n_decide,
                                 const uint8_t *rows_per_state, uint32_t *out_rows, uint8_t *out_mask,
                                 int8_t *out) {
  return mgp_decision_rows_seeded(nodes, node_offsets, n_states, consts, const_offsets, max_passes, n_vars, seed,
                                  state_keys, n_decide, rows_per_state, nullptr, nullptr, 0u, out_rows, out_mask, out);
}

extern "C" int mgp_decision_rows_seeded(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                        const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                        uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t n_decide,
                                        const uint8_t *rows_per_state, const uint32_t *seed_vals,
                                        const uint8_t *seed_mask, uint32_t seed_rows, uint32_t *out_rows,
                                        uint8_t *out_mask, int8_t *out) {
  return mgp_decision_rows_from(nodes, node_offsets, n_states, consts, const_offsets, max_passes, n_vars, seed,
                                state_keys, 0u, n_decide, rows_per_state, seed_vals, seed_mask, seed_rows, out_rows,
                                out_mask, out);
}

extern "C" int mgp_decision_rows_from(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                      const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                      uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t row0,
                                      uint32_t n_decide, const uint8_t *rows_per_state, const uint32_t *seed_vals,
                                      const uint8_t *seed_mask, uint32_t seed_rows, uint32_t *out_rows,
                                      uint8_t *out_mask, int8_t *out) {
  if (row0 > 255u) return MGP_E_ARG;
  if ((seed_vals == nullptr) != (seed_mask == nullptr)) return MGP_E_ARG;
  if (!node_offsets || !out || (n_states && (!nodes || !const_offsets)) ||
      (n_states && n_decide && (!out_rows || !out_mask)))
    return MGP_E_ARG;
  if (n_states && n_decide) memset(out_mask, 0, (size_t)n_states * n_decide * n_vars);
  // one row per state (the first round's row of large states): a state's analysis and its
  // row are one task, so the threads stay busy to the end instead of meeting at a barrier
  // between the analyses and the rows of every 256-state chunk (the same rows)
  if (n_decide == 1) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t st = 0; st < (int64_t)n_states; ++st) {
      if (skip_prep(rows_per_state, n_decide, (uint32_t)st)) {
        out[st] = 0;
        continue;
      }
      const uint64_t n0 = node_offsets[st], n1 = node_offsets[st + 1];
      const uint64_t c0 = const_offsets[st], c1 = const_offsets[st + 1];
      Prep P;
      prep_state(P, nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0, max_passes, n_vars);
      out[st] = (int8_t)P.r;
      const uint32_t rs = rows_per_state ? std::min<uint32_t>(rows_per_state[st], 1u) : 1u;
      if (P.r != 0 || rs == 0) continue;
      const uint64_t tag = state_keys ? state_keys[st] : (uint64_t)st << 32;
      const uint64_t r0 = (uint64_t)st * n_vars;
      auto put = [&](uint32_t sl, const V &v) {
        memcpy(out_rows + (r0 + sl) * 8ull, v.w, 32);
        out_mask[r0 + sl] = 1;
      };
      const uint64_t sb = (uint64_t)st * n_vars;
      decision_row(P, row0, 2u * row0, seed, tag, put, seed_vals ? seed_vals + sb * 8u : nullptr,
                   seed_mask ? seed_mask + sb : nullptr, seed_rows);
    }
    return MGP_OK;
  }
  constexpr uint32_t kChunk = 256;
  for (uint32_t cs = 0; cs < n_states; cs += kChunk) {
    const uint32_t ce = std::min<uint32_t>(n_states, cs + kChunk);
    std::vector<Prep> prep(ce - cs);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t st = cs; st < (int64_t)ce; ++st) {
      if (skip_prep(rows_per_state, n_decide, (uint32_t)st)) {  // no rows: not analysed
        prep[st - cs].r = 0;
        out[st] = 0;
        continue;
      }
      const uint64_t n0 = node_offsets[st], n1 = node_offsets[st + 1];
      const uint64_t c0 = const_offsets[st], c1 = const_offsets[st + 1];
      prep_state(prep[st - cs], nodes + n0, n1 - n0, consts ? consts + 8ull * c0 : nullptr, c1 - c0, max_passes,
                 n_vars);
      out[st] = (int8_t)prep[st - cs].r;
    }
    // one task per (state, row): a small batch spreads its rows over the host threads
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t task = (int64_t)cs * n_decide; task < (int64_t)ce * n_decide; ++task) {
      const int64_t st = task / n_decide;
      const uint32_t row = (uint32_t)(task % n_decide);
      const Prep &P = prep[st - cs];
      const uint32_t rs = rows_per_state ? std::min<uint32_t>(rows_per_state[st], n_decide) : n_decide;
      if (P.r != 0 || row >= rs) continue;
      const uint64_t tag = state_keys ? state_keys[st] : (uint64_t)st << 32;
      const uint64_t r0 = ((uint64_t)st * n_decide + row) * n_vars;
      auto put = [&](uint32_t sl, const V &v) {
        memcpy(out_rows + (r0 + sl) * 8ull, v.w, 32);
        out_mask[r0 + sl] = 1;
      };
      const uint64_t sb = (uint64_t)st * n_vars;
      const uint32_t ar = row0 + row;  // the absolute decision row
      decision_row(P, ar, 2u * ar, seed, tag, put, seed_vals ? seed_vals + sb * 8u : nullptr,
                   seed_mask ? seed_mask + sb : nullptr, seed_rows);
    }
  }
  return MGP_OK;
}

extern "C" int mgp_guided_candidates(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                                     const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                                     uint32_t n_cand, uint32_t n_vars, uint64_t seed, uint32_t every,
                                     uint32_t n_decide, uint32_t *cands, int8_t *out) {
  return mgp_guided_candidates_rows(nodes, node_offsets, n_states, consts, const_offsets, max_passes, n_cand, n_vars,
                                    seed, every, n_decide, nullptr, cands, out);
}
