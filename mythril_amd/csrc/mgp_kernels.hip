// mgp_kernels.hip — gfx950 kernels of the Mythril satisfiability pre-filter.
//
//   mgp_eval_kernel      constraint bytecode x candidate models, first-SAT
//   mgp_finalize_kernel  per-state min over candidate chunks + witness copy
//   mgp_fill_kernel      Philox4x32-10 benchmark candidates (untimed)
//   mgp_plant_kernel     scatter planted witnesses into the candidate array
//   mgp_transpose_kernel host AoS candidates -> device SoA layout
//   mgp_keccak_kernel    batched Keccak-256, one preimage per lane
//   mgp_preimage_kernel  benchmark mapping-slot preimages (untimed)
//
// Execution model: one 64-lane wave per (state,
// 64-candidate chunk).  The bytecode and constant pool are wave-uniform and
// are fetched through the scalar cache (s_load) — every lane of a wave runs
// the same instruction on its own candidate, so the opcode dispatch is a
// uniform branch with no divergence.  Each lane keeps the running
// accumulator (last BV result, 8 VGPRs) and 64 Bool bits (2 VGPRs) in
// registers; BV values that must outlive the next instruction go to per-lane
// LDS slots ([slot][half][lane] x 16 B: ds_read_b128 / ds_write_b128,
// conflict-free).  No MFMA: nothing here is a contraction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "../../include/mgp.h"
#include "mgp_bv.h"
#include "mgp_fe_sample.h"

#define MGP_WAVE 64
#define MGP_PARTIAL_NONE 0x7FFFFFFF
#define MGP_PARTIAL_UNDEC (-2)

namespace {

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// compile-time loop: f(std::integral_constant<int, i>) for i = 0..N-1, so that
// per-candidate register arrays are only ever indexed by constants (a runtime
// index would demote them to scratch)
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
  if constexpr (N > 0) {
    static_for<N - 1>(f);
    f(std::integral_constant<int, N - 1>{});
  }
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks dispatched round-robin over the 8 XCDs get
// consecutive logical ids per XCD, so neighbouring states (adjacent bytecode)
// share one L2.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nblk) {
  uint32_t xcd = bid & 7u, q = nblk >> 3, r = nblk & 7u;
  uint32_t base = (xcd < r) ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q;
  return base + (bid >> 3);
}

struct EvalCtx {
  const uint4 *lds;
  const uint32_t *cpool;
  uint4 *cbase;  // this state's candidates, device layout (spill rows are written)
  uint32_t n_cand;
  uint32_t lane;
  uint32_t spill0;  // candidate row of spill slot MGP_LDS_SLOTS (include/mgp_ir.h)
};

__device__ __forceinline__ U256 u256_from(uint4 lo, uint4 hi) {
  U256 v;
  v.w[0] = lo.x; v.w[1] = lo.y; v.w[2] = lo.z; v.w[3] = lo.w;
  v.w[4] = hi.x; v.w[5] = hi.y; v.w[6] = hi.z; v.w[7] = hi.w;
  return v;
}

// LDS slot image: [slot][cpl][half][lane] x 16 B (ds_read_b128, conflict-free)
template <int CPL>
__device__ __forceinline__ U256 fetch(uint32_t o, const U256 &acc, const EvalCtx &e, int c, uint32_t cand) {
  uint32_t kind = o >> 14, idx = o & 0x3FFFu;
  if (kind == MGP_K_ACC) return acc;
  if (kind == MGP_K_SLOT && idx >= MGP_LDS_SLOTS) {  // spill slot: this lane's candidate row
    const uint4 *p = e.cbase + (size_t)(e.spill0 + idx - MGP_LDS_SLOTS) * 2u * e.n_cand + cand;
    return u256_from(p[0], p[e.n_cand]);
  }
  if (kind == MGP_K_SLOT) {
    const uint4 *p = e.lds + ((size_t)idx * CPL + c) * 2u * MGP_WAVE + e.lane;
    return u256_from(p[0], p[MGP_WAVE]);
  }
  if (kind == MGP_K_CONST) {
    const uint32_t *cp = e.cpool + idx * 8u;  // uniform -> s_load_dwordx8
    U256 v;
#pragma unroll
    for (int l = 0; l < 8; ++l) v.w[l] = cp[l];
    return v;
  }
  const uint4 *p = e.cbase + (size_t)idx * 2u * e.n_cand + cand;
  return u256_from(p[0], p[e.n_cand]);
}

template <int CPL>
__device__ __forceinline__ void store_slot(uint4 *lds, uint32_t slot, int c, uint32_t lane, const U256 &v,
                                           const EvalCtx &e, uint32_t cand) {
  if (slot >= MGP_LDS_SLOTS) {  // spill slot: a later fetch by this lane reads the same address
    uint4 *p = e.cbase + (size_t)(e.spill0 + slot - MGP_LDS_SLOTS) * 2u * e.n_cand + cand;
    p[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
    p[e.n_cand] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
    return;
  }
  uint4 *p = lds + ((size_t)slot * CPL + c) * 2u * MGP_WAVE + lane;
  p[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
  p[MGP_WAVE] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
}

__device__ __forceinline__ bool is_bool_op(uint32_t op) { return op >= MGP_OP_BAND && op <= MGP_OP_BEQ; }
__device__ __forceinline__ bool is_cmp_op(uint32_t op) { return op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF; }
__device__ __forceinline__ bool is_signed_op(uint32_t op) {
  return op == MGP_OP_SDIV || op == MGP_OP_SREM || op == MGP_OP_SMOD || op == MGP_OP_ASHR;
}

}  // namespace

// --------------------------------------------------------------- eval
namespace {

__device__ __forceinline__ bool eval_cmp(uint32_t op, const U256 &a, const U256 &b, uint32_t width) {
  switch (op) {
    case MGP_OP_EQ: return bv_eq(a, b);
    case MGP_OP_ULT: return bv_ult(a, b);
    case MGP_OP_ULE: return !bv_ult(b, a);
    case MGP_OP_UGT: return bv_ult(b, a);
    case MGP_OP_UGE: return !bv_ult(a, b);
    case MGP_OP_SLT: return bv_slt(bv_sext(a, width), bv_sext(b, width));
    case MGP_OP_SLE: return !bv_slt(bv_sext(b, width), bv_sext(a, width));
    case MGP_OP_SGT: return bv_slt(bv_sext(b, width), bv_sext(a, width));
    case MGP_OP_SGE: return !bv_slt(bv_sext(a, width), bv_sext(b, width));
    case MGP_OP_UADD_NOOVF: {
      uint32_t carry;
      U256 s = bv_add(a, b, &carry);
      return (width >= 256u) ? (carry == 0u) : bv_eq(s, bv_mask(s, width));
    }
    case MGP_OP_UMUL_NOOVF: {
      U256 lo;
      U256 hi = bv_mul_full(a, b, &lo);
      return bv_is_zero(hi) && bv_eq(lo, bv_mask(lo, width));
    }
    default: return !bv_ult(a, b);  // USUB_NOUDF: b <= a
  }
}

// binary BV ops (a, b already fetched); division ops share one udivrem site
__device__ __forceinline__ U256 eval_bin(uint32_t op, U256 a, U256 b, uint32_t width, uint32_t imm) {
  if (op == MGP_OP_CONCAT) return bv_or(bv_shl(a, imm), b);
  if (is_signed_op(op) && width < 256u) {
    a = bv_sext(a, width);
    if (op != MGP_OP_ASHR) b = bv_sext(b, width);
  }
  if (op >= MGP_OP_UDIV && op <= MGP_OP_SMOD) {
    // SMT-LIB msb case split on |a|, |b|
    const bool sg = op >= MGP_OP_SDIV;
    const bool sa = sg && bv_sign(a), sb = sg && bv_sign(b);
    U256 q, m;
    bv_udivrem(sa ? bv_neg(a) : a, sb ? bv_neg(b) : b, &q, &m);
    if (op == MGP_OP_UDIV) return q;
    if (op == MGP_OP_UREM) return m;
    if (op == MGP_OP_SDIV) return (sa != sb) ? bv_neg(q) : q;
    if (op == MGP_OP_SREM) return sa ? bv_neg(m) : m;
    if (bv_is_zero(m) || (!sa && !sb)) return m;  // SMOD: sign follows the divisor
    if (sa && !sb) return bv_add(bv_neg(m), b, nullptr);
    if (!sa && sb) return bv_add(m, b, nullptr);
    return bv_neg(m);
  }
  switch (op) {
    case MGP_OP_ADD: return bv_add(a, b, nullptr);
    case MGP_OP_SUB: return bv_sub(a, b, nullptr);
    case MGP_OP_MUL: return bv_mul(a, b);
    case MGP_OP_AND: return bv_and(a, b);
    case MGP_OP_OR: return bv_or(a, b);
    case MGP_OP_XOR: return bv_xor(a, b);
    case MGP_OP_SHL: return bv_shl(a, bv_shift_amount(b));
    case MGP_OP_LSHR: return bv_lshr(a, bv_shift_amount(b));
    case MGP_OP_ASHR: return bv_ashr(a, bv_shift_amount(b));
    default: return bv_zero();
  }
}

__device__ __forceinline__ bool is_unary_bv(uint32_t op) {
  return op == MGP_OP_MOV || op == MGP_OP_ZEXT || op == MGP_OP_NOT || op == MGP_OP_NEG ||
         op == MGP_OP_EXTRACT || op == MGP_OP_SEXT;
}

__device__ __forceinline__ U256 eval_unary(uint32_t op, const U256 &a, uint32_t imm) {
  if (op == MGP_OP_NOT) return bv_not(a);
  if (op == MGP_OP_NEG) return bv_neg(a);
  if (op == MGP_OP_EXTRACT) return bv_lshr(a, imm);
  if (op == MGP_OP_SEXT) return bv_sext(a, imm);
  return a;  // MOV / ZEXT: storage is zero-extended, masking below
}

}  // namespace

// CPL = candidates per lane: a wave evaluates 64*CPL candidate models per
// pass over the bytecode, so the scalar decode/dispatch work of every
// instruction is shared by CPL independent 256-bit computations (which the
// scheduler interleaves for ILP).
template <int CPL>
__global__ __launch_bounds__(MGP_WAVE) void mgp_eval_kernel(
    const uint32_t *__restrict__ words, const uint64_t *__restrict__ offs,
    uint32_t n_states, uint4 *__restrict__ cands, uint32_t n_cand,
    uint32_t n_vars, uint32_t n_chunks, uint32_t n_slots,
    int32_t *__restrict__ partial, const uint32_t *__restrict__ order, uint32_t order_base) {
  extern __shared__ uint4 mgp_lds[];
  const uint32_t lid = xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t k = lid / n_chunks, chunk = lid - k * n_chunks;
  // a launch covers states order[order_base + k] (one slot-count bucket) or order_base + k
  const uint32_t state = order ? order[order_base + k] : order_base + k;
  if (state >= n_states) return;
  const uint32_t lane = threadIdx.x;

  const uint32_t *prog = words + offs[state];
  const uint32_t n_ins = uni(prog[0]);
  const uint32_t h_slots = uni(prog[2]);
  const uint32_t h_stat = uni(prog[3]);
  // spill slots live in candidate rows, not LDS: a spilling program needs MGP_LDS_SLOTS
  // slots of LDS and MGP_PROG_VARS rows per candidate
  const uint32_t hw[4] = {n_ins, uni(prog[1]), h_slots, h_stat};
  if ((h_stat & 0xFFu) != MGP_ST_OK || min(h_slots, MGP_LDS_SLOTS) > n_slots || MGP_PROG_VARS(hw) > n_vars) {
    if (lane == 0) partial[(size_t)state * n_chunks + chunk] = MGP_PARTIAL_UNDEC;
    return;
  }
  const uint32_t *ins = prog + MGP_HDR_WORDS;
  EvalCtx e;
  e.lds = mgp_lds;
  e.cpool = ins + (size_t)n_ins * MGP_INS_WORDS;
  e.cbase = cands + (size_t)state * n_vars * 2u * n_cand;
  e.n_cand = n_cand;
  e.lane = lane;
  e.spill0 = MGP_SPILL_BASE(h_stat >> 8);

  uint32_t cand[CPL];
  bool valid[CPL];
  U256 acc[CPL];
  uint64_t bools[CPL];
  bool root[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const uint32_t x = chunk * (MGP_WAVE * CPL) + c * MGP_WAVE + lane;
    valid[c] = x < n_cand;
    cand[c] = valid[c] ? x : n_cand - 1u;
    acc[c] = bv_zero();
    bools[c] = 1ull << MGP_BOOL_TRUE;
    root[c] = false;
  }

  // software-pipelined instruction fetch: the scalar loads of instruction
  // pc+1 are in flight while instruction pc executes (mgp_lower pads every
  // program with one zero instruction after RET)
  uint32_t n0 = uni(ins[0]), n1 = uni(ins[1]), n2 = uni(ins[2]), n3 = uni(ins[3]);
  for (uint32_t pc = 0; pc < n_ins; ++pc) {
    const uint32_t w0 = n0, w1 = n1, w2 = n2, w3 = n3;
    n0 = uni(ins[pc * 4u + 4u]);
    n1 = uni(ins[pc * 4u + 5u]);
    n2 = uni(ins[pc * 4u + 6u]);
    n3 = uni(ins[pc * 4u + 7u]);
    const uint32_t op = w0 & 0xFFu;
    const uint32_t width = ((w0 >> 8) & 0xFFu) + 1u;
    const uint32_t dst = ((w0 >> 16) & 0xFFu) | ((w3 & 0xFFu) << 8);  // BV slots past 255: high bits in w3
    const uint32_t flags = w0 >> 24;
    const uint32_t oa = w1 & 0xFFFFu, ob = w1 >> 16, oc = w2 & 0xFFFFu, imm = w2 >> 16;

    if (op == MGP_OP_RET) {
      static_for<CPL>([&](auto ic) __attribute__((always_inline)) {
        constexpr int c = decltype(ic)::value;
        root[c] = ((bools[c] >> oa) & 1ull) != 0ull;
      });
      break;
    }
    if (is_bool_op(op)) {
      static_for<CPL>([&](auto ic) __attribute__((always_inline)) {
        constexpr int c = decltype(ic)::value;
        const bool a = ((bools[c] >> oa) & 1ull) != 0ull;
        const bool b = ((bools[c] >> ob) & 1ull) != 0ull;
        const bool cc = ((bools[c] >> oc) & 1ull) != 0ull;
        bool r;
        switch (op) {
          case MGP_OP_BAND: r = a && b; break;
          case MGP_OP_BOR: r = a || b; break;
          case MGP_OP_BXOR: r = a != b; break;
          case MGP_OP_BNOT: r = !a; break;
          case MGP_OP_BITE: r = a ? b : cc; break;
          default: r = a == b; break;  // BEQ
        }
        bools[c] = (bools[c] & ~(1ull << dst)) | ((uint64_t)r << dst);
      });
      continue;
    }
    if (is_cmp_op(op)) {
      static_for<CPL>([&](auto ic) __attribute__((always_inline)) {
        constexpr int c = decltype(ic)::value;
        const U256 a = fetch<CPL>(oa, acc[c], e, c, cand[c]);
        const U256 b = fetch<CPL>(ob, acc[c], e, c, cand[c]);
        const bool r = eval_cmp(op, a, b, width);
        bools[c] = (bools[c] & ~(1ull << dst)) | ((uint64_t)r << dst);
      });
      continue;
    }

    // ---- BV-producing instructions
    static_for<CPL>([&](auto ic) __attribute__((always_inline)) {
      constexpr int c = decltype(ic)::value;
      U256 r;
      if (op == MGP_OP_ITE) {
        const bool cond = ((bools[c] >> oa) & 1ull) != 0ull;
        r = bv_sel(cond, fetch<CPL>(ob, acc[c], e, c, cand[c]), fetch<CPL>(oc, acc[c], e, c, cand[c]));
      } else if (op == MGP_OP_EQSEL) {  // select-chain step: (a == b) ? c : acc
        const bool hit = bv_eq(fetch<CPL>(oa, acc[c], e, c, cand[c]), fetch<CPL>(ob, acc[c], e, c, cand[c]));
        r = bv_sel(hit, fetch<CPL>(oc, acc[c], e, c, cand[c]), acc[c]);
      } else if (is_unary_bv(op)) {
        r = eval_unary(op, fetch<CPL>(oa, acc[c], e, c, cand[c]), imm);
      } else {
        r = eval_bin(op, fetch<CPL>(oa, acc[c], e, c, cand[c]), fetch<CPL>(ob, acc[c], e, c, cand[c]), width, imm);
      }
      if (width < 256u) r = bv_mask(r, width);
      acc[c] = r;
      if (flags & MGP_INS_STORE) store_slot<CPL>(mgp_lds, dst, c, lane, r, e, cand[c]);
    });
  }

  int32_t first = MGP_PARTIAL_NONE;
#pragma unroll
  for (int c = CPL - 1; c >= 0; --c) {
    const unsigned long long m = __ballot(valid[c] && root[c]);
    if (m) first = (int32_t)(chunk * (MGP_WAVE * CPL) + c * MGP_WAVE + (uint32_t)__ffsll((long long)m) - 1u);
  }
  if (lane == 0) partial[(size_t)state * n_chunks + chunk] = first;
}

__global__ void mgp_finalize_kernel(const int32_t *__restrict__ partial, uint32_t n_states,
                                    uint32_t n_chunks, const uint4 *__restrict__ cands,
                                    uint32_t n_cand, uint32_t n_vars,
                                    int32_t *__restrict__ first_sat, uint4 *__restrict__ witness) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_states) return;
  int32_t best = MGP_PARTIAL_NONE;
  bool undec = false, bad = false;
  for (uint32_t k = 0; k < n_chunks; ++k) {
    int32_t p = partial[(size_t)s * n_chunks + k];
    if (p == MGP_PARTIAL_UNDEC) undec = true;
    else if (p == MGP_PARTIAL_NONE) continue;
    else if (p < 0 || (uint32_t)p >= n_cand) bad = true;  // a chunk left no valid result
    else if (p < best) best = p;
  }
  int32_t res = bad ? MGP_EVAL_FAULT
                    : undec ? MGP_UNDECIDED : (best == MGP_PARTIAL_NONE ? MGP_NO_SAT : best);
  first_sat[s] = res;
  if (res >= 0 && witness) {
    const uint4 *cb = cands + (size_t)s * n_vars * 2u * n_cand;
    for (uint32_t v = 0; v < n_vars; ++v)
      for (uint32_t h = 0; h < 2u; ++h)
        witness[((size_t)s * n_vars + v) * 2u + h] = cb[(size_t)(v * 2u + h) * n_cand + (uint32_t)res];
  }
}

// --------------------------------------------------------------- Philox
namespace {
__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += 0x9E3779B9u;
    key.y += 0xBB67AE85u;
  }
  return ctr;
}
}  // namespace

// one thread per (state, var, cand); writes both 16-byte halves
__global__ void mgp_fill_kernel(const uint32_t *__restrict__ words, const uint64_t *__restrict__ offs,
                                uint32_t n_states, uint64_t state_base, uint64_t seed,
                                uint4 *__restrict__ cands, uint32_t n_cand, uint32_t n_vars) {
  const uint64_t total = (uint64_t)n_states * n_vars * n_cand;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = (uint32_t)(t % n_cand);
    const uint64_t sv = t / n_cand;
    const uint32_t v = (uint32_t)(sv % n_vars);
    const uint32_t s = (uint32_t)(sv / n_vars);
    const uint64_t gs = state_base + s;
    uint4 r0 = philox4x32_10(make_uint4(c, v, (uint32_t)gs, (uint32_t)(gs >> 32)), key);
    uint4 r1 = philox4x32_10(make_uint4(c, v | (1u << 16), (uint32_t)gs, (uint32_t)(gs >> 32)), key);
    uint4 sel = philox4x32_10(make_uint4(c, v | (2u << 16), (uint32_t)gs, (uint32_t)(gs >> 32)), key);
    uint32_t w[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    if ((sel.x & 3u) == 0u) {  // 25 % interesting values
      const uint32_t kind = sel.y & 15u;
      for (int l = 0; l < 8; ++l) w[l] = 0u;
      if (kind == 1u) {
        w[0] = 1u;
      } else if (kind == 2u) {
        for (int l = 0; l < 8; ++l) w[l] = 0xFFFFFFFFu;
      } else if (kind == 3u) {
        w[7] = 0x80000000u;
      } else if (kind == 4u) {
        for (int l = 0; l < 5; ++l) w[l] = 0xFFFFFFFFu;
      } else if (kind >= 5u && kind <= 7u) {  // ACTORS transaction/symbolic.py:25-27
        const uint32_t pat[3][5] = {
            {0xAFFEAFFEu, 0xAFFEAFFEu, 0xAFFEAFFEu, 0xAFFEAFFEu, 0xAFFEAFFEu},
            {0xDEADBEEFu, 0xDEADBEEFu, 0xDEADBEEFu, 0xDEADBEEFu, 0xDEADBEEFu},
            {0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu, 0xAAAAAAAAu}};
        for (int l = 0; l < 5; ++l) w[l] = pat[kind - 5u][l];
      } else if (kind >= 8u) {  // constant-pool entry + {-1, 0, +1}
        const uint32_t *prog = words + offs[s];
        const uint32_t n_ins = prog[0], n_c = prog[1];
        if (n_c) {
          const uint32_t *cp = prog + MGP_HDR_WORDS + (size_t)n_ins * MGP_INS_WORDS + (sel.z % n_c) * 8u;
          U256 x;
          for (int l = 0; l < 8; ++l) x.w[l] = cp[l];
          const uint32_t d = sel.w % 3u;
          if (d == 0u) x = bv_sub(x, bv_small(1u), nullptr);
          else if (d == 2u) x = bv_add(x, bv_small(1u), nullptr);
          for (int l = 0; l < 8; ++l) w[l] = x.w[l];
        }
      }
    }
    uint4 *dst = cands + ((size_t)s * n_vars + v) * 2u * n_cand + c;
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[n_cand] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

__global__ void mgp_plant_kernel(uint4 *__restrict__ cands, uint32_t n_cand, uint32_t n_vars,
                                 const uint32_t *__restrict__ pstate, const uint32_t *__restrict__ pidx,
                                 const uint4 *__restrict__ pwords, uint32_t n_plant) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = (uint64_t)n_plant * n_vars * 2u;
  if (t >= total) return;
  const uint32_t h = (uint32_t)(t & 1u);
  const uint32_t v = (uint32_t)((t >> 1) % n_vars);
  const uint32_t i = (uint32_t)((t >> 1) / n_vars);
  const uint32_t s = pstate[i], c = pidx[i];
  cands[((size_t)s * n_vars + v) * 2u * n_cand + (size_t)h * n_cand + c] = pwords[((size_t)i * n_vars + v) * 2u + h];
}

// host AoS [state][cand][var][2 x uint4] -> device [state][var][half][cand]
__global__ void mgp_transpose_kernel(const uint4 *__restrict__ aos, uint4 *__restrict__ soa,
                                     uint32_t n_states, uint32_t n_cand, uint32_t n_vars) {
  const uint64_t total = (uint64_t)n_states * n_vars * 2u * n_cand;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = (uint32_t)(t % n_cand);
    uint64_t r = t / n_cand;
    const uint32_t h = (uint32_t)(r & 1u);
    r >>= 1;
    const uint32_t v = (uint32_t)(r % n_vars);
    const uint64_t s = r / n_vars;
    soa[t] = aos[((s * n_cand + c) * n_vars + v) * 2u + h];
  }
}

// --------------------------------------------------------------- Keccak
namespace {
__constant__ uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

// Keccak-f[1600] on 32-bit halves.  A 64-bit lane is (lo, hi); the compiler sees only
// 32-bit operations, so theta's five-way parities become v_xor3_b32 / v_bitop3_b32,
// chi's a ^ (~b & c) one v_bitop3_b32 per word, and every rotation two v_alignbit_b32
// (a 64-bit rotate through lshl_b64 + lshr + or costs four).
template <int R>
__device__ __forceinline__ void rotl64_32(uint32_t lo, uint32_t hi, uint32_t &olo, uint32_t &ohi) {
  if constexpr (R == 0) {
    olo = lo;
    ohi = hi;
  } else if constexpr (R == 32) {
    olo = hi;
    ohi = lo;
  } else if constexpr (R < 32) {
    ohi = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
    olo = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
  } else {
    ohi = __builtin_amdgcn_alignbit(lo, hi, 64 - R);
    olo = __builtin_amdgcn_alignbit(hi, lo, 64 - R);
  }
}

template <int I>
struct KeccakRho;  // FIPS 202 rho offsets, lane (x,y) at index x + 5y
#define MGP_RHO(i, r) \
  template <>        \
  struct KeccakRho<i> { static constexpr int v = r; };
MGP_RHO(0, 0) MGP_RHO(1, 1) MGP_RHO(2, 62) MGP_RHO(3, 28) MGP_RHO(4, 27) MGP_RHO(5, 36) MGP_RHO(6, 44)
MGP_RHO(7, 6) MGP_RHO(8, 55) MGP_RHO(9, 20) MGP_RHO(10, 3) MGP_RHO(11, 10) MGP_RHO(12, 43) MGP_RHO(13, 25)
MGP_RHO(14, 39) MGP_RHO(15, 41) MGP_RHO(16, 45) MGP_RHO(17, 15) MGP_RHO(18, 21) MGP_RHO(19, 8)
MGP_RHO(20, 18) MGP_RHO(21, 2) MGP_RHO(22, 61) MGP_RHO(23, 56) MGP_RHO(24, 14)
#undef MGP_RHO

// one round on K independent states (K = 2: two hashes per lane, interleaved by the
// scheduler; A/B knob MGP_KECCAK_X2)
template <int K>
__device__ __forceinline__ void keccak_round_k(uint32_t (*lo)[25], uint32_t (*hi)[25], int round) {
#pragma unroll
  for (int q = 0; q < K; ++q) {
    uint32_t cl[5], ch[5], dl[5], dh[5], bl[25], bh[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      cl[x] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(lo[q][x], lo[q][x + 5], lo[q][x + 10], 0x96),
                                          lo[q][x + 15], lo[q][x + 20], 0x96);
      ch[x] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(hi[q][x], hi[q][x + 5], hi[q][x + 10], 0x96),
                                          hi[q][x + 15], hi[q][x + 20], 0x96);
    }
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      uint32_t rl, rh;
      rotl64_32<1>(cl[(x + 1) % 5], ch[(x + 1) % 5], rl, rh);
      dl[x] = cl[(x + 4) % 5] ^ rl;
      dh[x] = ch[(x + 4) % 5] ^ rh;
    }
    static_for<25>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int x = i % 5, y = i / 5;
      constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
      rotl64_32<KeccakRho<i>::v>(lo[q][i] ^ dl[x], hi[q][i] ^ dh[x], bl[dst], bh[dst]);
    });
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
      for (int x = 0; x < 5; ++x) {
        lo[q][x + 5 * y] = bl[x + 5 * y] ^ (~bl[(x + 1) % 5 + 5 * y] & bl[(x + 2) % 5 + 5 * y]);
        hi[q][x + 5 * y] = bh[x + 5 * y] ^ (~bh[(x + 1) % 5 + 5 * y] & bh[(x + 2) % 5 + 5 * y]);
      }
    const uint64_t rc = kKeccakRC[round];
    lo[q][0] ^= (uint32_t)rc;
    hi[q][0] ^= (uint32_t)(rc >> 32);
  }
}

template <int K>
__device__ __forceinline__ void keccak_f1600_32k(uint32_t (*lo)[25], uint32_t (*hi)[25]) {
#pragma unroll
  for (int round = 0; round < 24; ++round) keccak_round_k<K>(lo, hi, round);
}

__device__ __forceinline__ void keccak_f1600_32(uint32_t lo[25], uint32_t hi[25]) {
  // fully unrolled: the pi permutation then costs no moves and the round constants
  // become literals
#pragma unroll
  for (int round = 0; round < 24; ++round) {
    uint32_t cl[5], ch[5], dl[5], dh[5], bl[25], bh[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      // three-input XOR = v_bitop3_b32 with truth table 0x96
      cl[x] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(lo[x], lo[x + 5], lo[x + 10], 0x96),
                                          lo[x + 15], lo[x + 20], 0x96);
      ch[x] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(hi[x], hi[x + 5], hi[x + 10], 0x96),
                                          hi[x + 15], hi[x + 20], 0x96);
    }
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      uint32_t rl, rh;
      rotl64_32<1>(cl[(x + 1) % 5], ch[(x + 1) % 5], rl, rh);
      dl[x] = cl[(x + 4) % 5] ^ rl;
      dh[x] = ch[(x + 4) % 5] ^ rh;
    }
    static_for<25>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int x = i % 5, y = i / 5;
      constexpr int dst = y + 5 * ((2 * x + 3 * y) % 5);
      rotl64_32<KeccakRho<i>::v>(lo[i] ^ dl[x], hi[i] ^ dh[x], bl[dst], bh[dst]);
    });
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
      for (int x = 0; x < 5; ++x) {
        lo[x + 5 * y] = bl[x + 5 * y] ^ (~bl[(x + 1) % 5 + 5 * y] & bl[(x + 2) % 5 + 5 * y]);
        hi[x + 5 * y] = bh[x + 5 * y] ^ (~bh[(x + 1) % 5 + 5 * y] & bh[(x + 2) % 5 + 5 * y]);
      }
    const uint64_t rc = kKeccakRC[round];
    lo[0] ^= (uint32_t)rc;
    hi[0] ^= (uint32_t)(rc >> 32);
  }
}

__device__ __forceinline__ void keccak_f1600(uint64_t st[25]) {
  uint32_t lo[25], hi[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) {
    lo[i] = (uint32_t)st[i];
    hi[i] = (uint32_t)(st[i] >> 32);
  }
  keccak_f1600_32(lo, hi);
#pragma unroll
  for (int i = 0; i < 25; ++i) st[i] = ((uint64_t)hi[i] << 32) | lo[i];
}
}  // namespace

// generic path: any len, any stride (byte loads), multi-block absorb
__global__ void mgp_keccak_kernel(const uint8_t *__restrict__ in, uint64_t n, uint32_t len,
                                  uint32_t stride, uint8_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *p = in + i * stride;
  uint64_t st[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) st[k] = 0ull;
  uint32_t off = 0;
  while (len - off >= 136u) {
    for (int k = 0; k < 17; ++k) {
      uint64_t v = 0;
      for (int b = 7; b >= 0; --b) v = (v << 8) | p[off + 8 * k + b];
      st[k] ^= v;
    }
    keccak_f1600(st);
    off += 136u;
  }
  uint8_t blk[136];
  for (int b = 0; b < 136; ++b) blk[b] = 0;
  for (uint32_t b = 0; b < len - off; ++b) blk[b] = p[off + b];
  blk[len - off] ^= 0x01u;
  blk[135] ^= 0x80u;
  for (int k = 0; k < 17; ++k) {
    uint64_t v = 0;
    for (int b = 7; b >= 0; --b) v = (v << 8) | blk[8 * k + b];
    st[k] ^= v;
  }
  keccak_f1600(st);
  uint8_t *o = out + i * 32u;
  for (int k = 0; k < 4; ++k)
    for (int b = 0; b < 8; ++b) o[8 * k + b] = (uint8_t)(st[k] >> (8 * b));
}

// fast path, two hashes per lane (i and i + half): A/B variant (MGP_KECCAK_X2=1)
__global__ __launch_bounds__(256) void mgp_keccak64x2_kernel(const uint4 *__restrict__ in, uint64_t n,
                                                             uint32_t stride16, uint4 *__restrict__ out) {
  const uint64_t half = (n + 1) / 2;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  const uint64_t j = i + half < n ? i + half : i;  // odd n: the last lane hashes i twice
  uint32_t lo[2][25], hi[2][25];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint4 *p = in + (q ? j : i) * stride16;
#pragma unroll
    for (int k = 0; k < 25; ++k) lo[q][k] = hi[q][k] = 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 v = p[c];
      lo[q][2 * c] = v.x; hi[q][2 * c] = v.y; lo[q][2 * c + 1] = v.z; hi[q][2 * c + 1] = v.w;
    }
    lo[q][8] = 0x01u;
    hi[q][16] = 0x80000000u;
  }
  keccak_f1600_32k<2>(lo, hi);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    uint4 *o = out + (q ? j : i) * 2u;
    o[0] = make_uint4(lo[q][0], hi[q][0], lo[q][1], hi[q][1]);
    o[1] = make_uint4(lo[q][2], hi[q][2], lo[q][3], hi[q][3]);
  }
}

// fast path: 64-byte preimages, 16-byte aligned stride (mapping slots)
__global__ __launch_bounds__(256) void mgp_keccak64_kernel(const uint4 *__restrict__ in, uint64_t n,
                                                           uint32_t stride16, uint4 *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *p = in + i * stride16;
  uint64_t st[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) st[k] = 0ull;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint4 v = p[q];
    st[2 * q] = ((uint64_t)v.y << 32) | v.x;
    st[2 * q + 1] = ((uint64_t)v.w << 32) | v.z;
  }
  st[8] = 0x01ull;
  st[16] = 0x8000000000000000ull;
  keccak_f1600(st);
  uint4 *o = out + i * 2u;
  o[0] = make_uint4((uint32_t)st[0], (uint32_t)(st[0] >> 32), (uint32_t)st[1], (uint32_t)(st[1] >> 32));
  o[1] = make_uint4((uint32_t)st[2], (uint32_t)(st[2] >> 32), (uint32_t)st[3], (uint32_t)(st[3] >> 32));
}

// fast path at 8 waves/SIMD (<= 64 VGPRs, the compiler spills a few words): A/B variant (MGP_KECCAK_W8=1)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void mgp_keccak64w8_kernel(const uint4 *__restrict__ in, uint64_t n,
                                                           uint32_t stride16, uint4 *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 *p = in + i * stride16;
  uint64_t st[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) st[k] = 0ull;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint4 v = p[q];
    st[2 * q] = ((uint64_t)v.y << 32) | v.x;
    st[2 * q + 1] = ((uint64_t)v.w << 32) | v.z;
  }
  st[8] = 0x01ull;
  st[16] = 0x8000000000000000ull;
  keccak_f1600(st);
  uint4 *o = out + i * 2u;
  o[0] = make_uint4((uint32_t)st[0], (uint32_t)(st[0] >> 32), (uint32_t)st[1], (uint32_t)(st[1] >> 32));
  o[1] = make_uint4((uint32_t)st[2], (uint32_t)(st[2] >> 32), (uint32_t)st[3], (uint32_t)(st[3] >> 32));
}

namespace {
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
}  // namespace

// preimage i = pad32(addr_i) || pad32((first+i) mod 8), big-endian words
__global__ void mgp_preimage_kernel(uint8_t *__restrict__ out, uint64_t first, uint64_t n, uint64_t seed) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t g = first + i;
  const uint64_t x0 = splitmix64(seed + g), x1 = splitmix64(x0), x2 = splitmix64(x1);
  uint8_t b[64];
  for (int k = 0; k < 64; ++k) b[k] = 0;
  // addr = (x2 & 0xffffffff) << 128 | x1 << 64 | x0, 20 bytes big-endian at [12, 32)
  for (int k = 0; k < 8; ++k) b[31 - k] = (uint8_t)(x0 >> (8 * k));
  for (int k = 0; k < 8; ++k) b[23 - k] = (uint8_t)(x1 >> (8 * k));
  for (int k = 0; k < 4; ++k) b[15 - k] = (uint8_t)(x2 >> (8 * k));
  b[63] = (uint8_t)(g & 7u);
  uint4 *o = reinterpret_cast<uint4 *>(out + i * 64u);
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4];
    for (int j = 0; j < 4; ++j)
      w[j] = (uint32_t)b[16 * q + 4 * j] | ((uint32_t)b[16 * q + 4 * j + 1] << 8) |
             ((uint32_t)b[16 * q + 4 * j + 2] << 16) | ((uint32_t)b[16 * q + 4 * j + 3] << 24);
    o[q] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}


// ------------------------------------------------- front-end candidates
// Device twin of mgp_make_candidates (mgp_cands.cpp): the same splitmix64 stream keyed by
// (seed, state, row, variable), the same row structure (parent witness row, first-hint
// row, hint row with x == y aliases applied, then the 35/25/15/25 mixture) and the same
// final masking, bit for bit (tests/test_gpu_front.py), written straight into the
// device layout [state][var][half][cand] the interpreter reads.  One thread per
// (state, candidate row); the row is built in place (an alias copies the source cell as
// written so far, as on the host) and masked to the slot widths at the end.
namespace {
__device__ __forceinline__ uint64_t fe_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
struct FeRow {
  uint4 *out;
  uint32_t n_cand, n_vars, c;
  uint64_t s;
  __device__ uint4 *at(uint32_t v, uint32_t h) const {
    return out + (((s * n_vars + v) * 2u + h) * (uint64_t)n_cand + c);
  }
  __device__ void put(uint32_t v, const uint32_t *x) const {
    *at(v, 0) = make_uint4(x[0], x[1], x[2], x[3]);
    *at(v, 1) = make_uint4(x[4], x[5], x[6], x[7]);
  }
  __device__ void copy(uint32_t dst, uint32_t src) const {
    const uint4 a = *at(src, 0), b = *at(src, 1);
    *at(dst, 0) = a;
    *at(dst, 1) = b;
  }
};
}  // namespace

// One candidate row (s, c), built by `nl` cooperating lanes (lane = 0..nl-1; nl = 1 is
// one thread per row): every pass that writes only its own variable's cell is strided
// over the lanes, the two alias passes (an alias copies a cell as written so far, in
// variable order) run on lane 0, and SYNC separates the passes when nl > 1.  Same
// values either way.
template <bool BLOCK>
__device__ __forceinline__ void fe_cands_row(
    uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed, const uint64_t *__restrict__ var_off,
    const uint32_t *__restrict__ var_width, const uint8_t *__restrict__ var_kind,
    const uint64_t *__restrict__ hint_off, const uint32_t *__restrict__ hints,
    const uint64_t *__restrict__ alias_off, const uint32_t *__restrict__ aliases,
    const uint64_t *__restrict__ const_off, const uint32_t *__restrict__ consts, const uint32_t *__restrict__ fixed,
    uint32_t n_fixed, const int32_t *__restrict__ parent_idx, const uint32_t *__restrict__ pvals,
    const uint8_t *__restrict__ pmask, const uint32_t *__restrict__ dom, const uint32_t *__restrict__ asrc_off,
    const uint32_t *__restrict__ asrc, const uint32_t *__restrict__ wcls, const uint32_t *__restrict__ wlist,
    const uint64_t *__restrict__ state_keys, const uint32_t *__restrict__ xrows, const uint8_t *__restrict__ xmask,
    uint32_t n_xrows, uint32_t n_xvars, uint4 *__restrict__ out, uint64_t s, uint32_t c, uint32_t lane, uint32_t nl) {
#define SYNC()                      \
  do {                              \
    if constexpr (BLOCK) __syncthreads(); \
  } while (0)
  const uint64_t tag = state_keys ? state_keys[s] : s << 40;  // as mgp_make_candidates
  const FeRow R{out, n_cand, n_vars, c, s};
  uint32_t x[8];
  for (uint32_t v = lane; v < n_vars; v += nl) {  // uniform everywhere first (also padding variables)
    uint64_t k = fe_mix(seed ^ fe_mix(tag ^ ((uint64_t)c << 16) ^ v));
    for (int l = 0; l < 8; l += 2) {
      k = fe_mix(k);
      x[l] = (uint32_t)k;
      x[l + 1] = (uint32_t)(k >> 32);
    }
    R.put(v, x);
  }
  const uint64_t v0 = var_off[s], V = var_off[s + 1] - v0;
  if (V == 0 || V > n_vars) return;
  const uint64_t c0 = const_off[s], nc = const_off[s + 1] - c0;
  const uint64_t n_pool = 3 * nc + n_fixed;
  const uint64_t a0 = alias_off[s], na = alias_off[s + 1] - a0;
  auto n_hint = [&](uint64_t v) { return hint_off[v0 + v + 1] - hint_off[v0 + v]; };
  auto hint = [&](uint64_t v, uint64_t j) { return hints + (hint_off[v0 + v] + j) * 8u; };
  auto pool = [&](uint64_t i, uint32_t *r) {
    if (i >= 3 * nc) {
      for (int l = 0; l < 8; ++l) r[l] = fixed[(i - 3 * nc) * 8u + l];
      return;
    }
    const uint32_t *a = consts + (c0 + i % nc) * 8u;
    const int d = i < nc ? 0 : (i < 2 * nc ? 1 : -1);
    uint64_t carry = d > 0 ? 1u : 0u;
    const uint32_t ext = d < 0 ? 0xFFFFFFFFu : 0u;
    for (int l = 0; l < 8; ++l) {
      if (d == 0) {
        r[l] = a[l];
        continue;
      }
      const uint64_t t = (uint64_t)a[l] + ext + carry;
      r[l] = (uint32_t)t;
      carry = t >> 32;
    }
  };
  const int32_t pidx = parent_idx ? parent_idx[s] : -1;
  const uint32_t first_row = pidx >= 0 ? 1u : 0u;
  SYNC();
  if (pidx >= 0 && c == 0) {  // parent witness row (values of the same variables, by name)
    for (uint64_t v = lane; v < V; v += nl)
      if (pmask[(uint64_t)pidx * n_vars + v]) R.put((uint32_t)v, pvals + ((uint64_t)pidx * n_vars + v) * 8u);
  } else if (c == first_row || c == first_row + 1) {
    for (uint64_t v = lane; v < V; v += nl)
      if (n_hint(v)) R.put((uint32_t)v, hint(v, 0));
    SYNC();
    if (c == first_row + 1 && lane == 0)
      for (uint64_t a = 0; a < na; ++a) {
        const uint32_t dst = aliases[2 * (a0 + a)], src = aliases[2 * (a0 + a) + 1];
        if (dst < V && src < V && var_width[v0 + dst] == var_width[v0 + src] && n_hint(src) && !n_hint(dst))
          R.copy(dst, src);
      }
  } else if (c > first_row + 1) {
    auto draw = [&](uint64_t v, double *r, uint64_t *pick) {
      const uint64_t k = fe_mix(seed ^ 0xA5A5A5A5ull ^ fe_mix(tag ^ ((uint64_t)c << 16) ^ v));
      *r = (double)(k >> 11) * (1.0 / 9007199254740992.0);
      *pick = fe_mix(k);
    };
    for (uint64_t v = lane; v < V; v += nl) {
      double r;
      uint64_t pick;
      draw(v, &r, &pick);
      if (r < 0.35 && n_hint(v)) {
        R.put((uint32_t)v, hint(v, pick % n_hint(v)));
      } else if (r < 0.60 && n_pool) {
        pool(pick % n_pool, x);
        R.put((uint32_t)v, x);
      }
    }
    SYNC();
    for (uint64_t v = 0; v < V && lane == 0; ++v) {  // after the others, so an alias can copy any variable
      double r;
      uint64_t pick;
      draw(v, &r, &pick);
      const bool pend = !(r < 0.35 && n_hint(v)) && !(r < 0.60 && n_pool) && r < 0.75;
      if (!pend) continue;
      // x == y alias sources of v in alias order, and the equal-width variables in index
      // order, from the host's per-variable tables (mgp_fe_alias_tables): O(log V) per
      // variable instead of the host generator's scans, same choice
      const uint32_t *srcs = asrc + asrc_off[v0 + v];
      const uint32_t n_src = asrc_off[v0 + v + 1] - asrc_off[v0 + v];
      const uint64_t k = fe_mix(seed ^ 0x5A5A5A5Aull ^ fe_mix(tag ^ ((uint64_t)c << 16) ^ v));
      if (n_src) {
        R.copy((uint32_t)v, srcs[k % n_src]);
        continue;
      }
      // the next equal-width variable from a random start: the first u != v at or after
      // st0 (circularly) in the sorted list of v's width class
      const uint32_t *L = wlist + wcls[2 * (v0 + v)];
      const uint32_t len = wcls[2 * (v0 + v) + 1];
      const uint32_t st0 = (uint32_t)(k % V);
      uint32_t lo = 0, hi = len;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (L[mid] < st0) lo = mid + 1;
        else hi = mid;
      }
      for (uint32_t t = 0; t < 2 && t < len; ++t) {
        const uint32_t u = L[(lo + t) % len];
        if (u != v) {
          R.copy((uint32_t)v, u);
          break;
        }
      }
    }
    SYNC();
    const uint32_t kk = c - (first_row + 2u);  // domain rows: as mgp_make_candidates
    if (dom && (kk & 1u) == 0u)
      for (uint64_t v = lane; v < V; v += nl) {
        const uint32_t *d = dom + (v0 + v) * 33u;
        if (!d[32]) continue;
        U256 z, o, lo, hi;
        for (int l = 0; l < 8; ++l) {
          z.w[l] = d[l];
          o.w[l] = d[8 + l];
          lo.w[l] = d[16 + l];
          hi.w[l] = d[24 + l];
        }
        const uint64_t key = fe_mix64(seed ^ 0xD0D0D0D0ull ^ fe_mix64(tag ^ ((uint64_t)c << 16) ^ v));
        U256 xv = fe_sample_domain(z, o, lo, hi, var_width[v0 + v], kk / 2u, key);
        if (n_hint(v) && (fe_mix64(key ^ 0x9E37ull) & 1u)) {
          const uint32_t *hp = hint(v, fe_mix64(key ^ 0x7F4Aull) % n_hint(v));
          U256 h;
          for (int l = 0; l < 8; ++l) h.w[l] = hp[l];
          h = bv_mask(h, var_width[v0 + v]);
          if (fe_inside(z, o, lo, hi, h)) xv = h;
        }
        R.put((uint32_t)v, xv.w);
      }
    // explicit rows (host or device decision rows, mgp_decision_rows): the first n_xrows
    // mixture rows take the given values of the slots their mask marks
    if (xrows && kk < n_xrows) {
      const uint64_t r0 = (s * n_xrows + kk) * (uint64_t)n_xvars;
      for (uint64_t v = lane; v < V && v < n_xvars; v += nl)
        if (xmask[r0 + v]) R.put((uint32_t)v, xrows + (r0 + v) * 8u);
    }
  }
  SYNC();
  for (uint64_t v = lane; v < V; v += nl)  // pinned constants
    if (var_kind && var_kind[v0 + v] == 2 && n_hint(v)) R.put((uint32_t)v, hint(v, 0));
  SYNC();
  // the mask to the slot width, 8 variables per round trip: their 16 loads are
  // independent, so a small batch (a few waves on the chip) pays one load latency per
  // 8 variables instead of one per 16 bytes
  constexpr uint32_t kB = 8;
  for (uint64_t vb = (uint64_t)lane * kB; vb < V; vb += (uint64_t)nl * kB) {
    uint4 q[kB][2];
    uint32_t w[kB];
    const uint32_t nb = (uint32_t)((V - vb) < kB ? (V - vb) : kB);
#pragma unroll
    for (uint32_t j = 0; j < kB; ++j) {
      w[j] = j < nb ? var_width[v0 + vb + j] : 256u;
      if (w[j] < 256u) {
        q[j][0] = *R.at((uint32_t)(vb + j), 0);
        q[j][1] = *R.at((uint32_t)(vb + j), 1);
      }
    }
#pragma unroll
    for (uint32_t j = 0; j < kB; ++j) {
      if (w[j] >= 256u) continue;
      for (uint32_t h = 0; h < 2; ++h) {
        uint32_t *e = reinterpret_cast<uint32_t *>(&q[j][h]);
        for (int l = 0; l < 4; ++l) {
          const int lo = 32 * (4 * (int)h + l);
          e[l] &= (int)w[j] >= lo + 32 ? 0xFFFFFFFFu : ((int)w[j] <= lo ? 0u : ((1u << (w[j] - lo)) - 1u));
        }
        *R.at((uint32_t)(vb + j), h) = q[j][h];
      }
    }
  }
}

#undef SYNC

__global__ __launch_bounds__(256) void mgp_fe_cands_kernel(
    uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed, const uint64_t *__restrict__ var_off,
    const uint32_t *__restrict__ var_width, const uint8_t *__restrict__ var_kind,
    const uint64_t *__restrict__ hint_off, const uint32_t *__restrict__ hints,
    const uint64_t *__restrict__ alias_off, const uint32_t *__restrict__ aliases,
    const uint64_t *__restrict__ const_off, const uint32_t *__restrict__ consts, const uint32_t *__restrict__ fixed,
    uint32_t n_fixed, const int32_t *__restrict__ parent_idx, const uint32_t *__restrict__ pvals,
    const uint8_t *__restrict__ pmask, const uint32_t *__restrict__ dom, const uint32_t *__restrict__ asrc_off,
    const uint32_t *__restrict__ asrc, const uint32_t *__restrict__ wcls, const uint32_t *__restrict__ wlist,
    const uint64_t *__restrict__ state_keys, const uint32_t *__restrict__ xrows, const uint8_t *__restrict__ xmask,
    uint32_t n_xrows, uint32_t n_xvars, uint4 *__restrict__ out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (uint64_t)n_states * n_cand) return;
  fe_cands_row<false>(n_states, n_cand, n_vars, seed, var_off, var_width, var_kind, hint_off, hints, alias_off, aliases, const_off, consts, fixed, n_fixed, parent_idx, pvals, pmask, dom, asrc_off, asrc, wcls, wlist, state_keys, xrows, xmask, n_xrows, n_xvars, out, g / n_cand, (uint32_t)(g % n_cand), 0u, 1u);
}

// one 64-lane workgroup per row: a small batch of contract states (hundreds of variables
// per row, a few waves on the whole chip) builds a row in a few variable-steps per lane
// instead of one long sequential pass per thread
__global__ __launch_bounds__(64) void mgp_fe_cands_rowblock_kernel(
    uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed, const uint64_t *__restrict__ var_off,
    const uint32_t *__restrict__ var_width, const uint8_t *__restrict__ var_kind,
    const uint64_t *__restrict__ hint_off, const uint32_t *__restrict__ hints,
    const uint64_t *__restrict__ alias_off, const uint32_t *__restrict__ aliases,
    const uint64_t *__restrict__ const_off, const uint32_t *__restrict__ consts, const uint32_t *__restrict__ fixed,
    uint32_t n_fixed, const int32_t *__restrict__ parent_idx, const uint32_t *__restrict__ pvals,
    const uint8_t *__restrict__ pmask, const uint32_t *__restrict__ dom, const uint32_t *__restrict__ asrc_off,
    const uint32_t *__restrict__ asrc, const uint32_t *__restrict__ wcls, const uint32_t *__restrict__ wlist,
    const uint64_t *__restrict__ state_keys, const uint32_t *__restrict__ xrows, const uint8_t *__restrict__ xmask,
    uint32_t n_xrows, uint32_t n_xvars, uint4 *__restrict__ out) {
  const uint64_t g = blockIdx.x;
  if (g >= (uint64_t)n_states * n_cand) return;
  fe_cands_row<true>(n_states, n_cand, n_vars, seed, var_off, var_width, var_kind, hint_off, hints, alias_off, aliases, const_off, consts, fixed, n_fixed, parent_idx, pvals, pmask, dom, asrc_off, asrc, wcls, wlist, state_keys, xrows, xmask, n_xrows, n_xvars, out, g / n_cand, (uint32_t)(g % n_cand), threadIdx.x, blockDim.x);
}

// ------------------------------------------------------ VALU peak probe
// 8 independent v_add_u32 chains, 64 adds per chain per iteration, written as
// inline asm so nothing is folded: measures the INT32 VALU issue rate the
// roofline fraction is priced against ("confirm with a
// v_add_u32 microbenchmark").
__global__ __launch_bounds__(256) void mgp_valu_probe_kernel(uint32_t iters, uint32_t *__restrict__ sink) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  const uint32_t b = blockIdx.x | 1u;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      asm volatile(
          "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
          "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(b));
    }
  }
  const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0xFFFFFFFFu) sink[blockIdx.x] = r;  // keep the chains live
}

// ------------------------------------------------------------ launchers
template <int CPL>
static hipError_t launch_eval_cpl(const uint32_t *words, const uint64_t *offs, uint32_t n_states,
                                  const uint32_t *cands, uint32_t n_cand, uint32_t n_vars, uint32_t n_slots,
                                  int32_t *partial, const uint32_t *order, const uint32_t *bucket_bounds,
                                  const uint32_t *bucket_slots, uint32_t n_buckets, uint32_t n_chunks,
                                  hipStream_t st) {
  // One launch per slot-count bucket: the dynamic LDS (slots x CPL x 2 KiB
  // per 64-lane wave) is sized per bucket, so states with few live values run
  // at the occupancy their LDS footprint allows instead of the batch maximum.
  const bool bucketed = n_buckets && order && bucket_bounds && bucket_slots;
  const uint32_t nb = bucketed ? n_buckets : 1u;
  for (uint32_t bkt = 0; bkt < nb; ++bkt) {
    const uint32_t lo = bucketed ? bucket_bounds[bkt] : 0u;
    const uint32_t hi = bucketed ? bucket_bounds[bkt + 1] : n_states;
    // spill slots (>= MGP_LDS_SLOTS) take no LDS
    const uint32_t sl = std::min<uint32_t>(bucketed ? bucket_slots[bkt] : n_slots, MGP_LDS_SLOTS);
    if (hi <= lo) continue;
    const uint64_t nblk = (uint64_t)(hi - lo) * n_chunks;
    const size_t lds = (size_t)(sl ? sl : 1u) * CPL * 2u * MGP_WAVE * sizeof(uint4);
    hipLaunchKernelGGL(mgp_eval_kernel<CPL>, dim3((uint32_t)nblk), dim3(MGP_WAVE), lds, st, words, offs, n_states,
                       reinterpret_cast<uint4 *>(const_cast<uint32_t *>(cands)), n_cand, n_vars, n_chunks, sl,
                       partial,
                       bucketed ? order : nullptr, lo);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

// candidates per lane: 2 when a state has enough candidates to fill 128
// lanes; MGP_CPL=1|2 in the environment forces a value (A/B measurements)
static uint32_t cpl_override() {
  static const uint32_t v = [] {
    const char *e = getenv("MGP_CPL");
    return (e && (e[0] == '1' || e[0] == '2') && e[1] == 0) ? (uint32_t)(e[0] - '0') : 0u;
  }();
  return v;
}

// Launch descriptors of the gfx950 interpreter, one per position p of the launch
// order (order[p], or p): everything its prologue needs from the program headers, so
// that a wave reaches its page / pool / variable loads after one dependent load
// instead of four (offs -> v1 header -> uop header).  32 B each:
//   {state, undecided, slots, n_uops}  {page0 address lo, hi, pool offset from page 0,
//    n_pool | register-variable mask << 8}
__global__ void mgp_desc_kernel(const uint32_t *__restrict__ words, const uint64_t *__restrict__ offs,
                                uint32_t n_states, const uint32_t *__restrict__ order, uint32_t n_vars,
                                uint4 *__restrict__ desc) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_states) return;
  const uint32_t state = order ? order[p] : p;
  const uint32_t *w = words + offs[state];
  const uint4 h = make_uint4(w[0], w[1], w[2], w[3]);
  uint32_t undec = 1u, n_uops = 0u, pool_rel = 0u, npm = 0u;
  uint64_t page = 0u;
  if ((h.w & 0xFFu) == MGP_ST_OK && MGP_PROG_VARS(w) <= n_vars) {
    const uint32_t v1 = 4u + 4u * h.x + 8u * h.y;
    const uint32_t *u = w + ((v1 + 3u) & ~3u) + 4u;
    const uint4 uh = make_uint4(u[0], u[1], u[2], u[3]);
    n_uops = uh.x;
    npm = uh.w;
    undec = (uh.y == 0u && n_uops > 0u) ? 0u : 1u;
    page = reinterpret_cast<uint64_t>(u + 4);
    pool_rel = uh.z - 16u;
  }
  // slots: the LDS slots the interpreter allocates for the state (uop header word 3
  // bits 16..23: the v1 slot count minus the register slots)
  const uint32_t lds_slots = undec ? h.z : (npm >> 16) & 0xFFu;
  desc[2 * (size_t)p] = make_uint4(state, undec, lds_slots, n_uops);
  desc[2 * (size_t)p + 1] = make_uint4((uint32_t)page, (uint32_t)(page >> 32), pool_rel, npm);
}

extern "C" hipError_t mgp_asm_available(void);
extern "C" hipError_t mgp_launch_eval_asm(const void *desc, uint32_t n_states, const uint32_t *cands,
                                          uint32_t n_cand, uint32_t n_vars, uint32_t n_slots, int32_t *partial,
                                          const uint32_t *bucket_bounds, const uint32_t *bucket_slots,
                                          uint32_t n_buckets, uint32_t n_chunks, hipStream_t st);

// Launch-descriptor buffers, one per (device, stream), grow-only.  Kernels of one stream
// run in order, so a stream's buffer is free again for its next launch; growing it waits
// for the stream first (the old buffer may still be read by enqueued kernels).  Not
// stream-ordered allocation (hipMallocAsync / hipFreeAsync): a descriptor buffer must stay
// mapped until the interpreter launches that read it have finished.
//
// MGP_DESC_MODE (fault triage of DESIGN.md §4 "Launch descriptors"; never set in
// measurements): "exact" = a buffer of exactly n_states x 32 B per launch, freed after a
// stream synchronise (no floor, no slack: an out-of-bounds descriptor read faults);
// "async" = hipMallocAsync / hipFreeAsync of exactly that size on the launch stream
// (the round-1 variant whose lifetime was suspected).  Unset: the grow-only buffer.
static int desc_mode() {
  static const int v = [] {
    const char *e = getenv("MGP_DESC_MODE");
    if (!e) return 0;
    return e[0] == 'e' ? 1 : (e[0] == 'a' ? 2 : 0);
  }();
  return v;
}

static std::mutex g_desc_mu;
static std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> g_desc_bufs;

// A context's stream is about to be destroyed (mgp_destroy): free its descriptor buffer
// (the stream has been synchronised, so no launch still reads it).
extern "C" void mgp_desc_release(int dev, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_desc_mu);
  auto it = g_desc_bufs.find({dev, st});
  if (it == g_desc_bufs.end()) return;
  if (it->second.first) (void)hipFree(it->second.first);
  g_desc_bufs.erase(it);
}

static hipError_t desc_buffer(hipStream_t st, size_t bytes, void **out) {
  if (desc_mode() == 1) return hipMalloc(out, bytes);
  if (desc_mode() == 2) return hipMallocAsync(out, bytes, st);
  std::mutex &mu = g_desc_mu;
  auto &bufs = g_desc_bufs;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  auto &b = bufs[{dev, st}];
  if (b.second < bytes) {
    if (b.first) {
      e = hipStreamSynchronize(st);
      if (e != hipSuccess) return e;
      (void)hipFree(b.first);
      b = {nullptr, 0};
    }
    size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
    e = hipMalloc(&b.first, cap);
    if (e != hipSuccess) return e;
    b.second = cap;
  }
  *out = b.first;
  return hipSuccess;
}

// MGP_SYNC_DEBUG=1: synchronise after every launch of the evaluation path and name the
// kernel that failed (fault triage; never set in measurements)
static bool sync_debug() {
  static const bool v = getenv("MGP_SYNC_DEBUG") != nullptr;
  return v;
}

// Evaluation engine: MGP_ENGINE_ASM = the hand-written gfx950 interpreter
// (mgp_eval_gfx950, default), MGP_ENGINE_HIP = the HIP C++ interpreter above
// (kept as an independent second implementation; A/B and cross-checks).
// MGP_ENGINE=hip|asm in the environment sets the initial choice.
static thread_local void *g_last_desc = nullptr;  // the triage modes' per-launch buffer

static int g_engine = [] {
  const char *e = getenv("MGP_ENGINE");
  return (e && e[0] == 'h') ? MGP_ENGINE_HIP : MGP_ENGINE_ASM;
}();

extern "C" {

int mgp_set_eval_engine(int engine) {
  if (engine == MGP_ENGINE_HIP || engine == MGP_ENGINE_ASM) g_engine = engine;
  return g_engine;
}

hipError_t mgp_launch_eval(const uint32_t *words, const uint64_t *offs, uint32_t n_states,
                           const uint32_t *cands, uint32_t n_cand, uint32_t n_vars, uint32_t n_slots,
                           int32_t *first_sat, uint32_t *witness, int32_t *partial, const uint32_t *order,
                           const uint32_t *bucket_bounds, const uint32_t *bucket_slots, uint32_t n_buckets,
                           hipStream_t st) {
  if (n_states == 0) return hipSuccess;
  uint32_t n_chunks;
  hipError_t err;
  if (g_engine == MGP_ENGINE_ASM) {
    n_chunks = (n_cand + MGP_WAVE - 1) / MGP_WAVE;
    const bool bucketed = n_buckets && order && bucket_bounds && bucket_slots;
    void *desc = nullptr;
    err = desc_buffer(st, (size_t)n_states * 32u, &desc);
    if (err != hipSuccess) return err;
    g_last_desc = desc;
    hipLaunchKernelGGL(mgp_desc_kernel, dim3((n_states + 255) / 256), dim3(256), 0, st, words, offs, n_states,
                       bucketed ? order : nullptr, n_vars, reinterpret_cast<uint4 *>(desc));
    err = hipGetLastError();
    if (err == hipSuccess && sync_debug()) {
      err = hipStreamSynchronize(st);
      if (err != hipSuccess) fprintf(stderr, "[mgp] mgp_desc_kernel failed: %s\n", hipGetErrorString(err));
    }
    if (err == hipSuccess)
      err = mgp_launch_eval_asm(desc, n_states, cands, n_cand, n_vars, n_slots, partial,
                                bucketed ? bucket_bounds : nullptr, bucketed ? bucket_slots : nullptr,
                                bucketed ? n_buckets : 0u, n_chunks, st);

  } else {
    const uint32_t cpl = cpl_override() ? cpl_override() : 1u;  // CPL=2 measured slower (LDS occupancy halves)
    n_chunks = (n_cand + MGP_WAVE * cpl - 1) / (MGP_WAVE * cpl);
    err = (cpl == 2u) ? launch_eval_cpl<2>(words, offs, n_states, cands, n_cand, n_vars, n_slots, partial, order,
                                           bucket_bounds, bucket_slots, n_buckets, n_chunks, st)
                      : launch_eval_cpl<1>(words, offs, n_states, cands, n_cand, n_vars, n_slots, partial, order,
                                           bucket_bounds, bucket_slots, n_buckets, n_chunks, st);
  }
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(mgp_finalize_kernel, dim3((n_states + 255) / 256), dim3(256), 0, st, partial,
                     n_states, n_chunks, reinterpret_cast<const uint4 *>(cands), n_cand, n_vars,
                     first_sat, reinterpret_cast<uint4 *>(witness));
  err = hipGetLastError();
  if (g_engine == MGP_ENGINE_ASM && desc_mode() && g_last_desc) {  // triage modes: release the exact buffer
    const hipError_t fe = desc_mode() == 1 ? hipStreamSynchronize(st) : hipSuccess;
    if (fe == hipSuccess) (void)(desc_mode() == 1 ? hipFree(g_last_desc) : hipFreeAsync(g_last_desc, st));
    g_last_desc = nullptr;
    if (err == hipSuccess) err = fe;
  }
  if (err == hipSuccess && sync_debug()) {
    err = hipStreamSynchronize(st);
    if (err != hipSuccess) fprintf(stderr, "[mgp] mgp_finalize_kernel failed: %s\n", hipGetErrorString(err));
  }
  return err;
}

hipError_t mgp_launch_fill(const uint32_t *words, const uint64_t *offs, uint32_t n_states,
                           uint64_t state_base, uint64_t seed, uint32_t *cands, uint32_t n_cand,
                           uint32_t n_vars, hipStream_t st) {
  const uint64_t total = (uint64_t)n_states * n_vars * n_cand;
  if (total == 0) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 65536ull * 16) blocks = 65536ull * 16;
  hipLaunchKernelGGL(mgp_fill_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, words, offs, n_states,
                     state_base, seed, reinterpret_cast<uint4 *>(cands), n_cand, n_vars);
  return hipGetLastError();
}

hipError_t mgp_launch_plant(uint32_t *cands, uint32_t n_cand, uint32_t n_vars, const uint32_t *pstate,
                            const uint32_t *pidx, const uint32_t *pwords, uint32_t n_plant, hipStream_t st) {
  const uint64_t total = (uint64_t)n_plant * n_vars * 2u;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(mgp_plant_kernel, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<uint4 *>(cands), n_cand, n_vars, pstate, pidx,
                     reinterpret_cast<const uint4 *>(pwords), n_plant);
  return hipGetLastError();
}

hipError_t mgp_launch_transpose(const uint32_t *aos, uint32_t *soa, uint32_t n_states, uint32_t n_cand,
                                uint32_t n_vars, hipStream_t st) {
  const uint64_t total = (uint64_t)n_states * n_vars * 2u * n_cand;
  if (total == 0) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 65536ull * 16) blocks = 65536ull * 16;
  hipLaunchKernelGGL(mgp_transpose_kernel, dim3((uint32_t)blocks), dim3(256), 0, st,
                     reinterpret_cast<const uint4 *>(aos), reinterpret_cast<uint4 *>(soa), n_states,
                     n_cand, n_vars);
  return hipGetLastError();
}

static int g_keccak_engine = [] {
  const char *e = getenv("MGP_KECCAK_ENGINE");
  return !e ? MGP_ENGINE_ASM : e[0] == 'h' ? MGP_ENGINE_HIP : strcmp(e, "asm_dx") == 0 ? MGP_ENGINE_ASM_DX
                                                                                        : MGP_ENGINE_ASM;
}();

extern "C" int mgp_set_keccak_engine(int engine) {
  if (engine == MGP_ENGINE_HIP || engine == MGP_ENGINE_ASM || engine == MGP_ENGINE_ASM_DX) g_keccak_engine = engine;
  return g_keccak_engine;
}

extern "C" hipError_t mgp_launch_keccak64_asm(const void *in, uint64_t n, uint32_t stride16, void *out,
                                              int variant, hipStream_t st);

hipError_t mgp_launch_keccak(const uint8_t *in, uint64_t n, uint32_t len, uint32_t stride, uint8_t *out,
                             hipStream_t st) {
  if (n == 0) return hipSuccess;
  const bool fast = len == 64u && (stride % 16u) == 0u && ((uintptr_t)in % 16u) == 0u &&
                    ((uintptr_t)out % 16u) == 0u;
  const uint64_t blocks = (n + 255) / 256;
  if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
  static const bool x2 = [] {
    const char *e = getenv("MGP_KECCAK_X2");
    return e && e[0] == '1';
  }();
  static const bool w8 = [] {
    const char *e = getenv("MGP_KECCAK_W8");
    return e && e[0] == '1';
  }();
  // the hand-allocated kernel (gen_keccak_asm.py) unless the compiler-allocated one is
  // selected (mgp_set_keccak_engine / MGP_KECCAK_ENGINE=hip, A/B)
  if (fast && g_keccak_engine != MGP_ENGINE_HIP && !w8 && !x2 && n < (1ull << 32))
    return mgp_launch_keccak64_asm(in, n, stride / 16u, out, g_keccak_engine == MGP_ENGINE_ASM_DX ? 1 : 0, st);
  if (fast && w8) {
    hipLaunchKernelGGL(mgp_keccak64w8_kernel, dim3((uint32_t)blocks), dim3(256), 0, st,
                       reinterpret_cast<const uint4 *>(in), n, stride / 16u, reinterpret_cast<uint4 *>(out));
  } else if (fast && x2) {
    hipLaunchKernelGGL(mgp_keccak64x2_kernel, dim3((uint32_t)((n + 1) / 2 + 255) / 256), dim3(256), 0, st,
                       reinterpret_cast<const uint4 *>(in), n, stride / 16u, reinterpret_cast<uint4 *>(out));
  } else if (fast) {
    hipLaunchKernelGGL(mgp_keccak64_kernel, dim3((uint32_t)blocks), dim3(256), 0, st,
                       reinterpret_cast<const uint4 *>(in), n, stride / 16u, reinterpret_cast<uint4 *>(out));
  } else {
    hipLaunchKernelGGL(mgp_keccak_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, in, n, len, stride, out);
  }
  return hipGetLastError();
}

hipError_t mgp_launch_preimages(uint8_t *out, uint64_t first, uint64_t n, uint64_t seed, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(mgp_preimage_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, out, first, n,
                     seed);
  return hipGetLastError();
}

hipError_t mgp_launch_fe_cands(uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                               const uint64_t *var_off, const uint32_t *var_width, const uint8_t *var_kind,
                               const uint64_t *hint_off,
                               const uint32_t *hints, const uint64_t *alias_off, const uint32_t *aliases,
                               const uint64_t *const_off, const uint32_t *consts, const uint32_t *fixed,
                               uint32_t n_fixed, const int32_t *parent_idx, const uint32_t *pvals,
                               const uint8_t *pmask, const uint32_t *dom, const uint32_t *asrc_off,
                               const uint32_t *asrc, const uint32_t *wcls, const uint32_t *wlist,
                               const uint64_t *state_keys, const uint32_t *xrows, const uint8_t *xmask,
                               uint32_t n_xrows, uint32_t n_xvars, uint32_t *out, hipStream_t st) {
  const uint64_t total = (uint64_t)n_states * n_cand;
  if (total == 0) return hipSuccess;
  // few rows of many variables (LASER's 2-successor forks of contract states): a
  // workgroup per row; otherwise a thread per row (MGP_FE_ROWBLOCK=0/1 forces one, A/B)
  static const int rb_env = [] {
    const char *e = getenv("MGP_FE_ROWBLOCK");
    return e ? atoi(e) : -1;
  }();
  const bool rowblock = rb_env >= 0 ? rb_env != 0 : (total <= 16384u && n_vars >= 32u);
  if (rowblock) {
    hipLaunchKernelGGL(mgp_fe_cands_rowblock_kernel, dim3((uint32_t)total), dim3(64), 0, st, n_states, n_cand,
                       n_vars, seed, var_off, var_width, var_kind, hint_off, hints, alias_off, aliases, const_off,
                       consts, fixed, n_fixed, parent_idx, pvals, pmask, dom, asrc_off, asrc, wcls, wlist,
                       state_keys, xrows, xmask, n_xrows, n_xvars, reinterpret_cast<uint4 *>(out));
    return hipGetLastError();
  }
  const uint64_t blocks = (total + 255) / 256;
  if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mgp_fe_cands_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, n_states, n_cand, n_vars, seed,
                     var_off, var_width, var_kind, hint_off, hints, alias_off, aliases, const_off, consts, fixed, n_fixed,
                     parent_idx, pvals, pmask, dom, asrc_off, asrc, wcls, wlist, state_keys, xrows, xmask, n_xrows,
                     n_xvars, reinterpret_cast<uint4 *>(out));
  return hipGetLastError();
}

hipError_t mgp_launch_valu_probe(uint32_t iters, uint32_t blocks, uint32_t *sink, hipStream_t st) {
  hipLaunchKernelGGL(mgp_valu_probe_kernel, dim3(blocks), dim3(256), 0, st, iters, sink);
  return hipGetLastError();
}

}  // extern "C"
