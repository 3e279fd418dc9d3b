// mgp_decide.hip — decision rows on the GPU (the second witness round's hardest rows).
//
// A decision row fixes a state's variables one at a time, each drawn from its current
// abstract value, and re-propagates the known-bits x interval analysis after every
// choice (mgp_domain.h decision_row; DESIGN.md §4 "Domain-guided second witness round").
// The host restatement is mgp_refute.cpp's mgp_decision_rows; this kernel runs the SAME
// code (mgp_domain.h, compiled for gfx950), so its rows are bit-identical to the host's
// by construction (tests/test_gpu_decide.py checks it on the corpus).
//
// Execution model: one workgroup (one wave) per (state, row) task.  The 64 lanes copy
// the task's mutable arrays (node values, truth sets, variable values, pair orderings)
// from the state's base analysis into the task's workspace with 16-B loads, then lane 0
// runs the row: the propagation is a sequential work list over the DAG, so a task is
// latency-bound and the chip's parallelism is the tasks (hundreds to thousands per
// batch).  The base analyses, the DAGs and the propagation graphs are one read-only blob
// per batch (mgp_refute.cpp serialises them); workspaces and rows are written by vector
// stores only.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mgp_decide.h"
#include "mgp_domain.h"

using namespace mgpd;

namespace {

template <typename T>
__device__ __forceinline__ const T *at(const uint8_t *blob, uint64_t off) {
  return reinterpret_cast<const T *>(blob + off);
}

// 64 lanes copy `bytes` (a multiple of 16) from src to dst
__device__ __forceinline__ void copy16(void *dst, const void *src, uint64_t bytes) {
  const uint4 *s = reinterpret_cast<const uint4 *>(src);
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  for (uint64_t i = threadIdx.x; i < bytes / 16u; i += blockDim.x) d[i] = s[i];
}

struct RowPut {
  uint32_t *rows;
  uint8_t *mask;
  uint64_t base;  // (state * n_decide + row) * n_vars
  __device__ void operator()(uint32_t sl, const V &v) const {
    uint4 *o = reinterpret_cast<uint4 *>(rows + (base + sl) * 8u);
    o[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
    o[1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
    mask[base + sl] = 1u;
  }
};

__global__ __launch_bounds__(64) void mgp_decide_kernel(const uint8_t *__restrict__ blob,
                                                        const mgp_dec_state *__restrict__ states,
                                                        const mgp_dec_task *__restrict__ tasks, uint32_t n_tasks,
                                                        uint8_t *__restrict__ ws, uint64_t seed, uint32_t or_rows,
                                                        const uint32_t *__restrict__ seed_vals,
                                                        const uint8_t *__restrict__ seed_mask, uint32_t seed_rows,
                                                        uint32_t *__restrict__ out_rows,
                                                        uint8_t *__restrict__ out_mask) {
  const uint32_t t = blockIdx.x;
  if (t >= n_tasks) return;
  const mgp_dec_task T = tasks[t];
  const mgp_dec_state S = states[T.state];
  uint8_t *w = ws + T.ws;
  AV *av = reinterpret_cast<AV *>(w + S.ws_av);
  AV *vars = reinterpret_cast<AV *>(w + S.ws_vars);
  Pair *pairs = reinterpret_cast<Pair *>(w + S.ws_pairs);
  uint8_t *bs = w + S.ws_bs;
  copy16(av, blob + S.av, (uint64_t)S.n * sizeof(AV));
  copy16(vars, blob + S.vars, (uint64_t)S.n_vt * sizeof(AV));
  copy16(pairs, blob + S.pairs, ((uint64_t)S.n_pairs * sizeof(Pair) + 15u) / 16u * 16u);
  copy16(bs, blob + S.bs, ((uint64_t)S.n + 15u) / 16u * 16u);
  __syncthreads();
  if (threadIdx.x != 0) return;
  Stack<UndoRec> undo;
  undo.p = reinterpret_cast<UndoRec *>(w + S.ws_undo);
  undo.cap = S.ucap;
  Stack<uint32_t> work;
  work.p = reinterpret_cast<uint32_t *>(w + S.ws_work);
  work.cap = S.wcap;
  Dom d;
  d.nd = at<mgp_node>(blob, S.nd);
  d.orig = at<mgp_node>(blob, S.orig);
  d.n = S.n;
  d.consts = at<uint32_t>(blob, S.consts);
  d.n_consts = S.n_consts;
  d.av = av;
  d.bs = bs;
  d.isb = at<uint8_t>(blob, S.isb);
  d.vtie = at<int32_t>(blob, S.vtie);
  d.vars = vars;
  d.pairs = pairs;
  d.n_pairs = S.n_pairs;
  d.cmp_pair = at<int32_t>(blob, S.cmp_pair);
  d.cmp_dom = at<uint8_t>(blob, S.cmp_dom);
  d.cmp_t = at<uint8_t>(blob, S.cmp_t);
  d.pair_keys = at<uint64_t>(blob, S.pair_keys);
  d.pair_idx = at<int32_t>(blob, S.pair_idx);
  d.ufs = at<UfApp>(blob, S.ufs);
  d.n_ufs = S.n_ufs;
  d.tien = at<int32_t>(blob, S.tien);
  d.n_cmpn = S.n_cmpn;
  d.n_borp = S.n_borp;
  d.ufp = at<uint32_t>(blob, S.ufp);
  d.n_ufp = S.n_ufp;
  d.cong = at<int32_t>(blob, S.cong);
  d.n_cong = S.n_cong;
  d.arel = at<ArithRel>(blob, S.arel);
  d.n_arel = S.n_arel;
  d.og = at<OrGroup>(blob, S.og);
  d.n_og = S.n_og;
  d.odis = at<OrDis>(blob, S.odis);
  d.oatom = at<int32_t>(blob, S.oatom);
  d.otgt = at<int32_t>(blob, S.otgt);
  d.inj = at<InjApp>(blob, S.inj);
  d.n_inj = S.n_inj;
  d.uoff = at<uint32_t>(blob, S.uoff);
  d.ulist = at<uint32_t>(blob, S.ulist);
  d.voff = at<uint32_t>(blob, S.voff);
  d.vlist = at<uint32_t>(blob, S.vlist);
  d.tie_rel = at<uint8_t>(blob, S.tie_rel);
  d.heur = true;
  d.undo = &undo;
  d.touched = &work;
  PrepView pv;
  pv.n_slot = S.n_slot;
  pv.slot = at<uint32_t>(blob, S.slot);
  pv.width = at<uint32_t>(blob, S.width);
  pv.node = at<int32_t>(blob, S.node);
  pv.eqh_off = at<uint32_t>(blob, S.eqh_off);
  pv.eqh = at<V>(blob, S.eqh);
  RowPut put{out_rows, out_mask, T.out_row};
  decision_row(pv, d, T.row, 2u * T.row, seed, T.tag, or_rows, put, seed_vals ? seed_vals + T.seed_row * 8u : nullptr,
               seed_mask ? seed_mask + T.seed_row : nullptr, seed_rows);
}

}  // namespace

extern "C" hipError_t mgp_launch_decide(const uint8_t *blob, const mgp_dec_state *states, const mgp_dec_task *tasks,
                                        uint32_t n_tasks, uint8_t *ws, uint64_t seed, uint32_t or_rows,
                                        const uint32_t *seed_vals, const uint8_t *seed_mask, uint32_t seed_rows,
                                        uint32_t *out_rows, uint8_t *out_mask, hipStream_t st) {
  if (n_tasks == 0) return hipSuccess;
  hipLaunchKernelGGL(mgp_decide_kernel, dim3(n_tasks), dim3(64), 0, st, blob, states, tasks, n_tasks, ws, seed,
                     or_rows, seed_vals, seed_mask, seed_rows, out_rows, out_mask);
  return hipGetLastError();
}
