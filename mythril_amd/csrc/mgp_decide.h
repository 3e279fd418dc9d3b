// mgp_decide.h — layout of the device decision-row batch (mgp_refute.cpp writes it,
// mgp_decide.hip reads it).  All offsets are byte offsets, 16-B aligned: into the
// read-only blob (the prepared states) or into one task's workspace.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

struct mgp_dec_state {
  // blob: DAG, pre-relaxation DAG (congruence arguments), constants, base analysis,
  // propagation graph and the decision slots
  uint64_t nd, orig, consts, av, bs, isb, vtie, vars, pairs, cmp_pair, cmp_dom, cmp_t, pair_keys, pair_idx, ufs;
  uint64_t uoff, ulist, voff, vlist, tie_rel, slot, width, node, eqh_off, eqh, cong, arel, og, odis, oatom, otgt, inj;
  uint64_t tien, ufp;
  uint64_t n_consts;
  uint32_t n, n_vt, n_pairs, n_ufs, n_slot, ucap, wcap, n_cong, n_arel, n_og, n_inj, n_cmpn, n_borp, n_ufp;
  // workspace of one task of this state: private node values, variable values, pair
  // orderings, truth sets, undo log, work list
  uint64_t ws_av, ws_vars, ws_pairs, ws_bs, ws_undo, ws_work, ws_bytes;
};

struct mgp_dec_task {
  uint32_t state, row;  // index into the state table; decision row number
  uint64_t ws;          // byte offset of the task's workspace
  uint64_t tag;         // candidate-stream key of the state (MGP_FE_STATE_KEY)
  uint64_t out_row;     // (batch state * n_decide + row) * n_vars: first word-row of the output
  uint64_t seed_row;    // batch state * n_vars: the state's parent-seed slots (seed_vals / seed_mask)
};

extern "C" hipError_t mgp_launch_decide(const uint8_t *blob, const mgp_dec_state *states, const mgp_dec_task *tasks,
                                        uint32_t n_tasks, uint8_t *ws, uint64_t seed, uint32_t or_rows,
                                        const uint32_t *seed_vals, const uint8_t *seed_mask, uint32_t seed_rows,
                                        uint32_t *out_rows, uint8_t *out_mask, hipStream_t st);
