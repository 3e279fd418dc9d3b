/*
 * mgp.h — C ABI of libmgp.so, the MI355X-native satisfiability pre-filter
 * and batched Keccak-256 for Mythril's LASER engine.
 *
 * The reference (mythril v0.22.1, 100 % Python) reaches native code only
 * through z3py/ctypes and pysha3; these entry points are the native boundary
 * that replaces those calls on the hot path:
 *
 *   mgp_eval_batch      replaces the serial z3 check() behind
 *                        Constraints.is_possible
 *                        (mythril/laser/ethereum/state/constraints.py:34-51)
 *                        and the SAT-only analysis.solver.get_model calls
 *                        (mythril/analysis/solver.py:27-61) — witness search
 *                        only: a witness proves SAT, everything else stays z3.
 *   mgp_lower           lowers the constraint DAG (laser.smt vocabulary,
 *                        mythril/laser/smt/ *.py) to the flat bytecode.
 *   mgp_keccak256_batch replaces ethereum.utils.sha3 in
 *                        KeccakFunctionManager.find_concrete_keccak
 *                        (mythril/laser/ethereum/keccak_function_manager.py:40-54)
 *                        and pysha3 keccak_256 in get_code_hash
 *                        (mythril/support/support_utils.py:29-41).
 *
 * Conventions: every function returns 0 on success and a negative MGP_E_*
 * code on failure; no C++ exception crosses this boundary; host buffers are
 * caller-owned; the context owns device buffers and a HIP stream.  One context
 * per device per host thread.  Results are deterministic: first-SAT is the
 * lowest candidate index whose assignment makes the root true.
 *
 * The *_dev entry points take device pointers and a hipStream_t (as void*) so
 * that callers holding inputs resident in HBM (bench.py, torch tensors) skip
 * the PCIe copies.
 */
#ifndef MGP_H
#define MGP_H

#include <stddef.h>
#include <stdint.h>

#include "mgp_ir.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MGP_OK 0
#define MGP_E_ARG (-1)       /* bad argument / shape                       */
#define MGP_E_HIP (-2)       /* HIP runtime error (message in mgp_last_error) */
#define MGP_E_NOMEM (-3)     /* allocation failed                          */
#define MGP_E_CAPACITY (-4)  /* output buffer too small (mgp_lower)        */

typedef struct mgp_ctx mgp_ctx;

/* ------------------------------------------------------------ lifecycle */
int mgp_create(int device, mgp_ctx **out);
void mgp_destroy(mgp_ctx *ctx);
const char *mgp_last_error(mgp_ctx *ctx); /* ctx may be NULL: global error */
int mgp_device_count(int *out);
const char *mgp_version(void);
/* Host threads of the OpenMP stages started FROM THE CALLING THREAD (lowering, pre-check,
 * decision rows, ...): n > 0 sets it for this thread only; returns the previous value.
 * The background UNSAT-core shrink (mythril_amd.solver.UnsatCores) uses it so that it
 * does not oversubscribe the cores the foreground calls use. */
int mgp_set_thread_omp(int n);

/* -------------------------------------------------------------- lowering
 * Host-side, no device needed.  Lowers n_states node lists to bytecode.
 *   nodes[node_offsets[s] .. node_offsets[s+1])   nodes of state s
 *   consts[const_offsets[s]*8 ..]                  its constant pool (u32 limbs)
 * out_words receives the concatenated programs (capacity out_cap words),
 * out_prog_offsets[s] the word offset of state s (n_states+1 entries),
 * out_status[s] MGP_ST_OK or MGP_ST_UNSUPPORTED (an unsupported state still
 * gets a valid program header so that evaluation reports MGP_UNDECIDED).
 * max_slots caps the BV slots per state (0 = default 32).
 * Returns MGP_E_CAPACITY (and the needed size in *out_words_used) if too small. */
int mgp_lower(const mgp_node *nodes, const uint64_t *node_offsets,
              uint32_t n_states, const uint32_t *consts,
              const uint64_t *const_offsets, uint32_t max_slots,
              uint32_t *out_words, uint64_t out_cap,
              uint64_t *out_prog_offsets, uint8_t *out_status,
              uint64_t *out_words_used);

/* ----------------------------------------------------- constraint eval
 * prog_words/prog_offsets: output of mgp_lower (prog_offsets has n_states+1
 * entries; prog_offsets[n_states] = total words).
 * cand_words: n_states * n_cand * n_vars * 8 u32, layout [state][cand][var][limb]
 *   (limb 0 least significant).
 * out_first_sat[s]: lowest satisfying candidate index, MGP_NO_SAT (-1) if none,
 *   MGP_UNDECIDED (-2) if the state's program is unsupported (MGP_EVAL_FAULT (-3):
 *   an internal inconsistency, never expected).
 * out_witness (may be NULL): n_states * n_vars * 8 u32; filled for SAT states
 *   with the winning candidate's words, left untouched otherwise. */
int mgp_eval_batch(mgp_ctx *ctx, const uint32_t *prog_words,
                   const uint64_t *prog_offsets, uint32_t n_states,
                   const uint32_t *cand_words, uint32_t n_cand,
                   uint32_t n_vars, int32_t *out_first_sat,
                   uint32_t *out_witness);

/* Device-resident variant.  d_cands uses the DEVICE layout
 * [state][var][half][cand] of 16-byte groups.  With n_buckets == 0 one launch
 * covers all states with n_slots BV slots of LDS each (the max header slot
 * count).  Otherwise d_order (device) lists the states bucket by bucket:
 * bucket b = d_order[bucket_bounds[b] .. bucket_bounds[b+1]) runs with
 * bucket_slots[b] slots (bounds/slots are HOST arrays, see mgp_plan_buckets),
 * so each bucket gets the occupancy its LDS footprint allows. */
int mgp_eval_batch_dev(const uint32_t *d_prog_words,
                       const uint64_t *d_prog_offsets, uint32_t n_states,
                       const uint32_t *d_cands, uint32_t n_cand,
                       uint32_t n_vars, uint32_t n_slots,
                       int32_t *d_first_sat, uint32_t *d_witness,
                       int32_t *d_scratch /* n_states*ceil(n_cand/64) */,
                       const uint32_t *d_order,
                       const uint32_t *bucket_bounds,
                       const uint32_t *bucket_slots, uint32_t n_buckets,
                       void *stream);

/* Evaluation engine of mgp_eval_batch / mgp_eval_batch_dev:
 *   MGP_ENGINE_ASM  hand-written gfx950 interpreter (mgp_eval_gfx950), default
 *   MGP_ENGINE_HIP  HIP C++ interpreter (independent second implementation)
 * Sets the engine when `engine` is one of them; returns the current engine.
 * Process-wide; MGP_ENGINE=hip|asm in the environment sets the initial value. */
#define MGP_ENGINE_HIP 1
#define MGP_ENGINE_ASM 2
int mgp_set_eval_engine(int engine);

/* Keccak kernel of the 64-byte fast path (mgp_keccak256_batch / _dev with len = 64 and a
 * 16-B aligned stride): MGP_ENGINE_ASM = mgp_keccak64_gfx950 (gen_keccak_asm.py, VGPRs
 * placed by bank), default; MGP_ENGINE_ASM_DX = its variant with theta through D[x]
 * (two-source XORs); MGP_ENGINE_HIP = mgp_keccak64_kernel (compiler-allocated).  Same
 * digests.  Sets it when `engine` is one of them; returns the current one.
 * MGP_KECCAK_ENGINE=hip|asm|asm_dx sets the initial value. */
#define MGP_ENGINE_ASM_DX 3
int mgp_set_keccak_engine(int engine);

/* Diagnostic only: when d_diag (device memory, 16 B per state x chunk) is non-null the
 * MGP_ENGINE_ASM kernel writes per-wave clock stamps there (profiles/stamps.py). */
int mgp_set_eval_diag(void *d_diag);

/* Host-side launch plan: states grouped by the BV-slot count in their program
 * header.  Writes order_out[n_states], bounds_out[nb+1], slots_out[nb];
 * returns nb (<= max_buckets) or a negative error. */
int mgp_plan_buckets(const uint32_t *prog_words, const uint64_t *prog_offsets,
                     uint32_t n_states, uint32_t *order_out,
                     uint32_t *bounds_out, uint32_t *slots_out,
                     uint32_t max_buckets);

/* Fill device candidates with the benchmark mixture (Philox4x32-10 keyed by
 * (seed, state_base+s, cand, var)): 25 % interesting values (0, 1, 2^256-1,
 * 2^255, 2^160-1, ACTORS, constant-pool entries +-1), 75 % uniform. */
int mgp_fill_candidates_dev(const uint32_t *d_prog_words,
                            const uint64_t *d_prog_offsets, uint32_t n_states,
                            uint64_t state_base, uint64_t seed,
                            uint32_t *d_cands, uint32_t n_cand,
                            uint32_t n_vars, void *stream);

/* Overwrite candidate plant_idx[i] of state plant_state[i] with the n_vars*8
 * words plant_words[i] (device pointers, n_plant entries). */
int mgp_plant_candidates_dev(uint32_t *d_cands, uint32_t n_states,
                             uint32_t n_cand, uint32_t n_vars,
                             const uint32_t *d_plant_state,
                             const uint32_t *d_plant_idx,
                             const uint32_t *d_plant_words, uint32_t n_plant,
                             void *stream);

/* ----------------------------------------------------- UNSAT pre-check
 * Host-side, no device needed (OpenMP over states).  Replaces, for the states
 * it decides, the z3 check that follows a GPU miss: Constraints.is_possible
 * (mythril/laser/ethereum/state/constraints.py:34-51, unsat -> False) and
 * get_model (mythril/analysis/solver.py:27-61, unsat -> UnsatError).
 * Sound abstract interpretation (known bits x unsigned interval per BV node,
 * truth set per Bool node) with backward narrowing from root = true, at most
 * max_passes forward+backward passes (0 = 16).  Node lists / constant pools as
 * for mgp_lower.
 *   out[s] = 1   no assignment satisfies state s (proven UNSAT)
 *            0   not refuted (SAT or undecided: the caller's solver decides)
 *           -1   not analysed (width > 256, malformed node list)
 * A 1 is a proof; it never depends on candidates or randomness. */
int mgp_refute(const mgp_node *nodes, const uint64_t *node_offsets,
               uint32_t n_states, const uint32_t *consts,
               const uint64_t *const_offsets, uint32_t max_passes,
               int8_t *out);
/* mgp_refute plus case splitting for the states it leaves open: each open select
 * condition (BV ITE / BITE, nearest the root first; max_splits bits 0..15 = at most this
 * many per state) is assumed true and false in turn, and each branch is split again on
 * the others up to (max_splits >> 16) & 15 levels (0 = 1); both branches refuted -> 1;
 * one refuted -> the other polarity is kept.  Then (round 6; max_splits bit 20 clear)
 * interval bisection: a variable whose interval the analysis bounded is split in halves,
 * 8 levels deep, each half propagated; every leaf refuted -> 1 (rubixi.sol:130-151:
 * value * 90 / 100 > value * 300 / 100 between two require()s on value).  A 1 is a proof.
 * The product runs it on the states both witness rounds leave open (solver.Prefilter),
 * before they go to the caller's solver: ether_thief's balance comparisons after a
 * zero-value transfer whose recipient is open (mythril/analysis/module/modules/
 * ether_thief.py:55-95). */
int mgp_refute_split(const mgp_node *nodes, const uint64_t *node_offsets,
                     uint32_t n_states, const uint32_t *consts,
                     const uint64_t *const_offsets, uint32_t max_passes,
                     uint32_t max_splits, int8_t *out);
/* UNSAT cores of refuted constraint lists (round 5; replaces rebuilding a DAG per deletion
 * trial in the caller).  Each state is the DAG mgp_build_states builds from a list of
 * n_roots[s] constraints (roots AND-chained at its tail).  Per state: up to `halvings`
 * rounds keep the first or second half of the list when it alone is refuted, then (lists of
 * at most max_single) greedy single deletions drop every constraint whose removal keeps the
 * list refuted; each trial re-runs mgp_refute's analysis with only the kept constraints
 * required.  keep (one byte per constraint, states concatenated): 1 = in the core.
 * out[s]: 1 = core found (the kept set is refuted: a proof, the reference's z3 would answer
 * unsat for it, analysis/solver.py:56-61), 0 = the list is not refuted (all kept),
 * -1 = no root chain / malformed (all kept).  Host only (OpenMP over states). */
int mgp_refute_cores(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                     const uint32_t *consts, const uint64_t *const_offsets, const uint32_t *n_roots,
                     uint32_t max_passes, uint32_t halvings, uint32_t max_single, uint8_t *keep,
                     int8_t *out);
/* Diagnostic (tests): the refined abstract value of every node of ONE state,
 * 33 words per node: known-zero mask, known-one mask, lo, hi (8 u32 limbs
 * each) and the Bool truth set (bit0 = may be false, bit1 = may be true).
 * Returns 1 / 0 / -1 as mgp_refute. */
int mgp_refute_trace(const mgp_node *nodes, uint64_t n_nodes,
                     const uint32_t *consts, uint64_t n_consts,
                     uint32_t max_passes, uint32_t *out_av);

/* Guided candidates for the states the first witness round missed: runs the
 * same analysis as mgp_refute and, for every state it does not refute, writes
 * values drawn from each variable's refined abstract value (interval bounds,
 * then draws inside the interval with the known bits forced) into candidate
 * rows 0, every, 2*every, ... of `cands` (host layout of mgp_eval_batch:
 * [state][cand][var][8 limbs]); other rows and variables the DAG does not
 * read are left as given.  The first n_decide of those rows are built by
 * decisions: each variable in turn is fixed to a draw from its current
 * abstract value and the analysis re-propagated from the decided node (a
 * bounded worklist; MGP_DECIDE_PASSES=k re-runs k full passes instead), so
 * later variables see the narrowing the earlier choices cause.  Decision rows
 * 0-7 decide in variable order, rows 8-15 in reverse order, later rows in
 * either; the first eight take draw schedules 0, 4, 6, 8, 2, 10, 12, 14 (the
 * lo/hi schedule and three random-draw schedules first).  UF applications get their fresh value slot (p1)
 * from the application's abstract value (keccak intervals, alignment).
 * Deterministic in seed.  out[s] as mgp_refute.  Replaces nothing in the
 * reference: it feeds the GPU witness search that answers get_model /
 * is_possible (analysis/solver.py:27-61, constraints.py:34-51) before z3. */
int mgp_guided_candidates(const mgp_node *nodes, const uint64_t *node_offsets,
                          uint32_t n_states, const uint32_t *consts,
                          const uint64_t *const_offsets, uint32_t max_passes,
                          uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                          uint32_t every, uint32_t n_decide, uint32_t *cands,
                          int8_t *out);

/* mgp_guided_candidates with a decision-row count per state: state s gets
 * min(rows_per_state[s], n_decide) decision rows, the rest of its guided rows
 * are plain domain draws (the front end gives expensive states fewer rows so
 * that more of them fit its time budget).  rows_per_state = NULL is
 * mgp_guided_candidates. */
int mgp_guided_candidates_rows(const mgp_node *nodes, const uint64_t *node_offsets,
                               uint32_t n_states, const uint32_t *consts,
                               const uint64_t *const_offsets, uint32_t max_passes,
                               uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                               uint32_t every, uint32_t n_decide,
                               const uint8_t *rows_per_state, uint32_t *cands,
                               int8_t *out);

/* Decision rows only (host, OpenMP over (state, row) tasks): the rows the first n_decide
 * rows of mgp_guided_candidates_rows would write, as explicit rows for mgp_check_batch:
 * out_rows [n_states][n_decide][n_vars][8], out_mask [n_states][n_decide][n_vars] (1 =
 * the row sets that slot; a row of a refuted or unanalysed state sets none).  State s
 * gets min(rows_per_state[s], n_decide) rows (NULL = n_decide).  Draws are keyed by
 * (seed, state_keys[s] or s, row, slot); each decision propagates within
 * 4 x nodes + 64 transfer-function evaluations, so the rows depend on the state's
 * content and the seed only -- not on the thread count, the batch or the host's speed.
 * out[s] as mgp_refute. */
int mgp_decision_rows(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                      const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                      uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t n_decide,
                      const uint8_t *rows_per_state, uint32_t *out_rows, uint8_t *out_mask, int8_t *out);

/* mgp_decision_rows with parent seeds: seed_vals u32[n_states *
 * n_vars * 8] and seed_mask u8[n_states * n_vars] give, per variable slot, the parent
 * state's witness value (matched by slot key); decision row r with bit r of seed_rows set
 * first fixes every seeded slot to it (rolled back where the child's constraints reject
 * it), then decides the rest as usual (mgp_domain.h decision_row).  Both NULL = unseeded.
 * A child state extends its parent by one constraint (svm.py:251-255, the prune point). */
int mgp_decision_rows_seeded(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                             const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                             uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t n_decide,
                             const uint8_t *rows_per_state, const uint32_t *seed_vals, const uint8_t *seed_mask,
                             uint32_t seed_rows, uint32_t *out_rows, uint8_t *out_mask, int8_t *out);
/* mgp_decision_rows_seeded for rows row0 .. row0 + n_decide - 1: output row k is decision
 * row row0 + k (its schedule, case splits, draw stream and seed_rows bit are those of row
 * row0 + k); rows_per_state counts rows from row0.  row0 = 0 is mgp_decision_rows_seeded.
 * Prefilter's first round asks large states for row 1 alone (solver.py ROWS_FIRST_FROM). */
int mgp_decision_rows_from(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                           const uint32_t *consts, const uint64_t *const_offsets, uint32_t max_passes,
                           uint32_t n_vars, uint64_t seed, const uint64_t *state_keys, uint32_t row0,
                           uint32_t n_decide, const uint8_t *rows_per_state, const uint32_t *seed_vals,
                           const uint8_t *seed_mask, uint32_t seed_rows, uint32_t *out_rows, uint8_t *out_mask,
                           int8_t *out);
/* Candidate assignments for the first witness round (host, OpenMP over states):
 * per state, row 0 is left for the parent witness when has_parent[s], then the
 * first hint of every variable, that row with the x == y aliases applied, then
 * a seeded mixture per variable (35 % hint, 25 % pool = constants, +-1, the
 * fixed pool; 15 % alias of an equal-width variable; 25 % uniform), masked to
 * the slot width.  var_kind (may be NULL): slots of kind 2 (pinned constants,
 * MGP_FE_VAR_KIND) hold their first hint in every row.  Variables of state s are var_off[s]..var_off[s+1]; hints of
 * variable v are rows hint_off[v]..hint_off[v+1] of `hints` (8 limbs each);
 * aliases are (dst, src) pairs of state-local indices; consts as for
 * mgp_lower.  out: [n_states][n_cand][n_vars][8], the host layout of
 * mgp_eval_batch.  Deterministic in seed, independent of the thread count.
 * state_keys (may be NULL): per-state stream tags (MGP_FE_STATE_KEY), so that a
 * state's rows depend on its content, not on its index in the batch. */
int mgp_make_candidates(uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                        const uint64_t *var_off, const uint32_t *var_width, const uint8_t *var_kind,
                        const uint64_t *hint_off, const uint32_t *hints,
                        const uint64_t *alias_off, const uint32_t *aliases,
                        const uint64_t *const_off, const uint32_t *consts,
                        const uint32_t *fixed_pool, uint32_t n_fixed,
                        const uint8_t *has_parent, const uint32_t *dom, const uint64_t *state_keys,
                        uint32_t *out);
/* mgp_refute plus the refined abstract value of every variable slot of the states it
 * does not refute: out_dom has 33 u32 per slot of var_off (known-zero, known-one, lo,
 * hi as 8 limbs each, then 1 if the slot has a domain, else 0).  `dom` of
 * mgp_make_candidates / the device generator: every other mixture row draws those
 * slots from their domains (mgp_fe_sample.h), an inside hint half of the time. */
int mgp_refute_domains(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states,
                       const uint32_t *consts, const uint64_t *const_offsets, const uint64_t *var_off,
                       uint32_t max_passes, int8_t *out, uint32_t *out_dom);

/* ------------------------------------------------------ native front end
 * Flattens a batch of states' path constraints (the roots) into node lists, constant
 * pools, variable tables and candidate hints, OpenMP over states — what the reference
 * re-adds to a fresh z3 solver per state (constraints.py:34-51, analysis/solver.py:
 * 37-50).  Input: the term arena (mythril_amd/smt.py _Arena): per term op, width
 * (Bool = 0), 3 argument term ids (-1 = none, always < the term's own id), 2 params
 * (VAR: name id; CONST: limb offset, limb count; EXTRACT: hi, lo; UFAPP/UFINV:
 * function id, function-name id) and the little-endian u32 limbs of the constants.
 * roots[root_off[s] .. root_off[s+1]) are the term ids of state s's constraints.
 * The batch is read back with mgp_fe_get (arrays owned by the batch, valid until
 * mgp_fe_free; *count = number of ELEMENTS of the field's type listed below, e.g. 8
 * uint32_t per constant).  Per variable slot: width (<= 256), full width (first slot of a
 * value, else 0), name id, aux (slot index within a wide value; for a fresh
 * uninterpreted-function value the node index of its application; for a pinned
 * constant its pool index), kind (0 named variable, 1 fresh UF value, 2 pinned
 * constant: every candidate row holds hint 0 of the slot).  hint_off is per variable slot (8 limbs per hint);
 * aliases are (dst, src) slot pairs local to the state.  name_hash[id] (may be NULL, n_names
 * entries) is a stable hash of the text of arena name `id`; STATE_KEY folds it in place of the
 * id, so a state's key (and its candidates) do not depend on the order names were interned.
 * GPU_NODES (offsets
 * GPU_NODE_OFF) is the program the GPU evaluates: NODES except that padded key
 * equalities are replaced by the constant that strengthens the formula, and that
 * operand uses of pinned constants read VAR nodes placed in front of the state's
 * program (mgp_front.cpp); FLAGS per state: */
#define MGP_FE_SAT_UNSAFE 0x1u   /* a padded key equality under both polarities: no GPU SAT answer */
#define MGP_FE_STRENGTHENED 0x2u /* padded key equalities replaced in GPU_NODES */
#define MGP_FE_PINNED 0x4u       /* constants past the pool budget are pinned variable slots in GPU_NODES */
#define MGP_FE_POOL_KEEP 48u     /* constant-pool entries a GPU program keeps (the rest are pinned) */
typedef struct mgp_fe_batch mgp_fe_batch;
enum mgp_fe_field {
  MGP_FE_NODES = 0,     /* mgp_node                     */
  MGP_FE_GPU_NODES,     /* mgp_node                     */
  MGP_FE_NODE_OFF,      /* uint64_t, n_states + 1       */
  MGP_FE_CONSTS,        /* uint32_t, 8 per entry        */
  MGP_FE_CONST_OFF,     /* uint64_t, n_states + 1       */
  MGP_FE_VAR_OFF,       /* uint64_t, n_states + 1       */
  MGP_FE_VAR_WIDTH,     /* uint32_t per slot            */
  MGP_FE_VAR_FULL,      /* uint32_t per slot            */
  MGP_FE_VAR_NAME,      /* uint32_t per slot            */
  MGP_FE_VAR_AUX,       /* uint32_t per slot            */
  MGP_FE_VAR_KIND,      /* uint8_t per slot             */
  MGP_FE_HINT_OFF,      /* uint64_t, n_slots + 1        */
  MGP_FE_HINTS,         /* uint32_t, 8 per hint         */
  MGP_FE_ALIAS_OFF,     /* uint64_t, n_states + 1       */
  MGP_FE_ALIASES,       /* uint32_t, 2 per pair         */
  MGP_FE_FLAGS,         /* uint8_t per state            */
  MGP_FE_VAR_KEY,       /* uint64_t per slot: name id, kind, UF node, piece (parent matching) */
  MGP_FE_GPU_NODE_OFF,  /* uint64_t, n_states + 1: offsets into GPU_NODES */
  MGP_FE_VAR_TID,       /* int32_t per slot: arena id of the VAR / UF term it stands for (-1 pinned) */
  MGP_FE_STATE_KEY,     /* uint64_t per state: content key (nodes, constants, variable names by
                           name_hash, not arena ids); candidate streams are keyed by it */
  MGP_FE_DEC_NODES      /* mgp_node, offsets NODE_OFF: NODES with the GPU program's padded-key
                           strengthening applied and no pinning -- the formula witness searches
                           (decision rows, domain rows) aim at; never used for a refutation */
};
int mgp_build_states(const uint8_t *t_op, const uint32_t *t_width, const int32_t *t_args, const uint32_t *t_p,
                     uint64_t n_terms, const uint32_t *limbs, uint64_t n_limbs, const int32_t *roots,
                     const uint64_t *root_off, uint32_t n_states, const uint64_t *name_hash,
                     uint64_t n_names, mgp_fe_batch **out);
int mgp_fe_get(const mgp_fe_batch *batch, int field, const void **ptr, uint64_t *count);
void mgp_fe_free(mgp_fe_batch *batch);
/* States idx[0..n) of a built batch (indices < its n_states, any order, repeats allowed) as a
 * new batch, free with mgp_fe_free: every field equals what mgp_build_states gives for those
 * states' roots, without walking the term arena again.  solver.Prefilter cuts its
 * candidate-memory groups and retry rounds out of the call's one build this way. */
int mgp_fe_select(const mgp_fe_batch *batch, const uint32_t *idx, uint32_t n, mgp_fe_batch **out);

/* One batch through the whole pre-filter (mgp_pipeline.cpp): lower the GPU programs,
 * run the host pre-check (mgp_refute_domains: refutations + the variable domains the
 * candidates draw from), generate n_cand candidates per state ON THE GPU (the
 * mgp_make_candidates mixture, bit-identical, from the batch's hints/aliases/constants +
 * fixed_pool) and evaluate them.  Parent witnesses (optional):
 * parent_keys/parent_vals[parent_off[s] .. parent_off[s+1]) are (slot key, 8 limbs)
 * pairs of state s's parent witness; slot_keys = the batch's MGP_FE_VAR_KEY; a state
 * with a parent gets those values in candidate row 0.  Outputs: out_first[s] as
 * mgp_eval_batch, out_witness (may be NULL) n_states x n_vars x 8 u32 with n_vars =
 * *out_n_vars = the batch's widest state (SAT rows only), out_refuted[s] as
 * mgp_refute.  out_times (may be NULL) receives 5 stage times in ms: lower,
 * refute, upload+launch, GPU wait, copy-back.  Candidate streams are keyed by the
 * batch's MGP_FE_STATE_KEY, so a state's answer does not depend on the batch it is in.
 * Explicit rows (optional, n_xrows > 0): xrows [n_states][n_xrows][n_xvars][8] and
 * xmask [n_states][n_xrows][n_xvars] -- the first n_xrows mixture rows of state s take
 * the values of the slots the mask marks (decision rows, mgp_decision_rows).
 * Replaces, for one batch, the z3
 * checks of Constraints.is_possible (constraints.py:34-51) and the SAT-only get_model
 * calls (analysis/solver.py:27-61) it can decide. */
/* Size mgp_check_batch's pinned host staging buffer and device candidate block of ctx
 * up front (they otherwise grow on the first large batch: pinning ~200 MB of host memory
 * takes tens of ms).  solver.Prefilter reserves its cand_bytes at construction. */
int mgp_pipeline_reserve(mgp_ctx *ctx, uint64_t host_bytes, uint64_t cand_bytes);
#define MGP_CHECK_NO_REFUTE 0x1u   /* skip the host pre-check (and the domain rows) */
#define MGP_CHECK_NO_DOMAINS 0x2u  /* plain mixture rows only (A/B)                    */
#define MGP_CHECK_NO_WITNESS 0x4u  /* mgp_check_submit: first-SAT words only, no witness download */
int mgp_check_batch(mgp_ctx *ctx, const mgp_fe_batch *batch, uint32_t n_cand, uint64_t seed,
                    const uint32_t *fixed_pool, uint32_t n_fixed, const uint64_t *parent_keys,
                    const uint32_t *parent_vals, const uint64_t *parent_off, const uint64_t *slot_keys,
                    const uint32_t *xrows, const uint8_t *xmask, uint32_t n_xrows, uint32_t n_xvars,
                    uint32_t flags, int32_t *out_first, uint32_t *out_witness, int8_t *out_refuted,
                    uint32_t *out_n_vars, double *out_times);
/* mgp_check_batch in two halves, so that a caller overlaps one batch's GPU round with the
 * next batch's host stages.  mgp_check_submit does the host stages (lowering, pre-check,
 * staging into one of the context's two pinned buffers), enqueues the upload, kernels and
 * download on the context's stream, and returns without waiting: out_refuted and
 * *out_n_vars are final, out_times gets 3 stage times (lower, refute, upload+launch),
 * *out_ticket names the batch (-1 for an empty one).  At most two batches are in flight
 * per context (a third submit fails with MGP_E_ARG).  mgp_check_finish waits for the
 * ticket's batch and writes out_first / out_witness as mgp_check_batch does (out_witness
 * NULL, or a submit with MGP_CHECK_NO_WITNESS: none); out_times gets 2 (GPU wait,
 * copy-back).  Batches run on the device in submit order; the batch object and the
 * explicit rows need to live only until mgp_check_submit returns.  Answers are those of
 * mgp_check_batch on the same arguments. */
int mgp_check_submit(mgp_ctx *ctx, const mgp_fe_batch *batch, uint32_t n_cand, uint64_t seed,
                     const uint32_t *fixed_pool, uint32_t n_fixed, const uint64_t *parent_keys,
                     const uint32_t *parent_vals, const uint64_t *parent_off, const uint64_t *slot_keys,
                     const uint32_t *xrows, const uint8_t *xmask, uint32_t n_xrows, uint32_t n_xvars,
                     uint32_t flags, int8_t *out_refuted, uint32_t *out_n_vars, double *out_times,
                     int32_t *out_ticket);
int mgp_check_finish(mgp_ctx *ctx, int32_t ticket, int32_t *out_first, uint32_t *out_witness,
                     double *out_times);
/* mgp_check_batch keeps the programs it lowers in a process-wide cache keyed by the
 * exact node list and constants of each state (compared in full on a hit; 256 MiB,
 * oldest first out): a retry round or a repeated query skips the lowering.  This
 * empties it (cold measurements, tests); returns the number of programs dropped. */
uint64_t mgp_program_cache_clear(void);
/* Lower the GPU programs of `batch` into that cache (no device work): a caller that has
 * host work of its own before mgp_check_batch (the first-round decision rows of large
 * states, solver.Prefilter) runs it on another thread meanwhile, and the check then finds
 * every program lowered.  MGP_OK or the lowering's error. */
int mgp_program_cache_warm(const mgp_fe_batch *batch);
/* Test hook: the candidates mgp_check_batch would evaluate (no parents), device layout
 * [state][var][half][cand] of 16-byte groups, n_vars >= the batch's widest state. */
int mgp_fe_candidates(mgp_ctx *ctx, const mgp_fe_batch *batch, uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                      const uint32_t *fixed_pool, uint32_t n_fixed, const uint32_t *dom, const uint32_t *xrows,
                      const uint8_t *xmask, uint32_t n_xrows, uint32_t n_xvars, uint32_t *out);

/* ---------------------------------------------------------- Keccak-256
 * n preimages of len bytes each, preimage i at in + i*stride; 32-byte
 * big-endian digests to out32 + 32*i.  Keccak-256 = Keccak[r=1088,c=512]
 * with 0x01 domain padding (Ethereum), NOT NIST SHA3-256. */
int mgp_keccak256_batch(mgp_ctx *ctx, const uint8_t *in, uint64_t n,
                        uint32_t len, uint32_t stride, uint8_t *out32);
int mgp_keccak256_dev(const uint8_t *d_in, uint64_t n, uint32_t len,
                      uint32_t stride, uint8_t *d_out32, void *stream);

/* Benchmark preimages: pad32(addr_i) || pad32(i mod 8), addr_i = low 160 bits
 * of splitmix64 chain seeded with seed + first + i. */
int mgp_fill_mapping_preimages_dev(uint8_t *d_out64, uint64_t first,
                                   uint64_t n, uint64_t seed, void *stream);

/* --------------------------------------------------- synthetic workload
 * Seeded synthetic constraint DAGs: n_nodes op-nodes per
 * state over 4 free 256-bit vars + up to 2 keccak-UF apps (vars 4, 5) and a
 * <=16-entry constant pool; root = conjunction of the last 4 Bool nodes.
 * States are generated independently from (seed, state_base + s), so any
 * sub-range reproduces exactly.  For states with planted[s] = 1 a satisfying
 * assignment (n_vars*8 words) is written to plant_words[s] and the candidate
 * index to plant_idx[s] (< n_cand).
 * Capacities: nodes_out >= n_states*(n_nodes+32), consts_out >= n_states*16*8. */
int mgp_synth_generate(uint64_t seed, uint64_t state_base, uint32_t n_states,
                       uint32_t n_nodes, uint32_t n_cand,
                       mgp_node *nodes_out, uint64_t *node_offsets,
                       uint32_t *consts_out, uint64_t *const_offsets,
                       uint8_t *planted, uint32_t *plant_idx,
                       uint32_t *plant_words);
/* Ablation of the synthetic generator for the benchmark's division split: mode 1 draws
 * every division (UDIV/UREM/SDIV/SREM/SMOD) as an ADD, 2 every MUL, 3 both, 0 none; the
 * DAGs are otherwise the same.  Process-wide (default from MGP_SYNTH_ABLATE). */
int mgp_synth_set_ablate(int mode);

/* Nominal INT32 op counts summed over the op-nodes of
 * each state — the algorithmic work the roofline fraction is priced on. */
int mgp_nominal_ops(const mgp_node *nodes, const uint64_t *node_offsets,
                    uint32_t n_states, uint64_t *out_ops);

/* INT32 VALU issue-rate probe: blocks x 256 threads x iters x 512 v_add_u32
 * (the count is written to *ops_out); time it on `stream` to obtain the
 * measured peak the roofline fractions are priced against. */
int mgp_probe_valu_dev(uint32_t iters, uint32_t blocks, uint32_t *d_sink,
                       uint64_t *ops_out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MGP_H */
