// mgp_pipeline.cpp — one call per batch of states: lower, pre-check on the host,
// generate candidates on the GPU and evaluate (the pre-check runs before the upload: its
// domains feed the candidates).  A caller overlaps one batch's GPU round with the next
// batch's host stages through mgp_check_submit / mgp_check_finish.
//
// This is the native body of Prefilter.check_states (mythril_amd/solver.py), i.e. of
// the batched prune filter at LaserEVM.exec (mythril/laser/ethereum/svm.py:251-255)
// and of the SAT-only get_model calls (mythril/analysis/solver.py:27-61).  Input is a
// front-end batch (mgp_front.cpp).  Stages, in order, on the context's stream:
//   1. lower the GPU program of every state (mgp_lower.cpp, OpenMP);
//   2. the host UNSAT pre-check (mgp_refute_domains, original nodes: the sound
//      direction, see mgp_front.cpp), which also yields every variable's refined
//      abstract value;
//   3. upload programs and the candidate tables (variable widths, hints, aliases,
//      constants, parent-witness rows, domains) — a few hundred bytes per variable,
//      instead of n_cand x n_vars x 32 B of host-built candidates;
//   4. mgp_fe_cands_kernel writes the candidates straight into the interpreter's
//      [state][var][half][cand] layout (every other mixture row drawn from the
//      domains); launch descriptors, the gfx950 interpreter and the first-SAT
//      reduction follow (mgp_launch_eval);
//   5. first-SAT words and witnesses come back.
// Stage times (ms) go to out_times[0..4] when given: lower, refute, upload+launch,
// GPU wait, copy-back.
#include <hip/hip_runtime.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mgp.h"
#include "mgp_buf.h"

extern "C" {
hipError_t mgp_launch_eval(const uint32_t *words, const uint64_t *offs, uint32_t n_states, const uint32_t *cands,
                           uint32_t n_cand, uint32_t n_vars, uint32_t n_slots, int32_t *first_sat,
                           uint32_t *witness, int32_t *partial, const uint32_t *order,
                           const uint32_t *bucket_bounds, const uint32_t *bucket_slots, uint32_t n_buckets,
                           hipStream_t st);
hipError_t mgp_launch_fe_cands(uint32_t n_states, uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                               const uint64_t *var_off, const uint32_t *var_width, const uint8_t *var_kind,
                               const uint64_t *hint_off,
                               const uint32_t *hints, const uint64_t *alias_off, const uint32_t *aliases,
                               const uint64_t *const_off, const uint32_t *consts, const uint32_t *fixed,
                               uint32_t n_fixed, const int32_t *parent_idx, const uint32_t *pvals,
                               const uint8_t *pmask, const uint32_t *dom, const uint32_t *asrc_off,
                               const uint32_t *asrc, const uint32_t *wcls, const uint32_t *wlist,
                               const uint64_t *state_keys, const uint32_t *xrows, const uint8_t *xmask,
                               uint32_t n_xrows, uint32_t n_xvars, uint32_t *out, hipStream_t st);
int mgp_fe_get(const mgp_fe_batch *batch, int field, const void **ptr, uint64_t *count);
int mgp_ctx_stream(mgp_ctx *ctx, void **stream, int *device);
int mgp_ctx_fail(mgp_ctx *ctx, int code, const char *msg);
}
int mgp_lower_vec(const mgp_node *nodes, const uint64_t *node_offsets, uint32_t n_states, const uint32_t *consts,
                  const uint64_t *const_offsets, uint32_t max_slots, U32Buf &words,
                  std::vector<uint64_t> &offs, std::vector<uint8_t> &status);

namespace {

struct Arr {
  const void *p = nullptr;
  uint64_t n = 0;
};

Arr get(const mgp_fe_batch *B, int f) {
  Arr a;
  mgp_fe_get(B, f, &a.p, &a.n);
  return a;
}

// One submitted batch: its pinned staging buffer (one upload and one download per batch;
// pageable hipMemcpyAsync is a blocking staged copy, ~0.4 ms each), the event recorded
// after its download, and what mgp_check_finish needs to unpack the download.  Two slots
// per context: a caller submits the next batch -- lowering, pre-check and staging on the
// host -- while the previous one runs on the GPU (solver.Prefilter's group pipeline).
struct Slot {
  void *host = nullptr;
  size_t hcap = 0;
  hipEvent_t done = nullptr;
  bool busy = false;
  bool want_witness = false;
  uint32_t n_states = 0, n_vars = 0, user_vars = 0;
  size_t first_bytes = 0;
  std::vector<uint8_t> status;
  hipError_t ensure_host(size_t bytes) {
    if (bytes <= hcap) return hipSuccess;
    if (host) (void)hipHostFree(host);
    host = nullptr;
    hcap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1u << 20);
    hipError_t e = hipHostMalloc(&host, want, hipHostMallocDefault);
    if (e == hipSuccess) hcap = want;
    return e;
  }
};

// device buffers of the pipeline, one set per (context); grown on demand.  Every batch's
// device work is in order on the context's stream, so two submitted batches share them.
struct PipeBufs {
  void *p[16] = {};
  size_t cap[16] = {};
  U32Buf words;          // the batch's lowered programs (host), reused across calls
  U32Buf dom;            // the batch's variable domains (host), reused across calls
  Slot slot[2];
  hipError_t ensure(int i, size_t bytes) {
    if (bytes <= cap[i]) return hipSuccess;
    if (p[i]) (void)hipFree(p[i]);
    p[i] = nullptr;
    cap[i] = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1u << 16);
    hipError_t e = hipMalloc(&p[i], want);
    if (e == hipSuccess) cap[i] = want;
    return e;
  }
};

// one buffer set per context; contexts may be driven from several host threads at once
// (Prefilter(devices=[...]), ctypes releases the GIL), so the map is guarded and holds
// the sets by pointer: a reference handed out stays valid while other contexts insert
std::mutex &bufs_mu() {
  static std::mutex m;
  return m;
}
std::unordered_map<mgp_ctx *, std::unique_ptr<PipeBufs>> &bufs_map() {
  static std::unordered_map<mgp_ctx *, std::unique_ptr<PipeBufs>> m;
  return m;
}
PipeBufs &bufs_of(mgp_ctx *ctx) {
  std::lock_guard<std::mutex> lk(bufs_mu());
  auto &p = bufs_map()[ctx];
  if (!p) p.reset(new PipeBufs());
  return *p;
}

enum { B_WORDS, B_OFFS, B_ORDER, B_CANDS, B_FIRST, B_WIT, B_PART, B_TABLES, B_NUM };

// Per-variable tables of the device candidate generator (mgp_fe_cands_kernel), so that
// its alias step is a lookup instead of the host generator's scans: asrc_off / asrc =
// the x == y alias sources of each variable (global variable index, CSR, alias order,
// sources inside the state), wcls[2g] / wcls[2g+1] = offset / length in wlist of the
// sorted local indices of the variables with g's width in its state
struct AliasTables {
  std::vector<uint32_t> asrc_off, asrc, wcls, wlist;
};
void alias_tables(uint32_t n_states, const uint64_t *vo, const uint32_t *vw, const uint64_t *ao,
                  const uint32_t *al, AliasTables &T) {
  const uint64_t nv = n_states ? vo[n_states] : 0;
  T.asrc_off.assign(nv + 1, 0u);
  T.wcls.assign(2 * nv + 2, 0u);
  T.asrc.clear();
  T.wlist.clear();
  for (uint32_t s = 0; s < n_states; ++s) {
    const uint64_t v0 = vo[s], V = vo[s + 1] - v0;
    for (uint64_t a = ao[s]; a < ao[s + 1]; ++a)
      if (al[2 * a] < V && al[2 * a + 1] < V) T.asrc_off[v0 + al[2 * a] + 1]++;
  }
  for (uint64_t g = 0; g < nv; ++g) T.asrc_off[g + 1] += T.asrc_off[g];
  T.asrc.assign(T.asrc_off[nv] ? T.asrc_off[nv] : 1u, 0u);
  std::vector<uint32_t> fill(T.asrc_off.begin(), T.asrc_off.end() - 1);
  std::vector<std::pair<uint32_t, uint32_t>> byw;
  for (uint32_t s = 0; s < n_states; ++s) {
    const uint64_t v0 = vo[s], V = vo[s + 1] - v0;
    for (uint64_t a = ao[s]; a < ao[s + 1]; ++a)
      if (al[2 * a] < V && al[2 * a + 1] < V) T.asrc[fill[v0 + al[2 * a]]++] = al[2 * a + 1];
    byw.clear();
    for (uint64_t v = 0; v < V; ++v) byw.push_back({vw[v0 + v], (uint32_t)v});
    std::sort(byw.begin(), byw.end());
    for (size_t i = 0; i < byw.size();) {
      size_t j = i;
      while (j < byw.size() && byw[j].first == byw[i].first) ++j;
      const uint32_t off = (uint32_t)T.wlist.size();
      for (size_t k = i; k < j; ++k) T.wlist.push_back(byw[k].second);
      for (size_t k = i; k < j; ++k) {
        T.wcls[2 * (v0 + byw[k].second)] = off;
        T.wcls[2 * (v0 + byw[k].second) + 1] = (uint32_t)(j - i);
      }
      i = j;
    }
  }
  if (T.wlist.empty()) T.wlist.push_back(0u);
}

// Lowered programs of recent states, keyed by the exact content of the state's GPU node
// list and constants (compared in full on a hit, so a hash collision can only cost a
// lowering).  The retry round of a batch re-checks its open states (solver.py
// _retry_round) and detection modules re-ask queries of states already pruned, so the
// same programs come back; a WalletLibrary program costs milliseconds to lower.
struct ProgCache {
  struct Entry {
    std::vector<uint8_t> key;
    std::shared_ptr<const std::vector<uint32_t>> words;  // shared: a hit outlives its eviction
    uint8_t status;
  };
  std::mutex mu;
  std::unordered_map<uint64_t, Entry> map;
  std::vector<uint64_t> fifo;
  size_t head = 0, bytes = 0;
  static constexpr size_t kMaxBytes = 256u << 20;
};
ProgCache &prog_cache() {
  static ProgCache c;
  return c;
}
uint64_t fnv(const uint8_t *p, size_t n, uint64_t h = 1469598103934665603ull) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {  // 8 bytes per step (keys are tens of KiB)
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x100000001B3ull;
    h ^= h >> 29;
  }
  for (; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

// Keys and hashes are built in parallel without the lock; the lock covers the lookups
// and, later, the inserts.  A hit holds its program by shared_ptr, so the copy into the
// batch's program vector runs in parallel outside the lock, and other threads (one host
// thread per device) lower their misses concurrently.
int lower_cached(const mgp_node *nodes, const uint64_t *noff, uint32_t n_states, const uint32_t *consts,
                 const uint64_t *coff, U32Buf &words, std::vector<uint64_t> &offs,
                 std::vector<uint8_t> &status) {
  ProgCache &C = prog_cache();
  // MGP_FE_TIMING=1: the stages of this call on stderr (profiling aid)
  static const bool timing = getenv("MGP_FE_TIMING") != nullptr;
  double tt = omp_get_wtime();
  auto stage = [&](const char *what) {
    if (!timing) return;
    const double now = omp_get_wtime();
    fprintf(stderr, "[lower_cached] %u states: %s %.3f ms\n", n_states, what, 1e3 * (now - tt));
    tt = now;
  };
  std::vector<std::vector<uint8_t>> keys(n_states);
  std::vector<uint64_t> hs(n_states);
#pragma omp parallel for schedule(dynamic, 8)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    const size_t nb = (noff[s + 1] - noff[s]) * sizeof(mgp_node), cb = (coff[s + 1] - coff[s]) * 32u;
    keys[s].resize(16 + nb + cb);
    const uint64_t hdr[2] = {noff[s + 1] - noff[s], coff[s + 1] - coff[s]};
    memcpy(keys[s].data(), hdr, 16);
    memcpy(keys[s].data() + 16, nodes + noff[s], nb);
    if (cb) memcpy(keys[s].data() + 16 + nb, consts + coff[s] * 8u, cb);
    hs[s] = fnv(keys[s].data(), keys[s].size());
  }
  std::vector<std::shared_ptr<const std::vector<uint32_t>>> hit(n_states);
  std::vector<uint8_t> hit_status(n_states, 0);
  std::vector<uint32_t> miss;
  {
    std::lock_guard<std::mutex> lk(C.mu);
    for (uint32_t s = 0; s < n_states; ++s) {
      auto it = C.map.find(hs[s]);
      if (it != C.map.end() && it->second.key == keys[s]) {
        hit[s] = it->second.words;
        hit_status[s] = it->second.status;
      } else {
        miss.push_back(s);
      }
    }
  }
  stage("keys + lookup");
  // the lowered misses, in a per-thread buffer kept across calls: a cold 1 024-state batch
  // is ~60 MB of programs, and releasing that every call showed as ~10 ms on the call's path
  // (capped, ADVICE r5: a buffer past kKeepWords -- a batch larger than the 1 024-state bench
  // call -- is released here rather than pinned by this thread for the life of the process)
  static thread_local U32Buf mw_keep;
  constexpr size_t kKeepWords = (size_t)32 << 20;  // 128 MB
  if (mw_keep.capacity() > kKeepWords) U32Buf().swap(mw_keep);
  U32Buf &mw = mw_keep;
  mw.clear();
  std::vector<uint64_t> mo;
  std::vector<uint8_t> mst;
  if (miss.size() == n_states) {  // a cold batch: its own node lists, no gathered copy
    const int rc = mgp_lower_vec(nodes, noff, n_states, consts, coff, 0, mw, mo, mst);
    if (rc != MGP_OK) return rc;
    stage("lower");
  } else if (!miss.empty()) {
    std::vector<mgp_node> mn;
    std::vector<uint32_t> mc;
    std::vector<uint64_t> mno(1, 0), mco(1, 0);
    for (uint32_t s : miss) {
      mn.insert(mn.end(), nodes + noff[s], nodes + noff[s + 1]);
      mc.insert(mc.end(), consts + coff[s] * 8u, consts + coff[s + 1] * 8u);
      mno.push_back(mn.size());
      mco.push_back(mc.size() / 8u);
    }
    if (mc.empty()) mc.assign(8, 0u);
    stage("gather misses");
    const int rc = mgp_lower_vec(mn.data(), mno.data(), (uint32_t)miss.size(), mc.data(), mco.data(), 0, mw, mo, mst);
    if (rc != MGP_OK) return rc;
    stage("lower");
  }
  offs.assign((size_t)n_states + 1, 0u);
  status.assign(n_states, 0u);
  std::vector<int64_t> mi(n_states, -1);
  for (size_t k = 0; k < miss.size(); ++k) mi[miss[k]] = (int64_t)k;
  for (uint32_t s = 0; s < n_states; ++s)
    offs[s + 1] = offs[s] + (mi[s] >= 0 ? mo[mi[s] + 1] - mo[mi[s]] : hit[s]->size());
  words.resize(offs[n_states]);
  // the new programs as cache entries (built in parallel, inserted under the lock below)
  std::vector<ProgCache::Entry> ents(miss.size());
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t s = 0; s < (int64_t)n_states; ++s) {
    if (mi[s] >= 0) {
      const size_t k = (size_t)mi[s];
      memcpy(words.data() + offs[s], mw.data() + mo[k], (mo[k + 1] - mo[k]) * 4u);
      status[s] = mst[k];
      ents[k].key = std::move(keys[s]);
      ents[k].words = std::make_shared<const std::vector<uint32_t>>(mw.begin() + mo[k], mw.begin() + mo[k + 1]);
      ents[k].status = mst[k];
    } else {
      memcpy(words.data() + offs[s], hit[s]->data(), hit[s]->size() * 4u);
      status[s] = hit_status[s];
    }
  }
  stage("copy out + cache entries");
  if (!miss.empty()) {
    // insert the new programs, evicting the oldest past the byte budget
    std::lock_guard<std::mutex> lk(C.mu);
    for (size_t k = 0; k < miss.size(); ++k) {
      const uint32_t s = miss[k];
      ProgCache::Entry &e = ents[k];
      const size_t sz = e.key.size() + e.words->size() * 4u;
      if (sz > ProgCache::kMaxBytes / 8) continue;
      auto it = C.map.find(hs[s]);
      if (it != C.map.end()) {
        C.bytes -= it->second.key.size() + it->second.words->size() * 4u;
        it->second = std::move(e);
      } else {
        C.map.emplace(hs[s], std::move(e));
        C.fifo.push_back(hs[s]);
      }
      C.bytes += sz;
      while (C.bytes > ProgCache::kMaxBytes && C.head < C.fifo.size()) {
        auto old = C.map.find(C.fifo[C.head++]);
        if (old == C.map.end()) continue;
        C.bytes -= old->second.key.size() + old->second.words->size() * 4u;
        C.map.erase(old);
      }
      if (C.head > 4096 && C.head * 2 > C.fifo.size()) {
        C.fifo.erase(C.fifo.begin(), C.fifo.begin() + (ptrdiff_t)C.head);
        C.head = 0;
      }
    }
  }
  stage("insert");
  return MGP_OK;
}  // (the batch's key copies and gathered programs are released here)

}  // namespace

extern "C" {

uint64_t mgp_program_cache_clear(void) {
  ProgCache &C = prog_cache();
  std::lock_guard<std::mutex> lk(C.mu);
  const uint64_t n = C.map.size();
  C.map.clear();
  C.fifo.clear();
  C.head = 0;
  C.bytes = 0;
  return n;
}

int mgp_program_cache_warm(const mgp_fe_batch *B) {
  if (!B) return MGP_E_ARG;
  const Arr gnodes = get(B, MGP_FE_GPU_NODES), gnoff = get(B, MGP_FE_GPU_NODE_OFF), consts = get(B, MGP_FE_CONSTS),
            coff = get(B, MGP_FE_CONST_OFF);
  const uint32_t n_states = (uint32_t)(gnoff.n ? gnoff.n - 1 : 0);
  if (n_states == 0) return MGP_OK;
  static const uint32_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  U32Buf words;
  std::vector<uint64_t> offs;
  std::vector<uint8_t> status;
  return lower_cached((const mgp_node *)gnodes.p, (const uint64_t *)gnoff.p, n_states,
                      consts.n ? (const uint32_t *)consts.p : zero8, (const uint64_t *)coff.p, words, offs, status);
}

void mgp_pipeline_release(mgp_ctx *ctx) {
  std::unique_ptr<PipeBufs> b;
  {
    std::lock_guard<std::mutex> lk(bufs_mu());
    auto &m = bufs_map();
    auto it = m.find(ctx);
    if (it == m.end()) return;
    b = std::move(it->second);
    m.erase(it);
  }
  if (!b) return;
  for (Slot &s : b->slot)
    if (s.busy && s.done) (void)hipEventSynchronize(s.done);  // nothing in flight reads what is freed
  for (int i = 0; i < 16; ++i)
    if (b->p[i]) (void)hipFree(b->p[i]);
  for (Slot &s : b->slot) {
    if (s.host) (void)hipHostFree(s.host);
    if (s.done) (void)hipEventDestroy(s.done);
  }
}

int mgp_pipeline_reserve(mgp_ctx *ctx, uint64_t host_bytes, uint64_t cand_bytes) {
  if (!ctx) return MGP_E_ARG;
  PipeBufs &D = bufs_of(ctx);
  hipError_t e = hipSuccess;
  for (Slot &s : D.slot)
    if (e == hipSuccess && !s.busy) e = s.ensure_host((size_t)host_bytes);
  if (e == hipSuccess && cand_bytes) e = D.ensure(B_CANDS, (size_t)cand_bytes);
  return e == hipSuccess ? MGP_OK : mgp_ctx_fail(ctx, MGP_E_HIP, hipGetErrorString(e));
}

int mgp_check_submit(mgp_ctx *ctx, const mgp_fe_batch *B, uint32_t n_cand, uint64_t seed, const uint32_t *fixed_pool,
                     uint32_t n_fixed, const uint64_t *parent_keys, const uint32_t *parent_vals,
                     const uint64_t *parent_off, const uint64_t *slot_keys, const uint32_t *xrows,
                     const uint8_t *xmask, uint32_t n_xrows, uint32_t n_xvars, uint32_t flags, int8_t *out_refuted,
                     uint32_t *out_n_vars, double *out_times, int32_t *out_ticket) {
  if (!ctx || !B || !out_refuted || !out_ticket || n_cand == 0 || (n_fixed && !fixed_pool))
    return mgp_ctx_fail(ctx, MGP_E_ARG, "bad argument to mgp_check_submit");
  *out_ticket = -1;
  double t = omp_get_wtime();
  auto lap = [&](int k) {
    const double now = omp_get_wtime();
    if (out_times) out_times[k] = 1e3 * (now - t);
    t = now;
  };
  const Arr nodes = get(B, MGP_FE_NODES), gnodes = get(B, MGP_FE_GPU_NODES), noff = get(B, MGP_FE_NODE_OFF),
            gnoff = get(B, MGP_FE_GPU_NODE_OFF),
            consts = get(B, MGP_FE_CONSTS), coff = get(B, MGP_FE_CONST_OFF), voff = get(B, MGP_FE_VAR_OFF),
            vwidth = get(B, MGP_FE_VAR_WIDTH), hoff = get(B, MGP_FE_HINT_OFF), hints = get(B, MGP_FE_HINTS),
            aoff = get(B, MGP_FE_ALIAS_OFF), aliases = get(B, MGP_FE_ALIASES), vkind = get(B, MGP_FE_VAR_KIND),
            skey = get(B, MGP_FE_STATE_KEY);
  const uint32_t n_states = (uint32_t)(noff.n ? noff.n - 1 : 0);
  if (out_n_vars) *out_n_vars = 1;
  if (n_states == 0) return MGP_OK;  // ticket -1: nothing to finish
  if (n_xrows && (!xrows || !xmask || n_xvars == 0))
    return mgp_ctx_fail(ctx, MGP_E_ARG, "explicit rows need xrows, xmask and n_xvars");
  PipeBufs &D0 = bufs_of(ctx);
  const int ticket = !D0.slot[0].busy ? 0 : (!D0.slot[1].busy ? 1 : -1);
  if (ticket < 0) return mgp_ctx_fail(ctx, MGP_E_ARG, "two batches in flight on this context: finish one first");
  Slot &SL = D0.slot[ticket];
  const uint64_t *vo = (const uint64_t *)voff.p;
  uint32_t n_vars = 1;
  for (uint32_t s = 0; s < n_states; ++s) n_vars = std::max<uint32_t>(n_vars, (uint32_t)(vo[s + 1] - vo[s]));
  if (out_n_vars) *out_n_vars = n_vars;
  static const uint32_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint32_t *cp = consts.n ? (const uint32_t *)consts.p : zero8;

  // 1. lower the GPU programs (programs lowered by an earlier call come from the cache)
  // the batch's programs, in the context's kept buffer (the same ~60 MB every call; a
  // batch still in flight has its copy in its own staging buffer)
  U32Buf &words = D0.words;
  words.clear();
  std::vector<uint64_t> offs;
  std::vector<uint8_t> status;
  int rc = lower_cached((const mgp_node *)gnodes.p, (const uint64_t *)gnoff.p, n_states, cp,
                        (const uint64_t *)coff.p, words, offs, status);
  if (rc != MGP_OK) return mgp_ctx_fail(ctx, rc, "lowering failed");
  static const bool timing = getenv("MGP_FE_TIMING") != nullptr;
  if (timing) fprintf(stderr, "[check_batch] %u states: lowered at %.3f ms\n", n_states, 1e3 * (omp_get_wtime() - t));
  std::vector<uint32_t> order(n_states), bounds(257), bslots(256);
  const int nb = mgp_plan_buckets(words.data(), offs.data(), n_states, order.data(), bounds.data(), bslots.data(),
                                  256);
  if (nb < 0) return mgp_ctx_fail(ctx, MGP_E_ARG, "bucket planning failed");
  uint32_t max_slots = 0;
  for (int b = 0; b < nb; ++b) max_slots = std::max(max_slots, bslots[b]);
  // candidate rows per state: the variables, plus the spill rows of programs with more
  // live values than LDS slots (include/mgp_ir.h); only the variables come back
  const uint32_t user_vars = n_vars;
  for (uint32_t s = 0; s < n_states; ++s)
    if (status[s] == MGP_ST_OK) n_vars = std::max<uint32_t>(n_vars, MGP_PROG_VARS(words.data() + offs[s]));
  // parent-witness rows: for every state whose parent witness is given, the parent's
  // value of each of its variable slots (matched by slot key = name, kind, aux)
  std::vector<int32_t> pidx(n_states, -1);
  std::vector<uint32_t> pvals;
  std::vector<uint8_t> pmask;
  if (parent_off && parent_keys && parent_vals && slot_keys) {
    uint32_t np = 0;
    for (uint32_t s = 0; s < n_states; ++s)
      if (parent_off[s + 1] > parent_off[s]) pidx[s] = (int32_t)np++;
    pvals.assign((size_t)np * n_vars * 8u, 0u);
    pmask.assign((size_t)np * n_vars, 0u);
    const uint32_t *vw = (const uint32_t *)vwidth.p;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t s = 0; s < (int64_t)n_states; ++s) {
      if (pidx[s] < 0) continue;
      std::unordered_map<uint64_t, uint64_t> at;
      for (uint64_t k = parent_off[s]; k < parent_off[s + 1]; ++k) at.emplace(parent_keys[k], k);
      for (uint64_t v = vo[s]; v < vo[s + 1]; ++v) {
        auto it = at.find(slot_keys[v]);
        if (it == at.end()) continue;
        uint32_t *d = &pvals[((size_t)pidx[s] * n_vars + (v - vo[s])) * 8u];
        memcpy(d, parent_vals + it->second * 8u, 32);
        const uint32_t w = vw[v];
        for (int l = 0; l < 8; ++l) {
          const int lo = 32 * l;
          d[l] &= (int)w >= lo + 32 ? 0xFFFFFFFFu : ((int)w <= lo ? 0u : ((1u << (w - lo)) - 1u));
        }
        pmask[(size_t)pidx[s] * n_vars + (v - vo[s])] = 1;
      }
    }
  }
  if (timing) fprintf(stderr, "[check_batch] %u states: step 1 done at %.3f ms\n", n_states, 1e3 * (omp_get_wtime() - t));
  lap(0);

  // 2. host UNSAT pre-check + variable domains
  U32Buf &dom = D0.dom;  // kept across calls; mgp_refute_domains zeroes what it writes
  dom.clear();
  if (flags & MGP_CHECK_NO_REFUTE) {
    memset(out_refuted, 0, n_states);
  } else {
    const bool want_dom = !(flags & MGP_CHECK_NO_DOMAINS);
    if (want_dom) dom.resize((size_t)vo[n_states] * 33u);
    rc = want_dom ? mgp_refute_domains((const mgp_node *)nodes.p, (const uint64_t *)noff.p, n_states, cp,
                                       (const uint64_t *)coff.p, vo, 0, out_refuted, dom.data())
                  : mgp_refute((const mgp_node *)nodes.p, (const uint64_t *)noff.p, n_states, cp,
                               (const uint64_t *)coff.p, 0, out_refuted);
    if (rc != MGP_OK) return mgp_ctx_fail(ctx, rc, "mgp_refute failed");
  }
  lap(1);

  // 3. upload
  void *stp = nullptr;
  int dev = 0;
  mgp_ctx_stream(ctx, &stp, &dev);
  hipStream_t st = (hipStream_t)stp;
  hipError_t e = hipSetDevice(dev);
  PipeBufs &D = D0;
  const size_t cand_bytes = (size_t)n_states * n_cand * n_vars * 32u;
  const uint32_t n_chunks = (n_cand + 63u) / 64u;
  // one table buffer: var_off | var_width | hint_off | hints | alias_off | aliases | const_off | consts |
  // fixed | parent_idx | pvals | pmask | var_kind | dom, each 256-B aligned
  // (mgp_fe_get counts elements of each array: u32 limbs for consts / hints / aliases)
  AliasTables AT;
  alias_tables(n_states, vo, (const uint32_t *)vwidth.p, (const uint64_t *)aoff.p, (const uint32_t *)aliases.p, AT);
  const size_t xr_words = (size_t)n_states * n_xrows * n_xvars;
  const size_t sizes[21] = {voff.n * 8, vwidth.n * 4, hoff.n * 8, hints.n * 4, aoff.n * 8, aliases.n * 4,
                            coff.n * 8, consts.n ? consts.n * 4 : 32, (size_t)n_fixed * 32,
                            (size_t)n_states * 4, pvals.size() * 4, pmask.size(), vkind.n, dom.size() * 4,
                            AT.asrc_off.size() * 4, AT.asrc.size() * 4, AT.wcls.size() * 4, AT.wlist.size() * 4,
                            skey.n * 8, xr_words * 32, xr_words};
  const void *srcs[21] = {voff.p, vwidth.p, hoff.p, hints.p, aoff.p, aliases.p, coff.p, cp, fixed_pool,
                          pidx.data(), pvals.data(), pmask.data(), vkind.p, dom.data(),
                          AT.asrc_off.data(), AT.asrc.data(), AT.wcls.data(), AT.wlist.data(),
                          skey.p, xrows, xmask};
  // one upload: programs | program offsets | launch order | the 21 tables, 256-B aligned
  const size_t pre[3] = {words.size() * 4u, offs.size() * 8u, (size_t)n_states * 4u};
  size_t at[25];
  at[0] = 0;
  for (int i = 0; i < 3; ++i) at[i + 1] = (at[i] + pre[i] + 255) & ~(size_t)255;
  for (int i = 0; i < 21; ++i) at[i + 4] = (at[i + 3] + sizes[i] + 255) & ~(size_t)255;
  const size_t up = at[24];
  const size_t wit_bytes = (size_t)n_states * n_vars * 32u, first_bytes = ((size_t)n_states * 4u + 255) & ~(size_t)255;
  const bool want_witness = !(flags & MGP_CHECK_NO_WITNESS);
  if (e == hipSuccess) e = SL.ensure_host(std::max(up, first_bytes + (want_witness ? wit_bytes : 0)));
  if (e == hipSuccess && !SL.done) e = hipEventCreateWithFlags(&SL.done, hipEventDisableTiming);
  if (e != hipSuccess) return mgp_ctx_fail(ctx, MGP_E_HIP, hipGetErrorString(e));
  uint8_t *H = (uint8_t *)SL.host;
  {  // the programs (hundreds of MB for contract states): copied in 4-MiB pieces in parallel
    const size_t piece = (size_t)4 << 20, n_pieces = (pre[0] + piece - 1) / piece;
    const uint8_t *src = (const uint8_t *)words.data();
#pragma omp parallel for schedule(dynamic, 1) if (n_pieces > 1)
    for (int64_t k = 0; k < (int64_t)n_pieces; ++k) {
      const size_t o = (size_t)k * piece;
      memcpy(H + at[0] + o, src + o, std::min(piece, pre[0] - o));
    }
  }
  memcpy(H + at[1], offs.data(), pre[1]);
  memcpy(H + at[2], order.data(), pre[2]);
  for (int i = 0; i < 21; ++i)
    if (sizes[i] && srcs[i]) memcpy(H + at[i + 3], srcs[i], sizes[i]);
  // a device buffer that must grow is freed and reallocated: let the other slot's batch,
  // which may still read it, drain first
  const size_t need[5] = {cand_bytes, (size_t)n_states * 4u, wit_bytes, (size_t)n_states * n_chunks * 4u, up};
  const int which[5] = {B_CANDS, B_FIRST, B_WIT, B_PART, B_TABLES};
  bool grow = false;
  for (int i = 0; i < 5; ++i) grow |= need[i] > D.cap[which[i]];
  if (grow && D.slot[1 - ticket].busy && e == hipSuccess) e = hipStreamSynchronize(st);
  for (int i = 0; i < 5 && e == hipSuccess; ++i) e = D.ensure(which[i], need[i]);
  if (e == hipSuccess) e = hipMemcpyAsync(D.p[B_TABLES], H, up, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return mgp_ctx_fail(ctx, MGP_E_HIP, hipGetErrorString(e));
  const uint8_t *base = (const uint8_t *)D.p[B_TABLES], *tb = base + at[3];
  auto T = [&](int i) { return tb + (at[i + 3] - at[3]); };
  e = mgp_launch_fe_cands(n_states, n_cand, n_vars, seed, (const uint64_t *)T(0), (const uint32_t *)T(1),
                          vkind.n ? (const uint8_t *)T(12) : nullptr, (const uint64_t *)T(2), (const uint32_t *)T(3),
                          (const uint64_t *)T(4), (const uint32_t *)T(5), (const uint64_t *)T(6),
                          (const uint32_t *)T(7), (const uint32_t *)T(8), n_fixed, (const int32_t *)T(9),
                          (const uint32_t *)T(10), (const uint8_t *)T(11),
                          dom.empty() ? nullptr : (const uint32_t *)T(13), (const uint32_t *)T(14),
                          (const uint32_t *)T(15), (const uint32_t *)T(16), (const uint32_t *)T(17),
                          skey.n ? (const uint64_t *)T(18) : nullptr, n_xrows ? (const uint32_t *)T(19) : nullptr,
                          n_xrows ? (const uint8_t *)T(20) : nullptr, n_xrows, n_xvars, (uint32_t *)D.p[B_CANDS], st);
  if (e == hipSuccess) e = hipMemsetAsync(D.p[B_PART], 0x7E, (size_t)n_states * n_chunks * 4u, st);
  if (e == hipSuccess)
    e = mgp_launch_eval((const uint32_t *)(base + at[0]), (const uint64_t *)(base + at[1]), n_states,
                        (const uint32_t *)D.p[B_CANDS], n_cand, n_vars, max_slots, (int32_t *)D.p[B_FIRST],
                        (uint32_t *)D.p[B_WIT], (int32_t *)D.p[B_PART], (const uint32_t *)(base + at[2]),
                        bounds.data(), bslots.data(), (uint32_t)nb, st);
  // one download into the slot's pinned buffer (the upload has been consumed by then: same stream)
  if (e == hipSuccess) e = hipMemcpyAsync(H, D.p[B_FIRST], (size_t)n_states * 4u, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && want_witness)
    e = hipMemcpyAsync(H + first_bytes, D.p[B_WIT], wit_bytes, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipEventRecord(SL.done, st);
  if (e != hipSuccess) return mgp_ctx_fail(ctx, MGP_E_HIP, hipGetErrorString(e));
  SL.busy = true;
  SL.want_witness = want_witness;
  SL.n_states = n_states;
  SL.n_vars = n_vars;
  SL.user_vars = user_vars;
  SL.first_bytes = first_bytes;
  SL.status.swap(status);
  *out_ticket = ticket;
  lap(2);
  return MGP_OK;
}

int mgp_check_finish(mgp_ctx *ctx, int32_t ticket, int32_t *out_first, uint32_t *out_witness, double *out_times) {
  if (!ctx) return MGP_E_ARG;
  if (ticket < 0) return MGP_OK;  // an empty batch
  PipeBufs &D = bufs_of(ctx);
  if (ticket > 1 || !D.slot[ticket].busy) return mgp_ctx_fail(ctx, MGP_E_ARG, "mgp_check_finish: no such batch in flight");
  Slot &SL = D.slot[ticket];
  if (!out_first || (out_witness && !SL.want_witness)) return mgp_ctx_fail(ctx, MGP_E_ARG, "bad argument to mgp_check_finish");
  double t = omp_get_wtime();
  hipError_t e = hipEventSynchronize(SL.done);
  SL.busy = false;  // the slot is free again whatever happened to its batch
  if (e != hipSuccess) return mgp_ctx_fail(ctx, MGP_E_HIP, hipGetErrorString(e));
  double now = omp_get_wtime();
  if (out_times) out_times[0] = 1e3 * (now - t);
  t = now;
  // 5. first-SAT words and the witnesses of the SAT states
  const uint8_t *H = (const uint8_t *)SL.host;
  const uint32_t n_states = SL.n_states;
  memcpy(out_first, H, (size_t)n_states * 4u);
  if (out_witness) {
    const uint32_t *w = (const uint32_t *)(H + SL.first_bytes);
    for (uint32_t s = 0; s < n_states; ++s)
      if (out_first[s] >= 0) memcpy(out_witness + (size_t)s * SL.user_vars * 8u, w + (size_t)s * SL.n_vars * 8u,
                                    (size_t)SL.user_vars * 32u);
  }
  for (uint32_t s = 0; s < n_states; ++s)
    if (SL.status[s] != MGP_ST_OK && out_first[s] >= 0) out_first[s] = MGP_UNDECIDED;  // never expected
  if (out_times) out_times[1] = 1e3 * (omp_get_wtime() - t);
  return MGP_OK;
}

int mgp_check_batch(mgp_ctx *ctx, const mgp_fe_batch *B, uint32_t n_cand, uint64_t seed, const uint32_t *fixed_pool,
                    uint32_t n_fixed, const uint64_t *parent_keys, const uint32_t *parent_vals,
                    const uint64_t *parent_off, const uint64_t *slot_keys, const uint32_t *xrows,
                    const uint8_t *xmask, uint32_t n_xrows, uint32_t n_xvars, uint32_t flags, int32_t *out_first,
                    uint32_t *out_witness, int8_t *out_refuted, uint32_t *out_n_vars, double *out_times) {
  if (!ctx || !B || !out_first || !out_refuted || n_cand == 0 || (n_fixed && !fixed_pool))
    return mgp_ctx_fail(ctx, MGP_E_ARG, "bad argument to mgp_check_batch");
  int32_t ticket = -1;
  double tm[5] = {0, 0, 0, 0, 0};
  int rc = mgp_check_submit(ctx, B, n_cand, seed, fixed_pool, n_fixed, parent_keys, parent_vals, parent_off,
                            slot_keys, xrows, xmask, n_xrows, n_xvars,
                            out_witness ? (flags & ~MGP_CHECK_NO_WITNESS) : (flags | MGP_CHECK_NO_WITNESS),
                            out_refuted, out_n_vars, tm, &ticket);
  if (rc == MGP_OK) rc = mgp_check_finish(ctx, ticket, out_first, out_witness, tm + 3);
  if (out_times) memcpy(out_times, tm, sizeof(tm));
  return rc;
}

// Test hook: the candidates mgp_check_batch evaluates, copied back in the device layout
// [state][var][half][cand] of 16-byte groups (tests compare them with mgp_make_candidates).
int mgp_fe_candidates(mgp_ctx *ctx, const mgp_fe_batch *B, uint32_t n_cand, uint32_t n_vars, uint64_t seed,
                      const uint32_t *fixed_pool, uint32_t n_fixed, const uint32_t *dom, const uint32_t *xrows,
                      const uint8_t *xmask, uint32_t n_xrows, uint32_t n_xvars, uint32_t *out) {
  if (!ctx || !B || !out || n_cand == 0 || n_vars == 0) return mgp_ctx_fail(ctx, MGP_E_ARG, "bad argument");
  const Arr noff = get(B, MGP_FE_NODE_OFF), consts = get(B, MGP_FE_CONSTS), coff = get(B, MGP_FE_CONST_OFF),
            voff = get(B, MGP_FE_VAR_OFF), vwidth = get(B, MGP_FE_VAR_WIDTH), hoff = get(B, MGP_FE_HINT_OFF),
            hints = get(B, MGP_FE_HINTS), aoff = get(B, MGP_FE_ALIAS_OFF), aliases = get(B, MGP_FE_ALIASES),
            vkind = get(B, MGP_FE_VAR_KIND), skey = get(B, MGP_FE_STATE_KEY);
  const uint32_t n_states = (uint32_t)(noff.n ? noff.n - 1 : 0);
  if (n_states == 0) return MGP_OK;
  if (n_xrows && (!xrows || !xmask || n_xvars == 0)) return mgp_ctx_fail(ctx, MGP_E_ARG, "bad explicit rows");
  void *stp = nullptr;
  int dev = 0;
  mgp_ctx_stream(ctx, &stp, &dev);
  hipStream_t st = (hipStream_t)stp;
  static const uint32_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  AliasTables AT;
  alias_tables(n_states, (const uint64_t *)voff.p, (const uint32_t *)vwidth.p, (const uint64_t *)aoff.p,
               (const uint32_t *)aliases.p, AT);
  const size_t xr_words = (size_t)n_states * n_xrows * n_xvars;
  const size_t sizes[18] = {voff.n * 8, vwidth.n * 4, hoff.n * 8, hints.n * 4, aoff.n * 8, aliases.n * 4,
                            coff.n * 8, consts.n ? consts.n * 4 : 32, (size_t)n_fixed * 32, vkind.n,
                            dom ? (size_t)((const uint64_t *)voff.p)[n_states] * 33u * 4u : 0,
                            AT.asrc_off.size() * 4, AT.asrc.size() * 4, AT.wcls.size() * 4, AT.wlist.size() * 4,
                            skey.n * 8, xr_words * 32, xr_words};
  const void *srcs[18] = {voff.p, vwidth.p, hoff.p, hints.p, aoff.p, aliases.p, coff.p,
                          consts.n ? consts.p : zero8, fixed_pool, vkind.p, dom,
                          AT.asrc_off.data(), AT.asrc.data(), AT.wcls.data(), AT.wlist.data(), skey.p, xrows, xmask};
  size_t at[19];
  at[0] = 0;
  for (int i = 0; i < 18; ++i) at[i + 1] = (at[i] + sizes[i] + 255) & ~(size_t)255;
  std::vector<uint8_t> stage(at[18]);
  for (int i = 0; i < 18; ++i)
    if (sizes[i] && srcs[i]) memcpy(stage.data() + at[i], srcs[i], sizes[i]);
  const size_t cb = (size_t)n_states * n_cand * n_vars * 32u;
  void *dt = nullptr, *dc = nullptr;
  hipError_t e = hipSetDevice(dev);
  if (e == hipSuccess) e = hipMalloc(&dt, at[18]);
  if (e == hipSuccess) e = hipMalloc(&dc, cb);
  if (e == hipSuccess) e = hipMemcpyAsync(dt, stage.data(), at[18], hipMemcpyHostToDevice, st);
  const uint8_t *tb = (const uint8_t *)dt;
  if (e == hipSuccess)
    e = mgp_launch_fe_cands(n_states, n_cand, n_vars, seed, (const uint64_t *)(tb + at[0]),
                            (const uint32_t *)(tb + at[1]), vkind.n ? (const uint8_t *)(tb + at[9]) : nullptr,
                            (const uint64_t *)(tb + at[2]),
                            (const uint32_t *)(tb + at[3]), (const uint64_t *)(tb + at[4]),
                            (const uint32_t *)(tb + at[5]), (const uint64_t *)(tb + at[6]),
                            (const uint32_t *)(tb + at[7]), (const uint32_t *)(tb + at[8]), n_fixed, nullptr,
                            nullptr, nullptr, dom ? (const uint32_t *)(tb + at[10]) : nullptr,
                            (const uint32_t *)(tb + at[11]), (const uint32_t *)(tb + at[12]),
                            (const uint32_t *)(tb + at[13]), (const uint32_t *)(tb + at[14]),
                            skey.n ? (const uint64_t *)(tb + at[15]) : nullptr,
                            n_xrows ? (const uint32_t *)(tb + at[16]) : nullptr,
                            n_xrows ? (const uint8_t *)(tb + at[17]) : nullptr, n_xrows, n_xvars, (uint32_t *)dc, st);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dc, cb, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (dt) (void)hipFree(dt);
  if (dc) (void)hipFree(dc);
  return e == hipSuccess ? MGP_OK : mgp_ctx_fail(ctx, MGP_E_HIP, hipGetErrorString(e));
}

}  // extern "C"
