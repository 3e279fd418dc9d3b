// mgp_runtime.cpp — C-ABI context, device-buffer management and launch
// plumbing for libmgp.so (include/mgp.h).  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <omp.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/mgp.h"

extern "C" {
hipError_t mgp_launch_eval(const uint32_t *words, const uint64_t *offs, uint32_t n_states, const uint32_t *cands,
                           uint32_t n_cand, uint32_t n_vars, uint32_t n_slots, int32_t *first_sat,
                           uint32_t *witness, int32_t *partial, const uint32_t *order,
                           const uint32_t *bucket_bounds, const uint32_t *bucket_slots, uint32_t n_buckets,
                           hipStream_t st);
hipError_t mgp_launch_fill(const uint32_t *words, const uint64_t *offs, uint32_t n_states, uint64_t state_base,
                           uint64_t seed, uint32_t *cands, uint32_t n_cand, uint32_t n_vars, hipStream_t st);
hipError_t mgp_launch_plant(uint32_t *cands, uint32_t n_cand, uint32_t n_vars, const uint32_t *pstate,
                            const uint32_t *pidx, const uint32_t *pwords, uint32_t n_plant, hipStream_t st);
hipError_t mgp_launch_transpose(const uint32_t *aos, uint32_t *soa, uint32_t n_states, uint32_t n_cand,
                                uint32_t n_vars, hipStream_t st);
hipError_t mgp_launch_keccak(const uint8_t *in, uint64_t n, uint32_t len, uint32_t stride, uint8_t *out,
                             hipStream_t st);
hipError_t mgp_launch_preimages(uint8_t *out, uint64_t first, uint64_t n, uint64_t seed, hipStream_t st);
hipError_t mgp_launch_valu_probe(uint32_t iters, uint32_t blocks, uint32_t *sink, hipStream_t st);
void mgp_desc_release(int dev, hipStream_t st);
}

namespace {

thread_local std::string g_err;

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1u << 20);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// maximum program size accepted by the host-pointer entry point
constexpr uint32_t kMaxSlotsHard = MGP_MAX_SLOTS;

}  // namespace

struct mgp_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  DevBuf words, offs, cand_aos, cand_soa, first, wit, partial, kin, kout, order;
};

namespace {

int fail(mgp_ctx *ctx, int code, const std::string &msg) {
  if (ctx) ctx->err = msg;
  g_err = msg;
  return code;
}
int hip_fail(mgp_ctx *ctx, hipError_t e, const char *where) {
  return fail(ctx, MGP_E_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define MGP_HIP(ctx, call)                                  \
  do {                                                      \
    hipError_t _e = (call);                                 \
    if (_e != hipSuccess) return hip_fail(ctx, _e, #call);  \
  } while (0)

// Validate caller-provided bytecode on the host so that a malformed program can
// never make the kernel read outside its LDS slots, constant pool or
// candidate rows.  Returns the max slot count over the batch or -1.
int64_t validate_programs(const uint32_t *w, const uint64_t *offs, uint32_t n_states, uint32_t n_vars,
                          std::string *why, uint32_t *rows_needed) {
  uint32_t max_slots = 0;
  *rows_needed = n_vars;
  const uint64_t total = offs[n_states];
  for (uint32_t s = 0; s < n_states; ++s) {
    const uint64_t o = offs[s], e = offs[s + 1];
    if (e < o || e > total || (o & 3u) || e - o < MGP_HDR_WORDS) {
      *why = "bad program offsets at state " + std::to_string(s);
      return -1;
    }
    const uint32_t n_ins = w[o], n_c = w[o + 1], n_sl = w[o + 2], st = w[o + 3];
    if ((st & 0xFFu) != MGP_ST_OK) continue;  // reported as undecided by the kernel
    if (n_sl > kMaxSlotsHard || (st >> 8) > n_vars ||
        o + MGP_HDR_WORDS + (uint64_t)(n_ins + 1) * MGP_INS_WORDS > e ||
        o + MGP_HDR_WORDS + (uint64_t)n_ins * MGP_INS_WORDS + (uint64_t)n_c * 8u > e) {
      *why = "bad program header at state " + std::to_string(s);
      return -1;
    }
    bool has_ret = false;
    for (uint32_t i = 0; i < n_ins; ++i) {
      const uint32_t *I = w + o + MGP_HDR_WORDS + (uint64_t)i * MGP_INS_WORDS;
      const uint32_t op = I[0] & 0xFFu, dst = ((I[0] >> 16) & 0xFFu) | ((I[3] & 0xFFu) << 8), fl = I[0] >> 24;
      const uint32_t opnds[3] = {I[1] & 0xFFFFu, I[1] >> 16, I[2] & 0xFFFFu};
      const bool bool_in = (op >= MGP_OP_BAND && op <= MGP_OP_BEQ) || op == MGP_OP_RET;
      const bool bool_out = (op >= MGP_OP_EQ && op <= MGP_OP_USUB_NOUDF) || (op >= MGP_OP_BAND && op <= MGP_OP_BEQ);
      if (op == MGP_OP_RET) has_ret = true;
      if (bool_out && dst >= MGP_BOOL_BITS) return *why = "bool dst", -1;
      if (!bool_out && op != MGP_OP_RET && (fl & MGP_INS_STORE) && dst >= n_sl) {
        *why = "slot dst out of range at state " + std::to_string(s);
        return -1;
      }
      for (int k = 0; k < 3; ++k) {
        const uint32_t o16 = opnds[k];
        const bool is_bool = bool_in || (op == MGP_OP_ITE && k == 0);
        if (is_bool) {
          if (o16 >= MGP_BOOL_BITS) return *why = "bool operand", -1;
          continue;
        }
        const uint32_t kind = o16 >> 14, idx = o16 & 0x3FFFu;
        if ((kind == MGP_K_SLOT && idx >= std::max(n_sl, 1u) && o16 != 0) ||
            (kind == MGP_K_CONST && idx >= n_c) || (kind == MGP_K_VAR && idx >= n_vars)) {
          *why = "operand out of range at state " + std::to_string(s);
          return -1;
        }
      }
    }
    if (!has_ret) {
      *why = "program without RET at state " + std::to_string(s);
      return -1;
    }
    max_slots = std::max(max_slots, n_sl);
    *rows_needed = std::max<uint32_t>(*rows_needed, MGP_PROG_VARS(w + o));  // spill rows past the variables
  }
  return (int64_t)max_slots;
}

}  // namespace

extern "C" {

const char *mgp_version(void) { return "mgp 0.1 (gfx950)"; }

int mgp_set_thread_omp(int n) {
  const int old = omp_get_max_threads();
  if (n > 0) omp_set_num_threads(n);
  return old;
}

int mgp_device_count(int *out) {
  if (!out) return MGP_E_ARG;
  hipError_t e = hipGetDeviceCount(out);
  if (e != hipSuccess) {
    *out = 0;
    return hip_fail(nullptr, e, "hipGetDeviceCount");
  }
  return MGP_OK;
}

int mgp_create(int device, mgp_ctx **out) {
  if (!out) return fail(nullptr, MGP_E_ARG, "out is NULL");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hipGetDeviceCount");
  if (device < 0 || device >= n) return fail(nullptr, MGP_E_ARG, "device index out of range");
  mgp_ctx *c = new (std::nothrow) mgp_ctx();
  if (!c) return fail(nullptr, MGP_E_NOMEM, "context allocation");
  c->device = device;
  e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return hip_fail(nullptr, e, "mgp_create");
  }
  *out = c;
  return MGP_OK;
}

void mgp_pipeline_release(mgp_ctx *ctx);  // mgp_pipeline.cpp

int mgp_ctx_stream(mgp_ctx *ctx, void **stream, int *device) {
  if (!ctx) return MGP_E_ARG;
  *stream = ctx->stream;
  *device = ctx->device;
  return MGP_OK;
}

int mgp_ctx_fail(mgp_ctx *ctx, int code, const char *msg) { return fail(ctx, code, msg ? msg : ""); }

void mgp_destroy(mgp_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  mgp_pipeline_release(ctx);
  for (DevBuf *b : {&ctx->words, &ctx->offs, &ctx->cand_aos, &ctx->cand_soa, &ctx->first, &ctx->wit,
                    &ctx->partial, &ctx->kin, &ctx->kout, &ctx->order})
    b->release();
  if (ctx->stream) {
    mgp_desc_release(ctx->device, ctx->stream);  // the stream's launch-descriptor buffer
    (void)hipStreamDestroy(ctx->stream);
  }
  delete ctx;
}

const char *mgp_last_error(mgp_ctx *ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int mgp_eval_batch(mgp_ctx *ctx, const uint32_t *prog_words, const uint64_t *prog_offsets, uint32_t n_states,
                   const uint32_t *cand_words, uint32_t n_cand, uint32_t n_vars, int32_t *out_first_sat,
                   uint32_t *out_witness) {
  if (!ctx) return fail(nullptr, MGP_E_ARG, "ctx is NULL");
  if (n_states == 0) return MGP_OK;
  if (!prog_words || !prog_offsets || !cand_words || !out_first_sat || n_cand == 0 || n_vars == 0)
    return fail(ctx, MGP_E_ARG, "NULL buffer or zero n_cand/n_vars");
  std::string why;
  uint32_t rows = n_vars;
  const int64_t slots = validate_programs(prog_words, prog_offsets, n_states, n_vars, &why, &rows);
  if (slots < 0) return fail(ctx, MGP_E_ARG, why);
  MGP_HIP(ctx, hipSetDevice(ctx->device));
  // programs with spill slots (include/mgp_ir.h) use candidate rows past the caller's
  // n_vars as scratch: the device block gets `rows` rows per candidate, the extra ones
  // left for the program to write
  std::vector<uint32_t> padded;
  const uint32_t user_vars = n_vars;
  if (rows > n_vars) {
    padded.assign((size_t)n_states * n_cand * rows * 8u, 0u);
    for (size_t sc = 0; sc < (size_t)n_states * n_cand; ++sc)
      memcpy(padded.data() + sc * rows * 8u, cand_words + sc * n_vars * 8u, (size_t)n_vars * 32u);
    cand_words = padded.data();
    n_vars = rows;
  }
  const uint64_t total_words = prog_offsets[n_states];
  const size_t cand_bytes = (size_t)n_states * n_cand * n_vars * 32u;
  const uint32_t n_chunks = (n_cand + 63u) / 64u;
  MGP_HIP(ctx, ctx->words.ensure(total_words * 4u));
  MGP_HIP(ctx, ctx->offs.ensure(((size_t)n_states + 1) * 8u));
  MGP_HIP(ctx, ctx->cand_aos.ensure(cand_bytes));
  MGP_HIP(ctx, ctx->cand_soa.ensure(cand_bytes));
  MGP_HIP(ctx, ctx->first.ensure((size_t)n_states * 4u));
  MGP_HIP(ctx, ctx->wit.ensure((size_t)n_states * n_vars * 32u));
  MGP_HIP(ctx, ctx->partial.ensure((size_t)n_states * n_chunks * 4u));
  hipStream_t st = ctx->stream;
  MGP_HIP(ctx, hipMemcpyAsync(ctx->words.p, prog_words, total_words * 4u, hipMemcpyHostToDevice, st));
  MGP_HIP(ctx, hipMemcpyAsync(ctx->offs.p, prog_offsets, ((size_t)n_states + 1) * 8u, hipMemcpyHostToDevice, st));
  MGP_HIP(ctx, hipMemcpyAsync(ctx->cand_aos.p, cand_words, cand_bytes, hipMemcpyHostToDevice, st));
  MGP_HIP(ctx, mgp_launch_transpose((const uint32_t *)ctx->cand_aos.p, (uint32_t *)ctx->cand_soa.p, n_states,
                                    n_cand, n_vars, st));
  std::vector<uint32_t> order(n_states), bounds(kMaxSlotsHard + 2), bslots(kMaxSlotsHard + 1);
  const int nb = mgp_plan_buckets(prog_words, prog_offsets, n_states, order.data(), bounds.data(), bslots.data(),
                                  kMaxSlotsHard + 1);
  if (nb < 0) return fail(ctx, MGP_E_ARG, "bucket planning failed");
  MGP_HIP(ctx, ctx->order.ensure((size_t)n_states * 4u));
  MGP_HIP(ctx, hipMemcpyAsync(ctx->order.p, order.data(), (size_t)n_states * 4u, hipMemcpyHostToDevice, st));
  // partial results start as an invalid value: a chunk that leaves none shows up as
  // MGP_EVAL_FAULT instead of reusing a previous batch's result
  MGP_HIP(ctx, hipMemsetAsync(ctx->partial.p, 0x7E, (size_t)n_states * n_chunks * 4u, st));
  MGP_HIP(ctx, mgp_launch_eval((const uint32_t *)ctx->words.p, (const uint64_t *)ctx->offs.p, n_states,
                               (const uint32_t *)ctx->cand_soa.p, n_cand, n_vars, (uint32_t)slots,
                               (int32_t *)ctx->first.p, (uint32_t *)ctx->wit.p, (int32_t *)ctx->partial.p,
                               (const uint32_t *)ctx->order.p, bounds.data(), bslots.data(), (uint32_t)nb, st));
  MGP_HIP(ctx, hipMemcpyAsync(out_first_sat, ctx->first.p, (size_t)n_states * 4u, hipMemcpyDeviceToHost, st));
  MGP_HIP(ctx, hipStreamSynchronize(st));
  if (out_witness) {
    // copy back witness rows only for SAT states (others left untouched)
    std::vector<uint32_t> w((size_t)n_states * n_vars * 8u);
    MGP_HIP(ctx, hipMemcpyAsync(w.data(), ctx->wit.p, w.size() * 4u, hipMemcpyDeviceToHost, st));
    MGP_HIP(ctx, hipStreamSynchronize(st));
    for (uint32_t s = 0; s < n_states; ++s)
      if (out_first_sat[s] >= 0)
        memcpy(out_witness + (size_t)s * user_vars * 8u, w.data() + (size_t)s * n_vars * 8u, user_vars * 32u);
  }
  return MGP_OK;
}

int mgp_eval_batch_dev(const uint32_t *d_prog_words, const uint64_t *d_prog_offsets, uint32_t n_states,
                       const uint32_t *d_cands, uint32_t n_cand, uint32_t n_vars, uint32_t n_slots,
                       int32_t *d_first_sat, uint32_t *d_witness, int32_t *d_scratch, const uint32_t *d_order,
                       const uint32_t *bucket_bounds, const uint32_t *bucket_slots, uint32_t n_buckets,
                       void *stream) {
  if (n_states == 0) return MGP_OK;
  if (!d_prog_words || !d_prog_offsets || !d_cands || !d_first_sat || !d_scratch || n_cand == 0 || n_vars == 0 ||
      n_slots > kMaxSlotsHard || (n_buckets && (!d_order || !bucket_bounds || !bucket_slots)))
    return fail(nullptr, MGP_E_ARG, "bad argument to mgp_eval_batch_dev");
  for (uint32_t b = 0; b < n_buckets; ++b)
    if (bucket_slots[b] > kMaxSlotsHard || bucket_bounds[b] > bucket_bounds[b + 1] || bucket_bounds[b + 1] > n_states)
      return fail(nullptr, MGP_E_ARG, "bad bucket plan");
  hipError_t e = mgp_launch_eval(d_prog_words, d_prog_offsets, n_states, d_cands, n_cand, n_vars, n_slots,
                                 d_first_sat, d_witness, d_scratch, d_order, bucket_bounds, bucket_slots, n_buckets,
                                 (hipStream_t)stream);
  return e == hipSuccess ? MGP_OK : hip_fail(nullptr, e, "mgp_eval_batch_dev");
}

int mgp_fill_candidates_dev(const uint32_t *d_prog_words, const uint64_t *d_prog_offsets, uint32_t n_states,
                            uint64_t state_base, uint64_t seed, uint32_t *d_cands, uint32_t n_cand,
                            uint32_t n_vars, void *stream) {
  if (!d_prog_words || !d_prog_offsets || !d_cands) return fail(nullptr, MGP_E_ARG, "NULL device pointer");
  hipError_t e = mgp_launch_fill(d_prog_words, d_prog_offsets, n_states, state_base, seed, d_cands, n_cand, n_vars,
                                 (hipStream_t)stream);
  return e == hipSuccess ? MGP_OK : hip_fail(nullptr, e, "mgp_fill_candidates_dev");
}

int mgp_plant_candidates_dev(uint32_t *d_cands, uint32_t n_states, uint32_t n_cand, uint32_t n_vars,
                             const uint32_t *d_plant_state, const uint32_t *d_plant_idx,
                             const uint32_t *d_plant_words, uint32_t n_plant, void *stream) {
  (void)n_states;
  if (n_plant && (!d_cands || !d_plant_state || !d_plant_idx || !d_plant_words))
    return fail(nullptr, MGP_E_ARG, "NULL device pointer");
  hipError_t e = mgp_launch_plant(d_cands, n_cand, n_vars, d_plant_state, d_plant_idx, d_plant_words, n_plant,
                                  (hipStream_t)stream);
  return e == hipSuccess ? MGP_OK : hip_fail(nullptr, e, "mgp_plant_candidates_dev");
}

int mgp_keccak256_dev(const uint8_t *d_in, uint64_t n, uint32_t len, uint32_t stride, uint8_t *d_out32,
                      void *stream) {
  if (n && (!d_in || !d_out32 || stride < len)) return fail(nullptr, MGP_E_ARG, "bad keccak arguments");
  hipError_t e = mgp_launch_keccak(d_in, n, len, stride, d_out32, (hipStream_t)stream);
  return e == hipSuccess ? MGP_OK : hip_fail(nullptr, e, "mgp_keccak256_dev");
}

int mgp_keccak256_batch(mgp_ctx *ctx, const uint8_t *in, uint64_t n, uint32_t len, uint32_t stride,
                        uint8_t *out32) {
  if (!ctx) return fail(nullptr, MGP_E_ARG, "ctx is NULL");
  if (n == 0) return MGP_OK;
  if (!in || !out32 || stride < len) return fail(ctx, MGP_E_ARG, "bad keccak arguments");
  MGP_HIP(ctx, hipSetDevice(ctx->device));
  // pack to a dense, 16-byte aligned device layout (stride rounded up to 16)
  const uint32_t dstride = (len + 15u) & ~15u;
  const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(n, (1ull << 30) / std::max(dstride, 16u)));
  MGP_HIP(ctx, ctx->kin.ensure((size_t)chunk * std::max(dstride, 16u)));
  MGP_HIP(ctx, ctx->kout.ensure((size_t)chunk * 32u));
  std::vector<uint8_t> stage((size_t)chunk * dstride);
  hipStream_t st = ctx->stream;
  for (uint64_t base = 0; base < n; base += chunk) {
    const uint64_t m = std::min(chunk, n - base);
    for (uint64_t i = 0; i < m; ++i) memcpy(stage.data() + i * dstride, in + (base + i) * stride, len);
    if (m * dstride) MGP_HIP(ctx, hipMemcpyAsync(ctx->kin.p, stage.data(), m * dstride, hipMemcpyHostToDevice, st));
    MGP_HIP(ctx, mgp_launch_keccak((const uint8_t *)ctx->kin.p, m, len, dstride ? dstride : 16u,
                                   (uint8_t *)ctx->kout.p, st));
    MGP_HIP(ctx, hipMemcpyAsync(out32 + base * 32u, ctx->kout.p, m * 32u, hipMemcpyDeviceToHost, st));
    MGP_HIP(ctx, hipStreamSynchronize(st));
  }
  return MGP_OK;
}

int mgp_fill_mapping_preimages_dev(uint8_t *d_out64, uint64_t first, uint64_t n, uint64_t seed, void *stream) {
  if (n && !d_out64) return fail(nullptr, MGP_E_ARG, "NULL device pointer");
  hipError_t e = mgp_launch_preimages(d_out64, first, n, seed, (hipStream_t)stream);
  return e == hipSuccess ? MGP_OK : hip_fail(nullptr, e, "mgp_fill_mapping_preimages_dev");
}

int mgp_probe_valu_dev(uint32_t iters, uint32_t blocks, uint32_t *d_sink, uint64_t *ops_out, void *stream) {
  if (!d_sink || blocks == 0) return fail(nullptr, MGP_E_ARG, "bad probe arguments");
  if (ops_out) *ops_out = (uint64_t)blocks * 256u * iters * 64u * 8u;
  hipError_t e = mgp_launch_valu_probe(iters, blocks, d_sink, (hipStream_t)stream);
  return e == hipSuccess ? MGP_OK : hip_fail(nullptr, e, "mgp_probe_valu_dev");
}

}  // extern "C"
