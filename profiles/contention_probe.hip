// contention_probe.hip — throughput of the interpreter's per-uop instruction patterns
// with W co-resident waves per SIMD (profiles only; not part of libmgp).
//   hipcc --offload-arch=gfx950 -O3 -o build/contention_probe profiles/contention_probe.hip
// Every wave loops one pattern ITERS x 8 times; W waves per SIMD are forced by the LDS
// allocation (160 KiB per CU / 4W per single-wave block) and the kernel is long enough
// for all of them to be resident together.  Reported: SIMD-cycles per wave-pattern
// (kernel time x clock x 1024 SIMDs / patterns executed) and the per-wave latency.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 256
#define R8(x) x x x x x x x x

#define PREFETCH \
  "v_readlane_b32 s44, v108, s46\n v_readlane_b32 s45, v109, s46\n v_readlane_b32 s47, v110, s46\n" \
  "v_readlane_b32 s48, v111, s46\n v_readlane_b32 s49, v112, s46\n s_add_u32 s46, s46, 1\n s_and_b32 s46, s46, 31\n"
#define GIDX_ON "s_lshr_b32 s50, s52, 16\n s_set_gpr_idx_on s50, gpr_idx(SRC1)\n"
#define GIDX_OFF "s_set_gpr_idx_off\n"
#define ADD8 \
  "v_add_co_u32 v100, vcc, v100, v108\n v_addc_co_u32 v101, vcc, v101, v109, vcc\n" \
  "v_addc_co_u32 v102, vcc, v102, v110, vcc\n v_addc_co_u32 v103, vcc, v103, v111, vcc\n" \
  "v_addc_co_u32 v104, vcc, v104, v112, vcc\n v_addc_co_u32 v105, vcc, v105, v113, vcc\n" \
  "v_addc_co_u32 v106, vcc, v106, v114, vcc\n v_addc_co_u32 v107, vcc, v107, v115, vcc\n"
#define TAILMOV "s_mov_b64 s[54:55], s[44:45]\n s_mov_b64 s[56:57], s[48:49]\n"
#define SETPC "s_getpc_b64 s[42:43]\n s_add_u32 s42, s42, 12\n s_addc_u32 s43, s43, 0\n s_setpc_b64 s[42:43]\n"
#define SETPC_NOJUMP "s_getpc_b64 s[42:43]\n s_add_u32 s42, s42, 12\n s_addc_u32 s43, s43, 0\n s_nop 0\n"
#define LDSRD "ds_read_b128 v[116:119], v124\n ds_read_b128 v[120:123], v124 offset:1024\n s_waitcnt lgkmcnt(0)\n"
// next uop through the scalar cache: one s_load per uop into N, offset advanced in a 4 KiB window
#define SMEMPF "s_load_dwordx4 s[44:47], s[58:59], s40\n s_add_u32 s40, s40, 16\n s_and_b32 s40, s40, 0xff0\n"
// tail with the SMEM uop: wait, decode the first-handler offset, jump
#define SMEMTAIL "s_waitcnt lgkmcnt(0)\n s_and_b32 s54, s44, 0xffff\n s_lshl2_add_u32 s54, s54, s42\n s_mov_b64 s[56:57], s[46:47]\n"
// a pool constant into vB: 8 readlanes + 8 moves (the interpreter's const fetch)
#define CONST_RL \
  R8("v_readlane_b32 s48, v108, s46\n") \
  "v_mov_b32 v116, s48\n v_mov_b32 v117, s48\n v_mov_b32 v118, s48\n v_mov_b32 v119, s48\n" \
  "v_mov_b32 v120, s48\n v_mov_b32 v121, s48\n v_mov_b32 v122, s48\n v_mov_b32 v123, s48\n"
// a pool constant into vB through the scalar cache: one s_load_dwordx8, wait, 8 moves
#define CONST_SM \
  "s_load_dwordx8 s[24:31], s[58:59], 0x0\n s_waitcnt lgkmcnt(0)\n" \
  "v_mov_b32 v116, s24\n v_mov_b32 v117, s25\n v_mov_b32 v118, s26\n v_mov_b32 v119, s27\n" \
  "v_mov_b32 v120, s28\n v_mov_b32 v121, s29\n v_mov_b32 v122, s30\n v_mov_b32 v123, s31\n"
#define LDSWR "ds_write_b128 v124, v[100:103]\n ds_write_b128 v124, v[104:107] offset:1024\n"

#define CLOB                                                                                                   \
  "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",      \
      "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "s40",   \
      "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55",  \
      "s56", "s57", "s58", "s59", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "vcc", "memory"

#define PRE                                                                                       \
  "v_mov_b32 v108, %1\n v_mov_b32 v109, 3\n v_mov_b32 v110, 5\n v_mov_b32 v111, 7\n"              \
  "v_mov_b32 v112, 9\n v_mov_b32 v113, 11\n v_mov_b32 v114, 13\n v_mov_b32 v115, 17\n"            \
  "v_mov_b32 v100, 0\n v_mov_b32 v101, 0\n v_mov_b32 v102, 0\n v_mov_b32 v103, 0\n"              \
  "v_mov_b32 v104, 0\n v_mov_b32 v105, 0\n v_mov_b32 v106, 0\n v_mov_b32 v107, 0\n"              \
  "v_lshlrev_b32 v124, 4, %1\n s_mov_b32 s46, 0\n s_mov_b32 s52, 0\n s_mov_b64 s[40:41], -1\n"   \
  "s_mov_b64 s[58:59], %3\n s_mov_b32 s40, 0\n s_getpc_b64 s[42:43]\n"

extern __shared__ uint32_t lds_pad[];

template <int MODE>
__global__ __launch_bounds__(64) void cont_kernel(uint32_t *sink, const uint32_t *prog) {
  const uint32_t lane = threadIdx.x;
  lds_pad[lane] = lane;
  __syncthreads();
  uint32_t out = 0;
#define BODY(P)                                                                          \
  asm volatile(PRE "s_mov_b32 s53, %2\n 1:\n" R8(P)                                     \
               "s_sub_u32 s53, s53, 1\n s_cmp_lg_u32 s53, 0\n s_cbranch_scc1 1b\n v_mov_b32 %0, v100\n" \
               : "=v"(out)                                                               \
               : "v"(lane), "i"(ITERS), "s"(prog)                                        \
               : CLOB)
  if constexpr (MODE == 0) BODY(PREFETCH GIDX_ON ADD8 GIDX_OFF TAILMOV SETPC);   // XR_ADD uop
  if constexpr (MODE == 1) BODY(PREFETCH ADD8 TAILMOV SETPC);                    // without GPR-index mode
  if constexpr (MODE == 2) BODY(PREFETCH GIDX_ON ADD8 GIDX_OFF TAILMOV SETPC_NOJUMP);  // without the jump
  if constexpr (MODE == 3) BODY(GIDX_ON ADD8 GIDX_OFF TAILMOV SETPC);            // without the readlanes
  if constexpr (MODE == 4) BODY(ADD8);                                           // the arithmetic alone
  if constexpr (MODE == 5) BODY(GIDX_ON ADD8 GIDX_OFF);                          // arithmetic + index mode
  if constexpr (MODE == 6) BODY(PREFETCH ADD8);                                  // arithmetic + readlanes
  if constexpr (MODE == 7) BODY(ADD8 SETPC);                                     // arithmetic + jump
  if constexpr (MODE == 8) BODY(PREFETCH LDSRD ADD8 LDSWR TAILMOV SETPC);        // XS_ADD_S-like uop
  if constexpr (MODE == 9) BODY(SMEMPF ADD8 SMEMTAIL SETPC);                   // uop through SMEM, no readlanes
  if constexpr (MODE == 10) BODY(PREFETCH CONST_RL ADD8 TAILMOV SETPC);         // const operand by readlanes
  if constexpr (MODE == 11) BODY(PREFETCH CONST_SM ADD8 TAILMOV SETPC);         // const operand by s_load
  if constexpr (MODE == 12) BODY(SMEMPF CONST_SM ADD8 SMEMTAIL SETPC);          // both through SMEM
  if (out == 0xdeadbeefu) sink[blockIdx.x] = out;
}

template <int MODE>
static void run(const char *name, int waves) {
  const int blocks = 1024 * waves;
  const size_t lds = (160u * 1024u) / (4u * (unsigned)waves) - 256;
  uint32_t *sink, *prog;
  (void)hipMalloc(&sink, blocks * 4);
  (void)hipMalloc(&prog, 1 << 20);
  (void)hipMemset(prog, 0, 1 << 20);
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&cont_kernel<MODE>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(cont_kernel<MODE>, dim3(blocks), dim3(64), lds, 0, sink, prog);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (rep && ms < best) best = ms;
  }
  const double ghz = 2.4;
  const double patterns = (double)blocks * ITERS * 8;
  const double simd_cyc = best * 1e-3 * ghz * 1e9 * 1024 / patterns;
  printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"simd_cycles_per_wave_pattern\": %.1f, "
         "\"wave_latency_cycles\": %.1f}\n",
         name, waves, best, simd_cyc, simd_cyc * waves);
  (void)hipFree(sink);
  (void)hipFree(prog);
}

int main() {
  for (int w : {1, 2, 4}) {
    run<0>("XR_ADD uop: prefetch+gidx+add8+tail+setpc", w);
    run<1>("no gpr_idx", w);
    run<2>("no jump", w);
    run<3>("no readlanes", w);
    run<4>("add8 only", w);
    run<5>("add8 + gpr_idx", w);
    run<6>("add8 + readlanes", w);
    run<7>("add8 + setpc", w);
    run<8>("XS_ADD_S-like: prefetch+lds rd+add8+lds wr+tail+setpc", w);
    run<9>("uop via s_load (no readlanes) + add8 + setpc", w);
    run<10>("prefetch + const by 8 readlanes + add8 + setpc", w);
    run<11>("prefetch + const by s_load_dwordx8 + add8 + setpc", w);
    run<12>("uop and const via s_load + add8 + setpc", w);
  }
  return 0;
}
