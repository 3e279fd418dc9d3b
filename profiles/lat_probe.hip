// lat_probe.hip — per-wave issue latency of the instruction patterns the interpreter's
// handlers are built from (profiles only; not part of libmgp).
//   hipcc --offload-arch=gfx950 -O3 -o build/lat_probe profiles/lat_probe.hip && ./build/lat_probe
// Each mode repeats one pattern REP times inside the wave and reports the median over
// waves of shader clocks (s_memtime) per pattern, with W resident waves per SIMD forced
// by the LDS allocation (160 KiB per CU / (4 W) per single-wave block).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define REP 64
#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

// 256-bit add, vA += vB, carry through VCC (the interpreter's BIN_LIMBS ADD)
#define ADD256 \
  "v_add_co_u32 v100, vcc, v100, v108\n v_addc_co_u32 v101, vcc, v101, v109, vcc\n" \
  "v_addc_co_u32 v102, vcc, v102, v110, vcc\n v_addc_co_u32 v103, vcc, v103, v111, vcc\n" \
  "v_addc_co_u32 v104, vcc, v104, v112, vcc\n v_addc_co_u32 v105, vcc, v105, v113, vcc\n" \
  "v_addc_co_u32 v106, vcc, v106, v114, vcc\n v_addc_co_u32 v107, vcc, v107, v115, vcc\n"
// two independent 256-bit adds interleaved (carries in VCC and s[40:41])
#define ADD256X2 \
  "v_add_co_u32 v100, vcc, v100, v108\n v_add_co_u32 v116, s[40:41], v116, v108\n" \
  "v_addc_co_u32 v101, vcc, v101, v109, vcc\n v_addc_co_u32 v117, s[40:41], v117, v109, s[40:41]\n" \
  "v_addc_co_u32 v102, vcc, v102, v110, vcc\n v_addc_co_u32 v118, s[40:41], v118, v110, s[40:41]\n" \
  "v_addc_co_u32 v103, vcc, v103, v111, vcc\n v_addc_co_u32 v119, s[40:41], v119, v111, s[40:41]\n" \
  "v_addc_co_u32 v104, vcc, v104, v112, vcc\n v_addc_co_u32 v120, s[40:41], v120, v112, s[40:41]\n" \
  "v_addc_co_u32 v105, vcc, v105, v113, vcc\n v_addc_co_u32 v121, s[40:41], v121, v113, s[40:41]\n" \
  "v_addc_co_u32 v106, vcc, v106, v114, vcc\n v_addc_co_u32 v122, s[40:41], v122, v114, s[40:41]\n" \
  "v_addc_co_u32 v107, vcc, v107, v115, vcc\n v_addc_co_u32 v123, s[40:41], v123, v115, s[40:41]\n"
// 8 independent full-rate ops
#define IND8 \
  "v_xor_b32 v100, v100, v108\n v_xor_b32 v101, v101, v108\n v_xor_b32 v102, v102, v108\n" \
  "v_xor_b32 v103, v103, v108\n v_xor_b32 v104, v104, v108\n v_xor_b32 v105, v105, v108\n" \
  "v_xor_b32 v106, v106, v108\n v_xor_b32 v107, v107, v108\n"
// 8 dependent full-rate ops (one chain)
#define DEP8 \
  "v_xor_b32 v100, v100, v108\n v_xor_b32 v100, v100, v109\n v_xor_b32 v100, v100, v110\n" \
  "v_xor_b32 v100, v100, v111\n v_xor_b32 v100, v100, v112\n v_xor_b32 v100, v100, v113\n" \
  "v_xor_b32 v100, v100, v114\n v_xor_b32 v100, v100, v115\n"
// a jump to the next instruction through s_setpc (the dispatch tail)
#define SETPC \
  "s_getpc_b64 s[42:43]\n s_add_u32 s42, s42, 12\n s_addc_u32 s43, s43, 0\n s_setpc_b64 s[42:43]\n"
// the dispatch tail as the interpreter has it: 5 readlanes + counter + 2 moves + setpc
#define DISPATCH \
  "v_readlane_b32 s44, v108, s46\n v_readlane_b32 s45, v109, s46\n v_readlane_b32 s47, v110, s46\n" \
  "v_readlane_b32 s48, v111, s46\n v_readlane_b32 s49, v112, s46\n s_add_u32 s46, s46, 1\n" \
  "s_and_b32 s46, s46, 63\n s_mov_b64 s[50:51], s[44:45]\n s_mov_b64 s[52:53], s[48:49]\n" SETPC
// VALU -> SGPR -> SALU dependency
#define RDL "v_readlane_b32 s44, v100, s46\n s_add_u32 s46, s44, 1\n s_and_b32 s46, s46, 63\n"
// LDS round trip: two 16-B stores, two 16-B loads of the same slot, wait
#define LDSRT \
  "ds_write_b128 v124, v[100:103]\n ds_write_b128 v124, v[104:107] offset:1024\n" \
  "ds_read_b128 v[108:111], v124\n ds_read_b128 v[112:115], v124 offset:1024\n s_waitcnt lgkmcnt(0)\n"
// LDS load + wait only
#define LDSRD "ds_read_b128 v[108:111], v124\n ds_read_b128 v[112:115], v124 offset:1024\n s_waitcnt lgkmcnt(0)\n"
// dependent v_mad_u64_u32 chain
#define MAD "v_mad_u64_u32 v[100:101], s[40:41], v100, v108, v[100:101]\n"
#define MAD4I \
  "v_mad_u64_u32 v[100:101], s[40:41], v102, v108, v[100:101]\n" \
  "v_mad_u64_u32 v[102:103], s[40:41], v104, v108, v[102:103]\n" \
  "v_mad_u64_u32 v[104:105], s[40:41], v106, v108, v[104:105]\n" \
  "v_mad_u64_u32 v[106:107], s[40:41], v100, v108, v[106:107]\n"
// GPR-index-mode moves of 8 limbs (fetch of a register-bank operand)
#define GPRIDX \
  "s_set_gpr_idx_on s47, gpr_idx(SRC0)\n v_mov_b32 v100, v108\n v_mov_b32 v101, v109\n" \
  "v_mov_b32 v102, v110\n v_mov_b32 v103, v111\n v_mov_b32 v104, v112\n v_mov_b32 v105, v113\n" \
  "v_mov_b32 v106, v114\n v_mov_b32 v107, v115\n s_set_gpr_idx_off\n"
// compare -> VCC -> SALU test -> not-taken branch
#define CMPBR "v_cmp_eq_u32 vcc, v100, v108\n s_cmp_eq_u64 vcc, 0\n s_cbranch_scc1 1f\n 1:\n"
// a pure SALU op chain
#define SALU8 R8("s_add_u32 s46, s46, 1\n")
// v_cndmask from an SGPR mask (8 limbs)
#define CND8 \
  "v_cndmask_b32_e64 v100, v100, v108, s[40:41]\n v_cndmask_b32_e64 v101, v101, v109, s[40:41]\n" \
  "v_cndmask_b32_e64 v102, v102, v110, s[40:41]\n v_cndmask_b32_e64 v103, v103, v111, s[40:41]\n" \
  "v_cndmask_b32_e64 v104, v104, v112, s[40:41]\n v_cndmask_b32_e64 v105, v105, v113, s[40:41]\n" \
  "v_cndmask_b32_e64 v106, v106, v114, s[40:41]\n v_cndmask_b32_e64 v107, v107, v115, s[40:41]\n"

#define CLOB                                                                                                   \
  "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",      \
      "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "s40",   \
      "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "vcc", "memory"

#define PRE                                                                                       \
  "v_mov_b32 v108, %0\n v_mov_b32 v109, 3\n v_mov_b32 v110, 5\n v_mov_b32 v111, 7\n"              \
  "v_mov_b32 v112, 9\n v_mov_b32 v113, 11\n v_mov_b32 v114, 13\n v_mov_b32 v115, 17\n"            \
  "v_mov_b32 v100, 0\n v_mov_b32 v101, 0\n v_mov_b32 v102, 0\n v_mov_b32 v103, 0\n"              \
  "v_mov_b32 v104, 0\n v_mov_b32 v105, 0\n v_mov_b32 v106, 0\n v_mov_b32 v107, 0\n"              \
  "v_mov_b32 v116, 0\n v_mov_b32 v117, 0\n v_mov_b32 v118, 0\n v_mov_b32 v119, 0\n"              \
  "v_mov_b32 v120, 0\n v_mov_b32 v121, 0\n v_mov_b32 v122, 0\n v_mov_b32 v123, 0\n"              \
  "v_lshlrev_b32 v124, 4, %0\n s_mov_b32 s46, 0\n s_mov_b32 s47, 0\n s_mov_b64 s[40:41], -1\n"

extern __shared__ uint32_t lds_pad[];

template <int MODE>
__global__ __launch_bounds__(64) void lat_kernel(uint64_t *clk, uint32_t *sink) {
  uint64_t t0, t1;
  const uint32_t lane = threadIdx.x;
  lds_pad[lane] = lane;
  __syncthreads();
#define BODY(P)                                                                                   \
  asm volatile(PRE "s_waitcnt lgkmcnt(0)\n s_memtime %1\n s_waitcnt lgkmcnt(0)\n" R64(P)          \
               "s_memtime %2\n s_waitcnt lgkmcnt(0)\n v_mov_b32 %3, v100\n"                        \
               : "+v"(sink_v), "=s"(t0), "=s"(t1), "=v"(out)                                       \
               : "v"(lane)                                                                          \
               : CLOB)
  uint32_t sink_v = lane, out = 0;
  (void)sink_v;
  if constexpr (MODE == 0) BODY(ADD256);
  if constexpr (MODE == 1) BODY(ADD256X2);
  if constexpr (MODE == 2) BODY(IND8);
  if constexpr (MODE == 3) BODY(DEP8);
  if constexpr (MODE == 4) BODY(SETPC);
  if constexpr (MODE == 5) BODY(DISPATCH);
  if constexpr (MODE == 6) BODY(RDL);
  if constexpr (MODE == 7) BODY(LDSRT);
  if constexpr (MODE == 8) BODY(LDSRD);
  if constexpr (MODE == 9) BODY(MAD);
  if constexpr (MODE == 10) BODY(MAD4I);
  if constexpr (MODE == 11) BODY(GPRIDX);
  if constexpr (MODE == 12) BODY(CMPBR);
  if constexpr (MODE == 13) BODY(SALU8);
  if constexpr (MODE == 14) BODY(CND8);
  if (out == 0xdeadbeefu) sink[blockIdx.x] = out;
  if (lane == 0) clk[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(const char *name, int per_rep_insts, int waves, uint64_t *d_clk, uint32_t *d_sink) {
  const int blocks = 1024 * waves;
  const size_t lds = (160u * 1024u) / (4u * (unsigned)waves) - 64;
  hipFuncSetAttribute(reinterpret_cast<const void *>(&lat_kernel<MODE>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL(lat_kernel<MODE>, dim3(blocks), dim3(64), lds, 0, d_clk, d_sink);
  hipDeviceSynchronize();
  std::vector<uint64_t> h(blocks);
  hipMemcpy(h.data(), d_clk, blocks * sizeof(uint64_t), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  const double med = (double)h[blocks / 2] / REP;
  printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"clk_per_pattern\": %.1f, \"clk_per_inst\": %.2f}\n",
         name, waves, med, med / per_rep_insts);
}

int main() {
  uint64_t *clk;
  uint32_t *sink;
  hipMalloc(&clk, 8192 * sizeof(uint64_t));
  hipMalloc(&sink, 8192 * sizeof(uint32_t));
  for (int w : {1, 4}) {
    run<0>("add256 carry chain (8)", 8, w, clk, sink);
    run<1>("2 x add256 interleaved (16)", 16, w, clk, sink);
    run<2>("8 independent xor", 8, w, clk, sink);
    run<3>("8 dependent xor", 8, w, clk, sink);
    run<4>("s_setpc to next (4 salu)", 4, w, clk, sink);
    run<5>("dispatch tail (5 readlane+4 salu+setpc)", 13, w, clk, sink);
    run<6>("readlane -> salu (3)", 3, w, clk, sink);
    run<7>("lds 2 store + 2 load + wait", 5, w, clk, sink);
    run<8>("lds 2 load + wait", 3, w, clk, sink);
    run<9>("v_mad_u64_u32 dependent", 1, w, clk, sink);
    run<10>("4 v_mad_u64_u32 independent", 4, w, clk, sink);
    run<11>("gpr_idx 8 moves", 10, w, clk, sink);
    run<12>("cmp -> vcc -> s_cmp -> branch", 3, w, clk, sink);
    run<13>("8 dependent salu", 8, w, clk, sink);
    run<14>("8 cndmask (sgpr mask)", 8, w, clk, sink);
  }
  hipFree(clk);
  hipFree(sink);
  return 0;
}
