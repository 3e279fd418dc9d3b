// valu_mix.hip — VALU issue-rate microbenchmark for the instruction classes of
// the Keccak kernel (profiles only; not part of libmgp).
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_mix profiles/valu_mix.hip && ./build/valu_mix
// Each mode runs 8 independent chains of one instruction per lane (inline asm,
// nothing folded) and reports wave64 instructions per SIMD-cycle at the clock
// the kernel actually ran at (s_memtime shader clocks vs s_memrealtime 100 MHz).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHAINS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)

template <int MODE>
__global__ __launch_bounds__(256) void mix_kernel(uint32_t iters, uint32_t *sink, uint64_t *clk) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  const uint32_t b = blockIdx.x | 1u, c = blockIdx.x * 3u + 7u;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      if constexpr (MODE == 0)
        asm volatile(
            "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
            : CHAINS : "v"(b));
      if constexpr (MODE == 1)
        asm volatile(
            "v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %8\n\tv_xor_b32 %2, %2, %8\n\tv_xor_b32 %3, %3, %8\n\t"
            "v_xor_b32 %4, %4, %8\n\tv_xor_b32 %5, %5, %8\n\tv_xor_b32 %6, %6, %8\n\tv_xor_b32 %7, %7, %8"
            : CHAINS : "v"(b));
      if constexpr (MODE == 2)
        asm volatile(
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\t"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\t"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\t"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"
            : CHAINS : "v"(b), "v"(c));
      if constexpr (MODE == 3)
        asm volatile(
            "v_alignbit_b32 %0, %0, %8, 7\n\tv_alignbit_b32 %1, %1, %8, 7\n\tv_alignbit_b32 %2, %2, %8, 7\n\t"
            "v_alignbit_b32 %3, %3, %8, 7\n\tv_alignbit_b32 %4, %4, %8, 7\n\tv_alignbit_b32 %5, %5, %8, 7\n\t"
            "v_alignbit_b32 %6, %6, %8, 7\n\tv_alignbit_b32 %7, %7, %8, 7"
            : CHAINS : "v"(b));
      if constexpr (MODE == 4)  // bitop3 reading three chain registers (no shared operand)
        asm volatile(
            "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n\t"
            "v_bitop3_b32 %2, %2, %3, %4 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %4, %5 bitop3:0x96\n\t"
            "v_bitop3_b32 %4, %4, %5, %6 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %6, %7 bitop3:0x96\n\t"
            "v_bitop3_b32 %6, %6, %7, %0 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %0, %1 bitop3:0x96"
            : CHAINS);
      if constexpr (MODE == 5)  // VOP3 two-source xor (the e64 encoding)
        asm volatile(
            "v_xor_b32_e64 %0, %0, %8\n\tv_xor_b32_e64 %1, %1, %8\n\tv_xor_b32_e64 %2, %2, %8\n\t"
            "v_xor_b32_e64 %3, %3, %8\n\tv_xor_b32_e64 %4, %4, %8\n\tv_xor_b32_e64 %5, %5, %8\n\t"
            "v_xor_b32_e64 %6, %6, %8\n\tv_xor_b32_e64 %7, %7, %8"
            : CHAINS : "v"(b));
      if constexpr (MODE == 6)
        asm volatile(
            "v_lshl_or_b32 %0, %0, 7, %8\n\tv_lshl_or_b32 %1, %1, 7, %8\n\tv_lshl_or_b32 %2, %2, 7, %8\n\t"
            "v_lshl_or_b32 %3, %3, 7, %8\n\tv_lshl_or_b32 %4, %4, 7, %8\n\tv_lshl_or_b32 %5, %5, 7, %8\n\t"
            "v_lshl_or_b32 %6, %6, 7, %8\n\tv_lshl_or_b32 %7, %7, 7, %8"
            : CHAINS : "v"(b));
      if constexpr (MODE == 7)
        asm volatile(
            "v_lshrrev_b32 %0, 25, %0\n\tv_lshrrev_b32 %1, 25, %1\n\tv_lshrrev_b32 %2, 25, %2\n\t"
            "v_lshrrev_b32 %3, 25, %3\n\tv_lshrrev_b32 %4, 25, %4\n\tv_lshrrev_b32 %5, 25, %5\n\t"
            "v_lshrrev_b32 %6, 25, %6\n\tv_lshrrev_b32 %7, 25, %7"
            : CHAINS);
      if constexpr (MODE == 8)
        asm volatile(
            "v_alignbyte_b32 %0, %0, %8, 3\n\tv_alignbyte_b32 %1, %1, %8, 3\n\tv_alignbyte_b32 %2, %2, %8, 3\n\t"
            "v_alignbyte_b32 %3, %3, %8, 3\n\tv_alignbyte_b32 %4, %4, %8, 3\n\tv_alignbyte_b32 %5, %5, %8, 3\n\t"
            "v_alignbyte_b32 %6, %6, %8, 3\n\tv_alignbyte_b32 %7, %7, %8, 3"
            : CHAINS : "v"(b));
      if constexpr (MODE == 9)
        asm volatile(
            "v_perm_b32 %0, %0, %8, %9\n\tv_perm_b32 %1, %1, %8, %9\n\tv_perm_b32 %2, %2, %8, %9\n\t"
            "v_perm_b32 %3, %3, %8, %9\n\tv_perm_b32 %4, %4, %8, %9\n\tv_perm_b32 %5, %5, %8, %9\n\t"
            "v_perm_b32 %6, %6, %8, %9\n\tv_perm_b32 %7, %7, %8, %9"
            : CHAINS : "v"(b), "v"(c));
      if constexpr (MODE == 10)  // alternating alignbit / bitop3: is alignbit a separate pipe?
        asm volatile(
            "v_alignbit_b32 %0, %0, %8, 7\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\t"
            "v_alignbit_b32 %2, %2, %8, 7\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\t"
            "v_alignbit_b32 %4, %4, %8, 7\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\t"
            "v_alignbit_b32 %6, %6, %8, 7\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"
            : CHAINS : "v"(b), "v"(c));
      if constexpr (MODE == 12)  // four alignbit, then four bitop3: fewer slow/fast transitions
        asm volatile(
            "v_alignbit_b32 %0, %0, %8, 7\n\tv_alignbit_b32 %2, %2, %8, 7\n\t"
            "v_alignbit_b32 %4, %4, %8, 7\n\tv_alignbit_b32 %6, %6, %8, 7\n\t"
            "v_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\t"
            "v_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96"
            : CHAINS : "v"(b), "v"(c));
      if constexpr (MODE == 13)  // keccak-like ratio: 1 alignbit per 2 full-rate ops
        asm volatile(
            "v_alignbit_b32 %0, %0, %8, 7\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\t"
            "v_xor_b32 %2, %2, %8\n\tv_alignbit_b32 %3, %3, %8, 7\n\t"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_xor_b32 %5, %5, %8\n\t"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_xor_b32 %7, %7, %8"
            : CHAINS : "v"(b), "v"(c));
      if constexpr (MODE == 11)
        asm volatile(
            "v_lshl_add_u32 %0, %0, 7, %8\n\tv_lshl_add_u32 %1, %1, 7, %8\n\tv_lshl_add_u32 %2, %2, 7, %8\n\t"
            "v_lshl_add_u32 %3, %3, 7, %8\n\tv_lshl_add_u32 %4, %4, 7, %8\n\tv_lshl_add_u32 %5, %5, 7, %8\n\t"
            "v_lshl_add_u32 %6, %6, 7, %8\n\tv_lshl_add_u32 %7, %7, 7, %8"
            : CHAINS : "v"(b));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0xFFFFFFFFu) sink[blockIdx.x] = r;
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int MODE>
static void run(const char *name, uint32_t *sink, uint64_t *clk) {
  const uint32_t iters = 400, blocks = 8192;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL(mix_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, iters, sink, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (rep && ms < best) best = ms;
  }
  uint64_t h[2048];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < 1024; ++i) { cyc += (double)h[2 * i]; rt += (double)h[2 * i + 1]; }
  const double ghz = cyc / (rt * 10.0);  // realtime ticks at 100 MHz
  const double winst = (double)blocks * 4 * iters * 512;  // wave64 instructions
  const double per_simd_cycle = winst / (1024.0 * (best * 1e-3) * ghz * 1e9);
  printf("{\"mode\": \"%s\", \"ms\": %.3f, \"clock_ghz\": %.3f, \"lane_tops\": %.2f, "
         "\"wave_insts_per_simd_cycle\": %.3f}\n",
         name, best, ghz, winst * 64 / (best * 1e-3) / 1e12, per_simd_cycle);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  uint32_t *sink;
  uint64_t *clk;
  hipMalloc(&sink, 8192 * 4);
  hipMalloc(&clk, 2048 * 8);
  run<0>("v_add_u32", sink, clk);
  run<1>("v_xor_b32", sink, clk);
  run<5>("v_xor_b32_e64", sink, clk);
  run<3>("v_alignbit_b32 (2 vgpr + imm)", sink, clk);
  run<2>("v_bitop3_b32 (chain + 2 shared vgpr)", sink, clk);
  run<4>("v_bitop3_b32 (3 chain vgprs)", sink, clk);
  run<6>("v_lshl_or_b32", sink, clk);
  run<7>("v_lshrrev_b32", sink, clk);
  run<8>("v_alignbyte_b32", sink, clk);
  run<9>("v_perm_b32", sink, clk);
  run<10>("alignbit/bitop3 alternating", sink, clk);
  run<11>("v_lshl_add_u32", sink, clk);
  run<12>("4 alignbit then 4 bitop3", sink, clk);
  run<13>("alignbit : full-rate = 1 : 3", sink, clk);
  hipFree(sink);
  hipFree(clk);
  return 0;
}
