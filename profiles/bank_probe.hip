// VGPR bank probe (diagnostic, not part of libmgp): issue rate of v_bitop3_b32 / v_xor_b32
// whose VGPR sources sit in distinct banks (register index mod 4) against sources that
// share one bank.  Build: hipcc --offload-arch=gfx950 -O2 profiles/bank_probe.hip -o /tmp/bank_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP16(x) x x x x x x x x x x x x x x x x

template <int MODE>
__global__ void probe(int iters, unsigned *out) {
  unsigned acc = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // bitop3, sources v41 v42 v43: banks 1, 2, 3
      asm volatile(REP16("v_bitop3_b32 v40, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v44, v41, v42, v43 bitop3:0x96\n")
                   ::: "v40", "v41", "v42", "v43", "v44");
    } else if (MODE == 1) {  // bitop3, sources v40 v44 v48: all bank 0
      asm volatile(REP16("v_bitop3_b32 v41, v40, v44, v48 bitop3:0x96\n v_bitop3_b32 v45, v40, v44, v48 bitop3:0x96\n")
                   ::: "v40", "v41", "v44", "v45", "v48");
    } else if (MODE == 2) {  // xor, sources v41 v42
      asm volatile(REP16("v_xor_b32 v40, v41, v42\n v_xor_b32 v44, v41, v42\n") ::: "v40", "v41", "v42", "v44");
    } else if (MODE == 3) {  // xor, sources v40 v44 (same bank)
      asm volatile(REP16("v_xor_b32 v41, v40, v44\n v_xor_b32 v45, v40, v44\n") ::: "v40", "v41", "v44", "v45");
    } else if (MODE == 4) {  // mad_u64_u32, sources v42 v43 v[44:45]: banks 2, 3, 0/1
      asm volatile(REP16("v_mad_u64_u32 v[50:51], vcc, v42, v43, v[44:45]\n v_mad_u64_u32 v[52:53], vcc, v42, v43, v[44:45]\n")
                   ::: "v42", "v43", "v44", "v45", "v50", "v51", "v52", "v53", "vcc");
    } else {  // mad_u64_u32, sources v40 v44 v[48:49]: banks 0, 0, 0/1
      asm volatile(REP16("v_mad_u64_u32 v[50:51], vcc, v40, v44, v[48:49]\n v_mad_u64_u32 v[52:53], vcc, v40, v44, v[48:49]\n")
                   ::: "v40", "v44", "v48", "v49", "v50", "v51", "v52", "v53", "vcc");
    }
    acc += i;
  }
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

int main() {
  unsigned *out;
  hipMalloc(&out, 4);
  const int iters = 20000, blocks = 256 * 4 * 8, threads = 64;  // 8 waves per SIMD
  const char *names[6] = {"bitop3 distinct banks", "bitop3 one bank", "xor distinct banks", "xor one bank",
                          "mad_u64_u32 distinct banks", "mad_u64_u32 shared banks"};
  for (int mode = 0; mode < 6; ++mode) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) probe<0><<<blocks, threads>>>(iters, out);
      if (mode == 1) probe<1><<<blocks, threads>>>(iters, out);
      if (mode == 2) probe<2><<<blocks, threads>>>(iters, out);
      if (mode == 3) probe<3><<<blocks, threads>>>(iters, out);
      if (mode == 4) probe<4><<<blocks, threads>>>(iters, out);
      if (mode == 5) probe<5><<<blocks, threads>>>(iters, out);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double inst = (double)blocks * iters * 32;            // wave-instructions
    const double per_simd_per_s = inst / 1024.0 / (ms * 1e-3);
    printf("{\"mode\": \"%s\", \"ms\": %.3f, \"wave_inst_per_simd_per_ns\": %.4f}\n", names[mode], ms,
           per_simd_per_s * 1e-9);
  }
  return 0;
}
