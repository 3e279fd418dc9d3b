// Issue-rate probe for the Keccak instruction mix (diagnostic, not part of libmgp): how many
// wave-instructions per ns one SIMD issues for dependency-free streams of the instruction
// forms mgp_keccak64_gfx950 uses, alone and in the kernel's per-round mix (120 v_bitop3_b32
// : 58 v_alignbit_b32, gen_keccak_asm.py), at the kernel's occupancy (5 waves per SIMD) and
// at 8.  The mix rate is the issue bound the kernel is measured against.
// Build: hipcc --offload-arch=gfx950 -O2 profiles/issue_probe.hip -o profiles/issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP4(x) x x x x
#define REP16(x) REP4(x) REP4(x) REP4(x) REP4(x)
// distinct banks throughout: sources v41 v42 v43 (banks 1, 2, 3), destinations bank 0 / 1
#define BIT3A "v_bitop3_b32 v40, v41, v42, v43 bitop3:0x96\n"
#define BIT3B "v_bitop3_b32 v44, v41, v42, v43 bitop3:0x96\n"
#define ALIGN "v_alignbit_b32 v48, v41, v42, 31\n"
#define ALIGN2 "v_alignbit_b32 v52, v42, v43, 31\n"

template <int MODE>
__global__ void probe(int iters, unsigned *out) {
  unsigned acc = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // bitop3 only (32 per iteration)
      asm volatile(REP16(BIT3A BIT3B) ::: "v40", "v41", "v42", "v43", "v44");
    } else if (MODE == 1) {  // alignbit only (32)
      asm volatile(REP16(ALIGN ALIGN2) ::: "v41", "v42", "v43", "v48", "v52");
    } else {  // the kernel's mix: 2 bitop3 per alignbit (120 : 58 per round), 48 per iteration
      asm volatile(REP16(BIT3A BIT3B ALIGN) ::: "v40", "v41", "v42", "v43", "v44", "v48");
    }
    acc += i;
  }
  if (acc == 0xFFFFFFFFu) out[0] = acc;
}

int main() {
  unsigned *out;
  hipMalloc(&out, 4);
  const int iters = 20000;
  const char *names[3] = {"bitop3", "alignbit", "keccak mix 2:1"};
  const int per_iter[3] = {32, 32, 48};
  for (int waves = 5; waves <= 8; waves += 3) {
    const int blocks = 256 * 4 * waves, threads = 64;
    for (int mode = 0; mode < 3; ++mode) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      float ms = 0.f;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (mode == 0) probe<0><<<blocks, threads>>>(iters, out);
        if (mode == 1) probe<1><<<blocks, threads>>>(iters, out);
        if (mode == 2) probe<2><<<blocks, threads>>>(iters, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
      }
      const double inst = (double)blocks * iters * per_iter[mode];  // wave-instructions
      printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"wave_inst_per_simd_per_ns\": %.4f}\n",
             names[mode], waves, ms, inst / (1024.0 * ms * 1e6));
    }
  }
  hipFree(out);
  return 0;
}
