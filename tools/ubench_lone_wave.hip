// Lone-wavefront instruction costs on gfx950 (one wave on the whole GPU), in shader clocks
// (s_memtime).  Guides the hand-scheduled plan loop (gome_amd/csrc/gen_plan_asm.py).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lone_wave.hip -o tools/ubench_lone_wave
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void k(unsigned long long* out) {
  unsigned long long t0, t1;
  unsigned a = threadIdx.x, b = 1, c = 2, d1 = 3, d2 = 4;
  // 1) 512 dependent s_add
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_add_u32 %0, %0, 1\n\t")) : "+s"(b));
  t1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0;
  // 2) 512 independent s_add pairs (two chains interleaved)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\t")) : "+s"(b), "+s"(c));
  t1 = __builtin_amdgcn_s_memtime();
  out[1] = t1 - t0;
  // 3) 512 taken branches (to the next instruction)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_branch 1f\n\t1:\n\t")) ::);
  t1 = __builtin_amdgcn_s_memtime();
  out[2] = t1 - t0;
  // 4) 512 not-taken s_cbranch_scc1 after s_cmp (scc = 0)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_cmp_eq_u32 %0, 12345\n\ts_cbranch_scc1 2f\n\t2:\n\t")) : "+s"(b));
  t1 = __builtin_amdgcn_s_memtime();
  out[3] = t1 - t0;
  // 5) 512 v_readlane -> s_add dependent pairs
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("v_readlane_b32 %0, %1, 3\n\ts_add_u32 %0, %0, 1\n\t")) : "+s"(c) : "v"(a));
  t1 = __builtin_amdgcn_s_memtime();
  out[4] = t1 - t0;
  // 6) 512 v_writelane (m0 lane select) on one VGPR
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_mov_b32 m0, 5\n\t" REP8(REP64("v_writelane_b32 %0, %1, m0\n\t")) : "+v"(a) : "s"(b) : "m0");
  t1 = __builtin_amdgcn_s_memtime();
  out[5] = t1 - t0;
  // 7) 512 s_sub_u32/s_subb_u32 pairs (64-bit subtract chain)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_sub_u32 %0, %0, 1\n\ts_subb_u32 %1, %1, 0\n\t")) : "+s"(b), "+s"(c));
  t1 = __builtin_amdgcn_s_memtime();
  out[6] = t1 - t0;
  // 8) 512 v_add_u32 dependent
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("v_add_u32 %0, 1, %0\n\t")) : "+v"(a));
  t1 = __builtin_amdgcn_s_memtime();
  out[7] = t1 - t0;
  // 9) 512 s_cselect_b64 exec + v_add (exec-masked VALU)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_mov_b64 exec, 1\n\tv_add_u32 %0, 1, %0\n\t")) "s_mov_b64 exec, -1\n\t" : "+v"(a));
  t1 = __builtin_amdgcn_s_memtime();
  out[8] = t1 - t0;
  // 10) 512 s_bitcmp1 + s_cbranch_scc1 taken to next
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_bitcmp0_b32 %0, 31\n\ts_cbranch_scc1 3f\n\t3:\n\t")) : "+s"(b));
  t1 = __builtin_amdgcn_s_memtime();
  out[9] = t1 - t0;
  // 11) s_cmp, 3 independent s_add, s_cbranch (not taken): is the branch cost SCC latency?
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_cmp_eq_u32 %0, 12345\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\t"
                          "s_add_u32 %3, %3, 1\n\ts_cbranch_scc1 4f\n\t4:\n\t"))
               : "+s"(b), "+s"(c), "+s"(d1), "+s"(d2));
  t1 = __builtin_amdgcn_s_memtime();
  out[10] = t1 - t0;
  // 12) 4 s_add alone (reference for 11)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_cmp_eq_u32 %0, 12345\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\t"
                          "s_add_u32 %3, %3, 1\n\t"))
               : "+s"(b), "+s"(c), "+s"(d1), "+s"(d2));
  t1 = __builtin_amdgcn_s_memtime();
  out[11] = t1 - t0;
  // 13) s_cbranch_scc1 taken to a target 8 instructions ahead (skipping them)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_cmp_eq_u32 %0, %0\n\ts_cbranch_scc1 5f\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %1, %1, 1\n\t"
                          "s_add_u32 %1, %1, 1\n\ts_add_u32 %1, %1, 1\n\t5:\n\t"))
               : "+s"(b), "+s"(c));
  t1 = __builtin_amdgcn_s_memtime();
  out[12] = t1 - t0;
  // 14) v_readlane, then 5 independent SALU, then consume (hidden latency?)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("v_readlane_b32 %0, %4, 3\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\t"
                          "s_add_u32 %3, %3, 1\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %0, %0, 1\n\t"))
               : "+s"(c), "+s"(b), "+s"(d1), "+s"(d2) : "v"(a));
  t1 = __builtin_amdgcn_s_memtime();
  out[13] = t1 - t0;
  out[14] = a + b + c + d1 + d2;
}

int main() {
  unsigned long long* d;
  unsigned long long h[16];
  hipMalloc(&d, sizeof(h));
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  }
  const char* names[] = {"dep s_add", "2 indep s_add (per pair)", "s_branch taken", "s_cmp+cbranch not taken (pair)",
                         "v_readlane->s_add (pair)", "v_writelane", "s_sub+s_subb (pair)", "dep v_add",
                         "s_mov exec + v_add (pair)", "s_bitcmp + cbranch taken (pair)",
                         "cmp,3 add,cbranch nt (group)", "cmp,3 add (group)", "cmp,cbranch taken over 4 (group)",
                         "readlane,4 salu,consume (group)"};
  // s_memtime counts at a fixed 100 MHz reference on gfx9? print raw ticks per op
  for (int i = 0; i < 14; ++i) printf("%-34s %8.3f ticks/op\n", names[i], h[i] / 512.0);
  hipFree(d);
  return 0;
}
