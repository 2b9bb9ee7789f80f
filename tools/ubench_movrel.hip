// Lone-wave costs of the plan-latency candidates of DESIGN 4.1 (round 6), in s_memtime ticks per
// group: M0-relative SGPR reads/writes (s_movrels / s_movreld) against the v_readlane / v_writelane
// pair the plan uses for lane depths today, and the SGPR side-mask upkeep a level-empty fast path
// would need (s_bitset / s_ff1).  Same method as ubench_lone_wave.hip: one wave, 512 repetitions.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_movrel.hip -o tools/ubench_movrel
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void k(unsigned long long* out) {
  unsigned long long t0, t1;
  unsigned a = threadIdx.x, b = 1, c = 2, d = 3;
  unsigned long long msk = 0x00F0F0F0F0F0F0F0ull;
  // 1) v_readlane (SGPR lane select) -> dependent s_add: today's deep-level read
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_mov_b32 s10, 3\n\t" REP8(REP64("v_readlane_b32 %0, %1, s10\n\ts_add_u32 %0, %0, 1\n\t"))
               : "+s"(c) : "v"(a) : "s10");
  t1 = __builtin_amdgcn_s_memtime();
  out[0] = t1 - t0;
  // 2) s_movrels (M0 fixed) -> dependent s_add
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_mov_b32 m0, 3\n\ts_nop 1\n\t" REP8(REP64("s_movrels_b32 %0, s16\n\ts_add_u32 %0, %0, 1\n\t"))
               : "+s"(c) : : "m0", "s16", "s17", "s18", "s19");
  t1 = __builtin_amdgcn_s_memtime();
  out[1] = t1 - t0;
  // 3) s_mov m0 (a new index every time) + s_movrels + dependent s_add
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_and_b32 m0, %1, 3\n\ts_movrels_b32 %0, s16\n\ts_add_u32 %1, %0, %1\n\t"))
               : "+s"(c), "+s"(b) : : "m0", "s16", "s17", "s18", "s19");
  t1 = __builtin_amdgcn_s_memtime();
  out[2] = t1 - t0;
  // 4) s_mov m0 + s_movreld (indexed SGPR write) + read back
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_and_b32 m0, %1, 3\n\ts_movreld_b32 s16, %0\n\ts_mov_b32 %0, s17\n\ts_add_u32 %1, %1, 1\n\t"))
               : "+s"(c), "+s"(b) : : "m0", "s16", "s17", "s18", "s19");
  t1 = __builtin_amdgcn_s_memtime();
  out[3] = t1 - t0;
  // 5) v_writelane (M0 lane select, as the plan's staging) + v_readlane back -> s_add
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_mov_b32 m0, 5\n\t" REP8(REP64("v_writelane_b32 %1, %0, m0\n\tv_readlane_b32 %0, %1, m0\n\ts_add_u32 %0, %0, 1\n\t"))
               : "+s"(c), "+v"(a) : : "m0");
  t1 = __builtin_amdgcn_s_memtime();
  out[4] = t1 - t0;
  // 6) side-mask upkeep on a rest: s_bitset1_b64 (the level joins the side set)
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_bitset1_b64 %0, %1\n\ts_add_u32 %1, %1, 7\n\t")) : "+s"(msk), "+s"(b));
  t1 = __builtin_amdgcn_s_memtime();
  out[5] = t1 - t0;
  // 7) next level from the mask: s_and with the above-level mask, s_ff1, consume
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("s_lshr_b64 s[20:21], %0, %1\n\ts_ff1_i32_b64 %1, s[20:21]\n\ts_and_b32 %1, %1, 31\n\t"))
               : "+s"(msk), "+s"(d) : : "s20", "s21");
  t1 = __builtin_amdgcn_s_memtime();
  out[6] = t1 - t0;
  // 8) today's next level: v_cmp_ne_u64 over the pair registers + s_ff1 of VCC + v_readlane
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile(REP8(REP64("v_cmp_ne_u32 vcc, 0, %1\n\ts_ff1_i32_b64 %0, vcc\n\tv_readlane_b32 %0, %1, %0\n\t"))
               : "+s"(c) : "v"(a) : "vcc");
  t1 = __builtin_amdgcn_s_memtime();
  out[7] = t1 - t0;
  out[8] = a + b + c + d + msk;
}

int main() {
  unsigned long long* d;
  unsigned long long h[9];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  }
  const char* names[] = {"v_readlane(s) -> s_add",           "s_movrels (m0 fixed) -> s_add",
                         "m0 <- idx, s_movrels, s_add",      "m0 <- idx, s_movreld, read, add",
                         "v_writelane + v_readlane (m0) -> add", "s_bitset1_b64 + s_add",
                         "mask: lshr, ff1, and",             "v_cmp, s_ff1 vcc, v_readlane"};
  for (int i = 0; i < 8; ++i) printf("%-36s %8.3f ticks/group\n", names[i], h[i] / 512.0);
  hipFree(d);
  return 0;
}
