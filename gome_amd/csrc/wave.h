// wave.h — wavefront (64-lane) primitives for gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gome {

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned long long lt_mask() {
  const uint32_t l = lane_id();
  return l ? (~0ull >> (64 - l)) : 0ull;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ int64_t rl64(int64_t v, uint32_t j) {
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), j);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), j);
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ int64_t uni64(int64_t v) { return rl64(v, __builtin_amdgcn_readfirstlane(lane_id())); }

// v_writelane_b32: replace lane l of `reg` with the uniform value v (no exec masking).
// HIP exposes no builtin for it; bind the LLVM intrinsic so the compiler sees (and
// hazard-checks) a real v_writelane.
__device__ int gome_writelane_i32(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wl_u32(uint32_t reg, uint32_t v, uint32_t l) {
  return static_cast<uint32_t>(gome_writelane_i32(static_cast<int>(v), static_cast<int>(l), static_cast<int>(reg)));
}

// Inclusive scan of a 64-bit value over the whole wave (LDS-crossbar shuffles).
__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off);
    if (lane >= static_cast<uint32_t>(off)) x += y;
  }
  return x;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t x) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= static_cast<uint32_t>(off)) x += y;
  }
  return x;
}

__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t x) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= static_cast<uint32_t>(off)) x = max(x, y);
  }
  return x;
}

// Inclusive scan of a 64-bit value over lanes 0..31 (rows 0 and 1) with DPP row shifts
// (VALU-latency, no LDS crossbar) and one readlane to carry row 0 into row 1.
// Lanes 32..63 return unspecified values.
template <int CTRL>
__device__ __forceinline__ int64_t dpp_shr64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(x), CTRL, 0xF, 0xF, false);
  const uint32_t hi = __builtin_amdgcn_update_dpp(0u, static_cast<uint32_t>(static_cast<uint64_t>(x) >> 32),
                                                  CTRL, 0xF, 0xF, false);
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ int64_t scan32_i64(int64_t x) {
  x += dpp_shr64<0x111>(x);  // row_shr:1
  x += dpp_shr64<0x112>(x);  // row_shr:2
  x += dpp_shr64<0x114>(x);  // row_shr:4
  x += dpp_shr64<0x118>(x);  // row_shr:8
  const int64_t row0 = rl64(x, 15);
  if (lane_id() >= 16) x += row0;
  return x;
}

// Explicit address spaces.  Where one source line may store to LDS or to HBM, the compiler
// merges the two into a FLAT access, which counts against both vmcnt and lgkmcnt: every
// later LDS wait then also waits for the HBM write.  Route such stores through these.
#define GOME_LDS __attribute__((address_space(3)))
#define GOME_GLB __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GOME_LDS T* as_lds(T* p) { return (GOME_LDS T*)(p); }
template <class T>
__device__ __forceinline__ GOME_GLB T* as_glb(T* p) { return (GOME_GLB T*)(p); }
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u v4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  v4u r = {a, b, c, d};
  return r;
}
__device__ __forceinline__ void st16_lds(void* p, v4u v) { *(GOME_LDS v4u*)(p) = v; }
__device__ __forceinline__ void st16_glb(void* p, v4u v) { *(GOME_GLB v4u*)(p) = v; }
__device__ __forceinline__ uint32_t lo32(int64_t x) { return static_cast<uint32_t>(x); }
__device__ __forceinline__ uint32_t hi32(int64_t x) { return static_cast<uint32_t>(static_cast<uint64_t>(x) >> 32); }

// Keep a wave-uniform value in VGPRs: an inline-asm VGPR output is divergent to the
// compiler, so later arithmetic on it stays VALU instead of occupying the (scarce) SGPR file.
template <class T>
__device__ __forceinline__ T vreg(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

__host__ __device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

}  // namespace gome
