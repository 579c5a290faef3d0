// wave.h — wave-level helpers shared by the kernels (64-lane wavefronts).
#pragma once
#include <stdint.h>

#include "kernels.h"

namespace lcdev {
namespace {

// Number of set bits of m in lanes below this one (prefix-sum compaction).
__device__ __forceinline__ int lanes_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
// Minimum of v over the 64 lanes as a wave-uniform (SGPR) value: four DPP
// min steps inside each 16-lane row (quad_perm [1,0,3,2], quad_perm
// [2,3,0,1], row_half_mirror, row_mirror), then the four row minima are read
// with v_readlane and combined on the scalar unit.  No LDS round trip.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return umin(umin(r0, r1), umin(r2, r3));
}
// Signed minimum over the wave (wave-uniform): wave_min_u32 on the
// order-preserving flip of the sign bit.
__device__ __forceinline__ int wave_min_i32(int v) {
  return (int)(wave_min_u32((uint32_t)v ^ 0x80000000u) ^ 0x80000000u);
}
__device__ __forceinline__ int first_lane(uint64_t b) { return (int)__builtin_ctzll(b); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int4 uni4(int4 v) {
  return make_int4(uni(v.x), uni(v.y), uni(v.z), uni(v.w));
}
// Lane-1's value (lane 0: `first`): DPP wave_shr:1, a VALU op instead of an
// LDS-crossbar permute (ds_bpermute) and its round trip.
__device__ __forceinline__ int wave_shr1(int v, int first) {
  return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xF, 0xF, false);
}
// Inclusive prefix sum over the wave: four DPP row_shr steps inside each
// 16-lane row (lanes shifted in from outside the row add 0), then the totals
// of the earlier rows (v_readlane).  `lane` = this lane's index.
__device__ __forceinline__ int wave_prefix_sum(int v, int lane) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
  const int r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
  const int r2 = __builtin_amdgcn_readlane(v, 47);
  const int row = lane >> 4;
  return v + (row == 0 ? 0 : row == 1 ? r0 : row == 2 ? r0 + r1 : r0 + r1 + r2);
}
// Suffix minimum over the wave: returns the minimum over the lanes above
// this one (`none` for lane 63) and sets *incl to the one including it.
// DPP row_shl steps inside each row (lanes shifted in from outside read
// `none`, the identity), then the minima of the later rows (v_readlane).
__device__ __forceinline__ uint32_t wave_suffix_min_excl(uint32_t v, int lane, uint32_t none,
                                                         uint32_t *incl) {
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)none, (int)v, 0x101, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)none, (int)v, 0x102, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)none, (int)v, 0x104, 0xF, 0xF, false));
  v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp((int)none, (int)v, 0x108, 0xF, 0xF, false));
  // v: minimum from this lane to its row's end
  const uint32_t m1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t m2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
  const uint32_t m3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  const int row = lane >> 4;
  const uint32_t m23 = umin(m2, m3);
  const uint32_t above = row == 0 ? umin(m1, m23) : row == 1 ? m23 : row == 2 ? m3 : none;
  *incl = umin(v, above);
  const uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp((int)none, (int)v, 0x101, 0xF, 0xF, false);
  return umin(nxt, above);
}
// Makes this wave's earlier stores visible to all of its lanes (LDS:
// lgkmcnt; global memory: vmcnt, same CU so L1-coherent).
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

}  // namespace
}  // namespace lcdev
