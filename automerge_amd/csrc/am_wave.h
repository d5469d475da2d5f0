// am_wave.h -- wave64 cross-lane primitives for CDNA4 (gfx950) built on DPP and permlane swaps.
//
// HIP's __shfl_* lower to ds_bpermute_b32: an LDS-pipeline round trip (address VGPR, LDS
// crossbar, lgkmcnt wait) per 32 bits moved. The per-document kernels are chains of small scans,
// sorts and neighbour compares over one wave, so that latency is on their critical path. The
// fixed-pattern moves below stay in the VALU:
//   * row_shr / row_shl / quad_perm / wave_shr / wave_shl / row_bcast DPP modifiers
//     (GFX9 DPP: rows of 16 lanes, row_bcast:15 / row_bcast:31 carry across rows),
//   * v_permlane16_swap / v_permlane32_swap (gfx950) for the xor-16 / xor-32 exchanges,
//   * v_readlane for wave-uniform broadcasts.
// Only data-dependent gathers (__shfl with a per-lane index) still use ds_bpermute.
#pragma once
#include <cstdint>

namespace wave {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t identity, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int32_t dpp(int32_t identity, int32_t v) {
  return __builtin_amdgcn_update_dpp(identity, v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint64_t dpp(uint64_t identity, uint64_t v) {
  const uint32_t lo = dpp<CTRL, ROW_MASK>((uint32_t)identity, (uint32_t)v);
  const uint32_t hi = dpp<CTRL, ROW_MASK>((uint32_t)(identity >> 32), (uint32_t)(v >> 32));
  return (uint64_t)hi << 32 | lo;
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int64_t dpp(int64_t identity, int64_t v) {
  return (int64_t)dpp<CTRL, ROW_MASK>((uint64_t)identity, (uint64_t)v);
}

enum : int {
  QP_XOR1 = 0xB1,  // quad_perm [1,0,3,2]
  QP_XOR2 = 0x4E,  // quad_perm [2,3,0,1]
  ROW_SHL4 = 0x104, ROW_SHL8 = 0x108,
  ROW_SHR1 = 0x111, ROW_SHR2 = 0x112, ROW_SHR4 = 0x114, ROW_SHR8 = 0x118,
  WAVE_SHL1 = 0x130, WAVE_SHR1 = 0x138,
  ROW_BCAST15 = 0x142, ROW_BCAST31 = 0x143,
};

// value of lane l-1 (lane 0 gets `fill`): __shfl_up(v, 1) without the LDS round trip
template <typename T> struct same_t { using type = T; };
template <typename T>
__device__ __forceinline__ T up1(T v, typename same_t<T>::type fill) { return dpp<WAVE_SHR1>(fill, v); }
// value of lane l+1 (lane 63 gets `fill`)
template <typename T>
__device__ __forceinline__ T down1(T v, typename same_t<T>::type fill) { return dpp<WAVE_SHL1>(fill, v); }

__device__ __forceinline__ uint32_t bcast(uint32_t v, int src) { return (uint32_t)__builtin_amdgcn_readlane((int)v, src); }
__device__ __forceinline__ int32_t bcast(int32_t v, int src) { return __builtin_amdgcn_readlane(v, src); }
__device__ __forceinline__ uint64_t bcast(uint64_t v, int src) {
  return (uint64_t)bcast((uint32_t)(v >> 32), src) << 32 | bcast((uint32_t)v, src);
}
__device__ __forceinline__ int64_t bcast(int64_t v, int src) { return (int64_t)bcast((uint64_t)v, src); }

// inclusive scans over the 64 lanes (every lane must be active)
__device__ __forceinline__ uint32_t incl_add(uint32_t x) {
  x += dpp<ROW_SHR1>(0u, x);
  x += dpp<ROW_SHR2>(0u, x);
  x += dpp<ROW_SHR4>(0u, x);
  x += dpp<ROW_SHR8>(0u, x);
  x += dpp<ROW_BCAST15, 0xa>(0u, x);
  x += dpp<ROW_BCAST31, 0xc>(0u, x);
  return x;
}
__device__ __forceinline__ int32_t incl_max(int32_t x) {
  const int32_t I = INT32_MIN;
  x = max(x, dpp<ROW_SHR1>(I, x));
  x = max(x, dpp<ROW_SHR2>(I, x));
  x = max(x, dpp<ROW_SHR4>(I, x));
  x = max(x, dpp<ROW_SHR8>(I, x));
  x = max(x, dpp<ROW_BCAST15, 0xa>(I, x));
  x = max(x, dpp<ROW_BCAST31, 0xc>(I, x));
  return x;
}
// exclusive prefix sum; `total` = sum over all lanes
__device__ __forceinline__ uint32_t excl_add(uint32_t v, uint32_t& total) {
  const uint32_t x = incl_add(v);
  total = bcast(x, 63);
  return x - v;
}
__device__ __forceinline__ uint32_t sum_all(uint32_t v) { return bcast(incl_add(v), 63); }
__device__ __forceinline__ int64_t max_all(int64_t v) {
  // 64-bit max: reduce the halves through a 64-bit compare after each move
  const int64_t I = INT64_MIN;
  int64_t y;
  y = dpp<ROW_SHR1>(I, v); v = y > v ? y : v;
  y = dpp<ROW_SHR2>(I, v); v = y > v ? y : v;
  y = dpp<ROW_SHR4>(I, v); v = y > v ? y : v;
  y = dpp<ROW_SHR8>(I, v); v = y > v ? y : v;
  y = dpp<ROW_BCAST15, 0xa>(I, v); v = y > v ? y : v;
  y = dpp<ROW_BCAST31, 0xc>(I, v); v = y > v ? y : v;
  return bcast(v, 63);
}

// value of lane l ^ J for J in {1, 2, 4, 8, 16, 32}
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  const uint32_t l = lane_id();
  if constexpr (J == 1) return dpp<QP_XOR1>(0u, v);
  else if constexpr (J == 2) return dpp<QP_XOR2>(0u, v);
  else if constexpr (J == 4) {
    const uint32_t a = dpp<ROW_SHL4>(0u, v), b = dpp<ROW_SHR4>(0u, v);
    return (l & 4) ? b : a;
  } else if constexpr (J == 8) {
    const uint32_t a = dpp<ROW_SHL8>(0u, v), b = dpp<ROW_SHR8>(0u, v);
    return (l & 8) ? b : a;
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (l & 16) ? (uint32_t)r[0] : (uint32_t)r[1];
  } else {
    static_assert(J == 32, "xor_lane: J in {1,2,4,8,16,32}");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (l & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
  }
}
template <int J>
__device__ __forceinline__ uint64_t xor_lane(uint64_t v) {
  return (uint64_t)xor_lane<J>((uint32_t)(v >> 32)) << 32 | xor_lane<J>((uint32_t)v);
}

// one bitonic compare-exchange stage (k, J): ascending over the wave
template <int J>
__device__ __forceinline__ uint64_t bitonic_step(uint64_t v, uint32_t k) {
  const uint32_t l = lane_id();
  const uint64_t p = xor_lane<J>(v);
  const bool up = (l & k) == 0, lo = (l & J) == 0;
  const uint64_t mn = v < p ? v : p, mx = v < p ? p : v;
  return (lo == up) ? mn : mx;
}
// ascending sort of one u64 per lane (padding lanes hold ~0)
__device__ __forceinline__ uint64_t sort64(uint64_t v) {
  v = bitonic_step<1>(v, 2);
  v = bitonic_step<2>(v, 4);  v = bitonic_step<1>(v, 4);
  v = bitonic_step<4>(v, 8);  v = bitonic_step<2>(v, 8);  v = bitonic_step<1>(v, 8);
  v = bitonic_step<8>(v, 16); v = bitonic_step<4>(v, 16); v = bitonic_step<2>(v, 16); v = bitonic_step<1>(v, 16);
  v = bitonic_step<16>(v, 32); v = bitonic_step<8>(v, 32); v = bitonic_step<4>(v, 32); v = bitonic_step<2>(v, 32);
  v = bitonic_step<1>(v, 32);
  v = bitonic_step<32>(v, 64); v = bitonic_step<16>(v, 64); v = bitonic_step<8>(v, 64); v = bitonic_step<4>(v, 64);
  v = bitonic_step<2>(v, 64); v = bitonic_step<1>(v, 64);
  return v;
}

}  // namespace wave
