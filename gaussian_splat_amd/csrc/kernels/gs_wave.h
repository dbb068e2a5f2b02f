// gs_wave.h — wave64 / workgroup primitives for gfx950 (64-lane wavefronts).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Number of set bits of `mask` strictly below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t mbcnt(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += o;
    }
    return v;
}

// Exclusive scan over a 256-thread workgroup; `tmp` is >= 4 elements of LDS.
// Returns the exclusive prefix; *total receives the block sum.
template <typename T>
__device__ __forceinline__ T block256_exclusive_scan(T v, T* tmp, T* total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    T inc = wave_inclusive_scan(v);
    if (lane == 63) tmp[wave] = inc;
    __syncthreads();
    T w0 = tmp[0], w1 = tmp[1], w2 = tmp[2], w3 = tmp[3];
    T base = (wave > 0 ? w0 : T(0)) + (wave > 1 ? w1 : T(0)) + (wave > 2 ? w2 : T(0));
    *total = w0 + w1 + w2 + w3;
    __syncthreads();
    return base + inc - v;
}

}  // namespace gs
