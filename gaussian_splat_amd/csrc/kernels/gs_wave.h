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

// Hand-off of LDS data between lanes of ONE wave (no workgroup barrier):
// orders this wave's LDS writes before its later reads, for the hardware and
// for the compiler (which may otherwise forward a lane's own store).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// Workgroup barrier that orders LDS only (__syncthreads also waits for every
// outstanding global store of the wave, vmcnt(0), which a kernel that
// scatters stores between barriers cannot afford).
__device__ __forceinline__ void block_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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

// Inclusive wave64 scan with DPP (no LDS round trips): row_shr 1/2/4/8 scans
// each 16-lane row, row_bcast:15 / row_bcast:31 carry rows 0->1, 2->3 and
// 0-1 -> 2-3.  Out-of-range sources read 0, the identity of + and of max
// over unsigned values.
template <bool MAX>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
    auto op = [](uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : a + b; };
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
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
