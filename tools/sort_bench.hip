// sort_bench: our reduce-then-scan LSD sort vs rocPRIM (hipcub) on the frame's shapes.
// Measurement tool only (cross-check + headroom); not part of libgsplat.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
#include "kernels/gs_kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 26307856;
    const int bits = argc > 2 ? atoi(argv[2]) : 13;
    std::mt19937 rng(1);
    std::vector<uint32_t> hk(n), hv(n);
    for (uint32_t i = 0; i < n; ++i) { hk[i] = rng() & ((1u << bits) - 1); hv[i] = i; }
    uint32_t *k, *v, *k2, *v2, *tk, *tv;
    CK(hipMalloc(&k, n * 4)); CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&k2, n * 4)); CK(hipMalloc(&v2, n * 4));
    CK(hipMalloc(&tk, n * 4)); CK(hipMalloc(&tv, n * 4));
    CK(hipMemcpy(k, hk.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(v, hv.data(), n * 4, hipMemcpyHostToDevice));
    uint32_t* scratch; CK(hipMalloc(&scratch, gs::radix_sort_scratch_words(n) * 4));
    size_t tb = 0; void* tmp = nullptr;
    CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k, k2, v, v2, (int)n, 0, bits));
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(a));
        for (int it = 0; it < 10; ++it) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k, k2, v, v2, (int)n, 0, bits));
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("rocprim  n=%u bits=%d: %.1f us/sort\n", n, bits, ms * 100);
        CK(hipEventRecord(a));
        bool in_tmp;
        for (int it = 0; it < 10; ++it) CK(gs::launch_radix_sort(k, v, k2, v2, tk, tv, n, bits, scratch, &in_tmp, 0));
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipEventElapsedTime(&ms, a, b));
        printf("ours n=%u bits=%d: %.1f us/sort\n", n, bits, ms * 100);
    }
    std::vector<uint32_t> ok(n); CK(hipMemcpy(ok.data(), k2, n * 4, hipMemcpyDeviceToHost));
    printf("sorted: %d\n", (int)std::is_sorted(ok.begin(), ok.end()));
    return 0;
}
