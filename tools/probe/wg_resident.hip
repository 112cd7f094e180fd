// Probe (diagnostic, not product code): how many 128-lane workgroups with
// 20432 B of LDS are resident per CU at once, when the second wave exits at
// once (mode 0) or waits in a barrier for the first (mode 1).  Wave 0 of
// each workgroup records its CU and start time and sleeps ~2 ms.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

__global__ void __launch_bounds__(128) k_res(uint64_t* out, int mode) {
    __shared__ uint8_t pad[20432];
    const uint32_t wave = threadIdx.x >> 6;
    if (wave == 1) {
        if (mode == 1) __syncthreads();
        return;
    }
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));   // HW_REG_XCC_ID
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    pad[threadIdx.x] = 1;
    while (__builtin_amdgcn_s_memrealtime() - t0 < 200000) __builtin_amdgcn_s_sleep(10);   // 2 ms
    if (mode == 1) __syncthreads();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t0;
        out[2 * blockIdx.x + 1] = ((uint64_t)(xcc & 15) << 32) | hw | (pad[5] == 9 ? 1ull << 63 : 0ull);
    }
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nb = 8 * cus;
    uint64_t* d = nullptr;
    hipMalloc(&d, 16 * nb);
    std::vector<uint64_t> h(2 * nb);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(k_res, dim3(nb), dim3(128), 0, 0, d, mode);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), d, 16 * nb, hipMemcpyDeviceToHost);
        uint64_t tmin = ~0ull;
        for (int b = 0; b < nb; ++b) tmin = std::min(tmin, h[2 * b]);
        // per (xcc, se, sh, cu): workgroups started within 0.5 ms of the first start
        std::map<uint64_t, int> early, all;
        for (int b = 0; b < nb; ++b) {
            const uint64_t id = h[2 * b + 1];
            const uint32_t hw = (uint32_t)id;
            const uint64_t key = ((id >> 32) & 15) << 16 | ((hw >> 8) & 15) | ((hw >> 12) & 1) << 4 | ((hw >> 13) & 3) << 5;
            all[key]++;
            if (h[2 * b] - tmin < 50000) early[key]++;
        }
        int mx = 0, mn = 1 << 30;
        for (auto& kv : early) { mx = std::max(mx, kv.second); mn = std::min(mn, kv.second); }
        uint64_t tmax = 0;
        for (int b = 0; b < nb; ++b) tmax = std::max(tmax, h[2 * b]);
        printf("mode %d (%s): %zu CUs seen, workgroups started in the first 0.5 ms per CU: min %d max %d; "
               "last start %.2f ms after the first\n", mode, mode ? "second wave waits in a barrier" : "second wave exits",
               all.size(), mn, mx, (tmax - tmin) / 1e5);
    }
    return 0;
}
