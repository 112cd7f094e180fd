// Probe (diagnostic, not product code): which SIMD each wave of a workgroup
// lands on (HW_REG_HW_ID), for 64- and 128-lane workgroups at 8 workgroups per
// CU (20 KiB of LDS each, like k_decode / k_decode2).  Prints, per
// workgroup size, how many waves of wave index w landed on each SIMD.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int T>
__global__ void __launch_bounds__(T) k_where(uint32_t* out) {
    __shared__ uint8_t pad[20432];
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID, all 32 bits
    if ((threadIdx.x & 63) == 0) {
        pad[threadIdx.x] = 1;
        out[blockIdx.x * (T / 64) + threadIdx.x / 64] = hw;
    }
    // keep the workgroups resident together
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 200000) __builtin_amdgcn_s_sleep(10);
    if (pad[0] == 7) out[0] = 0;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nb = 8 * cus;
    uint32_t* d = nullptr;
    hipMalloc(&d, 4 * nb * 2);
    static uint32_t h[2048 * 8 * 2];
    for (int pass = 0; pass < 2; ++pass) {
        const int wpg = pass ? 2 : 1;
        if (pass) hipLaunchKernelGGL(k_where<128>, dim3(nb), dim3(128), 0, 0, d);
        else hipLaunchKernelGGL(k_where<64>, dim3(nb), dim3(64), 0, 0, d);
        hipDeviceSynchronize();
        hipMemcpy(h, d, 4 * nb * wpg, hipMemcpyDeviceToHost);
        int cnt[2][4] = {{0}};
        int samesimd = 0;
        for (int b = 0; b < nb; ++b) {
            for (int w = 0; w < wpg; ++w) cnt[w][(h[b * wpg + w] >> 4) & 3]++;
            if (wpg == 2 && ((h[b * 2] >> 4) & 3) == ((h[b * 2 + 1] >> 4) & 3)) samesimd++;
        }
        printf("%d-lane workgroups: ", 64 * wpg);
        for (int w = 0; w < wpg; ++w)
            printf("wave %d on SIMD0..3: %d %d %d %d; ", w, cnt[w][0], cnt[w][1], cnt[w][2], cnt[w][3]);
        if (wpg == 2) printf("both waves on one SIMD: %d of %d", samesimd, nb);
        printf("\n");
        if (pass) {   // the first few workgroups' placements
            for (int b = 0; b < 24; ++b)
                printf("wg %d: hw0 %08x (simd %u cu %u) hw1 %08x (simd %u cu %u)\n", b, h[2 * b], (h[2 * b] >> 4) & 3,
                       (h[2 * b] >> 8) & 15, h[2 * b + 1], (h[2 * b + 1] >> 4) & 3, (h[2 * b + 1] >> 8) & 15);
        }
    }
    return 0;
}
