// Probe (diagnostic, not product code): does a co-resident idle wave slow a
// working wave?  128-lane workgroups, 20432 B of LDS (8 per CU), wave 0 runs
// a fixed dependent LDS + VALU loop; wave 1 exits at once (mode 0), waits in
// a barrier (mode 1) or sleeps in s_sleep polls of an LDS word (mode 2).
// Prints wave 0's wall time (s_memrealtime, 100 MHz) and shader clocks
// (s_memtime) averaged over the workgroups.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(128) k_work(uint64_t* out, int mode, uint32_t iters, const uint32_t* __restrict__ g,
                                              int gmode) {
    __shared__ uint32_t pad[5108];
    __shared__ uint32_t flag;
    const uint32_t wave = threadIdx.x >> 6, L = threadIdx.x & 63;
    if (threadIdx.x == 0) flag = 0;
    for (uint32_t i = threadIdx.x; i < 5108; i += 128) pad[i] = i * 2654435761u;
    __syncthreads();
    if (wave == 1) {
        if (mode == 1) __syncthreads();
        if (mode == 2) while (__hip_atomic_load(&flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(127);
        return;
    }
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    uint32_t x = L, acc = 0;
    if (gmode) {   // a dependent global read (64 MiB table: HBM / MALL) + an LDS read per step
        uint32_t y = blockIdx.x * 977u + L;
        for (uint32_t i = 0; i < iters / 50; ++i) {
            y = g[(y * 2654435761u + i) & ((16u << 20) - 1u)];
            x = pad[(x + y) & 4095];
            acc += x * 3u + (y >> 7);
        }
    } else {
        for (uint32_t i = 0; i < iters; ++i) {   // a dependent LDS read + a few VALU ops per step
            x = pad[(x + i) & 4095];
            acc += x * 3u + (x >> 7);
        }
    }
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
    if (mode == 1) __syncthreads();
    if (mode == 2 && L == 0) __hip_atomic_store(&flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (L == 0) {
        out[3 * blockIdx.x] = r1 - r0;
        out[3 * blockIdx.x + 1] = c1 - c0;
        out[3 * blockIdx.x + 2] = acc;
    }
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int nb = 8 * cus;
    uint64_t* d = nullptr;
    hipMalloc(&d, 24 * nb);
    uint32_t* g = nullptr;
    hipMalloc(&g, 64u << 20);
    std::vector<uint32_t> hg(16u << 20);
    for (size_t i = 0; i < hg.size(); ++i) hg[i] = (uint32_t)(i * 2246822519u);
    hipMemcpy(g, hg.data(), 64u << 20, hipMemcpyHostToDevice);
    std::vector<uint64_t> h(3 * nb);
    for (int gmode = 0; gmode < 2; ++gmode)
        for (int mode = 0; mode < 3; ++mode) {
            hipLaunchKernelGGL(k_work, dim3(nb), dim3(128), 0, 0, d, mode, 200000u, g, gmode);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), d, 24 * nb, hipMemcpyDeviceToHost);
            double wall = 0, clk = 0;
            for (int b = 0; b < nb; ++b) { wall += h[3 * b] / 100.0 / nb; clk += (double)h[3 * b + 1] / nb; }
            printf("%s mode %d (%s): wave 0 %.1f us wall, %.0f shader clocks (%.2f GHz)\n",
                   gmode ? "global+LDS chain" : "LDS chain", mode, mode == 0 ? "wave 1 exits" : mode == 1 ? "wave 1 in a barrier" : "wave 1 polls in s_sleep",
                   wall, clk, clk / wall / 1000.0);
        }
    return 0;
}
