// Probe (diagnostic, not product code): how long s_sleep N sleeps on this GPU
// (shader clocks from s_memtime, 1000 sleeps per N, one wave).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <int N>
__global__ void k_sleep(uint64_t* out) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 1000; ++i) __builtin_amdgcn_s_sleep(N);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

int main() {
    uint64_t* d = nullptr;
    hipMalloc(&d, 8);
    uint64_t h = 0;
#define RUN(N)                                                                 \
    hipLaunchKernelGGL(k_sleep<N>, dim3(1), dim3(64), 0, 0, d);               \
    hipDeviceSynchronize();                                                    \
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);                                \
    printf("s_sleep %3d: %.1f clocks each\n", N, h / 1000.0);
    RUN(0) RUN(1) RUN(2) RUN(4) RUN(7) RUN(8) RUN(15) RUN(16) RUN(64) RUN(127)
    return 0;
}
