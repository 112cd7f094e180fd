// Probe (diagnostic, not product code): can a kernel launched BEFORE its
// input exists wait for it block by block?  The host fills a coherent pinned
// buffer (hipHostMallocCoherent: GPU reads of it are never served from a GPU
// cache) one 4 MiB block at a time and then sets that block's flag (a u32 in
// the same coherent memory, after a release fence); each wave polls its
// block's flag with system-scope loads (s_sleep between polls, a wall-clock
// timeout from s_memrealtime, 100 MHz), then pulls its block into device
// memory with 16-byte loads and XXH-like sums it.  Prints per-block pull
// latency after the flag, the overall pull rate, and whether every block's
// sum matches the host's.  No hang path: every wave exits by its deadline.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(64) k_wait_pull(const uint8_t* host, uint8_t* dev, const uint32_t* flags,
                                                  uint32_t bm, uint64_t deadline, uint32_t* sums, uint64_t* when) {
    const uint32_t b = blockIdx.x, L = threadIdx.x;
    uint32_t f = 0;
    for (;;) {
        f = __hip_atomic_load(flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (f) break;
        if (__builtin_amdgcn_s_memrealtime() > deadline) break;
        __builtin_amdgcn_s_sleep(64);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (!f) {   // timed out
        if (L == 0) { sums[b] = 0xDEADu; when[b] = 0; }
        return;
    }
    const v4u* src = reinterpret_cast<const v4u*>(host + (uint64_t)b * bm);
    v4u* dst = reinterpret_cast<v4u*>(dev + (uint64_t)b * bm);
    uint32_t acc = 0;
    for (uint32_t i = L; i < bm / 16; i += 64 * 8) {
        v4u v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = src[i + 64 * k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            dst[i + 64 * k] = v[k];
            acc += v[k].x * 3u + v[k].y * 5u + v[k].z * 7u + v[k].w * 11u;
        }
    }
    for (int d = 32; d > 0; d >>= 1) acc += __shfl_xor(acc, d, 64);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (L == 0) {
        sums[b] = acc;
        when[b] = __builtin_amdgcn_s_memrealtime() - t0;
    }
}

__global__ void k_now(uint64_t* o) { *o = __builtin_amdgcn_s_memrealtime(); }

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                      \
        }                                                                  \
    } while (0)

int main(int argc, char** argv) {
    const uint32_t nb = argc > 1 ? atoi(argv[1]) : 512, bm = 4u << 20;
    const uint64_t n = (uint64_t)nb * bm;
    uint8_t *h = nullptr, *d = nullptr;
    uint32_t *flags = nullptr, *sums = nullptr;
    uint64_t* when = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), n, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc(reinterpret_cast<void**>(&flags), nb * 4, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipMalloc(reinterpret_cast<void**>(&d), n));
    CK(hipMalloc(reinterpret_cast<void**>(&sums), nb * 4));
    CK(hipMalloc(reinterpret_cast<void**>(&when), nb * 8));
    for (int pass = 0; pass < 3; ++pass) {
        memset(flags, 0, nb * 4);
        std::atomic_thread_fence(std::memory_order_seq_cst);
        // deadline: 20 s from now on the GPU's 100 MHz clock (read by a tiny kernel)
        uint64_t* dnow = nullptr;
        CK(hipMalloc(reinterpret_cast<void**>(&dnow), 8));
        hipLaunchKernelGGL(k_now, dim3(1), dim3(1), 0, 0, dnow);
        uint64_t now = 0;
        CK(hipMemcpy(&now, dnow, 8, hipMemcpyDeviceToHost));
        CK(hipFree(dnow));
        hipStream_t st;
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_wait_pull, dim3(nb), dim3(64), 0, st, h, d, flags, bm, now + 20ull * 100000000ull, sums, when);
        CK(hipGetLastError());
        std::vector<uint32_t> want(nb);
        // the "reader": fill block by block (a memset-like pattern + mix), then publish
        for (uint32_t b = 0; b < nb; ++b) {
            uint32_t* w = reinterpret_cast<uint32_t*>(h + (uint64_t)b * bm);
            uint32_t acc = 0;
            for (uint32_t i = 0; i < bm / 4; i += 4) {
                for (int k = 0; k < 4; ++k) w[i + k] = (b * 2654435761u) ^ ((i + k) * 40503u) ^ (uint32_t)pass;
                acc += w[i] * 3u + w[i + 1] * 5u + w[i + 2] * 7u + w[i + 3] * 11u;
            }
            want[b] = acc;
            std::atomic_thread_fence(std::memory_order_release);
            __atomic_store_n(flags + b, 1u, __ATOMIC_RELEASE);
        }
        const double tRead = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CK(hipStreamSynchronize(st));
        const double tAll = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::vector<uint32_t> got(nb);
        std::vector<uint64_t> tw(nb);
        CK(hipMemcpy(got.data(), sums, nb * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(tw.data(), when, nb * 8, hipMemcpyDeviceToHost));
        uint32_t bad = 0;
        double mx = 0, avg = 0;
        for (uint32_t b = 0; b < nb; ++b) {
            bad += got[b] != want[b];
            mx = std::max(mx, tw[b] / 100.0);
            avg += tw[b] / 100.0 / nb;
        }
        printf("pass %d: %u blocks of 4 MiB: host fill %.1f ms (%.1f GB/s), all pulled %.1f ms after launch; "
               "per-block pull after its flag avg %.1f us max %.1f us; %u mismatches\n",
               pass, nb, tRead * 1e3, n / tRead / 1e9, tAll * 1e3, avg, mx, bad);
        CK(hipStreamDestroy(st));
    }
    return 0;
}
