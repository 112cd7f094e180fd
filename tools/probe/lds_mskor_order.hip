// Probe (diagnostic, not product code): one wave's same-address masked-OR
// exchanges (ds_mskor_rtn_b32, each lane replacing only its own 16-bit half or
// byte of a shared dword) -- are they applied in ascending lane order, like
// ds_wrxchg_rtn_b32 (lds_xchg_order.hip)?  Lane L writes field f(L) of dword
// a(L); it must get the field's value left by the highest lane < L writing the
// same field of the same dword (or the initial value), and the other fields of
// the dword must never be disturbed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

__device__ __forceinline__ uint32_t mskor_rtn(uint32_t* lds, uint32_t mask, uint32_t data) {
    uint32_t r;
    const uint32_t addr = (uint32_t)(uintptr_t)lds;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr), "v"(mask), "v"(data) : "memory");
    return r;
}

__global__ void __launch_bounds__(64) k_probe(const uint32_t* sel, uint32_t* ret, uint32_t* fin, int trials, int nWords, int fieldBits) {
    __shared__ uint32_t W[64];
    const int L = threadIdx.x;
    const int nf = 32 / fieldBits;
    const uint32_t fm = fieldBits == 32 ? 0xFFFFFFFFu : ((1u << fieldBits) - 1u);
    for (int t = blockIdx.x; t < trials; t += gridDim.x) {
        if (L < nWords) W[L] = 0xA5A5A5A5u ^ (uint32_t)L * 0x01010101u;
        __syncthreads();
        const uint32_t s = sel[t * 64 + L];
        const uint32_t a = s / nf, f = s % nf, sh = f * fieldBits;
        const uint32_t mine = (uint32_t)(t * 64 + L) & fm;
        const uint32_t old = mskor_rtn(&W[a], fm << sh, mine << sh);
        ret[t * 64 + L] = (old >> sh) & fm;
        __syncthreads();
        if (L < nWords) fin[t * 64 + L] = W[L];
        __syncthreads();
    }
}

int main() {
    const int trials = 20000;
    std::mt19937 rng(3);
    long bad = 0, badFin = 0, ok = 0;
    for (int fb : {16, 8}) {
        const int nf = 32 / fb;
        const uint32_t fm = (1u << fb) - 1u;
        for (int nWords : {1, 2, 8, 32}) {
            std::vector<uint32_t> sel(trials * 64), ret(trials * 64), fin(trials * 64);
            for (auto& x : sel) x = rng() % (uint32_t)(nWords * nf);
            uint32_t *dS, *dR, *dF;
            (void)hipMalloc(&dS, sel.size() * 4); (void)hipMalloc(&dR, ret.size() * 4); (void)hipMalloc(&dF, fin.size() * 4);
            (void)hipMemcpy(dS, sel.data(), sel.size() * 4, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k_probe, dim3(1024), dim3(64), 0, 0, dS, dR, dF, trials, nWords, fb);
            (void)hipMemcpy(ret.data(), dR, ret.size() * 4, hipMemcpyDeviceToHost);
            (void)hipMemcpy(fin.data(), dF, fin.size() * 4, hipMemcpyDeviceToHost);
            long b0 = bad, f0 = badFin;
            for (int t = 0; t < trials; ++t) {
                for (int L = 0; L < 64; ++L) {
                    const uint32_t s = sel[t * 64 + L], a = s / nf, f = s % nf;
                    uint32_t want = ((0xA5A5A5A5u ^ a * 0x01010101u) >> (f * fb)) & fm;
                    for (int j = L - 1; j >= 0; --j)
                        if (sel[t * 64 + j] == s) { want = (uint32_t)(t * 64 + j) & fm; break; }
                    (ret[t * 64 + L] == want ? ok : bad)++;
                }
                for (uint32_t a = 0; a < (uint32_t)nWords; ++a) {
                    uint32_t want = 0xA5A5A5A5u ^ a * 0x01010101u;
                    for (int L = 0; L < 64; ++L) {
                        const uint32_t s = sel[t * 64 + L];
                        if (s / nf == a) { const uint32_t sh = (s % nf) * fb; want = (want & ~(fm << sh)) | (((uint32_t)(t * 64 + L) & fm) << sh); }
                    }
                    if (fin[t * 64 + a] != want) badFin++;
                }
            }
            printf("field %2d bits, %2d words: %s (%ld lanes, %ld words off)\n", fb, nWords,
                   bad == b0 && badFin == f0 ? "ascending lane order" : "NOT in lane order", bad - b0, badFin - f0);
            (void)hipFree(dS); (void)hipFree(dR); (void)hipFree(dF);
        }
    }
    printf("lanes ok %ld bad %ld, final words bad %ld\n", ok, bad, badFin);
    return bad || badFin;
}
