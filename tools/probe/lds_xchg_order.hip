// Probe (diagnostic, not product code): the order in which one wave's
// same-address LDS exchanges (ds_wrxchg_rtn_b32) are applied on this GPU.
// For random address patterns it checks the hypothesis "ascending lane
// order": lane L gets the value of the highest lane < L with the same
// address (or the initial value), and memory ends holding the highest
// lane's value.  Prints the counts of trials that match / do not match.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

__global__ void __launch_bounds__(64) k_probe(const uint32_t* addr, uint32_t* ret, uint32_t* fin, int trials, int nAddr) {
    __shared__ uint32_t T[64];
    const int L = threadIdx.x;
    for (int t = blockIdx.x; t < trials; t += gridDim.x) {
        if (L < nAddr) T[L] = 0xFFFF0000u | (uint32_t)L;   // initial values
        __syncthreads();
        const uint32_t a = addr[t * 64 + L];
        const uint32_t mine = 0x1000u * (uint32_t)t + (uint32_t)L;
        ret[t * 64 + L] = __hip_atomic_exchange(&T[a], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        if (L < nAddr) fin[t * 64 + L] = T[L];
        __syncthreads();
    }
}

int main() {
    const int trials = 20000;
    std::mt19937 rng(1);
    long ok = 0, bad = 0, okFin = 0, badFin = 0, lowWins = 0;
    for (int nAddr : {1, 2, 4, 16, 64}) {
        std::vector<uint32_t> addr(trials * 64), ret(trials * 64), fin(trials * 64);
        for (auto& x : addr) x = rng() % nAddr;
        uint32_t *dA, *dR, *dF;
        hipMalloc(&dA, addr.size() * 4); hipMalloc(&dR, ret.size() * 4); hipMalloc(&dF, fin.size() * 4);
        hipMemcpy(dA, addr.data(), addr.size() * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_probe, dim3(1024), dim3(64), 0, 0, dA, dR, dF, trials, nAddr);
        hipMemcpy(ret.data(), dR, ret.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(fin.data(), dF, fin.size() * 4, hipMemcpyDeviceToHost);
        long b0 = bad;
        for (int t = 0; t < trials; ++t) {
            for (int L = 0; L < 64; ++L) {
                const uint32_t a = addr[t * 64 + L];
                uint32_t want = 0xFFFF0000u | a;
                for (int j = L - 1; j >= 0; --j)
                    if (addr[t * 64 + j] == a) { want = 0x1000u * (uint32_t)t + (uint32_t)j; break; }
                (ret[t * 64 + L] == want ? ok : bad)++;
            }
            for (int a = 0; a < nAddr; ++a) {
                int hi = -1, lo = -1;
                for (int L = 0; L < 64; ++L)
                    if (addr[t * 64 + L] == (uint32_t)a) { hi = L; if (lo < 0) lo = L; }
                if (hi < 0) continue;
                const uint32_t got = fin[t * 64 + a];
                (got == 0x1000u * (uint32_t)t + (uint32_t)hi ? okFin : badFin)++;
                if (got == 0x1000u * (uint32_t)t + (uint32_t)lo && lo != hi) lowWins++;
            }
        }
        printf("nAddr %2d: returns matching ascending-lane order %s (%ld mismatching lanes)\n", nAddr,
               bad == b0 ? "ALL" : "NOT ALL", bad - b0);
        hipFree(dA); hipFree(dR); hipFree(dF);
    }
    printf("lanes ok %ld bad %ld; final values ok %ld bad %ld (lowest-lane-wins %ld)\n", ok, bad, okFin, badFin, lowWins);
    return bad || badFin;
}
