// Probe (diagnostic, not product code): LDS issue cost of the decoder's copy
// patterns.  One workgroup of 64 lanes per CU slot (8 per CU, like k_decode),
// each wave repeating N rounds of 8 independent LDS ops of one kind, then the
// time per op from s_memtime (cycles at the shader clock's constant rate).
//   w8c   ds_write_b8, 64 consecutive bytes (4 lanes per dword: same-bank bytes)
//   w8s   ds_write_b8, stride 4 (one byte per dword, 64 dwords)
//   w32   ds_write_b32, 64 consecutive dwords
//   r8c   ds_read_u8, 64 consecutive bytes
//   r128b ds_read_b128, every lane the same 16 bytes (broadcast)
//   hop   ds_read_u16, every lane the same address, each read's address from
//         the previous one (the decoder's hop chain: latency, not rate)
//   r64b / r32b  ds_read_b64 / ds_read_b32, every lane the same address
// Prints cycles per op for 1 and 8 waves per CU.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int K>
__global__ void __launch_bounds__(64) k_lds(uint32_t rounds, uint64_t* cyc, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[16384];
    const uint32_t L = threadIdx.x;
    for (uint32_t i = L; i < 4096; i += 64) reinterpret_cast<uint32_t*>(buf)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t base = (r * 1664525u) & 8191u & ~255u;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint32_t o = base + 512u * g;
            if constexpr (K == 0) buf[o + L] = (uint8_t)(L + r);
            else if constexpr (K == 1) buf[o + 4 * L] = (uint8_t)(L + r);
            else if constexpr (K == 2) reinterpret_cast<uint32_t*>(buf + o)[L] = L + r;
            else if constexpr (K == 3) acc += buf[o + L];
            else if constexpr (K == 4) { const v4u q = *reinterpret_cast<const v4u*>(buf + o); acc += q.x ^ q.w; }
            else if constexpr (K == 5) acc = *reinterpret_cast<const uint16_t*>(buf + ((acc + o) & 0x3FFEu));   // dependent chain
            else if constexpr (K == 6) { const uint64_t q = *reinterpret_cast<const uint64_t*>(buf + o); acc += (uint32_t)q ^ (uint32_t)(q >> 32); }
            else acc += *reinterpret_cast<const uint32_t*>(buf + o);
        }
        __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (L == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + L] = acc;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const char* names[8] = {"w8c  ds_write_b8 x64 consecutive", "w8s  ds_write_b8 stride 4",
                            "w32  ds_write_b32 x64 consecutive", "r8c  ds_read_u8 x64 consecutive",
                            "r128b ds_read_b128 broadcast", "hop  ds_read_u16 dependent chain",
                            "r64b ds_read_b64 broadcast", "r32b ds_read_b32 broadcast"};
    uint64_t* cyc = nullptr;
    uint32_t* sink = nullptr;
    hipMalloc(&cyc, 8 * 8 * cus);
    hipMalloc(&sink, 4 * 64 * 8 * cus);
    const uint32_t rounds = 20000;
    for (int k = 0; k < 8; ++k) {
        for (int per = 1; per <= 8; per *= 8) {
            const uint32_t nb = per * cus;
            auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(nb), dim3(64), 0, 0, rounds, cyc, sink); };
            switch (k) {
                case 0: launch(k_lds<0>); break;
                case 1: launch(k_lds<1>); break;
                case 2: launch(k_lds<2>); break;
                case 3: launch(k_lds<3>); break;
                case 4: launch(k_lds<4>); break;
                case 5: launch(k_lds<5>); break;
                case 6: launch(k_lds<6>); break;
                default: launch(k_lds<7>); break;
            }
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            uint64_t h[8 * 256] = {0};
            hipMemcpy(h, cyc, 8 * nb, hipMemcpyDeviceToHost);
            double avg = 0;
            for (uint32_t b = 0; b < nb; ++b) avg += (double)h[b] / nb;
            printf("%-36s %d wave(s)/CU: %.2f memtime ticks per op per wave\n", names[k], per, avg / (rounds * 8.0));
        }
    }
    return 0;
}
