// Probe for DESIGN.md §4c, third hypothesis: under LDS traffic from a co-resident workgroup,
// does `s_waitcnt vmcnt(0)` + `s_barrier` still order an LDS-DMA (global_load_lds_dwordx4)
// write before other waves' ds_reads of the same bytes?
//
// victim: k_gl4's K-loop schedule without any extra wait: two LDS stages; per chunk c:
//         vmcnt(0); s_barrier; LDS-DMA of chunk c+1 into the other stage; every wave reads the
//         whole of stage c with ds_read_b128 and compares it with the value the source holds
//         there -- computed in registers (no global load, so no compiler vmcnt wait that would
//         retire the in-flight DMA early).  Counts stale words.
// partner: k_update's LDS pattern (static 16 x 16 tables, wave-uniform ds_read_b128 broadcasts),
//         looped to stay resident, on another stream.
// Cases: victim alone; victim with partner launched before / after it; LDS-DMA vs the
// register-staged control (global_load_dwordx4 + ds_write_b128, lgkmcnt(0) before the barrier).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_dma_race_probe tools/lds_dma_race_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

typedef __attribute__((address_space(3))) void lds_void;

__host__ __device__ __forceinline__ unsigned val(unsigned i) { return (i * 2654435761u) ^ 0xA5A5A5A5u; }

template <int METHOD>  // 0 LDS-DMA, 1 register staged
__global__ __launch_bounds__(512) void victim(const unsigned* __restrict__ src, unsigned* out, int stage_bytes,
                                              int chunks, int reps) {
    extern __shared__ __attribute__((aligned(16))) unsigned db[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int swords = stage_bytes / 4, pieces = stage_bytes / 1024;
    unsigned* st[2] = {db, db + swords};
    unsigned bad = 0;
    auto fill = [&](int c, unsigned* dst) {
        const unsigned* s = src + (size_t)c * swords;
        for (int p = wave; p < pieces; p += 8) {
            if (METHOD == 0) {
                __builtin_amdgcn_global_load_lds((const void*)(s + (size_t)p * 256 + lane * 4), (lds_void*)(dst + (size_t)p * 256),
                                                 16, 0, 0);
            } else {
                const uint4 v = *reinterpret_cast<const uint4*>(s + (size_t)p * 256 + lane * 4);
                *reinterpret_cast<uint4*>(dst + (size_t)p * 256 + lane * 4) = v;
            }
        }
    };
    for (int r = 0; r < reps; ++r) {
        fill(0, st[0]);
        for (int c = 0; c < chunks; ++c) {
            if (METHOD == 0) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            else __builtin_amdgcn_s_waitcnt(0xC07F);              // lgkmcnt(0): own ds_writes done
            __builtin_amdgcn_s_barrier();
            if (c + 1 < chunks) fill(c + 1, st[(c + 1) & 1]);
            const unsigned base = (unsigned)c * swords;
            // the reads as inline asm: hipcc tracks in-flight LDS-DMA and would put a vmcnt(0) in
            // front of a plain ds_read that may alias it (k_gl4's reads get none: see DESIGN.md)
            const unsigned lbase = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)st[c & 1];
            for (int q = threadIdx.x; q < swords / 4; q += 512) {
                uint4 v;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(lbase + 16u * q) : "memory");
                const unsigned i = base + 4 * q;
                bad += (v.x != val(i)) + (v.y != val(i + 1)) + (v.z != val(i + 2)) + (v.w != val(i + 3));
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_s_barrier();
    }
    for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor((int)bad, o);
    if (lane == 0 && bad) atomicAdd(out, bad);
}

__global__ __launch_bounds__(256) void partner(const float* C1, const float* C2, const float* U, float* out, int iters) {
    __shared__ float sC1[256], sC2[256], sU[256];
    for (int i = threadIdx.x; i < 256; i += 256) {
        sC1[i] = C1[i];
        sC2[i] = C2[i];
        sU[i] = U[i];
    }
    __syncthreads();
    float x[16];
    for (int j = 0; j < 16; ++j) x[j] = (float)(threadIdx.x + j);
    float acc = 0.f;
    for (int it = 0; it < iters; ++it)
        for (int i = 0; i < 16; ++i) {
            float m = 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) m += (sC1[i * 16 + j] + sC2[i * 16 + j] + sU[i * 16 + j]) * x[j];
            acc += m;
            x[i & 15] += 1e-7f * m;
        }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHECK(hipFuncSetAttribute((const void*)victim<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute((const void*)victim<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int chunks = 12, max_stage = 61 * 1024;
    std::vector<unsigned> h((size_t)chunks * max_stage / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = val((unsigned)i);
    unsigned *src, *bad;
    float *tab, *pout;
    CHECK(hipMalloc(&src, h.size() * 4));
    CHECK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&bad, 4));
    CHECK(hipMalloc(&tab, 3 * 256 * 4));
    CHECK(hipMemset(tab, 0, 3 * 256 * 4));
    const int p_wg = cus * 4;
    CHECK(hipMalloc(&pout, (size_t)p_wg * 256 * 4));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    unsigned long long total_dma = 0, total_reg = 0;
    for (int method = 0; method < 2; ++method)
        for (int order = 0; order < 3; ++order)  // 0 alone, 1 partner first, 2 victim first
            for (int stage_kb : {20, 30, 40, 41, 60, 61}) {
                for (int rep = 0; rep < 3; ++rep) {
                    CHECK(hipMemset(bad, 0, 4));
                    CHECK(hipDeviceSynchronize());
                    const size_t lds = (size_t)2 * stage_kb * 1024;
                    auto lv = [&] {
                        if (method == 0)
                            hipLaunchKernelGGL(victim<0>, dim3(cus * 2), dim3(512), lds, s2, src, bad, stage_kb * 1024, chunks, 40);
                        else
                            hipLaunchKernelGGL(victim<1>, dim3(cus * 2), dim3(512), lds, s2, src, bad, stage_kb * 1024, chunks, 40);
                    };
                    auto lp = [&] {
                        if (order) hipLaunchKernelGGL(partner, dim3(p_wg), dim3(256), 0, s1, tab, tab + 256, tab + 512, pout, 400);
                    };
                    if (order == 1) lp();
                    lv();
                    if (order == 2) lp();
                    CHECK(hipGetLastError());
                    CHECK(hipDeviceSynchronize());
                    unsigned b = 0;
                    CHECK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
                    (method ? total_reg : total_dma) += b;
                    printf("%-9s %-13s stage %2d KB (alloc %3d KB) rep %d: stale words %u\n", method ? "reg-stage" : "lds-dma",
                           order == 0 ? "alone" : order == 1 ? "partner-first" : "victim-first", stage_kb, 2 * stage_kb, rep, b);
                    fflush(stdout);
                }
            }
    printf("TOTAL stale words: lds-dma %llu, reg-stage %llu\n", total_dma, total_reg);
    return 0;
}
