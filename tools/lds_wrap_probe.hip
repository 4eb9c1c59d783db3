// Probe for DESIGN.md §4c (round 2): do two co-resident workgroups of DIFFERENT kernels, each
// using only plain ds_write / ds_read on its own dynamic LDS, keep their LDS intact?
//
// big:   one workgroup per CU, B KB of dynamic LDS filled with a pattern keyed by (kernel, block,
//        word), then re-verified for ~2 ms while it sleeps between passes;
// small: launched on another stream while `big` is resident, S KB per workgroup, several
//        workgroups per CU, same fill / verify loop with its own pattern.
// Each counts words that differ from its own pattern (and notes whether the bad value carries
// the OTHER kernel's tag).  Also reads HW_REG_LDS_ALLOC to report the LDS base each workgroup got.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_wrap_probe tools/lds_wrap_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

__device__ __forceinline__ unsigned lds_alloc_reg() { return __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 6); }

__device__ __forceinline__ unsigned pat(unsigned tag, unsigned blk, unsigned i) {
    return (tag << 28) | ((blk & 0xFFF) << 16) | (i & 0xFFFF);
}

// counters: [0] mismatches, [1] mismatches carrying the other kernel's tag, [2] max LDS base (x256 B)
__global__ void fillcheck(unsigned tag, unsigned other, int words, int passes, int sleeps, unsigned* cnt) {
    extern __shared__ unsigned sm[];
    const unsigned blk = blockIdx.x;
    for (int i = threadIdx.x; i < words; i += blockDim.x) sm[i] = pat(tag, blk, i);
    __syncthreads();
    unsigned bad = 0, foreign = 0;
    for (int p = 0; p < passes; ++p) {
        for (int s = 0; s < sleeps; ++s) __builtin_amdgcn_s_sleep(127);
        for (int i = threadIdx.x; i < words; i += blockDim.x) {
            const unsigned v = sm[i];
            if (v != pat(tag, blk, i)) {
                ++bad;
                foreign += (v >> 28) == other;
                sm[i] = pat(tag, blk, i);  // repair, so later passes count new hits only
            }
        }
        __syncthreads();
    }
    if (bad) atomicAdd(&cnt[0], bad);
    if (foreign) atomicAdd(&cnt[1], foreign);
    if (threadIdx.x == 0) atomicMax(&cnt[2], lds_alloc_reg() & 0xFFFF);
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHECK(hipFuncSetAttribute((const void*)fillcheck, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    unsigned *cb, *cs;
    CHECK(hipMalloc(&cb, 16));
    CHECK(hipMalloc(&cs, 16));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    unsigned long long tot_big = 0, tot_small = 0;
    printf("CUs %d\n", cus);
    for (int bkb : {0, 32, 60, 64, 66, 80, 100, 120, 140}) {
        for (int skb : {4, 20, 40}) {
            if (bkb + skb > 160) continue;
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipMemset(cb, 0, 16));
                CHECK(hipMemset(cs, 0, 16));
                CHECK(hipDeviceSynchronize());
                if (bkb) hipLaunchKernelGGL(fillcheck, dim3(cus), dim3(256), bkb * 1024, s1, 1u, 2u, bkb * 256, 40, 8, cb);
                hipLaunchKernelGGL(fillcheck, dim3(cus * 6), dim3(256), skb * 1024, s2, 2u, 1u, skb * 256, 20, 4, cs);
                CHECK(hipGetLastError());
                CHECK(hipDeviceSynchronize());
                unsigned hb[4], hs[4];
                CHECK(hipMemcpy(hb, cb, 16, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(hs, cs, 16, hipMemcpyDeviceToHost));
                tot_big += hb[0];
                tot_small += hs[0];
                printf("big %3d KB  small %2d KB x %d/CU rep %d: big bad %u (foreign %u, max base %u x256B) | small bad %u "
                       "(foreign %u, max base %u x256B)\n",
                       bkb, skb, 6, rep, hb[0], hb[1], hb[2], hs[0], hs[1], hs[2]);
                fflush(stdout);
            }
        }
    }
    printf("TOTAL bad words: big %llu, small %llu\n", tot_big, tot_small);
    return 0;
}
