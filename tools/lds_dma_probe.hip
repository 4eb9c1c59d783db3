// Probe for DESIGN.md §4c: does an LDS-DMA (global_load_lds_dwordx4) fill land where and when
// the ordering rules say, when another workgroup shares the CU?
//
// Partner kernels (one stream): small LDS allocations that
//   sleeper: fill their LDS with a pattern, re-check it between s_sleeps;
//   rmw:     read-modify-write their own words in a tight loop (heavy LDS traffic);
//   bcast:   wave-uniform broadcast reads of a table in a tight loop (k_update's access pattern);
// and count words that were not what they last wrote.
// Victim kernels (another stream, concurrently): a large dynamic LDS allocation filled by
//   flat:   sentinel fill (ds_write), barrier, LDS-DMA of the whole allocation, vmcnt(0),
//           barrier, check every word;
//   pipe:   k_gl4's K-loop schedule: two stages, per chunk c: vmcnt(0); s_barrier; LDS-DMA of
//           chunk c+1 into the other stage; check stage c against chunk c's source;
// with method lds-dma or (control) global load + ds_write.  Both kernels record their raw
// HW_REG_LDS_ALLOC.  Prints mismatch counts per case.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_dma_probe tools/lds_dma_probe.hip
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

// s_getreg_b32 hwreg(HW_REG_LDS_ALLOC) (id 6), 32 bits
__device__ __forceinline__ unsigned lds_alloc_reg() { return __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 6); }

__device__ __forceinline__ unsigned pat(unsigned wg, unsigned i) { return (wg * 2654435761u) ^ (i * 40503u) ^ 0x5A5A0000u; }

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor((int)v, o);
    return v;
}

// out[2 * blockIdx] = bad words, out[2 * blockIdx + 1] = LDS_ALLOC.  mode 0 sleeper, 1 rmw, 2 bcast
__global__ void partner(unsigned* out, int words, int iters, int mode) {
    extern __shared__ unsigned hb[];
    for (int i = threadIdx.x; i < words; i += blockDim.x) hb[i] = pat(blockIdx.x, i);
    __syncthreads();
    unsigned bad = 0, acc = 0;
    for (int it = 0; it < iters; ++it) {
        if (mode == 0) {
            __builtin_amdgcn_s_sleep(60);
            for (int i = threadIdx.x; i < words; i += blockDim.x) bad += hb[i] != pat(blockIdx.x, i);
        } else if (mode == 1) {
            const unsigned k0 = (unsigned)it * 0x9E3779B9u, k1 = (unsigned)(it + 1) * 0x9E3779B9u;
            for (int i = threadIdx.x; i < words; i += blockDim.x) {
                const unsigned v = hb[i];
                bad += v != (pat(blockIdx.x, i) ^ k0);
                hb[i] = pat(blockIdx.x, i) ^ k1;
            }
        } else {
            const int w = (threadIdx.x >> 6);
            for (int i = w; i < words; i += 4) {
                const unsigned v = hb[i];  // wave-uniform address: broadcast
                acc += v;
                bad += v != pat(blockIdx.x, i);
            }
        }
    }
    bad = wave_sum(bad) + (acc == 0x12345678u);
    __shared__ unsigned sb[16];
    if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = bad;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sb[w];
        out[2 * blockIdx.x] = t;
        out[2 * blockIdx.x + 1] = lds_alloc_reg();
    }
}

__device__ __forceinline__ void fill_piece(const unsigned* s, unsigned* d, int lane, int method) {
    if (method == 0) {
        __builtin_amdgcn_global_load_lds((const void*)(s + lane * 4), (lds_void*)d, 16, 0, 0);
    } else {
        const uint4 v = *reinterpret_cast<const uint4*>(s + lane * 4);
        *reinterpret_cast<uint4*>(d + lane * 4) = v;
    }
}

// out[4 * blockIdx] = wrong words, [+1] = LDS_ALLOC, [+2] = first wrong word (or ~0), [+3] = value
// kind 0 flat, 1 pipe (stage = bytes / 2, chunks = `chunks`, chunk c from src + c * stage)
__global__ void victim(const unsigned* __restrict__ src, unsigned* out, int bytes, int method, int kind, int reps,
                       int chunks) {
    extern __shared__ __attribute__((aligned(16))) unsigned db[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
    unsigned bad = 0, first = ~0u, val = 0;
    auto check = [&](const unsigned* ref, const unsigned* l, int words, int base) {
        for (int i = threadIdx.x; i < words; i += blockDim.x) {
            const unsigned v = l[i];
            if (v != ref[i]) {
                ++bad;
                if ((unsigned)(base + i) < first) {
                    first = (unsigned)(base + i);
                    val = v;
                }
            }
        }
    };
    if (kind == 0) {
        const int words = bytes / 4, pieces = bytes / 1024;
        for (int r = 0; r < reps; ++r) {
            for (int i = threadIdx.x; i < words; i += blockDim.x) db[i] = 0xDEADBEEFu;
            __syncthreads();
            for (int p = wave; p < pieces; p += nw) fill_piece(src + (size_t)p * 256, db + (size_t)p * 256, lane, method);
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            check(src, db, words, 0);
            __syncthreads();
        }
    } else {
        const int sbytes = (bytes / 2) & ~1023, swords = sbytes / 4, pieces = sbytes / 1024;
        unsigned* st[2] = {db, db + swords};
        for (int r = 0; r < reps; ++r) {
            for (int i = threadIdx.x; i < 2 * swords; i += blockDim.x) db[i] = 0xDEADBEEFu;
            __syncthreads();
            for (int p = wave; p < pieces; p += nw) fill_piece(src + (size_t)p * 256, st[0] + (size_t)p * 256, lane, method);
            for (int c = 0; c < chunks; ++c) {
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (lgkm / exp counts left at max)
                __builtin_amdgcn_s_barrier();
                if (c + 1 < chunks) {
                    const unsigned* s = src + (size_t)(c + 1) * swords;
                    for (int p = wave; p < pieces; p += nw)
                        fill_piece(s + (size_t)p * 256, st[(c + 1) & 1] + (size_t)p * 256, lane, method);
                }
                check(src + (size_t)c * swords, st[c & 1], swords, (c & 1) * swords);
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this chunk's reads retired
            }
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
        }
    }
    bad = wave_sum(bad);
    unsigned f = first, fv = val;
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned of = __shfl_xor((int)f, o), ov = __shfl_xor((int)fv, o);
        if (of < f) {
            f = of;
            fv = ov;
        }
    }
    // reuse the start of the allocation for the reduction (all checks done, all DMAs waited)
    __syncthreads();
    if (lane == 0) {
        db[3 * wave] = bad;
        db[3 * wave + 1] = f;
        db[3 * wave + 2] = fv;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned tb = 0, tf = ~0u, tv = 0;
        for (int w = 0; w < nw; ++w) {
            tb += db[3 * w];
            if (db[3 * w + 1] < tf) {
                tf = db[3 * w + 1];
                tv = db[3 * w + 2];
            }
        }
        out[4 * blockIdx.x] = tb;
        out[4 * blockIdx.x + 1] = lds_alloc_reg();
        out[4 * blockIdx.x + 2] = tf;
        out[4 * blockIdx.x + 3] = tv;
    }
}

int main(int argc, char** argv) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHECK(hipFuncSetAttribute((const void*)victim, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute((const void*)partner, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));
    const int chunks = 12;
    const size_t src_bytes = (size_t)chunks * 80 * 1024;
    std::vector<unsigned> hsrc(src_bytes / 4);
    for (size_t i = 0; i < hsrc.size(); ++i) hsrc[i] = 0x10000000u + (unsigned)(i * 7u);
    unsigned *src, *pout, *vout;
    const int p_wg = cus * 2, v_wg = cus;
    CHECK(hipMalloc(&src, src_bytes));
    CHECK(hipMemcpy(src, hsrc.data(), src_bytes, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&pout, sizeof(unsigned) * 2 * p_wg));
    CHECK(hipMalloc(&vout, sizeof(unsigned) * 4 * v_wg));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    printf("CUs %d; partner %d wgs x 256 threads; victim %d wgs x 512 threads\n", cus, p_wg, v_wg);
    const char* pname[] = {"none", "sleeper", "rmw", "bcast"};
    const char* kname[] = {"flat", "pipe"};
    const int piters[] = {0, 60, 3000, 2000};
    unsigned long long total_bad = 0;
    for (int victim_first = 0; victim_first < 2; ++victim_first)
    for (int method = 0; method < 2; ++method)
        for (int kind = 0; kind < 2; ++kind)
            for (int pm = 0; pm < 4; ++pm)
                for (int pk : {4, 16})
                    for (int vk : {40, 64, 82, 96, 122}) {
                        if (pm == 0 && pk != 4) continue;
                        if (2 * pk + vk > 160) continue;
                        CHECK(hipMemset(pout, 0, sizeof(unsigned) * 2 * p_wg));
                        CHECK(hipMemset(vout, 0, sizeof(unsigned) * 4 * v_wg));
                        CHECK(hipDeviceSynchronize());
                        auto launch_partner = [&] {
                            if (pm)
                                hipLaunchKernelGGL(partner, dim3(p_wg), dim3(256), pk * 1024, s1, pout, pk * 256,
                                                   piters[pm], pm - 1);
                        };
                        if (!victim_first) launch_partner();
                        hipLaunchKernelGGL(victim, dim3(v_wg), dim3(512), vk * 1024, s2, src, vout, vk * 1024, method, kind,
                                           victim_first ? (kind ? 200 : 600) : (kind ? 8 : 30), chunks);
                        if (victim_first) launch_partner();
                        CHECK(hipGetLastError());
                        CHECK(hipDeviceSynchronize());
                        std::vector<unsigned> po(2 * p_wg), vo(4 * v_wg);
                        CHECK(hipMemcpy(po.data(), pout, po.size() * 4, hipMemcpyDeviceToHost));
                        CHECK(hipMemcpy(vo.data(), vout, vo.size() * 4, hipMemcpyDeviceToHost));
                        unsigned long long pbad = 0, vbad = 0;
                        int pwb = 0, vwb = 0;
                        unsigned ex_first = ~0u, ex_val = 0, ex_alloc = 0, any_alloc = vo[1];
                        for (int w = 0; w < p_wg && pm; ++w)
                            if (po[2 * w]) {
                                pbad += po[2 * w];
                                ++pwb;
                            }
                        for (int w = 0; w < v_wg; ++w)
                            if (vo[4 * w]) {
                                if (!vwb) {
                                    ex_alloc = vo[4 * w + 1];
                                    ex_first = vo[4 * w + 2];
                                    ex_val = vo[4 * w + 3];
                                }
                                vbad += vo[4 * w];
                                ++vwb;
                            }
                        total_bad += pbad + vbad;
                        printf("%s %-8s %-4s partner %-7s %2d KB | victim %3d KB | partner bad: %3d wgs %9llu words | victim "
                               "bad: %3d wgs %9llu words, first byte %d = %08x (alloc %08x; wg0 alloc %08x)\n",
                               victim_first ? "V1" : "P1", method ? "ds_write" : "lds-dma", kname[kind], pname[pm], pm ? pk : 0, vk, pwb, pbad, vwb,
                               vbad, vwb ? (int)ex_first * 4 : -1, ex_val, ex_alloc, any_alloc);
                        if (pm) printf("    partner wg0 alloc %08x wg%d alloc %08x\n", po[1], p_wg - 1, po[2 * p_wg - 1]);
                        fflush(stdout);
                    }
    printf("TOTAL bad words %llu\n", total_bad);
    return 0;
}
