// Probe for DESIGN.md §4c, fourth hypothesis: does a k_update-shaped kernel (static J x J tables,
// wave-uniform ds_read_b128 broadcasts, packed f32 FMAs) compute bitwise the same while LDS-DMA
// (global_load_lds_dwordx4) fills of ANOTHER workgroup on the same CU are landing?
//
// victim (DMA side): k_gl4's K-loop LDS-DMA schedule (lds_dma_race_probe.hip's kernel), looped;
// upd_like: k_update's table pattern (lds_base_probe.hip's kernel), repeated on another stream.
// upd_like's outputs are compared bitwise with a run alone; the DMA side counts stale words.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_dma_upd_probe tools/lds_dma_upd_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <cmath>
#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

__device__ __forceinline__ unsigned lds_alloc_reg() { return __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 6); }

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

typedef float floatx2 __attribute__((ext_vector_type(2)));

template <int J>
__global__ __launch_bounds__(256) void upd_like(const float* C1, const float* C2, const float* U, const float* S,
                                                const float* x, const float* y, const float* e, float* out, int rows,
                                                int D, unsigned* alloc_out) {
    __shared__ float sC1[J * J], sC2[J * J], sU[J * J], sS[J];
    for (int i = threadIdx.x; i < J * J; i += 256) {
        sC1[i] = C1[i];
        sC2[i] = C2[i];
        sU[i] = U[i];
    }
    for (int i = threadIdx.x; i < J; i += 256) sS[i] = S[i];
    __syncthreads();
    if (threadIdx.x == 0) alloc_out[blockIdx.x] = lds_alloc_reg();
    const int DP = D / 2;
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = g / DP;
    if (row >= rows) return;
    const int d = 2 * (int)(g % DP);
    const int64_t rb = row * (int64_t)J * D;
    floatx2 xv[J], yv[J], ev[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        xv[j] = *reinterpret_cast<const floatx2*>(x + rb + j * D + d);
        yv[j] = *reinterpret_cast<const floatx2*>(y + rb + j * D + d);
        ev[j] = *reinterpret_cast<const floatx2*>(e + rb + j * D + d) * sS[j];
    }
    for (int i = 0; i < J; ++i) {
        floatx2 m1 = {0.f, 0.f}, m2 = {0.f, 0.f}, nz = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < J; ++j) {
            m1 += sC1[i * J + j] * xv[j];
            m2 += sC2[i * J + j] * yv[j];
            nz += sU[i * J + j] * ev[j];
        }
        *reinterpret_cast<floatx2*>(out + rb + i * D + d) = m1 + m2 + nz;
    }
}


int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHECK(hipFuncSetAttribute((const void*)victim<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CHECK(hipFuncSetAttribute((const void*)victim<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int J = 16, D = 96, rows = 3200;
    const size_t n = (size_t)rows * J * D;
    std::vector<float> h(3 * n + 3 * J * J + J);
    uint32_t st = 12345;
    for (auto& v : h) {
        st = st * 1664525u + 1013904223u;
        v = (float)((st >> 8) & 0xFFFF) / 65536.0f - 0.5f;
    }
    float *dx, *dt, *out_ref, *out;
    CHECK(hipMalloc(&dx, 3 * n * 4));
    CHECK(hipMalloc(&dt, (3 * J * J + J) * 4));
    CHECK(hipMalloc(&out_ref, n * 4));
    CHECK(hipMalloc(&out, n * 4));
    CHECK(hipMemcpy(dx, h.data(), 3 * n * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dt, h.data() + 3 * n, (3 * J * J + J) * 4, hipMemcpyHostToDevice));
    const int grid = (int)((rows * (D / 2) + 255) / 256);
    unsigned* ualloc;
    CHECK(hipMalloc(&ualloc, grid * 4));
    const int chunks = 12, max_stage = 61 * 1024;
    std::vector<unsigned> hs((size_t)chunks * max_stage / 4);
    for (size_t i = 0; i < hs.size(); ++i) hs[i] = val((unsigned)i);
    unsigned *src, *bad;
    CHECK(hipMalloc(&src, hs.size() * 4));
    CHECK(hipMemcpy(src, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMalloc(&bad, 4));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto run_upd = [&](float* o, hipStream_t s) {
        hipLaunchKernelGGL((upd_like<16>), dim3(grid), dim3(256), 0, s, dt, dt + J * J, dt + 2 * J * J, dt + 3 * J * J, dx,
                           dx + n, dx + 2 * n, o, rows, D, ualloc);
    };
    run_upd(out_ref, s2);
    CHECK(hipDeviceSynchronize());
    std::vector<float> ref(n), got(n);
    CHECK(hipMemcpy(ref.data(), out_ref, n * 4, hipMemcpyDeviceToHost));
    unsigned long long total_upd = 0, total_stale = 0;
    for (int method = 0; method < 2; ++method)
        for (int stage_kb : {20, 41, 61}) {
            for (int rep = 0; rep < 4; ++rep) {
                CHECK(hipMemset(out, 0, n * 4));
                CHECK(hipMemset(bad, 0, 4));
                CHECK(hipDeviceSynchronize());
                const size_t lds = (size_t)2 * stage_kb * 1024;
                if (method == 0)
                    hipLaunchKernelGGL(victim<0>, dim3(cus), dim3(512), lds, s1, src, bad, stage_kb * 1024, chunks, 2000);
                else
                    hipLaunchKernelGGL(victim<1>, dim3(cus), dim3(512), lds, s1, src, bad, stage_kb * 1024, chunks, 2000);
                size_t nbad = 0, first = (size_t)-1;
                double mx = 0;
                for (int k = 0; k < 40; ++k) {
                    run_upd(out, s2);
                    CHECK(hipStreamSynchronize(s2));
                    CHECK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
                    for (size_t i = 0; i < n; ++i)
                        if (got[i] != ref[i]) {
                            ++nbad;
                            if (first == (size_t)-1) first = i;
                            mx = std::fmax(mx, std::fabs((double)got[i] - ref[i]));
                        }
                }
                CHECK(hipDeviceSynchronize());
                unsigned b = 0;
                CHECK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
                total_upd += nbad;
                total_stale += b;
                printf("%-9s stage %2d KB rep %d: upd_like differing outputs %zu (max %.3g, first %zd: row %zd node %zd "
                       "feature %zd); dma-side stale words %u\n",
                       method ? "reg-stage" : "lds-dma", stage_kb, rep, nbad, mx, nbad ? (ssize_t)first : -1,
                       nbad ? (ssize_t)(first / (J * D)) : -1, nbad ? (ssize_t)((first / D) % J) : -1,
                       nbad ? (ssize_t)(first % D) : -1, b);
                fflush(stdout);
            }
        }
    printf("TOTAL upd_like differing %llu, stale %llu\n", total_upd, total_stale);
    return 0;
}
