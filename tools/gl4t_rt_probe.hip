// Probe (round 6): the tiled GEMM phase k_gl4t (sd_graph_linear_v4.hip) with
// RT 32-row tiles per wave.  RT = 1 is the product form (4 waves x 32 rows x 192 columns of one
// node, LDS-DMA ring of weights AND x, fill first, 2 chunks in flight); RT = 2 gives each wave 64
// rows: every weight fragment read from LDS feeds two row tiles (half the LDS fragment reads and
// half the weight DMA bytes per output), 36 MFMAs per chunk and wave, at twice the accumulators.
// NWV waves per workgroup.  Config-2 shape: J = 16, 10 node types, K = 192, N = 192 (and 768),
// row-blocked x, split-f16 weights, Y to the split route's column-tiled scratch.  Prints per-launch
// time (hipEvents over REPS back-to-back launches) and checks every variant bitwise against RT = 1.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Xclang -target-feature -Xclang -packed-fp32-ops
//        tools/gl4t_rt_probe.hip -o tools/gl4t_rt_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int J = 16, K = 192, NCH = K / 16, NTYPES = 10;
__constant__ int c_type[J] = {0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9};

template <int N>
struct VmCnt4 {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    static constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
};

__device__ __forceinline__ int64_t blk_off(int64_t row, int node, int f) {
    return ((((row >> 5) * J + node) * (int64_t)K) << 5) + ((f >> 3) << 8) + (((f >> 2) & 1) << 7) + ((row & 31) << 2) +
           (f & 3);
}
__device__ __forceinline__ int64_t zs_off(int64_t row, int j, int n, int N) {
    return ((((row >> 5) * (N >> 5) + (n >> 5)) * J + j) << 10) + ((row & 31) << 5) + (n & 31);
}

template <int RT, int NWV, int CT>
constexpr int smem_bytes() {
    constexpr int NS = 3, TS = 36;
    constexpr int SBW = NS * CT * 1024 * 2 + NS * NWV * RT * 2048;
    return SBW > NWV * 32 * TS * 4 ? SBW : NWV * 32 * TS * 4;
}

// one workgroup = NWV waves x RT 32-row tiles of ONE node x CT 32-column tiles
template <int RT, int NWV, int CT, int MINW>
__global__ __launch_bounds__(NWV * 64, MINW) void k_rt(const float* __restrict__ x, const _Float16* __restrict__ wsp,
                                                        float* __restrict__ y, int64_t ntile_r, int N) {
    constexpr int PF = 2, NS = 3, NT = NWV * 64, TILE_H = 1024, PPT = 128, TS = 36;
    constexpr int NPC = CT * PPT;  // 16-B weight pieces per chunk
    constexpr int XL = 2 * RT;     // x DMA instructions per chunk and wave
    constexpr int OPA = (NPC / 64 + NWV - 1) / NWV + XL, OPB = (NPC / 64) / NWV + XL;
    __shared__ __attribute__((aligned(16))) char smem[smem_bytes<RT, NWV, CT>()];
    _Float16(*sW)[CT * TILE_H] = reinterpret_cast<_Float16(*)[CT * TILE_H]>(smem);
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int ncg = N / (32 * CT);
    const int cg = (int)(u % ncg);
    const int64_t nrg = (ntile_r + NWV * RT - 1) / (NWV * RT);
    const int j = (int)((u / ncg) / nrg);
    const int64_t rgi = (u / ncg) % nrg;
    const int64_t tr0 = (rgi * NWV + wave) * RT;  // this wave's first 32-row tile
    const int nct = N / 32;
    const _Float16* wt0 = wsp + ((int64_t)c_type[j] * NCH * nct + cg * CT) * 1024;
    float* const xs0 = reinterpret_cast<float*>(smem + NS * CT * TILE_H * 2) + wave * (512 * RT);
    const float* xb[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int64_t t = tr0 + rt < ntile_r ? tr0 + rt : 0;  // dead tiles read tile 0 (never stored)
        xb[rt] = x + blk_off(t * 32 + l32, j, 4 * h);
    }
    floatx16 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[rt][ct][e] = 0.f;
    const bool wa = wave * 64 + NT * ((NPC / 64 + NWV - 1) / NWV - 1) < NPC;
    auto fill = [&](int c) {
        _Float16* dst = sW[c % NS];
#pragma unroll
        for (int k = 0; k < (NPC / 64 + NWV - 1) / NWV; ++k) {
            const int q0 = wave * 64 + NT * k;
            if (q0 >= NPC) continue;
            const int q = q0 + lane;
            const _Float16* src = wt0 + ((int64_t)c * nct + q / PPT) * 1024 + (q % PPT) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
        }
        float* xd = xs0 + (c % NS) * (NWV * 512 * RT);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            __builtin_amdgcn_global_load_lds((const void*)(xb[rt] + c * 512), (lds_void*)(xd + rt * 512), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(xb[rt] + c * 512 + 256), (lds_void*)(xd + rt * 512 + 256), 16, 0, 0);
        }
    };
    auto compute = [&](int c) {
        const float* xs = xs0 + (c % NS) * (NWV * 512 * RT) + h * 256 + l32 * 4;
        halfx8 xh[RT], xl[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const floatx4 a = *reinterpret_cast<const floatx4*>(xs + rt * 512);
            const floatx4 b = *reinterpret_cast<const floatx4*>(xs + rt * 512 + 128);
            const floatx8 f = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            xh[rt] = __builtin_convertvector(f, halfx8);
            xl[rt] = __builtin_convertvector(f - __builtin_convertvector(xh[rt], floatx8), halfx8);
        }
        const _Float16* wt = sW[c % NS] + lane * 8;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
            const halfx8 wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wh, acc[rt][ct], 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wl, t, 0, 0, 0);
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl[rt], wh, t, 0, 0, 0);
            }
        }
    };
    auto wait_chunk = [&](int younger) {
        if (younger == 0) {
            __builtin_amdgcn_s_waitcnt(VmCnt4<0>::imm & ~(0xF << 8));
        } else {
            if (wa) __builtin_amdgcn_s_waitcnt(VmCnt4<OPA>::imm & ~(0xF << 8));
            else __builtin_amdgcn_s_waitcnt(VmCnt4<OPB>::imm & ~(0xF << 8));
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
#pragma unroll
    for (int i = 0; i < PF; ++i) fill(i);
#pragma nounroll
    for (int c0 = 0; c0 < NCH - PF; c0 += PF) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int c = c0 + i;
            wait_chunk(PF - 1);
            fill(c + PF);
            asm volatile("" ::: "memory");
            compute(c);
        }
    }
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        wait_chunk(PF - 1 - i);
        compute(NCH - PF + i);
        asm volatile("" ::: "memory");
    }
    __syncthreads();
    float* sT = reinterpret_cast<float*>(smem) + wave * 32 * TS;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int64_t tr = tr0 + rt;
        if (tr >= ntile_r) break;  // wave-uniform
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sT[((r & 3) + 8 * (r >> 2) + 4 * h) * TS + l32] = acc[rt][ct][r];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 8 * q + (lane >> 3), c4 = (lane & 7) * 4;
                const floatx4 o = *reinterpret_cast<const floatx4*>(sT + row * TS + c4);
                *reinterpret_cast<floatx4*>(y + zs_off(tr * 32 + row, j, (cg * CT + ct) * 32 + c4, N)) = o;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int RT, int NWV, int CT, int MINW>
static void launch(const float* x, const _Float16* w, float* y, int64_t ntile_r, int N, hipStream_t s) {
    const int64_t nrg = (ntile_r + NWV * RT - 1) / (NWV * RT);
    const dim3 grid((unsigned)(nrg * J * (N / (32 * CT))));
    hipLaunchKernelGGL((k_rt<RT, NWV, CT, MINW>), grid, dim3(NWV * 64), 0, s, x, w, y, ntile_r, N);
}


// XV: x straight into registers by compiler-untracked global_load_dwordx4 (inline asm; waited for
// by the same counted vmcnt as the weight ring, then a register fence), weights by the LDS-DMA ring;
// the whole K loop unrolled so the 3-slot register ring of x has static slots (no back-edge copies)
__device__ __forceinline__ void g4_async(floatx4& d, const float* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}
template <int RT, int NWV, int CT, int MINW>
__global__ __launch_bounds__(NWV * 64, MINW) void k_xv(const float* __restrict__ x, const _Float16* __restrict__ wsp,
                                                        float* __restrict__ y, int64_t ntile_r, int N) {
    constexpr int PF = 2, NS = 3, NT = NWV * 64, TILE_H = 1024, PPT = 128, TS = 36;
    constexpr int NPC = CT * PPT;
    constexpr int XL = 2 * RT;
    constexpr int OPA = (NPC / 64 + NWV - 1) / NWV + XL, OPB = (NPC / 64) / NWV + XL;
    constexpr int SBW = NS * CT * TILE_H * 2;
    constexpr int SB = SBW > NWV * 32 * TS * 4 ? SBW : NWV * 32 * TS * 4;
    __shared__ __attribute__((aligned(16))) char smem[SB];
    _Float16(*sW)[CT * TILE_H] = reinterpret_cast<_Float16(*)[CT * TILE_H]>(smem);
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int ncg = N / (32 * CT);
    const int cg = (int)(u % ncg);
    const int64_t nrg = (ntile_r + NWV * RT - 1) / (NWV * RT);
    const int j = (int)((u / ncg) / nrg);
    const int64_t rgi = (u / ncg) % nrg;
    const int64_t tr0 = (rgi * NWV + wave) * RT;
    const int nct = N / 32;
    const _Float16* wt0 = wsp + ((int64_t)c_type[j] * NCH * nct + cg * CT) * 1024;
    const float* xr[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) xr[rt] = x + blk_off((tr0 + rt < ntile_r ? tr0 + rt : 0) * 32 + l32, j, 8 * h);
    floatx16 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[rt][ct][e] = 0.f;
    floatx4 xa[NS][RT], xb[NS][RT];
    const bool wa = wave * 64 + NT * ((NPC / 64 + NWV - 1) / NWV - 1) < NPC;
    auto fill = [&](int c) {
        _Float16* dst = sW[c % NS];
#pragma unroll
        for (int k = 0; k < (NPC / 64 + NWV - 1) / NWV; ++k) {
            const int q0 = wave * 64 + NT * k;
            if (q0 >= NPC) continue;
            const int q = q0 + lane;
            const _Float16* src = wt0 + ((int64_t)c * nct + q / PPT) * 1024 + (q % PPT) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            g4_async(xa[c % NS][rt], xr[rt] + c * 512);
            g4_async(xb[c % NS][rt], xr[rt] + c * 512 + 128);
        }
    };
    auto compute = [&](int c) {
        halfx8 xh[RT], xl[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const floatx4 a = xa[c % NS][rt], b = xb[c % NS][rt];
            const floatx8 f = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            xh[rt] = __builtin_convertvector(f, halfx8);
            xl[rt] = __builtin_convertvector(f - __builtin_convertvector(xh[rt], floatx8), halfx8);
        }
        const _Float16* wt = sW[c % NS] + lane * 8;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
            const halfx8 wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wh, acc[rt][ct], 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wl, t, 0, 0, 0);
                acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl[rt], wh, t, 0, 0, 0);
            }
        }
    };
    auto wait_chunk = [&](int c, int younger) {
        if (younger == 0) {
            __builtin_amdgcn_s_waitcnt(VmCnt4<0>::imm & ~(0xF << 8));
        } else {
            if (wa) __builtin_amdgcn_s_waitcnt(VmCnt4<OPA>::imm & ~(0xF << 8));
            else __builtin_amdgcn_s_waitcnt(VmCnt4<OPB>::imm & ~(0xF << 8));
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) asm volatile("" : "+v"(xa[c % NS][rt]), "+v"(xb[c % NS][rt]) :: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
#pragma unroll
    for (int i = 0; i < PF; ++i) fill(i);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        wait_chunk(c, c + 1 < NCH ? PF - 1 : 0);
        if (c + PF < NCH) fill(c + PF);
        asm volatile("" ::: "memory");
        compute(c);
    }
    __syncthreads();
    float* sT = reinterpret_cast<float*>(smem) + wave * 32 * TS;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int64_t tr = tr0 + rt;
        if (tr >= ntile_r) break;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sT[((r & 3) + 8 * (r >> 2) + 4 * h) * TS + l32] = acc[rt][ct][r];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 8 * q + (lane >> 3), c4 = (lane & 7) * 4;
                const floatx4 o = *reinterpret_cast<const floatx4*>(sT + row * TS + c4);
                *reinterpret_cast<floatx4*>(y + zs_off(tr * 32 + row, j, (cg * CT + ct) * 32 + c4, N)) = o;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}
template <int RT, int NWV, int CT, int MINW>
static void launch_xv(const float* x, const _Float16* w, float* y, int64_t ntile_r, int N, hipStream_t s) {
    const int64_t nrg = (ntile_r + NWV * RT - 1) / (NWV * RT);
    const dim3 grid((unsigned)(nrg * J * (N / (32 * CT))));
    hipLaunchKernelGGL((k_xv<RT, NWV, CT, MINW>), grid, dim3(NWV * 64), 0, s, x, w, y, ntile_r, N);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int64_t max_rows = 3200;
    const int64_t max_tiles = (max_rows + 31) / 32, rp = max_tiles * 32;
    const size_t nx = rp * J * K, nw = (size_t)NTYPES * NCH * 24 * 1024, ny = rp * J * 768;
    float *x, *y, *y2;
    _Float16* w;
    CHECK(hipMalloc(&x, nx * 4));
    CHECK(hipMalloc(&y, ny * 4));
    CHECK(hipMalloc(&y2, ny * 4));
    CHECK(hipMalloc(&w, nw * 2));
    {
        std::vector<float> hx(nx);
        for (size_t i = 0; i < nx; ++i) hx[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
        CHECK(hipMemcpy(x, hx.data(), nx * 4, hipMemcpyHostToDevice));
        std::vector<_Float16> hw(nw);
        for (size_t i = 0; i < nw; ++i) hw[i] = (_Float16)(((i * 40503u) % 2001) / 20000.f - 0.05f);
        CHECK(hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice));
    }
    hipStream_t st[3];
    for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // timing: `chains` streams each launching the kernel on its third of the rows (as the sampler's
    // three row chains do), REPS rounds; per-round time and the per-launch equivalent
    auto timeit = [&](const char* name, auto fn, int64_t rows, int N, int chains) {
        const int64_t tiles = (rows + 31) / 32;
        auto round = [&]() {
            for (int c = 0; c < chains; ++c) {
                const int64_t t0 = tiles * c / chains, t1 = tiles * (c + 1) / chains;
                fn(x + t0 * 32 * J * K, w, y + t0 * 32 * J * (int64_t)N, t1 - t0, N, chains > 1 ? st[c] : (hipStream_t)0);
            }
        };
        for (int i = 0; i < 5; ++i) round();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) {
            round();
            if (chains > 1) CHECK(hipDeviceSynchronize());
        }
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        const double bytes = (double)rows * J * (K + N) * 4;
        printf("%-34s rows %5lld N %3d chains %d: %8.2f us per round  %7.0f GB/s (x + Y)\n", name, (long long)rows, N,
               chains, us, bytes / us * 1e-3);
        fflush(stdout);
    };
    // correctness: every variant bitwise equal to RT = 1 (same products, same order per element)
    auto check = [&](const char* name, auto fn, int64_t rows, int N) {
        const int64_t tiles = (rows + 31) / 32;
        CHECK(hipMemset(y, 0, ny * 4));
        CHECK(hipMemset(y2, 0, ny * 4));
        launch<1, 4, 6, 2>(x, w, y, tiles, N, 0);
        fn(x, w, y2, tiles, N, (hipStream_t)0);
        CHECK(hipDeviceSynchronize());
        std::vector<float> a(tiles * 32 * J * (size_t)N), b(a.size());
        CHECK(hipMemcpy(a.data(), y, a.size() * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(b.data(), y2, b.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < a.size(); ++i) bad += memcmp(&a[i], &b[i], 4) != 0;
        double s = 0;
        for (size_t i = 0; i < a.size(); i += 97) s += a[i];
        printf("check %-28s rows %5lld N %3d: %zu of %zu differ (checksum %.6f)\n", name, (long long)rows, N, bad,
               a.size(), s);
        fflush(stdout);
    };
    auto v1 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch<1, 4, 6, 2>(a, b, c, t, n, s); };
    auto v2 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch<2, 4, 6, 1>(a, b, c, t, n, s); };
    auto v2b = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch<2, 2, 6, 2>(a, b, c, t, n, s); };
    auto v2c = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch<2, 4, 3, 1>(a, b, c, t, n, s); };
    auto xv6 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch_xv<1, 4, 6, 2>(a, b, c, t, n, s); };
    auto xv3 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch_xv<1, 4, 3, 2>(a, b, c, t, n, s); };
    auto xv8w = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch_xv<1, 8, 6, 1>(a, b, c, t, n, s); };
    auto xr2c3 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch_xv<2, 4, 3, 2>(a, b, c, t, n, s); };
    auto xr2c6 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch_xv<2, 4, 6, 1>(a, b, c, t, n, s); };
    auto xr2c6w2 = [](const float* a, const _Float16* b, float* c, int64_t t, int n, hipStream_t s) { launch_xv<2, 2, 6, 1>(a, b, c, t, n, s); };
    for (int64_t rows : {3200, 1067}) {
        check("XV 4w CT6", xv6, rows, 192);
        check("XV 4w CT3", xv3, rows, 192);
        check("XV 8w CT6", xv8w, rows, 192);
        check("XV RT2 4w CT3", xr2c3, rows, 192);
        check("XV RT2 4w CT6", xr2c6, rows, 192);
        check("XV RT2 2w CT6", xr2c6w2, rows, 192);
        check("XV 4w CT6 N768", xv6, rows, 768);
        check("RT2 4w CT6", v2, rows, 192);
        check("RT2 2w CT6", v2b, rows, 192);
        check("RT2 4w CT3", v2c, rows, 192);
        check("RT2 4w CT6 N768", v2, rows, 768);
    }
    for (int N : {192, 768}) {
        for (int chains : {1}) {
            timeit("RT1 4w CT6 (product)", v1, 3200, N, chains);
            timeit("RT1 4w CT6 (product) 1067 rows", v1, 1067, N, chains);
            timeit("XV 4w CT6", xv6, 3200, N, chains);
            timeit("XV 4w CT6 1067 rows", xv6, 1067, N, chains);
            timeit("XV 4w CT3", xv3, 3200, N, chains);
            timeit("XV 8w CT6", xv8w, 3200, N, chains);
            timeit("XV RT2 4w CT3", xr2c3, 3200, N, chains);
            timeit("XV RT2 4w CT3 1067 rows", xr2c3, 1067, N, chains);
            timeit("XV RT2 4w CT6", xr2c6, 3200, N, chains);
            timeit("XV RT2 2w CT6", xr2c6w2, 3200, N, chains);
            timeit("RT2 4w CT6", v2, 3200, N, chains);
            timeit("RT2 2w CT6", v2b, 3200, N, chains);
            timeit("RT2 4w CT3", v2c, 3200, N, chains);
        }
    }
    return 0;
}
