// Standalone probe of the tiled GEMM phase (k_gl4t, sd_graph_linear_v4.hip) at config 2's shape:
// N = 192, K = 192, J = 16, 10 node types, 3,200 (or ROWS) rows, row-blocked x, split-f16 weights,
// Y to the split route's scratch layout.  Variants isolate what bounds the K loop (VERDICT r03
// item 2): the production structure (register-staged weights, one barrier per chunk, x 4 chunks
// ahead) with its MFMAs, x loads, weight loads or Y stores removed one at a time, and alternative
// pipelines (LDS-DMA weight ring with the same lookahead as x; 8 waves per workgroup).  Timing:
// hipEvents around REPS back-to-back launches; bytes = x + Y + weights once (algorithmic).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Xclang -target-feature -Xclang -packed-fp32-ops
//        tools/gl4t_probe.hip -o tools/gl4t_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

constexpr int J = 16, K = 192, N = 192, NCH = K / 16, CT = 6, NTYPES = 10, NCT = 6;
__constant__ int c_type[J] = {0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9};

__device__ __forceinline__ int64_t blk_off(int64_t row, int node, int f) {
    return ((((row >> 5) * J + node) * (int64_t)K) << 5) + ((f >> 3) << 8) + (((f >> 2) & 1) << 7) + ((row & 31) << 2) +
           (f & 3);
}
__device__ __forceinline__ floatx4 g4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

enum Flags { NOMFMA = 1, NOX = 2, NOW = 4, NOY = 8, ACCY = 16 };
// ACCY: Y stored in the accumulator-native order [tile][g = r >> 2][lane][4] straight from the
// registers (one 1-KiB dwordx4 store per 4 accumulator registers; no LDS transpose)

// V 0: production structure.  V 1: weights by LDS-DMA into a ring of PF + 1 slots, PF chunks
// ahead like x (waiting for chunk c never waits for a younger chunk).  NWV waves per workgroup.
template <int V, int F, int NWV, int PF>
__global__ __launch_bounds__(NWV * 64, NWV == 4 ? 2 : 1) void k_probe(const float* __restrict__ x,
                                                                      const _Float16* __restrict__ wsp,
                                                                      float* __restrict__ y, int64_t ntile_r) {
    constexpr int NT = NWV * 64;
    constexpr int TILE_H = 1024, PPT = TILE_H / 8, NPC = CT * PPT;  // 16-B pieces per chunk: 768
    constexpr int NS = V == 1 ? PF + 1 : 2;                          // weight slots
    constexpr int TS = 36;
    constexpr int SBW = NS * CT * TILE_H * 2;
    constexpr int SB = SBW > NWV * 32 * TS * 4 ? SBW : NWV * 32 * TS * 4;
    __shared__ __attribute__((aligned(16))) char smem[SB];
    _Float16(*sW)[CT * TILE_H] = reinterpret_cast<_Float16(*)[CT * TILE_H]>(smem);
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int64_t nrg = (ntile_r + NWV - 1) / NWV;
    const int j = (int)(u / nrg);
    const int64_t tr = (u % nrg) * NWV + wave;
    const bool live = tr < ntile_r;
    const int64_t row0 = (live ? tr : 0) * 32;
    const float* xr = x + blk_off(row0 + l32, j, 8 * h);
    const _Float16* wb = wsp + (int64_t)c_type[j] * NCH * NCT * 1024;
    constexpr int NP = (NPC + NT - 1) / NT;  // pieces per thread per chunk
    floatx4 xa[PF], xb[PF];
    auto issue_x = [&](int c, int sl) {
        if constexpr (F & NOX) {
            xa[sl] = floatx4{0.5f, 0.25f, 0.125f, 1.f};
            xb[sl] = xa[sl];
        } else {
            xa[sl] = g4(xr + (c << 9));
            xb[sl] = g4(xr + (c << 9) + 128);
        }
    };
    floatx16 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[ct][e] = 0.f;
    auto compute = [&](int sl, const _Float16* wst) {
        const floatx8 f = {xa[sl].x, xa[sl].y, xa[sl].z, xa[sl].w, xb[sl].x, xb[sl].y, xb[sl].z, xb[sl].w};
        const halfx8 xh = __builtin_convertvector(f, halfx8);
        const halfx8 xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
        const _Float16* wt = wst + lane * 8;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
            const halfx8 wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
            if constexpr (F & NOMFMA) {
                acc[ct][0] += (float)wh[0] + (float)wl[1] + (float)xh[ct] + (float)xl[ct];
            } else {
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh, acc[ct], 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl, t, 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh, t, 0, 0, 0);
            }
        }
    };
    if constexpr (V == 0) {
        uint4 w0, w1, w2;
        static_assert(NP <= 3, "pieces");
        auto piece = [&](int k) { return wb + (min(tid + NT * k, NPC - 1) / PPT) * 1024 + (min(tid + NT * k, NPC - 1) % PPT) * 8; };
        const _Float16* s0 = piece(0);
        const _Float16* s1 = piece(1);
        const _Float16* s2 = piece(2);
        auto load_w = [&](int c) {
            if constexpr (!(F & NOW)) {
                const int64_t o = (int64_t)c * NCT * 1024;
                w0 = *reinterpret_cast<const uint4*>(s0 + o);
                if constexpr (NP > 1) w1 = *reinterpret_cast<const uint4*>(s1 + o);
                if constexpr (NP > 2) w2 = *reinterpret_cast<const uint4*>(s2 + o);
            }
        };
        auto store_w = [&](int sl) {
            if constexpr (!(F & NOW)) {
                uint4* d = reinterpret_cast<uint4*>(&sW[sl][tid * 8]);
                if (tid < NPC) d[0] = w0;
                if constexpr (NP > 1) if (tid + NT < NPC) d[NT] = w1;
                if constexpr (NP > 2) if (tid + 2 * NT < NPC) d[2 * NT] = w2;
            }
        };
        if constexpr (F & NOW) {  // one stage of constants, never refilled
            for (int q = tid; q < 2 * CT * TILE_H; q += NT) (&sW[0][0])[q] = (_Float16)(0.001f * (q & 7));
        }
        load_w(0);
#pragma unroll
        for (int i = 0; i < PF; ++i) issue_x(i, i);
#pragma nounroll
        for (int c0 = 0; c0 < NCH; c0 += PF) {
#pragma unroll
            for (int i = 0; i < PF; ++i) {
                const int c = c0 + i;
                store_w(i & 1);
                __builtin_amdgcn_s_waitcnt(0xC07F);
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                load_w(min(c + 1, NCH - 1));
                asm volatile("" ::: "memory");
                compute(i, sW[(F & NOW) ? 0 : (i & 1)]);
                asm volatile("" ::: "memory");
                issue_x(min(c + PF, NCH - 1), i);
            }
        }
    } else {
        // LDS-DMA ring: chunk c's slice in slot c % NS; pieces of wave w: q = w * 64 + lane + NT * k
        auto fill = [&](int c) {
            if constexpr (!(F & NOW)) {
                _Float16* dst = sW[c % NS];
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    const int q0 = wave * 64 + NT * k;
                    if (q0 >= NPC) continue;  // wave-uniform
                    const int q = min(q0 + lane, NPC - 1);
                    const _Float16* src = wb + ((int64_t)c * NCT + q / PPT) * 1024 + (q % PPT) * 8;
                    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
                }
            }
        };
        if constexpr (F & NOW) {
            for (int q = tid; q < NS * CT * TILE_H; q += NT) (&sW[0][0])[q] = (_Float16)(0.001f * (q & 7));
        }
        // prologue: chunks 0 .. PF-1 (weights and x), in chunk order
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            fill(i);
            issue_x(i, i);
        }
        // per chunk this wave issues npw DMA pieces (wave-uniform: 3 at 4 waves; 2 / 1 at 8) + 2 x loads
        constexpr int XL = (F & NOX) ? 0 : 2;
        constexpr int PA = (F & NOW) ? XL : (NPC / 64 + NWV - 1) / NWV + XL;  // waves with the extra piece
        constexpr int PB = (F & NOW) ? XL : (NPC / 64) / NWV + XL;
        const bool wa = (F & NOW) || wave * 64 + NT * ((NPC / 64 + NWV - 1) / NWV - 1) < NPC;
#pragma nounroll
        for (int c0 = 0; c0 < NCH; c0 += PF) {
#pragma unroll
            for (int i = 0; i < PF; ++i) {
                const int c = c0 + i;
                // chunk c's own loads done; the PF - 1 younger chunks stay in flight
                constexpr int NA = PA * (PF - 1), NB = PB * (PF - 1);
                static_assert(NA < 64, "vmcnt");
                if (wa) __builtin_amdgcn_s_waitcnt((NA & 0xF) | (0x7 << 4) | (0xF << 8) | ((NA >> 4) << 14));
                else __builtin_amdgcn_s_waitcnt((NB & 0xF) | (0x7 << 4) | (0xF << 8) | ((NB >> 4) << 14));
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_barrier();  // every wave's pieces of chunk c have landed
                asm volatile("" ::: "memory");
                compute(i, sW[(F & NOW) ? 0 : (c % NS)]);
                asm volatile("" ::: "memory");
                const int cn = min(c + PF, NCH - 1);
                fill(cn);
                issue_x(cn, i);
            }
        }
    }
    __syncthreads();
    if (!live) return;
    if constexpr (F & NOY) {
        float s = 0.f;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int e = 0; e < 16; ++e) s += acc[ct][e];
        if (s == 12345.f) y[lane] = s;
        return;
    }
    float* yo = y + ((tr * J + j) * 32) * (int64_t)N;
    if constexpr (F & ACCY) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<floatx4*>(yo + ct * 1024 + (g * 64 + lane) * 4) =
                    floatx4{acc[ct][4 * g], acc[ct][4 * g + 1], acc[ct][4 * g + 2], acc[ct][4 * g + 3]};
        return;
    }
    float* sT = reinterpret_cast<float*>(smem) + wave * 32 * TS;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sT[((r & 3) + 8 * (r >> 2) + 4 * h) * TS + l32] = acc[ct][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 8 * q + (lane >> 3), c4 = (lane & 7) * 4;
            *reinterpret_cast<floatx4*>(yo + (int64_t)row * N + ct * 32 + c4) = *reinterpret_cast<const floatx4*>(sT + row * TS + c4);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// V1 generalised: CTT 32-column tiles per workgroup (column group fastest in the XCD-aware order,
// as the library), NN output columns (192 or 768: to_qkv), LDS-DMA weight ring PF ahead.
template <int NN, int CTT, int NWV, int PF, int F>
__global__ __launch_bounds__(NWV * 64, 2) void k_ring(const float* __restrict__ x, const _Float16* __restrict__ wsp,
                                                      float* __restrict__ y, int64_t ntile_r) {
    constexpr int NT = NWV * 64, NCTT = NN / 32, ncg = NCTT / CTT;
    constexpr int TILE_H = 1024, PPT = TILE_H / 8, NPC = CTT * PPT;
    constexpr int NS = PF + 1, TS = 36;
    constexpr int SBW = NS * CTT * TILE_H * 2;
    constexpr int SB = SBW > NWV * 32 * TS * 4 ? SBW : NWV * 32 * TS * 4;
    __shared__ __attribute__((aligned(16))) char smem[SB];
    _Float16(*sW)[CTT * TILE_H] = reinterpret_cast<_Float16(*)[CTT * TILE_H]>(smem);
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int cg = (int)(u % ncg);
    const int64_t nrg = (ntile_r + NWV - 1) / NWV;
    const int j = (int)((u / ncg) / nrg);
    const int64_t tr = ((u / ncg) % nrg) * NWV + wave;
    const bool live = tr < ntile_r;
    const int64_t row0 = (live ? tr : 0) * 32;
    const float* xr = x + blk_off(row0 + l32, j, 8 * h);
    const _Float16* wb = wsp + ((int64_t)c_type[j] * NCH * NCTT + cg * CTT) * 1024;
    floatx4 xa[PF], xb[PF];
    auto issue_x = [&](int c, int sl) {
        xa[sl] = g4(xr + (c << 9));
        xb[sl] = g4(xr + (c << 9) + 128);
    };
    floatx16 acc[CTT];
#pragma unroll
    for (int ct = 0; ct < CTT; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[ct][e] = 0.f;
    auto compute = [&](int sl, const _Float16* wst) {
        const floatx8 f = {xa[sl].x, xa[sl].y, xa[sl].z, xa[sl].w, xb[sl].x, xb[sl].y, xb[sl].z, xb[sl].w};
        const halfx8 xh = __builtin_convertvector(f, halfx8);
        const halfx8 xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
        const _Float16* wt = wst + lane * 8;
#pragma unroll
        for (int ct = 0; ct < CTT; ++ct) {
            const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
            const halfx8 wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
            if constexpr (F & NOMFMA) {
                acc[ct][0] += (float)wh[0] + (float)wl[1] + (float)xh[ct & 7] + (float)xl[ct & 7];
            } else {
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh, acc[ct], 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl, t, 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh, t, 0, 0, 0);
            }
        }
    };
    constexpr int KW = (NPC / 64 + NWV - 1) / NWV;
    auto fill = [&](int c) {
        _Float16* dst = sW[c % NS];
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const int q0 = wave * 64 + NT * k;
            if (q0 >= NPC) continue;
            const int q = q0 + lane;
            __builtin_amdgcn_global_load_lds((const void*)(wb + ((int64_t)c * NCTT + q / PPT) * 1024 + (q % PPT) * 8),
                                             (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
        }
    };
    constexpr int PA = KW + 2, PB = (NPC / 64) / NWV + 2;
    const bool wa = wave * 64 + NT * (KW - 1) < NPC;
    auto wait = [&](int n) {
#define W_(m) if (wa) __builtin_amdgcn_s_waitcnt(((PA * (m)) & 0xF) | (0x7 << 4) | (0xF << 8) | (((PA * (m)) >> 4) << 14)); \
              else __builtin_amdgcn_s_waitcnt(((PB * (m)) & 0xF) | (0x7 << 4) | (0xF << 8) | (((PB * (m)) >> 4) << 14));
        if (n == 0) { W_(0) } else if (n == 1) { W_(1) } else if (n == 2) { W_(2) } else { W_(3) }
#undef W_
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        fill(i);
        issue_x(i, i);
    }
#pragma nounroll
    for (int c0 = 0; c0 < NCH - PF; c0 += PF) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int c = c0 + i;
            wait(PF - 1);
            compute(i, sW[c % NS]);
            asm volatile("" ::: "memory");
            fill(c + PF);
            issue_x(c + PF, i);
        }
    }
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        wait(PF - 1 - i);
        compute(i, sW[(NCH - PF + i) % NS]);
        asm volatile("" ::: "memory");
    }
    __syncthreads();
    if (!live) return;
    float* sT = reinterpret_cast<float*>(smem) + wave * 32 * TS;
    float* yo = y + ((tr * J + j) * 32) * (int64_t)NN + cg * CTT * 32;
#pragma unroll
    for (int ct = 0; ct < CTT; ++ct) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sT[((r & 3) + 8 * (r >> 2) + 4 * h) * TS + l32] = acc[ct][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 8 * q + (lane >> 3), c4 = (lane & 7) * 4;
            *reinterpret_cast<floatx4*>(yo + (int64_t)row * NN + ct * 32 + c4) = *reinterpret_cast<const floatx4*>(sT + row * TS + c4);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// V2: x too by LDS-DMA (each wave its own 2-KiB chunk image per slot), so the K loop holds no
// register-writing global load: no vmcnt the compiler must guess, all waits counted by hand.
template <int NN, int CTT, int NWV, int PF, int F>
__global__ __launch_bounds__(NWV * 64, 2) void k_ring2(const float* __restrict__ x, const _Float16* __restrict__ wsp,
                                                       float* __restrict__ y, int64_t ntile_r) {
    constexpr int NT = NWV * 64, NCTT = NN / 32, ncg = NCTT / CTT;
    constexpr int TILE_H = 1024, PPT = TILE_H / 8, NPC = CTT * PPT;
    constexpr int NS = PF + 1, TS = 36;
    constexpr int WSL = CTT * TILE_H * 2;          // bytes of a weight slot
    constexpr int XSL = NWV * 2048;                // bytes of an x slot (2 KiB per wave)
    constexpr int SBW = NS * (WSL + XSL);
    constexpr int SB = SBW > NWV * 32 * TS * 4 ? SBW : NWV * 32 * TS * 4;
    __shared__ __attribute__((aligned(16))) char smem[SB];
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int cg = (int)(u % ncg);
    const int64_t nrg = (ntile_r + NWV - 1) / NWV;
    const int j = (int)((u / ncg) / nrg);
    const int64_t tr = ((u / ncg) % nrg) * NWV + wave;
    const bool live = tr < ntile_r;
    const int64_t row0 = (live ? tr : 0) * 32;
    const float* xblk = x + blk_off(row0, j, 0);  // the wave's (row tile, node) region: chunk c at + 512 c floats
    const _Float16* wb = wsp + ((int64_t)c_type[j] * NCH * NCTT + cg * CTT) * 1024;
    auto wslot = [&](int sl) { return reinterpret_cast<_Float16*>(smem + sl * (WSL + XSL)); };
    auto xslot = [&](int sl) { return reinterpret_cast<float*>(smem + sl * (WSL + XSL) + WSL) + wave * 512; };
    floatx16 acc[CTT];
#pragma unroll
    for (int ct = 0; ct < CTT; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[ct][e] = 0.f;
    constexpr int KW = (NPC / 64 + NWV - 1) / NWV;
    auto fill = [&](int c) {
        _Float16* dst = wslot(c % NS);
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            const int q0 = wave * 64 + NT * k;
            if (q0 >= NPC) continue;
            const int q = q0 + lane;
            __builtin_amdgcn_global_load_lds((const void*)(wb + ((int64_t)c * NCTT + q / PPT) * 1024 + (q % PPT) * 8),
                                             (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
        }
        float* xd = xslot(c % NS);
        __builtin_amdgcn_global_load_lds((const void*)(xblk + c * 512 + lane * 4), (lds_void*)xd, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(xblk + c * 512 + 256 + lane * 4), (lds_void*)(xd + 256), 16, 0, 0);
    };
    auto compute = [&](int c) {
        const float* xs = xslot(c % NS);
        const floatx4 xa = *reinterpret_cast<const floatx4*>(xs + h * 256 + l32 * 4);
        const floatx4 xb = *reinterpret_cast<const floatx4*>(xs + h * 256 + 128 + l32 * 4);
        const floatx8 f = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
        const halfx8 xh = __builtin_convertvector(f, halfx8);
        const halfx8 xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
        const _Float16* wt = wslot(c % NS) + lane * 8;
#pragma unroll
        for (int ct = 0; ct < CTT; ++ct) {
            const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
            const halfx8 wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
            floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh, acc[ct], 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl, t, 0, 0, 0);
            acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh, t, 0, 0, 0);
        }
    };
    constexpr int PA = KW + 2, PB = (NPC / 64) / NWV + 2;
    const bool wa = wave * 64 + NT * (KW - 1) < NPC;
    auto wait = [&](int n) {
#define W_(m) if (wa) __builtin_amdgcn_s_waitcnt(((PA * (m)) & 0xF) | (0x7 << 4) | (0xF << 8) | (((PA * (m)) >> 4) << 14)); \
              else __builtin_amdgcn_s_waitcnt(((PB * (m)) & 0xF) | (0x7 << 4) | (0xF << 8) | (((PB * (m)) >> 4) << 14));
        if (n == 0) { W_(0) } else if (n == 1) { W_(1) } else if (n == 2) { W_(2) } else { W_(3) }
#undef W_
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
            wait(PF - 1);
            compute(c);
            asm volatile("" ::: "memory");
            fill(c + PF);
        }
    }
#pragma unroll
    for (int i = 0; i < PF; ++i) {
        wait(PF - 1 - i);
        compute(NCH - PF + i);
        asm volatile("" ::: "memory");
    }
    __syncthreads();
    if (!live) return;
    float* sT = reinterpret_cast<float*>(smem) + wave * 32 * TS;
    float* yo = y + ((tr * J + j) * 32) * (int64_t)NN + cg * CTT * 32;
#pragma unroll
    for (int ct = 0; ct < CTT; ++ct) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sT[((r & 3) + 8 * (r >> 2) + 4 * h) * TS + l32] = acc[ct][r];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = 8 * q + (lane >> 3), c4 = (lane & 7) * 4;
            *reinterpret_cast<floatx4*>(yo + (int64_t)row * NN + ct * 32 + c4) = *reinterpret_cast<const floatx4*>(sT + row * TS + c4);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// the x stream alone: every wave reads its 24 KB (row tile, node) region in 12 chunks of 2 x 1 KB,
// PF chunks in flight, and sums it (the bandwidth ceiling of k_gl4t's x access pattern)
template <int PF>
__global__ __launch_bounds__(256) void k_xstream(const float* __restrict__ x, float* __restrict__ y, int64_t ntile_r) {
    const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = tid >> 6;
    const int64_t u = blockIdx.x;
    const int64_t nrg = (ntile_r + 3) / 4;
    const int j = (int)(u / nrg);
    const int64_t tr = (u % nrg) * 4 + wave;
    if (tr >= ntile_r) return;
    const float* xr = x + blk_off(tr * 32 + l32, j, 8 * h);
    floatx4 s = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += g4(xr + (c << 9)) + g4(xr + (c << 9) + 128);
    if (s.x == 12345.f) y[tid] = s.y;
}

int main(int argc, char** argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : 3200;
    const int reps = argc > 2 ? atoi(argv[2]) : 50;
    const int64_t ntile_r = (rows + 31) / 32, rp = ntile_r * 32;
    const size_t nx = rp * J * K, ny = rp * J * N, nw = (size_t)NTYPES * NCH * NCT * 1024;
    const size_t ny4 = rp * J * 768, nw4 = (size_t)NTYPES * NCH * 24 * 1024;
    float *x, *y;
    _Float16* w;
    CHECK(hipMalloc(&x, nx * 4));
    CHECK(hipMalloc(&y, ny4 * 4));
    CHECK(hipMalloc(&w, nw4 * 2));
    {
        std::vector<float> hx(nx);
        for (size_t i = 0; i < nx; ++i) hx[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
        CHECK(hipMemcpy(x, hx.data(), nx * 4, hipMemcpyHostToDevice));
        std::vector<_Float16> hw(nw4);
        for (size_t i = 0; i < nw4; ++i) hw[i] = (_Float16)(((i * 40503u) % 2001) / 20000.f - 0.05f);
        CHECK(hipMemcpy(w, hw.data(), nw4 * 2, hipMemcpyHostToDevice));
    }
    const double bytes = (double)nx * 4 + (double)ny * 4 + (double)nw * 2;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch, double b) {
        for (int i = 0; i < 5; ++i) launch();
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("%-34s %8.2f us  %7.0f GB/s\n", name, us, b / us * 1e-3);
        fflush(stdout);
    };
#define RUN(NAME, V, F, NWV, PF)                                                                                 \
    timeit(NAME, [&] {                                                                                           \
        const unsigned g = (unsigned)(((ntile_r + NWV - 1) / NWV) * J);                                          \
        hipLaunchKernelGGL((k_probe<V, F, NWV, PF>), dim3(g), dim3(NWV * 64), 0, 0, x, w, y, ntile_r);           \
    }, bytes)
    printf("rows %lld: x %.1f MB, Y %.1f MB, weights %.1f MB\n", (long long)rows, nx * 4e-6, ny * 4e-6, nw * 2e-6);
    timeit("x stream alone (PF 12)", [&] {
        hipLaunchKernelGGL((k_xstream<12>), dim3((unsigned)(((ntile_r + 3) / 4) * J)), dim3(256), 0, 0, x, y, ntile_r);
    }, (double)nx * 4);
    RUN("V0 production", 0, 0, 4, 4);
    RUN("V1 DMA ring PF 2", 1, 0, 4, 2);
#define RING(NAME, NN, CTT, NWV, PF, F)                                                                          \
    timeit(NAME, [&] {                                                                                           \
        const unsigned g = (unsigned)(((ntile_r + NWV - 1) / NWV) * J * ((NN / 32) / CTT));                       \
        hipLaunchKernelGGL((k_ring<NN, CTT, NWV, PF, F>), dim3(g), dim3(NWV * 64), 0, 0, x, w, y, ntile_r);      \
    }, (double)nx * 4 + (double)rp * J * NN * 4 + (double)NTYPES * NCH * (NN / 32) * 2048)
#define RING2(NAME, NN, CTT, NWV, PF)                                                                            \
    timeit(NAME, [&] {                                                                                           \
        const unsigned g = (unsigned)(((ntile_r + NWV - 1) / NWV) * J * ((NN / 32) / CTT));                       \
        hipLaunchKernelGGL((k_ring2<NN, CTT, NWV, PF, 0>), dim3(g), dim3(NWV * 64), 0, 0, x, w, y, ntile_r);     \
    }, (double)nx * 4 + (double)rp * J * NN * 4 + (double)NTYPES * NCH * (NN / 32) * 2048)
    RING2("ring2 (x by DMA) N192 CT6 4w PF2", 192, 6, 4, 2);
    RING2("ring2 (x by DMA) N192 CT6 4w PF3", 192, 6, 4, 3);
    RING2("ring2 (x by DMA) N768 CT6 4w PF2", 768, 6, 4, 2);
    RING2("ring2 (x by DMA) N768 CT6 4w PF3", 768, 6, 4, 3);
    RING("ring N192 CT6 4w PF2", 192, 6, 4, 2, 0);
    RING("ring N192 CT3 4w PF2", 192, 3, 4, 2, 0);
    RING("ring N192 CT3 4w PF3", 192, 3, 4, 3, 0);
    RING("ring N192 CT2 4w PF2", 192, 2, 4, 2, 0);
    RING("ring N192 CT6 2w PF2", 192, 6, 2, 2, 0);
    RING("ring N192 CT3 2w PF2", 192, 3, 2, 2, 0);
    RING("ring N768 CT6 4w PF2", 768, 6, 4, 2, 0);
    RING("ring N768 CT6 4w PF3", 768, 6, 4, 3, 0);
    RING("ring N768 CT3 4w PF2", 768, 3, 4, 2, 0);
    RING("ring N768 CT6 4w PF2 no MFMA", 768, 6, 4, 2, NOMFMA);
    return 0;
}
