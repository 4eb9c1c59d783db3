// k_gl2: StaticGraphLinear (graph_structural.py:30-43) + fused epilogue, v2 schedule for gfx950.
//
// Same math and register tile as v1 (sd_kernels.hip, k_graph_linear): a wave owns 16 rows x
// (16*NCB) output columns for ALL J nodes, the exact-f32 MFMA v_mfma_f32_16x16x4_f32 does the
// per-node GEMM, and the G-hat node mixing + epilogue run in registers.  What changes is how the
// operands arrive:
//   * the weight tile of a 16-deep k chunk (all node types x 16*NCB columns) is brought into LDS
//     ONCE per workgroup by LDS-DMA (global_load_lds_dwordx4, no VGPRs), double-buffered, and
//     shared by the 4 waves (v1 re-read it from L1/L2 in every wave);
//   * LDS image [type][k-group][n][4 floats]: the 16 lanes of every ds_read_b128 lane group
//     read 16 distinct consecutive 16-B slots -> conflict-free;
//   * each node's x fragment for chunk c+1 is issued right after its last use in chunk c, so the
//     global latency hides under the other J-1 nodes' MFMAs (small J; large J loads on demand);
//   * __launch_bounds__(256, 2): <= 256 VGPR+AGPR, two workgroups per CU.
// One barrier per chunk: it retires the DMA for the next stage (RAW) and frees the stage the
// next fill overwrites (WAR).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sd_internal.h"

namespace sd {

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ floatx4 gld4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt immediate for "vmcnt <= n" with lgkmcnt / expcnt untouched (gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int N>
struct VmCnt {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    static constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
};

template <int NT>
__device__ __forceinline__ void fill_w_stage(const GLArgs& p, int c0, int k0, int K, float* dst, int wave,
                                             int lane) {
    // piece q (16 B) = (type, k-group, n), n fastest; one wave instruction = 64 pieces = 1 KiB
    const int npieces = p.ntypes * 4 * NT;
    for (int q0 = wave * 64; q0 < npieces; q0 += 256) {
        const int q = q0 + lane;
        const int n = q % NT;
        const int tl = q / NT;
        const int col = min(c0 + n, p.N - 1);  // tail columns: any valid row, never stored
        const float* src = p.W + ((int64_t)(tl >> 2) * p.N + col) * K + k0 + 4 * (tl & 3);
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 4), 16, 0, 0);
    }
}

}  // namespace

template <int JM, bool EXACT, int NCB, bool RMS, bool PREF, int MINW>
__global__ __launch_bounds__(256, MINW) void k_gl2(const GLArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NT = 16 * NCB;
    const int J = EXACT ? JM : p.J;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
    const int stage = p.ntypes * NT * 16;
    float* sW0 = smem;
    float* sW1 = smem + stage;
    float* sG = smem + 2 * stage;

    // XCD-aware tile order (cdna_hip_programming.md §5.5 T1): blocks b and b+8 share an XCD, so
    // logical tile L = (blocks of this XCD, in order) keeps the column tiles of one row tile -
    // which re-read the same x rows - inside one XCD's L2.  Bijective for any grid size.
    const int ntile_c = (p.N + NT - 1) / NT;
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int ct = L % ntile_c;
    const int64_t rt = L / ntile_c;
    const int64_t row0 = rt * 64 + wave * 16;
    const int c0 = ct * NT;
    const int K = p.K1 + p.K2;
    const int nchunk = K >> 4;

    const int64_t arow = row0 + lr;
    const bool rok = arow < p.B;
    const int64_t arow_c = rok ? arow : 0;
    const float* x1r = p.x1 + ((arow_c + p.x1_row0) / p.x1_div) * p.x1_rs + 4 * lg;
    const float* x2r = p.K2 ? p.x2 + arow_c * p.x2_rs + 4 * lg : nullptr;
    // Tail rows read row 0 (valid memory) and are never stored, so every wave issues exactly J
    // x loads per chunk - the counted vmcnt below relies on that count.
    auto load_a = [&](int c, int j) -> floatx4 {
        const int k0 = c << 4;
        const float* src = (k0 < p.K1) ? x1r + (int64_t)j * p.K1 + k0 : x2r + (int64_t)j * p.K2 + (k0 - p.K1);
        return gld4(src);
    };

    floatx4 acc[JM][NCB];
    floatx4 a[JM];
    float ss[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) {
        ss[j] = 0.f;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) acc[j][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

    fill_w_stage<NT>(p, c0, 0, K, sW0, wave, lane);
    for (int i = tid; i < J * J; i += 256) sG[i] = p.G[i];
    if (PREF) {
#pragma unroll
        for (int j = 0; j < JM; ++j)
            if (EXACT || j < J) a[j] = load_a(0, j);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int c = 0; c < nchunk; ++c) {
        const float* cur = (c & 1) ? sW1 : sW0;
        if (c + 1 < nchunk) fill_w_stage<NT>(p, c0, (c + 1) << 4, K, (c & 1) ? sW0 : sW1, wave, lane);
        const bool rms_chunk = RMS && (c << 4) < p.K1;
        const int cn = min(c + 1, nchunk - 1);  // branch-free prefetch (last chunk re-reads itself)
        // B fragments are read one node ahead so the ds_read latency hides under the MFMAs
        floatx4 bnext[NCB];
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
            bnext[cb] = *reinterpret_cast<const floatx4*>(cur + ((p.ntype[0] * 4 + lg) * NT + lr) * 4 + cb * 64);
#pragma unroll
        for (int j = 0; j < JM; ++j) {
            if (!EXACT && j >= J) continue;
            floatx4 bj[NCB];
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) bj[cb] = bnext[cb];
            if (j + 1 < JM && (EXACT || j + 1 < J)) {
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb)
                    bnext[cb] = *reinterpret_cast<const floatx4*>(
                        cur + ((p.ntype[j + 1] * 4 + lg) * NT + lr) * 4 + cb * 64);
            }
            floatx4 aj;
            if (PREF) {
                aj = a[j];
                a[j] = load_a(cn, j);
            } else {
                aj = load_a(c, j);
            }
            if (rms_chunk) ss[j] += aj.x * aj.x + aj.y * aj.y + aj.z * aj.z + aj.w * aj.w;
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                const floatx4 b = bj[cb];
                floatx4 cc = acc[j][cb];
                cc = mfma4(aj.x, b.x, cc);
                cc = mfma4(aj.y, b.y, cc);
                cc = mfma4(aj.z, b.z, cc);
                cc = mfma4(aj.w, b.w, cc);
                acc[j][cb] = cc;
            }
        }
        bool counted = false;
        if constexpr (PREF && EXACT) {
            if (c + 1 < nchunk) {
                // Issue order in this chunk: weight DMA for c+1 first, then the J x prefetches
                // for c+1.  vmcnt(J) retires the DMA while leaving the x loads in flight across
                // the barrier (a __syncthreads() would emit vmcnt(0) and drain them).
                __builtin_amdgcn_s_waitcnt(VmCnt<JM>::imm);
                __builtin_amdgcn_s_barrier();
                counted = true;
            }
        }
        if (!counted) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }

    if (row0 >= p.B) return;  // no barrier below
    if (RMS) {  // F.normalize(x, dim=-1): 1 / max(||x_bj||, 1e-12) per (row, node)
#pragma unroll
        for (int j = 0; j < JM; ++j) {
            if (!EXACT && j >= J) continue;
            float t = ss[j];
            t += __shfl_xor(t, 16);
            t += __shfl_xor(t, 32);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float s = 1.0f / fmaxf(sqrtf(__shfl(t, 4 * lg + r)), 1e-12f);
#pragma unroll
                for (int cb = 0; cb < NCB; ++cb) acc[j][cb][r] *= s;
            }
        }
    }
    if (p.bias) {  // per source node, before the mixing (graph_structural.py:38-41)
#pragma unroll
        for (int j = 0; j < JM; ++j) {
            if (!EXACT && j >= J) continue;
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) {
                const int n = c0 + 16 * cb + lr;
                acc[j][cb] += (n < p.N) ? p.bias[p.wrow[j] + n] : 0.f;
            }
        }
    }
    float fa[NCB], fb[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
        const int n = c0 + 16 * cb + lr;
        fa[cb] = 1.f;
        fb[cb] = 0.f;
        if (p.film && n < p.N) {
            fa[cb] = p.film[n] + 1.0f;
            fb[cb] = p.film[p.N + n];
        }
    }
    for (int i = 0; i < J; ++i) {
        floatx4 z[NCB];
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) z[cb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < JM; ++j) {
            if (!EXACT && j >= J) continue;
            const float g = sG[i * J + j];
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) z[cb] += g * acc[j][cb];
        }
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            const int n = c0 + 16 * cb + lr;
            if (n >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = row0 + 4 * lg + r;
                if (row >= p.B) continue;
                float v = z[cb][r];
                if (p.film) v = v * fa[cb] + fb[cb];
                if (p.act == 1) v = tanhf(v);
                if (p.res) v += p.res[row * p.res_rs + (int64_t)i * p.N + n];
                p.out[row * p.out_rs + (int64_t)i * p.N + n] = v;
            }
        }
    }
}

template <int JM, bool EXACT, int NCB, bool PREF, int MINW>
static hipError_t gl2_launch(const GLArgs& a, bool rms, hipStream_t s) {
    constexpr int NT = 16 * NCB;
    const int ntile_c = (a.N + NT - 1) / NT;
    const int64_t ntile_r = (a.B + 63) / 64;
    const dim3 grid((unsigned)(ntile_c * ntile_r));
    size_t lds = (size_t)(2 * a.ntypes * NT * 16 + a.J * a.J) * sizeof(float);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    auto kt = rms ? k_gl2<JM, EXACT, NCB, true, PREF, MINW> : k_gl2<JM, EXACT, NCB, false, PREF, MINW>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    g_route_bits |= kRouteExact;
    hipLaunchKernelGGL(kt, grid, dim3(256), lds, s, a);
    return hipGetLastError();
}

// Column-tile width: 32 (NCB=2) halves the x re-reads, 16 (NCB=1) doubles the number of
// workgroups; at small B*N the 32-wide grid cannot give every CU two workgroups, so go narrow.
// SKELDIFF_GL_NCB=1|2 forces a width (tuning / A-B runs).
static int ncb_choice(const GLArgs& a) {
    static const int forced = [] {
        const char* e = getenv("SKELDIFF_GL_NCB");
        return e ? atoi(e) : 0;
    }();
    if (forced == 1 || forced == 2) return forced;
    const int64_t wgs32 = (int64_t)((a.N + 31) / 32) * ((a.B + 63) / 64);
    return wgs32 >= 2 * 256 ? 2 : 1;
}

hipError_t launch_graph_linear_v2(const GLArgs& a, bool rms, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    // two 32-column weight stages must fit comfortably in LDS
    const bool wide = ncb_choice(a) == 2 && a.ntypes * 32 * 16 * 4 * 2 <= 96 * 1024;
    switch (a.J) {
        case 16: return wide ? gl2_launch<16, true, 2, true, 2>(a, rms, s) : gl2_launch<16, true, 1, true, 3>(a, rms, s);
        case 17: return wide ? gl2_launch<17, true, 2, true, 2>(a, rms, s) : gl2_launch<17, true, 1, true, 3>(a, rms, s);
        case 21: return gl2_launch<21, true, 1, true, 2>(a, rms, s);
        case 51: return gl2_launch<51, true, 1, false, 1>(a, rms, s);
        default: break;
    }
    if (a.J <= 8) return gl2_launch<8, false, 2, true, 2>(a, rms, s);
    if (a.J <= 16) return gl2_launch<16, false, 1, true, 2>(a, rms, s);
    if (a.J <= 32) return gl2_launch<32, false, 1, false, 2>(a, rms, s);
    return gl2_launch<64, false, 1, false, 1>(a, rms, s);
}

}  // namespace sd
