// k_gl3: StaticGraphLinear (graph_structural.py:30-43) + fused epilogue, v3 schedule.
//
// v2 kept all J node accumulators of a 16x16 output tile in every wave, which forces many small
// 16x16x4 MFMAs per loaded operand and a J^2 VALU node-mixing epilogue.  v3 splits the NODES
// over the 4 waves of a workgroup instead:
//   * workgroup tile = 32 rows x 32 output columns x all J nodes; wave w owns nodes w, w+4, ...
//     with one 32x32 accumulator each (v_mfma_f32_32x32x2_f32: 64-cycle issue = dependent
//     latency, so an 8-long chain per node per 16-deep chunk costs nothing; 2x the FLOPs per
//     operand register of 16x16x4);
//   * weights: LDS-DMA double-buffered stages, image [type][k-half][k-quad][col][4] so each
//     ds_read_b128 lane group reads 16 consecutive 16-B slots (conflict-free);
//   * x: each lane streams 8 contiguous k of its row (2 x float4) per node per chunk, prefetched
//     one chunk ahead; the counted vmcnt + raw s_barrier keeps those loads in flight;
//   * after the K loop, Y = s_j * acc + bias goes to LDS one 16-row half at a time (aliasing the
//     weight stages) and the node mixing Z = G-hat . Y runs as a 16x16x4 MFMA GEMM
//     (M = J, K = J, N = 16 rows x 32 cols), followed by FiLM / tanh / residual / store.
// Exact fp32 throughout (f32-input MFMA = k-ordered fmaf chain).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sd_internal.h"

namespace sd {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ floatx4 g4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }
__device__ __forceinline__ floatx4 l4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

template <int N>
struct VmCnt3 {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    static constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
};

// tanh(x) = 1 - 2 / (exp(2x) + 1): v_exp_f32 + v_rcp_f32; saturates cleanly at +-1 and is
// within ~2e-7 absolute of tanhf (the layer outputs feed a 1e-4 end-to-end bar)
__device__ __forceinline__ float fast_tanh(float x) {
    const float e = __expf(2.0f * x);
    return 1.0f - 2.0f * __frcp_rn(e + 1.0f);
}

constexpr int YSTRIDE = 528;  // floats per node in the Y half-tile (16 x 32 + 16 pad: lg rows -> other banks)

// weight chunk -> LDS stage, piece q = ((type*2 + h)*2 + kq)*32 + col  (16 B each)
__device__ __forceinline__ void fill_w3(const GLArgs& p, int c0, int k0, int K, float* dst, int wave, int lane) {
    const int npieces = p.ntypes * 128;
    for (int q0 = wave * 64; q0 < npieces; q0 += 256) {
        const int q = q0 + lane;
        const int col = q & 31;
        const int tk = q >> 5;  // (type*2 + h)*2 + kq
        const int n = min(c0 + col, p.N - 1);
        const float* src = p.W + ((int64_t)(tk >> 2) * p.N + n) * K + k0 + 4 * (tk & 3);
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 4), 16, 0, 0);
    }
}

}  // namespace

template <int J, bool RMS>
__global__ __launch_bounds__(256, 2) void k_gl3(const GLArgs p) {
    constexpr int NPW = (J + 3) / 4;      // nodes per wave
    constexpr int KS = (J + 3) / 4;       // 4-deep k steps of the mixing GEMM (K = J padded)
    constexpr int IB = (J + 15) / 16;     // 16-row i blocks of the mixing GEMM
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, h = lane >> 5, lr = lane & 15, lg = lane >> 4;
    const int stage = p.ntypes * 512;
    const int wbytes = 2 * stage;
    const int ybytes = J * YSTRIDE;
    float* sW0 = smem;
    float* sW1 = smem + stage;
    float* sY = smem;                                   // aliases the weight stages after the K loop
    float* sG = smem + (wbytes > ybytes ? wbytes : ybytes);

    const int ntile_c = (p.N + 31) >> 5;
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    const int ct = L % ntile_c;
    const int64_t row0 = (int64_t)(L / ntile_c) * 32;
    const int c0 = ct * 32;
    const int K = p.K1 + p.K2;
    const int nchunk = K >> 4;

    const int64_t arow = row0 + l32;
    const int64_t arow_c = arow < p.B ? arow : 0;  // tail rows read row 0, never stored
    const float* x1r = p.x1 + ((arow_c + p.x1_row0) / p.x1_div) * p.x1_rs + 8 * h;
    const float* x2r = p.K2 ? p.x2 + arow_c * p.x2_rs + 8 * h : nullptr;

    floatx16 acc[NPW];
    floatx4 a0[NPW], a1[NPW];
    float ss[NPW];
#pragma unroll
    for (int m = 0; m < NPW; ++m) {
        ss[m] = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[m][e] = 0.f;
    }
    auto node_of = [&](int m) { return wave + 4 * m; };
    auto load_x = [&](int c, int m, floatx4& lo, floatx4& hi) {
        const int j = min(node_of(m), J - 1);
        const int k0 = c << 4;
        const float* src = (k0 < p.K1) ? x1r + (int64_t)j * p.K1 + k0 : x2r + (int64_t)j * p.K2 + (k0 - p.K1);
        lo = g4(src);
        hi = g4(src + 4);
    };

    fill_w3(p, c0, 0, K, sW0, wave, lane);
#pragma unroll
    for (int m = 0; m < NPW; ++m) load_x(0, m, a0[m], a1[m]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int c = 0; c < nchunk; ++c) {
        const float* cur = (c & 1) ? sW1 : sW0;
        if (c + 1 < nchunk) fill_w3(p, c0, (c + 1) << 4, K, (c & 1) ? sW0 : sW1, wave, lane);
        const int cn = min(c + 1, nchunk - 1);
        const bool rms_chunk = RMS && (c << 4) < p.K1;
        auto wfrag = [&](int m) { return cur + (((p.ntype[min(node_of(m), J - 1)] * 2 + h) * 2) * 32 + l32) * 4; };
        floatx4 wa_n = l4(wfrag(0)), wb_n = l4(wfrag(0) + 128);  // weight fragments read one node ahead
#pragma unroll
        for (int m = 0; m < NPW; ++m) {
            const int j = node_of(m);
            const floatx4 xa = a0[m], xb = a1[m];
            const floatx4 wa = wa_n, wb = wb_n;
            if (m + 1 < NPW) {
                wa_n = l4(wfrag(m + 1));
                wb_n = l4(wfrag(m + 1) + 128);
            }
            load_x(cn, m, a0[m], a1[m]);  // every wave issues exactly 2*NPW loads (vmcnt below)
            if (j >= J) continue;         // wave-uniform: only the MFMAs are skipped
            if (rms_chunk)
                ss[m] += xa.x * xa.x + xa.y * xa.y + xa.z * xa.z + xa.w * xa.w + xb.x * xb.x + xb.y * xb.y +
                         xb.z * xb.z + xb.w * xb.w;
            floatx16 cc = acc[m];
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa.x, wa.x, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa.y, wa.y, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa.z, wa.z, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa.w, wa.w, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xb.x, wb.x, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xb.y, wb.y, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xb.z, wb.z, cc, 0, 0, 0);
            cc = __builtin_amdgcn_mfma_f32_32x32x2f32(xb.w, wb.w, cc, 0, 0, 0);
            acc[m] = cc;
        }
        if (c + 1 < nchunk) {
            // this chunk issued: weight DMA for c+1, then 2*NPW x prefetches -> retire the DMA only
            __builtin_amdgcn_s_waitcnt(VmCnt3<2 * NPW>::imm);
            __builtin_amdgcn_s_barrier();
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- per (row, node) scale + bias, in the accumulator layout:
    //      D[row = (r&3) + 8(r>>2) + 4h][col = l32] for register r of the 32x32 tile
    const int ncol = c0 + l32;
#pragma unroll
    for (int m = 0; m < NPW; ++m) {
        const int j = node_of(m);
        if (j >= J) continue;
        if (RMS) {
            float t = ss[m] + __shfl_xor(ss[m], 32);  // sum over the two k-halves of row l32
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float n2 = __shfl(t, (r & 3) + 8 * (r >> 2) + 4 * h);
                acc[m][r] *= 1.0f / fmaxf(sqrtf(n2), 1e-12f);
            }
        }
        if (p.bias) {
            const float bv = ncol < p.N ? p.bias[p.wrow[j] + ncol] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][r] += bv;
        }
    }

    // G-hat as the A operand of the mixing GEMM: A[i = ib*16 + lr][k = 4s + lg]
    for (int i = tid; i < J * J; i += 256) sG[i] = p.G[i];
    __syncthreads();  // also: every wave is done reading the weight stages (sY aliases them)
    float ga[IB][KS];
#pragma unroll
    for (int ib = 0; ib < IB; ++ib)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int i = ib * 16 + lr, jj = 4 * s + lg;
            ga[ib][s] = (i < J && jj < J) ? sG[i * J + jj] : 0.f;
        }

    float fa[2] = {1.f, 1.f}, fb[2] = {0.f, 0.f};  // FiLM for this lane's two output columns
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
        const int n = c0 + 16 * hb + lr;
        if (p.film && n < p.N) {
            fa[hb] = p.film[n] + 1.0f;
            fb[hb] = p.film[p.N + n];
        }
    }

#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        if (hf) __syncthreads();  // previous half's Y fully consumed
        // Y half -> LDS: sY[j][r][c], r = row within the half
#pragma unroll
        for (int m = 0; m < NPW; ++m) {
            const int j = node_of(m);
            if (j >= J) continue;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int r = (q & 3) + 8 * (q >> 2) + 4 * h;
                sY[j * YSTRIDE + r * 32 + l32] = acc[m][8 * hf + q];
            }
        }
        __syncthreads();
        // Z[i][rc] = sum_j G[i][j] Y[j][rc], rc = r*32 + c; wave w takes rc blocks w*8 .. w*8+7
#pragma unroll 2
        for (int b = 0; b < 8; ++b) {
            const int rc = (wave * 8 + b) * 16 + lr;
            const int r = rc >> 5, cc = rc & 31;
            const int64_t row = row0 + 16 * hf + r;
            const int n = c0 + cc;
            const int hb = cc >> 4;
            const bool ok = row < p.B && n < p.N;
            // residual loads first: their latency hides under the LDS reads + mixing MFMAs
            float rv[IB][4];
#pragma unroll
            for (int ib = 0; ib < IB; ++ib)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int i = ib * 16 + 4 * lg + e;
                    rv[ib][e] = (p.res && ok && i < J) ? p.res[row * p.res_rs + (int64_t)i * p.N + n] : 0.f;
                }
            float yb[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int jj = 4 * s + lg;
                yb[s] = jj < J ? sY[jj * YSTRIDE + rc] : 0.f;
            }
#pragma unroll
            for (int ib = 0; ib < IB; ++ib) {
                floatx4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < KS; ++s) z = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[ib][s], yb[s], z, 0, 0, 0);
                if (!ok) continue;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int i = ib * 16 + 4 * lg + e;
                    if (i >= J) continue;
                    float v = z[e];
                    if (p.film) v = v * fa[hb] + fb[hb];
                    if (p.act == 1) v = fast_tanh(v);
                    v += rv[ib][e];
                    p.out[row * p.out_rs + (int64_t)i * p.N + n] = v;
                }
            }
        }
    }
}

template <int J>
static hipError_t gl3_launch(const GLArgs& a, bool rms, hipStream_t s) {
    const int ntile_c = (a.N + 31) / 32;
    const int64_t ntile_r = (a.B + 31) / 32;
    const dim3 grid((unsigned)(ntile_c * ntile_r));
    const size_t wfl = (size_t)2 * a.ntypes * 512, yfl = (size_t)J * YSTRIDE;
    size_t lds = ((wfl > yfl ? wfl : yfl) + (size_t)J * J) * sizeof(float);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    auto kt = rms ? k_gl3<J, true> : k_gl3<J, false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    g_route_bits |= kRouteExact;
    hipLaunchKernelGGL(kt, grid, dim3(256), lds, s, a);
    return hipGetLastError();
}

// v3 covers the skeleton sizes of the release configs; returns hipErrorNotSupported otherwise.
hipError_t launch_graph_linear_v3(const GLArgs& a, bool rms, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if ((size_t)2 * a.ntypes * 512 * 4 > 120 * 1024) return hipErrorNotSupported;
    switch (a.J) {
        case 16: return gl3_launch<16>(a, rms, s);
        case 17: return gl3_launch<17>(a, rms, s);
        case 21: return gl3_launch<21>(a, rms, s);
        default: return hipErrorNotSupported;
    }
}

}  // namespace sd
