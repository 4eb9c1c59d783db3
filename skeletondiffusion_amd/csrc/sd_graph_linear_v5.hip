// v5: StaticGraphLinear (graph_structural.py:30-43) + fused epilogue for LARGE skeletons
// (J > 21: AMASS-MANO J = 51 with 43 node types, config 3).  The GEMM phase runs on the v4
// split-f16 products (k_gl4t, sd_graph_linear_v4.hip: launch_gemm_split) wherever the plan holds
// split weights; k_gl5_gemm below is the exact-f32 GEMM phase (kernel variant 5, other shapes).
//
// The one-kernel generations keep all J nodes of a row tile in one workgroup, so every k chunk
// stages the weights of every node type: at J = 51 that is 43 types (v3/v4 do not fit the LDS;
// v2 fits with 16-column tiles only and reaches 17.7 TF/s).  v5 splits the layer in two:
//   k_gl5_gemm   z[b, j, :] = s_bj W[type j] [x1_bj | x2_bj] + bias[type j]    per node j:
//                a row-batched GEMM (64 rows x 64 columns per workgroup, 2 x 2 waves of
//                v_mfma_f32_32x32x2_f32, K staged 32 deep in 16-B pieces, double-buffered with
//                register prefetch), one weight slab per workgroup; s_bj = 1 / max(||x1_bj||, 1e-12) (RMS)
//                from the staged x1 elements; z goes straight into `out`;
//   k_gl5_mix    out[b, i, :] = act(FiLM(sum_j G-hat[i, j] z[b, j, :])) + res[b, i, :]   in place:
//                one workgroup per (row, 64 columns) stages the row's J x 64 z slab in LDS before
//                it writes the same slab (each element read and written by its own workgroup).
// x1/x2 must not alias out.  When res aliases out (x = GL(h) + x), z goes to the caller's scratch
// (GLArgs::zs, a dead activation buffer of the step) instead, so the residual is read intact.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sd_internal.h"

namespace sd {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned uint4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
template <int N>
struct VmC {  // s_waitcnt vmcnt(N), expcnt / lgkmcnt not waited
    static_assert(N >= 0 && N < 64, "vmcnt range");
    static constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
};

constexpr int TM = 64, TN = 64, TK = 32;

struct Regs {
    float4 a[2], b[2];
};

// A (rows x K, k contiguous), 16-B pieces: thread piece q is row (tid >> 3) + 32q, k = k0 + 4 (tid & 7)
// (K1, K2, row strides and bases 16-B aligned: checked at launch; a piece never straddles K1)
__device__ __forceinline__ float4 x_piece(const GLArgs& p, int j, int64_t b, int k) {
    if (k < p.K1)
        return *reinterpret_cast<const float4*>(p.x1 + ((b + p.x1_row0) / p.x1_div) * p.x1_rs + (int64_t)j * p.K1 + k);
    return *reinterpret_cast<const float4*>(p.x2 + b * p.x2_rs + (int64_t)j * p.K2 + (k - p.K1));
}

template <bool RMS>
__device__ __forceinline__ void load_stage(const GLArgs& p, const float* W, int j, int64_t m0, int n0, int k0, int K,
                                           int tid, Regs& r, float* ssq) {
    const int kq = 4 * (tid & 7), mr = tid >> 3;
    const int gk = k0 + kq;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int64_t b = m0 + mr + 32 * q;
        const float4 v = (b < p.B && gk < K) ? x_piece(p, j, b, gk) : zero;
        r.a[q] = v;
        if (RMS && gk < p.K1) ssq[q] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        const int n = n0 + mr + 32 * q;
        r.b[q] = (n < p.N && gk < K) ? *reinterpret_cast<const float4*>(W + (int64_t)n * K + gk) : zero;
    }
}

__device__ __forceinline__ void store_stage(float (*As)[TM + 4], float (*Bs)[TN + 4], int tid, const Regs& r) {
    const int kq = 4 * (tid & 7), mr = tid >> 3;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int m = mr + 32 * q;
        As[kq + 0][m] = r.a[q].x; As[kq + 1][m] = r.a[q].y; As[kq + 2][m] = r.a[q].z; As[kq + 3][m] = r.a[q].w;
        Bs[kq + 0][m] = r.b[q].x; Bs[kq + 1][m] = r.b[q].y; Bs[kq + 2][m] = r.b[q].z; Bs[kq + 3][m] = r.b[q].w;
    }
}

template <bool RMS>
__global__ __launch_bounds__(256) void k_gl5_gemm(const GLArgs p, float* __restrict__ z, int64_t z_rs) {
    __shared__ float As[2][TK][TM + 4];
    __shared__ float Bs[2][TK][TN + 4];
    __shared__ float s_scale[TM];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int j = blockIdx.z;
    const int64_t m0 = (int64_t)blockIdx.y * TM;
    const int n0 = blockIdx.x * TN;
    const int K = p.K1 + p.K2;
    const float* W = p.W + (int64_t)p.wrow[j] * K;

    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    float ssq[2] = {0.f, 0.f};

    Regs r;
    load_stage<RMS>(p, W, j, m0, n0, 0, K, tid, r, ssq);
    store_stage(As[0], Bs[0], tid, r);
    __syncthreads();
    int cur = 0;
    for (int k0 = 0; k0 < K; k0 += TK) {
        const bool more = k0 + TK < K;
        if (more) load_stage<RMS>(p, W, j, m0, n0, k0 + TK, K, tid, r, ssq);
#pragma unroll
        for (int kk = 0; kk < TK; kk += 2) {
            const float a = As[cur][kk + (lane >> 5)][wm * 32 + (lane & 31)];
            const float b = Bs[cur][kk + (lane >> 5)][wn * 32 + (lane & 31)];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
        if (more) store_stage(As[cur ^ 1], Bs[cur ^ 1], tid, r);
        __syncthreads();
        cur ^= 1;
    }
    if (RMS) {  // F.normalize(x1, dim=-1): 8 consecutive lanes hold one row's k slice
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            float t = ssq[q];
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) t += __shfl_xor(t, o, 64);
            if ((tid & 7) == 0) s_scale[(tid >> 3) + 32 * q] = 1.0f / fmaxf(sqrtf(t), 1e-12f);
        }
        __syncthreads();
    }
    // C/D map: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
    const int n = n0 + wn * 32 + (lane & 31);
    if (n >= p.N) return;
    const float bv = p.bias ? p.bias[p.wrow[j] + n] : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int m = wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int64_t b = m0 + m;
        if (b < p.B) {
            const float v = RMS ? acc[e] * s_scale[m] : acc[e];
            z[b * z_rs + (int64_t)j * p.N + n] = v + bv;
        }
    }
}

// Each thread owns one column and the 16 rows i = 16 * wave + q: per source node one LDS read of
// z and four 16-B broadcast reads of G-hat^T[j][16 wave .. +15] feed 16 multiply-adds (the
// one-row-per-step form issued two LDS reads per multiply-add and was LDS-bound at ~1.3 TB/s).
__global__ __launch_bounds__(256) void k_gl5_mix(const GLArgs p, const float* z, int64_t z_rs, int vec) {
    __shared__ __attribute__((aligned(16))) float s_z[kMaxNodes][64];
    __shared__ __attribute__((aligned(16))) float s_gt[kMaxNodes][kMaxNodes + 4];
    const int tid = threadIdx.x, J = p.J, N = p.N;
    const int64_t b = blockIdx.x;
    const int n0 = blockIdx.y * 64;
    float* orow = p.out + b * p.out_rs;
    const float* zrow = z + b * z_rs;
    // G-hat^T staged from coalesced reads of G-hat's rows (reading its columns, one 4-B load per
    // lane from J different rows, was ~60 % of the kernel at J = 51); the padding nodes are zero
    for (int e = tid; e < J * J; e += 256) {
        const int i = e / J, jj = e - i * J;
        s_gt[jj][i] = p.G[e];
    }
    for (int e = tid; e < J * (kMaxNodes - J); e += 256) {
        const int jj = e / (kMaxNodes - J), i = J + e % (kMaxNodes - J);
        s_gt[jj][i] = 0.f;
    }
    if (vec && n0 + 64 <= N) {  // 16-B pieces (z, N and z_rs 16-B aligned: checked at launch)
        for (int e = tid; e < J * 16; e += 256) {
            const int jj = e >> 4, c4 = (e & 15) * 4;
            *reinterpret_cast<float4*>(&s_z[jj][c4]) =
                *reinterpret_cast<const float4*>(zrow + (int64_t)jj * N + n0 + c4);
        }
    } else {
        for (int e = tid; e < J * 64; e += 256) {
            const int jj = e >> 6, c = e & 63;
            s_z[jj][c] = (n0 + c < N) ? zrow[(int64_t)jj * N + n0 + c] : 0.f;
        }
    }
    // the residual pieces are loaded before the barrier, so their latency overlaps the mixing
    const int c = tid & 63, n = n0 + c, i0 = 16 * (tid >> 6);
    const bool live = n < N && i0 < J;
    float rv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) rv[q] = (p.res && live && i0 + q < J) ? p.res[b * p.res_rs + (int64_t)(i0 + q) * N + n] : 0.f;
    __syncthreads();
    if (!live) return;
    float acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
    for (int jj = 0; jj < J; ++jj) {
        const float zv = s_z[jj][c];
        const float4* g4 = reinterpret_cast<const float4*>(&s_gt[jj][i0]);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const float4 g = g4[v];
            acc[4 * v + 0] = fmaf(g.x, zv, acc[4 * v + 0]);
            acc[4 * v + 1] = fmaf(g.y, zv, acc[4 * v + 1]);
            acc[4 * v + 2] = fmaf(g.z, zv, acc[4 * v + 2]);
            acc[4 * v + 3] = fmaf(g.w, zv, acc[4 * v + 3]);
        }
    }
    float fa = 1.f, fb = 0.f;
    if (p.film) {
        fa = p.film[n] + 1.0f;
        fb = p.film[N + n];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int i = i0 + q;
        if (i >= J) break;
        float v = acc[q];
        if (p.film) v = v * fa + fb;
        if (p.act == 1) v = tanhf(v);  // (the v_exp / v_rcp form measured no faster here: 175 vs 174 us)
        orow[(int64_t)i * N + n] = v + rv[q];
    }
}

// The mixing pass on the matrix cores, R rows per workgroup.  k_gl5_mix above is bound by its LDS
// reads: per source node every wave issues one z read and four 16-B G-hat^T broadcast reads (4 LDS
// cycles each) for 16 multiply-adds, ~18 LDS cycles per 16 FMAs, with one row per workgroup.  Here
// per (row b, 64 columns) Z^T = z^T G-hat^T runs on v_mfma_f32_16x16x4_f32: A = z^T[col][j] from
// the row's z slab in LDS (one 4-B read per lane per MFMA), B = G-hat^T[j][i] in registers (wave w
// owns output nodes 16 w .. 16 w + 15; ceil(J / 4) fragments, loaded once per workgroup), D[col =
// 16 cb + 4 l4 + e][i = 16 w + l16]: four consecutive columns of one node per lane, so the
// residual loads and output stores are 16 B.  The f32 MFMA accumulates its 4 k products as an fmaf
// chain in k order, so each sum is k_gl5_mix's j-ordered fmaf chain (zero padding adds exact
// zeros).  The next row's slab is loaded to registers while the current row is mixed (two LDS
// slab buffers, one barrier per row).  J <= 64, N % 64 == 0, 16-B aligned z / res / out.
template <int R, int PD, bool TR = false>  // TR: mix with G-hat^T (the training backward, dz = G-hat^T dy)
__global__ __launch_bounds__(256) void k_gl5_mixm(const GLArgs p, const float* z, int64_t z_rs) {
    constexpr int ZS = 80;                 // floats per slab row (64 + 16: the 4 k lanes of a read hit 4 bank groups)
    constexpr int QPT = kMaxNodes * 16 / 256;  // 16-B slab pieces per thread at most (4)
    // two slab buffers of 4 ceil(J / 4) rows (the k extent of the MFMAs; rows >= J stay zero) in
    // dynamic LDS: 33 KB at J = 51, four workgroups per CU
    extern __shared__ __attribute__((aligned(16))) float s_z[];
    const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, l4 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int J = p.J, N = p.N, KS = (J + 3) >> 2;
    const int SLAB = 4 * KS * ZS, NQ = 4 * KS * 16;  // floats per slab buffer, 16-B pieces per slab
    const int n0 = blockIdx.y * 64;
    const int64_t b0 = (int64_t)blockIdx.x * R;
    const int nrows = (int)min((int64_t)R, p.B - b0);
    // B fragments: G-hat^T[j = 4 s + l4][i = 16 w + l16] = G-hat[i][j], zero outside J x J
    const int i = 16 * w + l16;
    float gb[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int j = 4 * s + l4;
        gb[s] = (s < KS && i < J && j < J) ? p.G[TR ? j * J + i : i * J + j] : 0.f;
    }
    // FiLM (scale + 1 | shift) of the workgroup's 64 columns, in LDS (read per row: registers
    // held across the row loop would cost an occupancy step)
    float* s_f = s_z + 2 * SLAB;
    if (tid < 64) {
        s_f[tid] = p.film ? p.film[n0 + tid] + 1.0f : 1.0f;
        s_f[64 + tid] = p.film ? p.film[N + n0 + tid] : 0.0f;
    }
    // slab piece q of thread t: node q >> 4, columns 4 (q & 15) .. + 3 (pieces of nodes >= J: zero).
    // PD = 2: a register ring of two slabs and two residual sets -- slab r + 2 and the residual of
    // row r + 1 are loaded while row r is mixed (about two rows of cover for each load); PD = 1:
    // slab r + 1 and row r's residual are loaded at the start of row r (one set each).
    float4 zv[PD][QPT];
    auto load_slab = [&](int r, int sl) {
        const float* zr = z + (b0 + r) * z_rs + n0;
#pragma unroll
        for (int k = 0; k < QPT; ++k) {
            const int q = tid + 256 * k, j = q >> 4;
            zv[sl][k] = (j < J && q < NQ) ? *reinterpret_cast<const float4*>(zr + (int64_t)j * N + 4 * (q & 15)) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_slab = [&](int buf, int sl) {
#pragma unroll
        for (int k = 0; k < QPT; ++k) {
            const int q = tid + 256 * k;
            if (q < NQ) *reinterpret_cast<float4*>(s_z + buf * SLAB + (q >> 4) * ZS + 4 * (q & 15)) = zv[sl][k];
        }
    };
    const bool live = i < J;  // this lane's output node
    float4 rv[PD][4];
    auto load_res = [&](int r, int sl) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
            rv[sl][cb] = (p.res && live) ? *reinterpret_cast<const float4*>(p.res + (b0 + r) * p.res_rs + (int64_t)i * N + n0 + 16 * cb + 4 * l4)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    // row r (slot sl = r & 1, a literal at each call site): its slab is in LDS buffer sl, its
    // residual in rv[sl]; zv[sl] is free (slab r is in LDS) and zv[sl ^ 1] holds slab r + 1
    auto row_step = [&](int r, const int sl) {
        const int zs = PD == 2 ? sl : 0, rs = PD == 2 ? sl : 0;  // ring slots of slab r + PD, residual r
        if constexpr (PD == 2) {
            if (r + 2 < nrows) load_slab(r + 2, zs);
            if (r + 1 < nrows) load_res(r + 1, rs ^ 1);
        } else {
            if (r + 1 < nrows) load_slab(r + 1, 0);
            load_res(r, 0);
        }
        floatx4 acc[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            floatx4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                if (s < KS) {  // wave-uniform
                    const float a = s_z[sl * SLAB + (4 * s + l4) * ZS + 16 * cb + l16];
                    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a, gb[s], t, 0, 0, 0);
                }
            }
            acc[cb] = t;
        }
        if (live) {
            float* orow = p.out + (b0 + r) * p.out_rs + (int64_t)i * N + n0 + 4 * l4;
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                float v[4] = {acc[cb][0], acc[cb][1], acc[cb][2], acc[cb][3]};
                const float4 fa = *reinterpret_cast<const float4*>(s_f + 16 * cb + 4 * l4);
                const float4 fb = *reinterpret_cast<const float4*>(s_f + 64 + 16 * cb + 4 * l4);
                const float fav[4] = {fa.x, fa.y, fa.z, fa.w};
                const float fbv[4] = {fb.x, fb.y, fb.z, fb.w};
                const float rvv[4] = {rv[rs][cb].x, rv[rs][cb].y, rv[rs][cb].z, rv[rs][cb].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (p.film) v[e] = v[e] * fav[e] + fbv[e];
                    if (p.act == 1) v[e] = tanhf(v[e]);
                    v[e] = v[e] + rvv[e];
                }
                *reinterpret_cast<float4*>(orow + 16 * cb) = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
        if (r + 1 < nrows) store_slab(sl ^ 1, PD == 2 ? zs ^ 1 : 0);  // LDS buffer sl ^ 1 was last read in row r - 1
        __syncthreads();
    };
    load_slab(0, 0);
    store_slab(0, 0);
    if constexpr (PD == 2) {
        if (nrows > 1) load_slab(1, 1);
        load_res(0, 0);
    }
    __syncthreads();
    for (int r = 0; r < nrows; r += 2) {
        row_step(r, 0);
        if (r + 1 < nrows) row_step(r + 1, 1);
    }
}

// k_gl5_mixm with its operands streamed by LDS-DMA (round 4).  k_gl5_mixm loads row r + 1's slab
// into registers while row r is mixed -- one row (52 MFMAs per wave at J = 51, ~0.8 us) of cover for
// a memory latency, with the VGPRs of a deeper ring costing occupancy (MFMA busy 29 %, SQ_WAIT_ANY
// 60 % at J = 51).  Here the z slab AND the residual slab of row r + PF go straight to LDS ring slot
// (r + PF) % NS by global_load_lds_dwordx4 (no VGPRs), issued after row r's barrier, so PF rows of
// MFMAs cover each load; the output leaves through raw buffer stores whose out-of-range offsets
// are dropped by the hardware (dead lanes and rows store nothing without a branch), so every wave
// issues a fixed number of memory operations per row and the wait for row r is an exact vmcnt.
// The same MFMA sequence (A = z^T from LDS, B = G-hat^T fragments, k steps in j order) and
// epilogue as k_gl5_mixm: bitwise equal.  Slab rows are 64 floats with the 16-B pieces of odd rows
// XOR-swizzled by 4 (the A reads of rows 4 s + l4, l4 = 0 / 1 then hit different bank halves).
// DMA instruction k of a slab covers rows 4 k .. 4 k + 3 and belongs to wave k % 4.
template <int R, int PF, bool RES>
__global__ __launch_bounds__(256, 2) void k_gl5_mixd(const GLArgs p, const float* z, int64_t z_rs) {
    constexpr int NS = PF + 1;
    const int J = p.J, N = p.N, KS = (J + 3) >> 2;
    const int SL = 4 * KS * 64;                   // floats per slab (4 KS rows x 64 columns)
    extern __shared__ __attribute__((aligned(16))) float s_m[];
    float* s_zr = s_m;                            // [NS][z | res][SL]
    const int tid = threadIdx.x, lane = tid & 63, l16 = lane & 15, l4 = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n0 = blockIdx.y * 64;
    const int64_t b0 = (int64_t)blockIdx.x * R;
    const int nrows = (int)min((int64_t)R, p.B - b0);
    const int i = 16 * w + l16;
    float gb[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int j = 4 * s + l4;
        gb[s] = (s < KS && i < J && j < J) ? p.G[i * J + j] : 0.f;
    }
    // this lane's FiLM values (the same for every row) straight to registers, issued with G-hat's
    // loads (one memory latency, waited at the first row's epilogue).  (Staged through LDS, they
    // were read back after the fills, a read the waitcnt pass cannot tell apart from a DMA
    // destination: vmcnt(0) -- the next rows' fills -- before every row's epilogue.)
    float4 fa[4], fb[4];
    if (p.film) {  // wave-uniform
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const float4 a = *reinterpret_cast<const float4*>(p.film + n0 + 16 * cb + 4 * l4);
            fa[cb] = make_float4(a.x + 1.0f, a.y + 1.0f, a.z + 1.0f, a.w + 1.0f);
            fb[cb] = *reinterpret_cast<const float4*>(p.film + N + n0 + 16 * cb + 4 * l4);
        }
    } else {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            fa[cb] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
            fb[cb] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
    }
    // the k padding rows J .. 4 KS - 1 of every z slot stay zero (never a DMA destination)
    for (int q = tid; q < NS * (4 * KS - J) * 64; q += 256) {
        const int sl = q / ((4 * KS - J) * 64), e = q % ((4 * KS - J) * 64);
        s_zr[sl * (RES ? 2 : 1) * SL + J * 64 + e] = 0.f;
    }
    const int nk = KS;                          // DMA instructions per slab
    const int nkw = (nk - w + 3) >> 2;          // this wave's share (instructions w, w + 4, ...)
    // a slab's 16-B pieces: lane L of instruction k -> LDS row 4 k + (L >> 4), piece L & 15, which
    // holds global piece (L & 15) ^ ((row & 1) << 2)
    auto fill = [&](int r) {  // row r (clamped to a valid row) into slot r % NS
        const int64_t br = b0 + min(r, nrows - 1);
        float* dz = s_zr + (r % NS) * (RES ? 2 : 1) * SL;
        const int row_in = lane >> 4, pc = lane & 15;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int k = w + 4 * kk;
            if (k >= nk) continue;  // wave-uniform
            const int row = 4 * k + row_in;
            const int gp = pc ^ ((row & 1) << 2);
            const int rowc = min(row, J - 1);  // lanes of rows >= J: a valid source, masked below
            if (row < J) {
                __builtin_amdgcn_global_load_lds((const void*)(z + br * z_rs + (int64_t)rowc * N + n0 + 4 * gp),
                                                 (lds_void*)(dz + 4 * k * 64), 16, 0, 0);
                if constexpr (RES)
                    __builtin_amdgcn_global_load_lds((const void*)(p.res + br * p.res_rs + (int64_t)rowc * N + n0 + 4 * gp),
                                                     (lds_void*)(dz + SL + 4 * k * 64), 16, 0, 0);
            }
        }
    };
    // output: raw buffer stores relative to the workgroup's first row; out-of-range offsets dropped
    const int64_t obase = b0 * p.out_rs;
    const uint32_t oreach = (uint32_t)min((int64_t)nrows * p.out_rs * 4, (int64_t)0x7fffffff);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(p.out + obase, 0, (int)oreach, 0x00020000);
    constexpr int ST = 4;                                        // stores per row and wave
    const int FO = nkw * (RES ? 2 : 1);                          // DMA operations per fill and wave
    auto wait_row = [&](int younger_fills, int younger_stores) {  // vmcnt: the ops issued after row r's fill
        const int n = younger_fills * FO + younger_stores * ST;
        // a switch over the possible immediates (n <= (PF - 1) * 8 + PF * 4)
        switch (n) {
#define SD_VMC(v) case v: __builtin_amdgcn_s_waitcnt(VmC<v>::imm); break;
            SD_VMC(0) SD_VMC(1) SD_VMC(2) SD_VMC(3) SD_VMC(4) SD_VMC(5) SD_VMC(6) SD_VMC(7) SD_VMC(8) SD_VMC(9)
            SD_VMC(10) SD_VMC(11) SD_VMC(12) SD_VMC(13) SD_VMC(14) SD_VMC(15) SD_VMC(16) SD_VMC(17) SD_VMC(18)
            SD_VMC(19) SD_VMC(20) SD_VMC(21) SD_VMC(22) SD_VMC(23) SD_VMC(24) SD_VMC(25) SD_VMC(26) SD_VMC(27)
            SD_VMC(28) SD_VMC(29) SD_VMC(30) SD_VMC(31) SD_VMC(32)
#undef SD_VMC
            default: __builtin_amdgcn_s_waitcnt(VmC<0>::imm); break;
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    __syncthreads();  // the zero rows before any DMA lands next to them
#pragma unroll
    for (int q = 0; q < PF; ++q) fill(q);  // rows 0 .. PF - 1 (clamped rows repeat a valid one)
    for (int r = 0; r < nrows; ++r) {
        // order per row m: wait(m), fill(m + PF), compute(m), stores(m); the prologue fills rows
        // 0 .. PF - 1.  Issued after fill(r): PF - 1 fills (prologue ones included) and min(r, PF)
        // rows' stores (stores(r - PF) when r >= PF, then fill(m + PF), stores(m) for m < r)
        const int m0 = max(r - PF + 1, 0);
        const int yrows = (r - m0) + (r < PF ? (PF - 1 - r) : 0);   // later fills (incl. prologue ones)
        const int ystores = r - m0 + (r >= PF ? 1 : 0);
        wait_row(yrows, ystores);
        const float* zs = s_zr + (r % NS) * (RES ? 2 : 1) * SL;
        // the row's residual out of LDS before the next fill is issued (read after it, the compiler
        // drained vmcnt(0) -- that fill too -- before the read: it cannot tell the two apart)
        // The reads are ds_read_b128 by inline asm: the waitcnt pass makes every LDS access it
        // knows wait for all LDS-DMA in flight (it cannot tell fill(r + 1)'s slot from slot r), so a
        // plain read here drained vmcnt(0) each row; wait_row already covers slot r, and the
        // lgkmcnt(0) below covers the asm reads themselves
        float4 rq[4];
        if constexpr (RES) {
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                const float* a = zs + SL + min(i, J - 1) * 64 + (((4 * cb + l4) ^ ((min(i, J - 1) & 1) << 2)) << 2);
                asm volatile("ds_read_b128 %0, %1" : "=v"(rq[cb]) : "v"((uint32_t)(uintptr_t)a) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        fill(r + PF);  // slot (r + PF) % NS = (r - 1) % NS: read in row r - 1, before this barrier
        // the four column blocks' chains interleaved (k step outer): consecutive MFMAs are
        // independent; each block still sums its k steps in order (bit-identical)
        floatx4 acc[4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            if (s < KS) {  // wave-uniform
                const int row = 4 * s + l4;
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    const float a = zs[row * 64 + ((((16 * cb + l16) >> 2) ^ ((l4 & 1) << 2)) << 2) + (l16 & 3)];
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, gb[s], acc[cb], 0, 0, 0);
                }
            }
        }
        const bool live = i < J;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            float v[4] = {acc[cb][0], acc[cb][1], acc[cb][2], acc[cb][3]};
            const float fav[4] = {fa[cb].x, fa[cb].y, fa[cb].z, fa[cb].w};
            const float fbv[4] = {fb[cb].x, fb[cb].y, fb[cb].z, fb[cb].w};
            float rvv[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (RES) {
                rvv[0] = rq[cb].x; rvv[1] = rq[cb].y; rvv[2] = rq[cb].z; rvv[3] = rq[cb].w;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (p.film) v[e] = v[e] * fav[e] + fbv[e];
                if (p.act == 1) v[e] = tanhf(v[e]);
                v[e] = v[e] + rvv[e];
            }
            const int off = live ? (int)((r * p.out_rs + (int64_t)i * N + n0 + 16 * cb + 4 * l4) * 4) : 0x7ffffff0;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, make_float4(v[0], v[1], v[2], v[3])), orsrc,
                                                   off, 0, 0);
        }
    }
    __builtin_amdgcn_s_waitcnt(VmC<0>::imm);  // the trailing (clamped) fills land before LDS is released
}

}  // namespace

// The mixing pass alone (the training graph-linear, sd_train.hip): out[r, i, :] = sum_j M[i, j]
// z[r, j, :] with M = G-hat (transpose 0) or G-hat^T (1), z and out (rows, J, N) row-major; the same
// j-ordered fmaf chains as sd_train.hip's k_mix.  hipErrorNotSupported unless N % 64 == 0 with
// 16-B aligned buffers and J <= 64.
hipError_t launch_mix_mfma(const float* z, const float* G, float* out, int64_t rows, int J, int N, bool transpose,
                           hipStream_t s) {
    if (J < 1 || J > kMaxNodes || N % 64 || ((uintptr_t)z & 15) || ((uintptr_t)out & 15) || rows / 8 >= 0x7fffffff)
        return hipErrorNotSupported;
    if (rows <= 0) return hipSuccess;
    GLArgs a{};
    a.G = G;
    a.out = out;
    a.out_rs = (int64_t)J * N;
    a.B = rows;
    a.N = N;
    a.J = J;
    const size_t lds = (2 * 4 * (size_t)((J + 3) / 4) * 80 + 128) * sizeof(float);
    const dim3 grid((unsigned)((rows + 7) / 8), (unsigned)(N / 64));
    if (transpose) hipLaunchKernelGGL((k_gl5_mixm<8, 1, true>), grid, dim3(256), lds, s, a, z, (int64_t)J * N);
    else hipLaunchKernelGGL((k_gl5_mixm<8, 1, false>), grid, dim3(256), lds, s, a, z, (int64_t)J * N);
    return hipGetLastError();
}

// Row-major operands only; J <= kMaxNodes.  hipErrorNotSupported where v5 does not apply.
hipError_t launch_graph_linear_v5(const GLArgs& a, bool rms, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (a.J < 1 || a.J > kMaxNodes || a.x1_blk || a.x2_blk || a.res_blk || a.out_blk) return hipErrorNotSupported;
    if (a.x1 == a.out || (a.x2 && a.x2 == a.out)) return hipErrorNotSupported;  // in-place GEMM would race
    // 16-B operand pieces
    if ((a.K1 & 3) || (a.K2 & 3) || (a.x1_rs & 3) || (a.K2 && (a.x2_rs & 3)) || ((uintptr_t)a.x1 & 15) ||
        ((uintptr_t)a.x2 & 15) || ((uintptr_t)a.W & 15))
        return hipErrorNotSupported;
    float* z = a.out;
    int64_t z_rs = a.out_rs;
    if (a.res && a.res == a.out) {  // the residual must survive the GEMM: z into the scratch
        if (!a.zs || a.zs_cap < a.B * a.J * (int64_t)a.N || a.zs == a.x1 || a.zs == a.x2) return hipErrorNotSupported;
        z = a.zs;
        z_rs = (int64_t)a.J * a.N;
    } else if (a.res && a.res < a.out + a.B * a.out_rs && a.out < a.res + a.B * a.res_rs) {
        return hipErrorNotSupported;  // partial overlap
    }
    const int64_t row_tiles = (a.B + TM - 1) / TM;
    if (row_tiles > 65535 || a.B > 65535 * 1024LL) return hipErrorNotSupported;
    // GEMM phase: split-f16 products (k_gl4y: 3 x v_mfma_f32_32x32x16_f16 per 16-deep k step, the
    // v4 arithmetic) unless the exact-f32 v5 is forced (kernel variant 5)
    hipError_t e = a.variant == 5 ? hipErrorNotSupported : launch_gemm_split(a, rms, z, z_rs, s);
    if (e == hipErrorNotSupported) {
        const dim3 g1((unsigned)((a.N + TN - 1) / TN), (unsigned)row_tiles, (unsigned)a.J);
        g_route_bits |= kRouteV5Mix;
        if (rms)
            hipLaunchKernelGGL(k_gl5_gemm<true>, g1, dim3(256), 0, s, a, z, z_rs);
        else
            hipLaunchKernelGGL(k_gl5_gemm<false>, g1, dim3(256), 0, s, a, z, z_rs);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return e;
    if (a.skip_mix) return z == a.out ? hipSuccess : hipErrorNotSupported;  // the pre-mix Y in out
    const int vec = ((uintptr_t)z & 15) == 0 && (a.N & 3) == 0 && (z_rs & 3) == 0;
    g_route_bits |= kRouteV5Mix;
    // the matrix-core mixing pass: 64-column blocks, 16-B z / residual / output pieces
    const bool mfma = !a.v5_valu && vec && a.N % 64 == 0 && ((uintptr_t)a.out & 15) == 0 && (a.out_rs & 3) == 0 &&
                      (!a.res || (((uintptr_t)a.res & 15) == 0 && (a.res_rs & 3) == 0)) && a.B / 8 < 0x7fffffff;
    if (mfma && (int64_t)a.B * a.out_rs * 4 < 0x7fffffff && (!a.res || a.res_rs % 4 == 0)) {
        // the LDS-DMA form: slabs of 4 ceil(J / 4) rows, 2 slots (row r + 1 in flight while row r is
        // mixed): 53 KiB of LDS at J = 51 with the residual, 3 workgroups per CU -- config 3 4,193 /
        // 4,195 vs 4,070 / 4,068 futures/s for 3 slots (2 workgroups per CU), profiles/r05k/ab_mixd.txt;
        // 8 rows per workgroup: 4,095 / 4,097 vs 4,065 / 4,044 (4 rows) and 4,003 / 3,999 (16 rows),
        // profiles/r05m/ab_mixd_rows.txt (the other forms: git history before round 6)
        const int KS = (a.J + 3) / 4;
        auto launch = [&](auto kt, int R, int PF) -> hipError_t {
            const size_t lds = (size_t)(PF + 1) * (a.res ? 2 : 1) * 4 * KS * 64 * sizeof(float);
            if (lds > 64 * 1024) {
                const hipError_t e = hipFuncSetAttribute((const void*)kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(kt, dim3((unsigned)((a.B + R - 1) / R), (unsigned)(a.N / 64)), dim3(256), lds, s, a,
                               (const float*)z, z_rs);
            return hipGetLastError();
        };
        return a.res ? launch(k_gl5_mixd<8, 1, true>, 8, 1) : launch(k_gl5_mixd<8, 1, false>, 8, 1);
    }
    if (mfma) {
        const dim3 blk(256);
        const unsigned ncb = (unsigned)(a.N / 64);
        const size_t lds = (2 * 4 * (size_t)((a.J + 3) / 4) * 80 + 128) * sizeof(float);  // <= 41.5 KB (J <= 64)
        hipLaunchKernelGGL((k_gl5_mixm<8, 1>), dim3((unsigned)((a.B + 7) / 8), ncb), blk, lds, s, a, (const float*)z, z_rs);
        return hipGetLastError();
    }
    const dim3 g2((unsigned)a.B, (unsigned)((a.N + 63) / 64));
    hipLaunchKernelGGL(k_gl5_mix, g2, dim3(256), 0, s, a, (const float*)z, z_rs, vec);
    return hipGetLastError();
}

}  // namespace sd
