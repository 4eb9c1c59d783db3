// Training side of the StaticGraphLinear (SURVEY.md §8f "next" #4): forward with the pre-mix
// activations kept for backward, and the backward the reference gets from torch autograd over
// GraphLinear.forward (src/core/network/layers/graph_structural.py:30-43, 105-114):
//   z[r, j, :] = W[type j] x[r, j, :] + bias[type j]         (per-node GEMM, rows x K -> rows x N)
//   y[r, i, :] = sum_j ghat[i, j] z[r, j, :]                  (node mixing)
// backward from dy:
//   dz[r, j, :] = sum_i ghat[i, j] dy[r, i, :]                (mixing with ghat^T)
//   dx[:, j, :] = dz[:, j, :] W[type j]                       (per-node GEMM)
//   dW[t]       = sum_{j: type j = t} dz[:, j, :]^T x[:, j, :] (per-type GEMM, reduction over rows)
//   dbias[t]    = sum_{r, j: type j = t} dz[r, j, :]
//   dghat[i, j] = sum_{r, n} dy[r, i, n] z[r, j, n]
// The three GEMMs are one strided kernel on v_mfma_f32_32x32x2_f32 (exact f32 products, f32
// accumulate): 64x64 C tile per 256-thread workgroup (2x2 waves of 32x32), K staged 16 at a time
// through LDS; the reduction over rows (dW) is split over row ranges into partial tiles that a
// fixed-order pass sums (deterministic, no float atomics).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/skeldiff.h"
#include "sd_internal.h"

namespace sd {
namespace {

constexpr int TM = 64, TN = 64, TK = 32;
constexpr int TE = TM * TK / 256;  // staged elements per thread and operand
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Strided batched GEMM: for batch z (grid.z = nbatch * splits):
//   node mode (by_type = 0): group = {node j = batch}, t = type(j)
//   type mode (by_type = 1): group = {nodes j with type(j) = batch}, t = batch
// C[c_off + m*cm + n] (+)= sum over the group, k of A[a_off + m*am + k*ak] * B[b_off + k*bk + n*bn]
// with a_off = j*aj + t*at, b_off = j*bj + t*bt, c_off = (by_type ? t : j)*cz + split*cs.
// splits > 1 (dW, where the reduction index k is the row index): split s takes k in
// [s*kchunk, min(K, (s+1)*kchunk)) and writes its own partial slab (c_off += s*cs).
struct GemmArgs {
    const float* A;
    const float* B;
    float* C;
    const float* bias;  // node mode only: C += bias[t*bt_bias + n]
    const int64_t* types;
    int M, N, K, J, by_type, splits, kchunk;
    int64_t am, ak, aj, at, bk, bn, bj, bt, cm, cz, cs, bias_t;
};

// Tile staging: TK = 32 deep (measured: 64-deep tiles halve the workgroups per CU through LDS and
// run 45 % slower), two LDS buffers, the next tile's global loads held in registers
// while the MFMAs of the current one run (one barrier per tile).  The unit-stride dimension of
// each operand runs over consecutive threads (am == 1 / bn == 1 select the mapping).
struct TileRegs {
    float a[TE], b[TE];
};

// ok ? v : 0 on a value already in registers (the asm pins it there: without it the select became
// a load through a selected address -- the tile registers went to scratch)
__device__ __forceinline__ float keep_or_zero(bool ok, float v) {
    asm volatile("" : "+v"(v));
    return ok ? v : 0.f;
}
__device__ __forceinline__ float4 keep_or_zero(bool ok, float4 v) {
    f32x4 t = {v.x, v.y, v.z, v.w};
    asm volatile("" : "+v"(t));
    return ok ? make_float4(t[0], t[1], t[2], t[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// LDS column swizzle of the k_gemm operand tiles: column m of k row k is stored at m ^ 4 ((k >> 2) & 7)
// (bits 2-4 only: 16-B pieces stay whole and aligned, a row's 32-column halves stay put).  The
// transposed stores of a k-contiguous operand (store_tile4, ak / bk == 1: a thread writes k rows
// kk .. kk + 3 of one column, lanes 8 apart in kk) hit 8 of the 32 banks at the 68-float row stride
// -- 4-way conflicts, 33 % of k_gemm's LDS cycles (profiles/r05d/pmc_kgemm.txt); swizzled they hit
// all 32, and the MFMA reads (32 consecutive columns of one k row) stay conflict-free
__device__ __forceinline__ int swz(int k, int m) { return m ^ (((k >> 2) & 7) << 2); }

__device__ __forceinline__ void load_tile(const GemmArgs& g, const float* A, const float* B, int m0, int n0, int k0,
                                          int kend, int kval, int tid, TileRegs& r) {
    // unconditional loads from clamped indices (kval: a valid k); the out-of-range values are
    // zeroed at the LDS store (store_tile), when they have arrived: a masked load beside a zero
    // write of the same register waited vmcnt(0) per element, and a select right after the load
    // would wait for it there
#pragma unroll
    for (int q = 0; q < TE; ++q) {
        const int idx = tid + 256 * q;
        int mm, kk;
        if (g.am == 1) { mm = idx & 63; kk = idx >> 6; } else { kk = idx & (TK - 1); mm = idx / TK; }
        const int gm = m0 + mm, gk = k0 + kk;
        r.a[q] = A[min(gm, g.M - 1) * g.am + (int64_t)(gk < kend ? gk : kval) * g.ak];
        int nn, kb;
        if (g.bn == 1) { nn = idx & 63; kb = idx >> 6; } else { kb = idx & (TK - 1); nn = idx / TK; }
        const int gn = n0 + nn, gkb = k0 + kb;
        r.b[q] = B[(int64_t)(gkb < kend ? gkb : kval) * g.bk + min(gn, g.N - 1) * g.bn];
    }
}

__device__ __forceinline__ void store_tile(const GemmArgs& g, float (*As)[TM + 4], float (*Bs)[TN + 4], int tid,
                                           const TileRegs& r, int m0, int n0, int k0, int kend) {
#pragma unroll
    for (int q = 0; q < TE; ++q) {
        const int idx = tid + 256 * q;
        int mm, kk;
        if (g.am == 1) { mm = idx & 63; kk = idx >> 6; } else { kk = idx & (TK - 1); mm = idx / TK; }
        As[kk][swz(kk, mm)] = keep_or_zero(m0 + mm < g.M && k0 + kk < kend, r.a[q]);
        int nn, kb;
        if (g.bn == 1) { nn = idx & 63; kb = idx >> 6; } else { kb = idx & (TK - 1); nn = idx / TK; }
        Bs[kb][swz(kb, nn)] = keep_or_zero(n0 + nn < g.N && k0 + kb < kend, r.b[q]);
    }
}

// 16-B pieces (VEC): 512 float4 per operand tile, 2 per thread, along the operand's unit-stride
// dimension (k: kq = 4 (tid & 7), row (tid >> 3) + 32 q;  m / n: 4 (tid & 15), k (tid >> 4) + 16 q).
// The host checks strides, extents and bases are multiples of 4 floats / 16 B (gemm_vec_ok).
struct TileRegs4 {
    float4 a[2], b[2];
};

__device__ __forceinline__ void load_tile4(const GemmArgs& g, const float* A, const float* B, int m0, int n0, int k0,
                                           int kend, int kval, int tid, TileRegs4& r) {
    // unconditional 16-B loads from clamped pieces (kval: a valid k; the last full piece of the m /
    // n extent, a multiple of 4: gemm_vec_ok); the out-of-range pieces are zeroed at the LDS store
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        int mm, kk;
        if (g.ak == 1) { kk = 4 * (tid & 7); mm = (tid >> 3) + 32 * q; } else { mm = 4 * (tid & 15); kk = (tid >> 4) + 16 * q; }
        const int gm = m0 + mm, gk = k0 + kk;
        const int gmc = gm < g.M ? gm : (g.am == 1 ? g.M - 4 : g.M - 1), gkc = gk < kend ? gk : kval;
        r.a[q] = *reinterpret_cast<const float4*>(A + gmc * g.am + (int64_t)gkc * g.ak);
        int nn, kb;
        if (g.bk == 1) { kb = 4 * (tid & 7); nn = (tid >> 3) + 32 * q; } else { nn = 4 * (tid & 15); kb = (tid >> 4) + 16 * q; }
        const int gn = n0 + nn, gkb = k0 + kb;
        const int gnc = gn < g.N ? gn : (g.bn == 1 ? g.N - 4 : g.N - 1), gkbc = gkb < kend ? gkb : kval;
        r.b[q] = *reinterpret_cast<const float4*>(B + (int64_t)gkbc * g.bk + gnc * g.bn);
    }
}

__device__ __forceinline__ void store_tile4(const GemmArgs& g, float (*As)[TM + 4], float (*Bs)[TN + 4], int tid,
                                            const TileRegs4& r, int m0, int n0, int k0, int kend) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        int mm, kk;
        if (g.ak == 1) { kk = 4 * (tid & 7); mm = (tid >> 3) + 32 * q; } else { mm = 4 * (tid & 15); kk = (tid >> 4) + 16 * q; }
        const float4 a = keep_or_zero(m0 + mm < g.M && k0 + kk < kend, r.a[q]);
        if (g.ak == 1) {
            As[kk][swz(kk, mm)] = a.x; As[kk + 1][swz(kk + 1, mm)] = a.y;
            As[kk + 2][swz(kk + 2, mm)] = a.z; As[kk + 3][swz(kk + 3, mm)] = a.w;
        } else {
            *reinterpret_cast<float4*>(&As[kk][swz(kk, mm)]) = a;
        }
        int nn, kb;
        if (g.bk == 1) { kb = 4 * (tid & 7); nn = (tid >> 3) + 32 * q; } else { nn = 4 * (tid & 15); kb = (tid >> 4) + 16 * q; }
        const float4 b = keep_or_zero(n0 + nn < g.N && k0 + kb < kend, r.b[q]);
        if (g.bk == 1) {
            Bs[kb][swz(kb, nn)] = b.x; Bs[kb + 1][swz(kb + 1, nn)] = b.y;
            Bs[kb + 2][swz(kb + 2, nn)] = b.z; Bs[kb + 3][swz(kb + 3, nn)] = b.w;
        } else {
            *reinterpret_cast<float4*>(&Bs[kb][swz(kb, nn)]) = b;
        }
    }
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) float As[2][TK][TM + 4];
    __shared__ __attribute__((aligned(16))) float Bs[2][TK][TN + 4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
    const int batch = blockIdx.z / g.splits, split = blockIdx.z % g.splits;
    const int kbeg = split * g.kchunk;
    const int kend = min(g.K, kbeg + g.kchunk);

    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;

    const int jbeg = g.by_type ? 0 : batch, jend = g.by_type ? g.J : batch + 1;
    for (int j = jbeg; j < jend; ++j) {
        const int t = g.types ? (int)g.types[j] : 0;
        if (g.by_type && t != batch) continue;  // uniform over the workgroup
        if (kbeg >= kend) continue;
        const float* A = g.A + j * g.aj + t * g.at;
        const float* B = g.B + j * g.bj + t * g.bt;
        auto mfma_tile = [&](int cur) {
#pragma unroll
            for (int kk = 0; kk < TK; kk += 2) {
                const int k = kk + (lane >> 5);
                const float a = As[cur][k][swz(k, wm * 32 + (lane & 31))];
                const float b = Bs[cur][k][swz(k, wn * 32 + (lane & 31))];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
            }
        };
        // the next tile's loads in registers while the MFMAs of this one run (one barrier per tile);
        // a three-deep register ring measured no faster (30.2 vs 29.4 us at N = K = 192, 1,024 rows,
        // with 180 VGPRs): the loop is not load-latency-bound
        TileRegs r;
        TileRegs4 r4;
        if (VEC) {
            load_tile4(g, A, B, m0, n0, kbeg, kend, kbeg, tid, r4);
            store_tile4(g, As[0], Bs[0], tid, r4, m0, n0, kbeg, kend);
        } else {
            load_tile(g, A, B, m0, n0, kbeg, kend, kbeg, tid, r);
            store_tile(g, As[0], Bs[0], tid, r, m0, n0, kbeg, kend);
        }
        __syncthreads();
        int cur = 0;
        for (int k0 = kbeg; k0 < kend; k0 += TK) {
            const bool more = k0 + TK < kend;
            if (more) {
                if (VEC) load_tile4(g, A, B, m0, n0, k0 + TK, kend, kbeg, tid, r4);
                else load_tile(g, A, B, m0, n0, k0 + TK, kend, kbeg, tid, r);
            }
            mfma_tile(cur);
            if (more) {
                if (VEC) store_tile4(g, As[cur ^ 1], Bs[cur ^ 1], tid, r4, m0, n0, k0 + TK, kend);
                else store_tile(g, As[cur ^ 1], Bs[cur ^ 1], tid, r, m0, n0, k0 + TK, kend);
            }
            __syncthreads();
            cur ^= 1;
        }
    }
    // C/D map: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
    float* C = g.C + batch * g.cz + split * g.cs;  // node j's or type t's output slab
    const int n = n0 + wn * 32 + (lane & 31);
    if (n >= g.N) return;
    float bv = 0.f;
    if (g.bias) {
        const int t = g.types ? (int)g.types[batch] : 0;
        bv = g.bias[t * g.bias_t + n];
    }
    // Every value and 32-bit byte offset first, pinned in registers, then the 16 stores (SGPR base +
    // VGPR offset): the compiler waits vmcnt(0) before it overwrites a pending store's data or
    // address registers, and reusing them per store waited out each store's completion in turn.
    // (Offsets past 4 GiB: the plain loop.)
    if ((int64_t)g.M * g.cm * 4 < 0xfffff000LL) {  // uniform
        float o[16];
        uint32_t off[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            o[r] = acc[r] + bv;
            off[r] = (uint32_t)((m * g.cm + n) * 4);
            asm volatile("" : "+v"(o[r]), "+v"(off[r]));
        }
        char* cb = reinterpret_cast<char*>(C);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (m < g.M) *reinterpret_cast<float*>(cb + off[r]) = o[r];
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < g.M) C[m * g.cm + n] = acc[r] + bv;
    }
}

// out[r, i, n] = sum_j M[i, j] in[r, j, n], M = ghat (transpose = 0) or ghat^T (transpose = 1).
// One workgroup per (row, 64-column chunk): the J x 64 input slab and M^T in LDS; each thread owns
// one column and RPT consecutive output rows (RPT * 4 >= J), fed per source node by one LDS read
// of the input and RPT / 4 16-B broadcast reads of M^T[j][i0 ..] (not two LDS reads per FMA).
// SKELDIFF_TRAIN_MIX=0 at load: the per-column k_mix everywhere (A/B)
static int g_train_mix_mfma = [] {
    const char* e = getenv("SKELDIFF_TRAIN_MIX");
    return e ? atoi(e) : 1;
}();

template <int RPT>
__global__ __launch_bounds__(256) void k_mix(const float* __restrict__ in, const float* __restrict__ ghat,
                                             float* __restrict__ out, int J, int N, int transpose) {
    __shared__ __attribute__((aligned(16))) float s_in[64][64];
    __shared__ __attribute__((aligned(16))) float s_mt[64][68];
    const int r = blockIdx.x, n0 = blockIdx.y * 64, tid = threadIdx.x;
    const int64_t base = (int64_t)r * J * N;
    for (int e = tid; e < J * 4 * RPT; e += 256) {
        const int jj = e / (4 * RPT), i = e % (4 * RPT);
        s_mt[jj][i] = i < J ? (transpose ? ghat[jj * J + i] : ghat[i * J + jj]) : 0.f;
    }
    for (int e = tid; e < J * 64; e += 256) {
        const int j = e >> 6, c = e & 63;
        s_in[j][c] = (n0 + c < N) ? in[base + (int64_t)j * N + n0 + c] : 0.f;
    }
    __syncthreads();
    const int c = tid & 63, i0 = RPT * (tid >> 6);
    if (n0 + c >= N || i0 >= J) return;
    float acc[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) acc[q] = 0.f;
    for (int j = 0; j < J; ++j) {
        const float x = s_in[j][c];
        const float4* m4 = reinterpret_cast<const float4*>(&s_mt[j][i0]);
#pragma unroll
        for (int v = 0; v < RPT / 4; ++v) {
            const float4 m = m4[v];
            acc[4 * v + 0] = fmaf(m.x, x, acc[4 * v + 0]);
            acc[4 * v + 1] = fmaf(m.y, x, acc[4 * v + 1]);
            acc[4 * v + 2] = fmaf(m.z, x, acc[4 * v + 2]);
            acc[4 * v + 3] = fmaf(m.w, x, acc[4 * v + 3]);
        }
    }
#pragma unroll
    for (int q = 0; q < RPT; ++q)
        if (i0 + q < J) out[base + (int64_t)(i0 + q) * N + n0 + c] = acc[q];
}

hipError_t launch_mix(const float* in, const float* ghat, float* out, int64_t rows, int J, int N, int transpose,
                      hipStream_t s) {
    // the matrix-core mixing pass (sd_graph_linear_v5.hip, k_gl5_mixm) for J > 32, where at least
    // three of its four waves own output nodes (at J = 16 three of four idle: 27.9 vs 15.8 us per
    // launch for the per-column form below, profiles/train_r03); the same fmaf chains
    if (g_train_mix_mfma && J > 32) {
        const hipError_t e = launch_mix_mfma(in, ghat, out, rows, J, N, transpose != 0, s);
        if (e != hipErrorNotSupported) return e;
    }
    const dim3 grid((unsigned)rows, (unsigned)((N + 63) / 64));
    if (J <= 16) hipLaunchKernelGGL(k_mix<4>, grid, dim3(256), 0, s, in, ghat, out, J, N, transpose);
    else if (J <= 32) hipLaunchKernelGGL(k_mix<8>, grid, dim3(256), 0, s, in, ghat, out, J, N, transpose);
    else hipLaunchKernelGGL(k_mix<16>, grid, dim3(256), 0, s, in, ghat, out, J, N, transpose);
    return hipGetLastError();
}

// partial dghat over a row range on v_mfma_f32_32x32x2_f32:
//   part[chunk][i][j] = sum_{r in chunk} (dY_r Z_r^T)[i][j],  dY_r, Z_r = (J x N) slabs of row r.
// Each wave takes every 4th row of the chunk; per 8-feature step a lane (node i or j = l & 31 of a
// 32-node tile, half h = l >> 5) loads 4 consecutive features k = k0 + 4h + s of its dy and z rows
// (16 B) and feeds them as MFMA k-step s: A and B use the same k permutation, so the sum over k
// is exact.  TI x TI 32x32 tiles cover J <= 32 * TI.  The 4 waves' tiles are summed in LDS in wave
// order (deterministic).
template <int TI>
__global__ __launch_bounds__(256) void k_dghat_part(const float* __restrict__ dy, const float* __restrict__ z,
                                                    float* __restrict__ part, int64_t rows, int J, int N,
                                                    int rows_per_chunk) {
    __shared__ float s_acc[TI * 32][TI * 32 + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 31, h = lane >> 5;
    f32x16 acc[TI][TI];
#pragma unroll
    for (int a = 0; a < TI; ++a)
#pragma unroll
        for (int b = 0; b < TI; ++b)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
    const int64_t r1 = min(rows, r0 + rows_per_chunk);
    const bool vec = (N & 7) == 0;
    for (int64_t r = r0 + w; r < r1; r += 4) {
        const float* dyr = dy + r * J * N;
        const float* zr = z + r * J * N;
        for (int k0 = 0; k0 < N; k0 += 8) {
            float av[TI][4], bv[TI][4];
#pragma unroll
            for (int a = 0; a < TI; ++a) {
                const int i = a * 32 + li;
                const int k = k0 + 4 * h;
                if (vec) {
                    float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
                    if (i < J) {
                        va = *(const float4*)(dyr + (int64_t)i * N + k);
                        vb = *(const float4*)(zr + (int64_t)i * N + k);
                    }
                    av[a][0] = va.x; av[a][1] = va.y; av[a][2] = va.z; av[a][3] = va.w;
                    bv[a][0] = vb.x; bv[a][1] = vb.y; bv[a][2] = vb.z; bv[a][3] = vb.w;
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const bool ok = i < J && k + q < N;
                        av[a][q] = ok ? dyr[(int64_t)i * N + k + q] : 0.f;
                        bv[a][q] = ok ? zr[(int64_t)i * N + k + q] : 0.f;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int a = 0; a < TI; ++a)
#pragma unroll
                    for (int b = 0; b < TI; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a][q], bv[b][q], acc[a][b], 0, 0, 0);
        }
    }
    // C/D map: col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
    for (int ww = 0; ww < 4; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int a = 0; a < TI; ++a)
#pragma unroll
                for (int b = 0; b < TI; ++b)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int i = a * 32 + (q & 3) + 8 * (q >> 2) + 4 * h, j = b * 32 + li;
                        s_acc[i][j] = (ww == 0 ? 0.f : s_acc[i][j]) + acc[a][b][q];
                    }
        }
        __syncthreads();
    }
    for (int p = tid; p < J * J; p += 256) part[(int64_t)blockIdx.x * J * J + p] = s_acc[p / J][p % J];
}

// J <= 16: the same partial dghat on v_mfma_f32_16x16x4_f32 (a 32x32 tile would leave three
// quarters of its products on padding): lane (node i = l & 15, quad kq = l >> 4) loads features
// k0 + 16u + 4kq .. +3 of its dy and z rows (16 B each, four 16-feature steps in flight) and feeds
// them as four k-steps; A and B share the permutation, so the sum over features is exact.
// One row per wave at a time; the 4 waves' tiles are summed in LDS in wave order.  N % 4 == 0.
__global__ __launch_bounds__(256) void k_dghat_part16(const float* __restrict__ dy, const float* __restrict__ z,
                                                      float* __restrict__ part, int64_t rows, int J, int N,
                                                      int rows_per_chunk) {
    __shared__ float s_acc[16][17];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = lane & 15, kq = lane >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_chunk;
    const int64_t r1 = min(rows, r0 + rows_per_chunk);
    for (int64_t r = r0 + w; r < r1; r += 4) {
        const float* dyr = dy + (r * J + i) * N;
        const float* zr = z + (r * J + i) * N;
        for (int k0 = 0; k0 < N; k0 += 64) {
            float4 va[4], vb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + 16 * u + 4 * kq;
                const bool ok = i < J && k < N;
                va[u] = ok ? *(const float4*)(dyr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
                vb[u] = ok ? *(const float4*)(zr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[u].x, vb[u].x, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[u].y, vb[u].y, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[u].z, vb[u].z, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[u].w, vb[u].w, acc, 0, 0, 0);
            }
        }
    }
    // C/D map: col = lane & 15, row = 4 (lane >> 4) + reg
    for (int ww = 0; ww < 4; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ii = 4 * kq + q;
                s_acc[ii][i] = (ww == 0 ? 0.f : s_acc[ii][i]) + acc[q];
            }
        }
        __syncthreads();
    }
    for (int p = tid; p < J * J; p += 256) part[(int64_t)blockIdx.x * J * J + p] = s_acc[p / J][p % J];
}

// partial dbias over a row range: part[chunk][t][n] = sum_{r in chunk, j: type j = t} dz[r,j,n]
__global__ __launch_bounds__(256) void k_dbias_part(const float* __restrict__ dz, const int64_t* __restrict__ types,
                                                    float* __restrict__ part, int64_t rows, int J, int N,
                                                    int n_types, int rows_per_chunk) {
    const int n = blockIdx.x * 256 + threadIdx.x, t = blockIdx.y;
    if (n >= N) return;
    const int64_t r0 = (int64_t)blockIdx.z * rows_per_chunk;
    const int64_t r1 = min(rows, r0 + rows_per_chunk);
    float acc = 0.f;
    for (int64_t r = r0; r < r1; ++r)
        for (int j = 0; j < J; ++j)
            if ((types ? (int)types[j] : 0) == t) acc += dz[(r * J + j) * N + n];
    part[((int64_t)blockIdx.z * n_types + t) * N + n] = acc;
}

// out[e] = sum_s part[s][e] in split order (deterministic)
__global__ __launch_bounds__(256) void k_sum_parts(const float* __restrict__ part, int splits, int64_t n,
                                                   float* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += part[s * n + e];
    out[e] = acc;
}

// out[e] = sum_s part[s][e] for few elements over many parts: one wave per element, lane l sums
// parts l, l + 64, ..., then a fixed xor-shuffle tree (deterministic)
__global__ __launch_bounds__(64) void k_sum_parts_wave(const float* __restrict__ part, int splits, int64_t n,
                                                       float* __restrict__ out) {
    const int64_t e = blockIdx.x;
    const int l = threadIdx.x;
    float acc = 0.f;
    for (int s = l; s < splits; s += 64) acc += part[s * n + e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (l == 0) out[e] = acc;
}

hipError_t sum_parts(const float* part, int splits, int64_t n, float* out, hipStream_t s) {
    if (splits >= 16 && n <= 65536)
        hipLaunchKernelGGL(k_sum_parts_wave, dim3((unsigned)n), dim3(64), 0, s, part, splits, n, out);
    else
        hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, splits, n, out);
    return hipGetLastError();
}

// 16-B pieces apply when each operand has a unit-stride dimension whose extent is a multiple of
// 4 and every other stride / offset / base is 16-B aligned
bool gemm_vec_ok(const GemmArgs& g) {
    auto m4 = [](int64_t v) { return (v & 3) == 0; };
    const bool a_ok = (g.ak == 1 && m4(g.K) && m4(g.kchunk) && m4(g.am)) || (g.am == 1 && m4(g.M) && m4(g.ak));
    const bool b_ok = (g.bk == 1 && m4(g.K) && m4(g.kchunk) && m4(g.bn)) || (g.bn == 1 && m4(g.N) && m4(g.bk));
    return a_ok && b_ok && m4(g.aj) && m4(g.at) && m4(g.bj) && m4(g.bt) && ((uintptr_t)g.A & 15) == 0 &&
           ((uintptr_t)g.B & 15) == 0;
}

hipError_t launch_gemm(const GemmArgs& g, dim3 grid, hipStream_t s) {
    if (gemm_vec_ok(g))
        hipLaunchKernelGGL(k_gemm<true>, grid, dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL(k_gemm<false>, grid, dim3(256), 0, s, g);
    return hipGetLastError();
}

constexpr int kRowsPerChunk = 16;  // dbias partials
constexpr int kDghatRows = 4;      // dghat partials (one row per wave)

int splits_for(int64_t rows) {
    // dW reduction: about 64 rows per split, at most 32 splits
    int64_t s = (rows + 255) / 256;
    return (int)(s < 1 ? 1 : (s > 32 ? 32 : s));
}

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }


// ---- attention over joints, training side (attention.py:122-136 under autograd) ---------------
// One workgroup per (row b, head h).  qkv (rows, J, 3 hid) row-major as to_qkv writes it, q at
// head h's columns [h dh, (h + 1) dh), k at hid + ..., v at 2 hid + ...; out (rows, J, hid).
//   S = (q scale) k^T, P = softmax_j(S), O = P v                                   (forward)
//   dV = P^T dO, dP = dO V^T, dS = P (dP - rowsum(P dP)), dQ = scale dS K, dK = dS^T (q scale)
// The head's q / k / v (and dO) go to LDS once; every product is a short f32 dot product from
// LDS (J, dh <= 64: at most 64 x 64 per operand).  P is recomputed in the backward instead of
// stored (one J x J product per (row, head)).  Row-wise softmax: one thread per query row.
template <bool BWD>
__global__ __launch_bounds__(256) void k_attn_train(const float* __restrict__ qkv, const float* __restrict__ dout,
                                                     float* __restrict__ out, int J, int heads, int dh, float scale) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int tid = threadIdx.x;
    const int64_t b = blockIdx.x / heads;
    const int h = blockIdx.x % heads;
    const int hid = heads * dh, JD = J * dh;
    const int DP = dh + 1;  // LDS row stride (odd: column walks across rows are conflict-free)
    const int JP = J + 1;
    float* sq = sm;               // [J][DP] q * scale
    float* sk = sq + J * DP;      // [J][DP]
    float* sv = sk + J * DP;      // [J][DP]
    float* sP = sv + J * DP;      // [J][JP] P
    float* sO = sP + J * JP;      // BWD: [J][DP] dO
    float* sS = sO + J * DP;      // BWD: [J][JP] dS
    const float* base = qkv + b * (int64_t)J * 3 * hid + h * dh;
    for (int e = tid; e < JD; e += 256) {
        const int n = e / dh, c = e - n * dh;
        const float* r = base + (int64_t)n * 3 * hid + c;
        sq[n * DP + c] = r[0] * scale;
        sk[n * DP + c] = r[hid];
        sv[n * DP + c] = r[2 * hid];
        if (BWD) sO[n * DP + c] = dout[(b * J + n) * (int64_t)hid + h * dh + c];
    }
    __syncthreads();
    for (int e = tid; e < J * J; e += 256) {
        const int n = e / J, j = e - n * J;
        float acc = 0.f;
        for (int c = 0; c < dh; ++c) acc = fmaf(sq[n * DP + c], sk[j * DP + c], acc);
        sP[n * JP + j] = acc;
    }
    __syncthreads();
    if (tid < J) {  // softmax over j of row n = tid
        float* row = sP + tid * JP;
        float m = -INFINITY;
        for (int j = 0; j < J; ++j) m = fmaxf(m, row[j]);
        float sum = 0.f;
        for (int j = 0; j < J; ++j) {
            const float e = expf(row[j] - m);
            row[j] = e;
            sum += e;
        }
        const float inv = 1.0f / sum;
        for (int j = 0; j < J; ++j) row[j] *= inv;
    }
    __syncthreads();
    if constexpr (!BWD) {
        for (int e = tid; e < JD; e += 256) {  // O[n][d] = sum_j P[n][j] v[j][d]
            const int n = e / dh, d = e - n * dh;
            float acc = 0.f;
            for (int j = 0; j < J; ++j) acc = fmaf(sP[n * JP + j], sv[j * DP + d], acc);
            out[(b * J + n) * (int64_t)hid + h * dh + d] = acc;
        }
        return;
    } else {
        // dP[n][j] = sum_d dO[n][d] v[j][d], kept in sS for the moment
        for (int e = tid; e < J * J; e += 256) {
            const int n = e / J, j = e - n * J;
            float acc = 0.f;
            for (int d = 0; d < dh; ++d) acc = fmaf(sO[n * DP + d], sv[j * DP + d], acc);
            sS[n * JP + j] = acc;
        }
        __syncthreads();
        if (tid < J) {  // dS = P (dP - sum_j P dP), row n = tid
            const float* pr = sP + tid * JP;
            float* dr = sS + tid * JP;
            float r = 0.f;
            for (int j = 0; j < J; ++j) r = fmaf(pr[j], dr[j], r);
            for (int j = 0; j < J; ++j) dr[j] = pr[j] * (dr[j] - r);
        }
        __syncthreads();
        float* g = out + b * (int64_t)J * 3 * hid + h * dh;  // dqkv
        for (int e = tid; e < JD; e += 256) {
            const int n = e / dh, c = e - n * dh;  // n: a query row (dq) and a key / value row (dk, dv)
            float dq = 0.f, dk = 0.f, dv = 0.f;
            for (int j = 0; j < J; ++j) {
                dq = fmaf(sS[n * JP + j], sk[j * DP + c], dq);  // sum_j dS[n][j] k[j][c]
                dk = fmaf(sS[j * JP + n], sq[j * DP + c], dk);  // sum_m dS[m][n] (q scale)[m][c]
                dv = fmaf(sP[j * JP + n], sO[j * DP + c], dv);  // sum_m P[m][n] dO[m][c]
            }
            float* r = g + (int64_t)n * 3 * hid + c;
            r[0] = dq * scale;
            r[hid] = dk;
            r[2 * hid] = dv;
        }
    }
}

size_t attn_train_lds(int J, int dh, bool bwd) {
    const size_t f = (size_t)3 * J * (dh + 1) + (size_t)J * (J + 1);
    return (bwd ? f + (size_t)J * (dh + 1) + (size_t)J * (J + 1) : f) * sizeof(float);
}

// ---- FiLM + tanh of a ResnetBlock's first Block (attention.py:67-75 under autograd) -----------
// out[b, j, c] = tanh(y[b, j, c] * (ss[b, c] + 1) + ss[b, C + c]), ss = the time MLP's (B, 2C)
// output (scale | shift, broadcast over the J nodes); the multiply and add rounded separately, as
// torch evaluates x * (scale + 1) + shift.  Backward: dpre = dout (1 - out^2),
// dy = dpre (scale + 1), dscale[b, c] = sum_j dpre y, dshift[b, c] = sum_j dpre (j in order).
__global__ __launch_bounds__(256) void k_film_tanh(const float* __restrict__ y, const float* __restrict__ ss,
                                                    float* __restrict__ out, int64_t n, int J, int C) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    const int c = (int)(e % C);
    const int64_t b = e / ((int64_t)J * C);
    const float sc = __fadd_rn(ss[b * 2 * C + c], 1.0f);
    out[e] = tanhf(__fadd_rn(__fmul_rn(y[e], sc), ss[b * 2 * C + C + c]));
}

__global__ __launch_bounds__(256) void k_film_tanh_bwd(const float* __restrict__ y, const float* __restrict__ ss,
                                                        const float* __restrict__ out, const float* __restrict__ dout,
                                                        float* __restrict__ dy, float* __restrict__ dss, int J, int C) {
    const int64_t b = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const float sc = __fadd_rn(ss[b * 2 * C + c], 1.0f);
    float gs = 0.f, gh = 0.f;
    for (int j = 0; j < J; ++j) {
        const int64_t o = (b * J + j) * (int64_t)C + c;
        const float t = out[o];
        const float dp = dout[o] * (1.0f - t * t);
        dy[o] = dp * sc;
        gs += dp * y[o];
        gh += dp;
    }
    dss[b * 2 * C + c] = gs;
    dss[b * 2 * C + C + c] = gh;
}

// ---- Ghat = G / max(rowsum|G|, eps) of a learnable influence matrix (graph_structural.py:107,
// F.normalize(G, p=1, dim=1)) ---------------------------------------------------------------------
// One workgroup of 64 threads: thread i owns row i (J <= 64, a J x J matrix is at most 16 KB and
// L2-resident).  Backward, with d_i = max(n_i, eps):
//   dG[i][j] = dGhat[i][j] / d_i - [n_i >= eps] sign(G[i][j]) (sum_k dGhat[i][k] G[i][k]) / d_i^2
// blockIdx.x = the matrix of a batch of `count` contiguous J x J matrices (every learnable G of a
// Denoiser in one launch each way).
__global__ __launch_bounds__(64) void k_l1norm_rows(const float* __restrict__ G, const float* __restrict__ dout,
                                                    float* __restrict__ out, int J, float eps, int bwd) {
    const int i = threadIdx.x;
    if (i >= J) return;
    const int64_t mat = (int64_t)blockIdx.x * J * J;
    G += mat;
    out += mat;
    if (bwd) dout += mat;
    const float* g = G + (int64_t)i * J;
    float n = 0.f;
    for (int j = 0; j < J; ++j) n += fabsf(g[j]);
    const float d = fmaxf(n, eps);
    float* o = out + (int64_t)i * J;
    if (!bwd) {
        for (int j = 0; j < J; ++j) o[j] = g[j] / d;
        return;
    }
    const float* dg = dout + (int64_t)i * J;
    float dot = 0.f;
    for (int j = 0; j < J; ++j) dot = fmaf(dg[j], g[j], dot);
    const float c = n >= eps ? dot / (d * d) : 0.f;
    for (int j = 0; j < J; ++j) {
        const float sg = g[j] > 0.f ? 1.f : (g[j] < 0.f ? -1.f : 0.f);
        o[j] = dg[j] / d - sg * c;
    }
}

// ---- RMSNorm of PreNorm (attention.py:30-36): out = (x / max(||x||, 1e-12)) g sqrt(C) ---------
// x (R, C) with R = rows x J vectors of C features; one wave per vector, kRmsRows vectors per
// workgroup.  The forward saves d = max(||x||, eps) per vector.  Backward, v = dy g s:
//   dx = v / d - [n >= eps] x (sum_c v_c x_c) / (d^2 n),    dg[c] = sum_vectors dy_c s x_c / d
// dg leaves as one partial per workgroup (waves summed in order), summed by sum_parts in order.
constexpr int kRmsRows = 16;  // 4 vectors per wave (64 per workgroup: 31.6 / 45.2 us fwd / bwd at 16,384 x 192)
constexpr int kRmsMaxC = 1024;

__device__ __forceinline__ float wave_sum(float v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <bool BWD>
__global__ __launch_bounds__(256) void k_rmsnorm(const float* __restrict__ x, const float* __restrict__ g,
                                                 const float* __restrict__ dy, float* __restrict__ out,
                                                 float* __restrict__ dnorm, float* __restrict__ dg_part, int64_t R,
                                                 int C, float s, float eps) {
    __shared__ float acc[BWD ? 4 * kRmsMaxC : 1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.x * kRmsRows;
    if constexpr (BWD) {
        for (int c = threadIdx.x; c < 4 * C; c += 256) acc[c] = 0.f;
        __syncthreads();
    }
#pragma unroll
    for (int q = w; q < kRmsRows; q += 4) {
        const int64_t r = r0 + q;
        if (r >= R) break;
        const float* xr = x + r * C;
        if constexpr (!BWD) {
            float ss = 0.f;
            for (int c = lane; c < C; c += 64) ss = fmaf(xr[c], xr[c], ss);
            const float n = sqrtf(wave_sum(ss));
            const float d = fmaxf(n, eps);
            for (int c = lane; c < C; c += 64) out[r * C + c] = (xr[c] / d) * g[c] * s;
            if (lane == 0) dnorm[r] = d;
        } else {
            const float* dr = dy + r * C;
            const float d = dnorm[r];
            float ss = 0.f, dot = 0.f;
            for (int c = lane; c < C; c += 64) {
                ss = fmaf(xr[c], xr[c], ss);
                dot = fmaf(dr[c] * g[c] * s, xr[c], dot);
            }
            const float n = sqrtf(wave_sum(ss));
            dot = wave_sum(dot);
            const float k = n >= eps ? dot / (d * d * n) : 0.f;
            for (int c = lane; c < C; c += 64) {
                const float v = dr[c] * g[c] * s;
                out[r * C + c] = v / d - xr[c] * k;
                acc[w * C + c] += dr[c] * s * (xr[c] / d);
            }
        }
    }
    if constexpr (BWD) {
        __syncthreads();
        for (int c = threadIdx.x; c < C; c += 256)
            dg_part[(int64_t)blockIdx.x * C + c] = ((acc[c] + acc[C + c]) + acc[2 * C + c]) + acc[3 * C + c];
    }
}

// ---- Mahalanobis loss of NonisotropicGaussianDiffusion (nonisotropic.py:177-190 + the
// 'b ... -> b' mean of base.py:298) ------------------------------------------------------------------
// Per row r: D = sgn (model_out - target) (J x F), M = S[t_r] D with S = mahalanobis_S_sqrt_recip
// (T, J, J); loss[r] = mean_{i,f} |M| (l1) or M^2 (mse).  One workgroup per row; D and S[t_r]
// staged in LDS, M in LDS, sums in a fixed order.  Backward recomputes M:
//   dM = (l1: sign(M), mse: 2M) * (dloss[r] / (J F)),   d model_out = sgn S^T dM.
template <bool BWD>
__global__ __launch_bounds__(256) void k_mahalanobis(const float* __restrict__ mo, const float* __restrict__ tg,
                                                     const float* __restrict__ S, const int64_t* __restrict__ t, int T,
                                                     const float* __restrict__ dloss, float* __restrict__ out, int J,
                                                     int F, float sgn, int mse) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int64_t r = blockIdx.x;
    const int JF = J * F;
    float* sD = sm;              // [J][F]
    float* sM = sD + JF;         // [J][F]
    float* sS = sM + JF;         // [J][J]
    float* red = sS + J * J;     // [256]
    const float* m = mo + r * JF;
    const float* tt = tg + r * JF;
    // a timestep outside [0, T) reads no table: its row's loss (or gradient) is NaN
    const int64_t tr = t[r];
    const bool tok = tr >= 0 && tr < T;
    const float* St = S + (tok ? tr : 0) * (int64_t)J * J;
    const float bad = tok ? 0.f : __builtin_nanf("");
    for (int e = threadIdx.x; e < JF; e += 256) sD[e] = sgn * (m[e] - tt[e]) + bad;
    for (int e = threadIdx.x; e < J * J; e += 256) sS[e] = St[e];
    __syncthreads();
    float part = 0.f;
    for (int e = threadIdx.x; e < JF; e += 256) {
        const int i = e / F, f = e - i * F;
        float a = 0.f;
        for (int j = 0; j < J; ++j) a = fmaf(sS[i * J + j], sD[j * F + f], a);
        sM[e] = a;
        part += mse ? a * a : fabsf(a);
    }
    if constexpr (!BWD) {
        red[threadIdx.x] = part;
        __syncthreads();
        if (threadIdx.x < 64) {
            const float v = ((red[threadIdx.x] + red[threadIdx.x + 64]) + red[threadIdx.x + 128]) + red[threadIdx.x + 192];
            const float tot = wave_sum(v);
            if (threadIdx.x == 0) out[r] = tot / (float)JF;
        }
    } else {
        __syncthreads();
        const float w = dloss[r] / (float)JF;
        for (int e = threadIdx.x; e < JF; e += 256) {
            const float a = sM[e];
            sM[e] = (mse ? 2.f * a : (a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f))) * w;
        }
        __syncthreads();
        float* o = out + r * JF;
        for (int e = threadIdx.x; e < JF; e += 256) {
            const int j = e / F, f = e - j * F;
            float a = 0.f;
            for (int i = 0; i < J; ++i) a = fmaf(sS[i * J + j], sM[i * F + f], a);
            o[e] = sgn * a + bad;  // an out-of-range timestep: NaN (sign(NaN) above gave 0)
        }
    }
}

size_t mahalanobis_lds(int J, int F) { return ((size_t)2 * J * F + (size_t)J * J + 256) * sizeof(float); }
}  // namespace
}  // namespace sd

using sd::GemmArgs;

#define TR_HIP(x)                                                                                     \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) return sd::set_error(SD_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" {

size_t sd_gl_train_workspace_bytes(int64_t rows, int32_t J, int32_t K, int32_t N, int32_t n_types) {
    if (rows < 0 || J < 1 || K < 1 || N < 1) return 0;
    const int types = n_types < 1 ? 1 : n_types;
    const int64_t s = sd::splits_for(rows);
    const int64_t chunks = sd::ceil_div(rows, sd::kRowsPerChunk);
    const int64_t gchunks = sd::ceil_div(rows, sd::kDghatRows);
    int64_t part = s * types * (int64_t)N * K;                    // dW partials
    part = part > gchunks * (int64_t)J * J ? part : gchunks * (int64_t)J * J;   // dghat partials
    part = part > chunks * (int64_t)types * N ? part : chunks * (int64_t)types * N;  // dbias partials
    return (size_t)(rows * J * (int64_t)N + part) * sizeof(float);
}

int sd_gl_train_forward(const float* x, const float* W, const float* bias, const int64_t* node_types,
                        int32_t n_types, const float* ghat, int64_t rows, int32_t J, int32_t K, int32_t N,
                        float* z, float* y, void* stream) {
    if (rows < 0 || J < 1 || J > 64 || K < 1 || N < 1 || n_types < 0)
        return sd::set_error(SD_E_INVALID, "gl_train_forward: need rows >= 0, 1 <= J <= 64, K, N >= 1");
    if (rows == 0) return SD_OK;
    if (!x || !W || !ghat || !z || !y) return sd::set_error(SD_E_INVALID, "gl_train_forward: null buffer");
    if (n_types > 0 && !node_types) return sd::set_error(SD_E_INVALID, "gl_train_forward: node_types missing");
    if (rows > INT32_MAX / 2) return sd::set_error(SD_E_INVALID, "gl_train_forward: too many rows");
    hipStream_t s = (hipStream_t)stream;
    GemmArgs g{};
    g.A = x; g.B = W; g.C = z; g.bias = bias; g.types = n_types > 0 ? node_types : nullptr;
    g.M = (int)rows; g.N = N; g.K = K; g.J = J; g.by_type = 0; g.splits = 1; g.kchunk = K;
    g.am = (int64_t)J * K; g.ak = 1; g.aj = K; g.at = 0;            // A[m][k] = x[m, j, k]
    g.bk = 1; g.bn = K; g.bj = 0; g.bt = (int64_t)N * K;            // B[k][n] = W[t][n][k]
    g.cm = (int64_t)J * N; g.cz = N; g.cs = 0; g.bias_t = N;        // C[m][n] = z[m, j, n]
    TR_HIP(sd::launch_gemm(g, dim3((unsigned)sd::ceil_div(N, sd::TN), (unsigned)sd::ceil_div(rows, sd::TM), J), s));
    TR_HIP(sd::launch_mix(z, ghat, y, rows, J, N, 0, s));
    return SD_OK;
}

int sd_gl_train_backward(const float* x, const float* z, const float* dy, const float* W, const int64_t* node_types,
                         int32_t n_types, const float* ghat, int64_t rows, int32_t J, int32_t K, int32_t N, float* dx,
                         float* dW, float* dbias, float* dghat, void* workspace, size_t workspace_bytes,
                         void* stream) {
    if (rows < 0 || J < 1 || J > 64 || K < 1 || N < 1 || n_types < 0)
        return sd::set_error(SD_E_INVALID, "gl_train_backward: need rows >= 0, 1 <= J <= 64, K, N >= 1");
    if (rows > INT32_MAX / 2) return sd::set_error(SD_E_INVALID, "gl_train_backward: too many rows");
    const int types = n_types > 0 ? n_types : 1;
    const int64_t* tp = n_types > 0 ? node_types : nullptr;
    if (n_types > 0 && !node_types) return sd::set_error(SD_E_INVALID, "gl_train_backward: node_types missing");
    hipStream_t s = (hipStream_t)stream;
    if (rows == 0) {  // empty batch: zero parameter gradients
        if (dW) TR_HIP(hipMemsetAsync(dW, 0, (size_t)types * N * K * sizeof(float), s));
        if (dbias) TR_HIP(hipMemsetAsync(dbias, 0, (size_t)types * N * sizeof(float), s));
        if (dghat) TR_HIP(hipMemsetAsync(dghat, 0, (size_t)J * J * sizeof(float), s));
        return SD_OK;
    }
    if (!x || !z || !dy || !W || !ghat) return sd::set_error(SD_E_INVALID, "gl_train_backward: null input");
    if (!workspace || workspace_bytes < sd_gl_train_workspace_bytes(rows, J, K, N, n_types))
        return sd::set_error(SD_E_INVALID, "gl_train_backward: workspace too small");
    float* dz = (float*)workspace;
    float* part = dz + rows * J * (int64_t)N;

    // dghat first (reads dy and z, independent of dz)
    if (dghat) {
        const int64_t chunks = sd::ceil_div(rows, sd::kDghatRows);
        if (J <= 16 && (N & 3) == 0)
            hipLaunchKernelGGL(sd::k_dghat_part16, dim3((unsigned)chunks), dim3(256), 0, s, dy, z, part, rows, J, N,
                               sd::kDghatRows);
        else if (J <= 32)
            hipLaunchKernelGGL(sd::k_dghat_part<1>, dim3((unsigned)chunks), dim3(256), 0, s, dy, z, part, rows, J, N,
                               sd::kDghatRows);
        else
            hipLaunchKernelGGL(sd::k_dghat_part<2>, dim3((unsigned)chunks), dim3(256), 0, s, dy, z, part, rows, J, N,
                               sd::kDghatRows);
        TR_HIP(hipGetLastError());
        TR_HIP(sd::sum_parts(part, (int)chunks, (int64_t)J * J, dghat, s));
    }
    if (!dx && !dW && !dbias) return SD_OK;
    TR_HIP(sd::launch_mix(dy, ghat, dz, rows, J, N, 1, s));
    if (dx) {
        GemmArgs g{};
        g.A = dz; g.B = W; g.C = dx; g.bias = nullptr; g.types = tp;
        g.M = (int)rows; g.N = K; g.K = N; g.J = J; g.by_type = 0; g.splits = 1; g.kchunk = N;
        g.am = (int64_t)J * N; g.ak = 1; g.aj = N; g.at = 0;         // A[m][n] = dz[m, j, n]
        g.bk = K; g.bn = 1; g.bj = 0; g.bt = (int64_t)N * K;         // B[n][k] = W[t][n][k]
        g.cm = (int64_t)J * K; g.cz = K; g.cs = 0;                   // C[m][k] = dx[m, j, k]
        TR_HIP(sd::launch_gemm(g, dim3((unsigned)sd::ceil_div(K, sd::TN), (unsigned)sd::ceil_div(rows, sd::TM), J), s));
    }
    if (dW) {
        const int splits = sd::splits_for(rows);
        const int kchunk = (int)sd::ceil_div(sd::ceil_div(rows, splits), sd::TK) * sd::TK;
        GemmArgs g{};
        g.A = dz; g.B = x; g.C = part; g.bias = nullptr; g.types = tp;
        g.M = N; g.N = K; g.K = (int)rows; g.J = J; g.by_type = 1; g.splits = splits; g.kchunk = kchunk;
        g.am = 1; g.ak = (int64_t)J * N; g.aj = N; g.at = 0;         // A[n][r] = dz[r, j, n]
        g.bk = (int64_t)J * K; g.bn = 1; g.bj = K; g.bt = 0;         // B[r][k] = x[r, j, k]
        g.cm = K; g.cz = (int64_t)N * K; g.cs = (int64_t)types * N * K;  // C[n][k] = part[s][t][n][k]
        TR_HIP(sd::launch_gemm(
            g, dim3((unsigned)sd::ceil_div(K, sd::TN), (unsigned)sd::ceil_div(N, sd::TM), types * splits), s));
        const int64_t n = (int64_t)types * N * K;
        TR_HIP(sd::sum_parts(part, splits, n, dW, s));
    }
    if (dbias) {
        const int64_t chunks = sd::ceil_div(rows, sd::kRowsPerChunk);
        hipLaunchKernelGGL(sd::k_dbias_part, dim3((unsigned)sd::ceil_div(N, 256), types, (unsigned)chunks), dim3(256), 0,
                           s, dz, tp, part, rows, J, N, types, sd::kRowsPerChunk);
        TR_HIP(hipGetLastError());
        const int64_t n = (int64_t)types * N;
        TR_HIP(sd::sum_parts(part, (int)chunks, n, dbias, s));
    }
    return SD_OK;
}

int sd_attn_train_forward(const float* qkv, float* out, int64_t rows, int32_t J, int32_t heads, int32_t dim_head,
                          float scale, void* stream) {
    if (rows < 0 || J < 1 || J > 64 || heads < 1 || dim_head < 1 || dim_head > 64)
        return sd::set_error(SD_E_INVALID, "sd_attn_train_forward: 1 <= J <= 64, 1 <= dim_head <= 64");
    if (rows == 0) return SD_OK;
    if (!qkv || !out) return sd::set_error(SD_E_INVALID, "sd_attn_train_forward: null buffer");
    if (rows * heads > 0x7fffffffLL) return sd::set_error(SD_E_INVALID, "sd_attn_train_forward: too many rows");
    const size_t lds = sd::attn_train_lds(J, dim_head, false);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)sd::k_attn_train<false>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return sd::set_error(SD_E_HIP, std::string("k_attn_train: ") + hipGetErrorString(e));
    }
    hipLaunchKernelGGL(sd::k_attn_train<false>, dim3((unsigned)(rows * heads)), dim3(256), lds, (hipStream_t)stream,
                       qkv, (const float*)nullptr, out, J, heads, dim_head, scale);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_attn_train: ") + hipGetErrorString(e));
}

int sd_attn_train_backward(const float* qkv, const float* dout, float* dqkv, int64_t rows, int32_t J, int32_t heads,
                           int32_t dim_head, float scale, void* stream) {
    if (rows < 0 || J < 1 || J > 64 || heads < 1 || dim_head < 1 || dim_head > 64)
        return sd::set_error(SD_E_INVALID, "sd_attn_train_backward: 1 <= J <= 64, 1 <= dim_head <= 64");
    if (rows == 0) return SD_OK;
    if (!qkv || !dout || !dqkv) return sd::set_error(SD_E_INVALID, "sd_attn_train_backward: null buffer");
    if (rows * heads > 0x7fffffffLL) return sd::set_error(SD_E_INVALID, "sd_attn_train_backward: too many rows");
    const size_t lds = sd::attn_train_lds(J, dim_head, true);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)sd::k_attn_train<true>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return sd::set_error(SD_E_HIP, std::string("k_attn_train: ") + hipGetErrorString(e));
    }
    hipLaunchKernelGGL(sd::k_attn_train<true>, dim3((unsigned)(rows * heads)), dim3(256), lds, (hipStream_t)stream,
                       qkv, dout, dqkv, J, heads, dim_head, scale);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_attn_train: ") + hipGetErrorString(e));
}

int sd_film_tanh_forward(const float* y, const float* ss, float* out, int64_t rows, int32_t J, int32_t C, void* stream) {
    if (rows < 0 || J < 1 || C < 1) return sd::set_error(SD_E_INVALID, "sd_film_tanh_forward: bad shape");
    if (rows == 0) return SD_OK;
    if (!y || !ss || !out) return sd::set_error(SD_E_INVALID, "sd_film_tanh_forward: null buffer");
    const int64_t n = rows * J * (int64_t)C;
    hipLaunchKernelGGL(sd::k_film_tanh, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, y, ss, out,
                       n, J, C);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_film_tanh: ") + hipGetErrorString(e));
}

int sd_film_tanh_backward(const float* y, const float* ss, const float* out, const float* dout, float* dy, float* dss,
                          int64_t rows, int32_t J, int32_t C, void* stream) {
    if (rows < 0 || J < 1 || C < 1 || rows > 65535) return sd::set_error(SD_E_INVALID, "sd_film_tanh_backward: bad shape");
    if (rows == 0) return SD_OK;
    if (!y || !ss || !out || !dout || !dy || !dss) return sd::set_error(SD_E_INVALID, "sd_film_tanh_backward: null buffer");
    hipLaunchKernelGGL(sd::k_film_tanh_bwd, dim3((unsigned)((C + 255) / 256), (unsigned)rows), dim3(256), 0,
                       (hipStream_t)stream, y, ss, out, dout, dy, dss, J, C);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_film_tanh_bwd: ") + hipGetErrorString(e));
}

int sd_l1norm_rows_forward(const float* G, float* ghat, int32_t J, int32_t count, float eps, void* stream) {
    if (J < 1 || J > 64 || count < 0) return sd::set_error(SD_E_INVALID, "sd_l1norm_rows_forward: 1 <= J <= 64, count >= 0");
    if (count == 0) return SD_OK;
    if (!G || !ghat) return sd::set_error(SD_E_INVALID, "sd_l1norm_rows_forward: null buffer");
    hipLaunchKernelGGL(sd::k_l1norm_rows, dim3((unsigned)count), dim3(64), 0, (hipStream_t)stream, G,
                       (const float*)nullptr, ghat, J, eps, 0);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_l1norm_rows: ") + hipGetErrorString(e));
}

int sd_l1norm_rows_backward(const float* G, const float* dghat, float* dG, int32_t J, int32_t count, float eps,
                            void* stream) {
    if (J < 1 || J > 64 || count < 0) return sd::set_error(SD_E_INVALID, "sd_l1norm_rows_backward: 1 <= J <= 64, count >= 0");
    if (count == 0) return SD_OK;
    if (!G || !dghat || !dG) return sd::set_error(SD_E_INVALID, "sd_l1norm_rows_backward: null buffer");
    hipLaunchKernelGGL(sd::k_l1norm_rows, dim3((unsigned)count), dim3(64), 0, (hipStream_t)stream, G, dghat, dG, J, eps,
                       1);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_l1norm_rows: ") + hipGetErrorString(e));
}

size_t sd_rmsnorm_workspace_bytes(int64_t R, int32_t C) {
    if (R < 0 || C < 1) return 0;
    return (size_t)sd::ceil_div(R, sd::kRmsRows) * C * sizeof(float);
}

int sd_rmsnorm_forward(const float* x, const float* g, float* out, float* dnorm, int64_t R, int32_t C, float scale,
                       float eps, void* stream) {
    if (R < 0 || C < 1 || C > sd::kRmsMaxC) return sd::set_error(SD_E_INVALID, "sd_rmsnorm_forward: 1 <= C <= 1024");
    if (R == 0) return SD_OK;
    if (!x || !g || !out || !dnorm) return sd::set_error(SD_E_INVALID, "sd_rmsnorm_forward: null buffer");
    if (sd::ceil_div(R, sd::kRmsRows) > 0x7fffffffLL) return sd::set_error(SD_E_INVALID, "sd_rmsnorm_forward: too many rows");
    hipLaunchKernelGGL(sd::k_rmsnorm<false>, dim3((unsigned)sd::ceil_div(R, sd::kRmsRows)), dim3(256), 0,
                       (hipStream_t)stream, x, g, (const float*)nullptr, out, dnorm, (float*)nullptr, R, C, scale, eps);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_rmsnorm: ") + hipGetErrorString(e));
}

int sd_rmsnorm_backward(const float* x, const float* g, const float* dnorm, const float* dy, float* dx, float* dg,
                        int64_t R, int32_t C, float scale, float eps, void* workspace, size_t workspace_bytes,
                        void* stream) {
    if (R < 0 || C < 1 || C > sd::kRmsMaxC) return sd::set_error(SD_E_INVALID, "sd_rmsnorm_backward: 1 <= C <= 1024");
    hipStream_t s = (hipStream_t)stream;
    if (R == 0) {
        if (dg) TR_HIP(hipMemsetAsync(dg, 0, (size_t)C * sizeof(float), s));
        return SD_OK;
    }
    if (!x || !g || !dnorm || !dy || !dx || !dg) return sd::set_error(SD_E_INVALID, "sd_rmsnorm_backward: null buffer");
    if (!workspace || workspace_bytes < sd_rmsnorm_workspace_bytes(R, C))
        return sd::set_error(SD_E_INVALID, "sd_rmsnorm_backward: workspace too small");
    const int64_t blocks = sd::ceil_div(R, sd::kRmsRows);
    if (blocks > 0x7fffffffLL) return sd::set_error(SD_E_INVALID, "sd_rmsnorm_backward: too many rows");
    float* part = (float*)workspace;
    hipLaunchKernelGGL(sd::k_rmsnorm<true>, dim3((unsigned)blocks), dim3(256), 0, s, x, g, dy, dx, (float*)dnorm, part, R,
                       C, scale, eps);
    TR_HIP(hipGetLastError());
    TR_HIP(sd::sum_parts(part, (int)blocks, C, dg, s));
    return SD_OK;
}

int sd_mahalanobis_loss_forward(const float* model_out, const float* target, const float* S, const int64_t* t,
                                int32_t T, int64_t rows, int32_t J, int32_t F, int32_t pred_noise, int32_t mse, float* loss,
                                void* stream) {
    if (rows < 0 || J < 1 || J > 64 || F < 1 || F > 256 || T < 1)
        return sd::set_error(SD_E_INVALID, "sd_mahalanobis_loss_forward: 1 <= J <= 64, 1 <= F <= 256, T >= 1");
    if (rows == 0) return SD_OK;
    if (!model_out || !target || !S || !t || !loss)
        return sd::set_error(SD_E_INVALID, "sd_mahalanobis_loss_forward: null buffer");
    if (rows > 0x7fffffffLL) return sd::set_error(SD_E_INVALID, "sd_mahalanobis_loss_forward: too many rows");
    const size_t lds = sd::mahalanobis_lds(J, F);
    if (lds > 64 * 1024)
        TR_HIP(hipFuncSetAttribute((const void*)sd::k_mahalanobis<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds));
    hipLaunchKernelGGL(sd::k_mahalanobis<false>, dim3((unsigned)rows), dim3(256), lds, (hipStream_t)stream, model_out,
                       target, S, t, T, (const float*)nullptr, loss, J, F, pred_noise ? -1.f : 1.f, mse);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_mahalanobis: ") + hipGetErrorString(e));
}

int sd_mahalanobis_loss_backward(const float* model_out, const float* target, const float* S, const int64_t* t,
                                 int32_t T, const float* dloss, int64_t rows, int32_t J, int32_t F, int32_t pred_noise,
                                 int32_t mse, float* dmodel_out, void* stream) {
    if (rows < 0 || J < 1 || J > 64 || F < 1 || F > 256 || T < 1)
        return sd::set_error(SD_E_INVALID, "sd_mahalanobis_loss_backward: 1 <= J <= 64, 1 <= F <= 256, T >= 1");
    if (rows == 0) return SD_OK;
    if (!model_out || !target || !S || !t || !dloss || !dmodel_out)
        return sd::set_error(SD_E_INVALID, "sd_mahalanobis_loss_backward: null buffer");
    if (rows > 0x7fffffffLL) return sd::set_error(SD_E_INVALID, "sd_mahalanobis_loss_backward: too many rows");
    const size_t lds = sd::mahalanobis_lds(J, F);
    if (lds > 64 * 1024)
        TR_HIP(hipFuncSetAttribute((const void*)sd::k_mahalanobis<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds));
    hipLaunchKernelGGL(sd::k_mahalanobis<true>, dim3((unsigned)rows), dim3(256), lds, (hipStream_t)stream, model_out,
                       target, S, t, T, dloss, dmodel_out, J, F, pred_noise ? -1.f : 1.f, mse);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SD_OK : sd::set_error(SD_E_HIP, std::string("k_mahalanobis: ") + hipGetErrorString(e));
}

}  // extern "C"
