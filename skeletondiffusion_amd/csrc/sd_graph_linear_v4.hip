// k_gl4: StaticGraphLinear (graph_structural.py:30-43) + fused epilogue on f16 MFMA with
// f32-accurate split products.
//
// gfx950 runs f32-input MFMA at 1/16 of the f16 rate (MI355X_MICROARCH.md: 157 vs 2,500 TF/s).
// v4 keeps f32 accuracy by splitting both operands into two f16 terms and summing three
// products in the f32 accumulator:
//     W' = W * 2^sW  (sW per layer: max|W'| < 2^15),  W'_hi = f16(W'),  W'_lo = f16(W' - W'_hi)
//     x_hi = f16(x),  x_lo = f16(x - x_hi)
//     y = 2^-sW * (x_hi W'_hi + x_hi W'_lo + x_lo W'_hi)          (all products exact in f32)
// Each operand keeps ~22 significant bits; the dropped x_lo W'_lo term is ~2^-22 relative and an
// f16-subnormal x_lo costs at most 2^-25 absolute per element.  tools/sim_split_f16.py measures
// the end-to-end effect on T=100 chains: within the f32-vs-f64 drift of the exact path
// (|split - f64| <= |f32 - f64|, ~1e-7, against the 1e-4 parity bar).
//
// Schedule (one workgroup = RT*32 rows x CT*32 output columns x all J nodes):
//   * NW waves; wave w owns nodes w, w+NW, ...; per node an RT x CT grid of 32x32 f32
//     accumulators on v_mfma_f32_32x32x16_f16 (3 MFMAs per 16-deep k step and tile);
//   * weights: pre-split at plan finalize into the exact B-fragment order
//     [type][k16 chunk][32-col tile][hi|lo][lane][8], so a chunk's slice for the workgroup's
//     columns is one contiguous span per type, streamed into LDS by LDS-DMA (16 B per lane,
//     double-buffered) and read back with conflict-free ds_read_b128 (lane l -> l*16 B);
//   * x: each lane streams 8 contiguous k of one row per node (2 float4) a chunk ahead and
//     splits them in registers (the activations stay f32 in HBM);
//   * epilogue as v3: scale/RMS/bias in the accumulator layout, Y through LDS in 16-row slabs,
//     G-hat mixing on 16x16x4 f32 MFMA, FiLM / tanh / residual / store.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <cmath>

#include "sd_internal.h"

namespace sd {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

namespace {

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
struct VmCnt4 {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    static constexpr int imm = (N & 0xF) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14);
};

__device__ __forceinline__ floatx4 g4(const float* p) { return *reinterpret_cast<const floatx4*>(p); }

// tanh(x) = 1 - 2 / (exp(2x) + 1) on v_exp_f32 + v_rcp_f32 (no IEEE division sequence):
// saturates cleanly at +-1, within ~3e-7 absolute of tanhf
__device__ __forceinline__ float tanh4(float x) {
    const float e = __builtin_amdgcn_exp2f(2.0f * 1.44269504088896341f * x);
    return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}

// Row-blocked activation layout of the v4 path: rows in blocks of 32; per (block, node) the F
// features as [F/8][2][32 rows][4], i.e. one aligned 16-B piece per (row, 4 features).  An x
// fragment load (32 rows x 8 features of one node) is then 2 x 512 contiguous bytes and an
// output quad one 16-B store.  Buffers are padded to a multiple of 32 rows.
__device__ __forceinline__ int64_t blk_off(int64_t row, int node, int f, int J, int F) {
    return ((((row >> 5) * J + node) * (int64_t)F) << 5) + ((f >> 3) << 8) + (((f >> 2) & 1) << 7) +
           ((row & 31) << 2) + (f & 3);
}

// ---- one-time weight preparation ------------------------------------------------------------

__global__ void k_absmax(const float* __restrict__ w, int64_t n, unsigned* __restrict__ out) {
    unsigned m = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = max(m, __float_as_uint(fabsf(w[i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

// out[type][c][ct][hl][lane][e] = split(W[type][32ct + (lane&31)][16c + 8(lane>>5) + e] * scale)
__global__ void k_split_w(const float* __restrict__ W, int ntypes, int N, int K, int nct, float scale,
                          _Float16* __restrict__ out) {
    const int nchunk = K >> 4;
    const int64_t total = (int64_t)ntypes * nchunk * nct * 64;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(g & 63);
        int64_t r = g >> 6;
        const int ct = (int)(r % nct);
        r /= nct;
        const int c = (int)(r % nchunk);
        const int t = (int)(r / nchunk);
        const int n = 32 * ct + (lane & 31);
        const int k0 = 16 * c + 8 * (lane >> 5);
        _Float16* hi = out + ((((int64_t)t * nchunk + c) * nct + ct) * 2) * 512 + lane * 8;
        _Float16* lo = hi + 512;
        for (int e = 0; e < 8; ++e) {
            const float v = n < N ? W[((int64_t)t * N + n) * K + k0 + e] * scale : 0.f;
            const _Float16 h = (_Float16)v;
            hi[e] = h;
            lo[e] = (_Float16)(v - (float)h);
        }
    }
}

// bf16 copy in the B-fragment layout of k_split_w: hi slots = bf16(W) (RNE), lo slots zero
__global__ void k_bf16_w(const float* __restrict__ W, int ntypes, int N, int K, int nct, __bf16* __restrict__ out) {
    const int nchunk = K >> 4;
    const int64_t total = (int64_t)ntypes * nchunk * nct * 64;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
        const int lane = (int)(g & 63);
        int64_t r = g >> 6;
        const int ct = (int)(r % nct);
        r /= nct;
        const int c = (int)(r % nchunk);
        const int t = (int)(r / nchunk);
        const int n = 32 * ct + (lane & 31);
        const int k0 = 16 * c + 8 * (lane >> 5);
        __bf16* hi = out + ((((int64_t)t * nchunk + c) * nct + ct) * 2) * 512 + lane * 8;
        __bf16* lo = hi + 512;
        for (int e = 0; e < 8; ++e) {
            hi[e] = (__bf16)(n < N ? W[((int64_t)t * N + n) * K + k0 + e] : 0.f);
            lo[e] = (__bf16)0.f;
        }
    }
}

}  // namespace

// row-blocked (blk_off) -> row-major (rows, J, F) copy (sd_denoiser_trace)
__global__ void k_unblock(float* __restrict__ out, const float* __restrict__ in, int64_t rows, int J, int F) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n4 = rows * J * (F / 4);
    if (g >= n4) return;
    const int f = (int)(g % (F / 4)) * 4;
    const int64_t rj = g / (F / 4);
    const int j = (int)(rj % J);
    const int64_t row = rj / J;
    *reinterpret_cast<floatx4*>(out + (row * J + j) * F + f) = *reinterpret_cast<const floatx4*>(in + blk_off(row, j, f, J, F));
}

hipError_t launch_unblock(float* out, const float* in, int64_t rows, int J, int F, hipStream_t s) {
    const int64_t n4 = rows * J * (F / 4);
    if (n4 <= 0) return hipSuccess;
    if (F % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_unblock, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, out, in, rows, J, F);
    return hipGetLastError();
}

hipError_t make_bf16_weights(const float* W, int ntypes, int N, int K, SplitW* out, hipStream_t s) {
    out->nct = ((N + 31) / 32 + 5) / 6 * 6;
    out->scale = out->unscale = 1.0f;
    const size_t halves = (size_t)ntypes * (K / 16) * out->nct * 1024;
    hipError_t e = hipMalloc(&out->w, halves * sizeof(_Float16));
    if (e != hipSuccess) return e;
    const int64_t total = (int64_t)ntypes * (K / 16) * out->nct * 64;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_bf16_w, dim3(blocks), dim3(256), 0, s, W, ntypes, N, K, out->nct,
                       reinterpret_cast<__bf16*>(out->w));
    return hipGetLastError();
}

hipError_t make_split_weights(const float* W, int ntypes, int N, int K, SplitW* out, hipStream_t s) {
    out->nct = ((N + 31) / 32 + 5) / 6 * 6;  // 32-col tiles, padded to a multiple of 6 (CT in 1, 2, 3)
    const int64_t n = (int64_t)ntypes * N * K;
    unsigned* dmax = nullptr;
    unsigned hmax = 0;
    hipError_t e = hipMalloc(&dmax, sizeof(unsigned));
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(dmax, 0, sizeof(unsigned), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_absmax, dim3(256), dim3(256), 0, s, W, n, dmax);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&hmax, dmax, sizeof(unsigned), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    (void)hipFree(dmax);
    const float amax = __builtin_bit_cast(float, hmax);
    int ex = 0;
    if (amax > 0.f && amax == amax && amax < 3.0e38f) (void)frexpf(amax, &ex);  // amax < 2^ex
    // W * 2^(15 - ex) < 2^15: inside f16 range, and the lo term of every weight within 2^-18
    // of the largest stays a normal f16
    out->scale = ldexpf(1.0f, 15 - ex);
    out->unscale = ldexpf(1.0f, ex - 15);
    const size_t halves = (size_t)ntypes * (K / 16) * out->nct * 1024;
    if ((e = hipMalloc(&out->w, halves * sizeof(_Float16))) != hipSuccess) return e;
    const int64_t total = (int64_t)ntypes * (K / 16) * out->nct * 64;
    const int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(k_split_w, dim3(blocks), dim3(256), 0, s, W, ntypes, N, K, out->nct, out->scale, out->w);
    return hipGetLastError();
}

// ---- split route, phase 1 (small grids) -----------------------------------------------------
// One wave per (32-row tile, node j, 32-column tile) walks the whole K extent with its x and
// weight fragments loaded straight into registers, PF chunks ahead (no LDS, no barriers), and
// stores Y = unscale * rms * acc + bias to ys[((tile * J + j) * 32 + r) * N + col].  Every
// accumulator element sees the same MFMA sequence (x_hi W'_hi, x_hi W'_lo, x_lo W'_hi per 16-deep
// chunk), RMS sum, range guard and scale arithmetic as in k_gl4, so phase 2 (k_gl4 MODE 2 / 3)
// reproduces the one-kernel results bit for bit.  Workgroup = 4 waves = 4 column tiles of one
// (row tile, node): the x fragments are shared through L1.
// Output: element (row 32 tr + r, node j, column 32 t + c) at y + tr y_ts + j y_js + t y_cs +
// r y_rs + c.  The split route's scratch p.zs is column-tiled, [tile][32-column tile][node][32
// rows][32] (y_cs = J * 1024: every (tile, column tile, node) block is 4 contiguous KiB, written
// whole by one wave and read back in 1-2 KiB runs by the mixing phase -- round 4; it was
// [tile][node][32 rows][N], 128-B runs); (ROWMAJOR, v5 for J > 21) row-major z with y_cs = 32,
// rows < B only.
struct YOut {
    float* y;
    int64_t y_rs, y_js, y_ts, y_cs;
};
// zs element (row, node j, column n) of the split route's column-tiled scratch
__device__ __forceinline__ int64_t zs_off(int64_t row, int j, int n, int J, int N) {
    return ((((row >> 5) * (N >> 5) + (n >> 5)) * J + j) << 10) + ((row & 31) << 5) + (n & 31);
}

// f16 range fallback (round 5; was a host-side re-run of the whole call): a wave whose split-f16
// operands reached |x| >= 65504 (x_hi would be inf) recomputes its 32 x 32 tile -- rows row0 ..
// row0 + 31, node j, columns col0 .. col0 + 31 -- on exact-f32 MFMA (v_mfma_f32_32x32x2_f32)
// straight from memory: the x operand as the split kernels address it (row-major with the x_cond
// row division and the tail rows clamped to row 0, or row-blocked), the plan's f32 weights p.W
// (types, N, K).  The sum is scaled by 1 / wsp_unscale (a power of two: exact), so the caller's
// epilogue (acc * unscale * rms + bias) is unchanged and the tile is f32-accurate for any finite
// input.  Taken only by the waves whose operands left the f16 range (wave-uniform ballot), so
// the in-range path keeps its arithmetic and its bitwise route equalities.
// Placement matters: run while the accumulators are live (before the epilogue), its loop raised the
// register count of every caller (k_gl4t 163 -> 235 VGPRs; the one-kernel J = 17 / 21 tiles
// spilled 4-8x more), as a call with acc live too (the live values move to callee-saved
// registers).  So the callers run it AFTER their normal stores, in a rolled loop over the tiles,
// inlined (no call frame, no scratch), and store the exact tile over the first.
__device__ __forceinline__ floatx16 exact_tile_f32_impl(const float* x1, int64_t x1_rs, int K1, int x1_div,
                                                                  int64_t x1_row0, int x1_blk, const float* x2,
                                                                  int64_t x2_rs, int K2, int x2_blk, int64_t B, int J,
                                                                  const float* W, int wrow, int N, float unscale,
                                                                  int64_t row0, int j, int col0) {
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int K = K1 + K2;
    const int col = col0 + l32;
    const float* wr = W + (int64_t)(wrow + (col < N ? col : 0)) * K + 4 * h;
    const int64_t row = row0 + l32, ac = row < B ? row : 0;
    // lane (l32, h) row `row`, features k0 + 4h .. + 3 (16-B pieces: K1, K2 multiples of 16)
    const float* xr1 = x1 + (x1_blk ? blk_off(row, j, 4 * h, J, K1) : ((ac + x1_row0) / x1_div) * x1_rs + (int64_t)j * K1 + 4 * h);
    const float* xr2 = !K2 ? xr1 : x2 + (x2_blk ? blk_off(row, j, 4 * h, J, K2) : ac * x2_rs + (int64_t)j * K2 + 4 * h);
    floatx16 c;
#pragma unroll
    for (int e = 0; e < 16; ++e) c[e] = 0.f;
#pragma nounroll
    for (int k0 = 0; k0 < K; k0 += 8) {  // A[row l32][k0 + 4h + i], B[k0 + 4h + i][col l32]
        // row-blocked: features f and f + 8 are 256 floats apart, row-major 8
        const float* xp = k0 < K1 ? xr1 + (x1_blk ? (k0 >> 3) * 256 : k0) : xr2 + (x2_blk ? ((k0 - K1) >> 3) * 256 : k0 - K1);
        const float4 xv = *reinterpret_cast<const float4*>(xp);
        float4 wv = *reinterpret_cast<const float4*>(wr + k0);
        if (col >= N) wv = float4{0.f, 0.f, 0.f, 0.f};
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(xv.x, wv.x, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(xv.y, wv.y, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(xv.z, wv.z, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(xv.w, wv.w, c, 0, 0, 0);
    }
    const float up = 1.0f / unscale;
#pragma unroll
    for (int e = 0; e < 16; ++e) c[e] *= up;
    return c;
}
__device__ __forceinline__ floatx16 exact_tile_f32(const GLArgs& p, int64_t row0, int j, int col0) {
    return exact_tile_f32_impl(p.x1, p.x1_rs, p.K1, p.x1_div, p.x1_row0, p.x1_blk, p.x2, p.x2_rs, p.K2, p.x2_blk, p.B,
                               p.J, p.W, p.wrow[j], p.N, p.wsp_unscale, row0, j, col0);
}

template <bool RMS, int PREC, bool ROWMAJOR, int PF = 8>  // PF: chunks in flight
__global__ __launch_bounds__(256) void k_gl4y(const GLArgs p, int ntile_c, int64_t ntile_r, const YOut yo) {
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    const int tc = (int)(u % ntile_c);
    const int64_t rj = u / ntile_c;
    const int J = p.J;
    const int j = (int)(rj % J);
    const int64_t tr = rj / J;
    if (tr >= ntile_r) return;  // wave-uniform
    const int64_t row0 = tr * 32;
    const int K = p.K1 + p.K2;
    const int nchunk = K >> 4;
    const int64_t arow = row0 + l32;
    const int64_t ac = arow < p.B ? arow : 0;
    const float* x1r = p.x1_blk ? p.x1 + blk_off(arow, j, 8 * h, J, p.K1)
                                : p.x1 + ((ac + p.x1_row0) / p.x1_div) * p.x1_rs + (int64_t)j * p.K1 + 8 * h;
    const float* x2r = !p.K2 ? nullptr
                             : p.x2_blk ? p.x2 + blk_off(arow, j, 8 * h, J, p.K2) : p.x2 + ac * p.x2_rs + (int64_t)j * p.K2 + 8 * h;
    const _Float16* wbase = p.wsp + ((int64_t)p.ntype[j] * nchunk * p.wsp_nct + tc) * 1024 + lane * 8;
    const int64_t wcs = (int64_t)p.wsp_nct * 1024;  // halves per chunk

    floatx4 xa[PF], xb[PF];
    halfx8 wh[PF], wl[PF];
    auto issue = [&](int c, int sl) {
        const int k0 = c << 4;
        const float* src;
        int step4;
        if (k0 < p.K1) {
            src = p.x1_blk ? x1r + (k0 << 5) : x1r + k0;
            step4 = p.x1_blk ? 128 : 4;
        } else {
            src = p.x2_blk ? x2r + ((k0 - p.K1) << 5) : x2r + (k0 - p.K1);
            step4 = p.x2_blk ? 128 : 4;
        }
        xa[sl] = g4(src);
        xb[sl] = g4(src + step4);
        const _Float16* w = wbase + c * wcs;
        wh[sl] = *reinterpret_cast<const halfx8*>(w);
        if constexpr (!PREC) wl[sl] = *reinterpret_cast<const halfx8*>(w + 512);
    };
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    float ss = 0.f, amx = 0.f;
    auto compute = [&](int c, int sl) {
        const floatx8 f = {xa[sl].x, xa[sl].y, xa[sl].z, xa[sl].w, xb[sl].x, xb[sl].y, xb[sl].z, xb[sl].w};
        if (RMS && (c << 4) < p.K1) {
            const floatx8 q = f * f;
            ss += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
        }
        const floatx8 a = __builtin_elementwise_abs(f);
        amx = fmaxf(amx, fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])), fmaxf(fmaxf(a[4], a[5]), fmaxf(a[6], a[7]))));
        const halfx8 xh = __builtin_convertvector(f, halfx8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh[sl], acc, 0, 0, 0);
        if constexpr (!PREC) {
            const halfx8 xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl[sl], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh[sl], acc, 0, 0, 0);
        }
    };
    // nchunk % PF == 0 (launch_gl4y): every load issued unconditionally -- a main loop that always
    // issues, a last round that never does.  (Round 4: the earlier `if (c + PF < nchunk) issue`
    // form made the waitcnt pass merge the paths and wait vmcnt(1-3) at every chunk, i.e. one
    // memory latency per chunk instead of one per launch.)
    // the bias before the operand loads: loaded after the K loop it was the youngest memory op, and
    // its vmcnt(0) put one more memory latency between the last MFMA and the stores
    const int ncol = tc * 32 + l32;
    const float bv = (p.bias && ncol < p.N) ? p.bias[p.wrow[j] + ncol] : 0.f;
#pragma unroll
    for (int i = 0; i < PF; ++i) issue(i, i);
    for (int c0 = 0; c0 < nchunk - PF; c0 += PF) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            compute(c0 + i, i);
            issue(c0 + i + PF, i);
        }
    }
#pragma unroll
    for (int i = 0; i < PF; ++i) compute(nchunk - PF + i, i);
    // the range guard sees the real rows only (the padding rows of a row-blocked buffer hold
    // whatever the workspace held: never stored, but they must not trigger the fallback)
    const bool oor = __builtin_amdgcn_ballot_w64(arow < p.B && amx >= 65504.0f) != 0;  // wave-uniform
    float sc[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = p.wsp_unscale;
    if (RMS) {
        const float t = ss + __shfl_xor(ss, 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float n2 = __shfl(t, (r & 3) + 8 * (r >> 2) + 4 * h);
            sc[r] *= 1.0f / fmaxf(sqrtf(n2), 1e-12f);
        }
    }
    auto store = [&](const floatx16& v) {
        if constexpr (ROWMAJOR) {
            if (ncol < p.N) {
                float* y = yo.y + tr * yo.y_ts + j * yo.y_js + tc * yo.y_cs + l32;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row0 + rr < p.B) y[rr * yo.y_rs] = v[r] * sc[r] + bv;
                }
            }
        } else {  // the split route's column-tiled scratch: every row of the tile, N % 32 == 0
            float* y = p.zs + zs_off(row0, j, tc * 32, J, p.N) + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) y[((r & 3) + 8 * (r >> 2) + 4 * h) << 5] = v[r] * sc[r] + bv;
        }
    };
    store(acc);
    // f16 range left: the tile again on exact-f32 MFMA, stored over the first (same lanes, same
    // addresses: program order); after the stores, so no accumulator is live across the call
    if (oor) {
        if (p.status && lane == 0) atomicOr(p.status, 1u);
        store(exact_tile_f32(p, row0, j, tc * 32));
    }
}

// ---- split route, phase 1 for full batches (tiled GEMM) --------------------------------------
// k_gl4y gives every (32-row tile, node, 32-column tile) its own wave and its own operand loads:
// 4 B of operands per output per k chunk, fine for latency at 50 rows, ingest-bound at 3,200.
// k_gl4t: one workgroup = 4 waves = 4 consecutive 32-row tiles of ONE node x CT 32-column tiles.
// The node's weight slice for the CT tiles (CT x 2 KiB per 16-deep chunk) is staged once per
// workgroup in LDS (register-staged, double-buffered: no LDS-DMA) and shared by the 4 waves; each
// wave streams its own x fragments PF chunks ahead and reuses them over CT tiles.  Per chunk a
// workgroup pulls 8 KiB of x + CT x 2 KiB of weights for 128 x 32 CT outputs (0.8 B per output
// at CT = 6 vs 2.2 B in the one-kernel k_gl4 32 x 64 tile).  Per accumulator element the MFMA
// sequence (x_hi W'_hi, x_hi W'_lo, x_lo W'_hi per chunk), RMS sum, scale and bias arithmetic are
// k_gl4's, so phase 2 (k_gl4 MODE 2 / 3) reproduces the one-kernel route bit for bit.
// K loop (round 6; the round-4 / round-5 forms and what they measured: DESIGN.md §4i / §4j, git
// history): the node's weight slice for the workgroup's CT column tiles goes through an LDS-DMA
// ring of PF + 1 slots (chunk c in slot c % NS by global_load_lds_dwordx4, PF chunks ahead, shared
// by the NWV waves), each fill issued right after its chunk's barrier ("fill first"); x is each
// wave's own (RT 32-row tiles), so it goes straight into a register ring of NS slots by
// global_load_dwordx4 the compiler does not track (inline asm: a tracked load beside in-flight
// LDS-DMA made the waitcnt pass drain vmcnt(0) at its first use), issued with the chunk's weight
// fill and covered by the same counted vmcnt wait, then fenced into the compiler's view.  The chunk
// loop is unrolled whole, so every register slot is static (no loop-carried copies of registers
// still being written).  RT = 2: every weight fragment read from LDS feeds two row tiles.
// tools/gl4t_rt_probe.hip (config-2 shape, alone on the GPU, bitwise equal to the round-5 ring):
// N = 192, 3,200 rows 17.1 vs 20.7 us (RT 2, CT 3), 1,067 rows 10.8 vs 12.5; N = 768 (RT 1, CT 6)
// 53.6 vs 56.6 and 23.3 vs 25.9 (profiles/r06f/probe.txt).  bf16 operands (PREC 2) are their own A
// fragments and keep the tracked register ring of the round-5 form (RT = 1).
template <int PREC, int CT, int NCH, int PF>
constexpr int gl4t_smem_bytes() {
    constexpr int TILE_H = PREC ? 512 : 1024, TS = 36, NWV = 4, NS = PF + 1;
    constexpr int SBW = NS * CT * TILE_H * 2;
    return SBW > NWV * 32 * TS * 4 ? SBW : NWV * 32 * TS * 4;
}

// A 16-B global load the compiler does not track (k_gl4t's x ring): waited for by hand (counted
// s_waitcnt vmcnt + a register fence)
__device__ __forceinline__ void g4_async(floatx4& d, const float* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
}

// The workgroup's work: unit u = (node j, row group, column group); smem_raw = its
// gl4t_smem_bytes of LDS.  A row group is NWV waves x RT 32-row tiles.
template <bool RMS, int PREC, int CT, int NCH, bool ROWMAJOR, int RT, int PF>
__device__ __forceinline__ void gl4t_body(const GLArgs& p, int ncg, int64_t ntile_r, const YOut& yo, const int64_t u,
                                          const int tid, char* __restrict__ smem_raw) {
    static_assert(PREC != 2 || RT == 1, "bf16 operands: one row tile per wave");
    static_assert(PF >= 2 && PF <= 4, "chunks in flight");
    constexpr int NWV = 4;                      // waves per workgroup
    constexpr int NT = NWV * 64;
    constexpr int TILE_H = PREC ? 512 : 1024;   // halves of one 32-column tile per chunk
    constexpr int PPT = TILE_H / 8;             // 16-B pieces per tile
    constexpr int TS = 36;                      // floats per row of a wave's 32 x 32 output transpose
    constexpr int NS = PF + 1;                  // ring slots: chunk c in slot c % NS
    constexpr bool XV = PREC != 2;              // x by untracked register loads
    _Float16(*sW)[CT * TILE_H] = reinterpret_cast<_Float16(*)[CT * TILE_H]>(smem_raw);
    const int lane = tid & 63, l32 = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int J = p.J;
    // node-major order: column group fastest (the ncg workgroups sharing one x tile), then row
    // groups, then nodes, so an XCD's contiguous share of u holds one or two nodes' weights
    // (N = 768: 5.9 MB of split weights for all 10 types did not fit a 4 MB L2 when every XCD
    // walked every node: 196 MB fetched per launch for ~45 MB of operands)
    const int cg = (int)(u % ncg);
    const int64_t nrg = (ntile_r + NWV * RT - 1) / (NWV * RT);
    const int j = (int)((u / ncg) / nrg);
    const int64_t rgi = (u / ncg) % nrg;
    const int64_t tr0 = (rgi * NWV + wave) * RT;  // this wave's first 32-row tile
    // per row tile: its rows (a dead tile -- past the batch -- reads tile 0 and stores nothing)
    int64_t row0[RT], arow[RT];
    const float* x1r[RT];
    const float* x2r[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        row0[rt] = (tr0 + rt < ntile_r ? tr0 + rt : 0) * 32;
        arow[rt] = row0[rt] + l32;
        const int64_t ac = arow[rt] < p.B ? arow[rt] : 0;
        // feature 8 h of chunk 0: the lane's A fragment (rows l32, k 8 h .. 8 h + 7)
        x1r[rt] = p.x1_blk ? p.x1 + blk_off(arow[rt], j, 8 * h, J, p.K1)
                           : p.x1 + ((ac + p.x1_row0) / p.x1_div) * p.x1_rs + (int64_t)j * p.K1 + 8 * h;
        x2r[rt] = !p.K2 ? x1r[rt]
                        : p.x2_blk ? p.x2 + blk_off(arow[rt], j, 8 * h, J, p.K2) : p.x2 + ac * p.x2_rs + (int64_t)j * p.K2 + 8 * h;
    }
    // chunk c's two 16-B pieces of row tile rt: k 16 c + 8 h .. + 3 and + 4 .. + 7 (row-blocked:
    // 128 floats apart, row-major: 4); x1 for the first K1 / 16 chunks, then x2.  One running
    // source pointer per row tile, advanced after each chunk's loads (fill runs in chunk order):
    // with the K loop unrolled whole, per-chunk addresses were hoisted and held live (spills)
    const int c1 = p.K1 >> 4;
    const int cs1 = p.x1_blk ? 512 : 16, cs2 = p.x2_blk ? 512 : 16;
    const int st1 = p.x1_blk ? 128 : 4, st2 = p.x2_blk ? 128 : 4;
    const float* xp[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) xp[rt] = c1 > 0 ? x1r[rt] : x2r[rt];
    auto xstep = [&](int c) { return c < c1 ? st1 : st2; };
    floatx4 xa[NS][RT], xb[NS][RT];
    floatx16 acc[RT][CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[rt][ct][e] = 0.f;
    float ss[RT], amx[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) ss[rt] = amx[rt] = 0.f;
    // the epilogue's bias, loaded before the K loop: loaded per tile in the epilogue, each load was
    // the youngest memory op and its vmcnt(0) also waited for the previous tile's stores -- CT
    // serial memory round trips in the store tail
    float bvp[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) bvp[ct] = p.bias ? p.bias[p.wrow[j] + (cg * CT + ct) * 32 + l32] : 0.f;
    const _Float16* wt0 = p.wsp + ((int64_t)p.ntype[j] * NCH * p.wsp_nct + cg * CT) * 1024;
    // Pieces of wave w per chunk: q0 = 64 w + NT k < CT * PPT (two counts, wave-uniform).
    constexpr int NPC = CT * PPT;
    constexpr int XL = 2 * RT;  // x loads per chunk and lane
    constexpr int OPA = (NPC / 64 + NWV - 1) / NWV + XL, OPB = (NPC / 64) / NWV + XL;
    static_assert(OPA * (PF - 1) < 64, "vmcnt range");
    const bool wa = wave * 64 + NT * ((NPC / 64 + NWV - 1) / NWV - 1) < NPC;
    // chunk c: its weight slice to slot c % NS (LDS-DMA), then its x pieces to register slot c % NS
    auto fill = [&](int c) {
        _Float16* dst = sW[c % NS];
#pragma unroll
        for (int k = 0; k < (NPC / 64 + NWV - 1) / NWV; ++k) {
            const int q0 = wave * 64 + NT * k;
            if (q0 >= NPC) continue;  // wave-uniform
            const int q = q0 + lane;
            const _Float16* src = wt0 + ((int64_t)c * p.wsp_nct + q / PPT) * 1024 + (q % PPT) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
        }
        const int s = c % NS;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const float* src = xp[rt];
            xp[rt] = c + 1 == c1 ? x2r[rt] : src + (c < c1 ? cs1 : cs2);
            if constexpr (XV) {
                g4_async(xa[s][rt], src);
                g4_async(xb[s][rt], src + xstep(c));
            } else {
                // a bf16 operand: its 8 k values (16 B) are the A fragment itself; the same two loads
                // on both paths (selected addresses, no branch), so the waitcnt pass keeps the ring
                const bool bsrc = c < c1 ? p.x1_bf16 : p.x2_bf16;
                const float* base = c < c1 ? p.x1 : p.x2;
                const float* qb = reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(base) + (src - base));
                xa[s][rt] = g4(bsrc ? qb : src);
                xb[s][rt] = g4(bsrc ? qb : src + xstep(c));
            }
        }
    };
    auto compute = [&](int c) {
        const int s = c % NS;
        const _Float16* wt = sW[s] + lane * 8;
        const bool rms_chunk = RMS && c < c1;
        if constexpr (PREC == 2) {  // bf16 mode: one bf16 product per k step (k_gl4 PREC 2's arithmetic)
            const bool bsrc = c < c1 ? p.x1_bf16 : p.x2_bf16;  // wave-uniform
            bf16x8 xb16;
            floatx8 f;
            if (bsrc) {
                xb16 = __builtin_bit_cast(bf16x8, xa[s][0]);
                f = __builtin_convertvector(xb16, floatx8);
            } else {
                f = floatx8{xa[s][0].x, xa[s][0].y, xa[s][0].z, xa[s][0].w, xb[s][0].x, xb[s][0].y, xb[s][0].z, xb[s][0].w};
                xb16 = __builtin_convertvector(f, bf16x8);
            }
            if (rms_chunk) {
                const floatx8 q = f * f;
                ss[0] += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const bf16x8 wb = *reinterpret_cast<const bf16x8*>(wt + ct * TILE_H);
                acc[0][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb16, wb, acc[0][ct], 0, 0, 0);
            }
            return;
        }
        halfx8 xh[RT], xl[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const floatx8 f = {xa[s][rt].x, xa[s][rt].y, xa[s][rt].z, xa[s][rt].w,
                               xb[s][rt].x, xb[s][rt].y, xb[s][rt].z, xb[s][rt].w};
            if (rms_chunk) {
                const floatx8 q = f * f;
                ss[rt] += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
            }
            const floatx8 a = __builtin_elementwise_abs(f);
            amx[rt] = fmaxf(amx[rt], fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])), fmaxf(fmaxf(a[4], a[5]), fmaxf(a[6], a[7]))));
            xh[rt] = __builtin_convertvector(f, halfx8);
            if constexpr (!PREC) xl[rt] = __builtin_convertvector(f - __builtin_convertvector(xh[rt], floatx8), halfx8);
            // the guard / norm reductions pinned to this chunk: the whole-unrolled K loop is one
            // block and, unpinned, the compiler sank the fmax chains into the epilogue (where the
            // ballot reads them), holding every chunk's x live to there -- 62..270 VGPRs spilled
            asm volatile("" : "+v"(amx[rt]), "+v"(ss[rt]));
        }
        // per accumulator element: x_hi W_hi, x_hi W_lo, x_lo W_hi per chunk, chunks in order --
        // the round-5 ring's sequence (bitwise equal to it and to the one-kernel route)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
            halfx8 wl;
            if constexpr (!PREC) wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wh, acc[rt][ct], 0, 0, 0);
                if constexpr (!PREC) {
                    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wl, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl[rt], wh, t, 0, 0, 0);
                }
                acc[rt][ct] = t;
            }
        }
    };
    // chunk c's weights and x landed: vmcnt(the ops of the younger chunks in flight) AND
    // lgkmcnt(0) (every LDS read this wave issued for the previous chunk has returned before it
    // arrives, so a fill issued after the barrier into that chunk's slot cannot overtake a read
    // still in flight), then the register fence (XV: the compiler sees chunk c's x defined here)
    // and the barrier (publishes every wave's weight pieces of chunk c)
    // (younger: chunks c + 1 .. issued before this wait, min(PF - 1, NCH - 1 - c); a constant in
    // the whole-unrolled loop, so the switch folds)
    auto wait_chunk = [&](int c, int younger) {
        switch (younger) {
            case 0: __builtin_amdgcn_s_waitcnt(VmCnt4<0>::imm & ~(0xF << 8)); break;
            case 1:
                if (wa) __builtin_amdgcn_s_waitcnt(VmCnt4<OPA>::imm & ~(0xF << 8));
                else __builtin_amdgcn_s_waitcnt(VmCnt4<OPB>::imm & ~(0xF << 8));
                break;
            case 2:
                if (wa) __builtin_amdgcn_s_waitcnt(VmCnt4<2 * OPA>::imm & ~(0xF << 8));
                else __builtin_amdgcn_s_waitcnt(VmCnt4<2 * OPB>::imm & ~(0xF << 8));
                break;
            default:
                if (wa) __builtin_amdgcn_s_waitcnt(VmCnt4<3 * OPA>::imm & ~(0xF << 8));
                else __builtin_amdgcn_s_waitcnt(VmCnt4<3 * OPB>::imm & ~(0xF << 8));
                break;
        }
        if constexpr (XV) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) asm volatile("" : "+v"(xa[c % NS][rt]), "+v"(xb[c % NS][rt]) :: "memory");
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    static_assert(NCH >= PF, "ring depth");
#pragma unroll
    for (int i = 0; i < PF; ++i) fill(i);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        wait_chunk(c, NCH - 1 - c < PF - 1 ? NCH - 1 - c : PF - 1);
        if constexpr (XV) {  // fill first: the slots of chunk c - 1 are free after the barrier
            if (c + PF < NCH) fill(c + PF);
            asm volatile("" ::: "memory");
            compute(c);
        } else {  // the tracked bf16 register ring: chunk c's registers are read before refilled
            compute(c);
            asm volatile("" ::: "memory");
            if (c + PF < NCH) fill(c + PF);
        }
        asm volatile("" ::: "memory");
    }
    __syncthreads();  // every wave past its last chunk: the stages become the output transposes
    // Y = acc * sc + bias through a per-wave 32 x 32 LDS transpose (the stages are dead: every
    // wave is past its last chunk), stored as 16-B pieces: 4 dwordx4 instead of 16 dword stores
    // per tile.  Launch shapes: N a multiple of 32 CT (launch_gl4t), so every column is real.
    float* sT = reinterpret_cast<float*>(smem_raw) + wave * 32 * TS;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int64_t tr = tr0 + rt;
        if (tr >= ntile_r) break;  // wave-uniform: dead tiles store nothing
        // (real rows only: the padding rows of a row-blocked buffer are never stored)
        const bool oor = PREC != 2 && __builtin_amdgcn_ballot_w64(arow[rt] < p.B && amx[rt] >= 65504.0f) != 0;
        float sc[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = p.wsp_unscale;
        if (RMS) {
            const float t = ss[rt] + __shfl_xor(ss[rt], 32);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float n2 = __shfl(t, (r & 3) + 8 * (r >> 2) + 4 * h);
                sc[r] *= 1.0f / fmaxf(sqrtf(n2), 1e-12f);
            }
        }
        float* y = yo.y + tr * yo.y_ts + j * yo.y_js + (int64_t)cg * CT * yo.y_cs;  // YOut as k_gl4y's
        auto store_tile = [&](int ct, const floatx16& v, float bv) {
#pragma unroll
            for (int r = 0; r < 16; ++r) sT[((r & 3) + 8 * (r >> 2) + 4 * h) * TS + l32] = v[r] * sc[r] + bv;
            __builtin_amdgcn_wave_barrier();  // DS operations of one wave complete in order
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = 8 * q + (lane >> 3), c4 = (lane & 7) * 4;
                const floatx4 o = *reinterpret_cast<const floatx4*>(sT + row * TS + c4);
                if (!ROWMAJOR || row0[rt] + row < p.B)  // row-major z holds rows < B only
                    *reinterpret_cast<floatx4*>(y + (int64_t)row * yo.y_rs + ct * yo.y_cs + c4) = o;
            }
            __builtin_amdgcn_wave_barrier();
        };
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) store_tile(ct, acc[rt][ct], bvp[ct]);
        // f16 range left: every tile of the row tile again on exact-f32 MFMA, stored over the first
        // (same lanes, same addresses: program order) -- after the stores
        if (oor) {
            if (p.status && lane == 0) atomicOr(p.status, 1u);
#pragma nounroll
            for (int ct = 0; ct < CT; ++ct) {
                const int col = (cg * CT + ct) * 32;
                store_tile(ct, exact_tile_f32(p, row0[rt], j, col), p.bias ? p.bias[p.wrow[j] + col + l32] : 0.f);
            }
        }
    }
}

template <bool RMS, int PREC, int CT, int NCH, bool ROWMAJOR, int RT, int PF>
__global__ __launch_bounds__(256, 2) void k_gl4t(const GLArgs p, int ncg, int64_t ntile_r, const YOut yo) {
    __shared__ __attribute__((aligned(16))) char smem_raw[gl4t_smem_bytes<PREC, CT, NCH, PF>()];
    // XCD-aware order (k_gl4's): consecutive u -- the column groups of one (row group, node), which
    // read the same x -- on one XCD (blocks b, b + 8, ... share one), so x reaches that L2 once
    const int nwg = gridDim.x, xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int64_t u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (blockIdx.x >> 3);
    gl4t_body<RMS, PREC, CT, NCH, ROWMAJOR, RT, PF>(p, ncg, ntile_r, yo, u, threadIdx.x, smem_raw);
}

// Epilogue of the fused to_qkv + Attention kernel (MODE 1), J <= 32, dh = 32, 8 waves, a
// 32-row tile.  Per 8-row slab: the mixed-in q|k|v (Z = G-hat Y) goes to LDS as [row][node][96],
// then wave w runs the attention of row 8*slab + w exactly as k_attention<JT> does (same f32 MFMA
// order over JT 16-node tiles, expf softmax), writing out[row][n][head*32 + d].
// FROM_YS (MODE 3, split route phase 2): k_gl4 MODE 3 has put slab q8only in sY already.
template <int J, int NW, int NPW, bool FROM_YS = false>
__device__ __forceinline__ void attention_epilogue(const GLArgs& p, floatx16 (&acc)[NPW][1][3], float* smem,
                                                   const float* sG, int64_t row0, int head, int wave, int lane,
                                                   int q8only = 0) {
    constexpr int COLS = 96;
    constexpr int JT = (J + 15) / 16;   // 16-node tiles (k_attention<JT>)
    constexpr int KS = (J + 3) / 4;     // 4-deep k steps of the mixing GEMM
    constexpr int YS8 = 8 * COLS + 16;  // floats per node in an 8-row Y slab (+16: bank shift)
    constexpr int ZN = 100;             // floats per node in a Z row (+4: bank shift)
    constexpr int ZR = J * ZN;          // floats per Z row
    const int l32 = lane & 31, h = lane >> 5, lr = lane & 15, lg = lane >> 4;
    const int hid = p.attn_heads * 32;
    float* sY = smem;
    // FROM_YS (MODE 3): Z overwrites the Y slab (mixed into registers first, one barrier between),
    // so the workgroup needs max(Y, Z) instead of Y + Z: 52 KB at J = 16, 54 KB at J = 17 -- under
    // 64 KB, two workgroups per CU instead of one holding the whole CU
    float* sZ = FROM_YS ? smem : smem + J * YS8;
    float ga[JT][KS];  // G-hat^T[k = j = 4s + lg][col = i = 16 it + lr]
#pragma unroll
    for (int it = 0; it < JT; ++it)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int i = 16 * it + lr, jj = 4 * s + lg;
            ga[it][s] = (i < J && jj < J) ? sG[i * J + jj] : 0.f;
        }
#pragma unroll
    for (int q8 = 0; q8 < 4; ++q8) {  // rows 8 q8 .. 8 q8 + 7 = accumulator registers 4 q8 .. 4 q8 + 3
        if (FROM_YS && q8 != q8only) continue;
        if constexpr (!FROM_YS) {
            __syncthreads();  // K loop / previous slab done with this LDS
#pragma unroll
            for (int m = 0; m < NPW; ++m) {
                const int j = wave + NW * m;
                if (j >= J) continue;
#pragma unroll
                for (int ct = 0; ct < 3; ++ct)
#pragma unroll
                    for (int e = 0; e < 4; ++e) sY[j * YS8 + (e + 4 * h) * COLS + 32 * ct + l32] = acc[m][0][ct][4 * q8 + e];
            }
            __syncthreads();
        }
        // node mixing: 48 blocks of 16 (row, column) positions, 6 per wave
        floatx4 zk[FROM_YS ? 48 / NW : 1][JT];  // FROM_YS: all of this wave's Z before the overwrite
#pragma unroll
        for (int k = 0; k < 48 / NW; ++k) {
            const int rc0 = (wave + NW * k) * 16;
            float ya[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int jj = 4 * s + lg;
                ya[s] = jj < J ? sY[jj * YS8 + rc0 + lr] : 0.f;
            }
            const int rc = rc0 + 4 * lg, r = rc / COLS, c = rc - r * COLS;
#pragma unroll
            for (int it = 0; it < JT; ++it) {
                floatx4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < KS; ++s) z = __builtin_amdgcn_mfma_f32_16x16x4f32(ya[s], ga[it][s], z, 0, 0, 0);
                const int i = 16 * it + lr;
                if constexpr (FROM_YS) zk[k][it] = z;
                else if (i < J) *reinterpret_cast<floatx4*>(sZ + r * ZR + i * ZN + c) = z;
            }
        }
        if constexpr (FROM_YS) {
            __syncthreads();  // every wave's Y reads done: Z may overwrite the slab
#pragma unroll
            for (int k = 0; k < 48 / NW; ++k) {
                const int rc = (wave + NW * k) * 16 + 4 * lg, r = rc / COLS, c = rc - r * COLS;
#pragma unroll
                for (int it = 0; it < JT; ++it) {
                    const int i = 16 * it + lr;
                    if (i < J) *reinterpret_cast<floatx4*>(sZ + r * ZR + i * ZN + c) = zk[k][it];
                }
            }
        }
        __syncthreads();
        // attention of one row per wave (k_attention<JT>'s math)
        const int64_t row = row0 + 8 * q8 + wave;
        const float* zr = sZ + wave * ZR;
        floatx4 S[JT][JT];
#pragma unroll
        for (int a = 0; a < JT; ++a)
#pragma unroll
            for (int c = 0; c < JT; ++c) S[a][c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cc = 0; cc < 32; cc += 16) {
            floatx4 ka[JT], qv[JT];
#pragma unroll
            for (int t = 0; t < JT; ++t) {
                const int j = t * 16 + lr;
                ka[t] = j < J ? *reinterpret_cast<const floatx4*>(zr + j * ZN + 32 + cc + 4 * lg) : floatx4{0.f, 0.f, 0.f, 0.f};
                qv[t] = j < J ? *reinterpret_cast<const floatx4*>(zr + j * ZN + cc + 4 * lg) * p.attn_scale
                              : floatx4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int nt = 0; nt < JT; ++nt) {
                    floatx4 cacc = S[jt][nt];
                    cacc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[jt].x, qv[nt].x, cacc, 0, 0, 0);
                    cacc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[jt].y, qv[nt].y, cacc, 0, 0, 0);
                    cacc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[jt].z, qv[nt].z, cacc, 0, 0, 0);
                    cacc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[jt].w, qv[nt].w, cacc, 0, 0, 0);
                    S[jt][nt] = cacc;
                }
        }
        // softmax over j (rows of S^T) for every query column n = nt * 16 + lr
#pragma unroll
        for (int nt = 0; nt < JT; ++nt) {
            float mx = -INFINITY;
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (jt * 16 + 4 * lg + e < J) mx = fmaxf(mx, S[jt][nt][e]);
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            float sum = 0.f;
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float ex = (jt * 16 + 4 * lg + e < J) ? expf(S[jt][nt][e] - mx) : 0.f;
                    S[jt][nt][e] = ex;
                    sum += ex;
                }
            sum += __shfl_xor(sum, 16);
            sum += __shfl_xor(sum, 32);
            const float inv = 1.0f / sum;
#pragma unroll
            for (int jt = 0; jt < JT; ++jt) S[jt][nt] *= inv;
        }
        // O^T[d][n] = sum_j V[j][d] P^T[j][n]
#pragma unroll
        for (int dc = 0; dc < 32; dc += 16) {
            floatx4 vv[JT];
#pragma unroll
            for (int jt = 0; jt < JT; ++jt)
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) {
                    const int j = jt * 16 + 4 * lg + s4;
                    vv[jt][s4] = j < J ? zr[j * ZN + 64 + dc + lr] : 0.f;
                }
#pragma unroll
            for (int nt = 0; nt < JT; ++nt) {
                floatx4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int jt = 0; jt < JT; ++jt) {
                    o = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[jt].x, S[jt][nt].x, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[jt].y, S[jt][nt].y, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[jt].z, S[jt][nt].z, o, 0, 0, 0);
                    o = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[jt].w, S[jt][nt].w, o, 0, 0, 0);
                }
                const int n = nt * 16 + lr;
                if (n < J && row < p.B) {
                    const int f = head * 32 + dc + 4 * lg;
                    float* dst = p.out_blk ? p.out + blk_off(row, n, f, J, hid) : p.out + row * p.out_rs + (int64_t)n * hid + f;
                    *reinterpret_cast<floatx4*>(dst) = o;
                }
            }
        }
    }
}

// Block.norm for norm_type 'layer' (attention.py:19-28, 55-58): nn.LayerNorm(J) over the node axis
// of the graph-linear output, per (row, column), eps 1e-5, biased variance, per-node affine.  In the
// mixing epilogue's layout lane (lr, lg) holds node i = 16 ib + lr of four consecutive columns, so a
// (row, column)'s J nodes are the 16 lanes of one lg group (x IB blocks): two xor-butterfly sums
// over lr, nodes i >= J masked out.
__device__ __forceinline__ floatx4 sum_lanes16(floatx4 v) {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
        v.x += __shfl_xor(v.x, m);
        v.y += __shfl_xor(v.y, m);
        v.z += __shfl_xor(v.z, m);
        v.w += __shfl_xor(v.w, m);
    }
    return v;
}

template <int IB>
__device__ __forceinline__ void node_layernorm(floatx4 (&z)[IB], const float* __restrict__ w, const float* __restrict__ b,
                                               int J, int lr) {
    const float inv = 1.0f / (float)J;
    floatx4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ib = 0; ib < IB; ++ib)
        if (16 * ib + lr < J) s += z[ib];
    const floatx4 mu = sum_lanes16(s) * inv;
    floatx4 q = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ib = 0; ib < IB; ++ib)
        if (16 * ib + lr < J) {
            const floatx4 d = z[ib] - mu;
            q += d * d;
        }
    q = sum_lanes16(q) * inv;
    floatx4 rs;
    rs.x = 1.0f / sqrtf(q.x + 1e-5f);
    rs.y = 1.0f / sqrtf(q.y + 1e-5f);
    rs.z = 1.0f / sqrtf(q.z + 1e-5f);
    rs.w = 1.0f / sqrtf(q.w + 1e-5f);
#pragma unroll
    for (int ib = 0; ib < IB; ++ib) {
        const int i = 16 * ib + lr;
        const float wi = i < J ? w[i] : 0.f, bi = i < J ? b[i] : 0.f;
        z[ib] = (z[ib] - mu) * rs * wi + bi;
    }
}

// MODE 0: StaticGraphLinear with the FiLM / tanh / residual epilogue.
// MODE 1: to_qkv + Attention fused (attention.py:105-136): the workgroup's three 32-column tiles
//   are head h's q, k and v columns (tiles h, heads + h, 2 heads + h), and the epilogue runs
//   softmax(q k^T * dh^-1/2) v per row over the J nodes instead of storing q/k/v; out = the
//   (B, J, heads * 32) attention output that to_out reads.  qkv never reaches HBM.
// PREC 1 ("half" precision mode): one product x_hi W'_hi per k step, so
//   only the hi halves of the weight fragments are streamed (half the weight bytes, a third of
//   the MFMAs); f32 accumulate, f32 activations in HBM, same epilogue.
// PREC 2 ("bf16" mode, config 5 as stated): one bf16 product per k step on
//   v_mfma_f32_32x32x16_bf16 (a.wsp = make_bf16_weights), f32 accumulate and epilogue; operands
//   and result may be stored as bf16 (GLArgs::x1_bf16 / x2_bf16 / res_bf16 / out_bf16,
//   row-major): a bf16 operand is its own A fragment (one 16-B load per 8 k).
// STG 0: weight stages filled by LDS-DMA (global_load_lds_dwordx4); STG 1: register-staged
//   (global_load_dwordx4 a chunk ahead, ds_write_b128 after the chunk's MFMAs).
// The workgroup's work for virtual block index bx of a grid of nwg (k_gl4 passes blockIdx.x /
// gridDim.x); smem = its dynamic LDS.
template <int J, int NW, int RT, int CT, bool RMS, int MODE = 0, int PREC = 0, int STG = 0>
__device__ __forceinline__ void gl4_body(const GLArgs& p, const int bx, const int nwg, float* __restrict__ smem) {
    static_assert(MODE == 0 || MODE == 2 || (CT == 3 && RT == 1 && J <= 32 && NW == 8), "attention mode: 32 x (q|k|v)");
    static_assert(MODE < 2 || (RT == 1 && STG == 0), "split-route phase 2: one 32-row tile");
    constexpr bool PH2 = MODE == 2 || MODE == 3;  // split-route phase 2: Y from the scratch, no K loop
    constexpr int NPW = (J + NW - 1) / NW;  // nodes per wave
    constexpr int KS = (J + 3) / 4;         // 4-deep k steps of the mixing GEMM (K = J padded)
    constexpr int IB = (J + 15) / 16;       // 16-row i blocks of the mixing GEMM
    constexpr int COLS = 32 * CT;
    constexpr int YR = COLS + 4;            // floats per Y row (+4: 4x4 blocks read conflict-free)
    constexpr int YS = 16 * YR + 16;        // floats per node in a 16-row Y slab (+16: bank shift)
    constexpr int NTH = NW * 64;
    constexpr int BPW = (COLS + NW - 1) / NW;  // 16-wide mixing blocks per wave per slab
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l32 = lane & 31, h = lane >> 5, lr = lane & 15, lg = lane >> 4;
    constexpr int TILE_H = PREC ? 512 : 1024;   // halves of one 32-column tile per k chunk (hi | hi+lo)
    const int stage_h = MODE >= 2 ? 0 : p.ntypes * CT * TILE_H;  // halves per weight stage
    const int wfl = stage_h;                   // two stages of halves = stage_h floats
    constexpr bool ATT = MODE == 1 || MODE == 3;
    // Y slab (+ Z rows; MODE 3: Z overwrites Y, attention_epilogue<…, FROM_YS>)
    const int yfl = MODE == 3 ? max(J * (8 * COLS + 16), 8 * J * 100) : ATT ? J * (8 * COLS + 16) + 8 * J * 100 : J * YS;
    _Float16* sW0 = reinterpret_cast<_Float16*>(smem);
    _Float16* sW1 = sW0 + stage_h;
    float* sY = smem;  // aliases the weight stages after the K loop
    float* sG = smem + (wfl > yfl ? wfl : yfl);
    float* sF = sG + J * J;  // FiLM (scale + 1 | shift) for this workgroup's columns

    const int ntile_c = ATT ? p.attn_heads : (p.N + COLS - 1) / COLS;
    const int xcd = bx & 7, q8 = nwg >> 3, r8 = nwg & 7;
    // XCD-aware order: consecutive L (the column tiles of one row tile) on one XCD, so x is
    // fetched into that XCD's L2 once.  attn_order 1 (fused attention): L = blockIdx, i.e. head
    // h = blockIdx % heads runs on XCD h % 8 and each XCD's L2 keeps only its heads' weights.
    // Split-route phase 2: workgroup = (tile, 16-row slab) in MODE 2, (tile, 8-row slab) in MODE 3.
    const int L = MODE == 2   ? (int)(bx >> 1)
                  : MODE == 3 ? (int)(bx >> 2)
                  : (MODE == 1 && p.attn_order == 1)
                      ? (int)bx
                      : (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3);
    const int slab = MODE == 2 ? (int)(bx & 1) : MODE == 3 ? (int)(bx & 3) : 0;
    const int ctile = L % ntile_c;
    const int64_t row0 = (int64_t)(L / ntile_c) * (32 * RT);
    const int c0 = ctile * COLS;
    const int K = p.K1 + p.K2;
    const int nchunk = K >> 4;  // even (checked at launch)

    // x row pointers: row-major (B, J, K) with the tail rows clamped to row 0 (never stored), or
    // row-blocked (padded to 32 rows: read as they are) -- see blk_off
    const float* x1r[RT];
    const float* x2r[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int64_t arow = row0 + 32 * rt + l32;
        const int64_t ac = arow < p.B ? arow : 0;
        x1r[rt] = p.x1_blk ? p.x1 + blk_off(arow, 0, 8 * h, J, p.K1) : p.x1 + ((ac + p.x1_row0) / p.x1_div) * p.x1_rs + 8 * h;
        x2r[rt] = !p.K2 ? nullptr : p.x2_blk ? p.x2 + blk_off(arow, 0, 8 * h, J, p.K2) : p.x2 + ac * p.x2_rs + 8 * h;
    }
    int jn[NPW], toff[NPW];  // wave-uniform (SGPR): clamped node, its type's stage offset
#pragma unroll
    for (int m = 0; m < NPW; ++m) {
        jn[m] = min(wave + NW * m, J - 1);
        toff[m] = p.ntype[jn[m]] * (CT * TILE_H);
    }

    // (mixing-epilogue helpers, defined before the phase-2 loads so MODE 2 can issue its residual
    // loads together with the Y slab's)
    // Mixing block b (0 <= b < COLS) of a 16-row slab = 16 (row, column) positions; the A lane lr
    // reads position lr, the output lane (lr = node, lg) owns positions 4 lg .. 4 lg + 3, which
    // are always 4 consecutive columns of one row (one 16-B piece).  Row-major output: a block is
    // 16 consecutive columns of one row, so the 4 lanes of a node cover 64 contiguous bytes.
    // Row-blocked output: a block is 4 rows x 4 columns (lg -> row), so the 4 lanes of a node
    // cover 4 consecutive rows of one 4-feature group = 64 contiguous bytes of that layout.
    const bool blk_out = p.out_blk != 0;  // wave-uniform
    auto a_off = [&](int b) {             // LDS offset (row * YR + col) of this lane's A position
        return blk_out ? ((b / (COLS / 4)) * 4 + (lr >> 2)) * YR + (b % (COLS / 4)) * 4 + (lr & 3)
                       : (b / (COLS / 16)) * YR + (b % (COLS / 16)) * 16 + lr;
    };
    auto out_pos = [&](int b, int& r, int& cc) {  // row in the slab and first column of this lane's quad
        if (blk_out) {
            r = (b / (COLS / 4)) * 4 + lg;
            cc = (b % (COLS / 4)) * 4;
        } else {
            r = b / (COLS / 16);
            cc = (b % (COLS / 16)) * 16 + 4 * lg;
        }
    };
    // J <= 16: a slab's residual pieces are all loaded before the Y exchange (latency hidden);
    // J > 16 (two node blocks): per group of PG blocks, halving the registers they hold
    constexpr bool RES_EARLY = IB == 1;
    constexpr int PG0 = (IB == 1 && BPW <= 8) ? BPW : (BPW < 4 ? BPW : 4);
    floatx4 rv[RES_EARLY ? BPW : PG0][IB];
    auto load_res = [&](int hc, int kfirst, int kcount) {
#pragma unroll
        for (int kk = 0; kk < (RES_EARLY ? BPW : PG0); ++kk) {
            if (kk >= kcount) continue;
            const int k = kfirst + kk;
            const int b = k < BPW ? wave + NW * k : COLS;
            int r, cc;
            out_pos(min(b, COLS - 1), r, cc);
            const int64_t row = row0 + 16 * hc + r;
            const int n = c0 + cc;
            const bool ok = b < COLS && row < p.B && n < p.N;  // N % 4 == 0 (checked at launch)
#pragma unroll
            for (int ib = 0; ib < IB; ++ib) {
                const int i = ib * 16 + lr;
                const int64_t ro = p.res_blk ? blk_off(row, i, n, J, p.N) : row * p.res_rs + (int64_t)i * p.N + n;
                if (PREC == 2 && p.res_bf16)
                    rv[kk][ib] = (ok && i < J) ? __builtin_convertvector(
                                                     *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(p.res) + ro), floatx4)
                                               : floatx4{0.f, 0.f, 0.f, 0.f};
                else
                    rv[kk][ib] = (ok && i < J) ? g4(p.res + ro) : floatx4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };

    floatx16 acc[NPW][RT][CT];
    if constexpr (PH2) {
        // split-route phase 2: the slab's Y (from phase 1's p.zs), G-hat and FiLM all loaded to
        // registers first (one memory round trip), then to LDS, one barrier
        constexpr int C4 = COLS / 4;
        constexpr int YQ = MODE == 2 ? J * 16 * C4 : J * 8 * 24;  // 16-B pieces of the slab
        constexpr int NYL = (YQ + NTH - 1) / NTH, NGL = (J * J + NTH - 1) / NTH;
        constexpr int YS8 = 8 * COLS + 16;  // MODE 3: attention_epilogue's slab layout
        const int64_t tb = (row0 >> 5) * J;
        // column-tiled zs (zs_off): consecutive q read consecutive 16-B pieces -- one node's rows of
        // the slab in one column tile are a contiguous 1-2 KiB run
        (void)tb;
        auto ysrc = [&](int q, float*& dst) -> const float* {
            if constexpr (MODE == 2) {
                static_assert(MODE != 2 || COLS == 32, "MODE 2: one 32-column tile");
                const int cc = (q % C4) * 4, r = (q / C4) & 15, j = q / (16 * C4);
                dst = sY + j * YS + r * YR + cc;
                return p.zs + zs_off(row0 + 16 * slab + r, j, c0 + cc, J, p.N);
            } else {
                const int cc = (q & 7) * 4, rr = (q >> 3) & 7, j = (q >> 6) % J, ct = (q >> 6) / J;
                dst = sY + j * YS8 + rr * COLS + 32 * ct + cc;
                return p.zs + zs_off(row0 + 8 * slab + rr, j, (ctile + ct * p.attn_heads) * 32 + cc, J, p.N);
            }
        };
        floatx4 yv[NYL];
        float gv[NGL];
        float f0 = 1.0f, f1 = 0.0f;
#pragma unroll
        for (int k = 0; k < NYL; ++k) {
            const int q = tid + k * NTH;
            float* d;
            if (q < YQ) {
                yv[k] = g4(ysrc(q, d));
            }
        }
        if constexpr (MODE == 2 && RES_EARLY)  // the residual in flight with the slab (one memory latency)
            if (p.res) load_res(slab, 0, BPW);
#pragma unroll
        for (int k = 0; k < NGL; ++k)
            if (tid + k * NTH < J * J) gv[k] = p.G[tid + k * NTH];
        if (tid < COLS && p.film && c0 + tid < p.N) {
            f0 = p.film[c0 + tid] + 1.0f;
            f1 = p.film[p.N + c0 + tid];
        }
#pragma unroll
        for (int k = 0; k < NYL; ++k) {
            const int q = tid + k * NTH;
            float* d;
            if (q < YQ) {
                (void)ysrc(q, d);
                *reinterpret_cast<floatx4*>(d) = yv[k];
            }
        }
#pragma unroll
        for (int k = 0; k < NGL; ++k)
            if (tid + k * NTH < J * J) sG[tid + k * NTH] = gv[k];
        if (tid < COLS) {
            sF[tid] = f0;
            sF[COLS + tid] = f1;
        }
        __syncthreads();
    } else {
    float ss[NPW][RT];
    float amx = 0.f;  // max |x| this lane split to f16 (range guard, GLArgs::status)
#pragma unroll
    for (int m = 0; m < NPW; ++m)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            ss[m][rt] = 0.f;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[m][rt][ct][e] = 0.f;
        }

    struct XBuf {
        floatx4 a[NPW][RT], b[NPW][RT];
    };
    XBuf X0, X1, X2;
    auto load_x = [&](int c, XBuf& xb) {
        const int k0 = c << 4;
#pragma unroll
        for (int m = 0; m < NPW; ++m)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const float* src;
                int step4;  // floats from k..k+3 to k+4..k+7
                if (k0 < p.K1) {
                    src = p.x1_blk ? x1r[rt] + (int64_t)jn[m] * p.K1 * 32 + (k0 << 5) : x1r[rt] + (int64_t)jn[m] * p.K1 + k0;
                    step4 = p.x1_blk ? 128 : 4;
                } else {
                    const int k2 = k0 - p.K1;
                    src = p.x2_blk ? x2r[rt] + (int64_t)jn[m] * p.K2 * 32 + (k2 << 5) : x2r[rt] + (int64_t)jn[m] * p.K2 + k2;
                    step4 = p.x2_blk ? 128 : 4;
                }
                if (PREC == 2 && (k0 < p.K1 ? p.x1_bf16 : p.x2_bf16)) {
                    // 8 bf16 k values (16 B): the A fragment itself, kept bit-exact in `a`; the
                    // element offset of src is that of the f32 layout (row-major)
                    const float* base = k0 < p.K1 ? p.x1 : p.x2;
                    const __bf16* bs = reinterpret_cast<const __bf16*>(base) + (src - base);
                    xb.a[m][rt] = *reinterpret_cast<const floatx4*>(bs);
                } else {
                    xb.a[m][rt] = g4(src);
                    xb.b[m][rt] = g4(src + step4);
                }
            }
    };
    // LDS-DMA of chunk c's weight slice for this workgroup's columns: per type one contiguous
    // span of CT * 2 KiB starting at tile (c0 / 32)
    auto fill_w = [&](int c, _Float16* dst) {
        constexpr int PPT = TILE_H / 8;     // 16-B pieces per tile (hi | hi+lo)
        const int per_type = CT * PPT;
        const int npieces = p.ntypes * per_type;
        for (int q0 = wave * 64; q0 < npieces; q0 += NTH) {
            const int q = min(q0 + lane, npieces - 1);
            const int t = q / per_type, rem = q - t * per_type;
            const int ct = rem / PPT;  // 32-column tile of this piece
            const int tile = MODE == 1 ? ctile + ct * p.attn_heads : (c0 >> 5) + ct;
            const _Float16* src = p.wsp + (((int64_t)t * nchunk + c) * p.wsp_nct + tile) * 1024 + (rem % PPT) * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(dst + (size_t)q0 * 8), 16, 0, 0);
        }
    };
#ifdef SD_DEBUG_LDS
    // stage c against its global source, read in the phase that reads the stage anyway
    auto check_stage = [&](int c) {
        constexpr int PPT = TILE_H / 8;
        const int per_type = CT * PPT;
        const int npieces = p.ntypes * per_type;
        const _Float16* st = (c & 1) ? sW1 : sW0;
        unsigned bad = 0;
        for (int q = tid; q < npieces; q += NTH) {
            const int t = q / per_type, rem = q - t * per_type;
            const int ct = rem / PPT;
            const int tile = MODE == 1 ? ctile + ct * p.attn_heads : (c0 >> 5) + ct;
            const uint4 g = *reinterpret_cast<const uint4*>(p.wsp + (((int64_t)t * nchunk + c) * p.wsp_nct + tile) * 1024 +
                                                            (rem % PPT) * 8);
            const uint4 l = *reinterpret_cast<const uint4*>(st + (size_t)q * 8);
            bad += (g.x != l.x) + (g.y != l.y) + (g.z != l.z) + (g.w != l.w);
        }
        if (bad) atomicAdd(&p.dbg[0], bad);
    };
#endif
    auto compute = [&](int c, const XBuf& xb) {
        const _Float16* cur = (c & 1) ? sW1 : sW0;
        const bool rms_chunk = RMS && (c << 4) < p.K1;
#pragma unroll
        for (int m = 0; m < NPW; ++m) {
            if (wave + NW * m >= J) continue;  // wave-uniform
            const _Float16* wt = cur + toff[m] + lane * 8;
            if constexpr (PREC == 2) {
                const bool bsrc = (c << 4) < p.K1 ? p.x1_bf16 : p.x2_bf16;  // wave-uniform
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    bf16x8 xb16;
                    floatx8 f;
                    if (bsrc) {
                        xb16 = __builtin_bit_cast(bf16x8, xb.a[m][rt]);
                        f = __builtin_convertvector(xb16, floatx8);
                    } else {
                        f = floatx8{xb.a[m][rt].x, xb.a[m][rt].y, xb.a[m][rt].z, xb.a[m][rt].w,
                                    xb.b[m][rt].x, xb.b[m][rt].y, xb.b[m][rt].z, xb.b[m][rt].w};
                        xb16 = __builtin_convertvector(f, bf16x8);
                    }
                    if (rms_chunk) {
                        const floatx8 q = f * f;
                        ss[m][rt] += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
                    }
#pragma unroll
                    for (int ct = 0; ct < CT; ++ct) {
                        const bf16x8 wb = *reinterpret_cast<const bf16x8*>(wt + ct * TILE_H);
                        acc[m][rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xb16, wb, acc[m][rt][ct], 0, 0, 0);
                    }
                }
                continue;
            }
            halfx8 xh[RT], xl[RT];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const floatx8 f = {xb.a[m][rt].x, xb.a[m][rt].y, xb.a[m][rt].z, xb.a[m][rt].w,
                                   xb.b[m][rt].x, xb.b[m][rt].y, xb.b[m][rt].z, xb.b[m][rt].w};
                if (rms_chunk) {
                    const floatx8 q = f * f;
                    ss[m][rt] += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
                }
                if (row0 + 32 * rt + l32 < p.B) {  // real rows only (row-blocked padding rows: any bits)
                    const floatx8 a = __builtin_elementwise_abs(f);
                    amx = fmaxf(amx, fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])),
                                           fmaxf(fmaxf(a[4], a[5]), fmaxf(a[6], a[7]))));
                }
                xh[rt] = __builtin_convertvector(f, halfx8);
                if constexpr (!PREC) xl[rt] = __builtin_convertvector(f - __builtin_convertvector(xh[rt], floatx8), halfx8);
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                const halfx8 wh = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H);
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    floatx16 a = acc[m][rt][ct];
                    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wh, a, 0, 0, 0);
                    if constexpr (!PREC) {
                        const halfx8 wl = *reinterpret_cast<const halfx8*>(wt + ct * TILE_H + 512);
                        a = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh[rt], wl, a, 0, 0, 0);
                        a = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl[rt], wh, a, 0, 0, 0);
                    }
                    acc[m][rt][ct] = a;
                }
            }
        }
    };
    // One k chunk: everything issued for chunk c (weight DMA + x loads) has landed -> barrier
    // (stage c visible to all waves; every wave is past chunk c-1, so its stage is free) ->
    // issue chunk c+1 into the other stage / register buffer -> MFMAs on chunk c.  The waitcnt
    // is a builtin (not inline asm) so the compiler knows x(c) is complete and inserts no
    // further vmcnt waits before the MFMAs.
    auto step = [&](int c, const XBuf& cur, XBuf& nxt) {
        __builtin_amdgcn_s_waitcnt(VmCnt4<0>::imm);
        __builtin_amdgcn_s_barrier();
        if (c + 1 < nchunk) {
            fill_w(c + 1, (c & 1) ? sW0 : sW1);
            load_x(c + 1, nxt);
        }
        compute(c, cur);
#if defined(SD_DEBUG_LDS) && !defined(SD_DEBUG_NO_GL)
        check_stage(c);
#endif
    };

    // G-hat and FiLM (scale + 1 | shift) for this workgroup's columns -> LDS, bias -> registers:
    // all read by the epilogue only, after the K loop's barriers
    for (int i = tid; i < J * J; i += NTH) sG[i] = p.G[i];
    for (int i = tid; i < COLS; i += NTH) {
        const int n = c0 + i;
        sF[i] = (p.film && n < p.N) ? p.film[n] + 1.0f : 1.0f;
        sF[COLS + i] = (p.film && n < p.N) ? p.film[p.N + n] : 0.0f;
    }
    float bv[NPW][CT];
#pragma unroll
    for (int m = 0; m < NPW; ++m)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) {
            const int ncol = (MODE == 1 ? (ctile + ct * p.attn_heads) * 32 : c0 + 32 * ct) + l32;
            bv[m][ct] = (p.bias && ncol < p.N) ? p.bias[p.wrow[jn[m]] + ncol] : 0.f;
        }
    if constexpr (STG == 1) {
        // register-staged weights: the pieces of chunk c+1 this thread carries are loaded right
        // after barrier c (with x(c+1)) and written to the other stage after compute(c); its
        // last reads were in phase c-1, before barrier c.  lgkmcnt(0) + barrier c+1 makes the
        // writes visible to every wave (no LDS-DMA anywhere in the K loop).
        constexpr int MAXP = 8;  // checked at launch: ntypes * CT * TILE_H / 8 <= MAXP * NTH
        constexpr int PPT = TILE_H / 8;
        const int per_type = CT * PPT;
        const int npieces = p.ntypes * per_type;
        // per carried piece: its offset in chunk 0's slice (halves; chunk c adds c * cstride)
        int woff[MAXP];
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            const int q = min(tid + k * NTH, npieces - 1);
            const int t = q / per_type, rem = q - t * per_type;
            const int ct = rem / PPT;
            const int tile = MODE == 1 ? ctile + ct * p.attn_heads : (c0 >> 5) + ct;
            woff[k] = ((t * nchunk) * p.wsp_nct + tile) * 1024 + (rem % PPT) * 8;
        }
        const int cstride = p.wsp_nct * 1024;
        // the carried pieces as MAXP named registers (an array here was kept in scratch)
        uint4 w0, w1, w2, w3, w4, w5, w6, w7;
#define SD_W8(OP) OP(0, w0) OP(1, w1) OP(2, w2) OP(3, w3) OP(4, w4) OP(5, w5) OP(6, w6) OP(7, w7)
#define SD_WLOAD(k, w) \
    if (tid + k * NTH < npieces) w = *reinterpret_cast<const uint4*>(p.wsp + woff[k] + c * cstride);
#define SD_WSTORE(k, w) \
    if (tid + k * NTH < npieces) *reinterpret_cast<uint4*>(dst + (size_t)(tid + k * NTH) * 8) = w;
        auto load_w = [&](int c) { SD_W8(SD_WLOAD) };
        auto store_w = [&](_Float16* dst) { SD_W8(SD_WSTORE) };
#undef SD_WLOAD
#undef SD_WSTORE
#undef SD_W8
        auto step_r = [&](int c, const XBuf& cur, XBuf& nxt) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's stage writes landed
            __builtin_amdgcn_s_barrier();
            if (c + 1 < nchunk) {
                load_w(c + 1);
                load_x(c + 1, nxt);
            }
            compute(c, cur);
            if (c + 1 < nchunk) store_w((c & 1) ? sW0 : sW1);
        };
        load_w(0);
        load_x(0, X0);
        store_w(sW0);
        for (int c = 0; c < nchunk; c += 2) {
            step_r(c, X0, X1);
            step_r(c + 1, X1, X0);
        }
    } else {
        fill_w(0, sW0);
        load_x(0, X0);
        for (int c = 0; c < nchunk; c += 2) {
            step(c, X0, X1);
            step(c + 1, X1, X0);
        }
    }
    // f16 range guard: a wave whose f16 operands reached |x| >= 65504 (x_hi would be inf) recomputes
    // its tiles on exact-f32 MFMA (exact_tile_f32, the split-route GEMM phases' fallback) before the
    // epilogue, whatever the f16 precision mode (round 6: the one-kernel tiles -- SD_OPT_SPLIT_ROUTE
    // 1, a gl4_tile option, half precision's J = 16 full-batch default -- only set the status bit
    // before).  The branch is wave-uniform and never taken in range, so the in-range arithmetic and
    // every bitwise route equality are unchanged; with the accumulators live the recompute costs
    // these tiles registers (spills at J = 17 / 21), which only a wave that left the range executes.
    if constexpr (PREC != 2) {
        if (__builtin_amdgcn_ballot_w64(amx >= 65504.0f) != 0) {
            if (p.status && lane == 0) atomicOr(p.status, 1u);
#pragma unroll
            for (int m = 0; m < NPW; ++m) {
                if (wave + NW * m >= J) continue;  // wave-uniform
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                    for (int ct = 0; ct < CT; ++ct)
                        acc[m][rt][ct] = exact_tile_f32(p, row0 + 32 * rt, jn[m],
                                                        MODE == 1 ? (ctile + ct * p.attn_heads) * 32 : c0 + 32 * ct);
            }
        }
    } else {
        if (p.status && __builtin_amdgcn_ballot_w64(amx >= 65504.0f) != 0 && lane == 0) atomicOr(p.status, 1u);
    }

    // ---- unscale, RMS, bias in the accumulator layout:
    //      D[row = (r&3) + 8(r>>2) + 4h][col = l32] for register r of a 32x32 tile
#pragma unroll
    for (int m = 0; m < NPW; ++m) {
        const int j = wave + NW * m;
        if (j >= J) continue;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            float sc[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) sc[r] = p.wsp_unscale;
            if (RMS) {
                const float t = ss[m][rt] + __shfl_xor(ss[m][rt], 32);  // full row l32 sum of squares
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float n2 = __shfl(t, (r & 3) + 8 * (r >> 2) + 4 * h);
                    sc[r] *= 1.0f / fmaxf(sqrtf(n2), 1e-12f);
                }
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[m][rt][ct][r] = acc[m][rt][ct][r] * sc[r] + bv[m][ct];
        }
    }
    }  // MODE < 2: K loop
#if defined(SD_DEBUG_LDS) && !defined(SD_DEBUG_NO_G)
    {
        unsigned bad = 0;
        for (int i = tid; i < J * J; i += NTH) bad += sG[i] != p.G[i];
        if (bad) atomicAdd(&p.dbg[2], bad);
    }
#endif
    if constexpr (MODE == 1) {
        attention_epilogue<J, NW, NPW>(p, acc, smem, sG, row0, ctile, wave, lane);
        return;
    } else if constexpr (MODE == 3) {
        attention_epilogue<J, NW, NPW, true>(p, acc, smem, sG, row0, ctile, wave, lane, slab);
        return;
    }
    // ---- mixing + epilogue, one 16-row slab at a time.  Z^T = Y^T G-hat^T on 16x16x4 f32 MFMA
    // with Y^T as the A operand: lane (lr, lg) ends up holding D[rc = 4lg + e][i = lr], i.e. four
    // consecutive columns of one row for node i, so residual loads and output stores are 16 B
    // per lane.  Mixing block b covers rc = 16b .. 16b+15 (one row, 16 consecutive columns).
    float ga[IB][KS];  // B operand: G-hat^T[k = j = 4s + lg][col = i = 16ib + lr]
#pragma unroll
    for (int ib = 0; ib < IB; ++ib)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int i = ib * 16 + lr, jj = 4 * s + lg;
            ga[ib][s] = (i < J && jj < J) ? sG[i * J + jj] : 0.f;
        }
#pragma unroll
    for (int hc0 = 0; hc0 < (MODE == 2 ? 1 : 2 * RT); ++hc0) {
        const int hc = MODE == 2 ? slab : hc0;
        const int rt = hc >> 1, hf = hc & 1;
        if (RES_EARLY && MODE != 2 && p.res) load_res(hc, 0, BPW);  // latency hides under the Y exchange below
        if constexpr (MODE != 2) {  // MODE 2: the slab is in sY already
            __syncthreads();        // K loop / previous slab done with the LDS that sY aliases
#pragma unroll
            for (int m = 0; m < NPW; ++m) {
                const int j = wave + NW * m;
                if (j >= J) continue;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int r = (q & 3) + 8 * (q >> 2) + 4 * h;
                        sY[j * YS + r * YR + 32 * ct + l32] = acc[m][rt][ct][8 * hf + q];
                    }
            }
            __syncthreads();
        }
        // per group of PG blocks: phase 1 every LDS read, phase 2 the mixing MFMAs, phase 3
        // FiLM / tanh / residual / 16-B stores -- no dependent chain per block
        constexpr int PG = (IB == 1 && BPW <= 8) ? BPW : (BPW < 4 ? BPW : 4);
        static_assert(PG == PG0, "residual group size");
#pragma unroll
        for (int k0 = 0; k0 < BPW; k0 += PG) {
            if (!RES_EARLY && p.res) load_res(hc, k0, min(PG, BPW - k0));
            float ya[PG][KS];  // A operand: Y^T[row = rc = 16b + lr][k = j = 4s + lg]
#pragma unroll
            for (int kk = 0; kk < PG; ++kk) {
                const int b = min(wave + NW * (k0 + kk), COLS - 1);
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const int jj = 4 * s + lg;
                    ya[kk][s] = (k0 + kk < BPW && jj < J) ? sY[jj * YS + a_off(b)] : 0.f;
                }
            }
            floatx4 z[PG][IB];
#pragma unroll
            for (int kk = 0; kk < PG; ++kk)
#pragma unroll
                for (int ib = 0; ib < IB; ++ib) {
                    floatx4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s = 0; s < KS; ++s)
                        t = __builtin_amdgcn_mfma_f32_16x16x4f32(ya[kk][s], ga[ib][s], t, 0, 0, 0);
                    z[kk][ib] = t;
                }
#pragma unroll
            for (int kk = 0; kk < PG; ++kk) {
                const int k = k0 + kk;
                if (k >= BPW) continue;
                const int b = wave + NW * k;
                int r, cc;
                out_pos(min(b, COLS - 1), r, cc);
                const int64_t row = row0 + 16 * hc + r;
                const int n = c0 + cc;
                const bool ok = b < COLS && row < p.B && n < p.N;
                const floatx4 fa = *reinterpret_cast<const floatx4*>(sF + cc);
                const floatx4 fb = *reinterpret_cast<const floatx4*>(sF + COLS + cc);
                if constexpr (MODE == 2)  // norm_type 'layer' (split route only: no registers taken from MODE 0)
                    if (p.ln_w) node_layernorm<IB>(z[kk], p.ln_w, p.ln_b, J, lr);
#pragma unroll
                for (int ib = 0; ib < IB; ++ib) {
                    const int i = ib * 16 + lr;
                    floatx4 v = z[kk][ib] * fa + fb;
                    if (p.act == 1) {
                        v.x = tanh4(v.x);
                        v.y = tanh4(v.y);
                        v.z = tanh4(v.z);
                        v.w = tanh4(v.w);
                    }
                    if (p.res) v += rv[RES_EARLY ? k : kk][ib];
                    if (ok && i < J) {
                        const int64_t oo = p.out_blk ? blk_off(row, i, n, J, p.N) : row * p.out_rs + (int64_t)i * p.N + n;
                        if (PREC == 2 && p.out_bf16)
                            *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(p.out) + oo) = __builtin_convertvector(v, bf16x4);
                        else
                            *reinterpret_cast<floatx4*>(p.out + oo) = v;
                    }
                }
            }
        }
    }
}

template <int J, int NW, int RT, int CT, bool RMS, int MODE = 0, int PREC = 0, int STG = 0>
__global__ __launch_bounds__(NW * 64, 1) void k_gl4(const GLArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    gl4_body<J, NW, RT, CT, RMS, MODE, PREC, STG>(p, blockIdx.x, gridDim.x, smem);
}

// v4 weight staging (GLArgs::gl4_stage): 0 = LDS-DMA stages, 1 = register-staged stages (2, a
// round-2 diagnostic setting, is now the same as 0: every launch takes its exact LDS).  Process
// default SKELDIFF_GL4_STAGE for new plans.
static int g_gl4_stage = [] {
    const char* e = getenv("SKELDIFF_GL4_STAGE");
    const int v = e ? atoi(e) : 0;
    return (v >= 0 && v <= 2) ? v : 0;
}();
int gl4_stage_default() { return g_gl4_stage; }

template <int J, int NW, int RT, int CT, int MODE = 0, int PREC = 0, int STG = 0>
static hipError_t gl4_launch_t(const GLArgs& a, bool rms, hipStream_t s);

template <int J, int NW, int RT, int CT, int MODE = 0, int PREC = 0>
static hipError_t gl4_launch(const GLArgs& a, bool rms, hipStream_t s) {
    constexpr int TILE_H = PREC ? 512 : 1024;
    // register staging: not for the J > 16 fused attention tile (3 nodes per wave: it would spill)
    if constexpr (MODE == 0 || (MODE == 1 && J <= 16)) {
        if (a.gl4_stage == 1 && a.ntypes * CT * (TILE_H / 8) <= 8 * NW * 64)
            return gl4_launch_t<J, NW, RT, CT, MODE, PREC, 1>(a, rms, s);
    }
    return gl4_launch_t<J, NW, RT, CT, MODE, PREC, 0>(a, rms, s);
}

template <int J, int NW, int RT, int CT, int MODE, int PREC, int STG>
static hipError_t gl4_launch_t(const GLArgs& a, bool rms, hipStream_t s) {
    constexpr int COLS = 32 * CT;
    constexpr bool ATT = MODE == 1 || MODE == 3;
    const int ntile_c = ATT ? a.attn_heads : (a.N + COLS - 1) / COLS;
    const int64_t ntile_r = (a.B + 32 * RT - 1) / (32 * RT);
    const dim3 grid((unsigned)(ntile_c * ntile_r * (MODE == 2 ? 2 : MODE == 3 ? 4 : 1)));
    const size_t wfl = MODE >= 2 ? 0 : (size_t)a.ntypes * CT * (PREC ? 512 : 1024);  // two stages of halves, in floats
    const size_t yfl = MODE == 3 ? std::max((size_t)J * (8 * COLS + 16), (size_t)8 * J * 100)
                       : ATT     ? (size_t)J * (8 * COLS + 16) + 8 * J * 100
                                 : (size_t)J * (16 * (COLS + 4) + 16);
    size_t lds = ((wfl > yfl ? wfl : yfl) + (size_t)J * J + 2 * COLS) * sizeof(float);
    if (lds > 160 * 1024) return hipErrorNotSupported;
    // Every launch takes exactly the LDS it uses and may share its CU with other kernels' workgroups
    // (row chains, concurrent plans): the co-residency hazard of rounds 1-2 was the packed-FP32
    // instructions of the co-resident update kernel, not these tiles (build.py).
    auto kt = rms ? k_gl4<J, NW, RT, CT, true, MODE, PREC, STG> : k_gl4<J, NW, RT, CT, false, MODE, PREC, STG>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    g_route_bits |= MODE >= 2 ? kRouteMixPhase : MODE == 1 ? kRouteFusedAttn : kRouteOneKernel;
    hipLaunchKernelGGL(kt, grid, dim3(NW * 64), lds, s, a);
    return hipGetLastError();
}

// SKELDIFF_GL4_CFG = <NW><RT><CT> (e.g. 822): process default of the plans' v4 tile (tuning);
// 0/unset = per shape.
static int g_gl4_cfg = [] {
    const char* e = getenv("SKELDIFF_GL4_CFG");
    return e ? atoi(e) : 0;
}();
int gl4_tile_default() { return g_gl4_cfg; }

// ---- split route (small grids) -------------------------------------------------
// A one-kernel launch is one workgroup's K-loop latency however few workgroups it has: at 50
// rows an N = 192 layer is 12 workgroups on 256 CUs.  The split route runs phase 1 (k_gl4y, one
// wave per (32-row tile, node, 32-column tile): J x more parallel work, no LDS) into the zs
// scratch and phase 2 (k_gl4 MODE 2: mixing + FiLM / tanh / residual per 16-row slab, or MODE 3:
// the attention epilogue per 8-row slab).  Same arithmetic in the same order as the one-kernel
// route, so the results are bitwise identical and the route can follow the shard size.
// Auto threshold on the rows of the whole sampling call (all row chains; GLArgs::route_rows):
// process default SKELDIFF_SPLIT_ROWS = 1200.  Measured (round 4, same box, T = 100, J = 16 f32,
// tools/sweep_routes.py, profiles/r04j/sweep.txt; k_gl4y with every chunk in flight): 800 rows
// 9,648 futures/s (k_gl4y, 2 chains) vs 7,737 (k_gl4t, 3); 1,600 rows 12,109 vs 12,172 (equal);
// 400 rows 6,165 vs 4,361.
static int64_t g_split_rows = [] {
    const char* e = getenv("SKELDIFF_SPLIT_ROWS");
    return e ? (int64_t)atoll(e) : (int64_t)1200;
}();
int64_t split_rows_default() { return g_split_rows; }

// 0: one-kernel route; 1: split route with the per-wave phase 1 (k_gl4y, small grids); 2: split
// route with the tiled phase 1 (k_gl4t, full batches).  GLArgs::split: 0 auto, 1 never, 2 always
// (k_gl4y), 3 always (k_gl4t).
static int split_route(const GLArgs& a, bool attn) {
    // norm_type 'layer': the Block LayerNorm runs in the split route's mixing phase only, so such a
    // layer takes a split route whatever SD_OPT_SPLIT_ROUTE 1 / a gl4_tile option / half or bf16
    // precision would choose (launch_graph_linear_v4 never hands it to a one-kernel tile)
    const bool ln = a.ln_w != nullptr;
    if ((a.split == 1 && !ln) || !a.zs || (a.N & 31) || a.J > 32) return 0;
    const int64_t tiles = (a.B + 31) / 32;
    if (tiles * 32 * a.J * (int64_t)a.N > a.zs_cap) return 0;
    if (a.zs == a.out || a.zs == a.x1 || a.zs == a.x2 || a.zs == a.res) return 0;
    if (attn && (a.attn_heads * 96 != a.N)) return 0;
    if (a.prec == 2 && a.split < 3 && !(a.split == 0 && a.J == 17)) return ln ? 2 : 0;  // bf16: tiled only (J = 17 auto)
    if (a.split == 2) return a.prec == 2 ? 0 : 1;
    if (a.split == 3) return 2;
    if (a.split == 4) return attn ? 0 : 2;  // tiled GEMM phase; to_qkv + attention on the one-kernel tile
    if (a.gl4_cfg != 0 && !ln) return 0;
    const int64_t rows = a.route_rows > 0 ? a.route_rows : a.B;
    if (rows <= g_split_rows) return a.prec == 2 ? (ln ? 2 : 0) : 1;
    // J = 17 / 21 full batches (f32 and half; bf16 at J = 17): the tiled route on one chain measured
    // faster than the one-kernel route on three (FreeMan J = 17 10,954 vs 9,547, AMASS J = 21 8,567
    // vs 8,371 futures/s at 3,200 rows, T = 100; config 5 half 133,002 vs 92,456, bf16 134,084 vs
    // 120,821; AMASS J = 21 bf16 9,563 vs 9,946 keeps the one-kernel route; DESIGN.md §4d'')
    // J = 16 (f32): the tiled route above the split-route threshold (three row chains sharing CUs,
    // round 3, same box: 800 rows 8,146 vs 7,516 futures/s for the one-kernel route, 1,600 rows
    // 12,385 vs 12,473, config 2 15,940 vs 14,972 with the fused one-kernel attention tile); in
    // half / bf16 mode the one-kernel tiles stay
    if (a.J == 16) return a.prec == 0 || ln ? 2 : 0;
    return (a.J == 17 || a.J == 21) ? 2 : 0;
}

template <bool ROWMAJOR, int PF>
static void launch_gl4y_pf(const GLArgs& a, bool rms, int ntc, int64_t ntile_r, const YOut& yo, dim3 grid, hipStream_t s) {
    if (a.prec == 1) {
        if (rms) hipLaunchKernelGGL((k_gl4y<true, 1, ROWMAJOR, PF>), grid, dim3(256), 0, s, a, ntc, ntile_r, yo);
        else hipLaunchKernelGGL((k_gl4y<false, 1, ROWMAJOR, PF>), grid, dim3(256), 0, s, a, ntc, ntile_r, yo);
    } else {
        if (rms) hipLaunchKernelGGL((k_gl4y<true, 0, ROWMAJOR, PF>), grid, dim3(256), 0, s, a, ntc, ntile_r, yo);
        else hipLaunchKernelGGL((k_gl4y<false, 0, ROWMAJOR, PF>), grid, dim3(256), 0, s, a, ntc, ntile_r, yo);
    }
}

template <bool ROWMAJOR>
static hipError_t launch_gl4y(const GLArgs& a, bool rms, int ntc, int64_t ntile_r, const YOut& yo, hipStream_t s) {
    const int64_t units = ntile_r * a.J * ntc;
    const dim3 grid((unsigned)((units + 3) / 4));
    // any chunk count: the v5 GEMM phase (launch_gemm_split) passes K = 16 / 48 (odd nchunk) too
    const int nchunk = (a.K1 + a.K2) / 16;
    if (nchunk < 1 || (a.K1 + a.K2) % 16) return hipErrorNotSupported;
    g_route_bits |= kRouteGemmWave;
    // chunks in flight: a divisor of nchunk (the K loop's rounds: the loop issues unconditionally,
    // so PF must divide nchunk); every chunk of a K = 192 layer in flight on grids of at most one
    // workgroup per CU (the wave pays one memory latency per launch)
    if (grid.x <= 256 && a.prec == 0 && nchunk % 12 == 0)
        launch_gl4y_pf<ROWMAJOR, 12>(a, rms, ntc, ntile_r, yo, grid, s);
    else if (nchunk % 8 == 0) launch_gl4y_pf<ROWMAJOR, 8>(a, rms, ntc, ntile_r, yo, grid, s);
    else if (nchunk % 6 == 0) launch_gl4y_pf<ROWMAJOR, 6>(a, rms, ntc, ntile_r, yo, grid, s);
    else if (nchunk % 4 == 0) launch_gl4y_pf<ROWMAJOR, 4>(a, rms, ntc, ntile_r, yo, grid, s);
    else if (nchunk % 3 == 0) launch_gl4y_pf<ROWMAJOR, 3>(a, rms, ntc, ntile_r, yo, grid, s);
    else if (nchunk % 2 == 0) launch_gl4y_pf<ROWMAJOR, 2>(a, rms, ntc, ntile_r, yo, grid, s);
    else launch_gl4y_pf<ROWMAJOR, 1>(a, rms, ntc, ntile_r, yo, grid, s);
    return hipGetLastError();
}

template <bool ROWMAJOR>
static hipError_t launch_gl4t(const GLArgs& a, bool rms, int64_t ntile_r, const YOut& yo, hipStream_t s);

// v5's GEMM phase on split-f16 products (J > 21; sd_graph_linear_v5.hip): z[b, j, n] row-major
// with row stride z_rs, rows < B only.  hipErrorNotSupported without split weights.
hipError_t launch_gemm_split(const GLArgs& a, bool rms, float* z, int64_t z_rs, hipStream_t s) {
    if (!a.wsp || a.prec == 2 || (a.K1 + a.K2) % 16 || a.K1 % 16 || a.x1_blk || a.x2_blk) return hipErrorNotSupported;
    const int64_t ntile_r = (a.B + 31) / 32;
    const int ntc = (a.N + 31) / 32;
    const YOut yo{z, z_rs, a.N, 32 * z_rs, 32};
    // the tiled phase (128 rows x up to 192 columns of one node per workgroup) where the shape
    // has one
    if (((uintptr_t)z & 15) == 0 && (z_rs & 3) == 0 && (a.N & 3) == 0) {  // 16-B Y pieces
        const hipError_t e = launch_gl4t<true>(a, rms, ntile_r, yo, s);
        if (e != hipErrorNotSupported) return e;
    }
    return launch_gl4y<true>(a, rms, ntc, ntile_r, yo, s);
}

template <int CT, int NCH, bool ROWMAJOR, int RT, int PF = 2>
static hipError_t launch_gl4t_v(const GLArgs& a, bool rms, int64_t ntile_r, const YOut& yo, hipStream_t s) {
    const int ncg = a.N / (32 * CT);  // column groups
    const dim3 grid((unsigned)(((ntile_r + 4 * RT - 1) / (4 * RT)) * a.J * ncg)), block(256);
    auto kt = a.prec == 1 ? (rms ? k_gl4t<true, 1, CT, NCH, ROWMAJOR, RT, PF> : k_gl4t<false, 1, CT, NCH, ROWMAJOR, RT, PF>)
                          : (rms ? k_gl4t<true, 0, CT, NCH, ROWMAJOR, RT, PF> : k_gl4t<false, 0, CT, NCH, ROWMAJOR, RT, PF>);
    if constexpr (!ROWMAJOR && RT == 1) {  // bf16 mode (precision 2): the split route's scratch output only
        if (a.prec == 2) kt = rms ? k_gl4t<true, 2, CT, NCH, false, 1, 2> : k_gl4t<false, 2, CT, NCH, false, 1, 2>;
    }
    g_route_bits |= kRouteGemmTiled;
    hipLaunchKernelGGL(kt, grid, block, 0, s, a, ncg, ntile_r, yo);
    return hipGetLastError();
}

// the release Denoiser's shapes: K = 192 (12 chunks), 256 (to_out, 16) or 384 (24), N a multiple
// of 96 (192 wide layers, 768 to_qkv, 96 final_glin); hipErrorNotSupported otherwise (k_gl4y).
// N = 192 / 96 (f32 / half): 2 row tiles x 3 column tiles per wave (tools/gl4t_rt_probe.hip: 17.1 vs
// 18.5 us for 1 x 6 at N = 192, 3,200 rows); N = 768 to_qkv: 1 x 6 (53.6 vs 56.4 us for 2 x 3).
// to_qkv (N = 768, K = 192) of the row-major v5 path (J > 21) on 256-column workgroups: 3 column
// groups of 8 tiles instead of 4 of 6 (0.75 of the x re-reads, 24 MFMAs per chunk and wave; MANO
// J = 51 3,757 / 3,766 vs 3,729 / 3,727 futures/s); on the tiled split route it measured slower
// (config 2 16,104 / 16,353 vs 16,498 / 16,375: its 72 KiB workgroups leave less room for the other
// row chains' kernels), profiles/r04_ab/gl4t_ct8.txt
template <bool ROWMAJOR>
static hipError_t launch_gl4t(const GLArgs& a, bool rms, int64_t ntile_r, const YOut& yo, hipStream_t s) {
    const int K = a.K1 + a.K2;
    if (a.K1 % 16 || (a.x1_div != 1 && a.x1_blk)) return hipErrorNotSupported;
    if (ROWMAJOR && a.N % 256 == 0 && K == 192 && a.prec != 2) return launch_gl4t_v<8, 12, ROWMAJOR, 1>(a, rms, ntile_r, yo, s);
    // f16 operands, row-blocked x, N = 96 / 192: 2 row tiles x 3 column tiles per wave (row-major x
    // -- the J > 21 path -- keeps 1 x 6: its x fragments are 16-B pieces of rows J K floats apart,
    // and a second row tile doubled them; MANO N = 192 29.1 vs 26.7 us, profiles/r06h)
#ifndef SD_GL4T_RT2
#define SD_GL4T_RT2 1
#endif
#ifndef SD_GL4T_PF
#define SD_GL4T_PF 2  // chunks in flight of the row-blocked forms (A/B builds: -DSD_GL4T_PF=3 / 4)
#endif
#ifndef SD_GL4T_PF6
#define SD_GL4T_PF6 2
#endif
    constexpr int PFB = ROWMAJOR ? 2 : SD_GL4T_PF, PF6 = ROWMAJOR ? 2 : SD_GL4T_PF6;
    if (!ROWMAJOR && SD_GL4T_RT2 && a.prec != 2 && a.N <= 192 && a.N % 96 == 0) {
        if (K == 192) return launch_gl4t_v<3, 12, ROWMAJOR, 2, PFB>(a, rms, ntile_r, yo, s);
        if (K == 256) return launch_gl4t_v<3, 16, ROWMAJOR, 2, PFB>(a, rms, ntile_r, yo, s);
        if (K == 384) return launch_gl4t_v<3, 24, ROWMAJOR, 2, PFB>(a, rms, ntile_r, yo, s);
    }
    if (a.N % 192 == 0) {
        if (K == 192) return launch_gl4t_v<6, 12, ROWMAJOR, 1, PF6>(a, rms, ntile_r, yo, s);
        if (K == 256) return launch_gl4t_v<6, 16, ROWMAJOR, 1, PF6>(a, rms, ntile_r, yo, s);
        if (K == 384) return launch_gl4t_v<6, 24, ROWMAJOR, 1, PF6>(a, rms, ntile_r, yo, s);
    } else if (a.N % 96 == 0) {
        if (K == 192) return launch_gl4t_v<3, 12, ROWMAJOR, 1>(a, rms, ntile_r, yo, s);
        if (K == 384) return launch_gl4t_v<3, 24, ROWMAJOR, 1>(a, rms, ntile_r, yo, s);
    }
    return hipErrorNotSupported;
}

template <int J>
static hipError_t gl4_split(const GLArgs& a, bool rms, bool attn, int route, hipStream_t s) {
    const int64_t ntile_r = (a.B + 31) / 32;
    const int ntc = a.N / 32;
    const YOut yo{a.zs, 32, 1024, (int64_t)(a.N / 32) * J * 1024, (int64_t)J * 1024};  // column-tiled (zs_off)
    hipError_t e = route == 2 ? launch_gl4t<false>(a, rms, ntile_r, yo, s) : hipErrorNotSupported;
    if (e == hipErrorNotSupported) {
        if (a.prec == 2) return hipErrorNotSupported;  // k_gl4y has no bf16 form
        e = launch_gl4y<false>(a, rms, ntc, ntile_r, yo, s);
    }
    if (e != hipSuccess) return e;
    if (a.prec == 2) {  // bf16 residual / output storage (PREC 2 epilogue)
        if (attn) return gl4_launch_t<J, 8, 1, 3, 3, 2, 0>(a, false, s);
        return gl4_launch_t<J, 8, 1, 1, 2, 2, 0>(a, false, s);
    }
    if (attn) return gl4_launch_t<J, 8, 1, 3, 3, 0, 0>(a, false, s);
    return gl4_launch_t<J, 8, 1, 1, 2, 0, 0>(a, false, s);
}

static hipError_t gl4_split_dispatch(const GLArgs& a, bool rms, bool attn, int route, hipStream_t s) {
    switch (a.J) {
        case 16: return gl4_split<16>(a, rms, attn, route, s);
        case 17: return gl4_split<17>(a, rms, attn, route, s);
        case 21: return gl4_split<21>(a, rms, attn, route, s);
        default: return hipErrorNotSupported;
    }
}

hipError_t launch_graph_linear_v4(const GLArgs& a, bool rms, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    // K1, K2 multiples of 16 and an even number of 16-deep chunks (the K loop is unrolled by 2)
    // 16-B row segments in the epilogue: N, row strides and buffers 16-B aligned
    if ((a.N & 3) || ((uintptr_t)a.out & 15) || ((uintptr_t)a.res & 15) || (a.res && (a.res_rs & 3)) || (a.out_rs & 3))
        return hipErrorNotSupported;
    if (!a.wsp || (a.K1 + a.K2) % 32 || a.K1 % 16 || (a.x1_blk && a.x1_div != 1)) return hipErrorNotSupported;
    if (a.J == 16 || a.J == 17 || a.J == 21)
        if (const int route = split_route(a, false)) {
            const hipError_t e = gl4_split_dispatch(a, rms, false, route, s);
            if (e != hipErrorNotSupported) return e;  // else: nothing launched, the one-kernel route
        }
    if (a.ln_w) return hipErrorNotSupported;  // the Block LayerNorm lives in the split mixing phase only
    const int cfg = a.gl4_cfg ? a.gl4_cfg : a.tile_hint;
    if (a.prec == 2) {  // bf16 mode: row-major operands, the default tiles only
        if (a.x1_blk || a.x2_blk || a.res_blk || a.out_blk) return hipErrorNotSupported;
        switch (a.J) {
            case 16: return gl4_launch<16, 8, 1, 3, 0, 2>(a, rms, s);
            case 17: return gl4_launch<17, 8, 1, 2, 0, 2>(a, rms, s);
            case 21: return gl4_launch<21, 8, 1, 2, 0, 2>(a, rms, s);
            default: return hipErrorNotSupported;
        }
    }
    if (a.prec == 1) {  // half precision mode: the default tiles only
        switch (a.J) {
            case 16:
                if (cfg == 812) return gl4_launch<16, 8, 1, 2, 0, 1>(a, rms, s);
                return gl4_launch<16, 8, 1, 3, 0, 1>(a, rms, s);
            case 17: return gl4_launch<17, 8, 2, 1, 0, 1>(a, rms, s);
            case 21: return gl4_launch<21, 8, 1, 2, 0, 1>(a, rms, s);
            default: return hipErrorNotSupported;
        }
    }
    switch (a.J) {
        case 16:
            if (cfg == 422) return gl4_launch<16, 4, 2, 2>(a, rms, s);
            if (cfg == 412) return gl4_launch<16, 4, 1, 2>(a, rms, s);
            if (cfg == 421) return gl4_launch<16, 4, 2, 1>(a, rms, s);
            if (cfg == 821) return gl4_launch<16, 8, 2, 1>(a, rms, s);
            if (cfg == 812) return gl4_launch<16, 8, 1, 2>(a, rms, s);
            if (cfg == 813) return gl4_launch<16, 8, 1, 3>(a, rms, s);
            if (cfg == 811) return gl4_launch<16, 8, 1, 1>(a, rms, s);  // small batches: 3x the workgroups
            if (cfg == 822) return gl4_launch<16, 8, 2, 2>(a, rms, s);
            // small grids (a few sequences: config 4, one sequence x 50 futures): 32 x 32 tiles give
            // 3x the workgroups of 32 x 96 and a third of the per-workgroup weight bytes; measured
            // 1.69x (59.0 vs 34.9 futures/s at 50 rows, T = 1000), but 0.91x at B = 3200
            if (cfg == 0 && (a.B + 31) / 32 * ((a.N + 95) / 96) < 32) return gl4_launch<16, 8, 1, 1>(a, rms, s);
            // 32 rows x 96 columns: 200 workgroups for an N = 192 layer at B = 3200 (64 x 64 gives
            // 150, leaving 40 % of the CUs idle); measured 1.28x faster on those layers
            return gl4_launch<16, 8, 1, 3>(a, rms, s);
        // J > 16 needs two 16-node blocks in the mixing epilogue: 96 columns spill there
        case 17:
            if (cfg == 821) return gl4_launch<17, 8, 2, 1>(a, rms, s);
            if (cfg == 813) return gl4_launch<17, 8, 1, 3>(a, rms, s);
            return gl4_launch<17, 8, 1, 2>(a, rms, s);
        case 21:
            if (cfg == 813) return gl4_launch<21, 8, 1, 3>(a, rms, s);
            return gl4_launch<21, 8, 1, 2>(a, rms, s);
        default: return hipErrorNotSupported;
    }
}

// to_qkv (RMSNorm-scaled, no bias) + Attention fused; a.out = (B, J, heads * 32) attention
// output.  hipErrorNotSupported where the fused tile does not apply (caller falls back to the
// graph-linear + k_attention pair).
hipError_t launch_qkv_attention_v4(const GLArgs& a, bool rms, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (!a.wsp || a.J > 32 || a.attn_heads < 1 || a.N != 3 * a.attn_heads * 32 || a.bias || a.film || a.res ||
        a.act || (a.K1 + a.K2) % 32 || a.K1 % 16 || ((uintptr_t)a.out & 15) || (a.out_rs & 3))
        return hipErrorNotSupported;
    GLArgs b = a;
    b.attn_order = a.gl4_cfg == 100 ? 1 : 0;
    if (a.J == 16 || a.J == 17 || a.J == 21)
        if (const int route = split_route(a, true)) {
            const hipError_t e = gl4_split_dispatch(b, rms, true, route, s);
            if (e != hipErrorNotSupported) return e;
        }
    // J = 17 / 21: 3 nodes per wave, two 16-node tiles in the softmax
    switch (a.J) {
        case 16:
            if (a.prec == 2) return gl4_launch<16, 8, 1, 3, 1, 2>(b, rms, s);
            return a.prec == 1 ? gl4_launch<16, 8, 1, 3, 1, 1>(b, rms, s) : gl4_launch<16, 8, 1, 3, 1>(b, rms, s);
        case 17:
            if (a.prec == 2) return gl4_launch<17, 8, 1, 3, 1, 2>(b, rms, s);
            return a.prec == 1 ? gl4_launch<17, 8, 1, 3, 1, 1>(b, rms, s) : gl4_launch<17, 8, 1, 3, 1>(b, rms, s);
        case 21:  // 13 node types: 2 x 78 KB weight stages + G-hat + FiLM = 158.5 KB of LDS
            if (a.prec == 2) return gl4_launch<21, 8, 1, 3, 1, 2>(b, rms, s);
            return a.prec == 1 ? gl4_launch<21, 8, 1, 3, 1, 1>(b, rms, s) : gl4_launch<21, 8, 1, 3, 1>(b, rms, s);
        default: return hipErrorNotSupported;
    }
}

}  // namespace sd

