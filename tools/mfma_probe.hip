// Instruction-mix probe for the split-f16 GEMM phase's chunk body (k_gl4t, sd_graph_linear_v4.hip):
// how many shader cycles one 16-deep k chunk of a wave's work costs when NO memory is involved
// beyond LDS, as a function of the pieces the production chunk carries:
//   M  18 v_mfma_f32_32x32x16_f16 (6 column tiles x 3 split products, each tile's 3 dependent)
//   L  + 12 ds_read_b128 of weight fragments (hi / lo per tile) from LDS, waited per tile pair
//   P  + the same reads issued for the whole chunk first, one lgkmcnt(0) (product-major)
//   X  + the f16 split of the x fragment (cvt, sub, cvt; |x| max for the range guard)
// Each wave runs ITERS chunks back to back; cycles from s_memtime around the loop (wave 0 of
// each workgroup), reported per chunk.  Grid: one workgroup per CU with 4 or 8 waves (1 or 2 per
// SIMD).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

enum { F_LDS = 1, F_PM = 2, F_X = 4 };
constexpr int CT = 6, ITERS = 256;

template <int F, int NW>
__global__ __launch_bounds__(NW * 64, 1) void k_mix(const float* __restrict__ xin, float* __restrict__ out,
                                                      unsigned long long* __restrict__ cyc) {
    __shared__ __attribute__((aligned(16))) _Float16 sW[2][CT * 1024];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 2 * CT * 1024; i += NW * 64) (&sW[0][0])[i] = (_Float16)(0.001f * (i & 63));
    __syncthreads();
    floatx16 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[ct][e] = 0.f;
    floatx8 f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = xin[(lane * 8 + e) & 255];
    halfx8 wr_h[CT], wr_l[CT];  // register weights for the M-only form
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
        wr_h[ct] = *reinterpret_cast<const halfx8*>(&sW[0][ct * 1024 + lane * 8]);
        wr_l[ct] = *reinterpret_cast<const halfx8*>(&sW[0][ct * 1024 + 512 + lane * 8]);
    }
    float amx = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
    for (int it = 0; it < ITERS; ++it) {
        halfx8 xh, xl;
        if constexpr (F & F_X) {
            const floatx8 a = __builtin_elementwise_abs(f);
            amx = fmaxf(amx, fmaxf(fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])), fmaxf(fmaxf(a[4], a[5]), fmaxf(a[6], a[7]))));
            xh = __builtin_convertvector(f, halfx8);
            xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
            f = f * 1.0000001f;  // a new x every chunk (as the x ring delivers)
        } else {
            xh = __builtin_convertvector(f, halfx8);
            xl = xh;
        }
        const _Float16* wt = &sW[it & 1][lane * 8];
        if constexpr (F & F_PM) {
            halfx8 wh[CT], wl[CT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                wh[ct] = *reinterpret_cast<const halfx8*>(wt + ct * 1024);
                wl[ct] = *reinterpret_cast<const halfx8*>(wt + ct * 1024 + 512);
            }
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh[ct], acc[ct], 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl[ct], t, 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh[ct], t, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                halfx8 wh = wr_h[ct], wl = wr_l[ct];
                if constexpr (F & F_LDS) {
                    wh = *reinterpret_cast<const halfx8*>(wt + ct * 1024);
                    wl = *reinterpret_cast<const halfx8*>(wt + ct * 1024 + 512);
                }
                floatx16 t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh, acc[ct], 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl, t, 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh, t, 0, 0, 0);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = amx;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) s += acc[ct][e];
    out[blockIdx.x * NW * 64 + tid] = s;
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int F, int NW>
static void run(const char* name, const float* x, float* out, unsigned long long* cyc, int grid) {
    hipLaunchKernelGGL((k_mix<F, NW>), dim3(grid), dim3(NW * 64), 0, 0, x, out, cyc);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL((k_mix<F, NW>), dim3(grid), dim3(NW * 64), 0, 0, x, out, cyc);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    static unsigned long long h[4096];
    CHECK(hipMemcpy(h, cyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    unsigned long long mn = ~0ull, mx = 0, sum = 0;
    for (int i = 0; i < grid; ++i) {
        mn = h[i] < mn ? h[i] : mn;
        mx = h[i] > mx ? h[i] : mx;
        sum += h[i];
    }
    printf("%-34s waves/SIMD %d  cycles/chunk min %7.1f avg %7.1f max %7.1f  (18 MFMA x 32 = 576 per wave)  %.1f us\n",
           name, NW / 4, (double)mn / ITERS, (double)sum / grid / ITERS, (double)mx / ITERS, ms * 1e3);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main() {
    const int grid = 256;
    float *x, *out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&x, 256 * sizeof(float)));
    CHECK(hipMemset(x, 0, 256 * sizeof(float)));
    CHECK(hipMalloc(&out, grid * 512 * sizeof(float)));
    CHECK(hipMalloc(&cyc, grid * sizeof(unsigned long long)));
    run<0, 4>("M (register weights)", x, out, cyc, grid);
    run<F_LDS, 4>("M + L (per-tile LDS reads)", x, out, cyc, grid);
    run<F_LDS | F_PM, 4>("M + P (chunk reads first)", x, out, cyc, grid);
    run<F_LDS | F_X, 4>("M + L + X (split)", x, out, cyc, grid);
    run<F_LDS | F_PM | F_X, 4>("M + P + X", x, out, cyc, grid);
    run<0, 8>("M (register weights)", x, out, cyc, grid);
    run<F_LDS, 8>("M + L (per-tile LDS reads)", x, out, cyc, grid);
    run<F_LDS | F_PM, 8>("M + P (chunk reads first)", x, out, cyc, grid);
    run<F_LDS | F_X, 8>("M + L + X (split)", x, out, cyc, grid);
    run<F_LDS | F_PM | F_X, 8>("M + P + X", x, out, cyc, grid);
    return 0;
}
