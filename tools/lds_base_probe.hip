// Probe for DESIGN.md §4c, second hypothesis: does a small-LDS kernel shaped like k_update
// (static J x J tables filled by ds_write, then wave-uniform ds_read_b128 broadcasts with
// immediate offsets) compute correctly when a co-resident workgroup holding a large LDS
// allocation pushes its LDS base up (past 64 KB)?
//
// hog:      one workgroup per CU with H KB of dynamic LDS, touches it, sleeps ~2 ms (no LDS-DMA);
// upd_like: k_update's table pattern: sC1/sC2/sU (16 x 16 f32) + sS (16) staged from global,
//           out[row][i][d] = sum_j C1[i][j] x[j][d] + C2[i][j] y[j][d] + U[i][j] (s_j e[j][d]).
// Each case runs upd_like alone (reference) and then launched right after a hog on another
// stream; prints differing outputs and the LDS bases both kernels saw (HW_REG_LDS_ALLOC).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/lds_base_probe tools/lds_base_probe.hip
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

__global__ void hog(unsigned* alloc_out, int words, int sleeps) {
    extern __shared__ unsigned hb[];
    for (int i = threadIdx.x; i < words; i += blockDim.x) hb[i] = i;
    __syncthreads();
    for (int s = 0; s < sleeps; ++s) __builtin_amdgcn_s_sleep(127);
    if (threadIdx.x == 0) alloc_out[blockIdx.x] = lds_alloc_reg() + (hb[words - 1] != (unsigned)(words - 1));
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
    CHECK(hipFuncSetAttribute((const void*)hog, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int J = 16, D = 96, rows = 4096;
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
    unsigned *halloc, *ualloc;
    CHECK(hipMalloc(&halloc, cus * 4));
    CHECK(hipMalloc(&ualloc, grid * 4));
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
    printf("CUs %d, upd_like grid %d x 256\n", cus, grid);
    unsigned long long total = 0;
    for (int hk : {0, 32, 48, 60, 63, 64, 65, 66, 72, 80, 82, 96, 100, 122, 128, 140, 150}) {
        for (int rep = 0; rep < 3; ++rep) {
            CHECK(hipMemset(out, 0, n * 4));
            CHECK(hipMemset(ualloc, 0, grid * 4));
            CHECK(hipDeviceSynchronize());
            if (hk) hipLaunchKernelGGL(hog, dim3(cus), dim3(256), hk * 1024, s1, halloc, hk * 256, 300);
            for (int k = 0; k < 20; ++k) run_upd(out, s2);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
            std::vector<unsigned> ua(grid), ha(cus);
            CHECK(hipMemcpy(ua.data(), ualloc, grid * 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(ha.data(), halloc, cus * 4, hipMemcpyDeviceToHost));
            size_t bad = 0, first = (size_t)-1;
            double mx = 0;
            for (size_t i = 0; i < n; ++i)
                if (got[i] != ref[i]) {
                    ++bad;
                    if (first == (size_t)-1) first = i;
                    mx = std::fmax(mx, std::fabs((double)got[i] - ref[i]));
                }
            unsigned maxbase = 0;
            for (unsigned a : ua) maxbase = std::max(maxbase, a & 0xFFF);
            total += bad;
            printf("hog %3d KB rep %d: %8zu outputs differ (max %.3g, first %zd); upd_like max base field %u (x256 B = "
                   "%u B); hog0 alloc %08x\n",
                   hk, rep, bad, mx, bad ? (ssize_t)first : (ssize_t)-1, maxbase, maxbase * 256, hk ? ha[0] : 0);
            fflush(stdout);
        }
    }
    printf("TOTAL differing %llu\n", total);
    return 0;
}
