// Probe for DESIGN.md §4c (round 2): two kernels that share nothing but CUs.
//
// mfma:   k_gl4y's shape -- per wave a 32x32 f32 accumulator over C chunks of
//         v_mfma_f32_32x32x16_f16 (3 per chunk), x / w fragments streamed from global memory
//         PF chunks ahead into registers, no LDS; result to global memory;
// tables: k_update's shape -- 3 J x J tables + J scales in LDS (ds_write, barrier, ds_read
//         broadcasts), per thread J-long register vectors, VALU FMAs; result to global memory.
// Each kernel first runs alone (reference), then both run repeatedly on two streams so their
// workgroups share CUs; every output is compared with its reference bit for bit.  Variants:
// mfma with its accumulator in AGPRs (compiler default here) or forced through VGPRs by an
// inline-asm copy, tables with / without LDS.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o build/coresidency_probe tools/coresidency_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

template <int PF>
__global__ __launch_bounds__(256) void k_mfma(const float* __restrict__ x, const _Float16* __restrict__ w, float* out,
                                             int nchunk) {
    const int lane = threadIdx.x & 63;
    const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const float* xr = x + (u % 64) * (int64_t)nchunk * 1024 + lane * 8;
    const _Float16* wr = w + (u % 16) * (int64_t)nchunk * 1024 + lane * 8;
    floatx4 xa[PF], xb[PF];
    halfx8 wh[PF], wl[PF];
    auto issue = [&](int c, int sl) {
        xa[sl] = *reinterpret_cast<const floatx4*>(xr + c * 1024);
        xb[sl] = *reinterpret_cast<const floatx4*>(xr + c * 1024 + 4);
        wh[sl] = *reinterpret_cast<const halfx8*>(wr + c * 1024);
        wl[sl] = *reinterpret_cast<const halfx8*>(wr + c * 1024 + 512);
    };
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int i = 0; i < PF; ++i)
        if (i < nchunk) issue(i, i);
    for (int c0 = 0; c0 < nchunk; c0 += PF) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int c = c0 + i;
            if (c < nchunk) {
                const floatx8 f = {xa[i].x, xa[i].y, xa[i].z, xa[i].w, xb[i].x, xb[i].y, xb[i].z, xb[i].w};
                const halfx8 xh = __builtin_convertvector(f, halfx8);
                const halfx8 xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh[i], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl[i], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh[i], acc, 0, 0, 0);
                if (c + PF < nchunk) issue(c + PF, i);
            }
        }
    }
    float* o = out + u * 1024 + lane;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r * 64] = acc[r];
}

// k_gl4y-like with a large by-value argument block (GLArgs is ~700 B) and a dynamically indexed
// per-wave table in it (GLArgs::ntype[j]): two launches with different arguments on two streams.
struct BigArgs {
    const float* x;
    const _Float16* w;
    float* out;
    int nchunk;
    int sel[64];
    int wrow[64];
    float scale[32];
};

__global__ __launch_bounds__(256) void k_mfma_args(const BigArgs p) {
    constexpr int PF = 8;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t u = (int64_t)blockIdx.x * 4 + wave;
    const int j = (int)(u % 64);
    const int nchunk = p.nchunk;
    const float* xr = p.x + (int64_t)p.wrow[j] * nchunk * 1024 + lane * 8;
    const _Float16* wr = p.w + (int64_t)p.sel[j] * nchunk * 1024 + lane * 8;
    floatx4 xa[PF], xb[PF];
    halfx8 wh[PF], wl[PF];
    auto issue = [&](int c, int sl) {
        xa[sl] = *reinterpret_cast<const floatx4*>(xr + c * 1024);
        xb[sl] = *reinterpret_cast<const floatx4*>(xr + c * 1024 + 4);
        wh[sl] = *reinterpret_cast<const halfx8*>(wr + c * 1024);
        wl[sl] = *reinterpret_cast<const halfx8*>(wr + c * 1024 + 512);
    };
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int i = 0; i < PF; ++i)
        if (i < nchunk) issue(i, i);
    for (int c0 = 0; c0 < nchunk; c0 += PF) {
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const int c = c0 + i;
            if (c < nchunk) {
                const floatx8 f = {xa[i].x, xa[i].y, xa[i].z, xa[i].w, xb[i].x, xb[i].y, xb[i].z, xb[i].w};
                const halfx8 xh = __builtin_convertvector(f, halfx8);
                const halfx8 xl = __builtin_convertvector(f - __builtin_convertvector(xh, floatx8), halfx8);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wh[i], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, wl[i], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, wh[i], acc, 0, 0, 0);
                if (c + PF < nchunk) issue(c + PF, i);
            }
        }
    }
    float* o = p.out + u * 1024 + lane;
    const float sc = p.scale[j & 31];
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r * 64] = acc[r] * sc;
}

template <bool LDS>
__global__ __launch_bounds__(256) void k_tables(const float* C, const float* x, float* out, int rows) {
    constexpr int J = 16, D = 96, DP = 48;
    __shared__ float sC1[J * J], sC2[J * J], sU[J * J], sS[J];
    if (LDS) {
        for (int i = threadIdx.x; i < J * J; i += 256) {
            sC1[i] = C[i];
            sC2[i] = C[256 + i];
            sU[i] = C[512 + i];
        }
        for (int i = threadIdx.x; i < J; i += 256) sS[i] = C[768 + i];
        __syncthreads();
    }
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = g / DP;
    if (row >= rows) return;
    const int d = 2 * (int)(g % DP);
    const int64_t rb = row * (int64_t)J * D;
    floatx2 a[J], b[J], e[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
        a[j] = *reinterpret_cast<const floatx2*>(x + rb + j * D + d);
        b[j] = *reinterpret_cast<const floatx2*>(x + rows * J * D + rb + j * D + d);
        e[j] = *reinterpret_cast<const floatx2*>(x + 2 * rows * J * D + rb + j * D + d) * (LDS ? sS[j] : C[768 + j]);
    }
    for (int i = 0; i < J; ++i) {
        floatx2 m1 = {0.f, 0.f}, m2 = {0.f, 0.f}, nz = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < J; ++j) {
            m1 += (LDS ? sC1[i * J + j] : C[i * J + j]) * a[j];
            m2 += (LDS ? sC2[i * J + j] : C[256 + i * J + j]) * b[j];
            nz += (LDS ? sU[i * J + j] : C[512 + i * J + j]) * e[j];
        }
        *reinterpret_cast<floatx2*>(out + rb + i * D + d) = m1 + m2 + nz;
    }
}

static uint32_t st = 12345;
static float rnd() {
    st = st * 1664525u + 1013904223u;
    return (float)((st >> 8) & 0xFFFF) / 65536.0f - 0.5f;
}

int main(int argc, char** argv) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nchunk = 12, mwg = cus * 2, rows = 400;
    const size_t nx = (size_t)64 * nchunk * 1024, nw = (size_t)16 * nchunk * 1024, nmo = (size_t)mwg * 4 * 1024;
    const size_t nt = (size_t)3 * rows * 16 * 96, nto = (size_t)rows * 16 * 96;
    std::vector<float> hx(nx), hc(1024), ht(nt);
    std::vector<_Float16> hw(nw);
    for (auto& v : hx) v = rnd();
    for (auto& v : hw) v = (_Float16)rnd();
    for (auto& v : hc) v = rnd();
    for (auto& v : ht) v = rnd();
    float *dx, *dc, *dt, *mo, *mref, *to, *tref;
    _Float16* dw;
    CHECK(hipMalloc(&dx, nx * 4));
    CHECK(hipMalloc(&dw, nw * 2));
    CHECK(hipMalloc(&dc, 1024 * 4));
    CHECK(hipMalloc(&dt, nt * 4));
    CHECK(hipMalloc(&mo, nmo * 4));
    CHECK(hipMalloc(&mref, nmo * 4));
    CHECK(hipMalloc(&to, nto * 4));
    CHECK(hipMalloc(&tref, nto * 4));
    CHECK(hipMemcpy(dx, hx.data(), nx * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dw, hw.data(), nw * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dc, hc.data(), 1024 * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dt, ht.data(), nt * 4, hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const int tgrid = (rows * 48 + 255) / 256;
    auto run_m = [&](float* o, hipStream_t s) { hipLaunchKernelGGL((k_mfma<8>), dim3(mwg), dim3(256), 0, s, dx, dw, o, nchunk); };
    auto run_t = [&](bool lds, float* o, hipStream_t s) {
        if (lds) hipLaunchKernelGGL((k_tables<true>), dim3(tgrid), dim3(256), 0, s, dc, dt, o, rows);
        else hipLaunchKernelGGL((k_tables<false>), dim3(tgrid), dim3(256), 0, s, dc, dt, o, rows);
    };
    std::vector<float> a(nmo), b(nmo), c(nto), e(nto);
    unsigned long long tot_m = 0, tot_t = 0;
    for (int lds = 1; lds >= 0; --lds) {
        run_m(mref, s1);
        run_t(lds, tref, s2);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(a.data(), mref, nmo * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(c.data(), tref, nto * 4, hipMemcpyDeviceToHost));
        for (int rep = 0; rep < 200; ++rep) {
            CHECK(hipMemset(mo, 0, nmo * 4));
            CHECK(hipMemset(to, 0, nto * 4));
            CHECK(hipDeviceSynchronize());
            // interleave: several table launches while the mfma kernel runs
            for (int k = 0; k < 4; ++k) {
                run_m(mo, s1);
                run_t(lds, to, s2);
            }
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(b.data(), mo, nmo * 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(e.data(), to, nto * 4, hipMemcpyDeviceToHost));
            size_t bm = 0, bt = 0;
            for (size_t i = 0; i < nmo; ++i) bm += memcmp(&a[i], &b[i], 4) != 0;
            for (size_t i = 0; i < nto; ++i) bt += memcmp(&c[i], &e[i], 4) != 0;
            tot_m += bm;
            tot_t += bt;
            if (bm || bt || rep % 50 == 0) {
                printf("tables %s rep %3d: mfma outputs differing %zu / %zu, tables outputs differing %zu / %zu\n",
                       lds ? "LDS " : "noLDS", rep, bm, nmo, bt, nto);
                fflush(stdout);
            }
        }
    }
    printf("TOTAL differing: mfma %llu, tables %llu\n", tot_m, tot_t);
    // two launches of k_mfma_args with different argument blocks on two streams
    {
        BigArgs A{}, B{};
        A.x = B.x = dx;
        A.w = B.w = dw;
        A.nchunk = B.nchunk = nchunk;
        float *oa, *ob, *ra, *rb;
        CHECK(hipMalloc(&oa, nmo * 4));
        CHECK(hipMalloc(&ob, nmo * 4));
        CHECK(hipMalloc(&ra, nmo * 4));
        CHECK(hipMalloc(&rb, nmo * 4));
        for (int j = 0; j < 64; ++j) {
            A.sel[j] = j % 16;
            B.sel[j] = (j * 7 + 3) % 16;
            A.wrow[j] = j;
            B.wrow[j] = 63 - j;
        }
        for (int j = 0; j < 32; ++j) {
            A.scale[j] = 1.0f + j;
            B.scale[j] = -1.0f - j;
        }
        auto la = [&](float* o, hipStream_t s) { A.out = o; hipLaunchKernelGGL(k_mfma_args, dim3(mwg), dim3(256), 0, s, A); };
        auto lb = [&](float* o, hipStream_t s) { B.out = o; hipLaunchKernelGGL(k_mfma_args, dim3(mwg), dim3(256), 0, s, B); };
        la(ra, s1);
        CHECK(hipDeviceSynchronize());
        lb(rb, s1);
        CHECK(hipDeviceSynchronize());
        std::vector<float> r1(nmo), r2(nmo), g1(nmo), g2(nmo);
        CHECK(hipMemcpy(r1.data(), ra, nmo * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(r2.data(), rb, nmo * 4, hipMemcpyDeviceToHost));
        unsigned long long ta = 0, tb = 0;
        for (int rep = 0; rep < 200; ++rep) {
            CHECK(hipMemset(oa, 0, nmo * 4));
            CHECK(hipMemset(ob, 0, nmo * 4));
            CHECK(hipDeviceSynchronize());
            for (int k = 0; k < 6; ++k) {
                la(oa, s1);
                lb(ob, s2);
            }
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(g1.data(), oa, nmo * 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(g2.data(), ob, nmo * 4, hipMemcpyDeviceToHost));
            size_t b1 = 0, b2 = 0;
            for (size_t i = 0; i < nmo; ++i) {
                b1 += memcmp(&r1[i], &g1[i], 4) != 0;
                b2 += memcmp(&r2[i], &g2[i], 4) != 0;
            }
            ta += b1;
            tb += b2;
            if (b1 || b2 || rep % 50 == 0) {
                printf("two-launch rep %3d: A differing %zu, B differing %zu (of %zu)\n", rep, b1, b2, nmo);
                fflush(stdout);
            }
        }
        printf("TOTAL two-launch differing: A %llu, B %llu\n", ta, tb);
    }
    return 0;
}
