// Block -> XCD placement across consecutive launches on one stream (speed only):
// each block records s_getreg(HW_REG_XCC_ID); the host prints, per launch, the XCD of block 0 and
// whether block b sits on XCD (xcd(0) + b) % 8 for every b.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void k_probe(int* out) {
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        out[blockIdx.x] = (int)(x & 0xf);
    }
    // a little work so the blocks overlap like a real layer
    volatile float acc = 0.f;
    for (int i = 0; i < 2000; ++i) acc = acc * 0.999f + 1.f;
}

int main() {
    const int grids[] = {400, 1600, 1200, 400, 512, 1024, 8, 256, 1200, 1600};
    int* d = nullptr;
    hipMalloc(&d, 4096 * sizeof(int));
    hipStream_t s;
    hipStreamCreate(&s);
    for (int rep = 0; rep < 2; ++rep)
        for (int g : grids) {
            hipLaunchKernelGGL(k_probe, dim3(g), dim3(256), 0, s, d);
            std::vector<int> h(g);
            hipMemcpyAsync(h.data(), d, g * sizeof(int), hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
            int rr = 1;
            for (int b = 0; b < g; ++b) rr &= h[b] == (h[0] + b) % 8;
            printf("grid %5d: block0 on XCD %d, round-robin from it: %s\n", g, h[0], rr ? "yes" : "no");
        }
    // back-to-back launches without a host sync between them (as in a graph): record both
    int* d2 = nullptr;
    hipMalloc(&d2, 4096 * sizeof(int));
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(k_probe, dim3(400), dim3(256), 0, s, d);
        hipLaunchKernelGGL(k_probe, dim3(1200), dim3(256), 0, s, d2);
        std::vector<int> a(400), b(1200);
        hipMemcpyAsync(a.data(), d, 400 * sizeof(int), hipMemcpyDeviceToHost, s);
        hipMemcpyAsync(b.data(), d2, 1200 * sizeof(int), hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        printf("pair %d: launch A block0 XCD %d, launch B block0 XCD %d\n", rep, a[0], b[0]);
    }
    hipFree(d);
    hipFree(d2);
    return 0;
}
