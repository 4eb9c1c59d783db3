// Compiler pitfall probe (ROCm 7.2 clang, gfx950): __builtin_bit_cast(int, v[e]) of an
// ext_vector_type element subscript reads element 0 for every e -- the kernel below loads ONE dword
// and reads lanes of it for all four e.  Through a scalar (float x = v[e]; __float_as_int(x)) the
// four elements are read.  k_attention's tail form (sd_kernels.hip) hit this.  Inspect with:
//   hipcc -c --offload-arch=gfx950 -O3 --save-temps tools/readlane_probe.hip -o /tmp/rl.o
//   grep -n 'readlane\|global_load' readlane_probe-hip-amdgcn-amd-amdhsa-gfx950.s
#include <hip/hip_runtime.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k(const floatx4* in, float* out) {
    floatx4 a = in[threadIdx.x];
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const float kk = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a[e]), 16 * g));
            acc = fmaf(kk, (float)(e + g), acc);
        }
    out[threadIdx.x] = acc;
}
