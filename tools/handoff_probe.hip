// Price of one inter-workgroup hand-off inside a launch vs a dependent kernel boundary (VERDICT r04
// item 3).  Ping-pong between two workgroups of one wave each (block 0 and block P):
// per round, A publishes (payload + flag), B waits for the flag, consumes the payload (and checks
// every word), then answers with a flag of its own; A waits for the answer.  One round = two
// hand-offs.  P = 8 puts the pair on one XCD, P = 1 on two (round-robin dealing, observed; each
// block records its s_getreg XCC_ID and the host prints the pair it actually got).
// Publish / consume forms:
//   flag      no payload, relaxed agent-scope atomic flag store / poll
//   rel       4 KiB payload by plain stores, agent release fence, flag; consumer acquire fence, plain loads
//   sc1       4 KiB payload by sc1 (write-through) stores + vmcnt(0), flag; consumer sc1 loads, no fences
//   l2plain   4 KiB payload by PLAIN stores + vmcnt(0), flag; consumer sc1 loads, no fences -- valid
//             only when both sides share an XCD's L2 (the probe counts stale words to show it)
// Every spin is bounded (a timed-out round is counted, never hangs).  The kernel boundary: 2,000
// back-to-back launches of a trivial 256-workgroup kernel on one stream (eager) and the same as a
// 100-node hipGraph replayed 20 times, timed with hipEvents.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/handoff_probe.hip -o tools/handoff_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef __attribute__((address_space(1))) unsigned gu32;
enum Form { FLAG = 0, REL = 1, SC1 = 2, L2PLAIN = 3 };
constexpr int WORDS = 1024;                 // 4 KiB payload: 16 floats per lane
constexpr unsigned long long SPIN_CAP = 1ull << 21;

__device__ __forceinline__ bool wait_eq(gu32* f, unsigned v, unsigned* tmo) {
    for (unsigned long long i = 0; i < SPIN_CAP; ++i) {
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == v) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    atomicAdd(tmo, 1u);
    return false;
}

template <int F>
__global__ __launch_bounds__(64) void k_pingpong(gu32* fa, gu32* fb, float* payload, int peer, int iters,
                                                 unsigned* xcc, unsigned long long* ticks, unsigned* stale,
                                                 unsigned* tmo) {
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b != 0 && b != peer) return;
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    if (lane == 0) xcc[b == 0 ? 0 : 1] = x & 0xf;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(payload, 0, WORDS * 4, 0x00020000);
    unsigned bad = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= iters; ++i) {
        if (b == 0) {  // A: publish round i, wait for the answer
            if (F != FLAG) {
#pragma unroll
                for (int k = 0; k < WORDS / 256; ++k) {
                    const float4 v = make_float4((float)i, (float)i, (float)i, (float)i);
                    const int off = (k * 64 + lane) * 16;
                    if (F == SC1)
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                               rsrc, off, 0, 16);
                    else
                        *reinterpret_cast<float4*>(payload + off / 4) = v;
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (F == REL) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            if (lane == 0) __hip_atomic_store(fa, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!wait_eq(fb, (unsigned)i, tmo)) break;
        } else {  // B: consume round i, answer
            if (!wait_eq(fa, (unsigned)i, tmo)) break;
            if (F == REL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (F != FLAG) {
#pragma unroll
                for (int k = 0; k < WORDS / 256; ++k) {
                    const int off = (k * 64 + lane) * 16;
                    float4 v;
                    if (F == REL)
                        v = *reinterpret_cast<const float4*>(payload + off / 4);
                    else
                        v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 16));
                    bad += (v.x != (float)i) + (v.y != (float)i) + (v.z != (float)i) + (v.w != (float)i);
                }
            }
            if (lane == 0) __hip_atomic_store(fb, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (bad) atomicAdd(stale, bad);
    if (b == 0 && lane == 0) *ticks = t1 - t0;
}

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0x7fffffff) *p = 1;
}

template <int F>
static void pingpong(const char* name, int peer, int iters) {
    unsigned *fa, *fb, *xcc, *stale, *tmo;
    float* payload;
    unsigned long long* ticks;
    CHECK(hipMalloc(&fa, 256));
    CHECK(hipMalloc(&fb, 256));
    CHECK(hipMalloc(&payload, WORDS * 4));
    CHECK(hipMalloc(&xcc, 16));
    CHECK(hipMalloc(&ticks, 8));
    CHECK(hipMalloc(&stale, 4));
    CHECK(hipMalloc(&tmo, 4));
    CHECK(hipMemset(fa, 0, 256));
    CHECK(hipMemset(fb, 0, 256));
    CHECK(hipMemset(payload, 0, WORDS * 4));
    CHECK(hipMemset(stale, 0, 4));
    CHECK(hipMemset(tmo, 0, 4));
    hipLaunchKernelGGL(k_pingpong<F>, dim3(16), dim3(64), 0, 0, (gu32*)fa, (gu32*)fb, payload, peer, iters, xcc, ticks,
                       stale, tmo);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned hx[2], hs, ht;
    unsigned long long tk;
    CHECK(hipMemcpy(hx, xcc, 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&hs, stale, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&ht, tmo, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&tk, ticks, 8, hipMemcpyDeviceToHost));
    // s_memrealtime: 100 MHz
    printf("%-8s pair XCD %u -> %u (%s)  one hand-off %6.3f us  (%d rounds)  stale words %u  timeouts %u\n", name, hx[0],
           hx[1], hx[0] == hx[1] ? "same XCD " : "cross-XCD", tk * 10e-3 / (2.0 * iters), iters, hs, ht);
    CHECK(hipFree(fa));
    CHECK(hipFree(fb));
    CHECK(hipFree(payload));
    CHECK(hipFree(xcc));
    CHECK(hipFree(ticks));
    CHECK(hipFree(stale));
    CHECK(hipFree(tmo));
}

int main() {
    const int iters = 2000;
    for (int peer : {8, 1}) {
        pingpong<FLAG>("flag", peer, iters);
        pingpong<REL>("rel", peer, iters);
        pingpong<SC1>("sc1", peer, iters);
        pingpong<L2PLAIN>("l2plain", peer, iters);
    }
    // dependent kernel boundary: trivial 256-workgroup kernels back to back
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t a, e;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&e));
    for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
    CHECK(hipStreamSynchronize(s));
    const int n = 2000;
    CHECK(hipEventRecord(a, s));
    for (int w = 0; w < n; ++w) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
    CHECK(hipEventRecord(e, s));
    CHECK(hipEventSynchronize(e));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, e));
    printf("kernel boundary, eager: %6.3f us per trivial 256-workgroup launch (%d launches)\n", ms * 1e3 / n, n);
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, nullptr);
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(a, s));
    for (int r = 0; r < 20; ++r) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipEventRecord(e, s));
    CHECK(hipEventSynchronize(e));
    CHECK(hipEventElapsedTime(&ms, a, e));
    printf("kernel boundary, hipGraph: %6.3f us per node (100-node graph x 20 replays)\n", ms * 1e3 / 2000);
    return 0;
}
