// On-device evaluation metrics over the sampler's outputs ("next" #2): the
// reference's multimodal metrics computed where the latents already are, one workgroup per
// sequence, fixed summation order (deterministic).
//   pairwise: mean over the sample pairs i < j of the L1 (lat_apd, multimodal.py:137-151) and
//             L2 (apd, multimodal.py:15-35) distances between the flattened samples;
//   ade / fde: per sample the mean over frames (ade, multimodal.py:44-57) or the last frame
//             (fde, :60-73) of the L2 distance to the target, then the minimum over samples;
//   mmade / mmfde: the same minimum against each of a sequence's multimodal ground truths,
//             averaged over them (multimodal.py:108-135): one workgroup per (sequence, gt) pair,
//             then a fixed-order mean per sequence.
// Samples are (S, X) rows of one sequence, X = T_frames * F (flattened frame-major, as
// `pred.reshape(batch, n_samples, seq_length, -1)`).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sd_internal.h"

namespace sd {

namespace {

constexpr int kMaxSamples = 64;
constexpr int kChunk = 64;  // features staged per step

// pair p (0 <= p < S(S-1)/2) -> (i, j), i < j, row-major over the upper triangle
__device__ __forceinline__ void pair_of(int p, int S, int& i, int& j) {
    int r = 0, base = 0;
    while (base + (S - 1 - r) <= p) {
        base += S - 1 - r;
        ++r;
    }
    i = r;
    j = r + 1 + (p - base);
}

__global__ __launch_bounds__(256) void k_pairwise(const float* __restrict__ x, int S, int64_t X,
                                                  float* __restrict__ l1_mean, float* __restrict__ l2_mean) {
    __shared__ float tile[kMaxSamples * kChunk];
    __shared__ float red1[kMaxSamples * (kMaxSamples - 1) / 2];
    __shared__ float red2[kMaxSamples * (kMaxSamples - 1) / 2];
    const int tid = threadIdx.x;
    const int P = S * (S - 1) / 2;
    const float* xs = x + (int64_t)blockIdx.x * S * X;
    constexpr int PPT = (kMaxSamples * (kMaxSamples - 1) / 2 + 255) / 256;  // pairs per thread
    float s1[PPT], s2[PPT];
    int pi[PPT], pj[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        s1[k] = s2[k] = 0.f;
        const int p = tid + 256 * k;
        pi[k] = pj[k] = 0;
        if (p < P) pair_of(p, S, pi[k], pj[k]);
    }
    for (int64_t f0 = 0; f0 < X; f0 += kChunk) {
        const int n = (int)min((int64_t)kChunk, X - f0);
        __syncthreads();
        for (int e = tid; e < S * kChunk; e += 256) {
            const int s = e / kChunk, f = e - s * kChunk;
            tile[e] = f < n ? xs[(int64_t)s * X + f0 + f] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PPT; ++k) {
            if (tid + 256 * k >= P) continue;
            const float* a = tile + pi[k] * kChunk;
            const float* b = tile + pj[k] * kChunk;
            float t1 = 0.f, t2 = 0.f;
            for (int f = 0; f < kChunk; ++f) {
                const float d = a[f] - b[f];
                t1 += fabsf(d);
                t2 = fmaf(d, d, t2);
            }
            s1[k] += t1;
            s2[k] += t2;
        }
    }
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        const int p = tid + 256 * k;
        if (p < P) {
            red1[p] = s1[k];
            red2[p] = sqrtf(s2[k]);
        }
    }
    __syncthreads();
    if (tid == 0) {
        double a = 0.0, b = 0.0;
        for (int p = 0; p < P; ++p) {
            a += red1[p];
            b += red2[p];
        }
        if (l1_mean) l1_mean[blockIdx.x] = (float)(a / P);
        if (l2_mean) l2_mean[blockIdx.x] = (float)(b / P);
    }
}

// pred (S, T, F) per sequence, target (T, F): per sample mean_t ||pred - target|| (ade) and the
// last frame's distance (fde), minimum over samples
// pair_seq (nullable): workgroup b compares target b with pred sequence pair_seq[b] (mm metrics)
__global__ __launch_bounds__(256) void k_ade_fde(const float* __restrict__ pred, const float* __restrict__ target,
                                                 int S, int T, int64_t F, float* __restrict__ ade,
                                                 float* __restrict__ fde, float* __restrict__ per_sample_ade,
                                                 float* __restrict__ per_sample_fde,
                                                 const int64_t* __restrict__ pair_seq) {
    __shared__ float sum_t[kMaxSamples], last_t[kMaxSamples];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t seq = pair_seq ? pair_seq[blockIdx.x] : (int64_t)blockIdx.x;
    const float* ps = pred + seq * S * T * F;
    const float* tg = target + (int64_t)blockIdx.x * T * F;
    for (int s = wave; s < S; s += 4) {
        float acc_t = 0.f, last = 0.f;
        for (int t = 0; t < T; ++t) {
            float d2 = 0.f;
            for (int64_t f = lane; f < F; f += 64) {
                const float d = ps[((int64_t)s * T + t) * F + f] - tg[(int64_t)t * F + f];
                d2 = fmaf(d, d, d2);
            }
            for (int o = 32; o > 0; o >>= 1) d2 += __shfl_xor(d2, o);
            const float dn = sqrtf(d2);
            acc_t += dn;
            if (t == T - 1) last = dn;
        }
        if (lane == 0) {
            sum_t[s] = acc_t;
            last_t[s] = last;
        }
    }
    __syncthreads();
    if (per_sample_ade)
        for (int s = tid; s < S; s += 256) per_sample_ade[(int64_t)blockIdx.x * S + s] = sum_t[s] / T;
    if (per_sample_fde)
        for (int s = tid; s < S; s += 256) per_sample_fde[(int64_t)blockIdx.x * S + s] = last_t[s];
    if (tid == 0) {
        float best = INFINITY, bestf = INFINITY;
        for (int s = 0; s < S; ++s) {
            best = fminf(best, sum_t[s] / T);
            bestf = fminf(bestf, last_t[s]);
        }
        if (ade) ade[blockIdx.x] = best;
        if (fde) fde[blockIdx.x] = bestf;
    }
}

// per sequence the mean of its pairs' values in pair order (offsets: nseq + 1); 0 pairs -> NaN
// (the mean of an empty tensor, as torch)
__global__ __launch_bounds__(256) void k_segment_mean(const float* __restrict__ v, const int64_t* __restrict__ off,
                                                      int64_t nseq, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nseq) return;
    const int64_t a = off[i], b = off[i + 1];
    float acc = 0.f;
    for (int64_t k = a; k < b; ++k) acc += v[k];
    out[i] = b > a ? acc / (float)(b - a) : __builtin_nanf("");
}

// ---- best-of-k training relaxation (reference trainer.py:207-222, get_ksimilarity_loss) ----------
// Per sequence the index of the smallest similarity among its k samples -- torch.min(dim).indices:
// the first minimum, and the first NaN if there is one (torch's min propagates NaN) -- and the
// diffusion loss at that index (torch.gather).  sim == loss in the latent space.
__global__ __launch_bounds__(256) void k_best_of_k(const float* __restrict__ sim, const float* __restrict__ loss,
                                                   int64_t nseq, int k, int64_t* __restrict__ idx,
                                                   float* __restrict__ sel) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nseq) return;
    const float* v = sim + b * k;
    int best = 0;
    float bv = v[0];
    for (int j = 1; j < k; ++j) {
        const float x = v[j];
        if (bv != bv) break;                  // a NaN already selected: the first NaN wins
        if (x != x || x < bv) {
            best = j;
            bv = x;
        }
    }
    if (idx) idx[b] = best;
    if (sel) sel[b] = loss[b * k + best];
}

// gradient of the gather: d loss[b, j] = d sel[b] at j = idx[b], else 0
__global__ __launch_bounds__(256) void k_best_of_k_bwd(const float* __restrict__ dsel, const int64_t* __restrict__ idx,
                                                       int64_t nseq, int k, float* __restrict__ dloss) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= nseq * k) return;
    const int64_t b = e / k;
    dloss[e] = (e - b * k == idx[b]) ? dsel[b] : 0.f;
}

// AutoEncoder.loss(pred, y, reduction='none') (reference autoencoder.py:80-98): per sample
// mean over frames of the mean over joints of the sum over coordinates of |d| (l1) or d^2 (mse);
// pred (nseq, S, T, J, C), target (nseq, T, J, C) (the future, not repeated).  One wave per
// (sequence, sample); frame sums in frame order.
__global__ __launch_bounds__(256) void k_pose_loss(const float* __restrict__ pred, const float* __restrict__ target,
                                                   int64_t nseq, int S, int T, int J, int C, int mse,
                                                   float* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nseq * S) return;  // wave-uniform
    const int64_t b = w / S;
    const int JC = J * C;
    const float* p = pred + w * (int64_t)T * JC;
    const float* tg = target + b * (int64_t)T * JC;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
        float fr = 0.f;  // sum over joints and coordinates of this frame
        for (int e = lane; e < JC; e += 64) {
            const float d = p[(int64_t)t * JC + e] - tg[(int64_t)t * JC + e];
            fr += mse ? d * d : fabsf(d);
        }
        for (int o = 32; o > 0; o >>= 1) fr += __shfl_xor(fr, o);
        acc += fr / (float)J;
    }
    if (lane == 0) out[w] = acc / (float)T;
}

}  // namespace

hipError_t launch_best_of_k(const float* sim, const float* loss, int64_t nseq, int k, int64_t* idx, float* sel,
                            hipStream_t s) {
    if (nseq <= 0) return hipSuccess;
    if (k < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_best_of_k, dim3((unsigned)((nseq + 255) / 256)), dim3(256), 0, s, sim ? sim : loss, loss,
                       nseq, k, idx, sel);
    return hipGetLastError();
}

hipError_t launch_best_of_k_bwd(const float* dsel, const int64_t* idx, int64_t nseq, int k, float* dloss,
                                hipStream_t s) {
    const int64_t n = nseq * k;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_best_of_k_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dsel, idx, nseq, k, dloss);
    return hipGetLastError();
}

hipError_t launch_pose_loss(const float* pred, const float* target, int64_t nseq, int S, int T, int J, int C, int mse,
                            float* out, hipStream_t s) {
    const int64_t waves = nseq * S;
    if (waves <= 0) return hipSuccess;
    if (T < 1 || J < 1 || C < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pose_loss, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, pred, target, nseq, S, T, J, C,
                       mse, out);
    return hipGetLastError();
}

hipError_t launch_pairwise(const float* x, int64_t nseq, int S, int64_t X, float* l1_mean, float* l2_mean,
                           hipStream_t s) {
    if (nseq <= 0) return hipSuccess;
    if (S < 2 || S > kMaxSamples || X <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pairwise, dim3((unsigned)nseq), dim3(256), 0, s, x, S, X, l1_mean, l2_mean);
    return hipGetLastError();
}

hipError_t launch_ade_fde(const float* pred, const float* target, int64_t nseq, int S, int T, int64_t F, float* ade,
                          float* fde, float* per_sample_ade, float* per_sample_fde, hipStream_t s) {
    if (nseq <= 0) return hipSuccess;
    if (S < 1 || S > kMaxSamples || T < 1 || F <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ade_fde, dim3((unsigned)nseq), dim3(256), 0, s, pred, target, S, T, F, ade, fde,
                       per_sample_ade, per_sample_fde, (const int64_t*)nullptr);
    return hipGetLastError();
}

hipError_t launch_mm_ade_fde(const float* pred, const float* gts, const int64_t* pair_seq, int64_t npairs,
                             const int64_t* seq_off, int64_t nseq, int S, int T, int64_t F, float* pair_ade,
                             float* pair_fde, float* mmade, float* mmfde, hipStream_t s) {
    if (nseq <= 0) return hipSuccess;
    if (S < 1 || S > kMaxSamples || T < 1 || F <= 0 || npairs < 0) return hipErrorInvalidValue;
    if (npairs > 0)
        hipLaunchKernelGGL(k_ade_fde, dim3((unsigned)npairs), dim3(256), 0, s, pred, gts, S, T, F, pair_ade, pair_fde,
                           (float*)nullptr, (float*)nullptr, pair_seq);
    const dim3 g((unsigned)((nseq + 255) / 256));
    if (mmade) hipLaunchKernelGGL(k_segment_mean, g, dim3(256), 0, s, pair_ade, seq_off, nseq, mmade);
    if (mmfde) hipLaunchKernelGGL(k_segment_mean, g, dim3(256), 0, s, pair_fde, seq_off, nseq, mmfde);
    return hipGetLastError();
}

}  // namespace sd
