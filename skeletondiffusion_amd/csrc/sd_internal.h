// Internal interfaces between the host plan (sd_plan.hip) and the gfx950 kernels
// (sd_kernels.hip).  Not part of the public ABI (see include/skeldiff.h).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <stdint.h>

namespace sd {

constexpr int kMaxNodes = 64;

#ifdef SD_DEBUG_LDS
// diagnostic build only (build.py debug=True): LDS integrity counters (device, 8 words) that
// GLArgs::dbg / UpdArgs::dbg point to: [0] k_gl4 weight stages vs their global source,
// [1] k_update tables vs global, [2] k_gl4 G-hat table
unsigned* debug_counters();
#endif

// One StaticGraphLinear (graph_structural.py:30-43) with its fused epilogue:
//   y_j   = s_j * (W_type(j) [x1_j | x2_j]) + bias_type(j)        (s_j = 1/max(|x1_j|,1e-12) if RMS)
//   z_i   = sum_j Ghat[i][j] y_j
//   z     = z * (film[n] + 1) + film[H + n]      (ResnetBlock FiLM, attention.py:71-73)
//   z     = act(z)                               (tanh)
//   z    += res                                  (residual, attention.py:16 / :102)
struct GLArgs {
    const float* x1; int64_t x1_rs; int K1; int x1_div;   // row b reads x1 row (b + x1_row0) / x1_div
    int64_t x1_row0;                                      // 0 <= x1_row0 < x1_div (a row chunk's phase)
    int tile_hint;                                        // v4 tile <NW><RT><CT> when gl4_cfg is 0 (0: per shape)
    // per-launch kernel selection (the plan's options, sd_plan_set_option; process defaults for
    // the test entry points): generation 0 auto / 1..5 forced, v4 tile <NW><RT><CT> (0 auto),
    // v4 weight staging 0 LDS-DMA (CU held exclusively) / 1 register-staged (CU shareable)
    int variant, gl4_cfg, gl4_stage;
    // v4 split route (phase 1 GEMM per (tile, node) into the zs scratch, phase 2 mixing epilogue;
    // bitwise identical to the one-kernel route): 0 auto, 1 never, 2 k_gl4y, 3 k_gl4t, 4 k_gl4t
    // except for to_qkv + attention
    int split;
    // v5 (J > 21) mixing pass (SD_OPT_V5_MIX): 0 the matrix-core form k_gl5_mixm, 1 the VALU form
    // k_gl5_mix (the same j-ordered fmaf chains)
    int v5_valu;
    int64_t route_rows;  // rows of the whole sampling call on this device (row chains: all chains); 0 = B
    const float* x2; int64_t x2_rs; int K2;               // optional second input (cat along K)
    const float* W;                                       // (types, N, K1+K2), K contiguous
    const float* bias;                                    // (types, N) or null
    const float* G;                                       // (J, J) Ghat, row-major
    const float* film;                                    // (2N): [scale | shift] or null
    const float* ln_w; const float* ln_b;                 // (J) Block.norm LayerNorm over nodes (norm_type 'layer', v4 only) or null
    const float* res; int64_t res_rs;                     // (B, J, N) or null
    float* out; int64_t out_rs;                           // (B, J, N)
    int64_t B;
    int N;
    int J;
    int act;                                              // 0 none, 1 tanh
    int ntypes;                                           // number of node types (rows of W / N)
    int wrow[kMaxNodes];                                  // type(j) * N  (row offset into W)
    int ntype[kMaxNodes];                                 // type(j)
    // v4 only: W pre-split into f16 hi/lo B fragments (make_split_weights); null -> v4 unusable
    const _Float16* wsp; int wsp_nct; float wsp_unscale;
    int prec;  // v4 products: 0 f32-accurate (3 split f16 products), 1 half (x_hi W'_hi only)
    // fused to_qkv + Attention (launch_qkv_attention_v4): heads of 32 dims, q scale dh^-1/2
    int attn_heads; float attn_scale; int attn_order;
    // v4 only: operand / result layouts, 0 = row-major (B, J, F), 1 = row-blocked (blk_off in
    // sd_graph_linear_v4.hip; rows padded to 32)
    int x1_blk, x2_blk, res_blk, out_blk;
    // v5: scratch for the pre-mix activations when res aliases out (zs_cap floats), or null;
    // v4 split route: the pre-mix Y of phase 1
    float* zs; int64_t zs_cap;
    unsigned* dbg;  // SD_DEBUG_LDS builds only: integrity counters (else unused)
    // v4: bit 0 set (atomicOr) when an activation is outside the f16 range of the split
    // (|x| >= 65504: x_hi would be inf); null = not checked
    unsigned* status;
    // bf16 storage of operands / result (precision mode 2): the tensor
    // holds bf16 elements at the same element offsets (row-major only)
    int x1_bf16, x2_bf16, res_bf16, out_bf16;
    // v5 only (J > 21): run the GEMM phase alone and leave the pre-mix Y in `out` (k_attention_mix
    // mixes the to_qkv layer); hipErrorNotSupported where the route cannot
    int skip_mix = 0;
};
int diag_flags();  // SKELDIFF_DIAG (sd_plan.hip)

// Kernels a sampling call launched (SD_OPT_LAST_ROUTE): every graph-linear / attention launch site
// ORs its bit into this host thread's word while run_denoiser records (eager) or captures (graph).
enum RouteBits : unsigned {
    kRouteOneKernel = 1,   // k_gl4 MODE 0: one-kernel graph-linear tile
    kRouteFusedAttn = 2,   // k_gl4 MODE 1: one-kernel to_qkv + attention
    kRouteGemmWave = 4,    // k_gl4y: small-batch split route, GEMM phase
    kRouteGemmTiled = 8,   // k_gl4t: tiled split route (and v5) GEMM phase
    kRouteMixPhase = 16,   // k_gl4 MODE 2 / 3: split-route mixing / attention phase
    kRouteV5Mix = 32,      // k_gl5_gemm / k_gl5_mix (J > 21)
    kRouteExact = 64,      // exact-f32 generations v1-v3
    kRouteAttention = 128,  // k_attention: the separate attention kernel (J > 21, unfused routes)
    // 256 / 512: round 5's small-batch fused tile and fused layer kernel (removed in round 6)
    kRouteAttnMix = 1024     // k_attention_mix: the to_qkv layer's mixing inside the attention kernel
};
extern thread_local unsigned g_route_bits;

// f16 hi/lo split of a (types, N, K) f32 weight in MFMA B-fragment order (sd_graph_linear_v4.hip)
struct SplitW {
    _Float16* w = nullptr;  // device, owned by the caller (hipFree)
    int nct = 0;            // 32-column tiles in the layout (padded to a multiple of 6)
    float scale = 1.f;      // W' = W * scale (a power of two)
    float unscale = 1.f;    // 1 / scale
};
hipError_t make_split_weights(const float* W, int ntypes, int N, int K, SplitW* out, hipStream_t s);
// bf16 copy of W in the same B-fragment layout (the hi slots hold bf16(W), unscaled; precision 2)
hipError_t make_bf16_weights(const float* W, int ntypes, int N, int K, SplitW* out, hipStream_t s);

// Multi-head attention over joints (attention.py:122-136) from a (B, J, 3*heads*dh) qkv buffer.
struct AttnArgs {
    const float* qkv; float* out; int64_t B; int J; int heads; int dh; float scale;
    // SD_OPT_ATTENTION 2: qkv holds the to_qkv layer's PRE-mix Y and the kernel mixes it with this
    // (J, J) G-hat first (k_attention_mix, 49 <= J <= 52, dh 32); null: qkv is mixed
    const float* G = nullptr;
};

// Posterior mean + correlated noise step (nonisotropic.py:196-210 / isotropic.py:85-95).
struct UpdArgs {
    const float* x0; const float* xt;
    const float* eps; int64_t eps_rs;      // given noise rows (noise_mode 1)
    const float* C1; const float* C2; const float* U; const float* sig;   // step-t tables
    float c1s, c2s, sigs;                  // isotropic scalars
    int obj; float xa, xb;                 // isotropic pred_noise / pred_v (obj 1): x0 = xa x_t - xb act(out)
    int iso; int act; int noise_mode;      // noise_mode: 0 none (t == 0), 1 given, 2 Philox
    int clip;                              // 1: x0 clamped to [-1, 1] (clip_denoised, base.py:318-319)
    uint64_t seed; int64_t row0; int step; const uint64_t* rng_dev;  // rng_dev: {seed,row0} or null
    int64_t row_shift;                     // added to row0 (either source): a row chunk's first row
    float* out; float* out2; int64_t out2_rs;
    float* mean_out; int64_t mean_rs; float* noise_out; int64_t noise_rs;
    int64_t B; int J; int D;
    unsigned* dbg;  // SD_DEBUG_LDS builds only
    int x0_bf16, xt_bf16, out_bf16;  // bf16 latents (precision mode 2); out2 / records stay f32
    int elementwise;  // SD_OPT_UPDATE_KERNEL: 0 k_update_mfma where it applies, 1 the element-per-thread forms
    // diagnostics only (sd_debug_update_dump): the J values of x0 (activation + clamp applied),
    // x_t and sigma eps each thread computed from, stored after its outputs; null = off
    float* dump_x0; float* dump_xt; float* dump_ev;
};

hipError_t launch_graph_linear(const GLArgs& a, bool rms, hipStream_t s);     // dispatches v1..v5
hipError_t launch_graph_linear_v5(const GLArgs& a, bool rms, hipStream_t s);  // J > 21: GEMM + mixing pass
hipError_t launch_graph_linear_v1(const GLArgs& a, bool rms, hipStream_t s);
hipError_t launch_graph_linear_v2(const GLArgs& a, bool rms, hipStream_t s);
hipError_t launch_graph_linear_v3(const GLArgs& a, bool rms, hipStream_t s);  // J in {16,17,21}
hipError_t launch_graph_linear_v4(const GLArgs& a, bool rms, hipStream_t s);  // needs a.wsp
hipError_t launch_qkv_attention_v4(const GLArgs& a, bool rms, hipStream_t s);  // J <= 16, dh 32
// split-f16 GEMM phase (k_gl4y) into row-major z (B, J, N) with row stride z_rs (v5, J > 21)
hipError_t launch_gemm_split(const GLArgs& a, bool rms, float* z, int64_t z_rs, hipStream_t s);
// process defaults that new plans (and the sd_test_* hooks) start from: SKELDIFF_GL_VARIANT
// (0 auto, 1..5), SKELDIFF_GL4_CFG (<NW><RT><CT>, 0 auto), SKELDIFF_GL4_STAGE (0 / 1), read at load
int graph_linear_variant();
int gl4_tile_default();
int gl4_stage_default();
int64_t split_rows_default();         // SKELDIFF_SPLIT_ROWS: auto split route at or below this many rows
hipError_t launch_attention(const AttnArgs& a, hipStream_t s);
hipError_t launch_update(const UpdArgs& a, hipStream_t s);
hipError_t launch_mix_mfma(const float* z, const float* G, float* out, int64_t rows, int J, int N, bool transpose,
                           hipStream_t s);  // G-hat (or G-hat^T) mixing of (rows, J, N), v5's MFMA pass
hipError_t launch_noise_fill(float* out, int64_t rows, int64_t n_per_row, uint64_t seed,
                             int64_t row0, int step, const uint64_t* rng_dev, hipStream_t s,
                             int64_t row_shift = 0,   // row_shift: added to row0 (either source)
                             int out_bf16 = 0);       // out holds bf16 elements
// dst[r * dst_rs + i] = src[r * src_rs + i] (i < n; n % 4 == 0) with f32 <-> bf16 conversion
hipError_t launch_convert_rows(void* dst, int dst_bf16, int64_t dst_rs, const void* src, int src_bf16,
                               int64_t src_rs, int64_t rows, int64_t n, hipStream_t s);
hipError_t launch_philox_raw(uint32_t* out, int64_t rows, int64_t quads, uint64_t seed,
                             int64_t row0, int step, hipStream_t s);
hipError_t launch_set_rng(uint64_t* rng_dev, uint64_t seed, int64_t row0, hipStream_t s);
hipError_t launch_delay(double us, hipStream_t s);  // a stream-ordered wait of `us` microseconds
hipError_t launch_copy_rows(float* dst, int64_t dst_rs, const float* src, int64_t src_rs,
                            int64_t rows, int64_t n, hipStream_t s);
// row-blocked v4 activation layout -> row-major (rows, J, F)
hipError_t launch_unblock(float* out, const float* in, int64_t rows, int J, int F, hipStream_t s);

// evaluation metrics (sd_metrics.hip)
hipError_t launch_pairwise(const float* x, int64_t nseq, int S, int64_t X, float* l1_mean, float* l2_mean,
                           hipStream_t s);
hipError_t launch_ade_fde(const float* pred, const float* target, int64_t nseq, int S, int T, int64_t F, float* ade,
                          float* fde, float* per_sample_ade, float* per_sample_fde, hipStream_t s);
hipError_t launch_mm_ade_fde(const float* pred, const float* gts, const int64_t* pair_seq, int64_t npairs,
                             const int64_t* seq_off, int64_t nseq, int S, int T, int64_t F, float* pair_ade,
                             float* pair_fde, float* mmade, float* mmfde, hipStream_t s);

// best-of-k training relaxation (sd_metrics.hip; trainer.py:182-222)
hipError_t launch_best_of_k(const float* sim, const float* loss, int64_t nseq, int k, int64_t* idx, float* sel,
                            hipStream_t s);
hipError_t launch_best_of_k_bwd(const float* dsel, const int64_t* idx, int64_t nseq, int k, float* dloss, hipStream_t s);
hipError_t launch_pose_loss(const float* pred, const float* target, int64_t nseq, int S, int T, int J, int C, int mse,
                            float* out, hipStream_t s);

// plan-finalize helpers (one-time)
hipError_t launch_sinusoidal(float* emb, int T, int dim, float neg_scale, hipStream_t s);
hipError_t launch_linear(const float* x, int M, int K, const float* W, const float* b, int N,
                         float* y, int in_act, int out_act, hipStream_t s);
hipError_t launch_ghat(const float* G, float* Ghat, int J, int normalize, hipStream_t s);
// sets the thread-local message sd_last_error() returns; returns `code` (sd_plan.hip)
int set_error(int code, const std::string& msg);
hipError_t launch_fold_gain(const float* W, const float* g, float mult, float* out,
                            int64_t rows, int K, hipStream_t s);
hipError_t launch_sigma(const float* logvar, float* sig, int64_t n, hipStream_t s);

}  // namespace sd
