/*
 * skeldiff.h — C ABI of libskeldiff.so, the MI355X (gfx950) sampling engine for the
 * SkeletonDiffusion hot path: NonisotropicGaussianDiffusion.sample().
 *
 * Boundary rules: plain pointers and sizes, no torch types.  Tensors are row-major fp32,
 * contiguous, in device memory (HBM) unless stated; `stream` is a hipStream_t passed as
 * void* (NULL = default stream).  Every function returns 0 on success and a negative
 * SD_E* code on error; sd_last_error() returns a thread-local message for the last failure.
 * No C++ exception crosses the ABI.  A plan is immutable after sd_plan_finalize() and may be
 * shared by several streams; a workspace belongs to one stream at a time.
 *
 * Which reference interface each entry point replaces (paths relative to the reference
 * tree, tum-vision/skeletondiffusion):
 *   sd_plan_create / sd_plan_set_tensor / sd_plan_finalize
 *       -> module construction + strict load_state_dict of the diffusion and Denoiser
 *          (src/core/diffusion_manager.py:16-27, src/eval_prepare_model.py:69-72,
 *           src/core/diffusion/nonisotropic.py:72-127, src/core/network/nn/generator.py:8-84).
 *          Tensors are handed over by their reference state_dict key.
 *   sd_denoiser_forward
 *       -> Denoiser.forward (src/core/network/nn/generator.py:86-107) as called by
 *          LatentDiffusion.feed_model (src/core/diffusion/base.py:243-255).
 *   sd_p_sample_update
 *       -> q_posterior + p_combine_mean_var_noise of one reverse step
 *          (src/core/diffusion/base.py:314-341, src/core/diffusion/nonisotropic.py:196-210;
 *           isotropic.py:85-95 for IsotropicGaussianDiffusion), x0 clamp included.
 *   sd_sample_loop
 *       -> LatentDiffusion.p_sample_loop / sample (src/core/diffusion/base.py:343-390,
 *          439-443).
 *   sd_noise_fill
 *       -> the white-noise draws get_noise/randn (src/core/diffusion/base.py:151-158,351),
 *          replaced by counter-based Philox4x32-10 keyed by (seed, global row, step) so that
 *          results do not depend on batch split or GPU count.
 */
#ifndef SKELDIFF_H
#define SKELDIFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history: 1 (rounds 1-3); 2 (round 5) -- sd_mahalanobis_loss_forward / _backward take T,
 * sd_set_kernel_variant / sd_set_row_chains / sd_set_update_kernel / sd_set_v5_mix removed
 * (per-plan options instead), sd_test_set_split_route and sd_plan_desc::objective added;
 * 3 (round 6) -- SD_FLAG_NO_CLIP (p_sample's clip_denoised = False), sd_p_sample_update takes
 * flags, the measured-slower kernel forms and option values removed; 4 (round 6) --
 * sd_plan_desc::norm_type (Block LayerNorm over the node axis).  Bindings check it at load. */
#define SD_ABI_VERSION 4

enum {
    SD_OK = 0,
    SD_E_INVALID = -1,   /* bad argument / shape / unsupported configuration */
    SD_E_STATE = -2,     /* plan not finalized, tensor missing, ... */
    SD_E_HIP = -3,       /* HIP runtime error */
    SD_E_NOMEM = -4,
    SD_E_INTERNAL = -5
};

/* flags for sd_sample_loop */
enum {
    SD_FLAG_GRAPH = 1,          /* capture the whole T-step chain in a hipGraph, cache, replay */
    SD_FLAG_DEVICE_START = 2,   /* x_T drawn on device (Philox, step index T) instead of x_T arg */
    SD_FLAG_DEVICE_NOISE = 4,   /* per-step noise drawn on device instead of eps_all */
    SD_FLAG_NO_CLIP = 8         /* x0 is not clamped to [-1, 1] (p_sample / p_mean_variance with
                                   clip_denoised = False, base.py:314-328; the flag also applies to
                                   sd_p_sample_update) */
};

typedef struct sd_plan sd_plan;

typedef struct sd_plan_desc {
    int32_t num_nodes;        /* J = channels = num_nodes (<= 64) */
    int32_t latent_dim;       /* Denoiser `dim` = diffusion latent_size (seq_length) */
    int32_t cond_dim;         /* 0, or latent_dim when diffusion_conditioning */
    int32_t out_dim;          /* Denoiser out_dim (== latent_dim for sampling) */
    int32_t depth;
    int32_t attn_heads;
    int32_t attn_dim_head;
    int32_t use_attention;    /* 1: Attention blocks, 0: Residual(PreNorm(StaticGraphLinear)) */
    int32_t self_condition;   /* must be 0 (no release config uses it) */
    int32_t learn_influence;  /* 1: G-hat = row-L1-normalised G (graph_structural.py:31-32) */
    int32_t num_node_types;   /* 0: shared weights (no node_types); else types in node_types */
    const int64_t* node_types;/* host array[J] (ignored when num_node_types == 0) */
    int32_t timesteps;        /* T */
    int32_t isotropic;        /* 1: IsotropicGaussianDiffusion posterior (scalar coefficients) */
    int32_t activation;       /* diffusion_activation: 0 identity, 1 tanh */
    float sinusoidal_theta;   /* SinusoidalPosEmb theta (10000) */
    int32_t objective;        /* 0 pred_x0 (release configs); isotropic only: 1 pred_noise, 2 pred_v
                                 (x0 = a[t] x_t - b[t] act(model_out): isotropic.py:48-70) */
    int32_t norm_type;        /* ResnetBlock Block.norm (attention.py:49-60): 0 'none' (release configs),
                                 1 'layer' = LayerNorm over the node axis (attention.py:19-28; J = 16, 17
                                 or 21, v4 kernels; tensors "...blockN.norm.norm.weight/bias") -- ABI 4 */
} sd_plan_desc;

int32_t sd_abi_version(void);
const char* sd_last_error(void);
/* How the device code was built: "no-packed-fp32" for the product build (skeletondiffusion_amd/
 * build.py compiles every kernel without packed-FP32 instructions, DESIGN.md §4c, and checks the
 * linked code objects); the Python binding refuses to load a library that says otherwise. */
const char* sd_build_info(void);

int sd_plan_create(sd_plan** out, const sd_plan_desc* desc);
void sd_plan_destroy(sd_plan* plan);

/* The tensors a plan requires, in reference state_dict key order ("model.init_lin.weight",
 * ..., "posterior_mean_coef1_x0", ...). */
int32_t sd_plan_num_tensors(const sd_plan* plan);
const char* sd_plan_tensor_name(const sd_plan* plan, int32_t index);
int64_t sd_plan_tensor_numel(const sd_plan* plan, int32_t index);

/* Copy one tensor (fp32, contiguous, host or device pointer) into the plan. */
int sd_plan_set_tensor(sd_plan* plan, const char* name, const float* data, int64_t numel,
                       void* stream);
/* Pack weights (G-hat, RMSNorm gain folding, time/FiLM tables, posterior tables). */
int sd_plan_finalize(sd_plan* plan, void* stream);

/* dims_out[4] = {J (num_nodes), D (latent_dim), T (timesteps), cond_dim} of the plan (host-side
 * shape validation at the boundary, e.g. the skeldiff::sample_loop torch op). */
int sd_plan_dims(const sd_plan* plan, int32_t* dims_out);

/* Bytes of device workspace needed for `rows` latent rows. */
size_t sd_workspace_bytes(const sd_plan* plan, int64_t rows);

/* x0_out(B,J,out_dim) = Denoiser(x_t(B,J,D), t, x_cond).  x_cond: (B / cond_repeat, J, cond_dim)
 * with row b reading x_cond row b / cond_repeat (the repeat_interleave of base.py:246-248), or
 * NULL when cond_dim == 0. */
int sd_denoiser_forward(const sd_plan* plan, const float* x_t, const float* x_cond,
                        int64_t cond_repeat, int32_t t, float* x0_out, int64_t rows,
                        void* workspace, size_t workspace_bytes, void* stream);

/* Status of the last sd_sample_loop / sd_denoiser_forward / sd_denoiser_trace on `workspace`
 * (synchronises `stream`): flags bit 0 (SD_STATUS_F16_RANGE) = an activation reached |x| >= 65504,
 * outside the f16 range of the split-f16 (v4) products; informational: every f16-product kernel
 * (the split routes' GEMM phases and, since ABI 3, the one-kernel tiles) recomputed the waves'
 * tiles that left the range on exact-f32 MFMA, so f32 mode stays f32-accurate for any finite
 * input.  The word is cleared at the start of each of those calls.  (Bit 1, the round-5 fused
 * layer kernel's timeout, went with that kernel in ABI 3.) */
enum { SD_STATUS_F16_RANGE = 1 };
int sd_workspace_status(const sd_plan* plan, const void* workspace, size_t workspace_bytes, uint32_t* flags,
                        void* stream);

/* sd_denoiser_forward that also copies every block output (rows, J, D + cond_dim), row-major,
 * into acts[0 .. 2 + 4 * depth): init_lin, then per layer i < 2 * depth the ResnetBlock output and
 * the Residual(PreNorm(Attention)) output (nn.Identity for the last layer: a copy of the
 * ResnetBlock output), then final_res_block -- the module outputs of generator.py:94-106 (test
 * hook: the per-layer parity against the reference's forward hooks). */
int sd_denoiser_trace(const sd_plan* plan, const float* x_t, const float* x_cond, int64_t cond_repeat,
                      int32_t t, float* x0_out, int64_t rows, void* workspace, size_t workspace_bytes,
                      float* const* acts, int32_t nacts, void* stream);

/* One reverse step for B rows at time t:
 *   x0 = clamp(act(x0_raw), -1, 1) (no clamp with SD_FLAG_NO_CLIP in flags); mean = C1[t] x0 + C2[t] x_t;
 *   x_prev = mean + U (sigma_t * eps)   (nonisotropic)   |  c1 x0 + c2 x_t + sigma_t eps (iso)
 * eps: (B, J, D) rows `eps_row_stride` floats apart, or NULL for device Philox noise
 * (seed, global row row0 + b, step t).  t == 0 adds no noise.  mean_out / noise_out are
 * optional (NULL) extra outputs with their own row strides (return_sampling_noise). */
int sd_p_sample_update(const sd_plan* plan, const float* x0_raw, const float* x_t,
                       const float* eps, int64_t eps_row_stride, uint64_t seed, int64_t row0,
                       int32_t t, float* x_prev, float* mean_out, int64_t mean_row_stride,
                       float* noise_out, int64_t noise_row_stride, int64_t rows, int32_t flags,
                       void* stream);

/* The full reverse chain t = T-1 .. 0 (base.py:365-367).
 *   x_T     : (B,J,D) start noise, or ignored with SD_FLAG_DEVICE_START
 *   eps_all : (B, T-1, J, D) sampling noise in the reference layout (step t reads
 *             eps_all[:, T-1-t]), or ignored with SD_FLAG_DEVICE_NOISE
 *   out     : (B,J,D) final latents
 *   means_out / noise_out / timages_out : optional (B, T-1, J, D) records of mean_t,
 *             the noise used and x_t for t = T-1..1 (return_sampling_noise / return_timages)
 *   start_out: optional (B,J,D) copy of the start noise used */
int sd_sample_loop(const sd_plan* plan, const float* x_T, const float* x_cond,
                   int64_t cond_repeat, const float* eps_all, uint64_t seed, int64_t row0,
                   float* out, float* means_out, float* noise_out, float* timages_out,
                   float* start_out, int64_t rows, void* workspace, size_t workspace_bytes,
                   int32_t flags, void* stream);

/* Fill out(B, n_per_row) with the device normals of (seed, rows row0.., step). n_per_row % 4 == 0. */
int sd_noise_fill(float* out, int64_t rows, int64_t n_per_row, uint64_t seed, int64_t row0,
                  int32_t step, void* stream);
/* Raw Philox4x32-10 words for tests: out[4*i .. 4*i+3] = philox(ctr = (i % quads, step,
 * row lo, row hi) with row = row0 + i / quads, key = seed). */
int sd_philox_raw(uint32_t* out, int64_t rows, int64_t quads, uint64_t seed, int64_t row0,
                  int32_t step, void* stream);

/* Number of kernel launches one reverse step (denoiser + update) issues. */
int32_t sd_plan_kernels_per_step(const sd_plan* plan);

/* Algorithmic FLOPs of one reverse step over `rows` rows, from the plan's own layer list:
 * flops_out[0] graph-linear GEMMs + G-hat mixing, [1] attention QK^T + PV, [2] posterior update. */
int sd_plan_step_flops(const sd_plan* plan, int64_t rows, double* flops_out);

/* Measurement hook: run one reverse step at time t `reps` times with HIP events recorded on
 * `stream` around every kernel.  ms_out[4] = mean ms per step in graph-linear, attention and
 * update kernels, and first-to-last event of the step; counts_out[3] (nullable) = launches per
 * step per class.  Device noise is used for the update. */
int sd_profile_step(const sd_plan* plan, const float* x_t, const float* x_cond, int64_t cond_repeat,
                    int32_t t, int64_t rows, void* workspace, size_t workspace_bytes, int32_t reps,
                    float* ms_out, int32_t* counts_out, void* stream);

/* Evaluation metrics on device, one workgroup per sequence, deterministic
 * fixed-order reductions, caller-owned device buffers, up to 64 samples per sequence.
 * sd_pairwise_distances: x (nseq, samples, features) -> per sequence the mean over sample pairs
 *   i < j of the L1 distance (l1_mean: the reference's lat_apd, src/metrics/multimodal.py:137-151)
 *   and of the L2 distance (l2_mean: apd, multimodal.py:15-35); either output may be NULL.
 * sd_ade_fde: pred (nseq, samples, frames, features), target (nseq, frames, features) -> per
 *   sequence min over samples of the mean-over-frames L2 distance (ade, multimodal.py:44-57) and
 *   of the last frame's distance (fde, :60-73); per_sample_* (nseq, samples) receive the
 *   distances before the minimum (reduction != 'mean'); any output may be NULL. */
int sd_pairwise_distances(const float* x, int64_t nseq, int32_t samples, int64_t features, float* l1_mean,
                          float* l2_mean, void* stream);
int sd_ade_fde(const float* pred, const float* target, int64_t nseq, int32_t samples, int32_t frames,
               int64_t features, float* ade, float* fde, float* per_sample_ade, float* per_sample_fde, void* stream);
/* Multimodal ADE / FDE (src/metrics/multimodal.py:108-135): sequence i has the ground truths
 * gts[seq_offsets[i] .. seq_offsets[i+1]) (each (frames, features); pair_seq[p] = the sequence
 * of ground truth p, npairs = seq_offsets[nseq]); per pair the min over samples of the ADE /
 * FDE against that ground truth (pair_ade / pair_fde, npairs each), then per sequence their
 * mean (mmade / mmfde, nseq; NaN for a sequence without ground truths, as the reference's
 * mean of an empty tensor).  pred (nseq, samples, frames, features).  seq_offsets and
 * pair_seq are device int64 arrays. */
int sd_mm_ade_fde(const float* pred, const float* gts, const int64_t* pair_seq, int64_t npairs,
                  const int64_t* seq_offsets, int64_t nseq, int32_t samples, int32_t frames, int64_t features,
                  float* pair_ade, float* pair_fde, float* mmade, float* mmfde, void* stream);

/* Best-of-k training relaxation (reference src/core/trainer.py:182-222,
 * Trainer.loss -> to_comparison_space_train -> get_ksimilarity_loss with train_pick_best_sample_among_k
 * = k): the diffusion loss of nseq sequences x k samples (nseq, k) (p_losses with n_train_samples = k,
 * base.py:262-300) and a similarity (nseq, k) -- the loss itself in the latent space (sim = NULL),
 * sd_pose_loss of the decoded samples in the input space, the per-sample ADE (sd_ade_fde
 * per_sample_ade) in the metric space.
 * sd_best_of_k: idx_out (nseq) int64 = per sequence the index of the smallest similarity
 *   (torch.min(dim).indices: the first minimum; the first NaN if any), loss_out (nseq) = the loss at
 *   that index (torch.gather).  Either output may be NULL.
 * sd_best_of_k_backward: dloss (nseq, k) = dloss_sel at the selected index, 0 elsewhere.
 * sd_pose_loss: AutoEncoder.loss(pred, y, reduction='none') (src/core/network/nn/autoencoder.py:80-98)
 *   per sample: mean over frames and joints of the sum over coordinates of |d| (mse = 0) or d^2 (mse
 *   = 1); pred (nseq, samples, frames, joints, dims), target (nseq, frames, joints, dims) ->
 *   per_sample (nseq, samples). */
int sd_best_of_k(const float* sim, const float* loss, int64_t nseq, int32_t k, int64_t* idx_out, float* loss_out,
                 void* stream);
int sd_best_of_k_backward(const float* dloss_sel, const int64_t* idx, int64_t nseq, int32_t k, float* dloss,
                          void* stream);
int sd_pose_loss(const float* pred, const float* target, int64_t nseq, int32_t samples, int32_t frames,
                 int32_t joints, int32_t dims, int32_t mse, float* per_sample, void* stream);

/* Test hooks: one kernel on caller buffers, for the per-kernel numerics tests.
 * sd_test_graph_linear: out(B,J,N) = act(FiLM(ghat @ (s_j W[type j] [x1_j | x2_j] + bias[type j]))) + res,
 *   W (types,N,K1+K2), bias (types,N) or NULL, ghat (J,J), film (2N) or NULL, res (B,J,N) or NULL,
 *   x1 row b read at b / x1_div, s_j = 1/max(||x1_j||,1e-12) when rms (else 1), act 0/1 = none/tanh.
 * sd_test_attention: out(B,J,heads*dh) = softmax(q k^T / sqrt(dh)) v per head, qkv (B,J,3*heads*dh). */
int sd_test_graph_linear(const float* x1, int32_t K1, int64_t x1_div, const float* x2, int32_t K2,
                         const float* W, const float* bias, const int64_t* node_types, const float* ghat,
                         const float* film, int32_t act, const float* res, float* out, int64_t rows,
                         int32_t J, int32_t N, int32_t rms, void* stream);
/* sd_test_graph_linear_layout: as sd_test_graph_linear with operand layouts: bit 0 x1, bit 1 x2,
 *   bit 2 res, bit 3 out in the v4 row-blocked layout (per 32-row block and node, features as
 *   [F/8][2][32 rows][4]; buffers padded to a multiple of 32 rows); needs the v4 kernels. */
int sd_test_graph_linear_layout(const float* x1, int32_t K1, int64_t x1_div, const float* x2, int32_t K2,
                                const float* W, const float* bias, const int64_t* node_types, const float* ghat,
                                const float* film, int32_t act, const float* res, float* out, int64_t rows,
                                int32_t J, int32_t N, int32_t rms, int32_t layout, void* stream);
int sd_test_attention(const float* qkv, float* out, int64_t rows, int32_t J, int32_t heads,
                      int32_t dim_head, void* stream);
/* sd_test_qkv_attention: the fused to_qkv + Attention kernel on caller buffers: qkv = G-hat-mixed
 *   StaticGraphLinear (s_j W[type j] x_j, s_j = RMS scale when rms, no bias) with W (types, 3*heads*32, K),
 *   then out(B,J,heads*32) = softmax(q k^T / sqrt(32)) v per head.  SD_E_INVALID where the fused
 *   kernel does not apply (J > 16).  layout bit 0 / bit 3: x / out row-blocked (as
 *   sd_test_graph_linear_layout).  Replaces to_qkv + Attention, attention.py:105-136. */
int sd_test_qkv_attention(const float* x, int32_t K, const float* W, const int64_t* node_types, const float* ghat,
                          float* out, int64_t rows, int32_t J, int32_t heads, int32_t rms, int32_t layout,
                          void* stream);
/* Test hook: the kernel generation of the sd_test_* entry points ONLY (plans never read it; a
 * plan's generation is its SD_OPT_KERNEL_VARIANT / SD_OPT_GL4_TILE):
 * gl_variant 0 = auto (v4 split-f16 where available, else exact-f32 v3/v2/v5), 1..3 = exact-f32
 * generations, 4 = v4, 5 = v5; gl4_tile = <waves><row tiles><col tiles> (e.g. 822) or 0 = auto,
 * -1 leaves it.  Returns the previous gl_variant, or -1 for an invalid one (nothing changed);
 * gl_variant = -1 only queries (returns the current value). */
int sd_test_set_kernel_variant(int32_t gl_variant, int32_t gl4_tile);
/* Test hook: the v4 split route of the sd_test_graph_linear* entry points ONLY (as
 * SD_OPT_SPLIT_ROUTE: 0 auto, 1 never, 2 k_gl4y GEMM phase, 3 k_gl4t GEMM phase, 4 k_gl4t except
 * to_qkv + attention; 2 / 3 / 4 allocate the pre-mix scratch per call).  Returns the previous route,
 * or -1 for an invalid one; route = -1 only queries. */
int sd_test_set_split_route(int32_t route);

/* Per-plan kernel options (read by the launches recorded after the call; part of the graph
 * cache key).  There is no process-wide kernel state: a plan starts from the SKELDIFF_*
 * environment read at library load and keeps its own options, so two plans may hold different
 * options and sample concurrently.  SD_E_INVALID for an unknown option or value. */
enum {
    SD_OPT_KERNEL_VARIANT = 1,  /* 0 auto, 1..5 force a graph-linear generation */
    SD_OPT_GL4_TILE = 2,        /* v4 tile <waves><row tiles><col tiles>, 0 = per shape */
    SD_OPT_ROW_CHAINS = 3,      /* 1..8 concurrent row chains in sd_sample_loop; 0 = auto
                                   (3, or 2 at <= SKELDIFF_SPLIT_ROWS rows) */
    SD_OPT_PRECISION = 4,       /* as sd_plan_set_precision */
    SD_OPT_GL4_STAGING = 5,     /* v4 weight stages: 0 LDS-DMA (default), 1 register-staged;
                                   2 = 0 (a round-2 diagnostic setting, kept for compatibility) */
    SD_OPT_SPLIT_ROUTE = 6,     /* v4 split route (GEMM phase per (tile, node) + mixing phase,
                                   DESIGN.md §4d'; bitwise identical results): 0 auto (k_gl4y at
                                   <= 1200 rows of the call; k_gl4t for full batches where measured
                                   faster), 1 never (the one-kernel k_gl4 tiles), 2 always (k_gl4y),
                                   3 always with the tiled GEMM phase (k_gl4t: 128 rows x up to 192
                                   columns of one node per workgroup), 4 the tiled GEMM phase except
                                   for to_qkv + attention (one-kernel fused tile).  ABI 3 removed 5
                                   (small-batch fused tile) and 6 (fused layer kernel k_gl4f):
                                   measured slower, DESIGN.md §4i / §4j */
    SD_OPT_LAST_CHAINS = 7,     /* read-only: row chains the plan's last sd_sample_loop ran (the
                                   SD_OPT_ROW_CHAINS value, fewer for batches of fewer than n
                                   32-row units, a ragged last unit counting; auto: 1 at <= 128
                                   rows, 2 at <= SKELDIFF_SPLIT_ROWS, else 3); 0 before the first
                                   call */
    SD_OPT_LAST_ROUTE = 8,      /* read-only: kernels the plan's last sd_sample_loop launched, bits
                                   1 one-kernel k_gl4, 2 fused to_qkv + attention k_gl4, 4 k_gl4y
                                   GEMM phase, 8 k_gl4t GEMM phase, 16 split-route mixing /
                                   attention phase, 32 v5 mixing (J > 21), 64 exact-f32 kernels,
                                   128 separate k_attention, 1024 k_attention_mix (256 / 512: the
                                   kernels ABI 3 removed) */
    SD_OPT_UPDATE_KERNEL = 9,   /* posterior update: 0 (default) the J x J projections on
                                   v_mfma_f32_16x16x4_f32 where they apply (nonisotropic, J <= 64),
                                   1 the element-per-thread forms; the same bits (ABI 3 removed the
                                   pipelined forms 2 / 3: measured no faster) */
    SD_OPT_V5_MIX = 10,         /* J > 21 mixing pass (v5): 0 (default) G-hat mixing on
                                   v_mfma_f32_16x16x4_f32 (k_gl5_mixm), 1 the VALU form (k_gl5_mix);
                                   the same j-ordered fmaf chains */
    SD_OPT_ATTENTION = 11       /* separate attention kernel at 49 <= J <= 52 (MANO), both forms
                                   the same bits: 0 (default) auto = 2; 2 the to_qkv layer's G-hat
                                   mixing inside the attention kernel, its pre-mix Y in the qkv
                                   buffer (k_attention_mix, 5 % faster); 3 after the mixing pass,
                                   padded to 64 nodes.  ABI 3 removed 1 (the 48-node
                                   tail form, 1 % slower) */
};
int sd_plan_set_option(sd_plan* plan, int32_t option, int64_t value);
int sd_plan_get_option(const sd_plan* plan, int32_t option, int64_t* value);

/* Graph-GRU latent decoder: AutoEncoder.decode -> Decoder.forward
 * (src/core/network/nn/decoder.py:60-104) with the StaticGraphGRU cell
 * (src/core/network/layers/recurrent.py:321-366), recurrent_arch_decoder = StaticGraphGRU, one
 * layer, clockwork off.  Tensors are the reference's `decoder.*` state_dict entries on the device
 * (types = num_node_types, or 1 with shared weights when num_node_types == 0):
 *   init_*  initial_hidden_h: G (J,J), weight (types, H, F+L), bias (types, H) or NULL
 *   G, G_add, weight_ih (types, 3H, F+L), weight_hh (types, 3H, H), bias_ih, bias_hh (types, 3H)
 *           rnn.layers.0 (G_add may be NULL: no additive influence)
 *   fc_*    fc: G (J,J), weight (types, F, H), bias (types, F) or NULL
 * x (rows, 2, J, F) = the last two observed frames (x[:, -2:]), h (rows, J, L) = the sampled
 * latents -> out (rows, ph, J, F).  F <= 16, L and H multiples of 16. */
typedef struct sd_gru_decoder_desc {
    int32_t num_nodes, feature_size, latent_size, hidden_size, num_node_types;
    const int64_t* node_types; /* host array[J] (ignored when num_node_types == 0) */
    const float *init_G, *init_weight, *init_bias;
    const float *G, *G_add, *weight_ih, *weight_hh, *bias_ih, *bias_hh;
    const float *fc_G, *fc_weight, *fc_bias;
} sd_gru_decoder_desc;
size_t sd_gru_decode_workspace_bytes(const sd_gru_decoder_desc* desc, int64_t rows, int32_t ph);
int sd_gru_decode(const sd_gru_decoder_desc* desc, const float* x, const float* h, int64_t rows, int32_t ph,
                  float* out, void* workspace, size_t workspace_bytes, void* stream);
/* Graph-GRU encoder + z_activation (src/core/network/nn/encoder.py:75-80, autoencoder.py:47-51,
 * encoder_act = z_activation = tanh): x (rows, frames, J, F) observed frames -> z (rows, J, L) =
 * tanh(tanh(fc(GRU over the frames from initial_hidden1(x[:, 0])))).  Same descriptor with the
 * `encoder.*` tensors: init_* = initial_hidden1 (weight (types, H, F)), weight_ih (types, 3H, F),
 * G_add = NULL, fc weight (types, L, H); latent_size = L. */
size_t sd_gru_encode_workspace_bytes(const sd_gru_decoder_desc* desc, int64_t rows, int32_t frames);
int sd_gru_encode(const sd_gru_decoder_desc* desc, const float* x, int64_t rows, int32_t frames, float* z,
                  void* workspace, size_t workspace_bytes, void* stream);
/* Arithmetic of the plan's graph-linear launches.  mode 0 (default):
 * f32-accurate -- 3 split f16 products per f32 product, within the f32-vs-f64 drift.  mode 1:
 * half -- one f16 product (x and W rounded to f16), f32 accumulate, f32 activations in HBM; the
 * latent ADE / APD stay within 1 % of mode 0 (tests/test_precision.py).  Applies to the split-f16
 * (v4) kernels (J in 16, 17, 21); plans on the exact-f32 kernels stay exact.  mode 2: bf16 --
 * "bf16 latents + fp32 Sigma_N projection" (BASELINE config 5): one bf16 product per
 * multiply-add (v_mfma_f32_32x32x16_bf16), f32 accumulate and epilogue; the latents between
 * steps (x_t, x0) and the residual-stream activations are bf16 in HBM; the posterior update
 * (C1 x0 + C2 x_t + U (sigma eps)) computes in f32; start noise, records and the final latents
 * are f32 at the ABI.  J in 16, 17, 21 only (SD_E_INVALID otherwise).  Affects launches recorded
 * after the call; SD_E_INVALID for another mode. */
int sd_plan_set_precision(sd_plan* plan, int32_t mode);

/* Training-side StaticGraphLinear (SURVEY.md §8f "next" #4): replaces GraphLinear.forward
 * (src/core/network/layers/graph_structural.py:30-43, StaticGraphLinear :105-114) and the backward
 * torch autograd derives for it in NonisotropicGaussianDiffusion.forward / p_losses training
 * (src/core/diffusion/base.py:262-307).  Caller-owned device buffers, row-major:
 *   x (rows, J, K), W (types, N, K), bias (types, N) or NULL, node_types device int64 (J) with
 *   values in [0, n_types) (n_types = 0: shared weights, W (1, N, K), node_types ignored),
 *   ghat (J, J) = the mixing matrix actually applied (G, or G / rowsum|G| when learn_influence).
 * sd_gl_train_forward: z = W[type j] x_j + bias[type j] (pre-mix, kept for backward), y = ghat @ z.
 * sd_gl_train_backward: from dy (rows, J, N) and the forward's z: dx (rows, J, K), dW (types, N, K),
 *   dbias (types, N), dghat (J, J); any output may be NULL (not computed).  Deterministic (fixed
 *   reduction order).  workspace >= sd_gl_train_workspace_bytes(rows, J, K, N, n_types).
 *   1 <= J <= 64. */
size_t sd_gl_train_workspace_bytes(int64_t rows, int32_t J, int32_t K, int32_t N, int32_t n_types);
int sd_gl_train_forward(const float* x, const float* W, const float* bias, const int64_t* node_types,
                        int32_t n_types, const float* ghat, int64_t rows, int32_t J, int32_t K, int32_t N,
                        float* z, float* y, void* stream);
int sd_gl_train_backward(const float* x, const float* z, const float* dy, const float* W, const int64_t* node_types,
                         int32_t n_types, const float* ghat, int64_t rows, int32_t J, int32_t K, int32_t N, float* dx,
                         float* dW, float* dbias, float* dghat, void* workspace, size_t workspace_bytes,
                         void* stream);

/* Attention over joints under autograd (training side; reference attention.py:122-136, the part
 * between to_qkv and to_out): qkv (rows, J, 3 * heads * dim_head) as to_qkv writes it.
 * sd_attn_train_forward: out (rows, J, heads * dim_head) = softmax((q scale) k^T) v per head.
 * sd_attn_train_backward: dqkv (rows, J, 3 * heads * dim_head) from dout, P recomputed.
 * 1 <= J <= 64, 1 <= dim_head <= 64; f32; one workgroup per (row, head). */
int sd_attn_train_forward(const float* qkv, float* out, int64_t rows, int32_t J, int32_t heads, int32_t dim_head,
                          float scale, void* stream);
int sd_attn_train_backward(const float* qkv, const float* dout, float* dqkv, int64_t rows, int32_t J, int32_t heads,
                           int32_t dim_head, float scale, void* stream);
/* FiLM + tanh of a ResnetBlock's first Block under autograd (reference attention.py:67-75):
 * y (rows, J, C), ss (rows, 2C) = scale | shift (the time MLP's output, broadcast over the J nodes):
 * out = tanh(y (scale + 1) + shift); backward: dy (rows, J, C) and dss (rows, 2C) from dout.
 * rows <= 65535 for the backward. */
int sd_film_tanh_forward(const float* y, const float* ss, float* out, int64_t rows, int32_t J, int32_t C, void* stream);
int sd_film_tanh_backward(const float* y, const float* ss, const float* out, const float* dout, float* dy, float* dss,
                          int64_t rows, int32_t J, int32_t C, void* stream);

/* Row-wise L1 normalisation of a learnable influence matrix under autograd (reference
 * graph_structural.py:107, F.normalize(G, p=1, dim=1)): ghat[i][j] = G[i][j] / max(sum_k |G[i][k]|, eps);
 * the backward writes dG from dghat.  `count` contiguous J x J row-major matrices (one launch for
 * all of a Denoiser's learnable G), 1 <= J <= 64, f32. */
int sd_l1norm_rows_forward(const float* G, float* ghat, int32_t J, int32_t count, float eps, void* stream);
int sd_l1norm_rows_backward(const float* G, const float* dghat, float* dG, int32_t J, int32_t count, float eps,
                            void* stream);
/* PreNorm's RMSNorm under autograd (reference attention.py:30-36): x (R, C), R vectors of C
 * features, out = x / max(||x||, eps) * g * scale (scale = sqrt(C)); the forward also writes
 * dnorm (R) = max(||x||, eps) for the backward, which writes dx (R, C) and dg (C), the latter
 * summed over vectors in a fixed order through a workspace of sd_rmsnorm_workspace_bytes.
 * 1 <= C <= 1024. */
size_t sd_rmsnorm_workspace_bytes(int64_t R, int32_t C);
int sd_rmsnorm_forward(const float* x, const float* g, float* out, float* dnorm, int64_t R, int32_t C, float scale,
                       float eps, void* stream);
int sd_rmsnorm_backward(const float* x, const float* g, const float* dnorm, const float* dy, float* dx, float* dg,
                        int64_t R, int32_t C, float scale, float eps, void* workspace, size_t workspace_bytes,
                        void* stream);
/* Mahalanobis loss of NonisotropicGaussianDiffusion reduced per row (reference
 * nonisotropic.py:177-190 and base.py:297-298): model_out, target (rows, J, F), S =
 * mahalanobis_S_sqrt_recip (T, J, J), t (rows) int64 timesteps (a row whose t is outside [0, T) gets a NaN
 * loss / gradient: no out-of-range table read);
 * loss[r] = mean_{i,f} |(S[t_r] D_r)[i][f]| (mse: squared), D = target - model_out when
 * pred_noise, else model_out - target.  The backward writes d model_out (rows, J, F) from dloss
 * (rows).  1 <= J <= 64, 1 <= F <= 256, f32. */
int sd_mahalanobis_loss_forward(const float* model_out, const float* target, const float* S, const int64_t* t,
                                int32_t T, int64_t rows, int32_t J, int32_t F, int32_t pred_noise, int32_t mse, float* loss,
                                void* stream);
int sd_mahalanobis_loss_backward(const float* model_out, const float* target, const float* S, const int64_t* t,
                                 int32_t T, const float* dloss, int64_t rows, int32_t J, int32_t F, int32_t pred_noise,
                                 int32_t mse, float* dmodel_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SKELDIFF_H */
