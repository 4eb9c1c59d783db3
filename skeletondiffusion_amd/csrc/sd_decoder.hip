// Graph-GRU latent decoder (SURVEY.md §8f "next" #1): AutoEncoder.decode -> Decoder.forward
// (src/core/network/nn/decoder.py:60-104) with the StaticGraphGRU cell of
// src/core/network/layers/recurrent.py:321-366, unrolled for `ph` frames.
//
// Per row (one sampled future) and frame t, with gx_t the cell's graph matrix:
//   gx_0 = normalize_L1(G),  gx_{t+1} = normalize_L1(gx_t + G_add)        (recurrent.py:361-364)
//   x_res  = W_ih[type] [x_last | h] + b_ih            (unmixed; the input never changes over t)
//   h_res  = gx_t (W_hh[type] hx + b_hh)               -> graph-linear launch with G = gx_t
//   r = sigmoid(gx_t x_res_r + h_r), z = sigmoid(gx_t x_res_z + h_z), n = tanh(gx_t x_res_n + r h_n)
//   hx <- n - n z + z hx                                -> k_gru_gate (mixes x_res on the fly)
//   out[:, t] = tanh(Ghat_fc (W_fc[type] hx + b_fc))    -> graph-linear launch, tanh epilogue
//   hx_0 = Ghat_init (W_init[type] [x_prev | h] + b_init)
// The graph linears run on the exact-f32 kernels (row-major); the 3-feature frame inputs are
// zero-padded to 16 so K stays a multiple of 16.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <string>

#include "../../include/skeldiff.h"
#include "sd_internal.h"

namespace sd {
namespace {

constexpr int KF = 16;  // padded width of the frame features (F <= 16)

// gx table: row i of gx_t for t = 0 .. ph-1 (rows are independent under the row-L1 normalize)
__global__ void k_gx_table(const float* __restrict__ G, const float* __restrict__ Gadd, int J, int ph,
                           float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= J) return;
    float row[kMaxNodes];
    float s = 0.f;
    for (int j = 0; j < J; ++j) s += fabsf(G[i * J + j]);
    float den = fmaxf(s, 1e-12f);
    for (int j = 0; j < J; ++j) row[j] = G[i * J + j] / den;
    for (int t = 0; t < ph; ++t) {
        for (int j = 0; j < J; ++j) out[((int64_t)t * J + i) * J + j] = row[j];
        s = 0.f;
        for (int j = 0; j < J; ++j) {
            row[j] += Gadd ? Gadd[i * J + j] : 0.f;
            s += fabsf(row[j]);
        }
        den = fmaxf(s, 1e-12f);
        for (int j = 0; j < J; ++j) row[j] /= den;
    }
}

__global__ void k_identity(float* I, int J) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < J * J) I[k] = (k / J == k % J) ? 1.f : 0.f;
}

// W (types, N, F + L) -> (types, N, KF + L), the F frame columns zero-padded to KF
__global__ void k_pad_w(const float* __restrict__ W, int64_t TN, int F, int L, float* __restrict__ Wp) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int KP = KF + L;
    if (g >= TN * KP) return;
    const int64_t tn = g / KP;
    const int k = (int)(g % KP);
    Wp[g] = k < F ? W[tn * (F + L) + k] : (k < KF ? 0.f : W[tn * (F + L) + F + (k - KF)]);
}

// frame `f` of x (rows, 2, J, F) -> (rows, J, KF) zero-padded
__global__ void k_pad_frame(const float* __restrict__ x, int64_t rows, int J, int F, int f, float* __restrict__ xp) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= rows * J * KF) return;
    const int k = (int)(g % KF);
    const int64_t rj = g / KF, r = rj / J;
    const int j = (int)(rj % J);
    xp[g] = k < F ? x[((r * 2 + f) * J + j) * F + k] : 0.f;
}

// frame `f` of x (rows, T, J, F) -> (rows, J, KF) zero-padded (encoder input)
__global__ void k_pad_frame_t(const float* __restrict__ x, int64_t rows, int T, int J, int F, int f,
                              float* __restrict__ xp) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= rows * J * KF) return;
    const int k = (int)(g % KF);
    const int64_t rj = g / KF, r = rj / J;
    const int j = (int)(rj % J);
    xp[g] = k < F ? x[((r * T + f) * J + j) * F + k] : 0.f;
}

__global__ void k_tanh_inplace(float* __restrict__ v, int64_t n) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g < n) v[g] = tanhf(v[g]);
}

// One workgroup per row: x_res (J, 3H) and gx_t in LDS; thread -> (node i, feature c) outputs.
__global__ __launch_bounds__(256) void k_gru_gate(const float* __restrict__ xres, const float* __restrict__ hres,
                                                  const float* __restrict__ gx, const float* __restrict__ hx,
                                                  float* __restrict__ hy, int J, int H) {
    extern __shared__ float lds[];
    float* sx = lds;               // (J, 3H)
    float* sg = lds + J * 3 * H;   // (J, J)
    const int64_t r = blockIdx.x;
    const int H3 = 3 * H;
    for (int k = threadIdx.x; k < J * H3; k += 256) sx[k] = xres[r * J * H3 + k];
    for (int k = threadIdx.x; k < J * J; k += 256) sg[k] = gx[k];
    __syncthreads();
    for (int o = threadIdx.x; o < J * H; o += 256) {
        const int i = o / H, c = o - i * H;
        float ir = 0.f, iz = 0.f, in = 0.f;
        for (int j = 0; j < J; ++j) {
            const float g = sg[i * J + j];
            ir = fmaf(g, sx[j * H3 + c], ir);
            iz = fmaf(g, sx[j * H3 + H + c], iz);
            in = fmaf(g, sx[j * H3 + 2 * H + c], in);
        }
        const float* hr = hres + (r * J + i) * H3;
        const float rg = 1.f / (1.f + expf(-(ir + hr[c])));
        const float zg = 1.f / (1.f + expf(-(iz + hr[H + c])));
        const float n = tanhf(in + rg * hr[2 * H + c]);
        const float h0 = hx[(r * J + i) * H + c];
        hy[(r * J + i) * H + c] = n - n * zg + zg * h0;
    }
}

struct DecWS {
    float *xprev, *xlast, *winit, *wih, *ghat_init, *ghat_fc, *ident, *gx, *xres, *hres, *h0, *h1;
};

size_t carve(const sd_gru_decoder_desc* d, int64_t rows, int ph, char* base, DecWS* w) {
    const int J = d->num_nodes, F = d->feature_size, L = d->latent_size, H = d->hidden_size;
    const int nt = d->num_node_types > 0 ? d->num_node_types : 1;
    size_t off = 0;
    auto take = [&](size_t nfloat) {
        float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
        off += (nfloat * sizeof(float) + 255) & ~(size_t)255;
        return p;
    };
    (void)F;
    DecWS t;
    DecWS& o = w ? *w : t;
    o.xprev = take((size_t)rows * J * KF);
    o.xlast = take((size_t)rows * J * KF);
    o.winit = take((size_t)nt * H * (KF + L));
    o.wih = take((size_t)nt * 3 * H * (KF + L));
    o.ghat_init = take((size_t)J * J);
    o.ghat_fc = take((size_t)J * J);
    o.ident = take((size_t)J * J);
    o.gx = take((size_t)ph * J * J);
    o.xres = take((size_t)rows * J * 3 * H);
    o.hres = take((size_t)rows * J * 3 * H);
    o.h0 = take((size_t)rows * J * H);
    o.h1 = take((size_t)rows * J * H);
    return off;
}

GLArgs gl(const sd_gru_decoder_desc* d, const float* x1, int K1, const float* x2, int K2, const float* W,
          const float* bias, const float* G, int N, float* out, int64_t out_rs, int64_t rows, int act) {
    GLArgs a{};
    a.x1 = x1;
    a.K1 = K1;
    a.x1_rs = (int64_t)d->num_nodes * K1;
    a.x1_div = 1;
    a.x2 = x2;
    a.K2 = K2;
    a.x2_rs = (int64_t)d->num_nodes * K2;
    a.W = W;
    a.bias = bias;
    a.G = G;
    a.out = out;
    a.out_rs = out_rs;
    a.B = rows;
    a.N = N;
    a.J = d->num_nodes;
    a.act = act;
    a.ntypes = d->num_node_types > 0 ? d->num_node_types : 1;
    for (int j = 0; j < d->num_nodes; ++j) {
        const int t = d->num_node_types > 0 ? (int)d->node_types[j] : 0;
        a.wrow[j] = t * N;
        a.ntype[j] = t;
    }
    return a;
}

}  // namespace
}  // namespace sd

namespace {
int dfail(int code, const std::string& m) { return sd::set_error(code, m); }
int check_desc(const sd_gru_decoder_desc* d) {
    if (!d) return dfail(SD_E_INVALID, "null decoder descriptor");
    if (d->num_nodes < 1 || d->num_nodes > sd::kMaxNodes) return dfail(SD_E_INVALID, "num_nodes must be in [1, 64]");
    if (d->feature_size < 1 || d->feature_size > sd::KF) return dfail(SD_E_INVALID, "feature_size must be in [1, 16]");
    if (d->latent_size < 16 || d->latent_size % 16 || d->hidden_size < 16 || d->hidden_size % 16)
        return dfail(SD_E_INVALID, "latent_size and hidden_size must be positive multiples of 16");
    if (d->num_node_types > 0 && !d->node_types) return dfail(SD_E_INVALID, "node_types missing");
    if (d->num_node_types > 0)
        for (int j = 0; j < d->num_nodes; ++j)
            if (d->node_types[j] < 0 || d->node_types[j] >= d->num_node_types)
                return dfail(SD_E_INVALID, "node_types out of range");
    if (!d->init_G || !d->init_weight || !d->G || !d->weight_ih || !d->weight_hh || !d->fc_G || !d->fc_weight)
        return dfail(SD_E_INVALID, "null decoder tensor");
    return SD_OK;
}
}  // namespace

extern "C" {

size_t sd_gru_decode_workspace_bytes(const sd_gru_decoder_desc* d, int64_t rows, int32_t ph) {
    if (check_desc(d) || rows < 0 || ph < 1) return 0;
    return sd::carve(d, rows, ph, nullptr, nullptr) + 256;
}

int sd_gru_decode(const sd_gru_decoder_desc* d, const float* x, const float* h, int64_t rows, int32_t ph,
                  float* out, void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_desc(d);
    if (rc) return rc;
    if (rows < 0 || ph < 1) return dfail(SD_E_INVALID, "rows >= 0 and ph >= 1 required");
    if (rows == 0) return SD_OK;
    if (!x || !h || !out) return dfail(SD_E_INVALID, "null input / output");
    const size_t need = sd::carve(d, rows, ph, nullptr, nullptr);
    char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    if (!workspace || (size_t)(base - (char*)workspace) + need > ws_bytes)
        return dfail(SD_E_INVALID, "workspace too small: need " + std::to_string(need + 256));
    sd::DecWS w;
    sd::carve(d, rows, ph, base, &w);
    hipStream_t s = (hipStream_t)stream;
    const int J = d->num_nodes, F = d->feature_size, L = d->latent_size, H = d->hidden_size;
    const int nt = d->num_node_types > 0 ? d->num_node_types : 1;
    const int KP = sd::KF + L;
#define DHIP(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return dfail(SD_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
    auto grid = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    // one-time per call: padded weights / frames, G-hats, the gx table
    hipLaunchKernelGGL(sd::k_pad_w, grid((int64_t)nt * H * KP), dim3(256), 0, s, d->init_weight, (int64_t)nt * H, F, L, w.winit);
    hipLaunchKernelGGL(sd::k_pad_w, grid((int64_t)nt * 3 * H * KP), dim3(256), 0, s, d->weight_ih, (int64_t)nt * 3 * H, F, L, w.wih);
    hipLaunchKernelGGL(sd::k_pad_frame, grid(rows * J * sd::KF), dim3(256), 0, s, x, rows, J, F, 0, w.xprev);
    hipLaunchKernelGGL(sd::k_pad_frame, grid(rows * J * sd::KF), dim3(256), 0, s, x, rows, J, F, 1, w.xlast);
    hipLaunchKernelGGL(sd::k_identity, grid((int64_t)J * J), dim3(256), 0, s, w.ident, J);
    hipLaunchKernelGGL(sd::k_gx_table, dim3(1), dim3(64), 0, s, d->G, d->G_add, J, (int)ph, w.gx);
    DHIP(hipGetLastError());
    DHIP(sd::launch_ghat(d->init_G, w.ghat_init, J, 1, s));
    DHIP(sd::launch_ghat(d->fc_G, w.ghat_fc, J, 1, s));
    // hx_0 = initial_hidden_h([x_prev | h]); x_res = W_ih [x_last | h] + b_ih (unmixed: G = I)
    const int64_t JH = (int64_t)J * H, JH3 = 3 * JH;
    DHIP(sd::launch_graph_linear(sd::gl(d, w.xprev, sd::KF, h, L, w.winit, d->init_bias, w.ghat_init, H, w.h0, JH, rows, 0), false, s));
    DHIP(sd::launch_graph_linear(sd::gl(d, w.xlast, sd::KF, h, L, w.wih, d->bias_ih, w.ident, 3 * H, w.xres, JH3, rows, 0), false, s));
    size_t gate_lds = ((size_t)J * 3 * H + (size_t)J * J) * sizeof(float);
    if (gate_lds > 64 * 1024)
        DHIP(hipFuncSetAttribute((const void*)sd::k_gru_gate, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gate_lds));
    float* hx = w.h0;
    float* hn = w.h1;
    for (int t = 0; t < ph; ++t) {
        const float* gxt = w.gx + (size_t)t * J * J;
        DHIP(sd::launch_graph_linear(sd::gl(d, hx, H, nullptr, 0, d->weight_hh, d->bias_hh, gxt, 3 * H, w.hres, JH3, rows, 0), false, s));
        hipLaunchKernelGGL(sd::k_gru_gate, dim3((unsigned)rows), dim3(256), gate_lds, s, w.xres, w.hres, gxt, hx, hn, J, H);
        DHIP(hipGetLastError());
        DHIP(sd::launch_graph_linear(sd::gl(d, hn, H, nullptr, 0, d->fc_weight, d->fc_bias, w.ghat_fc, F, out + (int64_t)t * J * F,
                                            (int64_t)ph * J * F, rows, 1), false, s));
        float* tmp = hx;
        hx = hn;
        hn = tmp;
    }
#undef DHIP
    return SD_OK;
}

size_t sd_gru_encode_workspace_bytes(const sd_gru_decoder_desc* d, int64_t rows, int32_t frames) {
    if (check_desc(d) || rows < 0 || frames < 1) return 0;
    return sd::carve(d, rows, frames, nullptr, nullptr) + 256;
}

// Encoder.forward + z_activation (encoder.py:75-80, autoencoder.py:47-51): the GRU over `frames`
// observed frames from hx_0 = initial_hidden1(x[:, 0]), then z = tanh(tanh(fc(hx_T))).  The
// descriptor's init_* are initial_hidden1 (input F), weight_ih is (types, 3H, F), latent_size is
// the fc output width (the latent), G_add must be NULL (no additive influence in the encoder).
int sd_gru_encode(const sd_gru_decoder_desc* d, const float* x, int64_t rows, int32_t frames, float* z,
                  void* workspace, size_t ws_bytes, void* stream) {
    int rc = check_desc(d);
    if (rc) return rc;
    if (rows < 0 || frames < 1) return dfail(SD_E_INVALID, "rows >= 0 and frames >= 1 required");
    if (rows == 0) return SD_OK;
    if (!x || !z) return dfail(SD_E_INVALID, "null input / output");
    if (d->G_add) return dfail(SD_E_INVALID, "the encoder GRU has no additive graph influence (G_add must be NULL)");
    const size_t need = sd::carve(d, rows, frames, nullptr, nullptr);
    char* base = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    if (!workspace || (size_t)(base - (char*)workspace) + need > ws_bytes)
        return dfail(SD_E_INVALID, "workspace too small: need " + std::to_string(need + 256));
    sd::DecWS w;
    sd::carve(d, rows, frames, base, &w);
    hipStream_t s = (hipStream_t)stream;
    const int J = d->num_nodes, F = d->feature_size, L = d->latent_size, H = d->hidden_size;
    const int nt = d->num_node_types > 0 ? d->num_node_types : 1;
#define DHIP(expr)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return dfail(SD_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
    auto grid = [](int64_t n) { return dim3((unsigned)((n + 255) / 256)); };
    // F-wide weights padded to KF (no latent part: L' = 0); frames padded one at a time into xprev
    hipLaunchKernelGGL(sd::k_pad_w, grid((int64_t)nt * H * sd::KF), dim3(256), 0, s, d->init_weight, (int64_t)nt * H, F, 0, w.winit);
    hipLaunchKernelGGL(sd::k_pad_w, grid((int64_t)nt * 3 * H * sd::KF), dim3(256), 0, s, d->weight_ih, (int64_t)nt * 3 * H, F, 0, w.wih);
    hipLaunchKernelGGL(sd::k_identity, grid((int64_t)J * J), dim3(256), 0, s, w.ident, J);
    hipLaunchKernelGGL(sd::k_gx_table, dim3(1), dim3(64), 0, s, d->G, (const float*)nullptr, J, (int)frames, w.gx);
    DHIP(hipGetLastError());
    DHIP(sd::launch_ghat(d->init_G, w.ghat_init, J, 1, s));
    DHIP(sd::launch_ghat(d->fc_G, w.ghat_fc, J, 1, s));
    const int64_t JH = (int64_t)J * H, JH3 = 3 * JH;
    size_t gate_lds = ((size_t)J * 3 * H + (size_t)J * J) * sizeof(float);
    if (gate_lds > 64 * 1024)
        DHIP(hipFuncSetAttribute((const void*)sd::k_gru_gate, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gate_lds));
    // x (rows, frames, J, F): frame t -> xprev via k_pad_frame's (rows, 2, J, F) view at stride
    // frames: done with a strided copy kernel of its own
    hipLaunchKernelGGL(sd::k_pad_frame_t, grid(rows * J * sd::KF), dim3(256), 0, s, x, rows, frames, J, F, 0, w.xprev);
    DHIP(sd::launch_graph_linear(sd::gl(d, w.xprev, sd::KF, nullptr, 0, w.winit, d->init_bias, w.ghat_init, H, w.h0, JH, rows, 0), false, s));
    float* hx = w.h0;
    float* hn = w.h1;
    for (int t = 0; t < frames; ++t) {
        const float* gxt = w.gx + (size_t)t * J * J;
        if (t > 0) hipLaunchKernelGGL(sd::k_pad_frame_t, grid(rows * J * sd::KF), dim3(256), 0, s, x, rows, frames, J, F, t, w.xprev);
        DHIP(sd::launch_graph_linear(sd::gl(d, w.xprev, sd::KF, nullptr, 0, w.wih, d->bias_ih, w.ident, 3 * H, w.xres, JH3, rows, 0), false, s));
        DHIP(sd::launch_graph_linear(sd::gl(d, hx, H, nullptr, 0, d->weight_hh, d->bias_hh, gxt, 3 * H, w.hres, JH3, rows, 0), false, s));
        hipLaunchKernelGGL(sd::k_gru_gate, dim3((unsigned)rows), dim3(256), gate_lds, s, w.xres, w.hres, gxt, hx, hn, J, H);
        DHIP(hipGetLastError());
        float* tmp = hx;
        hx = hn;
        hn = tmp;
    }
    // z = tanh(tanh(Ghat_fc (W_fc hx + b_fc))): the fc launch's tanh epilogue, then one more tanh
    DHIP(sd::launch_graph_linear(sd::gl(d, hx, H, nullptr, 0, d->fc_weight, d->fc_bias, w.ghat_fc, L, z, (int64_t)J * L, rows, 1), false, s));
    hipLaunchKernelGGL(sd::k_tanh_inplace, grid(rows * J * L), dim3(256), 0, s, z, rows * J * L);
    DHIP(hipGetLastError());
#undef DHIP
    return SD_OK;
}

}  // extern "C"
