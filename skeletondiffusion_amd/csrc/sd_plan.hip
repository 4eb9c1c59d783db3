// Host side of libskeldiff: plan construction (state_dict-keyed tensor registry), one-time
// packing, the per-step launch sequence of the Denoiser + posterior update, and the hipGraph
// capture of the whole T-step chain.  Implements include/skeldiff.h.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/skeldiff.h"
#include "sd_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

}  // namespace

int sd::set_error(int code, const std::string& msg) { return fail(code, msg); }
int sd::diag_flags() {
    static const int v = [] {
        const char* e = getenv("SKELDIFF_DIAG");
        return e ? atoi(e) : 0;
    }();
    return v;
}

#ifdef SD_DEBUG_LDS
unsigned* sd::debug_counters() {
    static unsigned* buf = [] {
        unsigned* b = nullptr;
        if (hipMalloc(&b, 8 * sizeof(unsigned)) != hipSuccess || hipMemset(b, 0, 8 * sizeof(unsigned)) != hipSuccess) abort();
        return b;
    }();
    return buf;
}
#endif

namespace {

#define SD_HIP(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return fail(SD_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Slot {
    std::string name;
    int64_t numel = 0;
    float* dev = nullptr;
    bool set = false;
};

// One StaticGraphLinear of the plan.
struct GL {
    int w = -1, g = -1, b = -1;  // slot indices (b = -1: no bias)
    int K1 = 0, K2 = 0, N = 0;
    float* ghat = nullptr;       // packed (J, J)
    const float* wuse = nullptr; // weights used by the kernel (folded copy for RMS layers)
    bool rms = false;
    int gain = -1;               // RMSNorm gain slot folded into this layer
    int lnw = -1, lnb = -1;      // Block.norm LayerNorm(J) affine slots (norm_type 'layer')
    sd::SplitW split;            // f16 hi/lo B fragments of wuse for the v4 kernel
    sd::SplitW split_bf;         // bf16 fragments of wuse (precision mode 2)
};

struct GraphKey {
    int64_t rows;
    const void* ptrs[10];
    int64_t cond_repeat;
    int32_t flags;
    int32_t chains;
    int32_t prec;
    int32_t variant, gl4_cfg, gl4_stage, split, upd_elem, v5_valu, attn_tail;  // the plan's kernel options at capture time
    void* stream;
    bool operator<(const GraphKey& o) const { return std::memcmp(this, &o, sizeof(GraphKey)) < 0; }
};

// The captured graphs of one sd_sample_loop shape (one per row chain).  Shared by the cache and
// every caller that is about to launch them, so an eviction by another thread never destroys an
// exec a caller still holds; the last holder destroys them after their own last launches are done
// (an event recorded behind each launch: no device-wide drain, other streams are not waited for).
struct GraphSet {
    std::vector<hipGraphExec_t> execs;
    // one per exec, recorded on the exec's stream after each launch; every launch first makes its
    // stream wait for the previous launch's record (under `mu`), so the last record completing
    // means every launch of the exec is done
    std::vector<hipEvent_t> done;
    std::mutex mu;
    unsigned route_bits = 0;       // sd::RouteBits the captured chains launch
    ~GraphSet() {
        for (auto e : done) {
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
        for (auto x : execs) (void)hipGraphExecDestroy(x);
    }
};

}  // namespace

// Diagnostics (tools/hazard_snap.py): when an arena is set (sd_debug_snapshot),
// every graph-linear call of run_denoiser copies its phase-1 scratch Y (zs) and its output rows
// into slot (step, call) of the arena at the chain's row offset, and the posterior update its
// output into call slot kSnapCalls - 1, so a run with row chains can be compared slot by slot
// with a one-chain run.  Never set on the product path.
namespace {
constexpr int kSnapCalls = 40;
struct Snap {
    float* arena = nullptr;
    int64_t slot = 0, half = 0;  // floats per slot; the Y region is [0, half), the output region the rest
    int nslots = 0;
    std::vector<int> meta;  // per slot: N, output floats per row, Y floats per row
};
Snap g_snap;
// diagnostics (sd_debug_update_dump): the first update of a sampling call dumps its inputs
struct UpdDump {
    float *x0 = nullptr, *xt = nullptr, *ev = nullptr;
};
UpdDump g_dump;
}  // namespace

// Row chains.  Rows never interact inside the Denoiser or the posterior update, so the T-step
// chain of rows [r0, r1) is independent of every other row range: record_loop splits the batch
// into `chains` row ranges (multiples of 32 rows) and records each range's
// T steps on its own stream, forked from and joined back into the caller's stream.  Kernels of
// different chains then run concurrently, so one chain's idle CUs (a 200-workgroup graph linear
// on 256 CUs, the last wave of a 800-workgroup attention launch) take the other chain's
// workgroups instead of waiting for the next kernel boundary.
static const int g_chains = [] {
    const char* e = getenv("SKELDIFF_CHAINS");
    const int v = e ? atoi(e) : 0;
    return (v >= 0 && v <= 8) ? v : 0;  // 0: per batch size (chain_count)
}();


struct sd_plan {
    sd_plan_desc d{};
    int J = 0, D = 0, C = 0, H = 0, O = 0, hid = 0, T = 0, depth = 0, nres = 0, ntypes = 1;
    std::vector<int> types;
    std::vector<Slot> slots;
    std::map<std::string, int> index;
    bool finalized = false;
    bool fuse_ok = false;  // to_qkv + attention fusable (v4 split weights, J <= 17 or 21, dim_head 32)
    bool blk_ok = false;   // every layer on v4 with row-blocked intermediate activations
    int prec = 0;          // sd_plan_set_precision: 0 f32-accurate, 1 half (f16 products)
    // kernel options (sd_plan_set_option), initialised from the process defaults at creation
    int variant = 0, gl4_cfg = 0, gl4_stage = 0, split = 0, chains = 0;
    int upd_elem = 0;  // SD_OPT_UPDATE_KERNEL: 1 = the element-per-thread update forms
    int v5_valu = 0;   // SD_OPT_V5_MIX: 1 = the VALU mixing pass of v5
    int attn_tail = 0;  // SD_OPT_ATTENTION: 0 auto (= 2 where it applies), 2 k_attention_mix, 3 separate mixing pass
    bool fuse_attention_now() const { return fuse_ok && (variant == 0 || variant == 4); }
    // SD_OPT_ATTENTION 2 where it applies: the v5 route's to_qkv mixing inside the attention kernel
    bool attn_mix_now() const {
        return (attn_tail == 0 || attn_tail == 2) && J >= 49 && J <= 52 && d.attn_dim_head == 32 && (variant == 0 || variant == 5) && prec != 2;
    }
    bool blocked_now() const { return blk_ok && fuse_attention_now() && prec != 2; }
    std::vector<void*> allocs;

    GL init_lin;
    std::vector<GL> r1, r2;        // ResnetBlock block1/block2 for layers.{L}.0, L < 2*depth, then final
    std::vector<int> mlp_w, mlp_b; // ResnetBlock mlp.1 weight/bias slots (FiLM)
    std::vector<GL> qkv, outp;     // attention (or single GL when use_attention == 0)
    std::vector<bool> has_attn;
    GL fres_res, fglin;
    int t1w = -1, t1b = -1, t3w = -1, t3b = -1;
    int s_c1 = -1, s_c2 = -1, s_lv = -1, s_u = -1;

    float* film = nullptr;  // (nres, T, 2H) raw Linear(tanh(temb)) outputs
    float* sig = nullptr;   // (T, J) or (T)
    std::vector<float> iso_c1, iso_c2, iso_sig;  // host copies of the scalar tables (isotropic)
    std::vector<float> iso_xa, iso_xb;           // pred_noise / pred_v: x0 = xa[t] x_t - xb[t] act(out)
    int s_xa = -1, s_xb = -1;

    std::mutex gmu;
    std::map<GraphKey, std::shared_ptr<GraphSet>> graphs;  // one graph per row chain
    // row chains (record_loop): auxiliary streams + fork/join events, created on first use
    static constexpr int kMaxChains = 8;
    std::mutex cmu;
    std::atomic<int> last_chains{0};  // SD_OPT_LAST_CHAINS
    std::atomic<unsigned> last_route{0};  // SD_OPT_LAST_ROUTE
    hipStream_t aux[kMaxChains] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kMaxChains] = {};

    ~sd_plan() {
        graphs.clear();
        for (int i = 0; i < kMaxChains; ++i) {
            if (aux[i]) (void)hipStreamDestroy(aux[i]);
            if (ev_join[i]) (void)hipEventDestroy(ev_join[i]);
        }
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (auto& s : slots)
            if (s.dev) (void)hipFree(s.dev);
        for (void* p : allocs) (void)hipFree(p);
    }

    int add(const std::string& name, int64_t numel) {
        const int id = (int)slots.size();
        slots.push_back(Slot{name, numel, nullptr, false});
        index[name] = id;
        return id;
    }
    GL add_gl(const std::string& name, int K1, int K2, int N, bool bias) {
        GL g;
        const int64_t K = K1 + K2;
        g.g = add(name + ".G", (int64_t)J * J);
        g.w = add(name + ".weight", (int64_t)ntypes * N * K);
        g.b = bias ? add(name + ".bias", (int64_t)ntypes * N) : -1;
        g.K1 = K1;
        g.K2 = K2;
        g.N = N;
        return g;
    }
    // ResnetBlock Block (attention.py:49-75): proj, then with norm_type 'layer' its LayerNorm(J)
    GL add_block(const std::string& name, int K1, int K2, int N) {
        GL g = add_gl(name + ".proj", K1, K2, N, true);
        if (d.norm_type == 1) {
            g.lnw = add(name + ".norm.norm.weight", J);
            g.lnb = add(name + ".norm.norm.bias", J);
        }
        return g;
    }
    const float* ptr(int slot) const { return slot < 0 ? nullptr : slots[slot].dev; }
};

namespace {

int check_dims(const sd_plan_desc* d) {
    if (!d) return fail(SD_E_INVALID, "null desc");
    if (d->num_nodes < 1 || d->num_nodes > sd::kMaxNodes)
        return fail(SD_E_INVALID, "num_nodes must be in [1, 64]");
    if (d->latent_dim <= 0 || d->latent_dim % 16) return fail(SD_E_INVALID, "latent_dim must be a positive multiple of 16");
    if (d->cond_dim != 0 && d->cond_dim % 16) return fail(SD_E_INVALID, "cond_dim must be 0 or a multiple of 16");
    if (d->out_dim != d->latent_dim) return fail(SD_E_INVALID, "out_dim must equal latent_dim for sampling");
    if (d->depth < 1) return fail(SD_E_INVALID, "depth must be >= 1");
    if (d->self_condition) return fail(SD_E_INVALID, "self_condition=True is not supported by the sampling engine");
    if (d->use_attention && (d->attn_heads < 1 || d->attn_dim_head <= 0 || d->attn_dim_head % 16))
        return fail(SD_E_INVALID, "attn_dim_head must be a positive multiple of 16");
    if (d->timesteps < 1) return fail(SD_E_INVALID, "timesteps must be >= 1");
    if (d->activation != 0 && d->activation != 1) return fail(SD_E_INVALID, "activation must be 0 (identity) or 1 (tanh)");
    if (d->objective < 0 || d->objective > 2) return fail(SD_E_INVALID, "objective must be 0 (pred_x0), 1 (pred_noise) or 2 (pred_v)");
    if (d->norm_type != 0 && d->norm_type != 1) return fail(SD_E_INVALID, "norm_type must be 0 ('none') or 1 ('layer')");
    if (d->norm_type == 1 && d->num_nodes != 16 && d->num_nodes != 17 && d->num_nodes != 21)
        return fail(SD_E_INVALID, "norm_type 'layer' runs in the v4 mixing epilogue: num_nodes 16, 17 or 21");
    if (d->objective != 0 && !d->isotropic)
        return fail(SD_E_INVALID, "the nonisotropic sampler supports objective pred_x0 only (the release configs; "
                                  "pred_v is not implemented in the reference, nonisotropic.py:122-124)");
    return SD_OK;
}

template <typename T>
int dalloc(sd_plan* p, T** out, size_t n) {
    void* q = nullptr;
    if (hipMalloc(&q, n * sizeof(T) + 16) != hipSuccess) return fail(SD_E_NOMEM, "hipMalloc failed");
    p->allocs.push_back(q);
    *out = (T*)q;
    return SD_OK;
}

// workspace carve (all offsets 256-B aligned)
struct WS {
    uint64_t* rng;      // {seed, row0} of the device noise (graph replays); rng + 4: status word
    float *x, *r, *h, *qkv, *o, *res, *x0, *img0, *img1;
};

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// floats per (row, node) of the qkv buffer: to_qkv's output, and the split route's pre-mix Y scratch
// of every graph-linear outside the attention block (the widest layer's N: at least H)
int64_t qkv_width(const sd_plan* p) {
    return std::max<int64_t>({p->d.use_attention ? 3 * (int64_t)p->hid : 0, (int64_t)p->H, (int64_t)p->O});
}

size_t carve(const sd_plan* p, int64_t rows, char* base, WS* w) {
    const size_t f = sizeof(float);
    const size_t rp = (size_t)((rows + 31) / 32 * 32);  // activations: padded to the 32-row blocks of the v4 layout
    const size_t nH = rp * p->J * p->H * f;
    const size_t nQ = rp * p->J * qkv_width(p) * f;
    const size_t nO = rp * p->J * (p->d.use_attention ? p->hid : p->H) * f;  // no attention: GL output
    const size_t nD = (size_t)rows * p->J * p->D * f;
    size_t off = 0;
    auto take = [&](size_t n) {
        char* q = base ? base + off : nullptr;
        off += align256(n);
        return q;
    };
    WS tmp;
    WS& W = w ? *w : tmp;
    W.rng = (uint64_t*)take(64);
    W.x = (float*)take(nH);
    W.r = (float*)take(nH);
    W.h = (float*)take(nH);
    W.qkv = (float*)take(nQ);
    W.o = (float*)take(nO);
    W.res = (float*)take(nH);
    W.x0 = (float*)take(nD);
    W.img0 = (float*)take(nD);
    W.img1 = (float*)take(nD);
    return off;
}

// the workspace's status word (range-guard flags, sd_workspace_status)
unsigned* ws_status(const WS& w) { return reinterpret_cast<unsigned*>(w.rng + 4); }
// entry points zero the status word
int ws_reset(const WS& w, hipStream_t s) {
    SD_HIP(hipMemsetAsync(ws_status(w), 0, sizeof(unsigned), s));
    return SD_OK;
}

sd::GLArgs gl_args(const sd_plan* p, const GL& g, const float* x1, int x1_div, const float* x2,
                   const float* film, const float* res, float* out, int64_t rows) {
    sd::GLArgs a{};
    a.x1 = x1;
    a.K1 = g.K1;
    a.x1_rs = (int64_t)p->J * g.K1;
    a.x1_div = x1_div;
    a.x2 = x2;
    a.K2 = g.K2;
    a.x2_rs = (int64_t)p->J * g.K2;
    a.W = g.wuse;
    a.bias = p->ptr(g.b);
    a.ln_w = p->ptr(g.lnw);
    a.ln_b = p->ptr(g.lnb);
    a.G = g.ghat;
    a.film = film;
    a.res = res;
    a.res_rs = (int64_t)p->J * g.N;
    a.out = out;
    a.out_rs = (int64_t)p->J * g.N;
    a.B = rows;
    a.N = g.N;
    a.J = p->J;
    a.act = 0;
    a.ntypes = p->ntypes;
    for (int j = 0; j < p->J; ++j) {
        a.wrow[j] = p->types[j] * g.N;
        a.ntype[j] = p->types[j];
    }
    const sd::SplitW& sw = p->prec == 2 ? g.split_bf : g.split;  // bf16 mode: the bf16 fragments
    a.wsp = sw.w;
    a.wsp_nct = sw.nct;
    a.wsp_unscale = sw.unscale;
    a.prec = p->prec;
    a.variant = p->variant;
    a.gl4_cfg = p->gl4_cfg;
    a.gl4_stage = p->gl4_stage;
    a.split = p->split;
    a.v5_valu = p->v5_valu;
#ifdef SD_DEBUG_LDS
    a.dbg = sd::debug_counters();
#endif
    return a;
}

// Optional per-launch event timing (sd_profile_step): classes 0 graph-linear, 1 attention,
// 2 update.  Events are recorded on the launch stream around each kernel.
struct Prof {
    std::vector<int> cls;
    std::vector<hipEvent_t> ev;  // pairs
    int pre(int c, hipStream_t s) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
        cls.push_back(c);
        ev.push_back(a);
        ev.push_back(b);
        return hipEventRecord(a, s) == hipSuccess ? 0 : -1;
    }
    int post(hipStream_t s) { return hipEventRecord(ev.back(), s) == hipSuccess ? 0 : -1; }
    ~Prof() {
        for (auto e : ev) (void)hipEventDestroy(e);
    }
};

#define SD_LAUNCH(prof, c, expr)                                                               \
    do {                                                                                       \
        if (prof && prof->pre(c, s)) return fail(SD_E_HIP, "hipEventRecord failed");          \
        SD_HIP(expr);                                                                          \
        if (prof && prof->post(s)) return fail(SD_E_HIP, "hipEventRecord failed");            \
    } while (0)

// Denoiser.forward (generator.py:86-107) for `rows` rows at time t.
// cond_phase: row 0 of this call is row cond_phase of a cond_repeat group (row chains)
int run_denoiser(const sd_plan* p, const float* x_t, const float* x_cond, int64_t cond_repeat,
                 int t, float* x0_out, int64_t rows, const WS& w, hipStream_t s, Prof* prof = nullptr,
                 int64_t cond_phase = 0, int tile_hint = 0, float* const* trace = nullptr,
                 int xt_bf16 = 0, int x0_bf16 = 0, int64_t route_rows = 0, int64_t snap_r0 = -1,
                 int snap_step = 0) {
    const int H = p->H;
    int snap_call = 0;
    auto snap = [&](const sd::GLArgs& g) -> int {
        const int call = snap_call++;
        if (!g_snap.arena || snap_r0 < 0) return SD_OK;
        const int64_t sl = (int64_t)snap_step * kSnapCalls + call;
        if (sl >= g_snap.nslots) return SD_OK;
        float* base = g_snap.arena + sl * g_snap.slot;
        const int64_t yrow = (int64_t)p->J * g.N;
        g_snap.meta[3 * sl] = g.N;
        g_snap.meta[3 * sl + 1] = (int)g.out_rs;
        g_snap.meta[3 * sl + 2] = (int)yrow;
        if (g.zs && (snap_r0 + rows) * yrow <= g_snap.half)
            SD_HIP(hipMemcpyAsync(base + snap_r0 * yrow, g.zs, rows * yrow * sizeof(float), hipMemcpyDeviceToDevice, s));
        if ((snap_r0 + rows) * g.out_rs <= g_snap.slot - g_snap.half)
            SD_HIP(hipMemcpyAsync(base + g_snap.half + snap_r0 * g.out_rs, g.out, rows * g.out_rs * sizeof(float),
                                  hipMemcpyDeviceToDevice, s));
        return SD_OK;
    };
    // v4 path: every intermediate activation in the row-blocked layout (coalesced x fragments);
    // the denoiser's inputs (x_t, x_cond) and output (x0) stay row-major
    const int B = p->blocked_now() ? 1 : 0;
    // bf16 mode (precision 2): the residual-stream activations (r, x, h, res; o without
    // attention) are bf16 in HBM, x_t / x0 as the caller says; x_cond, qkv and the attention
    // output stay f32
    const bool bf = p->prec == 2;
    auto bfl = [&](const float* q) -> int {
        if (!q) return 0;
        if (q == x_t) return xt_bf16;
        if (q == x0_out) return x0_bf16;
        return bf && (q == w.r || q == w.x || q == w.h || q == w.res || (!p->d.use_attention && q == w.o));
    };
    // sd_denoiser_trace: block outputs (rows, J, H) row-major, in the reference's module order
    int ntr = 0;
    auto record = [&](const float* buf) -> int {
        if (!trace) return SD_OK;
        float* dst = trace[ntr++];
        if (B) SD_HIP(sd::launch_unblock(dst, buf, rows, p->J, H, s));
        else SD_HIP(sd::launch_convert_rows(dst, 0, (int64_t)p->J * H, buf, bfl(buf), (int64_t)p->J * H, rows,
                                            (int64_t)p->J * H, s));
        return SD_OK;
    };
    // split-route / v5 scratch (pre-mix activations; v5: of layers whose residual aliases their
    // output): the qkv buffer, dead outside the attention block, as wide as the widest layer
    const int64_t zs_cap = (rows + 31) / 32 * 32 * p->J * qkv_width(p);
    auto lay = [B, tile_hint, &w, zs_cap, &bfl, route_rows](sd::GLArgs& g, int in, int res, int out) {
        g.status = ws_status(w);
        g.route_rows = route_rows;
        g.zs = w.qkv;
        g.zs_cap = zs_cap;
        g.tile_hint = tile_hint;
        g.x1_blk = g.x2_blk = B & in;
        g.res_blk = B & res;
        g.out_blk = B & out;
        g.x1_bf16 = bfl(g.x1);
        g.x2_bf16 = bfl(g.x2);
        g.res_bf16 = bfl(g.res);
        g.out_bf16 = bfl(g.out);
    };
    // init_lin on cat([x_cond, x]) (generator.py:91-94)
    sd::GLArgs a;
    // The init_lin output is `r` (generator.py:95, r = x.clone()); it is written to w.r and the
    // first ResnetBlock reads it from there and writes its result to w.x, so no copy is needed.
    if (p->C > 0) {
        a = gl_args(p, p->init_lin, x_cond, (int)cond_repeat, x_t, nullptr, nullptr, w.r, rows);
        a.x1_row0 = cond_phase;
    } else {
        a = gl_args(p, p->init_lin, x_t, 1, nullptr, nullptr, nullptr, w.r, rows);
    }
    lay(a, 0, 0, 1);
    SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
    int rc = snap(a);
    if (rc) return rc;
    rc = record(w.r);
    if (rc) return rc;

    const int L = 2 * p->depth;
    for (int l = 0; l < L; ++l) {
        const float* film = p->film + ((size_t)l * p->T + t) * 2 * H;
        const float* xin = (l == 0) ? w.r : w.x;
        // ResnetBlock: h = tanh(FiLM(GL1 x)); x = tanh(GL2 h) + x     (attention.py:96-102)
        a = gl_args(p, p->r1[l], xin, 1, nullptr, film, nullptr, w.h, rows);
        lay(a, 1, 1, 1);
        a.act = 1;
        SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
        if ((rc = snap(a))) return rc;
        a = gl_args(p, p->r2[l], w.h, 1, nullptr, nullptr, xin, w.x, rows);
        lay(a, 1, 1, 1);
        a.act = 1;
        SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
        if ((rc = snap(a))) return rc;
        if ((rc = record(w.x))) return rc;
        if (!p->has_attn[l]) {
            if ((rc = record(w.x))) return rc;  // nn.Identity in place of the last attention
            continue;
        }
        if (p->d.use_attention) {
            // Residual(PreNorm(Attention)): x = to_out(attn(to_qkv(rmsnorm(x)))) + x
            // q * dim_head ** -0.5 (attention.py:114,128): Python double scalar cast to fp32
            const float qscale = (float)std::pow((double)p->d.attn_dim_head, -0.5);
            hipError_t fused = hipErrorNotSupported;
            if (p->fuse_attention_now()) {  // to_qkv + attention in one kernel, qkv stays on chip
                a = gl_args(p, p->qkv[l], w.x, 1, nullptr, nullptr, nullptr, w.o, rows);
                a.out_rs = (int64_t)p->J * p->hid;
                a.attn_heads = p->d.attn_heads;
                a.attn_scale = qscale;
                lay(a, 1, 1, 1);
                if (prof && prof->pre(0, s)) return fail(SD_E_HIP, "hipEventRecord failed");
                fused = sd::launch_qkv_attention_v4(a, true, s);
                if (fused != hipSuccess && fused != hipErrorNotSupported) SD_HIP(fused);
                if (prof && prof->post(s)) return fail(SD_E_HIP, "hipEventRecord failed");
                if (fused == hipSuccess && (rc = snap(a))) return rc;
            }
            if (fused == hipErrorNotSupported) {
                if (B) return fail(SD_E_INTERNAL, "row-blocked plan without the fused attention kernel");
                a = gl_args(p, p->qkv[l], w.x, 1, nullptr, nullptr, nullptr, w.qkv, rows);
                lay(a, 0, 0, 0);
                // SD_OPT_ATTENTION 2: the GEMM phase alone, k_attention_mix mixes (else, or where
                // the route cannot leave the pre-mix Y in qkv, the whole layer)
                a.skip_mix = p->attn_mix_now() ? 1 : 0;
                if (prof && prof->pre(0, s)) return fail(SD_E_HIP, "hipEventRecord failed");
                hipError_t ge = sd::launch_graph_linear(a, true, s);
                if (ge == hipErrorNotSupported && a.skip_mix) {
                    a.skip_mix = 0;
                    ge = sd::launch_graph_linear(a, true, s);
                }
                SD_HIP(ge);
                if (prof && prof->post(s)) return fail(SD_E_HIP, "hipEventRecord failed");
                if ((rc = snap(a))) return rc;
                sd::AttnArgs aa{w.qkv, w.o, rows, p->J, p->d.attn_heads, p->d.attn_dim_head, qscale,
                                a.skip_mix ? a.G : nullptr};
                SD_LAUNCH(prof, 1, sd::launch_attention(aa, s));
            }
            a = gl_args(p, p->outp[l], w.o, 1, nullptr, nullptr, w.x, w.x, rows);
            lay(a, 1, 1, 1);
            SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
            if ((rc = snap(a))) return rc;
        } else {
            // Residual(PreNorm(StaticGraphLinear)): x = GL(rmsnorm(x)) + x, written to the `o`
            // buffer (sized like x in this configuration: a graph-linear may not write its own
            // input, sibling column tiles still read it) and copied back as x
            a = gl_args(p, p->qkv[l], w.x, 1, nullptr, nullptr, w.x, w.o, rows);
            lay(a, 1, 1, 1);
            SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, true, s));
            if ((rc = snap(a))) return rc;
            const int64_t rp = B ? (rows + 31) / 32 * 32 : rows;
            SD_LAUNCH(prof, 0, sd::launch_convert_rows(w.x, bfl(w.x), (int64_t)p->J * H, w.o, bfl(w.o), (int64_t)p->J * H, rp,
                                                       (int64_t)p->J * H, s));
        }
        if ((rc = record(w.x))) return rc;
    }
    // final_res_block on cat(x, r) (generator.py:104-106)
    const float* film = p->film + ((size_t)L * p->T + t) * 2 * H;
    a = gl_args(p, p->fres_res, w.x, 1, w.r, nullptr, nullptr, w.res, rows);
    lay(a, 1, 1, 1);
    SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
    if ((rc = snap(a))) return rc;
    a = gl_args(p, p->r1[L], w.x, 1, w.r, film, nullptr, w.h, rows);
    lay(a, 1, 1, 1);
    a.act = 1;
    SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
    if ((rc = snap(a))) return rc;
    a = gl_args(p, p->r2[L], w.h, 1, nullptr, nullptr, w.res, w.res, rows);
    lay(a, 1, 1, 1);
    a.act = 1;
    SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
    if ((rc = snap(a))) return rc;
    if ((rc = record(w.res))) return rc;
    // final_glin (generator.py:107)
    a = gl_args(p, p->fglin, w.res, 1, nullptr, nullptr, nullptr, x0_out, rows);
    lay(a, 1, 1, 0);
    SD_LAUNCH(prof, 0, sd::launch_graph_linear(a, false, s));
    if ((rc = snap(a))) return rc;
    return SD_OK;
}

int run_update(const sd_plan* p, const float* x0, const float* xt, const float* eps,
               int64_t eps_rs, int noise_mode, uint64_t seed, int64_t row0,
               const uint64_t* rng_dev, int t, float* out, float* out2, int64_t out2_rs,
               float* mean_out, int64_t mean_rs, float* noise_out, int64_t noise_rs, int64_t rows,
               hipStream_t s, Prof* prof = nullptr, int64_t row_shift = 0, int x0_bf16 = 0, int xt_bf16 = 0,
               int out_bf16 = 0, int clip = 1) {
    sd::UpdArgs u{};
    u.clip = clip;
    u.x0_bf16 = x0_bf16;
    u.xt_bf16 = xt_bf16;
    u.out_bf16 = out_bf16;
    u.x0 = x0;
    u.xt = xt;
    u.eps = eps;
    u.eps_rs = eps_rs;
    u.iso = p->d.isotropic;
    u.act = p->d.activation;
    u.noise_mode = (t > 0) ? noise_mode : 0;
    u.seed = seed;
    u.row0 = row0;
    u.step = t;
    u.rng_dev = rng_dev;
    u.row_shift = row_shift;
    u.out = out;
    u.out2 = out2;
    u.out2_rs = out2_rs;
    u.mean_out = mean_out;
    u.mean_rs = mean_rs;
    u.noise_out = noise_out;
    u.noise_rs = noise_rs;
    u.B = rows;
    u.J = p->J;
    u.D = p->D;
    u.elementwise = p->upd_elem == 1;
#ifdef SD_DEBUG_LDS
    u.dbg = sd::debug_counters();
#endif
    u.dump_x0 = g_dump.x0;
    u.dump_xt = g_dump.xt;
    u.dump_ev = g_dump.ev;
    if (p->d.isotropic) {
        u.c1s = p->iso_c1[t];
        u.c2s = p->iso_c2[t];
        u.sigs = p->iso_sig[t];
        if (p->d.objective) {
            u.obj = 1;
            u.xa = p->iso_xa[t];
            u.xb = p->iso_xb[t];
        }
    } else {
        const size_t JJ = (size_t)p->J * p->J;
        u.C1 = p->ptr(p->s_c1) + t * JJ;
        u.C2 = p->ptr(p->s_c2) + t * JJ;
        u.U = p->ptr(p->s_u);
        u.sig = p->sig + (size_t)t * p->J;
    }
    SD_LAUNCH(prof, 2, sd::launch_update(u, s));
    return SD_OK;
}

// algorithmic FLOPs of one reverse step for `rows` rows: [graph-linear, attention, update]
void step_flops(const sd_plan* p, int64_t rows, double* f) {
    const double J = p->J, R = (double)rows;
    auto gl = [&](const GL& g) { return 2.0 * R * J * g.N * (g.K1 + g.K2) + 2.0 * R * J * J * g.N; };
    f[0] = gl(p->init_lin) + gl(p->fres_res) + gl(p->fglin);
    for (auto& g : p->r1) f[0] += gl(g);
    for (auto& g : p->r2) f[0] += gl(g);
    f[1] = 0.0;
    for (size_t l = 0; l < p->has_attn.size(); ++l) {
        if (!p->has_attn[l]) continue;
        f[0] += gl(p->qkv[l]);
        if (p->d.use_attention) {
            f[0] += gl(p->outp[l]);
            f[1] += 4.0 * R * J * J * p->d.attn_dim_head * p->d.attn_heads;  // QK^T and PV
        }
    }
    // C1 x0 + C2 x_t + U (sigma eps): three J x J products per latent column
    f[2] = p->d.isotropic ? 6.0 * R * J * p->D : 6.0 * R * J * J * p->D;
}

}  // namespace

extern "C" {

int32_t sd_abi_version(void) { return SD_ABI_VERSION; }

#ifndef SD_BUILD_INFO
#define SD_BUILD_INFO "unknown (built outside build.py)"
#endif
const char* sd_build_info(void) { return SD_BUILD_INFO; }

// Diagnostics only (tools/hazard_snap.py; not in include/skeldiff.h): set (arena != null) or clear
// the snapshot arena of run_denoiser / record_loop.  slot_floats per slot, the first y_floats of
// it for the phase-1 scratch Y.  Not thread-safe; never used by the product path.
int sd_debug_snapshot(float* arena, int64_t slot_floats, int64_t y_floats, int32_t nslots) {
    g_snap.arena = arena;
    g_snap.slot = slot_floats;
    g_snap.half = y_floats;
    g_snap.nslots = arena ? nslots : 0;
    g_snap.meta.assign(3 * (size_t)std::max(nslots, 0), 0);
    return SD_OK;
}
// Diagnostics only: the first posterior update of the next sampling calls stores its inputs
// (x0 after activation and clamp, x_t, sigma eps; (rows, J, D) each) to these buffers; nulls = off
int sd_debug_update_dump(float* x0, float* xt, float* ev) {
    g_dump = UpdDump{x0, xt, ev};
    if (!x0 || !xt || !ev) g_dump = UpdDump{};
    return SD_OK;
}
int sd_debug_snapshot_meta(int32_t slot, int32_t* out3) {
    if (slot < 0 || 3 * (size_t)slot + 2 >= g_snap.meta.size()) return SD_E_INVALID;
    for (int i = 0; i < 3; ++i) out3[i] = g_snap.meta[3 * (size_t)slot + i];
    return SD_OK;
}

const char* sd_last_error(void) { return g_err.c_str(); }

int sd_plan_create(sd_plan** out, const sd_plan_desc* desc) {
    if (!out) return fail(SD_E_INVALID, "null out");
    *out = nullptr;
    int rc = check_dims(desc);
    if (rc) return rc;
    std::unique_ptr<sd_plan> p(new sd_plan());
    p->variant = sd::graph_linear_variant();
    if (desc->norm_type == 1 && p->variant != 0 && p->variant != 4)
        return fail(SD_E_INVALID, "norm_type 'layer' runs on the v4 kernels only (SKELDIFF_GL_VARIANT 0 or 4)");
    p->gl4_cfg = sd::gl4_tile_default();
    p->gl4_stage = sd::gl4_stage_default();
    p->chains = g_chains;
#ifdef SD_DEBUG_LDS
    (void)sd::debug_counters();  // allocated here, never during a stream capture
#endif
    p->d = *desc;
    p->J = desc->num_nodes;
    p->D = desc->latent_dim;
    p->C = desc->cond_dim;
    p->H = desc->latent_dim + desc->cond_dim;
    p->O = desc->out_dim;
    p->hid = desc->use_attention ? desc->attn_heads * desc->attn_dim_head : 0;
    p->T = desc->timesteps;
    p->depth = desc->depth;
    p->types.assign(p->J, 0);
    if (desc->num_node_types > 0) {
        if (!desc->node_types) return fail(SD_E_INVALID, "node_types is null");
        for (int j = 0; j < p->J; ++j) {
            const int64_t v = desc->node_types[j];
            if (v < 0 || v >= desc->num_node_types) return fail(SD_E_INVALID, "node_types out of range");
            p->types[j] = (int)v;
        }
        p->ntypes = desc->num_node_types;
    }
    const int J = p->J, H = p->H, hid = p->hid;
    p->ntypes = desc->num_node_types > 0 ? desc->num_node_types : 1;

    // tensor registry in the reference layout (generator.py:30-84)
    const std::string m = "model.";
    p->init_lin = p->add_gl(m + "init_lin", p->C > 0 ? p->C : p->D, p->C > 0 ? p->D : 0, H, true);
    p->t1w = p->add(m + "time_mlp.1.weight", (int64_t)4 * H * H);
    p->t1b = p->add(m + "time_mlp.1.bias", 4 * H);
    p->t3w = p->add(m + "time_mlp.3.weight", (int64_t)16 * H * H);
    p->t3b = p->add(m + "time_mlp.3.bias", 4 * H);
    const int L = 2 * p->depth;
    p->qkv.resize(L);
    p->outp.resize(L);
    p->has_attn.assign(L, false);
    for (int l = 0; l < L; ++l) {
        const std::string r = m + "layers." + std::to_string(l) + ".0.";
        p->mlp_w.push_back(p->add(r + "mlp.1.weight", (int64_t)2 * H * 4 * H));
        p->mlp_b.push_back(p->add(r + "mlp.1.bias", 2 * H));
        p->r1.push_back(p->add_block(r + "block1", H, 0, H));
        p->r2.push_back(p->add_block(r + "block2", H, 0, H));
        const bool attn = (l != L - 1);  // generator.py:71-76: last layer gets nn.Identity
        p->has_attn[l] = attn;
        if (!attn) continue;
        const std::string a = m + "layers." + std::to_string(l) + ".1.fn.";
        const int gain = p->add(a + "norm.g", H);
        if (desc->use_attention) {
            p->qkv[l] = p->add_gl(a + "fn.to_qkv", H, 0, 3 * hid, false);
            p->outp[l] = p->add_gl(a + "fn.to_out", hid, 0, H, false);
        } else {
            p->qkv[l] = p->add_gl(a + "fn", H, 0, H, false);
        }
        p->qkv[l].rms = true;
        p->qkv[l].gain = gain;
    }
    {
        const std::string r = m + "final_res_block.";
        p->mlp_w.push_back(p->add(r + "mlp.1.weight", (int64_t)2 * H * 4 * H));
        p->mlp_b.push_back(p->add(r + "mlp.1.bias", 2 * H));
        p->r1.push_back(p->add_block(r + "block1", H, H, H));
        p->r2.push_back(p->add_block(r + "block2", H, 0, H));
        p->fres_res = p->add_gl(r + "res_linear", H, H, H, false);
    }
    p->fglin = p->add_gl(m + "final_glin", H, 0, p->O, true);
    p->nres = L + 1;
    if (desc->isotropic) {
        p->s_c1 = p->add("posterior_mean_coef1", p->T);
        p->s_c2 = p->add("posterior_mean_coef2", p->T);
        p->s_lv = p->add("posterior_log_variance_clipped", p->T);
        if (desc->objective == 1) {  // predict_start_from_noise (isotropic.py:48-52)
            p->s_xa = p->add("sqrt_recip_alphas_cumprod", p->T);
            p->s_xb = p->add("sqrt_recipm1_alphas_cumprod", p->T);
        } else if (desc->objective == 2) {  // predict_start_from_v (isotropic.py:66-70)
            p->s_xa = p->add("sqrt_alphas_cumprod", p->T);
            p->s_xb = p->add("sqrt_one_minus_alphas_cumprod", p->T);
        }
    } else {
        p->s_c1 = p->add("posterior_mean_coef1_x0", (int64_t)p->T * J * J);
        p->s_c2 = p->add("posterior_mean_coef2_xt", (int64_t)p->T * J * J);
        p->s_lv = p->add("Lambda_posterior_log_variance_clipped", (int64_t)p->T * J);
        p->s_u = p->add("U", (int64_t)J * J);
    }
    *out = p.release();
    return SD_OK;
}

void sd_plan_destroy(sd_plan* plan) { delete plan; }

int32_t sd_plan_num_tensors(const sd_plan* plan) { return plan ? (int32_t)plan->slots.size() : 0; }

const char* sd_plan_tensor_name(const sd_plan* plan, int32_t i) {
    if (!plan || i < 0 || i >= (int32_t)plan->slots.size()) return nullptr;
    return plan->slots[i].name.c_str();
}

int64_t sd_plan_tensor_numel(const sd_plan* plan, int32_t i) {
    if (!plan || i < 0 || i >= (int32_t)plan->slots.size()) return -1;
    return plan->slots[i].numel;
}

int sd_plan_set_tensor(sd_plan* plan, const char* name, const float* data, int64_t numel, void* stream) {
    if (!plan || !name || !data) return fail(SD_E_INVALID, "null argument");
    if (plan->finalized) return fail(SD_E_STATE, "plan already finalized");
    auto it = plan->index.find(name);
    if (it == plan->index.end()) return fail(SD_E_INVALID, std::string("unexpected tensor: ") + name);
    Slot& s = plan->slots[it->second];
    if (numel != s.numel)
        return fail(SD_E_INVALID, std::string("size mismatch for ") + name + ": got " +
                                      std::to_string(numel) + ", expected " + std::to_string(s.numel));
    if (!s.dev) SD_HIP(hipMalloc(&s.dev, (size_t)numel * sizeof(float) + 16));
    SD_HIP(hipMemcpyAsync(s.dev, data, (size_t)numel * sizeof(float), hipMemcpyDefault, (hipStream_t)stream));
    // the source may be pageable host memory the caller frees right after: complete the copy
    SD_HIP(hipStreamSynchronize((hipStream_t)stream));
    s.set = true;
    return SD_OK;
}

int sd_plan_finalize(sd_plan* p, void* stream_) {
    if (!p) return fail(SD_E_INVALID, "null plan");
    if (p->finalized) return SD_OK;
    for (auto& s : p->slots)
        if (!s.set) return fail(SD_E_STATE, "missing tensor: " + s.name);
    hipStream_t s = (hipStream_t)stream_;
    const int J = p->J, H = p->H, T = p->T;
    int rc;

    auto pack_gl = [&](GL& g) -> int {
        int r = dalloc(p, &g.ghat, (size_t)J * J);
        if (r) return r;
        SD_HIP(sd::launch_ghat(p->ptr(g.g), g.ghat, J, p->d.learn_influence, s));
        g.wuse = p->ptr(g.w);
        if (g.rms) {  // fold RMSNorm gain * sqrt(dim) (attention.py:36) into the projection
            float* wf = nullptr;
            const int64_t K = g.K1 + g.K2;
            const int64_t rows = (int64_t)p->ntypes * g.N;
            r = dalloc(p, &wf, (size_t)(rows * K));
            if (r) return r;
            SD_HIP(sd::launch_fold_gain(p->ptr(g.w), p->ptr(g.gain), std::sqrt((float)H), wf, rows, (int)K, s));
            g.wuse = wf;
        }
        if ((g.K1 + g.K2) % 16 == 0 && g.K1 % 16 == 0) {
            SD_HIP(sd::make_split_weights(g.wuse, p->ntypes, g.N, g.K1 + g.K2, &g.split, s));
            p->allocs.push_back(g.split.w);
            SD_HIP(sd::make_bf16_weights(g.wuse, p->ntypes, g.N, g.K1 + g.K2, &g.split_bf, s));
            p->allocs.push_back(g.split_bf.w);
        }
        return SD_OK;
    };
    if ((rc = pack_gl(p->init_lin))) return rc;
    for (auto& g : p->r1)
        if ((rc = pack_gl(g))) return rc;
    for (auto& g : p->r2)
        if ((rc = pack_gl(g))) return rc;
    for (size_t l = 0; l < p->qkv.size(); ++l) {
        if (!p->has_attn[l]) continue;
        if ((rc = pack_gl(p->qkv[l]))) return rc;
        if (p->d.use_attention && (rc = pack_gl(p->outp[l]))) return rc;
    }
    if ((rc = pack_gl(p->fres_res))) return rc;
    if ((rc = pack_gl(p->fglin))) return rc;
    p->fuse_ok = p->d.use_attention && (J <= 17 || J == 21) && p->d.attn_dim_head == 32;
    for (size_t l = 0; l < p->qkv.size(); ++l)
        if (p->has_attn[l] && !p->qkv[l].split.w) p->fuse_ok = false;
    // row-blocked activations need every graph-linear on v4 (split weights, K multiple of 32)
    p->blk_ok = p->fuse_ok && J == 16;
    auto v4ok = [](const GL& g) { return g.split.w && (g.K1 + g.K2) % 32 == 0; };
    if (!v4ok(p->init_lin) || !v4ok(p->fres_res) || !v4ok(p->fglin)) p->blk_ok = false;
    for (auto& g : p->r1)
        if (!v4ok(g)) p->blk_ok = false;
    for (auto& g : p->r2)
        if (!v4ok(g)) p->blk_ok = false;
    for (size_t l = 0; l < p->outp.size(); ++l)
        if (p->has_attn[l] && !v4ok(p->outp[l])) p->blk_ok = false;

    // time MLP (generator.py:50-55, 97) and per-block FiLM tables (attention.py:81-84, 96-100)
    float *emb = nullptr, *t1 = nullptr, *temb = nullptr;
    if ((rc = dalloc(p, &emb, (size_t)T * H))) return rc;
    if ((rc = dalloc(p, &t1, (size_t)T * 4 * H))) return rc;
    if ((rc = dalloc(p, &temb, (size_t)T * 4 * H))) return rc;
    const int half = H / 2;
    if (half < 2) return fail(SD_E_INVALID, "model dim too small for the sinusoidal embedding");
    const float neg_scale = (float)(-(std::log((double)p->d.sinusoidal_theta) / (double)(half - 1)));
    SD_HIP(sd::launch_sinusoidal(emb, T, H, neg_scale, s));
    SD_HIP(sd::launch_linear(emb, T, H, p->ptr(p->t1w), p->ptr(p->t1b), 4 * H, t1, 0, 1, s));
    SD_HIP(sd::launch_linear(t1, T, 4 * H, p->ptr(p->t3w), p->ptr(p->t3b), 4 * H, temb, 0, 0, s));
    if ((rc = dalloc(p, &p->film, (size_t)p->nres * T * 2 * H))) return rc;
    for (int r = 0; r < p->nres; ++r)
        SD_HIP(sd::launch_linear(temb, T, 4 * H, p->ptr(p->mlp_w[r]), p->ptr(p->mlp_b[r]), 2 * H,
                                 p->film + (size_t)r * T * 2 * H, 1, 0, s));

    // posterior tables
    if (p->d.isotropic) {
        std::vector<float> lv(T);
        p->iso_c1.resize(T);
        p->iso_c2.resize(T);
        p->iso_sig.resize(T);
        SD_HIP(hipMemcpyAsync(p->iso_c1.data(), p->ptr(p->s_c1), T * sizeof(float), hipMemcpyDeviceToHost, s));
        SD_HIP(hipMemcpyAsync(p->iso_c2.data(), p->ptr(p->s_c2), T * sizeof(float), hipMemcpyDeviceToHost, s));
        SD_HIP(hipMemcpyAsync(lv.data(), p->ptr(p->s_lv), T * sizeof(float), hipMemcpyDeviceToHost, s));
        if (p->d.objective) {
            p->iso_xa.resize(T);
            p->iso_xb.resize(T);
            SD_HIP(hipMemcpyAsync(p->iso_xa.data(), p->ptr(p->s_xa), T * sizeof(float), hipMemcpyDeviceToHost, s));
            SD_HIP(hipMemcpyAsync(p->iso_xb.data(), p->ptr(p->s_xb), T * sizeof(float), hipMemcpyDeviceToHost, s));
        }
        SD_HIP(hipStreamSynchronize(s));
        for (int t = 0; t < T; ++t) p->iso_sig[t] = std::exp(0.5f * lv[t]);
    } else {
        if ((rc = dalloc(p, &p->sig, (size_t)T * J))) return rc;
        SD_HIP(sd::launch_sigma(p->ptr(p->s_lv), p->sig, (int64_t)T * J, s));
    }
    SD_HIP(hipStreamSynchronize(s));
    SD_HIP(hipFree(emb));
    SD_HIP(hipFree(t1));
    SD_HIP(hipFree(temb));
    for (auto it = p->allocs.begin(); it != p->allocs.end();) {
        if (*it == emb || *it == t1 || *it == temb) it = p->allocs.erase(it);
        else ++it;
    }
    p->finalized = true;
    return SD_OK;
}

size_t sd_workspace_bytes(const sd_plan* plan, int64_t rows) {
    if (!plan || rows < 0) return 0;
    return carve(plan, rows, nullptr, nullptr) + 256;
}

int32_t sd_plan_kernels_per_step(const sd_plan* p) {
    if (!p) return 0;
    int n = 1;  // init_lin
    for (size_t l = 0; l < p->has_attn.size(); ++l) n += 2 + (p->has_attn[l] ? (p->d.use_attention ? 3 : 1) : 0);
    n += 4 + 1;     // final res block (3) + final_glin + update
    return n;
}

static int ws_setup(const sd_plan* p, int64_t rows, void* ws, size_t bytes, WS* w) {
    if (!p || !p->finalized) return fail(SD_E_STATE, "plan is not finalized");
    if (rows < 0) return fail(SD_E_INVALID, "rows < 0");
    const size_t need = carve(p, rows, nullptr, nullptr);
    if (!ws || bytes < need) return fail(SD_E_INVALID, "workspace too small: need " + std::to_string(need));
    char* base = (char*)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    if ((size_t)(base - (char*)ws) + need > bytes) return fail(SD_E_INVALID, "workspace too small after alignment");
    carve(p, rows, base, w);
    return SD_OK;
}

int sd_denoiser_forward(const sd_plan* p, const float* x_t, const float* x_cond, int64_t cond_repeat,
                        int32_t t, float* x0_out, int64_t rows, void* workspace, size_t ws_bytes,
                        void* stream) {
    WS w;
    int rc = ws_setup(p, rows, workspace, ws_bytes, &w);
    if (rc) return rc;
    if (t < 0 || t >= p->T) return fail(SD_E_INVALID, "t out of range");
    if (!x_t || !x0_out) return fail(SD_E_INVALID, "null tensor");
    if (p->C > 0 && !x_cond) return fail(SD_E_INVALID, "x_cond is required (diffusion_conditioning)");
    if (cond_repeat < 1) return fail(SD_E_INVALID, "cond_repeat must be >= 1");
    if ((rc = ws_reset(w, (hipStream_t)stream))) return rc;
    return run_denoiser(p, x_t, x_cond, cond_repeat, t, x0_out, rows, w, (hipStream_t)stream);
}

int sd_workspace_status(const sd_plan* p, const void* workspace, size_t ws_bytes, uint32_t* flags, void* stream) {
    if (!flags) return fail(SD_E_INVALID, "null flags");
    WS w;
    int rc = ws_setup(p, 0, const_cast<void*>(workspace), ws_bytes, &w);
    if (rc) return rc;
    unsigned v = 0;
    SD_HIP(hipMemcpyAsync(&v, ws_status(w), sizeof(unsigned), hipMemcpyDeviceToHost, (hipStream_t)stream));
    SD_HIP(hipStreamSynchronize((hipStream_t)stream));
    *flags = v;
    return SD_OK;
}

int sd_denoiser_trace(const sd_plan* p, const float* x_t, const float* x_cond, int64_t cond_repeat, int32_t t,
                      float* x0_out, int64_t rows, void* workspace, size_t ws_bytes, float* const* acts,
                      int32_t nacts, void* stream) {
    WS w;
    int rc = ws_setup(p, rows, workspace, ws_bytes, &w);
    if (rc) return rc;
    if (t < 0 || t >= p->T) return fail(SD_E_INVALID, "t out of range");
    if (!x_t || !x0_out || !acts) return fail(SD_E_INVALID, "null tensor");
    if (nacts != 2 + 4 * p->depth) return fail(SD_E_INVALID, "nacts must be 2 + 4 * depth");
    for (int i = 0; i < nacts; ++i)
        if (!acts[i]) return fail(SD_E_INVALID, "null activation buffer");
    if (p->C > 0 && !x_cond) return fail(SD_E_INVALID, "x_cond is required (diffusion_conditioning)");
    if (cond_repeat < 1) return fail(SD_E_INVALID, "cond_repeat must be >= 1");
    if ((rc = ws_reset(w, (hipStream_t)stream))) return rc;
    return run_denoiser(p, x_t, x_cond, cond_repeat, t, x0_out, rows, w, (hipStream_t)stream, nullptr, 0, 0, acts);
}

int sd_p_sample_update(const sd_plan* p, const float* x0_raw, const float* x_t, const float* eps,
                       int64_t eps_rs, uint64_t seed, int64_t row0, int32_t t, float* x_prev,
                       float* mean_out, int64_t mean_rs, float* noise_out, int64_t noise_rs,
                       int64_t rows, int32_t flags, void* stream) {
    if (!p || !p->finalized) return fail(SD_E_STATE, "plan is not finalized");
    if (flags & ~SD_FLAG_NO_CLIP) return fail(SD_E_INVALID, "sd_p_sample_update flags: SD_FLAG_NO_CLIP only");
    if (t < 0 || t >= p->T) return fail(SD_E_INVALID, "t out of range");
    if (!x0_raw || !x_t || !x_prev) return fail(SD_E_INVALID, "null tensor");
    if (!eps && p->D % 4) return fail(SD_E_INVALID, "device noise needs latent_dim % 4 == 0");
    const int64_t JD = (int64_t)p->J * p->D;
    return run_update(p, x0_raw, x_t, eps, eps ? eps_rs : JD, eps ? 1 : 2, seed, row0, nullptr, t,
                      x_prev, nullptr, 0, mean_out, mean_out ? mean_rs : JD, noise_out,
                      noise_out ? noise_rs : JD, rows, (hipStream_t)stream, nullptr, 0, 0, 0, 0,
                      !(flags & SD_FLAG_NO_CLIP));
}

static WS shift_ws(const sd_plan* p, const WS& w, int64_t r0, int chain) {
    WS o = w;
    const int64_t J = p->J;
    o.x += r0 * J * p->H;
    o.r += r0 * J * p->H;
    o.h += r0 * J * p->H;
    o.res += r0 * J * p->H;
    o.qkv += r0 * J * (p->d.use_attention ? 3 * p->hid : p->H);
    o.o += r0 * J * (p->d.use_attention ? p->hid : p->H);
    o.x0 += r0 * J * p->D;
    o.img0 += r0 * J * p->D;
    o.img1 += r0 * J * p->D;
    return o;
}

// number of row chains for `rows` rows (multiples of 32 rows each; the plan's row_chains option,
// default 3).  Every route runs with any chain count: the kernels share CUs with each other's
// workgroups (the row-chain hazard of rounds 1-2 was packed-FP32 code, which the
// build no longer emits), and the results are bitwise independent of the chain count.
static int chain_count(const sd_plan* p, int64_t rows, int64_t cond_repeat, int64_t* unit) {
    (void)cond_repeat;  // a chain starting inside a sequence's futures reads x_cond via x1_row0
    const int64_t g = 32;
    *unit = g;
    // a partial last unit counts: 50 rows (config 4, one sequence) run as chains of 32 + 18 rows
    const int64_t units = (rows + g - 1) / g;
    // auto (0): 3 chains (+ the caller's stream = HIP's default 4 hardware queues; a 4th chain
    // shares a queue: config 2 11.9k vs 15.9k futures/s), 2 on the small-batch split route
    // (400 rows: 5,920 vs 5,398 on one, 3,279 on three), one at 128 rows and below, where every
    // kernel is a few microseconds long and a second chain slows both (config 4, 50 rows: 61 vs
    // 106 futures/s; tools/sweep_routes.py, profiles/r03/ab)
    int n = p->chains > 0 ? std::min(p->chains, (int)sd_plan::kMaxChains)
            : rows <= 128                       ? 1
            : rows <= sd::split_rows_default() ? 2
                                               : 3;
    if (units < n) n = (int)std::max<int64_t>(1, units);
    return n;
}
static int64_t chain_row(int i, int n, int64_t rows, int64_t unit) {
    return i >= n ? rows : std::min(rows, (rows + unit - 1) / unit * i / n * unit);
}

// Creates the auxiliary streams / fork-join events chains 1 .. n-1 use (caller holds cmu).
// Diagnostics (SKELDIFF_DIAG bit 13): every chain, the first included, on a stream
// of its own whose CU mask is a disjoint 1/n of the device's CUs (no two chains share a CU).
constexpr int kDiagCuMask = 1 << 13;
static int ensure_chains(sd_plan* mp, int n) {
    const bool masked = sd::diag_flags() & kDiagCuMask;
    if (!mp->ev_fork) SD_HIP(hipEventCreateWithFlags(&mp->ev_fork, hipEventDisableTiming));
    for (int i = masked ? 0 : 1; i < n; ++i) {
        if (!mp->aux[i]) {
            if (masked) {
                int dev = 0;
                hipDeviceProp_t pr;
                SD_HIP(hipGetDevice(&dev));
                SD_HIP(hipGetDeviceProperties(&pr, dev));
                const int ncu = pr.multiProcessorCount;
                std::vector<uint32_t> m((ncu + 31) / 32, 0u);
                const bool inter = sd::diag_flags() & (1 << 17);  // bit 17: interleaved (cu % n == i)
                for (int c = 0; c < ncu; ++c)
                    if (inter ? c % n == i : c * n / ncu == i) m[c / 32] |= 1u << (c % 32);
                SD_HIP(hipExtStreamCreateWithCUMask(&mp->aux[i], (uint32_t)m.size(), m.data()));
            } else {
                SD_HIP(hipStreamCreateWithFlags(&mp->aux[i], hipStreamNonBlocking));
            }
        }
        if (!mp->ev_join[i]) SD_HIP(hipEventCreateWithFlags(&mp->ev_join[i], hipEventDisableTiming));
    }
    return SD_OK;
}

// The whole T-step chain: start noise, then per step Denoiser + posterior update.  only = -1
// records every row chain (chain i on cs[i]; steps outer, chains inner, so an eager caller feeds
// every chain from the start); only = i records chain i alone on cs[i] (one captured graph per
// chain, see sd_sample_loop).
static int record_loop(const sd_plan* p, const float* x_T, const float* x_cond, int64_t cond_repeat,
                       const float* eps_all, uint64_t seed, int64_t row0, float* out, float* means,
                       float* noise_out, float* timages, float* start_out, int64_t rows, const WS& w,
                       int32_t flags, bool use_rng_dev, const hipStream_t* cs, int nch, int64_t unit, int only) {
    const int T = p->T;
    const int64_t JD = (int64_t)p->J * p->D;
    const int64_t step_rs = (int64_t)(T > 1 ? T - 1 : 1) * JD;  // row stride of (B, T-1, J, D)
    const uint64_t* rng = use_rng_dev ? w.rng : nullptr;
    const bool dev_start = (flags & SD_FLAG_DEVICE_START) != 0;
    const bool dev_noise = (flags & SD_FLAG_DEVICE_NOISE) != 0;
    const int bf = p->prec == 2;  // bf16 latents (x_t, x0 between steps); records and `out` f32
    struct Chain {
        int64_t r0, n;
        WS w;
        const float* cur;
    } ch[sd_plan::kMaxChains];
    const int c0 = only < 0 ? 0 : only, c1 = only < 0 ? nch : only + 1;
    for (int i = c0; i < c1; ++i) {
        Chain& c = ch[i];
        c.r0 = chain_row(i, nch, rows, unit);
        c.n = chain_row(i + 1, nch, rows, unit) - c.r0;
        c.w = shift_ws(p, w, c.r0, i);
        c.cur = (dev_start || bf) ? c.w.img1 : x_T + c.r0 * JD;
        if (dev_start) SD_HIP(sd::launch_noise_fill(c.w.img1, c.n, JD, seed, row0, T, rng, cs[i], c.r0, bf));
        else if (bf)  // bf16 latents: the caller's f32 start noise rounded once
            SD_HIP(sd::launch_convert_rows(c.w.img1, 1, JD, x_T + c.r0 * JD, 0, JD, c.n, JD, cs[i]));
        if (start_out) SD_HIP(sd::launch_convert_rows(start_out + c.r0 * JD, 0, JD, c.cur, bf, JD, c.n, JD, cs[i]));
    }
    for (int t = T - 1; t >= 0; --t) {
        const int64_t k = T - 1 - t;  // index into the (B, T-1, ...) records
        const bool rec = t > 0;
        for (int i = c0; i < c1; ++i) {
            Chain& c = ch[i];
            const int64_t r0 = c.r0;
            const float* xc = (p->C > 0) ? x_cond + (r0 / cond_repeat) * p->J * p->C : x_cond;
            // concurrent chains: 32 x 64 tiles (more, smaller workgroups to interleave) measured
            // 5 % faster than the single-chain 32 x 96 choice at B = 3200, 3 chains
            const int64_t wg813 = (c.n + 31) / 32 * 2;  // 32 x 96 workgroups of an N = 192 layer
            int rc = run_denoiser(p, c.cur, xc, cond_repeat, t, c.w.x0, c.n, c.w, cs[i], nullptr, r0 % cond_repeat,
                                  (nch > 1 && wg813 >= 32) ? 812 : 0, nullptr, bf, bf, rows, r0, (int)k);
            if (rc) return rc;
            float* nxt = (t == 0) ? out + r0 * JD : (((T - 1 - t) & 1) ? c.w.img1 : c.w.img0);
            const float* eps = (!dev_noise && t > 0) ? eps_all + r0 * step_rs + k * JD : nullptr;
            const UpdDump saved = g_dump;
            if (k != 0 || !g_dump.x0) g_dump = UpdDump{};
            else g_dump = UpdDump{g_dump.x0 + r0 * JD, g_dump.xt + r0 * JD, g_dump.ev + r0 * JD};
            rc = run_update(p, c.w.x0, c.cur, eps, step_rs, dev_noise ? 2 : 1, seed, row0, rng, t, nxt,
                            (rec && timages) ? timages + r0 * step_rs + k * JD : nullptr, step_rs,
                            (rec && means) ? means + r0 * step_rs + k * JD : nullptr, step_rs,
                            (rec && noise_out) ? noise_out + r0 * step_rs + k * JD : nullptr, step_rs, c.n,
                            cs[i], nullptr, r0, bf, bf, t > 0 ? bf : 0, !(flags & SD_FLAG_NO_CLIP));
            g_dump = saved;
            if (rc) return rc;
            const int64_t sl = k * kSnapCalls + kSnapCalls - 1;  // diagnostics: the update's output
            if (g_snap.arena && sl < g_snap.nslots && (r0 + c.n) * JD <= g_snap.slot - g_snap.half)
                SD_HIP(hipMemcpyAsync(g_snap.arena + sl * g_snap.slot + g_snap.half + r0 * JD, nxt, c.n * JD * sizeof(float),
                                      hipMemcpyDeviceToDevice, cs[i]));
            c.cur = nxt;
        }
    }
    return SD_OK;
}

// fork chains 1 .. n-1 off s (caller holds cmu, ensure_chains done)
static int fork_chains(sd_plan* mp, hipStream_t s, int n, hipStream_t* cs) {
    cs[0] = s;
    if (sd::diag_flags() & 4) {  // diagnostic: every chain on the caller's stream (no concurrency)
        for (int i = 1; i < n; ++i) cs[i] = s;
        return SD_OK;
    }
    if (n > 1) SD_HIP(hipEventRecord(mp->ev_fork, s));
    for (int i = (n > 1 && (sd::diag_flags() & kDiagCuMask)) ? 0 : 1; i < n; ++i) {
        SD_HIP(hipStreamWaitEvent(mp->aux[i], mp->ev_fork, 0));
        cs[i] = mp->aux[i];
    }
    return SD_OK;
}
static int join_chains(sd_plan* mp, hipStream_t s, int n, const hipStream_t* cs) {
    for (int i = (n > 1 && (sd::diag_flags() & kDiagCuMask)) ? 0 : 1; i < n; ++i) {
        SD_HIP(hipEventRecord(mp->ev_join[i], cs[i]));
        SD_HIP(hipStreamWaitEvent(s, mp->ev_join[i], 0));
    }
    return SD_OK;
}

int sd_sample_loop(const sd_plan* p, const float* x_T, const float* x_cond, int64_t cond_repeat,
                   const float* eps_all, uint64_t seed, int64_t row0, float* out, float* means_out,
                   float* noise_out, float* timages_out, float* start_out, int64_t rows,
                   void* workspace, size_t ws_bytes, int32_t flags, void* stream) {
    WS w;
    int rc = ws_setup(p, rows, workspace, ws_bytes, &w);
    if (rc) return rc;
    if (!out) return fail(SD_E_INVALID, "null out");
    if (!(flags & SD_FLAG_DEVICE_START) && !x_T) return fail(SD_E_INVALID, "x_T is null (pass SD_FLAG_DEVICE_START)");
    if (!(flags & SD_FLAG_DEVICE_NOISE) && p->T > 1 && !eps_all)
        return fail(SD_E_INVALID, "eps_all is null (pass SD_FLAG_DEVICE_NOISE)");
    if ((flags & (SD_FLAG_DEVICE_START | SD_FLAG_DEVICE_NOISE)) && p->D % 4)
        return fail(SD_E_INVALID, "device noise needs latent_dim % 4 == 0");
    if (p->C > 0 && !x_cond) return fail(SD_E_INVALID, "x_cond is required (diffusion_conditioning)");
    if (cond_repeat < 1) return fail(SD_E_INVALID, "cond_repeat must be >= 1");
    if (rows == 0) return SD_OK;
    hipStream_t s = (hipStream_t)stream;
    sd_plan* mp = const_cast<sd_plan*>(p);
    if ((rc = ws_reset(w, s))) return rc;
    int64_t unit = 32;
    const int nch = chain_count(p, rows, cond_repeat, &unit);
    mp->last_chains.store(nch);
    std::unique_lock<std::mutex> lk(mp->cmu, std::defer_lock);  // fork/join objects are shared
    hipStream_t cs[sd_plan::kMaxChains];
    cs[0] = s;
    if (nch > 1) {
        lk.lock();
        if ((rc = ensure_chains(mp, nch))) return rc;
        for (int i = 1; i < nch; ++i) cs[i] = mp->aux[i];
        if (sd::diag_flags() & kDiagCuMask) cs[0] = mp->aux[0];
    }
    if (!(flags & SD_FLAG_GRAPH)) {
        if ((rc = fork_chains(mp, s, nch, cs))) return rc;
        sd::g_route_bits = 0;
        rc = record_loop(p, x_T, x_cond, cond_repeat, eps_all, seed, row0, out, means_out, noise_out, timages_out,
                         start_out, rows, w, flags, false, cs, nch, unit, -1);
        mp->last_route.store(sd::g_route_bits);
        if (rc) return rc;
        return join_chains(mp, s, nch, cs);
    }

    // Graph mode: each row chain is captured once per (rows, pointers, flags, stream, chains) as a
    // graph of its own and replayed on its own stream (the chains' graphs overlap on the GPU, where
    // one graph holding parallel branches would be replayed in order); seed / row0 live in the
    // workspace so a replay can draw fresh noise.
    GraphKey key;
    std::memset(&key, 0, sizeof(key));
    key.rows = rows;
    const void* ptrs[10] = {x_T, x_cond, eps_all, out, means_out, noise_out, timages_out, start_out, workspace, nullptr};
    std::memcpy(key.ptrs, ptrs, sizeof(ptrs));
    key.cond_repeat = cond_repeat;
    key.flags = flags;
    key.chains = nch;
    key.prec = p->prec;
    key.variant = p->variant;
    key.gl4_cfg = p->gl4_cfg;
    key.gl4_stage = p->gl4_stage;
    key.split = p->split;
    key.upd_elem = p->upd_elem;
    key.v5_valu = p->v5_valu;
    key.attn_tail = p->attn_tail;
    key.stream = stream;
    SD_HIP(sd::launch_set_rng(w.rng, seed, row0, s));
    std::shared_ptr<GraphSet> set;
    {
        std::lock_guard<std::mutex> g(mp->gmu);
        auto it = p->graphs.find(key);
        if (it != p->graphs.end()) set = it->second;
    }
    if (!set) {
        set = std::make_shared<GraphSet>();
        std::vector<hipGraphExec_t>& execs = set->execs;
        sd::g_route_bits = 0;
        for (int i = 0; i < nch; ++i) {
            hipGraph_t graph = nullptr;
            hipGraphExec_t exec = nullptr;
            hipError_t e = hipStreamBeginCapture(cs[i], hipStreamCaptureModeThreadLocal);
            if (e == hipSuccess) {
                rc = record_loop(p, x_T, x_cond, cond_repeat, eps_all, seed, row0, out, means_out, noise_out,
                                 timages_out, start_out, rows, w, flags, true, cs, nch, unit, i);
                e = hipStreamEndCapture(cs[i], &graph);
                if (!rc && e == hipSuccess) e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
                if (graph) (void)hipGraphDestroy(graph);
            }
            if (rc || e != hipSuccess) {
                if (exec) (void)hipGraphExecDestroy(exec);
                if (rc) return rc;
                return fail(SD_E_HIP, std::string("graph capture: ") + hipGetErrorString(e));
            }
            execs.push_back(exec);
            hipEvent_t ev = nullptr;
            SD_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            set->done.push_back(ev);
        }
        set->route_bits = sd::g_route_bits;
        std::shared_ptr<GraphSet> evicted;  // destroyed (after its own launches) outside the lock
        {
            std::lock_guard<std::mutex> g(mp->gmu);
            auto& cache = mp->graphs;
            if (cache.size() >= 8) {  // bounded cache: callers that reuse buffers hit it every call
                evicted = cache.begin()->second;
                cache.erase(cache.begin());
            }
            cache[key] = set;
        }
    }
    mp->last_route.store(set->route_bits);
    if ((rc = fork_chains(mp, s, nch, cs))) return rc;
    {
        // SKELDIFF_CHAIN_STAGGER (µs, A/B): chain i starts i x that much later, so the chains run
        // different layer types at a time instead of the same one in lockstep
        static const double stagger = [] {
            const char* e = getenv("SKELDIFF_CHAIN_STAGGER");
            return e ? atof(e) : 0.0;
        }();
        std::lock_guard<std::mutex> g(set->mu);
        for (int i = 0; i < nch; ++i) {
            SD_HIP(hipStreamWaitEvent(cs[i], set->done[i], 0));  // the exec's previous launch (any stream)
            if (i > 0 && stagger > 0) SD_HIP(sd::launch_delay(stagger * i, cs[i]));
            SD_HIP(hipGraphLaunch(set->execs[i], cs[i]));
            SD_HIP(hipEventRecord(set->done[i], cs[i]));
        }
    }
    return join_chains(mp, s, nch, cs);
}

int sd_plan_dims(const sd_plan* p, int32_t* dims_out) {
    if (!p || !dims_out) return fail(SD_E_INVALID, "null argument");
    dims_out[0] = p->J;
    dims_out[1] = p->D;
    dims_out[2] = p->T;
    dims_out[3] = p->C;
    return SD_OK;
}

int sd_plan_step_flops(const sd_plan* p, int64_t rows, double* flops_out) {
    if (!p || !flops_out || rows < 0) return fail(SD_E_INVALID, "bad arguments");
    step_flops(p, rows, flops_out);
    return SD_OK;
}

int sd_profile_step(const sd_plan* p, const float* x_t, const float* x_cond, int64_t cond_repeat, int32_t t,
                    int64_t rows, void* workspace, size_t ws_bytes, int32_t reps, float* ms_out,
                    int32_t* counts_out, void* stream) {
    WS w;
    int rc = ws_setup(p, rows, workspace, ws_bytes, &w);
    if (rc) return rc;
    if (!x_t || !ms_out || reps < 1) return fail(SD_E_INVALID, "bad arguments");
    if (t < 0 || t >= p->T) return fail(SD_E_INVALID, "t out of range");
    if (p->C > 0 && !x_cond) return fail(SD_E_INVALID, "x_cond is required (diffusion_conditioning)");
    hipStream_t s = (hipStream_t)stream;
    if ((rc = ws_reset(w, s))) return rc;
    double acc[4] = {0, 0, 0, 0};
    int32_t counts[3] = {0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        Prof prof;
        rc = run_denoiser(p, x_t, x_cond, cond_repeat, t, w.x0, rows, w, s, &prof);
        if (rc) return rc;
        rc = run_update(p, w.x0, x_t, nullptr, 0, 2, 1234 + r, 0, nullptr, t, w.img0, nullptr, 0, nullptr, 0,
                        nullptr, 0, rows, s, &prof);
        if (rc) return rc;
        SD_HIP(hipStreamSynchronize(s));
        for (size_t i = 0; i < prof.cls.size(); ++i) {
            float ms = 0.f;
            SD_HIP(hipEventElapsedTime(&ms, prof.ev[2 * i], prof.ev[2 * i + 1]));
            acc[prof.cls[i]] += ms;
            if (r == 0) counts[prof.cls[i]]++;
        }
        float tot = 0.f;
        SD_HIP(hipEventElapsedTime(&tot, prof.ev.front(), prof.ev.back()));
        acc[3] += tot;
    }
    for (int i = 0; i < 4; ++i) ms_out[i] = (float)(acc[i] / reps);
    if (counts_out)
        for (int i = 0; i < 3; ++i) counts_out[i] = counts[i];
    return SD_OK;
}

int sd_pairwise_distances(const float* x, int64_t nseq, int32_t samples, int64_t features, float* l1_mean,
                          float* l2_mean, void* stream) {
    if (nseq < 0 || samples < 2 || samples > 64 || features < 1)
        return fail(SD_E_INVALID, "pairwise distances: need 2..64 samples, features >= 1");
    if (nseq == 0) return SD_OK;
    if (!x) return fail(SD_E_INVALID, "pairwise distances: null input");
    SD_HIP(sd::launch_pairwise(x, nseq, samples, features, l1_mean, l2_mean, (hipStream_t)stream));
    return SD_OK;
}

int sd_ade_fde(const float* pred, const float* target, int64_t nseq, int32_t samples, int32_t frames,
               int64_t features, float* ade, float* fde, float* per_sample_ade, float* per_sample_fde, void* stream) {
    if (nseq < 0 || samples < 1 || samples > 64 || frames < 1 || features < 1)
        return fail(SD_E_INVALID, "ade/fde: need 1..64 samples, frames >= 1, features >= 1");
    if (nseq == 0) return SD_OK;
    if (!pred || !target) return fail(SD_E_INVALID, "ade/fde: null input");
    SD_HIP(sd::launch_ade_fde(pred, target, nseq, samples, frames, features, ade, fde, per_sample_ade, per_sample_fde,
                              (hipStream_t)stream));
    return SD_OK;
}

int sd_mm_ade_fde(const float* pred, const float* gts, const int64_t* pair_seq, int64_t npairs,
                  const int64_t* seq_offsets, int64_t nseq, int32_t samples, int32_t frames, int64_t features,
                  float* pair_ade, float* pair_fde, float* mmade, float* mmfde, void* stream) {
    if (nseq < 0 || npairs < 0 || samples < 1 || samples > 64 || frames < 1 || features < 1)
        return fail(SD_E_INVALID, "mmade/mmfde: need 1..64 samples, frames >= 1, features >= 1");
    if (nseq == 0) return SD_OK;
    if (!seq_offsets || (npairs > 0 && (!pred || !gts || !pair_seq)) || (mmade && !pair_ade) || (mmfde && !pair_fde))
        return fail(SD_E_INVALID, "mmade/mmfde: null input (pair outputs are required for the means)");
    SD_HIP(sd::launch_mm_ade_fde(pred, gts, pair_seq, npairs, seq_offsets, nseq, samples, frames, features, pair_ade,
                                 pair_fde, mmade, mmfde, (hipStream_t)stream));
    return SD_OK;
}

int sd_best_of_k(const float* sim, const float* loss, int64_t nseq, int32_t k, int64_t* idx_out, float* loss_out,
                 void* stream) {
    if (nseq < 0 || k < 1) return fail(SD_E_INVALID, "best_of_k: nseq >= 0, k >= 1");
    if (nseq == 0) return SD_OK;
    if (!loss || (!idx_out && !loss_out)) return fail(SD_E_INVALID, "best_of_k: null buffer");
    SD_HIP(sd::launch_best_of_k(sim, loss, nseq, k, idx_out, loss_out, (hipStream_t)stream));
    return SD_OK;
}

int sd_best_of_k_backward(const float* dloss_sel, const int64_t* idx, int64_t nseq, int32_t k, float* dloss,
                          void* stream) {
    if (nseq < 0 || k < 1) return fail(SD_E_INVALID, "best_of_k_backward: nseq >= 0, k >= 1");
    if (nseq == 0) return SD_OK;
    if (!dloss_sel || !idx || !dloss) return fail(SD_E_INVALID, "best_of_k_backward: null buffer");
    SD_HIP(sd::launch_best_of_k_bwd(dloss_sel, idx, nseq, k, dloss, (hipStream_t)stream));
    return SD_OK;
}

int sd_pose_loss(const float* pred, const float* target, int64_t nseq, int32_t samples, int32_t frames,
                 int32_t joints, int32_t dims, int32_t mse, float* per_sample, void* stream) {
    if (nseq < 0 || samples < 1 || frames < 1 || joints < 1 || dims < 1)
        return fail(SD_E_INVALID, "pose_loss: samples, frames, joints, dims >= 1");
    if (nseq == 0) return SD_OK;
    if (!pred || !target || !per_sample) return fail(SD_E_INVALID, "pose_loss: null buffer");
    SD_HIP(sd::launch_pose_loss(pred, target, nseq, samples, frames, joints, dims, mse != 0, per_sample,
                                (hipStream_t)stream));
    return SD_OK;
}

// kernel generation / v4 tile of the sd_test_* hooks only (plans take theirs from SD_OPT_*)
static int g_test_variant = -1, g_test_tile = -1;  // -1: the process defaults (SKELDIFF_* at load)
static int test_variant() { return g_test_variant >= 0 ? g_test_variant : sd::graph_linear_variant(); }
static int test_tile() { return g_test_tile >= 0 ? g_test_tile : sd::gl4_tile_default(); }

// split route of the test entry points (GLArgs::split: 0 auto, 1 never, 2 k_gl4y, 3 k_gl4t, 4 k_gl4t
// except to_qkv + attention); 2 / 3 / 4 give sd_test_graph_linear* a scratch of its own for the pre-mix Y
static int g_test_split = 0;
int sd_test_set_split_route(int32_t route) {
    if (route == -1) return g_test_split;  // query
    if (route < 0 || route > 4) return fail(SD_E_INVALID, "split route out of range");
    const int old = g_test_split;
    g_test_split = route;
    return old;
}

int sd_test_set_kernel_variant(int32_t gl_variant, int32_t gl4_tile) {
    if (gl_variant == -1) return test_variant();  // query
    if (gl_variant < 0 || gl_variant > 5) return fail(SD_E_INVALID, "gl_variant out of range");
    const int old = test_variant();
    g_test_variant = gl_variant;
    if (gl4_tile >= 0) g_test_tile = gl4_tile;
    return old;
}

int sd_plan_set_option(sd_plan* p, int32_t option, int64_t value) {
    if (!p) return fail(SD_E_INVALID, "null plan");
    switch (option) {
        case SD_OPT_KERNEL_VARIANT:
            if (value < 0 || value > 5) return fail(SD_E_INVALID, "kernel variant must be in [0, 5]");
            if (p->prec == 2 && value != 0 && value != 4)
                return fail(SD_E_INVALID, "bf16 mode runs on the v4 kernels only (variant 0 or 4)");
            if (p->d.norm_type == 1 && value != 0 && value != 4)
                return fail(SD_E_INVALID, "norm_type 'layer' runs on the v4 kernels only (variant 0 or 4)");
            p->variant = (int)value;
            return SD_OK;
        case SD_OPT_GL4_TILE:
            if (value < 0) return fail(SD_E_INVALID, "gl4 tile must be >= 0");
            p->gl4_cfg = (int)value;
            return SD_OK;
        case SD_OPT_ROW_CHAINS:
            if (value < 0 || value > sd_plan::kMaxChains) return fail(SD_E_INVALID, "row chains must be in [0 (auto), 8]");
            p->chains = (int)value;
            return SD_OK;
        case SD_OPT_PRECISION: return sd_plan_set_precision(p, (int32_t)value);
        case SD_OPT_GL4_STAGING:
            if (value < 0 || value > 2)
                return fail(SD_E_INVALID, "gl4 staging must be 0 (LDS-DMA), 1 (registers) or 2 (diagnostic)");
            p->gl4_stage = (int)value;
            return SD_OK;
        case SD_OPT_LAST_CHAINS:
        case SD_OPT_LAST_ROUTE: return fail(SD_E_INVALID, "SD_OPT_LAST_CHAINS / SD_OPT_LAST_ROUTE are read-only");
        case SD_OPT_SPLIT_ROUTE:
            if (value < 0 || value > 4)
                return fail(SD_E_INVALID, "split route must be 0 (auto), 1 (never), 2 (always), 3 (always, tiled phase 1) "
                                          "or 4 (tiled phase 1 except to_qkv + attention)");
            p->split = (int)value;
            return SD_OK;
        case SD_OPT_UPDATE_KERNEL:
            if (value < 0 || value > 1)
                return fail(SD_E_INVALID, "update kernel must be 0 (matrix cores where they apply) or 1 (element-per-thread)");
            p->upd_elem = (int)value;
            return SD_OK;
        case SD_OPT_V5_MIX:
            if (value != 0 && value != 1) return fail(SD_E_INVALID, "v5 mix must be 0 (matrix cores) or 1 (VALU)");
            p->v5_valu = (int)value;
            return SD_OK;
        case SD_OPT_ATTENTION:
            if (value != 0 && value != 2 && value != 3)
                return fail(SD_E_INVALID, "attention must be 0 (auto: 2 where it applies), 2 (to_qkv mixing inside the "
                                          "attention kernel at 49 <= J <= 52) or 3 (the separate mixing pass)");
            p->attn_tail = (int)value;
            return SD_OK;
        default: return fail(SD_E_INVALID, "unknown option " + std::to_string(option));
    }
}

int sd_plan_get_option(const sd_plan* p, int32_t option, int64_t* value) {
    if (!p || !value) return fail(SD_E_INVALID, "null argument");
    switch (option) {
        case SD_OPT_KERNEL_VARIANT: *value = p->variant; return SD_OK;
        case SD_OPT_GL4_TILE: *value = p->gl4_cfg; return SD_OK;
        case SD_OPT_ROW_CHAINS: *value = p->chains; return SD_OK;
        case SD_OPT_PRECISION: *value = p->prec; return SD_OK;
        case SD_OPT_GL4_STAGING: *value = p->gl4_stage; return SD_OK;
        case SD_OPT_SPLIT_ROUTE: *value = p->split; return SD_OK;
        case SD_OPT_LAST_CHAINS: *value = p->last_chains.load(); return SD_OK;
        case SD_OPT_LAST_ROUTE: *value = p->last_route.load(); return SD_OK;
        case SD_OPT_UPDATE_KERNEL: *value = p->upd_elem; return SD_OK;
        case SD_OPT_V5_MIX: *value = p->v5_valu; return SD_OK;
        case SD_OPT_ATTENTION: *value = p->attn_tail; return SD_OK;
        default: return fail(SD_E_INVALID, "unknown option " + std::to_string(option));
    }
}

int sd_plan_set_precision(sd_plan* p, int32_t mode) {
    if (!p) return fail(SD_E_INVALID, "null plan");
    if (mode < 0 || mode > 2) return fail(SD_E_INVALID, "precision mode must be 0 (f32), 1 (half) or 2 (bf16)");
    if (mode == 2) {  // the bf16 operands exist only in the v4 tiles (J 16 / 17 / 21, row-major)
        if (p->J != 16 && p->J != 17 && p->J != 21)
            return fail(SD_E_INVALID, "bf16 mode needs the split-f16 (v4) tiles: num_nodes 16, 17 or 21");
        if (p->variant != 0 && p->variant != 4) return fail(SD_E_INVALID, "bf16 mode needs kernel variant 0 or 4");
        if (p->finalized) {
            auto v4ok = [](const GL& g) { return g.split_bf.w && (g.K1 + g.K2) % 32 == 0; };
            bool ok = v4ok(p->init_lin) && v4ok(p->fres_res) && v4ok(p->fglin);
            for (auto& g : p->r1) ok = ok && v4ok(g);
            for (auto& g : p->r2) ok = ok && v4ok(g);
            for (size_t l = 0; l < p->qkv.size(); ++l)
                if (p->has_attn[l]) ok = ok && v4ok(p->qkv[l]) && (!p->d.use_attention || v4ok(p->outp[l]));
            if (!ok) return fail(SD_E_INVALID, "bf16 mode needs every graph-linear on the v4 kernels (K % 32 == 0)");
        }
    }
    p->prec = mode;
    return SD_OK;
}

int sd_test_graph_linear(const float* x1, int32_t K1, int64_t x1_div, const float* x2, int32_t K2,
                         const float* W, const float* bias, const int64_t* node_types, const float* ghat,
                         const float* film, int32_t act, const float* res, float* out, int64_t rows,
                         int32_t J, int32_t N, int32_t rms, void* stream) {
    return sd_test_graph_linear_layout(x1, K1, x1_div, x2, K2, W, bias, node_types, ghat, film, act, res, out, rows,
                                       J, N, rms, 0, stream);
}

int sd_test_graph_linear_layout(const float* x1, int32_t K1, int64_t x1_div, const float* x2, int32_t K2,
                                const float* W, const float* bias, const int64_t* node_types, const float* ghat,
                                const float* film, int32_t act, const float* res, float* out, int64_t rows,
                                int32_t J, int32_t N, int32_t rms, int32_t layout, void* stream) {
    if (!x1 || !W || !ghat || !out || !node_types || J < 1 || J > sd::kMaxNodes || N < 1 || K1 % 16 ||
        K2 % 16 || x1_div < 1 || rows < 0)
        return fail(SD_E_INVALID, "bad arguments");
    sd::GLArgs a{};
    a.x1 = x1;
    a.K1 = K1;
    a.x1_rs = (int64_t)J * K1;
    a.x1_div = (int)x1_div;
    a.x2 = x2;
    a.K2 = x2 ? K2 : 0;
    a.x2_rs = (int64_t)J * K2;
    a.W = W;
    a.bias = bias;
    a.G = ghat;
    a.film = film;
    a.res = res;
    a.res_rs = (int64_t)J * N;
    a.out = out;
    a.out_rs = (int64_t)J * N;
    a.B = rows;
    a.N = N;
    a.J = J;
    a.act = act;
    a.ntypes = 1;
    for (int j = 0; j < J; ++j) {
        if (node_types[j] < 0) return fail(SD_E_INVALID, "negative node type");
        a.wrow[j] = (int)node_types[j] * N;
        a.ntype[j] = (int)node_types[j];
        a.ntypes = std::max(a.ntypes, (int)node_types[j] + 1);
    }
    // split weights for v4: made per call (tests), or cached by W pointer when
    // SKELDIFF_GL_CACHE_SPLIT=1 (tools/bench_gl.py: weights fixed across timed calls)
    static const bool cache = [] {
        const char* e = getenv("SKELDIFF_GL_CACHE_SPLIT");
        return e && atoi(e) == 1;
    }();
    static std::map<std::tuple<const float*, int, int, int>, sd::SplitW> cached;
    a.x1_blk = layout & 1;
    a.x2_blk = (layout >> 1) & 1;
    a.res_blk = (layout >> 2) & 1;
    a.out_blk = (layout >> 3) & 1;
    a.variant = test_variant();
    a.gl4_cfg = test_tile();
    a.gl4_stage = sd::gl4_stage_default();
    sd::SplitW sw;
    if (a.variant == 0 || a.variant == 4) {
        const auto key = std::make_tuple(W, a.ntypes, N, K1 + a.K2);
        auto it = cache ? cached.find(key) : cached.end();
        if (it != cached.end()) {
            sw = it->second;
        } else {
            SD_HIP(sd::make_split_weights(W, a.ntypes, N, K1 + a.K2, &sw, (hipStream_t)stream));
            if (cache) cached[key] = sw;
        }
        a.wsp = sw.w;
        a.wsp_nct = sw.nct;
        a.wsp_unscale = sw.unscale;
    }
    a.split = g_test_split;
    float* zs = nullptr;
    if (a.split >= 2 && rows > 0) {  // the split route's pre-mix Y scratch (zs_off layout)
        a.zs_cap = (rows + 31) / 32 * 32 * (int64_t)J * N;
        SD_HIP(hipMalloc(&zs, a.zs_cap * sizeof(float)));
        a.zs = zs;
    }
    const hipError_t e = sd::launch_graph_linear(a, rms != 0, (hipStream_t)stream);
    if ((sw.w && !cache) || zs) {
        (void)hipStreamSynchronize((hipStream_t)stream);
        if (sw.w && !cache) (void)hipFree(sw.w);
        if (zs) (void)hipFree(zs);
    }
    SD_HIP(e);
    return SD_OK;
}

int sd_test_qkv_attention(const float* x, int32_t K, const float* W, const int64_t* node_types, const float* ghat,
                          float* out, int64_t rows, int32_t J, int32_t heads, int32_t rms, int32_t layout,
                          void* stream) {
    if (!x || !W || !ghat || !out || !node_types || J < 1 || J > sd::kMaxNodes || heads < 1 || K % 32 || rows < 0)
        return fail(SD_E_INVALID, "bad arguments");
    sd::GLArgs a{};
    const int N = 3 * heads * 32;
    a.x1 = x;
    a.K1 = K;
    a.x1_rs = (int64_t)J * K;
    a.x1_div = 1;
    a.G = ghat;
    a.out = out;
    a.out_rs = (int64_t)J * heads * 32;
    a.B = rows;
    a.N = N;
    a.J = J;
    a.ntypes = 1;
    for (int j = 0; j < J; ++j) {
        if (node_types[j] < 0) return fail(SD_E_INVALID, "negative node type");
        a.wrow[j] = (int)node_types[j] * N;
        a.ntype[j] = (int)node_types[j];
        a.ntypes = std::max(a.ntypes, (int)node_types[j] + 1);
    }
    a.attn_heads = heads;
    a.attn_scale = (float)std::pow(32.0, -0.5);
    a.variant = test_variant();
    a.gl4_cfg = test_tile();
    a.gl4_stage = sd::gl4_stage_default();
    a.x1_blk = layout & 1;
    a.out_blk = (layout >> 3) & 1;
    sd::SplitW sw;
    SD_HIP(sd::make_split_weights(W, a.ntypes, N, K, &sw, (hipStream_t)stream));
    a.wsp = sw.w;
    a.wsp_nct = sw.nct;
    a.wsp_unscale = sw.unscale;
    const hipError_t e = sd::launch_qkv_attention_v4(a, rms != 0, (hipStream_t)stream);
    (void)hipStreamSynchronize((hipStream_t)stream);
    (void)hipFree(sw.w);
    if (e == hipErrorNotSupported) return fail(SD_E_INVALID, "fused qkv+attention not available for this shape");
    SD_HIP(e);
    return SD_OK;
}

int sd_test_attention(const float* qkv, float* out, int64_t rows, int32_t J, int32_t heads, int32_t dim_head,
                      void* stream) {
    if (!qkv || !out || J < 1 || J > sd::kMaxNodes || heads < 1 || dim_head % 16 || rows < 0)
        return fail(SD_E_INVALID, "bad arguments");
    sd::AttnArgs aa{qkv, out, rows, J, heads, dim_head, (float)std::pow((double)dim_head, -0.5)};
    SD_HIP(sd::launch_attention(aa, (hipStream_t)stream));
    return SD_OK;
}

#ifdef SD_DEBUG_LDS
// diagnostic build only: copy the LDS integrity counters to out[8] (host), then zero them
int sd_debug_lds_counters(uint32_t* out) {
    SD_HIP(hipDeviceSynchronize());
    SD_HIP(hipMemcpy(out, sd::debug_counters(), 8 * sizeof(unsigned), hipMemcpyDeviceToHost));
    SD_HIP(hipMemset(sd::debug_counters(), 0, 8 * sizeof(unsigned)));
    return SD_OK;
}
#endif

int sd_noise_fill(float* out, int64_t rows, int64_t n_per_row, uint64_t seed, int64_t row0, int32_t step,
                  void* stream) {
    if (!out || rows < 0 || n_per_row % 4) return fail(SD_E_INVALID, "bad arguments (n_per_row % 4 != 0?)");
    SD_HIP(sd::launch_noise_fill(out, rows, n_per_row, seed, row0, step, nullptr, (hipStream_t)stream));
    return SD_OK;
}

int sd_philox_raw(uint32_t* out, int64_t rows, int64_t quads, uint64_t seed, int64_t row0, int32_t step,
                  void* stream) {
    if (!out || rows < 0 || quads < 0) return fail(SD_E_INVALID, "bad arguments");
    SD_HIP(sd::launch_philox_raw(out, rows, quads, seed, row0, step, (hipStream_t)stream));
    return SD_OK;
}

}  // extern "C"
