// C-ABI implementation (include/mmvae_capi.h): handle lifecycle, parameter registry,
// dataset upload, step orchestration, RCCL gradient all-reduce, kernel timing.
#include <sys/mman.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mmvae/lbessel.hh"
#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"

using namespace mmvae;

static thread_local std::string g_last_error;

#define FAIL(e, code, msg)                         \
    do {                                           \
        std::string _m = (msg);                    \
        if (e) (e)->err = _m;                      \
        g_last_error = _m;                         \
        return (code);                             \
    } while (0)

#define HIPCHK(e, expr)                                                                             \
    do {                                                                                            \
        hipError_t _er = (expr);                                                                    \
        if (_er != hipSuccess)                                                                      \
            FAIL(e, MMVAE_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_er));               \
    } while (0)

namespace mmvae {

void timer_begin(Engine* e, const char* name, hipEvent_t* a) {
    auto it = e->timer_index.find(name);
    int idx;
    if (it == e->timer_index.end()) {
        idx = (int)e->timers.size();
        e->timers.push_back(TimerRec{name, 0.0, 0});
        e->timer_index[name] = idx;
    } else {
        idx = it->second;
    }
    hipEvent_t ev0, ev1;
    if (e->event_pool.size() >= 2) {
        ev0 = e->event_pool.back();
        e->event_pool.pop_back();
        ev1 = e->event_pool.back();
        e->event_pool.pop_back();
    } else {
        hipEventCreate(&ev0);
        hipEventCreate(&ev1);
    }
    hipEventRecord(ev0, e->stream);
    e->pending.push_back({idx, ev0, ev1});
    *a = ev1;
}

void timer_end(Engine* e, hipEvent_t a) { hipEventRecord(a, e->stream); }

}  // namespace mmvae

static void timer_collect(Engine* e) {
    if (e->pending.empty()) return;
    hipStreamSynchronize(e->stream);
    for (auto& p : e->pending) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, p.a, p.b);
        e->timers[p.idx].total_ms += ms;
        e->timers[p.idx].launches += 1;
        e->event_pool.push_back(p.a);
        e->event_pool.push_back(p.b);
    }
    e->pending.clear();
}

// ---------------------------------------------------------------------------------------
// parameter registry — LibTorch named_parameters() order (nb.hh:318-400, vmf.hh:325-388)
// ---------------------------------------------------------------------------------------
static void add_slot(Engine* e, const std::string& n, std::vector<int64_t> shape, bool reg) {
    ParamSlot s;
    s.name = n;
    s.shape = shape;
    s.numel = 1;
    for (auto v : shape) s.numel *= v;
    s.registered = reg;
    if (reg) {
        s.off = e->P_reg;
        e->P_reg += s.numel;
    } else {
        s.off = e->P_frz;
        e->P_frz += s.numel;
    }
    e->slot_index[n] = (int)e->slots.size();
    e->slots.push_back(s);
}

// Frozen hidden chains (nb.hh:331-379, vmf.hh:338-385): the first encoder layer (D -> KE) and
// the last decoder layer (KD -> D) are the big gene GEMMs; the layers between are small chain
// layers run inside the latent kernels.  Registers the frozen slots in the reference's names.
static void build_frozen_chains(Engine* e, bool vmf) {
    const int64_t D = e->D, K = e->K;
    const int ne = e->cfg.n_enc_hidden, nd = e->cfg.n_dec_hidden;
    const std::string ep = vmf ? "z_enc.encoding_" : "mu_enc.mu_encoding_";
    const std::string dp = vmf ? "z_dec.decoding_" : "mu_dec.mu_decoding_";
    int nl = 0, off = 0;
    auto chain_layer = [&](const std::string& w, const std::string& b, int in, int out) {
        e->ch_w[nl] = w;
        e->ch_b[nl] = b;
        e->ch_in[nl] = in;
        e->ch_out[nl] = out;
        e->ch_off[nl] = off;
        off += in * out + out;
        ++nl;
    };
    // encoder: Angular layers have no bias (angular.hh:34-42)
    if (ne == 0) {
        const std::string n0 = vmf ? "z_enc.0" : "mu_enc.mu_encoding";
        add_slot(e, n0 + ".weight", {K, D}, false);
        if (!vmf) add_slot(e, n0 + ".bias", {K}, false);
        e->fz_enc_w = n0 + ".weight";
        e->fz_enc_b = vmf ? "" : n0 + ".bias";
    }
    int64_t prev = D;
    for (int l = 0; l < ne; ++l) {
        const int64_t wl = e->cfg.enc_hidden[l];
        const std::string n = ep + std::to_string(l + 1);
        add_slot(e, n + ".weight", {wl, prev}, false);
        if (!vmf) add_slot(e, n + ".bias", {wl}, false);
        if (l == 0) {
            e->fz_enc_w = n + ".weight";
            e->fz_enc_b = vmf ? "" : n + ".bias";
        } else {
            chain_layer(n + ".weight", vmf ? "" : n + ".bias", (int)prev, (int)wl);
        }
        prev = wl;
    }
    e->nce = nl;
    prev = K;
    for (int l = 0; l < nd; ++l) {
        const int64_t wl = e->cfg.dec_hidden[l];
        const std::string n = dp + std::to_string(l + 1);
        add_slot(e, n + ".weight", {wl, prev}, false);
        add_slot(e, n + ".bias", {wl}, false);
        chain_layer(n + ".weight", n + ".bias", (int)prev, (int)wl);
        prev = wl;
    }
    e->ncd = nl - e->nce;
    const std::string nfin = vmf ? "z_dec.decoding" : "mu_dec.mu_decoding";
    add_slot(e, nfin + ".weight", {D, prev}, false);
    add_slot(e, nfin + ".bias", {D}, false);
    e->fz_dec_w = nfin + ".weight";
    e->fz_dec_b = nfin + ".bias";
}

// vmf_vae_tImpl registration order (vmf.hh:318-388); the Angular encoder and the decoder
// Sequential are never register_module'd (Q1) and stay frozen.
static void build_registry_vmf(Engine* e) {
    const int64_t D = e->D, C = e->C, K = e->K, E = e->E;
    add_slot(e, "x_mean", {1, D}, true);
    add_slot(e, "ln_x_sd", {1, D}, true);
    add_slot(e, "ln_kappa", {1}, true);
    add_slot(e, "covar_encoding.weight", {K, C}, true);
    add_slot(e, "covar_encoding.bias", {K}, true);
    add_slot(e, "representation_mean.weight", {K, E}, true);
    add_slot(e, "representation_mean.bias", {K}, true);
    add_slot(e, "representation_logvariance.weight", {K, E}, true);
    add_slot(e, "representation_logvariance.bias", {K}, true);
    add_slot(e, "covar_decoding_.weight", {D, C}, true);
    add_slot(e, "covar_decoding_.bias", {D}, true);
    build_frozen_chains(e, true);
}

static void build_registry_nb(Engine* e) {
    const int64_t D = e->D, C = e->C, K = e->K, H = e->H, R = e->R, E = e->E;
    add_slot(e, "x_mean", {1, D}, true);
    add_slot(e, "ln_x_sd", {1, D}, true);
    add_slot(e, "mu_bias", {1, D}, true);
    add_slot(e, "nu_bias", {1, D}, true);
    add_slot(e, "covar_encoding.weight", {K, C}, true);
    add_slot(e, "covar_encoding.bias", {K}, true);
    add_slot(e, "mu_representation_mean.weight", {K, E}, true);
    add_slot(e, "mu_representation_mean.bias", {K}, true);
    add_slot(e, "mu_representation_logvariance.weight", {K, E}, true);
    add_slot(e, "mu_representation_logvariance.bias", {K}, true);
    add_slot(e, "covar_decoding.weight", {D, C}, true);
    add_slot(e, "covar_decoding.bias", {D}, true);
    add_slot(e, "nu_encoding.weight", {H, D}, true);
    add_slot(e, "nu_encoding.bias", {H}, true);
    add_slot(e, "nu_representation_mean.weight", {R, H}, true);
    add_slot(e, "nu_representation_mean.bias", {R}, true);
    add_slot(e, "nu_representation_logvariance.weight", {R, H}, true);
    add_slot(e, "nu_representation_logvariance.bias", {R}, true);
    add_slot(e, "nu_decoding.weight", {D, R}, true);
    add_slot(e, "nu_decoding.bias", {D}, true);
    add_slot(e, "depth.weight", {1, D}, true);
    add_slot(e, "depth.bias", {1}, true);
    // frozen Sequentials (Q1: never register_module'd)
    build_frozen_chains(e, false);
}

template <class T>
static hipError_t dalloc(T** p, int64_t n) {
    return hipMalloc(p, sizeof(T) * (size_t)(n > 0 ? n : 1));
}

// point the current-slot views at pinned staging slot s
static void use_slot(Engine* e, int s) {
    const int64_t Bp = e->Bpad;
    auto& sl = e->slots2[s];
    e->cur_slot = s;
    e->h_cells_pin = sl.block;
    e->h_seg_pin = sl.block + Bp;
    e->h_perm_pin = reinterpret_cast<int32_t*>(e->h_seg_pin + Bp / 16 + 1);
    e->h_ss = reinterpret_cast<StepScalars*>(e->h_perm_pin + Bp);
    e->h_brp_pin = reinterpret_cast<int64_t*>(e->h_ss + 1);
    e->h_eps_pin = sl.eps;
    stream_bind(e, s);
    e->ev_staged = sl.ev;
}

extern "C" {

void mmvae_cfg_default(mmvae_cfg* c, int32_t model) {
    std::memset(c, 0, sizeof(*c));
    c->model = model;
    c->dtype = MMVAE_DTYPE_F32;
    c->C = 1;
    c->K = 2;   // --mean_latent / --latent default (nb.hh:59, vmf.hh:60)
    c->H = 1;
    c->R = 1;
    c->max_batch = 100;  // --batch_size default (mmvae.hh:35)
    c->lr = 1e-3f;
    c->weight_decay = 1e-4f;
    c->grad_clip = 1.f;
    c->kappa_min = 0.1f;
    c->kappa_max = 10.f;
    c->seed = 42;
}

const char* mmvae_last_error(mmvae_h h) { return h ? h->err.c_str() : g_last_error.c_str(); }

int mmvae_create(const mmvae_cfg* cfg, int device, mmvae_h* out) {
    if (!cfg || !out) FAIL((Engine*)nullptr, MMVAE_E_ARG, "null cfg/out");
    if (cfg->model != MMVAE_MODEL_NB && cfg->model != MMVAE_MODEL_VMF)
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "model must be MMVAE_MODEL_NB or MMVAE_MODEL_VMF");
    if (cfg->model == MMVAE_MODEL_VMF && !(cfg->kappa_min > 0.f && cfg->kappa_max >= cfg->kappa_min))
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "vMF needs 0 < kappa_min <= kappa_max");
    if (cfg->D < 1 || cfg->K < 1 || cfg->C < 1 || cfg->H < 1 || cfg->R < 1 || cfg->max_batch < 1)
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "cfg out of range (need D, K, C, H, R, max_batch >= 1)");
    if (cfg->dtype != MMVAE_DTYPE_F32 && cfg->dtype != MMVAE_DTYPE_BF16 && cfg->dtype != MMVAE_DTYPE_BF16X3 &&
        cfg->dtype != MMVAE_DTYPE_FP8)
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "dtype must be F32, BF16, BF16X3 or FP8");
    if (cfg->dtype == MMVAE_DTYPE_FP8 && cfg->model != MMVAE_MODEL_NB)
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "the fp8 mode is built for the NB decoder (BASELINE configs[4])");
    if (cfg->n_enc_hidden < 0 || cfg->n_enc_hidden > MMVAE_MAX_HIDDEN || cfg->n_dec_hidden < 0 ||
        cfg->n_dec_hidden > MMVAE_MAX_HIDDEN)
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "at most 16 hidden encoder / decoder layers (MMVAE_MAX_HIDDEN)");
    // nb.hh:334-337 pushes a hidden encoder Linear and its ReLU under the same name: LibTorch
    // throws at construction, so the reference has no such model
    if (cfg->model == MMVAE_MODEL_NB && cfg->relu && cfg->n_enc_hidden > 0)
        FAIL((Engine*)nullptr, MMVAE_E_ARG, "Submodule 'mu_encoding_1' already defined (reference nb.hh:334-337: "
                                            "--relu with hidden --mean_encoding layers)");
    for (int l = 0; l < cfg->n_enc_hidden; ++l)
        if (cfg->enc_hidden[l] < 1) FAIL((Engine*)nullptr, MMVAE_E_ARG, "hidden encoder widths must be >= 1");
    for (int l = 0; l < cfg->n_dec_hidden; ++l)
        if (cfg->dec_hidden[l] < 1) FAIL((Engine*)nullptr, MMVAE_E_ARG, "hidden decoder widths must be >= 1");
    // the fused tile kernels' shape envelope; anything else runs on the wide path (wide.hip)
    bool wide = cfg->K > 64 || cfg->C > CMAX || cfg->H > HMAX || cfg->R > RMAX || cfg->n_enc_hidden > 4 ||
                cfg->n_dec_hidden > 4;
    for (int l = 0; l < cfg->n_enc_hidden; ++l) wide = wide || cfg->enc_hidden[l] > 64;
    for (int l = 0; l < cfg->n_dec_hidden; ++l) wide = wide || cfg->dec_hidden[l] > 64;
    {  // the batch-list builder keeps a 16-row block's tile pointers in LDS (batch.hip)
        const int64_t NT = (cfg->D + 63) / 64;
        if (4 * (NT + 1 + 16 * (NT + 1) + 16 * NT) + 8 * 1024 + 256 > 160 * 1024) wide = true;
    }
    if (const char* v = std::getenv("MMVAE_WIDE"))  // diagnostics / tests: force the wide path
        if (v[0] == '1') wide = true;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0)
        FAIL((Engine*)nullptr, MMVAE_E_HIP, "no HIP device " + std::to_string(device));
    mmvae_engine* e = new mmvae_engine();
    e->cfg = *cfg;
    e->no_balance = std::getenv("MMVAE_NO_BALANCE") != nullptr;  // (read once: a graph-key input, graph_key.hpp)
    e->device = device;
    e->wide = wide;
    HIPCHK(e, hipSetDevice(device));
    HIPCHK(e, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    e->D = cfg->D;
    e->DP = (cfg->D + 63) / 64 * 64;
    e->NT = e->DP / 64;
    e->K = cfg->K;
    e->KE = cfg->n_enc_hidden ? cfg->enc_hidden[0] : cfg->K;
    e->E = cfg->n_enc_hidden ? cfg->enc_hidden[cfg->n_enc_hidden - 1] : cfg->K;
    e->KD = cfg->n_dec_hidden ? cfg->dec_hidden[cfg->n_dec_hidden - 1] : cfg->K;
    e->KP = (std::max(e->K, std::max(e->KE, e->KD)) <= 32) ? 32 : 64;  // (fused path only)
    e->C = cfg->C;
    e->H = cfg->H;
    e->R = cfg->R;
    e->Bmax = cfg->max_batch;
    e->Bpad = pad_rows(cfg->max_batch);
    e->nrb_max = e->Bpad / 64;
    if (cfg->model == MMVAE_MODEL_VMF) {
        e->H = e->R = 1;  // unused by the vMF model
        build_registry_vmf(e);
    } else {
        build_registry_nb(e);
    }

    // gene splits: one round of `per_cu` resident workgroups on each of the 256 CUs (the
    // occupancy the kernel's LDS / VGPR budget allows).  No tile kernel keeps split-long column
    // accumulators in LDS (every tile's partials stream out), so the split length is free: a
    // grid of one full round beats a longer grid with a partial second round (measured at
    // D = 30k: pass B 403 -> 302 us with 8 instead of 12 splits; at B = 8192 the encoders
    // ran 9 splits = 1.5 rounds).
    auto pick_split = [&](int per_cu) {
        int ns = (int)((256 * per_cu + e->nrb_max - 1) / e->nrb_max);
        if (ns < 1) ns = 1;
        if (ns > e->NT) ns = (int)e->NT;
        if (ns > 64) ns = 64;
        return ns;
    };
    // NB pass B holds ~150 KB of LDS per 8-wave workgroup (2 x 4-wave per CU); the vMF decoder
    // fits 4 (16 splits 46 + 71 us vs 12 splits 51 + 74 us); the shared encoder kernels (~37 KB, <= 104 VGPRs in bf16) fit 4 (measured at 64 row
    // blocks: 16 splits 58 + 31 us, 12 splits 62 + 34 us, 24 splits 61 + 36 us)
    // Resident 4-wave workgroups per CU by mode (LDS / VGPR budgets of the kernels, see
    // tools/resource_usage.py): bf16 operand tiles are the smallest; the x3 mode stages hi + lo
    // images and f32 four-byte elements, so both fit half as many (NB pass B: bf16 and x3 run one
    // 8-wave workgroup per CU = 2 units; f32 one 4-wave workgroup)
    const bool vmf_model = cfg->model == MMVAE_MODEL_VMF;
    const bool bf_ops = cfg->dtype == MMVAE_DTYPE_BF16 || cfg->dtype == MMVAE_DTYPE_FP8;  // fp8: bf16 encoders / dz
    // vMF x3 at K <= 32: ~48 KB of LDS per decoder workgroup (no WdT image): 3 per CU
    // NB x3 with MMVAE_DEC3=1: pass B at three 4-wave workgroups per CU (k_dec_nb D3)
    e->dec3 = !vmf_model && cfg->dtype == MMVAE_DTYPE_BF16X3 && getenv_is("MMVAE_DEC3", "1");
    const int dec_cu = vmf_model ? (bf_ops ? 4 : (cfg->dtype == MMVAE_DTYPE_BF16X3 && e->KP == 32 ? 3 : 2))
                                 : (cfg->dtype == MMVAE_DTYPE_F32 ? 1 : e->dec3 ? 3 : 2);
    e->nsplit_d = pick_split(dec_cu);
    // vMF forward decoder pass: ~29 KB of LDS and <= 128 VGPRs in the 16-bit operand modes at
    // K <= 32 with one covariate (VFwdOcc, vmf_kernels.hip): 4 per CU instead of the backward's 3
    e->nsplit_f = (vmf_model && e->KP == 32 && e->C == 1 && cfg->dtype != MMVAE_DTYPE_F32) ? pick_split(4) : e->nsplit_d;
    // passes A / C are light: a finer gene split gives 4x the waves for latency hiding
    e->nsplit_a = (int)std::min<int64_t>(e->NT, std::max<int64_t>(e->nsplit_d, (2048 + e->nrb_max - 1) / e->nrb_max));
    // encoder forward: bf16 ~37 KB (double-buffered), x3 ~39 KB single-buffered: 4 per CU; f32 2
    e->nsplit_e = pick_split(cfg->dtype == MMVAE_DTYPE_F32 ? 2 : 4);
    // encoder backward: bf16 ~37 KB LDS (4 per CU); x3 / f32 keep W in registers, ~43 KB (3 per CU)
    e->nsplit_b = pick_split((bf_ops || vmf_model) ? 4 : 3);  // vMF: no raw-count tile (enc_bwd.hpp)
    // tuning overrides (diagnostics): MMVAE_NSPLIT_E / _D / _A
    auto env_split = [&](const char* name, int& v) {
        if (const char* ev = std::getenv(name)) {
            const int x = std::atoi(ev);
            if (x >= 1) v = (int)std::min<int64_t>(x, e->NT);
        }
    };
    env_split("MMVAE_NSPLIT_E", e->nsplit_e);
    if (std::getenv("MMVAE_NSPLIT_E")) e->nsplit_b = e->nsplit_e;  // a forced encoder split covers both
    env_split("MMVAE_NSPLIT_B", e->nsplit_b);
    env_split("MMVAE_NSPLIT_D", e->nsplit_d);
    env_split("MMVAE_NSPLIT_F", e->nsplit_f);
    env_split("MMVAE_NSPLIT_A", e->nsplit_a);
    e->n_lat_wg = (int)(e->Bpad / LAT_CELLS);  // latent kernels: 16 cells per workgroup
    e->klp_off = e->nrb_max * e->nsplit_d;

    // latent state layout
    int64_t o = 0;
    e->LAT_H = o; o += e->KE;  // h0: the big encoder GEMM's output (post-ReLU)
    e->LAT_MEAN = o; o += e->K;
    e->LAT_A = o; o += e->K;
    e->LAT_EPS = o; o += e->K;
    e->LAT_NMEAN = o; o += e->R;
    e->LAT_AN = o; o += e->R;
    e->LAT_EPSN = o; o += e->R;
    e->LAT_ZNU = o; o += e->R;
    e->LAT_D = o; o += 1;
    e->LAT_W = o; o += 1;
    e->LAT_VALID = o; o += 1;
    e->LAT_HNU = o; o += e->H + 1;  // dhnu[H], dpre
    e->lat_stride = o;

    const int64_t Bp = e->Bpad, DP = e->DP, KP = e->KP, nrb = e->nrb_max;
    const int64_t SMALL = small_len((int)e->K, (int)e->E, (int)e->KE, (int)e->C,
                                    cfg->model == MMVAE_MODEL_VMF ? 0 : (int)(2 * e->R * e->H + 2 * e->R + e->H + 1));
    HIPCHK(e, dalloc(&e->d_params, e->P_reg));
    HIPCHK(e, dalloc(&e->d_grads, e->P_reg));
    HIPCHK(e, dalloc(&e->d_m, e->P_reg));
    HIPCHK(e, dalloc(&e->d_v, e->P_reg));
    HIPCHK(e, dalloc(&e->d_frozen, e->P_frz));
    HIPCHK(e, hipMemset(e->d_params, 0, sizeof(float) * e->P_reg));
    HIPCHK(e, hipMemset(e->d_grads, 0, sizeof(float) * e->P_reg));
    HIPCHK(e, hipMemset(e->d_m, 0, sizeof(float) * e->P_reg));
    HIPCHK(e, hipMemset(e->d_v, 0, sizeof(float) * e->P_reg));
    HIPCHK(e, hipMemset(e->d_frozen, 0, sizeof(float) * e->P_frz));
    // the fused path's operand images and per-step workspace: a wide-path handle (wide.hip) has
    // its own dense buffers and never reads these (they grow with K, E, B and C x D)
    if (!e->wide) {
    HIPCHK(e, dalloc(&e->d_WeP_f, KP * DP));
    HIPCHK(e, dalloc(&e->d_WeP_b, 2 * KP * DP));  // hi + lo planes (x3 mode)
    HIPCHK(e, dalloc(&e->d_WdP_f, KP * DP));
    HIPCHK(e, dalloc(&e->d_WdP_b, 2 * KP * DP));  // hi + lo planes (x3 mode)
    HIPCHK(e, dalloc(&e->d_WdT_f, KP * DP));
    if (cfg->dtype == MMVAE_DTYPE_FP8) {
        HIPCHK(e, dalloc(&e->d_WdP8, KP * DP));
        HIPCHK(e, dalloc(&e->d_WeS8, KP * DP));
        HIPCHK(e, dalloc(&e->d_escale, 2));
    }
    HIPCHK(e, dalloc(&e->d_WdT_b, 2 * KP * DP));  // hi + lo planes (x3 mode)
    HIPCHK(e, dalloc(&e->d_WeS_f, KP * DP));
    HIPCHK(e, dalloc(&e->d_WeS_b, 2 * KP * DP));  // hi + lo planes (x3 mode)
    }
    // per-step host->device staging in ONE pinned block and ONE device block, so a step issues a
    // single H2D copy (each copy is a ~4.5 us blit on the stream):  cells int64 [Bp] |
    // list segments int64 [Bp/16 + 1] | balancing permutation int32 [Bp]
    e->stage_bytes = sizeof(int64_t) * (size_t)(Bp + Bp / 16 + 1) + sizeof(int32_t) * (size_t)Bp + sizeof(StepScalars);
    e->stage_bytes = (e->stage_bytes + 15) / 16 * 16;  // copied in 16-byte chunks (StageCopy)
    e->stage_bytes_res = e->stage_bytes;
    // (+ the batch rowptr [Bp + 1] of a streamed dataset, staged only in that mode)
    const size_t stage_cap = (e->stage_bytes + sizeof(int64_t) * (size_t)(Bp + 1) + 15) / 16 * 16;
    HIPCHK(e, hipMalloc((void**)&e->d_cells, stage_cap));
    e->d_seg = e->d_cells + Bp;
    e->d_perm = reinterpret_cast<int32_t*>(e->d_seg + Bp / 16 + 1);
    e->d_ss = reinterpret_cast<const StepScalars*>(e->d_perm + Bp);  // 8-aligned: Bp % 128 == 0
    e->d_brp = reinterpret_cast<const int64_t*>(e->d_ss + 1);
    for (auto& sl : e->slots2) {
        // device-accessible, coherent: the step's prep kernel reads it directly (StageCopy)
        HIPCHK(e, hipHostMalloc((void**)&sl.block, stage_cap, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(sl.block, 0, stage_cap);
        HIPCHK(e, hipHostMalloc((void**)&sl.eps, sizeof(float) * Bp * (e->K + e->R)));
        HIPCHK(e, hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
    }
    use_slot(e, 0);
    HIPCHK(e, dalloc(&e->d_eps, Bp * (e->K + e->R)));
    if (!e->wide) {
    HIPCHK(e, hipMalloc(&e->d_toff, sizeof(int32_t) * (Bp / 16) * (e->NT + 1)));
    HIPCHK(e, dalloc(&e->d_gene, 10 * DP));
    HIPCHK(e, dalloc(&e->d_mvec, ((DP + 255) / 256) * KP));  // per-256-gene-block partials of mvec
    HIPCHK(e, dalloc(&e->d_rowx, Bp * (2 + e->H)));
    HIPCHK(e, dalloc(&e->d_rowxp, (int64_t)e->nsplit_e * Bp * (1 + e->H)));
    HIPCHK(e, dalloc(&e->d_hpart, (int64_t)e->nsplit_e * Bp * KP));
    HIPCHK(e, dalloc(&e->d_lat, Bp * e->lat_stride));
    HIPCHK(e, dalloc(&e->d_zf, Bp * KP));
    HIPCHK(e, dalloc(&e->d_zb, 2 * Bp * KP));  // hi + lo planes (x3 mode)
    HIPCHK(e, dalloc(&e->d_lsep, (int64_t)e->nsplit_a * Bp * 2));
    HIPCHK(e, dalloc(&e->d_rowB, (int64_t)std::max(e->nsplit_d, e->nsplit_f) * Bp * (2 + e->R)));
    HIPCHK(e, dalloc(&e->d_rowfin, Bp * 2));
    HIPCHK(e, dalloc(&e->d_dzp, (int64_t)e->nsplit_d * Bp * 2 * KP));
    HIPCHK(e, dalloc(&e->d_dh, Bp * KP));
    HIPCHK(e, dalloc(&e->d_dhT_f, Bp * KP));
    HIPCHK(e, dalloc(&e->d_dhT_b, 2 * Bp * KP));  // hi + lo planes (x3 mode)
    HIPCHK(e, dalloc(&e->d_slabB, nrb * ((1 + e->C) + 1 + e->R) * DP));
    HIPCHK(e, dalloc(&e->d_slabC, nrb * (1 + e->C) * DP));
    HIPCHK(e, dalloc(&e->d_slabE, nrb * (2 + e->H) * DP));
    HIPCHK(e, dalloc(&e->d_lossp, e->klp_off + e->n_lat_wg));
    HIPCHK(e, dalloc(&e->d_small, (int64_t)e->n_lat_wg * SMALL));
    HIPCHK(e, dalloc(&e->d_smallg, 128));
    }
    // clip-norm partials: k_sumsq's 256 blocks, or one per gradient-kernel block (NB world 1)
    HIPCHK(e, dalloc(&e->d_sumsq, 256 + (e->D + 31) / 32 + (SMALL + 2 * e->K + 31) / 32 + 1));
    if (!e->wide) {
        int64_t nch = 0;
        for (int l = 0; l < e->nce + e->ncd; ++l) nch = std::max<int64_t>(nch, e->ch_off[l] + e->ch_in[l] * e->ch_out[l] + e->ch_out[l]);
        HIPCHK(e, dalloc(&e->d_chain, nch));
        HIPCHK(e, dalloc(&e->d_rowv, Bp));
        HIPCHK(e, dalloc(&e->d_vk, 8));
    }
    // loss / total norm: written by the kernels straight into mapped pinned memory (no readback copy)
    HIPCHK(e, hipHostMalloc((void**)&e->h_out_pin, sizeof(float) * 4, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(e, hipHostGetDevicePointer((void**)&e->d_out, e->h_out_pin, 0));
    HIPCHK(e, hipHostMalloc((void**)&e->h_ticket, 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(e->h_ticket, 0, 64);
    HIPCHK(e, hipHostGetDevicePointer((void**)&e->d_ticket, e->h_ticket, 0));
    if (e->wide) HIPCHK(e, wide_create(e));
    for (auto& sl : e->slots2) HIPCHK(e, hipEventRecord(sl.ev, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    *out = e;
    return MMVAE_OK;
}

int mmvae_path(mmvae_h e, int32_t* wide) {
    if (!e || !wide) FAIL(e, MMVAE_E_ARG, "path: null");
    *wide = e->wide ? 1 : 0;
    return MMVAE_OK;
}

int mmvae_destroy(mmvae_h e) {
    if (!e) return MMVAE_OK;
    hipSetDevice(e->device);
    hipStreamSynchronize(e->stream);
    if (e->comm_stream) hipStreamSynchronize(e->comm_stream);
    // the gather stream first (its kernels read the slots' mapped pinned blocks: h_gcells,
    // h_brp_pin), then the slots
    stream_release(e);
    for (auto& sl : e->slots2) {
        for (auto& g : sl.graphs) hipGraphExecDestroy(g.second);
        if (sl.block) hipHostFree(sl.block);
        if (sl.eps) hipHostFree(sl.eps);
        if (sl.ev) hipEventDestroy(sl.ev);
    }
    if (e->comm) ncclCommDestroy(e->comm);
    wide_destroy(e);
    void* bufs[] = {e->d_rowptr, e->d_col, e->d_val, e->d_covar, e->d_params, e->d_grads, e->d_m, e->d_v,
                    e->d_frozen, e->d_WeP_f, e->d_WeP_b, e->d_WdP_f, e->d_WdP_b, e->d_WdT_f, e->d_WdT_b, e->d_WeS_f, e->d_WeS_b,
                    e->d_cells, e->d_eps, e->d_gene, e->d_mvec, e->d_rtp, e->d_cellnorm, e->d_pk, e->d_rowx, e->d_rowxp, e->d_hpart, e->d_lat,
                    e->d_zf, e->d_zb, e->d_lsep, e->d_rowB, e->d_rowfin, e->d_dzp, e->d_dh, e->d_dhT_f, e->d_dhT_b,
                    e->d_slabB, e->d_slabC, e->d_slabE, e->d_lossp, e->d_small, e->d_smallg, e->d_sumsq,
                    e->d_tmp, e->d_rowv, e->d_vk, e->d_tmp_ar, e->d_chain, e->d_WdP8, e->d_WeS8, e->d_escale, e->d_flag};
    for (void* b : bufs)
        if (b) hipFree(b);
    for (void* b : {(void*)e->d_toff, (void*)e->d_ents})  // d_seg / d_perm live in d_cells' block
        if (b) hipFree(b);
    if (e->h_out_pin) hipHostFree(e->h_out_pin);
    if (e->h_ticket) hipHostFree(e->h_ticket);
    for (auto ev : e->event_pool) hipEventDestroy(ev);
    for (auto& p : e->pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto ev : e->ev_bucket)
        if (ev) hipEventDestroy(ev);
    if (e->ev_comm_done) hipEventDestroy(e->ev_comm_done);
    if (e->comm_stream) hipStreamDestroy(e->comm_stream);
    hipStreamDestroy(e->stream);
    delete e;
    return MMVAE_OK;
}

}  // extern "C"

// Host -> device copy of a large pageable array through two pinned 32 MB chunks: the host copies
// chunk k + 1 into one while the DMA of chunk k reads the other (pageable hipMemcpy stages
// serially, at a fraction of the link rate).  Synchronous on return.
static hipError_t upload_chunked(Engine* e, void* dst, const void* src, size_t bytes) {
    constexpr size_t CH = (size_t)32 << 20;
    if (bytes <= CH) return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
    char* pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipError_t er = hipSuccess;
    for (int i = 0; i < 2 && er == hipSuccess; ++i) {
        er = hipHostMalloc((void**)&pin[i], CH);
        if (er == hipSuccess) er = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    }
    for (size_t off = 0, k = 0; off < bytes && er == hipSuccess; off += CH, ++k) {
        const int b = (int)(k & 1);
        const size_t n = std::min(CH, bytes - off);
        if (k >= 2) er = hipEventSynchronize(ev[b]);  // this pinned chunk's previous DMA is done
        if (er != hipSuccess) break;
        std::memcpy(pin[b], static_cast<const char*>(src) + off, n);
        er = hipMemcpyAsync(static_cast<char*>(dst) + off, pin[b], n, hipMemcpyHostToDevice, e->stream);
        if (er == hipSuccess) er = hipEventRecord(ev[b], e->stream);
    }
    const hipError_t es = hipStreamSynchronize(e->stream);
    for (int i = 0; i < 2; ++i) {
        if (pin[i]) hipHostFree(pin[i]);
        if (ev[i]) hipEventDestroy(ev[i]);
    }
    return er != hipSuccess ? er : es;
}

extern "C" {

}  // extern "C"

// a caller's cell-major CSR: rowptr monotone from 0, genes in range and strictly increasing per
// row (row validation on host threads; the first bad row of each thread's range is reported)
static int validate_csr(Engine* e, const char* what, const int64_t* rowptr, const int32_t* col, int64_t N, int64_t D) {
    if (D != e->D) FAIL(e, MMVAE_E_ARG, std::string(what) + ": D does not match the model's data_dim");
    if (rowptr[0] != 0) FAIL(e, MMVAE_E_ARG, std::string(what) + ": rowptr[0] must be 0");
    {
        const int nth = (int)std::max<int64_t>(1, std::min<int64_t>(16, N / 4096));
        std::vector<int> bad((size_t)nth, 0);  // 1 monotone, 2 range, 3 order
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t] {
                for (int64_t i = N * t / nth; i < N * (t + 1) / nth && !bad[(size_t)t]; ++i) {
                    if (rowptr[i + 1] < rowptr[i]) { bad[(size_t)t] = 1; break; }
                    for (int64_t j = rowptr[i]; j < rowptr[i + 1]; ++j) {
                        if (col[j] < 0 || col[j] >= D) { bad[(size_t)t] = 2; break; }
                        if (j > rowptr[i] && col[j] <= col[j - 1]) { bad[(size_t)t] = 3; break; }
                    }
                }
            });
        for (auto& x : th) x.join();
        for (int b : bad) {
            if (b == 1) FAIL(e, MMVAE_E_ARG, std::string(what) + ": rowptr not monotone");
            if (b == 2) FAIL(e, MMVAE_E_ARG, std::string(what) + ": gene index out of range");
            if (b == 3) FAIL(e, MMVAE_E_ARG, std::string(what) + ": gene indices must be strictly increasing within a row");
        }
    }
    return MMVAE_OK;
}

extern "C" {

// C == 1 covariates that are all exactly 1 (nullptr: the default ones) — Engine::unit_covar
static bool all_ones(const float* covar, int64_t N) {
    if (!covar) return true;
    for (int64_t i = 0; i < N; ++i)
        if (covar[i] != 1.f) return false;
    return true;
}

int mmvae_upload_csr(mmvae_h e, const int64_t* rowptr, const int32_t* col, const float* val, int64_t N,
                     int64_t D, const float* covar) {
    if (!e || !rowptr || N < 1) FAIL(e, MMVAE_E_ARG, "upload_csr: bad arguments");
    ++e->graph_gen;  // dataset buffers are replaced: step graphs are re-captured
    e->cap_synced = false;
    {
        const int rc = validate_csr(e, "upload_csr", rowptr, col, N, D);
        if (rc) return rc;
    }
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    stream_release(e);
    e->stage_bytes = e->stage_bytes_res;
    const int64_t nnz = rowptr[N];
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    hipFree(e->d_rowptr);
    hipFree(e->d_col);
    hipFree(e->d_val);
    hipFree(e->d_covar);
    e->d_rowptr = nullptr;
    e->d_col = nullptr;
    e->d_val = nullptr;
    e->d_covar = nullptr;
    // N + 2 row pointers: rowptr[N + 1] = nnz makes the empty padding row N (every row past the
    // batch points there) a valid zero-length row for readers that take rowptr[c + 1]
    HIPCHK(e, dalloc(&e->d_rowptr, N + 2));
    // +64: the clamped (unconditional) row loads of the empty padding row N read entry nnz
    HIPCHK(e, dalloc(&e->d_col, nnz + 64));
    HIPCHK(e, dalloc(&e->d_val, nnz + 64));
    HIPCHK(e, dalloc(&e->d_covar, (N + 1) * e->C));  // row N: zeros (padding rows)
    HIPCHK(e, hipMemset(e->d_covar + N * e->C, 0, sizeof(float) * e->C));
    HIPCHK(e, hipMemcpy(e->d_rowptr, rowptr, sizeof(int64_t) * (N + 1), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_rowptr + N + 1, rowptr + N, sizeof(int64_t), hipMemcpyHostToDevice));
    if (nnz > 0) {
        HIPCHK(e, upload_chunked(e, e->d_col, col, sizeof(int32_t) * nnz));
        HIPCHK(e, upload_chunked(e, e->d_val, val, sizeof(float) * nnz));
    }
    e->unit_covar = e->C == 1 && all_ones(covar, N);
    if (covar) {
        HIPCHK(e, hipMemcpy(e->d_covar, covar, sizeof(float) * N * e->C, hipMemcpyHostToDevice));
    } else {
        std::vector<float> ones((size_t)(N * e->C), 1.f);
        HIPCHK(e, hipMemcpy(e->d_covar, ones.data(), sizeof(float) * N * e->C, hipMemcpyHostToDevice));
    }
    e->N = N;
    e->N_host = N;
    e->nnz = nnz;
    e->cell_nnz.resize((size_t)N);
    for (int64_t i = 0; i < N; ++i) e->cell_nnz[(size_t)i] = (int32_t)(rowptr[i + 1] - rowptr[i]);
    HIPCHK(e, build_dataset_index(e));
    return MMVAE_OK;
}

}  // extern "C"

// allocate slot s's batch set for `cap` entries (rowptr / covariates / index sized by Bpad)
static hipError_t batch_set_alloc(Engine* e, int s, int64_t cap) {
    Engine::BatchSet& q = e->bset[s];
    hipFree(q.col);
    hipFree(q.val);
    q.col = nullptr;
    q.val = nullptr;
    hipError_t er;
    if ((er = dalloc(&q.col, cap)) != hipSuccess) return er;
    if ((er = dalloc(&q.val, cap)) != hipSuccess) return er;
    q.cap = cap;
    const int64_t Bp = e->Bpad;
    if (!q.rowptr) {
        if ((er = dalloc(&q.rowptr, Bp + 2)) != hipSuccess) return er;
        if ((er = dalloc(&q.covar, (Bp + 1) * e->C)) != hipSuccess) return er;
        if (!e->wide) {
            if ((er = hipMalloc(&q.rtp, sizeof(int32_t) * (size_t)(Bp + 1) * (size_t)(e->NT + 1))) != hipSuccess) return er;
            if ((er = hipMalloc(&q.cellnorm, sizeof(float2) * (size_t)(Bp + 1))) != hipSuccess) return er;
        }
    }
    return hipSuccess;
}

extern "C" {

int mmvae_stream_csr(mmvae_h e, const int64_t* rowptr, const int32_t* col, const float* val, int64_t N, int64_t D,
                     const float* covar) {
    if (!e || !rowptr || !col || !val || N < 1) FAIL(e, MMVAE_E_ARG, "stream_csr: bad arguments");
    {
        const int rc = validate_csr(e, "stream_csr", rowptr, col, N, D);
        if (rc) return rc;
    }
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    stream_release(e);  // a previous streamed dataset (its registrations, batch sets, buffers)
    const int64_t nnz = rowptr[N];
    // the DMA mode (packed copies only) rides on the prefetched gather; MMVAE_STREAM_SYNC=1 (the
    // in-step gather) and MMVAE_STREAM_DMA=0 read the packed copy over PCIe with the gather kernel
    const bool dma = !getenv_is("MMVAE_STREAM_SYNC", "1") && !getenv_is("MMVAE_STREAM_DMA", "0");
    // Everything of the new dataset is set up first; the resident dataset (if any) is dropped only
    // once it all succeeded, and a failure undoes this call's registrations.
    std::vector<void*> regs;
    uint32_t* packed = nullptr;
    const uint32_t* packed_dev = nullptr;
    size_t packed_map = 0;   // > 0: an mmap of that many bytes (else hipHostMalloc'd)
    bool packed_reg = false;  // the mmap is registered (mapped for the zero-copy gather)
    auto free_packed = [&]() {
        if (!packed) return;
        if (packed_reg) hipHostUnregister(packed);
        if (packed_map) munmap(packed, packed_map);
        else hipHostFree(packed);
        packed = nullptr;
        packed_dev = nullptr;
        packed_map = 0;
        packed_reg = false;
    };
    auto undo = [&]() {
        for (void* h : regs) hipHostFree(h);
        regs.clear();
        free_packed();
        (void)hipGetLastError();
    };
    // the arrays the gather / unpack kernels read over PCIe, as engine-owned mapped pinned copies.
    // The caller's memory itself is never registered: a registration outliving (or not fully
    // undone before) the caller's free let a later host -> device copy from a new array at the
    // same addresses go through the stale mapping (an illegal access in the next upload).
    auto reg = [&](const void* p, size_t bytes, const void** dev) -> hipError_t {
        if (!bytes) {
            *dev = p;
            return hipSuccess;
        }
        void* h = nullptr;
        hipError_t er = hipHostMalloc(&h, bytes, hipHostMallocMapped);
        if (er != hipSuccess) return er;
        regs.push_back(h);
        {  // host threads for the large ones
            const unsigned nth = bytes >= ((size_t)64 << 20) ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nth; ++t)
                th.emplace_back([&, t] {
                    const size_t a = bytes * t / nth, b = bytes * (t + 1) / nth;
                    std::memcpy(static_cast<char*>(h) + a, static_cast<const char*>(p) + a, b - a);
                });
            for (auto& x : th) x.join();
        }
        void* d = nullptr;
        er = hipHostGetDevicePointer(&d, h, 0);
        *dev = d;
        return er;
    };
    auto failed = [&](hipError_t er, const char* what) {
        undo();
        FAIL(e, MMVAE_E_HIP, std::string("stream_csr: ") + what + ": " + hipGetErrorString(er));
    };
    const void* d = nullptr;
    hipError_t er = reg(rowptr, sizeof(int64_t) * (size_t)(N + 1), &d);
    if (er != hipSuccess) return failed(er, "pinning rowptr");
    const int64_t* hs_rowptr = static_cast<const int64_t*>(d);
    // integer counts below 2^16 over at most 2^16 genes: the packed copy (bit-exact values).  In the
    // DMA mode only host threads read it (stream_dma_gather), so it stays pageable; the zero-copy
    // gather reads it over PCIe, so there it is mapped pinned memory.  If no such copy can be made
    // the caller's unpacked arrays serve instead.
    uint32_t cmax = 0;
    if (D <= 65536 && nnz > 0 && !getenv_is("MMVAE_STREAM_PACK", "0")) {
        const size_t bytes = sizeof(uint32_t) * (size_t)nnz;
        // MMVAE_STREAM_THP=1 (experiment): 2 MB transparent huge pages where the host gives them
        const bool thp = getenv_is("MMVAE_STREAM_THP", "1");
        if (dma || thp) {
            const size_t al2 = (size_t)(2u << 20);
            const size_t pbytes = thp ? (bytes + al2 - 1) & ~(al2 - 1) : bytes;
            void* m = mmap(nullptr, pbytes + (thp ? al2 : 0), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (m != MAP_FAILED) {
                if (thp) {  // 2 MB-aligned start inside the mapping, the rest unmapped
                    const uintptr_t a0 = reinterpret_cast<uintptr_t>(m), al = (a0 + al2 - 1) & ~(uintptr_t)(al2 - 1);
                    if (al > a0) munmap(m, al - a0);
                    if (al + pbytes < a0 + pbytes + al2) munmap(reinterpret_cast<void*>(al + pbytes), a0 + pbytes + al2 - (al + pbytes));
                    packed = reinterpret_cast<uint32_t*>(al);
                    madvise(packed, pbytes, MADV_HUGEPAGE);
                } else {
                    packed = static_cast<uint32_t*>(m);
                }
                packed_map = pbytes;
            }
        } else if (hipHostMalloc((void**)&packed, bytes, hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            packed = nullptr;
        }
        if (packed) {
            const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            std::vector<std::thread> th;
            std::vector<char> ok(nth, 1);
            std::vector<uint32_t> cm(nth, 0);
            for (unsigned t = 0; t < nth; ++t)
                th.emplace_back([&, t] {
                    const int64_t a = nnz * t / nth, b = nnz * (t + 1) / nth;
                    for (int64_t i = a; i < b; ++i) {
                        const float v = val[i];
                        const uint32_t c = (uint32_t)(v >= 0.f && v < 65536.f ? (int)v : 0);
                        const float back = (float)c;
                        if (std::memcmp(&back, &v, 4) != 0) {  // non-integer, negative, -0, too large
                            ok[t] = 0;
                            return;
                        }
                        packed[i] = ((uint32_t)col[i] << 16) | c;
                        cm[t] = std::max(cm[t], c);
                    }
                });
            for (auto& x : th) x.join();
            if (std::find(ok.begin(), ok.end(), 0) != ok.end()) {
                free_packed();
            } else {
                cmax = *std::max_element(cm.begin(), cm.end());
                if (dma) {
                    packed_dev = nullptr;  // host-only (the pool packs the step's rows from it)
                } else if (packed_map) {  // the zero-copy gather's THP copy: written, so backed: register
                    void* dp = nullptr;
                    if (hipHostRegister(packed, packed_map, hipHostRegisterMapped) == hipSuccess) {
                        packed_reg = true;
                        if (hipHostGetDevicePointer(&dp, packed, 0) == hipSuccess) packed_dev = static_cast<const uint32_t*>(dp);
                    }
                    if (!packed_dev) free_packed();
                } else {
                    packed_dev = packed;  // hipHostMallocMapped: one address space
                }
            }
        }
        (void)hipGetLastError();
    }
    const int32_t* hs_col = nullptr;
    const float* hs_val = nullptr;
    if (!packed) {
        if ((er = reg(col, sizeof(int32_t) * (size_t)nnz, &d)) != hipSuccess) return failed(er, "pinning col");
        hs_col = static_cast<const int32_t*>(d);
        if ((er = reg(val, sizeof(float) * (size_t)nnz, &d)) != hipSuccess) return failed(er, "pinning val");
        hs_val = static_cast<const float*>(d);
    }
    const float* hs_covar = nullptr;
    if (covar) {
        if ((er = reg(covar, sizeof(float) * (size_t)(N * e->C), &d)) != hipSuccess) return failed(er, "pinning covar");
        hs_covar = static_cast<const float*>(d);
    }
    // the new dataset is in place: the resident one (if any) goes
    for (void* b : {(void*)e->d_rowptr, (void*)e->d_col, (void*)e->d_val, (void*)e->d_covar, (void*)e->d_rtp,
                    (void*)e->d_cellnorm, (void*)e->d_pk})
        if (b) hipFree(b);
    e->d_pk = nullptr;
    e->d_rowptr = nullptr;
    e->d_col = nullptr;
    e->d_val = nullptr;
    e->d_covar = nullptr;
    e->d_rtp = nullptr;
    e->d_cellnorm = nullptr;
    ++e->graph_gen;
    e->cap_synced = false;
    e->hs_registered = regs;
    e->hs_rowptr = hs_rowptr;
    e->hs_packed = packed;
    e->hs_packed_dev = packed_dev;
    e->hs_packed_bytes = packed_map;
    e->hs_packed_reg = packed_reg;
    {
        // the batch lists carry integer counts below 2^22 in the entry word (tiles.hpp EntList);
        // the packed copy already proved counts below 2^16
        bool xm = getenv_is("MMVAE_LISTS_XM", "1");
        if (!packed && !xm) {
            const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            std::vector<char> bad(nth, 0);
            std::vector<std::thread> th;
            for (unsigned t = 0; t < nth; ++t)
                th.emplace_back([&, t] {
                    const int64_t a = nnz * t / nth, b = nnz * (t + 1) / nth;
                    for (int64_t i = a; i < b; ++i) {
                        const float v = val[i];
                        if (std::signbit(v) || !(v < 4194304.f && v == std::floor(v))) {
                            bad[t] = 1;
                            break;
                        }
                    }
                });
            for (auto& x : th) x.join();
            for (char b : bad) xm = xm || b;
        }
        e->ent_xm = xm;
    }
    e->hs_cmax = cmax;
    e->hs_col = hs_col;
    e->hs_val = hs_val;
    e->hs_covar = hs_covar;
    e->unit_covar = e->C == 1 && all_ones(covar, N);
    e->hh_rowptr = rowptr;
    e->hh_col = col;
    e->hh_val = val;
    e->streamed = true;
    e->N_host = N;
    e->N = e->Bpad;  // the device dataset: the batch's rows, row Bpad empty
    e->nnz = nnz;
    e->cell_nnz.resize((size_t)N);
    int64_t mx = 0;
    for (int64_t i = 0; i < N; ++i) {
        e->cell_nnz[(size_t)i] = (int32_t)(rowptr[i + 1] - rowptr[i]);
        mx = std::max<int64_t>(mx, e->cell_nnz[(size_t)i]);
    }
    // initial batch capacity: twice the mean row's share of a full batch (grown on demand)
    const int64_t cap = std::max<int64_t>(1024, 2 * (nnz / N + 1) * e->Bmax);
    for (int s2 = 0; s2 < 2; ++s2) HIPCHK(e, batch_set_alloc(e, s2, cap));
    e->stage_bytes = (e->stage_bytes_res + sizeof(int64_t) * (size_t)(e->Bpad + 1) + 15) / 16 * 16;
    stream_bind(e, e->cur_slot);
    // the prefetched gather (stream.hip stream_prefetch); MMVAE_STREAM_SYNC=1 keeps it in the step
    e->stream_prefetch = !getenv_is("MMVAE_STREAM_SYNC", "1");  // (dma above implies it)
    e->stream_index_step = getenv_is("MMVAE_STREAM_INDEX_STEP", "1");
    e->stream_dma = dma;  // (packed copies only)
    e->stream_b3 = e->stream_dma && e->hs_packed && e->hs_cmax < 256 && getenv_is("MMVAE_STREAM_B3", "1");
    if (e->stream_prefetch) {
        HIPCHK(e, hipStreamCreateWithFlags(&e->gstream, hipStreamNonBlocking));
        for (int s2 = 0; s2 < 2; ++s2) {
            HIPCHK(e, hipEventCreateWithFlags(&e->ev_gathered[s2], hipEventDisableTiming));
            HIPCHK(e, hipEventCreateWithFlags(&e->ev_setfree[s2], hipEventDisableTiming));
            HIPCHK(e, hipEventRecord(e->ev_setfree[s2], e->stream));  // no step on either set yet
            HIPCHK(e, hipHostMalloc((void**)&e->h_gcells[s2], sizeof(int64_t) * (size_t)(e->Bpad + 1),
                                    hipHostMallocMapped | hipHostMallocCoherent));
        }
    }
    return MMVAE_OK;
}

int mmvae_dataset_size(mmvae_h e, int64_t* N, int64_t* D) {
    if (!e) FAIL(e, MMVAE_E_ARG, "dataset_size: null");
    if (N) *N = e->N_host;
    if (D) *D = e->D;
    return MMVAE_OK;
}

int mmvae_synth_csr(mmvae_h e, int64_t N, double lib_size, uint64_t seed, int64_t* nnz_out) {
    if (!e || N < 1 || lib_size <= 0) FAIL(e, MMVAE_E_ARG, "synth_csr: bad arguments");
    HIPCHK(e, hipSetDevice(e->device));
    ++e->graph_gen;
    e->cap_synced = false;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    stream_release(e);
    e->stage_bytes = e->stage_bytes_res;
    HIPCHK(e, synth_dataset(e, N, lib_size, seed, nnz_out));
    e->N_host = e->N;
    return MMVAE_OK;
}

int mmvae_get_rows(mmvae_h e, const int64_t* rows, int64_t nrows, int64_t* rowptr_out, int32_t* col_out,
                   float* val_out, int64_t* nnz_io) {
    if (!e || !rows || !rowptr_out || !nnz_io) FAIL(e, MMVAE_E_ARG, "get_rows: bad arguments");
    if (!e->d_rowptr) FAIL(e, MMVAE_E_STATE, "get_rows: no dataset");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->streamed) {  // the caller's own host arrays
        int64_t need = 0;
        rowptr_out[0] = 0;
        for (int64_t i = 0; i < nrows; ++i) {
            if (rows[i] < 0 || rows[i] >= e->N_host) FAIL(e, MMVAE_E_ARG, "get_rows: row out of range");
            need += e->hh_rowptr[rows[i] + 1] - e->hh_rowptr[rows[i]];
            rowptr_out[i + 1] = need;
        }
        if (need <= *nnz_io && col_out && val_out)
            for (int64_t i = 0; i < nrows; ++i) {
                const int64_t a = e->hh_rowptr[rows[i]], n = e->hh_rowptr[rows[i] + 1] - a;
                std::memcpy(col_out + rowptr_out[i], e->hh_col + a, sizeof(int32_t) * (size_t)n);
                std::memcpy(val_out + rowptr_out[i], e->hh_val + a, sizeof(float) * (size_t)n);
            }
        *nnz_io = need;
        return MMVAE_OK;
    }
    std::vector<int64_t> rp(e->N + 1);
    HIPCHK(e, hipMemcpy(rp.data(), e->d_rowptr, sizeof(int64_t) * (e->N + 1), hipMemcpyDeviceToHost));
    int64_t need = 0;
    rowptr_out[0] = 0;
    for (int64_t i = 0; i < nrows; ++i) {
        if (rows[i] < 0 || rows[i] >= e->N) FAIL(e, MMVAE_E_ARG, "get_rows: row out of range");
        need += rp[rows[i] + 1] - rp[rows[i]];
        rowptr_out[i + 1] = need;
    }
    if (need > *nnz_io || !col_out || !val_out) {
        *nnz_io = need;
        return MMVAE_OK;
    }
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t a = rp[rows[i]], n = rp[rows[i] + 1] - a;
        if (n == 0) continue;
        HIPCHK(e, hipMemcpy(col_out + rowptr_out[i], e->d_col + a, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(val_out + rowptr_out[i], e->d_val + a, sizeof(float) * n, hipMemcpyDeviceToHost));
    }
    *nnz_io = need;
    return MMVAE_OK;
}

int mmvae_num_params(mmvae_h e, int32_t* count) {
    if (!e || !count) FAIL(e, MMVAE_E_ARG, "num_params: null");
    *count = (int32_t)e->slots.size();
    return MMVAE_OK;
}

int mmvae_param_info(mmvae_h e, int32_t idx, const char** name, int64_t* numel, int32_t* registered) {
    if (!e || idx < 0 || idx >= (int)e->slots.size()) FAIL(e, MMVAE_E_ARG, "param_info: index out of range");
    const ParamSlot& s = e->slots[idx];
    if (name) *name = s.name.c_str();
    if (numel) *numel = s.numel;
    if (registered) *registered = s.registered ? 1 : 0;
    return MMVAE_OK;
}

int mmvae_param_shape(mmvae_h e, int32_t idx, int32_t* ndim, int64_t* shape2) {
    if (!e || idx < 0 || idx >= (int)e->slots.size()) FAIL(e, MMVAE_E_ARG, "param_shape: index out of range");
    const ParamSlot& s = e->slots[idx];
    if (ndim) *ndim = (int32_t)s.shape.size();
    if (shape2) {
        shape2[0] = s.shape.size() > 0 ? s.shape[0] : 1;
        shape2[1] = s.shape.size() > 1 ? s.shape[1] : 1;
    }
    return MMVAE_OK;
}

static int find_slot(Engine* e, const char* name, int64_t numel, const ParamSlot** out) {
    if (!name) FAIL(e, MMVAE_E_ARG, "null parameter name");
    const ParamSlot* s = e->slot(name);
    if (!s) FAIL(e, MMVAE_E_NAME, std::string("unknown parameter ") + name);
    if (numel != s->numel)
        FAIL(e, MMVAE_E_ARG, std::string("numel mismatch for ") + name + ": expected " + std::to_string(s->numel));
    *out = s;
    return MMVAE_OK;
}

int mmvae_set_param(mmvae_h e, const char* name, const float* host, int64_t numel) {
    if (!e || !host) FAIL(e, MMVAE_E_ARG, "set_param: null");
    const ParamSlot* s;
    int rc = find_slot(e, name, numel, &s);
    if (rc) return rc;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    float* dst = s->registered ? e->d_params + s->off : e->d_frozen + s->off;
    HIPCHK(e, hipMemcpy(dst, host, sizeof(float) * numel, hipMemcpyHostToDevice));
    if (!s->registered) e->frozen_dirty = true;
    return MMVAE_OK;
}

int mmvae_get_param(mmvae_h e, const char* name, float* host, int64_t numel) {
    if (!e || !host) FAIL(e, MMVAE_E_ARG, "get_param: null");
    const ParamSlot* s;
    int rc = find_slot(e, name, numel, &s);
    if (rc) return rc;
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const float* src = s->registered ? e->d_params + s->off : e->d_frozen + s->off;
    HIPCHK(e, hipMemcpy(host, src, sizeof(float) * numel, hipMemcpyDeviceToHost));
    return MMVAE_OK;
}

int mmvae_get_grad(mmvae_h e, const char* name, float* host, int64_t numel) {
    if (!e || !host) FAIL(e, MMVAE_E_ARG, "get_grad: null");
    const ParamSlot* s;
    int rc = find_slot(e, name, numel, &s);
    if (rc) return rc;
    if (!s->registered) FAIL(e, MMVAE_E_ARG, std::string(name) + " is frozen (unregistered, Q1): no gradient");
    if (!e->have_grads) FAIL(e, MMVAE_E_STATE, "get_grad: no update step has run");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(host, e->d_grads + s->off, sizeof(float) * numel, hipMemcpyDeviceToHost));
    return MMVAE_OK;
}

int mmvae_init_params(mmvae_h e, uint64_t seed) {
    if (!e) FAIL(e, MMVAE_E_ARG, "init_params: null");
    std::mt19937_64 rng(seed);
    // fan_in of each weight; biases share their layer's bound (torch::nn::Linear::reset_parameters)
    auto fan_in_of = [&](const ParamSlot& s) -> int64_t {
        std::string base = s.name.substr(0, s.name.rfind('.'));
        const ParamSlot* w = e->slot(base + ".weight");
        if (!w || w->shape.size() < 2) return 1;
        return w->shape[1];
    };
    for (const ParamSlot& s : e->slots) {
        std::vector<float> v((size_t)s.numel, 0.f);
        if (s.name == "ln_x_sd") {
            std::fill(v.begin(), v.end(), 1.f);
        } else if (s.name == "ln_kappa") {
            std::fill(v.begin(), v.end(), std::log(e->cfg.kappa_min));  // vmf.hh:323 (float log, Q4)
        } else if (s.name == "x_mean" || s.name == "mu_bias" || s.name == "nu_bias") {
            // zeros (nb.hh:312-315)
        } else {
            const double bound = 1.0 / std::sqrt((double)fan_in_of(s));
            std::uniform_real_distribution<float> U((float)-bound, (float)bound);
            for (auto& x : v) x = U(rng);
        }
        int rc = mmvae_set_param(e, s.name.c_str(), v.data(), s.numel);
        if (rc) return rc;
    }
    return mmvae_reset_optimizer(e);
}

int mmvae_reset_optimizer(mmvae_h e) {
    if (!e) FAIL(e, MMVAE_E_ARG, "reset_optimizer: null");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipMemsetAsync(e->d_m, 0, sizeof(float) * e->P_reg, e->stream));
    HIPCHK(e, hipMemsetAsync(e->d_v, 0, sizeof(float) * e->P_reg, e->stream));
    e->adam_step = 0;
    return MMVAE_OK;
}

// Row balancing for the tile kernels: a workgroup's time is set by its heaviest 16-row wave,
// and the CSR entry count per row varies with the library size.  The batch's rows are ordered
// by nonzero count (bucketed counting sort, O(B)) and dealt to the B/16 waves in a snake, so
// every wave holds an even spread of light and heavy cells.  Per-row results are independent
// of the order and every batch sum is a fixed-order reduction; the reparameterisation noise
// stays keyed by the ORIGINAL batch position (perm), as is the injected eps.
static void balance_rows(Engine* e, int64_t B) {
    std::vector<int64_t> cells(e->h_cells_pin, e->h_cells_pin + B);
    int32_t mx = 1;
    for (int64_t j = 0; j < B; ++j) mx = std::max(mx, e->cell_nnz[(size_t)cells[(size_t)j]]);
    int sh = 0;
    while ((mx >> sh) >= 1024) ++sh;
    std::vector<int32_t> cnt(1025, 0), order((size_t)B);
    for (int64_t j = 0; j < B; ++j) ++cnt[(size_t)(1023 - (e->cell_nnz[(size_t)cells[(size_t)j]] >> sh)) + 1];
    for (int i = 0; i < 1024; ++i) cnt[(size_t)i + 1] += cnt[(size_t)i];
    for (int64_t j = 0; j < B; ++j) order[(size_t)cnt[(size_t)(1023 - (e->cell_nnz[(size_t)cells[(size_t)j]] >> sh))]++] = (int32_t)j;
    const int64_t nw = B / 16;
    for (int64_t s2 = 0; s2 < B; ++s2) {
        const int64_t pass = s2 / nw, q = s2 % nw, wv = (pass & 1) ? nw - 1 - q : q;
        const int64_t slot = wv * 16 + pass;
        e->h_cells_pin[slot] = cells[(size_t)order[(size_t)s2]];
        e->h_perm_pin[slot] = order[(size_t)s2];
    }
}

// the batch entry lists (+ the NB raw-count dots of depth / nu_enc, split 0 of rowxp)
static hipError_t build_lists(Engine* e, int64_t B) {
    if (e->cfg.model == MMVAE_MODEL_VMF) return build_batch_lists(e, B, nullptr, nullptr, nullptr);
    // the packed dot weights come from k_prep (nb_prep ran first on the same stream)
    return build_batch_lists(e, B, reinterpret_cast<const float2*>(e->d_gene + 8 * e->DP),
                             e->preg("nu_encoding.weight"), e->d_rowxp);
}

static inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#else
    std::this_thread::yield();
#endif
}

// until the device has written back staging ticket t (spin on the mapped word; a drained stream
// also frees the slot)
static hipError_t wait_ticket(Engine* e, int64_t t) {
    const volatile int64_t* p = e->h_ticket;
    for (uint32_t i = 1; *p < t; ++i) {
        if ((i & 63) == 0) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return q;
        }
        cpu_relax();
    }
    return hipSuccess;
}

// the slot's step: a fused-path step is tracked by its staging ticket, others by the slot's event
static hipError_t release_slot(Engine* e, bool ticketed) {
    auto& sl = e->slots2[e->cur_slot];
    sl.ticket = ticketed ? e->h_ss->ticket : 0;
    return ticketed ? hipSuccess : hipEventRecord(sl.ev, e->stream);
}

// host half of a step's staging: rows (+ balancing permutation, list segments) into the pinned
// block; the one H2D copy of the block is issued by the caller (stage_copy), inside a step graph
// when one is used
static int stage_rows(Engine* e, const int64_t* cell_ids, const int64_t* ridx, int64_t B, bool balance = false) {
    // the other pinned slot: wait until the step staged from it two steps ago is done with it
    use_slot(e, e->cur_slot ^ 1);
    {
        const auto& sl = e->slots2[e->cur_slot];
        HIPCHK(e, sl.ticket > 0 ? wait_ticket(e, sl.ticket) : hipEventSynchronize(e->ev_staged));
    }
    e->h_ss->ticket = ++e->ticket_seq;  // (only the fused path's k_batch_lists writes it back)
    for (int64_t j = 0; j < B; ++j) {
        int64_t r = j;
        if (ridx) {
            r = ridx[j];
            if (r < 0 || r >= B) FAIL(e, MMVAE_E_ARG, "ridx out of range [0, B)");
        }
        const int64_t c = cell_ids[r];
        if (c < 0 || c >= e->N_host) FAIL(e, MMVAE_E_ARG, "cell id out of range [0, N)");
        e->h_cells_pin[j] = c;
    }
    const int64_t Nv = e->N_host;  // the caller's cells (the padding marker: Nv)
    e->perm_active = balance && balance_rule(B, e->wide, (int64_t)e->cell_nnz.size() == Nv, e->no_balance);
    if (e->perm_active) {
        balance_rows(e, B);
    }
    // padding rows (up to the handle's padded max batch: the latent-head grids cover it) point
    // at row N: the empty row of the dataset index, a zero covariate row and rowptr[N] — so
    // every per-row load in the kernels is unconditional
    const int64_t Bp = e->Bpad;
    for (int64_t j = B; j < Bp; ++j) e->h_cells_pin[j] = Nv;
    // entry-list segments of the batch's 16-row wave blocks (batch.hip): host prefix of the
    // rows' nonzero counts; the list buffer grows (outside any step) when a batch needs more
    const int64_t Bq = pad_rows(B), WB = Bq / 16;
    int64_t tot = 0;
    for (int64_t wb = 0; wb < WB; ++wb) {
        e->h_seg_pin[wb] = tot;
        for (int r = 0; r < 16; ++r) {
            const int64_t c = e->h_cells_pin[wb * 16 + r];
            tot += (c < Nv) ? e->cell_nnz[(size_t)c] : 0;
        }
    }
    e->h_seg_pin[WB] = tot;
    if (e->streamed) {
        // the batch CSR's row offsets (every padded row; padding rows empty), staged for the
        // gather kernel; the slot's batch set grows (outside any step) when the batch needs more
        int64_t o = 0;
        for (int64_t b = 0; b < Bp; ++b) {
            e->h_brp_pin[b] = o;
            const int64_t c = e->h_cells_pin[b];
            o += (c < Nv) ? e->cell_nnz[(size_t)c] : 0;
        }
        e->h_brp_pin[Bp] = o;
        if (e->stream_prefetch) {
            // the gather reads the slot's row ids; the staged cells become the identity (the
            // batch's row b is batch-CSR row b), as the in-step gather leaves them
            int64_t* gc = e->h_gcells[e->cur_slot];
            for (int64_t b = 0; b < Bp; ++b) {
                gc[b] = e->h_cells_pin[b];
                e->h_cells_pin[b] = b;
            }
        }
        if (o > e->bset[e->cur_slot].cap) {
            HIPCHK(e, hipStreamSynchronize(e->stream));
            if (e->gstream) HIPCHK(e, hipStreamSynchronize(e->gstream));
            HIPCHK(e, batch_set_alloc(e, e->cur_slot, o + o / 4 + 1024));
            ++e->graph_gen;  // the slot's graphs point at the old buffers
        }
        stream_bind(e, e->cur_slot);
    }
    if (!e->wide && tot + 64 > e->ent_cap) {  // (the wide path reads the CSR rows directly)
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (e->d_ents) hipFree(e->d_ents);
        e->d_ents = nullptr;
        e->ent_cap = tot + tot / 4 + 1024;
        HIPCHK(e, hipMalloc(&e->d_ents, sizeof(uint2) * e->ent_cap));
        HIPCHK(e, hipMemset(e->d_ents, 0, sizeof(uint2) * e->ent_cap));
    }
    return MMVAE_OK;
}

}  // extern "C"

namespace mmvae {
// cells | segments | permutation | step scalars: copied from the current slot's mapped pinned
// block by the step's prep kernel (k_prep / k_vprep, StageCopy; the block is reused only after
// its slot's event)
StageCopy stage_copy_args(Engine* e) {
    return StageCopy{reinterpret_cast<const uint4*>(e->h_cells_pin), reinterpret_cast<uint4*>(e->d_cells),
                     (int)(e->stage_bytes / 16)};
}
}  // namespace mmvae

extern "C" {

// the device work of one step / eval, in stream order (eager, or captured into a step graph)
static int enqueue_run(Engine* e, const mmvae_step_args* a, int64_t n_total) {
    const bool vmf = e->cfg.model == MMVAE_MODEL_VMF;
    if (a->eps) {
        const int64_t ne = a->B * (e->K + (vmf ? 0 : e->R));
        HIPCHK(e, hipMemcpyAsync(e->d_eps, e->h_eps_pin, sizeof(float) * ne, hipMemcpyHostToDevice, e->stream));
    }
    e->grads_reduced = false;
    e->sq_parts = 0;
    if (e->wide) {
        HIPCHK(e, wide_forward_backward(e, a->B, n_total, a->beta, a->update != 0, a->eps != nullptr));  // + staged copy
    } else {
    HIPCHK(e, vmf ? vmf_prep(e, a->B, n_total, a->beta) : nb_prep(e, a->B, n_total, a->beta));  // + staged copy
    HIPCHK(e, stream_gather(e));  // (streamed dataset: the batch's rows from host memory)
    HIPCHK(e, build_lists(e, a->B));
    if (vmf) HIPCHK(e, vmf_forward_backward(e, a->B, n_total, a->beta, a->update != 0, a->eps != nullptr));
    else HIPCHK(e, nb_forward_backward(e, a->B, n_total, a->beta, a->update != 0, a->eps != nullptr));
    }
    if (a->update) {
        if (e->comm_active() && !e->grads_reduced) {
            ScopedTimer tm(e, "allreduce_grads");
            if (ncclAllReduce(e->d_grads, e->d_grads, (size_t)e->P_reg, ncclFloat, ncclSum, e->comm, e->stream) !=
                ncclSuccess)
                FAIL(e, MMVAE_E_COMM, "ncclAllReduce failed");
        }
        HIPCHK(e, opt_clip_adam(e));
    }
    return MMVAE_OK;  // loss and norm land in the mapped h_out_pin (d_out)
}

static void graph_drop(Engine* e) {
    for (auto& sl : e->slots2) {
        for (auto& g : sl.graphs) hipGraphExecDestroy(g.second);
        sl.graphs.clear();
    }
}

int mmvae_run(mmvae_h e, const mmvae_step_args* a, float* loss_out, double* total_norm_out) {
    if (!e || !a || !a->cell_ids) FAIL(e, MMVAE_E_ARG, "run: null arguments");
    if (a->B < 1 || a->B > e->Bmax) FAIL(e, MMVAE_E_ARG, "run: B must be in [1, max_batch]");
    if (!e->d_rowptr) FAIL(e, MMVAE_E_STATE, "run: no dataset uploaded");
    const int64_t n_total = a->n_total > 0 ? a->n_total : a->B;
    HIPCHK(e, hipSetDevice(e->device));
    // step graphs holding RCCL calls: the batch-dependent buffers sized for every rank's worst
    // batch first, so that no rank's graph key changes alone (comm_sync_capacity)
    const bool comm_graph_step = e->graph_on && !e->timing && e->comm_active() && e->comm_graph && !e->comm_graph_failed;
    if (comm_graph_step && a->B * (int64_t)e->world != n_total)  // (before any collective: graph_key.hpp)
        FAIL(e, MMVAE_E_ARG, "run: step graphs with RCCL calls (MMVAE_COMM_GRAPH=1) need B * world == n_total");
    if (comm_graph_step && !e->cap_synced) {
        const int crc = comm_sync_capacity(e);
        if (crc) return crc;
    }
    int rc = stage_rows(e, a->cell_ids, a->ridx, a->B, /*balance=*/true);
    if (rc) return rc;
    HIPCHK(e, stream_prefetch(e));  // (streamed dataset: the rows' gather on its own stream)
    const bool vmf = e->cfg.model == MMVAE_MODEL_VMF;
    if (a->eps) std::memcpy(e->h_eps_pin, a->eps, sizeof(float) * a->B * (e->K + (vmf ? 0 : e->R)));
    // the step's scalars travel in the staged block (the kernels read them from there)
    e->h_ss->step_id = (int64_t)a->step_id;
    e->h_ss->row_offset = a->row_offset;
    if (a->update) adam_scalars(e, e->adam_step + 1, e->h_ss);
    // frozen operands are repacked eagerly, never inside a step graph
    if (e->frozen_dirty) HIPCHK(e, e->wide ? wide_prepare_frozen(e) : vmf ? vmf_prepare_frozen(e) : nb_prepare_frozen(e));
    // one hipGraph per step: captured on the first step of a launch shape,
    // replayed while the shape holds; not with timers or diagnostics.  With an active
    // communicator the graph holds the RCCL bucket all-reduces too (comm_bucket's event fork onto
    // the comm stream and its join back are captured with them) when MMVAE_COMM_GRAPH=1 was set
    // at mmvae_comm_init (otherwise: eager steps).  Every rank takes the same capture decisions: the graph
    // key's batch-dependent buffers are sized for every rank's worst batch (comm_sync_capacity),
    // the capture outcome is agreed (comm_capture_agree), and a failed capture falls back to
    // eager launches for the handle's lifetime on every rank.
#ifdef MMVAE_DIAG
    static const bool dbg_env = std::getenv("MMVAE_DBG") != nullptr;
#else
    constexpr bool dbg_env = false;
#endif
    const bool with_comm = e->comm_active();
    const bool use_graph = e->graph_on && !e->timing && !dbg_env &&
                           (!with_comm || (e->comm_graph && !e->comm_graph_failed));
    if (use_graph) {
        GraphKey k;
        KeyInputs ki;
        ki.B = a->B;
        ki.n_total = n_total;
        ki.beta = a->beta;
        ki.update = a->update != 0;
        ki.use_eps = a->eps != nullptr;
        ki.perm = e->perm_active;
        ki.world = e->world;
        ki.comm_graph = with_comm;
        ki.ents = e->d_ents;
        ki.gen = e->graph_gen;
        if (derive_graph_key(ki, &k)) FAIL(e, MMVAE_E_ARG, "run: graph key (B * world != n_total)");
        Engine::StageSlot& sl = e->slots2[e->cur_slot];
        hipGraphExec_t gx = nullptr;
        for (auto& g : sl.graphs)
            if (g.first == k) gx = g.second;
        if (!gx) {
            constexpr size_t MAX_GRAPHS = 4;  // per slot; the oldest is dropped
            if (sl.graphs.size() >= MAX_GRAPHS) {
                hipGraphExecDestroy(sl.graphs.front().second);
                sl.graphs.erase(sl.graphs.begin());
            }
            HIPCHK(e, hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
            const int crc = enqueue_run(e, a, n_total);
            hipGraph_t g = nullptr;
            const hipError_t ce = hipStreamEndCapture(e->stream, &g);
            hipError_t ie = hipSuccess;
            if (!crc && ce == hipSuccess) ie = hipGraphInstantiate(&gx, g, nullptr, nullptr, 0);
            if (g) hipGraphDestroy(g);
            const bool cap_ok = !crc && ce == hipSuccess && ie == hipSuccess;
            // a failed capture or instantiation leaves a sticky error: cleared on every path (its
            // code is returned below, or the eager fallback runs on a clean runtime state)
            if (!cap_ok) (void)hipGetLastError();
            bool comm_fail = false;
            if (with_comm) {
                // the ranks agree before any of them launches: a graph one rank captured while
                // another fell back would pair a replayed collective with eager ones
                int agreed = 0;
                HIPCHK(e, comm_capture_agree(e, cap_ok, k, &agreed));
                comm_fail = !agreed;
            }
            if (comm_fail) {
                // the communicator's calls did not capture here or on another rank: this step and
                // the later ones with it run eagerly (nothing of the capture was executed)
                if (gx) hipGraphExecDestroy(gx);
                e->comm_graph_failed = true;
                gx = nullptr;
            } else {
                if (crc) return crc;
                HIPCHK(e, ce);
                HIPCHK(e, ie);
                sl.graphs.emplace_back(k, gx);
                ++e->graph_captures;
            }
        }
        if (gx) {
            HIPCHK(e, hipGraphLaunch(gx, e->stream));
            ++e->graph_replays;
        } else {
            rc = enqueue_run(e, a, n_total);
            if (rc) return rc;
        }
    } else {
        rc = enqueue_run(e, a, n_total);
        if (rc) return rc;
    }
    HIPCHK(e, release_slot(e, !e->wide));  // this slot's block is free after this step's copy
    HIPCHK(e, stream_step_done(e));
    if (a->update) {
        e->adam_step += 1;
        e->have_grads = true;
    }
    if (loss_out || total_norm_out) {
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (loss_out) *loss_out = e->h_out_pin[0];
        if (total_norm_out) *total_norm_out = a->update ? (double)e->h_out_pin[1] : 0.0;
    }
    if (e->timing) timer_collect(e);
    return MMVAE_OK;
}

static int step_or_eval(mmvae_h e, const int64_t* cell_ids, int64_t B, const int64_t* ridx, float beta,
                        const float* eps, float* loss_out, int update) {
    if (!e) FAIL(e, MMVAE_E_ARG, "step: null handle");
    mmvae_step_args a;
    std::memset(&a, 0, sizeof(a));
    a.cell_ids = cell_ids;
    a.ridx = ridx;
    a.B = B;
    a.n_total = B;
    a.beta = beta;
    a.eps = eps;
    a.step_id = e->auto_step++;
    a.update = update;
    return mmvae_run(e, &a, loss_out, nullptr);
}

int mmvae_step(mmvae_h e, const int64_t* cell_ids, int64_t B, const int64_t* ridx_or_null, float beta,
               const float* eps_or_null, float* loss_out) {
    return step_or_eval(e, cell_ids, B, ridx_or_null, beta, eps_or_null, loss_out, 1);
}

int mmvae_eval(mmvae_h e, const int64_t* cell_ids, int64_t B, float beta, const float* eps_or_null, float* loss_out) {
    return step_or_eval(e, cell_ids, B, nullptr, beta, eps_or_null, loss_out, 0);
}

int mmvae_encode(mmvae_h e, const int64_t* cell_ids, int64_t B, float* mean, float* lnvar) {
    if (!e || !cell_ids || !mean || !lnvar) FAIL(e, MMVAE_E_ARG, "encode: null arguments");
    if (B < 1 || B > e->Bmax) FAIL(e, MMVAE_E_ARG, "encode: B must be in [1, max_batch]");
    if (!e->d_rowptr) FAIL(e, MMVAE_E_STATE, "encode: no dataset uploaded");
    HIPCHK(e, hipSetDevice(e->device));
    int rc = stage_rows(e, cell_ids, nullptr, B);
    if (rc) return rc;
    HIPCHK(e, stream_prefetch(e));
    if (e->wide) {
        if (e->frozen_dirty) HIPCHK(e, wide_prepare_frozen(e));
        if (!e->d_tmp) HIPCHK(e, dalloc(&e->d_tmp, 2 * e->Bpad * e->K));
        HIPCHK(e, wide_encode(e, B, e->d_tmp, e->d_tmp + e->Bpad * e->K));  // + the staged copy
        HIPCHK(e, release_slot(e, false));
    } else {
    if (e->cfg.model != MMVAE_MODEL_VMF) HIPCHK(e, nb_prep(e, B, B, 1.f));  // + the staged copy
    else HIPCHK(e, vmf_prep(e, B, B, 1.f));
    HIPCHK(e, stream_gather(e));
    HIPCHK(e, release_slot(e, true));
    HIPCHK(e, build_lists(e, B));
    if (!e->d_tmp) HIPCHK(e, dalloc(&e->d_tmp, 2 * e->Bpad * e->K));
    if (e->cfg.model == MMVAE_MODEL_VMF) HIPCHK(e, vmf_encode(e, B, e->d_tmp, e->d_tmp + e->Bpad * e->K));
    else HIPCHK(e, nb_encode(e, B, e->d_tmp, e->d_tmp + e->Bpad * e->K));
    }
    HIPCHK(e, hipMemcpyAsync(mean, e->d_tmp, sizeof(float) * B * e->K, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipMemcpyAsync(lnvar, e->d_tmp + e->Bpad * e->K, sizeof(float) * B * e->K, hipMemcpyDeviceToHost,
                             e->stream));
    HIPCHK(e, stream_step_done(e));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MMVAE_OK;
}

int mmvae_sync(mmvae_h e) {
    if (!e) FAIL(e, MMVAE_E_ARG, "sync: null");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->timing) timer_collect(e);
    return MMVAE_OK;
}

int mmvae_comm_unique_id(void* out128) {
    if (!out128) FAIL((Engine*)nullptr, MMVAE_E_ARG, "comm_unique_id: null");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) FAIL((Engine*)nullptr, MMVAE_E_COMM, "ncclGetUniqueId failed");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(out128, &id, 128);
    return MMVAE_OK;
}

extern "C++" {
namespace mmvae {
static void build_buckets(Engine* e);
}
}

int mmvae_comm_init(mmvae_h e, int32_t rank, int32_t world, const void* id128) {
    if (!e || world < 1 || rank < 0 || rank >= world) FAIL(e, MMVAE_E_ARG, "comm_init: bad arguments");
    HIPCHK(e, hipSetDevice(e->device));
    ++e->graph_gen;  // rank-dependent launches (the vMF rank-0 term, bucket split) are re-captured
    e->cap_synced = false;
    if (!id128) {
        // local decomposition mode (tests): this handle computes rank `rank`'s shard of a
        // world-`world` step (rank-0-only terms included) but reduces nothing — the caller sums
        // the shards' gradients and losses itself
        if (e->comm) {
            ncclCommDestroy(e->comm);
            e->comm = nullptr;
        }
        e->comm_force = false;
        e->rank = rank;
        e->world = world;
        return MMVAE_OK;
    }
    ncclUniqueId id;
    std::memcpy(&id, id128, 128);
    if (e->comm) {
        ncclCommDestroy(e->comm);
        e->comm = nullptr;
    }
    ncclResult_t r = ncclCommInitRank(&e->comm, world, id, rank);
    if (r != ncclSuccess) FAIL(e, MMVAE_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    e->rank = rank;
    e->world = world;
    e->comm_force = getenv_is("MMVAE_FORCE_COMM", "1");
    // RCCL calls inside step graphs: opt-in (MMVAE_COMM_GRAPH=1).  No multi-rank run of captured
    // collectives has been made yet (one-GPU pool), so the default is the eager exchange.
    // One-GPU cost of the exchange at the headline shape (bench.py dp_exchange, forced 1-rank
    // communicator): flat eager -4 us per step, buckets eager +33 us, buckets captured +5 us
    e->comm_graph = getenv_is("MMVAE_COMM_GRAPH", "1");
    e->comm_graph_failed = false;
    if (!e->comm_stream) {
        HIPCHK(e, hipStreamCreateWithFlags(&e->comm_stream, hipStreamNonBlocking));
        for (auto& ev : e->ev_bucket) HIPCHK(e, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIPCHK(e, hipEventCreateWithFlags(&e->ev_comm_done, hipEventDisableTiming));
    }
    build_buckets(e);
    return MMVAE_OK;
}

extern "C++" {
namespace mmvae {
bool split_grads(const Engine* e) {
    // With a communicator: the two overlapped buckets when the step is captured into a graph
    // (their comm-stream fork / join is cheap there), otherwise one all-reduce of the whole flat
    // gradient on the main stream after the backward (eager fork / join costs more than the bucket
    // hides, bench.py dp_exchange).  MMVAE_NO_OVERLAP=1 forces the flat path, MMVAE_OVERLAP=1 the
    // buckets.
    if (e->comm_active()) {
        if (getenv_is("MMVAE_NO_OVERLAP", "1")) return false;
        if (getenv_is("MMVAE_OVERLAP", "1")) return true;
        return e->comm_graph && !e->comm_graph_failed;
    }
    const char* v = std::getenv("MMVAE_SPLIT_GRADS");
    return v && v[0] == '1';
}

// bucket 0: the decoder-side gene vectors — NB mu_bias, nu_bias, covar_decoding.*, nu_decoding.*
// (final after decoder pass C), vMF covar_decoding_.* (final after k_vdec_bwd); bucket 1: the
// complement (encoder gene vectors, latent heads, ln_kappa)
static void build_buckets(Engine* e) {
    const char* dec[] = {"mu_bias", "nu_bias", "covar_decoding.weight", "covar_decoding.bias",
                         "nu_decoding.weight", "nu_decoding.bias",
                         "covar_decoding_.weight", "covar_decoding_.bias"};  // (vMF names)
    std::vector<std::pair<int64_t, int64_t>> r0;
    for (const char* n : dec)
        if (const ParamSlot* sl = e->slot(n)) r0.push_back({sl->off, sl->numel});
    std::sort(r0.begin(), r0.end());
    e->bucket_ranges[0].clear();
    e->bucket_ranges[1].clear();
    for (auto& r : r0) {  // merge adjacent ranges
        auto& b = e->bucket_ranges[0];
        if (!b.empty() && b.back().first + b.back().second == r.first) b.back().second += r.second;
        else b.push_back(r);
    }
    int64_t at = 0;
    for (auto& r : e->bucket_ranges[0]) {
        if (r.first > at) e->bucket_ranges[1].push_back({at, r.first - at});
        at = r.first + r.second;
    }
    if (at < e->P_reg) e->bucket_ranges[1].push_back({at, e->P_reg - at});
}

hipError_t comm_bucket(Engine* e, int b) {
    if (!e->comm_active()) return hipSuccess;
    {
        // test hook (MMVAE_TEST_COMM_CAPTURE_FAIL=1): the bucket refuses to enqueue while its
        // stream is being captured, as a runtime whose RCCL cannot be captured would
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (getenv_is("MMVAE_TEST_COMM_CAPTURE_FAIL", "1") && hipStreamIsCapturing(e->stream, &cs) == hipSuccess &&
            cs == hipStreamCaptureStatusActive)
            return hipErrorStreamCaptureUnsupported;
    }
    hipError_t er = hipEventRecord(e->ev_bucket[b], e->stream);
    if (er != hipSuccess) return er;
    er = hipStreamWaitEvent(e->comm_stream, e->ev_bucket[b], 0);
    if (er != hipSuccess) return er;
    bool ok = ncclGroupStart() == ncclSuccess;
    for (auto& r : e->bucket_ranges[b])
        ok = ok && ncclAllReduce(e->d_grads + r.first, e->d_grads + r.first, (size_t)r.second, ncclFloat, ncclSum,
                                 e->comm, e->comm_stream) == ncclSuccess;
    ok = (ncclGroupEnd() == ncclSuccess) && ok;
    if (!ok) return hipErrorUnknown;
    if (b == 1) {
        er = hipEventRecord(e->ev_comm_done, e->comm_stream);
        if (er != hipSuccess) return er;
        er = hipStreamWaitEvent(e->stream, e->ev_comm_done, 0);
        if (er != hipSuccess) return er;
    }
    return hipSuccess;
}

constexpr size_t AGREE_BYTES = 16 * sizeof(int64_t);  // d_flag: the agreement words

// every rank's capture outcome and graph key, min-reduced over the communicator (eager, outside
// any capture; the key's max as the min of its negation): *agreed = 1 only when every rank
// captured its step graph and every rank's key words are equal (graph_key.hpp) — a rank whose key
// diverged makes all ranks fall back to eager steps instead of pairing mismatched graphs
hipError_t comm_capture_agree(Engine* e, bool ok, const GraphKey& k, int* agreed) {
    if (!e->d_flag) {
        hipError_t er = hipMalloc(&e->d_flag, AGREE_BYTES);
        if (er != hipSuccess) return er;
    }
    int64_t w[6], v[13];
    key_words(k, w);
    v[0] = ok ? 1 : 0;
    for (int i = 0; i < 6; ++i) {
        v[1 + i] = w[i];
        v[7 + i] = -w[i];
    }
    int64_t* dw = reinterpret_cast<int64_t*>(e->d_flag);
    hipError_t er = hipMemcpyAsync(dw, v, sizeof(v), hipMemcpyHostToDevice, e->stream);
    if (er != hipSuccess) return er;
    if (ncclAllReduce(dw, dw, 13, ncclInt64, ncclMin, e->comm, e->stream) != ncclSuccess) return hipErrorUnknown;
    er = hipMemcpyAsync(v, dw, sizeof(v), hipMemcpyDeviceToHost, e->stream);
    if (er == hipSuccess) er = hipStreamSynchronize(e->stream);
    bool same = v[0] == 1;
    for (int i = 0; i < 6; ++i) same = same && v[1 + i] == -v[7 + i];
    *agreed = same ? 1 : 0;
    return er;
}

// Step graphs with a communicator hold RCCL calls, so every rank must capture (and agree, above) at
// the same steps.  The graph cache key is rank-invariant except for the batch-dependent buffers a
// step graph points at: the entry lists (d_ents) and, for a streamed dataset, the batch sets and
// DMA copy buffers, which grow when one rank's batch needs more room than it has seen (a rank
// with a heavier batch would re-capture — and run the agreement all-reduce — alone, while its
// peers replayed: mismatched collectives).  So before the first graph step after a
// dataset or communicator change, the ranks agree (ncclMax, eager) on the largest batch any of
// them can stage — Bpad rows of its largest dataset row, resampled duplicates included — and
// size those buffers for it once; stage_rows then never grows them and every rank's key changes
// only with the step's shape, which all ranks share.  (Every rank calls this at the same step:
// dataset and communicator calls are collective in data-parallel use.)
int comm_sync_capacity(Engine* e) {
    int64_t mx = 0;
    for (int32_t v : e->cell_nnz) mx = std::max<int64_t>(mx, v);
    // [0] the batch capacity, [1] MMVAE_NO_BALANCE on any rank (so the permutation rule, a graph
    // key field, is the same function of B on every rank)
    int64_t w[2] = {e->Bpad * mx, e->no_balance ? 1 : 0};
    if (!e->d_flag) HIPCHK(e, hipMalloc(&e->d_flag, AGREE_BYTES));
    int64_t* dw = reinterpret_cast<int64_t*>(e->d_flag);
    HIPCHK(e, hipMemcpyAsync(dw, w, sizeof(w), hipMemcpyHostToDevice, e->stream));
    if (ncclAllReduce(dw, dw, 2, ncclInt64, ncclMax, e->comm, e->stream) != ncclSuccess)
        FAIL(e, MMVAE_E_COMM, "comm_sync_capacity: ncclAllReduce failed");
    HIPCHK(e, hipMemcpyAsync(w, dw, sizeof(w), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const int64_t need = w[0];
    e->no_balance = w[1] != 0;
    if (e->gstream) HIPCHK(e, hipStreamSynchronize(e->gstream));
    // the worst-case buffers; an allocation that fails leaves the buffer empty (eager steps grow
    // it per batch again) and, once the ranks agree on it below, every rank runs its communicator
    // steps eagerly instead of failing
    bool ok = true;
    if (!e->wide && need + 64 > e->ent_cap) {
        if (e->d_ents) hipFree(e->d_ents);
        e->d_ents = nullptr;
        e->ent_cap = 0;
        if (hipMalloc(&e->d_ents, sizeof(uint2) * (need + 64)) == hipSuccess &&
            hipMemset(e->d_ents, 0, sizeof(uint2) * (need + 64)) == hipSuccess) {
            e->ent_cap = need + 64;
        } else {
            if (e->d_ents) hipFree(e->d_ents);
            e->d_ents = nullptr;
            ok = false;
        }
    }
    if (e->streamed) {
        for (int s = 0; s < 2 && ok; ++s) {
            if (e->bset[s].cap < need && batch_set_alloc(e, s, need) != hipSuccess) ok = false;
            if (ok && e->stream_dma && e->hs_packed && e->bpk_cap[s] < need && stream_bpk_alloc(e, s, need) != hipSuccess)
                ok = false;
        }
        stream_bind(e, e->cur_slot);
    }
    if (!ok) (void)hipGetLastError();
    {
        int64_t okw = ok ? 1 : 0;
        HIPCHK(e, hipMemcpyAsync(dw, &okw, sizeof(okw), hipMemcpyHostToDevice, e->stream));
        if (ncclAllReduce(dw, dw, 1, ncclInt64, ncclMin, e->comm, e->stream) != ncclSuccess)
            FAIL(e, MMVAE_E_COMM, "comm_sync_capacity: ncclAllReduce failed");
        HIPCHK(e, hipMemcpyAsync(&okw, dw, sizeof(okw), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        if (!okw) e->comm_graph_failed = true;  // on every rank: eager communicator steps from here
        if (getenv_is("MMVAE_VERBOSE", "1"))
            std::fprintf(stderr, "[mmvae] rank %d: agreed batch capacity %lld entries (%.1f MB of entry lists)%s\n",
                         e->rank, (long long)need, 8e-6 * (double)need,
                         okw ? "" : "; an allocation failed on some rank: eager communicator steps");
    }
    ++e->graph_gen;  // on every rank at the same step
    e->cap_synced = true;
    return MMVAE_OK;
}
}  // namespace mmvae
}  // extern "C++"

int mmvae_comm_allreduce(mmvae_h e, float* values, int64_t n) {
    if (!e || !values || n < 0) FAIL(e, MMVAE_E_ARG, "comm_allreduce: bad arguments");
    if (n == 0 || !e->comm_active()) return MMVAE_OK;
    HIPCHK(e, hipSetDevice(e->device));
    if (!e->d_tmp_ar || e->n_tmp_ar < n) {
        if (e->d_tmp_ar) hipFree(e->d_tmp_ar);
        e->d_tmp_ar = nullptr;
        HIPCHK(e, dalloc(&e->d_tmp_ar, n));
        e->n_tmp_ar = n;
    }
    HIPCHK(e, hipMemcpyAsync(e->d_tmp_ar, values, sizeof(float) * n, hipMemcpyHostToDevice, e->stream));
    if (ncclAllReduce(e->d_tmp_ar, e->d_tmp_ar, (size_t)n, ncclFloat, ncclSum, e->comm, e->stream) != ncclSuccess)
        FAIL(e, MMVAE_E_COMM, "ncclAllReduce failed");
    HIPCHK(e, hipMemcpyAsync(values, e->d_tmp_ar, sizeof(float) * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MMVAE_OK;
}

int mmvae_timing_enable(mmvae_h e, int32_t on) {
    if (!e) FAIL(e, MMVAE_E_ARG, "timing_enable: null");
    if (!on) timer_collect(e);
    e->timing = on != 0;
    return MMVAE_OK;
}

int mmvae_timing_count(mmvae_h e, int32_t* n) {
    if (!e || !n) FAIL(e, MMVAE_E_ARG, "timing_count: null");
    timer_collect(e);
    *n = (int32_t)e->timers.size();
    return MMVAE_OK;
}

int mmvae_timing_get(mmvae_h e, int32_t idx, const char** name, double* total_ms, int64_t* launches) {
    if (!e || idx < 0 || idx >= (int)e->timers.size()) FAIL(e, MMVAE_E_ARG, "timing_get: index out of range");
    if (name) *name = e->timers[idx].name.c_str();
    if (total_ms) *total_ms = e->timers[idx].total_ms;
    if (launches) *launches = e->timers[idx].launches;
    return MMVAE_OK;
}

int mmvae_debug_copy(mmvae_h e, int32_t which, float* host, int64_t n) {
    if (!e || !host || n < 0 || which < 0 || which > 4) FAIL(e, MMVAE_E_ARG, "debug_copy: bad arguments");
    // 0: encoder split partials (k_enc_fwd stamps), 1: decoder dz partials (k_dec_nb stamps),
    // 2: pass-C column slab (k_dec_lse / latent stamps), 3: the last step's latent noise eps
    //    [Bpad][K] (rows in the step's staged order), 4: the encoder-backward slab (its stamps)
    if (which == 3) {
        if (n > e->Bpad * e->K) FAIL(e, MMVAE_E_ARG, "debug_copy: n exceeds Bpad * K");
        HIPCHK(e, hipSetDevice(e->device));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        std::vector<float> lat((size_t)(e->Bpad * e->lat_stride));
        HIPCHK(e, hipMemcpy(lat.data(), e->d_lat, sizeof(float) * lat.size(), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < n; ++i) host[i] = lat[(size_t)((i / e->K) * e->lat_stride + e->LAT_EPS + i % e->K)];
        return MMVAE_OK;
    }
    const int64_t cap = which == 0   ? (int64_t)e->nsplit_e * e->Bpad * e->KP
                        : which == 1 ? (int64_t)e->nsplit_d * e->Bpad * 2 * e->KP
                        : which == 4 ? (int64_t)e->nrb_max * (2 + e->H) * e->DP
                                     : (int64_t)e->nrb_max * (1 + e->C) * e->DP;
    if (n > cap) FAIL(e, MMVAE_E_ARG, "debug_copy: n exceeds the workspace");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    const float* src = which == 0 ? e->d_hpart : which == 1 ? e->d_dzp : which == 4 ? e->d_slabE : e->d_slabC;
    HIPCHK(e, hipMemcpy(host, src, sizeof(float) * n, hipMemcpyDeviceToHost));
    return MMVAE_OK;
}

int mmvae_graph_enable(mmvae_h e, int32_t on) {
    if (!e) FAIL(e, MMVAE_E_ARG, "graph_enable: null");
    HIPCHK(e, hipSetDevice(e->device));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->graph_on = on != 0;
    if (!e->graph_on) graph_drop(e);
    return MMVAE_OK;
}

int mmvae_graph_stats(mmvae_h e, int64_t* captures, int64_t* replays) {
    if (!e || !captures || !replays) FAIL(e, MMVAE_E_ARG, "graph_stats: null");
    *captures = e->graph_captures;
    *replays = e->graph_replays;
    return MMVAE_OK;
}

int mmvae_tiling_info(mmvae_h e, int32_t* out) {
    if (!e || !out) FAIL(e, MMVAE_E_ARG, "tiling_info: null");
    out[0] = (int32_t)e->NT;
    out[1] = e->nsplit_e;
    out[2] = e->nsplit_d;
    out[3] = e->nsplit_a;
    out[4] = e->nsplit_b;
    return MMVAE_OK;
}

// Fill every per-step workspace buffer with `byte` (stream-ordered).  A step must write
// everything it reads from these buffers before reading it, so results may not depend on
// their contents: the tests poison between steps and demand bit-identical outputs.
// Persistent state (dataset + its index, parameters, gradients, Adam moments, frozen weights
// and their packed operand images, the hidden-chain pack, injected noise) is left alone.
int mmvae_debug_poison(mmvae_h e, int32_t byte) {
    if (!e) FAIL(e, MMVAE_E_ARG, "debug_poison: null");
    HIPCHK(e, hipSetDevice(e->device));
    if (e->gstream) HIPCHK(e, hipStreamSynchronize(e->gstream));  // no gather in flight into a set
    const int64_t Bp = e->Bpad, DP = e->DP, KP = e->KP, nrb = e->nrb_max;
    const int64_t SMALL = small_len((int)e->K, (int)e->E, (int)e->KE, (int)e->C,
                                    e->cfg.model == MMVAE_MODEL_VMF ? 0 : (int)(2 * e->R * e->H + 2 * e->R + e->H + 1));
    const struct {
        void* p;
        size_t bytes;
    } bufs[] = {
        {e->d_cells, e->stage_bytes},
        {e->d_ents, sizeof(uint2) * (size_t)e->ent_cap},
        {e->d_toff, sizeof(int32_t) * (size_t)((Bp / 16) * (e->NT + 1))},
        {e->d_gene, sizeof(float) * (size_t)(10 * DP)},
        {e->d_mvec, sizeof(float) * (size_t)(((DP + 255) / 256) * KP)},
        {e->d_rowx, sizeof(float) * (size_t)(Bp * (2 + e->H))},
        {e->d_rowxp, sizeof(float) * (size_t)(e->nsplit_e * Bp * (1 + e->H))},
        {e->d_hpart, sizeof(float) * (size_t)(e->nsplit_e * Bp * KP)},
        {e->d_lat, sizeof(float) * (size_t)(Bp * e->lat_stride)},
        {e->d_zf, sizeof(float) * (size_t)(Bp * KP)},
        {e->d_zb, sizeof(__bf16) * (size_t)(2 * Bp * KP)},
        {e->d_lsep, sizeof(float) * (size_t)(e->nsplit_a * Bp * 2)},
        {e->d_rowB, sizeof(float) * (size_t)(std::max(e->nsplit_d, e->nsplit_f) * Bp * (2 + e->R))},
        {e->d_rowfin, sizeof(float) * (size_t)(Bp * 2)},
        {e->d_dzp, sizeof(float) * (size_t)(e->nsplit_d * Bp * 2 * KP)},
        {e->d_dh, sizeof(float) * (size_t)(Bp * KP)},
        {e->d_dhT_f, sizeof(float) * (size_t)(Bp * KP)},
        {e->d_dhT_b, sizeof(__bf16) * (size_t)(2 * Bp * KP)},
        {e->d_WeS_f, sizeof(float) * (size_t)(KP * DP)},
        {e->d_WeS_b, sizeof(__bf16) * (size_t)(2 * KP * DP)},
        {e->d_slabB, sizeof(float) * (size_t)(nrb * ((1 + e->C) + 1 + e->R) * DP)},
        {e->d_slabC, sizeof(float) * (size_t)(nrb * (1 + e->C) * DP)},
        {e->d_slabE, sizeof(float) * (size_t)(nrb * (2 + e->H) * DP)},
        {e->d_lossp, sizeof(float) * (size_t)(e->klp_off + e->n_lat_wg)},
        {e->d_small, sizeof(float) * (size_t)(e->n_lat_wg * SMALL)},
        {e->d_smallg, sizeof(float) * 128},
        {e->d_sumsq, sizeof(double) * (size_t)(256 + (e->D + 31) / 32 + (SMALL + 2 * e->K + 31) / 32 + 1)},
        {e->d_rowv, sizeof(float) * (size_t)Bp},
        {e->d_vk, sizeof(float) * 8},
        {e->d_WeS8, (size_t)(KP * DP)},
        {e->d_escale, sizeof(float) * 2},
    };
    for (const auto& b : bufs)
        if (b.p && b.bytes) HIPCHK(e, hipMemsetAsync(b.p, byte & 0xff, b.bytes, e->stream));
    if (e->streamed)  // the batch CSR sets are rewritten by every step's gather and index
        for (const auto& q : e->bset) {
            const size_t rows = (size_t)(Bp + 1);
            const struct {
                void* p;
                size_t bytes;
            } sb[] = {{q.rowptr, sizeof(int64_t) * (rows + 1)}, {q.col, sizeof(int32_t) * (size_t)q.cap},
                      {q.val, sizeof(float) * (size_t)q.cap}, {q.covar, sizeof(float) * rows * (size_t)e->C},
                      {q.rtp, sizeof(int32_t) * rows * (size_t)(e->NT + 1)}, {q.cellnorm, sizeof(float) * 2 * rows}};
            for (const auto& b : sb)
                if (b.p && b.bytes) HIPCHK(e, hipMemsetAsync(b.p, byte & 0xff, b.bytes, e->stream));
        }
    for (const auto& b : wide_poison_bufs(e))
        if (b.first && b.second) HIPCHK(e, hipMemsetAsync(b.first, byte & 0xff, b.second, e->stream));
    // and the LDS of every CU: a kernel reading LDS it did not write this launch (a tile row or
    // a correction plane left over from another workgroup) then sees the pattern
    HIPCHK(e, lds_poison(e, byte));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return MMVAE_OK;
}

int mmvae_timing_reset(mmvae_h e) {
    if (!e) FAIL(e, MMVAE_E_ARG, "timing_reset: null");
    timer_collect(e);
    for (auto& t : e->timers) {
        t.total_ms = 0;
        t.launches = 0;
    }
    return MMVAE_OK;
}

// ---- operators.hh scalars (host, fp32): include/mmvae/lbessel.hh ---------------------------
float mmvae_fasterlog(float x) { return mmvae_math::fasterlog(x); }
float mmvae_fasterlgamma(float x) { return mmvae_math::fasterlgamma(x); }
float mmvae_lbessel(float kappa, float nu) { return mmvae_math::lbessel(kappa, nu); }
float mmvae_lbessel_grad(float kappa, float nu) { return mmvae_math::lbessel_grad(kappa, nu); }

}  // extern "C"
