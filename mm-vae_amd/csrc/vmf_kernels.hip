// vMF-VAE ELBO step on gfx950: hand-written HIP kernels for the reference's second model
//   forward  vmf.hh:250-304      (encode: normalised log1p + Angular encoder; Gaussian latent;
//                                 decode: exp(z_dec(z)) + covar_dec(c), L2-normalised)
//            angular.hh:34-42    (W~ = normalize(relu(W) + 1e-4), frozen: precomputed once)
//   loss     vmf.hh:410-440      (kappa <y, r> + df log kappa - lbessel(kappa, df) - D/2 log 2pi)
//            operators.hh:13-101 (lbessel forward; backward = Baricz bound, ignores upstream, Q3)
//   backward hand-derived; the algebra is restated in oracle/vmf_analytic.py and proven equal
//            to LibTorch autograd there.
//
// Kernel chain per step (one stream), sharing the CSR tile machinery of tiles.hpp and the
// encoder GEMM kernels of nb_kernels.hip (enc_forward_launch / enc_backward_launch):
//   k_vprep        per-gene 1/(softplus(ln_x_sd)+eps), decoder gene records, W~/s, and the
//                  per-block partials of the dense encoder term mvec = (x_mean/s) W~^T
//   k_enc_fwd      sum_nnz l (W~/s)  on MFMA                    (shared with NB)
//   k_vlatent_fwd  h = that / ||l|| - mvec, heads, clamp, reparameterise, KL
//   (k_vprep's last block: kappa = clamp(exp(ln_kappa)), lbessel terms, one thread)
//   k_vdec<0>      logits on MFMA, u = exp, v = u + hc: row sums |v|^2, sum v, sum l v
//   k_vdec<1>      per-row cos_b, alpha_b, beta_b from the pass-0 split sums (vrow_coeffs);
//                  dv = alpha (l + eps) + beta v, da = dv u: column sums + dz GEMM on MFMA
//   (k_vrowfin     the same row coefficients, eval path only)
//   k_vlatent_bwd  heads backward, KL grads, dh (scaled by 1/||l|| for the encoder)
//   k_enc_bwd      sum_k W~ (dh/||l||)^T log1p(x)                (shared with NB)
//   k_vgrad_small / k_vgrad_genes   fixed-order reductions into the flat gradient
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"
#include "enc_bwd.hpp"

namespace mmvae {

struct VPtrs {
    const float *xm, *lsd, *lk, *Wce, *bce, *Wm, *bm, *Wl, *bl, *Wcd, *bcd;
    const float *We, *Wd, *bd;  // frozen (reference layouts: Angular W [Z][D], z_dec W [D][Z], b [D])
};

struct VGrads {
    float *xm, *lsd, *lk, *Wce, *bce, *Wm, *bm, *Wl, *bl, *Wcd, *bcd;
};

// Model scalars fixed by D (vmf.hh:252,421,427,435; operators.hh:75-76)
struct VScal {
    float epsD;    // 1e-2 / D
    float df;      // max(D/2 - 1, 0)
    float kmin, kmax;
    float lg_df1;  // fasterlgamma(df + 1)
    float c2;      // 0.5 D fasterlog(2 pi)
    int rank0;     // this rank adds the lbessel backward term (once per global batch)
};

// d_vk: kappa scalars written by the last block of k_vprep (vkappa_body)
enum { VK_KAPPA = 0, VK_EXP = 1, VK_MASK = 2, VK_T = 3, VK_BARICZ = 4 };

// =======================================================================================
// Frozen operand preparation (once per set_param of a frozen tensor)
//   W~ = normalize(relu(W) + 1e-4, dim 1)  (angular.hh:37-39)  -> packed [KP][DP] f32 / bf16
//   z_dec weight -> [DP][KP] (logit GEMM B operand) and [KP][DP] (dz GEMM B operand)
// =======================================================================================
__global__ __launch_bounds__(1024) void k_vnorm_enc(const float* __restrict__ W, int D, int DP, int K,
                                                    float* __restrict__ WeP_f, __bf16* __restrict__ WeP_b) {
    __shared__ float sb[16];
    const int k = blockIdx.x;
    float ss = 0.f;
    if (k < K)
        for (int g = threadIdx.x; g < D; g += 1024) {
            const float r = fmaxf(W[(int64_t)k * D + g], 0.f) + 1e-4f;
            ss = fmaf(r, r, ss);
        }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = ss;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += sb[q];
    const float nrm = fmaxf(sqrtf(t), 1e-12f);  // F::normalize: x / max(||x||, eps)
    for (int g = threadIdx.x; g < DP; g += 1024) {
        float v = 0.f;
        if (k < K && g < D) v = (fmaxf(W[(int64_t)k * D + g], 0.f) + 1e-4f) / nrm;
        WeP_f[(int64_t)k * DP + g] = v;
        put_op<X3>(WeP_b, k * DP + g, (int)gridDim.x * DP, v);  // lo plane KP * DP after the hi plane
    }
}

__global__ void k_vpack_dec(const float* Wd, int D, int DP, int KD, int KP, float* WdP_f, __bf16* WdP_b, float* WdT_f,
                            __bf16* WdT_b) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)KP * DP) return;
    const int k = (int)(i / DP), g = (int)(i % DP);
    const float wd = (k < KD && g < D) ? Wd[(int64_t)g * KD + k] : 0.f;  // [D][KD]
    const int pl = KP * DP;  // the x3 mode's lo planes
    WdT_f[i] = wd;
    put_op<X3>(WdT_b, (int)i, pl, wd);
    WdP_f[(int64_t)g * KP + k] = wd;
    put_op<X3>(WdP_b, g * KP + k, pl, wd);
}

// =======================================================================================
// k_vprep — per-gene constants of the step:
//   inv_g = 1 / (softplus(ln_x_sd_g) + eps)       (vmf.hh:255-256)
//   xmi_g = x_mean_g inv_g                         (dense part of the encoder input)
//   grec_g = (b_dec_g log2(e), b_cd_g, W_cd[g][0], epsD)  (vmf.hh:285-287); a padded gene holds
//            (-inf, 0, 0, 0), so its u = exp2(-inf), hc and dv are exact zeros with no mask
//   WeS[k][g] = inv_g W~[k][g]                     (encoder B operand, bf16 or f32)
// =======================================================================================
MMVAE_DEV void vkappa_body(const VPtrs& P, const VScal& s, float* __restrict__ vk);
// the last x-block (y = 0) computes the kappa scalars (vkappa_body, vmf.hh:301 + lbessel) — they
// depend only on ln_kappa, so they ride in this launch instead of a kernel of their own
__global__ __launch_bounds__(256) void k_vprep(VPtrs P, Dims d, float epsD, float* __restrict__ gene,
                                               const float* __restrict__ WeP_f, float* __restrict__ WeS_f,
                                               __bf16* __restrict__ WeS_b, float* __restrict__ mvecp, VScal sc,
                                               float* __restrict__ vk, StageCopy scp) {
    // every load before the first store (see k_prep, nb_kernels.hip), the staged block's
    // host-memory chunk last
    StageHold sh;
    if (blockIdx.x == gridDim.x - 1) {
        sh.load(scp);
        if (blockIdx.y == 0) vkappa_body(P, sc, vk);
        sh.store(scp);
        return;
    }
    const int g0 = blockIdx.x * 256 + threadIdx.x;
    const bool in = g0 < d.DP;
    const int g = in ? g0 : d.DP - 1;
    const bool v = in && g < d.D;
    const int gl = min(g, d.D - 1);
    const float lsd = P.lsd[gl];
    float wp[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wp[kk] = WeP_f[(int64_t)(blockIdx.y * 8 + kk) * d.DP + g];
    const float xm = P.xm[gl], bd = P.bd[gl], bcd = P.bcd[gl], wcd = P.Wcd[(int64_t)gl * d.C];
    __builtin_amdgcn_sched_barrier(0);  // the host-memory load stays behind the others
    sh.load(scp);
    __builtin_amdgcn_sched_barrier(0);
    const float inv = v ? 1.f / (softplus_acc(lsd) + epsD) : 0.f;
    if (blockIdx.y == 0 && in) {
        gene[g] = inv;
        gene[3 * d.DP + g] = v ? xm * inv : 0.f;
        reinterpret_cast<float4*>(gene + 4 * d.DP)[g] =
            float4{v ? bd * 1.4426950408889634f : -INFINITY, v ? bcd : 0.f, v ? wcd : 0.f, v ? epsD : 0.f};
    }
    const float xmv = v ? xm : 0.f;
    float mp[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const int k = blockIdx.y * 8 + kk;
        const float ws = inv * wp[kk];
        if (in) {  // bf16 image: hi plane, and the x3 mode's lo plane KP * DP elements after it
            if (WeS_b) put_op<X3>(WeS_b, (int)((int64_t)k * d.DP + g), d.KP * d.DP, ws);
            else WeS_f[(int64_t)k * d.DP + g] = ws;
        }
        mp[kk] = xmv * ws;  // xmi_g W~[k][g]
    }
    mvec_partial(mp, mvecp, d.KP, blockIdx.y * 8);  // summed by k_vlatent_fwd
    sh.store(scp);
}

// =======================================================================================
// k_vlatent_fwd — encoder head + Gaussian reparameterisation for 64 cells per workgroup
// (wave w owns cells 4w..4w+3, lane = latent k):
//   h = (sum_nnz l W~/s) / ||l|| - mvec              (vmf.hh:253-258, Angular has no bias)
//   mean = repr_mean(h) + covar_enc(c), lnvar = clamp(repr_lnvar(h), -4, 4)   (vmf.hh:259-264)
//   z = mean + eps exp(lnvar/2)                       (vmf.hh:394-404), KL (vmf.hh:410-414)
//   mode 1 = recorder encode(x) (vmf.hh:267-281): no covariate, writes mean/lnvar out.
// Per-row state kept for the backward: h, mean, pre-clamp a, eps, 1/||l|| (LAT_D), valid.
// =======================================================================================
// NW = 16 (one cell per wave, 1024 threads; no frozen chains): see k_latent_fwd (nb_kernels.hip).
// Every global load is issued before the first global store.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_vlatent_fwd(
    VPtrs P, Dims d, const int64_t* __restrict__ cells, const float* __restrict__ covar,
    const float* __restrict__ hpart, const float* __restrict__ mvec, const float2* __restrict__ cellnorm,
    float* __restrict__ rowx, const float* __restrict__ eps_in, const int32_t* __restrict__ perm, uint64_t seed,
    const StepScalars* __restrict__ ss,
    float* __restrict__ lat, float* __restrict__ zf, __bf16* __restrict__ zb,
    float* __restrict__ klpart, int mode, float* __restrict__ out_mean, float* __restrict__ out_lnvar) {
    constexpr int CPW = LAT_CELLS / NW;  // cells per wave
    constexpr bool CHAINS = NW == 4;     // the frozen chains' layers run on 256 threads
    const int K = d.K, KE = d.KE, E = d.E;
    const uint64_t step = (uint64_t)ss->step_id;  // the noise key (staged with the batch)
    const int64_t row_offset = ss->row_offset;
    __shared__ float sWm[64 * 65], sWl[64 * 65];
    __shared__ __attribute__((aligned(16))) float sH[LAT_CELLS * 68];
    __shared__ float sred[NW];
    HeadsStage<64 * NW> hst;
    hst.issue(P.Wm, P.Wl, K, E);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = lane;
    const int cw = CPW * w;                     // this wave's first cell in the workgroup
    const int bw = blockIdx.x * LAT_CELLS + cw;  // ... in the batch
    float hs[CPW];
    split_sum<CPW>(hpart, d.nsE, (int64_t)d.Bpad * d.KP, (int64_t)bw * d.KP + k, d.KP, k < KE, hs);
    // per-lane parameters and per-cell inputs (clamped, unconditional loads where possible)
    const int kk = min(k, K - 1);
    const float p_bm = P.bm[kk], p_bl = P.bl[kk], p_bce = P.bce[kk], p_wce = P.Wce[(int64_t)kk * d.C];
    float2 cn[CPW];
    int pbv[CPW];
    float epv[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        cn[c] = cellnorm[cells[b]];  // row norms from the dataset index (row Ncells = the empty padding row)
        pbv[c] = (perm && b < d.B) ? perm[b] : b;  // original batch position: the noise key
        epv[c] = (eps_in && k < K && b < d.B) ? eps_in[(int64_t)pbv[c] * K + k] : 0.f;
    }
    const float mvk = mvec_sum(mvec, d.nmv, d.KP, k);  // all threads (LDS combine)
    if (!CHAINS || d.nce == 0) hst.store(K, E, sWm, sWl);  // (with an encoder chain: after it, sWm stages its W)
    const float mk = (k < KE) ? mvk : 0.f;
    float inx[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        if (b >= d.B) hs[c] = 0.f;  // past this batch: partials unwritten this step (NB k_latent_fwd)
        inx[c] = 1.f / fmaxf(sqrtf(cn[c].x), 1e-12f);  // F::normalize
        if (mode == 0 && k == 0) {
            rowx[(int64_t)b * d.rowx_stride] = cn[c].x;
            rowx[(int64_t)b * d.rowx_stride + 1] = cn[c].y;
        }
        const float hv = hs[c] * inx[c] - mk;  // Angular output; --relu appends ReLU (vmf.hh:351-352)
        sH[(cw + c) * 68 + k] = (k < KE) ? (d.relu ? fmaxf(hv, 0.f) : hv) : 0.f;
    }
    __syncthreads();
    // the frozen Angular chain (encoding_l, l >= 2, + ReLU with --relu: vmf.hh:338-347)
    __shared__ float sZ[CHAINS ? 2 : 1][LAT_CELLS * 68];
    const float* hin = sH;
    if constexpr (CHAINS) {
        if (d.nce > 0) {
            hin = chain_run(d, 0, d.nce, sH, sZ[0], sZ[CHAINS ? 1 : 0], false, sWm, w, lane);
            hst.store(K, E, sWm, sWl);
            __syncthreads();
        }
    }
    // heads on f32 MFMA (vmf.hh:259-264), transposed back to lane = latent through LDS
    __shared__ float sM[LAT_CELLS * 68], sA[LAT_CELLS * 68];
    if (w < 4) heads_fwd(hin, sWm, sWl, K, E, w, lane, sM, sA);
    __syncthreads();
    float mean[CPW], av[CPW];
    const float bm = (k < K) ? p_bm : 0.f, bl = (k < K) ? p_bl : 0.f;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        mean[c] = bm + sM[(cw + c) * 68 + k];
        av[c] = bl + sA[(cw + c) * 68 + k];
    }
    float kl = 0.f;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        const bool valid = b < d.B;
        float* L = lat + (int64_t)b * d.lat_stride;
        float mn = mean[c];
        const float a = av[c];
        if (k < K && mode == 0) {
            float cm = p_bce;
            if (!covar) {  // unit covariate (Engine::unit_covar): c = 1, padding rows (row N) 0
                cm += valid ? p_wce : 0.f;
            } else {
                const int64_t cell = cells[b];  // padding rows hold the empty row N
                for (int q = 0; q < d.C; ++q) cm += P.Wce[k * d.C + q] * covar[cell * d.C + q];
            }
            mn += cm;
        }
        const float lnvar = fminf(fmaxf(a, -4.f), 4.f);
        if (mode == 1) {
            if (k < K && b < d.B) {
                out_mean[(int64_t)b * K + k] = mn;
                out_lnvar[(int64_t)b * K + k] = lnvar;
            }
            continue;
        }
        const float sig = expf(lnvar / 2.f);
        float eps = 0.f;
        const int pb = pbv[c];
        if (k < K && b < d.B) eps = eps_in ? epv[c] : philox_normal(seed, step, row_offset + pb, k);
        const float z = mn + eps * sig;
        if (k < KE) L[d.LAT_H + k] = sH[(cw + c) * 68 + k];
        if (k < K) {
            L[d.LAT_MEAN + k] = mn;
            L[d.LAT_A + k] = a;
            L[d.LAT_EPS + k] = eps;
            if (valid) kl += 1.f + lnvar - mn * mn - expf(lnvar);
        }
        if (CHAINS && d.ncd > 0) {
            sZ[0][(cw + c) * 68 + k] = (k < K) ? z : 0.f;  // the decoder chain's input (below)
        } else if (k < d.KP && b < d.Bpad) {  // rows past this batch's padded size: none
            const float zz = (k < K && valid) ? z : 0.f;
            zf[(int64_t)b * d.KP + k] = zz;
            put_op<X3>(zb, b * d.KP + k, d.Bpad * d.KP, zz);  // hi plane (+ the x3 lo plane)
        }
        if (k == 0) {
            L[d.LAT_D] = inx[c];
            L[d.LAT_VALID] = valid ? 1.f : 0.f;
        }
    }
    if (mode == 1) return;
    if constexpr (CHAINS) {
        if (d.ncd > 0) {
            // the frozen decoder chain (decoding_l + ReLU with --relu, vmf.hh:374-381): z -> zd
            __syncthreads();
            // ping-pong sZ[1] / sM (free: the means were read before the cell loop)
            const float* zd = chain_run(d, d.nce, d.nce + d.ncd, sZ[0], sZ[CHAINS ? 1 : 0], sM, false, sWm, w, lane);
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                const int b = bw + c;
                if (k < d.KP && b < d.Bpad) {
                    const float zz = (k < d.KD && b < d.B) ? zd[(cw + c) * 68 + k] : 0.f;
                    zf[(int64_t)b * d.KP + k] = zz;
                    put_op<X3>(zb, b * d.KP + k, d.Bpad * d.KP, zz);
                }
            }
        }
    }
    kl = wave_sum(kl);
    if (lane == 0) sred[w] = kl;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = (sred[0] + sred[1]) + (sred[2] + sred[3]);
#pragma unroll
        for (int i = 4; i < NW; i += 4) t += (sred[i] + sred[i + 1]) + (sred[i + 2] + sred[i + 3]);
        klpart[blockIdx.x] = -0.5f * t;
    }
}

// =======================================================================================
// vkappa_body — kappa = clamp(exp(ln_kappa), kappa_min, kappa_max) (vmf.hh:301) and the scalar
// loss terms T = df log kappa - lbessel(kappa, df) (vmf.hh:433, operators.hh:65-81) in the
// reference's fp32 operation order; the lbessel backward (Baricz bound, operators.hh:34-37).
// exp/log are evaluated in double and rounded once (correctly rounded fp32), so the clamp
// mask agrees with ATen's at the initial ln_kappa = log(kappa_min) (Q4).
// =======================================================================================
MMVAE_DEV void vkappa_body(const VPtrs& P, const VScal& s, float* __restrict__ vk) {
    if (threadIdx.x != 0) return;
    const float lk = P.lk[0];
    const float e = (float)exp((double)lk);
    const float kap = fminf(fmaxf(e, s.kmin), s.kmax);
    const float lkap = (float)log((double)kap);
    const double nu = s.df;
    const float eta = (float)((nu + 0.5) / (2. * (nu + 1.)));
    float s1 = s.df * lkap;
    s1 = s1 + eta * kap;
    s1 = s1 - (float)(((double)eta + nu) * log(2.));
    s1 = s1 - s.lg_df1;
    float s2 = kap - 0.5f * lkap;
    s2 = s2 - (float)(0.5 * log(2. * M_PI));
    const float lb = (kap <= s.df) ? s1 : s2;
    const float T = s.df * lkap - lb;
    const float x2 = kap * kap;
    const float lo = sqrtf(x2 * s.df / (s.df + 1.f) + s.df * s.df);
    const float up = sqrtf(x2 + s.df * s.df);
    vk[VK_KAPPA] = kap;
    vk[VK_EXP] = e;
    vk[VK_MASK] = (e >= s.kmin && e <= s.kmax) ? 1.f : 0.f;  // clamp backward mask (inclusive)
    vk[VK_T] = T;
    vk[VK_BARICZ] = 0.5f * (lo + up) / kap;
}

// =======================================================================================
// Decoder passes (vmf.hh:283-289, 419-440).  The [B, D] reconstruction is never stored:
//   k_vdec<0>: u = exp(z W_d^T + b_d), v = u + hc       -> per row |v|^2, sum v, sum_nnz l v
//   k_vdec<1>: dv = alpha_b (l + eps) + beta_b v, da = dv u
//              -> column sums of dv, dv c (covar_decoding_ grads) and dz = da W_d on MFMA
// Workgroup = 64 cells (4 waves x 16) x one gene split.  Per 64-gene tile the decoder rows
// (and in pass 1 the [KP][64] transposed tile) are register-staged once per workgroup into
// LDS; each wave densifies its 16 cells' log1p(x) into a wave-private 16x64 tile from the
// CSR (entries prefetched a tile ahead).  Lane l holds gene (l & 15) of cells 4(l>>4)+r.
// =======================================================================================
struct VDecPtrs {
    const float* lat;
    const float* zf;
    const __bf16* zb;
    const float* gene;
    const float* Wcd;
    const float* covar;
    const int64_t* cells;
    EntList ents;          // batch entry lists (k_batch_lists)
    const int64_t* seg;
    const int32_t* toff;
    const void* WdP;       // [DP][KP] T
    const void* WdT;       // [KP][DP] T
    const float* rowfin;   // [Bpad][2]: alpha, beta (eval path: k_vrowfin)
    float* rowB;           // [nsF][Bpad][3]: |v|^2, sum v, sum l v (forward pass splits)
    const float* rowx;     // [Bpad][..]: [1] = sum (l^2 + 2 eps l)
    const float* vk;       // kappa scalars (vkappa_body in k_vprep)
    float* rowcos;         // [Bpad] cos_b (written by split 0 of the backward pass)
    float* dzp;            // [nsD][Bpad][KP]
    float* slabB;          // [nrb][1+C][DP]
    int64_t zplane;        // x3 mode: element offset of the lo plane of zb
    int64_t wplane;        // x3 mode: element offset of the lo planes of WdP / WdT
};

// Per-row combine of pass 0's split sums (threads p0, p0 + np, ... of a row's np-thread group,
// combined with xor-shuffles over the group) -> alpha_b, beta_b, cos_b (vmf.hh:422-432):
//   alpha_b = -(kappa/n) / (nv ny),  beta_b = (kappa/n) cos_b / nv^2
// (below the normalize eps, r = v / eps and the clamp passes no gradient: beta = 0).
MMVAE_DEV void vrow_coeffs(const Dims& d, float epsD, const float* __restrict__ lat, const float* __restrict__ rowx,
                           const float* __restrict__ rowB, const float* __restrict__ vk, int b, int p0, int np,
                           float& al, float& be, float& cosb) {
    float Svv = 0.f, Sv = 0.f, Slv = 0.f;
    for (int s = p0; s < d.nsF; s += np) {  // the forward pass's splits
        const float* rp = rowB + ((int64_t)s * d.Bpad + b) * 3;
        Svv += rp[0];
        Sv += rp[1];
        Slv += rp[2];
    }
    for (int o = 1; o < np; o <<= 1) {
        Svv += __shfl_xor(Svv, o, 64);
        Sv += __shfl_xor(Sv, o, 64);
        Slv += __shfl_xor(Slv, o, 64);
    }
    const bool valid = lat[(int64_t)b * d.lat_stride + d.LAT_VALID] > 0.f;
    const float nvr = sqrtf(Svv);
    const float nv = fmaxf(nvr, 1e-12f);
    const float ny = fmaxf(sqrtf(rowx[(int64_t)b * d.rowx_stride + 1] + (float)d.D * epsD * epsD), 1e-12f);
    cosb = (Slv + epsD * Sv) / (ny * nv);
    const float kn = vk[VK_KAPPA] * d.inv_n;
    al = -kn / (nv * ny);
    be = kn * cosb / (nv * nv);
    if (!(nvr >= 1e-12f)) {
        al = -kn / (1e-12f * ny);
        be = 0.f;
    }
    if (!valid) {
        al = 0.f;
        be = 0.f;
        cosb = 0.f;
    }
}

// trw (16-bit operands): pass 1 reads the dz GEMM's B operand transposed from the W image, so
// no WdT image is staged (x3 at K <= 32: 3 workgroups per CU instead of 2)
#ifndef MMVAE_VDEC_SLOAD_LATE
#define MMVAE_VDEC_SLOAD_LATE 0
#endif
#ifndef MMVAE_VDEC_LPIPE
#define MMVAE_VDEC_LPIPE 1  // 0: each gene block's logits right before its element math (A/B)
#endif
#ifndef MMVAE_VDEC_DZ_LATE
#define MMVAE_VDEC_DZ_LATE 1  // 0: dz k-steps interleaved with the gene blocks (A/B: 90.6 vs 88.9 us x3)
#endif
static constexpr int VTAB = 512;  // log1p table entries of the fp32-accurate modes (x3, f32)
struct VDecLds {
    int o_g, o_t, o_part, o_wave, o_q1, o_toff, wave_bytes, o_tab, bytes;
    // nbuf: W stage buffers (the forward pass double-buffers: one barrier per tile)
    MMVAE_HOSTDEV VDecLds(int KP, int esz, int S, int nq, int pass, int planes = 1, int nbuf = 1) {
        const bool trw = esz == 2;
        o_g = nbuf * planes * 64 * KP * esz;                  // W images (hi [+ lo]) per buffer
        o_t = o_g + nbuf * 1024;                              // gene records per buffer
        o_part = o_t + (pass && !trw ? planes * KP * 64 * esz : 0);
        o_wave = o_part + (pass ? 4 * nq * 64 * 4 : 0);
        const int QS = 64 + (esz == 2 ? 8 : 4);
        o_q1 = 16 * 68 * 4;                                   // after the l tile
        o_toff = o_q1 + (pass ? ((planes * 16 * QS * esz + 15) / 16) * 16 : 0);
        wave_bytes = o_toff + ((S * 4 + 15) / 16) * 16;  // the wave block's tile offsets
        o_tab = o_wave + 4 * wave_bytes;
        bytes = o_tab + ((esz == 2 && planes == 1) ? 0 : VTAB * 4);  // the bf16 mode: one v_log, no table
    }
};

template <class P, int KP, int PASS, int CM>
MMVAE_DEV void vdec_body(VDecPtrs Q, Dims d, float epsD) {
    using T = typename Elem<P>::type;
    using M = MM<P>;
    using Fr = typename M::frag;
    constexpr bool X = IsX3<P>::value;
    constexpr int NPL = X ? 2 : 1;
    constexpr int KS = KP / M::KSTEP;
    constexpr int GK = 64 / M::KSTEP;
    constexpr bool BF = sizeof(T) == 2;
    constexpr int QS = 64 + (BF ? 8 : 4);
    constexpr int LS = 68;
    constexpr int RBW = KP * (int)sizeof(T);
    constexpr int RBT = 64 * (int)sizeof(T);
    constexpr bool TRW = BF;  // dz B operand read transposed from the W image (VDecLds)
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nsp = PASS ? d.nsD : d.nsF, tps = PASS ? d.tpsD : d.tpsF;  // the forward pass: own split
    int sp, rb;
    xcd_split_major((int)blockIdx.x, (int)gridDim.x / nsp, nsp, sp, rb);
    const int row0 = rb * 64 + 16 * w;
    const int t0 = sp * tps, t1 = min(d.NT, t0 + tps);
    const int S = tps + 1;
    // CM = 0: unit covariate (Engine::unit_covar, C = 1): covar_dec folds into a per-gene
    // constant, and the covariate gradient's column sums are the bias gradient's
    constexpr int CA = CM > 0 ? CM : 1;  // covariate array extent
    const int C = (CM <= 1) ? 1 : d.C;
    const int nq = 1 + C;
    // the forward pass double-buffers its W stage (~9 KB more LDS, still 4 workgroups per CU)
    // and meets one barrier per tile; the backward keeps one buffer (3 workgroups per CU)
    constexpr int NBF = PASS ? 1 : 2;
    const VDecLds L(KP, (int)sizeof(T), S, nq, PASS, NPL, NBF);
    constexpr int WIMG = 64 * KP * (int)sizeof(T);  // one plane of the W / WdT images
    constexpr int QPL = 16 * QS;                     // the pq tile's lo plane (x3)
    auto wbuf = [&](int b) { return smem + b * NPL * WIMG; };
    auto gbuf = [&](int b) { return reinterpret_cast<float4*>(smem + L.o_g + b * 1024); };
    char* tst = smem + L.o_t;
    float* part = reinterpret_cast<float*>(smem + L.o_part);
    char* wp = smem + L.o_wave + w * L.wave_bytes;
    float* lt = reinterpret_cast<float*>(wp);
    T* q1 = reinterpret_cast<T*>(wp + L.o_q1);
    int32_t* toffl = reinterpret_cast<int32_t*>(wp + L.o_toff);
    const T* Z = BF ? reinterpret_cast<const T*>(Q.zb) : reinterpret_cast<const T*>(Q.zf);
    const char* WdPc = reinterpret_cast<const char*>(Q.WdP);
    const char* WdTc = reinterpret_cast<const char*>(Q.WdT);
    const float4* grec = reinterpret_cast<const float4*>(Q.gene + 4 * d.DP);
    // log1p of integer counts from a per-workgroup LDS table in the fp32-accurate modes (the
    // libm log1pf per entry otherwise dominates the tile); the bf16 mode keeps one v_log
    using VTabT = Log1pTab<typename std::conditional<BF && !X, __bf16, float>::type, VTAB>;
    uint32_t* ltab = reinterpret_cast<uint32_t*>(smem + L.o_tab);
    VTabT::fill(ltab);  // published by the first barrier below

    DualStage<64, RBW, 256, X> wreg;
    DualStage<KP, RBT, 256, X> treg;
    float4 greg = float4{0.f, 0.f, 0.f, 0.f};
    const int64_t wplb = Q.wplane * (int64_t)sizeof(T);
    auto stage_load = [&](int t) {
        wreg.load(WdPc + (int64_t)64 * t * RBW, RBW, wplb);
        if (PASS && !TRW) treg.load(WdTc + (int64_t)64 * t * sizeof(T), (int64_t)d.DP * sizeof(T), wplb);
        if (threadIdx.x < 64) greg = grec[64 * t + threadIdx.x];
    };
    auto stage_store = [&](int b) {
        wreg.store(wbuf(b), WIMG);
        if (PASS && !TRW) treg.store(tst, WIMG);
        if (threadIdx.x < 64) gbuf(b)[threadIdx.x] = greg;
    };
    stage_load(min(t0, d.NT - 1));  // independent of everything below: issued first
    if (PASS) {  // the per-row backward coefficients from pass 0's split sums (k_vrowfin), 4 threads per row
        const int rr = threadIdx.x >> 2, pp = threadIdx.x & 3;
        const int b = rb * 64 + rr;
        float al, be, cosb;
        vrow_coeffs(d, epsD, Q.lat, Q.rowx, Q.rowB, Q.vk, b, pp, 4, al, be, cosb);
        if (pp == 0) {
            part[2 * rr] = al;
            part[2 * rr + 1] = be;
            if (sp == 0) Q.rowcos[b] = cosb;
        }
        __syncthreads();
    }
    Fr zfr[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
        zfr[s] = M::load(&Z[(int64_t)(row0 + (lane & 15)) * KP + s * M::KSTEP + (lane >> 4) * M::EPL], Q.zplane);
    // rows 4 (lane >> 4) + 2h + j live in component j of the pair h (packed-f32 element math)
    f2 crow2[2][CA], ra2[2], rbt2[2], svv2[2], sv2[2], slv2[2];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int h = r >> 1, j = r & 1;
        const int b = row0 + 4 * (lane >> 4) + r;
        const int64_t cell = Q.cells[b];  // padding rows hold the empty row N
#pragma unroll
        for (int c = 0; c < CM; ++c) crow2[h][c][j] = (c < C) ? Q.covar[cell * C + c] : 0.f;  // row N: zeros
        ra2[h][j] = PASS ? part[2 * (16 * w + 4 * (lane >> 4) + r)] : 0.f;
        rbt2[h][j] = PASS ? part[2 * (16 * w + 4 * (lane >> 4) + r) + 1] : 0.f;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        svv2[h] = splat2(0.f);
        sv2[h] = splat2(0.f);
        slv2[h] = splat2(0.f);
    }
    f32x4 dz[KP / 16];
#pragma unroll
    for (int lb = 0; lb < KP / 16; ++lb) dz[lb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int wbk = row0 >> 4;  // this wave's 16-row block of the batch entry lists
    fill_toffl(toffl, S, t0, d.NT, Q.toff, wbk, lane);
    const int64_t segw = Q.seg[wbk];
    wave_sync();

    // the tile's entries are fetched two tiles ahead (two register sets, the tile loop unrolled
    // by two): a global load's latency under load is about a tile of this kernel's work
    ListEntries pendA, pendB;
    // lt starts zeroed; afterwards each tile clears only the positions it wrote
    for (int i = lane; i < 16 * LS / 4; i += 64) reinterpret_cast<float4*>(lt)[i] = float4{0.f, 0.f, 0.f, 0.f};
    if (t0 < t1) {
        pendA.fetch(Q.ents, segw, toffl, 0, lane);
        pendB.fetch(Q.ents, segw, toffl, min(1, t1 - t0 - 1), lane);
        stage_store(0);
    }
    lds_barrier();  // the first tiles' entry loads stay in flight
    // bf16 mode: log1p of a set's two register entries (one v_log each) computed a tile before
    // their visit, off the densify's critical path (bf16 16.62M -> 16.93M cells/s).  The table
    // modes (x3, f32) read their LDS table in the visit: looked up early, the reads cost more in
    // the gene blocks than they saved (x3 13.34M -> 13.22M).
    constexpr bool PRE = !VTabT::ON;
    float lvA[2] = {0.f, 0.f}, lvB[2] = {0.f, 0.f};
    auto lookup = [&](const ListEntries& p, float (&lv)[2]) {
#pragma unroll
        for (int k = 0; k < 2; ++k) lv[k] = VTabT::value(ltab, fmaxf(p.x(Q.ents, k), 0.f));
    };
    if (PRE && t0 < t1) lookup(pendA, lvA);
    // diagnostic (MMVAE_DBG & 256, -DMMVAE_DIAG builds): per-wave phase cycles into dzp
    // (outputs invalid): densify, gene blocks, tile barrier, slab store, stage store + barrier
    const bool stamps = dbg_bit(d.dbg, 256);
    uint64_t st_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp_ = stamps ? stamp_now() : 0;
    auto lap = [&](int i_) {
        if (stamps) {
            const uint64_t tn = stamp_now();
            st_[i_] += tn - tp_;
            tp_ = tn;
        }
    };

    auto tile = [&](int t, ListEntries& pend, const float (&lv)[2], const ListEntries& pnext, float (&lvnext)[2]) {
        const int tl = t - t0;
        const int cb = NBF == 2 ? (tl & 1) : 0;  // this tile's stage buffer
        const char* wst = wbuf(cb);
        const float4* gst = gbuf(cb);
        // unconditional (clamped) next-stage loads: counted waits (MMVAE_VDEC_SLOAD_LATE: issued
        // after the densify instead, off the post-barrier burst of every wave's loads)
        if (!MMVAE_VDEC_SLOAD_LATE && !dbg_bit(d.dbg, 512)) stage_load(dbg_bit(d.dbg, 1024) ? t0 : min(t + 1, t1 - 1));
        lap(5);
        // ---- densify this wave's 16 x 64 log1p(relu x) tile (zero outside the entries) ----
        if constexpr (PRE) {
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (lane + 64 * k < pend.n) lt[ent_row(pend.raw[k]) * LS + ent_gene(pend.raw[k])] = lv[k];
            for (int e = 128 + lane; e < pend.n; e += 64) {  // past the register pair: read here
                const uint32_t r = Q.ents.w[pend.base + e];
                const float xv = ent_x(Q.ents, r, ent_xload(Q.ents, pend.base + e));
                VTabT::put(ltab, lt, ent_row(r) * LS + ent_gene(r), 0, fmaxf(xv, 0.f));
            }
        } else {
            pend.visit(Q.ents, lane, [&](int r, int gl, float x) { VTabT::put(ltab, lt, r * LS + gl, 0, fmaxf(x, 0.f)); });
        }
        wave_sync();
        lap(7);
        int zpos0 = pend.pos(0, lane), zpos1 = pend.pos(1, lane);
        // materialised here: pend's registers are free for the next fetch (no loop-carried copy)
        asm volatile("" : "+v"(zpos0), "+v"(zpos1));
        const bool zall = pend.n > 128;  // entries past the register pair: clear the whole tile
        pend.fetch(Q.ents, segw, toffl, min(tl + 2, t1 - t0 - 1), lane);
        if (MMVAE_VDEC_SLOAD_LATE && !dbg_bit(d.dbg, 512)) stage_load(min(t + 1, t1 - 1));
        lap(0);
        // the logits of gene block gb (16 genes x this wave's 16 rows); block gb + 1's MFMAs are
        // issued ahead of block gb's element math, so the two overlap inside the wave
        auto logit = [&](int gb) {
            const int gl = 16 * gb + (lane & 15);
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS; ++s)
                acc = M::mma(zfr[s], M::load(reinterpret_cast<const T*>(wst + swz_off<RBW>(gl, (s * M::KSTEP + (lane >> 4) * M::EPL) * (int)sizeof(T))), WIMG / (int)sizeof(T)), acc);
            return acc;
        };
        // dz[cell][latent] += sum_g da[cell][g] W_d[g][latent] over the k step s's genes — run as
        // soon as the gene blocks it covers have written their da (this wave's own q1 rows)
        auto dz_step = [&](int s) {
            Fr a1;
            if constexpr (X) {
                const char* qb = reinterpret_cast<const char*>(q1);
                a1 = Fr{pqt_frag<512>(qb, s * M::KSTEP), pqt_frag<512>(qb + 2048, s * M::KSTEP)};
            } else if constexpr (BF) {
                a1 = pqt_frag<512>(reinterpret_cast<const char*>(q1), s * M::KSTEP);
            } else {
                a1 = M::load(&q1[(lane & 15) * QS + s * M::KSTEP + (lane >> 4) * M::EPL], QPL);
            }
#pragma unroll
            for (int lb = 0; lb < KP / 16; ++lb) {
                Fr bw;
                if constexpr (TRW) bw = TrFrag<P, RBW>::load(wst, s * M::KSTEP, 16 * lb, WIMG);
                else
                    bw = M::load(reinterpret_cast<const T*>(
                        tst + swz_off<RBT>(16 * lb + (lane & 15), (s * M::KSTEP + (lane >> 4) * M::EPL) * (int)sizeof(T))),
                        WIMG / (int)sizeof(T));
                dz[lb] = M::mma(a1, bw, dz[lb]);
            }
        };
        // (bf16 operand modes: x3 89.1 -> 87.6 us; the f32 mode is faster without, 158 vs 163 us)
        constexpr bool LP = MMVAE_VDEC_LPIPE && BF;
        f32x4 accn = LP ? logit(0) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
            const int gl = 16 * gb + (lane & 15);
            const f32x4 acc = LP ? accn : logit(gb);
            if (LP && gb + 1 < 4) accn = logit(gb + 1);
            const float4 g4 = gst[gl];
            float wcd[CA];
            wcd[0] = g4.z;
#pragma unroll
            for (int c = 1; c < CM; ++c) wcd[c] = (c < C && 64 * t + gl < d.D) ? Q.Wcd[(int64_t)(64 * t + gl) * C + c] : 0.f;
            f2 csp[1 + CA];
#pragma unroll
            for (int c = 0; c < 1 + CA; ++c) csp[c] = splat2(0.f);
            constexpr float L2E = 1.4426950408889634f;
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // rows rl, rl + 1 as one packed pair
                const int rl = 4 * (lane >> 4) + 2 * h;
                const f2 ex = fma2(f2{acc[2 * h], acc[2 * h + 1]}, splat2(L2E), splat2(g4.x));
                const f2 u = f2{fexp2(ex.x), fexp2(ex.y)};      // exp(z_dec(z))   vmf.hh:285
                f2 hc = splat2(CM == 0 ? g4.y + g4.z : g4.y);  // covar_dec(c)    vmf.hh:286
#pragma unroll
                for (int c = 0; c < CM; ++c) hc = fma2(crow2[h][c], splat2(wcd[c]), hc);
                const f2 v = u + hc;                            // padded genes: 0 + 0
                const f2 l = f2{lt[rl * LS + gl], lt[(rl + 1) * LS + gl]};
                if (PASS == 0) {
                    svv2[h] = fma2(v, v, svv2[h]);
                    sv2[h] += v;
                    slv2[h] = fma2(l, v, slv2[h]);
                } else {
                    const f2 dv = fma2(ra2[h], l + g4.w, rbt2[h] * v);  // g4.w = epsD (padded: 0)
                    csp[0] += dv;
#pragma unroll
                    for (int c = 0; c < CM; ++c) csp[1 + c] = fma2(dv, crow2[h][c], csp[1 + c]);
                    const f2 da = dv * u;
                    if constexpr (BF) {
                        pqt_put<512, X>(reinterpret_cast<char*>(q1), 2048, gl, rl, da.x, da.y);
                    } else {
                        put_op<P>(q1, rl * QS + gl, QPL, da.x);
                        put_op<P>(q1, (rl + 1) * QS + gl, QPL, da.y);
                    }
                }
            }
            float cs[1 + CA];
#pragma unroll
            for (int c = 0; c < 1 + CA; ++c) cs[c] = csp[c].x + csp[c].y;
            if (CM == 0) cs[1] = cs[0];  // sum_b dv c_b with c_b = 1
            if (PASS) {
                float* pw = part + w * nq * 64 + gl;
                if (CM <= 1) {  // nq = 2
                    const float s = sum_rowgroups2(cs[0], cs[1]);
                    if (!(lane & 16)) pw[(lane >> 5) * 64] = s;
                } else {
#pragma unroll
                    for (int c = 0; c < 1 + CM; ++c)
                        if (c <= C) {
                            const float s = sum_rowgroups(cs[c]);
                            if (lane < 16) pw[c * 64] = s;
                        }
                }
                // the k steps whose last gene is in this block (x3 / bf16: one step per two
                // blocks; f32: four per block)
                constexpr int GPS = M::KSTEP;
                if (!MMVAE_VDEC_DZ_LATE && (16 * (gb + 1)) % GPS == 0) {
                    wave_sync();
#pragma unroll
                    for (int s = 0; s < GK; ++s)
                        if ((s + 1) * GPS > 16 * gb && (s + 1) * GPS <= 16 * (gb + 1)) dz_step(s);
                }
            }
        }
        if (PASS && MMVAE_VDEC_DZ_LATE) {
            wave_sync();
#pragma unroll
            for (int s = 0; s < GK; ++s) dz_step(s);
        }
        // clear what this tile wrote into lt (the gene blocks above were its last readers)
        if (zall) {
            for (int i = lane; i < 16 * LS / 4; i += 64) reinterpret_cast<float4*>(lt)[i] = float4{0.f, 0.f, 0.f, 0.f};
        } else {
            if (zpos0 >= 0) lt[(zpos0 >> 6) * LS + (zpos0 & 63)] = 0.f;
            if (zpos1 >= 0) lt[(zpos1 >> 6) * LS + (zpos1 & 63)] = 0.f;
        }
        if (PRE && t + 1 < t1) lookup(pnext, lvnext);
        lap(1);
        if (PASS || NBF == 1) lds_barrier();  // (the forward pass: its stage is double-buffered)
        lap(2);
        if (PASS) {
            for (int i = threadIdx.x; i < nq * 64; i += 256) {
                const int q = i >> 6, g = i & 63;
                Q.slabB[((int64_t)rb * nq + q) * d.DP + 64 * t + g] =
                    part[(0 * nq + q) * 64 + g] + part[(1 * nq + q) * 64 + g] + part[(2 * nq + q) * 64 + g] +
                    part[(3 * nq + q) * 64 + g];
            }
        }
        lap(3);
        if (t + 1 < t1) stage_store(NBF == 2 ? ((tl + 1) & 1) : 0);
        lds_barrier();
        lap(4);
    };
    for (int t = t0; t < t1; t += 2) {
        tile(t, pendA, lvA, pendB, lvB);
        if (t + 1 < t1) tile(t + 1, pendB, lvB, pendA, lvA);
    }
    if (stamps) {
        if (lane == 0) {
            float* o = Q.dzp + ((int64_t)blockIdx.x * 4 + w) * 12;
            for (int i = 0; i < 8; ++i) o[i] = (float)st_[i];
            o[8] = (float)(t1 - t0);
            o[9] = (float)wave_place();
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int b = row0 + 4 * (lane >> 4) + r;
        if (PASS == 0) {
            float a = svv2[r >> 1][r & 1], s1 = sv2[r >> 1][r & 1], s2 = slv2[r >> 1][r & 1];
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                a += __shfl_xor(a, o, 64);
                s1 += __shfl_xor(s1, o, 64);
                s2 += __shfl_xor(s2, o, 64);
            }
            if ((lane & 15) == 0) {
                float* rp = Q.rowB + ((int64_t)sp * d.Bpad + b) * 3;
                rp[0] = a;
                rp[1] = s1;
                rp[2] = s2;
            }
        } else {
#pragma unroll
            for (int lb = 0; lb < KP / 16; ++lb)
                Q.dzp[((int64_t)sp * d.Bpad + b) * KP + 16 * lb + (lane & 15)] = dz[lb][r];
        }
    }
}

// forward pass occupancy: 4 waves per SIMD (<= 128 VGPRs, no spills) for the 16-bit operand
// modes at K <= 32 with one covariate — the pass is latency-bound (phase stamps: one wave per SIMD
// takes ~3.1k cycles per tile, three take ~3.5k), so a fourth workgroup per CU adds throughput
template <class P, int KP, int CM> struct VFwdOcc {
    static constexpr int value = (sizeof(typename Elem<P>::type) == 2 && KP <= 32 && CM <= 1) ? 4 : 2;
};
template <class P, int KP, int CM>
__global__ __launch_bounds__(256, (VFwdOcc<P, KP, CM>::value)) void k_vdec_fwd(VDecPtrs Q, Dims d, float epsD) { vdec_body<P, KP, 0, CM>(Q, d, epsD); }
template <class P, int KP, int CM>
__global__ __launch_bounds__(256, 2) void k_vdec_bwd(VDecPtrs Q, Dims d, float epsD) { vdec_body<P, KP, 1, CM>(Q, d, epsD); }

// =======================================================================================
// k_vrowfin — per row (one thread): combine pass-0 splits, cos_b = <y_b, r_b>
// (vmf.hh:422-432) and the decoder backward coefficients (see oracle/vmf_analytic.py):
//   alpha_b = -(kappa/n) / (nv ny),  beta_b = (kappa/n) cos_b / nv^2
// (below the normalize eps, r = v / eps and the clamp passes no gradient: beta = 0).
// =======================================================================================
__global__ __launch_bounds__(256) void k_vrowfin(Dims d, float epsD, const float* __restrict__ lat,
                                                 const float* __restrict__ rowx, const float* __restrict__ rowB,
                                                 const float* __restrict__ vk, float* __restrict__ rowfin,
                                                 float* __restrict__ rowcos) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= d.Bpad) return;
    float al, be, cosb;
    vrow_coeffs(d, epsD, lat, rowx, rowB, vk, b, 0, 1, al, be, cosb);
    rowfin[2 * b] = al;
    rowfin[2 * b + 1] = be;
    rowcos[b] = cosb;
}

// =======================================================================================
// k_vlatent_bwd — backward of the reparameterisation, clamp, KL and the Z x Z heads for 64
// cells per workgroup (lane = latent):  dz = sum over decoder splits,
//   dmean = dz + (beta/n) mean,  da = [dz eps e^{lnvar/2}/2 + (beta/n)(e^{lnvar} - 1)/2] mask
//   dh = dmean Wm + da Wl;  dWm += dmean^T h, dWl += da^T h (per-workgroup partials)
// dhT (encoder backward operand) = dh / ||l||; the x_mean gradient needs the unscaled sum.
// =======================================================================================
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_vlatent_bwd(VPtrs P, Dims d, const int64_t* __restrict__ cells,
                                                     const float* __restrict__ covar, const float* __restrict__ lat,
                                                     const float* __restrict__ dzp, float* __restrict__ dhT_f,
                                                     __bf16* __restrict__ dhT_b, float* __restrict__ small) {
    constexpr int CPW = LAT_CELLS / NW;  // cells per wave (NW = 16: no frozen chains)
    constexpr bool CHAINS = NW == 4;
    const int K = d.K, C = d.C, KP = d.KP, E = d.E, KE = d.KE;
    const int SMALL = small_len(K, E, KE, C, 0);
    constexpr int NSM = 3 * 64 + 64 * CMAX;
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    float* sWm = lsm;               // [K][65]
    float* sWl = sWm + 64 * 65;     // [K][65]
    float* sDM = sWl + 64 * 65;            // [cell][68] dmean
    float* sDA = sDM + LAT_CELLS * 68;     // [cell][68] d(pre-clamp lnvar)
    float* sH = sDA + LAT_CELLS * 68;      // [cell][68] h0 (column 64: 1/||l||)
    float* sT = sH + LAT_CELLS * 68;       // [64][17] dh0 / ||l||, transposed (latent-major)
    float (*wpart)[NSM] = reinterpret_cast<float (*)[NSM]>(sT + 64 * 17);  // [NW][NSM]
    // frozen chains (only with hidden layers): W stage, two gradient images, the recomputed
    // chain outputs (ReLU masks): encoder [nce], decoder z + [ncd]
    float* sCW = &wpart[NW][0];
    float* const sG0 = sCW + 64 * 65;  // gradient images sG(0), sG(1)
    auto sG = [&](int i) { return sG0 + i * (LAT_CELLS * 68); };
    float* cimg = sG0 + 2 * LAT_CELLS * 68;
    // every global input first (one memory round): head weights, dz split partials, the cells' latent records
    HeadsStage<64 * NW> hst;
    hst.issue(P.Wm, P.Wl, K, E);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = lane;
    const int cw = CPW * w;                     // this wave's first cell in the workgroup
    const int bw = blockIdx.x * LAT_CELLS + cw;  // ... in the batch
    float dz4[CPW];  // the decoder GEMM input's gradient (KD wide)
    split_sum<CPW>(dzp, d.nsD, (int64_t)d.Bpad * KP, (int64_t)bw * KP + k, KP, k < d.KD, dz4);
    const int kk = min(k, K - 1), ke = min(k, KE - 1);
    float vval[CPW], vinx[CPW], vh[CPW], vmean[CPW], va[CPW], veps[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const float* L = lat + (int64_t)(bw + c) * d.lat_stride;
        vval[c] = L[d.LAT_VALID];
        vinx[c] = L[d.LAT_D];
        vh[c] = L[d.LAT_H + ke];
        vmean[c] = L[d.LAT_MEAN + kk];
        va[c] = L[d.LAT_A + kk];
        veps[c] = L[d.LAT_EPS + kk];
    }
    hst.store(K, E, sWm, sWl);
    // with a decoder chain: dz at the latent = the chain's backward from dzd (z recomputed, the
    // chain outputs kept for the ReLU masks)
    const float* dzimg = nullptr;
    if (CHAINS && d.ncd > 0) {
        float* zimg = cimg + d.nce * LAT_CELLS * 68;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const float lnvar = fminf(fmaxf(va[c], -4.f), 4.f);
            zimg[(cw + c) * 68 + k] = (k < K) ? vmean[c] + veps[c] * expf(lnvar / 2.f) : 0.f;
            sG(0)[(cw + c) * 68 + k] = (k < d.KD && vval[c] > 0.f) ? dz4[c] : 0.f;
        }
        __syncthreads();
        float* outs = zimg + LAT_CELLS * 68;  // decoder chain outputs [ncd]
        chain_run(d, d.nce, d.nce + d.ncd, zimg, outs, nullptr, true, sCW, w, lane);
        int g = 0;
        for (int l = d.ncd - 1; l >= 0; --l) {
            chain_stage_w(d, d.nce + l, sCW);
            __syncthreads();
            const f32x4 acc = chain_bwd(d, d.nce + l, sG(g), outs + l * LAT_CELLS * 68, sCW, d.relu != 0, w, lane);
            img_store(sG(g ^ 1), acc, w, lane);
            __syncthreads();
            g ^= 1;
        }
        dzimg = sG(g);
    }
    const float bn = d.beta * d.inv_n;
    float rbm = 0.f, rbl = 0.f, rWce[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) rWce[c] = 0.f;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        const bool valid = vval[c] > 0.f;
        float dmean = 0.f, da = 0.f;
        const float h = (k < KE && valid) ? vh[c] : 0.f;  // dW = dmean^T h: 0 * h must be 0
        if (k < K) {
            const float dz = dzimg ? dzimg[(cw + c) * 68 + k] : dz4[c];
            const float mean = vmean[c], a = va[c], eps = veps[c];
            const float lnvar = fminf(fmaxf(a, -4.f), 4.f);
            const float sig = expf(lnvar / 2.f);
            dmean = dz + bn * mean;
            const float dlnvar = dz * eps * sig * 0.5f + bn * 0.5f * (expf(lnvar) - 1.f);
            da = (a >= -4.f && a <= 4.f) ? dlnvar : 0.f;
            if (!valid) {
                dmean = 0.f;
                da = 0.f;
            }
        }
        sDM[(cw + c) * 68 + k] = dmean;
        sDA[(cw + c) * 68 + k] = da;
        sH[(cw + c) * 68 + k] = h;
        if (k == 0) sH[(cw + c) * 68 + 64] = vinx[c];  // 1/||l|| beside the cell's h
        rbm += dmean;
        rbl += da;
        if (!covar) {  // unit covariate (Engine::unit_covar): c = 1 (dmean is 0 on padding rows)
            rWce[0] += dmean;
        } else {
            const int64_t cell = cells[b];  // padding rows hold the empty row N
#pragma unroll
            for (int q = 0; q < CMAX; ++q)
                if (q < C) rWce[q] += dmean * covar[cell * C + q];
        }
    }
    for (int i = lane; i < NSM; i += 64) wpart[w][i] = 0.f;
    __syncthreads();
    float* wp = wpart[w];
    // the heads' input: h0, or the Angular chain's output (recomputed, outputs kept)
    const float* hin = sH;
    if (CHAINS && d.nce > 0) {
        hin = chain_run(d, 0, d.nce, sH, cimg, nullptr, true, sCW, w, lane);
    }
    if (w < 4) {  // dh0[16 cells][KE] on f32 MFMA (wave w: columns 16w..16w+15), scaled by 1/||l|| for k_enc_bwd
        f32x4 acc = heads_dh(sDM, sDA, sWm, sWl, K, E, w, lane);
        if (CHAINS && d.nce > 0) {  // back through the Angular chain
            img_store(sG(0), acc, w, lane);
            __syncthreads();
            int g = 0;
            for (int l = d.nce - 1; l >= 0; --l) {
                chain_stage_w(d, l, sCW);
                __syncthreads();
                acc = chain_bwd(d, l, sG(g), cimg + l * LAT_CELLS * 68, sCW, d.relu != 0, w, lane);
                if (l > 0) {
                    img_store(sG(g ^ 1), acc, w, lane);
                    __syncthreads();
                    g ^= 1;
                }
            }
        }
        const int j = 16 * w + (lane & 15);
        float rdhs = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cl = 4 * (lane >> 4) + r, b = blockIdx.x * LAT_CELLS + cl;
            if (j < KP && b < d.Bpad) {  // [KP][Bpad] images: rows past this batch's padded size write nothing
                // ReLU backward: the gradient passes where the (stored, post-ReLU) h is > 0
                const bool pass = j < KE && (!d.relu || sH[cl * 68 + j] > 0.f);
                const float v = pass ? acc[r] : 0.f;
                sT[j * 17 + cl] = v * sH[cl * 68 + 64];  // stored transposed below
                rdhs += v;
            }
        }
        rdhs = sum_rowgroups(rdhs);
        if (lane < 16) wp[128 + j] = rdhs;  // the other waves' partials of latent j stay 0
    }
    wp[k] = rbm;
    wp[64 + k] = rbl;
#pragma unroll
    for (int q = 0; q < CMAX; ++q) wp[192 + k * CMAX + q] = rWce[q];
    float* out = small + (int64_t)blockIdx.x * SMALL;
    if (w < 4) heads_dW(sDM, sDA, hin, K, E, w, lane, out);
    __syncthreads();
    // dh^T / ||l|| [KP][Bpad] (the encoder backward's A operand: f32 image, or the bf16 hi [+ lo]
    // planes) from the transposed LDS tile: 16 consecutive cells of one latent per 16 lanes
    for (int i = threadIdx.x; i < KP * LAT_CELLS; i += 64 * NW) {
        const int j = i >> 4, cl = i & 15, b = blockIdx.x * LAT_CELLS + cl;
        const float vs = sT[j * 17 + cl];
        if (b < d.Bpad) {
            if (dhT_f) dhT_f[(int64_t)j * d.Bpad + b] = vs;
            if (dhT_b) put_op<X3>(dhT_b, j * d.Bpad + b, KP * d.Bpad, vs);  // hi plane (+ the x3 lo plane)
        }
    }
    const int o_bm = 2 * K * E, o_bl = o_bm + K, o_ce = o_bl + K, o_dhs = o_ce + K * C;
    auto wsum = [&](int off) {  // fixed order over the waves, four at a time
        float t = (wpart[0][off] + wpart[1][off]) + (wpart[2][off] + wpart[3][off]);
#pragma unroll
        for (int i = 4; i < NW; i += 4) t += (wpart[i][off] + wpart[i + 1][off]) + (wpart[i + 2][off] + wpart[i + 3][off]);
        return t;
    };
    for (int i = threadIdx.x; i < K; i += 64 * NW) {
        out[o_bm + i] = wsum(i);
        out[o_bl + i] = wsum(64 + i);
        for (int q = 0; q < C; ++q) out[o_ce + i * C + q] = wsum(192 + i * CMAX + q);
    }
    for (int i = threadIdx.x; i < KE; i += 64 * NW) out[o_dhs + i] = wsum(128 + i);
}
// k_vlatent_bwd's LDS (+ the chain W stage, 2 gradient images and the chain outputs with hidden layers)
static size_t vlat_bwd_lds(const Engine* e, int nw) {
    size_t f = 2 * 64 * 65 + 3 * LAT_CELLS * 68 + 64 * 17 + (size_t)nw * (3 * 64 + 64 * CMAX);
    if (e->nce + e->ncd > 0) f += 64 * 65 + (size_t)(2 + e->nce + e->ncd + 1) * LAT_CELLS * 68;
    return f * 4;
}

// =======================================================================================
// k_vgrad_small — block 0: the loss (vmf.hh:429-439) and the ln_kappa gradient
//   L = beta KL / n - (kappa sum_b cos_b + B (T - c2)) / n
//   dkappa = -sum_b cos_b / n + df (-B/n) / kappa + [rank 0] Baricz(kappa)   (Q3: the lbessel
//   backward ignores its upstream gradient, so under DP only one rank adds it)
//   dln_kappa = dkappa exp(ln_kappa) [kappa_min <= exp(ln_kappa) <= kappa_max]
// other blocks: fixed-order reduction of k_vlatent_bwd's per-workgroup partials.
// =======================================================================================
MMVAE_DEV void vgrad_small_body(const Dims& d, const VScal& sc, const float* __restrict__ small, int nwg,
                                const VGrads& G, float* __restrict__ smallg, const float* __restrict__ rowcos,
                                const float* __restrict__ klpart, int nkl, const float* __restrict__ vk,
                                float* __restrict__ out, int with_grads, double* __restrict__ sqpart, const int bid) {
    const int K = d.K, C = d.C, E = d.E, KE = d.KE;
    const int SMALL = small_len(K, E, KE, C, 0);
    if (bid == 0) {
        __shared__ float sb[8];
        float cs = 0.f, ks = 0.f;
        for (int i = threadIdx.x; i < d.Bpad; i += 256) cs += rowcos[i];
        for (int i = threadIdx.x; i < nkl; i += 256) ks += klpart[i];
        const float tc = block_sum<4>(cs, sb);
        const float tk = block_sum<4>(ks, sb);
        if (threadIdx.x == 0) {
            const float kap = vk[VK_KAPPA];
            const float Bn = (float)d.B * d.inv_n;
            const float llik_sum = fmaf(kap, tc, (float)d.B * (vk[VK_T] - sc.c2));
            out[0] = tk * d.beta * d.inv_n - llik_sum * d.inv_n;
            if (with_grads) {
                float dk = -tc * d.inv_n;
                dk += (sc.df * -Bn) / kap;
                if (sc.rank0) dk += vk[VK_BARICZ];
                const float glk = (vk[VK_MASK] > 0.f) ? dk * vk[VK_EXP] : 0.f;
                G.lk[0] = glk;
                if (sqpart) sqpart[0] = (double)glk * glk;
            }
        }
        return;
    }
    if (!with_grads) return;
    __shared__ float red[8][32];
    const int i = (bid - 1) * 32 + (threadIdx.x & 31);
    const float s = sum_partials(small, nwg, SMALL, i, red);
    // store the small gradient; returns how many gradient elements received s (0: smallg)
    auto store = [&]() -> int {
        int o = i;
        if (o < K * E) { G.Wm[o] = s; return 1; }
        o -= K * E;
        if (o < K * E) { G.Wl[o] = s; return 1; }
        o -= K * E;
        if (o < K) { G.bm[o] = s; G.bce[o] = s; return 2; }
        o -= K;
        if (o < K) { G.bl[o] = s; return 1; }
        o -= K;
        if (o < K * C) { G.Wce[o] = s; return 1; }
        o -= K * C;
        smallg[o] = s;  // cdh = sum_b dh_b
        return 0;
    };
    double sq = 0.0;
    if ((threadIdx.x >> 5) == 0 && i < SMALL) sq = (double)s * s * store();
    if (sqpart && threadIdx.x < 64) {  // clip-norm partial of this block (fixed order)
        sq = wave_sum_d(sq);
        if (threadIdx.x == 0) sqpart[bid] = sq;
    }
}

__global__ __launch_bounds__(256) void k_vgrad_small(Dims d, VScal sc, const float* __restrict__ small, int nwg,
                                                     VGrads G, float* __restrict__ smallg,
                                                     const float* __restrict__ rowcos, const float* __restrict__ klpart,
                                                     int nkl, const float* __restrict__ vk, float* __restrict__ out,
                                                     int with_grads, double* __restrict__ sqpart) {
    vgrad_small_body(d, sc, small, nwg, G, smallg, rowcos, klpart, nkl, vk, out, with_grads, sqpart, (int)blockIdx.x);
}

// the encoder backward (log1p term only) and the small-gradient / loss blocks in one launch
template <class P, int KP>
__global__ __launch_bounds__(256) void k_enc_bwd_vsmall(EntList ents, const int64_t* __restrict__ seg,
                                                        const int32_t* __restrict__ toff, const float* __restrict__ lat,
                                                        const typename Elem<P>::type* __restrict__ dhT, int64_t dplane,
                                                        const typename WEnc<P>::type* __restrict__ WeP, Dims d,
                                                        float* __restrict__ slabE, int nenc, VScal sc,
                                                        const float* __restrict__ small, int nwg, VGrads G,
                                                        float* __restrict__ smallg, const float* __restrict__ rowcos,
                                                        const float* __restrict__ klpart, int nkl,
                                                        const float* __restrict__ vk, float* __restrict__ out,
                                                        double* __restrict__ sqpart) {
    const int bid = (int)blockIdx.x;
    if (bid < nenc) enc_bwd_body<P, KP, true, false>(ents, seg, toff, lat, dhT, dplane, WeP, d, slabE, bid);
    else vgrad_small_body(d, sc, small, nwg, G, smallg, rowcos, klpart, nkl, vk, out, 1, sqpart, bid - nenc);
}

// Per-gene gradients from the row-block slabs (fixed order): covar_decoding_ (decoder pass 1)
// and x_mean / ln_x_sd through the Angular encoder (k_enc_bwd's sum_k W~ M term).
// PART: 0 = all; 1 = covar_decoding_ only (slab B, final after k_vdec_bwd: its all-reduce overlaps
// the encoder backward); 2 = x_mean / ln_x_sd only (slab E)
static constexpr int VGG_GENES = 64;  // genes per k_vgrad_genes workgroup
template <int PART>
__global__ __launch_bounds__(256) void k_vgrad_genes(VPtrs P, Dims d, VGrads G, const float* __restrict__ gene,
                                                     const float* __restrict__ WeP_f, const float* __restrict__ slabB,
                                                     const float* __restrict__ slabE, const float* __restrict__ smallg,
                                                     int nrb, double* __restrict__ sqpart) {
    // 64 genes x 16 row-block partitions per workgroup: a thread reads 4 consecutive genes of
    // every slab row with one 16-byte load (all of them in flight together); the partitions'
    // partial sums meet in LDS and thread g < 64 adds them in partition order.
    constexpr int NQ = 1 + CMAX + 1 + 1;  // slab B [1 + C], slab E [1], the column dot sum_k cdh[k] W~[k][g]
    constexpr int NPART = 16, GPT = 4;
    __shared__ float cdh[64];
    __shared__ float red[NPART][NQ][VGG_GENES];
    const int C = d.C, nqB = 1 + C;
    const int part = threadIdx.x >> 4, gq = (threadIdx.x & 15) * GPT;
    const int g0 = blockIdx.x * VGG_GENES;  // DP is a multiple of 64: every slab / W read is in bounds
    auto ld = [&](const float* p) { return *reinterpret_cast<const f32x4*>(p); };
    // every load first (clamped, unconditional; one memory round): the column dot's W rows
    // (latent rows part, part + NPART, ...), dh's column sums, the final phase's gene parameters
    // (threads < 64), then the slab rows
    f32x4 wv[64 / NPART];
#pragma unroll
    for (int i = 0; i < 64 / NPART; ++i) wv[i] = ld(WeP_f + (int64_t)min(part + NPART * i, d.KE - 1) * d.DP + g0 + gq);
    const float cdv = smallg[min((int)threadIdx.x, d.KE - 1)];
    const int gf = min(g0 + (int)threadIdx.x, d.D - 1);
    const float f_inv = gene[gf], f_xm = P.xm[gf], f_lsd = P.lsd[gf];
    f32x4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int rb = part; rb < nrb; rb += NPART) {
        const float* sB = slabB + (int64_t)rb * nqB * d.DP + g0 + gq;
#pragma unroll
        for (int q = 0; q < 1 + CMAX; ++q)
            if (PART != 2 && q < nqB) acc[q] += ld(sB + (int64_t)q * d.DP);
        if (PART != 1) acc[NQ - 2] += ld(slabE + (int64_t)rb * d.DP + g0 + gq);
    }
    if (threadIdx.x < d.KE) cdh[threadIdx.x] = cdv;
    __syncthreads();
    if (PART != 1) {  // sum_k cdh[k] W~[k][g] in latent order
#pragma unroll
        for (int i = 0; i < 64 / NPART; ++i)
            if (part + NPART * i < d.KE)
#pragma unroll
                for (int e = 0; e < GPT; ++e) acc[NQ - 1][e] = fmaf(cdh[part + NPART * i], wv[i][e], acc[NQ - 1][e]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int i = 0; i < GPT; ++i) red[part][q][gq + i] = acc[q][i];
    __syncthreads();
    double sq = 0.0;  // sum of squares of the gradient elements this block writes (clip norm)
    auto put = [&](float* dst, float v) { *dst = v; sq += (double)v * v; };
    const int g = g0 + (int)threadIdx.x;
    if (threadIdx.x < VGG_GENES && g < d.D) {
        float t[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            float v = 0.f;
#pragma unroll
            for (int pp = 0; pp < NPART; ++pp) v += red[pp][q][threadIdx.x];
            t[q] = v;
        }
        if (PART != 2) {
            put(&G.bcd[g], t[0]);
            for (int c = 0; c < C; ++c) put(&G.Wcd[(int64_t)g * C + c], t[1 + c]);
        }
        if (PART != 1) {
            const float Gl = t[NQ - 2], gs = t[NQ - 1];
            const float inv = f_inv;
            put(&G.xm[g], -inv * gs);
            put(&G.lsd[g], -(inv * inv) * (Gl - f_xm * gs) * dsoftplus(f_lsd));
        }
    }
    if (sqpart && threadIdx.x < 64) {  // wave 0 holds every writer (threads 0..63)
        sq = wave_sum_d(sq);
        if (threadIdx.x == 0) sqpart[blockIdx.x] = sq;
    }
}

// =======================================================================================
// host-side launch orchestration
// =======================================================================================
static VPtrs vmf_ptrs(Engine* e) {
    VPtrs P;
    P.xm = e->preg("x_mean");
    P.lsd = e->preg("ln_x_sd");
    P.lk = e->preg("ln_kappa");
    P.Wce = e->preg("covar_encoding.weight");
    P.bce = e->preg("covar_encoding.bias");
    P.Wm = e->preg("representation_mean.weight");
    P.bm = e->preg("representation_mean.bias");
    P.Wl = e->preg("representation_logvariance.weight");
    P.bl = e->preg("representation_logvariance.bias");
    P.Wcd = e->preg("covar_decoding_.weight");
    P.bcd = e->preg("covar_decoding_.bias");
    P.We = e->pfrz(e->fz_enc_w);
    P.Wd = e->pfrz(e->fz_dec_w);
    P.bd = e->pfrz(e->fz_dec_b);
    return P;
}

static VGrads vmf_grads(Engine* e) {
    VGrads G;
    G.xm = e->greg("x_mean");
    G.lsd = e->greg("ln_x_sd");
    G.lk = e->greg("ln_kappa");
    G.Wce = e->greg("covar_encoding.weight");
    G.bce = e->greg("covar_encoding.bias");
    G.Wm = e->greg("representation_mean.weight");
    G.bm = e->greg("representation_mean.bias");
    G.Wl = e->greg("representation_logvariance.weight");
    G.bl = e->greg("representation_logvariance.bias");
    G.Wcd = e->greg("covar_decoding_.weight");
    G.bcd = e->greg("covar_decoding_.bias");
    return G;
}

static float host_fasterlog(float x) {
    uint32_t i;
    std::memcpy(&i, &x, 4);
    volatile float y = (float)i;
    y = y * 8.2629582881927490e-8f;
    return y - 87.989971088f;
}

static VScal vmf_scal(Engine* e) {
    VScal s;
    const int64_t D = e->D;
    s.epsD = (float)(1e-2 / (double)(float)D);
    s.df = (float)std::max(0.5 * (double)(float)D - 1., 0.);
    s.kmin = e->cfg.kappa_min;
    s.kmax = e->cfg.kappa_max;
    s.lg_df1 = mmvae_fasterlgamma((float)((double)s.df + 1));
    s.c2 = (float)(0.5 * (double)(float)D * (double)host_fasterlog((float)(2. * M_PI)));
    s.rank0 = e->rank == 0 ? 1 : 0;
    return s;
}

hipError_t vmf_prepare_frozen(Engine* e) {
    ScopedTimer tm(e, "k_vpack_frozen");
    hipLaunchKernelGGL(k_vnorm_enc, dim3((unsigned)e->KP), dim3(1024), 0, e->stream, e->pfrz(e->fz_enc_w),
                       (int)e->D, (int)e->DP, (int)e->KE, e->d_WeP_f, e->d_WeP_b);
    const int64_t n = e->KP * e->DP;
    hipLaunchKernelGGL(k_vpack_dec, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream,
                       e->pfrz(e->fz_dec_w), (int)e->D, (int)e->DP, (int)e->KD, (int)e->KP, e->d_WdP_f,
                       e->d_WdP_b, e->d_WdT_f, e->d_WdT_b);
    hipError_t er = pack_chain(e, true);
    if (er != hipSuccess) return er;
    e->frozen_dirty = false;
    // captured step graphs hold the old operands' scalars by value (the fp8 mode's 1 / wscale in
    // Dims): re-capture them
    ++e->graph_gen;
    return hipGetLastError();
}

static Dims vmf_dims(Engine* e, int64_t B, int64_t n_total, float beta) {
    Dims d{};
    d.D = (int)e->D;
    d.DP = (int)e->DP;
    d.NT = (int)e->NT;
    d.K = (int)e->K;
    d.KP = (int)e->KP;
    d.C = (int)e->C;
    d.H = 1;
    d.R = 1;
    d.B = (int)B;
    d.Bpad = (int)pad_rows(B);
    d.nrb = d.Bpad / 64;
    d.nsE = e->nsplit_e;
    d.tpsE = (int)((e->NT + d.nsE - 1) / d.nsE);
    d.nsB = e->nsplit_b;
    d.tpsB = (int)((e->NT + d.nsB - 1) / d.nsB);
    d.nsD = e->nsplit_d;
    d.tpsD = (int)((e->NT + d.nsD - 1) / d.nsD);
    d.nsF = e->nsplit_f;
    d.tpsF = (int)((e->NT + d.nsF - 1) / d.nsF);
    d.nsA = e->nsplit_a;
    d.tpsA = (int)((e->NT + d.nsA - 1) / d.nsA);
    d.inv_n = 1.f / (float)n_total;
    d.beta = beta;
    d.lat_stride = (int)e->lat_stride;
    d.LAT_H = (int)e->LAT_H;
    d.LAT_MEAN = (int)e->LAT_MEAN;
    d.LAT_A = (int)e->LAT_A;
    d.LAT_EPS = (int)e->LAT_EPS;
    d.LAT_D = (int)e->LAT_D;  // vMF: 1 / ||log1p x||
    d.LAT_VALID = (int)e->LAT_VALID;
    d.rowx_stride = 2 + (int)e->H;
    d.Ncells = (int)e->N;
    d.nmv = (int)((e->DP + 255) / 256);
#ifdef MMVAE_DIAG
    { const char* ev = getenv("MMVAE_DBG"); d.dbg = ev ? atoi(ev) : 0; }
#else
    d.dbg = 0;
#endif
    d.relu = e->cfg.relu != 0;
    d.inv_wscale = 1.f;
    dims_hidden(e, d);
    return d;
}

template <class PM, int KP>
static hipError_t vmf_launch_all(Engine* e, const Dims& d, const VPtrs& P, const VScal& sc, bool update,
                                 bool use_eps, int mode, float* out_mean,
                                 float* out_lnvar) {
    using T = typename Elem<PM>::type;
    constexpr int NPL = IsX3<PM>::value ? 2 : 1;
    const bool bf = sizeof(T) == 2;  // bf16 planes (bf16, x3)
    hipStream_t st = e->stream;
    const int nrb = d.nrb;
    float* gene = e->d_gene;  // k_vprep ran before the batch lists (vmf_prep)
    const bool ucov = d.C == 1 && e->unit_covar;  // the CM = 0 decoder instances
    const float* lat_covar = ucov ? nullptr : e->d_covar;  // latent kernels: no covariate gather
    // latent kernels: one cell per wave (16 waves) without frozen chains (k_latent_fwd, NB)
    static const bool lat_nw4 = getenv_is("MMVAE_LAT_NW", "4");
    const bool lat16 = !lat_nw4 && d.nce == 0 && d.ncd == 0;
    {
        ScopedTimer tm(e, "k_enc_fwd");
        hipError_t er = enc_forward_launch(e, d, e->d_hpart);
        if (er != hipSuccess) return er;
    }
    {
        ScopedTimer tm(e, "k_vlatent_fwd");
        auto go = [&](auto kern, int nth) {
            hipLaunchKernelGGL(kern, dim3(e->n_lat_wg), dim3(nth), 0, st, P, d, e->d_cells,
                               mode == 1 ? e->d_covar : lat_covar, e->d_hpart, e->d_mvec,
                               (const float2*)e->d_cellnorm, e->d_rowx, use_eps ? e->d_eps : nullptr,
                               (mode == 0 && e->perm_active) ? e->d_perm : nullptr, e->cfg.seed, e->d_ss, e->d_lat,
                               e->d_zf, e->d_zb, e->d_lossp, mode, out_mean, out_lnvar);
        };
        if (lat16) go(k_vlatent_fwd<16>, 1024);
        else go(k_vlatent_fwd<4>, 256);
    }
    if (mode == 1) return hipGetLastError();
    VDecPtrs Q;
    Q.lat = e->d_lat;
    Q.zf = e->d_zf;
    Q.zb = e->d_zb;
    Q.gene = gene;
    Q.Wcd = P.Wcd;
    Q.covar = e->d_covar;
    Q.cells = e->d_cells;
    Q.ents = ent_list(e);
    Q.seg = e->d_seg;
    Q.toff = e->d_toff;
    Q.WdP = bf ? (const void*)e->d_WdP_b : (const void*)e->d_WdP_f;
    Q.WdT = bf ? (const void*)e->d_WdT_b : (const void*)e->d_WdT_f;
    Q.rowfin = e->d_rowfin;
    Q.rowB = e->d_rowB;
    Q.rowx = e->d_rowx;
    Q.vk = e->d_vk;
    Q.rowcos = e->d_rowv;
    Q.dzp = e->d_dzp;
    Q.slabB = e->d_slabB;
    Q.zplane = (int64_t)d.Bpad * d.KP;
    Q.wplane = (int64_t)e->KP * e->DP;
    const dim3 gdec(nrb * d.nsD);
    const int nq = 1 + d.C;
    const int S = d.tpsD + 1;
    {
        ScopedTimer tm(e, "k_vdec_fwd");
        const dim3 gfwd(nrb * d.nsF);  // the forward pass's own split (VFwdOcc)
        const size_t lds = (size_t)VDecLds(KP, (int)sizeof(T), d.tpsF + 1, nq, 0, NPL, 2).bytes;
        if (ucov) hipLaunchKernelGGL((k_vdec_fwd<PM, KP, 0>), gfwd, dim3(256), lds, st, Q, d, sc.epsD);
        else if (d.C == 1) hipLaunchKernelGGL((k_vdec_fwd<PM, KP, 1>), gfwd, dim3(256), lds, st, Q, d, sc.epsD);
        else hipLaunchKernelGGL((k_vdec_fwd<PM, KP, CMAX>), gfwd, dim3(256), lds, st, Q, d, sc.epsD);
    }
    VGrads G = vmf_grads(e);
    const int SMALL = small_len(d.K, d.E, d.KE, d.C, 0);
    if (!update) {  // eval: cos_b for the loss (the update path derives it inside k_vdec_bwd)
        {
            ScopedTimer tm(e, "k_vrowfin");
            hipLaunchKernelGGL(k_vrowfin, dim3((d.Bpad + 255) / 256), dim3(256), 0, st, d, sc.epsD, e->d_lat,
                               e->d_rowx, e->d_rowB, e->d_vk, e->d_rowfin, e->d_rowv);
        }
        ScopedTimer tm(e, "k_loss");
        hipLaunchKernelGGL(k_vgrad_small, dim3(1), dim3(256), 0, st, d, sc, e->d_small, 0, G, e->d_smallg, e->d_rowv,
                           e->d_lossp, e->n_lat_wg, e->d_vk, e->d_out, 0, nullptr);
        return hipGetLastError();
    }
    {
        ScopedTimer tm(e, "k_vdec_bwd");
        const size_t lds = (size_t)VDecLds(KP, (int)sizeof(T), S, nq, 1, NPL).bytes;
        if (ucov) hipLaunchKernelGGL((k_vdec_bwd<PM, KP, 0>), gdec, dim3(256), lds, st, Q, d, sc.epsD);
        else if (d.C == 1) hipLaunchKernelGGL((k_vdec_bwd<PM, KP, 1>), gdec, dim3(256), lds, st, Q, d, sc.epsD);
        else hipLaunchKernelGGL((k_vdec_bwd<PM, KP, CMAX>), gdec, dim3(256), lds, st, Q, d, sc.epsD);
    }
    const bool split = split_grads(e);
    if (split) {  // covar_decoding_ gradients final: all-reduce them under the encoder backward
        ScopedTimer tm(e, "k_vgrad_genes_dec");
        hipLaunchKernelGGL(k_vgrad_genes<1>, dim3((d.D + VGG_GENES - 1) / VGG_GENES), dim3(256), 0, st, P, d, G, gene, e->d_WeP_f,
                           e->d_slabB, e->d_slabE, e->d_smallg, nrb, nullptr);
        hipError_t er = comm_bucket(e, 0);
        if (er != hipSuccess) return er;
    }
    {
        ScopedTimer tm(e, "k_vlatent_bwd");
        auto go = [&](auto kern, int nth) {
            hipLaunchKernelGGL(kern, dim3(e->n_lat_wg), dim3(nth), vlat_bwd_lds(e, lat16 ? 16 : 4), st, P, d, e->d_cells,
                               lat_covar, e->d_lat, e->d_dzp, bf ? nullptr : e->d_dhT_f, bf ? e->d_dhT_b : nullptr,
                               e->d_small);
        };
        if (lat16) go(k_vlatent_bwd<16>, 1024);
        else go(k_vlatent_bwd<4>, 256);
    }
    // world 1 (no split): the gradient kernels also write the clip norm's sum-of-squares partials
    const bool fuse_sq = !split && !(e->comm_active());
    const int gS = 1 + (SMALL + 31) / 32, gG = (d.D + VGG_GENES - 1) / VGG_GENES;
    double* sqS = fuse_sq ? e->d_sumsq : nullptr;
    double* sqG = fuse_sq ? e->d_sumsq + gS : nullptr;
    {
        // encoder backward + the small-parameter gradients / loss in one launch
        ScopedTimer tm(e, "k_enc_bwd");
        const int nenc = nrb * d.nsB;
        const T* dhT = reinterpret_cast<const T*>(bf ? (const void*)e->d_dhT_b : (const void*)e->d_dhT_f);
        const auto* WeT = reinterpret_cast<const typename WEnc<PM>::type*>(
            std::is_same<typename WEnc<PM>::type, __bf16>::value ? (const void*)e->d_WeP_b : (const void*)e->d_WeP_f);
        hipLaunchKernelGGL((k_enc_bwd_vsmall<PM, KP>), dim3(nenc + gS), dim3(256), (enc_bwd_lds<PM, KP, false>(d)), st, ent_list(e),
                           e->d_seg, e->d_toff, e->d_lat, dhT, (int64_t)KP * d.Bpad, WeT, d, e->d_slabE, nenc, sc,
                           e->d_small, e->n_lat_wg, G, e->d_smallg, e->d_rowv, e->d_lossp, e->n_lat_wg, e->d_vk,
                           e->d_out, sqS);
    }
    {
        ScopedTimer tm(e, "k_vgrad_genes");
        if (split)
            hipLaunchKernelGGL(k_vgrad_genes<2>, dim3(gG), dim3(256), 0, st, P, d, G, gene, e->d_WeP_f,
                               e->d_slabB, e->d_slabE, e->d_smallg, nrb, sqG);
        else
            hipLaunchKernelGGL(k_vgrad_genes<0>, dim3(gG), dim3(256), 0, st, P, d, G, gene, e->d_WeP_f,
                               e->d_slabB, e->d_slabE, e->d_smallg, nrb, sqG);
    }
    if (split) {
        hipError_t er = comm_bucket(e, 1);
        if (er != hipSuccess) return er;
        e->grads_reduced = e->comm_active();
    } else if (fuse_sq) {
        e->sq_parts = gS + gG;
    }
    return hipGetLastError();
}

template <class... A>
static hipError_t vmf_dispatch(Engine* e, A... a) {
    return dispatch_mode<false>(e, [&](auto p, auto kp) { return vmf_launch_all<decltype(p), decltype(kp)::value>(e, a...); });
}

// k_vprep (+ the staged block's copy): launched ahead of the batch lists
hipError_t vmf_prep(Engine* e, int64_t B, int64_t n_total, float beta) {
    if (e->frozen_dirty) {
        hipError_t er = vmf_prepare_frozen(e);
        if (er != hipSuccess) return er;
    }
    const Dims d = vmf_dims(e, B, n_total, beta);
    const VPtrs P = vmf_ptrs(e);
    const VScal sc = vmf_scal(e);
    const bool bf = e->cfg.dtype != MMVAE_DTYPE_F32;  // bf16 planes (bf16, x3)
    ScopedTimer tm(e, "k_vprep");
    hipLaunchKernelGGL(k_vprep, dim3((d.DP + 255) / 256 + 1, d.KP / 8), dim3(256), 0, e->stream, P, d, sc.epsD,
                       e->d_gene, e->d_WeP_f, e->d_WeS_f, bf ? e->d_WeS_b : nullptr, e->d_mvec, sc, e->d_vk,
                       stage_copy_args(e));
    return hipGetLastError();
}

hipError_t vmf_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps) {
    if (e->frozen_dirty) {
        hipError_t er = vmf_prepare_frozen(e);
        if (er != hipSuccess) return er;
    }
    const Dims d = vmf_dims(e, B, n_total, beta);
    return vmf_dispatch(e, d, vmf_ptrs(e), vmf_scal(e), update, use_eps, 0, (float*)nullptr,
                        (float*)nullptr);
}

hipError_t vmf_encode(Engine* e, int64_t B, float* d_mean, float* d_lnvar) {
    if (e->frozen_dirty) {
        hipError_t er = vmf_prepare_frozen(e);
        if (er != hipSuccess) return er;
    }
    const Dims d = vmf_dims(e, B, B, 1.f);
    return vmf_dispatch(e, d, vmf_ptrs(e), vmf_scal(e), false, false, 1, d_mean, d_lnvar);
}

}  // namespace mmvae
