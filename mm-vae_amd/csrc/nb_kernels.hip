// NB-VAE ELBO step on gfx950: hand-written HIP kernels for the reference's hot path
//   forward  nb.hh:403-508  (encode_mu, reparameterize, decode_mu, encode_nu, decode_nu, depth)
//   loss     nb.hh:510-548  (nllik_loss, kl_loss, loss)
//   backward (LibTorch autograd in the reference, mmvae_alg.hh:307) — hand-derived here; the
//            algebra is restated in oracle/nb_analytic.py and proven equal to autograd there.
//
// Data layout in HBM: dataset = cell-major CSR (int64 rowptr, int32 gene,
// f32 count); frozen encoder weight stored [KP][DP], frozen decoder weight stored both
// [DP][KP] (logit GEMM operand) and [KP][DP] (dz GEMM operand), bf16 or f32.  The dense
// [B,D] batch of the reference (mmvae_io.hh:208-245) is never materialised in HBM: every
// kernel densifies one 16-cell x 64-gene tile at a time into LDS from the CSR.
//
// Kernel chain per step (one stream):
//   k_prep        per-gene constants (softplus(ln_x_sd), bias sums), encoder mean term
//   k_enc_fwd     densify log1p(x)/sd tiles in LDS -> MFMA with the frozen encoder; the same
//                 entry walk accumulates the raw-x dots of depth / nu_enc per gene split
//   k_latent_fwd  K x K heads, clamp, reparameterise (Philox or injected eps), KL
//   k_dec<A>      logit GEMM (MFMA) + online max/sum-exp per cell        (pass A)
//   k_dec<B>      logit GEMM + softmax + NB likelihood + every gradient term that needs only
//                 the log-sum-exp; dz GEMM on MFMA from LDS-staged p*q, p  (pass B)
//   k_dec<C>      logit GEMM + exp + column sums weighted by the row term E_b (pass C)
//   k_latent_bwd  latent heads backward, KL grads, dh
//   k_enc_bwd     dh^T x log1p(x) tiles on MFMA -> ln_x_sd grad; raw-x column sums
//   k_grad_small / k_grad_genes   deterministic slab reductions -> flat gradient buffer
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"
#include "enc_bwd.hpp"

namespace mmvae {

struct NBPtrs {
    const float *xm, *lsd, *mub, *nub, *Wce, *bce, *Wm, *bm, *Wl, *bl, *Wcd, *bcd, *Wne, *bne, *Wnm,
        *bnm, *Wnl, *bnl, *Wnd, *bnd, *wdp, *bdp;
    const float *We, *be, *Wd, *bd;  // frozen (reference layouts: We [K][D], Wd [D][K])
    float* dbg_out;                  // diagnostics only (MMVAE_DBG stamps)
};

struct NBGrads {
    float *xm, *lsd, *mub, *nub, *Wce, *bce, *Wm, *bm, *Wl, *bl, *Wcd, *bcd, *Wne, *bne, *Wnm, *bnm,
        *Wnl, *bnl, *Wnd, *bnd, *wdp, *bdp;
};


// =======================================================================================
// k_enc_scale (fp8 mode) — the power-of-two scale of this step's e4m3 encoder image W / sd:
// amax(W / sd) <= max|W| / min_g sd_g, so scale = 2^floor(log2(448 / bound)) keeps every
// scaled value inside the e4m3 range (448); [0] = scale, [1] = 1 / scale (the accumulator's).
// =======================================================================================
__global__ __launch_bounds__(1024) void k_enc_scale(const float* __restrict__ lsd, int D, float wmax,
                                                   float* __restrict__ escale) {
    // min_g sd_g = softplus(min_g ln_x_sd_g) + 1e-4 (softplus is increasing): a plain min over
    // the genes, loads issued eight at a time per thread (independent accumulators)
    __shared__ float red[16];
    float m[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = INFINITY;
    for (int g0 = threadIdx.x; g0 < D; g0 += 8 * 1024) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int g = g0 + i * 1024;
            if (g < D) m[i] = fminf(m[i], lsd[g]);
        }
    }
    float v = fminf(fminf(fminf(m[0], m[1]), fminf(m[2], m[3])), fminf(fminf(m[4], m[5]), fminf(m[6], m[7])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 0; i < 16; ++i) v = fminf(v, red[i]);
        const float bound = wmax / (softplus_acc(v) + 1e-4f);
        const float sc = bound > 0.f ? exp2f(floorf(log2f(448.f / bound))) : 1.f;
        escale[0] = sc;
        escale[1] = 1.f / sc;
    }
}

// =======================================================================================
// k_prep — per-gene constants (nb.hh:408-410 softplus(ln_x_sd)+eps, nb.hh:440 bias terms,
// nb.hh:458 nu_dec bias - nu_bias) and the encoder's dense mean term
// mvec[k] = sum_g x_mean_g / (softplus(ln_x_sd_g) + 1e-4) * W_enc[k, g].
// =======================================================================================
__global__ __launch_bounds__(256) void k_prep(NBPtrs P, Dims d, float* gene, const float* __restrict__ WeP_f,
                                              float* __restrict__ WeS_f, __bf16* __restrict__ WeS_b,
                                              float* __restrict__ mvecp, StageCopy scp, uint8_t* __restrict__ WeS8,
                                              const float* __restrict__ escale) {
    // grid (genes / 256, KP / 8): every y-slice packs 8 latent rows of the scaled encoder weight
    // and writes its block's partial of mvec (mvec_partial; summed by k_latent_fwd).  Every load
    // is issued before the first store (clamped, unconditional: one in-order counter covers
    // loads and stores), the staged block's host-memory chunk last.
    const int g0 = blockIdx.x * 256 + threadIdx.x;
    const bool in = g0 < d.DP;
    const int g = in ? g0 : d.DP - 1;
    const bool v = g < d.D;
    const int gl = min(g, d.D - 1);
    const float lsd = P.lsd[gl];
    float wp[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) wp[kk] = WeP_f[(int64_t)(blockIdx.y * 8 + kk) * d.DP + g];
    const float xm = P.xm[gl], bd = P.bd[gl], bcd = P.bcd[gl], mub = P.mub[gl], bnd = P.bnd[gl], nub = P.nub[gl];
    const float wcd = P.Wcd[(int64_t)gl * d.C], wnd = P.Wnd[(int64_t)gl * d.R], wdp = P.wdp[gl], wne = P.Wne[gl];
    const float esc = WeS8 ? escale[0] : 1.f;
    StageHold sh;
    __builtin_amdgcn_sched_barrier(0);  // the host-memory load stays behind the others
    sh.load(scp);
    __builtin_amdgcn_sched_barrier(0);
    const float inv = v ? 1.f / (softplus_acc(lsd) + 1e-4f) : 0.f;
    if (blockIdx.y == 0 && in) {
        float bias = -INFINITY, cnu = 0.f, xmi = 0.f;
        if (v) {
            bias = bd + bcd + mub;
            cnu = bnd - nub;
            xmi = xm * inv;
        }
        gene[g] = inv;
        gene[d.DP + g] = bias;
        gene[2 * d.DP + g] = cnu;
        gene[3 * d.DP + g] = xmi;
        // packed decoder record (bias, cn, Wcd[g][0], Wnd[g][0])
        reinterpret_cast<float4*>(gene + 4 * d.DP)[g] = float4{bias, cnu, v ? wcd : 0.f, v ? wnd : 0.f};
        // packed raw-count dot weights (depth.weight, nu_encoding.weight row 0) for the batch
        // lists' dots (batch.hip): one 8-byte gather per entry
        reinterpret_cast<float2*>(gene + 8 * d.DP)[g] = float2{v ? wdp : 0.f, v ? wne : 0.f};
    }
    // encoder weight pre-scaled by 1/(softplus(ln_x_sd)+1e-4): x~ W^T = log1p(x) (W inv)^T - mvec
    const float xmv = (in && v) ? xm : 0.f;
    float mp[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const int k = blockIdx.y * 8 + kk;
        const float ws = inv * wp[kk];
        if (in) {  // bf16 image: hi plane, and the x3 mode's lo plane KP * DP elements after it
            if (WeS_b) put_op<X3>(WeS_b, (int)((int64_t)k * d.DP + g), d.KP * d.DP, ws);
            else WeS_f[(int64_t)k * d.DP + g] = ws;
            // fp8 mode: the forward GEMM's e4m3 image (the bf16 one stays for the backward)
            if (WeS8) WeS8[(int64_t)k * d.DP + g] = to_t<uint8_t>(ws * esc);
        }
        mp[kk] = xmv * ws;  // x_mean_g / sd_g * W_enc[k, g]
    }
    mvec_partial(mp, mvecp, d.KP, blockIdx.y * 8);
    sh.store(scp);
}

// =======================================================================================
// k_enc_fwd — mu encoder (nb.hh:410-411) on MFMA.  x~ W^T = log1p(x) (W/sd)^T - mvec, so only
// the nonzeros are densified.  Workgroup = 64 cells x one gene split; per 64-gene tile the
// pre-scaled frozen weight tile ([KP][DP], k_prep) is register-staged once per workgroup into
// LDS (double-buffered, swizzled), while each wave scatters its 16 cells' log1p(x) for the
// NEXT tile from the batch entry lists (tiles t+1, t+2 prefetched, entries balanced over the
// lanes) into a wave-private 16x64 LDS tile.  Partial h per gene split -> hpart.  (The raw-count
// dots of depth / nu_enc, nb.hh:448, 498, are taken by k_batch_lists, which visits every entry
// with its row known.)
// =======================================================================================
// SB (x3): single-buffered x tile and W stage — the wave's scatter into its x tile follows
// its own MFMA operand reads of the tile (one wave's LDS operations complete in order), and the
// W stage is rewritten between two barriers — so x3 fits 4 workgroups per CU (39 KB) instead of 2.
// NW waves (16 rows each) per workgroup: 8 in the x3 mode (the staged W tile serves 128 rows,
// two workgroups per CU), 4 otherwise
// W stage buffers of k_enc_fwd: 2 (double-buffered, one barrier per tile) in every mode; the x3
// mode's single-buffered x tiles keep its two 8-wave workgroups per CU with both W stages (75 KB)
#ifndef MMVAE_ENC_NBW
#define MMVAE_ENC_NBW 2
#endif
template <class P, int KP, bool SB = false, int NW = 4>
__global__ __launch_bounds__(64 * NW) void k_enc_fwd(EntList ents, const int64_t* __restrict__ seg,
                                                 const int32_t* __restrict__ toff,
                                                 const typename Elem<P>::type* __restrict__ WeS, int64_t wplane, Dims d,
                                                 float* __restrict__ hpart, const float* __restrict__ oscale) {
    using T = typename Elem<P>::type;
    using M = MM<P>;
    using Fr = typename M::frag;
    constexpr bool X = IsX3<P>::value;
    constexpr int NPL = X ? 2 : 1;                 // operand planes (x3: hi + lo)
    constexpr int XS = sizeof(T) == 4 ? 68 : 80;   // x tile row stride (elements): conflict-free
    constexpr int RB = 64 * (int)sizeof(T);        // staged W row = 64 genes of one latent
    constexpr int STB = KP * RB;
    constexpr int XT = 16 * XS;                    // elements of one x tile plane
    constexpr int NB = SB ? 1 : 2;                 // x tiles per wave
    constexpr int NBW = MMVAE_ENC_NBW;             // W stage buffers (2: one barrier per tile)
    constexpr int XB = NB * NPL * XT * (int)sizeof(T);  // per wave: x tiles [hi 0][hi 1][lo 0][lo 1]
    constexpr int XPL = NB * XT;                   // x plane stride (elements)
    using Tab = Log1pTab<P, SB ? 512 : LTAB>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint64_t t_entry = dbg_bit(d.dbg, 32) ? stamp_now() : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int sp = blockIdx.x % d.nsE, rb = blockIdx.x / d.nsE;
    const int row0 = rb * 16 * NW + 16 * w;
    const int t0 = sp * d.tpsE, t1 = min(d.NT, t0 + d.tpsE);
    const int S = d.tpsE + 1;
    const EncLds L(KP, (int)sizeof(T), S, XB, 0, NPL, Tab::BYTES, NBW, NW);
    char* wst = smem;
    uint32_t* ltab = reinterpret_cast<uint32_t*>(smem + L.o_tab);
    Tab::fill(ltab);
    T* xt = reinterpret_cast<T*>(smem + L.o_x + w * XB);
    int32_t* toffl = reinterpret_cast<int32_t*>(smem + L.o_toff) + w * S;

    DualStage<KP, RB, 64 * NW, X> wreg;
    auto wsrc = [&](int t) { return reinterpret_cast<const char*>(WeS) + (int64_t)64 * t * sizeof(T); };
    // prologue loads with no dependence on the lists go out first (W tile t0)
    wreg.load(wsrc(min(t0, d.NT - 1)), (int64_t)d.DP * sizeof(T), wplane * (int64_t)sizeof(T));
    const int wbk = row0 >> 4;
    fill_toffl(toffl, S, t0, d.NT, toff, wbk, lane);
    const int64_t segw = seg[wbk];
    auto zero_tile = [&](T* x0) {
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
            for (int i = lane; i < XT * (int)sizeof(T) / 16; i += 64)
                reinterpret_cast<uint4*>(x0 + pl * XPL)[i] = uint4{0, 0, 0, 0};
    };
    zero_tile(xt);
    if constexpr (Tab::ON) __syncthreads();  // the table
    else wave_sync();
    auto scatter = [&](const ListEntries& le, T* dst) {
        le.visit(ents, lane, [&](int r, int gl, float x) { Tab::put(ltab, dst, r * XS + gl, XPL, x); });
    };

    f32x4 acc[KP / 16];
#pragma unroll
    for (int lb = 0; lb < KP / 16; ++lb) acc[lb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nt = t1 - t0;
    // tile t + 1's entries come from one of two register sets, fetched two tiles ahead; the loop
    // is unrolled by two so neither set is ever copied (a loop-carried copy of a register with a
    // load in flight makes the compiler wait for that load at the loop latch)
    ListEntries qA, qB;
    // each x tile buffer is cleared only where its last scatter wrote (whole tile past 128 entries)
    int zp[NB][2];
    bool zall[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        zp[b][0] = zp[b][1] = -1;
        zall[b] = true;
    }
    auto keep = [&](const ListEntries& le, int b) {
        zp[b][0] = le.pos(0, lane);
        zp[b][1] = le.pos(1, lane);
        asm volatile("" : "+v"(zp[b][0]), "+v"(zp[b][1]));  // taken now: le is refetched next
        zall[b] = le.n > 128;
    };
    auto clear = [&](T* x0, int b) {
        if (zall[b]) {
            zero_tile(x0);
        } else {
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (zp[b][k] >= 0) {
                    const int idx = (zp[b][k] >> 6) * XS + (zp[b][k] & 63);
                    x0[idx] = T{};
                    if constexpr (NPL == 2) x0[idx + XPL] = T{};
                }
        }
    };
    if (t0 < t1) {
        ListEntries first;  // every prologue load is issued before the first wait
        first.fetch(ents, segw, toffl, 0, lane);
        qA.fetch(ents, segw, toffl, min(1, nt - 1), lane);
        qB.fetch(ents, segw, toffl, min(2, nt - 1), lane);
        wreg.store(wst, NBW * STB);
        scatter(first, xt);
        keep(first, 0);
    }
    lds_barrier();
    const bool stamps = dbg_bit(d.dbg, 32);
    uint64_t sa = 0, sb = 0, sc = 0, sd = 0, tp = stamps ? stamp_now() : 0;
    auto lap = [&](uint64_t& acc_) {
        if (stamps) {
            const uint64_t tn = stamp_now();
            acc_ += tn - tp;
            tp = tn;
        }
    };
    // q: tile t + 1's entries; buf: the x tile buffer holding tile t; wb: the W stage holding it
    auto tile = [&](int t, ListEntries& q, int buf, int wb) {
        const int tl = t - t0;
        // unconditional (clamped) prefetch of the next weight tile: counted vmcnt waits
        wreg.load(wsrc(min(t + 1, t1 - 1)), (int64_t)d.DP * sizeof(T), wplane * (int64_t)sizeof(T));
        const T* xb = xt + buf * XT;
#pragma unroll
        for (int s = 0; s < 64 / M::KSTEP; ++s) {
            const Fr a = M::load(&xb[(lane & 15) * XS + s * M::KSTEP + (lane >> 4) * M::EPL], XPL);
#pragma unroll
            for (int lb = 0; lb < KP / 16; ++lb) {
                const Fr bw = M::load(reinterpret_cast<const T*>(
                    wst + wb * STB + swz_off<RB>(16 * lb + (lane & 15), (s * M::KSTEP + (lane >> 4) * M::EPL) * (int)sizeof(T))),
                    NBW * STB / (int)sizeof(T));
                acc[lb] = M::mma(a, bw, acc[lb]);
            }
        }
        lap(sa);
        const int nb = SB ? 0 : (buf ^ 1);
        T* xn = xt + nb * XT;
        if (t + 1 < t1) {
            clear(xn, nb);  // SB: after this wave's own operand reads of it (LDS is in order)
            wave_sync();
            scatter(q, xn);
            keep(q, nb);
        }
        lap(sb);
        q.fetch(ents, segw, toffl, min(tl + 3, nt - 1), lane);  // the loads stay in flight across the barriers
        if constexpr (NBW == 1) {
            lds_barrier();  // every wave's reads of this W stage done
            if (t + 1 < t1) wreg.store(wst, STB);
        } else if (t + 1 < t1) {
            // the other stage: every wave read it in tile t - 1, before that tile's last barrier
            wreg.store(wst + (wb ^ 1) * STB, NBW * STB);
        }
        lap(sc);
        lds_barrier();
        lap(sd);
    };
    for (int t = t0; t < t1; t += 2) {
        tile(t, qA, 0, 0);
        if (t + 1 < t1) tile(t + 1, qB, SB ? 0 : 1, NBW == 2 ? 1 : 0);
    }
    if (stamps) {  // diagnostic build: per-wave phase cycles into hpart (outputs invalid)
        const uint64_t t_loop_end = stamp_now();
        vm_wait_all();
        __syncthreads();
        if (lane == 0) {
            float* o = hpart + ((int64_t)blockIdx.x * NW + w) * 8;
            o[0] = (float)sa;
            o[1] = (float)sb;
            o[2] = (float)sc;
            o[3] = (float)sd;
            o[4] = (float)(t_loop_end - t_entry - (sa + sb + sc + sd));  // prologue + tail
            o[5] = (float)(t_entry & 0xffffffu);                          // entry time (low bits)
            o[6] = (float)(t_loop_end - t_entry);
        }
        return;
    }
    // fp8 mode: the e4m3 weight image carries the step's power-of-two scale (k_enc_scale)
    const float osc = IsF8<P>::value ? oscale[1] : 1.f;
#pragma unroll
    for (int lb = 0; lb < KP / 16; ++lb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            hpart[((int64_t)sp * d.Bpad + row0 + 4 * (lane >> 4) + r) * KP + 16 * lb + (lane & 15)] = acc[lb][r] * osc;
}

// =======================================================================================
// k_latent_fwd — the K x K heads and the reparameterisation for LAT_CELLS = 16 cells per
// workgroup (lane = latent k; NW waves, each owning 16 / NW cells):
//   h = mu_enc(x~) (+ frozen bias), mean = mu_repr_mean(h) + covar_enc(c) (nb.hh:412-416),
//   lnvar = clamp(mu_repr_lnvar(h), -4, 4), z = mean + eps*exp(lnvar/2) (nb.hh:462-472),
//   nu path (nb.hh:444-451, 489-492), depth d = softplus(pre) (nb.hh:498), KL terms (nb.hh:533-537).
// The heads are [16 cells x K] x [K x K] products on f32 MFMA (waves 0..3), h from an LDS
// [cell][k] image.
//   mode 1 = recorder encode_mu(x) (nb.hh:419-431): no covariate, writes mean/lnvar out.
// NW = 16 (one cell per wave, 1024 threads): the kernel is a chain of memory rounds, and one
// wave per SIMD with 4 cells each leaves most of each round's loads queued behind the wave's
// load counter; 16 waves per CU keep every cell's loads in flight at once.  It has no frozen
// hidden chains (those run the NW = 4 instance, whose chain layers assume 256 threads).  Every
// global load is issued before the first global store (one in-order counter covers both).
// =======================================================================================
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_latent_fwd(
    NBPtrs P, Dims d, const int64_t* __restrict__ cells, const float* __restrict__ covar,
    const float* __restrict__ hpart, const float* __restrict__ mvec, const float* __restrict__ rowxp,
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
    __shared__ __attribute__((aligned(16))) float sH[LAT_CELLS * 68];  // [cell][k]
    __shared__ float sred[NW];
    __shared__ float sRX[LAT_CELLS][1 + HMAX];  // depth pre-activation, nu_enc(x)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = lane;
    const int cw = CPW * w;                     // this wave's first cell in the workgroup
    const int bw = blockIdx.x * LAT_CELLS + cw;  // ... in the batch
    // diagnostic (MMVAE_DBG & 2048): realtime stamps of the phases into P.dbg_out (outputs invalid)
    const bool rts = dbg_bit(d.dbg, 2048) && mode == 0;
    uint64_t rt_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto mark = [&](int i_) {  // constant index at every call: rt_ stays in registers
        if (rts) rt_[i_] = realtime_now();
    };
    mark(0);
    // every global input first, waits in issue order (one memory round, plus one for the loads
    // that depend on a cell id); the per-cell loop below then only stores
    HeadsStage<64 * NW> hst;
    hst.issue(P.Wm, P.Wl, K, E);
    const int nqx = 1 + d.H;
    float xs[CPW];  // raw-count dots (k_batch_lists), lanes < 1 + H
    split_sum<CPW>(rowxp, 1, (int64_t)d.Bpad * nqx, (int64_t)bw * nqx + (k < nqx ? k : 0), nqx, k < nqx, xs);
    float hs[CPW];  // the encoder's gene-split partials of h
    split_sum<CPW>(hpart, d.nsE, (int64_t)d.Bpad * d.KP, (int64_t)bw * d.KP + k, d.KP, k < KE, hs);
    // per-lane parameters (clamped, unconditional loads)
    const int kk = min(k, K - 1), kr = min(k, d.R - 1), ke = min(k, KE - 1);
    const float p_bx = (k == 0) ? P.bdp[0] : P.bne[min(max(k - 1, 0), d.H - 1)];  // raw-count dot bias
    const float p_be = P.be[ke], p_bm = P.bm[kk], p_bl = P.bl[kk];
    const float p_bce = P.bce[kk], p_wce = P.Wce[(int64_t)kk * d.C];
    const float p_bnm = P.bnm[kr], p_bnl = P.bnl[kr];
    float p_wnm[HMAX], p_wnl[HMAX];
#pragma unroll
    for (int hh = 0; hh < HMAX; ++hh) {
        p_wnm[hh] = P.Wnm[kr * d.H + min(hh, d.H - 1)];
        p_wnl[hh] = P.Wnl[kr * d.H + min(hh, d.H - 1)];
    }
    // rows past this batch (b >= B): the handle-wide grid covers them, but the lists / encoder
    // wrote their partials only up to pad_rows(B) — whatever the buffers hold there is dropped
#pragma unroll
    for (int c = 0; c < CPW; ++c)
        if (bw + c >= d.B) hs[c] = xs[c] = 0.f;
    int pbv[CPW];
    float cmv[CPW], epv[CPW], enp[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        const bool valid = b < d.B;
        pbv[c] = (perm && valid) ? perm[b] : b;  // original batch position: the noise key
        float cm = 0.f;
        if (k < K && mode == 0) {
            cm = p_bce;
            if (!covar) {  // unit covariate (Engine::unit_covar): c = 1, padding rows (row N) 0
                cm += valid ? p_wce : 0.f;
            } else {
                const int64_t cell = cells[b];  // padding rows hold the empty row N
                for (int q = 0; q < d.C; ++q) cm += P.Wce[k * d.C + q] * covar[cell * d.C + q];
            }
        }
        cmv[c] = cm;
        epv[c] = (eps_in && k < K && valid) ? eps_in[(int64_t)pbv[c] * K + k] : 0.f;
        enp[c] = (eps_in && k < d.R && valid) ? eps_in[(int64_t)d.B * K + (int64_t)pbv[c] * d.R + k] : 0.f;
    }
    // h = sum of the encoder's gene-split partials - mvec + bias (mvec: all threads, LDS combine)
    const float mvk = mvec_sum(mvec, d.nmv, d.KP, k);
    if (!CHAINS || d.nce == 0) hst.store(K, E, sWm, sWl);  // (with an encoder chain: after it, sWm stages its W)
    mark(1);
    {
        // raw-count dots (+ bias) -> sRX, and rowx for k_latent_bwd
        if (k < nqx) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                const float v = xs[c] + p_bx;
                sRX[cw + c][k] = v;
                if (mode == 0) rowx[(int64_t)(bw + c) * d.rowx_stride + (k == 0 ? 0 : 1 + k)] = v;
            }
        }
    }
    const float hb = (k < KE) ? p_be - mvk : 0.f;
    mark(2);
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const float hv = hb + hs[c];  // mu_enc Linear output; --relu appends ReLU(inplace) (nb.hh:345-346)
        sH[(cw + c) * 68 + k] = (k < KE) ? (d.relu ? fmaxf(hv, 0.f) : hv) : 0.f;
    }
    __syncthreads();
    // the frozen encoder chain (hidden mu_encoding_l, l >= 2: nb.hh:331-340) -> the heads' input
    __shared__ float sZ[CHAINS ? 2 : 1][LAT_CELLS * 68];
    const float* hin = sH;
    if constexpr (CHAINS) {
        if (d.nce > 0) {
            hin = chain_run(d, 0, d.nce, sH, sZ[0], sZ[CHAINS ? 1 : 0], false, sWm, w, lane);
            hst.store(K, E, sWm, sWl);
            __syncthreads();
        }
    }
    // heads on f32 MFMA (nb.hh:412-416), transposed back to lane = latent through LDS
    __shared__ float sM[LAT_CELLS * 68], sA[LAT_CELLS * 68];
    if (w < 4) heads_fwd(hin, sWm, sWl, K, E, w, lane, sM, sA);
    __syncthreads();
    mark(3);
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
        const int pb = pbv[c];
        float* L = lat + (int64_t)b * d.lat_stride;
        float mn = mean[c] + cmv[c], a = av[c];
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
        if (k < K && b < d.B)
            eps = eps_in ? epv[c] : (dbg_bit(d.dbg, 4096) ? 0.f : philox_normal(seed, step, row_offset + pb, k));  // 4096: diagnostic
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
        // ---- overdispersion latent (lanes r < R) ----
        const float* rx = &sRX[cw + c][0];  // [0] = depth pre-activation, [1 + h] = nu_enc_h
        if (k < d.R) {
            float nm = p_bnm, an = p_bnl;
#pragma unroll
            for (int hh = 0; hh < HMAX; ++hh)
                if (hh < d.H) {
                    nm += p_wnm[hh] * rx[1 + hh];
                    an += p_wnl[hh] * rx[1 + hh];
                }
            const float nlv = fminf(fmaxf(an, -4.f), 4.f);
            float en = 0.f;
            if (b < d.B)
                en = eps_in ? enp[c] : (dbg_bit(d.dbg, 4096) ? 0.f : philox_normal(seed, step, row_offset + pb, NU_LANE + k));
            const float zn = nm + en * expf(nlv / 2.f);
            L[d.LAT_NMEAN + k] = nm;
            L[d.LAT_AN + k] = an;
            L[d.LAT_EPSN + k] = en;
            L[d.LAT_ZNU + k] = valid ? zn : 0.f;
            if (valid) kl += 1.f + nlv - nm * nm - expf(nlv);
        }
        if (k == 0) {
            const float pre = rx[0];
            const float dd = softplus_acc(pre);
            L[d.LAT_D] = dd;
            L[d.LAT_W] = valid ? dd * d.inv_n : 0.f;
            L[d.LAT_VALID] = valid ? 1.f : 0.f;
        }
    }
    if (mode == 1) return;
    if constexpr (CHAINS) {
        if (d.ncd > 0) {
            // the frozen decoder chain (mu_decoding_l + ReLU with --relu, nb.hh:362-379): z -> zd,
            // the big decoder GEMM's input
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
    mark(4);
    kl = wave_sum(kl);
    if (lane == 0) sred[w] = kl;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        if constexpr (NW == 4) {
            t = (sred[0] + sred[1]) + (sred[2] + sred[3]);
        } else {
#pragma unroll
            for (int i = 0; i < NW; i += 4) t += (sred[i] + sred[i + 1]) + (sred[i + 2] + sred[i + 3]);
        }
        klpart[blockIdx.x] = -0.5f * t;
    }
    if (rts) {
        vm_wait_all();
        mark(5);
        if (lane == 0) {
            float* o = P.dbg_out + ((int64_t)blockIdx.x * NW + w) * 8;
            for (int i = 0; i < 6; ++i) o[i] = (float)(rt_[i] & 0xffffffu);
            o[6] = o[5];
            o[7] = (float)wave_place();
        }
    }
}

// =======================================================================================
// Decoder (nb.hh:433-442, 453-460, 510-531).  Three passes over the [B, D] logit matrix,
// which is never stored: the softmax backward needs the row sum E_b = sum_g P q, which is
// known only after a full sweep of the row.
//   k_dec<PASS 0> (A): online max / sum-exp per cell                      -> lsep[split][cell]
//   k_dec_nb     (B): softmax + NB terms + dz GEMM + column sums          (see below)
//   k_dec<PASS 2> (C): column sums of w_b E_b p_bg (the E_b P term of the softmax backward)
// Lane l holds, per 16-gene block, gene (l & 15) of cells 4(l>>4)+r, r = 0..3 (MFMA C layout).
// =======================================================================================
struct DecPtrs {
    const float* lat;
    const float* zf;
    const __bf16* zb;
    const float* gene;  // inv, bias, cnu  [3][DP]
    const float* Wcd;   // covar_decoding.weight [D][C]
    const float* Wnd;   // nu_decoding.weight [D][R]
    const float* covar;
    const int64_t* cells;
    const int64_t* rowptr;
    const int32_t* col;
    const float* val;
    const int32_t* rtp;
    const void* WdP;  // [DP][KP] T
    const void* WdT;  // [KP][DP] T
    float* lsep;      // [nsA][Bpad][2]
    float* rowfin;    // [Bpad][2]: lse (log2 units), published by k_dec_nb for pass C
    float* rowB;      // [nsD][Bpad][2+R]
    float* dzp;       // [nsD][Bpad][2][KP]
    float* slabB;     // [nrb][nqB][DP]
    float* slabC;     // [nrb][1+C][DP]
    float* lossp;     // [grid]
    EntList ents;          // per-step batch entry lists (batch.hip)
    const int64_t* seg;    // [Bpad/16 + 1]
    const int32_t* toff;   // [Bpad/16][NT+1]
    int64_t zplane;        // x3 mode: element offset of the lo plane of zb
    int64_t wplane;        // x3 mode: element offset of the lo planes of WdP / WdT
};

// Passes A and C: each tile's decoder rows + gene records are staged ONCE per workgroup into
// LDS (register-staged, double-buffered, swizzled image) and shared by the four waves; a wave
// owns 32 rows (two 16-row MFMA blocks), so every W fragment read from LDS feeds two MFMAs.
// Workgroup = 128 rows x one gene split.
#ifndef MMVAE_PASSC_PIPE
#define MMVAE_PASSC_PIPE 0  // 1: block gb + 1's logits issued ahead of block gb's element math (A/B: no gain)
#endif
static constexpr int AC_RPW = 2;  // 16-row MFMA blocks per wave
template <class P, int KP, int PASS, int CM>
MMVAE_DEV void dec_ac_body(DecPtrs Q, Dims d) {
    using T = typename Elem<P>::type;
    using M = MM<P>;
    using Fr = typename M::frag;
    constexpr bool X = IsX3<P>::value;
    constexpr bool F8M = IsF8<P>::value;     // fp8 logits: z from f32, W_dec pre-scaled e4m3
    constexpr int NPL = X ? 2 : 1;
    constexpr int KS = KP / M::KSTEP;
    constexpr bool BF = sizeof(T) == 2;
    constexpr int RB = KP * (int)sizeof(T);  // bytes per staged gene row
    constexpr int WIMG = 64 * RB;            // one W image plane
    constexpr int STB = NPL * WIMG + 1024;   // one stage buffer: W tile (hi [+ lo]) + grec tile
    constexpr int J = AC_RPW;
    constexpr int WR = 16 * J;               // rows per wave
    constexpr float L2E = 1.4426950408889634f;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint64_t rt_entry = dbg_bit(d.dbg, 256) ? realtime_now() : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int sp = blockIdx.x % d.nsA, rbw = blockIdx.x / d.nsA;
    const int row0 = rbw * 4 * WR + WR * w;
    const int t0 = sp * d.tpsA, t1 = min(d.NT, t0 + d.tpsA);
    // CM = 0: unit covariate (Engine::unit_covar, C = 1): the covariate Linear folds into the
    // gene's bias, and its weight gradient's column sums are the bias gradient's
    constexpr int CA = CM > 0 ? CM : 1;  // covariate array extent
    const int C = (CM <= 1) ? 1 : d.C;
    const int nq = 1 + C;
    char* stg = smem;
    float* part = reinterpret_cast<float*>(smem + 2 * STB);  // C: [2][4][nq][64]; prologue: [4 WR]
    const T* Z = BF ? reinterpret_cast<const T*>(Q.zb) : reinterpret_cast<const T*>(Q.zf);
    const char* WdPc = reinterpret_cast<const char*>(Q.WdP);
    const float4* grec = reinterpret_cast<const float4*>(Q.gene + 4 * d.DP);

    if (PASS == 2) {  // w_b E_b from pass B's per-split row sums, 4 threads per row
        for (int rr0 = 0; rr0 < 4 * WR; rr0 += 64) {
            const int rr = rr0 + (threadIdx.x >> 2), pp = threadIdx.x & 3;
            const int b = rbw * 4 * WR + rr;
            float E = 0.f;
            for (int s2 = pp; s2 < d.nsD; s2 += 4) E += Q.rowB[((int64_t)s2 * d.Bpad + b) * (2 + d.R)];
            E += __shfl_xor(E, 1, 64);
            E += __shfl_xor(E, 2, 64);
            if (pp == 0) part[rr] = Q.lat[(int64_t)b * d.lat_stride + d.LAT_W] * E;
        }
        __syncthreads();
    }
    Fr zfr[J][KS];
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int64_t zo = (int64_t)(row0 + 16 * j + (lane & 15)) * KP + s * M::KSTEP + (lane >> 4) * M::EPL;
            if constexpr (F8M) zfr[j][s] = M::load_f32(Q.zf + zo);
            else zfr[j][s] = M::load(&Z[zo], Q.zplane);
        }
    const float ainv = F8M ? d.inv_wscale : 1.f;  // logit accumulator unscale (fp8 W_dec)
    float lse2[J][4], wE[J][4], crow[J][4][CA], mrun[J][4], srun[J][4];
#pragma unroll
    for (int j = 0; j < J; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int b = row0 + 16 * j + 4 * (lane >> 4) + r;
            const int64_t cell = Q.cells[b];  // padding rows hold the empty row N
#pragma unroll
            for (int c = 0; c < CM; ++c) crow[j][r][c] = (c < C) ? Q.covar[cell * C + c] : 0.f;  // row N: zeros
            lse2[j][r] = (PASS == 2) ? Q.rowfin[2 * b] : 0.f;  // written by k_dec_nb (split 0)
            wE[j][r] = (PASS == 2) ? part[WR * w + 16 * j + 4 * (lane >> 4) + r] : 0.f;
            mrun[j][r] = -1e30f;
            srun[j][r] = 0.f;
        }
    if (PASS == 2) __syncthreads();  // part is reused for the column partials below
    // Register-staged decoder tiles, two in flight: tile t + 2 is loaded while tile t is
    // computed from LDS, tile t + 1 (loaded an iteration earlier) is written to the other LDS
    // buffer at the end — one LDS barrier per tile, no vmcnt(0) drain of a fresh DMA.
    using WStage = DualStage<64, RB, 256, X>;
    WStage wrA, wrB;
    float4 grA = float4{0.f, 0.f, 0.f, 0.f}, grB = grA;
    auto ld = [&](WStage& R, float4& G, int t) {
        R.load(WdPc + (int64_t)64 * t * RB, RB, Q.wplane * (int64_t)sizeof(T));
        if (threadIdx.x < 64) G = grec[64 * t + threadIdx.x];
    };
    auto st = [&](const WStage& R, const float4& G, int buf) {
        R.store(stg + buf * STB, WIMG);
        if (threadIdx.x < 64) reinterpret_cast<float4*>(stg + buf * STB + NPL * WIMG)[threadIdx.x] = G;
    };
    // diagnostic (MMVAE_DBG & 256): per-wave phase cycles into slabC (outputs invalid)
    const bool stamps = dbg_bit(d.dbg, 256);
    uint64_t st_[4] = {0, 0, 0, 0}, tp_ = 0;
    auto lap = [&](int i_) {
        if (stamps) {
            const uint64_t tn = stamp_now();
            st_[i_] += tn - tp_;
            tp_ = tn;
        }
    };
    auto tile = [&](int t, WStage& hold, float4& ghold, WStage& nxt, float4& gnxt) {
        const int buf = (t - t0) & 1;
        ld(nxt, gnxt, min(t + 2, t1 - 1));  // unconditional (clamped): counted waits
        const char* sb = stg + buf * STB;
        if (PASS == 0) {
            // online log-sum-exp in log2 units with one rescale per tile: the lane's 4 genes of
            // the tile (one per 16-gene block) are reduced to their max first
            f32x4 acc[4][J];
#pragma unroll
            for (int gb = 0; gb < 4; ++gb) {
                const int gl = 16 * gb + (lane & 15);
#pragma unroll
                for (int j = 0; j < J; ++j) acc[gb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const Fr bw = M::load(reinterpret_cast<const T*>(sb + swz_off<RB>(gl, (s * M::KSTEP + (lane >> 4) * M::EPL) * (int)sizeof(T))),
                                          WIMG / (int)sizeof(T));
#pragma unroll
                    for (int j = 0; j < J; ++j) acc[gb][j] = M::mma(zfr[j][s], bw, acc[gb][j]);
                }
            }
            lap(3);
            float b2[4], w2[4][CA];
#pragma unroll
            for (int gb = 0; gb < 4; ++gb) {
                const int gl = 16 * gb + (lane & 15);
                const float4 g4 = reinterpret_cast<const float4*>(sb + NPL * WIMG)[gl];
                b2[gb] = (CM == 0 ? g4.x + g4.z : g4.x) * L2E;  // padded genes: -inf
                w2[gb][0] = g4.z * L2E;
#pragma unroll
                for (int c = 1; c < CM; ++c)
                    w2[gb][c] = (c < C && 64 * t + gl < d.D) ? Q.Wcd[(int64_t)(64 * t + gl) * C + c] * L2E : 0.f;
            }
            // rows 2h, 2h + 1 as one packed-f32 pair
#pragma unroll
            for (int j = 0; j < J; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    f2 l2[4];
#pragma unroll
                    for (int gb = 0; gb < 4; ++gb) {
                        f2 v = splat2(b2[gb]);
#pragma unroll
                        for (int c = 0; c < CM; ++c) v = fma2(f2{crow[j][2 * h][c], crow[j][2 * h + 1][c]}, splat2(w2[gb][c]), v);
                        l2[gb] = fma2(f2{acc[gb][j][2 * h], acc[gb][j][2 * h + 1]}, splat2(L2E * ainv), v);
                    }
                    f2 mo = f2{mrun[j][2 * h], mrun[j][2 * h + 1]}, mn;
                    mn.x = fmaxf(mo.x, fmaxf(fmaxf(l2[0].x, l2[1].x), fmaxf(l2[2].x, l2[3].x)));
                    mn.y = fmaxf(mo.y, fmaxf(fmaxf(l2[0].y, l2[1].y), fmaxf(l2[2].y, l2[3].y)));
                    const f2 dm = mo - mn;
                    f2 sacc = f2{srun[j][2 * h], srun[j][2 * h + 1]} * f2{fexp2(dm.x), fexp2(dm.y)};
#pragma unroll
                    for (int gb = 0; gb < 4; ++gb) {
                        const f2 e2 = l2[gb] - mn;
                        sacc += f2{fexp2(e2.x), fexp2(e2.y)};
                    }
                    srun[j][2 * h] = sacc.x;
                    srun[j][2 * h + 1] = sacc.y;
                    mrun[j][2 * h] = mn.x;
                    mrun[j][2 * h + 1] = mn.y;
                }
        } else {
        // pass C: gene block gb + 1's logit MFMAs are issued ahead of block gb's element math
        auto logits = [&](int gb, f32x4 (&acc)[J]) {
            const int gl = 16 * gb + (lane & 15);
#pragma unroll
            for (int j = 0; j < J; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const Fr bw = M::load(reinterpret_cast<const T*>(sb + swz_off<RB>(gl, (s * M::KSTEP + (lane >> 4) * M::EPL) * (int)sizeof(T))),
                                      WIMG / (int)sizeof(T));
#pragma unroll
                for (int j = 0; j < J; ++j) acc[j] = M::mma(zfr[j][s], bw, acc[j]);
            }
        };
        f32x4 accn[J];
        if (MMVAE_PASSC_PIPE) logits(0, accn);
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
            const int gl = 16 * gb + (lane & 15);
            f32x4 acc[J];
#pragma unroll
            for (int j = 0; j < J; ++j) acc[j] = accn[j];
            if (MMVAE_PASSC_PIPE && gb + 1 < 4) logits(gb + 1, accn);
            if (!MMVAE_PASSC_PIPE) logits(gb, acc);
            const float4 g4 = reinterpret_cast<const float4*>(sb + NPL * WIMG)[gl];
            const float gx = CM == 0 ? g4.x + g4.z : g4.x;  // unit covariate: folded into the bias
            float wcd[CA];
            wcd[0] = g4.z;
#pragma unroll
            for (int c = 1; c < CM; ++c) wcd[c] = (c < C && 64 * t + gl < d.D) ? Q.Wcd[(int64_t)(64 * t + gl) * C + c] : 0.f;
            {  // pass C: rows 2h, 2h + 1 as one packed-f32 pair
                f2 csp[1 + CA];
#pragma unroll
                for (int c = 0; c < 1 + CA; ++c) csp[c] = splat2(0.f);
#pragma unroll
                for (int j = 0; j < J; ++j)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        f2 lg = fma2(f2{acc[j][2 * h], acc[j][2 * h + 1]}, splat2(ainv), splat2(gx));
#pragma unroll
                        for (int c = 0; c < CM; ++c) lg = fma2(f2{crow[j][2 * h][c], crow[j][2 * h + 1][c]}, splat2(wcd[c]), lg);
                        const f2 ex = fma2(lg, splat2(L2E), -f2{lse2[j][2 * h], lse2[j][2 * h + 1]});
                        const f2 wp = f2{wE[j][2 * h], wE[j][2 * h + 1]} * f2{fexp2(ex.x), fexp2(ex.y)};
                        csp[0] += wp;
#pragma unroll
                        for (int c = 0; c < CM; ++c) csp[1 + c] = fma2(wp, f2{crow[j][2 * h][c], crow[j][2 * h + 1][c]}, csp[1 + c]);
                    }
                float cs[1 + CA];
#pragma unroll
                for (int c = 0; c < 1 + CA; ++c) cs[c] = csp[c].x + csp[c].y;
                if (CM == 0) cs[1] = cs[0];  // sum_b w_b E_b p c_b with c_b = 1
                // per-wave partial of this tile (fixed-order combine after the tile barrier)
                float* pw = part + ((buf * 4 + w) * nq) * 64 + gl;
                if (CM <= 1) {  // nq = 2
                    const float v = sum_rowgroups2(cs[0], cs[1]);
                    if (!(lane & 16)) pw[(lane >> 5) * 64] = v;
                } else {
#pragma unroll
                    for (int c = 0; c < 1 + CM; ++c)
                        if (c <= C) {
                            const float v = sum_rowgroups(cs[c]);
                            if (lane < 16) pw[c * 64] = v;
                        }
                }
            }
        }
        }
        lap(0);
        if (t + 1 < t1) st(hold, ghold, buf ^ 1);
        lds_barrier();
        lap(1);
        if (PASS == 2) {  // one slab row per 128-row workgroup: (waves 0 + 1) + (waves 2 + 3)
            const float* pb = part + (buf * 4 * nq) * 64;
            for (int i = threadIdx.x; i < nq * 64; i += 256) {
                const int q = i >> 6, g = i & 63;
                Q.slabC[((int64_t)rbw * nq + q) * d.DP + 64 * t + g] =
                    (pb[(0 * nq + q) * 64 + g] + pb[(1 * nq + q) * 64 + g]) + (pb[(2 * nq + q) * 64 + g] + pb[(3 * nq + q) * 64 + g]);
            }
        }
    };
    if (t0 < t1) {
        ld(wrA, grA, t0);
        ld(wrB, grB, min(t0 + 1, t1 - 1));
        st(wrA, grA, 0);
    }
    __syncthreads();
    if (stamps) tp_ = stamp_now();
    const uint64_t rt_loop = stamps ? realtime_now() : 0;
    for (int t = t0; t < t1; t += 2) {
        tile(t, wrB, grB, wrA, grA);
        lap(2);
        if (t + 1 < t1) tile(t + 1, wrA, grA, wrB, grB);
        lap(2);
    }
    if (stamps) {
        if (lane == 0) {
            float* o = Q.slabC + ((int64_t)blockIdx.x * 4 + w) * 8;
            o[0] = (float)st_[0];
            o[1] = (float)st_[1];
            o[2] = (float)st_[2];
            o[3] = (float)(rt_entry & 0xffffffu);  // 100 MHz ticks: entry, loop start, loop end
            o[4] = (float)(rt_loop & 0xffffffu);
            o[5] = (float)(realtime_now() & 0xffffffu);
            o[6] = (float)wave_place();
            o[7] = (float)st_[3];
        }
        return;
    }
    if (PASS == 0) {
#pragma unroll
        for (int j = 0; j < J; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float m = mrun[j][r] * 0.6931471805599453f, s = srun[j][r];  // max back to natural units
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
                    const float mn = fmaxf(m, m2);
                    s = s * expf(m - mn) + s2 * expf(m2 - mn);
                    m = mn;
                }
                if ((lane & 15) == 0) {
                    float* lp = Q.lsep + ((int64_t)sp * d.Bpad + row0 + 16 * j + 4 * (lane >> 4) + r) * 2;
                    lp[0] = m;
                    lp[1] = s;
                }
            }
    }
}

// distinct kernel names per pass (profiles): A = log-sum-exp, C = the E_b P column term
template <class P, int KP, int CM>
__global__ __launch_bounds__(256, 2) void k_dec_lse(DecPtrs Q, Dims d) { dec_ac_body<P, KP, 0, CM>(Q, d); }
template <class P, int KP, int CM>
__global__ __launch_bounds__(256, 2) void k_dec_tail(DecPtrs Q, Dims d) { dec_ac_body<P, KP, 2, CM>(Q, d); }

// =======================================================================================
// k_dec_nb<T, KP, CM, RM> — decoder pass B: softmax + NB likelihood + every gradient term
// that needs only the row log-sum-exp (nb.hh:433-442, 453-460, 510-531 and their autograd).
// Workgroup = 64 cells (4 waves x 16) x one gene split.  Per 64-gene tile:
//   1. logits on MFMA against the decoder tile staged once per workgroup in LDS, p = softmax
//      (kept in registers in the MFMA C layout, also written to the wave's LDS p tile)
//   2. sparse pass over the tile's nonzeros (flattened over the wave's lanes): the
//      x-dependent terms (x log(s/mu), lgamma/digamma) -> loss, and the two per-element
//      corrections (p dq, d du) PLAIN-stored into the wave's correction tile (positions
//      are unique, so no atomics)
//   3. dense epilogue in the owner lanes (every element as if x = 0, plus its correction):
//      row sums in registers, column sums reduced across the wave's 16 rows with
//      permlane swaps and written as per-wave partials
//   4. dz partials on MFMA from the LDS-staged p*q and p tiles
//   5. barrier; the four waves' column partials are summed in a fixed order and stored to
//      this row block's slab in HBM (deterministic, no LDS or global atomics)
// The next tile's decoder rows, WdT rows and gene records are register-staged during the
// tile (loads early, ds_write after the barrier); CSR entries are prefetched a tile ahead.
// =======================================================================================
template <class T> struct CorrPair;
template <> struct CorrPair<float> {
    typedef float2 type;
    static MMVAE_DEV type pack(float a, float b) { return float2{a, b}; }
    static MMVAE_DEV void unpack(type v, float& a, float& b) { a = v.x; b = v.y; }
};
template <> struct CorrPair<X3> : CorrPair<float> {};  // x3 mode: f32 corrections
template <> struct CorrPair<__bf16> {  // bf16 mode: both corrections rounded to bf16
    typedef uint32_t type;
    static MMVAE_DEV type pack(float a, float b) {
        const __bf16 x = (__bf16)a, y = (__bf16)b;
        return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
    }
    static MMVAE_DEV void unpack(type v, float& a, float& b) {
        a = __uint_as_float(v << 16);
        b = __uint_as_float(v & 0xffff0000u);
    }
};

// Pass B runs NW = 8 waves (128 rows, two 64-row slab blocks) per workgroup and one
// workgroup per CU where the LDS allows (bf16): all waves of a CU advance tile by tile behind
// the same barriers (two co-resident 4-wave workgroups drift apart under the oldest-first
// issue arbitration and the younger one finishes alone at half occupancy), and the staged
// decoder tiles serve 128 rows instead of 64.  NW = 4 (64 rows, two workgroups per CU) otherwise.
// x3 mode (ALIAS): the dz GEMM's pq operand (hi + lo planes, 4 bytes per element) lives inside
// the wave's correction tile, laid out by 16-gene block: block gb of the correction tile is
// [16 rows][16 genes] f32 pairs (2 KB), its first 1 KB holds pq's hi plane then lo plane, each
// [16 genes][16 rows] (pqt_off: a row pair is one word; read back transposed, pqt_frag).  The epilogue reads all of a block's corrections before it writes that block's pq, and
// the tile is re-zeroed after the dz GEMM has read pq — saving the separate 4.6 KB pq tile per
// wave that would not fit 8 waves of x3 images in 160 KB.
struct DecNBLds {
    int o_gst, o_tst, o_part, o_fact, o_wave, wave_bytes, o_q1, o_q2, o_cc, o_toff, o_rsc, o_du = 0, bytes;
    int sw, st, sp;     // per-buffer strides: W tile, WdT tile (bytes, all planes), column partials (floats)
    int swp, stp;       // one plane of the W / WdT images (bytes)
    // eszw: element size of the staged logit operand (1 in the fp8 mode), esz: the dz operands'.
    // loss: the eval instance (no WdT stage, column partials, correction or pq tiles)
    // no_wdt: the dz GEMM reads its W operand transposed from the logit GEMM's W image (the
    // staggered x3 instance), so there is no WdT stage
    // d3: the three-waves-per-SIMD instance (k_dec_nb D3, x3): one stage buffer, no column
    // partial buffer (each wave's partials go into its own p tile after the dz GEMM), the p tile
    // unpadded (gene index XOR-swizzled by row), the correction tile holds p dq only (d du is
    // summed by the sparse pass into the wave's du accumulators), so 4 waves fit in 53 KB
    MMVAE_HOSTDEV DecNBLds(int KP, int esz, int S, int nq, int NRS, int csz, int NW, int nbuf, int planes, int eszw,
                           bool loss = false, bool no_wdt = false, bool d3 = false) {
        if (d3) {
            swp = 64 * KP * eszw;
            stp = 0;
            sw = planes * swp;
            st = 0;
            sp = 0;
            o_gst = sw;
            o_tst = o_gst + 1024;
            o_part = o_tst;
            o_fact = o_part;
            o_wave = o_fact + 64;
            o_q2 = 0;                 // p tile [16][64] f32 (x3: column partials [nq][64] after the dz GEMM)
            o_cc = 16 * 64 * 4;       // p dq plane per 16-gene block, 1 KB blocks (pq hi / lo aliased)
            o_q1 = o_cc;
            o_du = o_cc + 16 * 64 * 4;  // du sums: [64] genes, [64] genes x z_nu, [16] rows x w_nu
            // no LDS tile offsets (read from HBM with scalar loads) and two row scalars (d, z_nu):
            // 3 x 53,056 bytes fit the CU's 160 KB at its 2 KB allocation granule (4 x 9,200 + 17.5 KB
            // did not: 54,272 bytes ran two workgroups per CU)
            o_toff = o_du + (64 + 64 + 16) * 4;
            o_rsc = o_toff;
            wave_bytes = o_rsc + 16 * 2 * 4;
            bytes = o_wave + NW * wave_bytes;
            return;
        }
        const bool alias = planes == 2 && !loss;
        swp = 64 * KP * eszw;
        stp = (loss || no_wdt) ? 0 : KP * 64 * esz;
        sw = planes * swp;
        st = planes * stp;
        sp = loss ? ((16 * NW * 4 + 15) / 16) * 4 : ((NW * nq * 64 * 4 + 15) / 16) * 4;
        if (loss) csz = 0;
        o_gst = nbuf * sw;
        o_tst = o_gst + nbuf * 1024;
        o_part = o_tst + nbuf * st;
        o_fact = o_part + nbuf * sp * 4;  // x! for x = 0..8 (nb_gamma_terms)
        o_wave = o_fact + 48;
        const int QS = 64 + (esz == 2 ? 8 : 4);
        o_q1 = 0;
        o_q2 = (alias || loss) ? 0 : 16 * QS * esz;
        o_cc = o_q2 + 16 * 68 * 4;
        if (alias) o_q1 = o_cc;
        o_toff = o_cc + 16 * 64 * csz;
        o_rsc = o_toff + ((S * 4 + 15) / 16) * 16;
        wave_bytes = o_rsc + ((16 * NRS * 4 + 15) / 16) * 16;
        bytes = o_wave + NW * wave_bytes;
    }
};

// PL: the logit GEMM's operand policy (P, or F8 in the fp8 mode with P = bf16 for the dz GEMM)
// LOSS: the eval pass (mmvae_run update = 0) — the ELBO's likelihood terms only: the same
// arithmetic for the loss, without the corrections, column partials, dz GEMMs and WdT stage
// (the 8-wave loss instance fits two workgroups per CU: 128 VGPRs, ~60 KB of LDS in bf16)
// SG: the staggered instance (x3, NW = 8, training): waves 4-7 run half a tile behind waves 0-3
// (below), the W stage is double-buffered and serves the dz GEMM transposed (no WdT stage)
// TRW: no WdT stage, the dz GEMM reads W transposed (as SG does) — with DB, the x3 8-wave instance
// then double-buffers its stage and meets one barrier per tile (the default x3 training instance)
// D3: three waves per SIMD — 4-wave / 64-row workgroups, three per CU (<= 168 VGPRs, <= 53 KB of
// LDS: DecNBLds d3), so each SIMD holds waves of three independent workgroups and one wave's
// barrier wait leaves two others issuing.  The sparse pass stores only p dq per nonzero and
// adds its d du terms straight into the wave's LDS du sums (per-wave arrays, one wave's ds_add
// in program order: no cross-wave races); each wave's column partials go into its own p tile
// after the dz GEMM; one stage buffer, two barriers per tile.
template <class P, int KP, int CM, int RM, int NW, bool DB, class PL = P, bool LOSS = false, bool SG = false,
          bool TRW = false, bool D3 = false>
__global__ __launch_bounds__(64 * NW, D3 ? 3 : ((LOSS && NW == 8) ? 2 : 8 / NW)) void k_dec_nb(DecPtrs Q, Dims d) {
    using T = typename Elem<P>::type;
    using M = MM<P>;
    using Fr = typename M::frag;
    using TL = typename Elem<PL>::type;
    using ML = MM<PL>;
    constexpr bool F8M = IsF8<PL>::value;
    constexpr int KSL = KP / ML::KSTEP;  // k-steps of the logit GEMM
    using CP = CorrPair<P>;
    typedef typename CP::type CT;
    constexpr bool X = IsX3<P>::value;  // x3: split operands, pq aliased into the correction tile
    constexpr int NPL = X ? 2 : 1;
    constexpr int GK = 64 / M::KSTEP;   // k-steps of the dz GEMM over a 64-gene tile
    constexpr bool BF = sizeof(T) == 2;
    constexpr int QS = 64 + (BF ? 8 : 4);
    // pq (dz GEMM operand) element (r, g) and its lo-plane offset; the correction tile's (r, g)
    auto q1i = [](int r, int g) { return X ? ((g >> 4) * 1024 + r * 16 + (g & 15)) : r * QS + g; };
    constexpr int Q1PL = 256;
    auto cci = [](int r, int g) { return X ? ((g >> 4) * 256 + r * 16 + (g & 15)) : r * 64 + g; };
    // x3 corrections: per 16-gene block (2 KB) a p dq plane [16 genes][16 rows] and a d du plane
    // 1 KB after it, so a lane's row pair of one gene is one 8-byte read per plane (a packed-f32
    // operand as stored).  The f32 mode keeps (p dq, d du) pairs per element (its spilling pass B
    // ran 6 % slower with the planes)
    constexpr bool PLANAR = X;
    // (16-byte row quads XOR-swizzled by gene so the 16 genes of a lane group hit distinct banks)
    constexpr int PQBS = D3 ? 1024 : 2048;  // x3: bytes per 16-gene block of the correction / pq tile
    auto ccp = [](int r, int g) { return (g >> 4) * PQBS + (g & 15) * 64 + (((r >> 2) ^ ((g >> 2) & 3)) << 4) + (r & 3) * 4; };
    constexpr int PS = 68;
    // CM = 0: unit covariate (Engine::unit_covar, C = 1): the covariate Linear folds into the
    // gene's bias, and its weight gradient's column sums are the bias gradient's
    constexpr int CA = CM > 0 ? CM : 1;  // covariate array extent
    constexpr int NRS = 3 + RM + CA;    // row scalars: d, w, valid, znu[R], c[C]
    constexpr int RBW = KP * (int)sizeof(TL);  // staged decoder row (one gene)
    constexpr int RBT = 64 * (int)sizeof(T);  // staged WdT row (one latent, 64 genes)
    constexpr float L2E = 1.4426950408889634f;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // (D3: lane is re-made opaque every tile, so the lane-derived LDS addresses are recomputed
    // instead of being hoisted out of the tile loop and spilled)
    int lane = threadIdx.x & 63;
    int tido = threadIdx.x;  // (D3: opaque per tile, as lane)
    const int w = threadIdx.x >> 6;
    constexpr int NTH = 64 * NW;
    const int sp = blockIdx.x % d.nsD, rbw = blockIdx.x / d.nsD;
    const int row0 = rbw * 16 * NW + 16 * w;
    const int t0 = sp * d.tpsD, t1 = min(d.NT, t0 + d.tpsD);
    const int S = d.tpsD + 1;
    const int C = (CM <= 1) ? 1 : d.C, R = (RM == 1) ? 1 : d.R;
    const int nq = (1 + C) + 1 + R;
    static_assert(!SG || (X && DB && NW == 8 && !LOSS), "the staggered pass B is the x3 training instance");
    static_assert(!D3 || (X && NW == 4 && !DB && TRW && !LOSS && !SG && CM <= 1 && RM == 1 && !F8M),
                  "the three-waves-per-SIMD pass B is the x3 training instance for C = R = 1");
    const DecNBLds L(KP, (int)sizeof(T), S, nq, NRS, (int)sizeof(CT), NW, DB ? 2 : 1, NPL, (int)sizeof(TL), LOSS, SG || TRW, D3);
    char* wst = smem;
    const float4* gst = reinterpret_cast<const float4*>(smem + L.o_gst);
    char* tst = smem + L.o_tst;
    // [4][nq][64] column partials; D3: prologue / loss scratch in wave 0's p tile
    float* part = reinterpret_cast<float*>(smem + (D3 ? L.o_wave + L.o_q2 : L.o_part));
    float* ftab = reinterpret_cast<float*>(smem + L.o_fact);
    if (threadIdx.x < 9) {  // published by the barrier of the row lse block below
        float f = 1.f;
        for (int i = 2; i <= (int)threadIdx.x; ++i) f *= (float)i;
        ftab[threadIdx.x] = f;
    }
    char* wp = smem + L.o_wave + w * L.wave_bytes;
    T* q1 = reinterpret_cast<T*>(wp + L.o_q1);
    float* q2 = reinterpret_cast<float*>(wp + L.o_q2);
    CT* cc = reinterpret_cast<CT*>(wp + L.o_cc);
    int32_t* toffl = reinterpret_cast<int32_t*>(wp + L.o_toff);
    float* rsc = reinterpret_cast<float*>(wp + L.o_rsc);
    // row scalars per row: NRS (d, w, valid, z_nu[R], c[C]); D3 keeps only d and z_nu
    constexpr int RSS = D3 ? 2 : NRS, RSZ = D3 ? 1 : 3;
    float* duacc = reinterpret_cast<float*>(wp + L.o_du);  // D3: [64] sum du, [64] sum du z_nu, [16] sum du w_nu
    // the p tile's element (r, g): D3 unpadded with the gene XOR-swizzled by row (8-gene groups
    // stay contiguous for the dz GEMM's fragment reads), else a 68-float row stride
    auto qx = [](int r, int g) { return D3 ? r * 64 + (g ^ ((r & 7) << 3)) : r * 68 + g; };
    constexpr int CCBYTES = D3 ? 16 * 64 * 4 : 16 * 64 * (int)sizeof(CT);  // correction tile bytes
    const T* Z = BF ? reinterpret_cast<const T*>(Q.zb) : reinterpret_cast<const T*>(Q.zf);
    const char* WdPc = reinterpret_cast<const char*>(Q.WdP);
    const char* WdTc = reinterpret_cast<const char*>(Q.WdT);
    const float4* grec = reinterpret_cast<const float4*>(Q.gene + 4 * d.DP);  // (bias, cn, Wcd0, Wnd0)

    // ---- per-row state (lane holds rows 4(lane>>4)+r of the wave's 16) ----
    typename ML::frag zfr[KSL];
#pragma unroll
    for (int s = 0; s < KSL; ++s) {
        const int64_t zo = (int64_t)(row0 + (lane & 15)) * KP + s * ML::KSTEP + (lane >> 4) * ML::EPL;
        if constexpr (F8M) zfr[s] = ML::load_f32(Q.zf + zo);
        else zfr[s] = M::load(&Z[zo], Q.zplane);
    }
    const float ainv = F8M ? d.inv_wscale : 1.f;  // logit accumulator unscale (fp8 W_dec)
    // ---- staging of the decoder tile, its gene records and the WdT tile ----
    // SG: the stage is loaded and stored by the lagging half (waves 4-7, 256 threads) only
    constexpr int NST = SG ? NTH / 2 : NTH;
    const bool lag = SG && w >= NW / 2;
    const bool stager = !SG || lag;
    auto stid_ = [&]() { return (D3 ? tido : (int)threadIdx.x) & (NST - 1); };
    DualStage<64, RBW, NST, X> wreg;
    DualStage<KP, RBT, NTH, X> treg;
    float4 greg = float4{0.f, 0.f, 0.f, 0.f};
    const int64_t wplb = Q.wplane * (int64_t)sizeof(T);
    auto stage_load = [&](int t) {
        const int stid = stid_();
        wreg.load(WdPc + (int64_t)64 * t * RBW, RBW, wplb, D3 ? tido : (int)threadIdx.x);
        if constexpr (!LOSS && !SG && !TRW) treg.load(WdTc + (int64_t)64 * t * sizeof(T), (int64_t)d.DP * sizeof(T), wplb);
        if (stid < 64) greg = grec[64 * t + stid];
    };
    auto stage_store = [&](int b_) {
        const int stid = stid_();
        wreg.store(wst + b_ * L.sw, L.swp, D3 ? tido : (int)threadIdx.x);
        if constexpr (!LOSS && !SG && !TRW) treg.store(tst + b_ * L.st, L.stp);
        if (stid < 64) reinterpret_cast<float4*>(smem + L.o_gst)[64 * b_ + stid] = greg;
    };
    if (stager) stage_load(min(t0, d.NT - 1));  // independent of everything below: issued first
    // row log-sum-exp (log2 units) from pass A's split partials, 4 threads per row; split 0
    // also publishes it for pass C
    {
        const int rr = threadIdx.x >> 2, pp = threadIdx.x & 3;
        const int b = rbw * 16 * NW + rr;
        float mm = -INFINITY;
        for (int s2 = pp; s2 < d.nsA; s2 += 4) mm = fmaxf(mm, Q.lsep[((int64_t)s2 * d.Bpad + b) * 2]);
        mm = fmaxf(mm, __shfl_xor(mm, 1, 64));
        mm = fmaxf(mm, __shfl_xor(mm, 2, 64));
        float ss = 0.f;
        for (int s2 = pp; s2 < d.nsA; s2 += 4) {
            const float* lp = Q.lsep + ((int64_t)s2 * d.Bpad + b) * 2;
            ss += lp[1] * expf(lp[0] - mm);
        }
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        if (pp == 0) {
            const float l2 = (mm + logf(ss)) * L2E;
            part[rr] = l2;
            if (sp == 0) Q.rowfin[2 * b] = l2;
        }
        __syncthreads();
    }
    // rows 4(lane>>4) + 2h + j live in component j of the pair h (packed f32 epilogue)
    float lse2[4];
    f2 rv2[2], dv2[2], wv2[2], crow2[2][CA], znu2[2][RM];
    f2 Eacc2[2], dzn2[2][RM], wc2[2][CA];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int h = r >> 1, j = r & 1;
        const int b = row0 + 4 * (lane >> 4) + r;
        const float* Lr = Q.lat + (int64_t)b * d.lat_stride;
        rv2[h][j] = Lr[d.LAT_VALID];
        dv2[h][j] = Lr[d.LAT_D];
        wv2[h][j] = Lr[d.LAT_W];
        lse2[r] = part[16 * w + 4 * (lane >> 4) + r];
        const int64_t cell = Q.cells[b];  // padding rows hold the empty row N
#pragma unroll
        for (int c = 0; c < CM; ++c) crow2[h][c][j] = (c < C) ? Q.covar[cell * C + c] : 0.f;  // row N: zeros
#pragma unroll
        for (int q = 0; q < RM; ++q) {
            znu2[h][q][j] = (q < R) ? Lr[d.LAT_ZNU + q] : 0.f;
            dzn2[h][q][j] = 0.f;
        }
        Eacc2[h][j] = 0.f;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < CM; ++c) wc2[h][c] = wv2[h] * crow2[h][c];  // w_b c_b (covar_decoding column sums)
    f2 lossd2 = splat2(0.f);  // dense (x = 0) part of the loss
    f32x4 dzA[KP / 16], dzP[KP / 16];
#pragma unroll
    for (int lb = 0; lb < KP / 16; ++lb) {
        dzA[lb] = f32x4{0.f, 0.f, 0.f, 0.f};
        dzP[lb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float lossacc = 0.f;
    f2 lossacc2 = splat2(0.f);  // (the packed sparse pass's)
    constexpr float LN2c = 0.6931471805599453f;
    constexpr bool SPAIR = !std::is_same<P, float>::value;
    // ---- per-wave row data for the sparse pass ----
    const int wbk = row0 >> 4;  // this wave's 16-row block of the batch entry lists
    if constexpr (D3) toffl = const_cast<int32_t*>(Q.toff) + (int64_t)wbk * (d.NT + 1) + t0;  // (HBM, read-only)
    else fill_toffl(toffl, S, t0, d.NT, Q.toff, wbk, lane);
    const int64_t segw = Q.seg[wbk];
    if (D3 && lane < 16) {
        const int b = row0 + lane;
        const float* Lr = Q.lat + (int64_t)b * d.lat_stride;
        rsc[lane * 2] = Lr[d.LAT_D];
        rsc[lane * 2 + 1] = Lr[d.LAT_ZNU];
    } else if (lane < 16) {
        const int b = row0 + lane;
        const int64_t cell = Q.cells[b];  // padding rows hold the empty row N
        const float* Lr = Q.lat + (int64_t)b * d.lat_stride;
        float* rs = rsc + lane * NRS;
        rs[0] = Lr[d.LAT_D];
        rs[1] = Lr[d.LAT_W];
        rs[2] = Lr[d.LAT_VALID];
        for (int q = 0; q < RM; ++q) rs[3 + q] = (q < R) ? Lr[d.LAT_ZNU + q] : 0.f;
        for (int c = 0; c < CM; ++c) rs[3 + RM + c] = (c < C) ? Q.covar[cell * C + c] : 0.f;
    }
    if constexpr (!LOSS)
        for (int i = lane; i < CCBYTES / 16; i += 64) reinterpret_cast<uint4*>(cc)[i] = uint4{0, 0, 0, 0};
    if constexpr (D3)
        for (int i = lane; i < 64 + 64 + 16; i += 64) duacc[i] = 0.f;

    wave_sync();  // toffl
    ListEntries pend;
    if (t0 < t1) {
        pend.fetch(Q.ents, segw, toffl, 0, lane);
        if (stager) stage_store(0);
    }
    lds_barrier();  // the first tile's entry loads stay in flight

    // diagnostic (MMVAE_DBG & 64): per-wave phase cycles into dzp (outputs invalid)
    const bool stamps = dbg_bit(d.dbg, 64);
    const uint64_t rt0 = stamps ? realtime_now() : 0;
    uint64_t st_[7] = {0, 0, 0, 0, 0, 0, 0}, tp_ = stamps ? stamp_now() : 0;
    auto lap = [&](int i_) {
        if (stamps) {
            const uint64_t tn = stamp_now();
            st_[i_] += tn - tp_;
            tp_ = tn;
        }
    };
    // one tile's LDS stage / column-partial buffers
    struct TileCtx {
        int t;
        const char *wsb, *tsb;
        const float4* gsb;
        float* pb;
    };
    auto ctx = [&](int t) {
        const int buf = DB ? ((t - t0) & 1) : 0;
        return TileCtx{t, wst + buf * L.sw, tst + buf * L.st, gst + 64 * buf, part + buf * L.sp};
    };
    // ---- phases L + S of tile c.t: logits -> p, sparse pass, next tile's entry prefetch ----
    auto phase_ls = [&](const TileCtx& c) {
        const int t = c.t, tl = t - t0;
        const char* wsb = c.wsb;
        const float4* gsb = c.gsb;
        // ---- 1. logits -> p (into the wave's LDS p tile) ----
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
            const int gl = 16 * gb + (lane & 15);
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KSL; ++s)
                acc = ML::mma(zfr[s], ML::load(reinterpret_cast<const TL*>(wsb + swz_off<RBW>(gl, (s * ML::KSTEP + (lane >> 4) * ML::EPL) * (int)sizeof(TL))), L.swp / (int)sizeof(TL)), acc);
            const float4 g4 = gsb[gl];
            const float gx = CM == 0 ? g4.x + g4.z : g4.x;  // unit covariate: folded into the bias
            float wcd[CA];
            wcd[0] = g4.z;
#pragma unroll
            for (int c2 = 1; c2 < CM; ++c2) wcd[c2] = (c2 < C && 64 * t + gl < d.D) ? Q.Wcd[(int64_t)(64 * t + gl) * C + c2] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float lg = fmaf(acc[r], ainv, gx);
#pragma unroll
                for (int c2 = 0; c2 < CM; ++c2) lg = fmaf(crow2[r >> 1][c2][r & 1], wcd[c2], lg);
                q2[qx(4 * (lane >> 4) + r, gl)] = fexp2(fmaf(lg, L2E, -lse2[r]));  // nb.hh:440-441
            }
        }
        wave_sync();
        lap(0);
        if constexpr (D3) __builtin_amdgcn_sched_barrier(0);  // (phases not interleaved: register budget)
        // ---- 2. sparse pass: x-dependent terms of the tile's nonzeros ----
        // 16-bit operand modes (x3, bf16): two entries per lane as one packed pair (entries lane
        // and lane + 64, then + 128 / + 192 ...), packed arithmetic throughout (nb_nu2: the
        // epilogue's own overdispersion arithmetic, so an entry's nu is the dense pass's).  The f32
        // mode keeps one entry per lane (its pass B already spills).
        if constexpr (SPAIR) {
            if (!dbg_bit(d.dbg, 1)) pend.visit2(Q.ents, lane, [&](uint32_t ea, float xa, uint32_t eb, float xb, bool vb) {
                const int ra = ent_row(ea), ga = ent_gene(ea);
                const int rb = ent_row(eb), gb2 = ent_gene(eb);
                const f2 x = f2{xa, vb ? xb : 0.f};
                const float* rsa = rsc + ra * RSS;
                const float* rsb = rsc + rb * RSS;
                const f2 p = f2{q2[qx(ra, ga)], q2[qx(rb, gb2)]};
                const f2 mu = fma2(p, f2{rsa[0], rsb[0]}, splat2(1e-4f));  // nb.hh:519
                const float4 g4a = gsb[ga], g4b = gsb[gb2];
                f2 u = f2{g4a.y, g4b.y};
#pragma unroll
                for (int q = 0; q < RM; ++q) {  // nb.hh:456-457
                    const f2 wn = q == 0 ? f2{g4a.w, g4b.w}
                                         : ((q < R) ? f2{Q.Wnd[(int64_t)(64 * t + ga) * R + q], Q.Wnd[(int64_t)(64 * t + gb2) * R + q]}
                                                    : splat2(0.f));
                    u = fma2(wn, f2{rsa[RSZ + q], rsb[RSZ + q]}, u);
                }
                f2 nup, sgm;
                nb_nu2(u, nup, sgm);  // nb.hh:458-459
                const f2 sv = mu + nup;
                f2 rsv, rmu, lr;
                rsv.x = frcp(sv.x);
                rsv.y = frcp(sv.y);
                rmu.x = frcp(mu.x);
                rmu.y = frcp(mu.y);
                // nb.hh:522-523: the finite product for integer counts <= 8, the series otherwise
                const bool biga = !(x.x <= 8.f && x.x == floorf(x.x)), bigb = !(x.y <= 8.f && x.y == floorf(x.y));
                const f2 xf = f2{biga ? 0.f : x.x, bigb ? 0.f : x.y};
                f2 lgd, dgd;
                nb_gamma_terms2(nup, xf, (int)xf.x, (int)xf.y, lgd, dgd, ftab);
                if (biga || bigb) {
                    float l_, dg_;
                    if (biga) {
                        nb_gamma_terms<8>(nup.x, x.x, l_, dg_, ftab);
                        lgd.x = l_;
                        dgd.x = dg_;
                    }
                    if (bigb) {
                        nb_gamma_terms<8>(nup.y, x.y, l_, dg_, ftab);
                        lgd.y = l_;
                        dgd.y = dg_;
                    }
                }
                const f2 svm = sv * rmu;
                lr.x = flog2(svm.x);
                lr.y = flog2(svm.y);
                lossacc2 = fma2(x * LN2c, lr, lossacc2 + lgd);  // nb.hh:527: x (log(mu+nu) - log(mu))
                const f2 dq = x * (rsv - rmu);
                const f2 ddu = fma2(x, rsv, dgd) * sgm;          // (0 where the clamp bites)
                if constexpr (!LOSS) {
                    const f2 pdq = p * dq;
                    auto put = [&](int r, int gl, float a, float b) {
                        if constexpr (D3) {
                            *reinterpret_cast<float*>(reinterpret_cast<char*>(cc) + ccp(r, gl)) = a;
                        } else if constexpr (PLANAR) {
                            char* cb = reinterpret_cast<char*>(cc) + ccp(r, gl);
                            *reinterpret_cast<float*>(cb) = a;
                            *reinterpret_cast<float*>(cb + 1024) = b;
                        } else {
                            cc[cci(r, gl)] = CP::pack(a, b);
                        }
                    };
                    put(ra, ga, pdq.x, ddu.x);
                    if (vb) put(rb, gb2, pdq.y, ddu.y);
                    if constexpr (D3) {  // the d du terms into the wave's du sums (R = 1)
                        const f2 dz = ddu * f2{rsa[RSZ], rsb[RSZ]};  // x z_nu of the entry's row
                        const f2 dw = ddu * f2{g4a.w, g4b.w};    // x w_nu of the entry's gene
                        atomicAdd(&duacc[ga], ddu.x);
                        atomicAdd(&duacc[64 + ga], dz.x);
                        atomicAdd(&duacc[128 + ra], dw.x);
                        if (vb) {
                            atomicAdd(&duacc[gb2], ddu.y);
                            atomicAdd(&duacc[64 + gb2], dz.y);
                            atomicAdd(&duacc[128 + rb], dw.y);
                        }
                    }
                }
            });
        } else if (!dbg_bit(d.dbg, 1)) pend.visit(Q.ents, lane, [&](int r, int gl, float x) {
            const float* rs_ = rsc + r * NRS;
            const float p = q2[qx(r, gl)];
            const float mu = fmaf(p, rs_[0], 1e-4f);
            const float4 g4 = gsb[gl];
            float wnd[RM];
            wnd[0] = g4.w;
#pragma unroll
            for (int q = 1; q < RM; ++q) wnd[q] = (q < R) ? Q.Wnd[(int64_t)(64 * t + gl) * R + q] : 0.f;
            float u = g4.y;
#pragma unroll
            for (int q = 0; q < RM; ++q) u = fmaf(wnd[q], rs_[3 + q], u);
            float sig;
            const float spv = softplus_sig(u, sig);
            const float nu = clamp_nu(spv);
            const bool msk = nu == spv;                                 // clamp passes the gradient
            const float nup = nu + 1e-4f;
            const float sv = mu + nup;
            const float rsv = frcp(sv), rmu = frcp(mu);
            float lgd, dgd;
            nb_gamma_terms<std::is_same<P, float>::value ? 4 : 8>(nup, x, lgd, dgd, ftab);  // nb.hh:522-523
            lossacc += x * flog(sv * rmu) + lgd;                        // nb.hh:527: x (log(mu+nu) - log(mu))
            const float dq = x * (rsv - rmu);
            const float ddu = msk ? (x * rsv + dgd) * sig : 0.f;
            if constexpr (!LOSS) {
                if constexpr (PLANAR) {
                    char* cb = reinterpret_cast<char*>(cc) + ccp(r, gl);
                    *reinterpret_cast<float*>(cb) = p * dq;
                    *reinterpret_cast<float*>(cb + 1024) = ddu;
                } else {
                    cc[cci(r, gl)] = CP::pack(p * dq, ddu);
                }
            }
        });
        wave_sync();
        lap(1);
        if constexpr (D3) __builtin_amdgcn_sched_barrier(0);  // (phases not interleaved: register budget)
        // ---- prefetch the next tile's entries (rinc reused; loads stay in flight) ----
        pend.fetch(Q.ents, segw, toffl, min(tl + 1, t1 - t0 - 1), lane);
        lap(2);
        if constexpr (D3) __builtin_amdgcn_sched_barrier(0);  // (phases not interleaved: register budget)
    };
    // ---- phases E + Z of tile c.t: dense epilogue, dz GEMM ----
    auto phase_ez = [&](const TileCtx& c) {
        const int t = c.t;
        const float4* gsb = c.gsb;
        float* pb = c.pb;
        // ---- 3. dense epilogue in the owner lanes ----
        // MASK: some of the wave's rows (last row block) or the tile's genes (last tile) are
        // padding; the common case runs without the validity products.
        float colv[4];  // D3: the lane's column partial of each gene block (stored after the dz GEMM)
        auto epilogue = [&](auto mask_c) {
            constexpr bool MASK = decltype(mask_c)::value;
            constexpr float LN2 = 0.6931471805599453f;
            // (the general variant stays rolled; D3 too, for its register budget)
            constexpr int GBU = (CM <= 1 && RM == 1 && !D3) ? 4 : 1;
#pragma unroll GBU
            for (int gb = 0; gb < 4; ++gb) {
                const int gl = 16 * gb + (lane & 15);
                const int gene = 64 * t + gl;
                const bool gv = gene < d.D;
                const float4 g4 = gsb[gl];
                const float cn = g4.y;
                float wnd[RM];
                wnd[0] = g4.w;
#pragma unroll
                for (int q = 1; q < RM; ++q) wnd[q] = (q < R && gv) ? Q.Wnd[(int64_t)gene * R + q] : 0.f;
                const float gvf = gv ? 1.f : 0.f;
                f2 cs1[1 + CA], csdu = splat2(0.f), csduz[RM];
#pragma unroll
                for (int c2 = 0; c2 < 1 + CA; ++c2) cs1[c2] = splat2(0.f);
#pragma unroll
                for (int q = 0; q < RM; ++q) csduz[q] = splat2(0.f);
                // the block's corrections first (x3: this block's pq overwrites them below)
                CT ccv[4];
                f2 cpv[2], cdv[2];
                if constexpr (!LOSS) {
                    if constexpr (PLANAR) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const char* cb = reinterpret_cast<const char*>(cc) + ccp(4 * (lane >> 4) + 2 * h, gl);
                            cpv[h] = *reinterpret_cast<const f2*>(cb);
                            if constexpr (!D3) cdv[h] = *reinterpret_cast<const f2*>(cb + 1024);
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; ++r) ccv[r] = cc[cci(4 * (lane >> 4) + r, gl)];
                    }
                }
                if constexpr (X) asm volatile("" ::: "memory");
#pragma unroll
                for (int h = 0; h < 2; ++h) {  // rows rl, rl + 1 as one packed pair
                    const int rl = 4 * (lane >> 4) + 2 * h;
                    const f2 p = f2{q2[qx(rl, gl)], q2[qx(rl + 1, gl)]};
                    const f2 mu = fma2(p, dv2[h], splat2(1e-4f));                // nb.hh:519
                    f2 u = splat2(cn);
#pragma unroll
                    for (int q = 0; q < RM; ++q) u = fma2(splat2(wnd[q]), znu2[h][q], u);  // nb.hh:456-457
                    f2 nup, lg2, qv, sgm;
                    nb_dense2(mu, u, nup, lg2, qv, sgm);                         // nb.hh:458-459, 518-528
                    if (MASK) {
                        const f2 me = rv2[h] * gvf;
                        sgm *= me;
                        lossd2 = fma2(nup * me, lg2, lossd2);                    // nb.hh:528, x = 0 part
                    } else {
                        lossd2 = fma2(nup, lg2, lossd2);
                    }
                    if constexpr (LOSS) continue;
                    f2 cpp, cdp;  // the row pair's corrections: p dq, d du
                    if constexpr (PLANAR) {
                        cpp = cpv[h];
                        cdp = cdv[h];
                    } else {
                        float cpa, cda, cpb, cdb;
                        CP::unpack(ccv[2 * h], cpa, cda);
                        CP::unpack(ccv[2 * h + 1], cpb, cdb);
                        cpp = f2{cpa, cpb};
                        cdp = f2{cda, cdb};
                    }
                    const f2 pq = fma2(p, qv, cpp);                              // qv = n dL/dmu' - 1 at x = 0
                    // (D3: the nonzeros' d du terms went into the du sums in the sparse pass)
                    const f2 du = D3 ? fma2(lg2, splat2(LN2), qv) * sgm : fma2(fma2(lg2, splat2(LN2), qv), sgm, cdp);
                    Eacc2[h] += pq;
                    cs1[0] = fma2(wv2[h], pq, cs1[0]);
#pragma unroll
                    for (int c2 = 0; c2 < CM; ++c2) cs1[1 + c2] = fma2(wc2[h][c2], pq, cs1[1 + c2]);
                    csdu += du;
#pragma unroll
                    for (int qq = 0; qq < RM; ++qq) {
                        csduz[qq] = fma2(du, znu2[h][qq], csduz[qq]);
                        dzn2[h][qq] = fma2(du, splat2(wnd[qq]), dzn2[h][qq]);
                    }
                    if constexpr (X) {  // hi / lo planes of the row pair, one word each
                        pqt_put<PQBS, true>(reinterpret_cast<char*>(q1), 512, gl, rl, pq.x, pq.y);
                    } else if constexpr (BF) {  // bf16: the separate q1 tile, compact blocks
                        pqt_put<512, false>(reinterpret_cast<char*>(q1), 0, gl, rl, pq.x, pq.y);
                    } else {
                        put_op<P>(q1, q1i(rl, gl), Q1PL, pq.x);
                        put_op<P>(q1, q1i(rl + 1, gl), Q1PL, pq.y);
                    }
                }
                if constexpr (LOSS) continue;
                float* pw = pb + w * nq * 64 + gl;
                // (CM = 0: the covariate column sums sum_b w_b c_b pq with c_b = 1 are cs1[0])
                const f2 cs1c = (CM == 0) ? cs1[0] : cs1[1];
                if (CM <= 1 && RM == 1) {  // nq = 4: one transposed reduction, every lane stores
                    const float v = sum_rowgroups4(cs1[0].x + cs1[0].y, cs1c.x + cs1c.y, csdu.x + csdu.y,
                                                   csduz[0].x + csduz[0].y);
                    if constexpr (D3) {  // (rolled loop: selects keep colv in registers)
#pragma unroll
                        for (int k = 0; k < 4; ++k) colv[k] = (gb == k) ? v : colv[k];
                    }
                    else pw[(lane >> 4) * 64] = v;
                } else {
#pragma unroll
                    for (int c2 = 0; c2 < 1 + CA; ++c2)
                        if (c2 <= C) {
                            const f2 cv = (c2 == 1) ? cs1c : cs1[c2];
                            const float v = sum_rowgroups(cv.x + cv.y);
                            if (lane < 16) pw[c2 * 64] = v;
                        }
                    {
                        const float v = sum_rowgroups(csdu.x + csdu.y);
                        if (lane < 16) pw[(1 + C) * 64] = v;
                    }
#pragma unroll
                    for (int qq = 0; qq < RM; ++qq)
                        if (qq < R) {
                            const float v = sum_rowgroups(csduz[qq].x + csduz[qq].y);
                            if (lane < 16) pw[(2 + C + qq) * 64] = v;
                        }
                }
            }
        };
        if (!dbg_bit(d.dbg, 2)) {
            if (row0 + 16 <= d.B && 64 * t + 64 <= d.D) epilogue(std::false_type{});
            else epilogue(std::true_type{});
        }
        wave_sync();
        if constexpr (!X && !LOSS)
            for (int i = lane; i < 16 * 64 * (int)sizeof(CT) / 16; i += 64) reinterpret_cast<uint4*>(cc)[i] = uint4{0, 0, 0, 0};
        lap(3);
        if constexpr (D3) __builtin_amdgcn_sched_barrier(0);  // (phases not interleaved: register budget)
        // ---- 4. dz partial = sum_g Q[cell][g] W[g][latent] on MFMA ----
        if (!LOSS && !dbg_bit(d.dbg, 4))
#pragma unroll
            for (int s = 0; s < GK; ++s) {
                Fr a1;
                if constexpr (X) {
                    const char* qb = reinterpret_cast<const char*>(q1);
                    a1 = Fr{pqt_frag<PQBS>(qb, s * M::KSTEP, lane), pqt_frag<PQBS>(qb + 512, s * M::KSTEP, lane)};
                } else if constexpr (BF) {
                    a1 = pqt_frag<512>(reinterpret_cast<const char*>(q1), s * M::KSTEP);
                } else {
                    a1 = M::load(&q1[q1i(lane & 15, s * M::KSTEP + (lane >> 4) * M::EPL)], Q1PL);
                }
                const Fr a2 = M::load_f32(&q2[qx(lane & 15, s * M::KSTEP + (lane >> 4) * M::EPL)]);
#pragma unroll
                for (int lb = 0; lb < KP / 16; ++lb) {
                    Fr bw;
                    if constexpr (SG || TRW)  // transposed from the logit GEMM's W image (genes = k)
                        bw = TrFrag<P, RBW>::load(c.wsb, s * M::KSTEP, 16 * lb, L.swp, lane);
                    else
                        bw = M::load(reinterpret_cast<const T*>(
                            c.tsb + swz_off<RBT>(16 * lb + (lane & 15), (s * M::KSTEP + (lane >> 4) * M::EPL) * (int)sizeof(T))),
                            L.stp / (int)sizeof(T));
                    dzA[lb] = M::mma(a1, bw, dzA[lb]);
                    dzP[lb] = M::mma(a2, bw, dzP[lb]);
                }
            }
        if constexpr (X && !LOSS) {  // pq consumed: re-zero the correction tile it aliased
            wave_sync();
            for (int i = lane; i < CCBYTES / 16; i += 64) reinterpret_cast<uint4*>(cc)[i] = uint4{0, 0, 0, 0};
        }
        if constexpr (D3) {
            // the p tile is consumed: the wave's column partials [nq][64] go there (read by the
            // combine after the barrier), the du sums of the sparse pass added to theirs; the
            // per-tile du sums are cleared (the row sums at 128.. accumulate over the tiles)
            wave_sync();
            const int q = lane >> 4;
#pragma unroll
            for (int gb = 0; gb < 4; ++gb) {
                const int gl = 16 * gb + (lane & 15);
                q2[q * 64 + gl] = colv[gb] + (q >= 2 ? duacc[(q - 2) * 64 + gl] : 0.f);
            }
            wave_sync();
            duacc[lane] = 0.f;
            duacc[64 + lane] = 0.f;
        }
        lap(4);
    };
    // ---- 5. the waves' column partials of tile c.t -> slab (fixed order), by threads
    //      [th0, th0 + nth) ----
    auto combine = [&](const TileCtx& c, int th0, int nth) {
        if (LOSS || dbg_bit(d.dbg, 16384)) return;  // 16384: diagnostic, slab stores skipped
        // one slab row per workgroup (64 or 128 rows): the waves' partials in fixed order
        for (int i = (D3 ? tido : (int)threadIdx.x) - th0; i < nq * 64; i += nth) {
            const int q = i >> 6, g = i & 63;
            float v;
            if constexpr (D3) {  // each wave's partials in its p tile
                auto pw_ = [&](int wv) { return reinterpret_cast<const float*>(smem + L.o_wave + wv * L.wave_bytes + L.o_q2); };
                v = pw_(0)[q * 64 + g] + pw_(1)[q * 64 + g] + pw_(2)[q * 64 + g] + pw_(3)[q * 64 + g];
            } else {
                auto half = [&](int h) {
                    const float* ph = c.pb + 4 * h * nq * 64;
                    return ph[(0 * nq + q) * 64 + g] + ph[(1 * nq + q) * 64 + g] + ph[(2 * nq + q) * 64 + g] +
                           ph[(3 * nq + q) * 64 + g];
                };
                v = NW == 8 ? half(0) + half(1) : half(0);
            }
            Q.slabB[((int64_t)rbw * nq + q) * d.DP + 64 * c.t + g] = v;
        }
    };
    if constexpr (SG) {
        // Staggered pass B (MI355X_MICROARCH.md "Two waves per SIMD", item 9): waves w and w + 4
        // share a SIMD, so with both halves in the same phase the logit / dz MFMAs of one wave
        // meet the other's at the same time and the epilogue VALU likewise.  Waves 4-7 lag half a
        // tile: between barriers B(t-1) and B(t) the lead runs L S E Z of tile t while the lag
        // runs E Z of tile t-1 and L S of tile t.  Hazards, with the stage double-buffered:
        //  * stage(t+1) is written by the lag after its E Z(t-1) and L S(t), before B(t): every
        //    read of that buffer (stage(t-1)) is done — the lead's before B(t-1), the lag's
        //    earlier in its own program;
        //  * column partials of tile t (buffer t & 1) are complete at B(t+1) (the lag's E(t));
        //    the lead combines them after B(t+1), before its own E(t+2) rewrites the buffer,
        //    and the lag's E(t+2) follows B(t+2).
        for (int t = t0; t < t1; ++t) {
            const int tl = t - t0;
            if (lag) {
                stage_load(min(t + 1, t1 - 1));  // unconditional (clamped): counted waits
                if (t > t0) phase_ez(ctx(t - 1));
                phase_ls(ctx(t));
                if (t + 1 < t1) stage_store((tl + 1) & 1);
                lds_barrier();
            } else {
                phase_ls(ctx(t));
                phase_ez(ctx(t));
                lds_barrier();
                if (t > t0) combine(ctx(t - 1), 0, NTH / 2);
            }
        }
        if (t0 < t1) {
            if (lag) {
                phase_ez(ctx(t1 - 1));
                lds_barrier();
            } else {
                lds_barrier();
                combine(ctx(t1 - 1), 0, NTH / 2);
            }
        }
    } else {
        for (int t = t0; t < t1; ++t) {
            const int tl = t - t0;
            // (D3: the next stage is loaded after the tile's barrier, right before it is stored, so
            // its registers are not live across the tile; the latency is the other workgroups')
            if constexpr (!D3) stage_load(min(t + 1, t1 - 1));  // unconditional (clamped): counted waits, not vmcnt(0)
            if constexpr (D3) asm volatile("" : "+v"(lane), "+v"(tido));
            const TileCtx c = ctx(t);
            phase_ls(c);
            phase_ez(c);
            if constexpr (D3) {
                // the logit GEMM's z fragments are re-read (L2) after the dz GEMM, through an
                // address the compiler cannot prove loop-invariant: they are live from here to the
                // next tile's logits only, not through its sparse pass and epilogue
                const T* Zo = Z;
                asm volatile("" : "+s"(Zo));
#pragma unroll
                for (int s = 0; s < KSL; ++s)
                    zfr[s] = M::load(&Zo[(int64_t)(row0 + (lane & 15)) * KP + s * ML::KSTEP + (lane >> 4) * ML::EPL], Q.zplane);
            }
            // double-buffered (NW = 8): the next tile's stage goes into the other buffer before the
            // tile's single barrier; buffer b is rewritten only after the next barrier, which every
            // wave reaches after its combine reads of b
            if (DB && t + 1 < t1) stage_store((tl & 1) ^ 1);
            if (!dbg_bit(d.dbg, 32768)) lds_barrier();  // 32768: diagnostic, barrier skipped (outputs invalid)
            combine(c, 0, NTH);
            lap(5);
            if (!DB) {
                if constexpr (D3) {
                    if (t + 1 < t1) {
                        stage_load(t + 1);
                        stage_store(0);
                    }
                } else if (t + 1 < t1) {
                    stage_store(0);
                }
                lds_barrier();
            }
            lap(6);
        }
    }
    if (stamps) {
        vm_wait_all();
        __syncthreads();
        if (lane == 0) {
            float* o = Q.dzp + ((int64_t)blockIdx.x * NW + w) * 16;
            for (int i_ = 0; i_ < 7; ++i_) o[i_] = (float)st_[i_];
            o[8] = (float)wave_place();
            o[9] = (float)(rt0 & 0xffffffu);           // start / end, 100 MHz ticks (low bits)
            o[10] = (float)(realtime_now() & 0xffffffu);
        }
        return;
    }
    // ---- per-row outputs ----
#pragma unroll
    for (int r = 0; r < 4 && !LOSS; ++r) {
        float E = Eacc2[r >> 1][r & 1];
        float dz2[RM];
#pragma unroll
        for (int q = 0; q < RM; ++q) dz2[q] = dzn2[r >> 1][q][r & 1];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            E += __shfl_xor(E, o, 64);
#pragma unroll
            for (int q = 0; q < RM; ++q) dz2[q] += __shfl_xor(dz2[q], o, 64);
        }
        const int b = row0 + 4 * (lane >> 4) + r;
        if constexpr (D3) dz2[0] += duacc[128 + 4 * (lane >> 4) + r];  // the nonzeros' d du w_nu terms
        if ((lane & 15) == 0) {
            float* rp = Q.rowB + ((int64_t)sp * d.Bpad + b) * (2 + R);
            rp[0] = E;
            rp[1] = 0.f;  // unused slot (sum_g p_bg = 1: k_latent_bwd)
            for (int q = 0; q < R; ++q) rp[2 + q] = dz2[q < RM ? q : 0];
        }
#pragma unroll
        for (int lb = 0; lb < KP / 16; ++lb) {
            float* dp = Q.dzp + (((int64_t)sp * d.Bpad + b) * 2) * KP + 16 * lb + (lane & 15);
            dp[0] = dzA[lb][r];
            dp[KP] = dzP[lb][r];
        }
    }
    lossacc += lossacc2.x + lossacc2.y;
    const float lw = wave_sum(fmaf(0.6931471805599453f, lossd2.x + lossd2.y, lossacc));
    __syncthreads();
    if (lane == 0) part[w] = lw;
    __syncthreads();
    if (threadIdx.x == 0) {
        float l = 0.f;
#pragma unroll
        for (int i = 0; i < NW; ++i) l += part[i];
        Q.lossp[blockIdx.x] = l;
    }
}

// =======================================================================================
// k_latent_bwd — backward of reparameterisation, clamps, KL and the K x K heads
// (autograd of nb.hh:412-416, 449-450, 462-472, 498, 533-548) for 64 cells per workgroup:
//   dz = w_b (A''_b - E_b P_b),  w_b = d_b / n   (see oracle/nb_analytic.py)
// Per cell (lane = latent): dmean, dlnvar through the clamp; then the three small products
//   dh = dmean Wm + da Wl,  dWm += dmean^T h,  dWl += da^T h
// from LDS images with wave-uniform broadcast reads.  Every per-workgroup partial is a plain
// store (fixed-order sums, no atomics); k_grad_small reduces the partials.
// =======================================================================================
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_latent_bwd(NBPtrs P, Dims d, const int64_t* __restrict__ cells,
                                                    const float* __restrict__ covar,
                                                    float* __restrict__ lat, const float* __restrict__ rowx,
                                                    const float* __restrict__ rowB,
                                                    const float* __restrict__ dzp, float* __restrict__ dh,
                                                    float* __restrict__ dhT_f, __bf16* __restrict__ dhT_b,
                                                    float* __restrict__ small) {
    constexpr int CPW = LAT_CELLS / NW;  // cells per wave
    constexpr bool CHAINS = NW == 4;     // the frozen chains' layers run on 256 threads
    const int K = d.K, C = d.C, H = d.H, R = d.R, KP = d.KP, E = d.E, KE = d.KE;
    const int SMALL = small_len(K, E, KE, C, 2 * R * H + 2 * R + H + 1);
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    float* sWm = lsm;                 // [K][65]
    float* sWl = sWm + 64 * 65;       // [K][65]
    float* sDM = sWl + 64 * 65;       // [cell][68] dmean
    float* sDA = sDM + LAT_CELLS * 68;  // [cell][68] dlnvar-pre-clamp (a)
    float* sH = sDA + LAT_CELLS * 68;   // [cell][68] h0
    float* sT = sH + LAT_CELLS * 68;    // [64][17] dh0, transposed (latent-major)
    float* wpart = sT + 64 * 17;        // [NW][NSM] per-wave small partials
    const int NSM = 3 * 64 + 64 * CMAX + 2 * RMAX * HMAX + 2 * RMAX + HMAX + 1;
    // frozen chains (only with hidden layers): W stage, two gradient images, the recomputed
    // chain outputs (ReLU masks): encoder [nce], decoder z + [ncd]
    float* sCW = wpart + NW * NSM;
    float* const sG0 = sCW + 64 * 65;  // gradient images sG(0), sG(1)
    auto sG = [&](int i) { return sG0 + i * (LAT_CELLS * 68); };
    float* cimg = sG0 + 2 * LAT_CELLS * 68;  // [nce + ncd + 1][LAT_CELLS * 68]
    // diagnostic (MMVAE_DBG & 1024): realtime stamps of the phases into slabC (outputs invalid)
    const bool rts = dbg_bit(d.dbg, 1024);
    uint64_t rt_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto mark = [&](int i_) {  // constant index at every call: rt_ stays in registers
        if (rts) rt_[i_] = realtime_now();
    };
    mark(0);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = lane;
    const int cw = CPW * w;                     // this wave's first cell in the workgroup
    const int bw = blockIdx.x * LAT_CELLS + cw;  // ... in the batch
    // ---- every global input first (the waits are in issue order: one memory round) ----
    const int kk = min(k, K - 1), kr = min(k, R - 1), ke = min(k, KE - 1);
    float vval[CPW], vw[CPW], vmean[CPW], va[CPW], veps[CPW], vh[CPW], vnm[CPW], van[CPW], ven[CPW], vpre[CPW],
        vrx[CPW][HMAX];
    int64_t vcell[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        vcell[c] = covar ? cells[b] : 0;  // padding rows hold the empty row N (unit covariate: unread)
        const float* L = lat + (int64_t)b * d.lat_stride;
        vval[c] = L[d.LAT_VALID];
        vw[c] = L[d.LAT_W];
        vmean[c] = L[d.LAT_MEAN + kk];
        va[c] = L[d.LAT_A + kk];
        veps[c] = L[d.LAT_EPS + kk];
        vh[c] = L[d.LAT_H + ke];
        vnm[c] = L[d.LAT_NMEAN + kr];
        van[c] = L[d.LAT_AN + kr];
        ven[c] = L[d.LAT_EPSN + kr];
        const float* rx = rowx + (int64_t)b * d.rowx_stride;
        vpre[c] = rx[0];
#pragma unroll
        for (int hh = 0; hh < HMAX; ++hh) vrx[c][hh] = (hh < H) ? rx[2 + hh] : 0.f;
    }
    HeadsStage<64 * NW> hst;
    hst.issue(P.Wm, P.Wl, K, E);
    // the nu heads' weights (lanes k < H: dh_nu = sum_q Wnm[q][k] dnm_q + Wnl[q][k] dan_q)
    float p_wnm[RMAX], p_wnl[RMAX];
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
        p_wnm[q] = P.Wnm[min(q, R - 1) * H + min(k, H - 1)];
        p_wnl[q] = P.Wnl[min(q, R - 1) * H + min(k, H - 1)];
    }
    float dzA4[CPW], dzP4[CPW];  // the decoder GEMM input's gradient terms (KD wide)
    split_sum<CPW>(dzp, d.nsD, (int64_t)d.Bpad * 2 * KP, (int64_t)bw * 2 * KP + k, 2 * KP, k < d.KD, dzA4);
    split_sum<CPW>(dzp, d.nsD, (int64_t)d.Bpad * 2 * KP, (int64_t)bw * 2 * KP + KP + k, 2 * KP, k < d.KD, dzP4);
    float E4[CPW], dzn4[CPW];  // pass B's per-split row sums: E_b and dL/dznu_b (lanes < R)
    split_sum<CPW>(rowB, d.nsD, (int64_t)d.Bpad * (2 + R), (int64_t)bw * (2 + R), 2 + R, true, E4);
    split_sum<CPW>(rowB, d.nsD, (int64_t)d.Bpad * (2 + R), (int64_t)bw * (2 + R) + 2 + kr, 2 + R, k < R, dzn4);
    hst.store(K, E, sWm, sWl);
    mark(1);
    // with a decoder chain: dz at the latent = the chain's backward from dzd (z recomputed, the
    // chain outputs kept for the ReLU masks)
    const float* dzimg = nullptr;
    if (CHAINS && d.ncd > 0) {
        float* zimg = cimg + d.nce * LAT_CELLS * 68;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const int b = bw + c;
            const bool valid = (b < d.Bpad) && vval[c] > 0.f;
            const float lnvar = fminf(fmaxf(va[c], -4.f), 4.f);
            zimg[(cw + c) * 68 + k] = (k < K) ? vmean[c] + veps[c] * expf(lnvar / 2.f) : 0.f;
            sG(0)[(cw + c) * 68 + k] = (k < d.KD && valid) ? vw[c] * (dzA4[c] - E4[c] * dzP4[c]) : 0.f;
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
    mark(2);
    float* wp = wpart + w * NSM;
    float* p_dbm = wp;                 // [64]
    float* p_dbl = p_dbm + 64;         // [64]
    float* p_dhs = p_dbl + 64;         // [64]
    float* p_dWce = p_dhs + 64;        // [64][CMAX]
    float* p_dWnm = p_dWce + 64 * CMAX;  // [R][H]
    float* p_dWnl = p_dWnm + RMAX * HMAX;
    float* p_dbnm = p_dWnl + RMAX * HMAX;
    float* p_dbnl = p_dbnm + RMAX;
    float* p_dbne = p_dbnl + RMAX;
    float* p_dbdp = p_dbne + HMAX;
    for (int i = lane; i < NSM; i += 64) wp[i] = 0.f;
    const float bn = d.beta * d.inv_n;
    float rbm = 0.f, rbl = 0.f, rWce[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) rWce[c] = 0.f;
    float rdnm[HMAX], rdnl[HMAX], rbnm = 0.f, rbnl = 0.f, rbne = 0.f, rbdp = 0.f;
#pragma unroll
    for (int h = 0; h < HMAX; ++h) {
        rdnm[h] = 0.f;
        rdnl[h] = 0.f;
    }
    // ---- per cell: dmean, da (lane = k); the per-cell outputs to lat are stored after the loop ----
    float o_dhn[CPW], o_dpre[CPW];
    bool o_valid[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        const bool valid = (b < d.Bpad) && vval[c] > 0.f;
        const float E = E4[c];
        const float wb = vw[c];
        float dmean = 0.f, da = 0.f;
        if (k < K) {
            const float dz = dzimg ? dzimg[(cw + c) * 68 + k] : wb * (dzA4[c] - E * dzP4[c]);
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
        sH[(cw + c) * 68 + k] = (k < KE && valid) ? vh[c] : 0.f;  // dW = dmean^T h: 0 * h must be 0
        rbm += dmean;
        rbl += da;
#pragma unroll
        for (int q = 0; q < CMAX; ++q)
            if (q < C) rWce[q] += covar ? dmean * covar[vcell[c] * C + q] : dmean;  // unit: c = 1 (dmean 0 if invalid)
        // ---- overdispersion path (lanes < R) and depth (lane 0) ----
        float dnm = 0.f, dan = 0.f;
        if (k < R && valid) {
            const float dzn = dzn4[c] * d.inv_n;
            const float nm = vnm[c], an = van[c], en = ven[c];
            const float nlv = fminf(fmaxf(an, -4.f), 4.f);
            dnm = dzn + bn * nm;
            const float dnl = dzn * en * expf(nlv / 2.f) * 0.5f + bn * 0.5f * (expf(nlv) - 1.f);
            dan = (an >= -4.f && an <= 4.f) ? dnl : 0.f;
#pragma unroll
            for (int hh = 0; hh < HMAX; ++hh)
                if (hh < H) {
                    rdnm[hh] += dnm * vrx[c][hh];
                    rdnl[hh] += dan * vrx[c][hh];
                }
            rbnm += dnm;
            rbnl += dan;
        }
        float dhn = 0.f;
#pragma unroll
        for (int q = 0; q < RMAX; ++q)
            if (q < R) {
                const float a1 = __shfl(dnm, q, 64), a2 = __shfl(dan, q, 64);
                if (k < H) dhn += p_wnm[q] * a1 + p_wnl[q] * a2;
            }
        o_valid[c] = valid;
        o_dhn[c] = dhn;
        if (k < H && b < d.Bpad && valid) rbne += dhn;
        {
            const float dd = (E + 1.f) * d.inv_n;   // dL/dd_b = sum_g dmu' p = (E_b + sum_g p_bg) / n, sum p = 1
            o_dpre[c] = valid ? dd * dsoftplus(vpre[c]) : 0.f;
            if (k == 0 && b < d.Bpad) rbdp += o_dpre[c];
        }
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int b = bw + c;
        float* L = lat + (int64_t)b * d.lat_stride;
        if (k < H && b < d.Bpad) L[d.LAT_DHNU + k] = o_valid[c] ? o_dhn[c] : 0.f;
        if (k == 0 && b < d.Bpad) L[d.LAT_DPRE] = o_dpre[c];
    }
    mark(3);
    __syncthreads();
    // the heads' input: h0, or the frozen encoder chain's output (recomputed, outputs kept)
    const float* hin = sH;
    if (CHAINS && d.nce > 0) {
        hin = chain_run(d, 0, d.nce, sH, cimg, nullptr, true, sCW, w, lane);
    }
    // ---- dh0[16 cells][KE] on f32 MFMA (wave w: columns 16w..16w+15) ----
    if (w < 4) {  // (NW = 16: waves 4.. have no head columns)
        f32x4 acc = heads_dh(sDM, sDA, sWm, sWl, K, E, w, lane);
        if (CHAINS && d.nce > 0) {  // back through the encoder chain
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
                // ReLU backward: the gradient passes where the (stored, post-ReLU) h0 is > 0
                const bool pass = j < KE && (!d.relu || sH[cl * 68 + j] > 0.f);
                const float v = pass ? acc[r] : 0.f;
                sT[j * 17 + cl] = v;  // stored transposed below, 16 cells of a latent per 16 lanes
                rdhs += v;
            }
        }
        rdhs = sum_rowgroups(rdhs);
        if (lane < 16) p_dhs[j] = rdhs;  // the other waves' partials of latent j stay 0
    }
    p_dbm[k] = rbm;
    p_dbl[k] = rbl;
#pragma unroll
    for (int q = 0; q < CMAX; ++q) p_dWce[k * CMAX + q] = rWce[q];
    if (k < R) {
        for (int hh = 0; hh < H; ++hh) {
            p_dWnm[k * HMAX + hh] = rdnm[hh < HMAX ? hh : 0];
            p_dWnl[k * HMAX + hh] = rdnl[hh < HMAX ? hh : 0];
        }
        p_dbnm[k] = rbnm;
        p_dbnl[k] = rbnl;
    }
    if (k < H) p_dbne[k] = rbne;
    if (k == 0) p_dbdp[0] = rbdp;
    // ---- dWm, dWl = [dmean | da]^T h over the workgroup's cells on f32 MFMA ----
    float* out = small + (int64_t)blockIdx.x * SMALL;
    mark(4);
    if (w < 4) heads_dW(sDM, sDA, hin, K, E, w, lane, out);
    mark(5);
    __syncthreads();
    // dh^T [KP][Bpad] (the encoder backward's A operand: f32 image, or the bf16 hi [+ lo] planes)
    // from the transposed LDS tile: 16 consecutive cells of one latent per 16 lanes
    for (int i = threadIdx.x; i < KP * LAT_CELLS; i += 64 * NW) {
        const int j = i >> 4, cl = i & 15, b = blockIdx.x * LAT_CELLS + cl;
        const float v = sT[j * 17 + cl];
        if (b < d.Bpad) {
            if (dhT_f) dhT_f[(int64_t)j * d.Bpad + b] = v;
            if (dhT_b) put_op<X3>(dhT_b, j * d.Bpad + b, KP * d.Bpad, v);  // hi plane (+ the x3 lo plane)
        }
    }
    // ---- the small vectors: fixed-order sum of the four waves' partials ----
    const int o_bm = 2 * K * E, o_bl = o_bm + K, o_ce = o_bl + K, o_dhs = o_ce + K * C, o_nm = o_dhs + KE,
              o_bnm = o_nm + R * H, o_nl = o_bnm + R, o_bnl = o_nl + R * H, o_bne = o_bnl + R, o_bdp = o_bne + H;
    auto wsum = [&](int off) {  // fixed order over the waves, four at a time
        float t = (wpart[0 * NSM + off] + wpart[1 * NSM + off]) + (wpart[2 * NSM + off] + wpart[3 * NSM + off]);
#pragma unroll
        for (int i = 4; i < NW; i += 4)
            t += (wpart[i * NSM + off] + wpart[(i + 1) * NSM + off]) + (wpart[(i + 2) * NSM + off] + wpart[(i + 3) * NSM + off]);
        return t;
    };
    for (int i = threadIdx.x; i < K; i += 64 * NW) {
        out[o_bm + i] = wsum(i);
        out[o_bl + i] = wsum(64 + i);
        for (int q = 0; q < C; ++q) out[o_ce + i * C + q] = wsum(192 + i * CMAX + q);
    }
    for (int i = threadIdx.x; i < KE; i += 64 * NW) out[o_dhs + i] = wsum(128 + i);
    const int b_nm = 192 + 64 * CMAX, b_nl = b_nm + RMAX * HMAX, b_bnm = b_nl + RMAX * HMAX, b_bnl = b_bnm + RMAX,
              b_bne = b_bnl + RMAX, b_bdp = b_bne + HMAX;
    for (int i = threadIdx.x; i < R * H; i += 64 * NW) {
        const int r2 = i / H, h2 = i % H;
        out[o_nm + i] = wsum(b_nm + r2 * HMAX + h2);
        out[o_nl + i] = wsum(b_nl + r2 * HMAX + h2);
    }
    for (int i = threadIdx.x; i < R; i += 64 * NW) {
        out[o_bnm + i] = wsum(b_bnm + i);
        out[o_bnl + i] = wsum(b_bnl + i);
    }
    for (int i = threadIdx.x; i < H; i += 64 * NW) out[o_bne + i] = wsum(b_bne + i);
    if (threadIdx.x == 0) out[o_bdp] = wsum(b_bdp);
    if (rts) {
        vm_wait_all();
        mark(6);
        if (lane == 0) {
            float* o = P.dbg_out + ((int64_t)blockIdx.x * NW + w) * 8;
            for (int i = 0; i < 7; ++i) o[i] = (float)(rt_[i] & 0xffffffu);
            o[7] = (float)wave_place();
        }
    }
}

// =======================================================================================
// Gradient assembly (deterministic, fixed-order reductions)
// =======================================================================================
MMVAE_DEV void grad_small_body(const Dims& d, const float* __restrict__ small, int nwg, const NBGrads& G,
                               float* __restrict__ smallg, const float* __restrict__ lossp, int nlossp,
                               const float* __restrict__ klpart, int nkl, float* __restrict__ out, int with_grads,
                               double* __restrict__ sqpart, const int bid) {
    const int K = d.K, C = d.C, H = d.H, R = d.R, E = d.E, KE = d.KE;
    const int SMALL = small_len(K, E, KE, C, 2 * R * H + 2 * R + H + 1);
    if (bid == 0) {
        __shared__ float sb[8];
        float lsum = 0.f, ksum = 0.f;
        for (int i = threadIdx.x; i < nlossp; i += 256) lsum += lossp[i];
        for (int i = threadIdx.x; i < nkl; i += 256) ksum += klpart[i];
        float tl = block_sum<4>(lsum, sb);
        float tk = block_sum<4>(ksum, sb);
        if (threadIdx.x == 0) {
            out[0] = (tl + tk * d.beta) * d.inv_n;
            if (sqpart) sqpart[0] = 0.0;
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
    if (o < KE) { smallg[o] = s; return 0; }
    o -= KE;
    if (o < R * H) { G.Wnm[o] = s; return 1; }
    o -= R * H;
    if (o < R) { G.bnm[o] = s; return 1; }
    o -= R;
    if (o < R * H) { G.Wnl[o] = s; return 1; }
    o -= R * H;
    if (o < R) { G.bnl[o] = s; return 1; }
    o -= R;
    if (o < H) { G.bne[o] = s; return 1; }
    o -= H;
    G.bdp[0] = s;
    return 1;
    };
    double sq = 0.0;
    if ((threadIdx.x >> 5) == 0 && i < SMALL) sq = (double)s * s * store();
    if (sqpart && threadIdx.x < 64) {
        sq = wave_sum_d(sq);
        if (threadIdx.x == 0) sqpart[bid] = sq;
    }
}

__global__ __launch_bounds__(256) void k_grad_small(Dims d, const float* __restrict__ small, int nwg,
                                                    NBGrads G, float* __restrict__ smallg,
                                                    const float* __restrict__ lossp, int nlossp,
                                                    const float* __restrict__ klpart, int nkl,
                                                    float* __restrict__ out, int with_grads,
                                                    double* __restrict__ sqpart) {
    grad_small_body(d, small, nwg, G, smallg, lossp, nlossp, klpart, nkl, out, with_grads, sqpart, (int)blockIdx.x);
}

// k_enc_bwd and k_grad_small in ONE launch: both need only k_latent_bwd's outputs, so the small-
// gradient blocks (appended after the encoder blocks) run beside the encoder tail instead of as
// a separate kernel on the chain
template <class P, int KP, bool H1>
__global__ __launch_bounds__(256) void k_enc_bwd_small(EntList ents, const int64_t* __restrict__ seg,
                                                       const int32_t* __restrict__ toff, const float* __restrict__ lat,
                                                       const typename Elem<P>::type* __restrict__ dhT, int64_t dplane,
                                                       const typename WEnc<P>::type* __restrict__ WeP, Dims d,
                                                       float* __restrict__ slabE, int nenc, const float* __restrict__ small,
                                                       int nwg, NBGrads G, float* __restrict__ smallg,
                                                       const float* __restrict__ lossp, int nlossp,
                                                       const float* __restrict__ klpart, int nkl, float* __restrict__ out,
                                                       double* __restrict__ sqpart) {
    const int bid = (int)blockIdx.x;
    if (bid < nenc) enc_bwd_body<P, KP, H1, true>(ents, seg, toff, lat, dhT, dplane, WeP, d, slabE, bid);
    else grad_small_body(d, small, nwg, G, smallg, lossp, nlossp, klpart, nkl, out, 1, sqpart, bid - nenc);
}

// Per-gene gradients from the per-row-block column slabs of passes B, C and k_enc_bwd,
// summed in a fixed order (deterministic).  64 genes x NPART row-block partitions per
// workgroup: a thread reads 4 consecutive genes of every slab row with one 16-byte load (a
// wave covers 1 KB of 4 row blocks per load, all of a thread's loads independent and in
// flight together); the partitions' partial sums meet in LDS and thread g < 64 adds them in
// partition order.
// SMALL: the default widths C = R = H = 1 (9 slab rows per gene, all compile-time).
// PART: 0 = every per-gene gradient; 1 = decoder side only (slabs B, C: mu_bias, nu_bias,
// covar_decoding, nu_decoding — final after pass C, all-reduced while the encoder backward
// runs); 2 = encoder side only (slab E: x_mean, ln_x_sd, depth, nu_encoding).
static constexpr int GG_GENES = 64;  // genes per k_grad_genes workgroup
template <bool SMALL, int PART>
__global__ __launch_bounds__(256) void k_grad_genes(NBPtrs P, Dims d, NBGrads G,
                                                    const float* __restrict__ gene,
                                                    const float* __restrict__ slabB,
                                                    const float* __restrict__ slabC,
                                                    const float* __restrict__ slabE,
                                                    const float* __restrict__ smallg, int nrb, int nrbB, int nrbC,
                                                    double* __restrict__ sqpart) {
    constexpr int NQMAX = SMALL ? 9 : (1 + CMAX) + 1 + RMAX + (1 + CMAX) + 2 + HMAX;
    constexpr int NQR = NQMAX + 1;         // + the column dot sum_k cdh[k] W_enc[k][g]
    constexpr int NPART = SMALL ? 16 : 4;  // row-block partitions (LDS: NPART x NQR x 64 floats)
    constexpr int TPP = 256 / NPART;       // threads per partition: 16 (SMALL) or 64
    constexpr int GPT = GG_GENES / TPP;    // genes per thread: 4 or 1
    __shared__ float cdh[64];
    __shared__ float red[NPART][NQR][GG_GENES];
    const int C = SMALL ? 1 : d.C, R = SMALL ? 1 : d.R, H = SMALL ? 1 : d.H;
    const int nqB = (1 + C) + 1 + R, nqC = 1 + C, nqE = 2 + H;
    const int nq = nqB + nqC + nqE;
    for (int k = threadIdx.x; k < d.KE; k += 256) cdh[k] = smallg[k];
    const int part = threadIdx.x / TPP, gq = (threadIdx.x % TPP) * GPT;
    const int g0 = blockIdx.x * GG_GENES;  // DP is a multiple of 64: every slab read is in bounds
    typedef float vec __attribute__((ext_vector_type(GPT)));
    vec acc[NQMAX];
#pragma unroll
    for (int q = 0; q < NQMAX; ++q) acc[q] = vec(0.f);
    auto ld = [&](const float* p) { return *reinterpret_cast<const vec*>(p); };
    // the encoder-side column dot's W_enc loads go out first (every thread: latent rows
    // part, part + NPART, ... of its genes; W_enc is [KE][D], unpadded)
    vec gs = vec(0.f);
    if (PART != 1) {
        __syncthreads();  // cdh
#pragma unroll 4
        for (int k = part; k < d.KE; k += NPART)
#pragma unroll
            for (int i = 0; i < GPT; ++i) {
                const int gg = min(g0 + gq + i, d.D - 1);
                gs[i] = fmaf(cdh[k], P.We[(int64_t)k * d.D + gg], gs[i]);
            }
    }
#pragma unroll 2  // (4 at the headline shape: 15.4 -> 19.4 us)
    // slab rows: pass B one per workgroup (nrbB: 128 or 64 rows), pass C one per 128 rows (nrbC),
    // the encoder backward one per 64 rows (nrb)
    for (int rb = part; rb < nrb; rb += NPART) {
        const bool inB = rb < nrbB, inC = rb < nrbC;
        const float* sB = slabB + (int64_t)rb * nqB * d.DP + g0 + gq;
        const float* sC = slabC + (int64_t)rb * nqC * d.DP + g0 + gq;
        const float* sE = slabE + (int64_t)rb * nqE * d.DP + g0 + gq;
#pragma unroll
        for (int q = 0; q < NQMAX; ++q) {
            if (q < nqB) { if (PART != 2 && inB) acc[q] += ld(sB + (int64_t)q * d.DP); }
            else if (q < nqB + nqC) { if (PART != 2 && inC) acc[q] += ld(sC + (int64_t)(q - nqB) * d.DP); }
            else if (q < nq) { if (PART != 1) acc[q] += ld(sE + (int64_t)(q - nqB - nqC) * d.DP); }
        }
    }
#pragma unroll
    for (int q = 0; q < NQMAX; ++q)
#pragma unroll
        for (int i = 0; i < GPT; ++i) red[part][q][gq + i] = acc[q][i];
#pragma unroll
    for (int i = 0; i < GPT; ++i) red[part][NQMAX][gq + i] = gs[i];
    __syncthreads();
    // sum of squares of every gradient element this block writes (clip norm partial, world 1)
    double sq = 0.0;
    auto put = [&](float* dst, float v) { *dst = v; sq += (double)v * v; };
    const int g = g0 + (int)threadIdx.x;
    if (threadIdx.x < GG_GENES && g < d.D) {
    float acc[NQR];
#pragma unroll
    for (int q = 0; q < NQR; ++q) {
        float v = 0.f;
#pragma unroll
        for (int pp = 0; pp < NPART; ++pp) v += red[pp][q][threadIdx.x];
        acc[q] = v;
    }
    const float* cs1 = acc;               // [1+C]
    const float du = acc[1 + C];
    const float* duz = acc + 2 + C;       // [R]
    const float* tc = acc + nqB;          // [1+C]
    const float gl = acc[nqB + nqC];
    const float* raw = acc + nqB + nqC + 1;  // depth, nu_enc[H]
    const float inv_n = d.inv_n;
    if (PART != 2) {
        const float dl = cs1[0] - tc[0];
        put(&G.mub[g], dl);
        put(&G.bcd[g], dl);
        for (int c = 0; c < C; ++c) put(&G.Wcd[(int64_t)g * C + c], cs1[1 + c] - tc[1 + c]);
        put(&G.bnd[g], du * inv_n);
        put(&G.nub[g], -du * inv_n);
        for (int q = 0; q < R; ++q) put(&G.Wnd[(int64_t)g * R + q], duz[q] * inv_n);
    }
    if (PART != 1) {
    // encoder normalisation params (nb.hh:408-410)
    const float gs = acc[NQMAX];
    const float inv = gene[g];
    put(&G.xm[g], -inv * gs);
    const float th = P.lsd[g];
    put(&G.lsd[g], -(inv * inv) * (gl - P.xm[g] * gs) * dsoftplus(th));
    put(&G.wdp[g], raw[0]);
    for (int h = 0; h < H; ++h) put(&G.Wne[(int64_t)h * d.D + g], raw[1 + h]);
    }  // PART != 1
    }  // threadIdx.x < 64 && g < D
    if (sqpart && threadIdx.x < 64) {  // wave 0 holds every writer (threads 0..63)
        sq = wave_sum_d(sq);
        if (threadIdx.x == 0) sqpart[blockIdx.x] = sq;
    }
}

// =======================================================================================
// host-side launch orchestration
// =======================================================================================
static NBPtrs nb_ptrs(Engine* e) {
    NBPtrs P;
    P.dbg_out = e->d_slabC;
    P.xm = e->preg("x_mean");
    P.lsd = e->preg("ln_x_sd");
    P.mub = e->preg("mu_bias");
    P.nub = e->preg("nu_bias");
    P.Wce = e->preg("covar_encoding.weight");
    P.bce = e->preg("covar_encoding.bias");
    P.Wm = e->preg("mu_representation_mean.weight");
    P.bm = e->preg("mu_representation_mean.bias");
    P.Wl = e->preg("mu_representation_logvariance.weight");
    P.bl = e->preg("mu_representation_logvariance.bias");
    P.Wcd = e->preg("covar_decoding.weight");
    P.bcd = e->preg("covar_decoding.bias");
    P.Wne = e->preg("nu_encoding.weight");
    P.bne = e->preg("nu_encoding.bias");
    P.Wnm = e->preg("nu_representation_mean.weight");
    P.bnm = e->preg("nu_representation_mean.bias");
    P.Wnl = e->preg("nu_representation_logvariance.weight");
    P.bnl = e->preg("nu_representation_logvariance.bias");
    P.Wnd = e->preg("nu_decoding.weight");
    P.bnd = e->preg("nu_decoding.bias");
    P.wdp = e->preg("depth.weight");
    P.bdp = e->preg("depth.bias");
    P.We = e->pfrz(e->fz_enc_w);
    P.be = e->pfrz(e->fz_enc_b);
    P.Wd = e->pfrz(e->fz_dec_w);
    P.bd = e->pfrz(e->fz_dec_b);
    return P;
}

static NBGrads nb_grads(Engine* e) {
    NBGrads G;
    G.xm = e->greg("x_mean");
    G.lsd = e->greg("ln_x_sd");
    G.mub = e->greg("mu_bias");
    G.nub = e->greg("nu_bias");
    G.Wce = e->greg("covar_encoding.weight");
    G.bce = e->greg("covar_encoding.bias");
    G.Wm = e->greg("mu_representation_mean.weight");
    G.bm = e->greg("mu_representation_mean.bias");
    G.Wl = e->greg("mu_representation_logvariance.weight");
    G.bl = e->greg("mu_representation_logvariance.bias");
    G.Wcd = e->greg("covar_decoding.weight");
    G.bcd = e->greg("covar_decoding.bias");
    G.Wne = e->greg("nu_encoding.weight");
    G.bne = e->greg("nu_encoding.bias");
    G.Wnm = e->greg("nu_representation_mean.weight");
    G.bnm = e->greg("nu_representation_mean.bias");
    G.Wnl = e->greg("nu_representation_logvariance.weight");
    G.bnl = e->greg("nu_representation_logvariance.bias");
    G.Wnd = e->greg("nu_decoding.weight");
    G.bnd = e->greg("nu_decoding.bias");
    G.wdp = e->greg("depth.weight");
    G.bdp = e->greg("depth.bias");
    return G;
}

static Dims nb_dims(Engine* e, int64_t B, int64_t n_total, float beta) {
    Dims d;
    d.D = (int)e->D;
    d.DP = (int)e->DP;
    d.NT = (int)e->NT;
    d.K = (int)e->K;
    d.KP = (int)e->KP;
    d.C = (int)e->C;
    d.H = (int)e->H;
    d.R = (int)e->R;
    d.B = (int)B;
    d.Bpad = (int)pad_rows(B);
    d.nrb = d.Bpad / 64;
    d.nsE = e->nsplit_e;
    d.tpsE = (int)((e->NT + d.nsE - 1) / d.nsE);
    d.nsB = e->nsplit_b;
    d.tpsB = (int)((e->NT + d.nsB - 1) / d.nsB);
    d.nsD = e->nsplit_d;
    d.nsF = d.nsD;
    d.tpsD = (int)((e->NT + d.nsD - 1) / d.nsD);
    d.nsA = e->nsplit_a;
    d.tpsA = (int)((e->NT + d.nsA - 1) / d.nsA);
    d.inv_n = 1.f / (float)n_total;
    d.beta = beta;
    d.lat_stride = (int)e->lat_stride;
    d.LAT_H = (int)e->LAT_H;
    d.LAT_MEAN = (int)e->LAT_MEAN;
    d.LAT_A = (int)e->LAT_A;
    d.LAT_EPS = (int)e->LAT_EPS;
    d.LAT_NMEAN = (int)e->LAT_NMEAN;
    d.LAT_AN = (int)e->LAT_AN;
    d.LAT_EPSN = (int)e->LAT_EPSN;
    d.LAT_ZNU = (int)e->LAT_ZNU;
    d.LAT_D = (int)e->LAT_D;
    d.LAT_W = (int)e->LAT_W;
    d.LAT_VALID = (int)e->LAT_VALID;
    d.LAT_DHNU = (int)e->LAT_HNU;
    d.LAT_DPRE = (int)e->LAT_HNU + (int)e->H;
    d.rowx_stride = 2 + (int)e->H;
    d.Ncells = (int)e->N;
    d.nmv = (int)((e->DP + 255) / 256);
#ifdef MMVAE_DIAG
    { const char* ev = getenv("MMVAE_DBG"); d.dbg = ev ? atoi(ev) : 0; }
#else
    d.dbg = 0;
#endif
    d.relu = e->cfg.relu != 0;
    d.inv_wscale = 1.f / e->wscale;
    dims_hidden(e, d);
    return d;
}

__global__ void k_pack_frozen(const float* We, const float* Wd, int D, int DP, int KE, int KD, int KP,
                              float* WeP_f, __bf16* WeP_b, float* WdP_f, __bf16* WdP_b, float* WdT_f,
                              __bf16* WdT_b) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)KP * DP) return;
    const int k = (int)(i / DP), g = (int)(i % DP);
    const float we = (k < KE && g < D) ? We[(int64_t)k * D + g] : 0.f;   // [KE][D]
    const float wd = (k < KD && g < D) ? Wd[(int64_t)g * KD + k] : 0.f;  // [D][KD]
    // bf16 images carry the x3 mode's lo planes KP * DP elements after the hi planes
    const int64_t pl = (int64_t)KP * DP;
    WeP_f[i] = we;
    put_op<X3>(WeP_b, (int)i, (int)pl, we);
    WdT_f[i] = wd;
    put_op<X3>(WdT_b, (int)i, (int)pl, wd);
    WdP_f[(int64_t)g * KP + k] = wd;
    put_op<X3>(WdP_b, (int)((int64_t)g * KP + k), (int)pl, wd);
}

// ---- frozen hidden chains (shared with the vMF engine) ----------------------------------
void dims_hidden(const Engine* e, Dims& d) {
    d.KE = (int)e->KE;
    d.E = (int)e->E;
    d.KD = (int)e->KD;
    d.nce = e->nce;
    d.ncd = e->ncd;
    for (int l = 0; l < 8; ++l) {
        d.ch_in[l] = e->ch_in[l];
        d.ch_out[l] = e->ch_out[l];
        d.ch_off[l] = e->ch_off[l];
    }
    d.chain = e->d_chain;
}

// one chain layer into the chain buffer: W [out][in] (an Angular layer's normalize(relu(W) +
// 1e-4) rows, angular.hh:34-42), then the bias (0 without one).  One wave per output row.
__global__ __launch_bounds__(64) void k_chain_pack(const float* __restrict__ W, const float* __restrict__ b, int in,
                                                   int out, int angular, float* __restrict__ dst) {
    const int o = blockIdx.x, lane = threadIdx.x;
    float ss = 0.f;
    if (angular) {
        for (int i = lane; i < in; i += 64) {
            const float v = fmaxf(W[(int64_t)o * in + i], 0.f) + 1e-4f;
            ss += v * v;
        }
        ss = wave_sum(ss);
    }
    const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
    for (int i = lane; i < in; i += 64) {
        const float v = W[(int64_t)o * in + i];
        dst[(int64_t)o * in + i] = angular ? (fmaxf(v, 0.f) + 1e-4f) * inv : v;
    }
    if (lane == 0) dst[(int64_t)in * out + o] = b ? b[o] : 0.f;
}

hipError_t pack_chain(Engine* e, bool angular_enc) {
    for (int l = 0; l < e->nce + e->ncd; ++l) {
        const bool ang = angular_enc && l < e->nce;
        hipLaunchKernelGGL(k_chain_pack, dim3((unsigned)e->ch_out[l]), dim3(64), 0, e->stream, e->pfrz(e->ch_w[l]),
                           e->ch_b[l].empty() ? nullptr : e->pfrz(e->ch_b[l]), e->ch_in[l], e->ch_out[l], ang ? 1 : 0,
                           e->d_chain + e->ch_off[l]);
    }
    return hipGetLastError();
}

// fp8 mode: [DP][KP] e4m3 image of scale * W_dec[g][k] (0 past D / KD), two elements per thread
__global__ __launch_bounds__(256) void k_pack_w8(const float* __restrict__ Wd, int D, int DP, int KD, int KP,
                                                 float scale, uint8_t* __restrict__ WdP8) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (i >= (int64_t)DP * KP) return;
    const int g = (int)(i / KP), k = (int)(i % KP);
    const float a = (g < D && k < KD) ? Wd[(int64_t)g * KD + k] * scale : 0.f;
    const float b = (g < D && k + 1 < KD) ? Wd[(int64_t)g * KD + k + 1] * scale : 0.f;
    const int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    WdP8[i] = (uint8_t)(v & 0xff);
    WdP8[i + 1] = (uint8_t)((v >> 8) & 0xff);
}

hipError_t nb_prepare_frozen(Engine* e) {
    const int64_t n = e->KP * e->DP;
    if (e->cfg.dtype == MMVAE_DTYPE_FP8) {
        // power-of-two scale putting amax(W_dec) at the top of the e4m3 range (448): host amax of
        // the frozen tensor (repacked only when it changes)
        std::vector<float> w((size_t)(e->D * e->KD));
        hipError_t er = hipMemcpyAsync(w.data(), e->pfrz(e->fz_dec_w), sizeof(float) * w.size(), hipMemcpyDeviceToHost,
                                       e->stream);
        if (er == hipSuccess) er = hipStreamSynchronize(e->stream);
        if (er != hipSuccess) return er;
        float amax = 0.f;
        for (float v : w) amax = std::max(amax, std::fabs(v));
        e->wscale = amax > 0.f ? std::exp2(std::floor(std::log2(448.f / amax))) : 1.f;
        // max |W_enc| (frozen): the bound behind the encoder image's per-step scale (k_enc_scale)
        std::vector<float> we((size_t)(e->D * e->KE));
        er = hipMemcpyAsync(we.data(), e->pfrz(e->fz_enc_w), sizeof(float) * we.size(), hipMemcpyDeviceToHost, e->stream);
        if (er == hipSuccess) er = hipStreamSynchronize(e->stream);
        if (er != hipSuccess) return er;
        float wmax = 0.f;
        for (float v : we) wmax = std::max(wmax, std::fabs(v));
        e->wemax = wmax;
        hipLaunchKernelGGL(k_pack_w8, dim3((unsigned)((n / 2 + 255) / 256)), dim3(256), 0, e->stream,
                           e->pfrz(e->fz_dec_w), (int)e->D, (int)e->DP, (int)e->KD, (int)e->KP, e->wscale, e->d_WdP8);
    }
    ScopedTimer tm(e, "k_pack_frozen");
    hipLaunchKernelGGL(k_pack_frozen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream,
                       e->pfrz(e->fz_enc_w), e->pfrz(e->fz_dec_w), (int)e->D, (int)e->DP, (int)e->KE, (int)e->KD,
                       (int)e->KP, e->d_WeP_f, e->d_WeP_b, e->d_WdP_f, e->d_WdP_b, e->d_WdT_f, e->d_WdT_b);
    hipError_t er = pack_chain(e, false);
    if (er != hipSuccess) return er;
    e->frozen_dirty = false;
    // captured step graphs hold the old operands' scalars by value (the fp8 mode's 1 / wscale in
    // Dims): re-capture them
    ++e->graph_gen;
    return hipGetLastError();
}

// LDS of decoder passes A / C: double-buffered W stage (all planes) + grec tile
static size_t dec_lds(const Dims& d, int pass, int esz, int planes) {
    const int nq = 1 + d.C;
    size_t s = 2 * ((size_t)planes * 64 * d.KP * esz + 1024);
    if (pass == 2) s += (size_t)2 * 4 * nq * 64 * 4;
    return s;
}

// the single-buffered encoder forward in the x3 mode (f32: 3 waves / SIMD by VGPRs either way,
// and measured faster double-buffered at 2 workgroups per CU)
template <class P> struct EncSB { static constexpr bool value = IsX3<P>::value; };
template <class P> struct EncNW { static constexpr int value = sizeof(typename Elem<P>::type) == 2 ? 8 : 4; };
template <class P, int KP>
static size_t enc_fwd_lds(const Dims& d) {
    using T = typename Elem<P>::type;
    constexpr int NPL = IsX3<P>::value ? 2 : 1;
    constexpr int XS = sizeof(T) == 4 ? 68 : 80;
    constexpr bool SB = EncSB<P>::value;
    constexpr int NB = SB ? 1 : 2;
    return (size_t)EncLds(KP, (int)sizeof(T), d.tpsE + 1, NB * NPL * 16 * XS * (int)sizeof(T), 0, NPL,
                          Log1pTab<P, SB ? 512 : LTAB>::BYTES, MMVAE_ENC_NBW, EncNW<P>::value).bytes;
}
// the encoder operand images of mode P: bf16 planes (bf16, x3) or f32
template <class P> static const typename Elem<P>::type* op_img(const float* f, const __bf16* b) {
    if constexpr (sizeof(typename Elem<P>::type) == 2) return b;
    else return f;
}
// the encoder forward's scaled weight image: f32, bf16 planes, or the fp8 mode's e4m3 bytes
template <class P> static const typename Elem<P>::type* enc_img(const Engine* e) {
    if constexpr (IsF8<P>::value) return e->d_WeS8;
    else return op_img<P>(e->d_WeS_f, e->d_WeS_b);
}
template <class P, int KP>
static void enc_fwd_run(Engine* e, const Dims& d, float* hpart, hipStream_t st) {
    constexpr int NW = EncNW<P>::value;
    hipLaunchKernelGGL((k_enc_fwd<P, KP, EncSB<P>::value, NW>), dim3(d.nrb * 4 / NW * d.nsE), dim3(64 * NW),
                       (enc_fwd_lds<P, KP>(d)), st, ent_list(e),
                       e->d_seg, e->d_toff, enc_img<P>(e), (int64_t)e->KP * e->DP, d, hpart,
                       (const float*)e->d_escale);
}
// encoder backward operands: dh^T planes and the staged W (f32 in the x3 mode)
template <class P> static const typename WEnc<P>::type* enc_w(Engine* e) {
    if constexpr (std::is_same<typename WEnc<P>::type, __bf16>::value) return e->d_WeP_b;
    else return e->d_WeP_f;
}

static DecPtrs dec_ptrs(Engine* e, const Dims& d, const NBPtrs& P, bool bf) {
    DecPtrs Q;
    Q.lat = e->d_lat;
    Q.zf = e->d_zf;
    Q.zb = e->d_zb;
    Q.gene = e->d_gene;
    Q.Wcd = P.Wcd;
    Q.Wnd = P.Wnd;
    Q.covar = e->d_covar;
    Q.cells = e->d_cells;
    Q.rowptr = e->d_rowptr;
    Q.col = e->d_col;
    Q.val = e->d_val;
    Q.rtp = e->d_rtp;
    Q.ents = ent_list(e);
    Q.seg = e->d_seg;
    Q.toff = e->d_toff;
    Q.WdP = e->cfg.dtype == MMVAE_DTYPE_FP8 ? (const void*)e->d_WdP8 : bf ? (const void*)e->d_WdP_b : (const void*)e->d_WdP_f;
    Q.WdT = bf ? (const void*)e->d_WdT_b : (const void*)e->d_WdT_f;
    Q.lsep = e->d_lsep;
    Q.rowfin = e->d_rowfin;
    Q.rowB = e->d_rowB;
    Q.dzp = e->d_dzp;
    Q.slabB = e->d_slabB;
    Q.slabC = e->d_slabC;
    Q.lossp = e->d_lossp;
    Q.zplane = (int64_t)d.Bpad * d.KP;
    Q.wplane = (int64_t)e->KP * e->DP;
    return Q;
}

// k_latent_fwd: one cell per wave (16 waves, 1024 threads) when there are no frozen hidden
// chains; MMVAE_LAT_NW=4 forces the 4-wave instance (4 cells per wave)
static bool latent_nw16(const Dims& d) {
    static const bool nw4 = getenv_is("MMVAE_LAT_NW", "4");
    return !nw4 && d.nce == 0 && d.ncd == 0;
}
static void latent_fwd_launch(Engine* e, const NBPtrs& P, const Dims& d, const float* covar, const float* eps,
                              const int32_t* perm, int mode, float* out_mean, float* out_lnvar, hipStream_t st) {
    const bool nw16 = latent_nw16(d);
    auto go = [&](auto kern, int nth) {
        hipLaunchKernelGGL(kern, dim3(e->n_lat_wg), dim3(nth), 0, st, P, d, e->d_cells, covar, e->d_hpart, e->d_mvec,
                           e->d_rowxp, e->d_rowx, eps, perm, e->cfg.seed, e->d_ss, e->d_lat, e->d_zf, e->d_zb,
                           e->d_lossp + e->klp_off, mode, out_mean, out_lnvar);
    };
    if (nw16) go(k_latent_fwd<16>, 1024);
    else go(k_latent_fwd<4>, 256);
}

// k_latent_bwd's LDS: head weights, 3 cell images, the per-wave partials; with hidden layers
// also the chain W stage, 2 gradient images and the recomputed chain outputs
static size_t latent_bwd_lds(const Engine* e, int nw) {
    const int NSM = 3 * 64 + 64 * CMAX + 2 * RMAX * HMAX + 2 * RMAX + HMAX + 1;
    size_t f = 2 * 64 * 65 + 3 * LAT_CELLS * 68 + 64 * 17 + (size_t)nw * NSM;
    if (e->nce + e->ncd > 0) f += 64 * 65 + (size_t)(2 + e->nce + e->ncd + 1) * LAT_CELLS * 68;
    return f * 4;
}

template <class PM, int KP>
static hipError_t nb_launch_all(Engine* e, const Dims& d, const NBPtrs& P, bool update, bool use_eps) {
    // PB: the encoder / dz GEMM policy (bf16 in the fp8 mode), PM: the logit GEMM's
    using PB = typename Bf16If8<PM>::type;
    using T = typename Elem<PB>::type;
    using TL = typename Elem<PM>::type;
    constexpr bool X = IsX3<PB>::value;
    constexpr int NPL = X ? 2 : 1;
    const bool bf = sizeof(T) == 2;  // bf16 planes (bf16 and x3 modes)
    hipStream_t st = e->stream;
    const int nrb = d.nrb;
    float* gene = e->d_gene;  // k_prep ran before the batch lists (nb_prep)
    // unit covariate (no covariate file): the CM = 0 decoder instances fold it into per-gene
    // constants, and the latent kernels skip the covariate gather (a null pointer: c = 1)
    const bool ucov = d.C == 1 && e->unit_covar;
    const float* lat_covar = ucov ? nullptr : e->d_covar;
    {
        ScopedTimer tm(e, "k_enc_fwd");
        enc_fwd_run<PM, KP>(e, d, e->d_hpart, st);  // fp8 mode: the e4m3 encoder GEMM (PM = F8)
    }
    {
        ScopedTimer tm(e, "k_latent_fwd");
        latent_fwd_launch(e, P, d, lat_covar, use_eps ? e->d_eps : nullptr, e->perm_active ? e->d_perm : nullptr, 0,
                          nullptr, nullptr, st);
    }
    const DecPtrs Q = dec_ptrs(e, d, P, bf);
    const bool small_cr = (d.C == 1 && d.R == 1);
    // pass B: 16 NW rows per workgroup.  bf16: NW = 8 with double-buffered stages (one barrier
    // per tile); x3: NW = 8 single-buffered (the hi + lo images of double buffers exceed the
    // 160 KB LDS); f32 or MMVAE_DEC_NW=4: NW = 4 (64 rows, two workgroups per CU)
    const int nqB = (1 + d.C) + 1 + d.R;
    const int csz = (bf && !X) ? 4 : 8;
    const bool nw4 = getenv_is("MMVAE_DEC_NW", "4");
    const size_t ldsB8 = DecNBLds(KP, (int)sizeof(T), d.tpsD + 1, nqB, 3 + 1 + 1, csz, 8, X ? 1 : 2, NPL, (int)sizeof(TL)).bytes;
    // x3 with MMVAE_DEC3=1 (read at create, Engine::dec3): the three-waves-per-SIMD instance
    // (4-wave workgroups, three per CU; the gene split was sized for three at create)
    const size_t lds3 = DecNBLds(KP, (int)sizeof(T), d.tpsD + 1, nqB, 3 + 1 + 1, csz, 4, 1, NPL, (int)sizeof(TL), false, true, true).bytes;
    const bool use_d3 = X && e->dec3 && small_cr && 3 * ((lds3 + 2047) / 2048 * 2048) <= 160 * 1024;  // 2 KB LDS granule
    const int nwB = use_d3 ? 4 : (small_cr && bf && ldsB8 <= 160 * 1024 && !nw4) ? 8 : 4;
    const dim3 gdecB(nrb / (nwB / 4) * d.nsD);
    const dim3 gdecA(nrb / 2 * d.nsA);  // passes A / C: 128 rows per workgroup
    const size_t ldsA = dec_lds(d, 0, (int)sizeof(TL), NPL), ldsC = dec_lds(d, 2, (int)sizeof(TL), NPL);
    {
        ScopedTimer tm(e, "k_dec_lse");
        if (ucov) hipLaunchKernelGGL((k_dec_lse<PM, KP, 0>), gdecA, dim3(256), ldsA, st, Q, d);
        else if (d.C == 1) hipLaunchKernelGGL((k_dec_lse<PM, KP, 1>), gdecA, dim3(256), ldsA, st, Q, d);
        else hipLaunchKernelGGL((k_dec_lse<PM, KP, CMAX>), gdecA, dim3(256), ldsA, st, Q, d);
    }
    // x3 training, MMVAE_DEC_SG=1: the staggered instance (waves 4-7 half a tile behind).
    // Measured slower than the lock-step one (x3 k_dec_nb 264.9 vs 249.0 us at the headline
    // shape), so it is a diagnostic variant, not the default
    static const bool sg_on = getenv_is("MMVAE_DEC_SG", "1");
    const size_t ldsSG = DecNBLds(KP, (int)sizeof(T), d.tpsD + 1, nqB, 3 + 1 + 1, csz, 8, 2, NPL, (int)sizeof(TL), false, true).bytes;
    const bool use_sg = X && nwB == 8 && sg_on && ldsSG <= 160 * 1024;
    // the x3 instance double-buffered without a WdT stage (SG's layout, lock-step waves): one
    // barrier per tile instead of two (k_dec_nb 244.8 -> 241.2 us); MMVAE_DEC_TRWDB=0: the
    // single-buffered instance with its WdT stage
    static const bool trwdb_on = !getenv_is("MMVAE_DEC_TRWDB", "0");
    const bool use_trwdb = X && nwB == 8 && trwdb_on && !use_sg && ldsSG <= 160 * 1024;
    auto launch_b = [&](auto loss_c) {
        constexpr bool LS = decltype(loss_c)::value;
        if constexpr (X && !LS && std::is_same<PB, PM>::value) {
            if (use_d3) {
                if (ucov) hipLaunchKernelGGL((k_dec_nb<PB, KP, 0, 1, 4, false, PM, false, false, true, true>), gdecB, dim3(256), lds3, st, Q, d);
                else hipLaunchKernelGGL((k_dec_nb<PB, KP, 1, 1, 4, false, PM, false, false, true, true>), gdecB, dim3(256), lds3, st, Q, d);
                return;
            }
        }
        if (nwB == 8) {
            const size_t lds = LS ? DecNBLds(KP, (int)sizeof(T), d.tpsD + 1, nqB, 3 + 1 + 1, csz, 8, X ? 1 : 2, NPL, (int)sizeof(TL), true).bytes
                                  : ldsB8;
            if constexpr (X && !LS) {
                if (use_sg) {
                    hipLaunchKernelGGL((k_dec_nb<PB, KP, 1, 1, 8, true, PM, false, true>), gdecB, dim3(512), ldsSG, st, Q, d);
                    return;
                }
                if (use_trwdb) {
                    if (ucov) hipLaunchKernelGGL((k_dec_nb<PB, KP, 0, 1, 8, true, PM, false, false, true>), gdecB, dim3(512), ldsSG, st, Q, d);
                    else hipLaunchKernelGGL((k_dec_nb<PB, KP, 1, 1, 8, true, PM, false, false, true>), gdecB, dim3(512), ldsSG, st, Q, d);
                    return;
                }
            }
            if constexpr (sizeof(T) == 2) {
                if (ucov) hipLaunchKernelGGL((k_dec_nb<PB, KP, 0, 1, 8, !X, PM, LS>), gdecB, dim3(512), lds, st, Q, d);
                else hipLaunchKernelGGL((k_dec_nb<PB, KP, 1, 1, 8, !X, PM, LS>), gdecB, dim3(512), lds, st, Q, d);
            }
        } else if (small_cr) {
            const size_t lds4 = DecNBLds(KP, (int)sizeof(T), d.tpsD + 1, nqB, 3 + 1 + 1, csz, 4, 1, NPL, (int)sizeof(TL), LS).bytes;
            if (ucov) hipLaunchKernelGGL((k_dec_nb<PB, KP, 0, 1, 4, false, PM, LS>), gdecB, dim3(256), lds4, st, Q, d);
            else hipLaunchKernelGGL((k_dec_nb<PB, KP, 1, 1, 4, false, PM, LS>), gdecB, dim3(256), lds4, st, Q, d);
        } else
            hipLaunchKernelGGL((k_dec_nb<PB, KP, CMAX, RMAX, 4, false, PM, LS>), gdecB, dim3(256),
                               (size_t)DecNBLds(KP, (int)sizeof(T), d.tpsD + 1, nqB, 3 + RMAX + CMAX, csz, 4, 1, NPL, (int)sizeof(TL), LS).bytes, st, Q, d);
    };
    {
        // eval (update = 0): the loss-only instance (MMVAE_EVAL_FULL=1: the full pass, diagnostic)
        ScopedTimer tm(e, update ? "k_dec_nb" : "k_dec_nb_loss");
        static const bool eval_full = getenv_is("MMVAE_EVAL_FULL", "1");
        if (update || eval_full) launch_b(std::false_type{});
        else launch_b(std::true_type{});
    }
    NBGrads G = nb_grads(e);
    if (!update) {
        ScopedTimer tm(e, "k_loss");
        hipLaunchKernelGGL(k_grad_small, dim3(1), dim3(256), 0, st, d, e->d_small, 0, G, e->d_smallg, e->d_lossp,
                           (int)gdecB.x, e->d_lossp + e->klp_off, e->n_lat_wg, e->d_out, 0, nullptr);
        return hipGetLastError();
    }
    {
        ScopedTimer tm(e, "k_dec_tail");
        if (ucov) hipLaunchKernelGGL((k_dec_tail<PM, KP, 0>), gdecA, dim3(256), ldsC, st, Q, d);
        else if (d.C == 1) hipLaunchKernelGGL((k_dec_tail<PM, KP, 1>), gdecA, dim3(256), ldsC, st, Q, d);
        else hipLaunchKernelGGL((k_dec_tail<PM, KP, CMAX>), gdecA, dim3(256), ldsC, st, Q, d);
    }
    const bool split = split_grads(e);
    const bool small_genes = d.C == 1 && d.R == 1 && d.H == 1;
    const int nrbB = nrb / (nwB / 4), nrbC = nrb / 2;  // slab rows of passes B and C
    if (split) {  // decoder-side gene gradients final: all-reduce them under the encoder backward
        ScopedTimer tm(e, "k_grad_genes_dec");
        if (small_genes)
            hipLaunchKernelGGL((k_grad_genes<true, 1>), dim3((d.D + GG_GENES - 1) / GG_GENES), dim3(256), 0, st, P, d, G, gene,
                               e->d_slabB, e->d_slabC, e->d_slabE, e->d_smallg, nrb, nrbB, nrbC, nullptr);
        else
            hipLaunchKernelGGL((k_grad_genes<false, 1>), dim3((d.D + GG_GENES - 1) / GG_GENES), dim3(256), 0, st, P, d, G, gene,
                               e->d_slabB, e->d_slabC, e->d_slabE, e->d_smallg, nrb, nrbB, nrbC, nullptr);
        hipError_t er = comm_bucket(e, 0);
        if (er != hipSuccess) return er;
    }
    {
        ScopedTimer tm(e, "k_latent_bwd");
        const bool nw16 = latent_nw16(d);
        const size_t lds = latent_bwd_lds(e, nw16 ? 16 : 4);
        auto go = [&](auto kern, int nth) {
            // the encoder backward reads one dh^T image: bf16 planes (bf16, x3 and fp8 modes) or f32
            hipLaunchKernelGGL(kern, dim3(e->n_lat_wg), dim3(nth), lds, st, P, d, e->d_cells, lat_covar, e->d_lat,
                               e->d_rowx, e->d_rowB, e->d_dzp, e->d_dh, bf ? nullptr : e->d_dhT_f,
                               bf ? e->d_dhT_b : nullptr, e->d_small);
        };
        if (nw16) go(k_latent_bwd<16>, 1024);
        else go(k_latent_bwd<4>, 256);
    }
    // world 1 (no split): the gradient kernels also write the clip norm's sum-of-squares partials
    // (one double per block, fixed order), so k_adam folds them and k_sumsq is skipped
    const int SMALL = small_len(d.K, d.E, d.KE, d.C, 2 * d.R * d.H + 2 * d.R + d.H + 1);
    const int gS = 1 + (SMALL + 31) / 32, gG = (d.D + GG_GENES - 1) / GG_GENES;
    const bool fuse_sq = !split && !(e->comm_active());  // no all-reduce after these kernels
    double* sqS = fuse_sq ? e->d_sumsq : nullptr;
    double* sqG = fuse_sq ? e->d_sumsq + gS : nullptr;
    {
        // encoder backward + the small-parameter gradients / loss in one launch
        ScopedTimer tm(e, "k_enc_bwd");
        const auto* WeT = enc_w<PB>(e);
        const T* dhT = op_img<PB>(e->d_dhT_f, e->d_dhT_b);
        const int64_t dpl = (int64_t)KP * d.Bpad;
        const int nenc = nrb * d.nsB;
        if (d.H == 1)
            hipLaunchKernelGGL((k_enc_bwd_small<PB, KP, true>), dim3(nenc + gS), dim3(256), (enc_bwd_lds<PB, KP>(d)), st,
                               ent_list(e), e->d_seg, e->d_toff, e->d_lat, dhT, dpl, WeT, d, e->d_slabE, nenc, e->d_small,
                               e->n_lat_wg, G, e->d_smallg, e->d_lossp, (int)gdecB.x, e->d_lossp + e->klp_off,
                               e->n_lat_wg, e->d_out, sqS);
        else
            hipLaunchKernelGGL((k_enc_bwd_small<PB, KP, false>), dim3(nenc + gS), dim3(256), (enc_bwd_lds<PB, KP>(d)), st,
                               ent_list(e), e->d_seg, e->d_toff, e->d_lat, dhT, dpl, WeT, d, e->d_slabE, nenc, e->d_small,
                               e->n_lat_wg, G, e->d_smallg, e->d_lossp, (int)gdecB.x, e->d_lossp + e->klp_off,
                               e->n_lat_wg, e->d_out, sqS);
    }
    {
        ScopedTimer tm(e, "k_grad_genes");
        if (small_genes) {
            if (split)
                hipLaunchKernelGGL((k_grad_genes<true, 2>), dim3(gG), dim3(256), 0, st, P, d, G, gene,
                                   e->d_slabB, e->d_slabC, e->d_slabE, e->d_smallg, nrb, nrbB, nrbC, sqG);
            else
                hipLaunchKernelGGL((k_grad_genes<true, 0>), dim3(gG), dim3(256), 0, st, P, d, G, gene,
                                   e->d_slabB, e->d_slabC, e->d_slabE, e->d_smallg, nrb, nrbB, nrbC, sqG);
        } else {
            if (split)
                hipLaunchKernelGGL((k_grad_genes<false, 2>), dim3(gG), dim3(256), 0, st, P, d, G, gene,
                                   e->d_slabB, e->d_slabC, e->d_slabE, e->d_smallg, nrb, nrbB, nrbC, sqG);
            else
                hipLaunchKernelGGL((k_grad_genes<false, 0>), dim3(gG), dim3(256), 0, st, P, d, G, gene,
                                   e->d_slabB, e->d_slabC, e->d_slabE, e->d_smallg, nrb, nrbB, nrbC, sqG);
        }
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

// k_prep: launched ahead of the batch lists (whose raw-count dots read its packed weights)
hipError_t nb_prep(Engine* e, int64_t B, int64_t n_total, float beta) {
    if (e->frozen_dirty) {
        hipError_t er = nb_prepare_frozen(e);
        if (er != hipSuccess) return er;
    }
    const Dims d = nb_dims(e, B, n_total, beta);
    const NBPtrs P = nb_ptrs(e);
    const bool bf = e->cfg.dtype != MMVAE_DTYPE_F32;  // bf16 planes (bf16, x3)
    const bool f8 = e->cfg.dtype == MMVAE_DTYPE_FP8;
    if (f8) {
        ScopedTimer tm(e, "k_enc_scale");
        hipLaunchKernelGGL(k_enc_scale, dim3(1), dim3(1024), 0, e->stream, P.lsd, (int)e->D, e->wemax, e->d_escale);
    }
    ScopedTimer tm(e, "k_prep");
    hipLaunchKernelGGL(k_prep, dim3((d.DP + 255) / 256, d.KP / 8), dim3(256), 0, e->stream, P, d, e->d_gene, e->d_WeP_f,
                       e->d_WeS_f, bf ? e->d_WeS_b : nullptr, e->d_mvec, stage_copy_args(e),
                       f8 ? e->d_WeS8 : nullptr, (const float*)e->d_escale);
    return hipGetLastError();
}

hipError_t nb_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps) {
    if (e->frozen_dirty) {
        hipError_t er = nb_prepare_frozen(e);
        if (er != hipSuccess) return er;
    }
    const Dims d = nb_dims(e, B, n_total, beta);
    const NBPtrs P = nb_ptrs(e);
    return dispatch_mode(e, [&](auto p, auto kp) {
        return nb_launch_all<decltype(p), decltype(kp)::value>(e, d, P, update, use_eps);
    });
}

template <class PM, int KP>
static hipError_t nb_encode_t(Engine* e, const Dims& d, const NBPtrs& P, float* d_mean, float* d_lnvar) {
    hipStream_t st = e->stream;
    enc_fwd_run<PM, KP>(e, d, e->d_hpart, st);
    latent_fwd_launch(e, P, d, e->d_covar, nullptr, nullptr, 1, d_mean, d_lnvar, st);
    return hipGetLastError();
}

hipError_t nb_encode(Engine* e, int64_t B, float* d_mean, float* d_lnvar) {
    if (e->frozen_dirty) {
        hipError_t er = nb_prepare_frozen(e);
        if (er != hipSuccess) return er;
    }
    const Dims d = nb_dims(e, B, B, 1.f);
    const NBPtrs P = nb_ptrs(e);
    return dispatch_mode(e, [&](auto p, auto kp) {
        return nb_encode_t<decltype(p), decltype(kp)::value>(e, d, P, d_mean, d_lnvar);
    });
}

// ---- encoder kernels shared with the vMF engine (vmf_kernels.hip) ----------------------
hipError_t enc_forward_launch(Engine* e, const Dims& d, float* hpart) {
    if (e->cfg.dtype == MMVAE_DTYPE_FP8) {  // BASELINE configs[4]: the encoder GEMM on e4m3 too
        if (e->KP == 32) enc_fwd_run<F8, 32>(e, d, hpart, e->stream);
        else enc_fwd_run<F8, 64>(e, d, hpart, e->stream);
        return hipGetLastError();
    }
    return dispatch_mode<false>(e, [&](auto p, auto kp) {
        enc_fwd_run<decltype(p), decltype(kp)::value>(e, d, hpart, e->stream);
        return hipGetLastError();
    });
}

}  // namespace mmvae
