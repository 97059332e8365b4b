// Shared device-side pieces of the NB and vMF engines: launch dimensions, wave helpers,
// the batch entry-list reader (16 cells x 64 genes densified per tile) and the
// register-staged LDS tile copy.  Device-inline only: every __global__ kernel lives in
// exactly one translation unit (nb_kernels.hip / vmf_kernels.hip).
#pragma once
#include <type_traits>

#include "common.hpp"

namespace mmvae {

static constexpr int CMAX = 8, HMAX = 8, RMAX = 8;
static constexpr int LAT_CELLS = 16;  // cells per 256-thread workgroup of the latent-head kernels

struct Dims {
    int D, DP, NT, K, KP, C, H, R;
    int B, Bpad, nrb;
    int nsE, tpsE;  // encoder (forward) splits, tiles per split
    int nsB, tpsB;  // encoder backward splits
    int nsD, tpsD;  // decoder pass-B splits
    int nsF, tpsF;  // vMF decoder forward pass splits (its own occupancy; = nsD otherwise)
    int nsA, tpsA;  // decoder passes A / C splits
    float inv_n, beta;
    int lat_stride, LAT_H, LAT_MEAN, LAT_A, LAT_EPS, LAT_NMEAN, LAT_AN, LAT_EPSN, LAT_ZNU, LAT_D,
        LAT_W, LAT_VALID, LAT_DHNU, LAT_DPRE;
    int rowx_stride;  // 2 + H : pre, lnorm2, hnu[H]
    int Ncells;       // dataset rows: row Ncells of the per-cell tile index is the empty row
    int nmv;          // mvec partial blocks (256 genes each) written by the prep kernel
    int dbg;          // diagnostic ablation bits (MMVAE_DBG env, diagnostic builds only; dbg_bit)
    int relu;         // ReLU on the frozen encoder's output h (nb.hh:345-346, vmf.hh:351-352)
    float inv_wscale; // fp8 mode: 1 / the power-of-two scale of the e4m3 decoder weight (else 1)
    // frozen hidden layers (nb.hh:331-379, vmf.hh:338-385): KE = rows of the big encoder GEMM
    // (h0), E = input width of the heads, KD = input width of the big decoder GEMM (zd).  Chain
    // layer l (encoder layers 0 .. nce-1, then decoder layers nce .. nce+ncd-1) is
    // W [ch_out][ch_in] row-major at chain + ch_off[l], then its bias [ch_out] (zeros for an
    // Angular layer, whose W is stored normalised: k_chain_pack).  A ReLU follows every chain
    // layer when relu is set (NB encoder chains never have one: Q2 rejects --relu there).
    int KE, E, KD;
    int nce, ncd;
    int ch_in[8], ch_out[8], ch_off[8];
    const float* chain;
};

// Widths and the layout of the per-workgroup partials of the latent-head backward (k_latent_bwd
// / k_vlatent_bwd -> k_grad_small): dWm [K][E] | dWl [K][E] | dbm [K] | dbl [K] | dWce [K][C] |
// colsum dh0 [KE] | the NB overdispersion block (nb: 2RH + 2R + H + 1, vMF: 0)
// Diagnostic ablation / stamp bits (MMVAE_DBG): live only in diagnostic builds (-DMMVAE_DIAG,
// tools/build_variant.sh diag "-DMMVAE_DIAG"); product builds fold every test to false.
#ifdef MMVAE_DIAG
MMVAE_HOSTDEV bool dbg_bit(int dbg, int bit) { return (dbg & bit) != 0; }
#else
MMVAE_HOSTDEV constexpr bool dbg_bit(int, int) { return false; }
#endif

MMVAE_HOSTDEV int small_len(int K, int E, int KE, int C, int nbx) { return 2 * K * E + 2 * K + K * C + KE + nbx; }

// The step's staged block (cells | segments | permutation | step scalars, pinned host memory)
// copied into device memory by the prep kernel's y = 0 blocks: the first kernel of a step reads
// it straight from the mapped host block, instead of a separate copy launch.
struct StageCopy {
    const uint4* src;  // pinned host block (device-accessible)
    uint4* dst;
    int n16;           // 16-byte chunks
};
// The copy, split in two: load() issues this thread's first chunk (an unconditional load:
// blocks with y != 0, or with no staged block, read the first chunk of the destination block
// instead — engine-owned device memory, 16-byte aligned, at least one chunk long; the value is
// unused), store() writes it and copies any further chunks.  A kernel issues load() after its
// own loads, so waiting for those never waits for the slower host-memory read (loads retire in
// issue order).
struct StageHold {
    uint4 v;
    int i;
    bool on;
    MMVAE_DEV void load(const StageCopy& sc) {
        on = blockIdx.y == 0 && sc.src && sc.n16 > 0;
        i = blockIdx.x * 256 + threadIdx.x;
        v = *(on ? sc.src + min(i, sc.n16 - 1) : sc.dst);
    }
    MMVAE_DEV void store(const StageCopy& sc) const {
        if (!on) return;
        if (i < sc.n16) sc.dst[i] = v;
        for (int j = i + gridDim.x * 256; j < sc.n16; j += gridDim.x * 256) sc.dst[j] = sc.src[j];
    }
};

// out[c] = sum over splits s < ns of p[s * sstride + off + c * cstride], c < NC (NC = 4 or 1 cells):
// the split partials, loads issued 16 / NC splits at a time (independent, then summed).  The
// summation order is the same for any NC — groups of four splits, (v0 + v1) + (v2 + v3), added in
// split order, then the single splits — so a cell's sum does not depend on the cells per wave.
template <int NC>
MMVAE_DEV void split_sum(const float* __restrict__ p, int ns, int64_t sstride, int64_t off, int64_t cstride, bool on,
                         float (&out)[NC]) {
    static_assert(NC == 1 || NC == 2 || NC == 4, "split_sum: 1, 2 or 4 cells");
    constexpr int G = 16 / NC;  // splits per batch of loads
#pragma unroll
    for (int c = 0; c < NC; ++c) out[c] = 0.f;
    if (!on) return;
    int s = 0;
    for (; s + G <= ns; s += G) {
        float v[G][NC];
#pragma unroll
        for (int u = 0; u < G; ++u)
#pragma unroll
            for (int c = 0; c < NC; ++c) v[u][c] = p[(int64_t)(s + u) * sstride + off + c * cstride];
#pragma unroll
        for (int g = 0; g < G / 4; ++g)
#pragma unroll
            for (int c = 0; c < NC; ++c) out[c] += (v[4 * g][c] + v[4 * g + 1][c]) + (v[4 * g + 2][c] + v[4 * g + 3][c]);
    }
    for (; s + 4 <= ns; s += 4) {
        float v[4][NC];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < NC; ++c) v[u][c] = p[(int64_t)(s + u) * sstride + off + c * cstride];
#pragma unroll
        for (int c = 0; c < NC; ++c) out[c] += (v[0][c] + v[1][c]) + (v[2][c] + v[3][c]);
    }
    for (; s < ns; ++s)
#pragma unroll
        for (int c = 0; c < NC; ++c) out[c] += p[(int64_t)s * sstride + off + c * cstride];
}
MMVAE_DEV void split_sum4(const float* __restrict__ p, int ns, int64_t sstride, int64_t off, int64_t cstride, bool on,
                          float (&out)[4]) {
    split_sum<4>(p, ns, sstride, off, cstride, on, out);
}

// (gene split sp, row block rb) of flat workgroup id bid < nrb * ns.  Workgroups b and b + 8
// share an XCD and its L2 (round-robin dispatch, MI355X_MICROARCH.md "Workgroup dispatch"), so
// the nrb * ns / 8 items of one XCD are taken consecutively in split-major order: the workgroups
// reading a gene split's weight tiles sit on one or two XCDs, and each L2 holds about 1/8 of the
// weights instead of all of them.  (MMVAE_XCD_MAJOR=0 at build: bid % ns, bid / ns.)
#ifndef MMVAE_XCD_MAJOR
#define MMVAE_XCD_MAJOR 1
#endif
MMVAE_DEV void xcd_split_major(int bid, int nrb, int ns, int& sp, int& rb) {
    const int n = nrb * ns;
    if (MMVAE_XCD_MAJOR && (n & 7) == 0) {
        const int j = (bid & 7) * (n >> 3) + (bid >> 3);
        sp = j / nrb;
        rb = j - sp * nrb;
    } else {
        sp = bid % ns;
        rb = bid / ns;
    }
}

MMVAE_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NW>
MMVAE_DEV float block_sum(float v, float* sbuf) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sbuf[w] = v;
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x == 0)
        for (int i = 0; i < NW; ++i) t += sbuf[i];
    return t;  // valid in thread 0
}

// The per-step batch entry lists (batch.hip): one 32-bit word per entry, bits 0-9 the position
// (row-in-block << 6 | gene-in-tile), bits 10-31 the count when every value of the dataset is an
// integer in [0, 2^22) (Engine::ent_xm false, the counts of scRNA data and of the bench).  Other
// data (fractional values) keep the value as a float in a parallel array, words xoff.. of the
// same buffer.  The x word is loaded unconditionally (index 0 when xoff = 0: one broadcast word),
// so every load of a tile stays statically counted.
MMVAE_DEV int ent_row(uint32_t e) { return (int)((e >> 6) & 15); }
MMVAE_DEV int ent_gene(uint32_t e) { return (int)(e & 63); }
MMVAE_DEV float ent_x(const EntList& L, uint32_t e, float xw) { return L.xoff ? xw : (float)(e >> 10); }
MMVAE_DEV float ent_xload(const EntList& L, int64_t i) {
    return reinterpret_cast<const float*>(L.w)[L.xoff ? L.xoff + i : 0];
}
// One tile's entries of a wave's 16 rows: lane l takes entries l and l + 64 (prefetched a tile
// ahead), entries past 128 are read on the spot.  toffl = the wave block's tile offsets
// t0 .. t0 + S - 1 (LDS), seg = the block's first entry.
struct ListEntries {
    int n;
    int64_t base;
    uint32_t raw[2];  // the loaded words as they are: nothing reads them before visit (a select on
    float xw[2];      // them at fetch time would make the compiler wait for the loads right there)
    MMVAE_DEV void fetch(const EntList& L, int64_t seg, const int32_t* toffl, int tl, int lane) {
        const int a = toffl[tl];
        n = toffl[tl + 1] - a;
        base = seg + a;
#pragma unroll
        for (int k = 0; k < 2; ++k) {  // unconditional loads (the list buffer has 64 spare entries)
            const int e = lane + 64 * k;
            const int64_t i = base + (e < n ? e : 0);
            raw[k] = L.w[i];
            xw[k] = ent_xload(L, i);
        }
    }
    // packed position (row-in-block << 6 | gene-in-tile) of register entry k, -1 past the list
    MMVAE_DEV int pos(int k, int lane) const { return (lane + 64 * k < n) ? (int)(raw[k] & 1023u) : -1; }
    MMVAE_DEV float x(const EntList& L, int k) const { return ent_x(L, raw[k], xw[k]); }
    // f(pos A, x A, pos B, x B, B valid) for the tile's entries two at a time: A = lane,
    // B = lane + 64, then lane + 128 / + 192, ... (the packed-pair sparse passes; an invalid B
    // holds a real entry of the tile, to be neither stored nor counted)
    template <class F>
    MMVAE_DEV void visit2(const EntList& L, int lane, F&& f) const {
        if (lane < n) f(raw[0], x(L, 0), raw[1], x(L, 1), lane + 64 < n);
        for (int e = 128 + lane; e < n; e += 128) {
            const bool vb = e + 64 < n;
            const int64_t ia = base + e, ib = base + (vb ? e + 64 : e);
            const uint32_t ea = L.w[ia], eb = L.w[ib];
            const float xa = ent_xload(L, ia), xb = ent_xload(L, ib);
            f(ea, ent_x(L, ea, xa), eb, ent_x(L, eb, xb), vb);
        }
    }
    // f(row-in-block, gene-in-tile, x) for every entry of the tile
    template <class F>
    MMVAE_DEV void visit(const EntList& L, int lane, F&& f) const {
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (lane + 64 * k < n) f(ent_row(raw[k]), ent_gene(raw[k]), x(L, k));
        for (int e = 128 + lane; e < n; e += 64) {
            const uint32_t r = L.w[base + e];
            const float xv = ent_xload(L, base + e);
            f(ent_row(r), ent_gene(r), ent_x(L, r, xv));
        }
    }
};
// the wave block's tile offsets for the split's tiles t0 .. t0 + S - 1 into LDS
MMVAE_DEV void fill_toffl(int32_t* toffl, int S, int t0, int NT, const int32_t* __restrict__ toff, int wb, int lane) {
    for (int i = lane; i < S; i += 64) toffl[i] = toff[(int64_t)wb * (NT + 1) + min(t0 + i, NT)];
}

// log1p of a count: exact libm form in the fp32-accurate modes (f32, x3); for bf16 operand tiles
// one v_log of 1 + x (x >= 0: relative error <= 6e-8 / x, far below bf16's 4e-3 for any
// x >= 1e-4, and exact to f32 rounding for counts >= 1)
template <class P> MMVAE_DEV float log1p_cnt(float x) {
    if constexpr (std::is_same<P, __bf16>::value) return flog(1.f + x);
    else return log1pf(x);
}

// log1p of the integer counts 0 .. LTAB - 1 for the fp32-accurate modes' scatters (x3, f32):
// staged once per workgroup into LDS as the operand image of each value — x3: the hi / lo bf16
// pair packed in one word, f32: the float — so an entry is one LDS read instead of log1pf plus
// the split.  Other counts (non-integer, >= LTAB) take log1pf.  The bf16 mode keeps one v_log.
static constexpr int LTAB = 1024;
template <class P, int N = LTAB> struct Log1pTab {
    static constexpr bool ON = !std::is_same<P, __bf16>::value;
    static constexpr int BYTES = ON ? N * 4 : 0;
    MMVAE_DEV static void fill(uint32_t* tab) {
        if constexpr (ON)
            for (int i = threadIdx.x; i < N; i += blockDim.x) {
                const float v = log1pf((float)i);
                if constexpr (IsX3<P>::value) {
                    const __bf16 h = bf_hi(v), l = bf_lo(v, h);
                    tab[i] = (uint32_t)__builtin_bit_cast(uint16_t, h) | ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
                } else if constexpr (IsF8<P>::value) {
                    tab[i] = (uint32_t)to_t<uint8_t>(v);  // the e4m3 operand byte
                } else {
                    tab[i] = __float_as_uint(v);
                }
            }
    }
    // log1p(x) as the f32 the image of a float / bf16 table holds (P = float or __bf16)
    MMVAE_DEV static float value(const uint32_t* tab, float x) {
        static_assert(!IsX3<P>::value && !IsF8<P>::value, "f32 values only");
        if constexpr (!ON) {
            return flog(1.f + x);
        } else {
            const int xi = (int)x;
            float v;
            if (x == (float)xi && (unsigned)xi < (unsigned)N) v = __uint_as_float(tab[xi]);
            else v = log1pf(x);
            return v;
        }
    }
    // operand image of log1p(x) into tile t at idx (x3: lo plane `plane` elements after)
    template <class T>
    MMVAE_DEV static void put(const uint32_t* tab, T* t, int idx, int plane, float x) {
        if constexpr (!ON) {
            t[idx] = to_t<T>(flog(1.f + x));
        } else {
            const int xi = (int)x;
            if (x == (float)xi && (unsigned)xi < (unsigned)N) {
                const uint32_t v = tab[xi];
                if constexpr (IsX3<P>::value) {
                    t[idx] = __builtin_bit_cast(__bf16, (uint16_t)(v & 0xffffu));
                    t[idx + plane] = __builtin_bit_cast(__bf16, (uint16_t)(v >> 16));
                } else if constexpr (IsF8<P>::value) {
                    t[idx] = (uint8_t)v;
                } else {
                    t[idx] = __uint_as_float(v);
                }
            } else {
                const float v = log1pf(x);
                if constexpr (IsX3<P>::value) {
                    const __bf16 h = bf_hi(v);
                    t[idx] = h;
                    t[idx + plane] = bf_lo(v, h);
                } else {
                    t[idx] = to_t<T>(v);
                }
            }
        }
    }
};

// store v into operand tile t at element idx: plain (f32 / bf16), or as the hi / lo bf16 pair of
// the x3 mode with the lo plane `plane` elements after the hi plane
template <class P> MMVAE_DEV void put_op(typename Elem<P>::type* t, int idx, int plane, float v) {
    if constexpr (IsX3<P>::value) {
        const __bf16 h = bf_hi(v);
        t[idx] = h;
        t[idx + plane] = bf_lo(v, h);
    } else {
        t[idx] = to_t<typename Elem<P>::type>(v);
    }
}

// mvec[k] from the per-256-gene-block partials [nblk][KP] written by k_prep / k_vprep: the
// workgroup's first 256 threads each sum a quarter of the blocks of one latent (fixed order,
// loads issued 16 at a time), the quarters are combined in order through LDS.  All threads of
// the block call it; valid for k < 64.
MMVAE_DEV float mvec_sum(const float* __restrict__ mvecp, int nblk, int KP, int k) {
    __shared__ float smv[4][64];
    const int kk = threadIdx.x & 63, part = threadIdx.x >> 6;
    if (part < 4) {
        float s = 0.f;
        if (kk < KP) {
            int i = part;
            for (; i + 4 * 15 < nblk; i += 64) {
                float v[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = mvecp[(int64_t)(i + 4 * j) * KP + kk];
#pragma unroll
                for (int j = 0; j < 16; ++j) s += v[j];
            }
            for (; i < nblk; i += 4) s += mvecp[(int64_t)i * KP + kk];
        }
        smv[part][kk] = s;
    }
    __syncthreads();
    return (smv[0][k] + smv[1][k]) + (smv[2][k] + smv[3][k]);
}

// Per-block partial of mvec for 8 latents k0..k0+7: sum over the block's 256 genes of
// v[kk] (one per thread), written to mvecp[blockIdx.x][k0 + kk].  All 256 threads call it.
MMVAE_DEV void mvec_partial(const float (&v)[8], float* __restrict__ mvecp, int KP, int k0) {
    __shared__ float sred[4][8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
        const float t = wave_sum(v[kk]);
        if (lane == 0) sred[w][kk] = t;
    }
    __syncthreads();
    if (threadIdx.x < 8)
        mvecp[(int64_t)blockIdx.x * KP + k0 + threadIdx.x] =
            (sred[0][threadIdx.x] + sred[1][threadIdx.x]) + (sred[2][threadIdx.x] + sred[3][threadIdx.x]);
}

// Fixed-order sum over nwg per-workgroup partials [nwg][SMALL] for output i: a 256-thread block
// covers 32 outputs x 8 workgroup chunks (each thread's loads independent, 16 in flight), the
// chunk sums combined in chunk order through LDS.  Valid in threads 0..31 (threadIdx.x >> 5 == 0).
MMVAE_DEV float sum_partials(const float* __restrict__ small, int nwg, int SMALL, int i, float (*red)[32]) {
    const int col = threadIdx.x & 31, ch = threadIdx.x >> 5;
    float s = 0.f;
    if (i < SMALL) {
#pragma unroll 16
        for (int wg = ch; wg < nwg; wg += 8) s += small[(int64_t)wg * SMALL + i];
    }
    red[ch][col] = s;
    __syncthreads();
    float t = 0.f;
    if (ch == 0)
#pragma unroll
        for (int c = 0; c < 8; ++c) t += red[c][col];
    return t;
}

// The K x E head weights (Wm, Wl; K, E <= 64) into LDS [k][65]: issue() loads into registers
// (clamped, unconditional addresses: counted waits), store() writes LDS — other loads issued
// between the two share the same memory round.
template <int NTH = 256>
struct HeadsStage {
    static constexpr int NU = 4096 / NTH;  // K * E <= 64 * 64 values per thread group
    float tm[NU], tl[NU];
    MMVAE_DEV void issue(const float* __restrict__ Wm, const float* __restrict__ Wl, int K, int E) {
        const int KK = K * E;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int i = min((int)threadIdx.x + NTH * u, KK - 1);
            tm[u] = Wm[i];
            tl[u] = Wl[i];
        }
    }
    MMVAE_DEV void store(int K, int E, float* sWm, float* sWl) const {
        const int KK = K * E;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int i = (int)threadIdx.x + NTH * u;
            if (i < KK) {
                sWm[(i / E) * 65 + i % E] = tm[u];
                sWl[(i / E) * 65 + i % E] = tl[u];
            }
        }
    }
};
MMVAE_DEV void load_heads_lds(const float* __restrict__ Wm, const float* __restrict__ Wl, int K, int E, float* sWm,
                              float* sWl) {
    HeadsStage<> hs;
    hs.issue(Wm, Wl, K, E);
    hs.store(K, E, sWm, sWl);
}

// ---- latent-head products on f32 MFMA (exact f32 FMA chains) ---------------------------
// LDS images of the workgroup's LAT_CELLS = 16 cells: [cell][68], columns 0..63 always written
// (0 past the width); the head weights sWm / sWl [k][65] (valid for k < K, j < E).
// dh[cell][j] = sum_k dmean[cell][k] Wm[k][j] + da[cell][k] Wl[k][j]: wave w owns head inputs
// j = 16 w + (lane & 15); returns the C-layout tile, acc[r] = dh[4 (lane >> 4) + r][j].
MMVAE_DEV f32x4 heads_dh(const float* sDM, const float* sDA, const float* sWm, const float* sWl, int K, int E, int w,
                         int lane) {
    const int j = 16 * w + (lane & 15), row = lane & 15, kq = lane >> 4;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; 4 * s < K; ++s) {
        const int kk = 4 * s + kq;
        const bool ok = kk < K && j < E;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(sDM[row * 68 + kk], ok ? sWm[kk * 65 + j] : 0.f, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(sDA[row * 68 + kk], ok ? sWl[kk * 65 + j] : 0.f, acc, 0, 0, 0);
    }
    return acc;
}
// Forward heads for the 16 cells: mean_pre[cell][k] = sum_j h[cell][j] Wm[k][j] (j < E, and the
// same with Wl): wave w owns latents k = 16 w + (lane & 15); the C-layout results are stored to
// sM / sA [cell][68] (rows 4 (lane >> 4) + r).
MMVAE_DEV void heads_fwd(const float* sH, const float* sWm, const float* sWl, int K, int E, int w, int lane, float* sM,
                         float* sA) {
    const int kc = 16 * w + (lane & 15), row = lane & 15, jq = lane >> 4;
    f32x4 am = f32x4{0.f, 0.f, 0.f, 0.f}, al = am;
    for (int s = 0; 4 * s < E; ++s) {
        const int jj = 4 * s + jq;
        const bool ok = jj < E && kc < K;
        const float hj = sH[row * 68 + jj];
        am = __builtin_amdgcn_mfma_f32_16x16x4f32(hj, ok ? sWm[kc * 65 + jj] : 0.f, am, 0, 0, 0);
        al = __builtin_amdgcn_mfma_f32_16x16x4f32(hj, ok ? sWl[kc * 65 + jj] : 0.f, al, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sM[(4 * jq + r) * 68 + kc] = am[r];
        sA[(4 * jq + r) * 68 + kc] = al[r];
    }
}

// Per-workgroup partials of dWm = dmean^T h and dWl = da^T h over the 16 cells (h = the heads'
// input, E wide): wave w owns rows k = 16 w .. 16 w + 15; stored [k][j] into out[0 .. K*E) and
// out[K*E .. 2 K*E).
MMVAE_DEV void heads_dW(const float* sDM, const float* sDA, const float* sH, int K, int E, int w, int lane,
                        float* __restrict__ out) {
    const int kr = 16 * w + (lane & 15), cq = lane >> 4, jc = lane & 15;
    f32x4 am[4], al[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
        am[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
        al[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < LAT_CELLS / 4; ++s) {
        const int c = 4 * s + cq;
        const float a_m = sDM[c * 68 + kr], a_l = sDA[c * 68 + kr];
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            const float hb = sH[c * 68 + 16 * nb + jc];
            am[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_m, hb, am[nb], 0, 0, 0);
            al[nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_l, hb, al[nb], 0, 0, 0);
        }
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int kk = 16 * w + 4 * cq + r, jj = 16 * nb + jc;
            if (kk < K && jj < E) {
                out[kk * E + jj] = am[nb][r];
                out[K * E + kk * E + jj] = al[nb][r];
            }
        }
}

// ---- frozen hidden chains on the same LDS images (f32 MFMA) -----------------------------
// chain layer l's W into LDS sW [out][65] (all threads; the caller syncs before use)
MMVAE_DEV void chain_stage_w(const Dims& d, int l, float* sW) {
    const float* W = d.chain + d.ch_off[l];
    const int in = d.ch_in[l], n = in * d.ch_out[l];
    for (int i = threadIdx.x; i < n; i += 256) sW[(i / in) * 65 + i % in] = W[i];
}
// sOut = act(sIn W^T + b) over the 16 cells: wave w owns outputs 16 w .. 16 w + 15 (all 64
// columns of sOut written, 0 past the width)
MMVAE_DEV void chain_fwd(const Dims& d, int l, const float* sIn, const float* sW, bool relu, int w, int lane,
                         float* sOut) {
    const int in = d.ch_in[l], out = d.ch_out[l];
    const int oc = 16 * w + (lane & 15), row = lane & 15, iq = lane >> 4;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; 4 * s < in; ++s) {
        const int ii = 4 * s + iq;
        const bool ok = ii < in && oc < out;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(sIn[row * 68 + ii], ok ? sW[oc * 65 + ii] : 0.f, acc, 0, 0, 0);
    }
    const float bv = oc < out ? d.chain[d.ch_off[l] + in * out + oc] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float v = acc[r] + bv;
        if (relu) v = fmaxf(v, 0.f);
        sOut[(4 * iq + r) * 68 + oc] = oc < out ? v : 0.f;
    }
}
// Backward of one chain layer: dIn = (dOut masked by out > 0 when the layer has a ReLU) W.
// Wave w owns inputs i = 16 w + (lane & 15); returns acc[r] = dIn[4 (lane >> 4) + r][i].
MMVAE_DEV f32x4 chain_bwd(const Dims& d, int l, const float* sDOut, const float* sOut, const float* sW, bool relu, int w,
                          int lane) {
    const int in = d.ch_in[l], out = d.ch_out[l];
    const int i = 16 * w + (lane & 15), row = lane & 15, oq = lane >> 4;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; 4 * s < out; ++s) {
        const int oo = 4 * s + oq;
        float g = sDOut[row * 68 + oo];
        if (relu && !(sOut[row * 68 + oo] > 0.f)) g = 0.f;
        const bool ok = oo < out && i < in;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(g, ok ? sW[oo * 65 + i] : 0.f, acc, 0, 0, 0);
    }
    return acc;
}
// C-layout tile (wave w's 16 columns) -> LDS image
MMVAE_DEV void img_store(float* sImg, const f32x4& acc, int w, int lane) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sImg[(4 * (lane >> 4) + r) * 68 + 16 * w + (lane & 15)] = acc[r];
}
// Run chain layers [l0, l1) forward from image `in`: with keep, layer l's output goes to
// out0 + (l - l0) images (kept for the backward's ReLU masks), else ping-pong out0 / out1.  W
// staged through sW.  Returns the final image.  All threads; ends synced.
MMVAE_DEV const float* chain_run(const Dims& d, int l0, int l1, const float* in, float* out0, float* out1, bool keep,
                                 float* sW, int w, int lane) {
    const float* cur = in;
    for (int l = l0; l < l1; ++l) {
        chain_stage_w(d, l, sW);
        __syncthreads();
        float* o = keep ? out0 + (l - l0) * (LAT_CELLS * 68) : (((l - l0) & 1) ? out1 : out0);
        chain_fwd(d, l, cur, sW, d.relu != 0, w, lane, o);
        __syncthreads();
        cur = o;
    }
    return cur;
}

// LDS carve of k_enc_fwd (host computes the same size); planes = 2 in the x3 mode (hi + lo
// images of the double-buffered W stage: [hi 0][hi 1][lo 0][lo 1])
struct EncLds {
    int o_x, o_toff, o_tab, bytes;
    MMVAE_HOSTDEV EncLds(int KP, int esz, int S, int xbytes_per_wave, int pre, int planes = 1, int tab_bytes = 0,
                         int nbuf = 2, int nw = 4) {
        const int stb = KP * 64 * esz;
        o_x = pre + nbuf * planes * stb;
        o_toff = o_x + nw * xbytes_per_wave;  // [nw waves][S] tile offsets
        o_tab = o_toff + ((nw * S * 4 + 15) / 16) * 16;  // log1p table (Log1pTab)
        bytes = o_tab + tab_bytes;
    }
};

// Register-staged copy of a [NR rows][RB bytes] tile (row stride `ld` bytes in HBM) into the
// swizzled LDS image read by swz_off<RB>: loads issued early, ds_write_b128 late, so the
// copy overlaps a compute phase without an LDS-DMA in flight (hipcc drains vmcnt(0) before
// LDS reads while a DMA is outstanding).
template <int NR, int RB, int NTH = 256>
struct RegStage {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    static constexpr int CH = NR * RB / 16;             // 16-byte chunks of the tile
    static constexpr int NC = (CH + NTH - 1) / NTH;     // chunks per thread (1, 2 or 4)
    static constexpr bool PART = CH < NTH;              // fewer chunks than threads: the rest idle
    static_assert(NC >= 1 && NC <= 4 && (PART || CH % NTH == 0), "RegStage: 1..4 whole chunks per thread");
    static_assert((NTH & (NTH - 1)) == 0, "RegStage: a power-of-two thread group");
    // the staging threads are NTH consecutive threads of the block (a whole block, or one
    // aligned half of it): thread index within the group
    // (tx: the block's thread index — threadIdx.x, or a copy a kernel keeps opaque per tile so the
    // addresses derived from it are recomputed rather than held across its loop)
    static MMVAE_DEV int tid(int tx) { return tx & (NTH - 1); }
    u32x4 v0, v1, v2, v3;
    MMVAE_DEV u32x4 ld1(const char* src, int64_t ld, int i, int tx) const {
        const int c = PART ? min(tid(tx), CH - 1) : tid(tx) + NTH * i;
        return *reinterpret_cast<const u32x4*>(src + (int64_t)(c / (RB / 16)) * ld + (c % (RB / 16)) * 16);
    }
    MMVAE_DEV void st1(char* dst, int i, u32x4 x, int tx) const {
        const int c = tid(tx) + NTH * i;
        if (PART && c >= CH) return;
        *reinterpret_cast<u32x4*>(dst + swz_off<RB>(c / (RB / 16), (c % (RB / 16)) * 16)) = x;
    }
    MMVAE_DEV void load(const char* src, int64_t ld, int tx = (int)threadIdx.x) {
        v0 = ld1(src, ld, 0, tx);
        if constexpr (NC > 1) v1 = ld1(src, ld, 1, tx);
        if constexpr (NC > 2) v2 = ld1(src, ld, 2, tx);
        if constexpr (NC > 3) v3 = ld1(src, ld, 3, tx);
    }
    MMVAE_DEV void store(char* dst, int tx = (int)threadIdx.x) const {
        st1(dst, 0, v0, tx);
        if constexpr (NC > 1) st1(dst, 1, v1, tx);
        if constexpr (NC > 2) st1(dst, 2, v2, tx);
        if constexpr (NC > 3) st1(dst, 3, v3, tx);
    }
};

// RegStage of an operand tile and, in the x3 mode, of its lo plane: loaded from src and
// src + plane_bytes, stored to the LDS images dst and dst + img_bytes (same swizzle)
template <int NR, int RB, int NTH, bool X>
struct DualStage {
    RegStage<NR, RB, NTH> hi, lo;
    MMVAE_DEV void load(const char* src, int64_t ld, int64_t plane_bytes, int tx = (int)threadIdx.x) {
        hi.load(src, ld, tx);
        if constexpr (X) lo.load(src + plane_bytes, ld, tx);
    }
    MMVAE_DEV void store(char* dst, int img_bytes, int tx = (int)threadIdx.x) const {
        hi.store(dst, tx);
        if constexpr (X) lo.store(dst + img_bytes, tx);
    }
};

}  // namespace mmvae
