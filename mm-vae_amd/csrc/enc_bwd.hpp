// Encoder backward body shared by the NB (nb_kernels.hip) and vMF (vmf_kernels.hip) launches,
// so each model can put its small-gradient blocks into the same launch (k_enc_bwd_small /
// k_enc_bwd_vsmall).
#pragma once
#include "common.hpp"
#include "tiles.hpp"

namespace mmvae {

// =======================================================================================
// k_enc_bwd — gradient of x_mean / ln_x_sd through the frozen encoder (autograd of
// nb.hh:408-411) and of depth / nu_enc weights (raw x, nb.hh:448,498):
//   Gl_g  = sum_k W_enc[k,g] M[k,g],  M = dh^T log1p(x)   (MFMA on densified 64x64 tiles)
//   raw_g = sum_b a_b x_bg for a in {dpre, dhnu_h}        (gene-owner lanes over an f32 tile)
// Workgroup = 64 cells x one gene split.  The log1p(x) tile [64 genes][64 cells] and the raw
// count tile are shared by the four waves (each wave scatters its own 16 cells); wave w owns
// M's latent block w and the raw sums of gene block w.  Everything is written straight to the
// row block's slab in a fixed order — no atomics.  Single-buffered tiles, two barriers per tile.
// =======================================================================================
struct EncBwdLds {
    int o_lt, o_raw, o_part, o_scal, o_wave, wave_bytes, o_tab, bytes;
    // wsz: element size of the staged W image (f32 in the x3 mode: W only feeds a VALU dot);
    // planes: operand planes of the log1p tile (x3: hi + lo)
    // wsz 4 (f32 / x3): W stays in registers, no LDS image
    // raw: the raw-count tile (NB only; the vMF backward has no raw-count term, and without the
    // 17 KB tile its x3 workgroup fits 4 per CU instead of 3)
    MMVAE_HOSTDEV EncBwdLds(int KP, int esz, int S, int LS, int nsc, int wsz, int planes, int tab_bytes, bool raw) {
        o_lt = wsz == 4 ? 0 : KP * 64 * wsz;
        o_raw = o_lt + planes * 64 * LS * esz;
        o_part = o_raw + (raw ? 64 * 68 * 4 : 0);
        o_scal = o_part + 4 * 64 * 4;
        o_wave = o_scal + nsc * 64 * 4;
        wave_bytes = ((S * 4 + 15) / 16) * 16;  // the wave block's tile offsets
        o_tab = o_wave + 4 * wave_bytes;  // log1p table (Log1pTab)
        bytes = o_tab + tab_bytes;
    }
};

// staged encoder weight of the backward's VALU dot: the GEMM element type, f32 in the x3 mode
template <class P> struct WEnc { typedef typename Elem<P>::type type; };
template <> struct WEnc<X3> { typedef float type; };

template <class P, int KP, bool H1, bool RAW>
MMVAE_DEV void enc_bwd_body(EntList ents, const int64_t* __restrict__ seg,
                            const int32_t* __restrict__ toff, const float* __restrict__ lat,
                            const typename Elem<P>::type* __restrict__ dhT, int64_t dplane,
                            const typename WEnc<P>::type* __restrict__ WeP,
                            const Dims& d, float* __restrict__ slabE, const int bid) {
    using T = typename Elem<P>::type;
    using WT = typename WEnc<P>::type;
    using M = MM<P>;
    using Fr = typename M::frag;
    constexpr bool X = IsX3<P>::value;
    constexpr int LS = sizeof(T) == 2 ? 80 : 68;   // log1p tile row (gene) stride, elements
    constexpr int LT = 64 * LS;                    // elements of one log1p tile plane
    constexpr int RB = 64 * (int)sizeof(WT);       // staged W_enc row (one latent, 64 genes)
    // f32 W (x3 / f32 modes): each lane's 16 W values of a tile live in registers, loaded a tile
    // ahead from HBM / L2 (no 16 KB LDS image: one more workgroup per CU); bf16 W: LDS image
    constexpr bool WREG = sizeof(WT) == 4;
    constexpr int HN = H1 ? 1 : HMAX;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int sp, rb;
    xcd_split_major(bid, d.nrb, d.nsB, sp, rb);
    const int row0 = rb * 64 + 16 * w;
    const int t0 = sp * d.tpsB, t1 = min(d.NT, t0 + d.tpsB);
    const int S = d.tpsB + 1;
    const int H = H1 ? 1 : d.H;
    const int nq = RAW ? 2 + H : 1;  // vMF (RAW = false): only the log1p term
    const EncBwdLds L(KP, (int)sizeof(T), S, LS, 1 + HN, (int)sizeof(WT), X ? 2 : 1, Log1pTab<P>::BYTES, RAW);
    uint32_t* ltab = reinterpret_cast<uint32_t*>(smem + L.o_tab);
    Log1pTab<P>::fill(ltab);
    char* wst = smem;
    T* lt = reinterpret_cast<T*>(smem + L.o_lt);          // [64 genes][LS]  log1p(x)
    float* raw = reinterpret_cast<float*>(smem + L.o_raw);  // [64 genes][68] x
    float* part = reinterpret_cast<float*>(smem + L.o_part);  // [4][64]
    float* scal = reinterpret_cast<float*>(smem + L.o_scal);  // [1+H][64 cells]: dpre, dhnu_h
    int32_t* toffl = reinterpret_cast<int32_t*>(smem + L.o_wave + w * L.wave_bytes);  // [S] tile offsets
    // loads independent of the CSR index first: the W tile t0 and the dh^T A operand
    RegStage<KP, RB> wreg;
    auto wsrc = [&](int t) { return reinterpret_cast<const char*>(WeP) + (int64_t)64 * t * sizeof(WT); };
    // M = dh^T log1p(x) by (latent block lb) x (gene blocks): with KP = 64 wave w owns latent
    // block w and all four 16-gene blocks; with KP = 16 / 32 the waves split the gene blocks too
    // (NGB = KP / 16 blocks each, every wave busy); KP = 48 keeps one latent block per wave
    constexpr int NLB = KP / 16;
    constexpr bool GSPLIT = NLB < 4 && 4 % NLB == 0;
    constexpr int NGB = GSPLIT ? NLB : 4;   // gene blocks per wave
    const int lb = GSPLIT ? w % NLB : w;    // A operand: dh^T rows = latents of this wave's block, k = the workgroup's 64 cells
    const int gb0 = GSPLIT ? (w / NLB) * NGB : 0;
    float wr[4][4], wn[4][4];  // WREG: W[16 lb + 4 (lane >> 4) + r][64 t + 16 (gb0 + i) + (lane & 15)], this / next tile
    auto wload = [&](float (&dst)[4][4], int t) {
        const int kb = 16 * min(lb, KP / 16 - 1) + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < NGB; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                dst[i][r] = static_cast<float>(WeP[(int64_t)(kb + r) * d.DP + 64 * t + 16 * (gb0 + i) + (lane & 15)]);
    };
    if constexpr (WREG) wload(wr, min(t0, d.NT - 1));
    else wreg.load(wsrc(min(t0, d.NT - 1)), (int64_t)d.DP * sizeof(WT));
    constexpr int KSB = 64 / M::KSTEP;
    Fr afr[KSB];
#pragma unroll
    for (int s = 0; s < KSB; ++s)  // unconditional (clamped) loads; blocks past KP zeroed below
        afr[s] = M::load(&dhT[(int64_t)(16 * min(lb, KP / 16 - 1) + (lane & 15)) * d.Bpad + rb * 64 + s * M::KSTEP +
                              (lane >> 4) * M::EPL], dplane);

    const int wbk = row0 >> 4;  // this wave's 16-row block of the batch entry lists
    fill_toffl(toffl, S, t0, d.NT, toff, wbk, lane);
    const int64_t segw = seg[wbk];
    if (RAW && lane < 16) {
        const int b = row0 + lane;
        const float* Lr = lat + (int64_t)b * d.lat_stride;
        const float ok = (b < d.B) ? 1.f : 0.f;
        scal[16 * w + lane] = ok * Lr[d.LAT_DPRE];
        for (int h = 0; h < H; ++h) scal[(1 + h) * 64 + 16 * w + lane] = ok * Lr[d.LAT_DHNU + h];
    }
    // this wave's 16 cell columns of both tiles
    auto zero_cols = [&]() {
        constexpr int CB = 16 * (int)sizeof(T) / 16;
#pragma unroll
        for (int pl = 0; pl < (X ? 2 : 1); ++pl)
#pragma unroll
            for (int c = 0; c < CB; ++c) reinterpret_cast<uint4*>(lt + pl * LT + lane * LS + 16 * w)[c] = uint4{0, 0, 0, 0};
        if (RAW)
#pragma unroll
            for (int c = 0; c < 4; ++c) reinterpret_cast<uint4*>(raw + lane * 68 + 16 * w)[c] = uint4{0, 0, 0, 0};
    };
    auto scatter = [&](const ListEntries& le) {
        le.visit(ents, lane, [&](int r, int gl, float x) {
            Log1pTab<P>::put(ltab, lt, gl * LS + 16 * w + r, LT, x);
            if (RAW) raw[gl * 68 + 16 * w + r] = x;
        });
    };
    if (lb >= KP / 16)
#pragma unroll
        for (int s = 0; s < KSB; ++s) afr[s] = M::zero();

    wave_sync();  // toffl written above by this wave
    const int nt = t1 - t0;
    // tile t + 1's entries come from one of two register sets, fetched two tiles ahead, and the
    // loop is unrolled by two: no register set (nor the WREG W tile) is copied at the latch, where
    // a copy of a register with a load in flight would wait for that load
    ListEntries qA, qB;
    // this wave's cells in the shared tiles are cleared only where its last scatter wrote
    int zp0 = -1, zp1 = -1;
    bool zall = true;
    auto keep = [&](const ListEntries& le) {
        zp0 = le.pos(0, lane);
        zp1 = le.pos(1, lane);
        asm volatile("" : "+v"(zp0), "+v"(zp1));  // taken now: le is refetched next
        zall = le.n > 128;
    };
    auto clear = [&]() {
        if (zall) {
            zero_cols();
            wave_sync();
        } else {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int zp = k ? zp1 : zp0;
                if (zp >= 0) {
                    const int gl = zp & 63, r = zp >> 6;
                    lt[gl * LS + 16 * w + r] = T{};
                    if constexpr (X) lt[LT + gl * LS + 16 * w + r] = T{};
                    if (RAW) raw[gl * 68 + 16 * w + r] = 0.f;
                }
            }
        }
    };
    if (t0 < t1) {
        ListEntries first;
        first.fetch(ents, segw, toffl, 0, lane);
        qA.fetch(ents, segw, toffl, min(1, nt - 1), lane);
        qB.fetch(ents, segw, toffl, min(2, nt - 1), lane);
        if constexpr (!WREG) wreg.store(wst);
        zero_cols();
        if constexpr (Log1pTab<P>::ON) __syncthreads();  // the table
        else wave_sync();
        scatter(first);
        keep(first);
    }
    lds_barrier();
    // diagnostic (MMVAE_DBG & 16384, -DMMVAE_DIAG builds): per-wave phase cycles into slabE
    // (outputs invalid): raw sums, M + W dot, barrier 1, slab store + scatter, fetch + barrier 2
    const bool stamps = dbg_bit(d.dbg, 16384);
    uint64_t st_[6] = {0, 0, 0, 0, 0, 0}, tp_ = stamps ? stamp_now() : 0;
    const uint64_t t_start = tp_;
    auto lap = [&](int i_) {
        if (stamps) {
            const uint64_t tn = stamp_now();
            st_[i_] += tn - tp_;
            tp_ = tn;
        }
    };
    // q: tile t + 1's entries; wc / wx: this / the next tile's W registers (WREG)
    auto tile = [&](int t, ListEntries& q, float (&wc)[4][4], float (&wx)[4][4]) {
        const int tl = t - t0;
        if constexpr (WREG) wload(wx, min(t + 1, t1 - 1));
        else wreg.load(wsrc(min(t + 1, t1 - 1)), (int64_t)d.DP * sizeof(WT));
        // ---- raw-count column sums of gene block w: lane = (gene 16w + (l&15), cell quarter l>>4) ----
        if (RAW) {
            const int gl = 16 * w + (lane & 15), q4 = lane >> 4;
            const float4* xr = reinterpret_cast<const float4*>(raw + gl * 68 + 16 * q4);
            float4 xv[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) xv[c] = xr[c];
            for (int h = 0; h < 1 + H; ++h) {
                const float4* sc = reinterpret_cast<const float4*>(scal + h * 64 + 16 * q4);
                float v = 0.f;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float4 a = sc[c];
                    v = fmaf(xv[c].x, a.x, fmaf(xv[c].y, a.y, fmaf(xv[c].z, a.z, fmaf(xv[c].w, a.w, v))));
                }
                v = sum_rowgroups(v);
                if (lane < 16 && !stamps) slabE[((int64_t)rb * nq + 1 + h) * d.DP + 64 * t + gl] = v;
            }
        }
        lap(0);
        // ---- M block w on MFMA, then Gl partial = sum over the block's latents of W M ----
        if (lb < KP / 16) {
            if constexpr (GSPLIT)  // the other waves' gene blocks: zero partials from this wave
                if (lane < 16)
#pragma unroll
                    for (int gb = 0; gb < 4; ++gb)
                        if (gb < gb0 || gb >= gb0 + NGB) part[w * 64 + 16 * gb + lane] = 0.f;
#pragma unroll
            for (int i = 0; i < NGB; ++i) {
                const int gb = gb0 + i;
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < KSB; ++s) {
                    const Fr bx = M::load(&lt[(16 * gb + (lane & 15)) * LS + s * M::KSTEP + (lane >> 4) * M::EPL], LT);
                    acc = M::mma(afr[s], bx, acc);
                }
                const int gl = 16 * gb + (lane & 15);
                float v = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int k = 16 * lb + 4 * (lane >> 4) + r;
                    const float wv = WREG ? wc[i][r]
                                          : static_cast<float>(*reinterpret_cast<const WT*>(wst + swz_off<RB>(k, gl * (int)sizeof(WT))));
                    v = fmaf(wv, acc[r], v);
                }
                v = sum_rowgroups(v);
                if (lane < 16) part[w * 64 + gl] = v;
            }
        } else if (lane < 16) {
#pragma unroll
            for (int gb = 0; gb < 4; ++gb) part[w * 64 + 16 * gb + lane] = 0.f;
        }
        lap(1);
        lds_barrier();
        lap(2);
        if (threadIdx.x < 64 && !stamps) {
            const int g = threadIdx.x;
            slabE[((int64_t)rb * nq) * d.DP + 64 * t + g] = part[g] + part[64 + g] + part[128 + g] + part[192 + g];
        }
        if (t + 1 < t1) {
            clear();
            scatter(q);
            keep(q);
            if constexpr (!WREG) wreg.store(wst);
        }
        lap(3);
        q.fetch(ents, segw, toffl, min(tl + 3, nt - 1), lane);
        lds_barrier();
        lap(4);
    };
    for (int t = t0; t < t1; t += 2) {
        tile(t, qA, wr, wn);
        if (t + 1 < t1) tile(t + 1, qB, wn, wr);
    }
    if (stamps && lane == 0) {
        float* o = slabE + ((int64_t)bid * 4 + w) * 8;
        for (int i = 0; i < 5; ++i) o[i] = (float)st_[i];
        o[5] = (float)(stamp_now() - t_start);
        o[6] = (float)nt;
    }
}

template <class P, int KP, bool RAW = true>
inline size_t enc_bwd_lds(const Dims& d) {
    using T = typename Elem<P>::type;
    constexpr int LS = sizeof(T) == 2 ? 80 : 68;
    return (size_t)EncBwdLds(KP, (int)sizeof(T), d.tpsB + 1, LS, 1 + (d.H == 1 ? 1 : HMAX),
                             (int)sizeof(typename WEnc<P>::type), IsX3<P>::value ? 2 : 1, Log1pTab<P>::BYTES, RAW).bytes;
}

}  // namespace mmvae
