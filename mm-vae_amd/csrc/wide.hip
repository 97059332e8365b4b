// The wide path: the ELBO step for model shapes beyond the fused tile kernels' limits — a latent
// (K / Z) or any hidden width above 64, more than 4 hidden layers, covariate / overdispersion
// widths C, H, R above 8, or D above the batch lists' LDS tile index (75,264 genes).  The
// reference builds any Linear chain and latent width (nb.hh:331-379, vmf.hh:338-385); this path
// makes every such model train on the GPU.
//
// Layout: the step's B cells are densified into HBM as a row-major [B, D] f32 block (the
// reference's own dense batch, mmvae_io.hh:208-245; 328 MB at B = 4096, D = 20k — HBM has room),
// and the step is the reference's op sequence (oracle/nb_oracle.py, oracle/vmf_oracle.py) on:
//   * the big gene GEMMs (encoder / decoder, forward and both backward transposes) on the bf16
//     MFMA in the handle's mode — x3 split operands (fp32-accurate) or bf16 — with the operands
//     converted as they are staged (k_gemm_mf); the encoder's input normalisation applied as the
//     raw batch is loaded; the decoder's covariate Linear and both biases in the logit GEMM's
//     epilogue.  f32 handles and small or broadcast shapes use the exact f32 MFMA (k_gemm).
//     Split-K partials are reduced in a fixed order — deterministic, like the fused path;
//   * per-row kernels with the fused path's element arithmetic (NB: softmax + likelihood + its
//     gradient in three sweeps of a row; vMF: the row normalisations and their backward), the
//     small row Linears (depth, nu_enc, nu_dec, the covariate part) inline;
//   * fixed-order column reductions (k_colred) for every gene-vector gradient: one read of a
//     dense block serves all the sums over it.
#include <cmath>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"

extern "C" float mmvae_fasterlgamma(float x);

namespace mmvae {

// =======================================================================================
// Generic GEMM: C(m, n) [+]= act(alpha * sum_k A(m, k) B(k, n) + bias[n])
//   A(m, k) = A[m * sam + k * sak], B(k, n) = B[k * sbk + n * sbn], C(m, n) = C[m * scm + n * scn]
// =======================================================================================
struct GemmX {
    const float* xm = nullptr;   // x_mean [K]
    const float* isd = nullptr;  // 1 / (softplus(ln_x_sd) + eps) [K]
    const float* rs = nullptr;   // per-row scale of log1p(x) (vMF: 1 / |log1p(x_b)|), null: 1
};
struct GemmOp {
    int M = 0, N = 0, K = 0;
    const float* A = nullptr;
    int64_t sam = 0, sak = 0;
    const float* B = nullptr;
    int64_t sbk = 0, sbn = 0;
    float* C = nullptr;
    int64_t scm = 0, scn = 0;
    float alpha = 1.f;
    const float* bias = nullptr;   // [N]
    const float* bias2 = nullptr;  // [N], a second bias (the decoder's mu_bias, nb.hh:437-441)
    // rank-nc term sum_c ca[m * lca + c] * cw[n * lcw + c] (the covariate Linear of a decoder,
    // nb.hh:436 / vmf.hh:287, folded into the logit GEMM's epilogue; nc <= 8)
    const float* ca = nullptr;
    const float* cw = nullptr;
    const float* cbias = nullptr;  // that Linear's bias [N]
    int64_t lca = 0, lcw = 0;
    int nc = 0;
    int act = 0;                  // 1: ReLU
    int accumulate = 0;           // C += result
    // the column-sum epilogue (k_gemm_mf, one split): C is not stored; per 64-row tile mt,
    // cpart[(mt * 2 + 0) * N + n] = sum_m C(m, n) and [(mt * 2 + 1) * N + n] =
    // sum_m C(m, n) enc_in(cx(m, n)) with cxf's transform — the x_mean / ln_x_sd sums over the
    // encoder's input gradient straight from its GEMM (k_colred's XPROD pair, chunks = row tiles)
    float* cpart = nullptr;
    const float* cx = nullptr;
    int64_t ldcx = 0;
    GemmX cxf;
    // a frozen B operand's bf16 planes for k_gemm_skf (null: none): bpl[n * bkp + k], lo at + bplane
    const __bf16* bpl = nullptr;
    int bkp = 0;
    int64_t bplane = 0;
    const float* colv = nullptr;  // k_gemm_skf: gemm_colc of every column, combined by the host's launch
};

static constexpr int GT = 64, GK = 16, GLD = GT + 4;

// the column's constant: every bias of output column n, summed in a fixed order
MMVAE_DEV float gemm_colc(const GemmOp& g, int n) {
    float c = 0.f;
    if (g.bias) c += g.bias[n];
    if (g.bias2) c += g.bias2[n];
    if (g.cbias) c += g.cbias[n];
    return c;
}
// alpha acc + colc + the rank-nc term (cwn: column n's nc weights), ReLU, store / accumulate
MMVAE_DEV void gemm_store(const GemmOp& g, int m, int n, float acc, float colc, const float* cwn) {
    float v = fmaf(g.alpha, acc, colc);
    for (int c = 0; c < g.nc; ++c) v = fmaf(g.ca[(int64_t)m * g.lca + c], cwn[c], v);
    if (g.act == 1) v = fmaxf(v, 0.f);
    float* c = g.C + (int64_t)m * g.scm + (int64_t)n * g.scn;
    *c = g.accumulate ? *c + v : v;
}
MMVAE_DEV void gemm_epilogue(const GemmOp& g, int m, int n, float acc) {
    float cwn[8];
    for (int c = 0; c < g.nc; ++c) cwn[c] = g.cw[(int64_t)n * g.lcw + c];
    gemm_store(g, m, n, acc, gemm_colc(g, n), cwn);
}

// grid (tiles over N, tiles over M, splits); split s covers k chunks [s * cps, (s + 1) * cps)
// and, with more than one split, stores its raw sums into ws[s][M][N] for k_gemm_reduce.
// The exact f32 MFMA path (f32 handles, and every shape too small or too strided for k_gemm_mf).
__global__ __launch_bounds__(256) void k_gemm(GemmOp g, int cps, float* __restrict__ ws) {
    __shared__ float As[GK][GLD], Bs[GK][GLD];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;
    const int nch = (g.K + GK - 1) / GK;
    const int c0 = blockIdx.z * cps, c1 = min(nch, c0 + cps);
    const bool a_kfast = g.sak == 1, b_nfast = g.sbn == 1;
    float ra[4], rb[4];
    auto load = [&](int ch) {
        const int k0 = ch * GK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = t + 256 * i;
            int mm, kk;
            if (a_kfast) { mm = e >> 4; kk = e & 15; } else { mm = e & 63; kk = e >> 6; }
            const int m = m0 + mm, k = k0 + kk;
            ra[i] = (m < g.M && k < g.K) ? g.A[(int64_t)m * g.sam + (int64_t)k * g.sak] : 0.f;
            int nn, kb;
            if (b_nfast) { nn = e & 63; kb = e >> 6; } else { nn = e >> 4; kb = e & 15; }
            const int n = n0 + nn, kq = k0 + kb;
            rb[i] = (n < g.N && kq < g.K) ? g.B[(int64_t)kq * g.sbk + (int64_t)n * g.sbn] : 0.f;
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = t + 256 * i;
            if (a_kfast) As[e & 15][e >> 4] = ra[i]; else As[e >> 6][e & 63] = ra[i];
            if (b_nfast) Bs[e >> 6][e & 63] = rb[i]; else Bs[e & 15][e >> 4] = rb[i];
        }
    };
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (c0 < c1) load(c0);
    for (int ch = c0; ch < c1; ++ch) {
        __syncthreads();  // the previous chunk's operand reads are done
        store();
        __syncthreads();
        if (ch + 1 < c1) load(ch + 1);  // in flight under this chunk's MFMAs
#pragma unroll
        for (int s = 0; s < GK / 4; ++s) {
            const int kr = 4 * s + (lane >> 4);
            float a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[kr][wm + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[kr][wn + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    }
    const bool split = gridDim.z > 1;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r, n = n0 + wn + 16 * j + (lane & 15);
                if (m >= g.M || n >= g.N) continue;
                if (split) ws[((int64_t)blockIdx.z * g.M + m) * g.N + n] = acc[i][j][r];
                else gemm_epilogue(g, m, n, acc[i][j][r]);
            }
}

// the splits' partials summed in split order, then the epilogue
__global__ __launch_bounds__(256) void k_gemm_reduce(GemmOp g, int S, const float* __restrict__ ws) {
    const int64_t MN = (int64_t)g.M * g.N;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < MN; i += (int64_t)gridDim.x * 256) {
        float s = 0.f;  // (the splits in order, 8 loads issued at a time)
        int q = 0;
        for (; q + 8 <= S; q += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = ws[(q + u) * MN + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; q < S; ++q) s += ws[q * MN + i];
        gemm_epilogue(g, (int)(i / g.N), (int)(i % g.N), s);
    }
}

// =======================================================================================
// k_gemm_mf — the big GEMMs of the wide path on the bf16 MFMA (v_mfma_f32_16x16x32_bf16):
// one pass on bf16 operands (bf16 / fp8 handles) or the split "x3" products (bf16x3 handles,
// hi + lo planes, lo*hi + hi*lo + hi*hi: the fp32-accurate mode of the fused kernels).  The
// operands stay f32 in HBM; each 64 x 32 (rows x k) slice is loaded as float4 along its
// contiguous dimension, rounded to the bf16 planes in registers and stored into a
// double-buffered LDS image, one barrier per 32-deep k chunk (the next chunk's loads are in
// flight under the current chunk's MFMAs).  A slice whose k is contiguous in HBM is imaged
// [rows][k] and read with ds_read_b128; one whose rows are contiguous is imaged [k][rows] and
// read transposed (ds_read_b64_tr_b16, tr_frag) — so both transposes of every Linear's forward
// and backward run from the same kernel.  Workgroup: 64 x 64 outputs, four waves of 32 x 32.
// AT: the encoder's input transform on A (nb.hh:408-410, vmf.hh:253-257) applied as A is
// loaded, A(m, k) = (log1p(x) rs[m] - x_mean[k]) / sd[k] from the raw dense batch x, so the
// normalised input block is never stored.
// =======================================================================================

MMVAE_DEV float enc_in(float v, float rs, float xm, float isd) { return (log1p_pos(v) * rs - xm) * isd; }
// the same with libm log1pf (the f32 handles' input block, the ln_x_sd gradient's column sum)
__device__ __attribute__((noinline)) float log1p_libm(float v) { return log1pf(v); }
MMVAE_DEV float log1p_acc(float v) {
    // integer counts (0 included): 1 + v is exact and v_log's error is ~1 ulp of the result;
    // others libm, out of line (the branch is skipped by waves of counts, and the inlined libm
    // body would multiply the register use of every caller's unrolled loop)
    float r = flog(1.f + v);
    if (!(v >= 0.f && v < 16777216.f && v == floorf(v))) r = log1p_libm(v);
    return r;
}
MMVAE_DEV float enc_in_acc(float v, float rs, float xm, float isd) { return (log1p_acc(v) * rs - xm) * isd; }

template <class P>
struct MfOperand {
    static constexpr bool X = IsX3<P>::value;
    // one 64-row x 32-k slice: KF (k contiguous in HBM) -> image [64][32] (64-byte rows);
    // otherwise -> image [32][64] (128-byte rows); four f32 per thread per half.  Every load is
    // issued (indices clamped into the operand, out-of-range values zeroed after the load): the
    // count of loads in flight is then static and the compiler's waits let the next chunks'
    // loads stay outstanding (a bounds branch around a load made it wait for all of them).
    // The host routes here only float4-aligned operands whose contiguous extent is a multiple of 4.
    template <bool KF>
    static MMVAE_DEV void load(const float* base, int64_t srow, int64_t sk, int r0, int nrow, int k0, int K,
                               float4 (&v)[2]) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int r, k;
            bool ok;
            int64_t o;
            if constexpr (KF) {
                r = r0 + (t >> 3) + 32 * i;
                k = k0 + (t & 7) * 4;
                ok = r < nrow && k < K;
                o = (int64_t)min(r, nrow - 1) * srow + min(k, K - 4);
            } else {
                k = k0 + (t >> 4) + 16 * i;
                r = r0 + (t & 15) * 4;
                ok = k < K && r < nrow;
                o = (int64_t)min(k, K - 1) * sk + min(r, nrow - 4);
            }
            const float4 u = *reinterpret_cast<const float4*>(base + o);
            v[i].x = ok ? u.x : 0.f;
            v[i].y = ok ? u.y : 0.f;
            v[i].z = ok ? u.z : 0.f;
            v[i].w = ok ? u.w : 0.f;
        }
    }
    // the slice's bf16 planes (hi [, lo at +PL bytes]) into the image
    template <bool KF>
    static MMVAE_DEV void store(char* img, int PL, const float4 (&v)[2]) {
        const int t = threadIdx.x;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            int off;
            if constexpr (KF) off = swz_off<64>((t >> 3) + 32 * i, (t & 7) * 8);
            else off = swz_off<128>((t >> 4) + 16 * i, (t & 15) * 8);
            const float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            const uint32_t h01 = pk_bf16(e[0], e[1]), h23 = pk_bf16(e[2], e[3]);
            *reinterpret_cast<uint2*>(img + off) = uint2{h01, h23};
            if constexpr (X) {
                const uint32_t l01 = pk_bf16(e[0] - __uint_as_float(h01 << 16), e[1] - __uint_as_float(h01 & 0xffff0000u));
                const uint32_t l23 = pk_bf16(e[2] - __uint_as_float(h23 << 16), e[3] - __uint_as_float(h23 & 0xffff0000u));
                *reinterpret_cast<uint2*>(img + PL + off) = uint2{l01, l23};
            }
        }
    }
    // MFMA fragment of rows c0 .. c0 + 15 (lane & 15), k 8 (lane >> 4) .. + 7
    template <bool KF>
    static MMVAE_DEV typename MM<P>::frag frag(const char* img, int PL, int c0) {
        const int lane = threadIdx.x & 63;
        if constexpr (KF) {
            const int off = swz_off<64>(c0 + (lane & 15), (lane >> 4) * 16);
            if constexpr (X) return typename MM<P>::frag{*reinterpret_cast<const bf16x8*>(img + off),
                                                          *reinterpret_cast<const bf16x8*>(img + PL + off)};
            else return *reinterpret_cast<const bf16x8*>(img + off);
        } else {
            if constexpr (X) return typename MM<P>::frag{tr_frag<128>(img, 0, c0), tr_frag<128>(img + PL, 0, c0)};
            else return tr_frag<128>(img, 0, c0);
        }
    }
};

// NT: 64 or 128 output columns per workgroup (the four waves 32 x NT / 2 each); 128 halves
// the A re-reads of the K = D GEMMs whose N is the latent width
// XCD-aware tile order: blocks b and b + 8 share an XCD (its L2), so block b takes tile
// xcd * per + b / 8 of the (m fastest, then n, then split) order — an XCD walks the m tiles of
// its own n tiles / k splits and keeps their B slice in its L2 instead of every XCD cycling
// through all of B (MI355X_MICROARCH.md, workgroup dispatch; for speed only: any placement
// computes the same tiles)
MMVAE_DEV void mf_tile(int& tn, int& tm, int& tz) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int T = gx * gy * (int)gridDim.z;
    const int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int c = (T + 7) / 8, r = T % 8, xcd = L % 8, idx = L / 8;
    const int t = (r == 0 || xcd < r) ? xcd * c + idx : r * c + (xcd - r) * (c - 1) + idx;
    tm = t % gy;
    tn = (t / gy) % gx;
    tz = t / (gy * gx);
}

// NT: 64 or 128 output columns per workgroup (the four waves 32 x NT / 2 each); 128 halves
// the A re-reads of the K = D GEMMs whose N is the latent width.  PF: chunks whose loads are in
// flight in registers.  PF = 2 (the long-K GEMMs: K = D): two register stages, the loop unrolled
// by two so every register index is static — the chunk being stored into LDS and the next one
// load under the MFMAs of the current one; PF = 1 (a few chunks, K = a latent / hidden width):
// one stage, fewer registers and more workgroups per CU (two stages measured 272 -> 336 us on
// the logit GEMM, 4 chunks).
template <class P, bool AKF, bool BKF, bool AT, int NT, int PF>
__global__ __launch_bounds__(256) void k_gemm_mf(GemmOp g, GemmX x, int cps, float* __restrict__ ws, int vec) {
    static_assert(!AT || AKF, "the input transform follows the k-contiguous slice layout");
    using M = MM<P>;
    using Op = MfOperand<P>;
    constexpr int NPL = IsX3<P>::value ? 2 : 1;
    constexpr int PL = 4096;                // one plane of a 64 x 32 bf16 image
    constexpr int IMG = NPL * PL;           // one 64-row operand image
    constexpr int NB = NT / 64;             // B images per buffer
    constexpr int WJ = NT / 32;             // 16-column blocks per wave
    __shared__ __attribute__((aligned(16))) char lds[2][1 + NB][IMG];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int btn, btm, btz;
    if (vec & 2) mf_tile(btn, btm, btz);
    else btn = blockIdx.x, btm = blockIdx.y, btz = blockIdx.z;
    const int m0 = btm * 64, n0 = btn * NT;
    const int nch = (g.K + 31) / 32;
    const int c0 = btz * cps, c1 = min(nch, c0 + cps);
    float4 va[PF][2], vb[PF][NB][2];
    // AT: the transform's per-k vectors ride with the chunk's loads; the transform itself runs when
    // the chunk is stored into LDS, so the next chunk's loads stay in flight under this chunk's
    // MFMAs (applied inside load(), it made every chunk wait for its own loads: 263 us -> see
    // DESIGN.md §4b round 5)
    float xmv[PF][4], isv[PF][4], rsv[PF][2];
    int ktr[PF] = {};
    auto load = [&](auto S, int ch) {
        constexpr int st = decltype(S)::value;
        Op::template load<AKF>(g.A, g.sam, g.sak, m0, g.M, ch * 32, g.K, va[st]);
#pragma unroll
        for (int h = 0; h < NB; ++h) Op::template load<BKF>(g.B, g.sbn, g.sbk, n0 + 64 * h, g.N, ch * 32, g.K, vb[st][h]);
        if constexpr (AT) {
            const int t = threadIdx.x;
            ktr[st] = ch * 32 + (t & 7) * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = min(ktr[st] + j, g.K - 1);
                xmv[st][j] = x.xm[k];
                isv[st][j] = x.isd[k];
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = m0 + (t >> 3) + 32 * i;
                rsv[st][i] = x.rs ? x.rs[min(r, g.M - 1)] : 1.f;  // (x.rs: uniform)
            }
        }
    };
    const int wm = (w >> 1) * 32, wn = (w & 1) * (NT / 2);
    f32x4 acc[2][WJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // chunk ch in register stage / LDS buffer st = (ch - c0) & 1; buffer st was last read two
    // chunks ago, before the previous chunk's barrier
    auto chunk = [&](auto S, int buf, int ch) {
        constexpr int st = decltype(S)::value;
        if constexpr (AT) {  // the encoder input transform; k past K stays 0
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float* e = reinterpret_cast<float*>(&va[st][i]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    // (computed on every lane, the clamped k's loads are finite; pinned so the
                    // select stays a v_cndmask instead of a branch with its own load waits)
                    float tv = enc_in(e[j], rsv[st][i], xmv[st][j], isv[st][j]);
                    asm volatile("" : "+v"(tv));
                    e[j] = (ktr[st] + j < g.K) ? tv : 0.f;
                }
            }
        }
        Op::template store<AKF>(lds[buf][0], PL, va[st]);
#pragma unroll
        for (int h = 0; h < NB; ++h) Op::template store<BKF>(lds[buf][1 + h], PL, vb[st][h]);
        __syncthreads();
        // in flight under the MFMAs of this chunk (and with PF = 2 the next one).  PF = 2 issues
        // them unconditionally (past the split's end: its last chunk again, unused) so the loads
        // in flight are a static count; PF = 1 waits for all of them anyway and skips the spare
        if (PF == 2 || ch + 1 < c1) load(S, min(ch + PF, c1 - 1));
        typename M::frag fa[2], fb[WJ];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = Op::template frag<AKF>(lds[buf][0], PL, wm + 16 * i);
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
            const int cn = wn + 16 * j;
            fb[j] = Op::template frag<BKF>(lds[buf][1 + cn / 64], PL, cn & 63);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < WJ; ++j) acc[i][j] = M::mma(fa[i], fb[j], acc[i][j]);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    load(S0{}, c0);
    if constexpr (PF == 2) {
        load(S1{}, min(c0 + 1, max(c1 - 1, c0)));
        int ch = c0;
        for (; ch + 1 < c1; ch += 2) {  // (both stages every trip: the waits see one load pattern)
            chunk(S0{}, 0, ch);
            chunk(S1{}, 1, ch + 1);
        }
        if (ch < c1) chunk(S0{}, 0, ch);
    } else {
        for (int ch = c0; ch < c1; ++ch) chunk(S0{}, (ch - c0) & 1, ch);
    }
    if (g.cpart) {  // the column-sum epilogue (uniform; the host launches it with one split)
        __syncthreads();  // every wave's last fragment reads are done: the images are free
        float* red = reinterpret_cast<float*>(&lds[0][0][0]);  // [row half][2][NT]
        float xv[WJ][2][4];
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
            const int n = min(n0 + wn + 16 * j + (lane & 15), g.N - 1);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = min(m0 + wm + 16 * i + 4 * (lane >> 4) + r, g.M - 1);
                    xv[j][i][r] = g.cx[(int64_t)m * g.ldcx + n];
                }
        }
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
            const int n = n0 + wn + 16 * j + (lane & 15), nn = min(n, g.N - 1);
            const float xm = g.cxf.xm[nn], isd = g.cxf.isd[nn];
            float s0 = 0.f, s1 = 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
                    const float rs = g.cxf.rs ? g.cxf.rs[min(m, g.M - 1)] : 1.f;
                    const float v = (m < g.M && n < g.N) ? acc[i][j][r] : 0.f;
                    s0 += v;
                    s1 = fmaf(v, enc_in_acc(xv[j][i][r], rs, xm, isd), s1);
                }
            s0 += __shfl_xor(s0, 16, 64);
            s1 += __shfl_xor(s1, 16, 64);
            s0 += __shfl_xor(s0, 32, 64);
            s1 += __shfl_xor(s1, 32, 64);
            if (lane < 16) {
                red[((w >> 1) * 2 + 0) * NT + wn + 16 * j + lane] = s0;
                red[((w >> 1) * 2 + 1) * NT + wn + 16 * j + lane] = s1;
            }
        }
        __syncthreads();
        for (int t = threadIdx.x; t < 2 * NT; t += 256) {
            const int q = t / NT, c = t % NT, n = n0 + c;
            if (n < g.N) g.cpart[((int64_t)btm * 2 + q) * g.N + n] = red[q * NT + c] + red[(2 + q) * NT + c];
        }
        return;
    }
    const bool split = gridDim.z > 1;
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
        const int n = n0 + wn + 16 * j + (lane & 15);
        if (n >= g.N) continue;
        float colc = 0.f, cwn[8];
        if (!split) {
            colc = gemm_colc(g, n);
            for (int c = 0; c < g.nc; ++c) cwn[c] = g.cw[(int64_t)n * g.lcw + c];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
                if (m >= g.M) continue;
                if (split) ws[((int64_t)btz * g.M + m) * g.N + n] = acc[i][j][r];
                else gemm_store(g, m, n, acc[i][j][r], colc, cwn);
            }
    }
}

// =======================================================================================
// k_gemm_skf — the short-K, wide-output GEMMs against a frozen weight (K <= 128, N = D: the
// logit GEMM z W^T and the encoder input gradient dT W0, [B, D] outputs).  Their B operand is a
// frozen Linear weight, so it is kept pre-split as bf16 planes (hi [, lo]) in k-contiguous
// [N][Kp] layout (WideState::pl_*, rebuilt with the frozen parameters), and a lane reads its MFMA
// fragments straight from them (16-byte loads, no LDS, no per-tile conversion).  One wave per
// workgroup: it converts its 64 A rows (all of K) into fragments held in registers once, then
// walks the n tiles nt = blockIdx.x, + gridDim.x, ... (32 columns each) with the next tile's B
// fragments in flight under the current tile's MFMAs and epilogue — no barriers, no LDS.
// grid (G, row tiles), G a multiple of 8: blocks b and b + 8 share an XCD and walk the same
// columns, so a B tile is read from HBM about once per XCD.
// CS: the column-sum epilogue of GemmOp::cpart (chunks = 64-row tiles).
// =======================================================================================
template <class P>
MMVAE_DEV typename MM<P>::frag skf_split(const float4& a, const float4& b) {
    const float e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = pk_bf16(e[2 * i], e[2 * i + 1]);
    if constexpr (IsX3<P>::value) {
        uint32_t l[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            l[i] = pk_bf16(e[2 * i] - __uint_as_float(h[i] << 16), e[2 * i + 1] - __uint_as_float(h[i] & 0xffff0000u));
        return typename MM<P>::frag{__builtin_bit_cast(bf16x8, uint4{h[0], h[1], h[2], h[3]}),
                                    __builtin_bit_cast(bf16x8, uint4{l[0], l[1], l[2], l[3]})};
    } else {
        return __builtin_bit_cast(bf16x8, uint4{h[0], h[1], h[2], h[3]});
    }
}
template <class P>
MMVAE_DEV typename MM<P>::frag skf_bfrag(const __bf16* p, int64_t plane) {
    if constexpr (IsX3<P>::value)
        return typename MM<P>::frag{*reinterpret_cast<const bf16x8*>(p), *reinterpret_cast<const bf16x8*>(p + plane)};
    else
        return *reinterpret_cast<const bf16x8*>(p);
}
template <class P, bool CS>
__global__ __launch_bounds__(64) void k_gemm_skf(GemmOp g) {
    using M = MM<P>;
    using Fr = typename M::frag;
    const int lane = threadIdx.x;
    const int mt = blockIdx.y, m0 = mt * 64;
    const int KC = g.bkp / 32;  // <= 4 (host)
    const int ntiles = (g.N + 31) / 32;
    // the wave's A fragments: rows m0 + 16 i + (lane & 15), k = 32 kc + 8 (lane >> 4) .. + 7
    Fr fa[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + 16 * i + (lane & 15);
        const float* ar = g.A + (int64_t)min(m, g.M - 1) * g.sam;
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            if (kc >= KC) break;
            const int k0 = 32 * kc + 8 * (lane >> 4);
            const float4 u = *reinterpret_cast<const float4*>(ar + min(k0, g.K - 4));
            const float4 v = *reinterpret_cast<const float4*>(ar + min(k0 + 4, g.K - 4));
            const bool ok = m < g.M;
            const float4 z4 = float4{0.f, 0.f, 0.f, 0.f};
            fa[i][kc] = skf_split<P>((ok && k0 < g.K) ? u : z4, (ok && k0 + 4 < g.K) ? v : z4);
        }
    }
    // the lane's rows m0 + 16 i + 4 (lane >> 4) + r: store, the covariate rows (nc <= 2); CS, the row scale
    float car[4][4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = min(m0 + 16 * i + 4 * (lane >> 4) + r, g.M - 1);
            if constexpr (CS) {
                car[i][r][0] = g.cxf.rs ? g.cxf.rs[m] : 1.f;
            } else {
#pragma unroll
                for (int c = 0; c < 2; ++c) car[i][r][c] = c < g.nc ? g.ca[(int64_t)m * g.lca + c] : 0.f;
            }
        }
    // one n tile's operands, all issued together one tile ahead (tile t + 1's under tile t's MFMAs
    // and stores): the column constants (CS: the raw inputs and the transform's vectors) first,
    // then the B fragments (columns nt * 32 + 16 j + (lane & 15), k = 32 kc + 8 (lane >> 4)).  The
    // loop is unrolled by two over a ping-pong pair, so nothing is copied between registers.
    struct Tile {
        Fr fb[2][4];
        float cc[2], cw2[2][2], xv[CS ? 2 : 1][4][4];
    };
    auto fetch = [&](int nt, Tile& T) {
        const int n0 = nt * 32;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = min(n0 + 16 * j + (lane & 15), g.N - 1);
            if constexpr (CS) {
                T.cc[j] = g.cxf.xm[n];
                T.cw2[j][0] = g.cxf.isd[n];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int m = min(m0 + 16 * i + 4 * (lane >> 4) + r, g.M - 1);
                        T.xv[j][i][r] = g.cx[(int64_t)m * g.ldcx + n];
                    }
            } else {
                // unconditional loads (the host's combined column vector; the covariate columns past
                // nc re-read the last one, or the column vector, and meet zero rows): a load behind a
                // pointer test is consumed at once, and its wait would drain everything in flight
                T.cc[j] = g.colv[n];
#pragma unroll
                for (int c = 0; c < 2; ++c) T.cw2[j][c] = g.cw[(int64_t)n * g.lcw + min(c, max(g.nc - 1, 0))];
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // (issue order: the constants before the B fragments)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = min(n0 + 16 * j + (lane & 15), g.N - 1);
            const __bf16* bp = g.bpl + (int64_t)n * g.bkp + 8 * (lane >> 4);
#pragma unroll
            for (int kc = 0; kc < 4; ++kc)  // (all four: k chunks past KC reload the last, unused)
                T.fb[j][kc] = skf_bfrag<P>(bp + 32 * min(kc, KC - 1), g.bplane);
        }
    };
    auto compute = [&](int nt, const Tile& T) {
        const int n0 = nt * 32;
        f32x4 acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            if (kc >= KC) break;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = M::mma(fa[i][kc], T.fb[j][kc], acc[i][j]);
        }
        if constexpr (CS) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int n = n0 + 16 * j + (lane & 15);
                float s0 = 0.f, s1 = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int m = m0 + 16 * i + 4 * (lane >> 4) + r;
                        const float v = (m < g.M && n < g.N) ? acc[i][j][r] : 0.f;
                        s0 += v;
                        s1 = fmaf(v, enc_in_acc(T.xv[j][i][r], car[i][r][0], T.cc[j], T.cw2[j][0]), s1);
                    }
                s0 += __shfl_xor(s0, 16, 64);
                s1 += __shfl_xor(s1, 16, 64);
                s0 += __shfl_xor(s0, 32, 64);
                s1 += __shfl_xor(s1, 32, 64);
                if (lane < 16 && n < g.N) {
                    g.cpart[((int64_t)mt * 2 + 0) * g.N + n] = s0;
                    g.cpart[((int64_t)mt * 2 + 1) * g.N + n] = s1;
                }
            }
        } else {
            // (plain row-major stores, no read-modify-write: a load among the stores would make the
            // next tile's wait for its operands a wait for every store before it)
            float* cb = g.C + (int64_t)(m0 + 4 * (lane >> 4)) * g.scm + n0 + (lane & 15);
            float vv[4][4][2];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        float v = fmaf(g.alpha, acc[i][j][r], T.cc[j]);
#pragma unroll
                        for (int c = 0; c < 2; ++c) v = fmaf(car[i][r][c], T.cw2[j][c], v);  // (car = 0 past nc)
                        vv[i][r][j] = g.act == 1 ? fmaxf(v, 0.f) : v;
                    }
            if (m0 + 64 <= g.M && n0 + 32 <= g.N) {  // (uniform) a full tile: plain stores
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int j = 0; j < 2; ++j) cb[(int64_t)(16 * i + r) * g.scm + 16 * j] = vv[i][r][j];
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            if (m0 + 16 * i + 4 * (lane >> 4) + r < g.M && n0 + 16 * j + (lane & 15) < g.N)
                                cb[(int64_t)(16 * i + r) * g.scm + 16 * j] = vv[i][r][j];
            }
        }
    };
    const int G = gridDim.x;
    // every fetch is issued unconditionally (past the end: the last tile again, unused) so the
    // loads in flight are a static count and each tile waits for its own operands only
    Tile t0, t1;
    const int last = ntiles - 1;
    int nt = blockIdx.x;
    fetch(min(nt, last), t0);
    for (; nt < ntiles; nt += 2 * G) {
        fetch(min(nt + G, last), t1);
        compute(nt, t0);
        if (nt + G >= ntiles) break;
        fetch(min(nt + 2 * G, last), t0);
        compute(nt + G, t1);
    }
}

// every column's gemm_colc (the GEMM's biases, summed in its fixed order) into one vector
__global__ __launch_bounds__(256) void k_w_colc(GemmOp g, float* __restrict__ out) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n < g.N) out[n] = gemm_colc(g, n);
}

// bf16 planes (hi at out, lo at out + plane) of a frozen weight, B(k, n) = W[k sk + n sn], in
// the [N][Kp] k-contiguous layout of k_gemm_skf (k >= K: zero)
__global__ __launch_bounds__(256) void k_w_planes(const float* __restrict__ W, int64_t sk, int64_t sn, int N, int K,
                                                  int Kp, __bf16* __restrict__ out, int64_t plane) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)N * Kp) return;
    const int n = (int)(i % N), k = (int)(i / N);  // n fastest: coalesced reads when sn == 1
    const float v = k < K ? W[(int64_t)k * sk + (int64_t)n * sn] : 0.f;
    const __bf16 h = (__bf16)v;
    out[(int64_t)n * Kp + k] = h;
    out[plane + (int64_t)n * Kp + k] = (__bf16)(v - (float)h);
}

// =======================================================================================
// Wide-path state (device buffers sized at create, so a step allocates nothing and can be
// captured into a step graph)
// =======================================================================================
struct WLayer {
    const float* W = nullptr;  // [out][in] (frozen; vMF Angular layers: the normalised copy)
    const float* b = nullptr;  // [out] or null (Angular)
    int in = 0, out = 0;
    bool relu = false;         // ReLU after this layer
    float* act = nullptr;      // [Bpad][out] the layer's output (post-ReLU)
};

// a queued narrow column sum of the wide path (k_w_redsmall below)
struct RedJob {
    const float* Y;
    const float* X;
    float* out;
    int64_t ldy, ldx, wsoff;
    int KX, NJ, accumulate;
    float alpha;
};
static constexpr int RJ_MAX = 12;
struct RedJobs {
    int n = 0, M = 0, maxnj = 0;
    int64_t wsuse = 0;
    RedJob j[RJ_MAX];
};
struct WideState {
    int64_t Bp = 0, D = 0;
    // dense [Bpad][D] blocks: the raw batch, logits, their gradient, the nu pre-activation /
    // its gradient; Xn, the normalised encoder input, only on f32 handles (the bf16 / x3 GEMMs
    // transform the raw batch as they load it)
    float *X = nullptr, *Xn = nullptr, *LG = nullptr, *G = nullptr, *U = nullptr;
    float* Uin = nullptr;  // the nu pre-activation when R > RMAX (a GEMM output; U holds dL/du)
    // per-gene vectors [5][D]: sdv, softplus'(ln_x_sd), the encoder's two column sums, 1 / sdv
    float *gvec = nullptr;
    float* cr_part = nullptr;  // column-reduction partials (k_colred)
    int64_t cr_cap = 0;
    float* one = nullptr;    // a device 1.0f (ones operand of the column-sum GEMMs)
    float* ws = nullptr;     // split-K partials
    int64_t ws_cap = 0;
    // covariates of the batch rows, per-row scalars
    // rowv [8][Bpad]: loss, KL, depth d, depth pre-activation, its gradient, (vMF) kappa scalars,
    // (vMF) 1 / |log1p(x_b)|, 1 / |log1p(relu(x_b)) + eps|
    float *Cb = nullptr, *rowv = nullptr;
    // latent blocks [Bpad][K]: heads (raw mean, raw lnvar), covariate part, mean, z, eps, dz,
    // dmean, dlnvar(raw)
    float *Mr = nullptr, *Ar = nullptr, *Ce = nullptr, *Mn = nullptr, *Z = nullptr, *Ep = nullptr,
          *dZ = nullptr, *dM = nullptr, *dA = nullptr;
    // NB overdispersion side: hnu [Bpad][H], nu heads [Bpad][R] (raw mean / raw lnvar), znu, eps,
    // their gradients, dhnu
    float *Hn = nullptr, *NMr = nullptr, *NAr = nullptr, *Zn = nullptr, *En = nullptr, *dZn = nullptr,
          *dNM = nullptr, *dNA = nullptr, *dHn = nullptr;
    // hidden activations' gradient ping-pong [Bpad][maxw]
    float *dT0 = nullptr, *dT1 = nullptr;
    int maxw = 0;
    std::vector<WLayer> enc, dec;  // dec: hidden layers, then the final big layer (-> D)
    float* wtil = nullptr;         // vMF: normalised Angular weights of every encoder layer
    float* lossv = nullptr;        // [2]: scratch sums
    struct RedJobs redq;           // narrow column sums queued for one launch (red_flush)
    // bf16 planes of the frozen B operands of the two short-K GEMMs (k_gemm_skf, null: not
    // eligible): the decoder's final weight (logits) and the first encoder weight, transposed
    // (the encoder input gradient); [D][kp] each, the lo plane after the hi one
    __bf16 *pl_F = nullptr, *pl_E = nullptr;
    int kp_F = 0, kp_E = 0;
    float* colv = nullptr;  // [D] the short-K GEMM's combined column constants
};

static hipError_t walloc(float** p, int64_t n) { return hipMalloc(p, sizeof(float) * (size_t)(n > 0 ? n : 1)); }

// split-K count: one round of >= 512 workgroups where the tile grid is smaller, each split
// keeping >= min_ch chunks, capped by the partial buffer
static int split_count(const WideState* w, int64_t MN, int tiles, int nch, int min_ch) {
    int S = 1;
    if (tiles < 512 && nch >= 2 * min_ch) {
        S = std::min((512 + tiles - 1) / tiles, nch / min_ch);
        const int64_t cap = w->ws_cap / MN;
        if (S > cap) S = (int)cap;
        if (S < 2) S = 1;
    }
    return S;
}

static void launch_reduce(Engine* e, const GemmOp& g, int S) {
    const int64_t MN = (int64_t)g.M * g.N;
    const int nb = (int)std::min<int64_t>((MN + 255) / 256, 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, e->stream, g, S, (const float*)e->wide_st->ws);
}

template <class P, bool AT, int NT, int PF>
static void launch_mf(Engine* e, const GemmOp& g, const GemmX& x, dim3 grid, int cps, int vec) {
    float* ws = e->wide_st->ws;
    const bool akf = g.sak == 1, bkf = g.sbk == 1;
    if constexpr (AT) {
        if (bkf) hipLaunchKernelGGL((k_gemm_mf<P, true, true, true, NT, PF>), grid, dim3(256), 0, e->stream, g, x, cps, ws, vec);
        else hipLaunchKernelGGL((k_gemm_mf<P, true, false, true, NT, PF>), grid, dim3(256), 0, e->stream, g, x, cps, ws, vec);
    } else if (akf) {
        if (bkf) hipLaunchKernelGGL((k_gemm_mf<P, true, true, false, NT, PF>), grid, dim3(256), 0, e->stream, g, x, cps, ws, vec);
        else hipLaunchKernelGGL((k_gemm_mf<P, true, false, false, NT, PF>), grid, dim3(256), 0, e->stream, g, x, cps, ws, vec);
    } else {
        if (bkf) hipLaunchKernelGGL((k_gemm_mf<P, false, true, false, NT, PF>), grid, dim3(256), 0, e->stream, g, x, cps, ws, vec);
        else hipLaunchKernelGGL((k_gemm_mf<P, false, false, false, NT, PF>), grid, dim3(256), 0, e->stream, g, x, cps, ws, vec);
    }
}
// the input transform's GEMM runs over K = D (two stages); the others by their chunks per split
template <class P, bool AT>
static void launch_mf_nt(Engine* e, const GemmOp& g, const GemmX& x, dim3 grid, int cps, int vec, int nt) {
    if constexpr (AT) {
        if (nt == 128) launch_mf<P, true, 128, 2>(e, g, x, grid, cps, vec);
        else launch_mf<P, true, 64, 2>(e, g, x, grid, cps, vec);
    } else {
        const bool pf2 = cps >= 16;
        if (nt == 128) {
            if (pf2) launch_mf<P, false, 128, 2>(e, g, x, grid, cps, vec);
            else launch_mf<P, false, 128, 1>(e, g, x, grid, cps, vec);
        } else {
            if (pf2) launch_mf<P, false, 64, 2>(e, g, x, grid, cps, vec);
            else launch_mf<P, false, 64, 1>(e, g, x, grid, cps, vec);
        }
    }
}

// float4 operands: 16-byte aligned bases, strides and contiguous extents multiples of 4 floats
// (k_gemm_mf's loads are unconditional float4s with clamped indices)
static bool mf_vec(const GemmOp& g) {
    auto al = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool akf = g.sak == 1, bkf = g.sbk == 1;
    const int64_t sa = akf ? g.sam : g.sak, sb = bkf ? g.sbn : g.sbk;
    return al(g.A) && al(g.B) && sa % 4 == 0 && sb % 4 == 0 && (akf ? g.K : g.M) % 4 == 0 &&
           (bkf ? g.K : g.N) % 4 == 0;
}
static bool mf_modes(const Engine* e) {
    return e->cfg.dtype != MMVAE_DTYPE_F32 && !getenv_is("MMVAE_WIDE_F32GEMM", "1");
}
// the encoder input transform inside the first encoder GEMM (its A operand is the raw [B][D]
// batch, its B the [out][D] weight); otherwise the normalised block Xn is materialised
static bool at_in_gemm(const Engine* e) {
    if (!mf_modes(e) || e->D % 4 != 0) return false;
    if (e->cfg.model == MMVAE_MODEL_VMF) return true;  // layer 0 reads its Angular copy from wtil's start
    // (parameter slots are packed: the frozen weight's offset decides its alignment)
    const ParamSlot* sl = e->slot(e->fz_enc_w);
    return sl && sl->off % 4 == 0;
}
static bool use_mf(const Engine* e, const GemmOp& g) {
    if (!mf_modes(e)) return false;
    if (!(g.sak == 1 || g.sam == 1) || !(g.sbk == 1 || g.sbn == 1)) return false;
    if (g.sam == 0 || g.sbn == 0) return false;  // broadcast operands (column sums): the f32 kernel
    if (!mf_vec(g)) return false;
    return g.M >= 32 && g.N >= 32 && g.K >= 32 && (int64_t)g.M * g.N * (int64_t)g.K >= ((int64_t)1 << 22);
}

// the short-K kernel: a frozen B operand with planes, k-contiguous float4 A rows, K <= 128, at
// most two covariate columns in the epilogue
static bool use_sk(const Engine* e, const GemmOp& g) {
    if (!g.bpl || getenv_is("MMVAE_WIDE_NOSK", "1") || !mf_modes(e)) return false;
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return g.sak == 1 && al(g.A) && g.sam % 4 == 0 && g.K % 4 == 0 && g.K <= 128 && g.bkp >= g.K &&
           g.bkp % 32 == 0 && g.bkp <= 128 && g.nc <= 2 && g.M >= 1 && g.N >= 32 && !g.accumulate &&
           (g.cpart || g.scn == 1);
}

// C = epilogue(A . B); `x` non-null: the encoder input transform on A (the f32 handles
// materialise the normalised block instead, see enc_forward)
// ---- narrow shapes: the column sums / small weight gradients over the batch rows and the tiny
// Linears of the overdispersion side (H, R, C of a few units).  As GEMMs they cost a split-K
// launch of mostly idle 64 x 64 MFMA tiles plus a reduce (~20 us each, ~15 of them per step);
// here a column-parallel two-phase sum (fixed order: rows in RS splits, then the splits) and
// a thread-per-output kernel.
static constexpr int RS_SMALL = 16;  // row splits of k_w_redsmall
// A batch of such sums (RedJobs, one launch per phase): job z's ws[s][j] = sum over split s's
// rows m of Y[m][j / KX] * (X ? X[m][j % KX] : 1)  (j < NJ), then out[j] = alpha sum_s ws[s][j]
__global__ __launch_bounds__(256) void k_w_redsmall(RedJobs q, float* __restrict__ ws) {
    __shared__ float part[4][64];
    const RedJob& jb = q.j[blockIdx.z];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + lane;
    if ((int)blockIdx.x * 64 >= jb.NJ) return;  // (workgroup-uniform)
    const int M = q.M, per = (M + RS_SMALL - 1) / RS_SMALL;
    const int m0 = blockIdx.y * per, m1 = min(M, m0 + per);
    const float* Y = jb.Y;
    const float* X = jb.X;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (j < jb.NJ) {
        const int n = X ? j / jb.KX : j, k = X ? j % jb.KX : 0;
        int m = m0 + w;
        for (; m + 12 < m1; m += 16) {  // four rows in flight per lane
            float y[4], xv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                y[u] = Y[(int64_t)(m + 4 * u) * jb.ldy + n];
                xv[u] = X ? X[(int64_t)(m + 4 * u) * jb.ldx + k] : 1.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) s[u] = fmaf(y[u], xv[u], s[u]);
        }
        for (; m < m1; m += 4) s[0] = fmaf(Y[(int64_t)m * jb.ldy + n], X ? X[(int64_t)m * jb.ldx + k] : 1.f, s[0]);
    }
    part[w][lane] = (s[0] + s[1]) + (s[2] + s[3]);
    __syncthreads();
    if (w == 0 && j < jb.NJ)
        ws[jb.wsoff + (int64_t)blockIdx.y * jb.NJ + j] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
}
__global__ __launch_bounds__(256) void k_w_redsmall_fin(RedJobs q, const float* __restrict__ ws) {
    const RedJob& jb = q.j[blockIdx.z];
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= jb.NJ) return;
    float v = 0.f;
#pragma unroll 4
    for (int s = 0; s < RS_SMALL; ++s) v += ws[jb.wsoff + (int64_t)s * jb.NJ + j];
    v *= jb.alpha;
    jb.out[j] = jb.accumulate ? jb.out[j] + v : v;
}
static hipError_t red_flush(Engine* e);
static hipError_t redsmall(Engine* e, int M, int N, const float* Y, int64_t ldy, const float* X, int64_t ldx, int KX,
                           float* out, float alpha, int accumulate);

// C[m][n] = act(alpha sum_k A[m][k] B[k][n] + biases) (+ C), one thread per output: K <= 16 and N <= 256
__global__ __launch_bounds__(256) void k_w_lin_small(GemmOp g) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)g.M * g.N) return;
    const int m = (int)(i / g.N), n = (int)(i % g.N);
    float acc = 0.f;
    for (int k = 0; k < g.K; ++k) acc = fmaf(g.A[(int64_t)m * g.sam + (int64_t)k * g.sak], g.B[(int64_t)k * g.sbk + (int64_t)n * g.sbn], acc);
    gemm_epilogue(g, m, n, acc);
}

static hipError_t gemm(Engine* e, const GemmOp& g, const GemmX* x = nullptr) {
    if (g.M <= 0 || g.N <= 0) return hipSuccess;
    // per-kernel timers (bench.py's wide lines): the gene GEMMs apart from the small ones
    ScopedTimer tmg(e, (int64_t)g.M * g.N * g.K >= ((int64_t)1 << 26) ? "w_gemm_gene" : "w_gemm_small");
    if (!x && g.K <= 16 && g.N <= 256 && g.nc == 0) {
        hipLaunchKernelGGL(k_w_lin_small, dim3((unsigned)(((int64_t)g.M * g.N + 255) / 256)), dim3(256), 0, e->stream, g);
        return hipGetLastError();
    }
    WideState* w = e->wide_st;
    const int64_t MN = (int64_t)g.M * g.N;
    if (!x && use_sk(e, g)) {
        GemmOp gs = g;
        if (!g.cpart) {  // the column constants as one vector; cw pointed at something valid
            hipLaunchKernelGGL(k_w_colc, dim3((g.N + 255) / 256), dim3(256), 0, e->stream, g, w->colv);
            gs.colv = w->colv;
            if (g.nc == 0) {
                gs.cw = w->colv;  // (read, times the zero covariate rows)
                gs.lcw = 0;
            }
        }
        const int tmr = (g.M + 63) / 64, ntl = (g.N + 31) / 32;
        // one wave per SIMD over the chip (1024 SIMDs; ~400 registers a lane), G a multiple of 8
        int G = std::max(8, (1024 / std::max(1, tmr)) / 8 * 8);
        G = std::min(G, (ntl + 7) / 8 * 8);
        const dim3 grid((unsigned)G, (unsigned)tmr);
        if (e->cfg.dtype == MMVAE_DTYPE_BF16X3) {
            if (g.cpart) hipLaunchKernelGGL((k_gemm_skf<X3, true>), grid, dim3(64), 0, e->stream, gs);
            else hipLaunchKernelGGL((k_gemm_skf<X3, false>), grid, dim3(64), 0, e->stream, gs);
        } else {
            if (g.cpart) hipLaunchKernelGGL((k_gemm_skf<__bf16, true>), grid, dim3(64), 0, e->stream, gs);
            else hipLaunchKernelGGL((k_gemm_skf<__bf16, false>), grid, dim3(64), 0, e->stream, gs);
        }
        return hipGetLastError();
    }
    if (x || use_mf(e, g)) {
        const int nt = g.N >= 96 ? 128 : 64;
        const int tm = (g.M + 63) / 64, tn = (g.N + nt - 1) / nt, nch = (g.K + 31) / 32;
        int S = g.cpart ? 1 : split_count(w, MN, tm * tn, nch, 8);
        const int cps = (nch + S - 1) / S;
        S = std::max(1, (nch + cps - 1) / cps);
        if (x && !mf_vec(g)) return hipErrorInvalidValue;  // (at_in_gemm routes these to Xn)
        // (the XCD-aware tile order measured slower on every wide GEMM shape: opt-in only)
        const int vec = getenv_is("MMVAE_WIDE_XCD", "1") ? 2 : 0;
        const GemmX gx = x ? *x : GemmX{};
        const dim3 grid(tn, tm, S);
        if (e->cfg.dtype == MMVAE_DTYPE_BF16X3) {
            if (x) launch_mf_nt<X3, true>(e, g, gx, grid, cps, vec, nt);
            else launch_mf_nt<X3, false>(e, g, gx, grid, cps, vec, nt);
        } else {
            if (x) launch_mf_nt<__bf16, true>(e, g, gx, grid, cps, vec, nt);
            else launch_mf_nt<__bf16, false>(e, g, gx, grid, cps, vec, nt);
        }
        if (S > 1) launch_reduce(e, g, S);
        return hipGetLastError();
    }
    const int tm = (g.M + GT - 1) / GT, tn = (g.N + GT - 1) / GT;
    const int nch = (g.K + GK - 1) / GK;
    int S = split_count(w, MN, tm * tn, nch, 16);
    const int cps = (nch + S - 1) / S;
    S = std::max(1, (nch + cps - 1) / cps);
    hipLaunchKernelGGL(k_gemm, dim3(tn, tm, S), dim3(256), 0, e->stream, g, cps, w->ws);
    if (S > 1) launch_reduce(e, g, S);
    return hipGetLastError();
}

// C[M][N] (row-major, ldc) [+]= A[M][K] (row-major) . W^T, W [N][K] row-major (a Linear's weight)
static hipError_t linear_fwd(Engine* e, int M, int N, int K, const float* A, int64_t lda, const float* W,
                             const float* bias, float* C, int64_t ldc, int act = 0, int accumulate = 0) {
    GemmOp g;
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.sam = lda; g.sak = 1;
    g.B = W; g.sbk = 1; g.sbn = K;
    g.C = C; g.scm = ldc; g.scn = 1;
    g.bias = bias; g.act = act; g.accumulate = accumulate;
    return gemm(e, g);
}
// dX[M][K] [+]= dY[M][N] . W, W [N][K] row-major
static hipError_t linear_dx(Engine* e, int M, int N, int K, const float* dY, int64_t ldy, const float* W, float* dX,
                            int64_t ldx, int accumulate = 0) {
    GemmOp g;
    g.M = M; g.N = K; g.K = N;
    g.A = dY; g.sam = ldy; g.sak = 1;
    g.B = W; g.sbk = K; g.sbn = 1;
    g.C = dX; g.scm = ldx; g.scn = 1;
    g.accumulate = accumulate;
    return gemm(e, g);
}
// dW[N][K] = dY[M][N]^T . X[M][K]  (a Linear's weight gradient over the batch rows)
static hipError_t linear_dw(Engine* e, int M, int N, int K, const float* dY, int64_t ldy, const float* X, int64_t ldx,
                            float* dW) {
    if ((int64_t)N * K <= 4096 && (N < 32 || K < 32))  // a few hundred dot products over the rows
        return redsmall(e, M, N, dY, ldy, X, ldx, K, dW, 1.f, 0);
    GemmOp g;
    g.M = N; g.N = K; g.K = M;
    g.A = dY; g.sam = 1; g.sak = ldy;
    g.B = X; g.sbk = ldx; g.sbn = 1;
    g.C = dW; g.scm = K; g.scn = 1;
    return gemm(e, g);
}
// out[n] = sign * sum_{m < M} Y[m][n]  (column sums, fixed order)
// queue one narrow sum; red_flush launches the queued group (two launches for all of them)
static hipError_t redsmall(Engine* e, int M, int N, const float* Y, int64_t ldy, const float* X, int64_t ldx, int KX,
                           float* out, float alpha, int accumulate) {
    RedJobs& q = e->wide_st->redq;
    const int NJ = N * (X ? KX : 1);
    if (q.n == RJ_MAX || (q.n > 0 && q.M != M) || q.wsuse + (int64_t)RS_SMALL * NJ > e->wide_st->ws_cap) {
        const hipError_t er = red_flush(e);
        if (er != hipSuccess) return er;
    }
    RedJob& jb = q.j[q.n++];
    jb.Y = Y;
    jb.X = X;
    jb.out = out;
    jb.ldy = ldy;
    jb.ldx = ldx;
    jb.KX = KX;
    jb.NJ = NJ;
    jb.alpha = alpha;
    jb.accumulate = accumulate;
    jb.wsoff = q.wsuse;
    q.wsuse += (int64_t)RS_SMALL * NJ;
    q.M = M;
    q.maxnj = std::max(q.maxnj, NJ);
    return hipSuccess;
}
static hipError_t red_flush(Engine* e) {
    RedJobs& q = e->wide_st->redq;
    if (q.n == 0) return hipSuccess;
    ScopedTimer tm(e, "w_colsum_small");
    hipLaunchKernelGGL(k_w_redsmall, dim3((q.maxnj + 63) / 64, RS_SMALL, q.n), dim3(256), 0, e->stream, q, e->wide_st->ws);
    hipLaunchKernelGGL(k_w_redsmall_fin, dim3((q.maxnj + 255) / 256, 1, q.n), dim3(256), 0, e->stream, q,
                       (const float*)e->wide_st->ws);
    q = RedJobs{};
    return hipGetLastError();
}
static hipError_t colsum(Engine* e, int M, int N, const float* Y, int64_t ldy, float* out, float sign = 1.f,
                         int accumulate = 0) {
    return redsmall(e, M, N, Y, ldy, nullptr, 0, 1, out, sign, accumulate);
}

// =======================================================================================
// Batch densify, covariates, staged copy
// =======================================================================================
__global__ __launch_bounds__(256) void k_w_stage(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

// =======================================================================================
// Block reductions (256 threads, fixed order)
// =======================================================================================
MMVAE_DEV float wblock_sum(float v, float* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}
MMVAE_DEV float wblock_max(float v, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// =======================================================================================
// Batch densify (mmvae_io.hh:208-245), one workgroup per batch row: the row is zeroed with
// 16-byte stores, then the cell's nonzeros are scattered.  The same pass takes the row terms
// that need only the nonzeros (fixed-order block sums):
//   NB: the raw-count Linears depth(x) (nb.hh:400, 498) and nu_enc(x) (nb.hh:444-451) for
//       H <= HMAX (bias included);
//   vMF: 1 / |log1p(x_b)| (vmf.hh:253, F::normalize eps 1e-12) and 1 / |log1p(relu(x_b)) + eps|
//       (vmf.hh:421-422), the zeros' eps^2 terms in closed form.
// =======================================================================================
struct WDens {
    int D, C, H;
    const int64_t* cells;
    const int64_t* rowptr;
    const int32_t* col;
    const float* val;
    const float* covar;
    float *X, *Cb;
    // NB row dots (null: not taken here)
    const float *dw, *db, *Wne, *bne;
    float *dpre, *Hn;
    // vMF row scales (null: NB)
    float *rs1, *rs2;
    float epsD;
    int seg;  // 1: the LDS segment build; 0: the store pass (MMVAE_WIDE_DENSSTORE=1)
};
// The row is built in LDS segments of WSEG genes (zeroed, the segment's nonzeros scattered, then
// written out with coalesced 16-byte stores), so every byte of the dense row is written once.
// The segments' first entries come from one parallel pass over the row's entries (genes sorted:
// entry i starts every segment after its predecessor's, up to its own) — no serial search.
#ifndef MMVAE_WSEG
#define MMVAE_WSEG 4096
#endif
static constexpr int WSEG = MMVAE_WSEG, WSEG_MAX = 64;
__global__ __launch_bounds__(256) void k_w_densify2(WDens a) {
    __shared__ __attribute__((aligned(16))) float seg[WSEG];
    __shared__ float red[4];
    __shared__ int64_t bnd[WSEG_MAX + 1];
    const int b = blockIdx.x;
    const int64_t cell = a.cells[b];
    float* xr = a.X + (int64_t)b * a.D;
    const int64_t r0 = a.rowptr[cell], r1 = a.rowptr[cell + 1];
    const int32_t* cr = a.col;
    // the row terms over its nonzeros
    float dp = 0.f, hn[HMAX], n1 = 0.f, n2 = 0.f;
#pragma unroll
    for (int h = 0; h < HMAX; ++h) hn[h] = 0.f;
    for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
        const int g = cr[i];
        const float x = a.val[i];
        if (a.dpre) {
            dp = fmaf(x, a.dw[g], dp);
#pragma unroll
            for (int h = 0; h < HMAX; ++h)
                if (h < a.H) hn[h] = fmaf(x, a.Wne[(int64_t)h * a.D + g], hn[h]);
        }
        if (a.rs1) {
            const float l = log1pf(x), ly = log1pf(fmaxf(x, 0.f)) + a.epsD;
            n1 = fmaf(l, l, n1);
            n2 += ly * ly - a.epsD * a.epsD;
        }
    }
    const bool v4 = (a.D & 3) == 0;
    if (v4 && !a.seg) {
        // the row zeroed with 16-byte stores, then, after the barrier (its workgroup fence completes
        // those stores), the nonzeros written over it: one pass of stores, no LDS, one barrier —
        // the LDS segment build below is bound by its chain of per-segment barriers
        for (int i = threadIdx.x; i < a.D / 4; i += 256) reinterpret_cast<float4*>(xr)[i] = float4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) xr[cr[i]] = a.val[i];
    } else {
    const int nseg = (a.D + WSEG - 1) / WSEG;
    for (int sgi = 0; sgi < nseg; ++sgi) {
        const int s0 = sgi * WSEG, len = min(WSEG, a.D - s0);
        const int g0 = sgi % WSEG_MAX == 0 ? sgi : -1;  // the first segment of a group of WSEG_MAX
        if (g0 >= 0)
            for (int t = threadIdx.x; t <= WSEG_MAX; t += 256) bnd[t] = r1;
        for (int i = threadIdx.x; i < WSEG / 4; i += 256) reinterpret_cast<float4*>(seg)[i] = float4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        if (g0 >= 0) {  // bnd[t]: the first entry of the group's segment t (t = WSEG_MAX: the next group's)
            for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) {
                const int sg = cr[i] / WSEG, sp = i == r0 ? -1 : cr[i - 1] / WSEG;
                for (int t = max(sp + 1, g0); t <= min(sg, g0 + WSEG_MAX); ++t) bnd[t - g0] = i;
            }
            __syncthreads();
        }
        // this segment's entries: [bnd[j], bnd[j + 1])
        const int j = sgi % WSEG_MAX;
        for (int64_t i = bnd[j] + threadIdx.x; i < bnd[j + 1]; i += 256) seg[cr[i] - s0] = a.val[i];
        __syncthreads();
        if (v4) {
            for (int i = threadIdx.x; i < len / 4; i += 256)
                *reinterpret_cast<float4*>(xr + s0 + 4 * i) = reinterpret_cast<const float4*>(seg)[i];
        } else {
            for (int i = threadIdx.x; i < len; i += 256) xr[s0 + i] = seg[i];
        }
        __syncthreads();  // seg is rewritten by the next segment
    }
    }
    for (int c = threadIdx.x; c < a.C; c += 256) a.Cb[(int64_t)b * a.C + c] = a.covar[cell * a.C + c];
    if (a.dpre) {
        dp = wblock_sum(dp, red);
        if (threadIdx.x == 0) a.dpre[b] = dp + a.db[0];
        for (int h = 0; h < a.H && h < HMAX; ++h) {
            const float v = wblock_sum(hn[h], red);
            if (threadIdx.x == 0) a.Hn[(int64_t)b * a.H + h] = v + a.bne[h];
        }
    }
    if (a.rs1) {
        n1 = wblock_sum(n1, red);
        n2 = wblock_sum(n2, red);
        if (threadIdx.x == 0) {
            a.rs1[b] = 1.f / fmaxf(sqrtf(n1), 1e-12f);
            a.rs2[b] = 1.f / fmaxf(sqrtf(fmaf((float)a.D * a.epsD, a.epsD, n2)), 1e-12f);
        }
    }
}

// =======================================================================================
// Column reductions of a dense [M rows][N] block (the batch sums of the gene-vector gradients,
// nb.hh:410-460 / vmf.hh:256-290 backward), fixed order, no atomics:
//   s_j(n) = sum_m a_j(m) Y(m, n),  columns j: [a0 (null: ones)] then A1[:, j1 .. j1 + n1 - 1]
//   XPROD: s_0 = sum_m Y(m, n), s_1 = sum_m Y(m, n) enc_in(X2(m, n)) (ln_x_sd's sum)
// Stage 1 (k_colred): a thread owns 4 consecutive columns of one chunk of rows -> part[chunk];
// stage 2 (k_colred_fin): the chunks summed in order into the outputs.
// =======================================================================================
static constexpr int CR_QMAX = 9;
struct ColRed {
    int M, N, Q, has0, rows_per;
    const float* a0;
    const float* A1;
    int64_t la1;
    const float* Y;
    int64_t ly;
    const float* X2;  // XPROD (Q = 2)
    GemmX xf;
    float* part;  // [chunks][Q][N]
};
template <bool XPROD>
__global__ __launch_bounds__(256) void k_colred_gen(ColRed c) {
    constexpr int RG = 8;  // rows per group: their loads are all issued before the sums
    const int n = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (n >= c.N) return;
    const int r0 = blockIdx.y * c.rows_per, r1 = min(c.M, r0 + c.rows_per);
    const bool v4 = n + 3 < c.N && (c.ly & 3) == 0;
    float acc[CR_QMAX][4];
#pragma unroll
    for (int q = 0; q < CR_QMAX; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[q][j] = 0.f;
    float xm[4] = {0.f, 0.f, 0.f, 0.f}, isd[4] = {0.f, 0.f, 0.f, 0.f};
    if (XPROD)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (n + j < c.N) {
                xm[j] = c.xf.xm[n + j];
                isd[j] = c.xf.isd[n + j];
            }
    auto ld4 = [&](const float* base, int m, float (&v)[4]) {
        const float* p = base + (int64_t)m * c.ly + n;
        if (m >= r1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = 0.f;
        } else if (v4) {
            const float4 t = *reinterpret_cast<const float4*>(p);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (n + j < c.N) ? p[j] : 0.f;
        }
    };
    for (int m0 = r0; m0 < r1; m0 += RG) {
        float y[RG][4], x2[XPROD ? RG : 1][4];
#pragma unroll
        for (int i = 0; i < RG; ++i) ld4(c.Y, m0 + i, y[i]);
        if constexpr (XPROD)
#pragma unroll
            for (int i = 0; i < RG; ++i) ld4(c.X2, m0 + i, x2[i]);
#pragma unroll
        for (int i = 0; i < RG; ++i) {
            const int m = m0 + i;
            if (m >= r1) continue;
            if constexpr (XPROD) {
                const float rs = c.xf.rs ? c.xf.rs[m] : 1.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] += y[i][j];
                    acc[1][j] = fmaf(y[i][j], enc_in_acc(x2[i][j], rs, xm[j], isd[j]), acc[1][j]);
                }
            } else {
#pragma unroll
                for (int q = 0; q < CR_QMAX; ++q)
                    if (q < c.Q) {
                        const float a = (c.has0 && q == 0) ? (c.a0 ? c.a0[m] : 1.f) : c.A1[(int64_t)m * c.la1 + q - c.has0];
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[q][j] = fmaf(a, y[i][j], acc[q][j]);
                    }
            }
        }
    }
#pragma unroll
    for (int q = 0; q < CR_QMAX; ++q)
        if (q < c.Q)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (n + j < c.N) c.part[((int64_t)blockIdx.y * c.Q + q) * c.N + n + j] = acc[q][j];
}
// The float4 form (N and the row strides multiples of 4): a workgroup's rows in 64-row blocks,
// whose Q coefficient columns are staged into LDS first (block-uniform reads, no scalar load
// on the way to each fma), and the block's eight 8-row groups streamed through two register
// buffers — the next group's loads in flight under the current group's sums (ping-pong, fully
// unrolled, every load issued: rows past the chunk re-read its last row and meet a zero weight).
struct ColRed2 {
    ColRed c[2];  // blockIdx.z selects one (two independent sums over blocks of one shape in one launch)
};
template <bool XPROD>
__global__ __launch_bounds__(256) void k_colred(ColRed2 cc) {
    const ColRed& c = cc.c[blockIdx.z];
    constexpr int RG = 8;
    __shared__ float cf[CR_QMAX][64];
    const int n = (blockIdx.x * 256 + threadIdx.x) * 4;
    const int r0 = blockIdx.y * c.rows_per, r1 = min(c.M, r0 + c.rows_per);
    const int nq = XPROD ? 2 : c.Q;
    const int nc = min(n, c.N - 4);  // (threads past N load a valid column and store nothing)
    float acc[CR_QMAX][4];
#pragma unroll
    for (int q = 0; q < CR_QMAX; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[q][j] = 0.f;
    float xm[4] = {0.f, 0.f, 0.f, 0.f}, isd[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (XPROD)  // (x_mean is a packed parameter slot: no 16-byte alignment assumed)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            xm[j] = c.xf.xm[nc + j];
            isd[j] = c.xf.isd[nc + j];
        }
    float4 yb[2][RG], xb[XPROD ? 2 : 1][RG];
    auto load = [&](int buf, int m0) {
#pragma unroll
        for (int i = 0; i < RG; ++i) {
            const int m = min(m0 + i, r1 - 1);
            yb[buf][i] = *reinterpret_cast<const float4*>(c.Y + (int64_t)m * c.ly + nc);
            if constexpr (XPROD) xb[buf][i] = *reinterpret_cast<const float4*>(c.X2 + (int64_t)m * c.ly + nc);
        }
    };
    auto sum = [&](int buf, int i0) {  // rows i0 .. i0 + RG - 1 of the block
#pragma unroll
        for (int i = 0; i < RG; ++i) {
            const float* y = reinterpret_cast<const float*>(&yb[buf][i]);
            if constexpr (XPROD) {
                const float* x = reinterpret_cast<const float*>(&xb[buf][i]);
                const float w = cf[0][i0 + i], rs = cf[1][i0 + i];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float yv = w * y[j];
                    acc[0][j] += yv;
                    acc[1][j] = fmaf(yv, enc_in_acc(x[j], rs, xm[j], isd[j]), acc[1][j]);
                }
            } else {
#pragma unroll
                for (int q = 0; q < CR_QMAX; ++q)
                    if (q < nq) {
                        const float a = cf[q][i0 + i];
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[q][j] = fmaf(a, y[j], acc[q][j]);
                    }
            }
        }
    };
    for (int b0 = r0; b0 < r1; b0 += 64) {
        __syncthreads();  // the previous block's coefficient reads are done
        for (int t = threadIdx.x; t < nq * 64; t += 256) {
            const int q = t >> 6, m = b0 + (t & 63);
            float v = 0.f;
            if (m < r1) {
                if constexpr (XPROD) v = q == 0 ? 1.f : (c.xf.rs ? c.xf.rs[m] : 1.f);
                else v = (c.has0 && q == 0) ? (c.a0 ? c.a0[m] : 1.f) : c.A1[(int64_t)m * c.la1 + q - c.has0];
            }
            cf[q][t & 63] = v;
        }
        __syncthreads();
        // (sched barriers: each group's loads stay issued together, ahead of the sums that wait
        // for the other buffer — left alone, the scheduler sinks every load next to its use)
        load(0, b0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
        for (int gq = 0; gq < 64 / RG; gq += 2) {
            load(1, b0 + (gq + 1) * RG);
            __builtin_amdgcn_sched_barrier(0);
            sum(0, gq * RG);
            __builtin_amdgcn_sched_barrier(0);
            load(0, b0 + min(gq + 2, 64 / RG - 1) * RG);  // (the last trip: a spare re-read, unused)
            __builtin_amdgcn_sched_barrier(0);
            sum(1, (gq + 1) * RG);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (n >= c.N) return;
#pragma unroll
    for (int q = 0; q < CR_QMAX; ++q)
        if (q < nq)
            *reinterpret_cast<float4*>(c.part + ((int64_t)blockIdx.y * nq + q) * c.N + n) =
                float4{acc[q][0], acc[q][1], acc[q][2], acc[q][3]};
}
// outputs: column 0 -> o0[n s0] = alpha0 s (and o0b[n s0] = beta0 s); the A1 columns j ->
// o1[j q1 + n s1] = alpha1 s (the XPROD sum: o1[n s1])
struct ColOut {
    float* o0 = nullptr;
    float* o0b = nullptr;
    int64_t s0 = 1;
    float alpha0 = 1.f, beta0 = 1.f;
    float* o1 = nullptr;
    int64_t q1 = 0, s1 = 1;
    float alpha1 = 1.f;
};
__global__ __launch_bounds__(256) void k_colred_fin(int N, int Q, int has0, int chunks, const float* __restrict__ part,
                                                    ColOut o) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)N * Q) return;
    const int q = (int)(i / N), n = (int)(i % N);
    // the chunks in order, 16 loads issued at a time (one thread per output: a serial loop
    // waited for each load alone, ~17 us a launch)
    float s = 0.f;
    int c = 0;
    for (; c + 16 <= chunks; c += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = part[((int64_t)(c + u) * Q + q) * N + n];
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
    }
    for (; c < chunks; ++c) s += part[((int64_t)c * Q + q) * N + n];
    if (has0 && q == 0) {
        o.o0[n * o.s0] = o.alpha0 * s;
        if (o.o0b) o.o0b[n * o.s0] = o.beta0 * s;
    } else {
        const int j = q - has0;
        o.o1[j * o.q1 + n * o.s1] = o.alpha1 * s;
    }
}

// =======================================================================================
// NB kernels
// =======================================================================================
// per gene: sdv = softplus(ln_x_sd) + eps (nb.hh:408-410; vMF eps 1e-2 / D, vmf.hh:256), and
// softplus' derivative
__global__ __launch_bounds__(256) void k_w_gene(int D, const float* __restrict__ lsd, float eps, float* __restrict__ gv) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= D) return;
    const float u = lsd[g];
    const float sdv = softplus_acc(u) + eps;
    gv[g] = sdv;
    gv[D + g] = dsoftplus(u);
    gv[4 * D + g] = 1.f / sdv;  // the encoder input transform's scale (GemmX::isd)
}

// the normalised encoder input block of the exact-f32 handles (the bf16 / x3 GEMMs apply the
// same enc_in transform as they load the raw batch): nb.hh:408-410, vmf.hh:253-257
__global__ __launch_bounds__(256) void k_w_xn(int64_t n, int D, const float* __restrict__ X, GemmX x,
                                              float* __restrict__ Xn) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int g = (int)(i % D);
        Xn[i] = enc_in_acc(X[i], x.rs ? x.rs[i / D] : 1.f, x.xm[g], x.isd[g]);
    }
}

struct WLat {
    int B, K, R;
    const float *Mr, *Ar, *Ce;   // raw heads, covariate part (null: no covariate)
    float *Mn, *Z, *Ep;          // mean (with covariate), z, eps used
    const float *NMr, *NAr;      // NB nu heads (null for vMF)
    float *Zn, *En;
    const float* dpre;           // NB depth pre-activation [B] (null for vMF)
    float* dv;                   // NB depth d = softplus(dpre)
    float* kl;                   // [B] per-row KL: -0.5 sum (1 + lnvar - mean^2 - exp lnvar)
    const float* eps_in;         // injected noise (null: Philox)
    const StepScalars* ss;
    uint64_t seed;
    float* out_mean;             // encode mode: [B][K] outputs (mean without covariate, lnvar)
    float* out_lnvar;
};

// reparameterise + KL per row (nb.hh:412-416, 462-472, 533-537; vmf.hh:394-414)
__global__ __launch_bounds__(256) void k_w_latent(WLat a) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    const uint64_t step = (uint64_t)a.ss->step_id;
    const int64_t grow = a.ss->row_offset + b;
    float kl = 0.f;
    for (int k = threadIdx.x; k < a.K; k += 256) {
        const int64_t i = (int64_t)b * a.K + k;
        const float lnvar = fminf(fmaxf(a.Ar[i], -4.f), 4.f);
        if (a.out_mean) {
            a.out_mean[i] = a.Mr[i];
            a.out_lnvar[i] = lnvar;
            continue;
        }
        const float mn = a.Ce ? a.Mr[i] + a.Ce[i] : a.Mr[i];
        const float ep = a.eps_in ? a.eps_in[i] : philox_normal(a.seed, step, grow, k);
        a.Mn[i] = mn;
        a.Ep[i] = ep;
        a.Z[i] = mn + ep * expf(lnvar / 2.f);
        kl += 1.f + lnvar - mn * mn - expf(lnvar);
    }
    if (a.out_mean) return;
    if (a.NMr) {
        for (int k = threadIdx.x; k < a.R; k += 256) {
            const int64_t i = (int64_t)b * a.R + k;
            const float nm = a.NMr[i];
            const float nlv = fminf(fmaxf(a.NAr[i], -4.f), 4.f);
            const float en = a.eps_in ? a.eps_in[(int64_t)a.B * a.K + i] : philox_normal(a.seed, step, grow, NU_LANE + k);
            a.En[i] = en;
            a.Zn[i] = nm + en * expf(nlv / 2.f);
            kl += 1.f + nlv - nm * nm - expf(nlv);
        }
    }
    kl = wblock_sum(kl, red);
    if (threadIdx.x == 0) {
        a.kl[b] = -0.5f * kl;
        if (a.dpre) a.dv[b] = softplus_acc(a.dpre[b]);
    }
}

// latent backward per row: KL and reparameterisation gradients, the lnvar clamp mask (inclusive)
struct WLatB {
    int B, K, R;
    float beta_n, inv_n;
    const float *Mn, *Ar, *Ep, *dZ;
    float *dM, *dA;
    const float *NMr, *NAr, *En, *dZn;
    float *dNM, *dNA;
};
__global__ __launch_bounds__(256) void k_w_latent_bwd(WLatB a) {
    const int b = blockIdx.x;
    for (int k = threadIdx.x; k < a.K; k += 256) {
        const int64_t i = (int64_t)b * a.K + k;
        const float ar = a.Ar[i];
        const float lnvar = fminf(fmaxf(ar, -4.f), 4.f);
        const float sig = expf(lnvar / 2.f);
        const float dz = a.dZ[i];
        a.dM[i] = dz + a.beta_n * a.Mn[i];
        const float dl = dz * a.Ep[i] * 0.5f * sig - a.beta_n * 0.5f * (1.f - expf(lnvar));
        a.dA[i] = (ar >= -4.f && ar <= 4.f) ? dl : 0.f;
    }
    if (a.NMr) {
        for (int k = threadIdx.x; k < a.R; k += 256) {
            const int64_t i = (int64_t)b * a.R + k;
            const float ar = a.NAr[i];
            const float nlv = fminf(fmaxf(ar, -4.f), 4.f);
            const float dz = a.dZn[i];
            a.dNM[i] = dz + a.beta_n * a.NMr[i];
            const float dl = dz * a.En[i] * 0.5f * expf(nlv / 2.f) - a.beta_n * 0.5f * (1.f - expf(nlv));
            a.dNA[i] = (ar >= -4.f && ar <= 4.f) ? dl : 0.f;
        }
    }
}

// NB likelihood row (nb.hh:433-442, 453-460, 510-531) and its gradient, one workgroup per row,
// with the fused path's element arithmetic (nb_kernels.hip pass B: softplus_sig, nb_gamma_terms):
//   sweep 1: online max / sum-exp of the logits (every bias already added by the GEMM) -> lse;
//   sweep 2: p, mu' = p d + 1e-4, u = nu_dec(z_nu) - nu_bias (inline for R <= RMAX),
//            nu' = clamp(softplus(u)) + 1e-4, the NLL terms; G <- p dL/dmu' d,
//            U <- dL/du / n, row sums S = sum G, dd = sum p dL/dmu', dz_nu = sum U Wnd;
//   sweep 3: G <- (G - p S) / n  (the softmax backward: dL/dlogit).
struct WNbRow {
    int D, R;
    float inv_n;
    const float* LG;
    float *G, *U;
    const float* Uin;  // u when R > RMAX (else computed from Zn)
    const float* X;    // the dense batch (register-resident variant)
    // the row's nonzeros straight from the dataset CSR (cells[b]'s entries)
    const int64_t *cells, *rowptr;
    const int32_t* col;
    const float* val;
    const float *Zn, *Wnd, *bnd, *nu_bias;  // u inline (Zn non-null) or from U
    const float *dv, *dpre;
    float *lossr, *ddpre, *dZn;
    int with_grads;
};
// one (cell, gene) element of the NB row at x = 0 (every gene; the x-dependent terms of the
// nonzeros are added by nb_delta): loss term, G = p dL/dmu' d, dL/du / n (0 where the clamp
// bites), p dL/dmu'.  The dense part shares the fused path's arithmetic (nb_dense2's terms).
struct NbElem {
    float ll, gp, du, pg;
};
struct NbCore {
    float mu, nup, sv, rsv, lg2, sig;
    bool pass;  // the clamp passes the gradient
};
MMVAE_DEV NbCore nb_core(float p, float u, float d) {
    NbCore c;
    c.mu = fmaf(p, d, 1e-4f);
    const float sp = softplus_sig(u, c.sig);
    const float nu = clamp_nu(sp);
    c.pass = nu == sp;
    c.nup = nu + 1e-4f;
    c.sv = c.mu + c.nup;
    const float rr = frcp(c.nup * c.sv);
    c.rsv = c.nup * rr;                       // 1 / (mu + nu)
    c.lg2 = flog2(c.sv * (c.sv * rr));        // log2((mu + nu) / nu)
    return c;
}
MMVAE_DEV NbElem nb_elem(float p, float u, float d, float inv_n) {
    constexpr float LN2 = 0.6931471805599453f;
    const NbCore c = nb_core(p, u, d);
    const float gmu = c.nup * c.rsv;
    const float gnu = fmaf(c.lg2, LN2, fmaf(c.nup, c.rsv, -1.f));
    NbElem r;
    r.ll = c.nup * c.lg2 * LN2;                   // nb.hh:528
    r.du = c.pass ? gnu * c.sig * inv_n : 0.f;
    r.pg = gmu * p;
    r.gp = r.pg * d;
    return r;
}
// the x-dependent terms of a nonzero count x (nb.hh:522-527): added to the x = 0 element
MMVAE_DEV NbElem nb_delta(float p, float u, float d, float x, float inv_n, const float* ftab) {
    const NbCore c = nb_core(p, u, d);
    const float rmu = frcp(c.mu);
    float lgd, dgd;
    nb_gamma_terms<8>(c.nup, x, lgd, dgd, ftab);  // nb.hh:522-523
    const float dgmu = x * (c.rsv - rmu);          // x / s - x / mu
    const float dgnu = fmaf(x, c.rsv, dgd);
    NbElem r;
    r.ll = x * flog(c.sv * rmu) + lgd;             // nb.hh:527
    r.du = c.pass ? dgnu * c.sig * inv_n : 0.f;
    r.pg = dgmu * p;
    r.gp = r.pg * d;
    return r;
}

__global__ __launch_bounds__(256) void k_w_nb_row(WNbRow a) {
    __shared__ float red[4], red2[4], ftab[9];
    constexpr float L2E = 1.4426950408889634f;
    const int b = blockIdx.x;
    const int64_t o = (int64_t)b * a.D;
    const float* l = a.LG + o;
    if (threadIdx.x < 9) {
        float f = 1.f;
        for (int i = 2; i <= (int)threadIdx.x; ++i) f *= (float)i;
        ftab[threadIdx.x] = f;
    }
    // float4 sweeps when rows are 16-byte aligned (D % 4 == 0): thread t takes genes 4t + 1024 i
    const bool v4 = (a.D & 3) == 0;
    // sweep 1 (log2 units; -1e30: a thread without genes contributes nothing)
    float m = -1e30f, s = 0.f;
    if (v4) {
        for (int g = 4 * threadIdx.x; g < a.D; g += 1024) {
            const float4 v = *reinterpret_cast<const float4*>(l + g);
            const float v0 = v.x * L2E, v1 = v.y * L2E, v2 = v.z * L2E, v3 = v.w * L2E;
            const float mn = fmaxf(m, fmaxf(fmaxf(v0, v1), fmaxf(v2, v3)));
            s = s * fexp2(m - mn) + ((fexp2(v0 - mn) + fexp2(v1 - mn)) + (fexp2(v2 - mn) + fexp2(v3 - mn)));
            m = mn;
        }
    } else {
        for (int g = threadIdx.x; g < a.D; g += 256) {
            const float v = l[g] * L2E, mn = fmaxf(m, v);
            s = s * fexp2(m - mn) + fexp2(v - mn);
            m = mn;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
        const float mn = fmaxf(m, m2);
        s = s * fexp2(m - mn) + s2 * fexp2(m2 - mn);
        m = mn;
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = m;
        red2[threadIdx.x >> 6] = s;
    }
    __syncthreads();
    float M2 = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])), S2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) S2 += red2[i] * fexp2(red[i] - M2);
    const float lse2 = M2 + flog2(S2);
    __syncthreads();  // red reused below
    const float d = a.dv[b];
    float zn[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) zn[r] = (a.Zn && r < a.R) ? a.Zn[(int64_t)b * a.R + r] : 0.f;
    auto u_of = [&](int g) {
        if (!a.Zn) return a.Uin[o + g] - a.nu_bias[g];
        float u = a.bnd[g] - a.nu_bias[g];
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            if (r < a.R) u = fmaf(zn[r], a.Wnd[(int64_t)g * a.R + r], u);
        return u;
    };
    float lsum = 0.f, S = 0.f, dd = 0.f, dz[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) dz[r] = 0.f;
    auto take = [&](int g, const NbElem& q) {
        lsum += q.ll;
        S += q.gp;
        dd += q.pg;
        if (a.Zn)
#pragma unroll
            for (int r = 0; r < RMAX; ++r)
                if (r < a.R) dz[r] = fmaf(q.du, a.Wnd[(int64_t)g * a.R + r], dz[r]);
    };
    // sweep 2: every gene at x = 0 (no count-dependent branch: the nonzeros follow)
    if (v4) {
        for (int g = 4 * threadIdx.x; g < a.D; g += 1024) {
            const float4 lv = *reinterpret_cast<const float4*>(l + g);
            const float lgs[4] = {lv.x, lv.y, lv.z, lv.w};
            float gps[4], dus[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const NbElem q = nb_elem(fexp2(fmaf(lgs[j], L2E, -lse2)), u_of(g + j), d, a.inv_n);
                take(g + j, q);
                gps[j] = q.gp;
                dus[j] = q.du;
            }
            if (a.with_grads) {
                *reinterpret_cast<float4*>(a.U + o + g) = float4{dus[0], dus[1], dus[2], dus[3]};
                *reinterpret_cast<float4*>(a.G + o + g) = float4{gps[0], gps[1], gps[2], gps[3]};
            }
        }
    } else {
        for (int g = threadIdx.x; g < a.D; g += 256) {
            const NbElem q = nb_elem(fexp2(fmaf(l[g], L2E, -lse2)), u_of(g), d, a.inv_n);
            take(g, q);
            if (a.with_grads) {
                a.U[o + g] = q.du;
                a.G[o + g] = q.gp;
            }
        }
    }
    // the row's nonzeros (CSR, one gene at most once): their count-dependent terms, added onto
    // the x = 0 values just stored (the barrier orders the workgroup's stores before these
    // read-modify-writes)
    __syncthreads();
    {
        const int64_t cell = a.cells[b], e0 = a.rowptr[cell], e1 = a.rowptr[cell + 1];
        for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
            const int g = a.col[e];
            const float x = a.val[e];
            if (x == 0.f) continue;
            const NbElem q = nb_delta(fexp2(fmaf(l[g], L2E, -lse2)), u_of(g), d, x, a.inv_n, ftab);
            take(g, q);
            if (a.with_grads) {
                a.U[o + g] += q.du;
                a.G[o + g] += q.gp;
            }
        }
    }
    lsum = wblock_sum(lsum, red);
    if (threadIdx.x == 0) a.lossr[b] = lsum;
    if (!a.with_grads) return;
    S = wblock_sum(S, red);
    dd = wblock_sum(dd, red);
    if (threadIdx.x == 0) a.ddpre[b] = dd * a.inv_n * dsoftplus(a.dpre[b]);
    if (a.Zn)
        for (int r = 0; r < a.R && r < RMAX; ++r) {
            const float v = wblock_sum(dz[r], red);
            if (threadIdx.x == 0) a.dZn[(int64_t)b * a.R + r] = v;
        }
    // sweep 3: G <- (G - p S) / n
    if (v4) {
        for (int g = 4 * threadIdx.x; g < a.D; g += 1024) {
            const float4 lv = *reinterpret_cast<const float4*>(l + g);
            float4 gv = *reinterpret_cast<const float4*>(a.G + o + g);
            gv.x = a.inv_n * fmaf(-fexp2(fmaf(lv.x, L2E, -lse2)), S, gv.x);
            gv.y = a.inv_n * fmaf(-fexp2(fmaf(lv.y, L2E, -lse2)), S, gv.y);
            gv.z = a.inv_n * fmaf(-fexp2(fmaf(lv.z, L2E, -lse2)), S, gv.z);
            gv.w = a.inv_n * fmaf(-fexp2(fmaf(lv.w, L2E, -lse2)), S, gv.w);
            *reinterpret_cast<float4*>(a.G + o + g) = gv;
        }
    } else {
        for (int g = threadIdx.x; g < a.D; g += 256) {
            const float p = fexp2(fmaf(l[g], L2E, -lse2));
            a.G[o + g] = a.inv_n * fmaf(-p, S, a.G[o + g]);
        }
    }
}

// The LDS-resident variant for rows that fit (D % 4 == 0, 4 D bytes of LDS): 512 threads; the
// row's logits are read once into LDS and turned into p there, and the count-dependent terms
// come from the row's CSR entries after a branch-free x = 0 sweep of every gene — 5 passes over
// [B, D] (logits, U, G out, G back in and out) and no per-element divergence.
MMVAE_DEV float block_sum512(float v, float* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));
}
static constexpr int RCH = 5;  // float4 loads in flight per thread in the row sweeps
// GL: the row's G = p dL/dmu' d (+ the nonzeros' terms) is kept in LDS beside p (2 D floats, one
// workgroup per CU up to ~20k genes) instead of being stored, read back and stored again: the
// kernel is HBM-bound (≈ 2.4 GB a step at K = 128, D = 20k, B = 4096: logits in, U and G out,
// G in and out again, the sparse read-modify-writes), and G's round trip is 0.66 GB of it.
template <bool GL>
__global__ __launch_bounds__(512) void k_w_nb_row_lds(WNbRow a) {
    extern __shared__ __attribute__((aligned(16))) float prow[];  // [D] (GL: + [D] the row's G)
    float* grow = prow + a.D;  // (GL; D % 4 == 0 keeps it 16-byte aligned)
    __shared__ float red[8], red2[8], ftab[9];
    constexpr float L2E = 1.4426950408889634f;
    const int b = blockIdx.x;
    const int64_t o = (int64_t)b * a.D;
    if (threadIdx.x < 9) {
        float f = 1.f;
        for (int i = 2; i <= (int)threadIdx.x; ++i) f *= (float)i;
        ftab[threadIdx.x] = f;
    }
    // sweep 1: the logits into LDS (log2 units), online max / sum-exp.  Every sweep over the row
    // issues RCH float4 loads per thread before it uses any (one memory latency per RCH of them,
    // not one per float4)
    // (every batch's loads are issued unconditionally — clamped into the row, the spares unused —
    // and fenced from the math by a sched barrier: conditional or scheduler-sunk loads were
    // each waited for alone)
    float m = -1e30f, s = 0.f;
    for (int g0 = 4 * threadIdx.x; g0 < a.D; g0 += 2048 * RCH) {
        float4 vv[RCH];
#pragma unroll
        for (int j = 0; j < RCH; ++j) vv[j] = *reinterpret_cast<const float4*>(a.LG + o + min(g0 + 2048 * j, a.D - 4));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < RCH; ++j) {
            const int g = g0 + 2048 * j;
            if (g >= a.D) break;
            const float4 v = vv[j];
            const float v0 = v.x * L2E, v1 = v.y * L2E, v2 = v.z * L2E, v3 = v.w * L2E;
            *reinterpret_cast<float4*>(prow + g) = float4{v0, v1, v2, v3};
            const float mn = fmaxf(m, fmaxf(fmaxf(v0, v1), fmaxf(v2, v3)));
            s = s * fexp2(m - mn) + ((fexp2(v0 - mn) + fexp2(v1 - mn)) + (fexp2(v2 - mn) + fexp2(v3 - mn)));
            m = mn;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
        const float mn = fmaxf(m, m2);
        s = s * fexp2(m - mn) + s2 * fexp2(m2 - mn);
        m = mn;
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = m;
        red2[threadIdx.x >> 6] = s;
    }
    __syncthreads();
    float M2 = red[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) M2 = fmaxf(M2, red[i]);
    float S2 = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) S2 += red2[i] * fexp2(red[i] - M2);
    const float lse2 = M2 + flog2(S2);
    __syncthreads();  // red reused below
    const float d = a.dv[b];
    float zn[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) zn[r] = (a.Zn && r < a.R) ? a.Zn[(int64_t)b * a.R + r] : 0.f;
    float lsum = 0.f, S = 0.f, dd = 0.f, dz[RMAX];
#pragma unroll
    for (int r = 0; r < RMAX; ++r) dz[r] = 0.f;
    auto u_of = [&](int gg) {
        if (!a.Zn) return a.Uin[o + gg] - a.nu_bias[gg];
        float u = a.bnd[gg] - a.nu_bias[gg];
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            if (r < a.R) u = fmaf(zn[r], a.Wnd[(int64_t)gg * a.R + r], u);
        return u;
    };
    auto take = [&](int gg, const NbElem& q) {
        lsum += q.ll;
        S += q.gp;
        dd += q.pg;
        if (a.Zn)
#pragma unroll
            for (int r = 0; r < RMAX; ++r)
                if (r < a.R) dz[r] = fmaf(q.du, a.Wnd[(int64_t)gg * a.R + r], dz[r]);
    };
    // sweep 2: p (kept in LDS) and every gene's terms at x = 0 (branch free); U and G stored.
    // With one overdispersion latent (R = 1, u inline) the gene vectors u needs (bnd, nu_bias,
    // Wnd) are loaded RCH float4s at a time ahead of the math, as the logits are
    auto elem4 = [&](int g, float4 uv, float4 wv) {
        float4 lv = *reinterpret_cast<const float4*>(prow + g);
        float* pl = reinterpret_cast<float*>(&lv);
        const float* ul = reinterpret_cast<const float*>(&uv);
        const float* wl = reinterpret_cast<const float*>(&wv);
        float dus[4], gps[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float p = fexp2(pl[j] - lse2);
            pl[j] = p;
            const NbElem q = nb_elem(p, ul[j], d, a.inv_n);
            lsum += q.ll;
            S += q.gp;
            dd += q.pg;
            dz[0] = fmaf(q.du, wl[j], dz[0]);
            gps[j] = q.gp;
            dus[j] = q.du;
        }
        *reinterpret_cast<float4*>(prow + g) = lv;
        if (a.with_grads) {
            *reinterpret_cast<float4*>(a.U + o + g) = float4{dus[0], dus[1], dus[2], dus[3]};
            if (GL) *reinterpret_cast<float4*>(grow + g) = float4{gps[0], gps[1], gps[2], gps[3]};
            else *reinterpret_cast<float4*>(a.G + o + g) = float4{gps[0], gps[1], gps[2], gps[3]};
        }
    };
    if (a.Zn && a.R == 1) {
        for (int g0 = 4 * threadIdx.x; g0 < a.D; g0 += 2048 * RCH) {
            float4 bv[RCH], nv[RCH], wv[RCH];
#pragma unroll
            for (int j = 0; j < RCH; ++j) {
                const int g = min(g0 + 2048 * j, a.D - 4);  // (the registered gene vectors need not be 16-byte aligned)
                bv[j] = float4{a.bnd[g], a.bnd[g + 1], a.bnd[g + 2], a.bnd[g + 3]};
                nv[j] = float4{a.nu_bias[g], a.nu_bias[g + 1], a.nu_bias[g + 2], a.nu_bias[g + 3]};
                wv[j] = float4{a.Wnd[g], a.Wnd[g + 1], a.Wnd[g + 2], a.Wnd[g + 3]};
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < RCH; ++j) {
                const int g = g0 + 2048 * j;
                if (g >= a.D) break;
                const float4 uv = float4{fmaf(zn[0], wv[j].x, bv[j].x - nv[j].x), fmaf(zn[0], wv[j].y, bv[j].y - nv[j].y),
                                         fmaf(zn[0], wv[j].z, bv[j].z - nv[j].z), fmaf(zn[0], wv[j].w, bv[j].w - nv[j].w)};
                elem4(g, uv, wv[j]);
            }
        }
    } else {
    for (int g = 4 * threadIdx.x; g < a.D; g += 2048) {
        float4 lv = *reinterpret_cast<const float4*>(prow + g);
        float* pl = reinterpret_cast<float*>(&lv);
        float dus[4], gps[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float p = fexp2(pl[j] - lse2);
            pl[j] = p;
            const NbElem q = nb_elem(p, u_of(g + j), d, a.inv_n);
            take(g + j, q);
            gps[j] = q.gp;
            dus[j] = q.du;
        }
        *reinterpret_cast<float4*>(prow + g) = lv;
        if (a.with_grads) {
            *reinterpret_cast<float4*>(a.U + o + g) = float4{dus[0], dus[1], dus[2], dus[3]};
            if (GL) *reinterpret_cast<float4*>(grow + g) = float4{gps[0], gps[1], gps[2], gps[3]};
            else *reinterpret_cast<float4*>(a.G + o + g) = float4{gps[0], gps[1], gps[2], gps[3]};
        }
    }
    }
    // the row's nonzeros (CSR, each gene at most once): their count-dependent terms onto the
    // x = 0 values (the barrier orders the block's stores and LDS p before these reads), with
    // all of a thread's entries loaded before any is processed
    __syncthreads();
    {
        constexpr int NE = 4;
        const int64_t cell = a.cells[b], e0 = a.rowptr[cell], e1 = a.rowptr[cell + 1];
        for (int64_t eb = e0 + threadIdx.x; eb < e1; eb += 512 * NE) {
            int gs[NE];
            float xs[NE], gpo[NE], duo[NE];
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                const int64_t e = eb + 512 * k;
                gs[k] = e < e1 ? a.col[e] : 0;
                xs[k] = e < e1 ? a.val[e] : 0.f;
            }
            if (a.with_grads)
#pragma unroll
                for (int k = 0; k < NE; ++k) {
                    gpo[k] = xs[k] != 0.f ? (GL ? grow[gs[k]] : a.G[o + gs[k]]) : 0.f;
                    duo[k] = xs[k] != 0.f ? a.U[o + gs[k]] : 0.f;
                }
#pragma unroll
            for (int k = 0; k < NE; ++k) {
                if (xs[k] == 0.f) continue;
                const int gg = gs[k];
                const NbElem q = nb_delta(prow[gg], u_of(gg), d, xs[k], a.inv_n, ftab);
                take(gg, q);
                if (a.with_grads) {
                    if (GL) grow[gg] = gpo[k] + q.gp;
                    else a.G[o + gg] = gpo[k] + q.gp;
                    a.U[o + gg] = duo[k] + q.du;
                }
            }
        }
    }
    lsum = block_sum512(lsum, red);
    if (threadIdx.x == 0) a.lossr[b] = lsum;
    if (!a.with_grads) return;
    S = block_sum512(S, red);
    dd = block_sum512(dd, red);
    if (threadIdx.x == 0) a.ddpre[b] = dd * a.inv_n * dsoftplus(a.dpre[b]);
    if (a.Zn)
        for (int r = 0; r < a.R && r < RMAX; ++r) {
            const float v = block_sum512(dz[r], red);
            if (threadIdx.x == 0) a.dZn[(int64_t)b * a.R + r] = v;
        }
    // sweep 3: G = (G - p S) / n (each thread re-reads the G it stored: no barrier needed)
    for (int g0 = 4 * threadIdx.x; g0 < a.D; g0 += 2048 * RCH) {
        float4 gvv[RCH];
#pragma unroll
        for (int j = 0; j < RCH; ++j) {
            const int gj = min(g0 + 2048 * j, a.D - 4);
            gvv[j] = GL ? *reinterpret_cast<const float4*>(grow + gj) : *reinterpret_cast<const float4*>(a.G + o + gj);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < RCH; ++j) {
            const int g = g0 + 2048 * j;
            if (g >= a.D) break;
            const float4 pv = *reinterpret_cast<const float4*>(prow + g);
            float4 gv = gvv[j];
            gv.x = a.inv_n * fmaf(-pv.x, S, gv.x);
            gv.y = a.inv_n * fmaf(-pv.y, S, gv.y);
            gv.z = a.inv_n * fmaf(-pv.z, S, gv.z);
            gv.w = a.inv_n * fmaf(-pv.w, S, gv.w);
            *reinterpret_cast<float4*>(a.G + o + g) = gv;
        }
    }
}

// the ELBO scalar: (sum_b NLL_b [or the vMF llik terms] + beta sum_b KL_b) / n  (nb.hh:539-548)
__global__ __launch_bounds__(256) void k_w_loss(int B, const float* __restrict__ lossr, const float* __restrict__ kl,
                                                float beta, float inv_n, float extra, float* __restrict__ out) {
    __shared__ float red[4];
    float a = 0.f, k = 0.f;
    for (int b = threadIdx.x; b < B; b += 256) {
        a += lossr[b];
        k += kl[b];
    }
    a = wblock_sum(a, red);
    k = wblock_sum(k, red);
    if (threadIdx.x == 0) out[0] = (a + extra + beta * k) * inv_n;
}

// x_mean / ln_x_sd gradients from the column sums s1 = sum_b dXn, s2 = sum_b dXn Xn:
//   dxm = -s1 / sdv,  dlsd = -s2 / sdv * softplus'(ln_x_sd)   (nb.hh:408-410, vmf.hh:256-257)
__global__ __launch_bounds__(256) void k_w_xgrad(int D, const float* __restrict__ s12, const float* __restrict__ gv,
                                                 float* __restrict__ gxm, float* __restrict__ glsd) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= D) return;
    const float sdv = gv[g];
    gxm[g] = -s12[g] / sdv;
    glsd[g] = -s12[D + g] / sdv * gv[D + g];
}


// ReLU backward: dY[m][n] = 0 where the layer's (post-ReLU) output Y[m][n] is 0
__global__ __launch_bounds__(256) void k_w_relu_bwd(int64_t n, const float* __restrict__ Y, float* __restrict__ dY) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        if (!(Y[i] > 0.f)) dY[i] = 0.f;
}

// =======================================================================================
// vMF kernels (vmf.hh:250-304, 410-440; angular.hh:34-42)
// =======================================================================================
// Angular weights: W~ = normalize_rows(relu(W) + 1e-4)  (F::normalize eps 1e-12)
__global__ __launch_bounds__(256) void k_w_angular(int in, const float* __restrict__ W, float* __restrict__ Wt) {
    __shared__ float red[4];
    const int o = blockIdx.x;
    const float* w = W + (int64_t)o * in;
    float ss = 0.f;
    for (int i = threadIdx.x; i < in; i += 256) {
        const float v = fmaxf(w[i], 0.f) + 1e-4f;
        ss += v * v;
    }
    ss = wblock_sum(ss, red);
    const float nr = fmaxf(sqrtf(ss), 1e-12f);
    for (int i = threadIdx.x; i < in; i += 256) Wt[(int64_t)o * in + i] = (fmaxf(w[i], 0.f) + 1e-4f) / nr;
}

// vMF decoder row (vmf.hh:283-304, 419-440): h = exp(z_dec(z)) (the final Linear's output,
// exponentiated in place in LG), v = h + hc with hc = covar_decoding_(c) (inline for C <= CMAX,
// else read from U), r = normalize(v), y = normalize(log1p(relu(x)) + eps) from the raw batch and
// its row scale (k_w_densify2), cos_b = <y_b, r_b>; backward:
//   dr = -(kappa / n) y, dv = (dr - r <r, dr>) / |v|, U <- dv (covar_decoding_ grads),
//   G <- dv * h (the final Linear's output gradient)
struct WVRow {
    int D, C;
    float inv_n, epsD;
    float *LG, *U, *G;
    const float* X;
    const float* rs2;                    // 1 / |log1p(relu(x_b)) + eps|
    const float *Cb, *Wcd, *bcd;         // hc inline (Cb non-null) or from U
    const float* vk;  // kappa scalars (VK_KAPPA)
    float* cosr;
    int with_grads;
};
__global__ __launch_bounds__(256) void k_w_vmf_row(WVRow a) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    const int64_t o = (int64_t)b * a.D;
    float cb[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) cb[c] = (a.Cb && c < a.C) ? a.Cb[(int64_t)b * a.C + c] : 0.f;
    auto hc = [&](int g) {
        if (!a.Cb) return a.U[o + g];
        float v = a.bcd[g];
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
            if (c < a.C) v = fmaf(cb[c], a.Wcd[(int64_t)g * a.C + c], v);
        return v;
    };
    const float ry = a.rs2[b];
    auto yv = [&](int g) {
        const float x = a.X[o + g];
        return ((x > 0.f ? log1p_acc(x) : 0.f) + a.epsD) * ry;
    };
    float ss = 0.f, cr = 0.f;
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float h = fexp(a.LG[o + g]);
        a.LG[o + g] = h;
        const float v = h + hc(g);
        ss = fmaf(v, v, ss);
        cr = fmaf(yv(g), v, cr);
    }
    ss = wblock_sum(ss, red);
    cr = wblock_sum(cr, red);
    const float nv = sqrtf(ss), nr = fmaxf(nv, 1e-12f), inr = 1.f / nr;
    const float c = cr * inr;
    if (threadIdx.x == 0) a.cosr[b] = c;
    if (!a.with_grads) return;
    const float kn = a.vk[0] * a.inv_n;
    // <r, dr> = -(kappa / n) cos;  dv = (dr - r <r, dr>) / nr while nv > eps (else dr / eps)
    const float rdr = -kn * c;
    const bool big = nv > 1e-12f;
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float h = a.LG[o + g];
        const float r = (h + hc(g)) * inr;
        const float dr = -kn * yv(g);
        const float dv = (big ? fmaf(-r, rdr, dr) : dr) * inr;
        a.U[o + g] = dv;
        a.G[o + g] = dv * h;
    }
}

// vMF scalars (vmf.hh:301, operators.hh:13-101): kappa, T = df log kappa - lbessel, the Baricz
// bound — the fused path's vkappa_body restated (k_vprep)
struct WVScal {
    float df, kmin, kmax, lg_df1, c2;
    int rank0;
};
__global__ void k_w_vkappa(const float* __restrict__ lk_p, WVScal s, float* __restrict__ vk) {
    if (threadIdx.x != 0) return;
    const float lk = lk_p[0];
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
    const float x2 = kap * kap;
    const float lo = sqrtf(x2 * s.df / (s.df + 1.f) + s.df * s.df);
    const float up = sqrtf(x2 + s.df * s.df);
    vk[0] = kap;
    vk[1] = e;
    vk[2] = (e >= s.kmin && e <= s.kmax) ? 1.f : 0.f;
    vk[3] = s.df * lkap - lb;
    vk[4] = 0.5f * (lo + up) / kap;
}

// vMF loss and the ln_kappa gradient (vmf.hh:429-439; Q3 Baricz term on rank 0 only):
//   L = beta KL / n - (kappa sum_b cos_b + B (T - c2)) / n
__global__ __launch_bounds__(256) void k_w_vloss(int B, const float* __restrict__ cosr, const float* __restrict__ kl,
                                                 const float* __restrict__ vk, WVScal s, float beta, float inv_n,
                                                 float* __restrict__ out, float* __restrict__ glk, int with_grads) {
    __shared__ float red[4];
    float c = 0.f, k = 0.f;
    for (int b = threadIdx.x; b < B; b += 256) {
        c += cosr[b];
        k += kl[b];
    }
    c = wblock_sum(c, red);
    k = wblock_sum(k, red);
    if (threadIdx.x != 0) return;
    const float kap = vk[0];
    const float llik = fmaf(kap, c, (float)B * (vk[3] - s.c2));
    out[0] = k * beta * inv_n - llik * inv_n;
    if (with_grads) {
        float dk = -c * inv_n;
        dk += (s.df * -((float)B * inv_n)) / kap;
        if (s.rank0) dk += vk[4];
        glk[0] = (vk[2] > 0.f) ? dk * vk[1] : 0.f;
    }
}

// =======================================================================================
// Host side
// =======================================================================================
static int grid_for(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 8192); }

static void build_layers(Engine* e, WideState* w) {
    const bool vmf = e->cfg.model == MMVAE_MODEL_VMF;
    const bool relu = e->cfg.relu != 0;
    const int ne = e->cfg.n_enc_hidden, nd = e->cfg.n_dec_hidden;
    w->enc.clear();
    w->dec.clear();
    // encoder: the big first layer then the chain (nb.hh:331-349 / vmf.hh:338-355); NB ReLU only
    // without hidden layers (Q2 rejects --relu with them), vMF after every Angular layer
    if (ne == 0) {
        WLayer L;
        L.in = (int)e->D;
        L.out = (int)e->K;
        L.relu = relu;
        w->enc.push_back(L);
    }
    int prev = (int)e->D;
    for (int l = 0; l < ne; ++l) {
        WLayer L;
        L.in = prev;
        L.out = e->cfg.enc_hidden[l];
        L.relu = vmf && relu;
        w->enc.push_back(L);
        prev = L.out;
    }
    // decoder: hidden Linears (+ReLU with --relu), then the final Linear to D (no ReLU)
    prev = (int)e->K;
    for (int l = 0; l < nd; ++l) {
        WLayer L;
        L.in = prev;
        L.out = e->cfg.dec_hidden[l];
        L.relu = relu;
        w->dec.push_back(L);
        prev = L.out;
    }
    WLayer F;
    F.in = prev;
    F.out = (int)e->D;
    w->dec.push_back(F);
}

// frozen pointers of the layers (every frozen reload: the slots do not move, but the vMF
// Angular copies are recomputed)
static void bind_layers(Engine* e, WideState* w) {
    const bool vmf = e->cfg.model == MMVAE_MODEL_VMF;
    const int ne = e->cfg.n_enc_hidden, nd = e->cfg.n_dec_hidden;
    int64_t woff = 0;
    for (size_t l = 0; l < w->enc.size(); ++l) {
        std::string base;
        if (ne == 0) base = vmf ? "z_enc.0" : "mu_enc.mu_encoding";
        else base = (vmf ? "z_enc.encoding_" : "mu_enc.mu_encoding_") + std::to_string(l + 1);
        WLayer& L = w->enc[l];
        if (vmf) {
            L.W = w->wtil + woff;
            woff += (int64_t)L.in * L.out;
            L.b = nullptr;
        } else {
            L.W = e->pfrz(base + ".weight");
            L.b = e->pfrz(base + ".bias");
        }
    }
    for (size_t l = 0; l < w->dec.size(); ++l) {
        std::string base;
        if ((int)l < nd) base = (vmf ? "z_dec.decoding_" : "mu_dec.mu_decoding_") + std::to_string(l + 1);
        else base = vmf ? "z_dec.decoding" : "mu_dec.mu_decoding";
        w->dec[l].W = e->pfrz(base + ".weight");
        w->dec[l].b = e->pfrz(base + ".bias");
    }
}

hipError_t wide_create(Engine* e) {
    WideState* w = new WideState();
    e->wide_st = w;
    const int64_t Bp = e->Bpad, D = e->D, K = e->K, C = e->C, H = e->H, R = e->R;
    w->Bp = Bp;
    w->D = D;
    build_layers(e, w);
    hipError_t er;
#define WA(p, n) if ((er = walloc(&(p), (n))) != hipSuccess) return er
    WA(w->X, Bp * D);
    if (!at_in_gemm(e)) WA(w->Xn, Bp * D);
    if (e->cfg.model == MMVAE_MODEL_NB && R > RMAX) WA(w->Uin, Bp * D);
    WA(w->LG, Bp * D);
    WA(w->G, Bp * D);
    WA(w->U, Bp * D);
    WA(w->gvec, 5 * D);
    WA(w->colv, D);
    WA(w->one, 1);
    w->ws_cap = std::max<int64_t>(int64_t(8) << 20, 4 * D);
    WA(w->ws, w->ws_cap);
    w->cr_cap = 64 * CR_QMAX * ((D + 3) / 4 * 4);
    WA(w->cr_part, w->cr_cap);
    WA(w->Cb, Bp * C);
    WA(w->rowv, 8 * Bp);
    for (float** p : {&w->Mr, &w->Ar, &w->Ce, &w->Mn, &w->Z, &w->Ep, &w->dZ, &w->dM, &w->dA}) WA(*p, Bp * K);
    WA(w->Hn, Bp * H);
    WA(w->dHn, Bp * H);
    for (float** p : {&w->NMr, &w->NAr, &w->Zn, &w->En, &w->dZn, &w->dNM, &w->dNA}) WA(*p, Bp * R);
    int maxw = (int)K;
    int64_t wsum = 0;
    for (auto& L : w->enc) {
        WA(L.act, Bp * L.out);
        maxw = std::max(maxw, L.out);
        wsum += (int64_t)L.in * L.out;
    }
    for (size_t l = 0; l + 1 < w->dec.size(); ++l) {
        WA(w->dec[l].act, Bp * w->dec[l].out);
        maxw = std::max(maxw, w->dec[l].out);
    }
    w->maxw = maxw;
    WA(w->dT0, Bp * maxw);
    WA(w->dT1, Bp * maxw);
    if (e->cfg.model == MMVAE_MODEL_VMF) WA(w->wtil, wsum);
    WA(w->lossv, 8);
#undef WA
    const float one = 1.f;
    if ((er = hipMemcpy(w->one, &one, sizeof(float), hipMemcpyHostToDevice)) != hipSuccess) return er;
    if (mf_modes(e)) {  // the short-K GEMMs' weight planes (filled by wide_prepare_frozen)
        const int kf = w->dec.back().in, ke = w->enc[0].out;
        auto pl = [&](__bf16** p, int* kp, int k) -> hipError_t {
            if (k > 128 || k % 4 != 0) return hipSuccess;
            *kp = (k + 31) / 32 * 32;
            return hipMalloc(p, sizeof(__bf16) * 2 * (size_t)D * *kp);
        };
        if ((er = pl(&w->pl_F, &w->kp_F, kf)) != hipSuccess) return er;
        if ((er = pl(&w->pl_E, &w->kp_E, ke)) != hipSuccess) return er;
    }
    bind_layers(e, w);
    return hipSuccess;
}

void wide_destroy(Engine* e) {
    WideState* w = e->wide_st;
    if (!w) return;
    for (float* p : {w->X, w->Xn, w->Uin, w->LG, w->G, w->U, w->gvec, w->colv, w->one, w->ws, w->cr_part, w->Cb, w->rowv, w->Mr, w->Ar, w->Ce,
                     w->Mn, w->Z, w->Ep, w->dZ, w->dM, w->dA, w->Hn, w->dHn, w->NMr, w->NAr, w->Zn, w->En, w->dZn,
                     w->dNM, w->dNA, w->dT0, w->dT1, w->wtil, w->lossv})
        if (p) hipFree(p);
    for (auto& L : w->enc)
        if (L.act) hipFree(L.act);
    for (auto& L : w->dec)
        if (L.act) hipFree(L.act);
    if (w->pl_F) hipFree(w->pl_F);
    if (w->pl_E) hipFree(w->pl_E);
    delete w;
    e->wide_st = nullptr;
}

hipError_t wide_prepare_frozen(Engine* e) {
    WideState* w = e->wide_st;
    bind_layers(e, w);
    if (e->cfg.model == MMVAE_MODEL_VMF) {
        const int ne = e->cfg.n_enc_hidden;
        for (size_t l = 0; l < w->enc.size(); ++l) {
            const std::string base = ne == 0 ? std::string("z_enc.0") : "z_enc.encoding_" + std::to_string(l + 1);
            hipLaunchKernelGGL(k_w_angular, dim3(w->enc[l].out), dim3(256), 0, e->stream, w->enc[l].in,
                               (const float*)e->pfrz(base + ".weight"), const_cast<float*>(w->enc[l].W));
        }
    }
    const int D = (int)e->D;
    if (w->pl_F) {  // B(k, n) = W_F[n][k]
        const WLayer& F = w->dec.back();
        const int64_t n = (int64_t)D * w->kp_F;
        hipLaunchKernelGGL(k_w_planes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, F.W, (int64_t)1,
                           (int64_t)F.in, D, F.in, w->kp_F, w->pl_F, n);
    }
    if (w->pl_E) {  // B(k, n) = W0[k][n]
        const WLayer& L = w->enc[0];
        const int64_t n = (int64_t)D * w->kp_E;
        hipLaunchKernelGGL(k_w_planes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, L.W, (int64_t)L.in,
                           (int64_t)1, D, L.out, w->kp_E, w->pl_E, n);
    }
    e->frozen_dirty = false;
    ++e->graph_gen;
    return hipGetLastError();
}

wide_poison_t wide_poison_bufs(Engine* e) {
    wide_poison_t v;
    WideState* w = e->wide_st;
    if (!w) return v;
    const int64_t Bp = w->Bp, D = w->D, K = e->K, C = e->C, H = e->H, R = e->R;
    for (float* p : {w->X, w->Xn, w->Uin, w->LG, w->G, w->U})
        if (p) v.push_back({p, sizeof(float) * (size_t)(Bp * D)});
    v.push_back({w->gvec, sizeof(float) * (size_t)(5 * D)});
    v.push_back({w->ws, sizeof(float) * (size_t)w->ws_cap});
    v.push_back({w->cr_part, sizeof(float) * (size_t)w->cr_cap});
    v.push_back({w->Cb, sizeof(float) * (size_t)(Bp * C)});
    v.push_back({w->rowv, sizeof(float) * (size_t)(8 * Bp)});
    for (float* p : {w->Mr, w->Ar, w->Ce, w->Mn, w->Z, w->Ep, w->dZ, w->dM, w->dA})
        v.push_back({p, sizeof(float) * (size_t)(Bp * K)});
    for (float* p : {w->Hn, w->dHn}) v.push_back({p, sizeof(float) * (size_t)(Bp * H)});
    for (float* p : {w->NMr, w->NAr, w->Zn, w->En, w->dZn, w->dNM, w->dNA})
        v.push_back({p, sizeof(float) * (size_t)(Bp * R)});
    for (float* p : {w->dT0, w->dT1}) v.push_back({p, sizeof(float) * (size_t)(Bp * w->maxw)});
    for (auto& L : w->enc) v.push_back({L.act, sizeof(float) * (size_t)(Bp * L.out)});
    for (auto& L : w->dec)
        if (L.act) v.push_back({L.act, sizeof(float) * (size_t)(Bp * L.out)});
    v.push_back({w->lossv, sizeof(float) * 8});
    return v;
}

// staged block copy + densify (shared by step, eval and encode); the NB raw-count row dots and
// the vMF row scales ride along (k_w_densify2)
static hipError_t wide_input(Engine* e, int64_t B) {
    WideState* w = e->wide_st;
    const StageCopy sc = stage_copy_args(e);
    hipLaunchKernelGGL(k_w_stage, dim3((sc.n16 + 255) / 256), dim3(256), 0, e->stream, sc.src, sc.dst, sc.n16);
    {
        const hipError_t er = stream_gather(e);  // (streamed dataset: the batch's rows from host memory)
        if (er != hipSuccess) return er;
    }
    WDens a;
    std::memset(&a, 0, sizeof(a));
    a.D = (int)e->D;
    a.C = (int)e->C;
    a.H = (int)e->H;
    a.cells = e->d_cells;
    a.rowptr = e->d_rowptr;
    a.col = e->d_col;
    a.val = e->d_val;
    a.covar = e->d_covar;
    a.X = w->X;
    a.Cb = w->Cb;
    if (e->cfg.model == MMVAE_MODEL_VMF) {
        a.rs1 = w->rowv + 6 * w->Bp;
        a.rs2 = w->rowv + 7 * w->Bp;
        a.epsD = (float)(1e-2 / (double)(float)e->D);
    } else {
        a.dw = e->preg("depth.weight");
        a.db = e->preg("depth.bias");
        a.Wne = e->preg("nu_encoding.weight");
        a.bne = e->preg("nu_encoding.bias");
        a.dpre = w->rowv + 3 * w->Bp;
        a.Hn = w->Hn;
        if (e->H > HMAX) a.H = 0;  // (the wide nu encoder runs as a GEMM)
    }
    ScopedTimer tm(e, "w_densify");
    a.seg = getenv_is("MMVAE_WIDE_DENSSTORE", "1") ? 0 : 1;
    hipLaunchKernelGGL(k_w_densify2, dim3((unsigned)B), dim3(256), 0, e->stream, a);
    return hipGetLastError();
}

// the encoder input transform of this step (GemmX): x_mean, 1 / sdv, the vMF row scale
static GemmX enc_x(Engine* e) {
    WideState* w = e->wide_st;
    GemmX x;
    x.xm = e->preg("x_mean");
    x.isd = w->gvec + 4 * w->D;
    x.rs = e->cfg.model == MMVAE_MODEL_VMF ? w->rowv + 6 * w->Bp : nullptr;
    return x;
}

// the encoder chain from the raw batch X to the heads' input; returns it.  The first Linear
// takes enc_in(X) (nb.hh:408-410 / vmf.hh:253-257): on bf16 / x3 handles transformed inside the
// GEMM, on f32 handles from the materialised block Xn (the exact f32 GEMM)
static const float* enc_forward(Engine* e, int B, hipError_t& er) {
    WideState* w = e->wide_st;
    const GemmX gx = enc_x(e);
    const float* x = nullptr;
    int64_t ld = e->D;
    for (size_t l = 0; l < w->enc.size(); ++l) {
        WLayer& L = w->enc[l];
        GemmOp g;
        g.M = B; g.N = L.out; g.K = L.in;
        g.sam = ld; g.sak = 1;
        g.B = L.W; g.sbk = 1; g.sbn = L.in;
        g.C = L.act; g.scm = L.out; g.scn = 1;
        g.bias = L.b; g.act = L.relu ? 1 : 0;
        if (l == 0 && at_in_gemm(e)) {
            g.A = w->X;
            er = gemm(e, g, &gx);
        } else {
            if (l == 0) {
                const int64_t n = (int64_t)B * e->D;
                hipLaunchKernelGGL(k_w_xn, dim3(grid_for(n)), dim3(256), 0, e->stream, n, (int)e->D, (const float*)w->X,
                                   gx, w->Xn);
                x = w->Xn;
            }
            g.A = x;
            er = gemm(e, g);
        }
        if (er != hipSuccess) return nullptr;
        x = L.act;
        ld = L.out;
    }
    return x;
}

// column sums of Y [M][N] (row stride ly) into `o`: column 0 = a0 (null: ones) when has0, then
// the n1 columns of A1 (row stride la1), at most CR_QMAX per launch; X2: the XPROD pair
// (sum Y, sum Y enc_in(X2)) for the encoder's ln_x_sd gradient
static hipError_t colred_(Engine* e, int M, int N, const float* Y, int64_t ly, bool has0, const float* a0,
                         const float* A1, int64_t la1, int n1, ColOut o, const float* X2 = nullptr,
                         const GemmX* xf = nullptr) {
    WideState* w = e->wide_st;
    int done = 0;
    for (bool first = true; first || done < n1; first = false) {
        const int h0 = (first && has0) ? 1 : 0;
        const int nc = X2 ? 1 : std::min(n1 - done, CR_QMAX - h0);
        ColRed c;
        std::memset(&c, 0, sizeof(c));
        c.M = M;
        c.N = N;
        c.has0 = h0;
        c.Q = h0 + nc;
        c.a0 = a0;
        c.A1 = A1 ? A1 + done : nullptr;
        c.la1 = la1;
        c.Y = Y;
        c.ly = ly;
        c.X2 = X2;
        if (xf) c.xf = *xf;
        c.part = w->cr_part;
        const int64_t NQ = (int64_t)c.Q * ((N + 3) / 4 * 4);
        int chunks = (int)std::min<int64_t>(std::max(1, M / 64), w->cr_cap / NQ);
        chunks = std::max(1, std::min(chunks, 64));
        c.rows_per = (M + chunks - 1) / chunks;
        chunks = (M + c.rows_per - 1) / c.rows_per;
        const dim3 grid((unsigned)((N + 1023) / 1024), (unsigned)chunks);
        const bool f4 = N % 4 == 0 && ly % 4 == 0 && N >= 4 && (reinterpret_cast<uintptr_t>(Y) & 15) == 0 &&
                        (!X2 || (reinterpret_cast<uintptr_t>(X2) & 15) == 0);
        if (f4) {
            ColRed2 cc;
            cc.c[0] = c;
            if (X2) hipLaunchKernelGGL(k_colred<true>, grid, dim3(256), 0, e->stream, cc);
            else hipLaunchKernelGGL(k_colred<false>, grid, dim3(256), 0, e->stream, cc);
        } else {
            if (X2) hipLaunchKernelGGL(k_colred_gen<true>, grid, dim3(256), 0, e->stream, c);
            else hipLaunchKernelGGL(k_colred_gen<false>, grid, dim3(256), 0, e->stream, c);
        }
        ColOut oc = o;
        if (done) oc.o1 = o.o1 + done * o.q1;
        const int64_t nq = (int64_t)N * c.Q;
        hipLaunchKernelGGL(k_colred_fin, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, e->stream, N, c.Q, h0, chunks,
                           (const float*)w->cr_part, oc);
        done += nc;
        if (X2) break;
    }
    return hipGetLastError();
}
static hipError_t colred(Engine* e, int M, int N, const float* Y, int64_t ly, bool has0, const float* a0,
                         const float* A1, int64_t la1, int n1, ColOut o, const float* X2 = nullptr,
                         const GemmX* xf = nullptr) {
    ScopedTimer tm(e, "w_colred");
    return colred_(e, M, N, Y, ly, has0, a0, A1, la1, n1, o, X2, xf);
}
// two such sums (ones + A1 columns each, one launch each alone) over [M][N] blocks in one launch:
// the decoder's G and U sums, whose tails then overlap (falls back to two colred calls)
struct ColJob {
    const float* Y;
    const float* A1;
    int64_t la1;
    int n1;
    ColOut o;
};
static hipError_t colred_pair(Engine* e, int M, int N, const ColJob& j0, const ColJob& j1) {
    WideState* w = e->wide_st;
    const int64_t N4 = (N + 3) / 4 * 4;
    const int q0 = 1 + j0.n1, q1 = 1 + j1.n1;
    const int chunks = std::max(1, std::min(64, M / 64));
    auto al = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (q0 > CR_QMAX || q1 > CR_QMAX || N % 4 != 0 || N < 4 || !al(j0.Y) || !al(j1.Y) ||
        (int64_t)chunks * (q0 + q1) * N4 > w->cr_cap || getenv_is("MMVAE_WIDE_COLRED1", "1")) {
        hipError_t er = colred(e, M, N, j0.Y, N, true, nullptr, j0.A1, j0.la1, j0.n1, j0.o);
        if (er == hipSuccess) er = colred(e, M, N, j1.Y, N, true, nullptr, j1.A1, j1.la1, j1.n1, j1.o);
        return er;
    }
    ScopedTimer tm(e, "w_colred");
    ColRed2 cc;
    std::memset(&cc, 0, sizeof(cc));
    const int rows_per = (M + chunks - 1) / chunks;
    const ColJob* js[2] = {&j0, &j1};
    for (int z = 0; z < 2; ++z) {
        ColRed& c = cc.c[z];
        c.M = M;
        c.N = N;
        c.has0 = 1;
        c.Q = 1 + js[z]->n1;
        c.A1 = js[z]->A1;
        c.la1 = js[z]->la1;
        c.Y = js[z]->Y;
        c.ly = N;
        c.rows_per = rows_per;
        c.part = w->cr_part + (z ? (int64_t)chunks * q0 * N : 0);
    }
    const int ch = (M + rows_per - 1) / rows_per;
    hipLaunchKernelGGL(k_colred<false>, dim3((unsigned)((N + 1023) / 1024), (unsigned)ch, 2), dim3(256), 0, e->stream, cc);
    for (int z = 0; z < 2; ++z) {
        const int64_t nq = (int64_t)N * cc.c[z].Q;
        hipLaunchKernelGGL(k_colred_fin, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, e->stream, N, cc.c[z].Q, 1, ch,
                           (const float*)cc.c[z].part, js[z]->o);
    }
    return hipGetLastError();
}

// back through the encoder chain from dh [B][E] (in dT0) to the input gradient dXn [B][D] and
// its x_mean / ln_x_sd column sums (o: sum_b dXn, sum_b dXn Xn).  On the MFMA path the first
// layer's GEMM sums its output tiles itself (GemmOp::cpart) and dXn is never stored; otherwise
// dXn goes into G (the decoder's gradient block is consumed by then) and k_colred sums it.
static hipError_t enc_backward(Engine* e, int B, const ColOut& o) {
    WideState* w = e->wide_st;
    const int D = (int)e->D;
    float *cur = w->dT0, *nxt = w->dT1;
    for (int l = (int)w->enc.size() - 1; l >= 0; --l) {
        const WLayer& L = w->enc[l];
        hipError_t er;
        if (L.relu) {
            hipLaunchKernelGGL(k_w_relu_bwd, dim3(grid_for((int64_t)B * L.out)), dim3(256), 0, e->stream,
                               (int64_t)B * L.out, (const float*)L.act, cur);
        }
        if (l > 0) {
            if ((er = linear_dx(e, B, L.out, L.in, cur, L.out, L.W, nxt, L.in)) != hipSuccess) return er;
            std::swap(cur, nxt);
            continue;
        }
        const GemmX gx = enc_x(e);
        GemmOp g;  // dXn = dT . W0 (linear_dx's operands)
        g.M = B; g.N = L.in; g.K = L.out;
        g.A = cur; g.sam = L.out; g.sak = 1;
        g.B = L.W; g.sbk = L.in; g.sbn = 1;
        if (w->pl_E) {
            g.bpl = w->pl_E;
            g.bkp = w->kp_E;
            g.bplane = (int64_t)D * w->kp_E;
        }
        const int tm = (B + 63) / 64;  // the 64-row tiles = the partial chunks (both kernels)
        if (use_mf(e, g) && (int64_t)tm * 2 * D <= w->cr_cap && !getenv_is("MMVAE_WIDE_UNFUSED", "1")) {
            g.cpart = w->cr_part;
            g.cx = w->X;
            g.ldcx = D;
            g.cxf = gx;
            if ((er = gemm(e, g)) != hipSuccess) return er;
            ScopedTimer tm_(e, "w_colred");
            hipLaunchKernelGGL(k_colred_fin, dim3((unsigned)((2 * (int64_t)D + 255) / 256)), dim3(256), 0, e->stream, D, 2,
                               1, tm, (const float*)w->cr_part, o);
            return hipGetLastError();
        }
        g.C = w->G; g.scm = D; g.scn = 1;
        if ((er = gemm(e, g)) != hipSuccess) return er;
        return colred(e, B, D, w->G, D, true, nullptr, nullptr, 0, 1, o, w->X, &gx);
    }
    return hipGetLastError();
}

// decoder chain forward from z [B][K] to the last hidden output; returns the final layer's input
static const float* dec_hidden_fwd(Engine* e, int B, hipError_t& er) {
    WideState* w = e->wide_st;
    const float* x = w->Z;
    int64_t ld = e->K;
    for (size_t l = 0; l + 1 < w->dec.size(); ++l) {
        WLayer& L = w->dec[l];
        if ((er = linear_fwd(e, B, L.out, L.in, x, ld, L.W, L.b, L.act, L.out, L.relu ? 1 : 0)) != hipSuccess)
            return nullptr;
        x = L.act;
        ld = L.out;
    }
    return x;
}

// back through the decoder: from the final layer's output gradient G [B][D] to dz [B][K] (w->dZ)
static hipError_t dec_backward(Engine* e, int B) {
    WideState* w = e->wide_st;
    const int nl = (int)w->dec.size();
    const WLayer& F = w->dec[nl - 1];
    float* dst = (nl == 1) ? w->dZ : w->dT0;
    hipError_t er;
    if ((er = linear_dx(e, B, (int)e->D, F.in, w->G, e->D, F.W, dst, F.in)) != hipSuccess) return er;
    float *cur = w->dT0, *nxt = w->dT1;
    for (int l = nl - 2; l >= 0; --l) {
        const WLayer& L = w->dec[l];
        if (L.relu)
            hipLaunchKernelGGL(k_w_relu_bwd, dim3(grid_for((int64_t)B * L.out)), dim3(256), 0, e->stream,
                               (int64_t)B * L.out, (const float*)L.act, cur);
        float* d = (l == 0) ? w->dZ : nxt;
        if ((er = linear_dx(e, B, L.out, L.in, cur, L.out, L.W, d, L.in)) != hipSuccess) return er;
        std::swap(cur, nxt);
    }
    return hipGetLastError();
}

#define WCHK(x)                              \
    do {                                     \
        hipError_t er_ = (x);                \
        if (er_ != hipSuccess) return er_;   \
    } while (0)

// heads (nb.hh:412-416 / vmf.hh:258-263) from h [B][E]; names: mean, logvariance
static hipError_t heads_fwd(Engine* e, int B, const float* h, const std::string& wm, const std::string& wl, bool cov) {
    WideState* w = e->wide_st;
    const int K = (int)e->K, E = (int)w->enc.back().out;
    WCHK(linear_fwd(e, B, K, E, h, E, e->preg(wm + ".weight"), e->preg(wm + ".bias"), w->Mr, K));
    WCHK(linear_fwd(e, B, K, E, h, E, e->preg(wl + ".weight"), e->preg(wl + ".bias"), w->Ar, K));
    if (cov)
        WCHK(linear_fwd(e, B, K, (int)e->C, w->Cb, e->C, e->preg("covar_encoding.weight"),
                        e->preg("covar_encoding.bias"), w->Ce, K));
    return hipSuccess;
}

// heads backward: weight / bias / covariate gradients, then dh [B][E] into dT0
static hipError_t heads_bwd(Engine* e, int B, const float* h, const std::string& wm, const std::string& wl) {
    WideState* w = e->wide_st;
    const int K = (int)e->K, E = (int)w->enc.back().out, C = (int)e->C;
    WCHK(linear_dw(e, B, K, E, w->dM, K, h, E, e->greg(wm + ".weight")));
    WCHK(colsum(e, B, K, w->dM, K, e->greg(wm + ".bias")));
    WCHK(linear_dw(e, B, K, E, w->dA, K, h, E, e->greg(wl + ".weight")));
    WCHK(colsum(e, B, K, w->dA, K, e->greg(wl + ".bias")));
    WCHK(linear_dw(e, B, K, C, w->dM, K, w->Cb, C, e->greg("covar_encoding.weight")));
    WCHK(colsum(e, B, K, w->dM, K, e->greg("covar_encoding.bias")));
    WCHK(red_flush(e));  // (the group's sums in two launches)
    WCHK(linear_dx(e, B, K, E, w->dM, K, e->preg(wm + ".weight"), w->dT0, E));
    WCHK(linear_dx(e, B, K, E, w->dA, K, e->preg(wl + ".weight"), w->dT0, E, 1));
    return hipSuccess;
}

static hipError_t nb_step(Engine* e, int B, int64_t n_total, float beta, bool update, bool use_eps) {
    WideState* w = e->wide_st;
    const int D = (int)e->D, K = (int)e->K, H = (int)e->H, R = (int)e->R, C = (int)e->C;
    const float inv_n = 1.f / (float)n_total;
    float* r_loss = w->rowv;
    float* r_kl = w->rowv + w->Bp;
    float* r_d = w->rowv + 2 * w->Bp;
    float* r_dpre = w->rowv + 3 * w->Bp;
    float* r_ddpre = w->rowv + 4 * w->Bp;
    // the small Linears of the row side run inline (densify, the row kernel, the logit GEMM's
    // epilogue) up to the fused kernels' widths; wider ones as GEMMs
    const bool h_in = H <= HMAX, r_in = R <= RMAX, c_in = C <= CMAX;
    WCHK(wide_input(e, B));  // + depth(x), nu_enc(x) (h_in)
    hipLaunchKernelGGL(k_w_gene, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)e->preg("ln_x_sd"),
                       1e-4f, w->gvec);
    hipError_t er = hipSuccess;
    const float* h = enc_forward(e, B, er);
    WCHK(er);
    WCHK(heads_fwd(e, B, h, "mu_representation_mean", "mu_representation_logvariance", true));
    // overdispersion encoder on raw x (nb.hh:444-451)
    if (!h_in) WCHK(linear_fwd(e, B, H, D, w->X, D, e->preg("nu_encoding.weight"), e->preg("nu_encoding.bias"), w->Hn, H));
    WCHK(linear_fwd(e, B, R, H, w->Hn, H, e->preg("nu_representation_mean.weight"),
                    e->preg("nu_representation_mean.bias"), w->NMr, R));
    WCHK(linear_fwd(e, B, R, H, w->Hn, H, e->preg("nu_representation_logvariance.weight"),
                    e->preg("nu_representation_logvariance.bias"), w->NAr, R));
    WLat la;
    std::memset(&la, 0, sizeof(la));
    la.B = B; la.K = K; la.R = R;
    la.Mr = w->Mr; la.Ar = w->Ar; la.Ce = w->Ce;
    la.Mn = w->Mn; la.Z = w->Z; la.Ep = w->Ep;
    la.NMr = w->NMr; la.NAr = w->NAr; la.Zn = w->Zn; la.En = w->En;
    la.dpre = r_dpre; la.dv = r_d; la.kl = r_kl;
    la.eps_in = use_eps ? e->d_eps : nullptr;
    la.ss = e->d_ss;
    la.seed = e->cfg.seed;
    hipLaunchKernelGGL(k_w_latent, dim3(B), dim3(256), 0, e->stream, la);
    // logits = mu_dec(z) + covar_dec(c) + mu_bias (nb.hh:433-442) in one GEMM: the covariate
    // Linear and both biases in its epilogue
    const float* zd = dec_hidden_fwd(e, B, er);
    WCHK(er);
    const WLayer& F = w->dec.back();
    {
        GemmOp g;
        g.M = B; g.N = D; g.K = F.in;
        g.A = zd; g.sam = F.in; g.sak = 1;
        g.B = F.W; g.sbk = 1; g.sbn = F.in;
        g.C = w->LG; g.scm = D; g.scn = 1;
        g.bias = F.b;
        g.bias2 = e->preg("mu_bias");
        if (w->pl_F) {
            g.bpl = w->pl_F;
            g.bkp = w->kp_F;
            g.bplane = (int64_t)D * w->kp_F;
        }
        if (c_in) {
            g.ca = w->Cb; g.lca = C;
            g.cw = e->preg("covar_decoding.weight"); g.lcw = C;
            g.cbias = e->preg("covar_decoding.bias");
            g.nc = C;
        }
        WCHK(gemm(e, g));
    }
    if (!c_in)
        WCHK(linear_fwd(e, B, D, C, w->Cb, C, e->preg("covar_decoding.weight"), e->preg("covar_decoding.bias"), w->LG,
                        D, 0, 1));
    // u = nu_dec(z_nu) (nb.hh:458): inline in the row kernel, or a GEMM for R > RMAX
    if (!r_in) WCHK(linear_fwd(e, B, D, R, w->Zn, R, e->preg("nu_decoding.weight"), e->preg("nu_decoding.bias"), w->Uin, D));
    WNbRow rw;
    std::memset(&rw, 0, sizeof(rw));
    rw.D = D; rw.R = R; rw.inv_n = inv_n;
    rw.LG = w->LG; rw.G = w->G; rw.U = w->U; rw.Uin = w->Uin; rw.X = w->X;
    rw.cells = e->d_cells;
    rw.rowptr = e->d_rowptr;
    rw.col = e->d_col;
    rw.val = e->d_val;
    if (r_in) {
        rw.Zn = w->Zn;
        rw.Wnd = e->preg("nu_decoding.weight");
        rw.bnd = e->preg("nu_decoding.bias");
        rw.dZn = w->dZn;
    }
    rw.nu_bias = e->preg("nu_bias");
    rw.dv = r_d; rw.dpre = r_dpre; rw.lossr = r_loss; rw.ddpre = r_ddpre;
    rw.with_grads = update ? 1 : 0;
    {
        ScopedTimer tmr(e, "w_nb_row");
        if (D % 4 == 0 && (size_t)D * 8 <= 158 * 1024 && update && !getenv_is("MMVAE_WIDE_ROWG", "0"))
            // p and G in LDS (one workgroup per CU up to ~20k genes)
            hipLaunchKernelGGL(k_w_nb_row_lds<true>, dim3(B), dim3(512), (size_t)D * 8, e->stream, rw);
        else if (D % 4 == 0 && (size_t)D * 4 <= 150 * 1024)  // the row in LDS (2 workgroups per CU up to 20k genes)
            hipLaunchKernelGGL(k_w_nb_row_lds<false>, dim3(B), dim3(512), (size_t)D * 4, e->stream, rw);
        else
            hipLaunchKernelGGL(k_w_nb_row, dim3(B), dim3(256), 0, e->stream, rw);
    }
    hipLaunchKernelGGL(k_w_loss, dim3(1), dim3(256), 0, e->stream, B, (const float*)r_loss, (const float*)r_kl, beta,
                       inv_n, 0.f, e->d_out);
    if (!update) return hipGetLastError();
    // ---- backward ----
    // decoder-side gene vectors from the batch sums of dL/dlogit (G) and dL/du (U)
    {
        ColJob jg, ju;
        jg.Y = w->G;
        jg.A1 = w->Cb;
        jg.la1 = C;
        jg.n1 = C;
        jg.o.o0 = e->greg("mu_bias");
        jg.o.o0b = e->greg("covar_decoding.bias");
        jg.o.o1 = e->greg("covar_decoding.weight");
        jg.o.q1 = 1;
        jg.o.s1 = C;
        ju.Y = w->U;
        ju.A1 = w->Zn;
        ju.la1 = R;
        ju.n1 = R;
        ju.o.o0 = e->greg("nu_decoding.bias");
        ju.o.o0b = e->greg("nu_bias");
        ju.o.beta0 = -1.f;  // u = nu_dec(z_nu) - nu_bias
        ju.o.o1 = e->greg("nu_decoding.weight");
        ju.o.q1 = 1;
        ju.o.s1 = R;
        WCHK(colred_pair(e, B, D, jg, ju));
    }
    if (!r_in) WCHK(linear_dx(e, B, D, R, w->U, D, e->preg("nu_decoding.weight"), w->dZn, R));
    // decoder chain -> dz, then the latent
    WCHK(dec_backward(e, B));
    WLatB lb;
    lb.B = B; lb.K = K; lb.R = R;
    lb.beta_n = beta * inv_n; lb.inv_n = inv_n;
    lb.Mn = w->Mn; lb.Ar = w->Ar; lb.Ep = w->Ep; lb.dZ = w->dZ; lb.dM = w->dM; lb.dA = w->dA;
    lb.NMr = w->NMr; lb.NAr = w->NAr; lb.En = w->En; lb.dZn = w->dZn; lb.dNM = w->dNM; lb.dNA = w->dNA;
    hipLaunchKernelGGL(k_w_latent_bwd, dim3(B), dim3(256), 0, e->stream, lb);
    WCHK(heads_bwd(e, B, h, "mu_representation_mean", "mu_representation_logvariance"));
    // overdispersion encoder
    WCHK(linear_dw(e, B, R, H, w->dNM, R, w->Hn, H, e->greg("nu_representation_mean.weight")));
    WCHK(colsum(e, B, R, w->dNM, R, e->greg("nu_representation_mean.bias")));
    WCHK(linear_dw(e, B, R, H, w->dNA, R, w->Hn, H, e->greg("nu_representation_logvariance.weight")));
    WCHK(colsum(e, B, R, w->dNA, R, e->greg("nu_representation_logvariance.bias")));
    WCHK(linear_dx(e, B, R, H, w->dNM, R, e->preg("nu_representation_mean.weight"), w->dHn, H));
    WCHK(linear_dx(e, B, R, H, w->dNA, R, e->preg("nu_representation_logvariance.weight"), w->dHn, H, 1));
    // the raw-count Linears' weights from one pass over the batch: depth (nb.hh:400) and nu_enc
    {
        ColOut o;
        o.o0 = e->greg("depth.weight");
        o.o1 = e->greg("nu_encoding.weight");
        o.q1 = D;
        o.s1 = 1;
        WCHK(colred(e, B, D, w->X, D, true, r_ddpre, w->dHn, H, H, o));
    }
    WCHK(colsum(e, B, 1, r_ddpre, 1, e->greg("depth.bias")));
    WCHK(colsum(e, B, H, w->dHn, H, e->greg("nu_encoding.bias")));
    WCHK(red_flush(e));
    // encoder chain -> dXn and its column sums -> x_mean / ln_x_sd
    {
        ColOut o;
        o.o0 = w->gvec + 2 * D;
        o.o1 = w->gvec + 3 * D;
        WCHK(enc_backward(e, B, o));
    }
    hipLaunchKernelGGL(k_w_xgrad, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)(w->gvec + 2 * D),
                       (const float*)w->gvec, e->greg("x_mean"), e->greg("ln_x_sd"));
    return hipGetLastError();
}

static WVScal wvscal(Engine* e) {
    WVScal s;
    const int64_t D = e->D;
    s.df = (float)std::max(0.5 * (double)(float)D - 1., 0.);
    s.kmin = e->cfg.kappa_min;
    s.kmax = e->cfg.kappa_max;
    s.lg_df1 = mmvae_fasterlgamma((float)((double)s.df + 1));
    // fasterlog (fastlog.h:75-85) of 2 pi, as the fused path's host constant
    const float x = (float)(2. * M_PI);
    uint32_t i;
    std::memcpy(&i, &x, 4);
    volatile float y = (float)i;
    y = y * 8.2629582881927490e-8f;
    const float fl = y - 87.989971088f;
    s.c2 = (float)(0.5 * (double)(float)D * (double)fl);
    s.rank0 = e->rank == 0 ? 1 : 0;
    return s;
}

static hipError_t vmf_step(Engine* e, int B, int64_t n_total, float beta, bool update, bool use_eps) {
    WideState* w = e->wide_st;
    const int D = (int)e->D, K = (int)e->K, C = (int)e->C;
    const float inv_n = 1.f / (float)n_total;
    const float epsD = (float)(1e-2 / (double)(float)D);
    float* r_cos = w->rowv;
    float* r_kl = w->rowv + w->Bp;
    float* vk = w->rowv + 5 * w->Bp;
    const bool c_in = C <= CMAX;
    const WVScal sc = wvscal(e);
    WCHK(wide_input(e, B));  // + the row scales of log1p(x) and y
    hipLaunchKernelGGL(k_w_vkappa, dim3(1), dim3(64), 0, e->stream, (const float*)e->preg("ln_kappa"), sc, vk);
    hipLaunchKernelGGL(k_w_gene, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)e->preg("ln_x_sd"),
                       epsD, w->gvec);
    hipError_t er = hipSuccess;
    const float* h = enc_forward(e, B, er);
    WCHK(er);
    WCHK(heads_fwd(e, B, h, "representation_mean", "representation_logvariance", true));
    WLat la;
    std::memset(&la, 0, sizeof(la));
    la.B = B; la.K = K; la.R = 0;
    la.Mr = w->Mr; la.Ar = w->Ar; la.Ce = w->Ce;
    la.Mn = w->Mn; la.Z = w->Z; la.Ep = w->Ep;
    la.kl = r_kl;
    la.eps_in = use_eps ? e->d_eps : nullptr;
    la.ss = e->d_ss;
    la.seed = e->cfg.seed;
    hipLaunchKernelGGL(k_w_latent, dim3(B), dim3(256), 0, e->stream, la);
    const float* zd = dec_hidden_fwd(e, B, er);
    WCHK(er);
    const WLayer& F = w->dec.back();
    {  // linear_fwd's operands, with the frozen weight's planes for the short-K kernel
        GemmOp g;
        g.M = B; g.N = D; g.K = F.in;
        g.A = zd; g.sam = F.in; g.sak = 1;
        g.B = F.W; g.sbk = 1; g.sbn = F.in;
        g.C = w->LG; g.scm = D; g.scn = 1;
        g.bias = F.b;
        if (w->pl_F) {
            g.bpl = w->pl_F;
            g.bkp = w->kp_F;
            g.bplane = (int64_t)D * w->kp_F;
        }
        WCHK(gemm(e, g));
    }
    if (!c_in)
        WCHK(linear_fwd(e, B, D, C, w->Cb, C, e->preg("covar_decoding_.weight"), e->preg("covar_decoding_.bias"), w->U, D));
    WVRow rw;
    std::memset(&rw, 0, sizeof(rw));
    rw.D = D; rw.C = C; rw.inv_n = inv_n; rw.epsD = epsD;
    rw.LG = w->LG; rw.U = w->U; rw.G = w->G; rw.X = w->X; rw.rs2 = w->rowv + 7 * w->Bp;
    if (c_in) {
        rw.Cb = w->Cb;
        rw.Wcd = e->preg("covar_decoding_.weight");
        rw.bcd = e->preg("covar_decoding_.bias");
    }
    rw.vk = vk; rw.cosr = r_cos;
    rw.with_grads = update ? 1 : 0;
    {
        ScopedTimer tmr(e, "w_vmf_row");
        hipLaunchKernelGGL(k_w_vmf_row, dim3(B), dim3(256), 0, e->stream, rw);
    }
    hipLaunchKernelGGL(k_w_vloss, dim3(1), dim3(256), 0, e->stream, B, (const float*)r_cos, (const float*)r_kl,
                       (const float*)vk, sc, beta, inv_n, e->d_out, e->greg("ln_kappa"), update ? 1 : 0);
    if (!update) return hipGetLastError();
    {
        ColOut o;
        o.o0 = e->greg("covar_decoding_.bias");
        o.o1 = e->greg("covar_decoding_.weight");
        o.q1 = 1;
        o.s1 = C;
        WCHK(colred(e, B, D, w->U, D, true, nullptr, w->Cb, C, C, o));
    }
    WCHK(dec_backward(e, B));
    WLatB lb;
    std::memset(&lb, 0, sizeof(lb));
    lb.B = B; lb.K = K; lb.R = 0;
    lb.beta_n = beta * inv_n; lb.inv_n = inv_n;
    lb.Mn = w->Mn; lb.Ar = w->Ar; lb.Ep = w->Ep; lb.dZ = w->dZ; lb.dM = w->dM; lb.dA = w->dA;
    hipLaunchKernelGGL(k_w_latent_bwd, dim3(B), dim3(256), 0, e->stream, lb);
    WCHK(heads_bwd(e, B, h, "representation_mean", "representation_logvariance"));
    {
        ColOut o;
        o.o0 = w->gvec + 2 * D;
        o.o1 = w->gvec + 3 * D;
        WCHK(enc_backward(e, B, o));
    }
    hipLaunchKernelGGL(k_w_xgrad, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)(w->gvec + 2 * D),
                       (const float*)w->gvec, e->greg("x_mean"), e->greg("ln_x_sd"));
    return hipGetLastError();
}

hipError_t wide_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps) {
    // (per-kernel timers inside: w_gemm_gene, w_nb_row, w_colred, w_densify, ...; the rest of the
    // step's small kernels are untimed)
    if (e->cfg.model == MMVAE_MODEL_VMF) return vmf_step(e, (int)B, n_total, beta, update, use_eps);
    return nb_step(e, (int)B, n_total, beta, update, use_eps);
}

// recorder encode (nb.hh:419-431 / vmf.hh:267-281): mean and clamped lnvar, no covariate
hipError_t wide_encode(Engine* e, int64_t B, float* d_mean, float* d_lnvar) {
    WideState* w = e->wide_st;
    const int D = (int)e->D;
    const bool vmf = e->cfg.model == MMVAE_MODEL_VMF;
    WCHK(wide_input(e, B));
    const float epsD = (float)(1e-2 / (double)(float)D);
    hipLaunchKernelGGL(k_w_gene, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)e->preg("ln_x_sd"),
                       vmf ? epsD : 1e-4f, w->gvec);
    hipError_t er = hipSuccess;
    const float* h = enc_forward(e, (int)B, er);
    WCHK(er);
    if (vmf) WCHK(heads_fwd(e, (int)B, h, "representation_mean", "representation_logvariance", false));
    else WCHK(heads_fwd(e, (int)B, h, "mu_representation_mean", "mu_representation_logvariance", false));
    WLat la;
    std::memset(&la, 0, sizeof(la));
    la.B = (int)B; la.K = (int)e->K;
    la.Mr = w->Mr; la.Ar = w->Ar;
    la.ss = e->d_ss;
    la.out_mean = d_mean;
    la.out_lnvar = d_lnvar;
    hipLaunchKernelGGL(k_w_latent, dim3((unsigned)B), dim3(256), 0, e->stream, la);
    return hipGetLastError();
}

}  // namespace mmvae
