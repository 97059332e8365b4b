// The wide path: the ELBO step for model shapes beyond the fused tile kernels' limits — a latent
// (K / Z) or any hidden width above 64, more than 4 hidden layers, covariate / overdispersion
// widths C, H, R above 8, or D above the batch lists' LDS tile index (75,264 genes).  The
// reference builds any Linear chain and latent width (nb.hh:331-379, vmf.hh:338-385); this path
// makes every such model train on the GPU.
//
// Layout: the step's B cells are densified into HBM as a row-major [B, D] f32 block (the
// reference's own dense batch, mmvae_io.hh:208-245; 328 MB at B = 4096, D = 20k — HBM has room),
// and the step is the reference's op sequence (oracle/nb_oracle.py, oracle/vmf_oracle.py) on:
//   * one generic GEMM on the exact f32 MFMA (v_mfma_f32_16x16x4_f32, 64 x 64 tiles of four
//     waves, 16-deep k chunks staged through LDS, strided operands so every transpose of the
//     forward / backward is a stride swap), split-K into fixed-order partials when the tile grid
//     would not fill the 256 CUs — deterministic, like every reduction of the fused path;
//   * fused per-row kernels (softmax + NB likelihood + its gradient in three sweeps of a row;
//     the vMF row normalisations and their backward);
//   * per-gene kernels (the encoder's x_mean / ln_x_sd gradients from column sums).
// Column sums over the batch are GEMMs with a ones operand.  Every operand stays f32 (the dtype
// of the handle is ignored: this path is parity-grade in every mode).
#include <cmath>
#include <cstring>
#include <string>
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
struct GemmOp {
    int M = 0, N = 0, K = 0;
    const float* A = nullptr;
    int64_t sam = 0, sak = 0;
    const float* B = nullptr;
    int64_t sbk = 0, sbn = 0;
    float* C = nullptr;
    int64_t scm = 0, scn = 0;
    float alpha = 1.f;
    const float* bias = nullptr;  // [N]
    int act = 0;                  // 1: ReLU
    int accumulate = 0;           // C += result
};

static constexpr int GT = 64, GK = 16, GLD = GT + 4;

MMVAE_DEV void gemm_epilogue(const GemmOp& g, int m, int n, float acc) {
    float v = g.alpha * acc;
    if (g.bias) v += g.bias[n];
    if (g.act == 1) v = fmaxf(v, 0.f);
    float* c = g.C + (int64_t)m * g.scm + (int64_t)n * g.scn;
    *c = g.accumulate ? *c + v : v;
}

// grid (tiles over N, tiles over M, splits); split s covers k chunks [s * cps, (s + 1) * cps)
// and, with more than one split, stores its raw sums into ws[s][M][N] for k_gemm_reduce
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
        float s = 0.f;
        for (int q = 0; q < S; ++q) s += ws[q * MN + i];
        gemm_epilogue(g, (int)(i / g.N), (int)(i % g.N), s);
    }
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

struct WideState {
    int64_t Bp = 0, D = 0;
    // dense [Bpad][D] blocks
    float *X = nullptr, *Xn = nullptr, *LG = nullptr, *G = nullptr, *U = nullptr;
    // per-gene vectors: sdv, sigmoid(ln_x_sd), colsum scratch x2, (vMF) the eps-shifted y norm
    float *gvec = nullptr;
    float* one = nullptr;    // a device 1.0f (ones operand of the column-sum GEMMs)
    float* ws = nullptr;     // split-K partials
    int64_t ws_cap = 0;
    // covariates of the batch rows, per-row scalars
    float *Cb = nullptr, *rowv = nullptr;  // rowv: [8][Bpad]
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
};

static hipError_t walloc(float** p, int64_t n) { return hipMalloc(p, sizeof(float) * (size_t)(n > 0 ? n : 1)); }

static hipError_t gemm(Engine* e, const GemmOp& g) {
    if (g.M <= 0 || g.N <= 0) return hipSuccess;
    WideState* w = e->wide_st;
    const int tm = (g.M + GT - 1) / GT, tn = (g.N + GT - 1) / GT;
    const int nch = (g.K + GK - 1) / GK;
    int S = 1;
    const int tiles = tm * tn;
    if (tiles < 512 && nch >= 32) {
        S = std::min((512 + tiles - 1) / tiles, nch / 16);
        const int64_t cap = w->ws_cap / ((int64_t)g.M * g.N);
        if (S > cap) S = (int)cap;
        if (S < 2) S = 1;
    }
    const int cps = (nch + S - 1) / S;
    S = std::max(1, (nch + cps - 1) / cps);
    hipLaunchKernelGGL(k_gemm, dim3(tn, tm, S), dim3(256), 0, e->stream, g, cps, w->ws);
    if (S > 1) {
        const int64_t MN = (int64_t)g.M * g.N;
        const int nb = (int)std::min<int64_t>((MN + 255) / 256, 4096);
        hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, e->stream, g, S, (const float*)w->ws);
    }
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
    GemmOp g;
    g.M = N; g.N = K; g.K = M;
    g.A = dY; g.sam = 1; g.sak = ldy;
    g.B = X; g.sbk = ldx; g.sbn = 1;
    g.C = dW; g.scm = K; g.scn = 1;
    return gemm(e, g);
}
// out[n] = sign * sum_{m < M} Y[m][n]  (column sums, fixed order)
static hipError_t colsum(Engine* e, int M, int N, const float* Y, int64_t ldy, float* out, float sign = 1.f,
                         int accumulate = 0) {
    GemmOp g;
    g.M = 1; g.N = N; g.K = M;
    g.A = e->wide_st->one; g.sam = 0; g.sak = 0;
    g.B = Y; g.sbk = ldy; g.sbn = 1;
    g.C = out; g.scm = 0; g.scn = 1;
    g.alpha = sign; g.accumulate = accumulate;
    return gemm(e, g);
}

// =======================================================================================
// Batch densify, covariates, staged copy
// =======================================================================================
__global__ __launch_bounds__(256) void k_w_stage(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) dst[i] = src[i];
}

// one workgroup per batch row: zero the row, then scatter the cell's nonzeros (mmvae_io.hh:208-245)
__global__ __launch_bounds__(256) void k_w_densify(int D, int C, const int64_t* __restrict__ cells,
                                                   const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                   const float* __restrict__ val, const float* __restrict__ covar,
                                                   float* __restrict__ X, float* __restrict__ Cb) {
    const int b = blockIdx.x;
    const int64_t cell = cells[b];
    float* xr = X + (int64_t)b * D;
    for (int g = threadIdx.x; g < D; g += 256) xr[g] = 0.f;
    __syncthreads();
    const int64_t r0 = rowptr[cell], r1 = rowptr[cell + 1];
    for (int64_t i = r0 + threadIdx.x; i < r1; i += 256) xr[col[i]] = val[i];
    for (int c = threadIdx.x; c < C; c += 256) Cb[(int64_t)b * C + c] = covar[cell * C + c];
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

// digamma in double: recurrence up to 6, then the asymptotic series
MMVAE_DEV double digamma_d(double x) {
    double r = 0.0;
    while (x < 6.0) {
        r -= 1.0 / x;
        x += 1.0;
    }
    const double f = 1.0 / (x * x);
    return r + log(x) - 0.5 / x - f * (1.0 / 12 - f * (1.0 / 120 - f * (1.0 / 252 - f * (1.0 / 240 - f / 132))));
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
    gv[g] = softplus_acc(u) + eps;
    gv[D + g] = dsoftplus(u);
}

// NB encoder input: (log1p(x) - x_mean) / sdv (nb.hh:410)
__global__ __launch_bounds__(256) void k_w_xn_nb(int64_t n, int D, const float* __restrict__ X,
                                                 const float* __restrict__ xm, const float* __restrict__ gv,
                                                 float* __restrict__ Xn) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int g = (int)(i % D);
        Xn[i] = (log1pf(X[i]) - xm[g]) / gv[g];
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

// NB likelihood row (nb.hh:433-442, 453-460, 510-531) and its gradient, one workgroup per row:
//   sweep 1: l = logit + mu_bias (stored back), row max; sweep 2: sum exp -> lse;
//   sweep 3: p, mu' = p d + 1e-4, nu' = clamp(softplus(u - nu_bias)) + 1e-4, the NLL terms,
//            G = p dL/dp, U <- dL/du (x inv_n), row sums S = sum G, dd = sum p dL/dmu';
//   sweep 4: G <- inv_n (G - p S)  (the softmax backward: dL/dlogit)
struct WNbRow {
    int D;
    float inv_n;
    float *LG, *G, *U;
    const float *X, *mu_bias, *nu_bias, *dv, *dpre;
    float *lossr, *ddpre;
    int with_grads;
};
__global__ __launch_bounds__(256) void k_w_nb_row(WNbRow a) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    const int64_t o = (int64_t)b * a.D;
    float* l = a.LG + o;
    float mx = -INFINITY;
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float v = l[g] + a.mu_bias[g];
        l[g] = v;
        mx = fmaxf(mx, v);
    }
    mx = wblock_max(mx, red);
    float se = 0.f;
    for (int g = threadIdx.x; g < a.D; g += 256) se += expf(l[g] - mx);
    se = wblock_sum(se, red);
    const float lse = mx + logf(se);
    const float d = a.dv[b];
    float lsum = 0.f, S = 0.f, dd = 0.f;
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float p = expf(l[g] - lse);
        const float x = a.X[o + g];
        const float mu = p * d + 1e-4f;
        const float u = a.U[o + g] - a.nu_bias[g];
        const float sp = softplus_acc(u);
        const float nu = fminf(fmaxf(sp, 1e-4f), 1e4f);
        const float nup = nu + 1e-4f;
        const float s = mu + nup;
        const float ls = logf(s), lnu = logf(nup);
        float ll = nup * (ls - lnu);
        float dgd = 0.f;
        if (x != 0.f) {
            ll += lgammaf(nup) + lgammaf(x + 1.f) - lgammaf(nup + x) + x * (ls - logf(mu));
            dgd = (float)(digamma_d((double)nup) - digamma_d((double)nup + (double)x));
        }
        lsum += ll;
        if (a.with_grads) {
            const float gmu = x / s - x / mu + nup / s;
            const float gnu = dgd + (x + nup) / s + (ls - lnu) - 1.f;
            const float msk = (sp >= 1e-4f && sp <= 1e4f) ? 1.f : 0.f;
            a.U[o + g] = gnu * dsoftplus(u) * msk * a.inv_n;
            const float gp = p * gmu * d;
            a.G[o + g] = gp;
            S += gp;
            dd += gmu * p;
        }
    }
    lsum = wblock_sum(lsum, red);
    if (threadIdx.x == 0) a.lossr[b] = lsum;
    if (!a.with_grads) return;
    S = wblock_sum(S, red);
    dd = wblock_sum(dd, red);
    if (threadIdx.x == 0) a.ddpre[b] = dd * a.inv_n * dsoftplus(a.dpre[b]);
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float p = expf(l[g] - lse);
        a.G[o + g] = a.inv_n * (a.G[o + g] - p * S);
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

__global__ __launch_bounds__(256) void k_w_mul(int64_t n, const float* __restrict__ a, float* __restrict__ b) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] *= a[i];
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

// vMF encoder input per row: xn = normalize(log1p(x)); x~ = (xn - x_mean) / sdv  (vmf.hh:255-257)
// and the observed direction y = normalize(log1p(relu(x)) + eps) kept in X (vmf.hh:421-422)
__global__ __launch_bounds__(256) void k_w_xn_vmf(int D, float epsD, float* __restrict__ X, const float* __restrict__ xm,
                                                  const float* __restrict__ gv, float* __restrict__ Xn) {
    __shared__ float red[4];
    const int64_t o = (int64_t)blockIdx.x * D;
    float s1 = 0.f, s2 = 0.f;
    for (int g = threadIdx.x; g < D; g += 256) {
        const float x = X[o + g];
        const float lx = log1pf(x), ly = log1pf(fmaxf(x, 0.f)) + epsD;
        s1 += lx * lx;
        s2 += ly * ly;
    }
    s1 = wblock_sum(s1, red);
    s2 = wblock_sum(s2, red);
    const float n1 = fmaxf(sqrtf(s1), 1e-12f), n2 = fmaxf(sqrtf(s2), 1e-12f);
    for (int g = threadIdx.x; g < D; g += 256) {
        const float x = X[o + g];
        Xn[o + g] = (log1pf(x) / n1 - xm[g]) / gv[g];
        X[o + g] = (log1pf(fmaxf(x, 0.f)) + epsD) / n2;
    }
}

// vMF decoder row: LG = exp(z_dec(z)) (the final Linear's output, exponentiated in place) + hc
// (U holds c Wcd^T + bcd); r = normalize(v); cos_b = <y_b, r_b>; backward
//   dr = -(kappa / n) y, dv = (dr - r <r, dr>) / |v|, U <- dv (covar_decoding_ grads),
//   G <- dv * exp(.) (the final Linear's output gradient)
struct WVRow {
    int D;
    float inv_n;
    float *LG, *U, *G;
    const float* Y;
    const float* vk;  // kappa scalars (VK_KAPPA)
    float* cosr;
    int with_grads;
};
__global__ __launch_bounds__(256) void k_w_vmf_row(WVRow a) {
    __shared__ float red[4];
    const int64_t o = (int64_t)blockIdx.x * a.D;
    float ss = 0.f;
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float h = expf(a.LG[o + g]);
        a.LG[o + g] = h;
        const float v = h + a.U[o + g];
        ss += v * v;
    }
    ss = wblock_sum(ss, red);
    const float nv = sqrtf(ss), nr = fmaxf(nv, 1e-12f);
    float c = 0.f;
    for (int g = threadIdx.x; g < a.D; g += 256) c += a.Y[o + g] * ((a.LG[o + g] + a.U[o + g]) / nr);
    c = wblock_sum(c, red);
    if (threadIdx.x == 0) a.cosr[blockIdx.x] = c;
    if (!a.with_grads) return;
    const float kn = a.vk[0] * a.inv_n;
    // <r, dr> = -(kappa / n) cos;  dv = (dr - r <r, dr>) / nr while nv > eps (else dr / eps)
    const float rdr = -kn * c;
    const bool big = nv > 1e-12f;
    for (int g = threadIdx.x; g < a.D; g += 256) {
        const float h = a.LG[o + g];
        const float r = (h + a.U[o + g]) / nr;
        const float dr = -kn * a.Y[o + g];
        const float dv = big ? (dr - r * rdr) / nr : dr / nr;
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
    WA(w->Xn, Bp * D);
    WA(w->LG, Bp * D);
    WA(w->G, Bp * D);
    WA(w->U, Bp * D);
    WA(w->gvec, 4 * D);
    WA(w->one, 1);
    w->ws_cap = std::max<int64_t>(int64_t(8) << 20, 4 * D);
    WA(w->ws, w->ws_cap);
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
    bind_layers(e, w);
    return hipSuccess;
}

void wide_destroy(Engine* e) {
    WideState* w = e->wide_st;
    if (!w) return;
    for (float* p : {w->X, w->Xn, w->LG, w->G, w->U, w->gvec, w->one, w->ws, w->Cb, w->rowv, w->Mr, w->Ar, w->Ce,
                     w->Mn, w->Z, w->Ep, w->dZ, w->dM, w->dA, w->Hn, w->dHn, w->NMr, w->NAr, w->Zn, w->En, w->dZn,
                     w->dNM, w->dNA, w->dT0, w->dT1, w->wtil, w->lossv})
        if (p) hipFree(p);
    for (auto& L : w->enc)
        if (L.act) hipFree(L.act);
    for (auto& L : w->dec)
        if (L.act) hipFree(L.act);
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
    e->frozen_dirty = false;
    ++e->graph_gen;
    return hipGetLastError();
}

wide_poison_t wide_poison_bufs(Engine* e) {
    wide_poison_t v;
    WideState* w = e->wide_st;
    if (!w) return v;
    const int64_t Bp = w->Bp, D = w->D, K = e->K, C = e->C, H = e->H, R = e->R;
    for (float* p : {w->X, w->Xn, w->LG, w->G, w->U}) v.push_back({p, sizeof(float) * (size_t)(Bp * D)});
    v.push_back({w->gvec, sizeof(float) * (size_t)(4 * D)});
    v.push_back({w->ws, sizeof(float) * (size_t)w->ws_cap});
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

// staged block copy + densify (shared by step, eval and encode)
static hipError_t wide_input(Engine* e, int64_t B) {
    WideState* w = e->wide_st;
    const StageCopy sc = stage_copy_args(e);
    hipLaunchKernelGGL(k_w_stage, dim3((sc.n16 + 255) / 256), dim3(256), 0, e->stream, sc.src, sc.dst, sc.n16);
    hipLaunchKernelGGL(k_w_densify, dim3((unsigned)B), dim3(256), 0, e->stream, (int)e->D, (int)e->C,
                       (const int64_t*)e->d_cells, (const int64_t*)e->d_rowptr, (const int32_t*)e->d_col,
                       (const float*)e->d_val, (const float*)e->d_covar, w->X, w->Cb);
    return hipGetLastError();
}

// the encoder chain from its input block (Xn, [B][D]) to the heads' input; returns it
static const float* enc_forward(Engine* e, int B, const float* in, hipError_t& er) {
    WideState* w = e->wide_st;
    const float* x = in;
    int64_t ld = e->D;
    for (auto& L : w->enc) {
        if ((er = linear_fwd(e, B, L.out, L.in, x, ld, L.W, L.b, L.act, L.out, L.relu ? 1 : 0)) != hipSuccess)
            return nullptr;
        x = L.act;
        ld = L.out;
    }
    return x;
}

// back through the encoder chain from dh [B][E] (in dT0) to dXn [B][D] (into out)
static hipError_t enc_backward(Engine* e, int B, float* out) {
    WideState* w = e->wide_st;
    float *cur = w->dT0, *nxt = w->dT1;
    for (int l = (int)w->enc.size() - 1; l >= 0; --l) {
        const WLayer& L = w->enc[l];
        hipError_t er;
        if (L.relu) {
            hipLaunchKernelGGL(k_w_relu_bwd, dim3(grid_for((int64_t)B * L.out)), dim3(256), 0, e->stream,
                               (int64_t)B * L.out, (const float*)L.act, cur);
        }
        float* dst = (l == 0) ? out : nxt;
        if ((er = linear_dx(e, B, L.out, L.in, cur, L.out, L.W, dst, L.in)) != hipSuccess) return er;
        std::swap(cur, nxt);
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
    WCHK(wide_input(e, B));
    hipLaunchKernelGGL(k_w_gene, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)e->preg("ln_x_sd"),
                       1e-4f, w->gvec);
    const int64_t nBD = (int64_t)B * D;
    hipLaunchKernelGGL(k_w_xn_nb, dim3(grid_for(nBD)), dim3(256), 0, e->stream, nBD, D, (const float*)w->X,
                       (const float*)e->preg("x_mean"), (const float*)w->gvec, w->Xn);
    hipError_t er = hipSuccess;
    const float* h = enc_forward(e, B, w->Xn, er);
    WCHK(er);
    WCHK(heads_fwd(e, B, h, "mu_representation_mean", "mu_representation_logvariance", true));
    // overdispersion encoder on raw x (nb.hh:444-451), depth (nb.hh:400, 498)
    WCHK(linear_fwd(e, B, H, D, w->X, D, e->preg("nu_encoding.weight"), e->preg("nu_encoding.bias"), w->Hn, H));
    WCHK(linear_fwd(e, B, R, H, w->Hn, H, e->preg("nu_representation_mean.weight"),
                    e->preg("nu_representation_mean.bias"), w->NMr, R));
    WCHK(linear_fwd(e, B, R, H, w->Hn, H, e->preg("nu_representation_logvariance.weight"),
                    e->preg("nu_representation_logvariance.bias"), w->NAr, R));
    WCHK(linear_fwd(e, B, 1, D, w->X, D, e->preg("depth.weight"), e->preg("depth.bias"), r_dpre, 1));
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
    // decoders: logits = mu_dec(z) + covar_dec(c) (+ mu_bias in the row kernel), u = nu_dec(z_nu)
    const float* zd = dec_hidden_fwd(e, B, er);
    WCHK(er);
    const WLayer& F = w->dec.back();
    WCHK(linear_fwd(e, B, D, F.in, zd, F.in, F.W, F.b, w->LG, D));
    WCHK(linear_fwd(e, B, D, C, w->Cb, C, e->preg("covar_decoding.weight"), e->preg("covar_decoding.bias"), w->LG,
                    D, 0, 1));
    WCHK(linear_fwd(e, B, D, R, w->Zn, R, e->preg("nu_decoding.weight"), e->preg("nu_decoding.bias"), w->U, D));
    WNbRow rw;
    rw.D = D; rw.inv_n = inv_n;
    rw.LG = w->LG; rw.G = w->G; rw.U = w->U;
    rw.X = w->X; rw.mu_bias = e->preg("mu_bias"); rw.nu_bias = e->preg("nu_bias");
    rw.dv = r_d; rw.dpre = r_dpre; rw.lossr = r_loss; rw.ddpre = r_ddpre;
    rw.with_grads = update ? 1 : 0;
    hipLaunchKernelGGL(k_w_nb_row, dim3(B), dim3(256), 0, e->stream, rw);
    hipLaunchKernelGGL(k_w_loss, dim3(1), dim3(256), 0, e->stream, B, (const float*)r_loss, (const float*)r_kl, beta,
                       inv_n, 0.f, e->d_out);
    if (!update) return hipGetLastError();
    // ---- backward ----
    // decoder side gene vectors: mu_bias, covar_decoding.*, nu_bias, nu_decoding.*
    WCHK(colsum(e, B, D, w->G, D, e->greg("mu_bias")));
    WCHK(colsum(e, B, D, w->G, D, e->greg("covar_decoding.bias")));
    WCHK(linear_dw(e, B, D, C, w->G, D, w->Cb, C, e->greg("covar_decoding.weight")));
    WCHK(colsum(e, B, D, w->U, D, e->greg("nu_bias"), -1.f));
    WCHK(colsum(e, B, D, w->U, D, e->greg("nu_decoding.bias")));
    WCHK(linear_dw(e, B, D, R, w->U, D, w->Zn, R, e->greg("nu_decoding.weight")));
    WCHK(linear_dx(e, B, D, R, w->U, D, e->preg("nu_decoding.weight"), w->dZn, R));
    // depth
    WCHK(linear_dw(e, B, 1, D, r_ddpre, 1, w->X, D, e->greg("depth.weight")));
    WCHK(colsum(e, B, 1, r_ddpre, 1, e->greg("depth.bias")));
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
    WCHK(linear_dw(e, B, H, D, w->dHn, H, w->X, D, e->greg("nu_encoding.weight")));
    WCHK(colsum(e, B, H, w->dHn, H, e->greg("nu_encoding.bias")));
    // encoder chain -> dXn (into G: the decoder's gradient block is consumed), x_mean / ln_x_sd
    WCHK(enc_backward(e, B, w->G));
    WCHK(colsum(e, B, D, w->G, D, w->gvec + 2 * D));
    hipLaunchKernelGGL(k_w_mul, dim3(grid_for(nBD)), dim3(256), 0, e->stream, nBD, (const float*)w->Xn, w->G);
    WCHK(colsum(e, B, D, w->G, D, w->gvec + 3 * D));
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
    const WVScal sc = wvscal(e);
    WCHK(wide_input(e, B));
    hipLaunchKernelGGL(k_w_vkappa, dim3(1), dim3(64), 0, e->stream, (const float*)e->preg("ln_kappa"), sc, vk);
    hipLaunchKernelGGL(k_w_gene, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)e->preg("ln_x_sd"),
                       epsD, w->gvec);
    hipLaunchKernelGGL(k_w_xn_vmf, dim3(B), dim3(256), 0, e->stream, D, epsD, w->X, (const float*)e->preg("x_mean"),
                       (const float*)w->gvec, w->Xn);
    hipError_t er = hipSuccess;
    const float* h = enc_forward(e, B, w->Xn, er);
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
    WCHK(linear_fwd(e, B, D, F.in, zd, F.in, F.W, F.b, w->LG, D));
    WCHK(linear_fwd(e, B, D, C, w->Cb, C, e->preg("covar_decoding_.weight"), e->preg("covar_decoding_.bias"), w->U, D));
    WVRow rw;
    rw.D = D; rw.inv_n = inv_n;
    rw.LG = w->LG; rw.U = w->U; rw.G = w->G; rw.Y = w->X; rw.vk = vk; rw.cosr = r_cos;
    rw.with_grads = update ? 1 : 0;
    hipLaunchKernelGGL(k_w_vmf_row, dim3(B), dim3(256), 0, e->stream, rw);
    hipLaunchKernelGGL(k_w_vloss, dim3(1), dim3(256), 0, e->stream, B, (const float*)r_cos, (const float*)r_kl,
                       (const float*)vk, sc, beta, inv_n, e->d_out, e->greg("ln_kappa"), update ? 1 : 0);
    if (!update) return hipGetLastError();
    WCHK(colsum(e, B, D, w->U, D, e->greg("covar_decoding_.bias")));
    WCHK(linear_dw(e, B, D, C, w->U, D, w->Cb, C, e->greg("covar_decoding_.weight")));
    WCHK(dec_backward(e, B));
    WLatB lb;
    std::memset(&lb, 0, sizeof(lb));
    lb.B = B; lb.K = K; lb.R = 0;
    lb.beta_n = beta * inv_n; lb.inv_n = inv_n;
    lb.Mn = w->Mn; lb.Ar = w->Ar; lb.Ep = w->Ep; lb.dZ = w->dZ; lb.dM = w->dM; lb.dA = w->dA;
    hipLaunchKernelGGL(k_w_latent_bwd, dim3(B), dim3(256), 0, e->stream, lb);
    WCHK(heads_bwd(e, B, h, "representation_mean", "representation_logvariance"));
    WCHK(enc_backward(e, B, w->G));
    const int64_t nBD = (int64_t)B * D;
    WCHK(colsum(e, B, D, w->G, D, w->gvec + 2 * D));
    hipLaunchKernelGGL(k_w_mul, dim3(grid_for(nBD)), dim3(256), 0, e->stream, nBD, (const float*)w->Xn, w->G);
    WCHK(colsum(e, B, D, w->G, D, w->gvec + 3 * D));
    hipLaunchKernelGGL(k_w_xgrad, dim3((D + 255) / 256), dim3(256), 0, e->stream, D, (const float*)(w->gvec + 2 * D),
                       (const float*)w->gvec, e->greg("x_mean"), e->greg("ln_x_sd"));
    return hipGetLastError();
}

hipError_t wide_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps) {
    ScopedTimer tm(e, "wide_step");
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
    if (vmf)
        hipLaunchKernelGGL(k_w_xn_vmf, dim3((unsigned)B), dim3(256), 0, e->stream, D, epsD, w->X,
                           (const float*)e->preg("x_mean"), (const float*)w->gvec, w->Xn);
    else
        hipLaunchKernelGGL(k_w_xn_nb, dim3(grid_for(B * D)), dim3(256), 0, e->stream, (int64_t)B * D, D,
                           (const float*)w->X, (const float*)e->preg("x_mean"), (const float*)w->gvec, w->Xn);
    hipError_t er = hipSuccess;
    const float* h = enc_forward(e, (int)B, w->Xn, er);
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
