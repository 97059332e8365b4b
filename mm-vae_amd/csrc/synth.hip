// Device-side synthetic single-cell dataset (bench / smoke inputs):
//   p_g ~ Gamma(0.3, 1) normalised (host, seeded), L_c ~ LogNormal(ln lib, 0.5),
//   x_gc ~ Poisson(L_c p_g Gamma(2, 1/2)).
// Every (cell, gene) draw is a pure function of (seed, cell, gene) (Philox), so two passes
// (count, fill) produce a sorted cell-major CSR without storing the dense matrix.
#include <random>
#include <vector>

#include "common.hpp"
#include "engine.hpp"

namespace mmvae {

MMVAE_DEV float u01(uint32_t x) { return ((x >> 8) + 1) * (1.f / 16777217.f); }

MMVAE_DEV int synth_count(uint64_t seed, int64_t cell, int g, float lib_c, const float* pg) {
    uint32_t c[4] = {(uint32_t)g, (uint32_t)cell, (uint32_t)(cell >> 32), 0x5eedu};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ 0x9e37u);
    // Gamma(2, 1/2) = 0.5 * (E1 + E2)
    const float gam = -0.5f * (logf(u01(c[0])) + logf(u01(c[1])));
    const float lam = lib_c * pg[g] * gam;
    const float u = u01(c[2]);
    if (lam > 30.f) {
        const float n = sqrtf(-2.f * logf(u)) * cosf(6.2831853f * u01(c[3]));
        return max(0, (int)rintf(lam + sqrtf(lam) * n));
    }
    float pk = expf(-lam), cdf = pk;
    int k = 0;
    while (u > cdf && k < 200) {
        ++k;
        pk *= lam / (float)k;
        cdf += pk;
    }
    return k;
}

MMVAE_DEV float synth_lib(uint64_t seed, int64_t cell, float loglib) {
    uint32_t c[4] = {0xffffffffu, (uint32_t)cell, (uint32_t)(cell >> 32), 0x11bu};
    philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float n = sqrtf(-2.f * logf(u01(c[0]))) * cosf(6.2831853f * u01(c[1]));
    return expf(loglib + 0.5f * n);
}

__global__ __launch_bounds__(256) void k_synth_count(uint64_t seed, int64_t N, int D, float loglib,
                                                     const float* __restrict__ pg, int64_t* __restrict__ counts) {
    __shared__ int sb[4];
    const int64_t cell = blockIdx.x;
    const float L = synth_lib(seed, cell, loglib);
    int n = 0;
    for (int g = threadIdx.x; g < D; g += 256) n += synth_count(seed, cell, g, L, pg) > 0;
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
    if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = n;
    __syncthreads();
    if (threadIdx.x == 0) counts[cell] = sb[0] + sb[1] + sb[2] + sb[3];
}

__global__ __launch_bounds__(256) void k_synth_fill(uint64_t seed, int64_t N, int D, float loglib,
                                                    const float* __restrict__ pg, const int64_t* __restrict__ rowptr,
                                                    int32_t* __restrict__ col, float* __restrict__ val) {
    __shared__ int wcnt[4];
    const int64_t cell = blockIdx.x;
    const float L = synth_lib(seed, cell, loglib);
    int64_t base = rowptr[cell];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int g0 = 0; g0 < D; g0 += 256) {
        const int g = g0 + threadIdx.x;
        const int x = (g < D) ? synth_count(seed, cell, g, L, pg) : 0;
        const uint64_t m = __ballot(x > 0);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[w] = __popcll(m);
        __syncthreads();
        int off = 0;
        for (int i = 0; i < w; ++i) off += wcnt[i];
        const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        if (x > 0) {
            col[base + off + before] = g;
            val[base + off + before] = (float)x;
        }
        base += tot;
        __syncthreads();
    }
}

hipError_t synth_dataset(Engine* e, int64_t N, double lib, uint64_t seed, int64_t* nnz_out) {
    const int D = (int)e->D;
    std::mt19937_64 rng(seed);
    std::gamma_distribution<double> gam(0.3, 1.0);
    std::vector<float> pg(D);
    double tot = 0;
    std::vector<double> tmp(D);
    for (int g = 0; g < D; ++g) tot += (tmp[g] = gam(rng));
    for (int g = 0; g < D; ++g) pg[g] = (float)(tmp[g] / tot);
    float* d_pg = nullptr;
    int64_t* d_cnt = nullptr;
    hipError_t er;
    if ((er = hipMalloc(&d_pg, sizeof(float) * D)) != hipSuccess) return er;
    if ((er = hipMalloc(&d_cnt, sizeof(int64_t) * N)) != hipSuccess) return er;
    hipMemcpy(d_pg, pg.data(), sizeof(float) * D, hipMemcpyHostToDevice);
    const float loglib = (float)std::log(lib);
    hipLaunchKernelGGL(k_synth_count, dim3((unsigned)N), dim3(256), 0, e->stream, seed, N, D, loglib, d_pg, d_cnt);
    std::vector<int64_t> cnt(N), rp(N + 2, 0);  // rp[N + 1] = nnz: the empty padding row N
    if ((er = hipMemcpyAsync(cnt.data(), d_cnt, sizeof(int64_t) * N, hipMemcpyDeviceToHost, e->stream)) != hipSuccess)
        return er;
    if ((er = hipStreamSynchronize(e->stream)) != hipSuccess) return er;
    for (int64_t i = 0; i < N; ++i) rp[i + 1] = rp[i] + cnt[i];
    const int64_t nnz = rp[N];
    rp[N + 1] = nnz;
    hipFree(e->d_rowptr);
    hipFree(e->d_col);
    hipFree(e->d_val);
    hipFree(e->d_covar);
    e->d_rowptr = nullptr;
    e->d_col = nullptr;
    e->d_val = nullptr;
    e->d_covar = nullptr;
    if ((er = hipMalloc(&e->d_rowptr, sizeof(int64_t) * (N + 2))) != hipSuccess) return er;
    if ((er = hipMalloc(&e->d_col, sizeof(int32_t) * (nnz + 64))) != hipSuccess) return er;
    if ((er = hipMalloc(&e->d_val, sizeof(float) * (nnz + 64))) != hipSuccess) return er;
    if ((er = hipMalloc(&e->d_covar, sizeof(float) * (N + 1) * e->C)) != hipSuccess) return er;  // row N: zeros
    if ((er = hipMemset(e->d_covar + N * e->C, 0, sizeof(float) * e->C)) != hipSuccess) return er;
    hipMemcpy(e->d_rowptr, rp.data(), sizeof(int64_t) * (N + 2), hipMemcpyHostToDevice);
    std::vector<float> ones((size_t)N * e->C, 1.f);
    hipMemcpy(e->d_covar, ones.data(), sizeof(float) * N * e->C, hipMemcpyHostToDevice);
    e->unit_covar = e->C == 1;
    hipLaunchKernelGGL(k_synth_fill, dim3((unsigned)N), dim3(256), 0, e->stream, seed, N, D, loglib, d_pg,
                       e->d_rowptr, e->d_col, e->d_val);
    if ((er = hipStreamSynchronize(e->stream)) != hipSuccess) return er;
    e->N = N;
    e->nnz = nnz;
    e->cell_nnz.resize((size_t)N);
    for (int64_t i = 0; i < N; ++i) e->cell_nnz[(size_t)i] = (int32_t)cnt[(size_t)i];
    if ((er = build_dataset_index(e)) != hipSuccess) return er;
    hipFree(d_pg);
    hipFree(d_cnt);
    if (nnz_out) *nnz_out = nnz;
    return hipGetLastError();
}

// =======================================================================================
// Per-dataset index, built once after every upload / synth (the HBM-resident counterpart of the
// reference's ${mtx}.index, mmutil_index.hh:138-228): for every cell row
//   rtp_all[cell][t] = first CSR entry (relative) with gene >= 64 t, t = 0..NT  (the 16 x 64
//                      tile walk of every tile kernel; row N is the all-empty padding row)
//   cellnorm[cell]   = (sum log1p(x)^2, sum log1p(x)^2 + 2 eps log1p(x)), eps = 1e-2 / D:
//                      the vMF row norms of vmf.hh:253 and vmf.hh:422-423 (x only; accurate log1pf)
// One wave per row; the per-step kernels then never re-scan the batch's rows.
// =======================================================================================
__global__ __launch_bounds__(256) void k_dataset_index(const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                                       const float* __restrict__ val, int64_t N, int NT, float epsD,
                                                       int32_t* __restrict__ rtp, float2* __restrict__ cellnorm,
                                                       int32_t* __restrict__ xflag, uint32_t* __restrict__ pk) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    // log1pf of the integer counts 0 .. 511 from a workgroup table (the same log1pf values, so the
    // norms are bit-identical): the accurate log1pf is ~150 instructions
    __shared__ float l1tab[512];
    for (int i = threadIdx.x; i < 512; i += 256) l1tab[i] = log1pf((float)i);
    __syncthreads();
    if (row > N) return;
    int32_t* rt = rtp + row * (NT + 1);
    int n = 0;
    int64_t s = 0;
    if (row < N) {
        s = rowptr[row];
        n = (int)(rowptr[row + 1] - s);
    }
    const int32_t* cr = col + s;
    const float* vr = val + s;
    float sl2 = 0.f, sy = 0.f;
    bool nonint = false;  // a value the batch lists cannot carry in the entry word (tiles.hpp EntList)
    bool nonpk = false;   // a value the packed copy cannot carry (an integer count below 2^16)
    // four entries per lane per round, every load issued first (the per-step batch index of the
    // streamed dataset is latency-bound); each lane still sums its entries j = lane, lane + 64, ...
    // in order, so the norms are those of one entry per round
    constexpr int U = 4;
    for (int j0 = lane; j0 < n; j0 += 64 * U) {
        int g[U], gp[U];
        float x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = min(j0 + 64 * u, n - 1);
            g[u] = cr[j];
            gp[u] = cr[max(j - 1, 0)];  // unconditional: a predicated load would wait on its own
            x[u] = vr[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + 64 * u;
            if (j < n) {
                const float xv = x[u];
                nonint |= !((__float_as_uint(xv) >> 31) == 0u && xv < 4194304.f && xv == floorf(xv));  // (-0 and NaN too)
                nonpk |= !((__float_as_uint(xv) >> 31) == 0u && xv < 65536.f && xv == floorf(xv));
                if (pk) pk[s + j] = ((uint32_t)g[u] << 16) | (uint32_t)fminf(fmaxf(xv, 0.f), 65535.f);
                const int xi = (int)fminf(fmaxf(xv, 0.f), 511.f);
                // (x >= 0: log1pf(max(x, 0)) is l itself; else log1pf(0) = 0)
                const float l = ((float)xi == xv) ? l1tab[xi] : log1pf(xv);
                const float ly = xv >= 0.f ? l : 0.f;
                sl2 = fmaf(l, l, sl2);
                sy = fmaf(ly, ly + 2.f * epsD, sy);
                for (int tt = (j > 0 ? gp[u] >> 6 : -1) + 1; tt <= (g[u] >> 6); ++tt) rt[tt] = j;
            }
        }
    }
    const int tlast = (n == 0) ? -1 : (cr[n - 1] >> 6);
    for (int tt = tlast + 1 + lane; tt <= NT; tt += 64) rt[tt] = n;
    sl2 = wave_sum(sl2);
    sy = wave_sum(sy);
    if (lane == 0) cellnorm[row] = float2{sl2, sy};
    // (plain stores: every writer of a word stores the same value)
    if (xflag && __ballot(nonint) != 0ull && lane == 0) xflag[0] = 1;
    if (xflag && __ballot(nonpk) != 0ull && lane == 0) xflag[1] = 1;
}

// the index of rows [0, N] of a CSR (row N: the empty row) on the handle's stream, no sync
hipError_t index_rows(Engine* e, const int64_t* rowptr, const int32_t* col, const float* val, int64_t N, int32_t* rtp,
                      float* cellnorm, hipStream_t st) {
    const float epsD = (float)(1e-2 / (double)(float)e->D);
    hipLaunchKernelGGL(k_dataset_index, dim3((unsigned)((N + 1 + 3) / 4)), dim3(256), 0, st ? st : e->stream, rowptr, col, val, N,
                       (int)e->NT, epsD, rtp, (float2*)cellnorm, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t build_dataset_index(Engine* e) {
    if (e->wide) return hipSuccess;  // the wide path densifies straight from the CSR rows
    hipFree(e->d_rtp);
    hipFree(e->d_cellnorm);
    hipFree(e->d_pk);
    e->d_pk = nullptr;
    e->pk_on = false;
    e->d_rtp = nullptr;
    e->d_cellnorm = nullptr;
    hipError_t er;
    if ((er = hipMalloc(&e->d_rtp, sizeof(int32_t) * (size_t)(e->N + 1) * (size_t)(e->NT + 1))) != hipSuccess) return er;
    if ((er = hipMalloc(&e->d_cellnorm, sizeof(float2) * (size_t)(e->N + 1))) != hipSuccess) return er;
    const float epsD = (float)(1e-2 / (double)(float)e->D);
    // the packed copy for the list builder (MMVAE_LISTS_PK=0: none)
    if (e->D <= 65536 && e->nnz > 0 && !getenv_is("MMVAE_LISTS_PK", "0"))
        if ((er = hipMalloc(&e->d_pk, sizeof(uint32_t) * ((size_t)e->nnz + 64))) != hipSuccess) return er;  // (+64: the clamped loads of an empty row read word nnz)
    int32_t* d_xf = nullptr;  // [0]: some value is not an integer count in [0, 2^22); [1]: in [0, 2^16)
    if ((er = hipMalloc(&d_xf, 2 * sizeof(int32_t))) != hipSuccess) return er;
    if ((er = hipMemsetAsync(d_xf, 0, 2 * sizeof(int32_t), e->stream)) != hipSuccess) return er;
    {
        ScopedTimer tm(e, "k_dataset_index");
        hipLaunchKernelGGL(k_dataset_index, dim3((unsigned)((e->N + 1 + 3) / 4)), dim3(256), 0, e->stream, e->d_rowptr,
                           e->d_col, e->d_val, e->N, (int)e->NT, epsD, e->d_rtp, (float2*)e->d_cellnorm, d_xf, e->d_pk);
    }
    if ((er = hipGetLastError()) != hipSuccess) return er;
    int32_t xf = 0, xp[2] = {0, 0};
    er = hipMemcpyAsync(xp, d_xf, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream);
    if (er == hipSuccess) er = hipStreamSynchronize(e->stream);
    hipFree(d_xf);
    if (er != hipSuccess) return er;
    xf = xp[0];
    e->pk_on = e->d_pk && !xp[1];
    if (e->d_pk && xp[1]) {  // not counts: no packed copy
        hipFree(e->d_pk);
        e->d_pk = nullptr;
    }
    const bool xm = xf != 0 || getenv_is("MMVAE_LISTS_XM", "1");  // (test hook: the float-value lists)
    if (xm != e->ent_xm) ++e->graph_gen;  // the lists' format is baked into captured steps
    e->ent_xm = xm;
    return hipSuccess;
}

}  // namespace mmvae
