// Streamed dataset (mmvae_stream_csr): the caller's cell-major CSR stays in host memory, mapped
// into the device address space, and each step pulls its batch's rows over PCIe into a batch CSR
// in HBM.  The reference reads every batch from its BGZF file (mtx_data_block_t::read,
// mmvae_io.hh:208-245) and needs no more memory than one batch; this is its device counterpart
// for datasets beyond HBM: the step's device work opens with k_stream_gather (one workgroup per
// batch row: its entries and covariates from the host CSR, at the offsets the host computed from
// the rows' nonzero counts) and the batch rows' tile index (k_dataset_index), and every kernel
// after it runs on the batch CSR as the resident path runs on the whole dataset — the batch's row
// b is dataset row b, so the step's results are bit-identical to the resident path's.
#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"

namespace mmvae {

// rows 0 .. Bp - 1 of the batch (cells[b] = the caller's cell, >= Nh for padding rows), plus
// the batch's empty row Bp; afterwards cells[b] = b
__global__ __launch_bounds__(256) void k_stream_gather(const int64_t* __restrict__ hrp, const int32_t* __restrict__ hcol,
                                                       const float* __restrict__ hval, const float* __restrict__ hcov,
                                                       int64_t Nh, int C, int64_t* __restrict__ cells,
                                                       const int64_t* __restrict__ brp, int64_t Bp,
                                                       int64_t* __restrict__ rowptr, int32_t* __restrict__ col,
                                                       float* __restrict__ val, float* __restrict__ cov) {
    const int64_t b = blockIdx.x;
    if (b == Bp) {  // the empty row (and rowptr[N + 1] for readers of rowptr[c + 1])
        if (threadIdx.x == 0) {
            rowptr[Bp] = brp[Bp];
            rowptr[Bp + 1] = brp[Bp];
        }
        for (int c = threadIdx.x; c < C; c += 256) cov[Bp * C + c] = 0.f;
        return;
    }
    const int64_t g = cells[b];
    const bool real = g < Nh;
    const int64_t s = brp[b], n = brp[b + 1] - s;
    const int64_t src = real ? hrp[g] : 0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        col[s + i] = hcol[src + i];
        val[s + i] = hval[src + i];
    }
    for (int c = threadIdx.x; c < C; c += 256) cov[b * C + c] = (real && hcov) ? hcov[g * C + c] : (hcov ? 0.f : (real ? 1.f : 0.f));
    __syncthreads();  // every thread has read cells[b]
    if (threadIdx.x == 0) {
        rowptr[b] = s;
        cells[b] = b;
    }
}

void stream_bind(Engine* e, int s) {
    if (!e->streamed) return;
    const Engine::BatchSet& q = e->bset[s];
    e->d_rowptr = q.rowptr;
    e->d_col = q.col;
    e->d_val = q.val;
    e->d_covar = q.covar;
    e->d_rtp = q.rtp;
    e->d_cellnorm = q.cellnorm;
}

hipError_t stream_gather(Engine* e) {
    if (!e->streamed) return hipSuccess;
    ScopedTimer tm(e, "k_stream_gather");
    const int64_t Bp = e->Bpad;
    hipLaunchKernelGGL(k_stream_gather, dim3((unsigned)(Bp + 1)), dim3(256), 0, e->stream, e->hs_rowptr, e->hs_col,
                       e->hs_val, e->hs_covar, e->N_host, (int)e->C, e->d_cells, e->d_brp, Bp, e->d_rowptr, e->d_col,
                       e->d_val, e->d_covar);
    hipError_t er = hipGetLastError();
    if (er != hipSuccess) return er;
    if (e->wide) return hipSuccess;  // the wide path densifies from the CSR rows directly
    return index_rows(e, e->d_rowptr, e->d_col, e->d_val, Bp, e->d_rtp, e->d_cellnorm);
}

void stream_release(Engine* e) {
    for (auto& q : e->bset) {
        for (void* p : {(void*)q.rowptr, (void*)q.col, (void*)q.val, (void*)q.covar, (void*)q.rtp, (void*)q.cellnorm})
            if (p) hipFree(p);
        q = Engine::BatchSet{};
    }
    for (void* p : e->hs_registered) hipHostUnregister(p);
    e->hs_registered.clear();
    e->hs_rowptr = nullptr;
    e->hs_col = nullptr;
    e->hs_val = nullptr;
    e->hs_covar = nullptr;
    if (e->streamed) {  // the views pointed at the batch sets
        e->d_rowptr = nullptr;
        e->d_col = nullptr;
        e->d_val = nullptr;
        e->d_covar = nullptr;
        e->d_rtp = nullptr;
        e->d_cellnorm = nullptr;
    }
    e->streamed = false;
}

}  // namespace mmvae
