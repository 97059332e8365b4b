// Streamed dataset (mmvae_stream_csr): the caller's cell-major CSR stays in host memory, mapped
// into the device address space, and each step pulls its batch's rows over PCIe into a batch CSR
// in HBM.  The reference reads every batch from its BGZF file (mtx_data_block_t::read,
// mmvae_io.hh:208-245) and needs no more memory than one batch; this is its device counterpart
// for datasets beyond HBM: the step's device work opens with k_stream_gather (one workgroup per
// batch row: its entries and covariates from the host CSR, at the offsets the host computed from
// the rows' nonzero counts) and the batch rows' tile index (k_dataset_index), and every kernel
// after it runs on the batch CSR as the resident path runs on the whole dataset — the batch's row
// b is dataset row b, so the step's results are bit-identical to the resident path's.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"

namespace mmvae {

// rows 0 .. Bp - 1 of the batch (cells[b] = the caller's cell, >= Nh for padding rows), plus
// the batch's empty row Bp; afterwards cells[b] = b
// gcells (prefetched gather): the batch's dataset rows from the slot's mapped row-id array, the
// staged cells already the identity (cells is then not written).
// A few workgroups (gather_wgs) walk the rows, each thread keeping 8 loads per array in flight:
// PCIe latency wants many bytes in flight, not many waves — a grid of one workgroup per row held
// every CU's wave slots while it waited on PCIe and slowed the step it overlapped.
static constexpr int GU = 8;
// hpk (packed dataset): gene << 16 | count per entry instead of hcol / hval
__global__ __launch_bounds__(256) void k_stream_gather(const int64_t* __restrict__ hrp, const int32_t* __restrict__ hcol,
                                                       const float* __restrict__ hval, const uint32_t* __restrict__ hpk,
                                                       const float* __restrict__ hcov,
                                                       int64_t Nh, int C, int64_t* __restrict__ cells,
                                                       const int64_t* __restrict__ gcells,
                                                       const int64_t* __restrict__ brp, int64_t Bp,
                                                       int64_t* __restrict__ rowptr, int32_t* __restrict__ col,
                                                       float* __restrict__ val, float* __restrict__ cov) {
    for (int64_t b = blockIdx.x; b <= Bp; b += gridDim.x) {
        if (b == Bp) {  // the empty row (and rowptr[N + 1] for readers of rowptr[c + 1])
            if (threadIdx.x == 0) {
                rowptr[Bp] = brp[Bp];
                rowptr[Bp + 1] = brp[Bp];
            }
            for (int c = threadIdx.x; c < C; c += 256) cov[Bp * C + c] = 0.f;
            continue;
        }
        const int64_t g = gcells ? gcells[b] : cells[b];
        const bool real = g < Nh;
        const int64_t s = brp[b], n = brp[b + 1] - s;
        const int64_t src = real ? hrp[g] : 0;
        if (hpk) {
            // packed words: 16-byte loads from the row's first 16-byte boundary (4 entries per
            // lane, two loads in flight per lane), the unaligned head word by word
            const int64_t head = std::min<int64_t>(n, (4 - (src & 3)) & 3);
            if (threadIdx.x < head) {
                const uint32_t w = hpk[src + threadIdx.x];
                col[s + threadIdx.x] = (int32_t)(w >> 16);
                val[s + threadIdx.x] = (float)(w & 0xffffu);
            }
            const uint4* p4 = reinterpret_cast<const uint4*>(hpk + src + head);
            const int64_t n4 = (n - head) >> 2;
            for (int64_t q0 = 0; q0 < n4; q0 += 512) {
                uint4 w[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int64_t q = q0 + u * 256 + threadIdx.x;
                    if (q < n4) w[u] = p4[q];
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int64_t q = q0 + u * 256 + threadIdx.x;
                    if (q < n4) {
                        const int64_t o = s + head + 4 * q;
                        const uint32_t ww[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            col[o + j] = (int32_t)(ww[j] >> 16);
                            val[o + j] = (float)(ww[j] & 0xffffu);
                        }
                    }
                }
            }
            const int64_t tail0 = head + 4 * n4;
            if (tail0 + threadIdx.x < n) {
                const uint32_t w = hpk[src + tail0 + threadIdx.x];
                col[s + tail0 + threadIdx.x] = (int32_t)(w >> 16);
                val[s + tail0 + threadIdx.x] = (float)(w & 0xffffu);
            }
        } else {
            for (int64_t i0 = 0; i0 < n; i0 += 256 * GU) {
                int32_t cv[GU];
                float vv[GU];
#pragma unroll
                for (int u = 0; u < GU; ++u) {  // every load of the group in flight before the stores
                    const int64_t i = i0 + u * 256 + threadIdx.x;
                    if (i < n) {
                        cv[u] = hcol[src + i];
                        vv[u] = hval[src + i];
                    }
                }
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    const int64_t i = i0 + u * 256 + threadIdx.x;
                    if (i < n) {
                        col[s + i] = cv[u];
                        val[s + i] = vv[u];
                    }
                }
            }
        }
        for (int c = threadIdx.x; c < C; c += 256) cov[b * C + c] = (real && hcov) ? hcov[g * C + c] : (hcov ? 0.f : (real ? 1.f : 0.f));
        if (!gcells) __syncthreads();  // every thread has read cells[b]
        if (threadIdx.x == 0) {
            rowptr[b] = s;
            if (!gcells) cells[b] = b;
        }
    }
}

static unsigned gather_wgs(const Engine* e) {
    static const int env = [] { const char* v = std::getenv("MMVAE_GATHER_WGS"); return v ? std::atoi(v) : 0; }();
    const int64_t rows = e->Bpad + 1;
    return (unsigned)std::min<int64_t>(rows, env > 0 ? env : 64);
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

// in the step's stream (MMVAE_STREAM_SYNC=1, or a step graph's capture of it): nothing to do when
// stream_prefetch already enqueued the gather on gstream
hipError_t stream_gather(Engine* e) {
    if (!e->streamed || e->stream_prefetch) return hipSuccess;
    ScopedTimer tm(e, "k_stream_gather");
    const int64_t Bp = e->Bpad;
    hipLaunchKernelGGL(k_stream_gather, dim3(gather_wgs(e)), dim3(256), 0, e->stream, e->hs_rowptr, e->hs_col,
                       e->hs_val, (const uint32_t*)e->hs_packed, e->hs_covar, e->N_host, (int)e->C, e->d_cells, (const int64_t*)nullptr, e->d_brp, Bp,
                       e->d_rowptr, e->d_col, e->d_val, e->d_covar);
    hipError_t er = hipGetLastError();
    if (er != hipSuccess) return er;
    if (e->wide) return hipSuccess;  // the wide path densifies from the CSR rows directly
    return index_rows(e, e->d_rowptr, e->d_col, e->d_val, Bp, e->d_rtp, e->d_cellnorm);
}

// the staged step's gather on gstream, right after staging (host side, before the step's launch
// or graph): it starts once the last step on the slot's batch set is done and runs under the
// previous step's kernels; the step's stream waits for it.  The row ids and row offsets are read
// from the slot's mapped pinned memory, so nothing of the step's own staged copy is needed.
hipError_t stream_prefetch(Engine* e) {
    if (!e->streamed || !e->stream_prefetch) return hipSuccess;
    const int s = e->cur_slot;
    const int64_t Bp = e->Bpad;
    hipError_t er = hipStreamWaitEvent(e->gstream, e->ev_setfree[s], 0);
    if (er != hipSuccess) return er;
    hipLaunchKernelGGL(k_stream_gather, dim3(gather_wgs(e)), dim3(256), 0, e->gstream, e->hs_rowptr, e->hs_col,
                       e->hs_val, (const uint32_t*)e->hs_packed, e->hs_covar, e->N_host, (int)e->C, e->d_cells, (const int64_t*)e->h_gcells[s],
                       (const int64_t*)e->h_brp_pin, Bp, e->d_rowptr, e->d_col, e->d_val, e->d_covar);
    if ((er = hipGetLastError()) != hipSuccess) return er;
    if (!e->wide && (er = index_rows(e, e->d_rowptr, e->d_col, e->d_val, Bp, e->d_rtp, e->d_cellnorm, e->gstream)) != hipSuccess)
        return er;
    if ((er = hipEventRecord(e->ev_gathered[s], e->gstream)) != hipSuccess) return er;
    return hipStreamWaitEvent(e->stream, e->ev_gathered[s], 0);
}

// after the step's launches: its batch set is free once the step is done
hipError_t stream_step_done(Engine* e) {
    if (!e->streamed || !e->stream_prefetch) return hipSuccess;
    return hipEventRecord(e->ev_setfree[e->cur_slot], e->stream);
}

void stream_release(Engine* e) {
    if (e->gstream) hipStreamSynchronize(e->gstream);
    for (int s = 0; s < 2; ++s) {
        if (e->ev_gathered[s]) hipEventDestroy(e->ev_gathered[s]);
        if (e->ev_setfree[s]) hipEventDestroy(e->ev_setfree[s]);
        if (e->h_gcells[s]) hipHostFree(e->h_gcells[s]);
        e->ev_gathered[s] = e->ev_setfree[s] = nullptr;
        e->h_gcells[s] = nullptr;
    }
    if (e->gstream) hipStreamDestroy(e->gstream);
    e->gstream = nullptr;
    e->stream_prefetch = false;
    for (auto& q : e->bset) {
        for (void* p : {(void*)q.rowptr, (void*)q.col, (void*)q.val, (void*)q.covar, (void*)q.rtp, (void*)q.cellnorm})
            if (p) hipFree(p);
        q = Engine::BatchSet{};
    }
    for (void* p : e->hs_registered) hipHostUnregister(p);
    if (e->hs_packed) hipHostFree(e->hs_packed);
    e->hs_packed = nullptr;
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
