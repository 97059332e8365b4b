// Streamed dataset (mmvae_stream_csr): the caller's cell-major CSR stays in host memory, mapped
// into the device address space, and each step pulls its batch's rows over PCIe into a batch CSR
// in HBM.  The reference reads every batch from its BGZF file (mtx_data_block_t::read,
// mmvae_io.hh:208-245) and needs no more memory than one batch; this is its device counterpart
// for datasets beyond HBM: the step's device work opens with k_stream_gather (one workgroup per
// batch row: its entries and covariates from the host CSR, at the offsets the host computed from
// the rows' nonzero counts) and the batch rows' tile index (k_dataset_index), and every kernel
// after it runs on the batch CSR as the resident path runs on the whole dataset — the batch's row
// b is dataset row b, so the step's results are bit-identical to the resident path's.
#include <sys/mman.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>

#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"

namespace mmvae {

// rows 0 .. Bp - 1 of the batch (cells[b] = the caller's cell, >= Nh for padding rows), plus
// the batch's empty row Bp; afterwards cells[b] = b
// gcells (prefetched gather): the batch's dataset rows from the slot's mapped row-id array, the
// staged cells already the identity (cells is then not written).
// A few workgroups (gather_wgs) walk the rows, each thread keeping GU loads per array (unpacked) or two 16-byte words (packed) in flight:
// PCIe latency wants many bytes in flight, not many waves — a grid of one workgroup per row held
// every CU's wave slots while it waited on PCIe and slowed the step it overlapped.
static constexpr int GU = 6;
// a workgroup-uniform 64-bit value into scalar registers: the row's bases then cost no VGPRs, and
// the gather stays at <= 48 VGPRs, so its waves fit beside pass B's (2 x 232 of 512 per SIMD)
MMVAE_DEV int64_t uni64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// hpk (packed dataset): gene << 16 | count per entry instead of hcol / hval
// DEV (MMVAE_STREAM_DMA): hpk is the batch's packed rows already in HBM, row b at brp[b]
template <bool PK, bool DEV = false>
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
        const int64_t g = uni64(gcells ? gcells[b] : cells[b]);
        const bool real = g < Nh;
        const int64_t s = uni64(brp[b]);
        const int n = (int)(uni64(brp[b + 1]) - s);  // 32-bit offsets inside the row: few live VGPRs
        const int64_t src = DEV ? s : (real ? uni64(hrp[g]) : 0);
        int32_t* dc = col + s;
        float* dv = val + s;
        if (PK) {
            // packed words: 16-byte loads from the row's first 16-byte boundary (4 entries per
            // lane, two loads in flight per lane), the unaligned head word by word
            const uint32_t* hp = hpk + src;
            const int head = min(n, (int)((4 - (src & 3)) & 3));
            if ((int)threadIdx.x < head) {
                const uint32_t w = hp[threadIdx.x];
                dc[threadIdx.x] = (int32_t)(w >> 16);
                dv[threadIdx.x] = (float)(w & 0xffffu);
            }
            const uint4* p4 = reinterpret_cast<const uint4*>(hp + head);
            const int n4 = (n - head) >> 2;
            int32_t* dc4 = dc + head;
            float* dv4 = dv + head;
            // two 16-byte words per lane in flight, the four stores of a word at immediate offsets
            // of one address: <= 48 VGPRs, so the gather's waves fit beside pass B's
            auto put = [&](int q, const uint4& w) {
                int32_t* c4 = dc4 + 4 * (size_t)q;
                float* v4 = dv4 + 4 * (size_t)q;
                c4[0] = (int32_t)(w.x >> 16);
                c4[1] = (int32_t)(w.y >> 16);
                c4[2] = (int32_t)(w.z >> 16);
                c4[3] = (int32_t)(w.w >> 16);
                v4[0] = (float)(w.x & 0xffffu);
                v4[1] = (float)(w.y & 0xffffu);
                v4[2] = (float)(w.z & 0xffffu);
                v4[3] = (float)(w.w & 0xffffu);
            };
#pragma unroll 1
            for (int q = threadIdx.x; q < n4; q += 512) {
                const bool two = q + 256 < n4;
                const uint4 w0 = p4[q];
                uint4 w1 = uint4{0u, 0u, 0u, 0u};
                if (two) w1 = p4[q + 256];
                put(q, w0);
                if (two) put(q + 256, w1);
            }
            const int tail0 = head + 4 * n4;
            if (tail0 + (int)threadIdx.x < n) {
                const uint32_t w = hp[tail0 + threadIdx.x];
                dc[tail0 + threadIdx.x] = (int32_t)(w >> 16);
                dv[tail0 + threadIdx.x] = (float)(w & 0xffffu);
            }
        } else {
            const int32_t* hc = hcol + src;
            const float* hv = hval + src;
            for (int i0 = 0; i0 < n; i0 += 256 * GU) {
                int32_t cv[GU];
                float vv[GU];
#pragma unroll
                for (int u = 0; u < GU; ++u) {  // every load of the group in flight before the stores
                    const int i = i0 + u * 256 + threadIdx.x;
                    if (i < n) {
                        cv[u] = hc[i];
                        vv[u] = hv[i];
                    }
                }
#pragma unroll
                for (int u = 0; u < GU; ++u) {
                    const int i = i0 + u * 256 + threadIdx.x;
                    if (i < n) {
                        dc[i] = cv[u];
                        dv[i] = vv[u];
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

// DMA mode with 3-byte entries (stream_b3): genes as uint16, counts as uint8, both at the rows'
// batch offsets; four entries per lane in flight
__global__ __launch_bounds__(256) void k_stream_unpack3(const uint16_t* __restrict__ g16, const uint8_t* __restrict__ c8,
                                                        const float* __restrict__ hcov, int64_t Nh, int C,
                                                        const int64_t* __restrict__ gcells, const int64_t* __restrict__ brp,
                                                        int64_t Bp, int64_t* __restrict__ rowptr, int32_t* __restrict__ col,
                                                        float* __restrict__ val, float* __restrict__ cov) {
    for (int64_t b = blockIdx.x; b <= Bp; b += gridDim.x) {
        if (b == Bp) {
            if (threadIdx.x == 0) {
                rowptr[Bp] = brp[Bp];
                rowptr[Bp + 1] = brp[Bp];
            }
            for (int c = threadIdx.x; c < C; c += 256) cov[Bp * C + c] = 0.f;
            continue;
        }
        const int64_t g = uni64(gcells[b]);
        const bool real = g < Nh;
        const int64_t s = uni64(brp[b]);
        const int n = (int)(uni64(brp[b + 1]) - s);
        const uint16_t* gs = g16 + s;
        const uint8_t* cs = c8 + s;
        int32_t* dc = col + s;
        float* dv = val + s;
        for (int i0 = threadIdx.x; i0 < n; i0 += 1024) {
            uint32_t gg[4], cc[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = min(i0 + 256 * u, n - 1);
                gg[u] = gs[i];
                cc[u] = cs[i];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + 256 * u < n) {
                    dc[i0 + 256 * u] = (int32_t)gg[u];
                    dv[i0 + 256 * u] = (float)cc[u];
                }
        }
        for (int c = threadIdx.x; c < C; c += 256) cov[b * C + c] = (real && hcov) ? hcov[g * C + c] : (hcov ? 0.f : (real ? 1.f : 0.f));
        if (threadIdx.x == 0) rowptr[b] = s;
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

// in the step's stream (or a step graph's capture of it): the whole gather with MMVAE_STREAM_SYNC=1;
// with the prefetch, the DMA mode's unpack (HBM to HBM) and, with it or MMVAE_STREAM_INDEX_STEP=1,
// the batch's tile index — short full-GPU launches instead of more work on gstream's chain
static hipError_t stream_dma_unpack(Engine* e);

hipError_t stream_gather(Engine* e) {
    if (!e->streamed) return hipSuccess;
    if (e->stream_prefetch) {
        const bool dma = e->stream_dma && e->hs_packed;
        if (dma) {
            hipError_t er = stream_dma_unpack(e);
            if (er != hipSuccess) return er;
        }
        if (e->wide || !(e->stream_index_step || dma)) return hipSuccess;
        ScopedTimer tm(e, "k_dataset_index");
        return index_rows(e, e->d_rowptr, e->d_col, e->d_val, e->Bpad, e->d_rtp, e->d_cellnorm);
    }
    ScopedTimer tm(e, "k_stream_gather");
    const int64_t Bp = e->Bpad;
    // the gather kernel reads the dataset over PCIe: the packed copy's device address, or the
    // caller's registered arrays (a host-only packed copy belongs to the DMA mode)
    if (e->hs_packed ? !e->hs_packed_dev : !(e->hs_col && e->hs_val)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(e->hs_packed ? k_stream_gather<true> : k_stream_gather<false>, dim3(gather_wgs(e)), dim3(256), 0, e->stream, e->hs_rowptr, e->hs_col,
                       e->hs_val, e->hs_packed_dev, e->hs_covar, e->N_host, (int)e->C, e->d_cells, (const int64_t*)nullptr, e->d_brp, Bp,
                       e->d_rowptr, e->d_col, e->d_val, e->d_covar);
    hipError_t er = hipGetLastError();
    if (er != hipSuccess) return er;
    if (e->wide) return hipSuccess;  // the wide path densifies from the CSR rows directly
    return index_rows(e, e->d_rowptr, e->d_col, e->d_val, Bp, e->d_rtp, e->d_cellnorm);
}

// host gather pool (MMVAE_STREAM_DMA): persistent workers, the calling thread joins as worker 0
struct GatherPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, cv_done;
    std::function<void(int, int)> job;
    int gen = 0, pending = 0, nth = 1;
    bool stop = false;
    explicit GatherPool(int n) : nth(n) {
        for (int t = 1; t < n; ++t)
            th.emplace_back([this, t] {
                int seen = 0;
                for (;;) {
                    std::function<void(int, int)> j;
                    {
                        std::unique_lock<std::mutex> lk(m);
                        cv.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        j = job;
                    }
                    j(t, nth);
                    std::lock_guard<std::mutex> lk(m);
                    if (--pending == 0) cv_done.notify_one();
                }
            });
    }
    void run(std::function<void(int, int)> f) {
        {
            std::lock_guard<std::mutex> lk(m);
            job = f;
            pending = nth - 1;
            ++gen;
        }
        cv.notify_all();
        f(0, nth);
        std::unique_lock<std::mutex> lk(m);
        cv_done.wait(lk, [&] { return pending == 0; });
    }
    ~GatherPool() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        for (auto& x : th) x.join();
    }
};

// slot s's DMA copy buffers (pinned host + HBM) for `cap` packed entries; the caller bumps
// graph_gen (the step graphs' unpack reads d_bpk[s])
hipError_t stream_bpk_alloc(Engine* e, int s, int64_t cap) {
    hipError_t er;
    if (e->gstream && (er = hipStreamSynchronize(e->gstream)) != hipSuccess) return er;
    if (e->h_bpk[s]) hipHostFree(e->h_bpk[s]);
    if (e->d_bpk[s]) hipFree(e->d_bpk[s]);
    e->h_bpk[s] = nullptr;
    e->d_bpk[s] = nullptr;
    e->bpk_cap[s] = 0;
    if ((er = hipHostMalloc((void**)&e->h_bpk[s], sizeof(uint32_t) * (size_t)cap, hipHostMallocDefault)) != hipSuccess) return er;
    if ((er = hipMalloc(&e->d_bpk[s], sizeof(uint32_t) * (size_t)cap)) != hipSuccess) return er;
    e->bpk_cap[s] = cap;
    return hipSuccess;
}

// MMVAE_STREAM_DMA: the slot's rows packed on the host, one DMA copy, the unpack kernel on HBM
static hipError_t stream_dma_gather(Engine* e, int s, int64_t Bp) {
    hipError_t er;
    const int64_t tot = e->h_brp_pin[Bp];
    if ((er = hipEventSynchronize(e->ev_gathered[s])) != hipSuccess) return er;  // slot s's last copy has read h_bpk[s]
    if (tot > e->bpk_cap[s]) {
        if ((er = stream_bpk_alloc(e, s, tot + tot / 4 + 1024)) != hipSuccess) return er;
        ++e->graph_gen;  // the step graphs' unpack reads d_bpk[s]: re-captured with the new buffer
    }
    if (!e->gpool) {
        static const int env = [] { const char* v = std::getenv("MMVAE_STREAM_DMA_THREADS"); return v ? std::atoi(v) : 0; }();
        const int n = env > 0 ? env : (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
        e->gpool = new GatherPool(n);
    }
    const int64_t* gc = e->h_gcells[s];
    const int64_t* brp = e->h_brp_pin;
    uint32_t* dst = e->h_bpk[s];
    const uint32_t* src = e->hs_packed;
    const int64_t* hrp = e->hh_rowptr;
    const int64_t Nh = e->N_host;
    // 3-byte entries: genes (uint16) from the buffer's start, counts (uint8) from byte 2 * cap
    const bool b3 = e->stream_b3;
    uint16_t* g3 = reinterpret_cast<uint16_t*>(dst);
    uint8_t* c3 = reinterpret_cast<uint8_t*>(dst) + 2 * (size_t)e->bpk_cap[s];
    static_cast<GatherPool*>(e->gpool)->run([&](int t, int nth) {  // contiguous row ranges of about equal entries
        const int64_t a = tot * t / nth, z = tot * (t + 1) / nth;
        int64_t b = std::upper_bound(brp, brp + Bp + 1, a) - brp - 1;
        for (; b < Bp && brp[b] < z; ++b) {
            const int64_t n = brp[b + 1] - brp[b];
            if (n > 0 && gc[b] < Nh) {  // the part of row b inside [a, z)
                const int64_t lo = std::max(a, brp[b]), hi = std::min(z, brp[b + 1]);
                if (hi > lo) {
                    const uint32_t* w = src + hrp[gc[b]] + (lo - brp[b]);
                    if (b3) {
                        for (int64_t i = 0; i < hi - lo; ++i) {
                            g3[lo + i] = (uint16_t)(w[i] >> 16);
                            c3[lo + i] = (uint8_t)w[i];
                        }
                    } else {
                        std::memcpy(dst + lo, w, sizeof(uint32_t) * (size_t)(hi - lo));
                    }
                }
            }
        }
    });
    // only the copy runs on gstream: the unpack and the tile index are the step's first kernels
    // (stream_gather), so step n + 1's copy overlaps step n's whole kernel chain
    if (tot > 0 && b3) {
        if ((er = hipMemcpyAsync(e->d_bpk[s], e->h_bpk[s], 2 * (size_t)tot, hipMemcpyHostToDevice, e->gstream)) != hipSuccess) return er;
        const size_t co = 2 * (size_t)e->bpk_cap[s];
        return hipMemcpyAsync(reinterpret_cast<char*>(e->d_bpk[s]) + co, reinterpret_cast<char*>(e->h_bpk[s]) + co, (size_t)tot,
                              hipMemcpyHostToDevice, e->gstream);
    }
    if (tot > 0 && (er = hipMemcpyAsync(e->d_bpk[s], e->h_bpk[s], sizeof(uint32_t) * (size_t)tot, hipMemcpyHostToDevice, e->gstream)) != hipSuccess)
        return er;
    return hipSuccess;
}

// the DMA mode's unpack of the slot's packed rows (HBM to HBM, one workgroup per row up to 2048)
static hipError_t stream_dma_unpack(Engine* e) {
    const int64_t Bp = e->Bpad;
    const int s = e->cur_slot;
    ScopedTimer tm(e, "k_stream_gather");
    if (e->stream_b3) {
        const uint16_t* g16 = reinterpret_cast<const uint16_t*>(e->d_bpk[s]);
        const uint8_t* c8 = reinterpret_cast<const uint8_t*>(e->d_bpk[s]) + 2 * (size_t)e->bpk_cap[s];
        hipLaunchKernelGGL(k_stream_unpack3, dim3((unsigned)std::min<int64_t>(Bp + 1, 2048)), dim3(256), 0, e->stream, g16, c8,
                           e->hs_covar, e->N_host, (int)e->C, (const int64_t*)e->h_gcells[s], (const int64_t*)e->h_brp_pin, Bp,
                           e->d_rowptr, e->d_col, e->d_val, e->d_covar);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_stream_gather<true, true>), dim3((unsigned)std::min<int64_t>(Bp + 1, 2048)), dim3(256), 0, e->stream, e->hs_rowptr,
                       e->hs_col, e->hs_val, (const uint32_t*)e->d_bpk[s], e->hs_covar, e->N_host, (int)e->C, e->d_cells,
                       (const int64_t*)e->h_gcells[s], (const int64_t*)e->h_brp_pin, Bp, e->d_rowptr, e->d_col, e->d_val, e->d_covar);
    return hipGetLastError();
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
    if (e->stream_dma && e->hs_packed) {
        if ((er = stream_dma_gather(e, s, Bp)) != hipSuccess) return er;
    } else {
        if (e->hs_packed ? !e->hs_packed_dev : !(e->hs_col && e->hs_val)) return hipErrorInvalidValue;
        hipLaunchKernelGGL(e->hs_packed ? k_stream_gather<true> : k_stream_gather<false>, dim3(gather_wgs(e)), dim3(256), 0, e->gstream, e->hs_rowptr, e->hs_col,
                           e->hs_val, e->hs_packed_dev, e->hs_covar, e->N_host, (int)e->C, e->d_cells, (const int64_t*)e->h_gcells[s],
                           (const int64_t*)e->h_brp_pin, Bp, e->d_rowptr, e->d_col, e->d_val, e->d_covar);
        if ((er = hipGetLastError()) != hipSuccess) return er;
    }
    if (!e->wide && !e->stream_index_step && !(e->stream_dma && e->hs_packed) &&
        (er = index_rows(e, e->d_rowptr, e->d_col, e->d_val, Bp, e->d_rtp, e->d_cellnorm, e->gstream)) != hipSuccess)
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
    delete static_cast<GatherPool*>(e->gpool);
    e->gpool = nullptr;
    for (int s = 0; s < 2; ++s) {
        if (e->h_bpk[s]) hipHostFree(e->h_bpk[s]);
        if (e->d_bpk[s]) hipFree(e->d_bpk[s]);
        e->h_bpk[s] = nullptr;
        e->d_bpk[s] = nullptr;
        e->bpk_cap[s] = 0;
    }
    e->stream_dma = false;
    e->stream_b3 = false;
    e->hs_cmax = 0;
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
    for (void* p : e->hs_registered) hipHostFree(p);  // (the engine's pinned copies)
    if (e->hs_packed && e->hs_packed_bytes) {  // mmap'd: pageable (DMA mode) or registered (THP zero-copy)
        if (e->hs_packed_reg) hipHostUnregister(e->hs_packed);
        munmap(e->hs_packed, e->hs_packed_bytes);
    } else if (e->hs_packed) {
        hipHostFree(e->hs_packed);
    }
    e->hs_packed_reg = false;
    e->hs_packed = nullptr;
    e->hs_packed_dev = nullptr;
    e->hs_packed_bytes = 0;
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
