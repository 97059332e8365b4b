// Per-step batch entry lists: the batch's CSR entries regrouped by (16-row wave block, 64-gene
// tile), so every tile kernel reads a tile's entries of its 16 rows as one contiguous, lane-
// balanced list — no per-tile prefix scans over the rows, no per-row pointers in LDS.
//
//   ents  uint32 [E + 64]: pos = row-in-block << 6 | gene-in-tile in bits 0-9, the count in bits
//         10-31 (integer counts below 2^22); other data keep the value as a float in a parallel
//         array (Engine::ent_xm, tiles.hpp EntList).  Row-major inside a tile (rows ascending,
//         genes ascending — the order of the reference's dense row read, mmvae_io.hh:208-245)
//   seg   int64 [WB + 1]: first entry of wave block wb (host prefix of the rows' nonzero counts)
//   toff  int32 [WB][NT + 1]: first entry of tile t inside the block's segment
// Built from the per-dataset tile index (rtp) by one launch, k_batch_lists (one workgroup per
// wave block).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "engine.hpp"
#include "tiles.hpp"

namespace mmvae {

// One workgroup per 16-row wave block, one wave per row, everything in LDS:
//   1. the 16 rows' tile pointers (from the dataset index rtp) -> per-tile counts, the rows'
//      prefix inside every tile list and the block's tile offsets (exclusive scan) -> toff
//   2. the block's list segment is built in chunks of whole tiles (<= cap entries): every wave
//      drops its row's entries of the chunk's tiles at their final positions, then the workgroup
//      streams the chunk out with contiguous, full-line stores (no partial lines written from
//      different waves or CUs).
//   XM = false: the chunk is staged as entry words (4 B: a 16-row block of ~26k entries at the
//   headline is one chunk); XM = true: as (pos, value) pairs, streamed out to both arrays.
//   PK = true: the rows are read from the dataset's packed copy (gene << 16 | count, one word per
//   entry, Engine::d_pk), so a row's first 2048 entries are in flight before the index phase in
//   the registers the unpacked (col, val) pairs of 1024 take.
static constexpr int COPY_CAP_MAX = 32768;  // entries per LDS chunk (<= 128 KB), less for wide D
template <bool XM, bool PK>
__global__ __launch_bounds__(1024) void k_batch_lists(const int64_t* __restrict__ cells,
                                                      const int64_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col, const float* __restrict__ val,
                                                      const uint32_t* __restrict__ pk,
                                                      const int32_t* __restrict__ rtp, const int64_t* __restrict__ seg,
                                                      int NT, int cap, int32_t* __restrict__ toff,
                                                      uint32_t* __restrict__ ents, int64_t xoff, int dbg,
                                                      const float2* __restrict__ dotw, const float* __restrict__ Wne,
                                                      int H, int D, float* __restrict__ rowdots,
                                                      const StepScalars* __restrict__ ss, int64_t* ticket_out) {
    extern __shared__ __attribute__((aligned(16))) char csm[];
    using SE = typename std::conditional<XM, uint2, uint32_t>::type;  // staged entry
    SE* stage = reinterpret_cast<SE*>(csm);                            // [cap]
    int32_t* tw = reinterpret_cast<int32_t*>(csm + sizeof(SE) * (size_t)cap);  // [NT + 1] tile offsets
    int32_t* srt = tw + (NT + 1);                                       // [16][NT + 1] rows' tile pointers
    int32_t* sbase = srt + 16 * (NT + 1);                               // [16][NT] rows' list bases
    __shared__ int32_t wsum[16];
    __shared__ int32_t scarry;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tid = threadIdx.x;
    const int wb = blockIdx.x, b = wb * 16 + w;
    // the staged block is copied (the prep kernel ran before this one): release its slot to the
    // host with one system-scope vector store of the step's ticket
    if (wb == 0 && tid == 0) __hip_atomic_store(ticket_out, ss->ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int64_t c = cells[b];
    const int64_t s = rowptr[c];
    const int rn = (int)(rowptr[c + 1] - s);  // the row's nonzeros (rt[NT])
    // the row's first 1024 entries are requested before the index phase (chunk 0 starts at
    // entry 0 of every row) so their latency hides behind it
    constexpr int U = 16;
    struct GrpU {  // 64 U entries of the row: gene ids and values
        int g_[U];
        float x_[U];
        MMVAE_DEV int g(int u) const { return g_[u]; }
        MMVAE_DEV float x(int u) const { return x_[u]; }
    };
    struct GrpP {  // 64 U packed entries
        uint32_t w_[U];
        MMVAE_DEV int g(int u) const { return (int)(w_[u] >> 16); }
        MMVAE_DEV float x(int u) const { return (float)(w_[u] & 0xffffu); }
    };
    using Grp = typename std::conditional<PK, GrpP, GrpU>::type;
    Grp gA, gB;  // gB: PK only (the group after gA, in flight with it)
    auto load = [&](Grp& G, int jA, int jB) {
#pragma unroll
        for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads
            const int j = min(jA + 64 * u + lane, max(jB - 1, 0));
            if constexpr (PK) {
                G.w_[u] = pk[s + j];
            } else {
                G.g_[u] = col[s + j];
                G.x_[u] = val[s + j];
            }
        }
    };
    if (!dbg_bit(dbg, 512)) {
        load(gA, 0, rn);
        if constexpr (PK) load(gB, 64 * U, rn);
    }
    // the row's tile pointers: all loads of a group of 8 issued before the first LDS store
    {
        const int32_t* src = rtp + c * (int64_t)(NT + 1);
        for (int t0 = 0; t0 <= NT; t0 += 512) {
            int32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[min(t0 + 64 * u + lane, NT)];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (t0 + 64 * u + lane <= NT) srt[w * (NT + 1) + t0 + 64 * u + lane] = v[u];
        }
    }
    if (tid == 0) scarry = 0;
    __syncthreads();
    // per tile: the rows' prefix (sbase, before the tile offset) and the tile count (into tw)
    for (int t = tid; t < NT; t += 1024) {
        int32_t acc = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int32_t a0 = srt[r * (NT + 1) + t], a1 = srt[r * (NT + 1) + t + 1];
            sbase[r * NT + t] = acc - a0;
            acc += a1 - a0;
        }
        tw[t] = acc;
    }
    __syncthreads();
    // exclusive scan of the tile counts in chunks of 1024 tiles; tw[NT] = the block's total
    for (int t0 = 0; t0 <= NT; t0 += 1024) {
        const int t = t0 + tid;
        const int32_t v = (t < NT) ? tw[t] : 0;
        int32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        int32_t carry = scarry;
        for (int i = 0; i < w; ++i) carry += wsum[i];
        if (t <= NT) tw[t] = carry + incl - v;
        __syncthreads();
        if (tid == 0) {
            int32_t tot = 0;
            for (int i = 0; i < 16; ++i) tot += wsum[i];
            scarry += tot;
        }
        __syncthreads();
    }
    for (int t = tid; t <= NT; t += 1024) toff[(int64_t)wb * (NT + 1) + t] = tw[t];
    for (int i = tid; i < 16 * NT; i += 1024) sbase[i] += tw[i % NT];
    __syncthreads();
    if (dbg_bit(dbg, 512)) return;  // diagnostic: index phase only (lists invalid)
    const int64_t base = seg[wb];
    const int32_t* sb = sbase + w * NT;
    const int32_t* rt = srt + w * (NT + 1);
    // chunk bounds: the largest tB with tw[tB] - tw[tA] <= cap (a tile holds <= 1024 entries)
    auto chunk_end = [&](int tA) {
        int lo = tA + 1, hi = NT;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (tw[mid] - tw[tA] <= cap) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    // software pipeline over chunks: the next chunk's first 1024 entries of the row are loaded
    // while the current chunk streams out
    // NB (dotw != null): the raw-count dots of depth and nu_enc (nb.hh:448, 498) ride along,
    // every entry of the row passes through this wave exactly once
    const bool dots = dotw != nullptr && !dbg_bit(dbg, 4096);  // 4096: diagnostic, dots skipped
    float dpre = 0.f, dhn[HMAX];
#pragma unroll
    for (int h = 0; h < HMAX; ++h) dhn[h] = 0.f;
    auto drop = [&](const Grp& G, int j0, int jB, int cb) {  // masked LDS stores at the final positions
        float2 wv[U];
        if (dots) {  // every weight gather of the group in flight at once (clamped gene ids)
#pragma unroll
            for (int u = 0; u < U; ++u) wv[u] = dotw[(unsigned)G.g(u) < (unsigned)D ? G.g(u) : 0];
        }
        // every tile-base lookup first (the clamped loads give real gene ids, so each index is in
        // range), then the masked stores: a lookup inside each store's branch waited for its own
        // LDS round trip, sixteen in a row
        int pos[U];
#pragma unroll
        for (int u = 0; u < U; ++u) pos[u] = sb[min(G.g(u) >> 6, NT - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = j0 + 64 * u + lane;
            if (j < jB) {
                const uint32_t p = (uint32_t)((w << 6) | (G.g(u) & 63));
                if constexpr (XM) stage[pos[u] + j - cb] = uint2{p, __float_as_uint(G.x(u))};
                else stage[pos[u] + j - cb] = p | ((uint32_t)G.x(u) << 10);
            }
        }
        if (dots) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool in = j0 + 64 * u + lane < jB;
                const float xv = in ? G.x(u) : 0.f;
                dpre = fmaf(xv, wv[u].x, dpre);
                dhn[0] = fmaf(xv, wv[u].y, dhn[0]);
                for (int h = 1; h < H; ++h)
                    if (in) dhn[h < HMAX ? h : 0] = fmaf(xv, Wne[(int64_t)h * D + G.g(u)], dhn[h < HMAX ? h : 0]);
            }
        }
    };
    int tA = 0, tB = NT > 0 ? chunk_end(0) : 0;
    while (tA < NT) {
        const int cb = tw[tA], cnt = tw[tB] - cb;
        const int jA = rt[tA], jB = rt[tB];
        if constexpr (PK) {
            // gA, gB hold the chunk's first two groups; each is refilled two groups ahead
            for (int j0 = jA; j0 < jB; j0 += 2 * 64 * U) {
                drop(gA, j0, jB, cb);
                if (j0 + 2 * 64 * U < jB) load(gA, j0 + 2 * 64 * U, jB);
                if (j0 + 64 * U < jB) drop(gB, j0 + 64 * U, jB, cb);
                if (j0 + 3 * 64 * U < jB) load(gB, j0 + 3 * 64 * U, jB);
            }
        } else {
            drop(gA, jA, jB, cb);
            for (int j0 = jA + 64 * U; j0 < jB; j0 += 64 * U) {  // rows with more than 1024 entries in the chunk
                load(gA, j0, jB);
                drop(gA, j0, jB, cb);
            }
        }
        lds_barrier();
        const int tC = tB < NT ? chunk_end(tB) : NT;
        if (tB < NT) {  // next chunk in flight during the stream-out
            load(gA, rt[tB], rt[tC]);
            if constexpr (PK) load(gB, rt[tB] + 64 * U, rt[tC]);
        }
        uint32_t* dst = ents + base + cb;
        if (!dbg_bit(dbg, 8192)) {  // 8192: diagnostic, stream-out skipped (lists invalid)
            if constexpr (XM) {
                float* dx = reinterpret_cast<float*>(ents) + xoff + base + cb;
                for (int i = tid; i < cnt; i += 1024) {
                    const uint2 a = stage[i];
                    dst[i] = a.x;
                    dx[i] = __uint_as_float(a.y);
                }
            } else {
                // 16-byte stores (four entries each) from the first 16-byte-aligned entry on
                const int head = min(cnt, (int)((4 - ((base + cb) & 3)) & 3)), n4 = (cnt - head) >> 2;
                if (tid < head) dst[tid] = stage[tid];
                uint4* d4 = reinterpret_cast<uint4*>(dst + head);
                for (int i = tid; i < n4; i += 1024) {
                    const int k = head + 4 * i;
                    d4[i] = uint4{stage[k], stage[k + 1], stage[k + 2], stage[k + 3]};
                }
                const int rest = head + 4 * n4;
                if (tid < cnt - rest) dst[rest + tid] = stage[rest + tid];
            }
        }
        lds_barrier();  // stage reusable (the stores carry register copies)
        tA = tB;
        tB = tC;
    }
    if (dots) {
        dpre = wave_sum(dpre);
        for (int h = 0; h < H; ++h) dhn[h < HMAX ? h : 0] = wave_sum(dhn[h < HMAX ? h : 0]);
        if (lane == 0) {
            float* o = rowdots + (int64_t)b * (1 + H);
            o[0] = dpre;
            for (int h = 0; h < H; ++h) o[1 + h] = dhn[h < HMAX ? h : 0];
        }
    }
}

hipError_t build_batch_lists(Engine* e, int64_t B, const float2* dotw, const float* Wne, float* rowdots) {
    const int64_t Bp = pad_rows(B), WB = Bp / 16;
    ScopedTimer tm(e, "k_batch_lists");
    const size_t tab = sizeof(int32_t) * ((size_t)e->NT + 1 + 16 * ((size_t)e->NT + 1) + 16 * (size_t)e->NT);
    if (tab + 8 * 1024 > 160 * 1024) return hipErrorInvalidValue;  // D beyond ~75k genes
    const EntList L = ent_list(e);
    const size_t esz = L.xoff ? sizeof(uint2) : sizeof(uint32_t);
    const int cap = (int)std::min<size_t>(COPY_CAP_MAX, (160 * 1024 - 256 - tab) / esz) & ~3;  // 256: static LDS
    const bool pk = !L.xoff && e->pk_on && e->d_pk;  // the packed dataset (counts below 2^16)
    auto kern = L.xoff ? k_batch_lists<true, false> : pk ? k_batch_lists<false, true> : k_batch_lists<false, false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)WB), dim3(1024), esz * (size_t)cap + tab, e->stream, e->d_cells, e->d_rowptr, e->d_col,
                       e->d_val, e->d_pk, e->d_rtp, e->d_seg, (int)e->NT, cap, e->d_toff,
                       reinterpret_cast<uint32_t*>(e->d_ents), L.xoff,
#ifdef MMVAE_DIAG
                       [] { const char* v = std::getenv("MMVAE_DBG"); return v ? std::atoi(v) : 0; }(),
#else
                       0,
#endif
                       dotw, Wne,
                       (int)e->H, (int)e->D, rowdots, e->d_ss, e->d_ticket);
    return hipGetLastError();
}

}  // namespace mmvae
