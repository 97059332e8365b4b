// Internal state of one mmvae engine handle (one HIP device, one stream).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include <type_traits>

#include "../../include/mmvae_capi.h"
#include "common.hpp"
#include "graph_key.hpp"

namespace mmvae {

// environment switch: `name` is set to exactly `value`
inline bool getenv_is(const char* name, const char* value) {
    const char* v = std::getenv(name);
    return v && std::strcmp(v, value) == 0;
}

// Batch rows are padded to whole 128-row blocks: decoder pass B runs 128 rows per workgroup,
// the other row-blocked kernels 64 (padding rows point at the dataset's empty row N).
static constexpr int64_t ROW_ALIGN = 128;
inline int64_t pad_rows(int64_t B) { return (B + ROW_ALIGN - 1) / ROW_ALIGN * ROW_ALIGN; }

struct ParamSlot {
    std::string name;
    std::vector<int64_t> shape;
    int64_t off = 0;     // offset into the flat registered buffer (registered) or frozen buffer
    int64_t numel = 0;
    bool registered = true;
};

// Per-step scalars staged with the batch (in the same H2D copy) and read by the kernels, so a
// captured step graph replays unchanged with each step's values: the Philox noise key (step,
// global row offset) and Adam's bias-corrected rates (optim/adam.cpp).
struct StepScalars {
    int64_t step_id, row_offset;
    float lr_bc1, inv_sqrt_bc2;
    int64_t ticket;  // the staging ticket: k_batch_lists writes it back once the block is copied
};

// launch shape of a captured step graph: replayed while every field matches

struct TimerRec {
    std::string name;
    double total_ms = 0;
    int64_t launches = 0;
};

// Device buffers are plain hipMalloc allocations owned by the engine.
struct Engine {
    mmvae_cfg cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // ---- shapes ----
    int64_t D = 0, DP = 0, NT = 0;  // genes, padded to 64, #64-gene tiles
    int64_t K = 0, KP = 0;          // latent, padded (32 or 64) over K, KE, KD
    // frozen hidden layers: KE = width of the big encoder GEMM's output (h0), E = input width of
    // the latent heads, KD = input width of the big decoder GEMM; the small chain layers between
    // (nce encoder layers, then ncd decoder layers) packed in d_chain (see Dims)
    int64_t KE = 0, E = 0, KD = 0;
    int nce = 0, ncd = 0;
    int ch_in[2 * MMVAE_MAX_HIDDEN] = {}, ch_out[2 * MMVAE_MAX_HIDDEN] = {}, ch_off[2 * MMVAE_MAX_HIDDEN] = {};
    std::string ch_w[2 * MMVAE_MAX_HIDDEN], ch_b[2 * MMVAE_MAX_HIDDEN];  // frozen slot names of every chain layer (bias "" for Angular)
    float* d_chain = nullptr;
    std::string fz_enc_w, fz_enc_b, fz_dec_w, fz_dec_b;  // the big frozen layers' slots
    int64_t C = 1, H = 1, R = 1;
    int64_t Bmax = 0, Bpad = 0;     // max rows, padded (pad_rows)
    int64_t nrb_max = 0;            // row blocks of 64 at Bmax

    // ---- dataset ----
    // N = rows of the device dataset the kernels index (resident: every cell; streamed: the
    // batch's Bpad rows, row Bpad empty); N_host = the caller's cells (cell ids are validated
    // against it)
    int64_t N = 0, nnz = 0, N_host = 0;
    int64_t* d_rowptr = nullptr;
    int32_t* d_col = nullptr;
    float* d_val = nullptr;
    float* d_covar = nullptr;  // [N+1][C], row N = zeros (padding rows)
    // streamed dataset (mmvae_stream_csr): the caller's CSR as mapped pinned host memory (device
    // pointers), and per staging slot the batch CSR the step gathers into; d_rowptr / d_col /
    // d_val / d_covar / d_rtp / d_cellnorm then view the current slot's set
    bool streamed = false;
    // C == 1 and every dataset row's covariate is 1 (no covariate file: the reference's default):
    // the decoder kernels fold the covariate Linear into per-gene constants (instances CM = 0)
    bool unit_covar = false;
    const int64_t* hs_rowptr = nullptr;
    const int32_t* hs_col = nullptr;
    const float* hs_val = nullptr;
    const float* hs_covar = nullptr;
    std::vector<void*> hs_registered;  // the engine's mapped pinned copies of the streamed arrays (hipHostFree)
    // packed entries (streamed, D <= 65536, every value a 16-bit integer count): one word per
    // entry, gene << 16 | count, in engine-owned mapped pinned memory — the gather moves 4 bytes
    // per entry over PCIe instead of 8 (MMVAE_STREAM_PACK=0: the caller's arrays)
    bool stream_index_step = false;     // prefetch mode: the batch's tile index built inside the step, not on gstream
    uint32_t* hs_packed = nullptr;      // host address of the packed copy
    const uint32_t* hs_packed_dev = nullptr;  // its device address
    size_t hs_packed_bytes = 0;         // > 0: mmap'd (pageable in the DMA mode; 2 MB pages under MMVAE_STREAM_THP=1)
    bool hs_packed_reg = false;         // the mmap is registered as mapped pinned memory (zero-copy gather)
    const int64_t* hh_rowptr = nullptr;  // the same arrays' host addresses (mmvae_get_rows)
    const int32_t* hh_col = nullptr;
    const float* hh_val = nullptr;
    struct BatchSet {
        int64_t* rowptr = nullptr;  // [Bpad + 2]
        int32_t* col = nullptr;     // [cap]
        float* val = nullptr;
        float* covar = nullptr;     // [Bpad + 1][C]
        int32_t* rtp = nullptr;     // [Bpad + 1][NT + 1]
        float* cellnorm = nullptr;  // [Bpad + 1] float2
        int64_t cap = 0;
    } bset[2];
    int64_t* h_brp_pin = nullptr;   // pinned: the staged batch rowptr [Bpad + 1] (streamed)
    // prefetched gather (streamed, default; MMVAE_STREAM_SYNC=1: in the step's stream): the
    // step's rows are gathered on gstream as soon as the step is staged, under the previous
    // step's kernels.  h_gcells[s]: slot s's dataset row ids (mapped, read by the gather; the
    // staged block then carries the identity), ev_gathered[s]: the gather done, the step waits;
    // ev_setfree[s]: the last step on batch set s done, the next gather into it waits
    bool stream_prefetch = false;
    hipStream_t gstream = nullptr;
    hipEvent_t ev_gathered[2] = {nullptr, nullptr}, ev_setfree[2] = {nullptr, nullptr};
    // DMA mode (packed copy, prefetch; MMVAE_STREAM_DMA=0 turns it off): the host packs the batch's rows into h_bpk[s]
    // (worker threads), one DMA-engine copy moves them to d_bpk[s], and the unpack kernel reads
    // HBM instead of mapped host memory
    bool stream_dma = false;  // set by mmvae_stream_csr
    uint32_t hs_cmax = 0;     // the packed copy's largest count
    bool stream_b3 = false;   // DMA mode, every count < 256 (MMVAE_STREAM_B3=1): 3-byte entries on the copy
    uint32_t* h_bpk[2] = {nullptr, nullptr};
    uint32_t* d_bpk[2] = {nullptr, nullptr};
    int64_t bpk_cap[2] = {0, 0};
    void* gpool = nullptr;  // stream.hip's host gather pool
    int64_t* h_gcells[2] = {nullptr, nullptr};
    const int64_t* d_brp = nullptr;
    size_t stage_bytes_res = 0;     // the resident path's staged block (streamed adds the rowptr)

    // ---- parameters ----
    std::vector<ParamSlot> slots;
    std::map<std::string, int> slot_index;
    int64_t P_reg = 0, P_frz = 0;
    float* d_params = nullptr;  // registered, LibTorch order
    float* d_grads = nullptr;
    float* d_m = nullptr;
    float* d_v = nullptr;
    float* d_frozen = nullptr;  // frozen Sequentials (f32, reference layout)
    int64_t adam_step = 0;
    bool frozen_dirty = true;
    bool have_grads = false;

    // prepared frozen operand copies (rebuilt when frozen params change)
    float* d_WeP_f = nullptr;   // [KP][DP] encoder weight, zero padded
    __bf16* d_WeP_b = nullptr;
    float* d_WdP_f = nullptr;   // [DP][KP] decoder weight (gene-major)
    __bf16* d_WdP_b = nullptr;
    uint8_t* d_WdP8 = nullptr;  // [DP][KP] decoder weight x wscale, e4m3 (fp8 mode)
    float wscale = 1.f;         // power-of-two scale of d_WdP8
    uint8_t* d_WeS8 = nullptr;  // [KP][DP] encoder weight / sd x escale, e4m3 (fp8 mode, k_prep)
    float* d_escale = nullptr;  // [2] the step's power-of-two scale of d_WeS8 and its inverse (k_enc_scale)
    float wemax = 0.f;          // max |W_enc| (frozen), the scale's bound
    float* d_WdT_f = nullptr;   // [KP][DP] decoder weight transposed
    __bf16* d_WdT_b = nullptr;

    // ---- per-step workspace ----
    int64_t* d_cells = nullptr;      // [Bpad] gathered dataset rows (-1 = padding)
    int64_t* h_cells_pin = nullptr;  // pinned staging
    int32_t* h_perm_pin = nullptr;   // pinned: original batch position of every (balanced) row
    int32_t* d_perm = nullptr;       // [Bpad]
    StepScalars* h_ss = nullptr;     // pinned: this step's scalars (end of the staging block)
    const StepScalars* d_ss = nullptr;
    bool perm_active = false;        // the last staged batch was reordered (noise keyed by d_perm)
    bool no_balance = false;         // MMVAE_NO_BALANCE at create (max-agreed over the ranks, comm_sync_capacity)
    std::vector<int32_t> cell_nnz;   // host copy of every cell's nonzero count (row balancing, lists)
    // per-step batch entry lists (batch.hip)
    // [ent_cap] uint2 of storage: the 32-bit entry words [0, ent_cap), and with ent_xm the float
    // values [ent_cap, 2 ent_cap) (tiles.hpp EntList / ListEntries)
    uint2* d_ents = nullptr;
    bool ent_xm = false;             // some dataset value is not an integer in [0, 2^22)
    int64_t ent_cap = 0;
    int64_t* d_seg = nullptr;        // [Bpad/16 + 1]
    int64_t* h_seg_pin = nullptr;    // pinned staging of seg
    int32_t* d_toff = nullptr;       // [Bpad/16][NT+1]
    float* d_eps = nullptr;          // [Bpad][K] + [Bpad][R]
    float* h_eps_pin = nullptr;
    float* d_gene = nullptr;         // per-gene prep (k_prep / k_vprep): [10][DP] floats
    float* d_mvec = nullptr;         // [DP/256][KP] partials of mvec (k_prep / k_vprep)
    int32_t* d_rtp = nullptr;        // [N+1][NT+1] per-cell tile pointers (dataset index; row N = empty)
    // resident data with D <= 65536: the packed copy gene << 16 | count [nnz] written by the dataset
    // index kernel; pk_on when every value is an integer count below 2^16 (k_batch_lists reads it)
    uint32_t* d_pk = nullptr;
    bool pk_on = false;
    float* d_cellnorm = nullptr;     // [N+1] float2: vMF row norms of log1p(x) (dataset index)
    float* d_rowx = nullptr;         // [Bpad][2+H]  pre_depth, lnorm2, hnu[H]
    float* d_rowxp = nullptr;        // [nsE][Bpad][1+H]  gene-split partials of depth(x), nu_enc(x)
    float* d_hpart = nullptr;        // [nsplitE][Bpad][KP]
    float* d_lat = nullptr;          // latent state, see LAT_* offsets
    float* d_zf = nullptr;           // [Bpad][KP]
    __bf16* d_zb = nullptr;
    float* d_lsep = nullptr;         // [nsplit][Bpad][2]
    float* d_rowB = nullptr;         // [nsplit][Bpad][2+R]
    float* d_WeS_f = nullptr;        // [KP][DP] encoder weight / sd (per step)
    __bf16* d_WeS_b = nullptr;
    float* d_rowfin = nullptr;       // [Bpad][2]: lse2, w E
    float* d_dzp = nullptr;          // [nsplit][Bpad][2][KP]
    float* d_dh = nullptr;           // [Bpad][KP]
    float* d_dhT_f = nullptr;        // [KP][Bpad]
    __bf16* d_dhT_b = nullptr;
    float* d_slabB = nullptr;        // [nrb][nqB][DP]
    float* d_slabC = nullptr;        // [nrb][1+C][DP]
    float* d_slabE = nullptr;        // [nrb][2+H][DP]
    float* d_lossp = nullptr;        // loss partials
    float* d_small = nullptr;        // latent-bwd WG partials
    float* d_smallg = nullptr;       // reduced small grads scratch (colsum_dh etc.)
    double* d_sumsq = nullptr;       // sum-of-squares partials
    int sq_parts = 0;                // > 0: the gradient kernels wrote that many partials (k_sumsq skipped)
    float* d_out = nullptr;          // [0] loss, [1] total norm (float)
    float* d_rowv = nullptr;         // vMF: [Bpad] cos_b = <y_b, r_b>
    float* d_vk = nullptr;           // vMF: kappa scalars (k_vkappa)
    float* h_out_pin = nullptr;

    int nsplit_e = 1, nsplit_d = 1;  // D-splits of encoder / decoder pass-B grids
    bool dec3 = false;               // NB x3: the three-waves-per-SIMD pass B (MMVAE_DEC3=1)
    int nsplit_f = 1;                // vMF decoder forward pass (4 workgroups per CU where it fits)
    int nsplit_b = 1;                // D-split of the encoder backward
    int nsplit_a = 1;                // D-split of decoder passes A / C
    int n_lat_wg = 1;                // latent kernels' workgroups
    int64_t klp_off = 0;             // offset of KL partials inside d_lossp
    hipEvent_t ev_staged = nullptr;  // the current slot's: its last step is done with the pinned block
    // staging tickets (fused path): the step's k_batch_lists stores the ticket of the block it
    // follows into h_ticket (mapped, coherent) — stream order puts it after the prep kernel's copy
    int64_t* h_ticket = nullptr;
    int64_t* d_ticket = nullptr;
    int64_t ticket_seq = 0;
    // double-buffered pinned staging: the host fills slot s while the step staged from slot s ^ 1
    // runs; h_cells_pin / h_seg_pin / h_perm_pin / h_ss / h_eps_pin / ev_staged view the current
    // slot.  A step graph copies from its slot's block, so each slot has its own graph.
    struct StageSlot {
        int64_t* block = nullptr;  // cells | seg | perm | StepScalars
        float* eps = nullptr;
        hipEvent_t ev = nullptr;
        // > 0: the slot is free once the device has written back this ticket (*h_ticket, mapped
        // memory, no event marker between steps); 0: free after ev (wide path, upload)
        int64_t ticket = 0;
        // captured step graphs of this slot by launch shape (the training loop alternates an eval
        // forward and bootstrap updates, and the last batch of an epoch is ragged)
        std::vector<std::pair<GraphKey, hipGraphExec_t>> graphs;
    };
    StageSlot slots2[2];
    int cur_slot = 0;
    float* d_tmp = nullptr;          // encode outputs
    float* d_tmp_ar = nullptr;       // host-value all-reduce staging
    int32_t* d_flag = nullptr;       // the ranks' agreement words (comm_capture_agree, comm_sync_capacity)
    int64_t n_tmp_ar = 0;

    // ---- comm ----
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1;
    // MMVAE_FORCE_COMM=1 at mmvae_comm_init: a 1-rank communicator still runs the data-parallel
    // exchange (buckets, flat all-reduce, their graph capture) — the one-GPU test of that path
    bool comm_force = false;
    // RCCL calls inside step graphs: opt-in, MMVAE_COMM_GRAPH=1 (read at mmvae_comm_init)
    bool comm_graph = false;
    // the gradient exchange runs (a communicator of > 1 rank, or a forced 1-rank one)
    bool comm_active() const { return comm && (world > 1 || comm_force); }
    // bucketed gradient all-reduce overlapped with the encoder backward:
    // bucket 0 = the decoder-side gene vectors (ready after decoder pass C), bucket 1 = the rest.
    // Each bucket is a list of contiguous [offset, count) ranges of the flat gradient.
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_bucket[2] = {nullptr, nullptr};
    hipEvent_t ev_comm_done = nullptr;
    std::vector<std::pair<int64_t, int64_t>> bucket_ranges[2];
    bool grads_reduced = false;
    uint64_t auto_step = 0;  // Philox step counter of mmvae_step / mmvae_eval
    size_t stage_bytes = 0;  // the per-step H2D staging block (cells | seg | perm)  // set by a model step that already all-reduced its buckets

    // ---- the wide path (wide.hip): shapes beyond the fused kernels' limits ----
    bool wide = false;
    struct WideState* wide_st = nullptr;

    // ---- step graphs (A17: one hipGraph per step, mmvae_graph_enable) ----
    bool graph_on = false;
    // set when a capture with the communicator attached failed (RCCL calls not capturable in
    // this runtime): later steps with the communicator run eagerly
    bool comm_graph_failed = false;
    uint64_t graph_gen = 0;          // bumped when a buffer a step graph points at is replaced
    // step graphs with a communicator (the default): the batch-dependent buffers (entry
    // lists, streamed batch sets and DMA buffers) were sized for the worst batch of every rank
    // (comm_sync_capacity), so no rank re-captures alone; reset when the dataset or communicator
    // changes
    bool cap_synced = false;
    int64_t graph_captures = 0, graph_replays = 0;

    // ---- timing ----
    bool timing = false;
    std::vector<TimerRec> timers;
    std::map<std::string, int> timer_index;
    struct Pending { int idx; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;

    // latent state layout (floats per row)
    int64_t lat_stride = 0;
    int64_t LAT_H = 0, LAT_MEAN = 0, LAT_A = 0, LAT_EPS = 0, LAT_NMEAN = 0, LAT_AN = 0,
            LAT_EPSN = 0, LAT_ZNU = 0, LAT_D = 0, LAT_W = 0, LAT_VALID = 0, LAT_HNU = 0;

    const ParamSlot* slot(const std::string& n) const {
        auto it = slot_index.find(n);
        return it == slot_index.end() ? nullptr : &slots[it->second];
    }
    float* preg(const std::string& n) const { return d_params + slot(n)->off; }
    float* greg(const std::string& n) const { return d_grads + slot(n)->off; }
    float* pfrz(const std::string& n) const { return d_frozen + slot(n)->off; }
};

// timing helpers (capi.hip)
void timer_begin(Engine* e, const char* name, hipEvent_t* a);
void timer_end(Engine* e, hipEvent_t a);

struct ScopedTimer {
    Engine* e;
    hipEvent_t a = nullptr;
    int idx = -1;
    ScopedTimer(Engine* e_, const char* name) : e(e_) {
        if (e->timing) timer_begin(e, name, &a);
    }
    ~ScopedTimer() {
        if (e->timing && a) timer_end(e, a);
    }
};

inline EntList ent_list(const Engine* e) {
    return EntList{reinterpret_cast<const uint32_t*>(e->d_ents), e->ent_xm ? e->ent_cap : 0};
}

// NB launchers (nb_kernels.hip)
hipError_t nb_prepare_frozen(Engine* e);
hipError_t nb_prep(Engine* e, int64_t B, int64_t n_total, float beta);
hipError_t vmf_prep(Engine* e, int64_t B, int64_t n_total, float beta);
// the staged block's copy for the prep kernel (nullptr src: already on the device)
struct StageCopy;
StageCopy stage_copy_args(Engine* e);
// split gradient finalisation + bucketed all-reduce (capi.hip): true when the step runs the
// decoder-side / encoder-side gradient kernels separately (world > 1, or MMVAE_SPLIT_GRADS=1)
bool split_grads(const Engine* e);
// all-reduce gradient bucket b on the comm stream after the work queued so far on e->stream;
// bucket 1 also makes e->stream wait for both buckets.  No-op without a communicator.
hipError_t comm_bucket(Engine* e, int b);
// min-reduce every rank's step-graph capture outcome (eager): *agreed = 1 iff all captured
hipError_t comm_capture_agree(Engine* e, bool ok, const GraphKey& k, int* agreed);
// step graphs with a communicator: every batch-dependent buffer a step graph points at sized once
// for the largest batch any rank can stage, agreed over the communicator (capi.hip)
int comm_sync_capacity(Engine* e);
// slot s's DMA copy buffers of the streamed dataset (stream.hip)
hipError_t stream_bpk_alloc(Engine* e, int s, int64_t cap);
hipError_t nb_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps);
hipError_t nb_encode(Engine* e, int64_t B, float* d_mean, float* d_lnvar);
// vMF launchers (vmf_kernels.hip)
hipError_t vmf_prepare_frozen(Engine* e);
hipError_t vmf_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps);
hipError_t vmf_encode(Engine* e, int64_t B, float* d_mean, float* d_lnvar);
// encoder kernels shared by both models (nb_kernels.hip)
struct Dims;
hipError_t enc_forward_launch(Engine* e, const Dims& d, float* hpart);
// hidden-layer chain fields of Dims, and the chain buffer packing (nb_kernels.hip)
void dims_hidden(const Engine* e, Dims& d);
hipError_t pack_chain(Engine* e, bool angular_enc);
hipError_t build_batch_lists(Engine* e, int64_t B, const float2* dotw, const float* Wne, float* rowdots);

// Instantiate f(operand mode, latent padding) for the handle's dtype and KP: the mode is float
// (exact f32 MFMA), __bf16 (bf16 operands) or X3 (split-bf16, fp32-accurate products).
// (F8 = the fp8 mode, NB only; WITH_F8 = false maps it to bf16 for code that has no fp8 variant.)
template <bool WITH_F8 = true, class F>
hipError_t dispatch_mode(const Engine* e, F&& f) {
    using K32 = std::integral_constant<int, 32>;
    using K64 = std::integral_constant<int, 64>;
    const int dt = e->cfg.dtype;
    if (e->KP == 32) {
        if (dt == MMVAE_DTYPE_FP8) {
            if constexpr (WITH_F8) return f(F8{}, K32{});
            else return f(__bf16{}, K32{});
        }
        if (dt == MMVAE_DTYPE_BF16) return f(__bf16{}, K32{});
        if (dt == MMVAE_DTYPE_BF16X3) return f(X3{}, K32{});
        return f(float{}, K32{});
    }
    if (dt == MMVAE_DTYPE_FP8) {
        if constexpr (WITH_F8) return f(F8{}, K64{});
        else return f(__bf16{}, K64{});
    }
    if (dt == MMVAE_DTYPE_BF16) return f(__bf16{}, K64{});
    if (dt == MMVAE_DTYPE_BF16X3) return f(X3{}, K64{});
    return f(float{}, K64{});
}
// the wide path (wide.hip): dense [B, D] batch + generic f32-MFMA GEMMs for model shapes beyond
// the fused kernels (K or a hidden width > 64, > 4 hidden layers, C / H / R > 8, D > 75,264)
hipError_t wide_create(Engine* e);
void wide_destroy(Engine* e);
hipError_t wide_prepare_frozen(Engine* e);
hipError_t wide_forward_backward(Engine* e, int64_t B, int64_t n_total, float beta, bool update, bool use_eps);
hipError_t wide_encode(Engine* e, int64_t B, float* d_mean, float* d_lnvar);
typedef std::vector<std::pair<void*, size_t>> wide_poison_t;
wide_poison_t wide_poison_bufs(Engine* e);
// optimiser (opt_kernels.hip)
hipError_t opt_clip_adam(Engine* e);
// diagnostic: every CU's LDS filled with `byte` (mmvae_debug_poison)
hipError_t lds_poison(Engine* e, int byte);
void adam_scalars(const Engine* e, int64_t t, StepScalars* ss);
hipError_t synth_dataset(Engine* e, int64_t N, double lib, uint64_t seed, int64_t* nnz_out);
hipError_t build_dataset_index(Engine* e);
hipError_t index_rows(Engine* e, const int64_t* rowptr, const int32_t* col, const float* val, int64_t N, int32_t* rtp,
                      float* cellnorm, hipStream_t st = nullptr);  // st: e->stream when null
// streamed dataset: point the dataset views at staging slot s's batch set, and the step's gather
// (after the staged block's copy) + batch index (stream.hip)
void stream_bind(Engine* e, int s);
hipError_t stream_gather(Engine* e);
hipError_t stream_prefetch(Engine* e);
hipError_t stream_step_done(Engine* e);
void stream_release(Engine* e);

}  // namespace mmvae

// the opaque C handle is the engine itself
struct mmvae_engine : public mmvae::Engine {};
