/* mmvae_capi.h — C-ABI of the MI355X-native mmvae training engine.
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * (YPARK/mm-vae) has no FFI: its boundary is the C++ template
 *   train_vae_model<MODEL_PTR, VISITOR, DATA_BLOCK, LOSS>(...)   include/mmvae_alg.hh:200-210
 * whose per-batch body (mmvae_alg.hh:264-311) gathers a batch (DATA_BLOCK::read,
 * include/mmvae_io.hh:208-245), runs MODEL::forward + LOSS + autograd backward +
 * clip_grad_norm_ + Adam.  Every entry point below replaces one piece of that body; the
 * comment on each names the reference interface it replaces.  A host loop mirroring
 * train_vae_model (mm-vae_amd/host/) and the Python binding (mm-vae_amd/py/) sit on top.
 *
 * Conventions: plain C types; every call returns 0 on success or a negative MMVAE_E_*
 * code, with a message retrievable by mmvae_last_error(h) (no exceptions cross the ABI,
 * replacing the reference's CHK/ASSERT -> exit(1), include/utils/util.hh:35-56).  Host
 * buffers are caller-owned; device memory is owned by the handle.  One host thread per
 * handle.  All work is stream-ordered on the handle's HIP stream; the only host syncs are
 * mmvae_sync() and non-NULL scalar outputs of mmvae_run().
 */
#ifndef MMVAE_CAPI_H_
#define MMVAE_CAPI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mmvae_engine* mmvae_h;

enum {
    MMVAE_OK = 0,
    MMVAE_E_ARG = -1,    /* invalid argument / shape mismatch */
    MMVAE_E_HIP = -2,    /* HIP runtime failure (no device, OOM, launch error) */
    MMVAE_E_STATE = -3,  /* call out of order (e.g. step before upload) */
    MMVAE_E_COMM = -4,   /* RCCL failure */
    MMVAE_E_NAME = -5    /* unknown parameter name */
};

enum { MMVAE_MODEL_NB = 0, MMVAE_MODEL_VMF = 1 };
/* most hidden encoder / decoder layers of a cfg (the reference takes any number) */
#define MMVAE_MAX_HIDDEN 16
/* Operand precision of the encoder/decoder GEMMs; every epilogue, reduction, gradient and
 * optimiser update is fp32.
 *   F32     exact f32 MFMA (v_mfma_f32_16x16x4_f32): bitwise an fp32 FMA chain.
 *   BF16    bf16 operands, f32 accumulate (loss within ~2e-3 of fp32).
 *   BF16X3  fp32-accurate split operands: v = hi + lo (two bf16), each product accumulated in f32
 *           as lo*hi + hi*lo + hi*hi on the bf16 MFMA (relative product error <= ~2^-16), at a
 *           fraction of the f32 MFMA's cost — the parity-grade production mode.
 *   FP8     (NB only; BASELINE configs[4]) the decoder logit GEMM z W_dec^T of all three decoder
 *           passes and the encoder GEMM log1p(x) (W_enc / sd)^T on the fp8 e4m3 MFMA (W_dec scaled
 *           once, W_enc / sd every step, by a power of two below the e4m3 range; z and log1p(x)
 *           converted as loaded; f32 accumulate); the backward (dz, encoder) GEMMs as BF16. */
enum { MMVAE_DTYPE_F32 = 0, MMVAE_DTYPE_BF16 = 1, MMVAE_DTYPE_BF16X3 = 2, MMVAE_DTYPE_FP8 = 3 };

typedef struct mmvae_cfg {
    int32_t model;       /* MMVAE_MODEL_NB (src/nb_vae_main.cc) / MMVAE_MODEL_VMF (src/vmf_vae_main.cc) */
    int32_t dtype;       /* MMVAE_DTYPE_* */
    int64_t D;           /* genes: data_dim, nb.hh:214 / vmf.hh:200 (= MatrixMarket rows) */
    int64_t C;           /* covariate dim: covar_dim (1 for the auto ones-file, nb_vae_main.cc:68-73) */
    int64_t K;           /* NB --mean_latent (nb.hh:59) / vMF --latent (vmf.hh:60) */
    int64_t H;           /* NB --overdisp_encoding (nb.hh:60); ignored for vMF */
    int64_t R;           /* NB --overdispersion_latent (nb.hh:61); ignored for vMF */
    int64_t max_batch;   /* largest B passed to mmvae_run on this handle */
    float lr;            /* --lr (mmvae_alg.hh:19) default 1e-3 */
    float weight_decay;  /* AdamOptions.weight_decay, mmvae_alg.hh:236: 1e-4 */
    float grad_clip;     /* clip_grad_norm_ max norm, mmvae_alg.hh:308 (always 1.0 there: Q7) */
    float kappa_min;     /* vMF --kappa_min (vmf.hh:61) */
    float kappa_max;     /* vMF --kappa_max (vmf.hh:62) */
    uint64_t seed;       /* Philox seed for the reparameterisation noise when none is injected */
    int32_t relu;        /* --relu: NB ReLU after each frozen encoder / hidden decoder Linear
                            (nb.hh:336-346, 372-373); vMF after each Angular encoder / hidden
                            decoder Linear (vmf.hh:342-352, 378-379).  NB with relu and >= 1
                            hidden encoder layer is the reference's construction error (Q2,
                            nb.hh:334-337): mmvae_create returns MMVAE_E_ARG. */
    int32_t n_enc_hidden;    /* NB --mean_encoding / vMF --encoding: hidden widths, <= MMVAE_MAX_HIDDEN layers */
    int32_t n_dec_hidden;    /* NB --mean_decoding / vMF --decoding */
    int32_t enc_hidden[MMVAE_MAX_HIDDEN];
    int32_t dec_hidden[MMVAE_MAX_HIDDEN];
} mmvae_cfg;

/* Fill a cfg with the reference defaults (mmvae_alg.hh:19-23, nb.hh:58-61, vmf.hh:59-63). */
void mmvae_cfg_default(mmvae_cfg* cfg, int32_t model);

/* Create an engine on HIP device `device`.  Replaces constructing nbvae_t / vmf_vae_t
 * (nb.hh:299-401, vmf.hh:307-389) plus the torch::optim::Adam of mmvae_alg.hh:234-237.
 * Parameters start at zero; load them with mmvae_set_param or mmvae_init_params.
 * Shapes: D, K, C, H, R >= 1 and at most MMVAE_MAX_HIDDEN hidden encoder / decoder layers of any
 * width >= 1 (the reference has no limits).  Models with D <= 75,264 genes, K <= 64,
 * C, H, R <= 8, at most 4 hidden layers per side and hidden widths <= 64 run on the fused tile
 * kernels; any other shape runs on the wide path (a dense [B, D] batch in HBM and a generic GEMM:
 * the gene GEMMs on the bf16 MFMA as BF16X3 split operands or plain BF16 per the handle's dtype,
 * exact f32 MFMA for F32 handles and the small layers; mmvae_path reports which).  FP8 for the NB
 * model only. */
int mmvae_create(const mmvae_cfg* cfg, int device, mmvae_h* out);
int mmvae_destroy(mmvae_h h);
/* Which step path the handle runs: 0 = the fused tile kernels, 1 = the wide path. */
int mmvae_path(mmvae_h h, int32_t* wide);
/* Message for the last failing call on h (h may be NULL for mmvae_create failures). */
const char* mmvae_last_error(mmvae_h h);

/* ---- dataset (HBM-resident) --------------------------------------------------------
 * Replaces mtx_data_block_t (mmvae_io.hh:49-141) for the data AND the covariate blocks:
 * instead of re-reading BGZF per batch, the whole cell-major CSR is uploaded once
 * (rows = cells = MatrixMarket columns, 0-based gene ids, sorted within a row).
 * covar: [N, C] row-major (NULL -> all ones, the reference's auto covariate). */
int mmvae_upload_csr(mmvae_h h, const int64_t* rowptr, const int32_t* col, const float* val,
                     int64_t N, int64_t D, const float* covar);
/* Host-resident dataset for data beyond HBM (the reference streams each batch from its BGZF
 * file, mtx_data_block_t::read, mmvae_io.hh:208-245): the caller's cell-major CSR (and covariates,
 * or NULL for ones) stays in host memory; the caller keeps the arrays alive and unchanged until
 * mmvae_destroy or the next upload / synth / stream (host threads read them there).  The caller's
 * memory is never page-locked: what the GPU reads over PCIe is an engine-owned mapped pinned copy
 * — of the row offsets (8 B per row) and covariates (4 C B per row) always, and of col / val
 * (8 B per nonzero) only in the unpacked case (non-integer values or D > 65536); for 16-bit integer
 * counts the packed copy (4 B per nonzero) replaces them.  So pinned host memory is 8 B per row +
 * 4 B (packed) or 8 B (unpacked) per nonzero beyond the caller's arrays.  Every
 * step's rows are gathered over PCIe into a per-step batch CSR in HBM (two slots, alternating with
 * the staging slots) and indexed; the gather runs on its own stream as soon as the step is staged,
 * under the previous step's kernels, and the step waits for it.  When D <= 65536 and every value
 * is a 16-bit integer count, the engine keeps a packed copy (4 bytes per entry): host threads pack
 * the step's rows into a pinned slot buffer, one DMA-engine copy moves it to HBM and the step
 * unpacks it (MMVAE_STREAM_DMA=0: a zero-copy gather kernel reads the copy over PCIe instead).
 * The kernels after the gather are the resident path's, on the batch's rows.  Results
 * are bit-identical to mmvae_upload_csr of the same data.  HBM holds O(B nnz_b) of the dataset
 * instead of O(N nnz). */
int mmvae_stream_csr(mmvae_h h, const int64_t* rowptr, const int32_t* col, const float* val,
                     int64_t N, int64_t D, const float* covar);
/* Dataset size after upload/synth (mtx_data_block_t::ntot / nfeature, mmvae_io.hh:73-74). */
int mmvae_dataset_size(mmvae_h h, int64_t* N, int64_t* D);
/* Device-side synthetic dataset (bench / smoke): SURVEY §8(d) count distribution. */
int mmvae_synth_csr(mmvae_h h, int64_t N, double lib_size, uint64_t seed, int64_t* nnz_out);
/* Copy dataset rows back to the host (recorder / CPU baseline sampling).  rowptr_out
 * [nrows+1]; col/val sized by *nnz_io (in: capacity, out: needed). */
int mmvae_get_rows(mmvae_h h, const int64_t* rows, int64_t nrows, int64_t* rowptr_out,
                   int32_t* col_out, float* val_out, int64_t* nnz_io);

/* ---- parameters (names = LibTorch named_parameters() keys) -------------------------
 * Registered parameters (Adam + clip) keep their reference keys, e.g.
 * "mu_representation_mean.weight"; the frozen, unregistered Sequentials (Q1) are exposed
 * as "mu_enc.mu_encoding.weight|bias", "mu_dec.mu_decoding.weight|bias" (NB) and
 * "z_enc.0.weight", "z_dec.decoding.weight|bias" (vMF). */
int mmvae_num_params(mmvae_h h, int32_t* count);
int mmvae_param_info(mmvae_h h, int32_t idx, const char** name, int64_t* numel, int32_t* registered);
/* Tensor shape of parameter idx (1 or 2 dims, LibTorch layout) — the recorder writes 2-D
 * tensors as matrices and 1-D ones as columns (write_tensor, mmvae_io.hh:11-28). */
int mmvae_param_shape(mmvae_h h, int32_t idx, int32_t* ndim, int64_t* shape2);
int mmvae_set_param(mmvae_h h, const char* name, const float* host, int64_t numel);
int mmvae_get_param(mmvae_h h, const char* name, float* host, int64_t numel);
/* Pre-clip gradient of a registered parameter from the last update step (parity tests). */
int mmvae_get_grad(mmvae_h h, const char* name, float* host, int64_t numel);
/* Reference-default initialisation (torch::nn::Linear kaiming-uniform(a=sqrt 5) bounds,
 * zeros/ones per nb.hh:312-315, vmf.hh:321-323) from a seeded generator. */
int mmvae_init_params(mmvae_h h, uint64_t seed);
/* Reset the Adam moments and step counter. */
int mmvae_reset_optimizer(mmvae_h h);

/* ---- the ELBO step ------------------------------------------------------------------ */
typedef struct mmvae_step_args {
    const int64_t* cell_ids;  /* host [B]: dataset rows of this rank's batch (mmvae_alg.hh:264-266) */
    const int64_t* ridx;      /* host [B] or NULL: bootstrap resample, rows = cell_ids[ridx]
                                 (mmvae_alg.hh:292-301) */
    int64_t B;                /* rows on this rank */
    int64_t n_total;          /* rows over all ranks = the loss divisor n (nb.hh:543); 0 -> B */
    int64_t row_offset;       /* global index of this rank's first row (noise key) */
    float beta;               /* KL weight, nb_loss_t / vmf_loss_t (nb_vae_main.cc:26-32) */
    const float* eps;         /* host noise or NULL (Philox): NB [B*K] then [B*R] (nb.hh:480-492);
                                 vMF [B*K] (vmf.hh:299) */
    uint64_t step_id;         /* Philox counter when eps == NULL */
    int32_t update;           /* 1: forward+backward+all-reduce+clip+Adam (mmvae_alg.hh:303-310)
                                 0: forward-only train-mode loss (the eval pass, Q12, :277-285) */
} mmvae_step_args;

/* Run one step.  loss_out (nullable) receives the rank-local loss (sum over this rank's
 * rows / n_total; sum over ranks = the reference's loss).  total_norm_out (nullable)
 * receives the clip_grad_norm_ total norm.  Non-NULL outputs synchronise the stream. */
int mmvae_run(mmvae_h h, const mmvae_step_args* args, float* loss_out, double* total_norm_out);

/* The SURVEY §8(b) single-GPU entry points, thin forms of mmvae_run with n_total = B,
 * row_offset = 0 and an internal step counter for the Philox noise (when eps == NULL):
 *   mmvae_step — one update step (mmvae_alg.hh:290-310: resample through ridx, forward,
 *                loss, zero_grad, backward, clip_grad_norm_, Adam::step);
 *   mmvae_eval — the forward-only train-mode loss of mmvae_alg.hh:277-285 (Q12).
 * loss_out (nullable) synchronises the stream. */
int mmvae_step(mmvae_h h, const int64_t* cell_ids, int64_t B, const int64_t* ridx_or_null, float beta,
               const float* eps_or_null, float* loss_out);
int mmvae_eval(mmvae_h h, const int64_t* cell_ids, int64_t B, float beta, const float* eps_or_null,
               float* loss_out);

/* Recorder encoder (nb.hh:419-431 encode_mu(x); vmf.hh:267-281 encode(x)): mean/lnvar
 * [B*K] row-major, no covariate, no noise. */
int mmvae_encode(mmvae_h h, const int64_t* cell_ids, int64_t B, float* mean, float* lnvar);
int mmvae_sync(mmvae_h h);

/* ---- data parallel (RCCL over xGMI) -------------------------------------------------
 * One process per GPU.  Rank 0 creates the 128-byte unique id and shares it out of band;
 * every rank then calls mmvae_comm_init.  Afterwards each update step SUM-all-reduces the
 * registered gradients before clip + Adam (new: the reference has no distribution). */
int mmvae_comm_unique_id(void* out128);
int mmvae_comm_init(mmvae_h h, int32_t rank, int32_t world, const void* id128);
/* id128 == NULL: local decomposition mode (no communicator) — the handle computes rank
 * `rank`'s shard of a world-`world` step, including terms only rank 0 contributes (the vMF
 * lbessel backward, Q3), and reduces nothing; mmvae_get_grad then returns the shard's
 * gradient and the clip + Adam that follow act on it alone.  Used to test the data-parallel
 * decomposition on one GPU. */
/* SUM-all-reduce n host floats across the ranks (RCCL on the handle's stream; a copy when
 * world == 1).  Used by the host driver for the reported per-batch loss. */
int mmvae_comm_allreduce(mmvae_h h, float* values, int64_t n);

/* ---- instrumentation -----------------------------------------------------------------
 * HIP-event timing of every kernel launch on the handle's stream. */
int mmvae_timing_enable(mmvae_h h, int32_t on);
int mmvae_timing_count(mmvae_h h, int32_t* n);
int mmvae_timing_get(mmvae_h h, int32_t idx, const char** name, double* total_ms, int64_t* launches);
int mmvae_timing_reset(mmvae_h h);
/* Diagnostics: copy n floats of an internal workspace (0 = encoder partials, 1 = decoder dz, 2 = pass-C slab
 * partials, 4 = encoder-backward slab; the MMVAE_DBG stamp builds write per-wave phase cycles there;
 * 3 = the last step's latent noise eps [Bpad][K], rows in the staged order) to the host. */
int mmvae_debug_copy(mmvae_h h, int32_t which, float* host, int64_t n);
/* Gene tiling of the handle's tile kernels (tests assert that a split walks many tiles):
 * out[0] = 64-gene tiles NT, out[1..3] = gene splits of the encoder forward / decoder pass B /
 * decoder passes A and C, out[4] = the encoder backward's (each split walks ceil(NT / splits)
 * tiles). */
int mmvae_tiling_info(mmvae_h h, int32_t* out5);
/* Test hook: fill every per-step workspace buffer with the byte `byte` (parameters, optimiser
 * state, the dataset and the frozen operand images are untouched).  A step writes everything it
 * reads there, so results must be bit-identical whatever the workspace held before. */
int mmvae_debug_poison(mmvae_h h, int32_t byte);
/* Step graphs (the reference's per-batch step, mmvae_alg.hh:254-333, as one hipGraph): with
 * on != 0, mmvae_run / mmvae_step / mmvae_eval capture their device work (staging copy, kernels,
 * loss readback) once per launch shape (batch size, n_total, beta, update, injected eps) and
 * replay it; the step's variable scalars (Philox step / row offset, Adam's bias corrections)
 * travel in the staged copy.  Results are identical to eager launches.  Not used while kernel
 * timing is on.  With an active communicator (world > 1, or a 1-rank one under
 * MMVAE_FORCE_COMM=1) the steps run eagerly with one flat all-reduce of the gradient, unless
 * MMVAE_COMM_GRAPH=1 was set at mmvae_comm_init: then the two RCCL bucket all-reduces are captured
 * into the step graph too.  Every rank then captures at the same steps: the graph key is a
 * function of values all ranks share (csrc/graph_key.hpp; a step needs B * world == n_total),
 * before the first such step the ranks agree (ncclMax) on the largest batch any of them can stage
 * (Bpad x the largest dataset row: Bpad * max_nnz * 8 B of entry lists, doubled plus pinned DMA
 * buffers for a streamed dataset) and size the batch-dependent buffers for it once; each capture's
 * outcome and key are agreed (ncclMin) before any rank launches; if any rank's capture failed or
 * its key differed, all of them run that handle's communicator steps eagerly from then on.
 * Dataset, communicator, graph and timing calls are then collective (every rank makes them at the
 * same point of its step sequence).
 * graph_stats: captures and replays so far. */
int mmvae_graph_enable(mmvae_h h, int32_t on);
int mmvae_graph_stats(mmvae_h h, int64_t* captures, int64_t* replays);

/* ---- operators.hh (vMF observation model scalars) ----------------------------------
 * lbessel(kappa, nu): piecewise log I_nu(kappa) approximation (operators.hh:49-101) with
 * P. Mineiro's fasterlgamma (fastgamma.h:58-60); its custom backward returns the Baricz
 * bound 0.5(sqrt(k^2 nu/(nu+1)+nu^2)+sqrt(k^2+nu^2))/k, ignoring the upstream gradient
 * (operators.hh:20-40).  Host scalars, fp32. */
float mmvae_lbessel(float kappa, float nu);
float mmvae_lbessel_grad(float kappa, float nu);
float mmvae_fasterlog(float x);     /* fastlog.h:75-85 */
float mmvae_fasterlgamma(float x);  /* fastgamma.h:58-60 */

#ifdef __cplusplus
}
#endif
#endif /* MMVAE_CAPI_H_ */
