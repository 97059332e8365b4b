/* mmvae_host.h — C-ABI of the host-side runtime around the HIP engine (libmmvae_host.so).
 *
 * The reference's host path is C++ templates: the BGZF MatrixMarket mini-batch reader
 * (mtx_data_block_t, include/mmvae_io.hh:49-290, over mmutil_bgzf_util.hh:53-151) and the
 * training driver train_vae_model (include/mmvae_alg.hh:200-333) with its recorder
 * (include/models/nb.hh:569-662, vmf.hh:457-551).  On MI355X the dataset lives in HBM for the
 * whole run, so the reader becomes a one-time parallel loader into a cell-major CSR
 * (mmvae_mtx_read) and the driver a C++ loop over the engine C-ABI (mmvae_train).
 * Conventions as in mmvae_capi.h: 0 = success, negative MMVAE_E_* on failure with a message
 * from mmvae_host_last_error(); buffers returned in mmvae_csr are owned by the library and
 * released with mmvae_csr_free.
 */
#ifndef MMVAE_HOST_H_
#define MMVAE_HOST_H_

#include <stdint.h>

#include "mmvae_capi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Cell-major CSR of a genes x cells MatrixMarket matrix: row = cell (MatrixMarket column),
 * col = gene (0-based, strictly increasing within a row; duplicate entries: the last one in
 * file order wins, as the reference's dense scatter does, mmvae_io.hh:115-123). */
typedef struct mmvae_csr {
    int64_t N;        /* cells  = MatrixMarket columns (mtx_data_block_t::ntot, mmvae_io.hh:74) */
    int64_t D;        /* genes  = MatrixMarket rows (nfeature, mmvae_io.hh:73) */
    int64_t nnz;
    int64_t* rowptr;  /* [N + 1] */
    int32_t* col;     /* [nnz] */
    float* val;       /* [nnz] */
} mmvae_csr;

/* Read a MatrixMarket coordinate file — plain text, gzip, or BGZF (blocks inflated in
 * parallel) — with `threads` workers (<= 0: all hardware threads).  Replaces
 * mtx_data_block_t::init + read (mmvae_io.hh:208-245, 258-290) and visit_bgzf_block's
 * triplet parser (mmutil_bgzf_util.hh:53-151: 1-based, '%' comment lines and lines with
 * fewer than three fields skipped). */
int mmvae_mtx_read(const char* path, int threads, mmvae_csr* out);
/* Binary CSR cache (little-endian: magic "MMVAECSR", N, D, nnz, rowptr, col, val). */
int mmvae_csr_save(const char* path, const mmvae_csr* csr);
int mmvae_csr_load(const char* path, mmvae_csr* out);
void mmvae_csr_free(mmvae_csr* csr);
/* Dense [N][C] covariates from a MatrixMarket file (rows = covariate, columns = cells). */
int mmvae_mtx_read_dense_t(const char* path, int threads, int64_t* N, int64_t* C, float** out);
void mmvae_free(void* p);
/* The all-ones covariate file the CLIs write when --covar is absent
 * (create_ones_like, mmvae_io.hh:292-310): a 1 x N gzip MatrixMarket. */
int mmvae_mtx_write_ones(const char* path, int64_t N);
/* ${mtx}.index (build_mmutil_index, mmutil_index.hh:138-190): for a column-sorted BGZF
 * MatrixMarket file, the BGZF virtual offset of every column's first line as gzip text
 * "col voff" lines (0-based columns).  index_file NULL or "" -> mtx + ".index".  An existing
 * index is kept.  Errors as the reference: not BGZF, columns not sorted, last column missing. */
int mmvae_mtx_build_index(const char* mtx, const char* index_file);
/* read_mmutil_index (mmutil_index.hh:192-228): *voff [max col + 1] (free with mmvae_free),
 * missing columns back-filled with the next column's offset. */
int mmvae_mtx_read_index(const char* index_file, int64_t** voff, int64_t* ncol);
/* A cell-major CSR as a genes x cells BGZF MatrixMarket file, sorted by cell (bench / tests). */
int mmvae_mtx_write_csr(const char* path, const mmvae_csr* csr);
const char* mmvae_host_last_error(void);

/* ---- training driver (mmvae_alg.hh:200-333) ---------------------------------------------- */
typedef struct mmvae_train_opts {
    int64_t batch_size;   /* --batch_size (mmvae.hh:35, default 100) */
    int64_t max_epoch;    /* --max_epoch (mmvae_alg.hh:21, default 101) */
    int64_t nboot;        /* --nboot (mmvae_alg.hh:20, default 3) */
    int64_t recording;    /* --recording (mmvae_alg.hh:22, default 10) */
    float kl_discount;    /* --kl_discount (mmvae.hh:36, .1) */
    float kl_max;         /* --kl_max (1) */
    float kl_min;         /* --kl_min (.01) */
    uint64_t seed;        /* bootstrap resampling seed (the reference draws from random_device) */
    const char* out;      /* output header for the recorder files; NULL = no recorder */
    int32_t verbose;      /* per-epoch progress lines on stderr */
    int32_t rank, world;  /* data parallel: this process's shard of every batch (1 = single GPU) */
} mmvae_train_opts;

void mmvae_train_opts_default(mmvae_train_opts* o);
/* Bootstrap index j of resample `boot` of batch `b` in epoch `epoch`: uniform on [0, B)
 * (replaces the mt19937 uniform_int_distribution of mmvae_alg.hh:244,292-293 by a
 * counter-based generator so every rank, and the Python tests, draw the same indices). */
int64_t mmvae_ridx(uint64_t seed, int64_t epoch, int64_t batch, int64_t boot, int64_t j, int64_t B);
/* Run the training loop on an engine whose dataset (and covariates) are uploaded: per epoch,
 * per batch of the contiguous cells (b B + j) % N: one train-mode forward for the reported
 * loss, then nboot x (bootstrap resample, forward, backward, clip, Adam); recorder outputs
 * every `recording` epochs.  scores_out (nullable, [max_epoch]) receives the per-epoch loss
 * (sum_b loss_b B / (B nbatch), mmvae_alg.hh:268-320). */
int mmvae_train(mmvae_h h, const mmvae_train_opts* opts, float* scores_out);

#ifdef __cplusplus
}
#endif
#endif /* MMVAE_HOST_H_ */
