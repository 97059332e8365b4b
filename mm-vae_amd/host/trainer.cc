// train_vae_model (include/mmvae_alg.hh:200-333) as a host loop over the engine C-ABI, with the
// reference's recorders (nb.hh:569-662 nbvae_recorder_t, vmf.hh:457-551 vmf_vae_recorder_t).
//
// Per epoch, per batch of the contiguous cells (b B + j) % N (mmvae_alg.hh:264-266):
//   1. one train-mode forward for the reported loss (Q12, :277-285)       mmvae_run(update = 0)
//   2. nboot x { ridx ~ U[0, B)^B; rows = batch[ridx]; forward; backward;  mmvae_run(update = 1)
//               clip_grad_norm_; Adam }                                    (:290-311)
//   3. every `recording` epochs: encode the batch (no covariate, :314-316) into the recorder
// then the epoch score sum_b loss_b B / (B nbatch) (:268-320) and the recorder files.
// Data parallel: every batch of B rows splits into `world` contiguous slices; each rank runs
// its slice (n_total = B, Philox noise keyed by the global row), the engine all-reduces the
// gradients, and the reported loss is all-reduced here.  Only rank 0 writes files.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mmvae_host.h"
#include "host_common.hh"

namespace mmvae_host {

// util.hh:97-107
static std::string zeropad(int64_t t, int64_t tmax) {
    std::string tt = std::to_string(t), tm = std::to_string(tmax);
    while (tt.size() < tm.size()) tt = "0" + tt;
    return tt;
}

// splitmix64 finaliser over a keyed counter
static uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Recorder {
    std::string header;
    int64_t max_epoch = 0, K = 0, N = 0;
    bool vmf = false;
    std::vector<float> mean, lnvar;  // [N][K]

    // write_data_stream (io.hh:545-557): one row per line, space separated, ostream %g
    static bool write_matrix(const std::string& path, const float* m, int64_t rows, int64_t cols) {
        TextWriter w;
        if (!w.open(path)) return false;
        std::string line;
        for (int64_t r = 0; r < rows; ++r) {
            line.clear();
            for (int64_t c = 0; c < cols; ++c) {
                if (c) line += ' ';
                line += fmt_g(m[r * cols + c]);
            }
            line += '\n';
            w.write(line);
        }
        return w.close();
    }

    int on_epoch(mmvae_h h, int64_t epoch) {
        const std::string tag = header + "_" + zeropad(epoch, max_epoch);
        const char* sfx = vmf ? ".latent" : ".mu";
        if (!write_matrix(tag + sfx + "_mean.gz", mean.data(), N, K) ||
            !write_matrix(tag + sfx + "_lnvar.gz", lnvar.data(), N, K))
            return fail(MMVAE_E_ARG, "recorder: cannot write " + tag + sfx + "_*.gz");
        int32_t np = 0;
        mmvae_num_params(h, &np);
        std::vector<float> buf;
        for (int32_t i = 0; i < np; ++i) {
            const char* name;
            int64_t numel;
            int32_t reg, nd;
            int64_t sh[2];
            mmvae_param_info(h, i, &name, &numel, &reg);
            mmvae_param_shape(h, i, &nd, sh);
            std::string key(name);
            // frozen Sequentials write their own named_parameters (nb.hh:597-607, vmf.hh:485-495)
            if (!reg) key = key.substr(key.find('.') + 1);
            buf.resize((size_t)numel);
            if (mmvae_get_param(h, name, buf.data(), numel)) return fail(MMVAE_E_STATE, mmvae_last_error(h));
            // write_tensor (mmvae_io.hh:11-28): 2-D as a matrix, 1-D as a column
            const bool ok = nd == 2 ? write_matrix(tag + "_" + key + ".gz", buf.data(), sh[0], sh[1])
                                    : write_matrix(tag + "_" + key + ".gz", buf.data(), numel, 1);
            if (!ok) return fail(MMVAE_E_ARG, "recorder: cannot write " + tag + "_" + key + ".gz");
        }
        return MMVAE_OK;
    }
};

}  // namespace mmvae_host

using namespace mmvae_host;

extern "C" {

void mmvae_train_opts_default(mmvae_train_opts* o) {
    std::memset(o, 0, sizeof(*o));
    o->batch_size = 100;  // mmvae.hh:35
    o->max_epoch = 101;   // mmvae_alg.hh:21
    o->nboot = 3;         // mmvae_alg.hh:20
    o->recording = 10;    // mmvae_alg.hh:22
    o->kl_discount = .1f;  // mmvae.hh:36-38
    o->kl_max = 1.f;
    o->kl_min = 1e-2f;
    o->seed = 42;
    o->out = nullptr;
    o->verbose = 0;
    o->rank = 0;
    o->world = 1;
}

int64_t mmvae_ridx(uint64_t seed, int64_t epoch, int64_t batch, int64_t boot, int64_t j, int64_t B) {
    uint64_t x = mix64(seed ^ mix64((uint64_t)epoch * 0x100000001B3ull + (uint64_t)batch));
    x = mix64(x ^ ((uint64_t)boot << 40) ^ (uint64_t)j);
    return (int64_t)(((unsigned __int128)x * (unsigned __int128)(uint64_t)B) >> 64);
}

int mmvae_train(mmvae_h h, const mmvae_train_opts* o, float* scores_out) {
    if (!h || !o) return fail(MMVAE_E_ARG, "train: null argument");
    int64_t N = 0, D = 0;
    mmvae_dataset_size(h, &N, &D);
    if (N < 1) return fail(MMVAE_E_STATE, "train: no dataset uploaded");
    const int64_t B = o->batch_size;
    const int world = o->world > 0 ? o->world : 1, rank = o->rank;
    if (B < 1 || B % world) return fail(MMVAE_E_ARG, "train: batch_size must be >= 1 and divisible by world");
    if (o->max_epoch < 0 || o->nboot < 0 || o->recording < 1) return fail(MMVAE_E_ARG, "train: bad epoch/nboot/recording");
    const int64_t Bl = B / world, r0 = (int64_t)rank * Bl;
    int64_t nbatch = N / B;
    if (nbatch * B < N) ++nbatch;

    // model kind and latent width from the parameter registry
    int32_t np = 0;
    mmvae_num_params(h, &np);
    bool vmf = false;
    int64_t K = 0;
    for (int32_t i = 0; i < np; ++i) {
        const char* name;
        int64_t numel;
        int32_t reg, nd;
        int64_t sh[2];
        mmvae_param_info(h, i, &name, &numel, &reg);
        mmvae_param_shape(h, i, &nd, sh);
        if (!std::strcmp(name, "ln_kappa")) vmf = true;
        if (!std::strcmp(name, "covar_encoding.bias")) K = numel;
    }
    Recorder rec;
    const bool record = o->out && rank == 0;
    if (record) {
        rec.header = o->out;
        rec.max_epoch = o->max_epoch;
        rec.K = K;
        rec.N = N;
        rec.vmf = vmf;
        rec.mean.assign((size_t)(N * K), 0.f);
        rec.lnvar.assign((size_t)(N * K), 0.f);
    }
    std::vector<int64_t> batch((size_t)B), cells((size_t)Bl), enc_ids;
    std::vector<float> em, el;
    uint64_t fwd = 0;  // Philox step counter: one per forward, identical on every rank
    if (o->verbose && rank == 0)
        std::fprintf(stderr, "[mmvae] Batch size = %lld, Number of batches = %lld\n", (long long)B, (long long)nbatch);
    for (int64_t epoch = 0; epoch < o->max_epoch; ++epoch) {
        // nb_loss_t / vmf_loss_t (nb_vae_main.cc:26-32): max(kl_max exp(-discount t), kl_min)
        const float t = (float)epoch;
        const float rate = o->kl_max * std::exp(-o->kl_discount * t);
        const float beta = std::max(rate, o->kl_min);
        float loss_epoch = 0.f;
        const bool rec_now = (epoch + 1) % o->recording == 0;
        for (int64_t b = 0; b < nbatch; ++b) {
            for (int64_t j = 0; j < B; ++j) batch[(size_t)j] = (b * B + j) % N;
            // 1. reported loss: train-mode forward on the batch (Q12)
            for (int64_t j = 0; j < Bl; ++j) cells[(size_t)j] = batch[(size_t)(r0 + j)];
            mmvae_step_args a;
            std::memset(&a, 0, sizeof(a));
            a.cell_ids = cells.data();
            a.B = Bl;
            a.n_total = B;
            a.row_offset = r0;
            a.beta = beta;
            a.step_id = fwd++;
            a.update = 0;
            float lb = 0.f;
            if (mmvae_run(h, &a, &lb, nullptr)) return fail(MMVAE_E_STATE, mmvae_last_error(h));
            if (world > 1 && mmvae_comm_allreduce(h, &lb, 1)) return fail(MMVAE_E_COMM, mmvae_last_error(h));
            loss_epoch += lb * (float)B;
            // 2. bootstrap updates
            for (int64_t boot = 0; boot < o->nboot; ++boot) {
                for (int64_t j = 0; j < Bl; ++j)
                    cells[(size_t)j] = batch[(size_t)mmvae_ridx(o->seed, epoch, b, boot, r0 + j, B)];
                a.step_id = fwd++;
                a.update = 1;
                if (mmvae_run(h, &a, nullptr, nullptr)) return fail(MMVAE_E_STATE, mmvae_last_error(h));
            }
            // 3. recorder (encode_mu / encode without covariate, model in eval mode)
            if (record && rec_now) {
                const int64_t mb = Bl;  // the handle's max_batch is at least the rank slice
                for (int64_t s = 0; s < B; s += mb) {
                    const int64_t n = std::min(mb, B - s);
                    enc_ids.assign(batch.begin() + s, batch.begin() + s + n);
                    em.resize((size_t)(n * K));
                    el.resize((size_t)(n * K));
                    if (mmvae_encode(h, enc_ids.data(), n, em.data(), el.data())) return fail(MMVAE_E_STATE, mmvae_last_error(h));
                    for (int64_t j = 0; j < n; ++j) {
                        const int64_t r = enc_ids[(size_t)j];
                        std::memcpy(&rec.mean[(size_t)(r * K)], &em[(size_t)(j * K)], sizeof(float) * (size_t)K);
                        std::memcpy(&rec.lnvar[(size_t)(r * K)], &el[(size_t)(j * K)], sizeof(float) * (size_t)K);
                    }
                }
            }
        }
        loss_epoch /= (float)(B * nbatch);
        if (scores_out) scores_out[epoch] = loss_epoch;
        if (o->verbose && rank == 0)
            std::fprintf(stderr, "[mmvae] [%20lld] %20g\n", (long long)(epoch + 1), (double)loss_epoch);
        if (record && rec_now) {
            if (mmvae_sync(h)) return fail(MMVAE_E_STATE, mmvae_last_error(h));
            int rc = rec.on_epoch(h, epoch);
            if (rc) return rc;
        }
    }
    return mmvae_sync(h) ? fail(MMVAE_E_STATE, mmvae_last_error(h)) : MMVAE_OK;
}

}  // extern "C"
