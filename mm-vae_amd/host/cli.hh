// Options of the drop-in CLIs: the reference's four option structs (mmvae_options_t,
// training_options_t, nbvae_options_t / vmf_options_t; mmvae.hh:31-56, mmvae_alg.hh:14-34,
// nb.hh:53-71, vmf.hh:54-72) with their defaults, plus the engine's own.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mmvae_host.h"

namespace mmvae_host {

struct CliOptions {
    CliOptions() { mmvae_train_opts_default(&train); }
    // mmvae_options_t
    std::string mtx, idx, out, row, col, annot, covar_mtx, covar_idx;
    // training_options_t (lr here; the rest in `train`)
    float lr = 1e-3f;
    mmvae_train_opts train;
    // model options
    std::vector<int64_t> enc_layers, dec_layers;
    int64_t latent = 2;     // --mean_latent / --latent (nb.hh:59, vmf.hh:60)
    int64_t H = 1, R = 1;   // --overdisp_encoding, --overdispersion_latent (nb.hh:60-61)
    float kappa_min = .1f, kappa_max = 10.f;  // vmf.hh:61-62
    bool relu = false;
    // engine
    uint64_t seed = 42;
    std::string dtype = "f32";
    int device = -1;
    int threads = 0;
    bool csr_cache = true;
    bool verbose = true;
    bool help = false;
    int mm_rc = 0;  // parse_mmvae_options' result (EXIT_FAILURE: missing mtx / out)
};

int parse_options(int argc, const char** argv, int model, CliOptions& o);
const char* usage_text(int model);
// --dtype spelling -> MMVAE_DTYPE_*, -1 when unknown
int dtype_code(const std::string& s);
int run_cli(int argc, const char** argv, int model);

}  // namespace mmvae_host
