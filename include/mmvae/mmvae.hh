// mmvae.hh — the drop-in umbrella header of the MI355X engine for code written against the
// reference's include/mmvae.hh (+ mmvae_alg.hh / models' option headers):
//
//   * the option structs and parsers, same names and semantics (options.hh);
//   * the engine C-ABI (mmvae_capi.h): the model, optimiser, dataset and the ELBO step that the
//     reference builds from LibTorch modules (nbvae_t / vmf_vae_t + torch::optim::Adam);
//   * the host runtime C-ABI (mmvae_host.h): the MatrixMarket loader, ${mtx}.index and the
//     train_vae_model loop (mmvae_alg.hh:200-333) as mmvae_train.
//
// Header-only and torch-free; include operators.hh as well for the lbessel autograd op.
#ifndef MMVAE_DROPIN_HH_
#define MMVAE_DROPIN_HH_

#include "../mmvae_capi.h"
#include "../mmvae_host.h"
#include "options.hh"

// mmvae_options_t + nbvae/vmf options + training options -> engine cfg (the constructor
// arguments of nbvae_t, src/nb_vae_main.cc:103-112, and vmf_vae_t, src/vmf_vae_main.cc:100-107)
inline mmvae_cfg mmvae_cfg_from_nb(const mmvae::nb::nbvae_options_t& nb, const training_options_t& tr, int64_t D, int64_t C,
                                   int64_t batch_size) {
    mmvae_cfg c;
    mmvae_cfg_default(&c, MMVAE_MODEL_NB);
    c.D = D;
    c.C = C;
    c.K = nb.mean_latent;
    c.H = nb.overdispersion_encoding;
    c.R = nb.overdispersion_latent;
    c.max_batch = batch_size;
    c.lr = tr.lr;
    c.relu = nb.do_relu ? 1 : 0;
    c.n_enc_hidden = (int32_t)nb.mean_encoding_layers.size();
    c.n_dec_hidden = (int32_t)nb.mean_decoding_layers.size();
    for (size_t i = 0; i < nb.mean_encoding_layers.size() && i < 4; ++i) c.enc_hidden[i] = (int32_t)nb.mean_encoding_layers[i];
    for (size_t i = 0; i < nb.mean_decoding_layers.size() && i < 4; ++i) c.dec_hidden[i] = (int32_t)nb.mean_decoding_layers[i];
    return c;
}

inline mmvae_cfg mmvae_cfg_from_vmf(const mmvae::vmf::vmf_options_t& v, const training_options_t& tr, int64_t D, int64_t C,
                                    int64_t batch_size) {
    mmvae_cfg c;
    mmvae_cfg_default(&c, MMVAE_MODEL_VMF);
    c.D = D;
    c.C = C;
    c.K = v.latent;
    c.max_batch = batch_size;
    c.lr = tr.lr;
    c.kappa_min = v.kappa_min;
    c.kappa_max = v.kappa_max;
    c.relu = v.do_relu ? 1 : 0;
    c.n_enc_hidden = (int32_t)v.encoding_layers.size();
    c.n_dec_hidden = (int32_t)v.decoding_layers.size();
    for (size_t i = 0; i < v.encoding_layers.size() && i < 4; ++i) c.enc_hidden[i] = (int32_t)v.encoding_layers[i];
    for (size_t i = 0; i < v.decoding_layers.size() && i < 4; ++i) c.dec_hidden[i] = (int32_t)v.decoding_layers[i];
    return c;
}

#endif  // MMVAE_DROPIN_HH_
