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

// hidden widths of --mean_encoding / --mean_decoding (NB, nb.hh:331-379) or --encoding /
// --decoding (vMF, vmf.hh:338-385): every width up to MMVAE_MAX_HIDDEN layers per side is copied.
// A longer list keeps its true count in n_*_hidden (widths past the array are not stored), so
// mmvae_create rejects it with MMVAE_E_ARG instead of building a truncated model.
template <class V>
inline void mmvae_cfg_hidden_(mmvae_cfg& c, const V& enc, const V& dec) {
    c.n_enc_hidden = (int32_t)enc.size();
    c.n_dec_hidden = (int32_t)dec.size();
    for (size_t i = 0; i < enc.size() && i < (size_t)MMVAE_MAX_HIDDEN; ++i) c.enc_hidden[i] = (int32_t)enc[i];
    for (size_t i = 0; i < dec.size() && i < (size_t)MMVAE_MAX_HIDDEN; ++i) c.dec_hidden[i] = (int32_t)dec[i];
}

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
    mmvae_cfg_hidden_(c, nb.mean_encoding_layers, nb.mean_decoding_layers);
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
    mmvae_cfg_hidden_(c, v.encoding_layers, v.decoding_layers);
    return c;
}

#endif  // MMVAE_DROPIN_HH_
