// oracle/_ref recipe (TEST INFRASTRUCTURE ONLY): a seeded driver around the reference's own
// NB-VAE model, compiled from the sources where they lie under /root/reference.
//
// `make -C oracle` writes oracle/_ref/nb_model.hh = include/models/nb.hh:1-563 (the options,
// nbvae_tImpl, nllik_loss / kl_loss / loss) closed with the two namespace braces and the
// include guard's #endif.  Lines 564-666 (nbvae_recorder_t, the only Eigen user of the
// file) are left out, so the model builds against this image's LibTorch 2.10 with no
// stand-in header.  The build output stays in oracle/_ref/ (git-ignored); nothing from the
// reference is copied into the repository.
//
// The step is the reference's own (include/mmvae_alg.hh:234-236,290-310):
//   Adam(parameters(), AdamOptions(lr).weight_decay(1e-4))
//   xboot = index_select(x, 0, ridx); cboot = index_select(c, 0, ridx)
//   y = model->forward(xboot, cboot); loss = nb::loss(xboot, y, beta)
//   adam.zero_grad(); loss.backward(); clip_grad_norm_(parameters(), 1.0); adam.step()
// and the eval forward (mmvae_alg.hh:274-285, Q12) plus the recorder's encode_mu(x)
// (nb.hh:419-431).  The noise the reference draws with randn_like (nb.hh:467, mu then nu:
// nb.hh:480-492) is recovered bit-exactly by the SURVEY Appendix-A re-seed: manual_seed(s)
// right before forward, then manual_seed(s) again and randn({B,K}), randn({B,R}).  The
// harness checks the recovery (decode_mu / decode_nu of the recovered z equal the forward's
// outputs bit for bit) and exits non-zero otherwise.
//
// I/O: `ref_nb_harness DIR`.  DIR/spec.txt:
//   D C K H R relu init_seed
//   n_enc e1 .. ; n_dec d1 ..
//   steps, then per step: B beta seed      (DIR/x{t}.f32 [B,D] batch rows, c{t}.f32 [B,C],
//                                           ridx{t}.i64 [B])
//   B beta seed                            (eval: xe.f32, ce.f32)
// If DIR/in/<name>.f32 exists it overwrites the reference's seeded init of that parameter
// (registered names, frozen ones as mu_enc.<name> / mu_dec.<name>).
// Outputs: DIR/out/<key>.bin (raw little-endian) + DIR/out/manifest.txt (key dtype dims...).
#include <torch/torch.h>

#include "util.hh"
#include "check.hh"
#include "std_util.hh"
#include "nb_model.hh"

#include <sys/stat.h>

#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

namespace mmvae { namespace nb {
TORCH_MODULE(nbvae_t); // nb.hh:664 (after the recorder, which is not compiled here)
}}

using torch::Tensor;

static std::string g_dir;
static std::ofstream g_manifest;

static Tensor read_f32(const std::string &path, std::vector<int64_t> shape)
{
    int64_t n = 1;
    for (auto s : shape) n *= s;
    auto t = torch::empty(shape, torch::kFloat32);
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) { std::fprintf(stderr, "missing %s\n", path.c_str()); std::exit(2); }
    if (std::fread(t.data_ptr<float>(), 4, n, f) != (size_t)n) { std::fprintf(stderr, "short %s\n", path.c_str()); std::exit(2); }
    std::fclose(f);
    return t;
}

static Tensor read_i64(const std::string &path, int64_t n)
{
    auto t = torch::empty({ n }, torch::kLong);
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f || std::fread(t.data_ptr<int64_t>(), 8, n, f) != (size_t)n) { std::fprintf(stderr, "bad %s\n", path.c_str()); std::exit(2); }
    std::fclose(f);
    return t;
}

static void dump(const std::string &key, Tensor t)
{
    t = t.detach().contiguous();
    const bool dbl = t.scalar_type() == torch::kFloat64;
    std::string fname = key;
    for (auto &ch : fname) if (ch == '/') ch = '@';
    FILE *f = std::fopen((g_dir + "/out/" + fname + ".bin").c_str(), "wb");
    std::fwrite(t.data_ptr(), dbl ? 8 : 4, t.numel(), f);
    std::fclose(f);
    g_manifest << key << ' ' << (dbl ? "f64" : "f32");
    for (auto s : t.sizes()) g_manifest << ' ' << s;
    g_manifest << '\n';
}

static bool exists(const std::string &p)
{
    FILE *f = std::fopen(p.c_str(), "rb");
    if (f) std::fclose(f);
    return f != nullptr;
}

int main(int argc, char **argv)
{
    if (argc != 2) { std::fprintf(stderr, "usage: %s DIR\n", argv[0]); return 2; }
    g_dir = argv[1];
    torch::set_num_threads(1); // fixed reduction order
    std::ifstream spec(g_dir + "/spec.txt");
    int64_t D, C, K, H, R, relu, init_seed;
    spec >> D >> C >> K >> H >> R >> relu >> init_seed;
    using namespace mmvae::nb;
    std::vector<mu_encoder_h_dim> enc;
    std::vector<mu_decoder_h_dim> dec;
    int n;
    spec >> n;
    for (int i = 0; i < n; ++i) { int w; spec >> w; enc.emplace_back(w); }
    spec >> n;
    for (int i = 0; i < n; ++i) { int w; spec >> w; dec.emplace_back(w); }

    torch::manual_seed(init_seed);
    nbvae_t model(data_dim(D), covar_dim(C), enc, dec, mu_encoder_r_dim(K), nu_encoder_h_dim(H),
                  nu_encoder_r_dim(R), relu != 0);

    // parameters: the reference's seeded init, overwritten from DIR/in where given
    std::vector<std::pair<std::string, Tensor>> all;
    for (auto &p : model->named_parameters()) all.emplace_back(p.key(), p.value());
    for (auto &p : model->mu_enc->named_parameters()) all.emplace_back("mu_enc." + p.key(), p.value());
    for (auto &p : model->mu_dec->named_parameters()) all.emplace_back("mu_dec." + p.key(), p.value());
    {
        torch::NoGradGuard ng;
        for (auto &kv : all) {
            const std::string path = g_dir + "/in/" + kv.first + ".f32";
            if (exists(path)) kv.second.copy_(read_f32(path, kv.second.sizes().vec()));
        }
    }
    ::mkdir((g_dir + "/out").c_str(), 0755);
    g_manifest.open(g_dir + "/out/manifest.txt");
    for (auto &p : model->named_parameters()) dump("init/" + p.key(), p.value());
    for (auto &p : model->mu_enc->named_parameters()) dump("frozen/mu_enc." + p.key(), p.value());
    for (auto &p : model->mu_dec->named_parameters()) dump("frozen/mu_dec." + p.key(), p.value());

    // mmvae_alg.hh:234-236
    torch::optim::Adam adam(model->parameters(), torch::optim::AdamOptions(1e-3).weight_decay(1e-4));
    const float grad_clip = 1.0; // training_options_t default (mmvae_alg.hh:19-23)

    // The noise the forward just consumed, recovered by the re-seed; checked bit-exact.
    auto recover_eps = [&](const std::string &tag, int64_t seed, int64_t B, Tensor x, Tensor c,
                           const nbvae_out_t &y) {
        torch::manual_seed(seed);
        auto eps_mu = torch::randn({ B, K });
        auto eps_nu = torch::randn({ B, R });
        torch::NoGradGuard ng;
        auto zmu = y.mu_mean + eps_mu.mul(y.mu_lnvar.div(2.0).exp());
        auto znu = y.nu_mean + eps_nu.mul(y.nu_lnvar.div(2.0).exp());
        if (!torch::equal(model->decode_mu(zmu, c), y.recon_mu) ||
            !torch::equal(model->decode_nu(znu), y.recon_nu)) {
            std::fprintf(stderr, "%s: noise recovery is not bit-exact\n", tag.c_str());
            std::exit(3);
        }
        dump(tag + "/eps_mu", eps_mu);
        dump(tag + "/eps_nu", eps_nu);
    };

    int steps;
    spec >> steps;
    for (int t = 0; t < steps; ++t) {
        int64_t B, seed;
        float beta;
        spec >> B >> beta >> seed;
        const std::string tag = "s" + std::to_string(t);
        auto x = read_f32(g_dir + "/x" + std::to_string(t) + ".f32", { B, D });
        auto c = read_f32(g_dir + "/c" + std::to_string(t) + ".f32", { B, C });
        auto ridx = read_i64(g_dir + "/ridx" + std::to_string(t) + ".i64", B);
        model->train(true);
        // mmvae_alg.hh:300-310
        auto xboot = torch::index_select(x, 0, ridx);
        auto cboot = torch::index_select(c, 0, ridx);
        torch::manual_seed(seed);
        auto yboot = model->forward(xboot, cboot);
        recover_eps(tag, seed, B, xboot, cboot, yboot);
        auto L = mmvae::nb::loss(xboot, yboot, beta);
        adam.zero_grad();
        L.backward();
        for (auto &p : model->named_parameters()) dump(tag + "/grad/" + p.key(), p.value().grad());
        double total = torch::nn::utils::clip_grad_norm_(model->parameters(), grad_clip);
        adam.step();
        dump(tag + "/loss", L.detach().reshape({}));
        dump(tag + "/total_norm", torch::tensor(total, torch::kFloat64).reshape({}));
        for (auto &p : model->named_parameters()) dump(tag + "/param/" + p.key(), p.value());
    }
    {
        // the per-batch reported loss (mmvae_alg.hh:274-285): a train-mode forward, no update
        int64_t B, seed;
        float beta;
        spec >> B >> beta >> seed;
        auto x = read_f32(g_dir + "/xe.f32", { B, D });
        auto c = read_f32(g_dir + "/ce.f32", { B, C });
        model->train(true);
        torch::manual_seed(seed);
        auto y = model->forward(x, c);
        recover_eps("eval", seed, B, x, c, y);
        auto L = mmvae::nb::loss(x, y, beta);
        dump("eval/loss", L.detach().reshape({}));
        // the recorder (nb.hh:619-657 -> encode_mu(x), nb.hh:419-431) after train(false)
        model->train(false);
        torch::NoGradGuard ng;
        auto enc_out = model->encode_mu(x);
        dump("eval/enc_mean", enc_out.first);
        dump("eval/enc_lnvar", enc_out.second);
    }
    g_manifest.close();
    return 0;
}
