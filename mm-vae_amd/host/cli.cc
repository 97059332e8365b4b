// nb_vae_main / vmf_vae_main drop-in CLIs (src/nb_vae_main.cc, src/vmf_vae_main.cc) over the HIP
// engine.  The reference parses argv once per option group with getopt_long, unknown options
// ignored (opterr = 0): mmvae options (mmvae.hh:68-209), training options (mmvae_alg.hh:36-125),
// then the model's (nb.hh:73-194 / vmf.hh:75-186) — a short option therefore means one thing
// per group, and this parser keeps exactly that behaviour.  A fourth group holds the engine's
// own options (--seed, --dtype, --device, --threads, --no_csr_cache, --verbose).
//
// Outputs as the reference: ${out}.scores.gz (per-epoch loss), ${out}.covar.mtx.gz (+ .index) when
// --covar is absent (create_ones_like), ${mtx}.index when missing (BGZF inputs), recorder files
// every --recording epochs.  The dataset is loaded
// once into HBM; its parsed CSR is cached next to the mtx as ${mtx}.mmvae_csr (the role of the
// reference's ${mtx}.index: a faster second open).
// Data parallel: launched once per GPU with RANK / WORLD_SIZE / LOCAL_RANK in the environment;
// rank 0 publishes the RCCL id in ${out}.rccl_id, the other ranks read it.
#include <getopt.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mmvae/options.hh"
#include "../../include/mmvae_host.h"
#include "cli.hh"
#include "host_common.hh"

namespace mmvae_host {

static bool file_exists(const std::string& f) {
    struct stat st;
    return !f.empty() && stat(f.c_str(), &st) == 0;
}

int parse_options(int argc, const char** argv, int model, CliOptions& o) {
    // the reference's three option groups through the drop-in parsers (include/mmvae/options.hh)
    mmvae_options_t mo;
    bool help = false;
    o.mm_rc = parse_mmvae_options(argc, argv, mo, &help);
    o.help = help;
    o.mtx = mo.mtx;
    o.idx = mo.idx;
    o.out = mo.out;
    o.row = mo.row;
    o.col = mo.col;
    o.annot = mo.annot;
    o.covar_mtx = mo.covar_mtx;
    o.covar_idx = mo.covar_idx;
    o.train.batch_size = mo.batch_size;
    o.train.kl_discount = mo.kl_discount;
    o.train.kl_min = mo.kl_min;
    o.train.kl_max = mo.kl_max;
    training_options_t to;
    parse_training_options(argc, argv, to);
    o.lr = to.lr;
    o.train.nboot = to.nboot;
    o.train.max_epoch = to.max_epoch;
    o.train.recording = to.recording;
    if (model == MMVAE_MODEL_NB) {
        mmvae::nb::nbvae_options_t nb;
        parse_nbvae_options(argc, argv, nb);
        o.enc_layers = nb.mean_encoding_layers;
        o.dec_layers = nb.mean_decoding_layers;
        o.latent = nb.mean_latent;
        o.H = nb.overdispersion_encoding;
        o.R = nb.overdispersion_latent;
        o.relu = nb.do_relu;
    } else {
        mmvae::vmf::vmf_options_t vo;
        parse_vmf_options(argc, argv, vo);
        o.enc_layers = vo.encoding_layers;
        o.dec_layers = vo.decoding_layers;
        o.latent = vo.latent;
        o.kappa_min = vo.kappa_min;
        o.kappa_max = vo.kappa_max;
        o.relu = vo.do_relu;
    }
    // ---- engine options (not in the reference) ----
    static const option en_long[] = {{"seed", required_argument, nullptr, 1},      {"dtype", required_argument, nullptr, 2},
                                     {"device", required_argument, nullptr, 3},    {"threads", required_argument, nullptr, 4},
                                     {"no_csr_cache", no_argument, nullptr, 5},    {"verbose", no_argument, nullptr, 6},
                                     {"quiet", no_argument, nullptr, 7},           {nullptr, no_argument, nullptr, 0}};
    mmvae_opt_detail::each_opt(argc, argv, "", en_long, [&](int c, const std::string& v) {
        switch (c) {
            case 1: o.seed = std::stoull(v); break;
            case 2: o.dtype = v; break;
            case 3: o.device = std::stoi(v); break;
            case 4: o.threads = std::stoi(v); break;
            case 5: o.csr_cache = false; break;
            case 6: o.verbose = true; break;
            case 7: o.verbose = false; break;
            default: break;
        }
        return false;
    });
    if (o.idx.empty()) o.idx = o.mtx + ".index";
    if (o.covar_idx.empty()) o.covar_idx = o.covar_mtx + ".index";
    if (dtype_code(o.dtype) < 0) {
        std::fprintf(stderr, "unknown --dtype %s (f32 | bf16x3 | bf16 | fp8)\n", o.dtype.c_str());
        return MMVAE_E_ARG;
    }
    return MMVAE_OK;
}

// --dtype spellings (engine extension) -> MMVAE_DTYPE_*, or -1 for an unknown one
int dtype_code(const std::string& s) {
    if (s == "f32" || s == "fp32" || s == "float32") return MMVAE_DTYPE_F32;
    if (s == "bf16") return MMVAE_DTYPE_BF16;
    if (s == "bf16x3" || s == "x3") return MMVAE_DTYPE_BF16X3;
    if (s == "fp8" || s == "e4m3") return MMVAE_DTYPE_FP8;
    return -1;
}

const char* usage_text(int model) {
    return model == MMVAE_MODEL_NB
               ? "nb_vae_main --mtx X.mtx.gz --out OUT [--batch_size 100 --max_epoch 101 --nboot 3 --lr 1e-3\n"
                 "             --mean_latent 2 --overdisp_encoding 1 --overdispersion_latent 1 --kl_discount .1\n"
                 "             --kl_max 1 --kl_min .01 --recording 10 --covar C.mtx.gz]\n"
                 "engine: [--dtype f32|bf16x3|bf16|fp8 --seed S --device G --threads T --no_csr_cache --verbose]\n"
               : "vmf_vae_main --mtx X.mtx.gz --out OUT [--batch_size 100 --max_epoch 101 --nboot 3 --lr 1e-3\n"
                 "             --latent 2 --kappa_min .1 --kappa_max 10 --kl_discount .1 --kl_max 1 --kl_min .01\n"
                 "             --recording 10 --covar C.mtx.gz]\n"
                 "engine: [--dtype f32|bf16x3|bf16 --seed S --device G --threads T --no_csr_cache --verbose]\n"
                 "        (fp8 is built for the NB model only)\n";
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// bgzf_is_bgzf (bgzf.c:581-594): gzip magic with the FEXTRA flag and a 'BC' subfield
static bool looks_bgzf(const std::string& path) {
    unsigned char h[18];
    FILE* fp = std::fopen(path.c_str(), "rb");
    if (!fp) return false;
    const size_t n = std::fread(h, 1, 18, fp);
    std::fclose(fp);
    return n == 18 && h[0] == 31 && h[1] == 139 && h[2] == 8 && (h[3] & 4) && h[12] == 'B' && h[13] == 'C';
}

// nb_vae_main.cc:58-59 / 72-78: build the column index of a BGZF MatrixMarket file when it is
// missing (non-BGZF inputs, which the reference refuses, are read without one)
static void ensure_index(const std::string& mtx, const std::string& idx, bool verbose) {
    if (file_exists(idx) || !looks_bgzf(mtx)) return;
    if (mmvae_mtx_build_index(mtx.c_str(), idx.c_str()) != MMVAE_OK)
        std::fprintf(stderr, "warning: %s\n", mmvae_host_last_error());
    else if (verbose)
        std::fprintf(stderr, "[mmvae] Built the file: %s\n", idx.c_str());
}

static int load_dataset(const CliOptions& o, mmvae_csr& csr) {
    const std::string cache = o.mtx + ".mmvae_csr";
    struct stat sm, sc;
    if (o.csr_cache && stat(cache.c_str(), &sc) == 0 && stat(o.mtx.c_str(), &sm) == 0 && sc.st_mtime >= sm.st_mtime &&
        mmvae_csr_load(cache.c_str(), &csr) == MMVAE_OK)
        return MMVAE_OK;
    int rc = mmvae_mtx_read(o.mtx.c_str(), o.threads, &csr);
    if (rc) return rc;
    // best effort (read-only dirs are fine); one writer per node (tmp + rename inside csr_save)
    const char* lr = std::getenv("LOCAL_RANK");
    if (o.csr_cache && (!lr || std::atoi(lr) == 0)) mmvae_csr_save(cache.c_str(), &csr);
    return MMVAE_OK;
}

// The launch key ties the id file to THIS launch, so a file left by a crashed earlier run with
// the same --out is never read: torchrun's run id, else the rendezvous address, else the parent
// process (the launcher that started every rank).
static std::string launch_key() {
    if (const char* r = std::getenv("TORCHELASTIC_RUN_ID")) return std::string("run:") + r;
    const char* a = std::getenv("MASTER_ADDR");
    const char* p = std::getenv("MASTER_PORT");
    if (a && p) return std::string("addr:") + a + ":" + p;
    return "ppid:" + std::to_string((long long)getppid());
}

static std::string rccl_id_path(const CliOptions& o) { return o.out + ".rccl_id"; }

static int rendezvous(mmvae_h h, const CliOptions& o, int rank, int world) {
    const std::string path = rccl_id_path(o);
    std::string key = launch_key();
    key.resize(64, '\0');
    unsigned char id[128];
    if (rank == 0) {
        if (mmvae_comm_unique_id(id)) return fail(MMVAE_E_COMM, mmvae_last_error(nullptr));
        const std::string tmp = path + ".tmp";
        FILE* fp = std::fopen(tmp.c_str(), "wb");
        if (!fp || std::fwrite(key.data(), 1, 64, fp) != 64 || std::fwrite(id, 1, 128, fp) != 128 ||
            std::fclose(fp) != 0)
            return fail(MMVAE_E_COMM, "cannot write " + tmp);
        std::rename(tmp.c_str(), path.c_str());
    } else {
        const double t0 = now_s();
        for (;;) {
            FILE* fp = std::fopen(path.c_str(), "rb");
            if (fp) {
                char k2[64];
                const bool got = std::fread(k2, 1, 64, fp) == 64 && std::fread(id, 1, 128, fp) == 128;
                std::fclose(fp);
                if (got && std::memcmp(k2, key.data(), 64) == 0) break;  // else: a stale file, keep waiting
            }
            if (now_s() - t0 > 300) return fail(MMVAE_E_COMM, "timed out waiting for " + path);
            std::this_thread::sleep_for(std::chrono::milliseconds(50));
        }
    }
    if (mmvae_comm_init(h, rank, world, id)) return fail(MMVAE_E_COMM, mmvae_last_error(h));
    return MMVAE_OK;
}

// rank 0 removes the id file on every exit path once the ranks may have read it
struct RcclIdCleanup {
    std::string path;
    bool armed = false;
    ~RcclIdCleanup() {
        if (armed) std::remove(path.c_str());
    }
};

int run_cli(int argc, const char** argv, int model) {
    CliOptions o;
    if (parse_options(argc, argv, model, o) != MMVAE_OK && !o.help) {
        std::fputs(usage_text(model), stderr);
        return EXIT_FAILURE;
    }
    if (o.help) {
        std::fputs(usage_text(model), stderr);
        return EXIT_SUCCESS;
    }
    // mmvae.hh:197-198 (the parser printed the reason) and nb_vae_main.cc:51-52
    if (o.mm_rc != EXIT_SUCCESS) {
        std::fputs(usage_text(model), stderr);
        return EXIT_FAILURE;
    }
    if (o.enc_layers.size() > MMVAE_MAX_HIDDEN || o.dec_layers.size() > MMVAE_MAX_HIDDEN) {
        std::fprintf(stderr, "at most %d hidden encoder / decoder layers\n", MMVAE_MAX_HIDDEN);
        return EXIT_FAILURE;
    }
    const int rank = std::getenv("RANK") ? std::atoi(std::getenv("RANK")) : 0;
    const int world = std::getenv("WORLD_SIZE") ? std::atoi(std::getenv("WORLD_SIZE")) : 1;
    const int local = std::getenv("LOCAL_RANK") ? std::atoi(std::getenv("LOCAL_RANK")) : 0;
    const int device = o.device >= 0 ? o.device : local;
    if (o.train.batch_size % world) {
        std::fprintf(stderr, "--batch_size must be divisible by WORLD_SIZE\n");
        return EXIT_FAILURE;
    }
    if (rank == 0) ensure_index(o.mtx, o.idx, o.verbose);
    const double t0 = now_s();
    mmvae_csr csr;
    if (load_dataset(o, csr)) {
        std::fprintf(stderr, "failed to read %s: %s\n", o.mtx.c_str(), mmvae_host_last_error());
        return EXIT_FAILURE;
    }
    if (o.verbose && rank == 0)
        std::fprintf(stderr, "[mmvae] Sparse Mtx Data: %lld x %lld (%lld nonzeros) from %s in %.2f s\n", (long long)csr.D,
                     (long long)csr.N, (long long)csr.nnz, o.mtx.c_str(), now_s() - t0);
    // covariates (nb_vae_main.cc:63-83): a separate MatrixMarket, or the all-ones column
    std::vector<float> covar;
    int64_t C = 1;
    if (file_exists(o.covar_mtx)) {
        if (rank == 0) ensure_index(o.covar_mtx, o.covar_idx, o.verbose);
        int64_t Nc = 0;
        float* m = nullptr;
        if (mmvae_mtx_read_dense_t(o.covar_mtx.c_str(), o.threads, &Nc, &C, &m)) {
            std::fprintf(stderr, "failed to read %s: %s\n", o.covar_mtx.c_str(), mmvae_host_last_error());
            return EXIT_FAILURE;
        }
        if (Nc != csr.N) {
            std::fprintf(stderr, "data and covar on the same set of data points (%lld vs %lld)\n", (long long)csr.N,
                         (long long)Nc);
            return EXIT_FAILURE;
        }
        covar.assign(m, m + Nc * C);
        mmvae_free(m);
    } else if (rank == 0) {
        const std::string f = o.out + ".covar.mtx.gz";
        if (mmvae_mtx_write_ones(f.c_str(), csr.N)) {
            std::fprintf(stderr, "warning: %s\n", mmvae_host_last_error());
        } else {
            if (o.verbose) std::fprintf(stderr, "[mmvae] No covariate file is given. So we use this: %s\n", f.c_str());
            std::remove((f + ".index").c_str());  // a fresh ones-file gets a fresh index
            ensure_index(f, f + ".index", o.verbose);
        }
    }
    mmvae_cfg cfg;
    mmvae_cfg_default(&cfg, model);
    cfg.dtype = dtype_code(o.dtype);
    cfg.D = csr.D;
    cfg.C = C;
    cfg.K = o.latent;
    cfg.H = o.H;
    cfg.R = o.R;
    cfg.max_batch = o.train.batch_size / world;
    cfg.lr = o.lr;
    cfg.kappa_min = o.kappa_min;
    cfg.kappa_max = o.kappa_max;
    cfg.seed = o.seed;
    cfg.relu = o.relu ? 1 : 0;
    cfg.n_enc_hidden = (int32_t)o.enc_layers.size();
    cfg.n_dec_hidden = (int32_t)o.dec_layers.size();
    for (size_t i = 0; i < o.enc_layers.size(); ++i) cfg.enc_hidden[i] = (int32_t)o.enc_layers[i];
    for (size_t i = 0; i < o.dec_layers.size(); ++i) cfg.dec_hidden[i] = (int32_t)o.dec_layers[i];
    mmvae_h h = nullptr;
    if (mmvae_create(&cfg, device, &h)) {
        std::fprintf(stderr, "engine: %s\n", mmvae_last_error(nullptr));
        return EXIT_FAILURE;
    }
    int rc = mmvae_upload_csr(h, csr.rowptr, csr.col, csr.val, csr.N, csr.D, covar.empty() ? nullptr : covar.data());
    mmvae_csr_free(&csr);
    if (!rc) rc = mmvae_init_params(h, o.seed);
    // one hipGraph per step shape (single-rank runs; with a communicator the steps stay eager)
    if (!rc && !std::getenv("MMVAE_NO_GRAPH")) rc = mmvae_graph_enable(h, 1);
    RcclIdCleanup id_cleanup;
    id_cleanup.path = rccl_id_path(o);
    id_cleanup.armed = world > 1 && rank == 0;
    if (!rc && world > 1) rc = rendezvous(h, o, rank, world);
    if (rc) {
        std::fprintf(stderr, "engine: %s %s\n", mmvae_last_error(h), mmvae_host_last_error());
        mmvae_destroy(h);
        return EXIT_FAILURE;
    }
    mmvae_train_opts t = o.train;
    t.seed = o.seed;
    t.out = o.out.c_str();
    t.verbose = o.verbose ? 1 : 0;
    t.rank = rank;
    t.world = world;
    std::vector<float> scores((size_t)std::max<int64_t>(t.max_epoch, 1));
    const double t1 = now_s();
    rc = mmvae_train(h, &t, scores.data());
    if (rc) {
        std::fprintf(stderr, "training failed: %s\n", mmvae_host_last_error());
        mmvae_destroy(h);
        return EXIT_FAILURE;
    }
    if (o.verbose && rank == 0)
        std::fprintf(stderr, "[mmvae] trained %lld epochs in %.2f s\n", (long long)t.max_epoch, now_s() - t1);
    if (rank == 0) {  // write_vector_file(out + ".scores.gz") (nb_vae_main.cc:133)
        TextWriter w;
        const std::string f = o.out + ".scores.gz";
        if (!w.open(f)) {
            std::fprintf(stderr, "cannot write %s\n", f.c_str());
            mmvae_destroy(h);
            return EXIT_FAILURE;
        }
        for (int64_t e = 0; e < t.max_epoch; ++e) w.write(fmt_g(scores[(size_t)e]) + "\n");
        w.close();
    }
    mmvae_destroy(h);
    return EXIT_SUCCESS;
}

}  // namespace mmvae_host
