// options.hh — the reference's four command-line option groups, drop-in (header-only, inline).
//
// Same struct names, field names, defaults, long options, short letters and return codes as
//   mmvae_options_t      + parse_mmvae_options     include/mmvae.hh:31-209
//   training_options_t   + parse_training_options  include/mmvae_alg.hh:14-125
//   mmvae::nb::nbvae_options_t + parse_nbvae_options   include/models/nb.hh:53-194
//   mmvae::vmf::vmf_options_t  + parse_vmf_options     include/models/vmf.hh:54-186
// Each parser runs getopt_long over a private copy of argv with opterr = 0 (unknown options
// are ignored, so the groups can share one argv) and returns EXIT_SUCCESS /
// EXIT_FAILURE.  Differences, all deliberate:
//   * --grad_clip is accepted and ignored, as in the reference (no 'G' case, Q7);
//   * training_options_t::device is the HIP device ordinal (the reference holds a torch::Device
//     that its engine never uses on the GPU), default 0;
//   * inline definitions: the headers can be included by any number of translation units.
#ifndef MMVAE_OPTIONS_HH_
#define MMVAE_OPTIONS_HH_

#include <getopt.h>
#include <sys/stat.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

namespace mmvae_opt_detail {

// getopt_long permutes argv: every group parses a fresh copy (the reference's str2char copies)
template <class F>
inline void each_opt(int argc, const char* argv[], const char* shorts, const option* longs, F&& f) {
    std::vector<std::string> store(argv, argv + argc);
    std::vector<char*> ptrs;
    for (auto& s : store) ptrs.push_back(&s[0]);
    ptrs.push_back(nullptr);
    optind = 1;
    opterr = 0;
    while (true) {
        const int c = getopt_long(argc, ptrs.data(), shorts, longs, nullptr);
        if (c == -1) break;
        if (f(c, optarg ? std::string(optarg) : std::string())) break;
    }
}

inline std::vector<int64_t> split_ints(const std::string& s) {  // copy_int_arr (nb.hh:114-121)
    std::vector<int64_t> v;
    size_t p = 0;
    while (p <= s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        if (q > p) v.push_back(std::stol(s.substr(p, q - p)));
        p = q + 1;
    }
    return v;
}

inline bool file_exists(const std::string& f) {
    struct stat st;
    return !f.empty() && stat(f.c_str(), &st) == 0;
}

}  // namespace mmvae_opt_detail

// ---- mmvae.hh:31-209 -----------------------------------------------------------------------
struct mmvae_options_t {
    explicit mmvae_options_t() : batch_size(100), kl_discount(.1f), kl_min(1e-2f), kl_max(1.f) {}
    std::string mtx;
    std::string idx;
    std::string out;
    std::string row;
    std::string col;
    std::string annot;
    std::string covar_mtx;
    std::string covar_idx;
    int64_t batch_size;
    float kl_discount;
    float kl_min;
    float kl_max;
};

inline const char* mmvae_options_usage() {
    return "\n[options]\n\n"
           "--mtx         : a matrix market mtx file\n"
           "--idx         : an index file for the mtx (default: ${mtx}.index)\n"
           "--row         : the rows (line = one string)\n"
           "--col         : the columns (line = one string)\n"
           "--annot       : the list of column annotations (line = ${col} <space> ${k})\n"
           "--out         : output file header\n"
           "--covar       : a separate matrix market mtx for other covariates\n"
           "--covar_idx   : an index file for the covar mtx (default: ${covar}.index)\n"
           "--batch_size  : #samples in each batch (default: 100)\n\n"
           "--kl_discount : KL divergence discount (default: .1)\n"
           "              : Loss = likelihood_loss + beta * KL_loss\n"
           "              : where beta = exp(- ${discount} * epoch)\n"
           "--kl_max      : max KL divergence penalty (default: 1)\n"
           "--kl_min      : min KL divergence penalty (default: 1e-2)\n\n";
}

// help_out (nullable): set when --help was given (the reference prints the usage and returns
// EXIT_SUCCESS before checking the files)
inline int parse_mmvae_options(const int argc, const char* argv[], mmvae_options_t& options, bool* help_out = nullptr) {
    static const option longs[] = {{"mtx", required_argument, nullptr, 'M'},         {"idx", required_argument, nullptr, 'I'},
                                   {"out", required_argument, nullptr, 'O'},         {"output", required_argument, nullptr, 'O'},
                                   {"cov", required_argument, nullptr, 'V'},         {"covar", required_argument, nullptr, 'V'},
                                   {"cov_idx", required_argument, nullptr, 'J'},     {"covar_idx", required_argument, nullptr, 'J'},
                                   {"row", required_argument, nullptr, 'r'},         {"col", required_argument, nullptr, 'c'},
                                   {"column", required_argument, nullptr, 'c'},      {"annot", required_argument, nullptr, 'a'},
                                   {"annotation", required_argument, nullptr, 'a'},  {"batch_size", required_argument, nullptr, 'b'},
                                   {"batch", required_argument, nullptr, 'b'},       {"kl_discount", required_argument, nullptr, 'K'},
                                   {"kl_max", required_argument, nullptr, 'L'},      {"kl_min", required_argument, nullptr, 'l'},
                                   {"help", no_argument, nullptr, 'h'},              {nullptr, no_argument, nullptr, 0}};
    bool help = false;
    mmvae_opt_detail::each_opt(argc, argv, "M:I:O:V:J:r:c:a:b:K:L:l:h?", longs, [&](int c, const std::string& v) {
        switch (c) {
            case 'M': options.mtx = v; break;
            case 'I': options.idx = v; break;
            case 'V': options.covar_mtx = v; break;
            case 'J': options.covar_idx = v; break;
            case 'O': options.out = v; break;
            case 'r': options.row = v; break;
            case 'c': options.col = v; break;
            case 'a': options.annot = v; break;
            case 'b': options.batch_size = std::stol(v); break;
            case 'K': options.kl_discount = std::stof(v); break;
            case 'l': options.kl_min = std::stof(v); break;
            case 'L': options.kl_max = std::stof(v); break;
            case 'h': help = true; return true;
            default: break;
        }
        return false;
    });
    if (help_out) *help_out = help;
    if (help) {
        std::cerr << mmvae_options_usage() << std::endl;
        return EXIT_SUCCESS;
    }
    if (!mmvae_opt_detail::file_exists(options.mtx)) {  // ERR_RET (util.hh), mmvae.hh:197-198
        std::cerr << "missing mtx file" << std::endl;
        return EXIT_FAILURE;
    }
    if (options.out.size() == 0) {
        std::cerr << "need output file header" << std::endl;
        return EXIT_FAILURE;
    }
    if (options.idx.size() == 0) options.idx = options.mtx + ".index";
    if (options.covar_idx.size() == 0) options.covar_idx = options.covar_mtx + ".index";
    return EXIT_SUCCESS;
}

// ---- mmvae_alg.hh:14-125 -------------------------------------------------------------------
struct training_options_t {
    explicit training_options_t() : lr(1e-3f), grad_clip(1.f), nboot(3), max_epoch(101), recording(10), device(0) {}
    float lr;
    float grad_clip;    // parsed by nobody (Q7): clip_grad_norm_ always uses 1
    int64_t nboot;
    int64_t max_epoch;
    int64_t recording;
    int device;         // HIP device ordinal (the reference: torch::Device, mmvae_alg.hh:17,32)
};

inline int parse_training_options(const int argc, const char* argv[], training_options_t& options) {
    static const option longs[] = {{"lr", required_argument, nullptr, 'L'},          {"learning", required_argument, nullptr, 'L'},
                                   {"learn_rate", required_argument, nullptr, 'L'},  {"learning_rate", required_argument, nullptr, 'L'},
                                   {"rate", required_argument, nullptr, 'L'},        {"grad_clip", required_argument, nullptr, 'G'},
                                   {"nboot", required_argument, nullptr, 'B'},       {"boot", required_argument, nullptr, 'B'},
                                   {"bootstrap", required_argument, nullptr, 'B'},   {"max_epoch", required_argument, nullptr, 'E'},
                                   {"epoch", required_argument, nullptr, 'E'},       {"recording", required_argument, nullptr, 'R'},
                                   {"help", no_argument, nullptr, 'h'},              {nullptr, no_argument, nullptr, 0}};
    bool help = false;
    mmvae_opt_detail::each_opt(argc, argv, "L:G:B:E:R:h", longs, [&](int c, const std::string& v) {
        switch (c) {
            case 'L': options.lr = std::stof(v); break;
            case 'B': options.nboot = std::stol(v); break;
            case 'E': options.max_epoch = std::stol(v); break;
            case 'R': options.recording = std::stol(v); break;
            case 'h': help = true; return true;
            default: break;  // 'G': declared, never stored (Q7)
        }
        return false;
    });
    if (help)
        std::cerr << "[Training algorithm options]\n\n--lr         : learning rate (default: 1e-3)\n"
                     "--grad_clip  : gradient clip (default: 1)\n--nboot      : #bootstrapped gradients (default: 3)\n"
                     "--max_epoch  : maximum #epoch (default: 101)\n--recording  : recording interval (default: 10)\n"
                  << std::endl;
    return EXIT_SUCCESS;
}

// ---- models/nb.hh:53-194 (namespace mmvae::nb, as the reference) ---------------------------
namespace mmvae {
namespace nb {
struct nbvae_options_t {
    explicit nbvae_options_t() : mean_latent(2), overdispersion_encoding(1), overdispersion_latent(1), do_relu(false) {}
    std::vector<int64_t> mean_encoding_layers;
    std::vector<int64_t> mean_decoding_layers;
    int64_t mean_latent;
    int64_t overdispersion_encoding;
    int64_t overdispersion_latent;
    bool do_relu;
};

inline int parse_nbvae_options(const int argc, const char* argv[], nbvae_options_t& options) {
    static const option longs[] = {{"mean_encoding", required_argument, nullptr, 'E'},
                                   {"mean-encoding", required_argument, nullptr, 'E'},
                                   {"mean_decoding", required_argument, nullptr, 'D'},
                                   {"mean-decoding", required_argument, nullptr, 'D'},
                                   {"mean_latent", required_argument, nullptr, 'L'},
                                   {"mean-latent", required_argument, nullptr, 'L'},
                                   {"overdisp_encoding", required_argument, nullptr, 'e'},
                                   {"overdisp-encoding", required_argument, nullptr, 'e'},
                                   {"overdispersion_encoding", required_argument, nullptr, 'e'},
                                   {"overdispersion-encoding", required_argument, nullptr, 'e'},
                                   {"overdispersion_latent", required_argument, nullptr, 'l'},
                                   {"overdispersion-latent", required_argument, nullptr, 'l'},
                                   {"relu", no_argument, nullptr, 'R'},
                                   {"no_relu", no_argument, nullptr, 'r'},
                                   {"no-relu", no_argument, nullptr, 'r'},
                                   {"help", no_argument, nullptr, 'h'},
                                   {nullptr, no_argument, nullptr, 0}};
    mmvae_opt_detail::each_opt(argc, argv, "E:D:L:e:l:rRh", longs, [&](int c, const std::string& v) {
        switch (c) {
            case 'E': options.mean_encoding_layers = mmvae_opt_detail::split_ints(v); break;
            case 'D': options.mean_decoding_layers = mmvae_opt_detail::split_ints(v); break;
            case 'L': options.mean_latent = std::stol(v); break;
            case 'e': options.overdispersion_encoding = std::stol(v); break;
            case 'l': options.overdispersion_latent = std::stol(v); break;
            case 'r': options.do_relu = false; break;
            case 'R': options.do_relu = true; break;
            case 'h': return true;
            default: break;
        }
        return false;
    });
    return EXIT_SUCCESS;
}
}  // namespace nb
}  // namespace mmvae

// ---- models/vmf.hh:54-186 (namespace mmvae::vmf) -------------------------------------------
namespace mmvae {
namespace vmf {
struct vmf_options_t {
    explicit vmf_options_t() : latent(2), kappa_min(.1f), kappa_max(10.f), do_relu(false) {}
    std::vector<int64_t> encoding_layers;
    std::vector<int64_t> decoding_layers;
    int64_t latent;
    float kappa_min;
    float kappa_max;
    bool do_relu;
};

inline int parse_vmf_options(const int argc, const char* argv[], vmf_options_t& options) {
    static const option longs[] = {{"encoding", required_argument, nullptr, 'E'},  {"decoding", required_argument, nullptr, 'D'},
                                   {"latent", required_argument, nullptr, 'L'},    {"kappa_min", required_argument, nullptr, 'k'},
                                   {"kappa-min", required_argument, nullptr, 'k'}, {"kappa_max", required_argument, nullptr, 'K'},
                                   {"kappa-max", required_argument, nullptr, 'K'}, {"relu", no_argument, nullptr, 'R'},
                                   {"no_relu", no_argument, nullptr, 'r'},         {"no-relu", no_argument, nullptr, 'r'},
                                   {"help", no_argument, nullptr, 'h'},            {nullptr, no_argument, nullptr, 0}};
    mmvae_opt_detail::each_opt(argc, argv, "E:D:L:k:K:Rrh", longs, [&](int c, const std::string& v) {
        switch (c) {
            case 'E': options.encoding_layers = mmvae_opt_detail::split_ints(v); break;
            case 'D': options.decoding_layers = mmvae_opt_detail::split_ints(v); break;
            case 'L': options.latent = std::stol(v); break;
            case 'k': options.kappa_min = std::stof(v); break;
            case 'K': options.kappa_max = std::stof(v); break;
            case 'r': options.do_relu = false; break;
            case 'R': options.do_relu = true; break;
            case 'h': return true;
            default: break;
        }
        return false;
    });
    return EXIT_SUCCESS;
}
}  // namespace vmf
}  // namespace mmvae

#endif  // MMVAE_OPTIONS_HH_
