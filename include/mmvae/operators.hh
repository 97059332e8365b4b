// operators.hh — drop-in for the reference's custom autograd op (include/operators.hh:13-101):
//
//   torch::Tensor lbessel(const torch::Tensor kappa, at::Scalar df)
//
// log I_df(kappa), the piecewise approximation of Oh, Adamczewski & Park (2019): for kappa <= df
// df log kappa + eta kappa - (eta + df) log 2 - fasterlgamma(df + 1), eta = (df + 1/2)/(2(df + 1));
// otherwise kappa - log(kappa)/2 - log(2 pi)/2.  Its backward is the reference's custom node
// (LogModifiedBesselBackward, operators.hh:13-47): the Baricz bound
// (sqrt(k^2 df/(df + 1) + df^2) + sqrt(k^2 + df^2)) / (2 k), RETURNED AS IS — the upstream gradient
// is not multiplied in, which this op keeps so trajectories match.
//
// The arithmetic is the engine's host restatement (lbessel.hh — also behind the C-ABI's
// mmvae_lbessel / mmvae_lbessel_grad; bit-exact against the reference's fastgamma.h,
// tests/test_capi_cpu.py), header-only so a LibTorch program needs no link to libmmvae.so; it is
// wrapped as a public torch::autograd::Function instead of the reference's use of LibTorch
// internals (set_history, SavedVariable::reset_grad_function, which LibTorch 2.x removed).
// Elementwise on any shape; float math, result in kappa's dtype and device.
#ifndef MMVAE_OPERATORS_HH_
#define MMVAE_OPERATORS_HH_

#include <torch/torch.h>

#include "lbessel.hh"

namespace mmvae_ops_detail {

inline torch::Tensor map_scalar(const torch::Tensor& x, double df, float (*f)(float, float)) {  // elementwise
    auto c = x.detach().to(torch::kCPU, torch::kFloat).contiguous();
    auto out = torch::empty_like(c);
    const float* a = c.data_ptr<float>();
    float* o = out.data_ptr<float>();
    const int64_t n = c.numel();
    for (int64_t i = 0; i < n; ++i) o[i] = f(a[i], (float)df);
    return out.to(x.device(), x.scalar_type());
}

struct LBessel : public torch::autograd::Function<LBessel> {
    static torch::Tensor forward(torch::autograd::AutogradContext* ctx, torch::Tensor kappa, double df) {
        ctx->save_for_backward({kappa});
        ctx->saved_data["df"] = df;
        return map_scalar(kappa, df, mmvae_math::lbessel);
    }
    static torch::autograd::variable_list backward(torch::autograd::AutogradContext* ctx,
                                                   torch::autograd::variable_list /*grad_out: ignored, Q3*/) {
        const auto kappa = ctx->get_saved_variables()[0];
        const double df = ctx->saved_data["df"].toDouble();
        return {map_scalar(kappa, df, mmvae_math::lbessel_grad), torch::Tensor()};
    }
};

}  // namespace mmvae_ops_detail

inline torch::Tensor lbessel(const torch::Tensor self_, at::Scalar df_) {
    return mmvae_ops_detail::LBessel::apply(self_, df_.toDouble());
}

#endif  // MMVAE_OPERATORS_HH_
