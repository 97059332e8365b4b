// clip_grad_norm_ + torch::optim::Adam (L2 weight decay) over the flat registered-parameter
// buffer: the reference's mmvae_alg.hh:306-310 (LibTorch 2.10 clip_grad.h:54-86 and
// optim/adam.cpp).  Two launches: per-block sum of squares, then every block folds the
// partials, forms the clip coefficient and updates its slice (grad, wd, m, v, p in one pass).
#include "common.hpp"
#include "engine.hpp"

namespace mmvae {

static constexpr int SUMSQ_BLOCKS = 256;

__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
    __shared__ double sb[4];
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double v = g[i];
        s += v * v;
    }
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = sb[0] + sb[1] + sb[2] + sb[3];
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v, int64_t n,
                                              const double* __restrict__ part, int nparts, float max_norm,
                                              const StepScalars* __restrict__ ss, float b1, float b2, float wd,
                                              float eps, float* __restrict__ out) {
    const float lr_bc1 = ss->lr_bc1, inv_sqrt_bc2 = ss->inv_sqrt_bc2;  // this step's (staged with the batch)
    __shared__ float s_coef;
    __shared__ double sb[4];
    // the first EPT elements of this thread's grid-stride range are loaded before the clip norm's
    // partials are reduced: the update's loads do not wait for the norm
    constexpr int EPT = 4;
    const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
    float gv[EPT], pv[EPT], mv[EPT], vv[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int64_t i = i0 + e * stride;
        const bool in = i < n;
        gv[e] = in ? g[i] : 0.f;
        pv[e] = in ? p[i] : 0.f;
        mv[e] = in ? m[i] : 0.f;
        vv[e] = in ? v[i] : 0.f;
    }
    double tp = 0.0;
    for (int i = threadIdx.x; i < nparts; i += 256) tp += part[i];  // fixed order per block
    tp = wave_sum_d(tp);
    if ((threadIdx.x & 63) == 0) sb[threadIdx.x >> 6] = tp;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = (sb[0] + sb[1]) + (sb[2] + sb[3]);
        const float total = (float)sqrt(t);            // stack(norms).norm(2), fp32 tensor
        float coef = max_norm / (total + 1e-6f);       // clip_grad.h:81
        coef = fminf(coef, 1.f);                        // clamp(max=1), clip_grad.h:82-83
        s_coef = coef;
        if (blockIdx.x == 0) out[1] = total;
    }
    __syncthreads();
    const float coef = s_coef;
    auto update = [&](int64_t i, float gi, float pi, float m0, float v0) {
        gi = gi * coef;                                 // grad.mul_(clip_coef_clamped)
        gi = gi + wd * pi;                              // grad.add(p, weight_decay)
        const float mi = m0 * b1 + gi * (1.f - b1);     // exp_avg.mul_(b1).add_(grad, 1-b1)
        const float vi = v0 * b2 + (1.f - b2) * gi * gi;  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
        const float denom = sqrtf(vi) * inv_sqrt_bc2 + eps;
        m[i] = mi;
        v[i] = vi;
        p[i] = pi - lr_bc1 * (mi / denom);              // p.addcdiv_(exp_avg, denom, -lr/bc1)
    };
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int64_t i = i0 + e * stride;
        if (i < n) update(i, gv[e], pv[e], mv[e], vv[e]);
    }
    for (int64_t i = i0 + EPT * stride; i < n; i += stride) update(i, g[i], p[i], m[i], v[i]);
}

// Adam's bias-corrected rates of optimiser step t (optim/adam.cpp), into the staged scalars
void adam_scalars(const Engine* e, int64_t t, StepScalars* ss) {
    const double bc1 = 1.0 - std::pow(0.9, (double)t);
    const double bc2 = 1.0 - std::pow(0.999, (double)t);
    ss->lr_bc1 = (float)(e->cfg.lr / bc1);
    ss->inv_sqrt_bc2 = (float)(1.0 / std::sqrt(bc2));
}

// the staged scalars of the step hold adam_scalars(adam_step) (mmvae_run)
hipError_t opt_clip_adam(Engine* e) {
    const double b1 = 0.9, b2 = 0.999;
    const int64_t n = e->P_reg;
    // the NB world-1 step leaves its own partials (gradient kernels, one per block); otherwise
    // (vMF, or gradients all-reduced after the gradient kernels) k_sumsq computes them
    const int nparts = e->sq_parts > 0 ? e->sq_parts : SUMSQ_BLOCKS;
    if (e->sq_parts <= 0) {
        ScopedTimer tm(e, "k_sumsq");
        hipLaunchKernelGGL(k_sumsq, dim3(SUMSQ_BLOCKS), dim3(256), 0, e->stream, e->d_grads, n, e->d_sumsq);
    }
    e->sq_parts = 0;
    {
        ScopedTimer tm(e, "k_adam");
        hipLaunchKernelGGL(k_adam, dim3(SUMSQ_BLOCKS), dim3(256), 0, e->stream, e->d_params, e->d_grads, e->d_m,
                           e->d_v, n, e->d_sumsq, nparts, e->cfg.grad_clip, e->d_ss, (float)b1, (float)b2,
                           e->cfg.weight_decay, 1e-8f,
                           e->d_out);
    }
    return hipGetLastError();
}

// Diagnostic (mmvae_debug_poison): fill the whole LDS of every CU with a byte pattern.  One
// workgroup holds the full 160 KB, so a grid of a few rounds over the 256 CUs leaves the pattern
// in every CU's LDS for the kernels launched next.  Vector LDS stores only.
static constexpr int LDS_POISON_BYTES = 160 * 1024;
__global__ __launch_bounds__(256) void k_lds_poison(uint32_t word) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint4* s = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < LDS_POISON_BYTES / 16; i += 256) s[i] = uint4{word, word, word, word};
    __syncthreads();
}

hipError_t lds_poison(Engine* e, int byte) {
    const uint32_t b = (uint32_t)(byte & 0xff);
    static bool attr = false;
    if (!attr) {  // (the runtime may already allow the full LDS; a refusal is not an error here)
        (void)hipFuncSetAttribute((const void*)k_lds_poison, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  LDS_POISON_BYTES);
        (void)hipGetLastError();
        attr = true;
    }
    hipLaunchKernelGGL(k_lds_poison, dim3(4 * 256), dim3(256), LDS_POISON_BYTES, e->stream, b * 0x01010101u);
    return hipGetLastError();
}

}  // namespace mmvae
