// lbessel.hh — host fp32 scalars of the vMF observation model, header-only (shared by the
// engine's C-ABI exports mmvae_lbessel* / mmvae_faster* and the drop-in operators.hh):
//   fasterlog / fasterlgamma   P. Mineiro's bit-trick approximations (reference
//                              include/utils/fastlog.h:75-85, fastgamma.h:58-60), bit-exact
//                              against the reference headers compiled in oracle/_ref
//   lbessel / lbessel_grad     operators.hh:49-101 forward (ATen float ops with double scalars
//                              rounded to float, as the reference evaluates them) and the Baricz
//                              bound its custom backward returns (operators.hh:20-40, Q3)
#ifndef MMVAE_LBESSEL_HH_
#define MMVAE_LBESSEL_HH_

#include <cmath>
#include <cstdint>
#include <cstring>

namespace mmvae_math {

inline float fasterlog(float x) {
    uint32_t i;
    std::memcpy(&i, &x, 4);
    volatile float y = (float)i;
    y = y * 8.2629582881927490e-8f;
    return y - 87.989971088f;
}

inline float fasterlgamma(float x) {
    volatile float a = -0.0810614667f - x;
    a = a - fasterlog(x);
    volatile float b = (0.5f + x) * fasterlog(1.0f + x);
    return a + b;
}

// operators.hh:49-101 (forward) for a scalar kappa; nu = df
inline float lbessel(float kappa, float nu) {
    const double nud = nu;
    const float eta = (float)((nud + 0.5) / (2. * (nud + 1.)));
    const float lk = std::log(kappa);
    // stuff1 = nu*log(k) + eta*k - (eta+nu)*log(2) - fasterlgamma(nu+1)
    float s1 = (float)nud * lk;
    s1 = s1 + eta * kappa;
    s1 = s1 - (float)(((double)eta + nud) * std::log(2.));
    s1 = s1 - fasterlgamma((float)(nud + 1));
    float s2 = kappa - 0.5f * lk;
    s2 = s2 - (float)(0.5 * std::log(2. * M_PI));
    return (kappa <= nu) ? s1 : s2;
}

// operators.hh:20-40: Baricz bound, independent of the upstream gradient (Q3)
inline float lbessel_grad(float kappa, float nu) {
    const float df = nu;
    const float lb = std::sqrt(kappa * kappa * df / (float)(df + 1.) + df * df);
    const float ub = std::sqrt(kappa * kappa + df * df);
    return 0.5f * (lb + ub) / kappa;
}

}  // namespace mmvae_math

#endif  // MMVAE_LBESSEL_HH_
