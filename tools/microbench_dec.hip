// Micro-benchmark of the decoder pass-A inner loop with ablations (diagnostic tool, not shipped).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench_dec.hip -o /tmp/mb && /tmp/mb
// Variant bits: 1 = skip W loads (reuse registers), 2 = skip MFMA, 4 = skip epilogue.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../mm-vae_amd/csrc/common.hpp"

constexpr int KP = 64;
using M = MM<__bf16>;
using Fr = M::frag;
constexpr int KS = KP / 32;

template <int VAR>
__global__ __launch_bounds__(256, 2) void k_passA(const __bf16* __restrict__ Z, const __bf16* __restrict__ W,
                                                  const float4* __restrict__ grec, int DP, int NT, int nsp,
                                                  float* __restrict__ out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int sp = blockIdx.x % nsp, rb = blockIdx.x / nsp;
    const int row0 = rb * 64 + 16 * w;
    const int tps = (NT + nsp - 1) / nsp;
    const int t0 = sp * tps, t1 = min(NT, t0 + tps);
    Fr zfr[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) zfr[s] = M::load(&Z[(int64_t)(row0 + (lane & 15)) * KP + s * 32 + (lane >> 4) * 8]);
    float mrun[4] = {-1e30f, -1e30f, -1e30f, -1e30f}, srun[4] = {0, 0, 0, 0};
    Fr wc[4][KS], wn[4][KS];
    float4 gc[4], gn[4];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
            const int gene = 64 * t + 16 * gb + (lane & 15);
#pragma unroll
            for (int s = 0; s < KS; ++s) wn[gb][s] = M::load(&W[(int64_t)gene * KP + s * 32 + (lane >> 4) * 8]);
            gn[gb] = grec[gene];
        }
    };
    if (!(VAR & 1)) load_tile(t0);
    else {
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
#pragma unroll
            for (int s = 0; s < KS; ++s) wn[gb][s] = zfr[s];
            gn[gb] = float4{0.f, 0.f, 0.f, 0.f};
        }
    }
    for (int t = t0; t < t1; ++t) {
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
            gc[gb] = gn[gb];
#pragma unroll
            for (int s = 0; s < KS; ++s) wc[gb][s] = wn[gb][s];
        }
        if (!(VAR & 1) && t + 1 < t1) load_tile(t + 1);
#pragma unroll
        for (int gb = 0; gb < 4; ++gb) {
            f32x4 acc = f32x4{(float)t, 0.f, 0.f, 0.f};
            if (!(VAR & 2)) {
#pragma unroll
                for (int s = 0; s < KS; ++s) acc = M::mma(zfr[s], wc[gb][s], acc);
            } else {
                acc[1] = (float)wc[gb][0][0];
            }
            if (!(VAR & 4)) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float lg = acc[r] + gc[gb].x;
                    lg = fmaf(1.f, gc[gb].z, lg);
                    const float df = lg - mrun[r];
                    const float e = fexp(-fabsf(df));
                    const bool up = df > 0.f;
                    srun[r] = fmaf(srun[r], up ? e : 1.f, up ? 1.f : e);
                    mrun[r] = fmaxf(mrun[r], lg);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) srun[r] += acc[r] + gc[gb].x;
            }
        }
    }
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) v += srun[r] + mrun[r];
    out[blockIdx.x * 256 + threadIdx.x] = v;
}

int main() {
    const int D = 20000, DP = 20032, NT = DP / 64, B = 4096, nrb = B / 64;
    __bf16 *Z, *W;
    float4* grec;
    float* out;
    hipMalloc(&Z, sizeof(__bf16) * B * KP);
    hipMalloc(&W, sizeof(__bf16) * DP * KP);
    hipMalloc(&grec, sizeof(float4) * DP);
    hipMalloc(&out, sizeof(float) * 256 * nrb * 64);
    hipMemset(Z, 0, sizeof(__bf16) * B * KP);
    hipMemset(W, 0, sizeof(__bf16) * DP * KP);
    hipMemset(grec, 0, sizeof(float4) * DP);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](auto kern, int nsp, const char* name) {
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(nrb * nsp), dim3(256), 0, 0, Z, W, grec, DP, NT, nsp, out);
        hipEventRecord(a);
        const int it = 20;
        for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(nrb * nsp), dim3(256), 0, 0, Z, W, grec, DP, NT, nsp, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("%-28s nsp=%3d  %8.1f us\n", name, nsp, ms * 1000 / it);
    };
    for (int nsp : {8, 32}) {
        run(k_passA<0>, nsp, "full");
        run(k_passA<1>, nsp, "no W loads");
        run(k_passA<2>, nsp, "no MFMA");
        run(k_passA<4>, nsp, "no epilogue");
        run(k_passA<6>, nsp, "loads only");
        run(k_passA<7>, nsp, "nothing");
    }
    return 0;
}
