// Write / read bandwidth of the access shapes the wide path's [B, D] blocks see (a probe, not part
// of the engine): whole rows, MFMA-layout tiles (16 lanes x 4 B per row, 4 rows an instruction)
// and float4 tiles, over a 4096 x 20000 f32 block.   hipcc -O3 --offload-arch=gfx950 membw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

static constexpr int M = 4096, N = 20480;

// whole rows, float4 per lane, one workgroup (256) per row
__global__ void k_rows(float* C, int rd, float* sink) {
    float acc = 0.f;
    float* r = C + (size_t)blockIdx.x * N;
    for (int i = threadIdx.x; i < N / 4; i += 256) {
        if (rd) {
            float4 v = reinterpret_cast<float4*>(r)[i];
            acc += v.x + v.y + v.z + v.w;
        } else {
            reinterpret_cast<float4*>(r)[i] = float4{1.f, 2.f, 3.f, (float)i};
        }
    }
    if (rd && acc == 1234.5f) sink[0] = acc;
}

// one wave per tile of TR rows x TC columns; tiles (mt, nt) walked nt = blockIdx.x + k gridDim.x
// (as k_gemm_skf), MFMA layout: a store covers 4 rows x 16 columns
template <int TR, int TC>
__global__ __launch_bounds__(64) void k_tiles_mfma(float* C, int rd, float* sink) {
    const int lane = threadIdx.x;
    const int ntl = N / TC;
    float acc = 0.f;
    for (int nt = blockIdx.x; nt < ntl; nt += gridDim.x) {
        float* base = C + (size_t)(blockIdx.y * TR) * N + nt * TC;
#pragma unroll
        for (int i = 0; i < TR / 16; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < TC / 16; ++j) {
                    float* p = base + (size_t)(16 * i + 4 * (lane >> 4) + r) * N + 16 * j + (lane & 15);
                    if (rd) acc += *p;
                    else *p = (float)(i + r + j);
                }
    }
    if (rd && acc == 1234.5f) sink[0] = acc;
}

// the same tiles, float4 per lane: TC / 4 lanes per row, 64 / (TC / 4) rows an instruction
template <int TR, int TC>
__global__ __launch_bounds__(64) void k_tiles_f4(float* C, int rd, float* sink) {
    const int lane = threadIdx.x;
    constexpr int LPR = TC / 4, RPI = 64 / LPR;
    const int ntl = N / TC;
    float acc = 0.f;
    for (int nt = blockIdx.x; nt < ntl; nt += gridDim.x) {
        float* base = C + (size_t)(blockIdx.y * TR) * N + nt * TC;
#pragma unroll
        for (int q = 0; q < TR / RPI; ++q) {
            float4* p = reinterpret_cast<float4*>(base + (size_t)(q * RPI + lane / LPR) * N + 4 * (lane % LPR));
            if (rd) {
                float4 v = *p;
                acc += v.x + v.y + v.z + v.w;
            } else {
                *p = float4{1.f, 2.f, 3.f, (float)q};
            }
        }
    }
    if (rd && acc == 1234.5f) sink[0] = acc;
}

template <class F>
static float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main() {
    float *C, *sink;
    if (hipMalloc(&C, sizeof(float) * (size_t)M * N) != hipSuccess) return 1;
    hipMalloc(&sink, 64);
    const double bytes = 4.0 * M * N;
    for (int rd = 0; rd < 2; ++rd) {
        const char* what = rd ? "read " : "write";
        float t = timeit([&] { hipLaunchKernelGGL(k_rows, dim3(M), dim3(256), 0, 0, C, rd, sink); });
        printf("%s rows                     %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_mfma<64, 32>), dim3(16, M / 64), dim3(64), 0, 0, C, rd, sink); });
        printf("%s mfma tiles 64x32, G 16     %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_mfma<64, 32>), dim3(64, M / 64), dim3(64), 0, 0, C, rd, sink); });
        printf("%s mfma tiles 64x32, G 64     %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_mfma<16, 256>), dim3(16, M / 16), dim3(64), 0, 0, C, rd, sink); });
        printf("%s mfma tiles 16x256, G 16    %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_f4<64, 32>), dim3(16, M / 64), dim3(64), 0, 0, C, rd, sink); });
        printf("%s f4 tiles 64x32, G 16       %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_f4<64, 32>), dim3(64, M / 64), dim3(64), 0, 0, C, rd, sink); });
        printf("%s f4 tiles 64x32, G 64       %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_f4<16, 256>), dim3(16, M / 16), dim3(64), 0, 0, C, rd, sink); });
        printf("%s f4 tiles 16x256, G 16      %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_f4<64, 128>), dim3(16, M / 64), dim3(64), 0, 0, C, rd, sink); });
        printf("%s f4 tiles 64x128, G 16      %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL((k_tiles_f4<4, 256>), dim3(16, M / 4), dim3(64), 0, 0, C, rd, sink); });
        printf("%s f4 tiles 4x256, G 16       %8.1f us %7.0f GB/s\n", what, t * 1e3, bytes / t / 1e6);
    }
    return 0;
}
