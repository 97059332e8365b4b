// LDS float-atomic throughput probe (diagnostic tool, not shipped).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_lds_atomic.hip -o tools/bin/mb_lds && tools/bin/mb_lds
// Each wave issues ITER LDS ops; pattern: 0 = lane-distinct consecutive dwords, 1 = random
// dwords in 16 KB, 2 = 4 lanes per address (lane>>2), 3 = 16 lanes per address, 4 = all lanes
// one address.  OP: 0 = ds_add_f32 (atomicAdd, no return), 1 = ds_write_b32, 2 = ds_add_rtn.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 256;

template <int OP, int PAT>
__global__ __launch_bounds__(256) void k(float* out, int seed) {
    __shared__ float buf[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) buf[i] = 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned h = (unsigned)(lane * 2654435761u) ^ (unsigned)seed ^ (w * 97u);
    float acc = 0.f;
    for (int it = 0; it < ITER; ++it) {
        int a;
        if (PAT == 0) a = (lane + 64 * (it & 7) + 512 * w) & 4095;
        else if (PAT == 1) { h = h * 1664525u + 1013904223u; a = (h >> 8) & 4095; }
        else if (PAT == 2) a = ((lane >> 2) * 37 + it * 64 + w * 7) & 4095;
        else if (PAT == 3) a = ((lane >> 4) * 101 + it * 64 + w * 7) & 4095;
        else a = (it * 64 + w * 7) & 4095;
        if (OP == 0) atomicAdd(&buf[a], 1.f);
        else if (OP == 1) buf[a] = (float)it;
        else acc += atomicAdd(&buf[a], 1.f);
    }
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = buf[threadIdx.x] + acc;
}

template <int OP, int PAT>
void run(float* out, const char* name) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * 8;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k<OP, PAT>), dim3(grid), dim3(256), 0, 0, out, i);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k<OP, PAT>), dim3(grid), dim3(256), 0, 0, out, i);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 100.0;  // per launch
    const double wave_ops = (double)grid * 4 * ITER;
    // cycles per wave-instruction per CU at 2.4 GHz, 256 CUs
    const double cyc = us * 1e-6 * 2.4e9 * 256 / wave_ops;
    printf("%-34s %8.1f us   %6.2f CU-cycles per wave-op\n", name, us, cyc);
}

int main() {
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * 256 * 8);
    run<1, 0>(out, "write  distinct");
    run<1, 1>(out, "write  random");
    run<0, 0>(out, "atomic distinct");
    run<0, 1>(out, "atomic random");
    run<0, 2>(out, "atomic 4 lanes/addr");
    run<0, 3>(out, "atomic 16 lanes/addr");
    run<0, 4>(out, "atomic 64 lanes/addr");
    run<2, 0>(out, "atomic-rtn distinct");
    run<2, 1>(out, "atomic-rtn random");
    return 0;
}
