// fp64 VALU peak microbenchmark on MI355X: independent v_fma_f64 chains per lane.
// Reports TFLOP/s for 1..8 waves per SIMD (grid = 256 CUs x waves x 4 SIMDs).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ void __launch_bounds__(256) k_fma(double *out, int iters, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = fma(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    if (s == 12345.678) out[threadIdx.x] = s;
}

template <int CH>
void run(int waves_per_simd, double *d) {
    const int iters = 20000;
    dim3 grid(256 * waves_per_simd), block(256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_fma<CH>, grid, block, 0, 0, d, iters, 0.999999, 1e-7);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fma<CH>, grid, block, 0, 0, d, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * CH * (double)iters * grid.x * block.x;
    printf("chains %2d waves/SIMD %d : %7.2f TFLOP/s (%.3f ms)\n", CH, waves_per_simd, flops / ms / 1e9, ms);
}

int main() {
    double *d;
    hipMalloc(&d, 4096);
    for (int w : {1, 2, 3, 4, 8}) run<1>(w, d);
    for (int w : {1, 2, 3, 4}) run<2>(w, d);
    for (int w : {1, 2, 3, 4, 8}) run<4>(w, d);
    for (int w : {1, 2, 4, 8}) run<8>(w, d);
    return 0;
}
