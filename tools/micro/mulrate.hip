// Throughput of 32-bit integer multiplies vs 24-bit multiply-adds on gfx950 (independent chains,
// 8 per lane, every CU busy).  hipcc --offload-arch=gfx950 -O3 mulrate.hip -o mulrate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void k(int* out, int n, int c) {
    int x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x + j;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (KIND == 0) x[j] = x[j] * c;                 // v_mul_lo_u32
            else if (KIND == 1) x[j] = __mul24(x[j], c);    // v_mul_i32_i24
            else if (KIND == 2) x[j] = x[j] + c;            // v_add_u32
            else x[j] = __umulhi(uint32_t(x[j]), uint32_t(c));  // v_mul_hi_u32
        }
    }
    int s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND>
float run(int* d, int n) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k<KIND>, dim3(4096), dim3(256), 0, 0, d, n, 3);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<KIND>, dim3(4096), dim3(256), 0, 0, d, n, 3);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    int* d;
    hipMalloc(&d, 4096 * 256 * 4);
    const int n = 4096;
    const double ops = 4096.0 * 256 / 64 * n * 8;  // wave-instructions
    const char* names[4] = {"v_mul_lo_u32", "v_mul_i32_i24", "v_add_u32", "v_mul_hi_u32"};
    float ms[4] = {run<0>(d, n), run<1>(d, n), run<2>(d, n), run<3>(d, n)};
    for (int i = 0; i < 4; i++)
        printf("%-14s %8.3f ms  %6.2f cycles/wave-instr/SIMD (2.4 GHz, 1024 SIMDs)\n", names[i], ms[i],
               ms[i] * 1e-3 * 2.4e9 * 1024 / ops);
    return 0;
}
