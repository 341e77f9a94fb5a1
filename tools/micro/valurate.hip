// Issue rate of VALU instructions on gfx950 with every CU busy (16 waves per CU, 8 independent
// chains per lane; each instruction forced with inline asm so nothing folds).  Reports cycles per
// wave-instruction per SIMD at the clock the device reports.
// hipcc --offload-arch=gfx950 -O3 -Wno-unused-value valurate.hip -o valurate
#include <hip/hip_runtime.h>
#include <cstdio>

#define INS_LIST(X)                                                              \
    X(0, "v_add_u32 %0, %0, %1")                                                 \
    X(1, "v_add_u32_e64 %0, %0, %1")                                             \
    X(2, "v_and_b32 %0, %0, %1")                                                 \
    X(3, "v_lshlrev_b32 %0, %1, %0")                                             \
    X(4, "v_mul_u32_u24 %0, %0, %1")                                             \
    X(5, "v_max_i32 %0, %0, %1")                                                 \
    X(6, "v_cndmask_b32 %0, %0, %1, vcc")                                        \
    X(7, "v_cndmask_b32_e64 %0, %0, %1, vcc")                                    \
    X(8, "v_dot2c_i32_i16 %0, %1, %2")                                           \
    X(9, "v_add_f32 %0, %0, %1")                                                 \
    X(10, "v_fma_f32 %0, %0, %1, %2")                                            \
    X(11, "v_cvt_f32_i32 %0, %0")                                                \
    X(12, "v_alignbit_b32 %0, %0, %1, %2")                                       \
    X(13, "v_bfe_u32 %0, %0, %1, %2")                                            \
    X(14, "v_bfe_i32 %0, %0, %1, %2")                                            \
    X(15, "v_mad_u32_u24 %0, %0, %1, %2")                                        \
    X(16, "v_lshl_add_u32 %0, %0, %1, %2")                                       \
    X(17, "v_lshl_or_b32 %0, %0, %1, %2")                                        \
    X(18, "v_add3_u32 %0, %0, %1, %2")                                           \
    X(19, "v_or3_b32 %0, %0, %1, %2")                                            \
    X(20, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")                             \
    X(21, "v_med3_i32 %0, %0, %1, %2")                                           \
    X(22, "v_perm_b32 %0, %0, %1, %2")                                           \
    X(23, "v_mul_lo_u32 %0, %0, %1")                                             \
    X(24, "v_pk_add_u16 %0, %0, %1")                                             \
    X(25, "v_pk_max_i16 %0, %0, %1")                                             \
    X(26, "v_pk_mul_lo_u16 %0, %0, %1")                                          \
    X(27, "v_cvt_pk_u8_f32 %0, %1, 1, %0")                                       \
    X(28, "v_sat_pk_u8_i16 %0, %0")                                              \
    X(29, "v_xad_u32 %0, %0, %1, %2")                                            \
    X(30, "v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc")            \
    X(31, "v_min3_i32 %0, %0, %1, %2")                                          \
    X(32, "v_dot2_i32_i16 %0, %1, %2, %0")                                       \
    X(33, "v_mov_b32 %0, %1\n v_dot2c_i32_i16 %0, %1, %2")                       \
    X(34, "v_ashrrev_i32 %0, %1, %0")                                            \
    X(35, "v_mul_i32_i24 %0, %0, %1")                                            \
    X(36, "v_mad_i32_i24 %0, %0, %1, %2")                                        \
    X(37, "v_sub_u32 %0, %0, %1")                                                \
    X(38, "v_mul_hi_u32 %0, %0, %1")                                             \
    X(39, "v_floor_f32 %0, %0")                                                  \
    X(40, "v_mul_f32 %0, %0, %1")                                                \
    X(41, "v_mov_b32 %0, %1")

#define KCASE(N, S) else if (KIND == N) { _Pragma("unroll") for (int j = 0; j < 8; j++) asm volatile(S : "+v"(x[j]) : "v"(c), "v"(e) : "vcc"); }

template <int KIND>
__global__ void k(unsigned* out, int n, unsigned c, unsigned e) {
    unsigned x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x + j;
    for (int i = 0; i < n; i++) {
        if (KIND < 0) {}
        INS_LIST(KCASE)
    }
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 64-bit (packed f32) forms
template <int KIND>
__global__ void k64(unsigned long long* out, int n, unsigned long long c) {
    unsigned long long x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x + j;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (KIND == 0) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x[j]) : "v"(c));
            else if (KIND == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x[j]) : "v"(c));
            else if (KIND == 2) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(x[j]) : "v"(c));
            else asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x[j]) : "v"(c));
        }
    }
    unsigned long long s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static hipEvent_t ev0, ev1;
template <typename F, typename... A>
float timed(F f, A... a) {
    hipLaunchKernelGGL(f, dim3(4096), dim3(256), 0, 0, a...);
    hipEventRecord(ev0);
    hipLaunchKernelGGL(f, dim3(4096), dim3(256), 0, 0, a...);
    hipEventRecord(ev1);
    hipEventSynchronize(ev1);
    float ms;
    hipEventElapsedTime(&ms, ev0, ev1);
    return ms;
}

int main() {
    unsigned* d;
    hipMalloc(&d, 4096 * 256 * 8);
    hipEventCreate(&ev0);
    hipEventCreate(&ev1);
    const int n = 2048;
    const double ops = 4096.0 * 256 / 64 * n * 8;  // wave-instructions
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0);
    const double ghz = khz / 1e6;
    const double ref = timed(k<0>, d, n, 3u, 5u);
    printf("reference v_add_u32: %.3f ms (%.2f cycles at %.2f GHz)\n", ref, ref * 1e-3 * ghz * 1e9 * 1024 / ops, ghz);
#define KRUN(N, S) { const float ms = timed(k<N>, d, n, 3u, 5u); \
    printf("%-44s %7.3f ms  %5.2f cyc  x%.2f of v_add_u32\n", S, ms, ms * 1e-3 * ghz * 1e9 * 1024 / ops, ms / ref); }
    INS_LIST(KRUN)
    const char* n64[4] = {"v_pk_add_f32", "v_pk_fma_f32", "v_lshl_add_u64", "v_fma_f64"};
    for (int i = 0; i < 4; i++) {
        float ms = 0;
        auto* p = reinterpret_cast<unsigned long long*>(d);
        if (i == 0) ms = timed(k64<0>, p, n, 3ull);
        else if (i == 1) ms = timed(k64<1>, p, n, 3ull);
        else if (i == 2) ms = timed(k64<2>, p, n, 3ull);
        else ms = timed(k64<3>, p, n, 3ull);
        printf("%-44s %7.3f ms  %5.2f cyc  x%.2f of v_add_u32\n", n64[i], ms, ms * 1e-3 * ghz * 1e9 * 1024 / ops, ms / ref);
    }
    return 0;
}
