// Co-residency probe: which resources keep a small one-wave kernel (B, the IDCT
// shape: 64 threads, ~8 KB LDS, NVB live VGPRs) from starting beside a long resident kernel (A, the
// k_piece shape: one round of WA-thread workgroups with LDS_A bytes of dynamic LDS, NVA live VGPRs).
// A's workgroups spin for DUR us of wall clock; B is launched on a second stream right after.
// Prints, per case, how many of B's workgroups started before A's first workgroup ended.
//   hipcc -O3 --offload-arch=gfx950 -o cores tools/micro/cores.hip && ./cores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <int NV>
__device__ __forceinline__ void burn(uint32_t (&v)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; i++) asm volatile("v_add_u32 %0, 1, %0" : "+v"(v[i]));
}

template <int WA, int NVA>
__global__ __launch_bounds__(WA) void kA(unsigned long long* t, unsigned long long dur, uint32_t* sink) {
    extern __shared__ uint32_t lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v[NVA];
#pragma unroll
    for (int i = 0; i < NVA; i++) v[i] = threadIdx.x + i;
    lds[threadIdx.x] = v[0];
    while (__builtin_amdgcn_s_memrealtime() - t0 < dur) burn(v);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < NVA; i++) acc += v[i];
    if (acc == 0x12345u) sink[0] = acc + lds[threadIdx.x ^ 1];
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

template <int NVB>
__global__ __launch_bounds__(64) void kB(unsigned long long* t, unsigned long long dur, uint32_t* sink) {
    __shared__ uint32_t s[8112 / 4];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v[NVB];
#pragma unroll
    for (int i = 0; i < NVB; i++) v[i] = threadIdx.x * 3 + i;
    s[threadIdx.x] = v[1];
    while (__builtin_amdgcn_s_memrealtime() - t0 < dur) burn(v);
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < NVB; i++) acc += v[i];
    if (acc == 0x12345u) sink[0] = acc + s[threadIdx.x ^ 3];
    if (threadIdx.x == 0) t[blockIdx.x] = t0;
}

template <int WA, int NVA, int NVB>
void run_case(const char* name, size_t lds_a, int wgs_per_cu) {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int na = cus * wgs_per_cu, nb = cus * 8;
    unsigned long long *ta, *tb;
    uint32_t* sink;
    CHK(hipMalloc(&ta, sizeof(unsigned long long) * 2 * na));
    CHK(hipMalloc(&tb, sizeof(unsigned long long) * nb));
    CHK(hipMalloc(&sink, 64));
    CHK(hipFuncSetAttribute(reinterpret_cast<const void*>(&kA<WA, NVA>), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_a)));
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kA<WA, NVA>, WA, lds_a));
    hipStream_t s1, s2;
    CHK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL((kA<WA, NVA>), dim3(na), dim3(WA), lds_a, s1, ta, 200000ull /* 2 ms */, sink);
        hipLaunchKernelGGL(kB<NVB>, dim3(nb), dim3(64), 0, s2, tb, 2000ull /* 20 us */, sink);
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> ha(2 * na), hb(nb);
    CHK(hipMemcpy(ha.data(), ta, ha.size() * 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(hb.data(), tb, hb.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long a_start = ~0ull, a_end_min = ~0ull, a_end_max = 0;
    for (int i = 0; i < na; i++) {
        a_start = std::min(a_start, ha[2 * i]);
        a_end_min = std::min(a_end_min, ha[2 * i + 1]);
        a_end_max = std::max(a_end_max, ha[2 * i + 1]);
    }
    int before = 0;
    unsigned long long b_first = ~0ull;
    for (int i = 0; i < nb; i++) {
        before += hb[i] < a_end_min;
        b_first = std::min(b_first, hb[i]);
    }
    std::printf("%-44s A: %d x %d thr, lds %zu, occ %d/CU | B started beside A: %5d / %d (first B at %+.0f us of A's %.0f us)\n",
                name, na, WA, lds_a, occ, before, nb, (double(b_first) - double(a_start)) / 100.0,
                (double(a_end_max) - double(a_start)) / 100.0);
    CHK(hipFree(ta));
    CHK(hipFree(tb));
    CHK(hipFree(sink));
    CHK(hipStreamDestroy(s1));
    CHK(hipStreamDestroy(s2));
}

int main() {
    // k_piece<1024> at 96 VGPRs beside the 88-VGPR IDCT wave (co1024): fits by VGPR and LDS
    run_case<1024, 88, 80>("1024 x 96v A, lds 128640 | 88v B", 128640, 1);
    run_case<1024, 88, 80>("1024 x 96v A, lds 96000 | 88v B", 96000, 1);
    run_case<1024, 88, 24>("1024 x 96v A, lds 96000 | 32v B", 96000, 1);
    run_case<1024, 24, 24>("1024 x 32v A, lds 96000 | 32v B", 96000, 1);
    run_case<1024, 24, 24>("1024 x 32v A, lds 16384 | 32v B", 16384, 1);
    run_case<512, 24, 24>("512 x 32v A x2, lds 16384 | 32v B", 16384, 2);
    run_case<512, 104, 80>("512 x 112v A x2, lds 81536 | 88v B (control)", 81536, 2);
    return 0;
}
