// Micro-test: global_load_lds_dwordx4 lane -> LDS address mapping on gfx950 (M0 = wave base).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(const uint4* src, uint32_t* out, int off) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) buf[i] = 0xDEADBEEFu;
    __syncthreads();
    const uint32_t base = uint32_t(size_t((__attribute__((address_space(3))) uint32_t*)buf)) + off;
    const uint4* p = src + threadIdx.x;
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_waitcnt vmcnt(0)" :: "s"(base), "v"(p) : "memory", "m0");
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 64) out[i] = buf[i];
}
int main() {
    std::vector<uint32_t> h(256);
    for (int i = 0; i < 256; i++) h[i] = 0x1000u + i;
    uint4* s; uint32_t* o;
    hipMalloc(&s, 4096); hipMalloc(&o, 8192);
    hipMemcpy(s, h.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, s, o, 1024);
    std::vector<uint32_t> r(2048);
    hipMemcpy(r.data(), o, 8192, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 2048; i++) {
        const uint32_t want = (i >= 256 && i < 512) ? 0x1000u + (i - 256) : 0xDEADBEEFu;
        if (r[i] != want) { if (bad < 8) printf("word %d: %08x want %08x\n", i, r[i], want); bad++; }
    }
    printf("ldsdma mapping (lane l -> M0 + 16 l): %s (%d bad words)\n", bad ? "MISMATCH" : "ok", bad);
    return bad != 0;
}
