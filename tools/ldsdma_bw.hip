// Per-CU load bandwidth of LDS-DMA (global_load_lds_dwordx4) and of plain global_load_dwordx4
// into registers, for an L2-resident source (a small buffer every workgroup re-reads) and an
// HBM-streaming one.  One 512-thread workgroup per CU, `iters` stages of 64 KB each.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ldsdma_bw.hip -o tools/probe/ldsdma_bw
// Measured (1xMI355X): glds 98 B/ns/CU from L2, 30 B/ns/CU (7.75 TB/s) streaming from HBM;
// register loads 117 / 26 B/ns/CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void __launch_bounds__(512, 1) dma_kernel(const char* src, size_t span, int iters, unsigned* sink) {
    __shared__ __attribute__((aligned(16))) char L[2][65536];
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    size_t base = (size_t)blockIdx.x * 65536 * 4;
    for (int it = 0; it < iters; ++it) {
        const size_t off = (base + (size_t)it * 65536) % span;
        // 64 KB per stage: 64 wave-instructions of 1 KB, 8 per wave
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int j = 8 * wave + q;
            const char* g = src + off + (size_t)j * 1024 + lane * 16;
            __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(&L[it & 1][j * 1024]), 16, 0, 0);
        }
        __syncthreads();
    }
    if (tid == 0) sink[blockIdx.x] = L[0][lane] + L[1][lane * 3];
}

__global__ void __launch_bounds__(512, 1) reg_kernel(const char* src, size_t span, int iters, unsigned* sink) {
    const int tid = threadIdx.x;
    size_t base = (size_t)blockIdx.x * 65536 * 4;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (int it = 0; it < iters; ++it) {
        const size_t off = (base + (size_t)it * 65536) % span;
        uint4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const uint4*>(src + off + (size_t)q * 8192 + tid * 16);
#pragma unroll
        for (int q = 0; q < 8; ++q) { acc.x ^= v[q].x; acc.y += v[q].y; acc.z ^= v[q].z; acc.w += v[q].w; }
    }
    if (acc.x == 0x12345678u) sink[blockIdx.x] = acc.y + acc.z + acc.w;
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const size_t big = (size_t)1 << 31;   // 2 GiB: HBM streaming
    char* buf;
    unsigned* sink;
    hipMalloc(&buf, big);
    hipMalloc(&sink, 4096 * 4);
    hipMemset(buf, 1, big);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 256;
    struct { const char* name; size_t span; } spans[] = {{"L2 (2 MiB)", (size_t)2 << 20}, {"MALL (64 MiB)", (size_t)64 << 20}, {"HBM (2 GiB)", big}};
    for (int kind = 0; kind < 2; ++kind)
        for (auto& sp : spans) {
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (kind == 0) dma_kernel<<<cus, 512>>>(buf, sp.span, iters, sink);
                else reg_kernel<<<cus, 512>>>(buf, sp.span, iters, sink);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)cus * iters * 65536;
            printf("%-4s %-14s %8.1f us  %7.2f TB/s  %6.1f B/ns/CU\n", kind == 0 ? "glds" : "regs", sp.name,
                   ms * 1e3, bytes / ms / 1e9, bytes / ms / 1e6 / cus);
        }
    return 0;
}
