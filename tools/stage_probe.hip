// Diagnostic: how fast can every CU stage the same weight image (L2-shared)
// into its LDS?  The code act's layer 0 needs its 160 KB hi + lo image in each
// CU's LDS every launch; this times that staging alone, by size, waves per
// workgroup and load form (LDS-DMA vs register loads + ds_write), against an
// empty launch of the same grid and LDS size (hipEvents, back-to-back launches:
// L2-warm, as the act runs after the step in the train loop... which evicts it;
// the "flush" rows overwrite 256 MB between launches).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stage_probe.hip -o tools/stage_probe.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void g_void;

__global__ void __launch_bounds__(512) k_empty(int* out) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    if (threadIdx.x == 1000) out[0] = wl[0].x;
}

// LDS-DMA: n_kb KB from src (the same for every block) into LDS, 1 KB per wave-instruction
__global__ void __launch_bounds__(512) k_dma(const uint4* __restrict__ src, int n_kb, int* out) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int k = wave; k < n_kb; k += nw)
        __builtin_amdgcn_global_load_lds((g_void*)(src + k * 64 + lane), (lds_void*)(wl + k * 64), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = wl[(n_kb - 1) * 64 + 7].x;
}

// register loads, then ds_write_b128
__global__ void __launch_bounds__(512) k_reg(const uint4* __restrict__ src, int n_kb, int* out) {
    extern __shared__ __attribute__((aligned(16))) uint4 wl[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint4 r[24];
    int k0 = wave;
    while (k0 < n_kb) {
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int k = k0 + i * nw;
            if (k < n_kb) r[i] = src[k * 64 + lane];
        }
#pragma unroll
        for (int i = 0; i < 24; ++i) {
            const int k = k0 + i * nw;
            if (k < n_kb) wl[k * 64 + lane] = r[i];
        }
        k0 += 24 * nw;
    }
    __syncthreads();
    if (threadIdx.x == 0 && wl[(n_kb - 1) * 64 + 7].x == 0xdeadbeef) out[0] = 1;
}

static void check(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        printf("%s: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

template <class F>
static float time_it(F f, int reps = 100, uint4* junk = nullptr, size_t junk_bytes = 0) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    check("launch");
    hipDeviceSynchronize();
    check("sync");
    if (!junk) {
        hipEventRecord(a, 0);
        for (int i = 0; i < reps; ++i) f();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        return ms * 1e3f / reps;
    }
    float tot = 0;
    for (int i = 0; i < reps; ++i) {
        hipMemsetAsync(junk, i & 0xff, junk_bytes, 0);
        hipEventRecord(a, 0);
        f();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        tot += ms;
    }
    return tot * 1e3f / reps;
}

int main() {
    int* d;
    uint4* src;
    uint4* junk;
    hipMalloc(&d, 64);
    hipMalloc(&src, 256 * 1024);
    hipMemset(src, 1, 256 * 1024);
    const size_t jb = 256u << 20;
    hipMalloc(&junk, jb);
    int dev = 0, cus = 0;
    for (void* k : {(void*)k_empty, (void*)k_dma, (void*)k_reg})
        hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    printf("CUs %d\n", cus);
    for (int waves : {4, 8}) {
        for (int kb : {8, 16, 32, 64, 96, 128, 160}) {
            const size_t lds = (size_t)kb * 1024;
            const dim3 g(cus), blk(64 * waves);
            const float te = time_it([&] { hipLaunchKernelGGL(k_empty, g, blk, lds, 0, d); });
            const float td = time_it([&] { hipLaunchKernelGGL(k_dma, g, blk, lds, 0, src, kb, d); });
            const float tr = time_it([&] { hipLaunchKernelGGL(k_reg, g, blk, lds, 0, src, kb, d); });
            const float tdf = time_it([&] { hipLaunchKernelGGL(k_dma, g, blk, lds, 0, src, kb, d); }, 30, junk, jb);
            const float tef = time_it([&] { hipLaunchKernelGGL(k_empty, g, blk, lds, 0, d); }, 30, junk, jb);
            printf("waves %d  %3d KB/CU: empty %6.2f us  dma %6.2f us (%5.1f B/ns/CU over empty)  reg %6.2f us  "
                   "| after a 256 MB overwrite: empty %6.2f dma %6.2f us\n",
                   waves, kb, te, td, kb * 1024.0 / ((td - te) * 1e3), tr, tef, tdf);
        }
    }
    int h[2] = {0, 0};
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("LDS word after the DMA: %08x (expect 01010101)\n", h[1]);
    printf("done\n");
    return 0;
}
