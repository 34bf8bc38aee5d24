// Diagnostic: how fast does the chip launch workgroups of the drl_step shape?
// Times empty / tiny kernels over the same grid geometries (hipEvents).
// Build: hipcc --offload-arch=gfx950 -O3 tools/dispatch_probe.hip -o gpurun_out/dispatch_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void __launch_bounds__(64) k_empty64(int* p) {
    extern __shared__ int s[];
    if (threadIdx.x == 1000) p[0] = s[0];
}
__global__ void __launch_bounds__(256) k_empty256(int* p) {
    extern __shared__ int s[];
    if (threadIdx.x == 1000) p[0] = s[0];
}
// persistent: each 64-lane block loops over `iters` virtual blocks
__global__ void __launch_bounds__(64) k_loop64(int* p, int iters) {
    extern __shared__ int s[];
    int acc = 0;
    for (int i = 0; i < iters; ++i) acc += s[(threadIdx.x + i) & 63];
    if (acc == 123456789) p[0] = acc;
}

template <class F>
static float time_it(F f, int reps = 50) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main() {
    int* d;
    hipMalloc(&d, 64);
    const int lds = 5 * 1024;
    for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
        float t = time_it([&] { hipLaunchKernelGGL(k_empty64, dim3(blocks), dim3(64), lds, 0, d); });
        printf("empty 64-thr blocks=%6d lds=%d: %7.2f us  (%.2f ns/block)\n", blocks, lds, t, t * 1e3 / blocks);
    }
    for (int blocks : {1024, 2048, 4096}) {
        float t = time_it([&] { hipLaunchKernelGGL(k_empty256, dim3(blocks), dim3(256), 4 * lds, 0, d); });
        printf("empty 256-thr blocks=%6d lds=%d: %7.2f us  (%.2f ns/wave)\n", blocks, 4 * lds, t, t * 1e3 / (4 * blocks));
    }
    for (int blocks : {8192}) {
        float t = time_it([&] { hipLaunchKernelGGL(k_empty64, dim3(blocks), dim3(64), 0, 0, d); });
        printf("empty 64-thr blocks=%6d lds=0: %7.2f us\n", blocks, t);
    }
    printf("done\n");
    return 0;
}
