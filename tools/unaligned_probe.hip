// Diagnostic: do 16-B global loads at 8-B (not 16-B) aligned addresses return
// the right data on this GPU?  (Obs rows of 294 floats are 8-B aligned.)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const float* src, float* dst, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* p = src + 2 + 6 * i;  // 8 mod 16 (i even) / 0 mod 16 alternating
    float4 v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 8), 16);
    const float4 w = *reinterpret_cast<const float4*>(p);  // compiler assumes 16-B alignment
    dst[8 * i + 0] = v.x; dst[8 * i + 1] = v.y; dst[8 * i + 2] = v.z; dst[8 * i + 3] = v.w;
    dst[8 * i + 4] = w.x; dst[8 * i + 5] = w.y; dst[8 * i + 6] = w.z; dst[8 * i + 7] = w.w;
}
int main() {
    const int n = 4096, m = 6 * n + 16;
    float *hs = (float*)malloc(m * 4), *hd = (float*)malloc(8 * n * 4);
    for (int i = 0; i < m; ++i) hs[i] = (float)i;
    float *ds, *dd;
    hipMalloc(&ds, m * 4);
    hipMalloc(&dd, 8 * n * 4);
    hipMemcpy(ds, hs, m * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, ds, dd, n);
    hipError_t e = hipDeviceSynchronize();
    hipMemcpy(hd, dd, 8 * n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 8; ++j) bad += hd[8 * i + j] != (float)(2 + 6 * i + (j & 3));
    printf("status %s, mismatches %d of %d\n", hipGetErrorString(e), bad, 8 * n);
    return bad ? 1 : 0;
}
