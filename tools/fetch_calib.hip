// FETCH_SIZE calibration per access width on gfx950 (diagnostic; not the product).
//
// MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a wide
// (16 B/lane) coalesced read; other widths are uncalibrated.  drl_step reads
// 16-B LDS-DMA rows (ground) but also 4-B-per-lane rows (records, actions, MT
// words).  Each kernel below reads a known 1 GiB (past the 256 MiB Infinity
// Cache) with one access width; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/fetch_calib.bin
// and divide FETCH_SIZE*1024 by the byte count printed here.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <class T>
__global__ void read_width(const T* __restrict__ p, int64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const T v = p[i];
        if constexpr (sizeof(T) == 16) acc ^= v.x ^ v.y ^ v.z ^ v.w;
        else if constexpr (sizeof(T) == 8) acc ^= (uint32_t)v ^ (uint32_t)(v >> 32);
        else acc ^= (uint32_t)v;
    }
    if (acc == 0x12345679u) out[0] = acc;  // keeps the loads
}

// 8 lanes per 32-B row, rows 32 B apart: drl_step's record / action loads
__global__ void read_rows32(const uint32_t* __restrict__ p, int64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc ^= __builtin_nontemporal_load(p + i);
    if (acc == 0x12345679u) out[0] = acc;
}

int main() {
    const int64_t bytes = 1ll << 30;
    void* buf;
    uint32_t* out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(buf, 1, bytes));
    const dim3 grid(256 * 8 * 4), block(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(read_width<uint8_t>, grid, block, 0, 0, (const uint8_t*)buf, bytes, out);
        hipLaunchKernelGGL(read_width<uint16_t>, grid, block, 0, 0, (const uint16_t*)buf, bytes / 2, out);
        hipLaunchKernelGGL(read_width<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, bytes / 4, out);
        hipLaunchKernelGGL(read_width<uint64_t>, grid, block, 0, 0, (const uint64_t*)buf, bytes / 8, out);
        hipLaunchKernelGGL(read_width<uint4>, grid, block, 0, 0, (const uint4*)buf, bytes / 16, out);
        hipLaunchKernelGGL(read_rows32, grid, block, 0, 0, (const uint32_t*)buf, bytes / 4, out);
    }
    CHECK(hipDeviceSynchronize());
    printf("bytes read per kernel: %lld\n", (long long)bytes);
    return 0;
}
