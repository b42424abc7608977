// Memory-system microbenchmarks for the routing engine's access patterns on
// MI355X (experiments only; not part of the product).
//   stream     : coalesced 16 B/lane reads of a large array (HBM peak reference)
//   gather<R>  : random R-byte rows (R/8 lanes x 8 B), the relaxation's dist-row read
//   amin<R>    : random 8 B atomicMin (workgroup / agent scope) into R-byte rows
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench.hip -o tools/ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k_stream(const uint4* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// each group of L lanes reads one random row of L*8 bytes; `iters` rows per group
template <int L>
__global__ void k_gather(const uint64_t* __restrict__ a, uint32_t nrows, int iters, uint32_t* out) {
    const int lane = threadIdx.x & 63, sub = lane / L, l = lane % L;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / L;
    uint64_t acc = 0;
#pragma unroll 8
    for (int k = 0; k < iters; ++k) {
        const uint32_t r = hash32(gid * 7919u + k * 104729u) % nrows;
        acc += a[size_t(r) * L + l];
    }
    (void)sub;
    if (acc == 0x1234567ull) out[0] = 1;
}

template <int L, int SCOPE>
__global__ void k_amin(uint64_t* a, uint32_t nrows, int iters) {
    const int lane = threadIdx.x & 63, l = lane % L;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / L;
    for (int k = 0; k < iters; ++k) {
        const uint32_t r = hash32(gid * 7919u + k * 104729u) % nrows;
        __hip_atomic_fetch_min(&a[size_t(r) * L + l], uint64_t(k), __ATOMIC_RELAXED, SCOPE);
    }
}

// L-lane rows, only the first P lanes of each row take part (an improvement event
// where P of the bucket's sources improve)
template <int L, int P>
__global__ void k_amin_part(uint64_t* a, uint32_t nrows, int iters) {
    const int lane = threadIdx.x & 63, l = lane % L;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / L;
    for (int k = 0; k < iters; ++k) {
        const uint32_t r = hash32(gid * 7919u + k * 104729u) % nrows;
        if (l < P) __hip_atomic_fetch_min(&a[size_t(r) * L + l], uint64_t(k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

template <int L>
__global__ void k_store(uint64_t* a, uint32_t nrows, int iters) {
    const int lane = threadIdx.x & 63, l = lane % L;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / L;
    for (int k = 0; k < iters; ++k) {
        const uint32_t r = hash32(gid * 7919u + k * 104729u) % nrows;
        a[size_t(r) * L + l] = uint64_t(k);
    }
}

template <typename F>
float timeit(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main(int argc, char** argv) {
    size_t bytes = (argc > 1 ? atol(argv[1]) : 8192) * (1ull << 20);
    void* buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0xff, bytes));
    uint32_t* out;
    CK(hipMalloc(&out, 64));
    const int grid = 256 * 16, block = 256;
    float ms = timeit([&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, bytes / 16, out); });
    printf("stream read            %8.1f GB/s (%zu MiB)\n", bytes / ms / 1e6, bytes >> 20);
    const int iters = 256;
#define GATHER(L)                                                                                               \
    {                                                                                                           \
        uint32_t nrows = uint32_t(bytes / (L * 8));                                                             \
        float t = timeit([&] { hipLaunchKernelGGL(k_gather<L>, dim3(grid), dim3(block), 0, 0, (const uint64_t*)buf, nrows, iters, out); }); \
        double rows = double(grid) * block / L * iters;                                                         \
        printf("gather row %4d B      %8.1f GB/s useful, %8.2f Grows/s\n", L * 8, rows * L * 8 / t / 1e6, rows / t / 1e6); \
    }
    GATHER(1) GATHER(2) GATHER(4) GATHER(8) GATHER(16) GATHER(32) GATHER(64)
#define AMIN(L, S, NAME)                                                                                        \
    {                                                                                                           \
        uint32_t nrows = uint32_t(bytes / (L * 8));                                                             \
        float t = timeit([&] { hipLaunchKernelGGL((k_amin<L, S>), dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, nrows, 64); }); \
        double ops = double(grid) * block * 64;                                                                 \
        printf("atomicMin %-9s rows %3d B  %8.2f Gatomics/s\n", NAME, L * 8, ops / t / 1e6);                   \
    }
    AMIN(1, __HIP_MEMORY_SCOPE_WORKGROUP, "wg") AMIN(16, __HIP_MEMORY_SCOPE_WORKGROUP, "wg")
    AMIN(1, __HIP_MEMORY_SCOPE_AGENT, "agent") AMIN(16, __HIP_MEMORY_SCOPE_AGENT, "agent")
    // partial-row atomics: lane rate and event (row) rate
#define APART(P)                                                                                              \
    for (size_t sb : {size_t(192) << 20, bytes}) {                                                            \
        uint32_t nrows = uint32_t(sb / 128);                                                                  \
        float t = timeit([&] { hipLaunchKernelGGL((k_amin_part<16, P>), dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, nrows, 64); }); \
        double ev = double(grid) * block / 16 * 64;                                                           \
        printf("atomicMin %2d of 16 lanes, ws %6zu MiB: %8.2f Glane-atomics/s  %8.2f Gevents/s\n", P, sb >> 20, ev * P / t / 1e6, ev / t / 1e6); \
    }
    APART(1) APART(2) APART(4) APART(8) APART(16)
    // atomics and stores on small (L2-resident) and large working sets
    {
        size_t sizes[] = {2ull << 20, 192ull << 20, bytes};
        for (size_t sb : sizes) {
            uint32_t n1 = uint32_t(sb / 8), n16 = uint32_t(sb / 128);
            double ops = double(grid) * block * 64;
            float t1 = timeit([&] { hipLaunchKernelGGL((k_amin<1, __HIP_MEMORY_SCOPE_WORKGROUP>), dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, n1, 64); });
            float t2 = timeit([&] { hipLaunchKernelGGL((k_amin<1, __HIP_MEMORY_SCOPE_AGENT>), dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, n1, 64); });
            float t3 = timeit([&] { hipLaunchKernelGGL((k_store<1>), dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, n1, 64); });
            float t4 = timeit([&] { hipLaunchKernelGGL((k_store<16>), dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, n16, 64); });
            printf("ws %6zu MiB: atomicMin 8B wg %6.2f G/s, agent %6.2f G/s; store 8B %6.2f G/s; store 128B rows %6.2f Grows/s\n",
                   sb >> 20, ops / t1 / 1e6, ops / t2 / 1e6, ops / t3 / 1e6, ops / 16 / t4 / 1e6);
        }
    }
    // small working set (L2/MALL resident) gather
    {
        size_t small[] = {2ull << 20, 32ull << 20, 192ull << 20};
        for (size_t sb : small) {
            uint32_t nrows = uint32_t(sb / 128);
            float t = timeit([&] { hipLaunchKernelGGL(k_gather<16>, dim3(grid), dim3(block), 0, 0, (const uint64_t*)buf, nrows, iters, out); });
            double rows = double(grid) * block / 16 * iters;
            printf("gather 128 B rows in %4zu MiB  %8.1f GB/s useful\n", sb >> 20, rows * 128 / t / 1e6);
        }
    }
    return 0;
}
