// Row-gather microbenchmark in the relaxation's geometry (experiments only, not the
// product): one 1,024-thread workgroup per CU (256 workgroups), each sub-group of L
// lanes reading random 128-B rows of a large buffer, U independent rows in flight
// per sub-group per step. Compares the kernel's form (16 lanes x 8 B per row) with
// 8 lanes x 16 B per row (two sources' distances per lane), at equal rows in flight
// per wave, to tell whether the per-CU limit is per lane-request or per line.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_rows.hip -o tools/ubench_rows
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// L lanes per row, each loading 128 / L bytes (L = 16: 8 B; L = 8: 16 B); U rows per step
template <int L, int U>
__global__ void __launch_bounds__(1024, 1) k_rows(const uint4* __restrict__ a, uint32_t nrows, int steps, uint32_t* out) {
    const int lane = threadIdx.x & 63, l = lane % L;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / L;
    uint64_t acc = 0;
    for (int k = 0; k < steps; ++k) {
        uint64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t r = hash32(gid * 7919u + (k * U + u) * 104729u) % nrows;
            if constexpr (L == 16) {
                v[u] = reinterpret_cast<const uint64_t*>(a)[size_t(r) * 16 + l];
            } else {
                const uint4 x = a[size_t(r) * 8 + l];
                v[u] = (uint64_t(x.y) << 32 | x.x) + (uint64_t(x.w) << 32 | x.z);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc == 0x1234567ull) out[0] = 1;
}

// the relaxation's mix per step: M random rows of the large buffer plus U - M re-reads
// of the step's first row (the L1-resident padding / tail rows of an arc block)
template <int L, int U, int M>
__global__ void __launch_bounds__(1024, 1) k_mix(const uint4* __restrict__ a, uint32_t nrows, int steps, uint32_t* out) {
    const int lane = threadIdx.x & 63, l = lane % L;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / L;
    uint64_t acc = 0;
    for (int k = 0; k < steps; ++k) {
        uint64_t v[U];
        const uint32_t r0 = hash32(gid * 7919u + (k * U) * 104729u) % nrows;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t r = u < M ? hash32(gid * 7919u + (k * U + u) * 104729u) % nrows : r0;
            if constexpr (L == 16) {
                v[u] = reinterpret_cast<const uint64_t*>(a)[size_t(r) * 16 + l];
            } else {
                const uint4 x = a[size_t(r) * 8 + l];
                v[u] = (uint64_t(x.y) << 32 | x.x) + (uint64_t(x.w) << 32 | x.z);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc == 0x1234567ull) out[0] = 1;
}

// 16 lanes x 8-B atomicMin into one random 128-B row per sub-group per step (the flush's
// improvement events): request counting with rocprofv3 --pmc
__global__ void __launch_bounds__(1024, 1) k_amin16(uint64_t* a, uint32_t nrows, int steps) {
    const int lane = threadIdx.x & 63, l = lane % 16;
    const uint32_t gid = (blockIdx.x * blockDim.x + threadIdx.x) / 16;
    for (int k = 0; k < steps; ++k) {
        const uint32_t r = hash32(gid * 7919u + k * 104729u) % nrows;
        __hip_atomic_fetch_min(&a[size_t(r) * 16 + l], uint64_t(k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
    const size_t bytes = size_t(argc > 1 ? atol(argv[1]) : 8192) << 20;
    void* buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0x11, bytes));
    uint32_t* out;
    CK(hipMalloc(&out, 64));
    const uint32_t nrows = uint32_t(bytes / 128);
    const int grid = 256, block = 1024, steps = 256;
#define RUN(L, U)                                                                                                \
    {                                                                                                            \
        float t = timeit([&] { hipLaunchKernelGGL((k_rows<L, U>), dim3(grid), dim3(block), 0, 0, (const uint4*)buf, nrows, steps, out); }); \
        const double rows = double(grid) * block / L * U * steps;                                                \
        printf("rows: %2d lanes x %2d B, %2d rows/sub-group/step (%3d per wave in flight): %7.2f Grows/s  %7.1f GB/s\n", \
               L, 128 / L, U, U * 64 / L, rows / t / 1e6, rows * 128 / t / 1e6);                                 \
    }
    if (argc > 2) {  // request counting: one launch each of the 128-B row forms
        hipLaunchKernelGGL((k_rows<16, 8>), dim3(grid), dim3(block), 0, 0, (const uint4*)buf, nrows, 64, out);
        hipLaunchKernelGGL((k_rows<8, 8>), dim3(grid), dim3(block), 0, 0, (const uint4*)buf, nrows, 64, out);
        hipLaunchKernelGGL(k_amin16, dim3(grid), dim3(block), 0, 0, (uint64_t*)buf, nrows, 64);
        CK(hipDeviceSynchronize());
        printf("counting launches: each form %.0f rows\n", double(grid) * block / 16 * 8 * 64);
        return 0;
    }
    RUN(16, 4) RUN(16, 8) RUN(16, 16) RUN(8, 2) RUN(8, 4) RUN(8, 8) RUN(8, 16)
#define MIX(L, U, M)                                                                                             \
    {                                                                                                            \
        float t = timeit([&] { hipLaunchKernelGGL((k_mix<L, U, M>), dim3(grid), dim3(block), 0, 0, (const uint4*)buf, nrows, steps, out); }); \
        const double rows = double(grid) * block / L * U * steps;                                                \
        printf("mix: %2d lanes x %2d B, %2d rows per step of which %d random: %7.2f Grows/s (all row accesses)\n", \
               L, 128 / L, U, M, rows / t / 1e6);                                                                \
    }
    MIX(16, 8, 8) MIX(8, 8, 8) MIX(16, 8, 6) MIX(8, 8, 6) MIX(16, 8, 5) MIX(8, 8, 5) MIX(16, 8, 3) MIX(8, 8, 3)
    return 0;
}
