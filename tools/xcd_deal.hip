// Which XCD does each workgroup of a launch land on? (round-5 diagnosis of the
// PM 1 cluster fault, not product code.) Cluster mode assumes that blocks b, b+8,
// b+16, ... of a grid share one XCD (blocks dealt round-robin over the 8 XCDs).
// This launches a one-workgroup-per-CU grid (1,024 threads, 64 KB of dynamic
// LDS, like the routes kernel) with a plain launch and with
// hipLaunchCooperativeKernel, records HW_REG_XCC_ID per block, and counts the
// blocks whose XCD is not (block % 8), and the 4-wide clusters {b, b+8, b+16, b+24}
// (the kernel's member rule) whose members span several XCDs.
// Build: hipcc -O3 --offload-arch=gfx950 tools/xcd_deal.hip -o tools/xcd_deal
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));               \
            return 2;                                                         \
        }                                                                     \
    } while (0)

__global__ void __launch_bounds__(1024) k_where(int* xcc) {
    extern __shared__ int lds[];
    lds[threadIdx.x] = int(threadIdx.x);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        // (a vector store: the value is moved to a VGPR first)
        const int v = int(x & 15) + lds[1] - 1;
        __hip_atomic_store(&xcc[blockIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

static void report(const char* name, const std::vector<int>& x, int cl) {
    const int n = int(x.size());
    int off = 0, span = 0, nclu = 0;
    for (int b = 0; b < n; ++b) off += x[b] != (b & 7);
    // the kernel's member rule when grid % (8 * cl) == 0: member r of cluster
    // (b & 7) + 8 * q is block ((q * cl + r) << 3) | (b & 7)
    if (n % (8 * cl) == 0)
        for (int q = 0; q < n / (8 * cl); ++q)
            for (int lo = 0; lo < 8; ++lo) {
                int mask = 0;
                for (int r = 0; r < cl; ++r) mask |= 1 << x[((q * cl + r) << 3) | lo];
                ++nclu;
                span += (mask & (mask - 1)) != 0;
            }
    std::printf("%-12s grid %d: blocks not on XCD (b %% 8): %d; %d-wide clusters spanning XCDs: %d of %d; first 16:",
                name, n, off, cl, span, nclu);
    for (int b = 0; b < 16 && b < n; ++b) std::printf(" %d", x[b]);
    std::printf("\n");
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t dyn = 64 << 10;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_where), hipFuncAttributeMaxDynamicSharedMemorySize, int(dyn)));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_where, 1024, dyn));
    const int grid = cus * occ;
    std::printf("CUs %d, blocks per CU %d, grid %d\n", cus, occ, grid);
    int* d;
    CK(hipMalloc(&d, grid * sizeof(int)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<int> h(grid);
    for (int r = 0; r < reps; ++r)
        for (int coop = 0; coop < 2; ++coop) {
            CK(hipMemsetAsync(d, 0xFF, grid * sizeof(int), st));
            if (coop) {
                void* args[] = {&d};
                CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_where), dim3(grid), dim3(1024), args,
                                              unsigned(dyn), st));
            } else {
                hipLaunchKernelGGL(k_where, dim3(grid), dim3(1024), dyn, st, d);
                CK(hipGetLastError());
            }
            CK(hipMemcpyAsync(h.data(), d, grid * sizeof(int), hipMemcpyDeviceToHost, st));
            CK(hipStreamSynchronize(st));
            report(coop ? "cooperative" : "plain", h, 4);
        }
    return 0;
}
