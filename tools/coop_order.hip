// Stream-order check for cooperative launches (round-4 diagnosis, not product code).
//
// The cluster kernels are launched with hipLaunchCooperativeKernel on the engine's
// stream right after asynchronous work on that stream: a pageable host-to-device
// copy (the sorted sources), hipMemsetAsync (guard word and bucket tickets) and
// hipMemset2DAsync (cluster records and private far sets). This program repeats
// that sequence with known patterns and has the cooperative kernel count the
// words it does not see in their final state. A kernel that only reads (bounded
// indices, no spin) cannot fault whatever it finds.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            return 2;                                                                     \
        }                                                                                 \
    } while (0)

__global__ void k_check(const unsigned* src, int n_src, unsigned pat, const unsigned* zw, int n_zw,
                        const unsigned char* z2d, size_t pitch, int width, int rows, unsigned long long* bad) {
    unsigned long long b0 = 0, b1 = 0, b2 = 0;
    const int t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    for (int i = t; i < n_src; i += nt) b0 += src[i] != (pat ^ unsigned(i));
    for (int i = t; i < n_zw; i += nt) b1 += zw[i] != 0u;
    for (int r = 0; r < rows; ++r)
        for (int i = t; i < width; i += nt) b2 += z2d[size_t(r) * pitch + i] != 0;
    if (b0) atomicAdd(&bad[0], b0);
    if (b1) atomicAdd(&bad[1], b1);
    if (b2) atomicAdd(&bad[2], b2);
}

__global__ void k_dirty(unsigned* zw, int n_zw, unsigned char* z2d, size_t bytes) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
    for (int i = t; i < n_zw; i += nt) zw[i] = 0xABCDEFu;
    for (size_t i = t; i < bytes; i += nt) z2d[i] = 0x5A;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    const int coop = argc > 2 ? atoi(argv[2]) : 1;
    const int n_src = 1 << 16, n_zw = 16;
    const int rows = 64, width = 36864;
    const size_t pitch = 638976;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned *d_src, *d_zw;
    unsigned char* d_2d;
    unsigned long long* d_bad;
    CK(hipMalloc(&d_src, n_src * 4));
    CK(hipMalloc(&d_zw, n_zw * 4));
    CK(hipMalloc(&d_2d, pitch * rows));
    CK(hipMalloc(&d_bad, 3 * 8));
    CK(hipMemset(d_bad, 0, 24));
    std::vector<unsigned> h(n_src);
    unsigned long long tot[3] = {0, 0, 0};
    int grid = 256, block = 1024;
    for (int r = 0; r < reps; ++r) {
        // make the state wrong first (kernel on the same stream), then the async
        // producers, then the cooperative consumer
        hipLaunchKernelGGL(k_dirty, dim3(256), dim3(256), 0, st, d_zw, n_zw, d_2d, pitch * rows);
        const unsigned pat = 0x9E3779B9u * unsigned(r + 1);
        for (int i = 0; i < n_src; ++i) h[i] = pat ^ unsigned(i);
        CK(hipMemcpyAsync(d_src, h.data(), n_src * 4, hipMemcpyHostToDevice, st));
        CK(hipMemsetAsync(d_zw, 0, n_zw * 4, st));
        CK(hipMemset2DAsync(d_2d, pitch, 0, width, rows, st));
        const unsigned* a0 = d_src; int a1 = n_src; unsigned a2 = pat; const unsigned* a3 = d_zw; int a4 = n_zw;
        const unsigned char* a5 = d_2d; size_t a6 = pitch; int a7 = width; int a8 = rows; unsigned long long* a9 = d_bad;
        void* args[] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7, &a8, &a9};
        if (coop)
            CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_check), dim3(grid), dim3(block), args, 0, st));
        else
            hipLaunchKernelGGL(k_check, dim3(grid), dim3(block), 0, st, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st));
        unsigned long long b[3];
        CK(hipMemcpy(b, d_bad, 24, hipMemcpyDeviceToHost));
        CK(hipMemset(d_bad, 0, 24));
        for (int k = 0; k < 3; ++k) tot[k] += b[k];
    }
    std::printf("coop=%d reps=%d stale words: copied sources %llu, memset words %llu, memset2D bytes %llu\n", coop, reps,
                tot[0], tot[1], tot[2]);
    return (tot[0] | tot[1] | tot[2]) ? 1 : 0;
}
