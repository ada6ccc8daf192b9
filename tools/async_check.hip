// async_check.hip -- does memory from hipMallocAsync hold what is written to it, for very
// large sizes (tool)?  For each size: allocate (hipMallocAsync, default pool), write
// p[i] = i (uint32, wrapping) with one kernel, count mismatches with another, free.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/async_check tools/async_check.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__global__ void fill(uint32_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)(i * 2654435761u);
}

__global__ void check(const uint32_t *p, size_t n, unsigned long long *bad, unsigned long long *first) {
    unsigned long long b = 0, f = ~0ull;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != (uint32_t)(i * 2654435761u)) {
            ++b;
            if (i < f) f = i;
        }
    if (b) {
        atomicAdd(bad, b);
        atomicMin(first, f);
    }
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;  // 0 = async, 1 = hipMalloc
    const double gbs[] = {8, 100, 140, 150, 200, 215};
    unsigned long long *d = nullptr;
    CK(hipMalloc(&d, 16));
    for (double gb : gbs) {
        size_t bytes = (size_t)(gb * 1e9) & ~(size_t)4095;
        size_t n = bytes / 4;
        uint32_t *p = nullptr;
        if (mode == 0) {
            CK(hipMallocAsync(reinterpret_cast<void **>(&p), bytes, nullptr));
            CK(hipStreamSynchronize(nullptr));
        } else {
            CK(hipMalloc(&p, bytes));
        }
        unsigned long long h[2] = {0, ~0ull};
        CK(hipMemcpy(d, h, 16, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(fill, dim3(16384), dim3(256), 0, 0, p, n);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, 0, p, n, d, d + 1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        printf("{\"mode\": \"%s\", \"GB\": %.0f, \"ptr\": \"%p\", \"bad\": %llu, \"first_bad_byte\": %llu}\n",
               mode == 0 ? "async" : "hipMalloc", gb, (void *)p, h[0], h[0] ? h[1] * 4 : 0ull);
        fflush(stdout);
        if (mode == 0) {
            CK(hipFreeAsync(p, nullptr));
            CK(hipStreamSynchronize(nullptr));
        } else {
            CK(hipFree(p));
        }
    }
    return 0;
}
