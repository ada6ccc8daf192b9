// alloc_overlap.hip -- can a process compute on the GPU while another of its threads waits
// in hipMalloc for the driver's wipe of HBM freed by an earlier process (tool)?
// Run right after a process that wrote and freed 200 GB (tools/alloc_once 200 w): allocates
// a small buffer (clean memory: fast), starts a thread that allocates BIG GB, and meanwhile
// runs a memory-bound kernel on the small buffer in a loop on its own stream, printing when
// each one finished relative to the big allocation's start and end.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/alloc_overlap tools/alloc_overlap.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <thread>

__global__ void touch(float4 *p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(v, v, v, v);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const double small_gb = argc > 1 ? atof(argv[1]) : 20.0, big_gb = argc > 2 ? atof(argv[2]) : 150.0;
    const size_t sb = (size_t)(small_gb * 1e9) & ~(size_t)((2 << 20) - 1);
    const size_t bb = (size_t)(big_gb * 1e9) & ~(size_t)((2 << 20) - 1);
    if (hipFree(nullptr) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    void *s = nullptr;
    const double t0 = now();
    if (hipMalloc(&s, sb) != hipSuccess) return 1;
    printf("{\"small_GB\": %.0f, \"alloc_s\": %.4f}\n", small_gb, now() - t0);
    std::atomic<double> big_start{0}, big_end{0};
    void *b = nullptr;
    std::thread th([&] {
        big_start = now() - t0;
        hipError_t e = hipMalloc(&b, bb);
        big_end = now() - t0;
        if (e != hipSuccess) fprintf(stderr, "big hipMalloc: %s\n", hipGetErrorString(e));
    });
    int k = 0;
    double last = now() - t0;
    while (big_end.load() == 0 && k < 2000) {
        hipLaunchKernelGGL(touch, dim3(8192), dim3(256), 0, st, (float4 *)s, sb / 16, (float)k);
        if (hipStreamSynchronize(st) != hipSuccess) return 1;
        ++k;
        const double t = now() - t0;
        if (t - last > 0.25) {
            printf("{\"kernels_done\": %d, \"t_s\": %.3f}\n", k, t);
            fflush(stdout);
            last = t;
        }
    }
    th.join();
    printf("{\"big_GB\": %.0f, \"big_start_s\": %.4f, \"big_end_s\": %.4f, \"kernels_during\": %d}\n", big_gb,
           big_start.load(), big_end.load(), k);
    return 0;
}
