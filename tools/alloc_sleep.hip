// alloc_sleep.hip -- is the driver's wipe of freed HBM done in the background (tool)?
// Dirties GB bytes (allocate, write, free), then for each pause S: sleep S seconds, time a
// hipMalloc of the same size, write it, free it.  If the wipe runs in the background after
// a free, a longer pause makes the next allocation fast; if it runs when the memory is
// handed out again, every allocation waits the same.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/alloc_sleep tools/alloc_sleep.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <chrono>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__global__ void touch(float4 *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 150.0;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)((2 << 20) - 1);
    const double pauses[] = {0.0, 0.0, 2.0, 5.0, 10.0, 0.0};
    void *p = nullptr;
    for (double s : pauses) {
        if (s > 0) usleep((useconds_t)(s * 1e6));
        double t0 = now();
        CK(hipMalloc(&p, bytes));
        const double ta = now() - t0;
        t0 = now();
        hipLaunchKernelGGL(touch, dim3(8192), dim3(256), 0, 0, (float4 *)p, bytes / 16);
        CK(hipDeviceSynchronize());
        const double tw = now() - t0;
        t0 = now();
        CK(hipFree(p));
        const double tf = now() - t0;
        printf("{\"GB\": %.0f, \"pause_s\": %.1f, \"alloc_s\": %.4f, \"write_s\": %.4f, \"free_s\": %.4f}\n", gb, s, ta,
               tw, tf);
        fflush(stdout);
    }
    return 0;
}
