// alloc_once.hip -- one process, one large hipMalloc, timed (tool).  With "w" it also writes
// the memory, so that its exit leaves that much freed HBM for the driver to wipe.  Run
// back to back (tools/alloc_seq.sh) to see how an allocation right after another process's
// exit depends on its own size.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/alloc_once tools/alloc_once.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

__global__ void touch(float4 *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 20.0;
    const bool wr = argc > 2 && strcmp(argv[2], "w") == 0;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)((2 << 20) - 1);
    double t0 = now();
    if (hipFree(nullptr) != hipSuccess) return 1;  // runtime initialisation, not timed below
    const double tinit = now() - t0;
    void *p = nullptr;
    t0 = now();
    hipError_t e = hipMalloc(&p, bytes);
    const double ta = now() - t0;
    if (e != hipSuccess) {
        fprintf(stderr, "hipMalloc: %s\n", hipGetErrorString(e));
        return 1;
    }
    double tw = 0;
    if (wr) {
        t0 = now();
        hipLaunchKernelGGL(touch, dim3(8192), dim3(256), 0, 0, (float4 *)p, bytes / 16);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        tw = now() - t0;
    }
    printf("{\"GB\": %.0f, \"init_s\": %.4f, \"alloc_s\": %.4f, \"write_s\": %.4f}\n", gb, tinit, ta, tw);
    fflush(stdout);
    return 0;  // exit frees it
}
