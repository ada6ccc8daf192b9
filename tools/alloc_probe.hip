// alloc_probe.hip -- how long do very large device allocations take on the MI355X (tool)?
// First dirties the memory (allocate, write and free 200 GB), then times, each followed by
// a free: one hipMalloc of GB bytes; the same as 8 pieces from 8 host threads at once;
// hipExtMallocWithFlags(default); hipMallocAsync; and one hipMalloc again.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/alloc_probe tools/alloc_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <thread>
#include <vector>

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

static void write_all(void *p, size_t bytes) {
    hipLaunchKernelGGL(touch, dim3(8192), dim3(256), 0, 0, (float4 *)p, bytes / 16);
    CK(hipDeviceSynchronize());
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 150.0;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)((2 << 20) - 1);
    void *p = nullptr;
    double t0;
    {
        const size_t dirty = (size_t)200e9;
        t0 = now();
        CK(hipMalloc(&p, dirty));
        double t1 = now();
        write_all(p, dirty);
        CK(hipFree(p));
        printf("{\"step\": \"dirty 200 GB\", \"alloc_s\": %.4f, \"write_s\": %.4f}\n", t1 - t0, now() - t1);
        fflush(stdout);
    }
    auto one = [&](const char *name) {
        t0 = now();
        CK(hipMalloc(&p, bytes));
        double ta = now() - t0;
        t0 = now();
        write_all(p, bytes);
        double tw = now() - t0;
        CK(hipFree(p));
        printf("{\"step\": \"%s\", \"GB\": %.0f, \"alloc_s\": %.4f, \"first_write_s\": %.4f}\n", name, gb, ta, tw);
        fflush(stdout);
    };
    one("hipMalloc");
    {
        const int nt = 8;
        const size_t piece = (bytes / nt) & ~(size_t)((2 << 20) - 1);
        std::vector<void *> ps(nt, nullptr);
        t0 = now();
        std::vector<std::thread> th;
        for (int i = 0; i < nt; ++i)
            th.emplace_back([&, i] {
                CK(hipSetDevice(0));
                CK(hipMalloc(&ps[i], piece));
            });
        for (auto &t : th) t.join();
        printf("{\"step\": \"8 threads x hipMalloc\", \"GB\": %.0f, \"alloc_s\": %.4f}\n", gb, now() - t0);
        fflush(stdout);
        for (void *q : ps) write_all(q, piece);
        for (void *q : ps) CK(hipFree(q));
    }
    one("hipMalloc after threads");
    {
        t0 = now();
        CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocDefault));
        printf("{\"step\": \"hipExtMallocWithFlags\", \"GB\": %.0f, \"alloc_s\": %.4f}\n", gb, now() - t0);
        write_all(p, bytes);
        CK(hipFree(p));
    }
    {
        hipStream_t s;
        CK(hipStreamCreate(&s));
        t0 = now();
        CK(hipMallocAsync(&p, bytes, s));
        CK(hipStreamSynchronize(s));
        printf("{\"step\": \"hipMallocAsync\", \"GB\": %.0f, \"alloc_s\": %.4f}\n", gb, now() - t0);
        write_all(p, bytes);
        CK(hipFreeAsync(p, s));
        CK(hipStreamSynchronize(s));
    }
    one("hipMalloc last");
    return 0;
}
