// alloc_probe.hip -- how long do very large device allocations take on the MI355X (tool)?
// Times several allocation APIs for one large size: hipMalloc, hipMalloc again after a
// hipFree, hipExtMallocWithFlags (default / uncached), hipMallocAsync (default pool, then
// again after a free), the VMM path (hipMemCreate + hipMemMap), and 16 GB pieces.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/alloc_probe tools/alloc_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
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

static void report(const char *what, double gb, double t_alloc, void *p, size_t bytes) {
    double t0 = now();
    hipLaunchKernelGGL(touch, dim3(8192), dim3(256), 0, 0, (float4 *)p, bytes / 16);
    CK(hipDeviceSynchronize());
    printf("{\"api\": \"%s\", \"GB\": %.0f, \"alloc_s\": %.4f, \"first_write_s\": %.4f}\n", what, gb, t_alloc,
           now() - t0);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const double gb = argc > 1 ? atof(argv[1]) : 100.0;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)((2 << 20) - 1);
    void *p = nullptr;
    double t0;
    // 1. hipMalloc, twice (the second after a free)
    for (int rep = 0; rep < 2; ++rep) {
        t0 = now();
        CK(hipMalloc(&p, bytes));
        report(rep ? "hipMalloc_again" : "hipMalloc", gb, now() - t0, p, bytes);
        t0 = now();
        CK(hipFree(p));
        printf("{\"api\": \"hipFree\", \"s\": %.4f}\n", now() - t0);
    }
    // 2. hipExtMallocWithFlags
    t0 = now();
    CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocDefault));
    report("hipExtMallocWithFlags_default", gb, now() - t0, p, bytes);
    CK(hipFree(p));
    t0 = now();
    CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
    report("hipExtMallocWithFlags_uncached", gb, now() - t0, p, bytes);
    CK(hipFree(p));
    // 3. stream-ordered allocator (default pool), twice
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int rep = 0; rep < 2; ++rep) {
        t0 = now();
        CK(hipMallocAsync(&p, bytes, s));
        CK(hipStreamSynchronize(s));
        report(rep ? "hipMallocAsync_again" : "hipMallocAsync", gb, now() - t0, p, bytes);
        CK(hipFreeAsync(p, s));
        CK(hipStreamSynchronize(s));
    }
    // 4. VMM: physical handle + map
    {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        size_t gran = 0;
        CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
        size_t sz = (bytes + gran - 1) / gran * gran;
        t0 = now();
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, sz, &prop, 0));
        double t1 = now();
        void *va = nullptr;
        CK(hipMemAddressReserve(&va, sz, 0, nullptr, 0));
        CK(hipMemMap(va, sz, 0, h, 0));
        hipMemAccessDesc acc = {};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CK(hipMemSetAccess(va, sz, &acc, 1));
        printf("{\"api\": \"hipMemCreate\", \"s\": %.4f, \"map_s\": %.4f, \"gran\": %zu}\n", t1 - t0, now() - t1, gran);
        report("vmm", gb, now() - t0, va, sz);
        CK(hipMemUnmap(va, sz));
        CK(hipMemRelease(h));
        CK(hipMemAddressFree(va, sz));
    }
    // 5. 16 GB pieces
    {
        const size_t piece = (size_t)16e9 & ~(size_t)((2 << 20) - 1);
        std::vector<void *> ps;
        t0 = now();
        for (size_t done = 0; done < bytes; done += piece) {
            void *q;
            CK(hipMalloc(&q, piece));
            ps.push_back(q);
        }
        printf("{\"api\": \"hipMalloc_16GB_pieces\", \"GB\": %.0f, \"alloc_s\": %.4f}\n", gb, now() - t0);
        for (void *q : ps) CK(hipFree(q));
    }
    return 0;
}
