// vmm_check.hip -- can the score buffer come from the virtual memory API (hipMemCreate +
// hipMemMap) without the driver's wipe wait that hipMalloc pays on HBM freed before, and
// does such memory hold what is written to it (tool)?
//   1. dirty:   hipMalloc(D GB), write it, free            (HBM now needs a wipe)
//   2. malloc:  time hipMalloc(S GB) (+ first write), check a pattern, free
//   3. dirty again
//   4. vmm:     time reserve + create + map + set access of S GB, check a pattern twice, release
//   5. vmm grow: 100 GB mapped, checked, released; then S GB at a new reservation, checked
// Prints one JSON line per step.  build: hipcc --offload-arch=gfx950 -O2 -o tools/vmm_check tools/vmm_check.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

__device__ __host__ inline uint32_t pat(size_t i, uint32_t seed) { return (uint32_t)(i * 2654435761u) ^ seed; }

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = pat(i, seed);
}

__global__ void check(const uint32_t *p, size_t n, uint32_t seed, unsigned long long *bad) {
    unsigned long long b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += (p[i] != pat(i, seed));
    for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
    if ((threadIdx.x & 63u) == 0 && b) atomicAdd(bad, b);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));                         \
            fflush(stdout);                                                                         \
            return false;                                                                           \
        }                                                                                           \
    } while (0)

static unsigned long long *d_bad = nullptr;

static bool fill_check(uint32_t *p, size_t bytes, uint32_t seed, unsigned long long out[2]) {
    const size_t n = bytes / 4;
    hipLaunchKernelGGL(fill, dim3(16384), dim3(256), 0, 0, p, n, seed);
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 2; ++r) {
        CK(hipMemset(d_bad, 0, sizeof(unsigned long long)));
        hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, 0, p, n, seed, d_bad);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&out[r], d_bad, sizeof(unsigned long long), hipMemcpyDeviceToHost));
    }
    return true;
}

static bool dirty(double gb) {
    void *p = nullptr;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)4095;
    CK(hipMalloc(&p, bytes));
    hipLaunchKernelGGL(fill, dim3(16384), dim3(256), 0, 0, (uint32_t *)p, bytes / 4, 7u);
    CK(hipDeviceSynchronize());
    CK(hipFree(p));
    printf("{\"step\": \"dirty\", \"GB\": %.0f}\n", gb);
    fflush(stdout);
    return true;
}

static bool step_malloc(double gb) {
    void *p = nullptr;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)4095;
    double t0 = now();
    CK(hipMalloc(&p, bytes));
    double t1 = now();
    unsigned long long bad[2] = {0, 0};
    if (!fill_check((uint32_t *)p, bytes, 11u, bad)) return false;
    CK(hipFree(p));
    printf("{\"step\": \"malloc\", \"GB\": %.0f, \"alloc_s\": %.3f, \"bad\": %llu, \"bad_recheck\": %llu}\n", gb, t1 - t0,
           bad[0], bad[1]);
    fflush(stdout);
    return true;
}

struct vmm_buf {
    void *ptr = nullptr;
    size_t size = 0;
    hipMemGenericAllocationHandle_t h{};
};

static bool vmm_alloc(vmm_buf &b, double gb, double *secs) {
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof(prop));
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    if (gran == 0) gran = 2u << 20;
    b.size = (((size_t)(gb * 1e9)) + gran - 1) / gran * gran;
    const double t0 = now();
    CK(hipMemAddressReserve(&b.ptr, b.size, 0, nullptr, 0));
    CK(hipMemCreate(&b.h, b.size, &prop, 0));
    CK(hipMemMap(b.ptr, b.size, 0, b.h, 0));
    hipMemAccessDesc acc;
    memset(&acc, 0, sizeof(acc));
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = 0;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(b.ptr, b.size, &acc, 1));
    *secs = now() - t0;
    return true;
}

static bool vmm_free(vmm_buf &b) {
    CK(hipMemUnmap(b.ptr, b.size));
    CK(hipMemRelease(b.h));
    CK(hipMemAddressFree(b.ptr, b.size));
    b = vmm_buf();
    return true;
}

static bool step_vmm(const char *name, double gb, uint32_t seed) {
    vmm_buf b;
    double s = 0;
    if (!vmm_alloc(b, gb, &s)) return false;
    unsigned long long bad[2] = {0, 0};
    if (!fill_check((uint32_t *)b.ptr, b.size, seed, bad)) return false;
    printf("{\"step\": \"%s\", \"GB\": %.0f, \"ptr\": \"%p\", \"alloc_s\": %.3f, \"bad\": %llu, \"bad_recheck\": %llu}\n",
           name, gb, b.ptr, s, bad[0], bad[1]);
    fflush(stdout);
    return vmm_free(b);
}

int main(int argc, char **argv) {
    const double S = argc > 1 ? atof(argv[1]) : 150.0, D = argc > 2 ? atof(argv[2]) : 200.0;
    if (hipMalloc(&d_bad, sizeof(unsigned long long)) != hipSuccess) return 1;
    bool ok = dirty(D) && step_malloc(S) && dirty(D) && step_vmm("vmm", S, 13u) && step_vmm("vmm_100", 100.0, 17u) &&
              step_vmm("vmm_after_100", S, 19u) && dirty(D) && step_vmm("vmm_dirty_again", S, 23u);
    (void)hipFree(d_bad);
    return ok ? 0 : 1;
}
