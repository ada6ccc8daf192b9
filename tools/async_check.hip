// async_check.hip -- does memory from the stream-ordered allocator hold what is written to
// it at very large sizes (tool)?  For each size of a growing sequence:
// allocate, write p[i] = hash(i) ^ seed_a (seed_a distinct per allocation a) with one
// kernel, count mismatches with another (twice, to see whether they move), then free.
// Mismatches are classified: the word of the PREVIOUS allocation's pattern at the same
// index (the write went to, or the read came from, the old backing of a reused address),
// zero, or other.  Pool attributes (reserved / used bytes) are printed after each step.
//
// modes:  pool    the device's default pool (hipMallocAsync / hipFreeAsync)
//         trim    the same, with hipMemPoolTrimTo(pool, 0) after every free
//         own     an explicitly created pool (hipMemPoolCreate)
//         malloc  hipMalloc / hipFree (control)
//         sleep   the default pool, waiting 12 s after every free (time for the driver to
//                 finish clearing the freed memory) before the next allocation
// argv[2] = largest size in GB (default 200)
// An allocation that fails ends the sequence cleanly (everything outstanding is freed
// before the process exits: the round-2 version called exit(1) with a pool block live,
// and the runtime's teardown then aborted with "double free").
// build: hipcc --offload-arch=gfx950 -O2 -o tools/async_check tools/async_check.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

__device__ __host__ inline uint32_t pat(size_t i, uint32_t seed) { return (uint32_t)(i * 2654435761u) ^ seed; }

__global__ void fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = pat(i, seed);
}

// out[0] bad, [1] bad == previous allocation's word, [2] bad == 0, [3] first bad index, [4] last bad index
__global__ void check(const uint32_t *p, size_t n, uint32_t seed, uint32_t prev, unsigned long long *out) {
    unsigned long long b = 0, bp = 0, bz = 0, f = ~0ull, l = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = p[i];
        if (v != pat(i, seed)) {
            ++b;
            bp += (v == pat(i, prev));
            bz += (v == 0u);
            if (i < f) f = i;
            if (i > l) l = i;
        }
    }
    if (b) {
        atomicAdd(out + 0, b);
        atomicAdd(out + 1, bp);
        atomicAdd(out + 2, bz);
        atomicMin(out + 3, f);
        atomicMax(out + 4, l);
    }
}

static bool ok(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        printf("{\"error\": \"%s: %s\"}\n", what, hipGetErrorString(e));
        fflush(stdout);
        (void)hipGetLastError();
        return false;
    }
    return true;
}

static void pool_attrs(hipMemPool_t pool, const char *tag) {
    if (!pool) return;
    uint64_t res = 0, used = 0, hi = 0;
    (void)hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemCurrent, &res);
    (void)hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, &used);
    (void)hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemHigh, &hi);
    printf("{\"pool\": \"%s\", \"reserved_GB\": %.3f, \"used_GB\": %.3f, \"reserved_high_GB\": %.3f}\n", tag,
           res / 1e9, used / 1e9, hi / 1e9);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "pool";
    const bool use_pool = strcmp(mode, "malloc") != 0;
    const double max_gb = argc > 2 ? atof(argv[2]) : 200.0;
    const double gbs[] = {8, 100, 140, 150, 200};
    hipStream_t s = nullptr;
    if (!ok(hipStreamCreate(&s), "hipStreamCreate")) return 1;
    hipMemPool_t pool = nullptr;
    if (strcmp(mode, "own") == 0) {
        hipMemPoolProps props;
        memset(&props, 0, sizeof(props));
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = 0;
        if (!ok(hipMemPoolCreate(&pool, &props), "hipMemPoolCreate")) return 1;
    } else if (use_pool) {
        if (!ok(hipDeviceGetDefaultMemPool(&pool, 0), "hipDeviceGetDefaultMemPool")) return 1;
    }
    unsigned long long *d = nullptr;
    if (!ok(hipMalloc(&d, 5 * sizeof(unsigned long long)), "hipMalloc counters")) return 1;
    uint32_t prev = 0;
    int a = 0;
    for (double gb : gbs) {
        if (gb > max_gb) break;
        ++a;
        const uint32_t seed = 0x9e3779b9u * (uint32_t)a;
        const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)4095, n = bytes / 4;
        uint32_t *p = nullptr;
        hipError_t e;
        if (!use_pool)
            e = hipMalloc(reinterpret_cast<void **>(&p), bytes);
        else if (pool && strcmp(mode, "own") == 0)
            e = hipMallocFromPoolAsync(reinterpret_cast<void **>(&p), bytes, pool, s);
        else
            e = hipMallocAsync(reinterpret_cast<void **>(&p), bytes, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (!ok(e, "allocate")) {
            printf("{\"mode\": \"%s\", \"GB\": %.0f, \"allocated\": false}\n", mode, gb);
            break;
        }
        pool_attrs(pool, "after alloc");
        unsigned long long h[2][5];
        hipLaunchKernelGGL(fill, dim3(16384), dim3(256), 0, s, p, n, seed);
        bool good = ok(hipStreamSynchronize(s), "fill");
        for (int rep = 0; rep < 2 && good; ++rep) {
            unsigned long long init[5] = {0, 0, 0, ~0ull, 0};
            good = ok(hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice), "reset");
            if (!good) break;
            hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, s, p, n, seed, prev, d);
            good = ok(hipStreamSynchronize(s), "check") && ok(hipMemcpy(h[rep], d, sizeof(h[rep]), hipMemcpyDeviceToHost), "read");
        }
        if (good)
            printf("{\"mode\": \"%s\", \"GB\": %.0f, \"ptr\": \"%p\", \"bad\": %llu, \"bad_prev_pattern\": %llu, "
                   "\"bad_zero\": %llu, \"first_bad_byte\": %llu, \"last_bad_byte\": %llu, \"bad_recheck\": %llu}\n",
                   mode, gb, (void *)p, h[0][0], h[0][1], h[0][2], h[0][0] ? h[0][3] * 4 : 0ull,
                   h[0][0] ? h[0][4] * 4 : 0ull, h[1][0]);
        fflush(stdout);
        if (!use_pool)
            e = hipFree(p);
        else
            e = hipFreeAsync(p, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (!ok(e, "free")) break;
        if (strcmp(mode, "trim") == 0 && !ok(hipMemPoolTrimTo(pool, 0), "trim")) break;
        pool_attrs(pool, "after free");
        if (strcmp(mode, "sleep") == 0) sleep(12);
        prev = seed;
        if (!good) break;
    }
    (void)hipFree(d);
    if (pool && strcmp(mode, "own") == 0) (void)hipMemPoolDestroy(pool);
    (void)hipStreamDestroy(s);
    return 0;
}
