// async_oom.hip -- the smallest program that shows the abort seen at the end of
// tools/async_check: a stream-ordered allocation that fails with "out of
// memory", then a clean exit with nothing outstanding.  One step per mode, in a fresh
// process each (tools/async_oom.sh):
//   oom       hipMallocAsync(GB) on a fresh default pool, nothing allocated before
//   after     hipMallocAsync(8 GB) + hipFreeAsync first, then hipMallocAsync(GB)
//   grown     hipMallocAsync(100 GB) + hipFreeAsync first (the pool has grown to 100 GB)
//   regrown   100 GB, then 140 GB (re-served from the freed 100 GB block, the allocation
//             async_check found corrupt), each freed, then hipMallocAsync(GB)
//   malloc    hipMalloc(GB) (control: the non-pool allocator's out-of-memory path)
// Prints one JSON line; the exit status shows whether the runtime's teardown aborts.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/async_oom tools/async_oom.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "oom";
    const double gb = argc > 2 ? atof(argv[2]) : 400.0;
    hipStream_t s = nullptr;
    if (hipStreamCreate(&s) != hipSuccess) return 2;
    const double before[3][2] = {{8, 0}, {100, 0}, {100, 140}};
    const int pre = strcmp(mode, "after") == 0 ? 0 : strcmp(mode, "grown") == 0 ? 1 : strcmp(mode, "regrown") == 0 ? 2 : -1;
    for (int i = 0; pre >= 0 && i < 2 && before[pre][i] > 0; ++i) {
        void *q = nullptr;
        hipError_t e = hipMallocAsync(&q, (size_t)(before[pre][i] * 1e9), s);
        if (e == hipSuccess) e = hipFreeAsync(q, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        printf("{\"mode\": \"%s\", \"first_GB\": %.0f, \"result\": \"%s\"}\n", mode, before[pre][i],
               hipGetErrorString(e));
    }
    void *p = nullptr;
    const size_t bytes = (size_t)(gb * 1e9) & ~(size_t)4095;
    hipError_t e = strcmp(mode, "malloc") == 0 ? hipMalloc(&p, bytes) : hipMallocAsync(&p, bytes, s);
    if (e == hipSuccess && strcmp(mode, "malloc") != 0) e = hipStreamSynchronize(s);
    printf("{\"mode\": \"%s\", \"GB\": %.0f, \"result\": \"%s\"}\n", mode, gb, hipGetErrorString(e));
    fflush(stdout);
    (void)hipGetLastError();
    if (e == hipSuccess) {  // (only if the device really has that much)
        if (strcmp(mode, "malloc") == 0)
            (void)hipFree(p);
        else {
            (void)hipFreeAsync(p, s);
            (void)hipStreamSynchronize(s);
        }
    }
    (void)hipStreamDestroy(s);
    printf("{\"mode\": \"%s\", \"exit\": \"returning from main\"}\n", mode);
    fflush(stdout);
    return 0;
}
