// Probe: what does a process's exit cost after it holds page-locked host
// memory or device memory?  (The command line leaves both to the exit: the
// driver's wall clock sees the teardown, round 3 g4g: 0.9-1.0 s after the
// end-to-end runs.)  Usage: exit_probe MODE GB
//   pinned: hipHostMalloc in 400 MB chunks (the reader's text windows today)
//   thp:    2 MiB-aligned malloc + MADV_HUGEPAGE + hipHostRegister, same chunks
//   dev:    hipMalloc in 4 GB pieces
// Prints the allocation time and the CLOCK_MONOTONIC stamp at _Exit;
// scripts/micro/exit_probe.py reaps it and prints the teardown.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <time.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double mono()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    const char* mode = argv[1];
    const double gb = atof(argv[2]);
    if (hipSetDevice(0) != hipSuccess) return 3;
    void* warm = nullptr;
    if (hipMalloc(&warm, 1 << 20) != hipSuccess) return 3;
    const double t0 = mono();
    const size_t chunk = !strcmp(mode, "dev") ? (4ull << 30) : (400ull << 20);
    const size_t n = (size_t)(gb * 1e9 / (double)chunk + 0.5);
    for (size_t i = 0; i < n; i++) {
        void* p = nullptr;
        if (!strcmp(mode, "pinned")) {
            if (hipHostMalloc(&p, chunk, hipHostMallocDefault) != hipSuccess) return 4;
            memset(p, 1, chunk);
        } else if (!strcmp(mode, "thp")) {
            if (posix_memalign(&p, 2u << 20, chunk) != 0) return 4;
            madvise(p, chunk, MADV_HUGEPAGE);
            memset(p, 1, chunk);
            if (hipHostRegister(p, chunk, hipHostRegisterDefault) != hipSuccess) return 4;
        } else {
            if (hipMalloc(&p, chunk) != hipSuccess) return 4;
            if (hipMemset(p, 1, chunk) != hipSuccess) return 4;
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 5;
    const double t1 = mono();
    printf("%s %.1f GB: allocated in %.3f s\nexit %.6f\n", mode, (double)(n * chunk) / 1e9, t1 - t0, mono());
    fflush(stdout);
    std::_Exit(0);
}
