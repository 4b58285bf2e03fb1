// exit_probe: how long the kernel takes to tear down a process that holds
// device memory (VRAM buffers) and page-locked host memory -- the time between
// seqarc_amd's _Exit and its parent's wait returning (bench.py's
// "exit_to_reaped_s").  The parent never touches the GPU; each case runs in a
// forked child that initialises HIP, allocates, touches, and exits.
//   hipcc -O2 -o exit_probe scripts/exit_probe.cpp
//   ./exit_probe [vram_gb ...]   (default 0 50 100 200)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <vector>

static double mono()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// child: vram_gb in chunk_gb buffers (touched by a memset), pin_gb of
// page-locked host memory; writes its exit stamp to fd, then _Exit
static void child(double vram_gb, double chunk_gb, double pin_gb, int fd, bool release)
{
    if (hipInit(0) != hipSuccess) _Exit(3);
    std::vector<void*> bufs;
    const size_t chunk = (size_t)(chunk_gb * (1ull << 30));
    for (double got = 0; got + 1e-9 < vram_gb; got += chunk_gb) {
        void* p = nullptr;
        if (hipMalloc(&p, chunk) != hipSuccess) _Exit(4);
        if (hipMemsetAsync(p, 0, chunk, 0) != hipSuccess) _Exit(5);
        bufs.push_back(p);
    }
    void* h = nullptr;
    const size_t pin = (size_t)(pin_gb * (1ull << 30));
    if (pin) {
        if (posix_memalign(&h, 2u << 20, pin) != 0) _Exit(6);
        madvise(h, pin, MADV_HUGEPAGE);
        if (hipHostRegister(h, pin, hipHostRegisterPortable) != hipSuccess) _Exit(7);
    }
    hipDeviceSynchronize();
    double t_rel = 0;
    if (release) {   // the buffers freed by the process itself before the exit
        const double t0 = mono();
        for (void* p : bufs) hipFree(p);
        if (pin) hipHostUnregister(h);
        t_rel = mono() - t0;
    }
    double st[2] = {mono(), t_rel};
    if (write(fd, st, sizeof st) != (ssize_t)sizeof st) _Exit(8);
    _Exit(0);
}

int main(int argc, char** argv)
{
    std::vector<double> sizes;
    for (int i = 1; i < argc; i++) sizes.push_back(atof(argv[i]));
    if (sizes.empty()) sizes = {0, 50, 100, 200};
    struct Case {
        double chunk, pin;
        bool release;
    };
    const Case cases[] = {{4, 0, false}, {32, 0, false}, {4, 10, false}, {4, 0, true}};
    printf("%8s %8s %6s %8s %12s %12s\n", "vram_GB", "chunk_GB", "pin_GB", "release", "free_s", "exit->reap_s");
    for (double v : sizes)
        for (const Case& c : cases) {
            if (v == 0 && c.chunk != 4) continue;
            int p[2];
            if (pipe(p) != 0) return 1;
            const pid_t pid = fork();
            if (pid == 0) {
                close(p[0]);
                child(v, c.chunk, c.pin, p[1], c.release);
            }
            close(p[1]);
            double st[2] = {0, 0};
            const bool got = read(p[0], st, sizeof st) == (ssize_t)sizeof st;
            int status = 0;
            waitpid(pid, &status, 0);
            const double reaped = mono();
            close(p[0]);
            if (!got || !WIFEXITED(status) || WEXITSTATUS(status) != 0) {
                printf("%8.0f %8.0f %6.0f %8d  child failed (status %d)\n", v, c.chunk, c.pin, (int)c.release, status);
                continue;
            }
            printf("%8.0f %8.0f %6.0f %8d %12.3f %12.3f\n", v, c.chunk, c.pin, (int)c.release, st[1], reaped - st[0]);
            fflush(stdout);
        }
    return 0;
}
