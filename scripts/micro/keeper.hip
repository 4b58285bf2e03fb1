// keeper: a second process that keeps a light VALU load on every CU for D
// seconds (kernels of W waves per CU, each a dependent FMA loop of ~X us,
// relaunched back to back).  The experiment: does the GPU's activity-based
// clock control (amd-smi's "low utilization" record) keep the shader clock up
// for seqarc_amd -c's latency-bound pass-R tails when the GPU also sees this
// load?  (profiles/round5_r5i_*: with only the tails running the clock fell to
// 1.0-1.5 GHz and the last batch's pass R took 1.34 s instead of 0.65 s.)
//   hipcc --offload-arch=gfx950 -O3 -o keeper scripts/micro/keeper.hip
//   ./keeper SECONDS [WAVES_PER_CU] [ITERS] [MODE]
// MODE 0: a dependent FMA loop (r5k: the clock held at 2.37 GHz, but pass R's
// chains were no faster -- the keeper's VALU stream delays the chains' moves on
// the SIMDs they share); MODE 1: the waves resident but asleep (s_sleep, no
// issue); MODE 2: FMA bursts of 64 between sleeps (a ~1/8 duty).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

__global__ void k_sleep(float* out, int iters)
{
    for (int i = 0; i < iters; i++) __builtin_amdgcn_s_sleep(127);   // (~8k cycles each)
    if (iters < 0) out[threadIdx.x] = 0.0f;
}

__global__ void k_burst(float* out, int iters)
{
    float a = threadIdx.x * 1e-3f, b = 1.000001f, c = 1e-7f;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 64; k++) a = __builtin_fmaf(a, b, c);
        __builtin_amdgcn_s_sleep(8);
    }
    if (a == 12345.0f) out[threadIdx.x] = a;
}

__global__ void k_keep(float* out, int iters)
{
    float a = threadIdx.x * 1e-3f, b = 1.000001f, c = 1e-7f;
    for (int i = 0; i < iters; i++) {
        a = __builtin_fmaf(a, b, c);
        a = __builtin_fmaf(a, b, c);
        a = __builtin_fmaf(a, b, c);
        a = __builtin_fmaf(a, b, c);
    }
    if (a == 12345.0f) out[threadIdx.x] = a;   // (never: keeps the loop)
}

int main(int argc, char** argv)
{
    const double secs = argc > 1 ? atof(argv[1]) : 10.0;
    const int wpc = argc > 2 ? atoi(argv[2]) : 1;
    const int iters = argc > 3 ? atoi(argv[3]) : 2000;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    void (*k)(float*, int) = mode == 1 ? k_sleep : mode == 2 ? k_burst : k_keep;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    float* out;
    hipMalloc(&out, 4096);
    hipStream_t st;
    hipStreamCreate(&st);
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    long launches = 0;
    for (;;) {
        hipLaunchKernelGGL(k, dim3(p.multiProcessorCount * wpc), dim3(64), 0, st, out, iters);
        launches++;
        if (launches % 16 == 0) {
            hipStreamSynchronize(st);
            clock_gettime(CLOCK_MONOTONIC, &t1);
            if ((t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec) > secs) break;
        }
    }
    hipStreamSynchronize(st);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double el = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    printf("keeper (mode %d): %ld launches of %d waves in %.2f s (%.3f ms per launch)\n", mode, launches, p.multiProcessorCount * wpc,
           el, 1e3 * el / launches);
    return 0;
}
