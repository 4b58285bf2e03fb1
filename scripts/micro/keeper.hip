// keeper: a second process that keeps a light VALU load on every CU for D
// seconds (kernels of W waves per CU, each a dependent FMA loop of ~X us,
// relaunched back to back).  The experiment: does the GPU's activity-based
// clock control (amd-smi's "low utilization" record) keep the shader clock up
// for seqarc_amd -c's latency-bound pass-R tails when the GPU also sees this
// load?  (profiles/round5_r5i_*: with only the tails running the clock fell to
// 1.0-1.5 GHz and the last batch's pass R took 1.34 s instead of 0.65 s.)
//   hipcc --offload-arch=gfx950 -O3 -o keeper scripts/micro/keeper.hip
//   ./keeper SECONDS [WAVES_PER_CU] [ITERS]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

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
        hipLaunchKernelGGL(k_keep, dim3(p.multiProcessorCount * wpc), dim3(64), 0, st, out, iters);
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
    printf("keeper: %ld launches of %d waves in %.2f s (%.3f ms per launch)\n", launches, p.multiProcessorCount * wpc,
           el, 1e3 * el / launches);
    return 0;
}
