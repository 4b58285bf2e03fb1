// Microbenchmark of k_replay_aux_long on one synthetic hot quality-model run
// (symbols 37 / 25 / 11 with p = 0.90 / 0.07 / 0.03, like the bench's hottest
// context), plus a time split of one run's steps when built with -DSA_PROF.
// Mode 1 (third argument): 24 symbols with a geometric distribution (symbols
// beyond position 8, bubble swaps).  The records are checked against the
// serial host replay (replay_simple_run).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include "../../fastqueeze_amd/csrc/sa_kernels.hip"

using namespace sa;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main(int argc, char** argv)
{
    const uint32_t L = argc > 1 ? atoi(argv[1]) : 2000000;
    const int nruns = argc > 2 ? atoi(argv[2]) : 1;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const uint32_t model = M_QUAL + 12345;
    std::vector<uint32_t> keys((size_t)L * nruns + 1024, SORT_PAD), vals((size_t)L * nruns + 1024, 0);
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> U(0, 1);
    for (size_t i = 0; i < (size_t)L * nruns; i++) {
        double u = U(rng);
        uint32_t sym = u < 0.9 ? 37 : (u < 0.97 ? 25 : 11);
        if (mode == 1) {
            sym = 40;
            while (U(rng) < 0.55 && sym > 17) sym--;   // 40, 39, ... with ratio 0.55
        }
        keys[i] = (model << AUX_SYM_BITS) | sym;
        vals[i] = (uint32_t)(i % L);
    }
    std::vector<LongRun> runs(nruns);
    for (int r = 0; r < nruns; r++) runs[r] = LongRun{(uint64_t)r * L, (uint64_t)(r + 1) * L, (uint64_t)r * L, model, 0};
    uint32_t *dk, *dv, *dn, *derr; LongRun* dl; PRec* dp; uint16_t* dc;
    CK(hipMalloc(&dk, keys.size() * 4)); CK(hipMalloc(&dv, vals.size() * 4));
    CK(hipMalloc(&dl, runs.size() * sizeof(LongRun))); CK(hipMalloc(&dn, 16)); CK(hipMalloc(&derr, 4));
    CK(hipMalloc(&dp, (size_t)L * nruns * sizeof(PRec))); CK(hipMalloc(&dc, (size_t)L * nruns * 2));
    CK(hipMemcpy(dk, keys.data(), keys.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, vals.data(), vals.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(derr, 0, 4));
    CK(hipMemcpy(dl, runs.data(), runs.size() * sizeof(LongRun), hipMemcpyHostToDevice));
    const uint32_t ctr[4] = {0u, (uint32_t)nruns, 0u, 0u};   // short, huge, long, queue
    RunLists rl{nullptr, dn, dl, dn + 1, dn + 2, (uint64_t)nruns, dn + 3, dl};
    CK(hipMemset(derr, 0, 4));
    SymSink sink{dp, dc};
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int it = 0; it < 3; it++) {
        CK(hipMemcpy(dn, ctr, 16, hipMemcpyHostToDevice));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_replay_aux_long, dim3(nruns), dim3(128), 0, 0, rl, dk, dv, sink, derr);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("run of %u symbols x %d: %.2f ms = %.1f ns/symbol, %.2f us/step\n", L, nruns, ms, ms * 1e6 / L, ms * 1e3 / (L / 64.0));
    }
    uint32_t e; CK(hipMemcpy(&e, derr, 4, hipMemcpyDeviceToHost));
    printf("err bits %u\n", e);
    {
        std::vector<PRec> gp((size_t)L * nruns), hp((size_t)L * nruns);
        std::vector<uint16_t> gc((size_t)L * nruns), hc((size_t)L * nruns);
        CK(hipMemcpy(gp.data(), dp, gp.size() * sizeof(PRec), hipMemcpyDeviceToHost));
        CK(hipMemcpy(gc.data(), dc, gc.size() * 2, hipMemcpyDeviceToHost));
        std::vector<uint32_t> F(256);
        size_t bad = 0, first = ~(size_t)0;
        for (int r = 0; r < nruns; r++) {
            SymSink hs{hp.data() + (size_t)r * L, hc.data() + (size_t)r * L};
            replay_simple_run(keys.data(), vals.data(), (size_t)r * L, (size_t)(r + 1) * L, model, hs, F.data());
        }
        for (size_t i = 0; i < gp.size(); i++)
            if (gp[i].tf != hp[i].tf || gc[i] != hc[i]) { bad++; if (first == ~(size_t)0) first = i; }
        printf("records vs host replay: %zu of %zu differ (first %zd)\n", bad, gp.size(), (ssize_t)first);
    }
#ifdef SA_PROF
    unsigned long long pr[8];
    CK(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_prof), sizeof pr));
    const char* nm[5] = {"ring wait", "distinct pass", "events", "records", "tail"};
    for (int k = 0; k < 5; k++) printf("  %-14s %8.1f cycles/step (s_memtime)\n", nm[k], pr[k] / (L / 64.0));
#endif
    return 0;
}
