// Probe: cost of dependent global-memory round trips inside graph-replayed
// kernels, each kernel reading what the previous one wrote (the engine's
// producer -> consumer pattern).  k_chain<K>: every thread does K dependent
// loads from `in` (index from the previous value) and one store to `out`.
//   hipcc -shared -fPIC --offload-arch=gfx950 -O3 -std=c++17 latency_chain.hip -o liblatency_chain.so
#include <hip/hip_runtime.h>

template <int K>
__global__ __launch_bounds__(256) void k_chain(const int* __restrict__ in, int* __restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    int v = i;
#pragma unroll
    for (int k = 0; k < K; ++k) v = in[(unsigned)(v * 2654435761u + i) % (unsigned)n] + i;
    out[i % n] = v & 0xffff;
}

template <int K>
static double run(int* a, int* b, int n, int grid, int reps) {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int r = 0; r < reps; ++r) {
        if (r & 1) k_chain<K><<<grid, 256, 0, s>>>(b, a, n);
        else k_chain<K><<<grid, 256, 0, s>>>(a, b, n);
    }
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    for (int it = 0; it < 5; ++it) hipGraphLaunch(ge, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    hipStreamDestroy(s);
    return 1000.0 * ms / (5.0 * reps);
}

extern "C" int probe_chain(int grid, int n, double* us) {
    int *a, *b;
    if (hipMalloc(&a, sizeof(int) * (size_t)n) != hipSuccess) return -1;
    if (hipMalloc(&b, sizeof(int) * (size_t)n) != hipSuccess) return -1;
    hipMemset(a, 0, sizeof(int) * (size_t)n);
    hipMemset(b, 0, sizeof(int) * (size_t)n);
    us[0] = run<0>(a, b, n, grid, 200);
    us[1] = run<1>(a, b, n, grid, 200);
    us[2] = run<2>(a, b, n, grid, 200);
    us[3] = run<4>(a, b, n, grid, 200);
    us[4] = run<8>(a, b, n, grid, 200);
    hipFree(a);
    hipFree(b);
    return 0;
}
