// Probe: per-dispatch duration floor of trivial kernels (rocprofv3 --kernel-trace).
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { char pad[320]; };

__global__ void k_empty() {}
__global__ void k_empty_big(Big b) { if (b.pad[0] == 123 && threadIdx.x == 999) asm volatile("s_nop 0"); }
__global__ void k_touch(float* p) { p[blockIdx.x * blockDim.x + threadIdx.x] += 1.f; }
__global__ void k_lds(float* p) {
    extern __shared__ float s[];
    s[threadIdx.x] = p[blockIdx.x * blockDim.x + threadIdx.x];
    __syncthreads();
    p[blockIdx.x * blockDim.x + threadIdx.x] = s[255 - threadIdx.x];
}

int main() {
    float* p;
    hipMalloc(&p, 1 << 24);
    hipMemset(p, 0, 1 << 24);
    hipStream_t s;
    hipStreamCreate(&s);
    Big b{};
    for (int rep = 0; rep < 2; ++rep) {
        for (int i = 0; i < 50; ++i) k_empty<<<1, 64, 0, s>>>();
        for (int i = 0; i < 50; ++i) k_empty<<<1024, 256, 0, s>>>();
        for (int i = 0; i < 50; ++i) k_empty_big<<<1024, 256, 0, s>>>(b);
        for (int i = 0; i < 50; ++i) k_touch<<<1024, 256, 0, s>>>(p);
        for (int i = 0; i < 50; ++i) k_lds<<<1024, 256, 48 * 1024, s>>>(p);
    }
    // per-kernel-type graphs: steady-state cost per dispatch inside a graph
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int kind = 0; kind < 5; ++kind) {
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < 200; ++i) {
            if (kind == 0) k_empty<<<1, 64, 0, s>>>();
            if (kind == 1) k_empty<<<1024, 256, 0, s>>>();
            if (kind == 2) k_empty_big<<<1024, 256, 0, s>>>(b);
            if (kind == 3) k_touch<<<1024, 256, 0, s>>>(p);
            if (kind == 4) k_lds<<<1024, 256, 48 * 1024, s>>>(p);
        }
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0, s);
            hipGraphLaunch(ge, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2) printf("graph kind %d: 200 kernels %.1f us, %.2f us/kernel\n", kind, ms * 1e3, ms * 1e3 / 200);
        }
    }
    hipDeviceSynchronize();
    printf("done\n");
    return 0;
}
