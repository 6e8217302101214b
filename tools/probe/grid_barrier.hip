// Probe: cost of an in-kernel grid barrier (persistent launch) against a
// kernel boundary in a captured graph.  Each phase every workgroup writes one
// value and, after the barrier, reads another workgroup's value of that phase
// (cross-XCD visibility check).  The barrier is the generation/count form the
// persistent net kernels use, with a bounded spin (no hang on a non-resident
// grid: it sets the abort word and every later barrier falls through).
#include <hip/hip_runtime.h>
#include <cstdio>

struct Bar { unsigned count, gen, abort, pad; };

__device__ __forceinline__ void grid_sync(Bar* bar, unsigned nb) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(&bar->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned old = __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == nb - 1) {
            __hip_atomic_store(&bar->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&bar->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(&bar->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (__hip_atomic_load(&bar->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                if (wall_clock64() - t0 > 20000000ull) {   // 200 ms at 100 MHz
                    __hip_atomic_store(&bar->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// B: count and generation on separate 128-byte lines (pollers do not
// contend with the arrivals' atomics)
struct BarB { unsigned count, p0[31]; unsigned gen, p1[31]; unsigned abort, p2[31]; };
__device__ __forceinline__ void grid_sync_b(BarB* bar, unsigned nb) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(&bar->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned old = __hip_atomic_fetch_add(&bar->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == nb - 1) {
            __hip_atomic_store(&bar->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&bar->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(&bar->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (wall_clock64() - t0 > 20000000ull) { __hip_atomic_store(&bar->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// C: hierarchical -- 8 group counters (workgroup % 8, one line each), the
// last of a group arrives at the top counter, the last group bumps 8 group
// generation words (one line each) that the group's workgroups poll
struct BarC { unsigned top, p0[31]; unsigned abort, p1[31]; unsigned grp[8][32]; unsigned gen[8][32]; };
__device__ __forceinline__ void grid_sync_c(BarC* bar, unsigned nb) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned x = blockIdx.x & 7, per = nb >> 3;
        unsigned* gw = &bar->gen[x][0];
        const unsigned g = __hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned old = __hip_atomic_fetch_add(&bar->grp[x][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool done = false;
        if (old == per - 1) {
            __hip_atomic_store(&bar->grp[x][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned o2 = __hip_atomic_fetch_add(&bar->top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (o2 == 7) {
                __hip_atomic_store(&bar->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (int k = 0; k < 8; ++k) __hip_atomic_fetch_add(&bar->gen[k][0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                done = true;
            }
        }
        if (!done) {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (wall_clock64() - t0 > 20000000ull) { __hip_atomic_store(&bar->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

template <int V>
__global__ void k_phases_v(void* bar, float* data, int nphase, int* bad) {
    const unsigned nb = gridDim.x, b = blockIdx.x;
    for (int ph = 0; ph < nphase; ++ph) {
        if (threadIdx.x == 0) data[(size_t)(ph & 1) * nb + b] = (float)(ph * 7 + b);
        if (V == 1) grid_sync_b((BarB*)bar, nb);
        else grid_sync_c((BarC*)bar, nb);
        if (threadIdx.x == 0) {
            const unsigned o = (b + 37) % nb;
            if (data[(size_t)(ph & 1) * nb + o] != (float)(ph * 7 + o)) atomicAdd(bad, 1);
        }
    }
}

__global__ void k_phases(Bar* bar, float* data, int nphase, int* bad) {
    const unsigned nb = gridDim.x, b = blockIdx.x;
    for (int ph = 0; ph < nphase; ++ph) {
        if (threadIdx.x == 0) data[(size_t)(ph & 1) * nb + b] = (float)(ph * 7 + b);
        grid_sync(bar, nb);
        if (threadIdx.x == 0) {
            const unsigned o = (b + 37) % nb;
            if (data[(size_t)(ph & 1) * nb + o] != (float)(ph * 7 + o)) atomicAdd(bad, 1);
        }
    }
}

__global__ void k_one(float* data, int ph) {
    if (threadIdx.x == 0) data[blockIdx.x] = (float)(ph + blockIdx.x);
}

int main() {
    Bar* bar;
    float* data;
    int* bad;
    hipMalloc(&bar, sizeof(Bar));
    hipMemset(bar, 0, sizeof(Bar));
    hipMalloc(&data, 1 << 20);
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", cus);
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int nph = 2000;
    for (int nb : {64, 128, 256, 512, 1024}) {
        for (int threads : {256, 512}) {
            k_phases<<<nb, threads, 0, s>>>(bar, data, 10, bad);
            hipEventRecord(e0, s);
            k_phases<<<nb, threads, 0, s>>>(bar, data, nph, bad);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            Bar hb;
            int hbad;
            hipMemcpy(&hb, bar, sizeof(Bar), hipMemcpyDeviceToHost);
            hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost);
            printf("grid %4d x %3d: %d barriers %.1f us, %.3f us/barrier  abort=%u bad=%d count=%u\n", nb, threads,
                   nph, ms * 1e3, ms * 1e3 / nph, hb.abort, hbad, hb.count);
        }
    }
    void* bar2;
    hipMalloc(&bar2, sizeof(BarC) + sizeof(BarB));
    for (int v = 1; v <= 2; ++v) {
        for (int nb : {256, 512}) {
            hipMemset(bar2, 0, sizeof(BarC) + sizeof(BarB));
            hipMemset(bad, 0, 4);
            auto k = v == 1 ? k_phases_v<1> : k_phases_v<2>;
            k<<<nb, 256, 0, s>>>(bar2, data, 10, bad);
            hipEventRecord(e0, s);
            k<<<nb, 256, 0, s>>>(bar2, data, nph, bad);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            int hbad;
            unsigned ab[2];
            hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost);
            hipMemcpy(ab, v == 1 ? (char*)bar2 + 256 : (char*)bar2 + 128, 4, hipMemcpyDeviceToHost);
            printf("variant %c grid %4d: %.3f us/barrier  abort=%u bad=%d\n", v == 1 ? 'B' : 'C', nb, ms * 1e3 / nph,
                   ab[0], hbad);
        }
    }
    // kernel boundaries in a graph with the same per-phase work
    for (int nb : {256, 1024}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < 200; ++i) k_one<<<nb, 256, 0, s>>>(data, i);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0, s);
            hipGraphLaunch(ge, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2) printf("graph of 200 x k_one<<<%d>>>: %.3f us/kernel\n", nb, ms * 1e3 / 200);
        }
    }
    hipDeviceSynchronize();
    printf("done\n");
    return 0;
}
