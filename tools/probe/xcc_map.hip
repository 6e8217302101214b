// Probe: which XCD (XCC) runs each workgroup of a plain launch -- the tile
// orders of the conv kernels assume workgroup b lands on XCD b % 8.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_xcc(unsigned* out) {
    if (threadIdx.x == 0) {
        unsigned v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
        out[blockIdx.x] = v;
    }
}

int main() {
    const int n = 1024;
    unsigned* d;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
    for (int threads : {64, 256}) {
        k_xcc<<<n, threads>>>(d);
        unsigned h[n];
        if (hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int match = 0;
        for (int i = 0; i < n; ++i) match += (h[i] & 0xf) == (unsigned)(i % 8);
        printf("block size %d: %d of %d blocks on XCC (b %% 8); first 24:", threads, match, n);
        for (int i = 0; i < 24; ++i) printf(" %u", h[i] & 0xf);
        printf("\n");
    }
    return 0;
}
