// Probe build of the wide-scale streaming 1x1 conv (conv_s1.hip) with
// per-workgroup phase stamps (s_memrealtime, 100 MHz).
//   hipcc -shared -fPIC --offload-arch=gfx950 -O3 -std=c++17 -I../../include \
//     -I../../dl-normalizing-flows_amd/csrc s1_stamps.hip -o libs1_stamps.so
#define RNVP_S1_STAMPS 1
#include "../../dl-normalizing-flows_amd/csrc/conv_s1.hip"

extern "C" int rnvp_stat_shards(long long M) {
    long long s = M / 8192;
    int r = 1;
    while (r < 32 && r * 2 <= s) r *= 2;
    return r;
}

extern "C" int probe_s1(const rnvp_conv_args* a, void* stream, unsigned long long* stamps) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_s1_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                               (hipStream_t)stream) != hipSuccess)
        return -3;
    return rnvp_conv_s1_launch(a, (hipStream_t)stream);
}
