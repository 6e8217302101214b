// Probe build of the persistent band kernel with per-workgroup phase stamps
// (s_memrealtime, 100 MHz): where a wide-scale 3x3 launch spends its time.
//   hipcc -shared -fPIC --offload-arch=gfx950 -O3 -std=c++17 -I../../include \
//     -I../../dl-normalizing-flows_amd/csrc band_stamps.hip -o libband_stamps.so
#define RNVP_BAND_STAMPS 1
#include "../../dl-normalizing-flows_amd/csrc/conv_band.hip"

extern "C" int rnvp_stat_shards(long long M) {
    long long s = M / 8192;
    int r = 1;
    while (r < 32 && r * 2 <= s) r *= 2;
    return r;
}

extern "C" int probe_band(const rnvp_conv_args* a, void* stream, unsigned long long* stamps) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_band_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                               (hipStream_t)stream) != hipSuccess)
        return -3;
    return rnvp_conv_band2_launch(a, (hipStream_t)stream);
}
