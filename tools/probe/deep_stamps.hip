// Probe build of the deep-scale conv family with per-workgroup phase stamps
// (s_memrealtime, 100 MHz): where a short launch spends its time.
//   hipcc -shared -fPIC --offload-arch=gfx950 -O3 -std=c++17 -I../../include \
//     -I../../dl-normalizing-flows_amd/csrc deep_stamps.hip -o libdeep_stamps.so
#define RNVP_DEEP_STAMPS 1
#include "../../dl-normalizing-flows_amd/csrc/conv_deep.hip"

extern "C" int rnvp_stat_shards(long long M) {
    long long s = M / 8192;
    int r = 1;
    while (r < 32 && r * 2 <= s) r *= 2;
    return r;
}

// the wide-scale fan-out groups live in conv_s1.hip (not part of this probe)
int rnvp_s1_fanout_prepare(rnvp_net_step*, int, int*, int*, int*) { return RNVP_E_UNSUPPORTED; }
int rnvp_s1_fanout_launch(const rnvp_group_kargs&, int, int, int, hipStream_t) { return RNVP_E_UNSUPPORTED; }

extern "C" int probe_deep(const rnvp_conv_args* a, void* stream, int cfg, unsigned long long* stamps) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_deep_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                               (hipStream_t)stream) != hipSuccess)
        return -3;
    return rnvp_deep_launch(a, (hipStream_t)stream, cfg);
}
