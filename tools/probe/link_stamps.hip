// Probe build of the coupling-link kernels with per-workgroup phase stamps
// (s_memrealtime, 100 MHz): where a link launch spends its time.
//   hipcc -c -fPIC --offload-arch=gfx950 -O3 -std=c++17 -I../../include \
//     -I../../dl-normalizing-flows_amd/csrc link_stamps.hip -o link_stamps.o, then linked like csrc/Makefile
//   (g++ -shared against torch/lib/libamdhip64.so: one HIP runtime per process)
#define RNVP_LINK_STAMPS 1
#include "../../dl-normalizing-flows_amd/csrc/coupling_link.hip"

extern "C" int probe_link_bwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n, const rnvp_link_args* l,
                              void* stream, unsigned long long* stamps) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_link_stamps), &stamps, sizeof(stamps), 0, hipMemcpyHostToDevice,
                               (hipStream_t)stream) != hipSuccess)
        return -3;
    return rnvp_coupling_link_bwd(a, n, l, stream);
}
