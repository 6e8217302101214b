"""One-off source edit: BN statistics partials in fp64, DPP row reductions."""
import re
import sys

ROOT = "/root/repo/dl-normalizing-flows_amd/csrc/"


def sub(s, old, new, count=1):
    n = s.count(old)
    if n != count:
        sys.exit("expected %d x %r, found %d" % (count, old[:60], n))
    return s.replace(old, new)


p = ROOT + "common.h"
s = open(p).read()
if "row_sum16" not in s:
    s = sub(s, "// block-wide sum (blockDim.x multiple of 64, <= 1024); every thread gets the result", r'''// Sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15 = one MFMA column
// group); every lane of the row gets the result.  row_ror butterfly on the
// VALU (no LDS round trip: __shfl_xor lowers to ds_bpermute).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_f<0x128>(v); v += dpp_f<0x124>(v); v += dpp_f<0x122>(v); v += dpp_f<0x121>(v);
    return v;
}
__device__ __forceinline__ double row_sum16(double v) {
    v += dpp_d<0x128>(v); v += dpp_d<0x124>(v); v += dpp_d<0x122>(v); v += dpp_d<0x121>(v);
    return v;
}

// block-wide sum (blockDim.x multiple of 64, <= 1024); every thread gets the result''')
open(p, "w").write(s)

p = ROOT + "conv.hip"
s = open(p).read()
# epilogue statistics: per-lane partials in fp64 (sum of squares of values
# whose mean can be >> their spread: fp32 partials lose the variance)
s = sub(s, "bool epi_bn, const float* et, int pitch, float* s1, float* s2, int nvalid) {",
        "bool epi_bn, const float* et, int pitch, double* s1, double* s2, int nvalid) {")
s = sub(s, "            s2[r] += v[r] * v[r];", "            s2[r] += (double)v[r] * v[r];")
s = sub(s, "float s1[TN][4], s2[TN][4];", "double s1[TN][4], s2[TN][4];")
s = sub(s, "float s1[NT][4], s2[NT][4];", "double s1[NT][4], s2[NT][4];")
s = sub(s, "float s1[FR][4], s2[FR][4];", "double s1[FR][4], s2[FR][4];", 2)
s = sub(s, "float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};",
        "double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};")
pat = re.compile(r"float u1 = (s1\[\w+\]\[r\]), u2 = (s2\[\w+\]\[r\]);\n#pragma unroll\n\s*for \(int o = 1; o < 16; o <<= 1\) \{\n"
                 r"\s*u1 \+= __shfl_xor\(u1, o, 64\);\n\s*u2 \+= __shfl_xor\(u2, o, 64\);\n\s*\}")
s, n = pat.subn(r"const double u1 = row_sum16(\1), u2 = row_sum16(\2);", s)
if n != 4:
    sys.exit("row_sum16 sites: %d" % n)
s = sub(s, "float t1 = 0.f, t2 = 0.f;", "double t1 = 0.0, t2 = 0.0;", 5)
s = sub(s, "    __shared__ float red[WM * BN * 2];", "    __shared__ double red[WM * BN * 2];")
s = sub(s, "    __shared__ float red[16][64][2];", "    __shared__ double red[16][64][2];")
s = sub(s, "    float* red = btab + NC;                // [4 waves][NC][2]",
        "    double* red = (double*)(btab + NC);    // [4 waves][NC][2]")
s = sub(s, "+ 4 * (size_t)nc + 32 * (size_t)nc +", "+ 4 * (size_t)nc + 64 * (size_t)nc +")
s = sub(s, "    float sred[4][BN][2];                     // per-wave BN-stat partials",
        "    double sred[4][BN][2];                    // per-wave BN-stat partials")
s = sub(s, "    float* sred = btab + BN;                   // [TM][BN][2]",
        "    double* sred = (double*)(btab + BN);       // [TM][BN][2]")
s = sub(s, "    const size_t head = 4 * (4 * BN + BN + 2 * TM * BN);",
        "    const size_t head = 4 * (4 * BN + BN) + 8 * (2 * TM * BN);")
open(p, "w").write(s)

p = ROOT + "coupling.hip"
s = open(p).read()
s = sub(s, r'''__device__ __forceinline__ float seg_sum(float v, int seg) {
    for (int o = 1; o < seg; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}''', r'''__device__ __forceinline__ float seg_sum(float v, int seg) {
    for (int o = 1; o < seg; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double seg_sum(double v, int seg) {
    for (int o = 1; o < seg; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}''')
s = sub(s, "const float s1 = seg_sum(v, seg), s2 = seg_sum(v * v, seg);",
        "const double s1 = seg_sum((double)v, seg), s2 = seg_sum((double)v * v, seg);")
s = sub(s, "const float s1 = seg_sum(u, seg), s2 = seg_sum(u * u, seg);",
        "const double s1 = seg_sum((double)u, seg), s2 = seg_sum((double)u * u, seg);")
s = sub(s, "const float s1 = seg_sum(gxa, seg), s2 = seg_sum(gxa * xh, seg);",
        "const double s1 = seg_sum((double)gxa, seg), s2 = seg_sum((double)gxa * xh, seg);")
s = sub(s, r'''        vA = seg_sum(vA, seg);
        vB = seg_sum(vB, seg);
        vG = seg_sum(vG, seg);
        if (ok && (lane & (seg - 1)) == 0) {
            atomicAdd(&red[cb], (double)vA);
            atomicAdd(&red[g.Cb + cb], (double)vB);
            atomicAdd(&red[2 * g.Cb + cb], (double)vG);''', r'''        const double dA = seg_sum((double)vA, seg), dB = seg_sum((double)vB, seg), dG = seg_sum((double)vG, seg);
        if (ok && (lane & (seg - 1)) == 0) {
            atomicAdd(&red[cb], dA);
            atomicAdd(&red[g.Cb + cb], dB);
            atomicAdd(&red[2 * g.Cb + cb], dG);''')
s = sub(s, "atomicAdd(&red[cb], (double)s1);", "atomicAdd(&red[cb], s1);", 3)
s = sub(s, "atomicAdd(&red[g.Cb + cb], (double)s2);", "atomicAdd(&red[g.Cb + cb], s2);", 3)
# scale / scale_shift gradients: block partials in fp64
s = sub(s, "    __shared__ float redl[16];\n    const Geo g = geo(a);\n    const Tile t = tile_of(g, TP);\n    float* tab = (float*)dsm;",
        "    __shared__ double redl[16];\n    const Geo g = geo(a);\n    const Tile t = tile_of(g, TP);\n    float* tab = (float*)dsm;")
s = sub(s, "    float gsc = 0.f, gss = 0.f;", "    double gsc = 0.0, gss = 0.0;")
s = sub(s, "            gsc += glr * th;\n            gss += glr;", "            gsc += (double)glr * th;\n            gss += glr;")
s = sub(s, "    const float dsc = block_sum(gsc, redl);   // (barriers also publish gs)\n    const float dss = block_sum(gss, redl);",
        "    const float dsc = (float)block_sum(gsc, redl);   // (barriers also publish gs)\n    const float dss = (float)block_sum(gss, redl);")
open(p, "w").write(s)
print("ok")
