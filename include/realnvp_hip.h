/*
 * realnvp_hip.h -- C ABI of the MI355X (gfx950) RealNVP coupling-layer engine.
 *
 * The reference (alisher-turubayev/dl-normalizing-flows) has no FFI: its hot
 * path is the Python nn.Module API of flow_realnvp.RealNVP and
 * modules_realnvp.{Checkerboard,Channelwise}AffineCoupling.  This header is
 * the boundary those modules bind to (via ctypes): plain
 * pointers, sizes and a hipStream_t passed as void*.  Every entry point
 *   - is stream-ordered: no host synchronisation, no allocation (HIP-graph
 *     capture safe);
 *   - returns 0 on success, a positive hipError_t from the launch, or a
 *     negative RNVP_E_* code for invalid arguments (nothing is launched then);
 *   - never takes ownership: the caller (PyTorch's caching allocator in the
 *     Python host) owns every buffer, including workspaces.
 *
 * Layouts: "flow" tensors (x, z, log|det J|) are NCHW fp32 exactly as in the
 * reference.  "net" tensors (the s/t ResNet activations) are NHWC with a
 * padded channel stride `cs` (multiple of 8), dtype RNVP_F32 (parity mode)
 * or RNVP_BF16 (perf mode, fp32 accumulation).  Reductions that feed batch
 * statistics accumulate fp64 sums: layout [2*C] = {sum x, sum x^2}.
 */
#ifndef REALNVP_HIP_H
#define REALNVP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { RNVP_F32 = 0, RNVP_BF16 = 1 };
enum { RNVP_OK = 0, RNVP_E_INVALID = -1, RNVP_E_UNSUPPORTED = -2 };

/* ---- version / capabilities ------------------------------------------- */
int rnvp_version(void);
/* sizeof the library's argument structs, in this order: rnvp_bn_src,
 * rnvp_bn_running, rnvp_conv_args, rnvp_wgrad_conv, rnvp_wgrad_group,
 * rnvp_bn_bwd_args, rnvp_wn_desc, rnvp_adam_args, rnvp_coupling_args,
 * rnvp_net_step, rnvp_range, rnvp_link_args (-1 past the end).  A binding compares them with
 * its own mirrors at load time: a library built from another header revision
 * is refused instead of reading descriptor tables at the wrong stride. */
int rnvp_struct_size(int which);
const char* rnvp_status_string(int status);
/* empty one-lane dispatch: delimits engine launches in PMC traces (profiling only) */
int rnvp_marker(int tag, void* stream);

/* ---- index maps (bit-exact permutations) --------------------------------
 * replace AbstractCoupling.build_mask   modules_realnvp.py:211-226
 *         RealNVP.squeeze/undo_squeeze  flow_realnvp.py:121-135
 *         RealNVP.factor_out/restore    flow_realnvp.py:167-193 (the 0/1
 *         order_matrix conv of 139-165 is the permutation implemented here)
 * Shapes are those of the *larger* tensor: squeeze/undo_squeeze take the
 * [B,C,H,W] un-squeezed shape; factor_out/restore the [B,C,H,W] full shape
 * (on/off are [B,2C,H/2,W/2]). */
int rnvp_checkerboard_mask(float* mask, int size, int config, void* stream);
int rnvp_squeeze(const float* x, float* y, int B, int C, int H, int W, void* stream);
int rnvp_undo_squeeze(const float* y, float* x, int B, int C, int H, int W, void* stream);
int rnvp_factor_out(const float* x, float* on, float* off, int B, int C, int H, int W, void* stream);
int rnvp_restore(const float* on, const float* off, float* x, int B, int C, int H, int W, void* stream);

/* ---- logit transform (utils.py:33-72) ----------------------------------
 * y = logit(((x*255+u)/256*2-1)*c+1)/2), logdet[b] = sum softplus(y)+softplus(-y)-softplus(-logit(c)).
 * u = noise[i] when noise != NULL, else a counter-based Philox4x32-10 uniform
 * in [0,1) keyed by (seed, offset + i), where offset is advanced by
 * (*epoch) * B * n_per_sample when epoch (a device int64, e.g. the optimizer
 * step) is non-NULL -- so a replayed HIP graph draws fresh noise every step.
 * n_per_sample = C*H*W. */
int rnvp_logit_fwd(const float* x, const float* noise, uint64_t seed, uint64_t offset, const long long* epoch,
                   float constraint, float* y, float* logdet, int B, int n_per_sample, void* stream);
int rnvp_logit_inv(const float* x, float* y, float constraint, long long n, void* stream);

/* ---- transforms.ToTensor of a uint8 batch (train.py:65-71) -------------
 * y[i] = x[i] / 255.f (correctly rounded), x and y 16-byte aligned.  Lets the
 * real-data pipeline ship 1 B/pixel over PCIe and convert on the device. */
int rnvp_u8_to_unit(const uint8_t* x, float* y, long long n, void* stream);

/* ---- NCHW fp32 <-> NHWC layout moves (standalone WeightNormConv2d) -----
 * modules_realnvp.py:64-71 called on its own: the operand moves into the
 * engine's NHWC layout (channel stride cs >= C, zero padded; dtype
 * RNVP_F32 / RNVP_BF16) and the result back. */
int rnvp_nchw_to_nhwc(const float* x, void* y, int B, int C, int H, int W, int cs, int dtype, void* stream);
int rnvp_nhwc_to_nchw(const void* x, float* y, int B, int C, int H, int W, int cs, int dtype, void* stream);

/* ---- prior log-prob and per-sample reduction (flow_realnvp.py:329-340) --
 * out[b] = ldj[b] + sum_i (-z_i^2/2 - log(2 pi)/2)       (N(0,1) prior)
 * bwd: gz_i = -z_i * gout[b] */
int rnvp_prior_logprob(const float* z, const float* ldj, float* out, int B, int n_per_sample, void* stream);
int rnvp_prior_logprob_bwd(const float* z, const float* gout, float* gz, int B, int n_per_sample, void* stream);

/* ---- batch-norm statistic sources --------------------------------------
 * Batch sums written by many workgroups are SHARDED to keep fp64 atomic
 * contention bounded: layout [shards][2][C]; a reader adds the shards.
 * rnvp_stat_shards(M) is the shard count the conv kernels use for an M-pixel
 * output (callers size their sum buffers with it). */
typedef struct rnvp_bn_src {
    const double* sums;   /* [shards][2*C] {sum, sum of squares} of the batch, or NULL */
    double count;         /* elements per channel behind sums */
    const float* mean;    /* running mean (used when sums == NULL) */
    const float* var;     /* running var */
    const float* gamma;   /* affine weight, NULL = 1 */
    const float* beta;    /* affine bias, NULL = 0 */
    float eps;
    int shards;           /* >= 1 */
} rnvp_bn_src;
int rnvp_stat_shards(long long M);

/* running-stat update of nn.BatchNorm2d in train mode, for n BN sites at once.
 * rm = (1-mom) rm + mom mean; rv = (1-mom) rv + mom var*count/(count-1); nbt += 1 */
typedef struct rnvp_bn_running {
    const double* sums; double count; int C; int shards;
    float* rmean; float* rvar; long long* nbt;
} rnvp_bn_running;
int rnvp_bn_running_update(const rnvp_bn_running* descs_device, int n, int max_c, float momentum, void* stream);

/* ---- s/t ResNet convolution (MFMA implicit GEMM) -----------------------
 * replaces WeightNormConv2d.forward (modules_realnvp.py:64-71) inside
 * ResidualModule/ResidualBlock (73-194) with the surrounding
 * BatchNorm2d+ReLU fused into the operand load and bias / residual add /
 * skip accumulation / BN statistics fused into the epilogue.
 * y[m, n] (+)= sum_k act(x)[m + tap(k), ci(k)] * w[n, k] (+ bias[n]) (+ residual[m, n])
 * act = relu(bn(x)) when pro_bn_relu, identity otherwise; zero padding is
 * applied AFTER act (as nn.Conv2d pads its input).  k = (ky*ks+kx)*cs_in + ci.
 * epi_relu_bn_bwd (used for the data gradient): the result g is multiplied
 * by [relu(bn(epi_x)) > 0] before being stored, and epi_sums accumulates
 * {sum g, sum g*xhat} per output channel.  out_sums / epi_sums are sharded
 * with rnvp_stat_shards(B*H*W) shards and must be zeroed by the caller.
 * Small grids split K over workgroups when a workspace is given
 * (ws: fp32, >= splits * M * n elements; the epilogue then runs in a second
 * kernel that reduces the splits).
 * variant: 0 = automatic kernel choice per shape; 1 = the generic LDS-tiled
 * implicit GEMM (+ split-K) wherever the streaming kernel does not apply;
 * RNVP_VARIANT_DEEP = the deep-scale family (LDS activation tile + weight
 * ring) with its automatic configuration where it applies;
 * RNVP_VARIANT_DEEP0 + c = that family's configuration c, no fallback
 * (per call: used by the parity tests to cross-check the kernel families). */
#define RNVP_VARIANT_DEEP 2
#define RNVP_VARIANT_DEEP0 16
typedef struct rnvp_conv_args {
    int dtype;
    int B, H, W, ks;
    const void* x; int cs_in; int cin;
    const void* w; int kp;              /* packed weights [n][kp], kp % 64 == 0 */
    void* y; int cs_out; int n;
    const float* bias;
    const void* residual;
    int accumulate;
    int pro_bn_relu; rnvp_bn_src pro;
    double* out_sums;
    int epi_relu_bn_bwd; const void* epi_x; rnvp_bn_src epi; double* epi_sums;
    float* ws; long long ws_elems;      /* split-K workspace (optional) */
    int variant;
    /* optional (NULL: none): the same weights as w in the fragment-major image
     * -- block (n / 16, k / 32) of 512 bf16 at ((n / 16) * kp / 32 + k / 32) * 512,
     * element (n % 16 + 16 * (k % 32 / 8)) * 8 + k % 8 inside it (n padded to
     * 16 rows with zeros).  The bf16 3x3 deep-scale kernels read it instead of
     * w: each weight load of a wave is one contiguous KiB in MFMA lane order. */
    const void* w_frag;
    /* optional BatchNorm-backward prologue (bp = 1; bf16/fp32 data-gradient
     * convs on the deep-scale tiles, bf16 ones on the wide scales' streaming
     * 1x1 and band 3x3 kernels -- see rnvp_conv2d_check): x is the gradient g of
     * BatchNorm bp_bn's OUTPUT (the producing dgrad's relu/BN epilogue
     * output), bp_x that BatchNorm's saved input t (both [M][cs_in]), and the
     * conv's operand is dL/dt = gamma rstd (g - k1 - xhat k2) with
     * k1 = sum g / count, k2 = sum g xhat / count from bp_sums (the producing
     * epilogue's epi_sums, bp_shards shards <= 2) -- rnvp_bn_bwd_apply's
     * formula, formed while the operand tile is staged, so that apply's
     * launch and its dL/dt round trip disappear.  Workgroups of output
     * channel tile 0 store dL/dt to bp_out ([M][cs_in], for the weight
     * gradient); workgroup 0 writes bp_dbeta[c] = sum g and bp_dgamma[c] =
     * sum g xhat (BatchNorm2d's parameter gradients, modules_realnvp.py:36-52). */
    int bp; const void* bp_x; rnvp_bn_src bp_bn; const double* bp_sums; int bp_shards;
    void* bp_out; float* bp_dgamma; float* bp_dbeta;
} rnvp_conv_args;
int rnvp_conv2d(const rnvp_conv_args* a, void* stream);
/* RNVP_OK when rnvp_conv2d(a) would launch (argument checks and the
 * dispatch's own support limits, nothing launched): the host uses it to
 * decide which BatchNorm-backward applies fold into their consumer (bp). */
int rnvp_conv2d_check(const rnvp_conv_args* a);

/* grouped weight gradient: the wgrads of every conv of one coupling's s/t
 * network in ONE launch (they are independent of each other once the
 * coupling's data-gradient chain has run).  Conv c's pixel range is cut into
 * nz slabs; a workgroup owns one [64 n] x [64 k] tile of one slab and adds
 * its fp32 partial into replica z % nrep of ws[nrep][n][kp] (fp32 atomics,
 * <= nz/nrep adders per word; plain stores when nrep == nz); the bias partial
 * of k tile 0 goes to wsb[nrep][n] the same way.  ws / wsb must be zero on
 * entry; the weight-norm backward (rnvp_weight_norm_bwd, nz = nrep) sums the
 * replicas (and re-zeroes them when zero_after).  The library fills m_per_slab / task0 / tk.
 * Replaces the per-conv backward of WeightNormConv2d (modules_realnvp.py:53-59)
 * for the whole ResidualModule. */
#define RNVP_WGRAD_GROUP_MAX 24
typedef struct rnvp_wgrad_conv {
    const void* x; const void* dy;
    float* ws;                          /* [nrep][n][kp] fp32 partial sums */
    float* wsb;                         /* [nrep][n] bias partial sums or NULL */
    rnvp_bn_src pro;
    int cs_in, cin, ks, cs_dy, n, kp, pro_bn_relu, nz, nrep;
    long long m_per_slab;               /* filled by the library */
    int task0, tk, cls;                 /* filled by the library */
} rnvp_wgrad_conv;
typedef struct rnvp_wgrad_group {
    int dtype, B, H, W, n_conv;
    rnvp_wgrad_conv conv[RNVP_WGRAD_GROUP_MAX];
} rnvp_wgrad_group;
/* slab count the grouped wgrad uses for a conv over M pixels, and the
 * replica count (size ws with the latter) */
int rnvp_wgrad_slabs(long long M);
int rnvp_wgrad_replicas(int nz);
int rnvp_conv2d_wgrad_grouped(const rnvp_wgrad_group* g, void* stream);

/* batch-norm backward apply (train mode), the second half of BN backward:
 * dx = gamma*rstd*(g - sum_g/M - xhat * sum_gxhat/M) (+ residual) (+= dx if accumulate)
 * also writes dgamma = sum_gxhat, dbeta = sum_g (when non-NULL) */
typedef struct rnvp_bn_bwd_args {
    int dtype; long long M; int C; int cs;
    const void* g; const void* x; rnvp_bn_src bn;
    const double* sums; int sum_shards;  /* the dgrad epilogue's epi_sums */
    void* dx; const void* residual; int accumulate;
    float* dgamma; float* dbeta;
} rnvp_bn_bwd_args;
int rnvp_bn_bwd_apply(const rnvp_bn_bwd_args* a, void* stream);

/* weight normalisation (torch.nn.utils.weight_norm dim=0, modules_realnvp.py:53-59)
 * w = g * v / ||v||, packed into the forward layout wf[co][(ky*ks+kx)*cs_in+ci]
 * and the flipped, transposed data-gradient layout wd[ci][(ky'*ks+kx')*cs_out+co]
 * (w[co][ci][ks-1-ky'][ks-1-kx']).  g == NULL means a plain conv (w = v).
 * bwd: dv = (g/|v|)(dw - (v.dw/|v|^2) v), dg = v.dw/|v| from the packed dw
 * (sum of nz slabs), written at grad_base + dv_off / dg_off (elements;
 * dg_off < 0 = frozen g); dbias = sum of the nz bias partials at db_off;
 * zero_after: leave the slabs zero for the next atomic accumulation. */
typedef struct rnvp_wn_desc {
    const float* v; const float* g;
    void* wf; void* wd; float* norm;
    float* dw;                         /* packed [nz][cout][kp_f] fp32 (bwd), summed over nz */
    long long dv_off; long long dg_off;
    int cout, cin, ks, cs_in, kp_f, cs_out, kp_d;
    int row0;                          /* first global row (prefix sum of cout) */
    int tile0;                         /* first pack tile (prefix sum of rnvp_weight_norm_tiles) */
    int nz;                            /* dw partial slabs (>= 1) */
    float* dbp;                        /* bias partials [nz][cout] or NULL */
    long long db_off;                  /* bias gradient offset (elements) */
    int zero_after;                    /* re-zero dw / dbp after use (atomic accumulation) */
    int blk0;                          /* first row block (prefix sum of rnvp_weight_norm_opt_blocks) */
    /* optional fragment-major copies of wf / wd (rnvp_conv_args.w_frag; 3x3,
     * cs_in resp. cs_out a multiple of 32, rows padded to 16), written beside
     * the row-major images by rnvp_weight_norm_fwd / _transpose, or NULL */
    void* wf_frag; void* wd_frag;
} rnvp_wn_desc;
/* fwd, for any number of convs (a whole model): one launch computes every
 * row norm, one writes both packed images on [32 co] x [32 ci] tiles
 * ([32 co] x [256 ci] for 1x1 convs; total_tiles = sum over the convs of
 * rnvp_weight_norm_tiles(cout, cin, ks), < 0 for an invalid shape).
 * The images' padding must be zero on entry (it is never written). */
int rnvp_weight_norm_tiles(int cout, int cin, int ks);
int rnvp_weight_norm_fwd(const rnvp_wn_desc* descs_device, int n_desc, int total_rows, int total_tiles, int dtype,
                         void* stream);
/* zero0 / zero1: byte ranges (8-byte multiples, 8-byte aligned, may be
 * NULL / 0) zeroed by the same launch -- the caller's batch-statistic sums,
 * left zero for the next step once the coupling's backward has consumed them */
int rnvp_weight_norm_bwd(const rnvp_wn_desc* descs_device, int n_desc, int total_rows, float* grad_base,
                         void* zero0, long long zero0_bytes, void* zero1, long long zero1_bytes, void* stream);

/* Row-local parameter pass (weight-norm backward + Adam + next weight norm).
 * One launch per coupling replaces rnvp_weight_norm_bwd + that coupling's
 * share of rnvp_adam_step + the next step's rnvp_weight_norm_fwd: for every
 * output row co of every conv in the table, with dv_off / dg_off / db_off
 * indexing the adam arenas (param, grad, exp_avg, exp_avg_sq, mask):
 *   from_slabs = 1: dW = sum of the nz slabs, dv / dg / dbias as
 *     rnvp_weight_norm_bwd (also stored into grad); from_slabs = 0: dv / dg /
 *     dbias read from grad (data parallel, after the all-reduce);
 *   Adam (rnvp_adam_update semantics, t = *step + step_add) on the row of v
 *     (mask 1 assumed: the caller checks), g[co] (when dg_off >= 0) and the
 *     bias (db_off >= 0; db_off < 0 = no bias), with their mask bytes;
 *   norm[co] = ||v'||, and the forward packed image (rnvp_weight_norm_fwd
 *     layout) of w' = g' v' / ||v'|| for the next step; the data-gradient
 *     image then follows from rnvp_weight_norm_transpose.
 * blk0: prefix sums of rnvp_weight_norm_opt_blocks(cout, cin, ks) (negative:
 * the row does not fit the kernel's LDS -- use the unfused calls); the block
 * count assumes the packed row layout cs_in == round_up(cin, 8), which every
 * descriptor of this call must have (the binding checks its tables).
 * zero0 / zero1 as rnvp_weight_norm_bwd.  Replaces modules_realnvp.py:53-59
 * (weight_norm) and train.py:134, 200 (Adam) for the s/t convs. */
typedef struct rnvp_adam_args {
    float* param; float* grad; float* exp_avg; float* exp_avg_sq; const uint8_t* mask;
    const long long* step; long long step_add;
    float lr, beta1, beta2, eps, weight_decay, reg_coef;
} rnvp_adam_args;
int rnvp_weight_norm_opt_blocks(int cout, int cin, int ks);
int rnvp_weight_norm_bwd_adam(const rnvp_wn_desc* descs_device, int n_desc, int total_blocks, int from_slabs,
                              int dtype, const rnvp_adam_args* adam, void* zero0, long long zero0_bytes,
                              void* zero1, long long zero1_bytes, void* stream);
/* wd from wf (the transposed, flipped data-gradient image from the forward
 * image; bitwise what rnvp_weight_norm_fwd writes for the same weights), on
 * rnvp_weight_norm_fwd's tiles (tile0 / total_tiles) */
int rnvp_weight_norm_transpose(const rnvp_wn_desc* descs_device, int n_desc, int total_tiles, int dtype,
                               void* stream);
/* zero n byte ranges (8-byte multiples and alignment; max_bytes >= every
 * range's size): the batch-statistic sums a deferred parameter pass leaves
 * zero for the next step */
typedef struct rnvp_range { void* p; long long bytes; } rnvp_range;
int rnvp_zero_ranges(const rnvp_range* ranges_device, int n, long long max_bytes, void* stream);
/* Adam on the arena elements idx[0..n) (the parameters outside the convs:
 * BatchNorm affines, coupling scales, ...), rnvp_adam_update semantics */
int rnvp_adam_gather(const rnvp_adam_args* adam, const long long* idx, long long n, void* stream);

/* ---- affine coupling (modules_realnvp.py:239-370) -----------------------
 * kind 0 = CheckerboardAffineCoupling, 1 = ChannelwiseAffineCoupling.
 * Cb = channels seen by in_bn/out_bn: C (ckbd) or C/2 (chan).
 * Net input h0 = relu(cat(bn_in(xm), -bn_in(xm)[, mask])) with xm = x*mask
 * (ckbd, 2C+1 channels) or the "off" half (chan, C channels).  Net output
 * st = [shift | log_rescale] (2*Cb channels). */
/* the coupling's per-channel fp64 reductions are spread over this many
 * shards (workgroup % shards) so no word takes more than ~32 atomic adders */
#ifndef RNVP_COUPLING_SHARDS
#define RNVP_COUPLING_SHARDS 16
#endif
typedef struct rnvp_coupling_args {
    int kind, B, C, H, W, mask_config, coupling_bn, training, dtype;
    float momentum, eps;
    const float* x;                       /* coupling input (reverse: the output) */
    const float* in_gamma; const float* in_beta;
    float* in_rmean; float* in_rvar; long long* in_nbt;
    double* in_sums;                      /* [RNVP_COUPLING_SHARDS][2*Cb] */
    void* h0; int cs_h0;
    const void* st; int cs_st;
    const float* scale; const float* scale_shift;
    float* u;                             /* pre-out_bn value, [B,C,H,W] */
    float* z;                             /* output [B,C,H,W] */
    double* out_sums;                     /* [RNVP_COUPLING_SHARDS][2*Cb] */
    float* out_rmean; float* out_rvar; long long* out_nbt;
    float* ldj_sample;                    /* [B], += */
    float* ldj_full;                      /* [B,C,H,W] or NULL, written */
    /* backward */
    const float* gz;                      /* [B,C,H,W] */
    const float* gl_full;                 /* [B,C,H,W] or NULL */
    const float* gl_sample;               /* [B] used when gl_full == NULL */
    float* gx;                            /* [B,C,H,W] */
    void* gst; int cs_gst;
    double* bwd_sums;                     /* [RNVP_COUPLING_SHARDS][3*Cb] */
    float* g_scale; float* g_scale_shift; /* += */
    const void* gh0; int cs_gh0;
    double* in_bwd_sums;                  /* [RNVP_COUPLING_SHARDS][2*Cb] */
    float* g_in_gamma; float* g_in_beta;  /* written */
    /* optional, forward (rnvp_coupling_out_fwd): running-stat updates of the
     * s/t net's BatchNorms (what rnvp_bn_running_update does), folded into
     * the out launch; net_running is a device table of n_net_running sites
     * with at most net_running_cmax channels */
    const rnvp_bn_running* net_running; int n_net_running; int net_running_cmax;
    /* optional: [RNVP_COUPLING_SHARDS][2] fp64 partials of the scale /
     * scale_shift gradients -- zero on entry to rnvp_coupling_out_bwd, which
     * adds into them (one shard per group of workgroups instead of every
     * workgroup on one address); rnvp_coupling_in_bwd folds them into
     * g_scale / g_scale_shift (+=) and leaves them zero */
    double* gscale_part;
    /* optional, coupling links (rnvp_coupling_out_u, rnvp_coupling_link_fwd /
     * _bwd; see "coupling links" below).  All [RNVP_COUPLING_SHARDS][...] fp64,
     * zeroed on entry to the step that accumulates them:
     *   cls_sums   [nclass][2][C]  sums of u and u^2 per (pixel class, channel),
     *              every channel; pixel classes by nclass: 1 = one class,
     *              2 = (i+j)&1, 4 = (i&1)*2+(j&1) at pixel (i, j)
     *   prior_sums [nclass][2][C]  sums of -z*g_lp[b] and -z^2*g_lp[b] over the
     *              elements the link hands to the prior (factored out / final)
     *   outp_sums  [2][2][C]       sums of gx and gx*x per ((i+j)&1, channel) of
     *              this coupling's direct input gradient (written by its out
     *              part's link backward, read by the previous link's)
     *   in_bwd_ext [2][Cb]         sums of dL/dxa and dL/dxa * xm over the
     *              positions in_bn normalises (the kept squares / the
     *              conditioning half)
     * and two fp32 tables the forward leaves for the backward (written by the
     * link launch that computes them, or rnvp_coupling_in_apply):
     *   out_tab    [2][Cb]         out_bn batch mean, 1/sqrt(var + eps)
     *   in_tab     [4][Cb]         in_bn scale, shift, mean, 1/sqrt(var + eps) */
    int nclass;
    double* cls_sums;
    double* prior_sums;
    double* outp_sums;
    double* in_bwd_ext;
    float* out_tab;
    float* in_tab;
} rnvp_coupling_args;
int rnvp_coupling_in_fwd(const rnvp_coupling_args* a, void* stream);   /* in_sums must be zeroed */
int rnvp_coupling_out_fwd(const rnvp_coupling_args* a, void* stream);  /* out_sums must be zeroed */
int rnvp_coupling_reverse(const rnvp_coupling_args* a, void* stream);  /* z = inverse(x) */
/* backward of rnvp_coupling_reverse (training or eval; the out_bn inverse uses
 * the running statistics, modules_realnvp.py:284-291): from gz = dL/dz and
 * gl_full = dL/dlog_diag_J (or NULL) writes gx's direct part, the net output
 * gradient gst and the scale / scale_shift partials into gscale_part (which
 * rnvp_coupling_in_bwd folds into g_scale / g_scale_shift); the net backward
 * and rnvp_coupling_in_bwd then run as after rnvp_coupling_out_bwd. */
int rnvp_coupling_reverse_bwd(const rnvp_coupling_args* a, void* stream);
int rnvp_coupling_out_bwd(const rnvp_coupling_args* a, void* stream);  /* bwd_sums zeroed; writes gx, gst */
int rnvp_coupling_in_bwd(const rnvp_coupling_args* a, void* stream);   /* in_bwd_sums zeroed; gx += */

/* ---- coupling links (the training step's flow program) ----------------------
 * A link joins coupling a to what consumes its output z (flow_realnvp.py:252-327):
 *   RNVP_LINK_SAME      coupling n with n->x = z (same kind and shape, the
 *                       opposite mask: checkerboard_combo / channelwise_combo,
 *                       flow_realnvp.py:98-116)
 *   RNVP_LINK_SQUEEZE   checkerboard a -> channelwise n, n->x = squeeze(z)
 *                       (flow_realnvp.py:260; squeeze 121-127)
 *   RNVP_LINK_UNFACTOR  channelwise a -> the next scale's checkerboard n,
 *                       (n->x, off) = factor_out(undo_squeeze(z)) (264-267, 167-177):
 *                       n->x channel c = z channel 4c (c < K) / 4(c-K)+3, off
 *                       channel c = z channel 4c+1 / 4(c-K)+2 (K = n->C/2); the
 *                       off half goes to the prior
 *   RNVP_LINK_FINAL     z is the last scale's output: all of it goes to the
 *                       prior (312-327, 336-338)
 * The squeeze / factor-out permutations live in the link's addressing: no
 * permuted copy is made.  The prior log N(0,1) of what the link hands to the
 * prior is added into prior[b] (fp64, flow_realnvp.py:336-338).
 *
 * Forward, per coupling a: rnvp_coupling_out_u(a) (after a's s/t net: the
 * per-class sums of u and the per-sample sum of log_rescale) then
 * rnvp_coupling_link_fwd(a, n, l): z = out_bn(u) (u recomputed from x and the
 * net output), a's log-det constant and running statistics, n->x, n's in_bn
 * statistics in closed form from a's class sums (n->in_sums shard 0; n's in_bn
 * reads positions that are each wholly transformed or wholly kept by a), n's
 * net input h0 and in_bn running statistics.  a->nclass must be
 * rnvp_link_nclass(type, a->kind).
 *
 * Backward, per coupling a (n's backward done first): rnvp_coupling_link_bwd(a,
 * n, l) forms dL/dz of a (n's direct input gradient n->gx + n's in_bn backward
 * from n->gh0, or the prior's -z*g_lp) and runs a's out part with it (a->gx,
 * a->gst, a's scale partials, a->outp_sums) -- the out_bn backward sums it needs
 * are closed forms of n->outp_sums, n->in_bwd_sums, n->in_bwd_ext, n->in_sums and
 * a's class / prior sums; block 0 writes n's in_bn affine gradients.  Then a's
 * net backward and rnvp_coupling_in_bwd(a) with a->in_bwd_ext set (only the
 * reduction pass runs when a->gx is NULL: the first coupling keeps the apply
 * pass for dL/dx).  Requires training, coupling_bn, per-sample log-det. */
enum { RNVP_LINK_SAME = 0, RNVP_LINK_SQUEEZE = 1, RNVP_LINK_UNFACTOR = 2, RNVP_LINK_FINAL = 3 };
typedef struct rnvp_link_args {
    int type;
    const float* g_lp;       /* [B] dL/dlog_prob[b] (the prior's and every log-det's gradient weight) */
    double* prior;           /* [B] += (UNFACTOR, FINAL) */
    float* off;              /* UNFACTOR: [B, n->C, H, W] factored-out half, or NULL (not stored) */
    float* z;                /* FINAL: a's output [B, C, H, W], or NULL (not stored) */
} rnvp_link_args;
int rnvp_link_nclass(int type, int kind);
int rnvp_coupling_out_u(const rnvp_coupling_args* a, void* stream);
int rnvp_coupling_link_fwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n, const rnvp_link_args* l,
                           void* stream);
int rnvp_coupling_link_bwd(const rnvp_coupling_args* a, const rnvp_coupling_args* n, const rnvp_link_args* l,
                           void* stream);
/* only the in part's apply pass (rnvp_coupling_in_fwd without its statistics
 * pass: a->in_sums already hold the batch sums, e.g. from rnvp_flow_in_fwd) */
int rnvp_coupling_in_apply(const rnvp_coupling_args* a, void* stream);
/* the step's input: logit_transform of raw pixels with device Philox noise
 * (rnvp_logit_fwd semantics, logdet[b] += instead of =) fused with the first
 * coupling's in_bn batch sums (first->in_sums +=, NULL = none; first->x must
 * be y).  Spread over every CU (pixel tiles, not one workgroup per sample). */
int rnvp_flow_in_fwd(const float* x, uint64_t seed, const long long* epoch, float constraint, float* y,
                     float* logdet, const rnvp_coupling_args* first, int B, int C, int H, int W, void* stream);
/* end of the forward: lp[b] = prior[b] + ldj[b]; ll_acc[0] += mean_b(lp[b] +
 * logdet[b]) (fp64); prior and ldj are left zero for the next step, and
 * logdet too when zero_logdet */
int rnvp_flow_lp_finish(double* prior, float* ldj, float* logdet, int zero_logdet, float* lp, double* ll_acc, int B,
                        void* stream);

/* ---- regulariser and optimizer ------------------------------------------
 * weight_scale = sum over tensors of sum p^2  (flow_realnvp.py:362-369);
 * out must be zeroed.  bwd: grad_i += 2 * gout * p_i. */
typedef struct rnvp_tensor_ref { float* p; float* g; long long n; } rnvp_tensor_ref;
int rnvp_sumsq_multi(const rnvp_tensor_ref* refs_device, int n_refs, float* out, void* stream);
int rnvp_sumsq_bwd_multi(const rnvp_tensor_ref* refs_device, int n_refs, const float* gout, float coef, void* stream);

/* torch.optim.Adam step (coupled L2 weight decay, train.py:134) over a flat
 * fp32 parameter arena (n % 4 == 0, 16-B aligned).  step is a device int64
 * incremented by this call.  mask (optional, uint8 per element): 0 = frozen
 * (requires_grad=False: parameter and moments untouched, as torch skips
 * params without grad), 1 = trainable, 2 = trainable and regularised, i.e.
 * reg_coef*2*p is added to its gradient (the 5e-5*weight_scale term of
 * train.py:194 for trainable weight_g / scale).  NULL = all trainable. */
int rnvp_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                   long long* step, float lr, float beta1, float beta2, float eps, float weight_decay,
                   const uint8_t* mask, float reg_coef, void* stream);

/* the same update over one range [param, param+n) of the arena WITHOUT
 * touching the step counter: bias corrections use t = *step + step_add.  Lets
 * the optimizer run per parameter group as soon as that group's gradient is
 * final (e.g. per coupling, overlapped with the rest of the backward); the
 * caller advances the counter once per step with rnvp_step_increment. */
int rnvp_adam_update(float* param, float* grad, float* exp_avg, float* exp_avg_sq, long long n,
                     const long long* step, long long step_add, float lr, float beta1, float beta2, float eps,
                     float weight_decay, const uint8_t* mask, float reg_coef, void* stream);
int rnvp_step_increment(long long* step, void* stream);

/* ---- net steps ------------------------------------------------------------
 * One s/t-net step as a table entry (rnvp_net_group): a conv (rnvp_conv2d
 * semantics) or a BatchNorm-backward apply (rnvp_bn_bwd_apply semantics).
 * grad_base-relative dgamma_off / dbeta_off (elements, < 0 = not written)
 * locate a BN step's affine gradients. */
enum { RNVP_STEP_CONV = 0, RNVP_STEP_BN_BWD = 1 };
typedef struct rnvp_net_step {
    int kind;
    rnvp_conv_args conv;
    rnvp_bn_bwd_args bn;
    long long dgamma_off, dbeta_off;
    /* filled by rnvp_net_group_prepare */
    int cfg, nc, shards, xa, xb, tiles;
} rnvp_net_step;

/* ---- grouped 1x1 convs --------------------------------------------------
 * Up to RNVP_NET_GROUP_MAX INDEPENDENT 1x1 convs of one net (same pixels; no
 * conv reads what another writes) in ONE launch: the workgroups of all of
 * them share the grid, so one conv's memory waits overlap another's MFMAs
 * and the kernel boundaries between them disappear.  Used for the skip convs
 * of ResidualModule (modules_realnvp.py:184-189): each core_skips[i] forward
 * runs beside the next block's first 1x1, and the data gradients of
 * in_skip + every core_skips[i] (all read d out) run as one launch.
 * Steps are rnvp_net_step with kind RNVP_STEP_CONV (rnvp_conv2d semantics,
 * with or without the BN prologue).  rnvp_net_group_prepare (host) validates
 * and fills the derived fields (RNVP_E_UNSUPPORTED: no grouped form -- launch
 * them one by one); rnvp_net_group launches the filled HOST table: the
 * members travel by value in the kernel arguments (pointers read from the
 * argument segment address global memory; read from a device table they
 * would be generic, flat operations).  The table may be reused or freed as
 * soon as the call returns (stream capture records the arguments). */
#define RNVP_NET_GROUP_MAX 8
int rnvp_net_group_prepare(rnvp_net_step* steps_host, int n, int* klass, int* grid, int* lds_bytes);
int rnvp_net_group(const rnvp_net_step* steps_host, int n, int dtype, int klass, int grid, int lds_bytes,
                   void* stream);

/* misc */
int rnvp_fill_f64(double* p, long long n, double v, void* stream);

#ifdef __cplusplus
}
#endif
#endif
