/*
 * stcgan_hip.h -- C-ABI of the MI355X (gfx950) ST-CGAN hot-path library
 * (libstcgan_hip.so, built from the .hip sources in shadow-removal-istd_amd/csrc).
 *
 * The reference (nhchiu/Shadow-Removal-ISTD) has no native boundary: its hot
 * path is torch.nn modules running on cuDNN/ATen.  Each entry
 * point below replaces one implicit vendor kernel family on that path and
 * names the reference call site it serves:
 *
 *   stc_conv_fwd     Conv2d 4x4 s2/s1 p1 forward     STCGAN/networks.py:104-105,156-157,167-169,176-178,183-184
 *                    ConvTranspose2d 4x4 s2 p1 fwd   STCGAN/networks.py:112-114,119-121,126-128
 *                    and both layers' input gradient (conv dgrad == convT fwd geometry and vice versa)
 *   stc_conv_wgrad   weight gradient of both         (autograd of the same lines)
 *   stc_conv_fwd_ex  the same forward with the BatchNorm batch statistics of its output fused in
 *                    (Conv/ConvT -> BatchNorm2d pairs, networks.py:104-109,112-121,167-170,176-179)
 *   stc_conv_bwd_bn  input-gradient conv with the consumer BatchNorm-backward reduction fused in
 *   stc_pack_weight / stc_pack_weights  torch weight layout -> GEMM operand layout (one / many tensors)
 *   stc_chan_stats / stc_bn_finalize               BatchNorm2d train/eval forward, STCGAN/networks.py:107,109,170,179
 *   stc_bn_bwd_reduce / stc_bn_bwd_apply            BatchNorm2d backward fused with LeakyReLU/ReLU backward
 *                    (with mean == NULL: LeakyReLU(0.2)/ReLU backward alone, networks.py:106,108,158)
 *   stc_tanh_bias_bwd Tanh backward + outermost ConvT bias grad (networks.py:112-116)
 *   stc_gather_nchw / stc_scatter_nchw              torch.cat input concat (stcgan.py:219-227,269-272) / its backward
 *   stc_loss_fwd / stc_loss_bwd                     DataLoss (L1) and AdversarialLoss (MSE / BCE-with-logits), loss.py:14-26,59-86
 *   stc_adam_step    torch.optim.Adam                STCGAN/stcgan.py:60-65
 *   stc_infer_output infer() output stage: x*0.5+0.5, cv.resize INTER_LINEAR, float2uint
 *                    (STCGAN/stcgan.py:355-377, STCGAN/utils.py:63-65)
 *   stc_istd_errors  ISTD evaluation: masked LAB RMSE/MAE sums + PSNR squared error (src/eval.py:41-139)
 *   stc_istd_ssim    ISTD evaluation: SSIM (src/eval.py:137-139)
 *   stc_prepare_batch / stc_prepare_batch_f32 / stc_resize_area  training batch: uint2float, (v-0.5)*2,
 *                    Resize (INTER_AREA), RandomHorizontalFlip, RandomCrop (STCGAN/dataset.py:89-147, transform.py:103-181)
 *
 * Conventions
 *   - Activations are NHWC ("view" = base pointer + explicit strides, so a
 *     channel slice of a concat buffer is addressed in place, zero-copy).
 *   - The library never allocates device memory; all workspace comes from the
 *     caller.  Every call enqueues on the given hipStream_t only.
 *   - Every call returns 0 on success, or a non-zero code; stc_last_error()
 *     returns a thread-local message.  No C++ exception crosses the ABI.
 *   - dtype: STC_F32 = 0, STC_BF16 = 1 (activation / operand storage type;
 *     accumulation, BN statistics and optimizer state are always fp32).
 */
#ifndef STCGAN_HIP_H
#define STCGAN_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { STC_F32 = 0, STC_BF16 = 1 };

/* 4-D NHWC tensor view: element (b, y, x, c) lives at
 *   p + b*bs + y*rs + x*ps + (co + c)*cs                                    */
typedef struct {
  void* p;
  int32_t H, W;   /* logical extent (bounds for reads / reductions)        */
  int64_t bs;     /* batch stride, elements                                */
  int64_t rs;     /* row stride, elements                                  */
  int32_t ps;     /* pixel stride, elements                                */
  int32_t co;     /* channel offset                                        */
  int32_t cs;     /* channel stride (1 for NHWC, H*W for NCHW)             */
  int32_t pad_;
} stc_view;

/* ---- implicit-GEMM convolution -------------------------------------------
 * kind:
 *   STC_CONV_S2  : Conv2d k4 s2 p1 forward           (also ConvT dgrad)
 *   STC_CONV_S1  : Conv2d k4 s1 p1 forward
 *   STC_CONVT_S2 : ConvTranspose2d k4 s2 p1 forward  (also Conv-s2 dgrad), 4 phases
 *   STC_CONV_S1_DGRAD : input gradient of Conv2d k4 s1 p1
 * The packed weight comes from stc_pack_weight with the matching pack mode.
 * prologue (applied to every in-bounds input element before the product,
 * zero padding stays zero): v = v*scale[c] + shift[c] (if scale != NULL),
 * then v = v > 0 ? v : v*slope (if pro_act != 0).
 * epilogue: + bias[n] (if bias != NULL), tanh (if epi_tanh).                */
enum { STC_CONV_S2 = 0, STC_CONV_S1 = 1, STC_CONVT_S2 = 2, STC_CONV_S1_DGRAD = 3 };

int stc_conv_fwd(int dtype, int kind, int B,
                 stc_view x, int Cin,
                 const float* pro_scale, const float* pro_shift, int pro_act, float pro_slope,
                 const void* w_packed, int Cout,
                 stc_view y,
                 const float* bias, int epi_tanh, int out_f32,
                 void* workspace, int64_t workspace_bytes, void* stream);

/* Workspace bytes stc_conv_fwd needs for this problem (split-K slabs).
 * Hg x Wg = GEMM grid: the output grid for the conv kinds, the input grid for STC_CONVT_S2. */
int64_t stc_conv_fwd_workspace(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout);
/* Launch plan chosen for this problem: out[4] = {BM, BN, ksplit, narrow_n}; narrow_n = 1 means
 * the N <= 8 wave-per-pixel kernel (HBM-bound layers) instead of an MFMA tile. */
int stc_conv_fwd_plan(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout, int32_t* out);

/* Conv forward with the BatchNorm batch statistics of its output fused in (the reference's
 * Conv2d/ConvTranspose2d -> BatchNorm2d pairs, STCGAN/networks.py:104-109,112-121,167-170,176-179).
 * stats_part (optional): [stats_chunks][Cout][4] partials in stc_chan_stats format, merged by
 * stc_bn_finalize.  bf16 operands run on the LDS-DMA MFMA kernel, which computes the partials
 * in its epilogue (or in the split-K reduction); other cases run stc_conv_fwd + stc_chan_stats.
 * force_plan (optional, tuning/tests): {tile config, ksplit} for the bf16 kernel.
 * stc_conv_fwd_query returns the workspace bytes, the number of partial-stat chunks and the
 * plan {BM, BN, ksplit, narrow_n, tile config} for the same arguments.                       */
int stc_conv_fwd_query(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout, int out_f32,
                       const int32_t* force_plan, int64_t* workspace_bytes, int32_t* stats_chunks,
                       int32_t* plan_out);
int stc_conv_fwd_ex(int dtype, int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout,
                    stc_view y, const float* bias, int epi_tanh, int out_f32,
                    float* stats_part, int stats_chunks, const int32_t* force_plan,
                    void* workspace, int64_t workspace_bytes, void* stream);

/* Input-gradient conv with the BatchNorm-backward reduction of its consumer fused in.
 * The conv output v is the gradient reaching the output of a BatchNorm (through an activation)
 * at BN channel ch = n - ch_off; with the BN input x (raw conv output of the forward), the same
 * pixel's optional second gradient g_other and the BN tables:
 *   nn = x*scale + shift,  dn = v*act'(nn, slope_self) + g_other*act'(nn, slope_other),
 *   part2[chunk][ch] = {sum dn, sum dn*(x - mean)*rstd}     (stc_bn_bwd_reduce format)
 * over the pixels inside x's extent; stc_bn_bwd_apply then finishes the BN backward
 * (STCGAN/networks.py:107-109,170-171,179-180 backward).  bf16 NHWC outputs compute the sums in
 * the GEMM epilogue / split-K reduction; other cases run the conv and stc_bn_bwd_reduce.
 * stc_conv_bwd_bn_chunks_ex: the part2 chunk count for the same arguments (the kernel that runs, and so
 * the count, depends on the views' layout); stc_conv_bwd_bn_chunks: the same from the shape alone, for dense
 * 16-byte NHWC views at channel offset 0 (and no second gradient on the 31 x 31 logits-layer gradient).   */
typedef struct {
  stc_view x;        /* BN input (raw pre-BN values), C channels, extent = the BN domain  */
  stc_view g_other;  /* optional second gradient into the BN output (p == NULL: none)     */
  const float* scale;
  const float* shift;
  const float* mean;
  const float* rstd;
  float slope_self, slope_other;
  int32_t C, ch_off;
} stc_bnb_fuse;
int stc_conv_bwd_bn_chunks(int dtype, int kind, int B, int Hg, int Wg, int Cin, int Cout, int xH, int xW);
int stc_conv_bwd_bn_chunks_ex(int dtype, int kind, int B, stc_view dy, int Cin, int Cout, stc_view out,
                              const stc_bnb_fuse* bnb);
int stc_conv_bwd_bn(int dtype, int kind, int B, stc_view dy, int Cin, const void* w_packed, int Cout, stc_view out,
                    const stc_bnb_fuse* bnb, float* part2, int nchunks,
                    void* workspace, int64_t workspace_bytes, void* stream);
/* stc_conv_bwd_bn + stc_bn_bwd_apply from one call: the BN layer's input gradient dx (and dgamma / dbeta), with the
 * conv output at channels ch_off.. over x's extent as the gradient reaching the BN output (through slope_self).  */
int stc_conv_bwd_bn_apply(int dtype, int kind, int B, stc_view dy, int Cin, const void* w_packed, int Cout,
                          stc_view out, const stc_bnb_fuse* bnb, float* part2, int nchunks, const float* gamma,
                          stc_view dx, float* dgamma, float* dbeta, void* workspace, int64_t workspace_bytes,
                          void* stream);

/* ---- conv + train-mode BatchNorm + activation in one call -----------------------------------------
 * A BN layer's forward (STCGAN/networks.py:104-109,118-128,167-171: conv -> BatchNorm2d (batch statistics, running
 * statistics update) -> LeakyReLU / ReLU): stc_conv_fwd_ex with the statistics into fws, stc_bn_finalize, then
 * stc_bn_apply of apply_x (the conv output, or its cropped extent) into y1 [and y2] -- the same three launches,
 * enqueued by one call.  fws (fp32) = [nchunks*Cout*4 partials | mean | rstd | scale | shift], nchunks from
 * stc_conv_fwd_query; y1.p == NULL skips the apply.                                                       */
int stc_conv_bn_fwd(int dtype, int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout, stc_view y,
                    float* fws, int nchunks, const float* gamma, const float* beta, float* running_mean,
                    float* running_var, int64_t* num_batches_tracked, float momentum, float eps, stc_view apply_x,
                    stc_view y1, float slope1, stc_view y2, float slope2, void* workspace, int64_t workspace_bytes,
                    void* stream);

/* ---- input-gradient conv with the activation backward of a layer without BatchNorm ---------------
 * The backward of the first conv's activation (no BatchNorm there): G's outermost level, whose output feeds
 * the next conv through LeakyReLU(0.2) and the skip through ReLU (STCGAN/networks.py:99-106, the in-place skip
 * activation), and the PatchGAN's first layer (networks.py:165-166: LeakyReLU(0.2)).  Replaces stc_conv_fwd into
 * a gradient tensor followed by stc_bn_bwd_apply(no table): with this conv's output v (the gradient reaching the
 * activation, slope_self) and the optional second gradient g_other (slope_other) at the same pixel,
 *   out = g_other*act'(x, slope_other) + v*act'(x, slope_self)    (x = the activation's input)
 * is stored in place of v, rounded to bf16 from the same fp32 values as the two-call form (bit-identical), with
 * no intermediate gradient written or re-read.  stc_conv_bwd_act_ok: 1 when the layer takes the halo kernels
 * with 16-byte NHWC bf16 views of one extent (else use the two-call form).                              */
int stc_conv_bwd_act_ok(int dtype, int kind, int B, stc_view dy, int Cin, int Cout, stc_view out, stc_view x,
                        stc_view g_other);
int stc_conv_bwd_act(int dtype, int kind, int B, stc_view dy, int Cin, const void* w_packed, int Cout,
                     stc_view out, stc_view x, float slope_self, stc_view g_other, float slope_other, void* stream);

/* ---- conv with an activation epilogue (the layers without BatchNorm) -----------------------------
 * The outermost down conv of the generators (STCGAN/networks.py:99-101: conv, then LeakyReLU(0.2) for the
 * next conv and -- in-place on the skip -- ReLU for the up path) and the PatchGAN's first conv
 * (networks.py:165-166: conv + bias, LeakyReLU(0.2)).  Replaces stc_conv_fwd into a raw tensor followed by
 * stc_bn_apply(table = NULL): y1 = act(v, slope1) and, when y2.p != NULL, y2 = act(v, slope2), computed from
 * the bf16-rounded conv output v exactly as stc_bn_apply would (bit-identical), with no raw tensor written
 * or re-read.  stc_conv_fwd_act_ok: 1 when the shape runs as one bf16 LDS-DMA GEMM launch with 16-byte
 * NHWC views (else use the two-call form).                                                            */
int stc_conv_fwd_act_ok(int dtype, int kind, int B, stc_view x, int Cin, int Cout, stc_view y1, stc_view y2);
int stc_conv_fwd_act(int dtype, int kind, int B, stc_view x, int Cin, const void* w_packed, int Cout,
                     stc_view y1, float slope1, stc_view y2, float slope2, const float* bias,
                     void* workspace, int64_t workspace_bytes, void* stream);

/* split-K forward / input-gradient GEMMs (bf16): 1 (default) = the slabs are combined inside the launch by each
 * tile's last-arriving block (a ticket per tile) and it runs the epilogue; 0 = a separate reduction launch (A/B).
 * on < 0 only queries.  Returns the previous setting.  Workspace sizes and statistics chunk counts
 * (stc_conv_fwd_query / stc_conv_bwd_bn_chunks) follow the setting: query after changing it.                     */
int stc_set_splitk_inlaunch(int on);

/* ---- weight gradient ---------------------------------------------------------
 * dW[r][ci][kh][kw] = sum_{b,oy,ox} D[b,oy,ox,r] * G[b, oy*s+kh-1, ox*s+kw-1, ci]
 *   Conv2d s2/s1 : D = dy (grid = output), G = x (input), s = stride
 *   ConvT s2     : D = x (grid = input),  G = dy (output), s = 2
 * D grid is D.H x D.W; prologues (optional) apply to D and G like stc_conv_fwd.
 * dW is written in torch layout [R][Cg_out][4][4] (fp32), Cg_out <= Cg.          */
int stc_conv_wgrad(int dtype, int B, int stride,
                   stc_view D, int R,
                   const float* d_scale, const float* d_shift, int d_act, float d_slope,
                   stc_view G, int Cg, int Cg_out,
                   const float* g_scale, const float* g_shift, int g_act, float g_slope,
                   float* dW, void* workspace, int64_t workspace_bytes, void* stream);
int64_t stc_conv_wgrad_workspace(int dtype, int B, int Hd, int Wd, int R, int Cg);
/* The same with an optional per-call plan (tuning / tests): force_plan = {tile config 0..5, pixel
 * splits (0 = auto)} for the bf16 LDS-DMA kernel, NULL = automatic.  No global state.
 * stc_conv_wgrad_query: workspace bytes and plan_out[5] = {tile config (-1: fp32 / prologue kernel),
 * BM, BN, pixel splits, slab (1: fp32 split slabs + the fixed-order transposing reduction)} for the
 * same arguments (bf16 assumes the LDS-DMA kernel's eligibility: aligned NHWC views, no prologue). */
int stc_conv_wgrad_ex(int dtype, int B, int stride,
                      stc_view D, int R,
                      const float* d_scale, const float* d_shift, int d_act, float d_slope,
                      stc_view G, int Cg, int Cg_out,
                      const float* g_scale, const float* g_shift, int g_act, float g_slope,
                      float* dW, const int32_t* force_plan, void* workspace, int64_t workspace_bytes, void* stream);
int stc_conv_wgrad_query(int dtype, int B, int Hd, int Wd, int R, int Cg, const int32_t* force_plan,
                         int64_t* workspace_bytes, int32_t* plan_out);
/* Narrow-R stride-1 weight gradient (the PatchGAN logits layer, 512 -> 1: STCGAN/networks.py:183-184):
 * as stc_conv_wgrad for stride 1 when only the first R_out (1..2) of the R channels of D are nonzero
 * (channel padding); rows R_out..R-1 of dW are written as zeros.  D: [B][G.H-1][G.W-1][>=R],
 * G: NHWC, Cg % 64 == 0, D plane in LDS.  Workspace: stc_conv_wgrad_rows_workspace(B, G.H, R_out, Cg). */
int stc_conv_wgrad_rows(int dtype, int B, stc_view D, int R, int R_out, stc_view G, int Cg, int Cg_out,
                        float* dW, void* workspace, int64_t workspace_bytes, void* stream);
int64_t stc_conv_wgrad_rows_workspace(int B, int IH, int R_out, int Cg);

/* ---- weight packing ----------------------------------------------------------
 * W is a torch weight [P][Q][4][4] fp32.  out is [phases][N_pad][T][C_pad] of dtype.
 *   STC_PACK_CONV_FWD    : conv  W[co][ci] -> n=co, c=ci, 16 taps          (P=Cout,Q=Cin)
 *   STC_PACK_CONV_DGRAD  : conv  W[co][ci] -> n=ci, c=co, 4 phases x 4 taps (convT geometry)
 *   STC_PACK_CONV_S1_DGRAD: conv W[co][ci] -> n=ci, c=co, 16 taps
 *   STC_PACK_CONVT_FWD   : convT W[ci][co] -> n=co, c=ci, 4 phases x 4 taps (P=Cin,Q=Cout)
 *   STC_PACK_CONVT_DGRAD : convT W[ci][co] -> n=ci, c=co, 16 taps (conv-s2 geometry)      */
enum { STC_PACK_CONV_FWD = 0, STC_PACK_CONV_DGRAD = 1, STC_PACK_CONV_S1_DGRAD = 2,
       STC_PACK_CONVT_FWD = 3, STC_PACK_CONVT_DGRAD = 4 };
int stc_pack_weight(int dtype, int mode, const float* W, int P, int Q,
                    void* out, int N_pad, int C_pad, void* stream);
/* Multi-tensor packing: all stale packed operands of a network after an optimiser step in one
 * launch (n <= STC_PACK_MAX descriptors, each as stc_pack_weight's arguments).               */
#define STC_PACK_MAX 40
typedef struct {
  int32_t mode;
  int32_t P, Q, N_pad, C_pad;
  int32_t pad_;
  const float* W;
  void* out;
} stc_pack_desc;
int stc_pack_weights(int dtype, int n, const stc_pack_desc* descs, void* stream);

/* ---- batch norm -------------------------------------------------------------
 * stc_chan_stats: per-channel partial statistics of x over pixel chunks:
 *   part[chunk][c] = {count, shifted sum, shifted sum of squares, shift}.
 * stc_bn_finalize: combines partials (fixed order -> deterministic), writes
 *   mean/rstd (train), the affine table scale/shift used as a consumer prologue
 *   (scale = gamma*rstd, shift = beta - mean*scale), and updates running stats
 *   (momentum, unbiased var) + num_batches_tracked.  With part == NULL (eval)
 *   the table is built from the running statistics.                         */
int stc_chan_stats(int dtype, int B, stc_view x, int C, float* part, int nchunks, void* stream);
int stc_chan_stats_chunks(int B, int H, int W);
/* out[c] = sum over pixels of x[..., c] for c < Cout (conv bias gradient), fixed order.
 * part needs nchunks*C floats.                                               */
int stc_chan_sum(int dtype, int B, stc_view x, int C, int Cout, float* part, int nchunks, float* out, void* stream);
int stc_bn_finalize(const float* part, int nchunks, int C,
                    const float* gamma, const float* beta,
                    float* running_mean, float* running_var, int64_t* num_batches_tracked,
                    float momentum, float eps,
                    float* mean, float* rstd, float* scale, float* shift, void* stream);

/* Activation materialisation (BatchNorm apply + LeakyReLU/ReLU, STCGAN/networks.py:106-109,
 * 158, 170-171, 179-180): n = x*scale + shift (identity if scale == NULL), y1 = act(n, slope1),
 * y2 = act(n, slope2) if y2.p != NULL; act(v, s) = v > 0 ? v : s*v (s = 0 ReLU, 0.2 LeakyReLU,
 * 1 identity).  One pass per BN'd tensor; the consuming GEMMs then stage plain operands. */
int stc_bn_apply(int dtype, int B, stc_view x, int C, const float* scale, const float* shift,
                 stc_view y1, float slope1, stc_view y2, float slope2, void* stream);

/* BN backward fused with the activation backward of its consumers:
 *   n  = x*scale + shift (the BN output; scale/shift from stc_bn_finalize)
 *   dn = g1 * act1'(n) + g2 * act2'(n)   (g1/g2 optional; act' = 1 if n>0 else slope)
 *   reduce: part2[chunk][c] = {sum dn, sum dn*xhat}
 *   apply : dx = gamma*rstd*(dn - sum(dn)/P - xhat*sum(dn*xhat)/P); dgamma, dbeta.
 * With mean == NULL the BN is absent (identity affine): apply writes dx = dn. */
int stc_bn_bwd_reduce(int dtype, int B, stc_view x, int C,
                      const float* scale, const float* shift, const float* mean, const float* rstd,
                      stc_view g1, float slope1, stc_view g2, float slope2,
                      float* part2, int nchunks, void* stream);
int stc_bn_bwd_apply(int dtype, int B, stc_view x, int C,
                     const float* scale, const float* shift, const float* mean, const float* rstd,
                     const float* gamma,
                     stc_view g1, float slope1, stc_view g2, float slope2,
                     const float* part2, int nchunks,
                     stc_view dx, float* dgamma, float* dbeta, void* stream);

/* y = tanh(q) stored NCHW fp32 (the generator output).  dq = gy*(1-y^2) into NHWC
 * view dq; dbias[c] = sum dq (deterministic).                               */
int stc_tanh_bias_bwd(int dtype, int B, int C, int H, int W, const float* y, const float* gy,
                      stc_view dq, float* dbias, float* part, int nchunks, void* stream);

/* ---- layout -------------------------------------------------------------------
 * Gather up to 4 NCHW fp32 sources (channels concatenated, like torch.cat dim=1)
 * into an NHWC view with Cpad channels (extra channels zero).               */
int stc_gather_nchw(int dtype, int B, int H, int W, int nsrc, const float* const* src,
                    const int* src_c, stc_view dst, int Cpad, void* stream);
/* Scatter channel ranges of an NHWC view back to NCHW fp32 tensors (backward of the gather);
 * dst pointers may be NULL to skip a source.                                */
int stc_scatter_nchw(int dtype, int B, int H, int W, stc_view src, int nsrc, float* const* dst,
                     const int* dst_c, void* stream);

/* ---- losses ---------------------------------------------------------------------
 * kind: STC_LOSS_L1 (|p - t|, t tensor), STC_LOSS_MSE_CONST ((p - c)^2),
 *       STC_LOSS_BCE_CONST (BCE-with-logits vs constant label c).
 * fwd: out[0] = mean loss (deterministic two-level reduction, part >= stc_loss_parts(n) floats).
 * bwd: grad = gout[0] * dloss/dp (gout is a device scalar).                  */
enum { STC_LOSS_L1 = 0, STC_LOSS_MSE_CONST = 1, STC_LOSS_BCE_CONST = 2 };
int stc_loss_parts(int64_t n);
/* One objective of several loss terms (replaces the per-term AdversarialLoss / DataLoss calls and the
 * torch scalar arithmetic combining them, STCGAN/stcgan.py:240-251 (D, loss type "normal") and
 * :291-299 (G)).  Term k: kind (STC_LOSS_*), constant target consts[k] or targets[k], numels[k] elements.
 * fwd: vals[k] = mean loss of term k (bit-identical to stc_loss_fwd), then
 *   STC_LOSS_COMBINE_D (terms fake1, real1, fake2, real2; w = {lambda2, lambda3, -}):
 *     out[0] = D, vals[4] = D1, vals[5] = D2 with D1 = (fake1 + real1) * 0.5, D2 = (fake2 + real2) * 0.5,
 *     D = l2*D1 + l3*D2 (vals: 6 floats);
 *   STC_LOSS_COMBINE_G (terms data1, data2, G1, G2; w = {lambda1, lambda2, lambda3}):
 *     out[0] = G = ((data1 + l1*data2) + l2*G1) + l3*G2;
 *   fp32, one rounding per operation in that order (the torch evaluation).  part: stc_loss_multi_parts floats.
 * bwd: grads[k] (nullable) = ((gout * wa[k]) * wb[k]) / n_k * dloss_k/dp. */
#define STC_LOSS_MAX_TERMS 8
#define STC_LOSS_COMBINE_D 0
#define STC_LOSS_COMBINE_G 1
int stc_loss_multi_parts(int nterm, const int64_t* numels);
int stc_loss_multi_fwd(int nterm, const int32_t* kinds, const float* consts, const float* const* preds,
                       const float* const* targets, const int64_t* numels, int mode, const float* w,
                       float* part, float* vals, float* out, void* stream);
int stc_loss_multi_bwd(int nterm, const int32_t* kinds, const float* consts, const float* const* preds,
                       const float* const* targets, const int64_t* numels, const float* wa, const float* wb,
                       const float* gout, float* const* grads, void* stream);
int stc_loss_fwd(int kind, const float* p, const float* t, float c, int64_t n,
                 float* part, float* out, void* stream);
int stc_loss_bwd(int kind, const float* p, const float* t, float c, int64_t n,
                 const float* gout, float* grad, void* stream);

/* ---- inference output stage ---------------------------------------------------
 * src: generator output NCHW fp32 [B][C][H][W] (tanh range); dst: HWC uint8 [B][OH][OW][C],
 * dst = uint8(trunc(255 * resize_linear(src * 0.5 + 0.5))) with OpenCV's float32 INTER_LINEAR
 * geometry (exact 2x2 downscale: INTER_AREA block mean, as cv::resize does).  C in 1..4.
 * Replaces the per-image numpy / cv.resize / float2uint loop of STCGAN.infer (stcgan.py:355-377). */
int stc_infer_output(const float* src, int B, int C, int H, int W, int OH, int OW, unsigned char* dst,
                     void* stream);

/* ---- ISTD evaluation errors ----------------------------------------------------
 * img1, img2: uint8 RGB [B][H][W][3] (skimage.io.imread order); mask: uint8 [B][H][W] or NULL
 * (shadow = mask/255 >= 0.5; NULL = every pixel is "shadow", eval.py's no-maskdir case).
 * out: fp64 [B][7] = {sum |dLab|_2, sum |dLab|_1, count} over shadow pixels, the same over
 * non-shadow pixels, and sum (v1 - v2)^2 over all pixels and channels (v = u/255), with
 * Lab = skimage.color.rgb2lab (D65, 2 degrees).  ws: >= stc_istd_errors_workspace(B, H, W) bytes. */
int64_t stc_istd_errors_workspace(int B, int H, int W);
int stc_istd_errors(const unsigned char* img1, const unsigned char* img2, const unsigned char* mask, int B, int H,
                    int W, double* out, void* ws, int64_t ws_bytes, void* stream);
/* SSIM of each RGB pair as skimage 0.17 structural_similarity(X, Y, multichannel=True) computes it
 * on float32 images (7x7 uniform window, sample covariance, data_range 2): out fp64 [B].
 * H, W >= 7; ws as for stc_istd_errors (same workspace size query).                          */
int stc_istd_ssim(const unsigned char* img1, const unsigned char* img2, int B, int H, int W, double* out, void* ws,
                  int64_t ws_bytes, void* stream);

/* ISTD evaluation with the reference's resize branches (src/eval.py:64-81), one image pair per call.
 * Images are typed planes [H][W][C]:
 *   STC_IMG_U8F32 (0): uint8 read as util.img_as_float32 (float32(u) * float32(1/255))
 *   STC_IMG_U8F64 (1): uint8 read as util.img_as_float   (u * (1/255) in float64)
 *   STC_IMG_F64   (2): float64
 * stc_image_resize_f64: skimage 0.17 transform.resize(src, (OH, OW), mode="edge", order 1) -> float64,
 *   with anti_alias: the gaussian prefilter of resize's anti_aliasing (sigma = max(0, (in/out-1)/2)
 *   per axis, scipy mode 'nearest', truncate 4); ws >= stc_image_resize_workspace(H, W, C) bytes.
 * stc_istd_errors_ex: out[7] as stc_istd_errors for img1 (U8F32 or F64) vs img2 (U8F32 or F64), the
 *   sRGB gamma in each image's dtype and float64 from the xyz product on (skimage.color.rgb2lab);
 *   mask: float64 [H][W] (shadow = value > 0.5, util.img_as_bool) or NULL.
 * stc_istd_ssim_ex: out[1] = SSIM of the pair (as stc_istd_ssim, typed inputs).
 *   ws for both: >= stc_istd_typed_workspace(H, W) bytes.                                        */
enum { STC_IMG_U8F32 = 0, STC_IMG_U8F64 = 1, STC_IMG_F64 = 2 };
int64_t stc_image_resize_workspace(int H, int W, int C);
int stc_image_resize_f64(const void* src, int kind, int H, int W, int C, int OH, int OW, int anti_alias, double* dst,
                         void* ws, int64_t ws_bytes, void* stream);
int64_t stc_istd_typed_workspace(int H, int W);
int stc_istd_errors_ex(const void* img1, int kind1, const void* img2, int kind2, const double* mask, int H, int W,
                       double* out, void* ws, int64_t ws_bytes, void* stream);
int stc_istd_ssim_ex(const void* img1, int kind1, const void* img2, int kind2, int H, int W, double* out, void* ws,
                     int64_t ws_bytes, void* stream);

/* ---- training-batch preparation ---------------------------------------------------
 * src: uint8 [B][H][W][C] (decoded images, the loader's channel order); params: device int32
 * [B][3] = {flip, row_offset, col_offset} drawn on the host in the reference's order; pad_h /
 * pad_w: the zero border RandomCrop adds when the image is smaller than the crop.
 * dst: fp32 NCHW [B][C][OH][OW] = crop(flip((u / 255 - 0.5) * 2)), border value 0.              */
int stc_prepare_batch(const unsigned char* src, int B, int H, int W, int C, const int* params, int pad_h, int pad_w,
                      int OH, int OW, float* dst, void* stream);
/* The same flip / crop on an already normalised fp32 NHWC source (the output of stc_resize_area). */
int stc_prepare_batch_f32(const float* src, int B, int H, int W, int C, const int* params, int pad_h, int pad_w,
                          int OH, int OW, float* dst, void* stream);
/* Resize of transform.py:159-181 when the image shrinks in both dimensions: cv.resize INTER_AREA of
 * the normalised image ((u / 255 - 0.5) * 2), uint8 [B][H][W][C] -> fp32 NHWC [B][OH][OW][C]. */
int stc_resize_area(const unsigned char* src, int B, int H, int W, int C, int OH, int OW, float* dst, void* stream);

/* Resize (transform.py:173-178) when the image does not shrink in both axes: cv.resize INTER_LINEAR of
 * the float32 image (OpenCV's generic float path); src: uint8 [B][H][W][C] (src_u8 = 1, normalised
 * (u / 255 - 0.5) * 2 on the fly) or fp32 NHWC; dst fp32 NHWC [B][OH][OW][C].                     */
int stc_resize_linear(const void* src, int src_u8, int B, int H, int W, int C, int OH, int OW, float* dst,
                      void* stream);
/* RandomScale / RandomRotate (transform.py:59-100): cv.warpAffine(img, M_b, (W, H), INTER_LINEAR,
 * BORDER_CONSTANT 0) of every image b with its forward matrix M_b (device, float64 [B][6], the
 * getRotationMatrix2D result); OpenCV's inversion and fixed-point (1/32 pixel) sampling.  src as for
 * stc_resize_linear, dst fp32 NHWC [B][H][W][C].                                                  */
int stc_warp_affine(const void* src, int src_u8, int B, int H, int W, int C, const double* M, float* dst,
                    void* stream);

/* ---- optimizer --------------------------------------------------------------------
 * One launch over many tensors.  table: device array of ntensors records
 * {param*, grad*, exp_avg*, exp_avg_sq*, numel, first_block} (6 x int64), where
 * first_block is the prefix sum of ceil(numel / stc_adam_elems_per_block()) and
 * total_blocks the grand total.  torch.optim.Adam semantics (amsgrad=False,
 * weight_decay=0): exp_avg.lerp_(g, 1-b1); exp_avg_sq = b2*v + (1-b2)*g*g;
 * p += -(lr/bc1) * exp_avg / (sqrt(exp_avg_sq)/sqrt(bc2) + eps).              */
int stc_adam_step(const int64_t* table, int ntensors, int64_t total_blocks,
                  float lr, float beta1, float beta2, float eps, int step, void* stream);
int stc_adam_elems_per_block(void);
/* Adam fused with the weight repack (replaces stc_adam_step + stc_pack_weights after a step):
 * table = ntensors records of 24 int64
 *   {param*, grad*, exp_avg*, exp_avg_sq*, numel, first_block, kind, P, Q, q_tiles, npacks,
 *    npacks x {mode, out*, N_pad, C_pad, dtype}, padding}
 * kind 0: a flat tensor, ceil(numel / 1024) blocks.  kind 1: a [P][Q][4][4] weight, one block per
 * 16 x 16 (p, q) tile (q_tiles = ceil(Q / 16)), whose updated values are also written to each of
 * its npacks (<= 2) packed operands exactly as stc_pack_weight(dtype, mode, ..., N_pad, C_pad)
 * would (padding entries are left as they are).  Same Adam arithmetic as stc_adam_step.           */
int stc_adam_pack_step(const int64_t* table, int ntensors, int64_t total_blocks,
                       float lr, float beta1, float beta2, float eps, int step, void* stream);
/* stc_adam_pack_step with the step count on the device, for a train step captured as a HIP graph and
 * replayed (torch.optim.Adam's host-side step count would be frozen into the graph): one thread
 * advances *step_dev and forms lr/(1 - beta1^step) (double, then float) and sqrt(1 - beta2^step)
 * from bc1_tab[s] = 1 - beta1^s (double) and bc2s_tab[s] = (float)sqrt(1 - beta2^s), tables of tab_len
 * entries the caller fills with the host formulas, and *lr_dev (the double value of the float lr);
 * coef_dev: 2 floats of scratch.  Bit-identical to stc_adam_pack_step at the same step.            */
int stc_adam_pack_step_dev(const int64_t* table, int ntensors, int64_t total_blocks, int64_t* step_dev,
                           const double* lr_dev, const double* bc1_tab, const float* bc2s_tab, int tab_len,
                           float* coef_dev, float beta1, float beta2, float eps, void* stream);
/* The update of one optimiser step split over several launches -- each a table of a subset of the
 * parameters, launched as the backward completes their gradients (the optimiser overlapped with the
 * backward; torch.optim.Adam.step() of STCGAN/stcgan.py:229/303 updates every tensor independently, so
 * the split changes no result).  stc_adam_coef_dev: the device step count advanced once for the step
 * (the first half of stc_adam_pack_step_dev).  stc_adam_pack_apply: one table launch with either the
 * host coefficients of (lr, step) (coef_dev == NULL, as stc_adam_pack_step) or the device ones.      */
int stc_adam_coef_dev(int64_t* step_dev, const double* lr_dev, const double* bc1_tab, const float* bc2s_tab,
                      int tab_len, float* coef_dev, void* stream);
int stc_adam_pack_apply(const int64_t* table, int ntensors, int64_t total_blocks, float lr, int step,
                        const float* coef_dev, float beta1, float beta2, float eps, void* stream);
/* dst[e] += src[e] (fp32, numel[e] elements) for ntensors <= 16 tensors in one launch (host arrays of
 * device pointers).  Sums the weight gradients of two calls of one network inside one differentiated
 * graph -- the discriminators' real and fake calls, STCGAN/stcgan.py:215-227 -- which autograd would
 * otherwise add with one ATen kernel per parameter.                                               */
int stc_grad_accumulate(int ntensors, float* const* dst, const float* const* src, const int64_t* numel,
                        void* stream);

/* ---- misc ------------------------------------------------------------------------
 * stc_time_next_main_kernel: instrumentation (bench.py).  The next call ON THIS THREAD that launches a
 * GEMM-family main kernel (stc_conv_fwd, stc_conv_fwd_ex, stc_conv_bwd_bn, stc_conv_wgrad) records
 * ev_begin / ev_end (hipEvent_t, timing enabled) on its stream immediately before and after that kernel
 * -- not around the split-K / split-pixel reduction it may enqueue afterwards -- then disarms.  Both
 * NULL disarms.  Thread-local one-shot state: calls on other threads are unaffected.               */
int stc_time_next_main_kernel(void* ev_begin, void* ev_end);
/* waiter (hipStream_t) waits for everything enqueued so far on src: a pooled event (never destroyed, so it also
 * outlives a graph capture) recorded on src and waited on by waiter -- the host schedule's stream forks and joins
 * (the reference's implicit single stream has none; STCGAN/stcgan.py:203-312 runs the same work serially).     */
int stc_stream_wait(void* waiter, void* src);
const char* stc_last_error(void);
int stc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* STCGAN_HIP_H */
