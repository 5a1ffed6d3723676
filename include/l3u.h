/*
 * l3u.h — C ABI of the MI355X (gfx950) hot path of the Light-3D-U-Net
 *         (Lightweight3DUNet training / inference step + FocalTverskyLoss).
 *
 * Library: light-3d-unet-front_amd/lib/libl3u_hip.so  (built by `make` in that directory).
 *
 * Conventions (every entry point):
 *   - plain device pointers + sizes, no framework types; the caller owns all memory, nothing is
 *     allocated inside, so every call is hipGraph-capturable;
 *   - the last argument is the hipStream_t to enqueue on; calls are asynchronous;
 *   - the return value is a hipError_t as int (0 = hipSuccess; hipErrorInvalidValue for a shape
 *     the kernels do not support, e.g. an H*W plane above 4096 voxels for the stencil);
 *   - activations are NCDHW with the spatial volume S = D*H*W contiguous per (n, c), stored as fp32
 *     or — entry points with the suffix _bf16, same arguments otherwise — as bf16 (l3u_bf16, the
 *     raw 16-bit pattern); kernels compute in fp32 either way (bf16 loads widen, stores round to
 *     nearest even), weights / records / partial sums are always fp32 (fp64 where marked); a tensor
 *     is (pointer, batch stride in elements) — channel stride is always S.  A batch stride larger
 *     than C*S addresses one channel range of a concatenation buffer (zero-copy torch.cat);
 *   - "rec" is the per-(n,c) InstanceNorm record of 8 floats:
 *       {mean, rstd, scale = k*gamma*rstd, shift = k*beta, k, gamma, beta, 0}
 *     and the normalised, activated value is lrelu(scale*(y - mean) + shift)
 *     with k the Dropout3d keep scale (0 or 1/(1-p); 1 without dropout);
 *   - partial-sum buffers are reduced in a fixed order (l3u_reduce_segments), so results are
 *     bitwise run-to-run reproducible.
 *
 * The reference (xxxxxxyp/Light-3D-Unet-Front) is pure Python/PyTorch: it has no native FFI.  Each
 * entry point below names the reference module call it replaces (file:line in the reference);
 * the Python host mirror (light_unet/) binds them through ctypes.
 */
#ifndef L3U_H
#define L3U_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned short l3u_bf16;   /* bfloat16 bit pattern (torch.bfloat16 storage) */

/* ABI version of this header (L3U_ABI_VERSION); the ctypes binding refuses a library that reports
 * another.  3: l3u_norm_src.rank1, L3U_ADAMW_TICKET_INTS tickets, the l3u_sblock_* entry points
 * removed (round 3); the round-4 entry points.  5: l3u_pw_bwd_chunk (round 6). */
#define L3U_ABI_VERSION 5
int l3u_abi_version(void);

/* Where an InstanceNorm record comes from when a consumer kernel finalizes it itself (no separate
 * l3u_in_finalize launch): the (count, mean, M2) partials l3u_pw_fwd emitted for the producing
 * GEMM, the affine parameters and the Dropout3d stream.  Every workgroup of the consumer merges
 * the partials of its (n, c) in the same fixed order (identical values everywhere) and the first
 * workgroup of each (n, c) stores the record to rec_out for the backward pass.                 */
typedef struct l3u_norm_src {
  const float* stat_part;      /* [N][C][nsb][3] */
  int nsb;
  int layer;                   /* dropout stream id */
  const float* gamma;          /* [C] or NULL (1) */
  const float* beta;           /* [C] or NULL (0) */
  float drop_p;                /* 0: no dropout */
  unsigned long long seed;
  const int* step;             /* device step counter or NULL */
  float* rec_out;              /* [N][C][8] or NULL */
  const float* rank1;          /* [C] or NULL: the normalised tensor is rank-1, channel c =
                                  rank1[c] * ONE stored channel (see "rank-1 operands" below);
                                  the record's slot 7 carries rank1[c] (0 otherwise) */
} l3u_norm_src;

/* Rank-1 operands (the first block's y1 = w1[c] * z1 and r = wsc[c] * x, unet3d.py:163-167 with
 * one input channel): a NEGATIVE batch stride (-ns) on the normalised operand of
 *   l3u_dwpw_fwd (x, with src/rec), l3u_norm_act_fwd / l3u_norm_act_pool_fwd (r),
 *   l3u_norm_act_bwd_reduce[_r1|_up] (r), l3u_pw_bwd (y), l3u_pw_bwd_tail[_r1|_up] (yr),
 *   l3u_dw3_bwd (x, with rec) and l3u_dw3_fwd (x, with rec or src; the shapes of
 *   l3u_dw3_bwd_rank1)
 * means that operand holds ONE channel per sample (batch stride ns) and channel c is
 * record[c][7] * it, the float product the materialised tensor would hold (bit for bit).  The
 * record's slot 7 is set when it is finalized from an l3u_norm_src with rank1 != NULL.  fp32
 * entry points only.                                                                          */

/* ---- depthwise 3x3x3 conv, stride 1, padding 1, no bias ------------------------------------
 * replaces nn.Conv3d(C, C, 3, 1, 1, groups=C, bias=False)
 *          (DepthwiseSeparableConv3d.depthwise, light_unet/models/unet3d.py:16-17, forward :21)
 * w: [C][27].  rec != NULL fuses a = lrelu(scale*(x-mean) + shift) into the input load (the
 * InstanceNorm1 + LeakyReLU + Dropout3d that precede conv2.depthwise, unet3d.py:84-89).      */
int l3u_dw3_nchunk(int N, int C, int D, int H, int W);   /* z/y chunks per (n, c) */
int l3u_dw3_bwd_rank1(int N, int C, int D, int H, int W); /* 1: l3u_dw3_bwd and l3u_dw3_fwd
                                                             take a rank-1 x at this shape */
int l3u_dw3_fwd(const float* x, long long x_nstride, const float* w, const float* rec,
                const l3u_norm_src* src, float* y, long long y_nstride, int N, int C, int D,
                int H, int W, hipStream_t stream);   /* src != NULL: finalize rec in-kernel */
/* fused backward (autograd of the same module): dx = conv^T(dz) (accumulate != 0: dx += ...),
 * dw_part[C][N*nchunk][27] partial weight gradients.  rec != NULL: dx receives
 * dpre = dA * k * lrelu'(pre) and in_part[C][N][nchunk][2] (fp64) = {sum dpre, sum dpre*xhat}.*/
int l3u_dw3_bwd(const float* dz, long long dz_nstride, const float* x, long long x_nstride,
                const float* w, const float* rec, float* dx, long long dx_nstride, int accumulate,
                float* dw_part, double* in_part, int N, int C, int D, int H, int W,
                hipStream_t stream);

/* ---- channel-contraction GEMM on MFMA (v_mfma_f32_16x16x4_f32) ------------------------------
 * Y[n][j][s] = sum_k Wm[j][k] X[n][k][s] (+ bias[j]) (+ Y if accumulate)
 * w_layout 0: Wm[j][k] = w[j*K + k]   (torch Conv3d 1x1 weight [Co][Ci]: forward)
 * w_layout 1: Wm[j][k] = w[k*Nout + j] (transposed: backward-data of a 1x1 conv, and
 *                                       ConvTranspose3d weight [Ci][Co*8])
 * replaces nn.Conv3d(Ci, Co, 1, bias=False)  (DepthwiseSeparableConv3d.pointwise, unet3d.py:18;
 *          shortcut conv unet3d.py:70-73; out_conv unet3d.py:201) and the GEMM of
 *          nn.ConvTranspose3d(Ci, Ci//2, 2, 2) (unet3d.py:119).
 * stat_part != NULL: emits InstanceNorm partials [N][Nout][l3u_pw_stat_nsb(K, Nout, S)][3] = (count, mean, M2)
 * of the output for the nn.InstanceNorm3d that follows (unet3d.py:51,62,72).                  */
int l3u_pw_stat_nsb(int K, int Nout, int S);
int l3u_pw_fwd(const float* x, long long x_nstride, const float* w, int w_layout,
               const float* bias, float* y, long long y_nstride, int accumulate,
               float* stat_part, int N, int K, int Nout, int S, hipStream_t stream);
/* two independent 1x1 convs of the same shape (no bias, no accumulate, w [Nout][K]) in ONE launch
 * (a ResidualBlock's Conv1x1 shortcut, unet3d.py:70-73, and its conv1.pointwise, :18: both
 * K = Cin -> Nout = Cout over the same volume); statistics partials as l3u_pw_fwd, both or none.
 * S and every batch stride % 4 == 0.                                                           */
int l3u_pw_fwd2(const float* xa, long long xa_nstride, const float* wa, float* ya,
                long long ya_nstride, float* stat_a, const float* xb, long long xb_nstride,
                const float* wb, float* yb, long long yb_nstride, float* stat_b, int N, int K,
                int Nout, int S, hipStream_t stream);
/* ---- fused depthwise-separable conv forward (one launch per DepthwiseSeparableConv3d) -------
 * replaces DepthwiseSeparableConv3d.forward (unet3d.py:20-23: depthwise 3^3 then pointwise 1x1)
 * and, with w_sc, the ResidualBlock's Conv1x1 shortcut on the same input (unet3d.py:70-73,80):
 *   Z = dw3(A) (A = x, or lrelu(IN(x))*dropout when rec / src is given: unet3d.py:84-89),
 *   y = w_pw . Z,  r = w_sc . x,  z (optional, may be NULL) = Z for the backward.
 * y_stat / r_stat: InstanceNorm (count, mean, M2) partials in the l3u_pw_fwd format with
 * l3u_dwpw_stat_nsb(...) partials per (n, c).  Supported shapes: l3u_dwpw_supported.          */
int l3u_dwpw_supported(int K, int Nout, int D, int H, int W, int shortcut);
int l3u_dwpw_stat_nsb(int K, int Nout, int D, int H, int W);
int l3u_dwpw_fwd(const float* x, long long x_nstride, const float* w_dw, const float* rec,
                 const l3u_norm_src* src, const float* w_pw, float* y, long long y_nstride,
                 float* y_stat, const float* w_sc, float* r, long long r_nstride, float* r_stat,
                 float* z, long long z_nstride, int N, int K, int Nout, int D, int H, int W,
                 hipStream_t stream);
/* weight gradient partials: part[N*nsc][J][K] = sum_s dY[n][j][s] X[n][k][s] per voxel chunk   */
int l3u_pw_bwd_weight_nparts(int N, int S);
/* the voxel chunk of those partials (nsc = ceil(S / chunk)); a multiple of 256, at most 512: each
 * chunk is one workgroup sweep of the kernels that write them (csrc/pwconv.hip pw_chunk_ok)     */
int l3u_pw_bwd_chunk(int S);
int l3u_pw_bwd_weight(const float* dy, long long dy_nstride, const float* x, long long x_nstride,
                      float* part, int N, int J, int K, int S, hipStream_t stream);

/* fused backward of the same 1x1 conv (Y = W X, W = w[j*K + k], torch weight [J][K]) in one
 * pass over dY: dx[n][k][s] = sum_j W[j][k] dY[n][j][s] (accumulate != 0: dx += ...) and
 * part[l3u_pw_bwd_nparts(N, J, K, S)][J][K] weight-gradient partials (summed over the first
 * index they give the gradient).
 * y != NULL: dy holds dpre of the preceding InstanceNorm and dY is formed on the fly as
 * l3u_in_bwd_apply would (rec / in_part[J][N][npart][2] as for that call); dY is not stored.
 * Replaces the autograd backward of DepthwiseSeparableConv3d.pointwise (unet3d.py:18) and of the
 * shortcut conv (unet3d.py:70-73), with the InstanceNorm backward of unet3d.py:51 folded in.
 * Supported shapes: l3u_pw_bwd_supported(J, K, S) != 0: S % 4 == 0 and either J <= 32, K <= 64
 * (one workgroup per voxel chunk) or J in {64, 128}, any K (one per 64-voxel tile and 16 columns
 * of K, for the small latency-bound levels).                                                     */
int l3u_pw_bwd_supported(int J, int K, int S);
/* the same backward for conv2.pointwise (sel 1: yr = y2, rec = rec2) or the Conv1x1 shortcut
 * (sel 2: yr = r, rec = rec_r) with the block tail's backward (l3u_norm_act_bwd_apply) formed on
 * the fly from dout, out, yr and the l3u_norm_act_bwd_reduce partials tail_part[J][N][npart][3]:
 * dY = rstd*gamma*(g - mean(g) - xhat*mean(g*xhat)), g = dout*lrelu'(out), never written.
 * Supported: l3u_pw_bwd_supported(J, K, S) with J <= 32 (the 48^3 / 24^3 levels).
 * Replaces the autograd backward of norm2 / relu2 / the residual add (unet3d.py:62-63,87-91)
 * fused with that of conv2.pointwise (:18) or the shortcut (:70-73).                            */
int l3u_pw_bwd_tail(const float* dout, long long dout_nstride, const float* out,
                    long long out_nstride, const float* yr, long long yr_nstride, const float* rec,
                    const double* tail_part, int npart, int sel, const float* x,
                    long long x_nstride, const float* w, float* dx, long long dx_nstride,
                    int accumulate, float* part, int N, int J, int K, int S, hipStream_t stream);
/* the same with a rank-1 dout[j] = dscale[j] * dz (dz one channel: l3u_outconv_bwd_dz)       */
int l3u_pw_bwd_tail_r1(const float* dz, long long dz_nstride, const float* dscale,
                       const float* out, long long out_nstride, const float* yr,
                       long long yr_nstride, const float* rec, const double* tail_part, int npart,
                       int sel, const float* x, long long x_nstride, const float* w, float* dx,
                       long long dx_nstride, int accumulate, float* part, int N, int J, int K,
                       int S, hipStream_t stream);
/* the same with dout = dskip + the next level's MaxPool3d backward (as l3u_norm_act_bwd_reduce_up) */
int l3u_pw_bwd_tail_up(const float* dskip, long long dskip_nstride, const float* dpool,
                       long long dpool_nstride, const unsigned char* idx, const float* out,
                       long long out_nstride, const float* yr, long long yr_nstride,
                       const float* rec, const double* tail_part, int npart, int sel,
                       const float* x, long long x_nstride, const float* w, float* dx,
                       long long dx_nstride, int accumulate, float* part, int N, int J, int K, int D,
                       int H, int W, hipStream_t stream);

int l3u_pw_bwd_nparts(int N, int J, int K, int S);
int l3u_pw_bwd(const float* dy, long long dy_nstride, const float* y, long long y_nstride,
               const float* rec, const double* in_part, int npart, const float* x,
               long long x_nstride, const float* w, float* dx, long long dx_nstride, int accumulate,
               float* part, int N, int J, int K, int S, hipStream_t stream);
/* two plain l3u_pw_bwd calls (y == NULL) of the same J, N and S in ONE launch (a ResidualBlock's
 * conv2.pointwise and Conv1x1 shortcut backwards, unet3d.py:18,70-73: both read the block tail's
 * dy2 / dr), for the shapes l3u_pw_bwd2_supported(J, S) accepts (J in {64, 128}, the 12^3 / 6^3
 * levels); each problem gets l3u_pw_bwd_nparts(N, J, K, S) partials and the results are the two
 * calls' bit for bit.                                                                            */
/* the block tail's two pointwise backwards (conv2.pointwise: sel 1, yr = y2; the Conv1x1
 * shortcut: sel 2, yr = r) of l3u_pw_bwd_tail in ONE launch, dout as l3u_pw_bwd_tail (dscale and
 * dpool NULL), l3u_pw_bwd_tail_r1 (dscale) or l3u_pw_bwd_tail_up (dpool, idx and the plane Hf x Wf);
 * a rank-1 yr (negative yrb_nstride, fp32) only for the second problem and only when J, Ka, Kb
 * <= 16; each problem's partials as l3u_pw_bwd_nparts(N, J, K, S), results bit-identical to the
 * two calls.                                                                                    */
int l3u_pw_bwd_tail_pair(const float* dout, long long dout_nstride, const float* dscale,
                         const float* dpool, long long dpool_nstride, const unsigned char* idx,
                         int Hf, int Wf, const float* out, long long out_nstride,
                         const double* tail_part, int npart, const float* yra, long long yra_nstride,
                         const float* reca, const float* xa, long long xa_nstride, const float* wa,
                         float* dxa, long long dxa_nstride, int acc_a, float* part_a, int Ka,
                         int sel_a, const float* yrb, long long yrb_nstride, const float* recb,
                         const float* xb, long long xb_nstride, const float* wb, float* dxb,
                         long long dxb_nstride, int acc_b, float* part_b, int Kb, int sel_b, int N,
                         int J, int S, hipStream_t stream);
int l3u_pw_bwd2_supported(int J, int S);
int l3u_pw_bwd2(const float* dya, long long dya_nstride, const float* xa, long long xa_nstride,
                const float* wa, float* dxa, long long dxa_nstride, int acc_a, float* part_a, int Ka,
                const float* dyb, long long dyb_nstride, const float* xb, long long xb_nstride,
                const float* wb, float* dxb, long long dxb_nstride, int acc_b, float* part_b, int Kb,
                int N, int J, int S, hipStream_t stream);

/* ---- InstanceNorm3d(affine=True, eps=1e-5) + LeakyReLU(0.01) + Dropout3d + residual --------
 * replaces nn.InstanceNorm3d / nn.LeakyReLU / nn.Dropout3d / "out + residual"
 *          (ResidualBlock.forward, unet3d.py:77-93)
 * in_finalize: merge (count, mean, M2) partials -> rec; drop_p > 0 draws the Dropout3d channel
 * mask from a counter hash of (seed, *step, layer, n, c) (graph-replay safe).               */
int l3u_in_finalize(const float* stat_part, int nsb, const float* gamma, const float* beta,
                    float drop_p, unsigned long long seed, const int* step, int layer, float* rec,
                    int N, int C, hipStream_t stream);
/* block output: out = lrelu(scale2*(y2-mean2) + shift2 + R), R = r (rec_r == NULL, nn.Identity
 * shortcut) or scale_r*(r-mean_r) + shift_r (Conv1x1 + InstanceNorm shortcut)                        */
int l3u_norm_act_nblocks(int S);
/* records come either ready (rec2 / rec_r) or are finalized in-kernel from src2 / src_r
 * (then also stored to src->rec_out); shortcut == 0 means the identity residual (R = r).       */
int l3u_norm_act_fwd(const float* y2, long long y2_nstride, const float* rec2,
                     const l3u_norm_src* src2, const float* r, long long r_nstride,
                     const float* rec_r, const l3u_norm_src* src_r, int shortcut, float* out,
                     long long out_nstride, int N, int C, int S, hipStream_t stream);
/* the same block tail fused with the MaxPool3d(kernel 2, stride 2) that follows it in the encoder
 * (DownBlock, unet3d.py:104-105): also writes pooled [N][C][D/2*H/2*W/2] (batch stride
 * pooled_nstride) and idx (argmax in the window, as l3u_maxpool2_fwd).  Needs even D, H,
 * W % 4 == 0 and 16-byte aligned activations.                                              */
int l3u_norm_act_pool_fwd(const float* y2, long long y2_nstride, const float* rec2,
                          const l3u_norm_src* src2, const float* r, long long r_nstride,
                          const float* rec_r, const l3u_norm_src* src_r, int shortcut, float* out,
                          long long out_nstride, float* pooled, long long pooled_nstride,
                          unsigned char* idx, int N, int C, int D, int H, int W,
                          hipStream_t stream);
/* backward of the block tail: part[C][N][nblocks][3] (fp64) = {sum g, sum g*xhat2, sum g*xhat_r},
 * g = dout * lrelu'(out); then dy2 / dr (dr = g for the identity shortcut)                   */
int l3u_norm_act_bwd_reduce(const float* dout, long long dout_nstride, const float* out,
                            long long out_nstride, const float* y2, long long y2_nstride,
                            const float* rec2, const float* r, long long r_nstride,
                            const float* rec_r, double* part, int N, int C, int S,
                            hipStream_t stream);
/* the same with a rank-1 dout[c] = dscale[c] * dz (dz one channel: l3u_outconv_bwd_dz)      */
int l3u_norm_act_bwd_reduce_r1(const float* dz, long long dz_nstride, const float* dscale,
                               const float* out, long long out_nstride, const float* y2,
                               long long y2_nstride, const float* rec2, const float* r,
                               long long r_nstride, const float* rec_r, double* part, int N, int C,
                               int S, hipStream_t stream);
/* the same with dout = dskip + the MaxPool3d(2) backward of the next level (DownBlock,
 * unet3d.py:104: l3u_maxpool2_bwd's expression applied on load, so the level-output gradient is
 * never stored): dpool [N][C][S/8] (batch stride dpool_nstride), idx [N][C][S/8] as written by
 * l3u_maxpool2_fwd; even D and H, W % 4 == 0.                                                 */
int l3u_norm_act_bwd_reduce_up(const float* dskip, long long dskip_nstride, const float* dpool,
                               long long dpool_nstride, const unsigned char* idx, const float* out,
                               long long out_nstride, const float* y2, long long y2_nstride,
                               const float* rec2, const float* r, long long r_nstride,
                               const float* rec_r, double* part, int N, int C, int D, int H, int W,
                               hipStream_t stream);
int l3u_norm_act_bwd_apply(const float* dout, long long dout_nstride, const float* out,
                           long long out_nstride, const float* y2, long long y2_nstride,
                           const float* rec2, const float* r, long long r_nstride,
                           const float* rec_r, const double* part, float* dy2,
                           long long dy2_nstride, float* dr, long long dr_nstride, int N, int C,
                           int S, hipStream_t stream);
/* reduce + apply as ONE launch when l3u_norm_act_nblocks(S) == 1 (one workgroup per plane: the
 * small levels); same part layout (nblocks = 1) and bit-identical results (unet3d.py:87-91)      */
int l3u_norm_act_bwd(const float* dout, long long dout_nstride, const float* out,
                     long long out_nstride, const float* y2, long long y2_nstride,
                     const float* rec2, const float* r, long long r_nstride, const float* rec_r,
                     double* part, float* dy2, long long dy2_nstride, float* dr,
                     long long dr_nstride, int N, int C, int S, hipStream_t stream);
/* the same with dout = dskip + the next level's MaxPool3d backward of dpool (l3u_maxpool2_bwd
 * folded in: no level-output gradient tensor, one launch fewer; unet3d.py:104,109), for planes of
 * <= 2048 voxels with even D / H and W % 4 == 0; bit-identical to l3u_maxpool2_bwd followed by
 * l3u_norm_act_bwd                                                                              */
int l3u_norm_act_bwd_up(const float* dskip, long long dskip_nstride, const float* dpool,
                        long long dpool_nstride, const unsigned char* idx, const float* out,
                        long long out_nstride, const float* y2, long long y2_nstride,
                        const float* rec2, const float* r, long long r_nstride,
                        const float* rec_r, double* part, float* dy2, long long dy2_nstride,
                        float* dr, long long dr_nstride, int N, int C, int D, int H, int W,
                        hipStream_t stream);
/* inner InstanceNorm backward: dy = rstd*gamma*(dpre - mean(dpre) - xhat*mean(dpre*xhat))     */
int l3u_in_bwd_apply(const float* dpre, long long dpre_nstride, const float* y, long long y_nstride,
                     const float* rec, const double* in_part, int npart, float* dy,
                     long long dy_nstride, int N, int C, int S, hipStream_t stream);

/* ---- MaxPool3d(2, 2) (DownBlock.pool, unet3d.py:101, forward :109) ------------------------
 * idx: uint8 [N][C][So] argmax slot (first max in (dz,dy,dx) order, as torch CPU)
 * bwd: dx = route(dy) + add (add may be NULL) — writes every input voxel                      */
int l3u_maxpool2_fwd(const float* x, long long x_nstride, float* y, long long y_nstride,
                     unsigned char* idx, int N, int C, int D, int H, int W, hipStream_t stream);
int l3u_maxpool2_bwd(const float* dy, long long dy_nstride, const unsigned char* idx,
                     const float* add, long long add_nstride, float* dx, long long dx_nstride,
                     int N, int C, int D, int H, int W, hipStream_t stream);

/* ---- ConvTranspose3d(Ci, Co, 2, 2) (UpBlock.up, unet3d.py:119, forward :127) ---------------
 * the whole forward in one launch: the [Co*8 x Ci] GEMM on MFMA with the scatter (and bias) in
 * its epilogue (x: [N][Ci][D*H*W], w: torch ConvTranspose3d weight [Ci][Co][2][2][2])        */
int l3u_convt_fwd(const float* x, long long x_nstride, const float* w, const float* bias,
                  float* out, long long out_nstride, int N, int Ci, int Co, int D, int H, int W,
                  hipStream_t stream);
/* the whole backward reading dY in place from the up-sampled gradient (no space-to-depth copy):
 * dx = the data-gradient GEMM with its X operand gathered from dy; wpart[P][Ci][Co*8] weight
 * partials and bpart[P][Co] bias partials (fp32, from the weight-gradient launch), P =
 * l3u_pw_bwd_weight_nparts(N, D*H*W) (dy: [N][Co][2D][2H][2W] with batch stride dy_nstride,
 * e.g. the lower half of the decoder's concat gradient)                                        */
int l3u_convt_bwd(const float* dy, long long dy_nstride, const float* x, long long x_nstride,
                  const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart,
                  int N, int Ci, int Co, int D, int H, int W, hipStream_t stream);
/* the same backward as ONE launch (one workgroup per 64 low-res voxels and 16 input channels,
 * split over Co*8 rows by wave): dx, wpart[P][Ci][Co*8] and bpart[P][Co] (fp32) partials with
 * P = l3u_convt_bwd_fused_nparts(...) (0: shape not offered -> use l3u_convt_bwd; offered for
 * Co in {8, 16, 32, 64}, W % 4 == 0 and D*H*W <= 8192, where it beats the three-launch form).
 * Replaces the autograd backward of UpBlock.up (unet3d.py:119).                              */
int l3u_convt_bwd_fused_nparts(int N, int Ci, int Co, int D, int H, int W);
int l3u_convt_bwd_fused(const float* dy, long long dy_nstride, const float* x, long long x_nstride,
                        const float* w, float* dx, long long dx_nstride, float* wpart, float* bpart,
                        int N, int Ci, int Co, int D, int H, int W, hipStream_t stream);
/* ---- out_conv (1x1x1, C->1, bias) + Sigmoid (unet3d.py:201-202, forward :220-221) ----------
 * fwd: p = sigmoid(b + w.h); t != NULL also emits the FocalTversky first-stage partials
 *      ftl_part[N*nblocks][3] = {sum p*t, sum p, sum t} (reduce them with l3u_ftl_reduce)
 * bwd: dz = g*p*(1-p) with g = dp, or (dp == NULL) the FocalTversky gradient of the global sums
 *      (closed form, * gscale[0] if given); dh[c] = w[c]*dz;
 *      part[N*nblocks][C+1] (fp64) = {sum dz*h[c].., sum dz}; loss != NULL (dp == NULL): also
 *      loss[0] = (1 - TI)^gamma of the sums (what l3u_ftl_loss computes; saves that launch)    */
int l3u_outconv_nblocks(int S);
int l3u_outconv_fwd(const float* h, long long h_nstride, const float* w, const float* b, float* p,
                    const float* t, float* ftl_part, int N, int C, int S, hipStream_t stream);
int l3u_outconv_bwd(const float* dp, const float* p, const float* t, const double* sums,
                    double alpha, double beta, double gamma, double smooth, const float* gscale,
                    const float* h, long long h_nstride, const float* w, float* dh,
                    long long dh_nstride, double* part, float* loss, int N, int C, int S,
                    hipStream_t stream);
/* The FocalTversky form of l3u_outconv_bwd with the loss reduction folded in: instead of the
 * global sums it takes the out_conv forward's FocalTversky partials (ftl_part[ftl_nparts][3],
 * l3u_outconv_fwd) and every workgroup reduces them itself, in l3u_ftl_reduce's order (so the
 * sums, the loss and the gradient are bit-identical to l3u_ftl_reduce + l3u_outconv_bwd): the
 * single-process training step needs no separate reduce launch (losses.py:40-54). */
int l3u_outconv_bwd_ftl(const float* p, const float* t, const float* ftl_part, int ftl_nparts,
                        double alpha, double beta, double gamma, double smooth,
                        const float* gscale, const float* h, long long h_nstride, const float* w,
                        float* dh, long long dh_nstride, double* part, float* loss, int N, int C,
                        int S, hipStream_t stream);
/* the two out_conv backward forms writing dz = d(pre-sigmoid) [N][S] (batch stride dh_nstride)
 * into dh instead of dh[c] = w[c] * dz: out_conv (unet3d.py:201) is rank-1, so the last block's
 * tail backward takes dz and w through the _r1 entry points below and the [N][C][S] output
 * gradient is never stored (same values, bit for bit).                                       */
int l3u_outconv_bwd_dz(const float* dp, const float* p, const float* t, const double* sums,
                       double alpha, double beta, double gamma, double smooth, const float* gscale,
                       const float* h, long long h_nstride, const float* w, float* dh,
                       long long dh_nstride, double* part, float* loss, int N, int C, int S,
                       hipStream_t stream);
int l3u_outconv_bwd_ftl_dz(const float* p, const float* t, const float* ftl_part, int ftl_nparts,
                           double alpha, double beta, double gamma, double smooth,
                           const float* gscale, const float* h, long long h_nstride,
                           const float* w, float* dh, long long dh_nstride, double* part,
                           float* loss, int N, int C, int S, hipStream_t stream);

/* ---- Training patches (light_unet/datasets/patch_dataset.py:114-220) -----------------------
 * One record per patch: the case volume it is cut from (device pointers, [sd][sh][sw] fp32), the
 * crop start (max(0, center - patch // 2), zero padded past the volume end), and the augmentation
 * the host drew with the reference's RNG calls: flip axis (-1 none), rotation plane (rot_a0 < rot_a1,
 * -1 none) with scipy.ndimage.rotate's matrix entries and offsets, zoom (zoomed shape zs, the
 * out -> in factor zf = (in - 1) / (out - 1), the centre-crop start zst of the fit back to the
 * patch), intensity shift, gaussian noise on / off (the float64 noise values come in `noise`,
 * [B][pz][py][px], drawn by the host). */
typedef struct l3u_aug_param {
  const float* image;
  const float* label;
  int z0, y0, x0;
  int sd, sh, sw;
  int pz, py, px;
  int flip;
  int rot_a0, rot_a1;
  double rot_c, rot_s, rot_off0, rot_off1;
  int zoom;
  int zs[3];
  int zst[3];
  double zf[3];
  int shift_on;
  float shift;
  int noise_on;
} l3u_aug_param;

/* out_img / out_lab [B][pz][py][px] fp32 (the DataLoader batch, [B, 1, pz, py, px]); tmp_* the
 * same size (the rotated patches the zoom interpolates from). */
int l3u_aug_patches(const l3u_aug_param* params, int B, int pz, int py, int px, const double* noise,
                    float* tmp_img, float* tmp_lab, float* out_img, float* out_lab,
                    hipStream_t stream);

/* ---- Lesion post-processing (light_unet/models/metrics.py:38-63,107-213;
 *      light_unet/core/inferencer.py:62-111) -------------------------------------------------
 * l3u_ccl_label: connected components of (src >= threshold) over the 6 face neighbours
 * (scipy.ndimage.label's default structure in 3 dims), numbered 1..n in the order of each
 * component's first voxel in a C-order scan (scipy's numbering); background 0.  Workspace:
 * parent[D*H*W] int32, chunk_count[l3u_ccl_nchunks(D*H*W) + 1] int32; the component count
 * lands in chunk_count[l3u_ccl_nchunks(D*H*W)].  label[D*H*W] int32.
 * l3u_ccl_stats: per component l (1-based) 12 uint64: size, sum z, sum y, sum x, min z, y, x,
 * max z, y, x, max prob as float bits (prob optional, >= 0), 0; remap (optional, int32 indexed by
 * the old label) renumbers the labels in place first (0 drops the voxel: the min_size filter).
 * l3u_ccl_pairs: inter[a * (nb + 1) + b] += voxels labelled a in label_a and b in label_b (both
 * > 0); inter zeroed by the caller. */
int l3u_ccl_nchunks(long long n);
int l3u_ccl_label(const float* src, float threshold, int* parent, int* label, int* chunk_count,
                  int D, int H, int W, hipStream_t stream);
int l3u_ccl_stats(int* label, const int* remap, const float* prob, unsigned long long* stats,
                  int ncomp, int D, int H, int W, hipStream_t stream);
int l3u_ccl_pairs(const int* label_a, const int* label_b, int nb, unsigned int* inter, long long n,
                  hipStream_t stream);
/* The batched forms (get_connected_components / match_components / calculate_lesion_metrics on a
 * [B, D, H, W] array, metrics.py:38-63,99-124): ndimage.label's default structure in 4 dims adds
 * the batch axis as a fourth face neighbour (voxel (b, z, y, x) touches (b - 1, z, y, x)), with the
 * same C-order numbering over the whole array; workspace and label sized B*D*H*W.  l3u_ccl_stats_b
 * records the array's three LEADING coordinates: (z, y, x) with lead4 = 0 (a 3-dimensional array,
 * B = 1) and (b, z, y) with lead4 = 1 (a 4-dimensional array, any B) -- the reference keeps the
 * first three of center_of_mass's coordinates whatever the rank.  l3u_ccl_label / l3u_ccl_stats
 * are the B = 1, lead4 = 0 forms. */
int l3u_ccl_label_b(const float* src, float threshold, int* parent, int* label, int* chunk_count,
                    int B, int D, int H, int W, hipStream_t stream);
int l3u_ccl_stats_b(int* label, const int* remap, const float* prob, unsigned long long* stats,
                    int ncomp, int B, int D, int H, int W, int lead4, hipStream_t stream);

/* ---- UpBlock pad / crop (light_unet/models/unet3d.py:130-138) -----------------------------
 * dst[n][c][z][y][x] = src[n][c][z-oz][y-oy][x-ox] inside src's (sd, sh, sw) box, 0 elsewhere,
 * over the whole (dd, dh, dw) dst box.  Forward: the ConvTranspose3d output padded to the skip
 * volume (F.pad with diff//2 before, the rest after), written straight into the concat buffer;
 * backward (offsets negated): the concat gradient cropped to the ConvTranspose3d output. */
int l3u_box_copy(const float* src, long long src_nstride, int sd, int sh, int sw, float* dst,
                 long long dst_nstride, int dd, int dh, int dw, int oz, int oy, int ox, int N, int C,
                 hipStream_t stream);

/* ---- FocalTverskyLoss (light_unet/models/losses.py:11-54) ----------------------------------
 * sums = {sum p*t, sum p, sum t} over ALL voxels of the batch (pred.view(-1), losses.py:40-46),
 * reduced in double; loss = (1 - TI)^gamma; bwd writes dL/dp (* gscale[0] if given) or, with
 * through_sigmoid, dL/dz = dL/dp * p(1-p).  Under data parallelism the 3 sums are all-reduced
 * between l3u_ftl_sums and l3u_ftl_loss/bwd (exact global-batch semantics).                  */
int l3u_ftl_nblocks(long long numel);
int l3u_ftl_sums(const float* p, const float* t, long long numel, float* part, double* sums,
                 hipStream_t stream);
/* second stage only (partials from l3u_outconv_fwd): sums[3] = fixed-order sum of part[nparts][3] */
int l3u_ftl_reduce(const float* part, int nparts, double* sums, hipStream_t stream);
int l3u_ftl_loss(const double* sums, double alpha, double beta, double gamma, double smooth,
                 float* loss, hipStream_t stream);
int l3u_ftl_bwd(const float* p, const float* t, long long numel, const double* sums, double alpha,
                double beta, double gamma, double smooth, const float* gscale,
                int through_sigmoid, float* g, hipStream_t stream);

/* ---- the first block's front (in_channels = 1, unet3d.py:163-167) --------------------------
 * one launch for the Conv1x1 shortcut r[c] = wr[c]*x, conv1.depthwise z1 = dw3(x) (one channel,
 * w_dw [27]) and conv1.pointwise y1[c] = w1[c]*z1, with the (count, mean, M2) partials of r and y1
 * ([N][C][l3u_front_nblocks(S)][3], the l3u_pw_fwd format) from the channel's own moments.
 * Replaces three launches of unet3d.py:70-73,16-18 for the init_conv block.  W % 4 == 0.
 * x is the caller's fp32 input; x_copy != NULL also receives x in the storage type (the bf16
 * network's backward reads its input in bf16).  y1 / r == NULL (fp32): not written; the
 * consumers take them as rank-1 operands (w1[c] * z1, w_sc[c] * x: see "Rank-1 operands").      */
int l3u_front_nblocks(int S);
int l3u_front_fwd(const float* x, long long x_nstride, const float* w_dw, const float* w1,
                  const float* wr, float* z1, float* y1, float* r, float* stat1, float* statr,
                  float* x_copy, int N, int C, int D, int H, int W, hipStream_t stream);

/* ---- grouped / dense 3x3x3 conv (stride 1, padding 1, no bias): the
 * use_depthwise_separable=False path of ResidualBlock (GroupedConv3d unet3d.py:26-34, chosen at
 * :46-47 / :57-58; nn.Conv3d unet3d.py:49 / :60, G = 1).  w: torch weight [Cout][Cin/G][3][3][3].
 * fwd: rec != NULL transforms the input on load, a = lrelu(scale*(x-mean)+shift) (the record of
 *      the preceding InstanceNorm + LeakyReLU + Dropout3d, unet3d.py:84-88); stat_part != NULL
 *      also writes the (count, mean, M2) partials [N][Cout][l3u_gconv3_nblocks(S)][3] that
 *      l3u_in_finalize / l3u_norm_src consume (the format of l3u_pw_fwd).
 * bwd_data: dx (+)= conv^T(dy); rec != NULL: the IN-fused form, dx = dpre = conv^T(dy)*k*
 *      lrelu'(pre) with pre from ep (the saved pre-IN activation) and the IN-backward partials
 *      in_part[Cin][N][l3u_gconv3_nblocks(S)][2] as l3u_dw3_bwd writes them.
 * bwd_weight: part[P][Cout][Cin/G][27], P = l3u_gconv3_wgrad_nparts(N, S); rec as in fwd.      */
int l3u_gconv3_nblocks(int S);
int l3u_gconv3_wgrad_nparts(int N, int S);
int l3u_gconv3_fwd(const float* x, long long x_nstride, const float* w, const float* rec,
                   float* y, long long y_nstride, float* stat_part, int N, int Cin, int Cout,
                   int G, int D, int H, int W, hipStream_t stream);
int l3u_gconv3_bwd_data(const float* dy, long long dy_nstride, const float* w, const float* rec,
                        const float* ep, long long ep_nstride, float* dx, long long dx_nstride,
                        int accumulate, double* in_part, int N, int Cin, int Cout, int G, int D,
                        int H, int W, hipStream_t stream);
int l3u_gconv3_bwd_weight(const float* dy, long long dy_nstride, const float* x,
                          long long x_nstride, const float* rec, float* part, int N, int Cin,
                          int Cout, int G, int D, int H, int W, hipStream_t stream);

/* ---- AdamW on the flat parameter buffer (torch.optim.AdamW, trainer.py:75-79) -------------
 * lr and step live on the device (graph-replay safe).  ONE launch: the last workgroup
 * to finish (ticket order; *ticket starts at 0 and is reset) advances *step and, when
 * counter2 != NULL, *counter2 (the model's Dropout3d stream counter, unet3d.py:66, so a
 * captured training step needs no separate counter launches)                                   */
int l3u_adamw_tick(float* p, const float* g, float* m, float* v, long long numel, const float* lr,
                   float beta1, float beta2, float eps, float weight_decay, int* step,
                   float grad_scale, int* ticket, int* counter2, hipStream_t stream);

/* ---- deterministic second-stage reduction --------------------------------------------------
 * items[nitems][8] int64 = {src_off, count, istride, tstride, len<=256, dst_off, accumulate, f64}:
 * dst[dst_off+t] (+)= sum_{i<count} src[src_off + i*istride + t*tstride], summed in fp64;
 * f64 != 0: the source is fp64 and offsets/strides count doubles from the same base.
 * src is 16-byte aligned (checked), and every item's per-lane offsets fit 32 bits:
 * (count-1)*istride + (len-1)*tstride < 2^31 (the engine checks it when it records an item). */
int l3u_reduce_segments(const float* src, const long long* items, int nitems, float* dst,
                        hipStream_t stream);
/* the same reduction fused with the AdamW update (l3u_adamw_tick's arithmetic and step /
 * counter2 / ticket protocol) of the parameters it produces, for one process (no gradient
 * exchange between the two): requires that every one of the numel parameters is the output of
 * exactly one item and that no item accumulates; g receives the reduced gradient as well.
 * ticket: L3U_ADAMW_TICKET_INTS zeroed ints (left zeroed; element 0 may be the l3u_adamw_tick
 * ticket of the same optimizer)                                                                */
#define L3U_TICKET_GROUPS 32
#define L3U_TICKET_STRIDE 32
#define L3U_ADAMW_TICKET_INTS (L3U_TICKET_STRIDE * (L3U_TICKET_GROUPS + 1))
int l3u_reduce_segments_adamw(const float* src, const long long* items, int nitems, float* g,
                              float* p, float* m, float* v, const float* lr, float beta1,
                              float beta2, float eps, float weight_decay, int* step,
                              float grad_scale, int* ticket, int* counter2, hipStream_t stream);

/* ---- whole-volume sliding-window inference (light_unet/utils.py:11-173) --------------------
 * gather: out[b] = volume[z:z+pd, y:y+ph, x:x+pw] of window b (pos[b] = {z, y, x}), zero past
 *         the volume edge (utils.py:96-113)
 * blend:  prob[v] = sum_w pred_w[v] * imp[v - pos_w] / sum_w imp[v - pos_w] over the windows
 *         covering v, in the reference's window order (z, y, x) with separate fp32 multiply and
 *         add; windows are the grid zpos x ypos x xpos, preds[(iz*ny + iy)*nx + ix][pd*ph*pw] */
int l3u_window_gather(const float* img, int D, int H, int W, const int* pos, int B, int pd, int ph,
                      int pw, float* out, hipStream_t stream);
int l3u_window_blend(const float* preds, const int* zpos, int nz, const int* ypos, int ny,
                     const int* xpos, int nx, const float* imp, int D, int H, int W, int pd, int ph,
                     int pw, float* prob, hipStream_t stream);

/* storage casts (the bf16 network's input / input gradient); n elements                      */
int l3u_cast_f32_bf16(const float* x, l3u_bf16* y, long long n, hipStream_t stream);
int l3u_cast_bf16_f32(const l3u_bf16* x, float* y, long long n, hipStream_t stream);

/* device counter += value (Dropout3d RNG stream position, advanced once per training forward) */
int l3u_counter_add(int* counter, int value, hipStream_t stream);

/* ---- bf16 twins (BASELINE config 3) --------------------------------------------------------
 * The same calls with the saved activations (forward inputs and outputs: what the backward
 * re-reads) stored as bf16; argument order and meaning are those of the fp32 entry point without
 * the suffix.  Gradients (every backward input/output gradient), weights, biases, InstanceNorm
 * records and the statistics / weight-gradient partials stay fp32 (fp64 where marked), and every
 * kernel computes in fp32 (bf16 loads widen exactly, stores round to nearest even).
 * l3u_outconv_* keep p / dp / t fp32 (the loss runs on fp32 probabilities); l3u_front_fwd reads
 * the caller's fp32 x and can write its bf16 copy (x_copy) for the backward.  l3u_maxpool2_bwd
 * has no bf16 twin: it reads no saved activation.                                          */
int l3u_dw3_fwd_bf16(const l3u_bf16* x, long long x_nstride, const float* w, const float* rec,
                     const l3u_norm_src* src, l3u_bf16* y, long long y_nstride, int N, int C, int D,
                     int H, int W, hipStream_t stream);
int l3u_dw3_bwd_bf16(const float* dz, long long dz_nstride, const l3u_bf16* x, long long x_nstride,
                     const float* w, const float* rec, float* dx, long long dx_nstride,
                     int accumulate, float* dw_part, double* in_part, int N, int C, int D, int H,
                     int W, hipStream_t stream);
int l3u_dwpw_fwd_bf16(const l3u_bf16* x, long long x_nstride, const float* w_dw, const float* rec,
                      const l3u_norm_src* src, const float* w_pw, l3u_bf16* y, long long y_nstride,
                      float* y_stat, const float* w_sc, l3u_bf16* r, long long r_nstride,
                      float* r_stat, l3u_bf16* z, long long z_nstride, int N, int K, int Nout,
                      int D, int H, int W, hipStream_t stream);
int l3u_maxpool2_fwd_bf16(const l3u_bf16* x, long long x_nstride, l3u_bf16* y, long long y_nstride,
                          unsigned char* idx, int N, int C, int D, int H, int W,
                          hipStream_t stream);
int l3u_outconv_fwd_bf16(const l3u_bf16* h, long long h_nstride, const float* w, const float* b,
                         float* p, const float* t, float* ftl_part, int N, int C, int S,
                         hipStream_t stream);
int l3u_outconv_bwd_bf16(const float* dp, const float* p, const float* t, const double* sums,
                         double alpha, double beta, double gamma, double smooth,
                         const float* gscale, const l3u_bf16* h, long long h_nstride,
                         const float* w, float* dh, long long dh_nstride, double* part, float* loss,
                         int N, int C, int S, hipStream_t stream);
int l3u_outconv_bwd_ftl_bf16(const float* p, const float* t, const float* ftl_part, int ftl_nparts,
                             double alpha, double beta, double gamma, double smooth,
                             const float* gscale, const l3u_bf16* h, long long h_nstride,
                             const float* w, float* dh, long long dh_nstride, double* part,
                             float* loss, int N, int C, int S, hipStream_t stream);
int l3u_outconv_bwd_dz_bf16(const float* dp, const float* p, const float* t, const double* sums,
                            double alpha, double beta, double gamma, double smooth,
                            const float* gscale, const l3u_bf16* h, long long h_nstride,
                            const float* w, float* dh, long long dh_nstride, double* part,
                            float* loss, int N, int C, int S, hipStream_t stream);
int l3u_outconv_bwd_ftl_dz_bf16(const float* p, const float* t, const float* ftl_part,
                                int ftl_nparts, double alpha, double beta, double gamma,
                                double smooth, const float* gscale, const l3u_bf16* h,
                                long long h_nstride, const float* w, float* dh,
                                long long dh_nstride, double* part, float* loss, int N, int C,
                                int S, hipStream_t stream);
int l3u_box_copy_bf16(const l3u_bf16* src, long long src_nstride, int sd, int sh, int sw,
                      l3u_bf16* dst, long long dst_nstride, int dd, int dh, int dw, int oz, int oy,
                      int ox, int N, int C, hipStream_t stream);
int l3u_front_fwd_bf16(const float* x, long long x_nstride, const float* w_dw, const float* w1,
                       const float* wr, l3u_bf16* z1, l3u_bf16* y1, l3u_bf16* r, float* stat1,
                       float* statr, l3u_bf16* x_copy, int N, int C, int D, int H, int W,
                       hipStream_t stream);
int l3u_norm_act_fwd_bf16(const l3u_bf16* y2, long long y2_nstride, const float* rec2,
                          const l3u_norm_src* src2, const l3u_bf16* r, long long r_nstride,
                          const float* rec_r, const l3u_norm_src* src_r, int shortcut,
                          l3u_bf16* out, long long out_nstride, int N, int C, int S,
                          hipStream_t stream);
int l3u_norm_act_pool_fwd_bf16(const l3u_bf16* y2, long long y2_nstride, const float* rec2,
                               const l3u_norm_src* src2, const l3u_bf16* r, long long r_nstride,
                               const float* rec_r, const l3u_norm_src* src_r, int shortcut,
                               l3u_bf16* out, long long out_nstride, l3u_bf16* pooled,
                               long long pooled_nstride, unsigned char* idx, int N, int C, int D,
                               int H, int W, hipStream_t stream);
int l3u_norm_act_bwd_reduce_bf16(const float* dout, long long dout_nstride, const l3u_bf16* out,
                                 long long out_nstride, const l3u_bf16* y2, long long y2_nstride,
                                 const float* rec2, const l3u_bf16* r, long long r_nstride,
                                 const float* rec_r, double* part, int N, int C, int S,
                                 hipStream_t stream);
int l3u_norm_act_bwd_reduce_up_bf16(const float* dskip, long long dskip_nstride, const float* dpool,
                                    long long dpool_nstride, const unsigned char* idx,
                                    const l3u_bf16* out, long long out_nstride, const l3u_bf16* y2,
                                    long long y2_nstride, const float* rec2, const l3u_bf16* r,
                                    long long r_nstride, const float* rec_r, double* part, int N,
                                    int C, int D, int H, int W, hipStream_t stream);
int l3u_norm_act_bwd_reduce_r1_bf16(const float* dz, long long dz_nstride, const float* dscale,
                                    const l3u_bf16* out, long long out_nstride, const l3u_bf16* y2,
                                    long long y2_nstride, const float* rec2, const l3u_bf16* r,
                                    long long r_nstride, const float* rec_r, double* part, int N,
                                    int C, int S, hipStream_t stream);
int l3u_norm_act_bwd_apply_bf16(const float* dout, long long dout_nstride, const l3u_bf16* out,
                                long long out_nstride, const l3u_bf16* y2, long long y2_nstride,
                                const float* rec2, const l3u_bf16* r, long long r_nstride,
                                const float* rec_r, const double* part, float* dy2,
                                long long dy2_nstride, float* dr, long long dr_nstride, int N,
                                int C, int S, hipStream_t stream);
int l3u_norm_act_bwd_bf16(const float* dout, long long dout_nstride, const l3u_bf16* out,
                          long long out_nstride, const l3u_bf16* y2, long long y2_nstride,
                          const float* rec2, const l3u_bf16* r, long long r_nstride,
                          const float* rec_r, double* part, float* dy2, long long dy2_nstride,
                          float* dr, long long dr_nstride, int N, int C, int S, hipStream_t stream);
int l3u_norm_act_bwd_up_bf16(const float* dskip, long long dskip_nstride, const float* dpool,
                             long long dpool_nstride, const unsigned char* idx,
                             const l3u_bf16* out, long long out_nstride, const l3u_bf16* y2,
                             long long y2_nstride, const float* rec2, const l3u_bf16* r,
                             long long r_nstride, const float* rec_r, double* part, float* dy2,
                             long long dy2_nstride, float* dr, long long dr_nstride, int N, int C,
                             int D, int H, int W, hipStream_t stream);
int l3u_in_bwd_apply_bf16(const float* dpre, long long dpre_nstride, const l3u_bf16* y,
                          long long y_nstride, const float* rec, const double* in_part, int npart,
                          float* dy, long long dy_nstride, int N, int C, int S, hipStream_t stream);
int l3u_pw_fwd_bf16(const l3u_bf16* x, long long x_nstride, const float* w, int w_layout,
                    const float* bias, l3u_bf16* y, long long y_nstride, int accumulate,
                    float* stat_part, int N, int K, int Nout, int S, hipStream_t stream);
int l3u_pw_fwd2_bf16(const l3u_bf16* xa, long long xa_nstride, const float* wa, l3u_bf16* ya,
                     long long ya_nstride, float* stat_a, const l3u_bf16* xb, long long xb_nstride,
                     const float* wb, l3u_bf16* yb, long long yb_nstride, float* stat_b, int N,
                     int K, int Nout, int S, hipStream_t stream);
int l3u_convt_fwd_bf16(const l3u_bf16* x, long long x_nstride, const float* w, const float* bias,
                       l3u_bf16* out, long long out_nstride, int N, int Ci, int Co, int D, int H,
                       int W, hipStream_t stream);
int l3u_pw_bwd_weight_bf16(const float* dy, long long dy_nstride, const l3u_bf16* x,
                           long long x_nstride, float* part, int N, int J, int K, int S,
                           hipStream_t stream);
int l3u_pw_bwd_tail_bf16(const float* dout, long long dout_nstride, const l3u_bf16* out,
                         long long out_nstride, const l3u_bf16* yr, long long yr_nstride,
                         const float* rec, const double* tail_part, int npart, int sel,
                         const l3u_bf16* x, long long x_nstride, const float* w, float* dx,
                         long long dx_nstride, int accumulate, float* part, int N, int J, int K,
                         int S, hipStream_t stream);
int l3u_pw_bwd_tail_up_bf16(const float* dskip, long long dskip_nstride, const float* dpool,
                            long long dpool_nstride, const unsigned char* idx, const l3u_bf16* out,
                            long long out_nstride, const l3u_bf16* yr, long long yr_nstride,
                            const float* rec, const double* tail_part, int npart, int sel,
                            const l3u_bf16* x, long long x_nstride, const float* w, float* dx,
                            long long dx_nstride, int accumulate, float* part, int N, int J, int K,
                            int D, int H, int W, hipStream_t stream);
int l3u_pw_bwd_tail_r1_bf16(const float* dz, long long dz_nstride, const float* dscale,
                            const l3u_bf16* out, long long out_nstride, const l3u_bf16* yr,
                            long long yr_nstride, const float* rec, const double* tail_part,
                            int npart, int sel, const l3u_bf16* x, long long x_nstride,
                            const float* w, float* dx, long long dx_nstride, int accumulate,
                            float* part, int N, int J, int K, int S, hipStream_t stream);
int l3u_pw_bwd_tail_pair_bf16(const float* dout, long long dout_nstride, const float* dscale,
                              const float* dpool, long long dpool_nstride, const unsigned char* idx,
                              int Hf, int Wf, const l3u_bf16* out, long long out_nstride,
                              const double* tail_part, int npart, const l3u_bf16* yra,
                              long long yra_nstride, const float* reca, const l3u_bf16* xa,
                              long long xa_nstride, const float* wa, float* dxa,
                              long long dxa_nstride, int acc_a, float* part_a, int Ka, int sel_a,
                              const l3u_bf16* yrb, long long yrb_nstride, const float* recb,
                              const l3u_bf16* xb, long long xb_nstride, const float* wb, float* dxb,
                              long long dxb_nstride, int acc_b, float* part_b, int Kb, int sel_b,
                              int N, int J, int S, hipStream_t stream);
int l3u_pw_bwd_bf16(const float* dy, long long dy_nstride, const l3u_bf16* y, long long y_nstride,
                    const float* rec, const double* in_part, int npart, const l3u_bf16* x,
                    long long x_nstride, const float* w, float* dx, long long dx_nstride,
                    int accumulate, float* part, int N, int J, int K, int S, hipStream_t stream);
int l3u_pw_bwd2_bf16(const float* dya, long long dya_nstride, const l3u_bf16* xa,
                     long long xa_nstride, const float* wa, float* dxa, long long dxa_nstride,
                     int acc_a, float* part_a, int Ka, const float* dyb, long long dyb_nstride,
                     const l3u_bf16* xb, long long xb_nstride, const float* wb, float* dxb,
                     long long dxb_nstride, int acc_b, float* part_b, int Kb, int N, int J, int S,
                     hipStream_t stream);
int l3u_convt_bwd_fused_bf16(const float* dy, long long dy_nstride, const l3u_bf16* x,
                             long long x_nstride, const float* w, float* dx, long long dx_nstride,
                             float* wpart, float* bpart, int N, int Ci, int Co, int D, int H, int W,
                             hipStream_t stream);
int l3u_convt_bwd_bf16(const float* dy, long long dy_nstride, const l3u_bf16* x,
                       long long x_nstride, const float* w, float* dx, long long dx_nstride,
                       float* wpart, float* bpart, int N, int Ci, int Co, int D, int H, int W,
                       hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* L3U_H */
