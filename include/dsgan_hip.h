/*
 * dsgan_hip.h -- C ABI of libdsgan_hip.so, the MI355X (gfx950) kernels of the DS-GAN
 * G+D train step.
 *
 * The reference (yglbgyx/DS-GAN) has no native code: its hot path is PyTorch modules whose
 * math runs in cuDNN/cuBLAS/ATen.  Each entry point below replaces the reference op(s) cited
 * next to it (paths relative to the reference's DSGAN/ directory).  The binding the reference
 * side would add is the ctypes table in ds-gan_amd/dsgan_hip/_lib.py.
 *
 * Conventions
 *   - All tensors are caller-owned device pointers (fp32 unless stated), NCHW activations,
 *     OIHW weights.  `*_bs` = batch stride in elements (lets a channel slice of a concat
 *     buffer be read/written in place).  No allocation happens inside the library.
 *   - Every call is asynchronous on `stream` and returns 0, or a hipError_t / -1 with a
 *     message available from dsgan_last_error_string().
 *   - Weight-gradient entry points ACCUMULATE (+=) into their outputs: the caller zeroes the
 *     flat gradient buffer once per optimizer step, exactly like autograd's accumulation.
 *   - act codes: 0 none, 1 GELU (erf), 2 ReLU, 3 LeakyReLU(slope), 4 sigmoid.
 *   - prec: 0 = exact f32 MFMA (v_mfma_f32_32x32x2_f32), 1 = 16-bit MFMA operands with fp32
 *     accumulation (v_mfma_f32_32x32x16_bf16 / _f16).
 *   - 16-bit type: every "bf16" operand or storage flag, every 16-bit weight copy and every
 *     16-bit MFMA below uses the library's HALF TYPE, set process-wide by dsgan_set_half_type:
 *     0 = bf16 (default, --precision bf16), 1 = IEEE fp16 (--precision fp16, BASELINE configs[4]).
 *     Names keep "bf16" for the default; in fp16 mode the same entry points read/write fp16.
 *     The host selects it once per precision switch (dsgan_hip.functional.set_precision); calls
 *     issued after a switch use the new type.
 */
#ifndef DSGAN_HIP_H
#define DSGAN_HIP_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

int dsgan_abi_version(void);   /* 3: every scratch-taking entry point takes the scratch size */
const char* dsgan_last_error_string(void);
/* Scratch contract.  Every entry point that takes a scratch buffer (ws / work) takes its size
 * right after it (`ws_elems`, fp32 elements).  The launcher plans the launch it is about to issue,
 * computes the scratch that plan writes and returns -1 (message in dsgan_last_error_string) if
 * the buffer is NULL or smaller -- an undersized buffer is an error code, never an out-of-bounds
 * write.  Size a buffer with the matching *_workspace query.
 * dsgan_set_plan_only(1) (thread-local, returns the previous setting): scratch-taking entry points
 * validate, plan and check, then return 0 before any HIP call -- the planners run without a GPU
 * (tests/test_planner_cpu.py).  dsgan_last_ws_need(): the scratch the last planned launch of this
 * thread needed (elements; 0 = none). */
int dsgan_set_plan_only(int on);
long dsgan_last_ws_need(void);
/* the 16-bit operand type (see Conventions): 0 bf16, 1 fp16; -1 for anything else */
int dsgan_set_half_type(int t);
int dsgan_get_half_type(void);
/* Reads and clears the HIP runtime's pending launch error (0 = none): the host calls it after a
 * failed HIP-graph capture, whose invalidation error would otherwise be reported by the next
 * eager launch's check. */
int dsgan_clear_launch_error(void);
/* Kernel-only timer (bench.py's roofline leg; no reference counterpart -- measurement plumbing):
 * while on, the pointwise GEMM launchers record a HIP event pair around the GEMM kernel launch
 * itself, not around the split-K finishing pass or split reduction the same entry point issues, so
 * the figure is the kernel's own duration as rocprofv3 reports it.  dsgan_ktimer(1) on, (0) off,
 * (-1) reset the pair count; returns the count.  dsgan_ktimer_read fills ms[] with the first
 * min(count, max) pairs' elapsed ms (synchronise first) and returns how many, or -1 when an event
 * could not be recorded or read (e.g. events recorded by a replayed HIP graph's nodes). */
int dsgan_ktimer(int on);
int dsgan_ktimer_read(float* ms, int max);

/* ---- implicit-GEMM convolution (igemm.hip) ------------------------------------------------
 * Replaces nn.Conv2d / nn.Linear / nn.ConvTranspose2d forward+backward:
 *   Block.pwconv1/2 + shortcut   models/model/MixConvNeXtML.py:218-242
 *   1x1 convs (downSkip*, OriginMLKA, MidMLKA.conv)  :85,122-157,334-419
 *   ConvTranspose2d 3x3 s2       :53,150   (fwd = dsgan_conv_dgrad, dgrad = dsgan_conv_fwd)
 *   res 3x3 head                 :459
 *   PatchGAN 4x4 s2/s1           models/networks.py:543-569
 *   VGG16 3x3 + ReLU             models/vgg.py:15-24
 * y = act(conv(xact(x), w) + bias) [+ y if accumulate]; ypre (nullable) receives the
 * pre-activation; xact (act code) is applied to x as it is loaded (the Block MLP stores only
 * the pre-GELU hidden z and both of its consumers read gelu(z) this way). */
int dsgan_conv_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y,
                   long y_bs, float* ypre, long ypre_bs, int N, int Cin, int H, int W, int Cout,
                   int KH, int KW, int stride, int pad, int Ho, int Wo, int act, float slope,
                   int accumulate, int xact, int prec, hipStream_t stream);
/* dx = conv^T(dy, w) (+bias) ; if gpre: dx *= act'(gpre) with act code gact (fuses the
 * backward of the activation that produced the conv input).  stride 2 runs as four dense
 * parity-class GEMMs (no MFMA work on the structural zeros of the strided transpose). */
int dsgan_conv_dgrad(const float* dy, long dy_bs, const float* w, const float* bias, float* dx,
                     long dx_bs, float* ypre, long ypre_bs, const float* gpre, long gpre_bs,
                     int gact, int N, int Cin, int H, int W, int Cout, int KH, int KW, int stride,
                     int pad, int Ho, int Wo, int act, float slope, int accumulate, int prec,
                     hipStream_t stream);
/* dw[Cout][Cin][KH][KW] += sum_{n,oh,ow} dy * xact(x)  (split-K partials in ws, summed in a fixed
 * order: deterministic; ws = dsgan_conv_wgrad_workspace(...) floats, NULL when that is 0) */
long dsgan_conv_wgrad_workspace(int N, int Cin, int Cout, int KH, int KW, int Ho, int Wo, int prec);
int dsgan_conv_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, int N,
                     int Cin, int H, int W, int Cout, int KH, int KW, int stride, int pad, int Ho,
                     int Wo, int xact, int prec, float* ws, long ws_elems, hipStream_t stream);

/* ---- pointwise (1x1 / Linear) GEMM fast path (pwgemm.hip): bf16 MFMA, fp32 in HBM ----------
 * mode 0 FWD  : Y[b][M][P] = act(W[M][K] . xact(X[b][K][P]) + bias) (+Y), ypre = pre-act
 * mode 1 DGRAD: DX[b][M][P] = (W[K][M]^T . DY[b][K][P]) * gact'(gpre)
 * mode 2 WGRAD: DW[M][N] += sum_{b,p} DY[b][M][p] * xact(X[b][N][p])   (K = P, nb images)
 *              split over pixels into partials in `ws` (dsgan_pw_wgrad_workspace(M, N, P, nb)
 *              floats; NULL allowed when that is 0), summed in a fixed order: deterministic.
 *              `bias` (nullable) is an OUTPUT here: bias[m] += sum_{b,p} DY[b][m][p] (the layer's
 *              bias grad, from the same staged tiles -- no separate channel-sum pass).
 * FWD / DGRAD: ws (nullable) = dsgan_pw_fd_workspace(mode, M, K, P, nb) floats lets a launch whose
 *              tiles under-fill the chip split K; the partials are added in split order by a
 *              finishing pass that applies the epilogue (deterministic).
 * dsgan_pw_supported() reports whether a shape/alignment takes this path (else use igemm). */
int dsgan_pw_supported(int mode, int M, int K, int P, long a_bs, long b_bs, const void* a,
                       const void* b);
int dsgan_pw_gemm(int mode, const float* A, long a_bs, const float* B, long b_bs, float* Y,
                  long y_bs, const float* bias, float* ypre, long ypre_bs, const float* gpre,
                  long gpre_bs, int M, int N, int K, int P, int nb, int act, int gact, int bact,
                  int accumulate, float slope, float* ws, long ws_elems, hipStream_t stream);
long dsgan_pw_wgrad_workspace(int M, int N, int P, int nb);
long dsgan_pw_fd_workspace(int mode, int M, int K, int P, int nb);
/* planner knob `key` <- val (val < 0: read only), returns the previous value (measurement tools) */
int dsgan_pw_tune(int key, int val);

/* ---- exact-fp32 pointwise GEMMs (pwf32.hip): v_mfma_f32_32x32x2_f32, same modes and argument
 * meaning as dsgan_pw_gemm (no ypre / activation-on-load); the MidMLKA 1x1 conv (fp32 by policy,
 * MixConvNeXtML.py:85,112) and every 1x1 conv in the fp32 parity mode.  WGRAD: ws =
 * dsgan_pw_f32_wgrad_workspace(M, N, P, nb) floats (deterministic split reduction); `bias`
 * (nullable) is an OUTPUT there, as in dsgan_pw_gemm: bias[m] += sum_{b,p} DY[b][m][p]. */
int dsgan_pw_f32_supported(int mode, int M, int K, int P, long a_bs, long b_bs, const void* a, const void* b);
long dsgan_pw_f32_wgrad_workspace(int M, int N, int P, int nb);
int dsgan_pw_gemm_f32(int mode, const float* A, long a_bs, const float* B, long b_bs, float* Y, long y_bs,
                      const float* bias, const float* gpre, long gpre_bs, int M, int N, int K, int P, int nb, int act,
                      int gact, int accumulate, float slope, float* ws, long ws_elems, hipStream_t stream);

/* Weight-grad with bf16 operand(s) (pwgemm.hip): DW[M][N] += sum_{b,p} A[b][M][p] * B[b][N][p];
 * a_bf16 / b_bf16 select bf16 storage (h, gelu(z), dz of the MLP blocks).  P % 32 == 0.
 * db (nullable): db[m] += sum_{b,p} A[b][m][p], the bias grad (of the bf16 values when A is bf16).
 * ws: dsgan_pw_wgrad_workspace(M, N, P, nb) floats (deterministic split reduction). */
int dsgan_pw_wgrad_mixed(const void* A, long a_bs, int a_bf16, const void* B, long b_bs, int b_bf16,
                         float* dw, float* db, int M, int N, int P, int nb, float* ws, long ws_elems,
                         hipStream_t stream);
/* forward with bf16 activations in and/or out (unfused ConvNeXt MLP blocks c4/c5/uc1/uc2,
 * MixConvNeXtML.py:221-240): Y (+)= act(W X + bias), X/Y fp32 or bf16; ypre (nullable) = fp32
 * pre-activation, or with ypre_grad_bf16 the bf16 act'(pre) the backward multiplies by */
int dsgan_pw_fwd_io(const void* W, int w_bf16, const void* X, long x_bs, int x_bf16, void* Y, long y_bs, int y_bf16,
                    const void* ypre, long ypre_bs, int ypre_grad_bf16, const float* bias, int M, int K, int P, int nb,
                    int act, int accumulate, float slope, hipStream_t stream);
/* same, with the split-K scratch of dsgan_pw_fd_workspace(0, M, K, P, nb) (NULL: never split) */
int dsgan_pw_fwd_io_ws(const void* W, int w_bf16, const void* X, long x_bs, int x_bf16, void* Y, long y_bs, int y_bf16,
                       const void* ypre, long ypre_bs, int ypre_grad_bf16, const float* bias, int M, int K, int P,
                       int nb, int act, int accumulate, float slope, float* ws, long ws_elems, hipStream_t stream);
/* DX (+)= (W^T DY) (* GP): DY fp32 or bf16, DX fp32 or bf16, GP (nullable) the bf16 act'(pre) of
 * dsgan_pw_fwd_io.  Unfused-block pwconv2 / pwconv1 data-grads. */
int dsgan_pw_dgrad_io(const void* W, int w_bf16, const void* DY, long dy_bs, int dy_bf16, void* DX, long dx_bs,
                      int dx_bf16, const void* GP, long gp_bs, int M, int K, int P, int nb, int accumulate,
                      hipStream_t stream);
/* same, with the split-K scratch of dsgan_pw_fd_workspace(1, M, K, P, nb) (NULL: never split) */
int dsgan_pw_dgrad_io_ws(const void* W, int w_bf16, const void* DY, long dy_bs, int dy_bf16, void* DX, long dx_bs,
                         int dx_bf16, const void* GP, long gp_bs, int M, int K, int P, int nb, int accumulate,
                         float* ws, long ws_elems, hipStream_t stream);

/* ---- fused ConvNeXt MLP (mlp.hip), replaces Block.pwconv1 -> GELU -> pwconv2 -------------------
 * DSGAN/models/model/MixConvNeXtML.py:221-223,236-240 (nn.Linear(C,4C) + GELU + nn.Linear(4C,P) on
 * the NHWC permute of the InstanceNorm output).  bf16 MFMA, fp32 accumulation, hidden kept on chip.
 * dsgan_mlp_supported: 0 if (C, P, HW) has no fused kernel, else the backward pixel tile BN
 *   (the bsum partials buffer has nb*HW/BN rows of 4C floats).
 * dsgan_mlp_fwd: out[b][p][n] (+)= b2[p] + sum_m w2[p][m] gelu(b1[m] + sum_c w1[m][c] h[b][c][n]);
 *   w1 [4C][C], w2 [P][4C] bf16 copies of the Linear weights.
 * dsgan_mlp_bwd: recomputes z, writes dh (fp32), gelu(z) and dz (bf16 [nb][4C][HW]), and per-tile
 *   row sums of dz (bsum) for the pwconv1 bias grad (reduce with dsgan_colsum).
 * h is fp32, or bf16 when h_bf16 (dsgan_instnorm_fwd_bf16's output: the kernels round h to bf16
 *   on load either way, so the two forms give identical results). */
int dsgan_mlp_supported(int C, int P, int HW);
int dsgan_mlp_fwd(const void* h, long h_bs, int h_bf16, const void* w1, const float* b1, const void* w2,
                  const float* b2, float* out, long out_bs, int nb, int C, int P, int HW,
                  int accumulate, hipStream_t stream);
int dsgan_mlp_bwd(const void* h, long h_bs, int h_bf16, const float* dy, long dy_bs, const void* w1,
                  const float* b1, const void* w2, float* dh, long dh_bs, void* g_out, void* dz_out,
                  float* bsum, int nb, int C, int P, int HW, hipStream_t stream);
/* bsum may be NULL (the b1 grad then comes from dsgan_pw_wgrad_mixed's db on dz).
 * dsgan_mlp_bwd with g_out = dz_out = bsum = NULL writes dh only; the weight-grads then come from
 * dsgan_mlp_wgrad: dw1 [4C][C] += dz h^T, dw2 [P][4C] += dy gelu(z)^T, db1 [4C] += sum dz, with z and
 * dz recomputed per (hidden chunk, pixel split) workgroup so neither reaches HBM.  ws:
 * dsgan_mlp_wgrad_workspace() floats of per-split partials, summed in a fixed order. */
long dsgan_mlp_wgrad_workspace(int C, int P, int HW, int nb);
int dsgan_mlp_wgrad(const void* h, long h_bs, int h_bf16, const float* dy, long dy_bs, const void* w1,
                    const float* b1, const void* w2, float* dw1, float* db1, float* dw2, float* ws, long ws_elems,
                    int nb, int C, int P, int HW, hipStream_t stream);
/* planner knob `key` <- val (val < 0: read only), returns the previous value (measurement tools):
 * key 0 = the C = 256 backward with g / dz out, 0 LDS-DMA weight ring, 1 register-staged, 2 the ring with
 *         precomputed addresses (default) */
int dsgan_mlp_tune(int key, int val);
/* out[c] += sum_r part[r][c], rows added in a fixed order (deterministic); part is read only. */
int dsgan_colsum(float* part, int rows, int cols, float* out, hipStream_t stream);

/* ---- deferred split reductions (split_reduce.hip) --------------------------------------------
 * Every weight-grad entry point finishes with a fixed-order split reduction dw += sum_s partials[s]
 * of its scratch.  With deferral on, those reductions are queued (scratch pointers and outputs
 * recorded) instead of launched; dsgan_split_flush issues the queue as a few multi-segment launches
 * on the stream the producers ran on (segments with overlapping outputs in separate launches, in
 * queue order) -- the same per-element order of additions as the immediate form.  The caller keeps
 * every scratch buffer and output of a queued reduction alive, and reads no such output, until the
 * flush.  Training-loop replacement for the reference's per-layer autograd weight-grad sums
 * (DSGAN/models/pix2pix_model.py:201-217, loss.backward()). */
int dsgan_split_defer(int on);        /* returns the previous setting; turning off does not flush */
int dsgan_split_pending(void);        /* reductions queued */
int dsgan_split_flush(hipStream_t stream);  /* on the producers' stream; `stream` waits for them */
/* dst (bf16) = src (fp32), round to nearest even */
int dsgan_f32_to_bf16(const float* src, void* dst, long n, hipStream_t stream);

/* ---- direct convs for <= 8 channels on one side (skinny.hip) -----------------------------------
 * dsgan_conv_small_out: out[b][m][oh][ow] (+)= bias[m] + sum_{k,kh,kw} w(m,k,kh,kw) * in(b,k,tap),
 *   M <= 8; w(m,k,kh,kw) = w[m*wm + k*wk + kh*wh + kw*ww] (element strides, may be negative).
 *   transposed=0: conv (in = x[oh*s-pad+kh][ow*s-pad+kw]); transposed=1: the data-grad/ConvTranspose
 *   gather (in = x[(oh+pad-kh)/s][(ow+pad-kw)/s] where divisible, s in {1,2}).
 *   Replaces: G head Conv2d(64,3,3) (DSGAN/models/model/MixConvNeXtML.py:459), PatchGAN last Conv2d
 *   (DSGAN/models/networks.py:567), data-grads into 3/6-channel tensors (VGG conv1_1
 *   DSGAN/models/vgg.py:17, PatchGAN conv 0 networks.py:543) -- torch.nn.Conv2d forward/backward.
 * dsgan_conv_wgrad_small: dw[Cout][Cin][KH][KW] += conv weight-grad, Cout <= 8 or Cin <= 8,
 *   KH*KW in {1, 9, 16}; per-pixel-chunk partials in ws (dsgan_conv_wgrad_small_workspace floats,
 *   NULL when that is 0) summed in a fixed order: deterministic. */
int dsgan_conv_small_out(const float* x, long x_bs, const float* w, long wm, long wk, long wh, long ww,
                         const float* bias, float* y, long y_bs, int nb, int K, int M, int Hin, int Win,
                         int Ho, int Wo, int KH, int KW, int stride, int pad, int transposed,
                         int accumulate, hipStream_t stream);
/* dsgan_conv_small_in: y (+)= act(bias + conv) with K*KH*KW <= 36 input taps and any M (exact
 *   fp32, thread per output pixel); transposed=1 is the stride-1 data-grad gather.  Replaces:
 *   VGG16 conv1_1 forward (DSGAN/models/vgg.py:17) and the G head data-grad 3 -> 64
 *   (DSGAN/models/model/MixConvNeXtML.py:459, backward of the final nn.Conv2d(64, 3, 3, 1, 1)). */
int dsgan_conv_small_in(const float* x, long x_bs, const float* w, long wm, long wk, long wh, long ww,
                        const float* bias, float* y, long y_bs, int nb, int K, int M, int Hin, int Win,
                        int Ho, int Wo, int KH, int KW, int stride, int pad, int transposed, int act,
                        float slope, int accumulate, hipStream_t stream);
long dsgan_conv_wgrad_small_workspace(int N, int Cin, int Cout, int KH, int KW, int Ho, int Wo);
int dsgan_conv_wgrad_small(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, int N,
                           int Cin, int H, int W, int Cout, int KH, int KW, int stride, int pad, int Ho,
                           int Wo, float* ws, long ws_elems, hipStream_t stream);

/* ---- PatchGAN head (pglast.hip, exact fp32) --------------------------------------------------
 * NLayerDiscriminator's last layer Conv2d(ndf * 8, 1, 4, stride 1, pad 1) -> raw logits
 * (DSGAN/models/networks.py:567-568): x [N][K][H][W] -> y [N][1][H-1][W-1], w [1][K][4][4].
 * dsgan_pglast_supported(K, H, W): a channel chunk of the planes stages in 40 KB of LDS.
 *   fwd  : y (+)= bias + conv (bias nullable); per-chunk partials in ws (dsgan_pglast_workspace);
 *   wgrad: dw += dW, db += dB (db nullable); per-image partials in ws summed in a fixed order;
 *   dgrad: dx (+)= the input gradient. */
int dsgan_pglast_supported(int K, int H, int W);
long dsgan_pglast_workspace(int N, int K, int H, int W);
int dsgan_pglast_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int N, int K,
                     int H, int W, int accumulate, float* ws, long ws_elems, hipStream_t stream);
int dsgan_pglast_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* db, int N, int K,
                       int H, int W, float* ws, long ws_elems, hipStream_t stream);
int dsgan_pglast_dgrad(const float* dy, long dy_bs, const float* w, float* dx, long dx_bs, int N, int K, int H, int W,
                       int accumulate, hipStream_t stream);

/* ---- PatchGAN stem (pgstem.hip, exact fp32) -------------------------------------------------
 * NLayerDiscriminator layer 0: Conv2d(input_nc, ndf, 4, stride 2, pad 1) + bias + LeakyReLU(0.2, True)
 * (DSGAN/models/networks.py:543-545), one kernel per direction instead of the generic conv + the
 * LeakyReLU backward + the bias channel sum.  Cin in {3, 6}, Cout in {32, 64}, H % 8 == 0,
 * W % 64 == 0, W <= 512 (dsgan_pgstem_supported).  NCHW fp32, w OIHW [Cout][Cin][4][4].
 *   fwd  : y = lrelu(bias + conv(x)) (bias nullable), y [N][Cout][H/2][W/2];
 *   wgrad: dw += dW, db += dB (db nullable) from dy (grad of y) and y (the LeakyReLU slope is
 *          taken where y <= 0); per-workgroup partials in ws (dsgan_pgstem_wgrad_workspace floats)
 *          summed in a fixed order: deterministic;
 *   dgrad: dx (+)= the input gradient from dy and y. */
int dsgan_pgstem_supported(int Cin, int Cout, int H, int W);
int dsgan_pgstem_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int N,
                     int Cin, int Cout, int H, int W, float slope, hipStream_t stream);
long dsgan_pgstem_wgrad_workspace(int N, int Cin, int Cout, int H, int W);
int dsgan_pgstem_wgrad(const float* dy, long dy_bs, const float* y, long y_bs, const float* x, long x_bs, float* dw,
                       float* db, int N, int Cin, int Cout, int H, int W, float slope, float* ws, long ws_elems,
                       hipStream_t stream);
int dsgan_pgstem_dgrad(const float* dy, long dy_bs, const float* y, long y_bs, const float* w, float* dx,
                       long dx_bs, int N, int Cin, int Cout, int H, int W, float slope, int accumulate,
                       hipStream_t stream);

/* ---- thin 3x3 / stride 1 / pad 1 convs at full resolution (thin3.hip, exact fp32) ----------
 * The G head res = nn.Conv2d(64, 3, 3, padding=1) (DSGAN/models/model/MixConvNeXtML.py:459, applied
 * at :492): forward, weight-grad and data-grad.  M (the small side) 1..4, H % 4 == 0, W % 256 == 0,
 * 16-byte aligned planes (dsgan_thin3_supported).  w / dw are [M][K][3][3].
 *   fwd  : y[nb][M][H][W] (+)= bias + conv(x[nb][K][H][W]);
 *   wgrad: dw += sum over pixels (dy [nb][M][H][W], x [nb][K][H][W]); per-split partials in ws
 *          (dsgan_thin3_wgrad_workspace floats) summed in a fixed order: deterministic;
 *   dgrad: dx[nb][K][H][W] (+)= data-grad from dy [nb][M][H][W]. */
int dsgan_thin3_supported(int M, int H, int W, long bs_small, long bs_big);
int dsgan_thin3_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int nb, int K,
                    int M, int H, int W, int accumulate, hipStream_t stream);
long dsgan_thin3_wgrad_workspace(int nb, int K, int M, int H, int W);
int dsgan_thin3_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* ws, long ws_elems,
                      int nb, int K, int M, int H, int W, hipStream_t stream);
int dsgan_thin3_dgrad(const float* dy, long dy_bs, const float* w, float* dx, long dx_bs, int nb, int K, int M, int H,
                      int W, int accumulate, hipStream_t stream);

/* ---- tap-major implicit-GEMM conv for channel counts % 32 == 0 (tconv.hip, bf16 MFMA) -------
 * out[b][m][dst(o)] = act(sum_{tap,k} Wt[tap][m][k] * X[b][k][o*stride + (dh,dw)[tap]] + bias[m])
 *                     (* gact'(gpre) if gpre); dst(o) = (oh*os+ph, ow*os+pw) in Hdst x Wdst.
 * dsgan_conv_wtrans builds Wt from an OIHW weight: mode 0 forward, 1 stride-1 data-grad (flipped,
 * transposed), 2 one stride-2 data-grad parity class (kh0, kw0, nth, ntw). */
int dsgan_conv_wtrans(const float* W, float* Wt, int Co, int Ci, int KH, int KW, int mode, int kh0,
                      int kw0, int nth, int ntw, hipStream_t stream);
int dsgan_tconv(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                int os, int ph, int pw, int act, int gact, float slope, hipStream_t stream);
/* Split-K form: a launch whose tiles under-fill the chip (fewer than 512, e.g. the ConvTranspose
 * data-grads at 16^2 / 32^2, DSGAN/models/model/MixConvNeXtML.py:53) splits its K steps over
 * about 1024 workgroups; raw partials in ws (dsgan_tconv_workspace floats; 0 = not split, ws may
 * be NULL) are summed in a fixed order by a finishing pass that applies bias / act / gact'.
 * wt_bf16: Wt is the bf16 copy of dsgan_conv_wtrans_bf16 (same [tap][M][K] layout, K % 8 == 0). */
long dsgan_tconv_workspace(int nb, int K, int M, int Hout, int Wout, int ntaps);
int dsgan_tconv_ws(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                   const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                   int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                   int os, int ph, int pw, int act, int gact, float slope, int wt_bf16, float* ws,
                   long ws_elems, hipStream_t stream);
/* Same with X in the library's 16-bit half type (x_bs in elements) and the 16-bit Wt of
 * dsgan_conv_wtrans_bf16: the ConvTranspose2d data-grad (MixConvNeXtML.py:53,149-152) on the
 * 16-bit output grad of dsgan_instnorm_bwd_h -- the operand values the fp32 form rounds to on load. */
int dsgan_tconv_ws_xh(const void* Xh, long x_bs, const void* Wt, const float* bias, float* Y, long y_bs,
                      const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                      int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                      int os, int ph, int pw, int act, int gact, float slope, float* ws, long ws_elems,
                      hipStream_t stream);

/* ---- patch-staged implicit-GEMM conv (pconv.hip): VGG16 3x3 s1 (DSGAN/models/vgg.py:15-24) fwd
 * and data-grad, PatchGAN 4x4 s2/s1 (DSGAN/models/networks.py:543-569) fwd and s1 data-grad ------
 * y[b][m][oh][ow] (+)= act(bias[m] + sum_{c,kh,kw} Wb[tap][m][c] x[b][c][oh*s-pad+kh][ow*s-pad+kw])
 *                     (* gact'(gpre[b][m][oh][ow]) when gpre != NULL).  bf16 MFMA, Cin % 32 == 0.
 * dsgan_conv_wtrans_bf16 builds Wb from an OIHW weight: mode 0 forward, mode 1 the flipped
 * transposed kernel of the stride-1 data-grad (then call with pad' = KH-1-pad), mode 2 the
 * unflipped transposed kernel for dsgan_pconvt. */
int dsgan_pconv_supported(int K, int KH, int KW, int stride);
int dsgan_conv_wtrans_bf16(const float* W, void* Wb, int Co, int Ci, int KH, int KW, int mode,
                           hipStream_t stream);
/* n 16-bit weight copies in one launch (per 48): W[i] fp32 [Co][Ci][KH][KW] -> Wb[i], desc[5i..5i+4] =
 * (Co, Ci, KH, KW, mode): mode 0-2 as dsgan_conv_wtrans_bf16, -1 a plain cast (dsgan_f32_to_bf16).
 * The optimizer step refreshes every cached copy of the parameters it updated with one call. */
int dsgan_wtrans_multi(const void* const* W, void* const* Wb, const int* desc, int n, hipStream_t stream);
int dsgan_pconv(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                const float* gpre, long gpre_bs, int nb, int K, int M, int H, int W, int Ho, int Wo,
                int KH, int KW, int stride, int pad, int act, int gact, float slope, int accumulate,
                hipStream_t stream);
/* Split-K form of dsgan_pconv: a launch whose tiles under-fill the chip (the PatchGAN stride-1
 * layers at 31^2, DSGAN/models/networks.py:560-569) splits its 32-channel blocks over about 1024
 * workgroups; raw partials in ws (dsgan_pconv_workspace floats; 0 = not split, ws may be NULL)
 * are summed in a fixed order by a finishing pass applying bias / gact' / act / accumulate. */
long dsgan_pconv_workspace(int nb, int K, int M, int Ho, int Wo);
int dsgan_pconv_ws(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                   const float* gpre, long gpre_bs, int nb, int K, int M, int H, int W, int Ho, int Wo,
                   int KH, int KW, int stride, int pad, int act, int gact, float slope, int accumulate,
                   float* ws, long ws_elems, hipStream_t stream);

/* ---- 1x1 contractions with <= 16 channels on one side (pwsmall.hip): the 3/12-channel layers
 * at 256^2 -- c1 pwconv1/pwconv2/shortcut, OriginMLKA.to32/shortcut (MixConvNeXtML.py:122,145,
 * 218-224) and the data-grads into the 12-channel hidden.  Exact fp32 VALU (both modes):
 * Y[b][m][p] (+)= act(bias[m] + sum_k W[m*wm + k*wk] * xact(X[b][k][p])) (* gact'(G[b][m][p])). */
int dsgan_pw_small_supported(int K, int M, int P, long x_bs, long y_bs);
int dsgan_pw_small(const float* X, long x_bs, const float* W, int wm, int wk, const float* bias, float* Y,
                   long y_bs, const float* G, long g_bs, int nb, int K, int M, int P, int act, int xact,
                   int gact, int accumulate, float slope, hipStream_t stream);
/* two-input form (K + K2 <= 16): Y = act(bias + W X + W2 xact(X2)), W2 [M][K2] -- the c1 Block
 * tail shortcut(x) + pwconv2(gelu(z)) (MixConvNeXtML.py:236-242) in one pass */
int dsgan_pw_small2(const float* X, long x_bs, const float* W, int wm, int wk, const float* X2,
                    long x2_bs, const float* W2, int K2, const float* bias, float* Y, long y_bs,
                    const float* G, long g_bs, int nb, int K, int M, int P, int act, int xact, int gact,
                    int accumulate, float slope, hipStream_t stream);

/* ---- patch-staged stride-2 transposed conv (pconvt.hip): ConvTranspose2d(3, s2, p1, op1) forward
 * (MixConvNeXtML.py:53,149-152) and the data-grad of the PatchGAN Conv2d(4, s2, p1)
 * (DSGAN/models/networks.py:545-563) -- all four output parities from one staged input patch.
 * y[b][m][2i+ph][2j+pw] (+)= (bias[m] + sum Wb[kh][kw][m][c] x[b][c][i+(ph+1-kh)/2][j+(pw+1-kw)/2])
 *                          (* gact'(gpre)), bf16 MFMA, K % 32 == 0; Wb: dsgan_conv_wtrans_bf16 mode 2. */
int dsgan_pconvt_supported(int K, int KS, int stride, int pad);
int dsgan_pconvt(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                 const float* gpre, long gpre_bs, int nb, int K, int M, int Hi, int Wi, int Ho, int Wo,
                 int KS, int stride, int pad, int gact, float slope, int accumulate, hipStream_t stream);

/* ---- patch-staged conv weight-grad (wconv.hip): ConvTranspose2d 3x3/s2 weight-grads
 * (MixConvNeXtML.py:53,149-152, as the equivalent stride-2 conv) and PatchGAN 4x4 s2/s1
 * (DSGAN/models/networks.py:543-569) -- replaces the weight-grad half of torch's
 * convolution_backward for these layers.
 * dw[M][C][KH][KW] += sum_{b,oh,ow} D[b][m][oh][ow] * X[b][c][oh*s-pad+kh][ow*s-pad+kw], bf16 MFMA,
 * C % 32 == 0.  ws: dsgan_wconv_workspace() fp32 elements (per-split partials, reduced in fixed
 * order: deterministic). */
int dsgan_wconv_supported(int C, int KH, int KW, int stride);
long dsgan_wconv_workspace(int nb, int C, int M, int Ho, int Wo, int KH, int KW);
int dsgan_wconv(const float* D, long d_bs, const float* X, long x_bs, float* dw, float* ws, long ws_elems,
                int nb, int C, int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride, int pad,
                hipStream_t stream);
/* dsgan_wconv plus the conv's bias grad: db[m] += sum_{b,oh,ow} D[b][m][oh][ow] (fp32, fixed order),
 * from the staged D tiles (ws from dsgan_wconv_workspace, which includes the bias partials). */
int dsgan_wconv_db(const float* D, long d_bs, const float* X, long x_bs, float* dw, float* db, float* ws,
                   long ws_elems, int nb, int C, int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride,
                   int pad, hipStream_t stream);
/* Same with X in the library's 16-bit half type (x_bs in elements, rows 8-byte aligned), 3x3
 * stride 2 only: the ConvTranspose2d weight-grad on dsgan_instnorm_bwd_h's output (two resident
 * workgroups per CU; ws sized by dsgan_wconv_workspace, which covers both forms). */
int dsgan_wconv_xh(const float* D, long d_bs, const void* Xh, long x_bs, float* dw, float* ws, long ws_elems,
                   int nb, int C, int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride, int pad,
                   hipStream_t stream);

/* ---- depthwise conv (dwconv.hip): Block.dwconv :220, MidMLKA.X3..X9 :94-97 ----------------
 * y (+)= dwconv_KxK(x, w) + bias; flip = 1 with bias = NULL is the data-grad; accumulate adds into
 * y (data-grad of a tensor with a second consumer). */
int dsgan_dwconv_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y,
                     long y_bs, int N, int C, int H, int W, int K, int flip, int accumulate,
                     hipStream_t stream);
/* dw += sum dy*x (KxK), db += sum dy; per-workgroup partials in ws (dsgan_dwconv_wgrad_workspace
 * floats; aligned16 = x, dy 16-byte aligned with batch strides % 4 == 0) summed in a fixed order. */
long dsgan_dwconv_wgrad_workspace(int N, int C, int H, int W, int K, int aligned16);
/* MidMLKA's chunk(4) -> X3/X5/X7/X9 depthwise convs (MixConvNeXtML.py:94-97,110-111) as ONE launch
 * per pass over the four channel quarters (q channels each, quarter i has K = 3 + 2i):
 * dsgan_dwconv_multi_fwd: y (+)= dwconv_K(x) + b_K (flip = 1 with NULL biases: the data-grad);
 * dsgan_dwconv_multi_wgrad: dw_K += sum dy*x, db_K += sum dy, deterministic slot reduction in ws
 * (dsgan_dwconv_multi_wgrad_workspace floats).  Supported: dsgan_dwconv_multi_supported != 0. */
int dsgan_dwconv_multi_supported(int H, int W, const void* x, long x_bs, const void* y, long y_bs);
int dsgan_dwconv_multi_fwd(const float* x, long x_bs, const float* w3, const float* b3, const float* w5,
                           const float* b5, const float* w7, const float* b7, const float* w9, const float* b9,
                           float* y, long y_bs, int N, int q, int H, int W, int flip, int accumulate,
                           hipStream_t stream);
long dsgan_dwconv_multi_wgrad_workspace(int N, int q, int H, int W);
int dsgan_dwconv_multi_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw3, float* db3,
                             float* dw5, float* db5, float* dw7, float* db7, float* dw9, float* db9, int N, int q,
                             int H, int W, float* ws, long ws_elems, hipStream_t stream);
int dsgan_dwconv_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw,
                       float* db, int N, int C, int H, int W, int K, float* ws, long ws_elems,
                       hipStream_t stream);

/* ---- InstanceNorm2d(affine=False, eps) fused with per-plane scale, residual and activation
 * (norm_pointwise.hip): nn.InstanceNorm2d at MixConvNeXtML.py:54,80,113-116,151,158,221,
 * 335-420 and networks.py:556,565.  y = act(IN(scale*x) + res). */
int dsgan_instnorm_fwd(const float* x, long x_bs, const float* scale, const float* res,
                       long res_bs, float* y, long y_bs, float* mean, float* rstd, int N, int C,
                       int HW, int act, float slope, float eps, hipStream_t stream);
int dsgan_instnorm_bwd(const float* dy, long dy_bs, const float* x, long x_bs, const float* scale,
                       const float* res, long res_bs, const float* mean, const float* rstd,
                       float* dx, long dx_bs, float* dres, long dres_bs, float* dscale, int N,
                       int C, int HW, int act, float slope, float eps, hipStream_t stream);
/* The same two with scratch (ws_elems fp32 elements, at least dsgan_instnorm_workspace(N, C, HW)):
 * fewer than 128 planes of >= 16K pixels (the 3-channel block at 256^2) are split over several
 * workgroups per plane, with the plane statistics summed from per-chunk partials in a fixed order.
 * Other shapes need no scratch and run the kernels above. */
long dsgan_instnorm_workspace(int N, int C, int HW);
int dsgan_instnorm_fwd_ws(const float* x, long x_bs, const float* scale, const float* res, long res_bs,
                          float* y, long y_bs, float* mean, float* rstd, int N, int C, int HW, int act,
                          float slope, float eps, float* ws, long ws_elems, hipStream_t stream);
int dsgan_instnorm_bwd_ws(const float* dy, long dy_bs, const float* x, long x_bs, const float* scale,
                          const float* res, long res_bs, const float* mean, const float* rstd,
                          float* dx, long dx_bs, float* dres, long dres_bs, float* dscale, int N,
                          int C, int HW, int act, float slope, float eps, float* ws, long ws_elems,
                          hipStream_t stream);
/* Backward with dx stored in the library's 16-bit half type (dxh, batch stride dxh_bs elements,
 * 8-byte aligned) plus dxsum[n*C + c] = sum over the plane of the fp32 dx (nullable); no scale.
 * The ConvTranspose2d that feeds each decoder InstanceNorm (upSample :61-66, OriginMLKA :150-152)
 * reads dx only as 16-bit MFMA operands (dsgan_tconv_ws_xh, dsgan_wconv_xh) and its bias grad is
 * sum_n dxsum.  HW % 4 == 0, float4-aligned planes. */
int dsgan_instnorm_bwd_h(const float* dy, long dy_bs, const float* x, long x_bs, const float* res, long res_bs,
                         const float* mean, const float* rstd, void* dxh, long dxh_bs, float* dxsum, float* dres,
                         long dres_bs, int N, int C, int HW, int act, float slope, float eps, hipStream_t stream);
/* y (bf16, round-to-nearest-even) = IN(x): Block.norm (MixConvNeXtML.py:221) whose only consumers
 * are the block's bf16-operand MLP GEMMs.  HW % 4 == 0, 16-byte aligned. */
int dsgan_instnorm_fwd_bf16(const float* x, long x_bs, void* y, long y_bs, float* mean, float* rstd, int N,
                            int C, int HW, float eps, hipStream_t stream);

/* ---- MaxPool2d(k) with int32 plane-flat argmax (bit-exact with torch's indices):
 * downSample :68-74, downSkip* :333-417, OriginMLKA :123-136, VGG pools vgg.py. */
int dsgan_maxpool_fwd(const float* x, long x_bs, float* y, long y_bs, int* idx, int N, int C,
                      int H, int W, int k, hipStream_t stream);
int dsgan_maxpool_bwd(const float* dy, long dy_bs, const int* idx, float* dx, long dx_bs, int N,
                      int C, int H, int W, int k, int accumulate, hipStream_t stream);
/* The generator's skip pyramids (MixConvNeXtML.py:328-426: R1 -> k 2/4/8/16, R2 -> 2/4/8, R3 -> 2/4)
 * from one read of the source: levels 1-4 = MaxPool2d(2), (4), (8), (16), each output dense
 * [N][C][H/k][W/k] with its int32 plane-flat argmax (the same bits as dsgan_maxpool_fwd per k).
 * The backward adds every level's output grad (NULL = none) into dx in one pass (accumulate: dx +=).
 * Needs H % 16 == 0, W % 64 == 0 (dsgan_maxpool_pyr_supported). */
int dsgan_maxpool_pyr_supported(int H, int W, int levels);
int dsgan_maxpool_pyr_fwd(const float* x, long x_bs, int levels, float* y2, int* i2, float* y4, int* i4, float* y8,
                          int* i8, float* y16, int* i16, int N, int C, int H, int W, hipStream_t stream);
int dsgan_maxpool_pyr_bwd(const float* dy2, long dy2_bs, const int* i2, const float* dy4, long dy4_bs, const int* i4,
                          const float* dy8, long dy8_bs, const int* i8, const float* dy16, long dy16_bs,
                          const int* i16, float* dx, long dx_bs, int levels, int N, int C, int H, int W,
                          int accumulate, hipStream_t stream);

/* ---- channel attention CA (MixConvNeXtML.py:5-22) --------------------------------------- */
int dsgan_plane_stats(const float* x, long x_bs, float* avg, float* mx, int* amax, int N, int C,
                      int HW, hipStream_t stream);
int dsgan_plane_stats_bwd(const float* davg, const float* dmx, const int* amax, float* dx,
                          long dx_bs, int N, int C, int HW, hipStream_t stream);
int dsgan_ca_fwd(const float* avg, const float* mx, const float* w1, const float* w2,
                 const float* prelu_a, float* att, float* hsave, int N, int C, int R,
                 hipStream_t stream);
int dsgan_ca_bwd(const float* datt, const float* att, const float* avg, const float* mx,
                 const float* hsave, const float* w1, const float* w2, const float* prelu_a,
                 float* davg, float* dmx, float* dw1, float* dw2, float* dprelu_a, int N, int C,
                 int R, float* ws, long ws_elems, hipStream_t stream);   /* ws: N*(2*R*C+1) floats (per-image partials) */

/* ---- elementwise / reductions ------------------------------------------------------------
 * add_n: the decoder skip sums MixConvNeXtML.py:482-492; copy_strided: torch.cat :66;
 * channel_sum: conv/linear bias gradients (deterministic); act_bwd: ReLU/LeakyReLU/GELU backward. */
int dsgan_add_n(const float* const* ins, const long* in_bs, int nin, float* out, long out_bs,
                int N, long E, hipStream_t stream);
int dsgan_copy_strided(const float* src, long src_bs, float* dst, long dst_bs, int N, long E,
                       hipStream_t stream);
/* dst[i][0..E) <- src[i][0..E), i < count; src / dst are HOST arrays of device pointers (packed into
 * the launch, 32 pairs per launch): the ImagePool's per-query gather and scatter
 * (DSGAN/util/image_pool.py:12-32) in one launch each instead of one copy per image */
int dsgan_copy_multi(const float* const* src, float* const* dst, int count, long E, hipStream_t stream);
int dsgan_fill(float* p, float v, long n, hipStream_t stream);
int dsgan_scale(float* p, float a, long n, hipStream_t stream);
int dsgan_act_bwd(const float* dy, const float* pre, float* dx, long n, int act, float slope,
                  int accumulate, hipStream_t stream);
/* out[c] += sum_{n,p} dy[n][c][p]; ws: N*C floats (per-plane sums, added over n in a fixed order) */
int dsgan_channel_sum(const float* dy, long dy_bs, float* out, int N, int C, int HW, float* ws,
                      long ws_elems, hipStream_t stream);

/* ---- losses (losses.hip): scalars written to device memory, upstream grads read from it ----
 * GANLoss/BCEWithLogits networks.py:143-163; L1 pix2pix_model.py:177,182-186;
 * TV :189-191; ssim MS_SSIM.py:95-150 (coef: 3*planes*(H-10)*(W-10) floats of scratch).
 * Reductions are deterministic: block partials in `part` (dsgan_loss_parts() floats; ssim:
 * dsgan_ssim_parts(planes, H, W)) summed in a fixed order by one final workgroup. */
long dsgan_loss_parts(void);
/* The step's scalar loss combination in one launch (pix2pix_model.py:141-151 loss_G, :193-199
 * loss_D): out[0] = scale * sum_i a_i * (b_i + c_i * x_i[0]), summed left to right, c_i = +-1, each
 * product / sum rounded to fp32 once like the torch scalar-op chain it replaces (<= 8 terms; x_i
 * device scalars, a/b/c host arrays).  _bwd: gx[i] = gout[0] * scale * a_i * c_i. */
int dsgan_loss_combine(const float* const* x, const float* a, const float* b, const float* c, int n, float scale,
                       float* out, hipStream_t stream);
int dsgan_loss_combine_bwd(const float* gout, const float* a, const float* c, int n, float scale, float* gx,
                           hipStream_t stream);
long dsgan_ssim_parts(int planes, int H, int W);
int dsgan_bce_logits_fwd(const float* x, long n, float target, float* out, float* part, hipStream_t stream);
int dsgan_bce_logits_bwd(const float* x, long n, float target, const float* gout, float* dx,
                         int accumulate, hipStream_t stream);
int dsgan_l1_fwd(const float* a, const float* b, long n, float* out, float* part, hipStream_t stream);
int dsgan_l1_bwd(const float* a, const float* b, long n, const float* gout, float* da,
                 int accumulate, hipStream_t stream);
/* VGG perceptual tap backward (DSGAN/models/vgg.py:30-42, pix2pix_model.py:182-186): the grad at
 * the pre-ReLU output of a tapped conv, dx = (maxpool_bwd(dpool, idx) [dpool != NULL]
 * + gout*sign(y - r)/numel) * (y > 0) -- L1 backward + the two consumers' sum + ReLU backward. */
int dsgan_vgg_tap_bwd(const float* dpool, const int* idx, const float* y, const float* r, float* dx,
                      long planes, int H, int W, const float* gout, hipStream_t stream);
int dsgan_tv_fwd(const float* y, long planes, int H, int W, float coef, float* out, float* part,
                 hipStream_t stream);
int dsgan_tv_bwd(const float* y, long planes, int H, int W, float coef, const float* gout,
                 float* dy, int accumulate, hipStream_t stream);
int dsgan_ssim_fwd(const float* real, const float* fake, float a, float b, int planes, int H,
                   int W, const float* win11, float C1, float C2, float* coef, float* out,
                   float* part, hipStream_t stream);
int dsgan_ssim_bwd(const float* real, const float* fake, float a, float b, int planes, int H,
                   int W, const float* win11, const float* coef, const float* gout, float gcoef,
                   float* dfake, int accumulate, hipStream_t stream);
/* input pipeline, DSGAN/data/aligned_dataset.py:38-86 (ToTensor, crop, Normalize(0.5,0.5), flip,
 * optional gray): src uint8 [N][H][W][3] (already cropped), flip int [N] (device), dst fp32
 * [N][3 or 1][H][W]; bit-exact with the reference's torch CPU transforms. */
int dsgan_u8_to_image(const unsigned char* src, const int* flip, float* dst, int N, int H, int W, int gray,
                      hipStream_t stream);
/* train.py per-iteration metrics (DSGAN/train.py:27-44,110-124): acc[0..2] (device float) +=
 * {skimage-SSIM, PSNR, 1} of one [C][H][W] pair in [-1,1] after the reference's uint8
 * conversion; part = 128 doubles of scratch.  No host sync. */
int dsgan_img_metrics(const float* fake, const float* real, int C, int H, int W, double* part, float* acc,
                      hipStream_t stream);
/* MS-SSIM evaluation of (a*real+b, a*fake+b), DSGAN/MS_SSIM.py:153-225 (ms_ssim, forward only;
 * the differentiable form is dsgan_ms_ssim_fwd_train + dsgan_ms_ssim_bwd below): per scale the SSIM / contrast-structure plane means, then the padded 2x2 average pool;
 * weights_host = the level weights (host array, levels <= 8).  work: dsgan_ms_ssim_workspace
 * floats, stats: 2*levels*N*C floats, out: N+1 floats (per image, then the batch mean). */
long dsgan_ms_ssim_workspace(int N, int C, int H, int W);
int dsgan_ms_ssim(const float* real, const float* fake, float a, float b, int N, int C, int H, int W,
                  const float* win11, float C1, float C2, const float* weights_host, int levels,
                  float* work, long work_elems, float* stats, float* out, hipStream_t stream);
/* MS-SSIM as a differentiable loss (C4 opt-in, --ssim_loss ms_ssim): the same value with every
 * pyramid level kept in `work` (dsgan_ms_ssim_train_workspace floats), then the backward
 * dfake (+)= d(gout[0] * out[N])/d(fake) through the per-level SSIM / contrast-structure maps,
 * the relu'd product over levels and the padded 2x2 average pools (DSGAN/MS_SSIM.py:206-225).
 * stats: 2*levels*N*C floats, written by the forward, read by the backward. */
long dsgan_ms_ssim_train_workspace(int N, int C, int H, int W, int levels);
int dsgan_ms_ssim_fwd_train(const float* real, const float* fake, float a, float b, int N, int C, int H, int W,
                            const float* win11, float C1, float C2, const float* weights_host, int levels,
                            float* work, long work_elems, float* stats, float* out, hipStream_t stream);
int dsgan_ms_ssim_bwd(const float* real, const float* fake, float a, float b, int N, int C, int H, int W,
                      const float* win11, float C1, float C2, const float* weights_host, int levels, float* work,
                      long work_elems, const float* stats, const float* gout, float* dfake, int accumulate,
                      hipStream_t stream);

/* ---- VGG16 perceptual pass in channel-blocked bf16 (vggconv.hip): DSGAN/models/vgg.py:15-42 ----
 * Layout CB16 = [n][c/16][h][w][c%16].  vconv3x3: 3x3/pad 1/stride 1 implicit GEMM on bf16 MFMA,
 * Y = [relu](conv(X, W) + bias) [* (mask > 0)], Y bf16 or fp32 (y_f32); Wt = dsgan_vconv_wtrans
 * (dgrad = 0: forward weights; dgrad = 1: flipped/transposed, the data-grad of that conv, M = Ci).
 * Supported when K % 16 == 0, M % 64 == 0, W % 32 == 0, H % 4 == 0.
 * vgg_conv1_fwd / _dgrad: conv1_1 (3 -> 64) between the NCHW fp32 image and CB16 bf16.
 * cb16_maxpool: MaxPool2d(2) fp32 -> bf16 + u8 window argmax; cb16_tap_bwd: (maxpool backward +
 * L1 backward of the tapped feature) * ReLU' -> bf16 (pix2pix_model.py:182-186). */
int dsgan_vconv_supported(int K, int M, int H, int W);
/* planner knob `key` <- val (val < 0: read only), returns the previous value (measurement tools):
 * key 0 = kernel form, 0 the LDS-DMA ring kernel where a launch fills the chip, 1 the
 * register-staged kernel everywhere */
int dsgan_vconv_tune(int key, int val);
long dsgan_vconv_wtrans_size(int Co, int Ci);
int dsgan_vconv_wtrans(const float* W, void* Wt, int Co, int Ci, int dgrad, hipStream_t stream);
int dsgan_vconv3x3(const void* X, const void* Wt, const float* bias, const void* mask, void* Y, int y_f32, int relu,
                   int N, int K, int M, int H, int W, hipStream_t stream);
int dsgan_vgg_conv1_fwd(const float* x, long x_bs, const float* w, const float* b, void* y, int N, int H, int W,
                        hipStream_t stream);
int dsgan_vgg_conv1_dgrad(const void* d, const float* w, float* dx, long dx_bs, int N, int H, int W,
                          hipStream_t stream);
int dsgan_cb16_maxpool(const float* x, void* y, void* idx, int N, int C, int H, int W, hipStream_t stream);
/* dsgan_cb16_maxpool plus out[0] = mean |x - r| over the whole feature (the perceptual L1 of that
 * tap, DSGAN/models/pix2pix_model.py:182-186) from the same read of x; r = the real image's feature
 * (same CB16 fp32 layout); part: >= dsgan_cb16_maxpool_l1_parts floats of scratch; codes (nullable):
 * one byte per element of x (bit 0 = x > 0, bit 1 = x > r, bit 2 = x < r) for dsgan_cb16_tap_bwd_codes */
long dsgan_cb16_maxpool_l1_parts(int N, int C, int H, int W);
int dsgan_cb16_maxpool_l1(const float* x, const float* r, void* y, void* idx, void* codes, float* out, float* part,
                          long part_elems, int N, int C, int H, int W, hipStream_t stream);
/* dsgan_cb16_tap_bwd of a pooled tap (dpool, idx required) from those codes instead of f and r */
int dsgan_cb16_tap_bwd_codes(const void* dpool, const void* idx, const void* codes, void* d, int N, int C, int H,
                             int W, const float* gout, hipStream_t stream);
int dsgan_cb16_tap_bwd(const void* dpool, const void* idx, const float* f, const float* r, void* d, int N, int C,
                       int H, int W, const float* gout, hipStream_t stream);

/* ---- fused Adam over a flat buffer (adam.hip): torch.optim.Adam pix2pix_model.py:122-125 -- */
/* lr, betas, eps are torch's python doubles; each scalar the update uses is formed in double and
 * rounded to fp32 once, as torch's fp32 kernels receive them */
int dsgan_adam(float* p, const float* g, float* m, float* v, long n, double lr, double beta1,
               double beta2, double eps, int step, hipStream_t stream);
/* fp16 mode (--precision fp16) dynamic loss scaling, device-resident (torch GradScaler semantics,
 * no host sync).  state = fp32[5] {scale, skip, clean steps, 1/scale of this step, applied steps}.
 * dsgan_amp_check: inf/nan scan of the flat gradient (16-byte aligned) + state update (skip the
 * step and scale *= backoff on overflow; scale *= growth after `interval` clean steps);
 * part = dsgan_amp_parts() ints of scratch.  dsgan_adam_amp: dsgan_adam on g * state[3] with the
 * step count state[4]; no-op when state[1] != 0 (pix2pix_model.py:204-217 optimizer steps). */
long dsgan_amp_parts(void);
int dsgan_amp_check(const float* grad, long n, int* part, float* state, float backoff, float growth, int interval,
                    hipStream_t stream);
int dsgan_adam_amp(float* p, const float* g, float* m, float* v, long n, double lr, double beta1, double beta2,
                   double eps, const float* state, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DSGAN_HIP_H */
