/* pggan_hip.h — C ABI of libpggan_hip.so, the gfx950 (MI355X) kernels of the
 * PGGAN G+D+R1 training step.
 *
 * The reference (yukyeongleee/pggan) has no native FFI on this path: its ops are
 * torch.nn.Conv2d / nn.Linear inside ConstrainedLayer (lib/layers.py:28-108)
 * and autograd supplies backward and the R1 double-backward
 * (lib/loss.py:125-135).  Each entry point below replaces one reference op (or a
 * fused group of them) and names the reference lines it stands in for.  A
 * maintainer binds these with ctypes.
 *
 * Conventions
 *  - every function returns 0 (PG_OK) or a negative error code; the message is
 *    available from pg_last_error();
 *  - all pointers are DEVICE pointers owned by the caller; the library never
 *    allocates; `stream` is a hipStream_t passed as void* (0 = null stream);
 *  - dtype: PG_F32 (exact-fp32 parity mode) or PG_BF16 (bf16 storage, fp32
 *    accumulation); weights/biases/gradients/optimizer state are always fp32;
 *  - activations are NHWC with an explicit channel stride `*_cs` (elements);
 *    images at the API boundary are NCHW fp32 like the reference;
 *  - kernels are stateless and re-entrant; outputs are written fully unless an
 *    ACCUM flag / "accumulates" note says the result is added;
 *  - results are deterministic: a call repeated on the same inputs and geometry gives
 *    bitwise the same outputs (no order-dependent float atomics).  Sums over workgroups
 *    go through a caller-provided `scratch` (PG_SCRATCH_BYTES, see below).
 */
#ifndef PGGAN_HIP_H
#define PGGAN_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PG_OK 0
#define PG_ERR_ARG (-1)
#define PG_ERR_HIP (-2)
#define PG_ERR_UNSUPPORTED (-3)

#define PG_F32 0
#define PG_BF16 1

const char* pg_last_error(void);
int pg_version(void);

/* Reduction scratch of the entry points that sum over workgroups (the 1x1 RGB weight and bias
 * gradients, the penalties' per-sample norms, pg_bias_grad, pg_r1_penalty, pg_gp_penalty): each
 * workgroup stores its partial sums there and the last one to finish adds them in workgroup
 * order (a fixed-order sum instead of float atomics), so results are bitwise reproducible.
 * Contract: PG_SCRATCH_BYTES of device memory, zero-filled ONCE by the caller when allocated;
 * one scratch per stream (calls on one stream may share it, calls that can run concurrently on
 * different streams may not); every call returns it to its zero state. */
#define PG_SCRATCH_BYTES (4u << 20)
size_t pg_scratch_bytes(void);

/* ---- equalized-LR 3x3 convolution (lib/layers.py:66-89, ConstrainedLayer.forward :58-63)
 * y = out_scale * post(conv3x3(pre(x), wpk) + bias)
 * wpk: packed weights from pg_conv3x3_pack with the He constant folded in.
 * The same kernel runs the forward pass, the input-gradient pass (dgrad, with
 * PG_PACK_DGRAD weights) and the R1 tangent pass (no bias, PG_CONV_MASK). */
#define PG_CONV_UPS_IN 1  /* x is H/2 x W/2; nearest x2 upsample on load (lib/utils.py:106-118) */
#define PG_CONV_BIAS 2    /* + bias[cout] (fp32, He constant folded) */
#define PG_CONV_LRELU 4   /* leaky relu(slope) on the conv result */
#define PG_CONV_MASK 8    /* multiply by lrelu'(aux) (aux at output resolution, channel stride aux_cs) */
#define PG_CONV_POOL 16   /* 2x2 pool of the activated result (avg: out_scale=0.25, sum: 1.0) */
#define PG_CONV_ACCUM 32  /* y += result */
/* PixelNorm fused into the epilogue (lib/layers.py:8-14 applied after the conv+LReLU of a
 * generator block, lib/blocks.py:128-129,138-139): y = v * rsqrt(mean_c v^2 + 1e-8) with v
 * the activated result rounded to the storage dtype; if y2 != NULL it receives the
 * per-pixel factor rsqrt(...) as fp32 [B*H*W] (for pg_pixnorm_lrelu_bwd_y).  Needs every
 * output channel in one tile: query pg_conv3x3_supported().  Not with POOL/MASK/ACCUM. */
#define PG_CONV_PIXNORM 64
/* Sign-bit masks (bf16, the H,W >= 16 kernel; query pg_conv3x3_supported).  A bit tensor
 * holds the leaky-relu sign (activation > 0) of every channel: [B][H][W][bytes], channel c
 * at byte c/8, bit c%8.  1 bit replaces a 16-bit activation wherever only its sign is read
 * again (the discriminator's conv+LReLU+pool outputs, lib/blocks.py:189-193). */
#define PG_CONV_Y2_BITS 128   /* y2 receives the sign bits of the activated output: with POOL
                                 of the pre-pool output; without POOL (16 / 32 output channels)
                                 of y itself, the lrelu' operand of the layer's later masks */
#define PG_CONV_AUX_BITS 256  /* MASK operand aux is a bit tensor (aux_cs = bytes per pixel);
                                 with POOL the mask applies before pooling; may be combined
                                 with X_BITS (input and output masks both from bits) */
#define PG_CONV_X_BITS 512    /* x is masked on load by lrelu'(xbits) at conv resolution
                                 (pg_conv3x3_fwd_ex; xb_cs = bytes per pixel) */
#define PG_CONV_GZ_BITS 1024  /* wgrad: gz is at H/2 x W/2 and the effective gradient is
                                 up2(gz) * lrelu'(gzbits) (pg_conv3x3_wgrad_ex) */
/* PixelNorm + LReLU backward fused into an input-gradient conv (bf16, H,W >= 16 kernel; query
 * pg_conv3x3_supported): with v the conv result = dL/dy of a PG_CONV_PIXNORM output y, the
 * launch writes dL/du = r * (v - y * mean_c(y * v)) * lrelu'(y), u the pre-norm activation
 * (pg_pixnorm_lrelu_bwd_y without the round trip of v through HBM).  aux = y (storage
 * dtype, aux_cs), y2 = r (fp32 [B*H*W], from the forward).  With POOL (32 output channels):
 * applied to the pooled result, y and r at the pooled resolution (the generator's input
 * gradient through an upsampling conv a, then the previous block's PixelNorm).  Not with
 * BIAS / MASK / ACCUM / PIXNORM / bit flags. */
#define PG_CONV_PNBWD 2048
/* fromRGB weight gradient in the epilogue of the input-gradient conv that produces the
 * fromRGB output's gradient gz (the discriminator's top conv a, lib/blocks.py:153-170 with
 * pggan/nets.py:255): the conv result gz is NOT stored; instead
 *   dw[n*3 + i] += s * sum_pix gz[n] * img[i],  db[n] += s * sum_pix gz[n]
 * (img fp32 NCHW [B][3][H][W], summed over workgroups in a fixed order through `scratch`).
 * Only through pg_conv3x3_rgbw; query pg_conv3x3_supported. */
#define PG_CONV_RGBW 4096
/* fromRGB input gradient in the same epilogue (the penalty's input-gradient pass and the G
 * half's, pggan/nets.py:255 backward): the conv result gz is not stored; instead
 *   gimg[b][i] = f * sum_n W[n][i] gz[n]   (fp32 NCHW, written),
 *   norms[b] += sum_pix sum_i gimg[b][i]^2 (if norms; the R1 / GP squared norms),
 *   dw[n*3 + i] += s * sum_pix gz[n] gimg[i] (if dw; the R1 tangent's fromRGB weight term,
 *                                             s = f / B: gbar = gimg / B)
 * summed over workgroups in a fixed order through `scratch`.  Only through pg_conv3x3_rgbd. */
#define PG_CONV_RGBD 8192
/* toRGB output in the epilogue of the generator's top conv b forward (with PG_CONV_PIXNORM:
 * lib/blocks.py:131-139 then toRGBBlock, lib/blocks.py:153-170, pggan/nets.py:140-156 at
 * alpha = 1): y (and y2 = the PixelNorm factor) are written as by pg_conv3x3_fwd, and
 *   img[b][k] = c * (sum_n w_rgb[k][n] y[n] + b_rgb[k])   (fp32 NCHW, y as stored in bf16)
 * so the top activation is not read back by a separate toRGB pass.  Only through
 * pg_conv3x3_rgbo. */
#define PG_CONV_RGBO 16384

typedef struct {
  int B, H, W;     /* conv output spatial size (after the optional input upsample) */
  int cin, cout;   /* channels as packed (cin: multiple of 8, <=16 or multiple of 32) */
  int x_cs, y_cs, aux_cs, y2_cs; /* channel strides (elements) of x, y, aux, y2 */
  int flags;
  float slope;     /* leaky relu slope */
  float out_scale;
  int xb_cs;       /* bytes per pixel of the X_BITS / GZ_BITS bit tensor */
} pg_conv_desc;

#define PG_PACK_FWD 0    /* wpk[cout_p][9][cin_p]   = scale * W[o][c][tap]          */
#define PG_PACK_DGRAD 1  /* wpk[cin_p16][9][cout_p] = scale * W[o][c][8 - tap]      */
size_t pg_conv3x3_packed_elems(int mode, int cout, int cin);
int pg_conv3x3_pack(int dtype, int mode, int cout, int cin, const float* w_oihw, float scale,
                    void* wpk, void* stream);
/* All conv weights of a net in one launch: for each item, fwd and dgrad packs (as
 * pg_conv3x3_pack) and bias_scaled[o] = scale * bias[o] (bias may be NULL).  `items` is a
 * DEVICE array of n pg_pack_item (built once; the pointers are stable across steps);
 * max_tiles = max over items of ceil(max(cout16, cinp(cout))/32) * ceil(max(cinp(cin), cin16)/32). */
typedef struct {
  const float* w;       /* [cout][cin][3][3] fp32 */
  const float* bias;    /* [cout] or NULL */
  void* fwd;            /* PG_PACK_FWD layout, dtype */
  void* dgrad;          /* PG_PACK_DGRAD layout, dtype */
  float* bias_scaled;   /* [cout] */
  float scale;
  int cout, cin;
  int pad_;
} pg_pack_item;
int pg_conv3x3_pack_batch(int dtype, int n, const pg_pack_item* items, int max_tiles,
                          void* stream);
/* ws: optional fp32 workspace (>= pg_conv3x3_workspace_size bytes) that enables split-K
 * over input-channel chunks for small-spatial convs (deterministic: partial slabs + a
 * reduction/epilogue kernel); NULL or too small -> single pass. */
size_t pg_conv3x3_workspace_size(const pg_conv_desc* d);
int pg_conv3x3_fwd(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                   const float* bias, const void* aux, void* y, void* y2, void* ws,
                   size_t ws_bytes, void* stream);
/* pg_conv3x3_fwd with the input-mask bit tensor of PG_CONV_X_BITS */
int pg_conv3x3_fwd_ex(int dtype, const pg_conv_desc* d, const void* x, const void* xbits,
                      const void* wpk, const float* bias, const void* aux, void* y, void* y2,
                      void* ws, size_t ws_bytes, void* stream);
/* The input-gradient conv of PG_CONV_RGBW (d->flags includes it, y is not written): x, wpk,
 * aux as pg_conv3x3_fwd; img the fromRGB layer's input image, s its He constant, dw [C*3] /
 * db [C] the fromRGB weight / bias gradients (accumulated), scratch a PG_SCRATCH_BYTES
 * reduction scratch of the stream.  Replaces pg_conv3x3_fwd + pg_from_rgb_bwd(dw, db) of the
 * final backward pass (lib/model.py:95-97 through autograd in the reference). */
int pg_conv3x3_rgbw(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                    const void* aux, const float* img, float s, float* dw, float* db,
                    void* scratch, void* stream);
/* The input-gradient conv of PG_CONV_RGBD (d->flags includes it, y not written, B <= 16): x,
 * wpk, aux as pg_conv3x3_fwd; w_rgb [C][3] the fromRGB weights, f their He constant; gimg the
 * image gradient written; norms [B] accumulated or NULL; dw [C*3] accumulated or NULL with
 * scale s; scratch a PG_SCRATCH_BYTES reduction scratch of the stream.  Replaces
 * pg_conv3x3_fwd + pg_from_rgb_bwd(gimg, norms) (+ the tangent's pg_from_rgb_bwd(dw)). */
int pg_conv3x3_rgbd(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                    const void* aux, const float* w_rgb, float f, float* gimg, float* norms,
                    float* dw, float s, void* scratch, void* stream);
/* The generator's top conv b forward with PG_CONV_RGBO (d->flags = PIXNORM | LRELU | BIAS |
 * RGBO): x, wpk, bias, y, y2 as pg_conv3x3_fwd; w_rgb [3][C] / b_rgb [3] the toRGB layer's
 * weights and bias, c its He constant, img [B][3][H][W] fp32 written.  Replaces pg_conv3x3_fwd
 * + pg_rgb_out at alpha = 1 (pggan/nets.py:140-156). */
int pg_conv3x3_rgbo(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                    const float* bias, void* y, void* y2, const float* w_rgb, const float* b_rgb,
                    float c, float* img, void* stream);
/* 1 if pg_conv3x3_fwd supports d->flags for this shape/dtype (the fused epilogues depend
 * on the tile the dispatcher picks), 0 otherwise.  ws_bytes as passed to the launch. */
int pg_conv3x3_supported(int dtype, const pg_conv_desc* d, size_t ws_bytes);
/* weight gradient, accumulates: dw[o][c][ky][kx] += scale * sum_p gz[p][o] * x[p+tap][c]
 * and, if db != NULL, the bias gradient db[o] += scale * sum_p gz[p][o] (fused: gz is read
 * once).  desc: B,H,W, cin, cout, x_cs, y_cs = gz channel stride, flags may hold
 * PG_CONV_UPS_IN.  bf16: cout and both channel strides must be multiples of 8. */
/* ws: optional fp32 workspace (>= pg_conv3x3_wgrad_workspace_size bytes).  When the pixel
 * range is split over workgroups the partial sums go to per-split slabs of ws and a
 * second kernel adds them into dw/db; NULL or too small -> fp32 atomics per split. */
size_t pg_conv3x3_wgrad_workspace_size(int dtype, const pg_conv_desc* d);
int pg_conv3x3_wgrad(int dtype, const pg_conv_desc* d, const void* x, const void* gz, float scale,
                     float* dw, float* db, void* ws, size_t ws_bytes, void* stream);
/* pg_conv3x3_wgrad with PG_CONV_GZ_BITS: gz at half resolution (channel stride y_cs),
 * gzbits at full resolution (xb_cs bytes per pixel); bf16 only */
int pg_conv3x3_wgrad_ex(int dtype, const pg_conv_desc* d, const void* x, const void* gz,
                        const void* gzbits, float scale, float* dw, float* db, void* ws,
                        size_t ws_bytes, void* stream);
/* bias gradient, accumulates: db[c] += scale * sum_p g[p][c] */
int pg_bias_grad(int dtype, int npix, int C, int cs, const void* g, float scale, float* db,
                 void* scratch, void* stream);

/* ---- PixelwiseVectorNorm (lib/layers.py:8-14) over the channel axis of NHWC */
int pg_pixnorm_fwd(int dtype, int npix, int C, int cs, const void* x, void* y, void* stream);
/* gz = PN^T(gy) * lrelu'(u), u = the PN input (a leaky-relu output) (lib/blocks.py:128-139) */
int pg_pixnorm_lrelu_bwd(int dtype, int npix, int C, int cs, const void* u, const void* gy,
                         float slope, int apply_mask, void* gz, void* stream);

/* ---- elementwise helpers (NHWC, channel stride cs) */
/* out[p] = scale * g[ups ? p/2 : p] * (y ? lrelu'(y[p]) : 1)   (avg-pool backward, lib/blocks.py:193) */
/* the same backward from the fused conv's outputs (PG_CONV_PIXNORM): y = normalised
 * activation, r = per-pixel factor (fp32 [npix]); u = y / r is never stored */
int pg_pixnorm_lrelu_bwd_y(int dtype, int npix, int C, int cs, const void* y, const float* r,
                           const void* gy, float slope, void* gz, void* stream);
int pg_unpool_mask(int dtype, int B, int H, int W, int C, int g_cs, const void* g, int y_cs,
                   const void* y, float scale, float slope, int ups, int out_cs, void* out,
                   void* stream);
/* pg_unpool_mask (bf16, C % 8 == 0) with the lrelu' operand as sign bits, uint8 [B][H][W][C / 8]
 * (PG_CONV_Y2_BITS of the pooled conv that produced it) instead of the bf16 activation y */
int pg_unpool_mask_bits(int dtype, int B, int H, int W, int C, int g_cs, const void* g,
                        const void* bits, float scale, float slope, int ups, int out_cs, void* out,
                        void* stream);
/* 2x2 average pool (lib/utils.py:120-124), input B x H x W */
int pg_avgpool2(int dtype, int B, int H, int W, int C, int x_cs, const void* x, int y_cs, void* y,
                void* stream);
/* out = a*x + b*y over n elements (fade-in blends, pggan/nets.py:155-156, 263-265) */
int pg_blend(int dtype, size_t n, float a, const void* x, float b, const void* y, void* out,
             void* stream);

/* ---- RGB layers (toRGBBlock lib/blocks.py:153-170, fromRGBBlock :271-292) */
/* G output image (NCHW fp32): img = alpha*toRGB_s(x) + (1-alpha)*up2(toRGB_{s-1}(xp));
 * xp == NULL -> img = toRGB_s(x) (stage 0).  w: [3][C] fp32 raw, b: [3], c: He constant. */
int pg_rgb_out(int dtype, int B, int R, int C, int x_cs, const void* x, const float* w,
               const float* b, float c, int Cp, int xp_cs, const void* xp, const float* wp,
               const float* bp, float cp, float alpha, float* img, void* stream);
/* backward of pg_rgb_out: writes gx (NHWC, T) and gxp; accumulates dw/db/dwp/dbp */
int pg_rgb_out_bwd(int dtype, int B, int R, int C, int x_cs, const void* x, const float* w,
                   float c, int Cp, int xp_cs, const void* xp, const float* wp, float cp,
                   float alpha, const float* gimg, void* gx, void* gxp, float* dw, float* db,
                   float* dwp, float* dbp, void* scratch, void* stream);
/* fromRGB: y = lrelu(c*(W . img_in + b)), img_in = down ? avgpool2(img) : img  (img NCHW fp32);
 * R = output resolution.  b == NULL -> no bias; mask_y != NULL -> tangent mode:
 * y = c*(W . img_in) * lrelu'(mask_y) (no activation) */
/* the toRGB input gradient fused with the PixelNorm + LReLU backward of its input y (the level's
 * PG_CONV_PIXNORM output, r its per-pixel factor fp32 [B*R*R]): gz = r (v - y mean_c(y v))
 * lrelu'(y), v = c W^T gimg (pg_rgb_out_bwd's gx then pg_pixnorm_lrelu_bwd_y, without v's round
 * trip through HBM); C 16 or 32, alpha = 1 (no fade-in branch) */
int pg_rgb_out_bwd_pn(int dtype, int B, int R, int C, int y_cs, const void* y, const float* r,
                      const float* w, float c, const float* gimg, float slope, int gz_cs, void* gz,
                      void* stream);
/* pg_rgb_out_bwd_pn with the toRGB weight / bias gradients of the same pass (dw[i][k] +=
 * c sum gimg[i] y[k], db[i] += c sum gimg[i]; scratch: the stream's PG_SCRATCH_BYTES reduction
 * scratch): y and gimg are streamed once for both (lib/blocks.py toRGB, pggan/nets.py:140-156) */
int pg_rgb_out_bwd_pn_wg(int dtype, int B, int R, int C, int y_cs, const void* y, const float* r,
                         const float* w, float c, const float* gimg, float slope, int gz_cs,
                         void* gz, float* dw, float* db, void* scratch, void* stream);
int pg_from_rgb(int dtype, int B, int R, int C, const float* img, int down, const float* w,
                const float* b, float c, float slope, const void* mask_y, int y_cs, void* y,
                void* stream);
/* backward: gimg[b][i][p] += c * sum_o gz[p(/2)][o] W[o][i] * (down ? 0.25 : 1) (if gimg);
 * dw[o][i] += c sum gz*img_in, db[o] += c sum gz (if dw/db) */
int pg_from_rgb_bwd(int dtype, int B, int R, int C, const float* img, int down, const float* w,
                    float c, int gz_cs, const void* gz, float* gimg, float* dw, float* db,
                    void* scratch, void* stream);
/* An image operand of the fromRGB layers given as a per-sample mix instead of a tensor:
 * img[b] = a[b] * x0[b] + c[b] * x1[b] (NCHW fp32; a, c: DEVICE arrays of B floats; x1 and c
 * may be NULL; a == NULL means img = x0).  The gradient-penalty passes read the interpolated
 * image eps x_real + (1 - eps) x_fake (pggan/loss.py:75) and the penalty-weighted input
 * gradient this way, so neither is materialised. */
typedef struct {
  const float* x0;
  const float* x1;
  const float* a;
  const float* c;
} pg_img_src;
/* pg_from_rgb with the image operand as a pg_img_src */
int pg_from_rgb_src(int dtype, int B, int R, int C, const pg_img_src* img, int down, const float* w,
                    const float* b, float c, float slope, const void* mask_y, int y_cs, void* y,
                    void* stream);
/* pg_from_rgb_src (bf16, C % 8 == 0, C <= 64) with the lrelu sign bits as an operand instead of
 * a bf16 activation: ybits != NULL (forward) also writes the bits of the result y > 0, uint8
 * [B][R][R][C / 8] (channel o at byte o / 8, bit o % 8); mask_bits != NULL (the R1 tangent) masks
 * with those bits where pg_from_rgb reads mask_y (16x fewer bytes: 134 MB -> 8.4 MB per launch at
 * 1024^2, 16 channels, B = 4).  At most one of the two. */
int pg_from_rgb_bits(int dtype, int B, int R, int C, const pg_img_src* img, int down,
                     const float* w, const float* b, float c, float slope, const void* mask_bits,
                     int y_cs, void* y, void* ybits, void* stream);
/* pg_from_rgb_bwd with the image operand (of the weight gradient) as a pg_img_src, and for the
 * input gradient: gimg_overwrite = 1 writes gimg instead of accumulating into it; norms !=
 * NULL: norms[b] += sum over sample b of the final gimg^2 (the penalties' per-sample squared
 * norms, fused into the pass that writes the input gradient) */
int pg_from_rgb_bwd_src(int dtype, int B, int R, int C, const pg_img_src* img, int down,
                        const float* w, float c, int gz_cs, const void* gz, float* gimg,
                        int gimg_overwrite, float* norms, float* dw, float* db, void* scratch,
                        void* stream);
/* The penalty and the tangent-pass scale from the per-sample squared norms n_b of g = dD/dx:
 * mode 0 (R1, lib/loss.py:125-135): loss_out[0] += 0.5 * sum_b n_b / B, scale_b = 1 / B;
 * mode 1 (WGAN-GP, pggan/loss.py:81-87): loss_out[0] += w * sum_b (sqrt(n_b) - 1)^2,
 * scale_b = 2 w (sqrt(n_b) - 1) / sqrt(n_b) (0 where n_b = 0).  scale: DEVICE [B].  The
 * norms are reset to 0 (ready for the next accumulating pass: no memset per step). */
int pg_penalty_scale(int mode, int B, float* norms, float w, float* loss_out, float* scale,
                     void* stream);

/* real-image fade (pggan/model.py:217-221): out = (1-a)*up2(avgpool2(x)) + a*x, NCHW fp32 */
int pg_img_fade(int B, int C, int R, const float* x, float alpha, float* out, void* stream);

/* ---- equalized linear (lib/layers.py:92-108)
 * x: [B][K] (or NHWC [B][16][C] when PG_LIN_IN_CHW: k = c*16 + hw, the reference's NCHW flatten)
 * y: [B][N] (or NHWC [B][16][N/16] when PG_LIN_OUT_CHW: n = c*16 + hw, pggan/nets.py:130) */
#define PG_LIN_BIAS 1
#define PG_LIN_LRELU 2
#define PG_LIN_MASK 4     /* multiply by lrelu'(aux), aux laid out like y */
#define PG_LIN_IN_CHW 8
#define PG_LIN_OUT_CHW 16
#define PG_LIN_F32_IN 32  /* x is fp32 regardless of dtype */
#define PG_LIN_F32_OUT 64 /* y is fp32 regardless of dtype */
typedef struct {
  int B, K, N;
  int in_cs, out_cs;  /* channel strides for the CHW-mapped sides */
  int flags;
  float scale, slope;
} pg_linear_desc;
int pg_linear_fwd(int dtype, const pg_linear_desc* d, const void* x, const float* w,
                  const float* b, const void* aux, void* y, void* stream);
/* gx[b][k] = scale * sum_n gy[b][n] W[n][k]  (* lrelu'(aux[b][k]) if PG_LIN_MASK); flags
 * IN_CHW/F32_IN describe gx, OUT_CHW/F32_OUT describe gy */
int pg_linear_dgrad(int dtype, const pg_linear_desc* d, const void* gy, const float* w,
                    const void* aux, void* gx, void* stream);
/* bf16 split-reduction forms of the two passes above (deterministic: fp32 partials of
 * weight slices in ws, then a small epilogue kernel); pass 0 = fwd, 1 = dgrad.  A NULL or
 * too small ws (or the fp32 mode) falls back to pg_linear_fwd / pg_linear_dgrad. */
size_t pg_linear_workspace_size(int dtype, const pg_linear_desc* d, int pass);
int pg_linear_fwd_ws(int dtype, const pg_linear_desc* d, const void* x, const float* w,
                     const float* b, const void* aux, void* y, void* ws, size_t ws_bytes,
                     void* stream);
int pg_linear_dgrad_ws(int dtype, const pg_linear_desc* d, const void* gy, const float* w,
                       const void* aux, void* gx, void* ws, size_t ws_bytes, void* stream);
/* accumulates dw[n][k] += scale sum_b gy[b][n] x[b][k]; db[n] += scale sum_b gy[b][n] */
int pg_linear_wgrad(int dtype, const pg_linear_desc* d, const void* x, const void* gy, float* dw,
                    float* db, void* stream);

/* ---- minibatch stddev (lib/blocks.py:204-233), x: [B][HW][C] (cs x_cs) -> y: [B][HW][y_cs]
 * (channel C = group stddev, channels C+1..y_cs-1 = 0) */
int pg_mbstd_fwd(int dtype, int B, int HW, int C, int x_cs, const void* x, int y_cs, void* y,
                 void* stream);
/* gx = gy[:, :C] + d mbstd/dx ^T gy[:, C] */
int pg_mbstd_bwd(int dtype, int B, int HW, int C, int x_cs, const void* x, int y_cs,
                 const void* gy, void* gx, void* stream);
/* R1 second-order pieces at mbstd: tangent output tout = [a, sdot, 0..] and the injection
 * inj = d/dx <a, J^T gy> (added into the second backward), a = tangent at the input */
int pg_mbstd_r1(int dtype, int B, int HW, int C, int x_cs, const void* x, const void* a,
                int y_cs, const void* gy, void* tout, void* inj, void* stream);

/* ---- losses (lib/loss.py:119-135, pggan/loss.py:5-27); all fp32, device-resident scalars
 * logits [B]: loss = mean softplus(target ? -l : l); u = dloss/dl (scaled by w);
 * h = d u / d l (for the R1 double-backward).  loss_out[0] += w * loss. */
int pg_bce_loss(int B, const float* logits, int target, float w, float* loss_out, float* u,
                float* h, void* stream);
/* WGAN-GP mode drift term (pggan/loss.py:94-100 get_drift_loss): loss_out[0] += w * sum_b l_b^2
 * and u_b += 2 w l_b (u: the logit gradient of the real-image BCE, accumulated) */
int pg_drift_loss(int B, const float* logits, float w, float* loss_out, float* u, void* stream);
/* R1 = 0.5 * mean_b sum g^2 accumulated into r1_out[0]; gbar = g / B  (g: [n] fp32, B samples) */
int pg_r1_penalty(int B, size_t n, const float* g, float* r1_out, float* gbar, void* scratch,
                  void* stream);
/* WGAN-GP optional mode (pggan/loss.py:54-92): interp = eps*xr + (1-eps)*xf (per-sample eps) */
int pg_gp_interp(int B, size_t per, const float* xr, const float* xf, const float* eps,
                 float* out, void* stream);
/* gp = w * sum_b (||g_b|| - 1)^2 -> gp_out[0] (accumulate); gbar_b = w*2*(||g_b||-1)/||g_b|| g_b;
 * norms[B] workspace */
int pg_gp_penalty(int B, size_t per, const float* g, float w, float* gp_out, float* norms,
                  float* gbar, void* scratch, void* stream);

/* out = x + y*z (fp32; the R1 logit injection u + h*t, pggan/loss.py:16-27) */
int pg_mul_add(size_t n, const float* x, const float* y, const float* z, float* out, void* stream);

/* ---- Adam (torch.optim.Adam, lib/model.py:95-97; single-tensor update order) over one flat
 * fp32 range (the live parameters of a net are kept contiguous; dead ones are not passed) */
int pg_adam(size_t n, float* p, const float* g, float* m, float* v, float lr, float beta1,
            float beta2, float eps, int step, void* stream);

/* Adam with the step count in DEVICE memory, for a step captured once and replayed as a
 * hipGraph: bumps *step, then updates with the bias corrections of the new count taken from
 * `table` (DEVICE, tlen pairs {lr / (1 - beta1^t), sqrt(1 - beta2^t)} for t = 1..tlen, built
 * by pg_adam_table on the host with pg_adam's double arithmetic; counts past tlen use the last
 * pair, which pg_adam_table_len makes exact) -- the same update as pg_adam at that step. */
int pg_adam_table_len(float lr, float beta1, float beta2);
int pg_adam_table(float lr, float beta1, float beta2, int tlen, float* host_table);
int pg_adam_dev(size_t n, float* p, const float* g, float* m, float* v, float beta1, float beta2,
                float eps, const float* table, int tlen, int* step, void* stream);

/* ---- N(0,1) latents (counter-based, deterministic in (seed, offset)) */
int pg_randn(size_t n, uint64_t seed, uint64_t offset, float* out, void* stream);
/* the same draw with the offset in DEVICE memory; *offset then advances by n (graph replay) */
int pg_randn_dev(size_t n, uint64_t seed, uint64_t* offset, float* out, void* stream);
/* dtype conversion helpers */
int pg_cast(int dtype_in, int dtype_out, size_t n, const void* x, void* y, void* stream);

/* ---- training-image augmentation (SURVEY §8(f) GPU input pipeline): the transform chain
 * of lib/dataset.py:106-117 after Resize -- RandomHorizontalFlip(0.5), ColorJitter(0.2, 0.2,
 * 0.2, 0.01) in torchvision's random op order, ToTensor, Normalize(0.5, 0.5) -- on a batch of
 * decoded, resized images: src uint8 [B][H][W][3] (4-byte aligned), dst fp32 [B][3][H][W]
 * (16-byte aligned), params fp32 [B][12] = {flip (0/1), brightness, contrast, saturation,
 * hue factor, fn_idx[0..3] (0 brightness, 1 contrast, 2 saturation, 3 hue), 1 - contrast,
 * 1 - saturation, 0}.
 * Jitter arithmetic: the reference's PIL path (torchvision functional_pil: ImageEnhance
 * Brightness / Contrast / Color blends and the uint8 shift of PIL's HSV hue band) in Pillow's
 * libImaging arithmetic, uint8 after every op: byte-identical to the reference transform.
 * W % 4 == 0.  The caller provides pg_augment_workspace_bytes(B, H, W) of device workspace
 * (16-byte aligned). */
size_t pg_augment_workspace_bytes(int B, int H, int W);
int pg_augment_u8(int B, int H, int W, const void* src, const float* params, float* ws,
                  size_t ws_bytes, float* dst, void* stream);

/* ---- stream ordering between the engine's streams (weight gradients on a side stream).
 * torch's cross-stream events record with a system-scope release: every record writes back and
 * invalidates the L2 of all XCDs and the next kernel on that stream starts ~6.5 us late.  The
 * two streams are on one device, so these events release to device scope only
 * (hipEventReleaseToDevice).  `timing` != 0: a timing event that skips the system fence
 * (hipEventDisableSystemFence; a default timing event where the runtime rejects that flag), for
 * the bench's per-launch timers.  Handles are opaque. */
int pg_event_create(int timing, void** ev);
int pg_event_record(void* ev, void* stream);
int pg_stream_wait_event(void* stream, void* ev);
int pg_event_elapsed_ms(void* ev_start, void* ev_end, float* ms);
/* A non-blocking stream of the library's own; lowest_priority != 0: at the device's least
 * priority (its own hardware-queue pool, so never the queue of a normal-priority stream) */
int pg_stream_create(int lowest_priority, void** stream);
int pg_stream_destroy(void* stream);
int pg_event_destroy(void* ev);

/* ---- device memory helpers that take part in recordings: zero `bytes` at p / copy `bytes`
 * device to device, asynchronously on `stream` (the step's gradient and loss resets and its
 * input copies, so a recorded step needs no torch op) */
int pg_fill_zero(void* p, size_t bytes, void* stream);
int pg_copy(void* dst, const void* src, size_t bytes, void* stream);

/* ---- launch recorder (the training step replayed from C++; reference hot loop train.py:39-66).
 * Between pg_record_begin and pg_record_end every kernel launch, pg_event_record,
 * pg_stream_wait_event, pg_fill_zero and pg_copy this host thread issues runs as usual AND is
 * appended to a recording (function, geometry, stream, arguments by value).  pg_replay issues
 * the same sequence again on the same streams: one C++ loop instead of the Python layer that
 * produced it, and -- unlike a hipGraph -- the streams and their hardware queues are the
 * recorded ones.  The caller guarantees that every pointer the recording holds still points to
 * the same live buffers and that their contents (inputs, step counters) are meant to be
 * re-read; a recording is replayed on the thread's current device.  Handles are opaque. */
int pg_record_begin(void);
int pg_record_end(void** rec);
int pg_record_count(const void* rec);
int pg_replay(const void* rec);
void pg_record_destroy(void* rec);

/* ---- step plan: the kernel path of every 3x3 conv pass (forward, input
 * gradient, weight gradient) of one train_step at (stage, batch, dtype) -- the layer list of
 * pggan/nets.py:53-119 (G) and :164-239 (D) at scale_index = stage -- and the split-reduction
 * workspace the step needs (the max over its conv / wgrad launches).  Plans are immutable
 * after creation (thread-safe to read); the caller owns the workspace memory. */
typedef struct pg_step_plan pg_step_plan;
int pg_step_plan_create(int dtype, int n_depths, const int* depths, int stage, int batch,
                        pg_step_plan** out);
size_t pg_step_plan_workspace_size(const pg_step_plan* plan);
/* human-readable table of the plan (one line per conv layer) into buf */
int pg_step_plan_describe(const pg_step_plan* plan, char* buf, size_t len);
void pg_step_plan_destroy(pg_step_plan* plan);

#ifdef __cplusplus
}
#endif
#endif
