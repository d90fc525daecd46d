/*
 * spotter_hip.h — C-ABI of libspotter_hip.so, the MI355X (gfx950) kernels of
 * the RT-DETRv2 /detect hot path.
 *
 * The reference has no C-ABI: its hot path is the duck-typed HF interface
 * AmenitiesDetector calls (apps/spotter/src/spotter/serve.py:98-117):
 *   processor(images=PIL, return_tensors="pt")           -> sp_preprocess_u8
 *   model(**inputs) (RTDetrV2ForObjectDetection.forward) -> sp_conv2d, sp_maxpool3x3s2,
 *        sp_avgpool2x2_ceil, sp_upsample2x_nearest, sp_layernorm, sp_attention,
 *        sp_msda, sp_rowmax, sp_topk_rows, sp_gather_rows, sp_add_rows, sp_ref_init, sp_box_refine
 *   processor.post_process_object_detection(...)         -> sp_postprocess
 * (HF sources: transformers/models/rt_detr/image_processing_pil_rt_detr.py:
 * 451-462, 508-578; transformers/models/rt_detr_v2/modeling_rt_detr_v2.py:
 * 44-225, 1461-1656, 1797-1881.) spotter_amd/ (Python) implements that
 * interface on top of these entry points; INTEGRATION.md shows the binding.
 *
 * Conventions: plain device pointers (fp32 unless stated), sizes in elements,
 * `stream` is a hipStream_t (NULL = default stream). Every call is async on
 * `stream`, allocates nothing and is safe to capture in a hipGraph (except the
 * first sp_preprocess_u8 per (in, out) size, which uploads its coefficient
 * table). Return: 0 ok, >0 hipError_t, <0 argument error; the message is in
 * sp_last_error() (thread-local). No C++ exception crosses the ABI.
 */
#ifndef SPOTTER_HIP_H
#define SPOTTER_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SP_ABI_VERSION 15

enum sp_act { SP_ACT_NONE = 0, SP_ACT_RELU = 1, SP_ACT_SILU = 2, SP_ACT_GELU = 3 };
/* GEMM operand precision:
 *  SP_PREC_FP32  fp32 MFMA (v_mfma_f32_32x32x2_f32: an exact fp32 fmaf chain);
 *  SP_PREC_BF16  bf16 MFMA with fp32 accumulate (activations rounded RNE to bf16 on load,
 *                weights from Wt_bf16) — the separately reported bf16 variant;
 *  SP_PREC_F32X3 fp32 operands as 3-way bf16 splits x = hi + mid + lo (24 significand bits,
 *                exact for normal fp32), products hi·hi + hi·mid + mid·hi + hi·lo + lo·hi +
 *                mid·mid on bf16 MFMA with fp32 accumulate; the dropped terms sum to <= 2^-24
 *                of |a·b| (one fp32 rounding), so the result is fp32-accurate (checked against
 *                fp64 next to the fp32 MFMA path in tests/test_gpu_kernels.py).
 *                Weights from Wt_bf16 as three planes [3][Cout][K] (plane stride
 *                wt_plane_stride); activations are split while staging. */
enum sp_precision { SP_PREC_FP32 = 0, SP_PREC_BF16 = 1, SP_PREC_F32X3 = 2 };

/* One uint8 RGB HWC image in device memory. */
typedef struct {
  const uint8_t* data;
  int32_t height, width;
  int32_t row_stride; /* bytes between rows (>= 3*width) */
} sp_image_u8;

/*
 * Implicit-GEMM convolution / linear layer on fp32 MFMA (v_mfma_f32_32x32x2f32):
 *   out[m, n] = act( (Σ_k A[m, k] · W[n, k]) · row_scale[m % row_period] · scale[n]
 *                    + shift[n] + res1[m, n] ) + res2[m, n]
 * A is NHWC: pixel (b, y, x) starts at A + ((b*H + y)*W + x)*lda, channels [0, Cin).
 * A2 (optional) is added to A element-wise on load (same indexing, lda2).
 * W is [Cout][KH][KW][Cin] (k contiguous). m = (b*Ho + oy)*Wo + ox.
 * Output row m goes to C + (m / out_rows_per_group)*out_group_stride + (m % out_rows_per_group)*ldc
 * (out_rows_per_group = 0 means M, i.e. plain row-major with ldc).
 * res1/res2 rows use (m*ldr). Linear layers: N=1, H=1, W=rows, KH=KW=1.
 * With a workspace, launches whose tile grid cannot fill the chip split K over the
 * grid's z dimension and combine the partial sums (fixed order) before the epilogue.
 * Corresponds to nn.Conv2d + (Frozen)BatchNorm2d + activation (+ residual)
 * (RN:38-68, RN:225-231, M2:817-835) and nn.Linear (+ activation).
 */
typedef struct {
  const float* A; int64_t lda;
  const float* A2; int64_t lda2;
  int32_t N, H, W, Cin;
  int32_t KH, KW, stride, pad;
  int32_t Ho, Wo;
  const float* Wt; int32_t Cout;
  const float* scale;     /* [Cout] or NULL (1) */
  const float* shift;     /* [Cout] or NULL (0) */
  const float* row_scale; int32_t row_period; /* NULL or [row_period] */
  const float* res1; int64_t ldr1;
  int32_t act;
  const float* res2; int64_t ldr2;
  float* C; int64_t ldc;
  int32_t out_rows_per_group; int64_t out_group_stride;
  float* workspace; int64_t workspace_elems; /* optional fp32 scratch enabling split-K (small M) */
  int32_t precision;         /* sp_precision */
  const uint16_t* Wt_bf16;   /* [Cout][K] bf16 weights (SP_PREC_BF16), [3][Cout][K] (SP_PREC_F32X3) */
  int64_t wt_plane_stride;   /* elements between the hi / mid / lo planes (SP_PREC_F32X3) */
  /* Optional row LayerNorm fused into the epilogue (ABI v8): when ln_gamma is set,
   *   out[m, :] = LayerNorm(acc·row_scale·scale + shift + res1)[m, :] · ln_gamma + ln_beta   (eps ln_eps)
   * over the whole output row — the post-norm "Linear → +residual → LayerNorm" of the AIFI and decoder
   * layers (M2:395-404, 409-423, 426-429, 856-904) and enc_output (M2:1376-1381). Needs the fp32 weights
   * (precision SP_PREC_FP32), Cout a multiple of 128 up to 512, act none, no res2 / grouped rows. */
  const float* ln_gamma;
  const float* ln_beta;
  float ln_eps;
  /* ABI v10: A_bf16 (non-NULL, SP_PREC_BF16) replaces A for sp_conv2d's LDS-DMA tiles: the activations as
   * bf16 rows written by their producer (the bf16 variant's maps), staged as they are instead of rounded per
   * fragment; lda counts elements. */
  const uint16_t* A_bf16;
  /* ABI v10: bf16 activations (the bf16 variant keeps the backbone's maps in bf16). C_bf16 (non-NULL)
   * replaces C: the epilogue result is stored as bf16 (RNE) rows, ldc / out_group_stride in elements.
   * res1_bf16 / res2_bf16 (non-NULL) replace res1 / res2 (bf16 rows, ldr1 / ldr2 in elements). Not with
   * LayerNorm. */
  uint16_t* C_bf16;
  const uint16_t* res1_bf16;
  const uint16_t* res2_bf16;
  /* ABI v13: split-K arrival counters (optional, with a workspace). When set, a split-K launch combines its
   * partial sums inside the GEMM launch: each output tile's last-arriving workgroup adds the tile's partials in
   * fixed split order and applies the epilogue (the same arithmetic as the separate reduce launch, so the
   * result is bit-identical), instead of a second reduce launch. The caller zeroes the array once before first
   * use and gives each concurrently running stream its own; every launch leaves it zero. Launches whose tile
   * grid exceeds splitk_counters_len entries, or tiles without the in-launch form, use the reduce launch. */
  int32_t* splitk_counters; int64_t splitk_counters_len;
} sp_conv_desc;

/*
 * Multi-scale deformable attention v2 core + softmax + sampling-location math
 * (M2:166-225, M2:44-115, method "default"), one decoder layer.
 *   value   [B, S, ld_value] rows, head h channel c at column value_col + h*Dh + c
 *   off_aw  [B*Q, ld_off_aw]: columns [0, H*L*P*2) sampling offsets (h, l, p, xy),
 *           then [H*L*P*2, +H*L*P) attention logits (h, l*P + p)
 *   ref     [B*Q, 4] reference boxes (cx, cy, w, h) in (0, 1)
 *   out     [B*Q, ld_out] with column h*Dh + c
 */
typedef struct {
  const float* value; int64_t ld_value; int32_t value_col;
  const float* off_aw; int64_t ld_off_aw;
  const float* ref;
  float* out; int64_t ld_out;
  int32_t B, S, Q, heads, head_dim, levels, points;
  int32_t level_h[4], level_w[4], level_start[4];
  float offset_scale;
  /* ABI v10: value_bf16 (non-NULL) replaces value — the bf16 variant's value projection stored as bf16
   * rows (same ld_value / value_col in elements); sampling and accumulation stay fp32. */
  const uint16_t* value_bf16;
} sp_msda_desc;

int sp_abi_version(void);
const char* sp_last_error(void);
/* ABI v14: what this library was compiled with (no device call). SP_BUILD_FUSED_LN: the fused-LayerNorm
 * GEMM epilogue (sp_conv_desc.ln_gamma; diagnostic builds only); SP_BUILD_BOUNDS: the bounds-check build. */
enum sp_build_flag { SP_BUILD_FUSED_LN = 1, SP_BUILD_BOUNDS = 2 };
int sp_build_flags(void);
/* ABI v14, bounds-check builds (SP_BUILD_BOUNDS): synchronises the device, returns the number of index
 * violations the kernels recorded since the last call (and resets the counts), and writes one line per
 * offending source unit ("file:line hits=… index=… extent=…") into buf. -1 on a product build. */
int64_t sp_bounds_report(char* buf, int64_t cap);
int sp_device_init(int device);
/* Frees the cached resample coefficient tables (the only state kept across
 * calls). Safe to call at any time; the next sp_preprocess_u8 rebuilds what it needs. */
int sp_shutdown(void);

/* RTDetrImageProcessorPil resize (PIL BILINEAR, bit-exact) + rescale 1/255 + HWC→CHW
 * (IPP:451-462, IT:118-122, IT:367). out: [n, 3, out_h, out_w] fp32. */
int sp_preprocess_u8(const sp_image_u8* images, int n, int out_h, int out_w, float* out,
                     void* stream);

int sp_conv2d(const sp_conv_desc* d, void* stream);
/* Test / tuning hook (ABI v7): force the GEMM tile configuration of later sp_conv2d calls made by
 * the CALLING THREAD (-1, the default, = chosen by shape). Nothing on the product path calls it, and
 * no environment variable is read: the production tile choice cannot be changed from outside. */
int sp_set_conv_config(int cfg);
/* The same override for split-K launches only (ABI v11; cfg -1 = the library's choice), a cap on the split-K
 * factor of this thread's later launches (max_splits < 1 = the default, 16) and the fewest 32-deep k-tiles a
 * launch needs to split at all (min_ktiles < 1 = the default, 8): bs1 tuning hooks. */
int sp_set_splitk_config(int cfg, int max_splits, int min_ktiles);
/* Tuning knobs of this thread's later launches (ABI v11; value -1 = the product default), for same-process
 * A/B measurements; nothing on the product path calls it. */
enum sp_tuning_knob {
  SP_TUNE_GLDS_EPILOGUE = 3,  /* split-mode slab epilogue: 4 = outputs stored from the accumulators, else the slab pass */
  SP_TUNE_MSDA_GENERIC = 4,   /* ABI v14: 1 = sp_msda's per-lane kernel where the point-sharing one applies (A/B) */
};
int sp_set_tuning(int knob, int value);

/* 3x3 stride-1 pad-1 convolution by Winograd F(2x2, 3x3) (ABI v9): the same result contract as
 * sp_conv2d on the same descriptor (KH = KW = 3, stride 1, pad 1; act, scale / shift, res1 / res2 as
 * above; no A2, row_scale, grouped rows or LayerNorm; Cin % 32 == 0, Cout % 4 == 0, 16-byte aligned
 * operands), computed as input transform V = B^T d B per 2x2 output tile → 16 batched GEMMs
 * V_ab · U_ab on the split (SP_PREC_F32X3) or bf16 (SP_PREC_BF16) MFMA kernels → output transform
 * Y = A^T M A + the fused epilogue. 2.25x fewer GEMM multiply-adds than the implicit GEMM; fp32 error
 * on par with the direct fp32 conv. wt_wino: the transformed weights U = G g G^T (computed in fp64 on
 * the host, rounded to fp32) as bf16 planes [planes][16][Cout][Cin] (component ab = 4a + b), planes
 * wino_plane_stride elements apart (3 planes for SP_PREC_F32X3, 1 for SP_PREC_BF16); d->Wt /
 * d->Wt_bf16 are not read. work: fp32 scratch of >= 16 * T * (Cin + Cout) elements,
 * T = N * ceil(H/2) * ceil(W/2). Replaces sp_conv2d for the RepVGG 3x3 (M2:921-923) and other
 * stride-1 3x3 convs (M2:817-835, RN:78-103). */
int sp_conv3x3_winograd(const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride, float* work,
                        int64_t work_elems, void* stream);
/* The three stages of sp_conv3x3_winograd as separate launches (same arguments and checks; work holds
 * V = work[0 : 16*T*Cin) and M = work[16*T*Cin : 16*T*(Cin+Cout))), so a caller can time the component
 * GEMM apart from the two HBM-bound transforms: input transform A → V; the 16 batched GEMMs V → M;
 * output transform + epilogue M → C. */
int sp_winograd_f23_input(const sp_conv_desc* d, float* work, int64_t work_elems, void* stream);
int sp_winograd_f23_gemm(const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride, float* work,
                         int64_t work_elems, void* stream);
int sp_winograd_f23_output(const sp_conv_desc* d, const float* work, int64_t work_elems, void* stream);
/* The same three stages for F(4x4, 3x3) (ABI v9): 4x4 output tiles, T = N * ceil(H/4) * ceil(W/4), 36
 * components (component ab = 6a + b), interpolation points (0, -1, 1, 1/2, -2, inf); wt_wino
 * [planes][36][Cout][Cin] (U = G g G^T in fp64 on the host), work >= 36 * T * (Cin + Cout) elements.
 * 1/4 of the direct conv's multiply-adds; fp32 error 3-5x the direct conv's, under 1e-5 of the output
 * scale (tests/test_gpu_kernels.py::test_winograd_is_fp32_accurate). */
int sp_winograd_f43_input(const sp_conv_desc* d, float* work, int64_t work_elems, void* stream);
int sp_winograd_f43_gemm(const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride, float* work,
                         int64_t work_elems, void* stream);
int sp_winograd_f43_output(const sp_conv_desc* d, const float* work, int64_t work_elems, void* stream);

/* NCHW → NHWC (pixel_values layout of the processor contract → conv layout). */
int sp_nchw_to_nhwc(const float* x, float* y, int n, int c, int h, int w, void* stream);
/* Backbone stem conv 1 (RN:71-114: 3x3 stride 2 pad 1, Cin 3, FrozenBN affine M2:748-758, ReLU)
 * read directly from NCHW pixel_values x [n,3,h,w]; wt [cout][27] in (kh, kw, ci) order; y NHWC
 * [n, (h-1)/2+1, (w-1)/2+1, cout]. Replaces sp_nchw_to_nhwc + sp_conv2d for this layer. cout 32 or 64,
 * act 0 (none) or 1 (relu). (ABI v6) */
int sp_stem_conv3x3s2_nchw(const float* x, const float* wt, const float* scale, const float* shift, float* y,
                           int n, int h, int w, int cout, int act, void* stream);
/* The same with bf16 output rows (ABI v10: the bf16 variant; fp32 arithmetic, RNE at the store). */
int sp_stem_conv3x3s2_nchw_bf16(const float* x, const float* wt, const float* scale, const float* shift, uint16_t* y,
                                int n, int h, int w, int cout, int act, void* stream);
/* Stem convs 2 and 3 of the bf16 variant (ABI v10): 3x3 stride 1 pad 1, Cin 32 → Cout 32 or 64, dense NHWC
 * bf16 rows in and out, weights w16 bf16 [Cout][3][3][32], FrozenBN (scale, shift) + act (0 none, 1 relu)
 * in fp32, RNE at the store. Direct LDS-halo convolution (RN:78-103). */
int sp_conv3x3_c32_bf16(const uint16_t* x, const uint16_t* w16, const float* scale, const float* shift, uint16_t* y,
                        int n, int h, int w, int cout, int act, void* stream);
/* The same two convs on fp32 rows (ABI v10, the fp32 modes): dense NHWC fp32 rows in and out, weights fp32
 * [Cout][3][3][32] (the packed [Cout][K] form), exact fp32 products with fp32 accumulation
 * (v_mfma_f32_32x32x2_f32). Direct LDS-halo convolution (RN:78-103). */
int sp_conv3x3_c32(const float* x, const float* wt, const float* scale, const float* shift, float* y, int n, int h,
                   int w, int cout, int act, void* stream);
/* The ResNet stage-0 3x3 (Cin 64 → Cout 64, stride 1 pad 1, RN:170-231) on bf16 rows (the bf16 variant):
 * bf16 [64][3][3][64] weights, rows ldx (% 8) / ldy (% 4)
 * elements apart, fp32 accumulate, BN (+ the optional pre-activation residual res, bf16 rows ldr apart: the
 * basic block's shortcut, RN:170-200) + act in fp32, RNE at the store. */
int sp_conv3x3_c64_bf16(const uint16_t* x, int64_t ldx, const uint16_t* w16, const float* scale, const float* shift,
                        uint16_t* y, int64_t ldy, const uint16_t* res, int64_t ldr, int n, int h, int w, int act,
                        void* stream);
/* nn.MaxPool2d(3, 2, 1) on NHWC (RN:88). y rows are ldy floats apart (ldy >= c, ldy % 4 == 0), so the
 * result can land in a channel slice of a wider buffer (the fused bottleneck shortcut, ABI v6). */
int sp_maxpool3x3s2(const float* x, float* y, int64_t ldy, int n, int h, int w, int c, void* stream);
/* The same on bf16 rows (ABI v10: the bf16 variant's backbone maps); c % 8 == 0, ldy % 8 == 0. */
int sp_maxpool3x3s2_bf16(const uint16_t* x, uint16_t* y, int64_t ldy, int n, int h, int w, int c, void* stream);
/* nn.AvgPool2d(2, 2, 0, ceil_mode=True) on NHWC (RN:150, RN:202); y rows ldy floats apart as above. */
int sp_avgpool2x2_ceil(const float* x, float* y, int64_t ldy, int n, int h, int w, int c, void* stream);
/* The same on bf16 rows (ABI v10; fp32 sum and divide, RNE to bf16); c % 8 == 0, ldy % 8 == 0. */
int sp_avgpool2x2_ceil_bf16(const uint16_t* x, uint16_t* y, int64_t ldy, int n, int h, int w, int c, void* stream);
/* F.interpolate(scale_factor=2, mode="nearest") into a channel slice (M2:1192). */
int sp_upsample2x_nearest(const float* x, int64_t ldx, float* y, int64_t ldy, int n, int h,
                          int w, int c, void* stream);
/* nn.LayerNorm over the last dim (d <= 1024). */
int sp_layernorm(const float* x, int64_t ldx, const float* gamma, const float* beta, float* y,
                 int64_t ldy, int rows, int d, float eps, void* stream);
/* ABI v15. sp_layernorm at d = 256 with the output rounded RNE to bf16 rows: the bf16 variant's encoder head,
 * whose score projection rounds its operand to bf16 anyway (M2:1587-1593). */
int sp_layernorm_bf16(const float* x, int64_t ldx, const float* gamma, const float* beta, uint16_t* y, int64_t ldy,
                      int rows, int d, float eps, void* stream);
/* softmax(Q Kᵀ · scale) V per (batch, head); Q/K/V rows [batch*n, ld], head h at col h*dh. */
int sp_attention(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                 int64_t ldv, float* o, int64_t ldo, int batch, int n, int heads, int dh,
                 float scale, void* stream);
/* The same on bf16 operands (ABI v11, the bf16 variant): Q / K / V rounded to bf16 as staged, scores, softmax and
 * accumulation in fp32; fp32 rows in and out. */
int sp_attention_bf16(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                      int64_t ldv, float* o, int64_t ldo, int batch, int n, int heads, int dh,
                      float scale, void* stream);
int sp_msda(const sp_msda_desc* d, void* stream);
/* Per row: top-k of x[r, 0:n] (values reduced by max over groups of `reduce_c` consecutive
 * columns first when reduce_c > 1; sigmoid applied first when apply_sigmoid), sorted by
 * value descending, ties by lower index. vals may be NULL. Requires k <= 512. */
int sp_topk_rows(const float* x, int64_t ldx, int rows, int n, int reduce_c, int apply_sigmoid,
                 int k, float* vals, int32_t* idx, void* stream);
/* out[r] = max_c x[r*ldx + c], c < C: the per-anchor class max in front of query selection
 * (enc_outputs_class.max(-1).values, M2:1599), spread over the chip; sp_topk_rows(reduce_c = 1)
 * then ranks one key per anchor. */
int sp_rowmax(const float* x, int64_t ldx, int64_t rows, int c, float* out, void* stream);
/* ABI v15. out[r] = max_c (a[r, :] · w[c, :] + bias[c]), c < n: the bf16 variant's score head and its per-anchor
 * class max in one pass (M2:1587-1599), equal bit for bit to sp_conv2d (SP_PREC_BF16, bf16 A rows) + sp_rowmax.
 * a: bf16 rows [rows, lda], w: bf16 [n, k] (k contiguous), n <= 96, k = 256, 16-byte aligned. */
int sp_linear_rowmax_bf16(const uint16_t* a, int64_t lda, const uint16_t* w, const float* bias, int rows, int n,
                          int k, float* out, void* stream);
/* dst[b, i, :] = src[b*src_rows + idx[b, i], :] */
int sp_gather_rows(const float* src, int64_t ld_src, int src_rows, const int32_t* idx, int k,
                   int batch, int d, float* dst, int64_t ld_dst, void* stream);
/* ABI v15. y[r, 0:cols] = a[r, :] + b[r, :] in fp32, written as fp32 rows (y) or rounded RNE to bf16 rows
 * (y_bf16; exactly one of the two): the decoder / AIFI attention input h + pos (M2:395-404, M2:409-423),
 * materialised so the q/k and offset projections load it by LDS-DMA instead of adding it in a register-staged
 * loader (sp_conv_desc.A2). cols % 8 == 0, lda / ldb % 4 == 0, ldy % 8 == 0, 16-byte aligned rows. */
int sp_add_rows(const float* a, int64_t lda, const float* b, int64_t ldb, float* y, uint16_t* y_bf16, int64_t ldy,
                int rows, int cols, void* stream);
/* ref[b,i,:] = sigmoid(delta[b,i,:] + anchors[idx[b,i],:]) (M2:1597-1603, M2:616). */
int sp_ref_init(const float* delta, int64_t ld_delta, const float* anchors, const int32_t* idx,
                int batch, int k, float* ref, void* stream);
/* ref = sigmoid(delta + inverse_sigmoid(ref, 1e-5)) (M2:636-639, M2:548-552). */
int sp_box_refine(const float* delta, int64_t ld_delta, float* ref, int rows, void* stream);
/* post_process_object_detection, use_focal_loss=True (IPP:536-576):
 * scores = sigmoid(logits) → top-k over Q*C → label = i % C, query = i / C, box = xyxy(boxes[query])
 * × (w, h, w, h); counts[b] = #(score > threshold) (results are sorted, so the kept ones are a
 * prefix). target_hw: device int32 [B, 2] (h, w). work: device int32 [B*k]. */
int sp_postprocess(const float* logits, const float* boxes, const int32_t* target_hw, int batch,
                   int q, int c, int k, float threshold, float* scores, int64_t* labels,
                   float* boxes_xyxy, int32_t* counts, int32_t* work, void* stream);

/*
 * JPEG decode (ABI v11): the step in front of A1 — serve.py:96-97 `Image.open(BytesIO(...)).convert("RGB")`,
 * which Pillow runs through libjpeg-turbo (ISLOW integer IDCT, fancy upsampling, integer YCbCr→RGB).
 * Split as the hardware wants it: the Huffman entropy decode (a serial bit stream) on the host, everything
 * per pixel on the GPU. Supported: 8-bit baseline / extended / progressive Huffman JPEGs with 1 (gray) or 3
 * (YCbCr, or RGB per the Adobe / component-id rules of libjpeg) components, luma at the maximum sampling
 * factors and chroma at 1x or 2x below it in each direction, restart intervals. Anything else returns
 * SP_JPEG_UNSUPPORTED (the caller keeps the reference's host decode for that image).
 */
#define SP_JPEG_UNSUPPORTED (-10)
typedef struct {
  int32_t width, height;
  int32_t ncomp;            /* 1 or 3 */
  int32_t color;            /* 0 gray, 1 YCbCr, 2 RGB */
  int32_t progressive;
  int32_t max_h, max_v;     /* maximum sampling factors */
  int32_t h[3], v[3];       /* sampling factors per component */
  int32_t bw[3], bh[3];     /* coefficient blocks per row / block rows per component (MCU-padded) */
  int64_t block_off[3];     /* first block of each component in the coefficient array */
  int64_t total_blocks;     /* coefficient array: total_blocks * 64 int16, natural (row-major) order */
  int64_t plane_off[3];     /* byte offset of each component's sample plane (bw*8 x bh*8) in `work` */
  int64_t plane_bytes;      /* bytes of `work` sp_jpeg_to_rgb needs */
  uint16_t quant[3][64];    /* dequantisation tables (natural order), latched at each component's first scan */
} sp_jpeg_layout;
/* Host: parse the JPEG in data[0:len) into *lay; with coefs != NULL (coef_elems >= total_blocks*64) also run
 * the entropy decode (jdhuff.c / jdphuff.c semantics, including progressive refinement scans and restart
 * markers; truncated data decodes as zeros, as libjpeg does) and write the quantised coefficients. No device
 * call: safe without a GPU. */
int sp_jpeg_decode_coefs(const uint8_t* data, int64_t len, sp_jpeg_layout* lay, int16_t* coefs, int64_t coef_elems);
/* Device: coefficients (device copy of the array above) → RGB: dequantise + ISLOW IDCT per 8x8 block into the
 * component planes in `work`, then fancy upsampling + YCbCr→RGB into rgb (uint8 HWC rows rgb_stride bytes
 * apart, the exact pixels Pillow's convert("RGB") produces). status (device int32, zeroed by the caller; may
 * be NULL) is set to 1 when a block leaves the range in which this integer IDCT and libjpeg-turbo's SIMD one
 * agree (only corrupt or crafted coefficient data does): the caller then keeps Pillow's decode (ABI v12). */
int sp_jpeg_to_rgb(const int16_t* coefs, const sp_jpeg_layout* lay, uint8_t* work, int64_t work_bytes, uint8_t* rgb,
                   int64_t rgb_stride, int32_t* status, void* stream);

/*
 * JPEG encode (ABI v12): serve.py:139-142 `image.save(buffer, format="JPEG")`, which Pillow runs through
 * libjpeg-turbo with quality 75 (or the caller's), 4:2:0 (or the caller's subsampling), the ISLOW forward DCT,
 * the Annex K Huffman tables and a JFIF header. Split as the hardware wants it: colour conversion,
 * downsampling, FDCT, quantisation and the Huffman coding itself (per-MCU bit counts, a prefix sum, then
 * every MCU writes its bits at its own offset) on the GPU; the header bytes, the 0xFF byte stuffing and the
 * final padding on the host. The bytes equal Pillow's (tests/test_jpeg_enc.py, tests/test_gpu_jpeg.py).
 */
typedef struct {
  int32_t width, height;
  int32_t quality;              /* 1..100 (Pillow's default -1 resolved to libjpeg's 75) */
  int32_t h0, v0;               /* luma sampling factors (1x1, 2x1 or 2x2); chroma is 1x1 */
  int32_t mcux, mcuy, bpm;      /* MCU grid; blocks per MCU = h0*v0 + 2 */
  int32_t wb0, hb0;             /* luma blocks holding image data (the rest of the MCU grid: dummy blocks) */
  int64_t total_blocks;         /* mcux * mcuy * bpm, in scan (MCU-interleaved) order */
  int64_t work_bytes;           /* device workspace sp_jpeg_enc_rgb needs */
  int64_t bits_cap;             /* device bytes of the entropy-coded bit buffer (worst case) */
  uint16_t quant[2][64];        /* natural order, luma / chroma (jcparam.c jpeg_set_quality) */
  uint16_t recip[2][64];        /* jcdctmgr.c compute_reciprocal of quant << 3: reciprocal, correction, shift */
  uint16_t corr[2][64];
  int16_t shift[2][64];
} sp_jpeg_enc_layout;
/* Host: the layout for a width x height RGB image at quality (-1 = 75) and Pillow's subsampling code (-1 or 2:
 * 4:2:0, 1: 4:2:2, 0: 4:4:4). */
int sp_jpeg_enc_plan(int32_t width, int32_t height, int32_t quality, int32_t subsampling, sp_jpeg_enc_layout* lay);
/* Device: RGB pixels (uint8 rows row_stride bytes apart, pixel_bytes 3 (RGB) or 4 (RGBX)) → the entropy-coded
 * segment, unstuffed and unpadded, MSB first, in bits[0 : ceil(*nbits / 8)); *nbits (device int64) is written.
 * work: lay->work_bytes; bits: lay->bits_cap bytes. */
int sp_jpeg_enc_rgb(const uint8_t* rgb, int64_t row_stride, int32_t pixel_bytes, const sp_jpeg_enc_layout* lay,
                    uint8_t* work, int64_t work_bytes, uint8_t* bits, int64_t bits_cap, int64_t* nbits, void* stream);
/* Host: the JPEG file: SOI, JFIF APP0, COM (comment_len > 0), DQT x2, SOF0, DHT x4, SOS, the segment with 0xFF
 * stuffing and 1-bit padding, EOI. out_cap >= sp_jpeg_enc_max_bytes(lay, nbits, comment_len). */
int64_t sp_jpeg_enc_max_bytes(const sp_jpeg_enc_layout* lay, int64_t nbits, int64_t comment_len);
int sp_jpeg_enc_finish(const sp_jpeg_enc_layout* lay, const uint8_t* bits, int64_t nbits, const uint8_t* comment,
                       int64_t comment_len, uint8_t* out, int64_t out_cap, int64_t* out_len);

#ifdef __cplusplus
}
#endif
#endif /* SPOTTER_HIP_H */
