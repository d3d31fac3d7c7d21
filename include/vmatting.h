/*
 * vmatting.h — C ABI of the MI355X (gfx950) per-frame alpha-matting path.
 *
 * Drop-in boundary for the hot path of tangih/video-matting.  The reference is
 * TensorFlow-1.x graph code: its "FFI" is the TF op set reached through
 * sess.run (train.py:81,330).  Each entry point below replaces the TF/OpenCV
 * op(s) the reference's model builders and flow helpers call, cited per
 * function.  A Python host (video-matting_amd/vmatting/_lib.py) binds this with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - All tensor pointers are DEVICE pointers owned by the caller (e.g. from
 *     torch.Tensor.data_ptr() on ROCm); nothing is allocated inside a call.
 *   - Activations are NHWC views (vm_tensor): element (n,h,w,c) lives at
 *     ptr + ((n*H + h)*W + w)*cstride + coff + c, in elements of `dtype`.
 *     A channel slice of a wider buffer (coff, cstride) is how a tf.concat is
 *     expressed without a copy (unet.py:62, unet_simple.py:41, small.py:22).
 *   - `stream` is a hipStream_t (void* here so the header needs no HIP include);
 *     every call is asynchronous on it and is capturable into a hipGraph.
 *   - Return value: VM_OK (0) or a negative VM_E* code; vm_last_error() gives a
 *     per-thread message.  No exception crosses the ABI.
 *   - Thread-safety: reentrant; calls on different streams may run concurrently.
 */
#ifndef VMATTING_H
#define VMATTING_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VM_ABI_VERSION 1

enum vm_dtype {
  VM_F32 = 0,
  VM_BF16 = 1,
  VM_U8 = 2,
  VM_F64 = 3, /* loader outputs only */
  VM_F16 = 4  /* IEEE half: the split-fp16 x3 conv operands only (vm_split3h_nhwc, vm_conv3x3_ex_nhwc, head_acc) */
};

enum vm_act {
  VM_ACT_NONE = 0,
  VM_ACT_RELU = 1,     /* tf.nn.relu            (unet.py:96 ...)            */
  VM_ACT_SIGMOID = 2,  /* tf.nn.sigmoid         (unet.py:145,205)           */
  VM_ACT_SOFTMAX = 3   /* tf.nn.softmax, last axis (refine.py:31)           */
};

enum vm_status {
  VM_OK = 0,
  VM_EINVAL = -1,        /* bad argument / shape mismatch (TF: ValueError at build) */
  VM_EUNSUPPORTED = -2,  /* valid but not supported by this build                    */
  VM_EHIP = -3,          /* HIP runtime error                                        */
  VM_EINDEX = -4         /* data-dependent index error (flow.correct_alpha IndexError) */
};

typedef struct vm_tensor {
  void* ptr;
  int32_t n, h, w, c;     /* logical shape                                  */
  int32_t cstride, coff;  /* channel stride of the pixel row / first channel */
  int32_t dtype;          /* enum vm_dtype                                   */
} vm_tensor;

int vm_abi_version(void);
const char* vm_last_error(void);
/* Process-wide tuning knobs (no reference counterpart; TF picks kernels itself):
 *   "conv_kernel"    0 = auto (default: patch kernel when legal, else by shape), 1 = register-staged MFMA kernel
 *                    only, 2 = LDS-DMA kernel when legal, 3 = patch-reuse kernel when legal (bf16, cin % 32 == 0,
 *                    bf16 output, no softmax)
 *   "patch_cfg"      patch-kernel tiling override (0 = dispatcher's choice; 19, 22, 25, 30 = one of the tilings it
 *                    picks); the other sweep tilings and the timing-only ablations ("patch_ablate", "patch_rowslot",
 *                    "pair_kernel" 10..18, garbage results) exist only in the study build (`make study`), never here
 *   "up_skip"        folded 2x upconvs: 1 = skip the exact-zero taps of the odd phases' filters (25 of 36 taps run,
 *                    bit-identical, default), 0 = run all 36
 *   "src_span_limit" byte span of split sources the 32-bit-offset conv kernels take (default 0x7ffffff0; wider
 *                    spans return VM_EUNSUPPORTED and the caller materialises the concat); lowered by tests
 *   "conv_min_tiles" grid size (256-wide output tiles) from which auto uses the LDS-DMA kernel (default 128)
 *   "glds_rb"        K-step bytes of the 256x256 LDS-DMA tile: 128 (2-slot ring, default) or 64 (4-slot)
 *   "head_kernel"    cout == 1 convs: 0 = MFMA tap-GEMM kernel (default), 1 = generic per-pixel kernel,
 *                    2 = register-strip kernel
 *   "softmax_kernel" cin <= 8 -> 64 conv + softmax (refine.py conv4): 0 = generic kernels' epilogue; bf16: 1 =
 *                    conv3x3_first_softmax (register stores), 2 = its nontemporal form, 3 / 4 = per-wave LDS transpose
 *                    with whole-pixel plain / nontemporal stores, 5 = 4 with the weights in LDS, 6 = wave-private
 *                    strips, no per-tile block barrier (default); f32: any value but 0 = conv3x3_first_softmax_f32
 *   "softmax_blocks" persistent grid of the conv3x3_first_softmax kernels (default 2048)
 *   "pair_xin_wide"  pair kernel, f32 frames with 4..8 channels: 1 = two 16-byte loads per pixel (default),
 *                    0 = one dword load per channel
 *   "pair_strip"     first pair: 1 = strip-walking kernel where it applies (default), 0 = tile kernels
 *   "patch_repi"     patch kernel register epilogue: 1 (default) / 0 = LDS-staged epilogue
 *   "patch_persist"  1 = persistent row-slot patch kernel where the round policy says it pays (default), 0 = off
 *   "persist_rounds", "persist_up_rounds"  its minimum rounds of items for plain convs (default 2) and folded
 *                    upconvs (default 6); 0 = any grid (tests)
 *   "persist_all"    1 = every plain grid of >= persist_rounds rounds (A/B); "persist_rot" 0 = walkers rotate
 *                    through the output tiles for folded upconvs only (default), 1 = always, 2 = never
 *   "rows_kernel", "rows_min_blocks", "rows_min_cin", "rows_up"  row-stationary kernel dispatch (1, 400, 128, 0)
 *   "border_ks"      folded-upconv border pass granule split: 1 (default), 2 or 4
 *   The patch / row-stationary / persistent / strip choices and "up_skip" are bit-identical (every output keeps its
 *   MFMA sequence); "conv_kernel", "head_kernel" and "softmax_kernel" pick kernels with another f32 summation order
 *   (within the stated tolerances). */
int vm_set_option(const char* key, long value);
/* Name of the conv kernel the calling thread's last vm_conv3x3_nhwc launched, spelled the way
 * rocprofv3 reports it (e.g. "vm::conv3x3_mfma<unsigned short, 128, 128>"); "" before the first call.
 * Used to attribute per-kernel profiler counters (bench.py); no reference counterpart. */
const char* vm_conv3x3_last_kernel(void);

/* ---------------------------------------------------------------- 3x3 convolution
 * Replaces tf.nn.conv2d(x, w, [1,1,1,1], 'SAME') + tf.nn.bias_add + the activation /
 * inference batch-norm that follows it:
 *   unet.py:35-42 (new_conv), 44-63 (upconv conv), 65-74 (conv_layer);
 *   unet_simple.py:19-27, 30-42, 98-107; small.py:13-34; refine.py:18-25.
 * y = act((conv(x, w) + bias) * scale + shift) per output channel; bias/scale/shift
 * may be NULL (f32 device arrays of length cout).  Weights are first packed from
 * TF's HWIO f32 layout into the kernel's [cout_pad][K_pad] layout (K ordered channel-chunk-major:
 * the 9 taps of each 128-byte channel chunk are consecutive, so shared input rows stay L2-resident).
 * Computes in x->dtype (bf16 -> MFMA 16x16x32 bf16, f32 -> exact-f32 MFMA 16x16x4),
 * accumulates in f32.  cout == 1 dispatches the memory-bound head kernel.
 * act == VM_ACT_SOFTMAX needs cout <= 128 (whole channel row in one tile).
 */
size_t vm_conv3x3_packed_bytes(int cin, int cout, int dtype);
int vm_conv3x3_pack_weights(const float* w_hwio, int cin, int cout, int dtype, void* packed, void* stream);

/* Many packs in ONE launch (the optimizer step re-packs every trainable filter, train.py:302-304).  A job packs the
 * conv geometry (cin, cout, dtype) from an f32 HWIO source filter of (w_cin, w_cout) channels, zero outside it
 * (a cout-padded narrow conv); flip = 1 packs the data-gradient filter of that source instead (spatially flipped,
 * in/out transposed: cin = the source's output channels (padded), cout = its input channels). */
typedef struct vm_pack_job {
  const float* w;
  void* packed;
  int32_t cin, cout, dtype, flip, w_cin, w_cout;
} vm_pack_job;
int vm_conv3x3_pack_weights_batch(int njobs, const vm_pack_job* jobs, void* stream);
int vm_conv3x3_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                    const float* scale, const float* shift, int act, vm_tensor* y, void* stream);
/* The same conv over the channel concat of nsrc sources (unet_simple.py:153-168's per-level concat of the three
 * towers, tower-major in HBM so the towers run as one batch): x is the [n,h,w,c_src] view of source 0, source s
 * lies src_stride elements further; cin = nsrc * x->c, and x->c must be whole 64-byte granules. */
/* vm_conv3x3_nhwc / vm_conv3x3_sources_nhwc with a caller workspace: small-grid bf16 convs with a long K loop
 * (the deep levels of unet_simple's towers and heads) split their channel granules over ~1024 blocks and reduce the
 * f32 partial sums in a fixed order (deterministic).  nsrc 0/1 = one source.  work: vm_conv3x3_workspace_bytes. */
size_t vm_conv3x3_workspace_bytes(const vm_tensor* x, int cin, int cout);
int vm_conv3x3_ex_nhwc(const vm_tensor* x, int nsrc, long src_stride, const void* packed, int cin, int cout,
                       const float* bias, const float* scale, const float* shift, int act, vm_tensor* y, void* work,
                       size_t work_bytes, void* stream);
int vm_conv3x3_sources_nhwc(const vm_tensor* x, int nsrc, long src_stride, const void* packed, int cin, int cout,
                            const float* bias, const float* scale, const float* shift, int act, vm_tensor* y,
                            void* stream);
/* Same conv, and additionally the 2x2/2 SAME max-pool of its output written to ypool
 * ([n, ceil(h/2), ceil(w/2), cout], same dtype) — replaces the conv_layer + max_pool pairs
 * unet.py:170-187 (conv1_2/pool1 ... conv4_3/pool4; max_pool at unet.py:32-33).
 * Only the bf16 patch kernel fuses pooling: other cases return VM_EUNSUPPORTED and the caller runs
 * vm_conv3x3_nhwc + vm_maxpool2x2_same_nhwc instead. */
int vm_conv3x3_pool_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                         const float* scale, const float* shift, int act, vm_tensor* y, vm_tensor* ypool,
                         void* stream);

/* cout == 1 head conv, y = act(conv(x, w) + bias ...), and optionally alpha = sigmoid of the pre-activation value
 * (f32, contiguous [n*h*w]) from the same pass — unet.py:203-205 (conv1_5 = self.conv1_3 logits, then
 * tf.nn.sigmoid -> self.output; unet_simple.py:142, small.py:49-50).  alpha may be NULL. */
int vm_conv3x3_head_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias, const float* scale,
                         const float* shift, int act, vm_tensor* y, float* alpha, void* stream);

/* The same cout == 1 head over one channel chunk of its input, adding y_acc (f32, contiguous [n*h*w], e.g. the
 * previous chunk's y) to the pre-activation: a head over more channels than one MFMA head tile holds, chunk by chunk
 * (the split-bf16 x6 path's conv1_5 over 6 x 128 channels, unet.py:203-205).  cin <= 256 (bf16). */
int vm_conv3x3_head_acc_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias, const float* y_acc,
                             vm_tensor* y, float* alpha, void* stream);
/* The same with the per-channel affine of vm_conv3x3_nhwc: pre-activation = (conv + y_acc + bias) * scale + shift
 * (y_acc may be NULL) — the split-fp16 x3 path's conv1_5, whose fp16 filter parts are pre-scaled by a power of two
 * that the last chunk's scale undoes (exactly) before the sigmoid (unet.py:203-205).  x may be VM_F16 (cin <= 256), or a two-slab
 * split-fp16 view [l, h] of 128-channel slabs with cin 384 (read as [l, h, h]; conv1_5 of the f16x3 forward). */
int vm_conv3x3_head_acc_ex_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias, const float* scale,
                                const float* shift, const float* y_acc, vm_tensor* y, float* alpha, void* stream);

/* Two chained convs whose 64-channel intermediate never leaves the chip: y = act2(conv3x3(relu(conv3x3(x, w1) + bias1),
 * w2) + bias2 ...), optionally with the fused 2x2 SAME max-pool of y into ypool (NULL = none) — replaces
 * unet.py:170-172 (conv1_1 -> conv1_2 -> pool1; conv_layer at :65-74) and the VGG towers' first pair
 * (unet_simple.py:60-62).  x: [n,h,w,cin1 <= 8], either a bf16 view whose 8-element pixel row from coff is
 * readable (the channels >= cin1 meet zero weights) or the caller's f32 frame itself (any channel stride; rounded
 * to bf16 on load, which replaces the vm_convert_nhwc pass); packed1 = vm_conv3x3_pack_weights(cin1, 64, bf16),
 * packed2 = (64, cout2, bf16).  bf16 compute only: an f32 y returns VM_EUNSUPPORTED and the caller runs the two
 * convs separately. */
int vm_conv3x3_pair_first_nhwc(const vm_tensor* x, const void* packed1, int cin1, const float* bias1,
                               const void* packed2, int cout2, const float* bias2, const float* scale2,
                               const float* shift2, int act2, vm_tensor* y, vm_tensor* ypool, void* stream);

/* The pair with conv1_1's own output kept too (mid: bf16 [n,h,w,64] view, 16-byte aligned channel chunks) — the
 * training towers (unet_simple.py:60-62), whose select convs read conv1_1 (unet_simple.py:160-168).
 * VM_EUNSUPPORTED when the strip-walking kernel cannot take the case (the caller runs the two convs). */
int vm_conv3x3_pair_first_mid_nhwc(const vm_tensor* x, const void* packed1, int cin1, const float* bias1,
                                   const void* packed2, int cout2, const float* bias2, const float* scale2,
                                   const float* shift2, int act2, vm_tensor* y, vm_tensor* ypool, vm_tensor* mid,
                                   void* stream);

/* The pair kernel with the head split (unet.py:170-172 + 203-205): conv1_5 over cat1 = [up, skip] is linear in
 * its input channels, so the skip half's share is taken where conv1_2's output is made.  Besides y/ypool the pair
 * kernel writes partial[pixel][12] (f32, n*h*w*12 floats): taps 0..8 of sum_c y[pixel][c] * head_w[tap][head_coff+c]
 * (head_w = conv1_5's HWIO f32 filter [3,3,head_cin,1], bf16-rounded like the packed head; 9..11 = 0).  store_y = 0
 * leaves y unwritten (only the pool and the partials leave the chip).  vm_conv3x3_head_partial_nhwc then runs the
 * head over the other channels (x = the up half, packed for that many channels) and adds
 * sum_tap partial[pixel + offset(tap)][tap] (zero outside the frame) before bias / act / alpha. */
int vm_conv3x3_pair_first_head_nhwc(const vm_tensor* x, const void* packed1, int cin1, const float* bias1,
                                    const void* packed2, int cout2, const float* bias2, const float* scale2,
                                    const float* shift2, int act2, vm_tensor* y, vm_tensor* ypool,
                                    const float* head_w, int head_cin, int head_coff, float* partial, int store_y,
                                    void* stream);
int vm_conv3x3_head_partial_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias,
                                 const float* scale, const float* shift, int act, vm_tensor* y, float* alpha,
                                 const float* partial, void* stream);

/* tf.image.resize_images(x, [2h, 2w]) (TF-1 legacy bilinear, exact 2x) followed by the 3x3 SAME conv, without
 * materialising the resized tensor — unet.py:44-63 (upconv_concat: resize_images at :58, conv2d at :60) for the
 * levels whose skip tensor is exactly twice the input's size.  Bilinear 2x is linear, so every output pixel
 * (2i+a, 2j+b) is a 3x3 conv of the low-res frame at (i, j) with one of four "phase" filters:
 * vm_conv3x3_fold_up2x_weights folds the HWIO f32 filter [3,3,cin,cout] into [3,3,cin,4*cout] (channel
 * p*cout + co = phase p = 2a+b of channel co); pack that with vm_conv3x3_pack_weights(cin, 4*cout) as packed_up
 * and the plain filter as packed.  The frame border (output rows 0 and 2h-1, columns 0 and 2w-1), where the
 * resized image's zero padding breaks the folding, is recomputed from packed the unfused way.
 * x: low-res [n,h,w,cin]; y: [n,2h,2w,cout].  bf16 only (f32 callers use resize + conv3x3: VM_EUNSUPPORTED),
 * cout % 64 == 0, 16-byte aligned channel views.  Numerics: the folded filter is rounded to bf16 instead of the
 * resized activations (same bf16 tolerance class as the unfused path). */
int vm_conv3x3_fold_up2x_weights(const float* w_hwio, int cin, int cout, float* w_up_hwio, void* stream);
int vm_conv3x3_up2x_nhwc(const vm_tensor* x, const void* packed_up, const void* packed, int cin, int cout,
                         const float* bias, const float* scale, const float* shift, int act, vm_tensor* y,
                         void* stream);

/* The folded upconv with the head split (unet.py:200-205: upconv_4 -> cat1 -> conv1_5): besides y (store_y = 0
 * leaves it unwritten) the conv writes partial[pixel][12] of its [n,2h,2w] output (f32): taps 0..8 of
 * sum_c y[pixel][c] * head_w[tap][head_coff + c] over the conv's bf16 outputs (head_w = conv1_5's HWIO f32 filter
 * [3,3,head_cin,1], bf16-rounded like a packed head; taps 9..11 zero), the frame border included (from the border
 * pass's values).  cout == 64; VM_EUNSUPPORTED when a kernel-selection option rules out the patch kernel's register
 * epilogue (the caller then stores y and runs vm_conv3x3_head_partial_nhwc). */
/* The folded upconv of the split-fp16 x3 path (unet.py:44-63 at f32 accuracy): x is the low-res split input [l, h]
 * (VM_F16, S = x.c / 2 channels per slab, S % 32 == 0), packed_up the fp16 parts [Wh', Wl', Wh'] (cin = 3 S) of the
 * folded filter of vm_conv3x3_fold_up2x_weights (pre-scaled by 2^t), packed the plain filter's parts at the same
 * scale (the border pass: the resize of x = h + l in f32, split again); y = act((conv + bias) * scale + shift) in f32,
 * written split as vm_conv3x3_split3_nhwc writes it ([n, 2h, 2w, cout], cout % 64 == 0, slab y_slab). */
int vm_conv3x3_up2x_split3_nhwc(const vm_tensor* x, const void* packed_up, const void* packed, int cin, int cout,
                                const float* bias, const float* scale, const float* shift, int act, vm_tensor* y,
                                int y_slab, int* overflow, void* stream);
int vm_conv3x3_up2x_head_nhwc(const vm_tensor* x, const void* packed_up, const void* packed, int cin, int cout,
                              const float* bias, const float* scale, const float* shift, int act, vm_tensor* y,
                              const float* head_w, int head_cin, int head_coff, float* partial, int store_y,
                              void* stream);

/* conv1_5 + sigmoid from two partial sets (unet.py:203-205 with both halves of cat1 taken where they were made,
 * vm_conv3x3_up2x_head_nhwc and vm_conv3x3_pair_first_head_nhwc): logits[p] = bias[0] + sum_tap (pa[p + off(tap)][tap]
 * + pb[p + off(tap)][tap]) (zero outside the frame), alpha[p] = sigmoid(logits[p]).  pa, pb: f32 [n*h*w][12];
 * logits: f32 [n,h,w,1] view or NULL; alpha: contiguous f32 [n*h*w] or NULL. */
int vm_conv3x3_head_from_partials(const float* pa, const float* pb, int n, int h, int w, const float* bias,
                                  vm_tensor* logits, float* alpha, void* stream);

/* tf.nn.max_pool(ksize 2, stride 2, 'SAME') — unet.py:32-33, unet_simple.py:95-96, small.py:40,42 */
int vm_maxpool2x2_same_nhwc(const vm_tensor* x, vm_tensor* y, void* stream);

/* tf.image.resize_images(x, [H, W]) TF-1.x bilinear legacy — unet.py:58, unet_simple.py:33, small.py:17 */
int vm_resize_bilinear_tf1_nhwc(const vm_tensor* x, vm_tensor* y, void* stream);

/* dtype / channel-padding copy with optional per-channel affine and activation
 * (packs the caller's f32 [N,H,W,7] frame into the compute layout; loader.py:76-78 mean/shift
 * can be folded in via shift).  Channels >= x->c of y are zero-filled. */
int vm_convert_nhwc(const vm_tensor* x, vm_tensor* y, const float* scale, const float* shift, int act, void* stream);
/* A HIP stream created with a full CU mask (hipExtStreamCreateWithCUMask), for the trainers' side streams (the
 * filter gradients beside the data-gradient chain, train.py:37-52 / 288-304): a plain stream shares one of the
 * process's hardware queues, possibly the caller's, which serialises the two.  vm_stream_destroy releases it. */
int vm_stream_create_masked(void** stream);
int vm_stream_destroy(void* stream);
/* One wave spinning for `microseconds` of the device wall clock on `stream`: the trainers' probe for a side stream
 * that runs beside theirs (a plain stream may share the caller's hardware queue). */
int vm_spin(int microseconds, void* stream);
/* Split-bf16 x6 operand of an f32 activation (no reference counterpart: the operand format of the split-bf16 conv
 * path, which evaluates unet.py's tf.nn.conv2d (unet.py:39,60,70) at f32 accuracy on bf16 MFMA).  x (f32 view,
 * x.c channels) -> three bf16 parts h = bf16(x), m = bf16(x - h), l = bf16(x - h - m), written as six slabs
 * [l, m, h, m, h, h] at channel p*S + y.coff + c of y (bf16, S = y.cstride / 6; y.c >= x.c, the extra channels 0).
 * A conv over the 6*S channels with the filter parts [h, m, l, h, m, h] stacked along cin is the sum of the six
 * cross products down to 2^-16 of the leading one.  y_pool (optional, same layout at ceil(h/2) x ceil(w/2)): the
 * split of tf.nn.max_pool 2x2 SAME (unet.py:33) of x, from the same pass. */
int vm_split6_nhwc(const vm_tensor* x, vm_tensor* y, vm_tensor* y_pool, void* stream);
/* Split-fp16 x3 operand of an f32 activation (no reference counterpart: the operand format of the split-fp16 conv path,
 * which evaluates unet.py's tf.nn.conv2d (unet.py:39,60,70) at f32 accuracy in three fp16 MFMA products).  x (f32
 * view) -> h = fp16(x), l = fp16(x - h) (RNE; 22 significant bits), written as slabs [l, h] at channel p*S + y.coff + c
 * of y (VM_F16; S = slab, or y.cstride / 2 when slab <= 0; y.c >= x.c, the extra channels 0), and a third slab [h]
 * at 2*S + y.coff + c when the pixel row holds it (3*S <= y.cstride).  A conv over [l, h, h] with the filter parts
 * [Wh, Wl, Wh] stacked along cin is l*Wh + h*Wl + h*Wh; vm_conv3x3_ex_nhwc / split3 read a two-slab view (x.c = 2S,
 * cin = 3S, S % 32 == 0) as [l, h, h], so h is stored once.  y_pool (optional, same layout at ceil(h/2) x ceil(w/2)):
 * the split of tf.nn.max_pool 2x2 SAME (unet.py:33) of x from the same pass.  overflow (device int, may be NULL): set
 * to 1 when some |x| >= 65520 (fp16's range; the split is then invalid). */
int vm_split3h_nhwc(const vm_tensor* x, vm_tensor* y, vm_tensor* y_pool, int slab, int* overflow, void* stream);
/* tf.image.resize_images(x, [y.h, y.w]) TF-1 legacy bilinear (unet.py:58) of an f32 activation, written as its
 * split-fp16 x3 operand (the vm_split3h_nhwc layout of y, slab / overflow as there) without the f32 resized tensor;
 * the same float32 arithmetic as vm_resize_bilinear_tf1_nhwc, so bit-identical to that resize followed by the split.
 * 16-byte aligned views, c % 8 == 0 (the split-fp16 path's upconv_concat inputs, unet.py:44-63). */
int vm_resize_split3h_nhwc(const vm_tensor* x, vm_tensor* y, int slab, int* overflow, void* stream);
/* The split-fp16 x3 conv with the split of its output fused into the epilogue (no f32 round trip): x is an fp16 split
 * input (slabs [l, h] read as [l, h, h], or three stored slabs; cin = 3 x its channels) and packed its fp16 filter
 * parts; y = act((conv + bias) * scale + shift) is computed in f32 as vm_conv3x3_nhwc does, then written split as
 * vm_split3h_nhwc writes it: slabs [l, h] (+ [h] where 3 * y_slab <= y.cstride) of y (VM_F16, cout % 8 == 0 channels
 * at y.coff inside the first slab) at slab distance y_slab (<= 0: y.cstride / 2);
 * ypool (optional, same layout, pool_slab) receives the split of tf.nn.max_pool 2x2 SAME (unet.py:33) of y.  overflow
 * (device int, may be NULL) is set when some |y| >= 65520.  work / work_bytes: vm_conv3x3_workspace_bytes (split-K on
 * small grids; not with ypool). */
int vm_conv3x3_split3_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                           const float* scale, const float* shift, int act, vm_tensor* y, int y_slab, vm_tensor* ypool,
                           int pool_slab, int* overflow, void* work, size_t work_bytes, void* stream);

/* tf.contrib.layers.batch_norm(is_training=True): batch mean / biased variance over N,H,W
 * (unet_simple.py:25,41; small.py:22,32).  work: vm_bn_workspace_bytes(x) bytes of device scratch. */
size_t vm_bn_workspace_bytes(const vm_tensor* x);
int vm_bn_stats_nhwc(const vm_tensor* x, float* mean, float* var, void* work, void* stream);
/* y = act((x - mean) * rsqrt(var + eps) * gamma + beta); y may alias x. NULL mean/var = 0/1. */
int vm_bn_apply_nhwc(const vm_tensor* x, vm_tensor* y, const float* mean, const float* var, const float* gamma,
                     const float* beta, float eps, int act, void* stream);

/* tf.nn.softmax over channels — refine.py:31 */
int vm_softmax_lastdim_nhwc(const vm_tensor* x, vm_tensor* y, void* stream);

/* reader.create_composite_image (reader.py:72-79): out = a*fg + (1-a)*bg on channels 0..2 (channels >= 3: bg),
 * over `pixels` pixels of `cn` interleaved channels.  fg/bg: img_dtype VM_U8 / VM_F32 / VM_F64; alpha: one
 * VM_F32 / VM_F64 value per pixel; out: VM_F32 / VM_F64.  Computed in float64 (numpy's promotion), rounded to
 * out_dtype, so a VM_F64 output is bit-identical to the reference's numpy expression. */
int vm_composite_image(const void* fg, const void* bg, int img_dtype, const void* alpha, int alpha_dtype,
                       long pixels, int cn, void* out, int out_dtype, void* stream);

/* flow.warp_img (flow.py:9-18): out[y,x] = bilinear(img, x + flow[y,x,0], y + flow[y,x,1]),
 * cv2.remap INTER_LINEAR / BORDER_CONSTANT 0.  mode 0 = OpenCV 1/32-pixel fixed point, 1 = exact.
 * img [ih,iw] f32, flow [h,w,2] f32, out [h,w] f32.  Batched over `n` frames (contiguous). */
int vm_remap_bilinear_f32(const float* img, int ih, int iw, const float* flow, int h, int w, int n, float* out,
                          int mode, void* stream);
/* flow.warp_bgr (flow.py:21-33): uint8 [ih,iw,cn] HWC, OpenCV 15-bit fixed-point weights. */
int vm_remap_bilinear_u8(const uint8_t* img, int ih, int iw, int cn, const float* flow, int h, int w, uint8_t* out,
                         void* stream);

/* flow.correct_alpha (flow.py:36-65): forward/backward consistency; alpha [h,w] f32 zeroed IN PLACE
 * where the round-trip error > thresh.  promote 0 = numpy-1.x float64 index arithmetic, 1 = numpy-2
 * float32.  *err_flag (device int, zeroed by the caller) is set when an index falls below -dim
 * (the reference's IndexError); the host turns that into VM_EINDEX. */
int vm_fb_consistency(const float* backward, const float* forward, int h, int w, float* alpha, float thresh,
                      int promote, int* err_flag, void* stream);

/* BASELINE config 3 in one pass (flow.py:69-77 chain, refine.py:27 input): per pixel
 *   alpha_w = warp_img(prev_alpha, backward)      (as vm_remap_bilinear_f32 mode 0, flow.py:9-18)
 *   correct_alpha(backward, forward, alpha_w)     (as vm_fb_consistency, flow.py:36-65, threshold thresh)
 *   out[pixel] = [cmp B, G, R, alpha, alpha_w, 0, 0, 0]   (the RefineNet input, Cin 5 padded to 8)
 * prev_alpha / alpha [h,w] f32, backward / forward [h,w,2] f32, cmp [h,w,3] f32 (BGR - VGG_MEAN), out [h,w,8]
 * in out_dtype (VM_F32 or VM_BF16), warped [h,w] f32 or NULL.  *err_flag (zeroed by the caller) is set where
 * the reference raises IndexError; the output is then undefined. */
int vm_temporal_refine_input(const float* prev_alpha, const float* backward, const float* forward, const float* cmp,
                             const float* alpha, int h, int w, float thresh, int promote, void* out, int out_dtype,
                             float* warped, int* err_flag, void* stream);

/* train.py:14-28,42-47 loss: out[0] = mean(0.5*charb(pred,gt) + 0.5*charb(composite(raw_fg,bg,pred), cmp)),
 * out[1] = mean alpha loss, out[2] = mean compositional loss.  pred/gt [n,h,w,1], others [n,h,w,3] f32.
 * work: vm_loss_workspace_bytes(n*h*w) bytes. */
size_t vm_loss_workspace_bytes(long pixels);
int vm_matting_loss(const float* pred, const float* gt, const float* raw_fg, const float* bg, const float* cmp,
                    long pixels, float* out, void* work, void* stream);

/* ---------------------------------------------------------------- training-sample loader
 * Replaces the per-pixel part of loader.py's sample builders after decoding: load_and_crop (loader.py:39-85),
 * simple_load_crop (:119-157), video_load_crop (:285-330) and their batch loops get_batch / simple_batch /
 * video_batch (:93-116, 160-171, 333-345) — get_padded_img canvases (:10-36), crops, flow.warp_img of the
 * previous alpha (:291-293), cv2.resize(INTER_LINEAR) of fg / alpha / warped alpha / bg to the network size
 * (:70-73, 146-148, 316-319), reader.create_composite_image and the VGG_MEAN subtraction (:75-77).
 * The random draws stay on the host (same np.random calls, same order); the host passes their outcome as
 * window maps.  One axis of a padded + cropped source: resize-source index u in [0, n) is canvas index
 * t = u + off; the canvas holds image data on [lo, hi) at image index t + shift, zeros elsewhere. */
typedef struct vm_crop_axis {
  int32_t n, off, lo, hi, shift;
} vm_crop_axis;

typedef struct vm_loader_sample {
  const uint8_t* fg;   /* foreground BGRA u8 [fg_h, fg_w, 4] (reader.read_fg_img: BGR + alpha), 4-byte aligned */
  const uint8_t* prev; /* previous frame BGRA u8 [prev_h, prev_w, 4] (its alpha is warped) or NULL */
  const float* flow;   /* backward flow f32 [fg_h, fg_w, 2] (reader.read_flow), 8-byte aligned, or NULL */
  const uint8_t* bg;   /* background BGR u8 [bg_h, bg_w, 3] (cv2.imread) */
  int32_t fg_h, fg_w, prev_h, prev_w, bg_h, bg_w;
  vm_crop_axis fg_rows, fg_cols, bg_rows, bg_cols;
  int32_t mirror;      /* get_batch rd_mirror: flip this sample's outputs left-right (loader.py:105-109) */
  int32_t reserved;
} vm_loader_sample;

enum vm_loader_plane { VM_LOADER_CMP = 0, VM_LOADER_BG = 1, VM_LOADER_LABEL = 2, VM_LOADER_WARPED = 3,
                       VM_LOADER_FG = 4 };

/* Output planes [n, out_h, out_w, *] (NULL = not produced); element (i, y, x, k) of plane p is at
 * ptr[p][((i*out_h + y)*out_w + x)*pixstride[p] + k].  cmp, bg: 3 channels, mean-subtracted; label: 1 channel
 * (alpha); warped: 3 identical channels (loader.py:293); fg: 3 channels, the resized raw foreground. */
typedef struct vm_loader_outputs {
  void* ptr[5];
  int32_t pixstride[5];
  int32_t reserved;
} vm_loader_outputs;

/* samples: HOST array of n descriptors whose image pointers are device pointers; validated, then uploaded into
 * work (device, vm_loader_workspace_bytes(n) bytes) on `stream`.  dtype VM_F32 or VM_F64 (float64 = the
 * reference's values bit for bit).  Output size (out_h, out_w) = (input_size[1], input_size[0]). */
size_t vm_loader_workspace_bytes(int n);
int vm_loader_compose(const vm_loader_sample* samples, int n, int out_h, int out_w, int dtype,
                      const vm_loader_outputs* out, void* work, void* stream);

/* ---------------------------------------------------------------- augmentation
 * tps.py (thin-plate-spline warp) and augmentation.py (augment's per-pixel work).  The TPS coefficient solve
 * (tps._make_warp's 28x28 pinv, tps.py:110-115) and the np.random draws stay on the host, as in the reference;
 * the per-pixel evaluation, resampling and colour work run here. */

/* tps._make_inverse_warp's grid evaluation (tps.py:41-51 with tps._calculate_f, tps.py:100-108):
 * grid[c][i][j] = a1_c + ax_c*x_i + ay_c*y_j + sum_k w_kc * U(|(x_i, y_j) - P_k|), U(r) = (r*r)*log(r) (0 below
 * 1e-100, tps.py:80-81), x_i = i*x_step + x_lo, y_j = j*y_step + y_lo (np.mgrid).  points [npts,2] and coeffs
 * [npts+3,2] (w_k rows, then a1, ax, ay) are DEVICE f64; grid is DEVICE f64 [2, nx, ny]. */
int vm_tps_grid(const double* points, const double* coeffs, int npts, int nx, int ny, double x_lo, double x_step,
                double y_lo, double y_step, double* grid, void* stream);

/* The inverse map tps.warp_images samples with.  upsample = 0 (approximate_grid == 1): the grid is the map and the
 * output is nx x ny.  upsample = 1: the output is (x_span+1) x (y_span+1) (x_span = x_max - x_min) and each pixel's
 * map is the bilinear upsampling of tps.py:55-74 with x_steps = (x_max - x_min) / approximate_grid. */
typedef struct vm_tps_map {
  const double* grid;
  int32_t nx, ny;
  int32_t upsample;
  int32_t x_span, y_span;
  int32_t reserved;
  double x_steps, y_steps;
} vm_tps_map;

/* tps.warp_images' resampling (tps.py:34): scipy.ndimage.map_coordinates(plane, map, order) with mode 'constant'
 * (cval 0) on `cn` interleaved planes.  img [ih, iw, cn] and out [oh, ow, cn] of dtype VM_U8 / VM_F32 / VM_F64
 * (integer outputs round as scipy does: (type)(t + 0.5)).  order 0 or 1. */
int vm_tps_sample(const vm_tps_map* map, const void* img, int ih, int iw, int cn, int dtype, int order, void* out,
                  void* stream);

/* cv2.warpAffine(src, M, (w, h)) with INTER_LINEAR, BORDER_CONSTANT 0 (augmentation.py:58-61): m is the FORWARD
 * 2x3 matrix (HOST, 6 doubles), inverted in double as warpAffine does.  src [ih, iw, cn], dst [h, w, cn], dtype
 * VM_U8 (15-bit fixed-point weights), VM_F32 or VM_F64 (float table weights). */
int vm_warp_affine(const void* src, int ih, int iw, int cn, int dtype, const double* m, void* dst, int h, int w,
                   void* stream);
/* augmentation.warp_image without its TPS part (augmentation.py:59-63): cv2.warpAffine by the integer translation
 * [[1,0,tu],[0,1,tv]] to (w, h), then cv2.warpAffine by m (the forward getRotationMatrix2D, inverted as warpAffine
 * does) to (w, h) — fused into one pass, bit-identical to the two vm_warp_affine calls (the translation's fixed-point
 * fraction is zero, so its output is src shifted with zero fill).  lut (optional, u8 BGR only): then
 * change_illumination (augmentation.py:86-98, 133-134) with that S/V map, as vm_change_illumination_u8. */
int vm_warp_image(const void* src, int ih, int iw, int cn, int dtype, int tu, int tv, const double* m,
                  const uint8_t* lut, void* dst, int h, int w, void* stream);

/* augmentation.change_illumination (augmentation.py:86-98): cvtColor BGR2HSV (uint8, hrange 180), S and V through
 * lut (HOST, 256 bytes: lut[u] = uint8(255 * clip(a * (u/255.)**b + c, 0, 1)), built by the caller with the
 * reference's float64 arithmetic), cvtColor HSV2BGR.  bgr / out: device uint8 [pixels, 3]. */
int vm_change_illumination_u8(const uint8_t* bgr, long pixels, const uint8_t* lut, uint8_t* out, void* stream);

/* augmentation.object_size / fg_center (augmentation.py:10-20): stats (device int64[3]) = number of nonzero
 * alpha pixels, sum of their row indices, sum of their column indices.  alpha [h, w] VM_F64 / VM_F32 / VM_U8. */
int vm_nonzero_stats(const void* alpha, int h, int w, int dtype, long long* stats, void* stream);

/* augmentation.augmentation's BGRA frame (augmentation.py:154-155, 162-163): out[p] = [fg B, G, R,
 * uint8(255. * alpha[p])] (the product in the alpha's precision, f64 / f32, truncated like numpy's astype). */
int vm_bgra_u8(const uint8_t* fg, const void* alpha, int alpha_dtype, long pixels, uint8_t* out, void* stream);

/* augmentation.augment (augmentation.py:101-135) for a batch of samples in four launches per 4 samples (the
 * config-5 pipeline, vmatting.augmentation.augment_many): per sample the TPS lattice of tps._make_inverse_warp
 * (output region (0, 0, h, w), approximate_grid 2), ONE resampling pass for the fg planes and the alpha through its
 * upsampled map (tps.warp_images, order 1), the fused translate + similarity warps (vm_warp_image) of the background
 * (its own size, camera motion) and of the resampled fg / alpha (object motion), and change_illumination with the
 * sample's S/V map on fg and bg (the fg and alpha object-motion warps share one pass, which can also write the
 * BGRA frame).  Bit-identical to the per-sample entry points.  The np.random draws, the TPS solve
 * and the maps stay on the host (the caller's), as in vm_tps_grid / vm_warp_image. */
typedef struct vm_augment_job {
  const uint8_t* fg;        /* [h, w, 3] u8 BGR (device) */
  const uint8_t* bg;        /* [bg_h, bg_w, 3] u8 BGR */
  const double* alpha;      /* [h, w] f64 */
  const double* tps_points; /* [npts, 2] f64 (device): the deformed landmarks, the reverse map's from-points */
  const double* tps_coeffs; /* [npts + 3, 2] f64 (device): their solve, tps._make_warp (pinv(L) @ [landmarks; 0]) */
  void* scratch;            /* vm_augment_scratch_bytes(h, w) device bytes (lattice, resampled fg and alpha) */
  uint8_t* new_fg;          /* [h, w, 3] u8 */
  uint8_t* new_bg;          /* [bg_h, bg_w, 3] u8 */
  double* new_alpha;        /* [h, w] f64 */
  uint8_t* new_bgra;        /* optional [h, w, 4] u8: the augmented frame as augmentation.augmentation writes it
                             * (augmentation.py:162-163, vm_bgra_u8 of new_fg and new_alpha); NULL: not written */
  int32_t h, w, bg_h, bg_w, npts;
  int32_t tu_bg, tv_bg, tu_fg, tv_fg;
  int32_t reserved;
  double m_bg[6];           /* the forward getRotationMatrix2D matrices (host values), inverted as warpAffine does */
  double m_fg[6];
  uint8_t lut[256];         /* change_illumination's S/V map (augmentation.py:89-95), shared by fg and bg */
} vm_augment_job;
size_t vm_augment_scratch_bytes(int h, int w);
int vm_augment_batch(const vm_augment_job* jobs, int n, void* stream);

/* vm_bgra_u8 for n (fg u8 [px, 3], f64 alpha [px]) pairs (host arrays of device pointers) in one launch per 8. */
int vm_bgra_u8_batch(const uint8_t* const* fg, const double* const* alpha, const long* pixels, uint8_t* const* out,
                     int n, void* stream);

/* vm_nonzero_stats for n f64 alphas (host arrays of device pointers and sizes) in one launch per 8: stats is device
 * int64 [n][3] (count, row-index sum, column-index sum per alpha). */
int vm_nonzero_stats_batch(const double* const* alphas, const int* h, const int* w, int n, long long* stats,
                           void* stream);

/* data.trimap_from_matte (data.py:37-67; the reference uses dilate 1, crop 3): trimap u8 [h, w] from a float64
 * matte [h, w] (device), 255 / 0 where the matte is exactly 1 / 0, 128 elsewhere and — reproducing the reference's
 * raster-order overwrites — on 1-pixels (0-pixels) with a non-0/1 pixel later in raster order within crop (dilate)
 * in the max-norm.  dilate, crop <= 8. */
int vm_trimap_from_matte(const double* matte, int h, int w, int dilate, int crop, uint8_t* trimap, void* stream);

/* ---------------------------------------------------------------- training step (config 5)
 * Backward of train.py's loss through UNetSimple's trainable layers and tf.train.AdamOptimizer
 * (train.py:288-343 video_procedure, 176-227 simple_procedure; unet_simple.py:19-42,116-142).  Gradients are f32;
 * forward activations (x, y views) may be f32 or bf16. */

/* dL/dlogits for alpha = sigmoid(logits) (unet_simple.py:142) under train.py:294-298's loss
 * (regular_l1 train.py:21-28, composite :14-18); pred/gt [P], raw_fg/bg/cmp [P,3] f32 device; dlogits [P]. */
int vm_matting_loss_backward(const float* pred, const float* gt, const float* raw_fg, const float* bg, const float* cmp,
                             long pixels, float* dlogits, void* stream);

/* Workspace of vm_bn_backward_nhwc for a c-channel view. */
size_t vm_bn_backward_workspace_bytes(int channels);

/* Gradient of tf.contrib.layers.batch_norm(is_training=True) (unet_simple.py:25,41) w.r.t. its input x, gamma and
 * beta, given dy (f32) = dL/d(BN output); y (optional) = the relu output that followed the BN (unet_simple.py:120-141:
 * tf.nn.relu(new_conv(...))), so g = dy * (y > 0).  mean/var: the batch statistics the forward normalised with.
 * x == NULL: only dbeta = sum(g) (a bias gradient: the channel sum of dy).  dx / dgamma / dbeta may be NULL. */
int vm_bn_backward_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                        const float* var, const float* gamma, float eps, vm_tensor* dx, float* dgamma, float* dbeta,
                        void* work, void* stream);
/* The same with dx2 (optional, may be NULL): a second copy of dx in dx2's dtype (the bf16 operand of the
 * data-gradient conv in the bf16 training path, written in the same pass); dbias (optional, needs x): the
 * gradient of a bias added before the BN (new_conv's conv bias, unet_simple.py:23-25) = sum of dx over the
 * pixels, from the same double sums (zero in exact arithmetic). */
int vm_bn_backward_ex_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                           const float* var, const float* gamma, float eps, vm_tensor* dx, vm_tensor* dx2,
                           float* dgamma, float* dbeta, float* dbias, void* work, void* stream);

/* The input-gradient pass of vm_bn_backward_ex_nhwc alone, with the two channel sums given: sum_g = sum(g),
 * sum_gx = sum(g * xhat) over `count` pixels.  SyncBN (DDP with statistics over the global batch, the single-device
 * reference's unet_simple.py:25,41 normalisation): each replica takes its local sums (vm_bn_backward_ex_nhwc with
 * dx NULL), all-reduces them, and applies them here with count = all replicas' pixels. */
int vm_bn_backward_apply_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                              const float* var, const float* gamma, float eps, const float* sum_g,
                              const float* sum_gx, long count, vm_tensor* dx, vm_tensor* dx2, void* stream);

/* tf.nn.relu gradient: dx = dy * (y > 0); dx f32. */
int vm_relu_backward_nhwc(const vm_tensor* dy, const vm_tensor* y, vm_tensor* dx, void* stream);
/* The same with an optional second (e.g. bf16) copy of dx. */
int vm_relu_backward_ex_nhwc(const vm_tensor* dy, const vm_tensor* y, vm_tensor* dx, vm_tensor* dx2, void* stream);
/* The same over a decoder level's concat in one pass (upconv_concat, unet_simple.py:30-42): channels [0, split) of
 * the gradient go to dx_lo [n,h,w,split] (f32: the select convs' already-masked gradients, read densely by their
 * BN backward), channels [split, c) to dx [n,h,w,c-split] and optionally dx2 (the upconv's).  0 < split < c, or
 * split 0 with dx_lo NULL (= vm_relu_backward_ex_nhwc). */
int vm_relu_backward_split_nhwc(const vm_tensor* dy, const vm_tensor* y, int split, vm_tensor* dx_lo, vm_tensor* dx,
                                vm_tensor* dx2, void* stream);

/* Adjoint of vm_maxpool2x2_same_nhwc (tf.nn.max_pool 2x2/2 SAME: small.py:40,42; unet.py:32-33): x is the pool's
 * input [n,h,w,c] (any dtype), dy its output gradient [n,ceil(h/2),ceil(w/2),c]; dx [n,h,w,c] (f32 or bf16)
 * = add + the window gradient at the window's first maximum in row-major order (TF MaxPoolGrad's tie rule), 0
 * elsewhere.  add (optional, may alias dx): a gradient reaching x by another path (small.py:20's skip concat). */
int vm_maxpool2x2_backward_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* add, vm_tensor* dx,
                                void* stream);

/* The front end of a relu conv's backward (train.py training_procedure through unet.py's y = relu(conv(x) + b),
 * :35-42,65-74): dz = (y > 0) * g written as dz (e.g. the bf16 copy the filter / data-gradient convs read) and the
 * bias gradient dbias[c] = sum_p dz (f64 partials, fixed-order fold) from one pass.  g = dy (+ add) when dy is y's
 * shape; when dy is the 2x2 SAME pool's shape, g = add (optional) + tf.nn.max_pool's adjoint of dy (the window's
 * first maximum of y in row-major order, TF MaxPoolGrad) — the skip half of an [up, skip] concat (unet.py:62) and its
 * pool in one pass.  dy / add f32; y any dtype; work = vm_relu_backward_bias_workspace_bytes(c). */
size_t vm_relu_backward_bias_workspace_bytes(int channels);
int vm_relu_backward_bias_nhwc(const vm_tensor* dy, const vm_tensor* y, const vm_tensor* add, vm_tensor* dz,
                               float* dbias, void* work, void* stream);

/* Adjoint of vm_resize_bilinear_tf1_nhwc (tf.image.resize_images, unet_simple.py:33): dy [n,oh,ow,c] (f32 or bf16
 * view) -> dx contiguous f32 [n,ih,iw,c] (overwritten). */
int vm_resize_bilinear_tf1_backward(const vm_tensor* dy, float* dx, int ih, int iw, void* stream);
/* The same with dx a dense view [n,ih,iw,c]: f32, or bf16 (c % 4 == 0; each f32 sum rounded once to nearest even). */
int vm_resize_bilinear_tf1_backward_nhwc(const vm_tensor* dy, vm_tensor* dx, void* stream);

/* Workspace of vm_conv3x3_wgrad_nhwc (per-block partial filter gradients, <= 64 MiB). */
size_t vm_conv3x3_wgrad_workspace_bytes(int n, int h, int w, int cin, int cout);

/* Weight gradient of the 3x3 SAME conv (tf.nn.conv2d, unet_simple.py:23,35): dw[3][3][cin][cout] (HWIO, f32) +=
 * sum over pixels of x (view, cin = x->c) patch x dy (f32 view [n,h,w,cout]); cout <= 48.  Accumulates;
 * deterministic (fixed-order two-pass sum through ``work``). */
int vm_conv3x3_wgrad_nhwc(const vm_tensor* x, const vm_tensor* dy, float* dw, void* work, void* stream);
/* The weight gradient with options: x_src_c > 0 reads x as x->c / x_src_c sources of x_src_c channels each,
 * source s at x_src_stride elements from the view base (the frozen towers' features stored tower-major,
 * unet_simple.py:153-168's concat); mode 0 = the exact-f32 FMA kernel above, mode 1 = MFMA with bf16 operands
 * (x a bf16 view of 16-byte channel chunks, dy rounded to bf16 on load, f32 sums; the bf16 training path).
 * cout <= 48; dw += result; work: vm_conv3x3_wgrad_ex_workspace_bytes(..., mode) bytes. */
size_t vm_conv3x3_wgrad_ex_workspace_bytes(int n, int h, int w, int cin, int cout, int mode);
int vm_conv3x3_wgrad_ex_nhwc(const vm_tensor* x, int x_src_c, long x_src_stride, const vm_tensor* dy, float* dw,
                             void* work, int mode, void* stream);

/* The data-gradient filter of a 3x3 SAME conv: w_flipped[kh][kw][co][ci] = w[2-kh][2-kw][ci][co]; dx is then
 * vm_conv3x3_nhwc(dy, pack(w_flipped)). */
int vm_conv3x3_flip_weights(const float* w_hwio, int cin, int cout, float* w_flipped, void* stream);

/* tf.train.AdamOptimizer's ApplyAdam (train.py:302-304) over n f32 values, g = grad * grad_scale:
 * m += (g - m)(1 - beta1); v += (g^2 - v)(1 - beta2); var -= m * lr_t / (sqrt(v) + eps), with the caller's
 * lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t). */
int vm_adam_tf(float* var, float* m, float* v, const float* grad, long n, float lr_t, float beta1, float beta2,
               float eps, float grad_scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VMATTING_H */
