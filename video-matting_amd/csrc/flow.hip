// Two-frame temporal path: optical-flow backward warp (flow.warp_img / warp_bgr) and the
// forward/backward consistency mask (flow.correct_alpha).  Gather-bound: one thread per output
// pixel, coalesced reads of the flow field and the output, L2-served bilinear taps.

#include "vm_common.h"

namespace vm {

// cv2.remap(img, identity+flow (CV_32FC2), None, INTER_LINEAR), BORDER_CONSTANT 0 (flow.py:12-18).
// mode 0 (OpenCV): X = cvRound(x*32) (round-half-even), integer X>>5, fraction (X&31)/32, weights from
// the 32x32 table (exact products of k/32), taps summed TL,TR,BL,BR; a tap outside the frame reads 0.
// mode 1: exact bilinear on the float coordinate.
__global__ void remap_f32_kernel(const float* __restrict__ img, int ih, int iw, const float* __restrict__ flow, int h,
                                 int w, int nfr, float* __restrict__ out, int mode) {
  const long per = (long)h * w;
  const long total = per * nfr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long f = i / per;
    const long pi = i - f * per;
    const int y = (int)(pi / w), x = (int)(pi - (long)y * w);
    const float2 fl = reinterpret_cast<const float2*>(flow)[i];
    const float mx = (float)x + fl.x;  // (identity + flow).astype(float32): one rounding
    const float my = (float)y + fl.y;
    int x0, y0;
    float fx, fy;
    if (mode == 0) {
      const int X = (int)rintf(mx * 32.f);
      const int Y = (int)rintf(my * 32.f);
      x0 = X >> 5;
      y0 = Y >> 5;
      fx = (float)(X & 31) * (1.f / 32.f);
      fy = (float)(Y & 31) * (1.f / 32.f);
    } else {
      const float flx = floorf(mx), fly = floorf(my);
      x0 = (int)flx;
      y0 = (int)fly;
      fx = mx - flx;
      fy = my - fly;
    }
    const float* im = img + f * (long)ih * iw;
    auto tap = [&](int yy, int xx) -> float {
      return ((unsigned)yy < (unsigned)ih && (unsigned)xx < (unsigned)iw) ? im[(long)yy * iw + xx] : 0.f;
    };
    const float w00 = (1.f - fy) * (1.f - fx), w01 = (1.f - fy) * fx, w10 = fy * (1.f - fx), w11 = fy * fx;
    float s = tap(y0, x0) * w00;
    s += tap(y0, x0 + 1) * w01;
    s += tap(y0 + 1, x0) * w10;
    s += tap(y0 + 1, x0 + 1) * w11;
    out[i] = s;
  }
}

// uint8 planes (flow.py:29-31): 15-bit integer weights (32-fy)(32-fx)*32 etc. (exact), (sum + 2^14) >> 15.
__global__ void remap_u8_kernel(const uint8_t* __restrict__ img, int ih, int iw, int cn, const float* __restrict__ flow,
                                int h, int w, uint8_t* __restrict__ out) {
  const long total = (long)h * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int y = (int)(i / w), x = (int)(i - (long)y * w);
    const float2 fl = reinterpret_cast<const float2*>(flow)[i];
    const int X = (int)rintf(((float)x + fl.x) * 32.f);
    const int Y = (int)rintf(((float)y + fl.y) * 32.f);
    const int x0 = X >> 5, y0 = Y >> 5, ax = X & 31, ay = Y & 31;
    const int w00 = (32 - ay) * (32 - ax) * 32, w01 = (32 - ay) * ax * 32, w10 = ay * (32 - ax) * 32, w11 = ay * ax * 32;
    for (int k = 0; k < cn; ++k) {
      auto tap = [&](int yy, int xx) -> int {
        return ((unsigned)yy < (unsigned)ih && (unsigned)xx < (unsigned)iw) ? (int)img[((long)yy * iw + xx) * cn + k] : 0;
      };
      const int s = tap(y0, x0) * w00 + tap(y0, x0 + 1) * w01 + tap(y0 + 1, x0) * w10 + tap(y0 + 1, x0 + 1) * w11;
      int v = (s + (1 << 14)) >> 15;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      out[i * cn + k] = (uint8_t)v;
    }
  }
}

// flow.correct_alpha (flow.py:41-50): j0 = min(int(bw[i,j,0] + j), w-1), i0 = min(int(bw[i,j,1] + i), h-1)
// (int() truncates toward 0; negative indices wrap numpy-style, below -dim the reference raises IndexError);
// (j1, i1) the same through fw[i0, j0]; alpha[i,j] = 0 where ||(i1 - i, j1 - j)|| > thresh.
template <int PROMOTE>
__device__ __forceinline__ long step_index(float u, long base, long lim) {
  long t;
  if (PROMOTE == 0) t = (long)((double)u + (double)base);  // numpy-1: float64, exact
  else t = (long)(u + (float)base);                         // numpy-2: float32 add
  return t < lim - 1 ? t : lim - 1;
}

// Pass 1 only validates the indices; pass 2 returns early when pass 1 flagged an IndexError, so on
// error alpha is left untouched — as in the reference, where the exception escapes the loop before
// the masked assignment (flow.py:41-50).
template <int PROMOTE>
__global__ void fb_check_kernel(const float* __restrict__ bw, int h, int w, int* err) {
  const long total = (long)h * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / w), c = (int)(i - (long)r * w);
    const float2 b = reinterpret_cast<const float2*>(bw)[i];
    const long j0 = step_index<PROMOTE>(b.x, c, w);
    const long i0 = step_index<PROMOTE>(b.y, r, h);
    if (j0 < -(long)w || i0 < -(long)h) atomicOr(err, 1);
  }
}

template <int PROMOTE>
__global__ void fb_consistency_kernel(const float* __restrict__ bw, const float* __restrict__ fw, int h, int w,
                                      float* __restrict__ alpha, double thresh, const int* err) {
  if (*err) return;
  const long total = (long)h * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / w), c = (int)(i - (long)r * w);
    const float2 b = reinterpret_cast<const float2*>(bw)[i];
    const long j0 = step_index<PROMOTE>(b.x, c, w);
    const long i0 = step_index<PROMOTE>(b.y, r, h);
    const long ji = j0 < 0 ? j0 + w : j0, ii = i0 < 0 ? i0 + h : i0;  // numpy negative-index wrap
    const float2 f = reinterpret_cast<const float2*>(fw)[ii * w + ji];
    const long j1 = step_index<PROMOTE>(f.x, j0, w);
    const long i1 = step_index<PROMOTE>(f.y, i0, h);
    const double di = (double)(i1 - r), dj = (double)(j1 - c);
    if (sqrt(di * di + dj * dj) > thresh) alpha[i] = 0.f;
  }
}

// ---------------------------------------------------------------- config 3: warp + occlusion + refine input
// One pass per pixel of the two-frame chain flow.py's demo runs (flow.py:69-77): alpha_w = warp_img(prev, flow_b)
// (the remap_f32 mode-0 arithmetic above), correct_alpha(flow_b, flow_f, alpha_w) (fb_consistency above: one
// gather of flow_f at the backward target), and the RefineNet input row [cmp B,G,R, alpha_t, alpha_w, 0, 0, 0]
// (refine.py:27, Cin = 5 padded to 8, the concat of SURVEY.md 8(a) a14) written as one 16- or 32-byte NHWC pixel.
// Every value is bit-identical to the separate kernels; the IndexError flag is raised as in fb_check (the caller
// raises before using the output).
template <typename T, int PROMOTE>
__global__ __launch_bounds__(256) void temporal_input_kernel(const float* __restrict__ prev,
                                                             const float* __restrict__ bw,
                                                             const float* __restrict__ fw,
                                                             const float* __restrict__ cmp,
                                                             const float* __restrict__ cur, int h, int w,
                                                             double thresh, T* __restrict__ out,
                                                             float* __restrict__ warped, int* err) {
  const long total = (long)h * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int y = (int)(i / w), x = (int)(i - (long)y * w);
    const float2 fl = reinterpret_cast<const float2*>(bw)[i];
    // warp_img: cv2.remap 1/32-pixel fixed point (remap_f32_kernel, mode 0)
    const int X = (int)rintf(((float)x + fl.x) * 32.f);
    const int Y = (int)rintf(((float)y + fl.y) * 32.f);
    const int x0 = X >> 5, y0 = Y >> 5;
    const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
    auto tap = [&](int yy, int xx) -> float {
      return ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) ? prev[(long)yy * w + xx] : 0.f;
    };
    const float w00 = (1.f - fy) * (1.f - fx), w01 = (1.f - fy) * fx, w10 = fy * (1.f - fx), w11 = fy * fx;
    float a = tap(y0, x0) * w00;
    a += tap(y0, x0 + 1) * w01;
    a += tap(y0 + 1, x0) * w10;
    a += tap(y0 + 1, x0 + 1) * w11;
    // correct_alpha (fb_consistency_kernel)
    const long j0 = step_index<PROMOTE>(fl.x, x, w);
    const long i0 = step_index<PROMOTE>(fl.y, y, h);
    if (j0 < -(long)w || i0 < -(long)h) {
      atomicOr(err, 1);
    } else {
      const long ji = j0 < 0 ? j0 + w : j0, ii = i0 < 0 ? i0 + h : i0;
      const float2 f = reinterpret_cast<const float2*>(fw)[ii * w + ji];
      const long j1 = step_index<PROMOTE>(f.x, j0, w);
      const long i1 = step_index<PROMOTE>(f.y, i0, h);
      const double di = (double)(i1 - y), dj = (double)(j1 - x);
      if (sqrt(di * di + dj * dj) > thresh) a = 0.f;
    }
    if (warped) warped[i] = a;
    float v[8] = {cmp[i * 3], cmp[i * 3 + 1], cmp[i * 3 + 2], cur[i], a, 0.f, 0.f, 0.f};
    if constexpr (sizeof(T) == 2) {
      reinterpret_cast<uint4*>(out)[i] = Chunk<T>::pack(v);
    } else {
      reinterpret_cast<float4*>(out)[2 * i] = make_float4(v[0], v[1], v[2], v[3]);
      reinterpret_cast<float4*>(out)[2 * i + 1] = make_float4(v[4], 0.f, 0.f, 0.f);
    }
  }
}

// ---------------------------------------------------------------- training loss (train.py:14-28, 42-47)
constexpr int LOSS_NBLK = 512;

__global__ __launch_bounds__(256) void loss_partial_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                           const float* __restrict__ fg, const float* __restrict__ bg,
                                                           const float* __restrict__ cmp, long P, double* part) {
  __shared__ double sh[2][256];
  double sa = 0.0, sc = 0.0;
  const float eps2 = 1e-6f * 1e-6f;  // tf.square(tf.constant(1e-6)) in f32
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    const float a = pred[i];
    const float d = a - gt[i];
    sa += sqrtf(d * d + eps2);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float pc = a * fg[i * 3 + k] + (1.f - a) * bg[i * 3 + k];
      const float e = pc - cmp[i * 3 + k];
      sc += sqrtf(e * e + eps2);
    }
  }
  sh[0][threadIdx.x] = sa;
  sh[1][threadIdx.x] = sc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + s];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x * 2] = sh[0][0];
    part[blockIdx.x * 2 + 1] = sh[1][0];
  }
}

// one 256-thread block folds the nblk partial pairs (a fixed tree: deterministic; a single thread's serial walk of
// 1024 dependent loads took 47 us)
__global__ __launch_bounds__(256) void loss_final_kernel(const double* part, int nblk, long P, float* out) {
  __shared__ double sh[2][256];
  double sa = 0.0, sc = 0.0;
  for (int b = threadIdx.x; b < nblk; b += 256) {
    sa += part[2 * b];
    sc += part[2 * b + 1];
  }
  sh[0][threadIdx.x] = sa;
  sh[1][threadIdx.x] = sc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + s];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double la = sh[0][0] / (double)P, lc = sh[1][0] / (3.0 * (double)P);
    out[0] = (float)(0.5 * la + 0.5 * lc);
    out[1] = (float)la;
    out[2] = (float)lc;
  }
}

}  // namespace vm

using namespace vm;

extern "C" int vm_remap_bilinear_f32(const float* img, int ih, int iw, const float* flow, int h, int w, int n,
                                     float* out, int mode, void* stream) {
  if (!img || !flow || !out || ih <= 0 || iw <= 0 || h <= 0 || w <= 0 || n <= 0 || (mode != 0 && mode != 1))
    return fail(VM_EINVAL, "remap_f32: bad argument");
  if (reinterpret_cast<uintptr_t>(flow) % 8) return fail(VM_EUNSUPPORTED, "remap_f32: flow must be 8-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long total = (long)h * w * n;
  hipLaunchKernelGGL(remap_f32_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, img, ih, iw, flow, h, w, n, out,
                     mode);
  return check_launch("remap_f32");
}

extern "C" int vm_remap_bilinear_u8(const uint8_t* img, int ih, int iw, int cn, const float* flow, int h, int w,
                                    uint8_t* out, void* stream) {
  if (!img || !flow || !out || ih <= 0 || iw <= 0 || cn <= 0 || h <= 0 || w <= 0)
    return fail(VM_EINVAL, "remap_u8: bad argument");
  if (reinterpret_cast<uintptr_t>(flow) % 8) return fail(VM_EUNSUPPORTED, "remap_u8: flow must be 8-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(remap_u8_kernel, dim3(grid_for((long)h * w, 256)), dim3(256), 0, st, img, ih, iw, cn, flow, h, w,
                     out);
  return check_launch("remap_u8");
}

extern "C" int vm_fb_consistency(const float* backward, const float* forward, int h, int w, float* alpha, float thresh,
                                 int promote, int* err_flag, void* stream) {
  if (!backward || !forward || !alpha || !err_flag || h <= 0 || w <= 0 || (promote != 0 && promote != 1))
    return fail(VM_EINVAL, "fb_consistency: bad argument");
  if ((reinterpret_cast<uintptr_t>(backward) | reinterpret_cast<uintptr_t>(forward)) % 8)
    return fail(VM_EUNSUPPORTED, "fb_consistency: flows must be 8-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_for((long)h * w, 256);
  if (promote == 0) {
    hipLaunchKernelGGL(fb_check_kernel<0>, dim3(grid), dim3(256), 0, st, backward, h, w, err_flag);
    hipLaunchKernelGGL(fb_consistency_kernel<0>, dim3(grid), dim3(256), 0, st, backward, forward, h, w, alpha,
                       (double)thresh, err_flag);
  } else {
    hipLaunchKernelGGL(fb_check_kernel<1>, dim3(grid), dim3(256), 0, st, backward, h, w, err_flag);
    hipLaunchKernelGGL(fb_consistency_kernel<1>, dim3(grid), dim3(256), 0, st, backward, forward, h, w, alpha,
                       (double)thresh, err_flag);
  }
  return check_launch("fb_consistency");
}

extern "C" int vm_temporal_refine_input(const float* prev_alpha, const float* backward, const float* forward,
                                        const float* cmp, const float* alpha, int h, int w, float thresh, int promote,
                                        void* out, int out_dtype, float* warped, int* err_flag, void* stream) {
  if (!prev_alpha || !backward || !forward || !cmp || !alpha || !out || !err_flag || h <= 0 || w <= 0 ||
      (promote != 0 && promote != 1) || (out_dtype != VM_F32 && out_dtype != VM_BF16))
    return fail(VM_EINVAL, "temporal_refine_input: bad argument");
  if ((reinterpret_cast<uintptr_t>(backward) | reinterpret_cast<uintptr_t>(forward)) % 8 ||
      reinterpret_cast<uintptr_t>(out) % 16)
    return fail(VM_EUNSUPPORTED, "temporal_refine_input: flows 8-byte and out 16-byte aligned");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_for((long)h * w, 256);
#define VM_TEMPORAL(TT, PR)                                                                                           \
  hipLaunchKernelGGL((temporal_input_kernel<TT, PR>), dim3(grid), dim3(256), 0, st, prev_alpha, backward, forward, cmp, \
                     alpha, h, w, (double)thresh, reinterpret_cast<TT*>(out), warped, err_flag)
  if (out_dtype == VM_BF16) {
    if (promote == 0) VM_TEMPORAL(uint16_t, 0); else VM_TEMPORAL(uint16_t, 1);
  } else {
    if (promote == 0) VM_TEMPORAL(float, 0); else VM_TEMPORAL(float, 1);
  }
#undef VM_TEMPORAL
  return check_launch("temporal_refine_input");
}

extern "C" size_t vm_loss_workspace_bytes(long pixels) {
  (void)pixels;
  return (size_t)LOSS_NBLK * 2 * sizeof(double);
}

extern "C" int vm_matting_loss(const float* pred, const float* gt, const float* raw_fg, const float* bg,
                               const float* cmp, long pixels, float* out, void* work, void* stream) {
  if (!pred || !gt || !raw_fg || !bg || !cmp || !out || !work || pixels <= 0)
    return fail(VM_EINVAL, "matting_loss: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nblk = grid_for(pixels, 256, LOSS_NBLK);
  double* part = reinterpret_cast<double*>(work);
  hipLaunchKernelGGL(loss_partial_kernel, dim3(nblk), dim3(256), 0, st, pred, gt, raw_fg, bg, cmp, pixels, part);
  int rc = check_launch("loss_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(256), 0, st, part, nblk, pixels, out);
  return check_launch("loss_final");
}
