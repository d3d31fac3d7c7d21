// Training-sample preprocessing of the reference's loader (loader.py:39-85 load_and_crop,
// :119-157 simple_load_crop, :285-330 video_load_crop, and the batch loops :93-116, 160-171, 333-345)
// after image decoding: pad/crop windows, the previous-alpha optical-flow warp, cv2.resize to the
// network size, compositing and VGG-mean subtraction, for a whole batch in one launch.
//
// One thread per output pixel (grid.y = sample).  Each thread gathers the 1, 2x2 or 2x2-block source
// pixels its resize needs straight from the decoded u8 images (foreground BGRA, background BGR,
// previous-frame alpha + flow for the warp) through the crop/pad window maps, so the padded canvases,
// the crops, the full-frame warp of the previous alpha (loader.py:292) and the float64 copies the
// reference allocates never exist.  HBM traffic is the decoded bytes the windows touch plus the outputs.
//
// Arithmetic is float64 with float32 resize coefficients, operation for operation as OpenCV's
// resize/remap and numpy's compositing; this file is compiled with -ffp-contract=off (no fused
// multiply-adds), so the f64 outputs are bit-identical to oracle/loader.py and the f32 outputs are
// those values rounded once.

#include <cfloat>

#include <type_traits>

#include "vm_common.h"

namespace vm {
namespace {

template <int C>
struct Vd {
  double v[C];
};

template <int C>
__device__ __forceinline__ Vd<C> vscale(Vd<C> a, double s) {
#pragma unroll
  for (int k = 0; k < C; ++k) a.v[k] = a.v[k] * s;
  return a;
}

template <int C>
__device__ __forceinline__ Vd<C> vsum(Vd<C> a, const Vd<C>& b) {
#pragma unroll
  for (int k = 0; k < C; ++k) a.v[k] = a.v[k] + b.v[k];
  return a;
}

// OpenCV resize(): scale = 1 / ((double)dsize / ssize); the INTER_LINEAR -> INTER_AREA switch needs both
// scales to be exactly the integer 2 (|scale - cvRound(scale)| < DBL_EPSILON).
__device__ __forceinline__ bool area2(int n, int dn) {
  const double scale = 1.0 / ((double)dn / (double)n);
  const double is = rint(scale);
  return fabs(scale - is) < DBL_EPSILON && is == 2.0;
}

// cv2.resize(src, (ow, oh), INTER_LINEAR) of a float64 image at output pixel (dy, dx); fetch(r, c) returns the
// source pixel.  Paths as OpenCV 3.x imgproc/resize.cpp: copy when sizes match; the area fast path for an exact
// 2x reduction (sum = ((a + b) + c) + d over the row-major 2x2 block, times 0.25f); otherwise HResizeLinear
// (columns: coefficient pair in float, s < 0 -> (0, 0), s >= n-1 -> copied column) then VResizeLinear (rows
// clamped, coefficients kept).
template <int C, typename F>
__device__ Vd<C> cv_resize_at(const F& fetch, int sh, int sw, int oh, int ow, int dy, int dx) {
  if (sh == oh && sw == ow) return fetch(dy, dx);
  if (area2(sw, ow) && area2(sh, oh)) {
    const int y = 2 * dy, x = 2 * dx;
    Vd<C> s = vsum(vsum(vsum(fetch(y, x), fetch(y, x + 1)), fetch(y + 1, x)), fetch(y + 1, x + 1));
    return vscale(s, 0.25);
  }
  const double scx = 1.0 / ((double)ow / (double)sw);
  float fx = (float)((dx + 0.5) * scx - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) {
    fx = 0.f;
    sx = 0;
  }
  const bool single = sx + 1 >= sw;
  if (sx >= sw - 1) {
    fx = 0.f;
    sx = sw - 1;
  }
  const double a0 = (double)(1.f - fx), a1 = (double)fx;
  const double scy = 1.0 / ((double)oh / (double)sh);
  float fy = (float)((dy + 0.5) * scy - 0.5);
  const int sy = (int)floorf(fy);
  fy -= (float)sy;
  const int r0 = min(max(sy, 0), sh - 1), r1 = min(max(sy + 1, 0), sh - 1);
  const double b0 = (double)(1.f - fy), b1 = (double)fy;
  auto hrow = [&](int r) -> Vd<C> {
    if (single) return fetch(r, sx);
    return vsum(vscale(fetch(r, sx), a0), vscale(fetch(r, sx + 1), a1));
  };
  return vsum(vscale(hrow(r0), b0), vscale(hrow(r1), b1));
}

// resize-source index u along one axis -> image index, or -1 where the padded canvas is zero
__device__ __forceinline__ int axis_map(const vm_crop_axis& a, int u) {
  const int t = u + a.off;
  return (t >= a.lo && t < a.hi) ? t + a.shift : -1;
}

// cv2.remap(prev_alpha, identity + flow, INTER_LINEAR) at image pixel (y, x) for a float64 image (flow.py:9-18):
// X = cvRound(mx * 32), integer part X >> 5, table weights (exact products of k/32, float), taps TL, TR, BL, BR
// summed in that order in float64, a tap outside the previous frame reads 0.
__device__ __forceinline__ double warp_prev_alpha(const vm_loader_sample& s, int y, int x) {
  const float2 fl = reinterpret_cast<const float2*>(s.flow)[(long)y * s.fg_w + x];
  const float mx = (float)x + fl.x, my = (float)y + fl.y;
  const float lim = 1073741824.f;  // |X| < 2^30: anything that far out reads zeros anyway (NaN -> -2^30)
  const int X = (int)fminf(fmaxf(rintf(mx * 32.f), -lim), lim);
  const int Y = (int)fminf(fmaxf(rintf(my * 32.f), -lim), lim);
  const int x0 = X >> 5, y0 = Y >> 5;
  const float fx = (float)(X & 31) * (1.f / 32.f), fy = (float)(Y & 31) * (1.f / 32.f);
  auto tap = [&](int yy, int xx) -> double {
    if ((unsigned)yy >= (unsigned)s.prev_h || (unsigned)xx >= (unsigned)s.prev_w) return 0.0;
    return (double)s.prev[((long)yy * s.prev_w + xx) * 4 + 3] / 255.0;
  };
  double acc = tap(y0, x0) * (double)((1.f - fy) * (1.f - fx));
  acc = acc + tap(y0, x0 + 1) * (double)((1.f - fy) * fx);
  acc = acc + tap(y0 + 1, x0) * (double)(fy * (1.f - fx));
  acc = acc + tap(y0 + 1, x0 + 1) * (double)(fy * fx);
  return acc;
}

__device__ __forceinline__ double vgg_mean(int k) { return k == 0 ? 103.939 : (k == 1 ? 116.779 : 123.68); }

template <typename T>
__device__ __forceinline__ void put(void* base, long pix, int stride, int k, double v) {
  reinterpret_cast<T*>(base)[pix * stride + k] = (T)v;
}

// up to kLoaderJobs descriptors travel by value in the kernel arguments (no upload copy per batch)
constexpr int kLoaderJobs = 8;
struct LoaderJobs {
  vm_loader_sample s[kLoaderJobs];
};

template <typename T, typename SRC>
__global__ __launch_bounds__(256) void loader_compose_kernel(SRC samples, int oh, int ow, vm_loader_outputs out) {
  const vm_loader_sample& s = [&]() -> const vm_loader_sample& {
    if constexpr (std::is_same_v<SRC, LoaderJobs>) return samples.s[blockIdx.y];
    else return samples[blockIdx.y];
  }();
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= oh * ow) return;
  const int dy = p / ow, dxo = p - dy * ow;
  const int dx = s.mirror ? ow - 1 - dxo : dxo;  // get_batch rd_mirror: np.flip(axis=1) of the outputs

  // foreground stack of the (padded) crop: B, G, R, alpha, warped previous alpha
  auto fg_fetch = [&](int r, int c) -> Vd<5> {
    Vd<5> o = {{0.0, 0.0, 0.0, 0.0, 0.0}};
    const int y = axis_map(s.fg_rows, r), x = axis_map(s.fg_cols, c);
    if (y < 0 || x < 0) return o;
    const uchar4 q = *reinterpret_cast<const uchar4*>(s.fg + ((long)y * s.fg_w + x) * 4);
    o.v[0] = (double)q.x;
    o.v[1] = (double)q.y;
    o.v[2] = (double)q.z;
    o.v[3] = (double)q.w / 255.0;  // reader.py:16
    if (s.prev) o.v[4] = warp_prev_alpha(s, y, x);
    return o;
  };
  auto bg_fetch = [&](int r, int c) -> Vd<3> {
    Vd<3> o = {{0.0, 0.0, 0.0}};
    const int y = axis_map(s.bg_rows, r), x = axis_map(s.bg_cols, c);
    if (y < 0 || x < 0) return o;
    const uint8_t* q = s.bg + ((long)y * s.bg_w + x) * 3;
    o.v[0] = (double)q[0];
    o.v[1] = (double)q[1];
    o.v[2] = (double)q[2];
    return o;
  };
  const Vd<5> f = cv_resize_at<5>(fg_fetch, s.fg_rows.n, s.fg_cols.n, oh, ow, dy, dx);
  const Vd<3> b = cv_resize_at<3>(bg_fetch, s.bg_rows.n, s.bg_cols.n, oh, ow, dy, dx);

  const long pix = (long)blockIdx.y * oh * ow + (long)dy * ow + dxo;
  const double a = f.v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double cmp = a * f.v[k] + (1.0 - a) * b.v[k];  // reader.py:78
    if (out.ptr[VM_LOADER_CMP]) put<T>(out.ptr[VM_LOADER_CMP], pix, out.pixstride[VM_LOADER_CMP], k, cmp - vgg_mean(k));
    if (out.ptr[VM_LOADER_BG]) put<T>(out.ptr[VM_LOADER_BG], pix, out.pixstride[VM_LOADER_BG], k, b.v[k] - vgg_mean(k));
    if (out.ptr[VM_LOADER_FG]) put<T>(out.ptr[VM_LOADER_FG], pix, out.pixstride[VM_LOADER_FG], k, f.v[k]);
    if (out.ptr[VM_LOADER_WARPED]) put<T>(out.ptr[VM_LOADER_WARPED], pix, out.pixstride[VM_LOADER_WARPED], k, f.v[4]);
  }
  if (out.ptr[VM_LOADER_LABEL]) put<T>(out.ptr[VM_LOADER_LABEL], pix, out.pixstride[VM_LOADER_LABEL], 0, a);
}

// every image index an axis can produce lies inside the image
bool axis_ok(const vm_crop_axis& a, int img_n) {
  if (a.n <= 0 || a.lo < 0 || a.hi < a.lo) return false;
  const long t0 = a.off > a.lo ? a.off : a.lo;
  const long t1 = (long)a.off + a.n < a.hi ? (long)a.off + a.n : a.hi;  // exclusive
  if (t0 >= t1) return true;                                            // the window sees only zeros
  return t0 + a.shift >= 0 && t1 - 1 + a.shift < img_n;
}

}  // namespace
}  // namespace vm

using namespace vm;

extern "C" size_t vm_loader_workspace_bytes(int n) { return n > 0 ? (size_t)n * sizeof(vm_loader_sample) : 0; }

extern "C" int vm_loader_compose(const vm_loader_sample* samples, int n, int out_h, int out_w, int dtype,
                                 const vm_loader_outputs* out, void* work, void* stream) {
  if (!samples || n <= 0 || out_h <= 0 || out_w <= 0 || !out || !work || (dtype != VM_F32 && dtype != VM_F64))
    return fail(VM_EINVAL, "loader_compose: bad argument");
  static const int nch[5] = {3, 3, 1, 3, 3};
  for (int o = 0; o < 5; ++o)
    if (out->ptr[o] && out->pixstride[o] < nch[o]) return fail(VM_EINVAL, "loader_compose: output %d stride", o);
  for (int i = 0; i < n; ++i) {
    const vm_loader_sample& s = samples[i];
    if (!s.fg || !s.bg || s.fg_h <= 0 || s.fg_w <= 0 || s.bg_h <= 0 || s.bg_w <= 0)
      return fail(VM_EINVAL, "loader_compose: sample %d: missing image", i);
    if (reinterpret_cast<uintptr_t>(s.fg) % 4) return fail(VM_EUNSUPPORTED, "loader_compose: fg must be 4-byte aligned");
    if ((s.prev == nullptr) != (s.flow == nullptr))
      return fail(VM_EINVAL, "loader_compose: sample %d: prev and flow go together", i);
    if (out->ptr[VM_LOADER_WARPED] && !s.prev)
      return fail(VM_EINVAL, "loader_compose: warped output needs prev/flow (sample %d)", i);
    if (s.prev && (s.prev_h <= 0 || s.prev_w <= 0 || reinterpret_cast<uintptr_t>(s.flow) % 8))
      return fail(VM_EINVAL, "loader_compose: sample %d: bad previous frame / flow", i);
    if (!axis_ok(s.fg_rows, s.fg_h) || !axis_ok(s.fg_cols, s.fg_w) || !axis_ok(s.bg_rows, s.bg_h) ||
        !axis_ok(s.bg_cols, s.bg_w))
      return fail(VM_EINVAL, "loader_compose: sample %d: crop window outside the image", i);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((out_h * out_w + 255) / 256, n);
  if (n <= kLoaderJobs) {  // the descriptors by value: one launch, no upload
    LoaderJobs J{};
    for (int i = 0; i < n; ++i) J.s[i] = samples[i];
    if (dtype == VM_F32)
      hipLaunchKernelGGL((loader_compose_kernel<float, LoaderJobs>), grid, dim3(256), 0, st, J, out_h, out_w, *out);
    else
      hipLaunchKernelGGL((loader_compose_kernel<double, LoaderJobs>), grid, dim3(256), 0, st, J, out_h, out_w, *out);
    return check_launch("loader_compose");
  }
  hipError_t e = hipMemcpyAsync(work, samples, (size_t)n * sizeof(vm_loader_sample), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return fail(VM_EHIP, "loader_compose: descriptor upload: %s", hipGetErrorString(e));
  const auto* dev = reinterpret_cast<const vm_loader_sample*>(work);
  if (dtype == VM_F32)
    hipLaunchKernelGGL((loader_compose_kernel<float, const vm_loader_sample*>), grid, dim3(256), 0, st, dev, out_h,
                       out_w, *out);
  else
    hipLaunchKernelGGL((loader_compose_kernel<double, const vm_loader_sample*>), grid, dim3(256), 0, st, dev, out_h,
                       out_w, *out);
  return check_launch("loader_compose");
}
