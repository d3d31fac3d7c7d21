// Augmentation path: tps.py's thin-plate-spline warp and augmentation.py's
// per-pixel work (warpAffine, HSV illumination change, the foreground statistics).  All of it is gather- or
// HBM-bound integer/f64 work: one thread per output pixel, rows of consecutive threads write consecutive
// pixels (coalesced stores), taps are L2-served gathers.  Built with -ffp-contract=off: every expression is
// evaluated in the reference's order with IEEE rounding at each step (numpy / scipy / OpenCV do not fuse).

#include "vm_common.h"

namespace vm {

// ---------------------------------------------------------------------------------------------------- tps.py

// uint8 HWC outputs: a block's run of 256 consecutive pixels (cn bytes each) is staged in LDS and written back as
// 4-byte stores (one lane per dword) instead of cn scattered byte stores per lane.
constexpr int kRun = 256;

__device__ __forceinline__ void flush_run(uint8_t* __restrict__ dst, const uint8_t* stage, int nbytes) {
  if ((reinterpret_cast<uintptr_t>(dst) & 3) == 0) {
    const int nw = nbytes >> 2;
    for (int t = threadIdx.x; t < nw; t += blockDim.x)
      reinterpret_cast<uint32_t*>(dst)[t] = reinterpret_cast<const uint32_t*>(stage)[t];
    for (int t = (nw << 2) + threadIdx.x; t < nbytes; t += blockDim.x) dst[t] = stage[t];
  } else {
    for (int t = threadIdx.x; t < nbytes; t += blockDim.x) dst[t] = stage[t];
  }
}

// (row, col) of flat pixel i in a row-major [*, w] image: 32-bit unsigned division (callers check total < 2^31);
// a 64-bit divide is a long emulated sequence on CDNA.
__device__ __forceinline__ int row_of(long i, int w) { return (int)((unsigned)i / (unsigned)w); }

// One output pixel per lane.  uint8 outputs go through the LDS run (blockDim.x == kRun, cn <= 8); wider types
// store straight from the lane (consecutive lanes, consecutive pixels).
template <typename T, class F>
__device__ __forceinline__ void for_pixels(long total, int cn, T* __restrict__ out, F&& pixel) {
  if constexpr (sizeof(T) == 1) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kRun * 8];
    for (long base = (long)blockIdx.x * kRun; base < total; base += (long)gridDim.x * kRun) {
      const long i = base + threadIdx.x;
      if (i < total) pixel(i, reinterpret_cast<T*>(stage) + threadIdx.x * cn);
      __syncthreads();
      const long n = total - base < kRun ? total - base : kRun;
      flush_run(reinterpret_cast<uint8_t*>(out) + base * cn, stage, (int)(n * cn));
      __syncthreads();
    }
  } else {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
      pixel(i, out + i * cn);
  }
}

// tps._calculate_f (tps.py:100-108) on the approximate grid of tps._make_inverse_warp (tps.py:41-51):
// x_i = i*x_step + x_lo (np.mgrid), f = a1 + ax*x + ay*y + sum_k w_k * U(r_k), U(r) = (r*r)*log(r), 0 below
// 1e-100 (tps.py:80-81).  Both coordinates share the distance evaluation; each keeps its own accumulator in the
// reference's order.
__device__ __forceinline__ void tps_grid_body(const double* __restrict__ pts, const double* __restrict__ coef,
                                              int npts, int nx, int ny, double x_lo, double x_step, double y_lo,
                                              double y_step, double* __restrict__ grid) {
  const long total = (long)nx * ny;
  const double a1x = coef[2 * npts], a1y = coef[2 * npts + 1];
  const double axx = coef[2 * npts + 2], axy = coef[2 * npts + 3];
  const double ayx = coef[2 * npts + 4], ayy = coef[2 * npts + 5];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ix = row_of(i, ny), iy = (int)(i - (long)ix * ny);
    const double x = (double)ix * x_step + x_lo;
    const double y = (double)iy * y_step + y_lo;
    double sx = 0.0, sy = 0.0;
    for (int k = 0; k < npts; ++k) {
      // U(r) = r^2 log r as d2 * log(d2) / 2 (d2 = r^2): one log and no sqrt per term (the f64 lattice is
      // compute-bound: 13M terms per 1080p sample), contracted to FMAs here only; a few ulp from the reference's
      // sqrt-then-log, far inside the 1e-9 px the map is held to (tests/test_gpu_augment.py)
#pragma clang fp contract(fast)
      const double dx = x - pts[2 * k], dy = y - pts[2 * k + 1];
      const double d2 = dx * dx + dy * dy;
      const double u = d2 < 1e-200 ? 0.0 : 0.5 * d2 * log(d2);  // r < 1e-100 -> 0 (tps.py:80-81)
      sx += coef[2 * k] * u;
      sy += coef[2 * k + 1] * u;
    }
    grid[i] = a1x + axx * x + ayx * y + sx;
    grid[total + i] = a1y + axy * x + ayy * y + sy;
  }
}

__global__ void tps_grid_kernel(const double* __restrict__ pts, const double* __restrict__ coef, int npts, int nx,
                                int ny, double x_lo, double x_step, double y_lo, double y_step,
                                double* __restrict__ grid) {
  tps_grid_body(pts, coef, npts, nx, ny, x_lo, x_step, y_lo, y_step, grid);
}

// One axis of the grid upsampling (tps.py:55-63): frac, idx = modf((steps - 1) * u / span); idx1 =
// int(clip(idx + 1, 0, steps - 1)).
struct UpAxis {
  int i0, i1;
  double f, f1;
};

__device__ __forceinline__ UpAxis up_axis(int u, double steps, int span) {
  const double v = (steps - 1.0) * (double)u / (double)span;
  const double ip = trunc(v);
  UpAxis a;
  a.i0 = (int)ip;
  a.f = v - ip;
  a.f1 = 1.0 - a.f;
  double c = (double)(a.i0 + 1);
  c = c < 0.0 ? 0.0 : c;
  c = c > steps - 1.0 ? steps - 1.0 : c;
  a.i1 = (int)c;
  return a;
}

template <typename T>
__device__ __forceinline__ double to_f64(T v) {
  return (double)v;
}

template <typename T>
__device__ __forceinline__ T from_f64(double t);
template <>
__device__ __forceinline__ uint8_t from_f64<uint8_t>(double t) {  // scipy CASE_INTERP_OUT_UINT: (type)(t + 0.5)
  return (uint8_t)(t + 0.5);
}
template <>
__device__ __forceinline__ float from_f64<float>(double t) {
  return (float)t;
}
template <>
__device__ __forceinline__ double from_f64<double>(double t) {
  return t;
}

// tps.warp_images' sampling (tps.py:34): the per-pixel source coordinate is the grid (UP = false) or its bilinear
// upsampling t00*x1*y1 + t01*x1*yf + t10*xf*y1 + t11*xf*yf (tps.py:64-74); then scipy.ndimage.map_coordinates
// (order 0 / 1, mode 'constant', cval 0): a coordinate outside [0, n-1] gives 0; order 1 sums
// t += (v * w_row) * w_col over the taps (r0,c0) (r0,c1) (r1,c0) (r1,c1), weights (1 - f, 1 - (1 - f)).
template <typename T, int ORDER, bool UP>
__global__ void tps_sample_kernel(const double* __restrict__ grid, int nx, int ny, double x_steps, int x_span,
                                  double y_steps, int y_span, const T* __restrict__ img, int ih, int iw, int cn,
                                  T* __restrict__ out, int oh, int ow) {
  const long total = (long)oh * ow;
  const long gsz = (long)nx * ny;
  for_pixels(total, cn, out, [&](long i, T* o) {
    const int oy = row_of(i, ow), ox = (int)(i - (long)oy * ow);
    double tr, tc;
    if (UP) {
      const UpAxis ax = up_axis(oy, x_steps, x_span);
      const UpAxis ay = up_axis(ox, y_steps, y_span);
      const long a00 = (long)ax.i0 * ny + ay.i0, a01 = (long)ax.i0 * ny + ay.i1;
      const long a10 = (long)ax.i1 * ny + ay.i0, a11 = (long)ax.i1 * ny + ay.i1;
      tr = grid[a00] * ax.f1 * ay.f1 + grid[a01] * ax.f1 * ay.f + grid[a10] * ax.f * ay.f1 + grid[a11] * ax.f * ay.f;
      tc = grid[gsz + a00] * ax.f1 * ay.f1 + grid[gsz + a01] * ax.f1 * ay.f + grid[gsz + a10] * ax.f * ay.f1 +
           grid[gsz + a11] * ax.f * ay.f;
    } else {
      tr = grid[i];
      tc = grid[gsz + i];
    }
    const bool inside = tr >= 0.0 && tr <= (double)(ih - 1) && tc >= 0.0 && tc <= (double)(iw - 1);
    if (!inside) {
      for (int k = 0; k < cn; ++k) o[k] = from_f64<T>(0.0);
      return;
    }
    if (ORDER == 0) {
      const int r = (int)floor(tr + 0.5), c = (int)floor(tc + 0.5);
      const T* p = img + ((long)r * iw + c) * cn;
      for (int k = 0; k < cn; ++k) o[k] = from_f64<T>(to_f64(p[k]));
    } else {
      const double fr0 = floor(tr), fc0 = floor(tc);
      const int r0 = (int)fr0, c0 = (int)fc0;
      const double fr = tr - fr0, fc = tc - fc0;
      const double wr0 = 1.0 - fr, wr1 = 1.0 - wr0, wc0 = 1.0 - fc, wc1 = 1.0 - wc0;
      const bool r1ok = r0 + 1 < ih, c1ok = c0 + 1 < iw;
      const T* p00 = img + ((long)r0 * iw + c0) * cn;
      for (int k = 0; k < cn; ++k) {
        const double v00 = to_f64(p00[k]);
        const double v01 = c1ok ? to_f64(p00[cn + k]) : 0.0;
        const double v10 = r1ok ? to_f64(p00[(long)iw * cn + k]) : 0.0;
        const double v11 = (r1ok && c1ok) ? to_f64(p00[((long)iw + 1) * cn + k]) : 0.0;
        double t = 0.0;
        t += (v00 * wr0) * wc0;
        t += (v01 * wr0) * wc1;
        t += (v10 * wr1) * wc0;
        t += (v11 * wr1) * wc1;
        o[k] = from_f64<T>(t);
      }
    }
  });
}

// ---------------------------------------------------------------------------------------------------- OpenCV

struct Affine {
  double m[6];  // the inverted matrix (dst -> src), as WarpAffineInvoker uses it
};

__device__ __forceinline__ int cv_round(double v) { return (int)rint(v); }  // cvRound: round half to even

// cv2.warpAffine INTER_LINEAR, BORDER_CONSTANT 0 (OpenCV 3.x imgwarp.cpp WarpAffineInvoker + remapBilinear):
// X = (cvRound((M1*y + M2)*1024) + 16 + cvRound(M0*x*1024)) >> 5, tap (X>>5, Y>>5) saturated to short, fraction
// (X&31, Y&31) into the 32x32 bilinear table.  uint8: 15-bit weights (32-ay)(32-ax)*32 ..., (s + 2^14) >> 15;
// float: the exact float table weights, v0*w0 + v1*w1 + v2*w2 + v3*w3 in the source type's arithmetic.
template <typename T>
__global__ void warp_affine_kernel(const T* __restrict__ src, int ih, int iw, int cn, Affine a, T* __restrict__ dst,
                                   int h, int w) {
  const long total = (long)h * w;
  for_pixels(total, cn, dst, [&](long i, T* o) {
    const int y = row_of(i, w), x = (int)(i - (long)y * w);
    const int adelta = cv_round(a.m[0] * (double)x * 1024.0);
    const int bdelta = cv_round(a.m[3] * (double)x * 1024.0);
    const int X0 = cv_round((a.m[1] * (double)y + a.m[2]) * 1024.0) + 16;
    const int Y0 = cv_round((a.m[4] * (double)y + a.m[5]) * 1024.0) + 16;
    const int X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
    int sx = X >> 5, sy = Y >> 5;
    sx = sx < -32768 ? -32768 : (sx > 32767 ? 32767 : sx);
    sy = sy < -32768 ? -32768 : (sy > 32767 ? 32767 : sy);
    const int ax = X & 31, ay = Y & 31;
    const bool y0ok = (unsigned)sy < (unsigned)ih, y1ok = (unsigned)(sy + 1) < (unsigned)ih;
    const bool x0ok = (unsigned)sx < (unsigned)iw, x1ok = (unsigned)(sx + 1) < (unsigned)iw;
    const T* p = src + ((long)sy * iw + sx) * cn;
    for (int k = 0; k < cn; ++k) {
      const T v0 = (y0ok && x0ok) ? p[k] : T(0);
      const T v1 = (y0ok && x1ok) ? p[cn + k] : T(0);
      const T v2 = (y1ok && x0ok) ? p[(long)iw * cn + k] : T(0);
      const T v3 = (y1ok && x1ok) ? p[((long)iw + 1) * cn + k] : T(0);
      if constexpr (sizeof(T) == 1) {
        const int s = (int)v0 * ((32 - ay) * (32 - ax) * 32) + (int)v1 * ((32 - ay) * ax * 32) +
                      (int)v2 * (ay * (32 - ax) * 32) + (int)v3 * (ay * ax * 32);
        int r = (s + (1 << 14)) >> 15;
        o[k] = (T)(r < 0 ? 0 : (r > 255 ? 255 : r));
      } else {
        const float wy0 = 1.f - (float)ay * (1.f / 32.f), wy1 = (float)ay * (1.f / 32.f);
        const float wx0 = 1.f - (float)ax * (1.f / 32.f), wx1 = (float)ax * (1.f / 32.f);
        const T w0 = (T)(wy0 * wx0), w1 = (T)(wy0 * wx1), w2 = (T)(wy1 * wx0), w3 = (T)(wy1 * wx1);
        o[k] = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
      }
    }
  });
}

struct Lut256 {
  uint8_t t[256];
};

// augmentation.change_illumination (augmentation.py:86-98): cvtColor BGR2HSV (RGB2HSV_b, hsv_shift 12, hrange
// 180), S and V through the host-built map lut[u] = uint8(255 * clip(a * (u/255)^b + c, 0, 1)), cvtColor HSV2BGR
// (HSV2RGB_b: float32 HSV2RGB_f, then cvRound(x * 255) saturated).  The division tables live in LDS.
// HSV round trip of one BGR pixel with S, V through lut (the division tables sdiv / hdiv in LDS)
__device__ __forceinline__ void illum_px(int b, int g, int r, const Lut256& lut, const int* sdiv, const int* hdiv,
                                         uint8_t* o) {
  const float hscale = 6.f / 180.f;
  const float inv255 = 1.f / 255.f;
  int v = b > g ? b : g;
  v = v > r ? v : r;
  int vmin = b < g ? b : g;
  vmin = vmin < r ? vmin : r;
  const int diff = v - vmin;
  const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
  const int s = (diff * sdiv[v] + (1 << 11)) >> 12;
  int hh = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
  hh = (hh * hdiv[diff] + (1 << 11)) >> 12;
  hh += hh < 0 ? 180 : 0;
  // new_hsv = (h, lut[s], lut[v]) -> HSV2RGB_b
  float hf = (float)(uint8_t)hh;
  const float sf = (float)lut.t[s] * inv255;
  const float vf = (float)lut.t[v] * inv255;
  float ob, og, orr;
  if (sf == 0.f) {
    ob = og = orr = vf;
  } else {
    hf *= hscale;
    while (hf < 0.f) hf += 6.f;
    while (hf >= 6.f) hf -= 6.f;
    int sector = (int)floorf(hf);
    hf -= (float)sector;
    if ((unsigned)sector >= 6u) {
      sector = 0;
      hf = 0.f;
    }
    float tab[4];
    tab[0] = vf;
    tab[1] = vf * (1.f - sf);
    tab[2] = vf * (1.f - sf * hf);
    tab[3] = vf * (1.f - sf * (1.f - hf));
    const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
    ob = tab[sd[sector][0]];
    og = tab[sd[sector][1]];
    orr = tab[sd[sector][2]];
  }
  auto sat = [](float x) -> uint8_t {
    const int q = (int)rintf(x * 255.f);
    return (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
  };
  o[0] = sat(ob);
  o[1] = sat(og);
  o[2] = sat(orr);
}

__device__ __forceinline__ void illum_tables(int* sdiv, int* hdiv) {
  for (int t = threadIdx.x; t < 256; t += blockDim.x) {
    sdiv[t] = t ? (int)rint((double)(255 << 12) / (1.0 * t)) : 0;
    hdiv[t] = t ? (int)rint((double)(180 << 12) / (6.0 * t)) : 0;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) illumination_kernel(const uint8_t* __restrict__ bgr, long pixels, Lut256 lut,
                                                           uint8_t* __restrict__ out) {
  __shared__ int sdiv[256], hdiv[256];
  illum_tables(sdiv, hdiv);
  for_pixels(pixels, 3, out, [&](long i, uint8_t* o) {
    illum_px(bgr[3 * i], bgr[3 * i + 1], bgr[3 * i + 2], lut, sdiv, hdiv, o);
  });
}

// augmentation.warp_image without the TPS part (augmentation.py:59-63) in ONE pass, optionally followed by
// change_illumination (augmentation.py:133-134, u8 BGR only).  The first cv2.warpAffine is the integer translation
// [[1, 0, tu], [0, 1, tv]]: its fixed-point coordinates have zero fraction, so translated(y, x) = src(y - tv, x - tu)
// inside src, else 0, exactly (u8: (v*32768 + 2^14) >> 15 = v; float: v*1 + 0 + 0 + 0).  The second warpAffine
// (getRotationMatrix2D, inverted on the host side as warpAffine does) then gathers its 4 taps from that virtual
// translated image (size h x w, zero outside) — no intermediate image in HBM.
template <typename T, bool ILLUM>
__global__ void __launch_bounds__(256) warp_image_kernel(const T* __restrict__ src, int ih, int iw, int cn, int tu,
                                                         int tv, Affine a, Lut256 lut, T* __restrict__ dst, int h,
                                                         int w) {
  __shared__ int sdiv[256], hdiv[256];
  if constexpr (ILLUM) illum_tables(sdiv, hdiv);
  const long total = (long)h * w;
  for_pixels(total, cn, dst, [&](long i, T* o) {
    const int y = row_of(i, w), x = (int)(i - (long)y * w);
    const int adelta = cv_round(a.m[0] * (double)x * 1024.0);
    const int bdelta = cv_round(a.m[3] * (double)x * 1024.0);
    const int X0 = cv_round((a.m[1] * (double)y + a.m[2]) * 1024.0) + 16;
    const int Y0 = cv_round((a.m[4] * (double)y + a.m[5]) * 1024.0) + 16;
    const int X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
    int sx = X >> 5, sy = Y >> 5;
    sx = sx < -32768 ? -32768 : (sx > 32767 ? 32767 : sx);
    sy = sy < -32768 ? -32768 : (sy > 32767 ? 32767 : sy);
    const int ax = X & 31, ay = Y & 31;
    // a tap (ty, tx) of the translated image: inside it AND its source pixel inside src
    auto ok = [&](int ty, int tx) {
      return (unsigned)ty < (unsigned)h && (unsigned)tx < (unsigned)w && (unsigned)(ty - tv) < (unsigned)ih &&
             (unsigned)(tx - tu) < (unsigned)iw;
    };
    const bool k0 = ok(sy, sx), k1 = ok(sy, sx + 1), k2 = ok(sy + 1, sx), k3 = ok(sy + 1, sx + 1);
    const T* p = src + ((long)(sy - tv) * iw + (sx - tu)) * cn;
    uint8_t px[8];
    for (int k = 0; k < cn; ++k) {
      const T v0 = k0 ? p[k] : T(0);
      const T v1 = k1 ? p[cn + k] : T(0);
      const T v2 = k2 ? p[(long)iw * cn + k] : T(0);
      const T v3 = k3 ? p[((long)iw + 1) * cn + k] : T(0);
      if constexpr (sizeof(T) == 1) {
        const int s = (int)v0 * ((32 - ay) * (32 - ax) * 32) + (int)v1 * ((32 - ay) * ax * 32) +
                      (int)v2 * (ay * (32 - ax) * 32) + (int)v3 * (ay * ax * 32);
        const int r = (s + (1 << 14)) >> 15;
        const T q = (T)(r < 0 ? 0 : (r > 255 ? 255 : r));
        if constexpr (ILLUM) px[k] = q;
        else o[k] = q;
      } else {
        const float wy0 = 1.f - (float)ay * (1.f / 32.f), wy1 = (float)ay * (1.f / 32.f);
        const float wx0 = 1.f - (float)ax * (1.f / 32.f), wx1 = (float)ax * (1.f / 32.f);
        const T w0 = (T)(wy0 * wx0), w1 = (T)(wy0 * wx1), w2 = (T)(wy1 * wx0), w3 = (T)(wy1 * wx1);
        o[k] = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
      }
    }
    if constexpr (ILLUM) illum_px(px[0], px[1], px[2], lut, sdiv, hdiv, reinterpret_cast<uint8_t*>(o));
  });
}

// augmentation.augmentation's BGRA frame (augmentation.py:154-155, 162-163): concat(fg u8 BGR, (255. * alpha)
// .astype(uint8)) — the product in the alpha's precision (f64 like numpy), truncated — one 4-byte store per pixel.
template <typename TA>
__global__ void __launch_bounds__(256) bgra_kernel(const uint8_t* __restrict__ fg, const TA* __restrict__ alpha,
                                                   long pixels, uint32_t* __restrict__ out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < pixels; i += (long)gridDim.x * blockDim.x) {
    const uint32_t a8 = (uint32_t)(uint8_t)(int)(255.0 * (double)alpha[i]);
    out[i] = (uint32_t)fg[3 * i] | ((uint32_t)fg[3 * i + 1] << 8) | ((uint32_t)fg[3 * i + 2] << 16) | (a8 << 24);
  }
}

// augmentation.object_size / fg_center (augmentation.py:10-20): count, row-index sum and column-index sum of the
// nonzero alpha pixels (exact integers; the host forms sqrt(count) and int(sum / count) like numpy).
template <typename T>
__global__ void __launch_bounds__(256) nonzero_stats_kernel(const T* __restrict__ a, int h, int w,
                                                            unsigned long long* __restrict__ stats) {
  unsigned long long cnt = 0, sr = 0, sc = 0;
  for (int r = blockIdx.x; r < h; r += gridDim.x) {
    const T* row = a + (long)r * w;
    for (int c = threadIdx.x; c < w; c += blockDim.x) {
      if (row[c] != T(0)) {
        ++cnt;
        sr += (unsigned long long)r;
        sc += (unsigned long long)c;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    cnt += __shfl_xor(cnt, off, 64);
    sr += __shfl_xor(sr, off, 64);
    sc += __shfl_xor(sc, off, 64);
  }
  // one set of atomics per block (not per wave): the three counters are single addresses
  __shared__ unsigned long long part[3][4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][wv] = cnt;
    part[1][wv] = sr;
    part[2][wv] = sc;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long v = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += part[threadIdx.x][k];
    if (v) atomicAdd(&stats[threadIdx.x], v);
  }
}


// ---------------------------------------------------------------------------------------------------- batches
// augmentation.augment over a batch of samples (augment_many: the config-5 pipeline) in a handful of launches: every
// launch takes up to kAugJobs samples' parameters by value (grid.y = the sample), so a batch of 8 costs 2 x 4
// launches where the per-sample calls cost 8 x 6 (their ~25 us of host issue each bounded the chained step).  Per
// pixel the arithmetic is the per-sample kernels' own (tps_grid_body, the UP / order-1 path of tps_sample_kernel,
// warp_image_kernel): outputs bit-identical.  The fg and alpha TPS resamplings share one map, so they are ONE pass
// here (one upsampled coordinate per pixel, then the 3 u8 and the f64 taps).
constexpr int kAugJobs = 4;

struct AugGridJobs {
  const double* pts[kAugJobs];
  const double* coef[kAugJobs];
  double* grid[kAugJobs];
  UpAxis* axes[kAugJobs];  // the upsampling's per-row ([h+1]) then per-column ([w+1]) terms
  int npts[kAugJobs], nx[kAugJobs], ny[kAugJobs], h[kAugJobs], w[kAugJobs];
  double xstep[kAugJobs], ystep[kAugJobs], xsteps[kAugJobs], ysteps[kAugJobs];
};

// the lattice, and the resampling's up_axis terms of every output row and column (each an f64 division): formed
// once per sample here instead of twice per output pixel
__global__ void __launch_bounds__(256) tps_grid_batch_kernel(AugGridJobs J) {
  const int j = blockIdx.y;
  tps_grid_body(J.pts[j], J.coef[j], J.npts[j], J.nx[j], J.ny[j], 0.0, J.xstep[j], 0.0, J.ystep[j], J.grid[j]);
  const int h = J.h[j], w = J.w[j];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < h + w + 2; i += gridDim.x * blockDim.x)
    J.axes[j][i] = i <= h ? up_axis(i, J.xsteps[j], h) : up_axis(i - h - 1, J.ysteps[j], w);
}

struct AugSampleJobs {
  const double* grid[kAugJobs];
  const UpAxis* axes[kAugJobs];
  const uint8_t* fg[kAugJobs];
  const double* al[kAugJobs];
  uint8_t* fg_t[kAugJobs];
  double* al_t[kAugJobs];
  int h[kAugJobs], w[kAugJobs], nx[kAugJobs], ny[kAugJobs];
  double xsteps[kAugJobs], ysteps[kAugJobs];
};

// tps.warp_images' resampling of the fg planes (u8) and of the alpha plane (f64) through the same upsampled map
// (tps.py:55-74, output (h+1) x (w+1)): tps_sample_kernel<uint8_t, 1, true> and <double, 1, true> in one pass
__global__ void __launch_bounds__(256) tps_sample_pair_kernel(AugSampleJobs J) {
  const int j = blockIdx.y;
  const int ih = J.h[j], iw = J.w[j], oh = ih + 1, ow = iw + 1, nx = J.nx[j], ny = J.ny[j];
  const double* __restrict__ grid = J.grid[j];
  const uint8_t* __restrict__ img = J.fg[j];
  const double* __restrict__ al = J.al[j];
  double* __restrict__ alt = J.al_t[j];
  const long total = (long)oh * ow, gsz = (long)nx * ny;
  const UpAxis* __restrict__ axes = J.axes[j];
  (void)J.xsteps[j];
  (void)J.ysteps[j];
  for_pixels(total, 3, J.fg_t[j], [&](long i, uint8_t* o) {
    const int oy = row_of(i, ow), ox = (int)(i - (long)oy * ow);
    const UpAxis ax = axes[oy];            // == up_axis(oy, xsteps, ih)
    const UpAxis ay = axes[oh + ox];       // == up_axis(ox, ysteps, iw)
    const long a00 = (long)ax.i0 * ny + ay.i0, a01 = (long)ax.i0 * ny + ay.i1;
    const long a10 = (long)ax.i1 * ny + ay.i0, a11 = (long)ax.i1 * ny + ay.i1;
    const double tr = grid[a00] * ax.f1 * ay.f1 + grid[a01] * ax.f1 * ay.f + grid[a10] * ax.f * ay.f1 +
                      grid[a11] * ax.f * ay.f;
    const double tc = grid[gsz + a00] * ax.f1 * ay.f1 + grid[gsz + a01] * ax.f1 * ay.f +
                      grid[gsz + a10] * ax.f * ay.f1 + grid[gsz + a11] * ax.f * ay.f;
    const bool inside = tr >= 0.0 && tr <= (double)(ih - 1) && tc >= 0.0 && tc <= (double)(iw - 1);
    if (!inside) {
      o[0] = o[1] = o[2] = 0;
      alt[i] = 0.0;
      return;
    }
    const double fr0 = floor(tr), fc0 = floor(tc);
    const int r0 = (int)fr0, c0 = (int)fc0;
    const double fr = tr - fr0, fc = tc - fc0;
    const double wr0 = 1.0 - fr, wr1 = 1.0 - wr0, wc0 = 1.0 - fc, wc1 = 1.0 - wc0;
    const bool r1ok = r0 + 1 < ih, c1ok = c0 + 1 < iw;
    const uint8_t* p00 = img + ((long)r0 * iw + c0) * 3;
    for (int k = 0; k < 3; ++k) {
      const double v00 = (double)p00[k];
      const double v01 = c1ok ? (double)p00[3 + k] : 0.0;
      const double v10 = r1ok ? (double)p00[(long)iw * 3 + k] : 0.0;
      const double v11 = (r1ok && c1ok) ? (double)p00[((long)iw + 1) * 3 + k] : 0.0;
      double t = 0.0;
      t += (v00 * wr0) * wc0;
      t += (v01 * wr0) * wc1;
      t += (v10 * wr1) * wc0;
      t += (v11 * wr1) * wc1;
      o[k] = from_f64<uint8_t>(t);
    }
    const double* q00 = al + (long)r0 * iw + c0;
    const double v00 = q00[0];
    const double v01 = c1ok ? q00[1] : 0.0;
    const double v10 = r1ok ? q00[iw] : 0.0;
    const double v11 = (r1ok && c1ok) ? q00[iw + 1] : 0.0;
    double t = 0.0;
    t += (v00 * wr0) * wc0;
    t += (v01 * wr0) * wc1;
    t += (v10 * wr1) * wc0;
    t += (v11 * wr1) * wc1;
    alt[i] = t;
  });
}

// warp_image_kernel's per-pixel work, one job per blockIdx.y
template <typename T, bool ILLUM>
__device__ __forceinline__ void warp_image_body(const T* __restrict__ src, int ih, int iw, int cn, int tu, int tv,
                                                const Affine& a, const Lut256& lut, const int* sdiv, const int* hdiv,
                                                T* __restrict__ dst, int h, int w) {
  const long total = (long)h * w;
  for_pixels(total, cn, dst, [&](long i, T* o) {
    const int y = row_of(i, w), x = (int)(i - (long)y * w);
    const int adelta = cv_round(a.m[0] * (double)x * 1024.0);
    const int bdelta = cv_round(a.m[3] * (double)x * 1024.0);
    const int X0 = cv_round((a.m[1] * (double)y + a.m[2]) * 1024.0) + 16;
    const int Y0 = cv_round((a.m[4] * (double)y + a.m[5]) * 1024.0) + 16;
    const int X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
    int sx = X >> 5, sy = Y >> 5;
    sx = sx < -32768 ? -32768 : (sx > 32767 ? 32767 : sx);
    sy = sy < -32768 ? -32768 : (sy > 32767 ? 32767 : sy);
    const int ax = X & 31, ay = Y & 31;
    auto ok = [&](int ty, int tx) {
      return (unsigned)ty < (unsigned)h && (unsigned)tx < (unsigned)w && (unsigned)(ty - tv) < (unsigned)ih &&
             (unsigned)(tx - tu) < (unsigned)iw;
    };
    const bool k0 = ok(sy, sx), k1 = ok(sy, sx + 1), k2 = ok(sy + 1, sx), k3 = ok(sy + 1, sx + 1);
    const T* p = src + ((long)(sy - tv) * iw + (sx - tu)) * cn;
    uint8_t px[8];
    for (int k = 0; k < cn; ++k) {
      const T v0 = k0 ? p[k] : T(0);
      const T v1 = k1 ? p[cn + k] : T(0);
      const T v2 = k2 ? p[(long)iw * cn + k] : T(0);
      const T v3 = k3 ? p[((long)iw + 1) * cn + k] : T(0);
      if constexpr (sizeof(T) == 1) {
        const int s = (int)v0 * ((32 - ay) * (32 - ax) * 32) + (int)v1 * ((32 - ay) * ax * 32) +
                      (int)v2 * (ay * (32 - ax) * 32) + (int)v3 * (ay * ax * 32);
        const int r = (s + (1 << 14)) >> 15;
        const T q = (T)(r < 0 ? 0 : (r > 255 ? 255 : r));
        if constexpr (ILLUM) px[k] = q;
        else o[k] = q;
      } else {
        const float wy0 = 1.f - (float)ay * (1.f / 32.f), wy1 = (float)ay * (1.f / 32.f);
        const float wx0 = 1.f - (float)ax * (1.f / 32.f), wx1 = (float)ax * (1.f / 32.f);
        const T w0 = (T)(wy0 * wx0), w1 = (T)(wy0 * wx1), w2 = (T)(wy1 * wx0), w3 = (T)(wy1 * wx1);
        o[k] = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
      }
    }
    if constexpr (ILLUM) illum_px(px[0], px[1], px[2], lut, sdiv, hdiv, reinterpret_cast<uint8_t*>(o));
  });
}

// the camera motion of a batch: each sample's background through its translation + scale and its S/V map
// (augmentation.py:113-116, 133-134)
struct AugWarpU8Jobs {
  const uint8_t* src[kAugJobs];
  uint8_t* dst[kAugJobs];
  int ih[kAugJobs], iw[kAugJobs], h[kAugJobs], w[kAugJobs], tu[kAugJobs], tv[kAugJobs];
  Affine a[kAugJobs];
  Lut256 lut[kAugJobs];
};

__global__ void __launch_bounds__(256) warp_bg_batch_kernel(AugWarpU8Jobs J) {
  __shared__ int sdiv[256], hdiv[256];
  illum_tables(sdiv, hdiv);
  const int j = blockIdx.y;
  warp_image_body<uint8_t, true>(J.src[j], J.ih[j], J.iw[j], 3, J.tu[j], J.tv[j], J.a[j], J.lut[j], sdiv, hdiv,
                                 J.dst[j], J.h[j], J.w[j]);
}

// the object motion of a batch: the TPS-resampled fg (u8 BGR, then the illumination change) and alpha (f64) go through
// the SAME translation and similarity (augmentation.py:121-129), so one pass forms each pixel's fixed-point source
// coordinate once and gathers both images' taps; optionally it also writes the sample's BGRA frame (vm_bgra_u8 of the
// two outputs, augmentation.py:162-163).  Per image, warp_image_body's arithmetic: bit-identical.
struct AugWarpObjJobs {
  const uint8_t* fg[kAugJobs];
  const double* al[kAugJobs];
  uint8_t* dfg[kAugJobs];
  double* dal[kAugJobs];
  uint32_t* bgra[kAugJobs];
  int ih[kAugJobs], iw[kAugJobs], h[kAugJobs], w[kAugJobs], tu[kAugJobs], tv[kAugJobs];
  Affine a[kAugJobs];
  Lut256 lut[kAugJobs];
};

__global__ void __launch_bounds__(256) warp_object_batch_kernel(AugWarpObjJobs J) {
  __shared__ int sdiv[256], hdiv[256];
  illum_tables(sdiv, hdiv);
  const int j = blockIdx.y;
  const int ih = J.ih[j], iw = J.iw[j], h = J.h[j], w = J.w[j], tu = J.tu[j], tv = J.tv[j];
  const Affine a = J.a[j];
  const uint8_t* __restrict__ src = J.fg[j];
  const double* __restrict__ asrc = J.al[j];
  double* __restrict__ dal = J.dal[j];
  uint32_t* __restrict__ bgra = J.bgra[j];
  const long total = (long)h * w;
  for_pixels(total, 3, J.dfg[j], [&](long i, uint8_t* o) {
    const int y = row_of(i, w), x = (int)(i - (long)y * w);
    const int adelta = cv_round(a.m[0] * (double)x * 1024.0);
    const int bdelta = cv_round(a.m[3] * (double)x * 1024.0);
    const int X0 = cv_round((a.m[1] * (double)y + a.m[2]) * 1024.0) + 16;
    const int Y0 = cv_round((a.m[4] * (double)y + a.m[5]) * 1024.0) + 16;
    const int X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
    int sx = X >> 5, sy = Y >> 5;
    sx = sx < -32768 ? -32768 : (sx > 32767 ? 32767 : sx);
    sy = sy < -32768 ? -32768 : (sy > 32767 ? 32767 : sy);
    const int ax = X & 31, ay = Y & 31;
    auto ok = [&](int ty, int tx) {
      return (unsigned)ty < (unsigned)h && (unsigned)tx < (unsigned)w && (unsigned)(ty - tv) < (unsigned)ih &&
             (unsigned)(tx - tu) < (unsigned)iw;
    };
    const bool k0 = ok(sy, sx), k1 = ok(sy, sx + 1), k2 = ok(sy + 1, sx), k3 = ok(sy + 1, sx + 1);
    const long base = (long)(sy - tv) * iw + (sx - tu);
    const uint8_t* p = src + base * 3;
    uint8_t px[3];
    for (int k = 0; k < 3; ++k) {
      const int v0 = k0 ? p[k] : 0, v1 = k1 ? p[3 + k] : 0;
      const int v2 = k2 ? p[(long)iw * 3 + k] : 0, v3 = k3 ? p[((long)iw + 1) * 3 + k] : 0;
      const int s = v0 * ((32 - ay) * (32 - ax) * 32) + v1 * ((32 - ay) * ax * 32) + v2 * (ay * (32 - ax) * 32) +
                    v3 * (ay * ax * 32);
      const int r = (s + (1 << 14)) >> 15;
      px[k] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
    illum_px(px[0], px[1], px[2], J.lut[j], sdiv, hdiv, o);
    const double* q = asrc + base;
    const double v0 = k0 ? q[0] : 0.0, v1 = k1 ? q[1] : 0.0, v2 = k2 ? q[iw] : 0.0, v3 = k3 ? q[iw + 1] : 0.0;
    const float wy0 = 1.f - (float)ay * (1.f / 32.f), wy1 = (float)ay * (1.f / 32.f);
    const float wx0 = 1.f - (float)ax * (1.f / 32.f), wx1 = (float)ax * (1.f / 32.f);
    const double w0 = (double)(wy0 * wx0), w1 = (double)(wy0 * wx1), w2 = (double)(wy1 * wx0), w3 = (double)(wy1 * wx1);
    const double al = v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3;
    dal[i] = al;
    if (bgra) {
      const uint32_t a8 = (uint32_t)(uint8_t)(int)(255.0 * al);
      bgra[i] = (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16) | (a8 << 24);
    }
  });
}

// augmentation.augmentation's BGRA frames of a batch (vm_bgra_u8 per job, f64 alpha), grid.y = the job
struct AugBgraJobs {
  const uint8_t* fg[2 * kAugJobs];
  const double* al[2 * kAugJobs];
  uint32_t* out[2 * kAugJobs];
  long px[2 * kAugJobs];
};

__global__ void __launch_bounds__(256) bgra_batch_kernel(AugBgraJobs J) {
  const int j = blockIdx.y;
  const uint8_t* __restrict__ fg = J.fg[j];
  const double* __restrict__ alpha = J.al[j];
  uint32_t* __restrict__ out = J.out[j];
  const long pixels = J.px[j];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < pixels; i += (long)gridDim.x * blockDim.x) {
    const uint32_t a8 = (uint32_t)(uint8_t)(int)(255.0 * alpha[i]);
    out[i] = (uint32_t)fg[3 * i] | ((uint32_t)fg[3 * i + 1] << 8) | ((uint32_t)fg[3 * i + 2] << 16) | (a8 << 24);
  }
}

// the foreground statistics of a batch of alphas, one launch (grid.y = the alpha)
struct AugStatsJobs {
  const double* a[2 * kAugJobs];
  int h[2 * kAugJobs], w[2 * kAugJobs];
};

__global__ void __launch_bounds__(256) nonzero_stats_batch_kernel(AugStatsJobs J, unsigned long long* __restrict__ stats) {
  const int j = blockIdx.y;
  const int h = J.h[j], w = J.w[j];
  const double* a = J.a[j];
  unsigned long long cnt = 0, sr = 0, sc = 0;
  for (int r = blockIdx.x; r < h; r += gridDim.x) {
    const double* row = a + (long)r * w;
    for (int c = threadIdx.x; c < w; c += blockDim.x) {
      if (row[c] != 0.0) {
        ++cnt;
        sr += (unsigned long long)r;
        sc += (unsigned long long)c;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    cnt += __shfl_xor(cnt, off, 64);
    sr += __shfl_xor(sr, off, 64);
    sc += __shfl_xor(sc, off, 64);
  }
  __shared__ unsigned long long part[3][4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    part[0][wv] = cnt;
    part[1][wv] = sr;
    part[2][wv] = sc;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long v = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += part[threadIdx.x][k];
    if (v) atomicAdd(&stats[3 * j + threadIdx.x], v);
  }
}

// ---------------------------------------------------------------------------------------------------- data.py

// data.trimap_from_matte (data.py:37-67).  The reference's raster loop lets a known pixel's own assignment (255 for
// matte 1, 0 for matte 0) overwrite every earlier 128-mark, so the result is 128 for unknown pixels and for known
// pixels with an unknown pixel LATER in raster order within radius crop (matte 1) / dilate (matte 0).  A 16x64
// tile's classes (0 / 1 / unknown / outside) are staged in LDS with the half-window halo below and to the sides.
constexpr int kTriH = 16, kTriW = 64, kTriMaxSide = 8;

__global__ void __launch_bounds__(256) trimap_kernel(const double* __restrict__ m, int h, int w, int dilate, int crop,
                                                     uint8_t* __restrict__ out) {
  __shared__ uint8_t cls[(kTriH + kTriMaxSide) * (kTriW + 2 * kTriMaxSide)];
  const int side = dilate > crop ? dilate : crop;
  const int r0 = blockIdx.y * kTriH, c0 = blockIdx.x * kTriW;
  const int lw = kTriW + 2 * side, lh = kTriH + side;
  for (int t = threadIdx.x; t < lh * lw; t += blockDim.x) {
    const int rr = r0 + t / lw, cc = c0 - side + t % lw;
    uint8_t k = 3;  // outside the image
    if (rr < h && cc >= 0 && cc < w) {
      const double v = m[(long)rr * w + cc];
      k = v == 1. ? 1 : (v == 0. ? 0 : 2);
    }
    cls[t] = k;
  }
  __syncthreads();
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = c0 + tx;
  if (c >= w) return;
  for (int j = 0; j < kTriH / 4; ++j) {
    const int lr = ty * (kTriH / 4) + j, r = r0 + lr;
    if (r >= h) break;
    const uint8_t own = cls[lr * lw + tx + side];
    uint8_t v = 128;
    if (own <= 1) {
      v = own ? 255 : 0;
      const int rad = own ? crop : dilate;
      for (int dk = 0; dk <= rad && v != 128; ++dk)
        for (int dl = (dk == 0 ? 1 : -rad); dl <= rad; ++dl)
          if (cls[(lr + dk) * lw + tx + side + dl] == 2) {
            v = 128;
            break;
          }
    }
    out[(long)r * w + c] = v;
  }
}

}  // namespace vm

using namespace vm;

extern "C" int vm_tps_grid(const double* points, const double* coeffs, int npts, int nx, int ny, double x_lo,
                           double x_step, double y_lo, double y_step, double* grid, void* stream) {
  if (!points || !coeffs || !grid || npts <= 0 || nx <= 0 || ny <= 0) return fail(VM_EINVAL, "tps_grid: bad argument");
  if ((long)nx * ny >= (1L << 31)) return fail(VM_EUNSUPPORTED, "tps_grid: more than 2^31 grid points");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long total = (long)nx * ny;
  hipLaunchKernelGGL(tps_grid_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, points, coeffs, npts, nx, ny, x_lo,
                     x_step, y_lo, y_step, grid);
  return check_launch("tps_grid");
}

template <typename T>
static void launch_tps_sample(const vm_tps_map* m, const void* img, int ih, int iw, int cn, int order, void* out,
                              int oh, int ow, hipStream_t st) {
  const dim3 g(grid_for((long)oh * ow, 256)), b(256);
  const T* s = static_cast<const T*>(img);
  T* o = static_cast<T*>(out);
#define VM_TPS_LAUNCH(ORD, UP)                                                                                      \
  hipLaunchKernelGGL((tps_sample_kernel<T, ORD, UP>), g, b, 0, st, m->grid, m->nx, m->ny, m->x_steps, m->x_span,    \
                     m->y_steps, m->y_span, s, ih, iw, cn, o, oh, ow)
  if (order == 0) {
    if (m->upsample) VM_TPS_LAUNCH(0, true);
    else VM_TPS_LAUNCH(0, false);
  } else {
    if (m->upsample) VM_TPS_LAUNCH(1, true);
    else VM_TPS_LAUNCH(1, false);
  }
#undef VM_TPS_LAUNCH
}

extern "C" int vm_tps_sample(const vm_tps_map* map, const void* img, int ih, int iw, int cn, int dtype, int order,
                             void* out, void* stream) {
  if (!map || !map->grid || !img || !out || ih <= 0 || iw <= 0 || cn <= 0 || map->nx <= 0 || map->ny <= 0 ||
      (order != 0 && order != 1))
    return fail(VM_EINVAL, "tps_sample: bad argument");
  if (dtype == VM_U8 && cn > 8) return fail(VM_EUNSUPPORTED, "tps_sample: uint8 images with more than 8 planes");
  if ((long)map->nx * map->ny >= (1L << 31) || ((long)map->x_span + 1) * (map->y_span + 1) >= (1L << 31))
    return fail(VM_EUNSUPPORTED, "tps_sample: more than 2^31 pixels");
  int oh = map->nx, ow = map->ny;
  if (map->upsample) {
    if (map->x_span <= 0 || map->y_span <= 0) return fail(VM_EINVAL, "tps_sample: empty output region");
    // every grid index the upsampling can form must lie inside the grid
    if (!(map->x_steps - 1.0 < (double)map->nx) || !(map->y_steps - 1.0 < (double)map->ny) || map->x_steps < 1.0 ||
        map->y_steps < 1.0)
      return fail(VM_EINVAL, "tps_sample: grid %dx%d too small for steps %g x %g", map->nx, map->ny, map->x_steps,
                  map->y_steps);
    oh = map->x_span + 1;
    ow = map->y_span + 1;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (dtype) {
    case VM_U8: launch_tps_sample<uint8_t>(map, img, ih, iw, cn, order, out, oh, ow, st); break;
    case VM_F32: launch_tps_sample<float>(map, img, ih, iw, cn, order, out, oh, ow, st); break;
    case VM_F64: launch_tps_sample<double>(map, img, ih, iw, cn, order, out, oh, ow, st); break;
    default: return fail(VM_EUNSUPPORTED, "tps_sample: dtype %d", dtype);
  }
  return check_launch("tps_sample");
}

// warpAffine without WARP_INVERSE_MAP inverts the forward matrix in double (imgwarp.cpp)
static Affine invert_affine(const double* m) {
  Affine a;
  for (int i = 0; i < 6; ++i) a.m[i] = m[i];
  double d = a.m[0] * a.m[4] - a.m[1] * a.m[3];
  d = d != 0 ? 1. / d : 0.;
  const double a11 = a.m[4] * d, a22 = a.m[0] * d;
  a.m[0] = a11;
  a.m[1] *= -d;
  a.m[3] *= -d;
  a.m[4] = a22;
  const double b1 = -a.m[0] * a.m[2] - a.m[1] * a.m[5];
  const double b2 = -a.m[3] * a.m[2] - a.m[4] * a.m[5];
  a.m[2] = b1;
  a.m[5] = b2;
  return a;
}

extern "C" int vm_warp_image(const void* src, int ih, int iw, int cn, int dtype, int tu, int tv, const double* m,
                             const uint8_t* lut, void* dst, int h, int w, void* stream) {
  if (!src || !dst || !m || ih <= 0 || iw <= 0 || cn <= 0 || h <= 0 || w <= 0)
    return fail(VM_EINVAL, "warp_image: bad argument");
  if (dtype == VM_U8 && cn > 8) return fail(VM_EUNSUPPORTED, "warp_image: uint8 images with more than 8 channels");
  if (lut && (dtype != VM_U8 || cn != 3)) return fail(VM_EINVAL, "warp_image: the illumination change needs u8 BGR");
  if ((long)h * w >= (1L << 31) || (long)ih * iw >= (1L << 31))
    return fail(VM_EUNSUPPORTED, "warp_image: more than 2^31 pixels");
  const Affine a = invert_affine(m);
  Lut256 l{};
  if (lut)
    for (int i = 0; i < 256; ++i) l.t[i] = lut[i];
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g(grid_for((long)h * w, 256)), b(256);
  switch (dtype) {
    case VM_U8:
      if (lut)
        hipLaunchKernelGGL((warp_image_kernel<uint8_t, true>), g, b, 0, st, static_cast<const uint8_t*>(src), ih, iw,
                           cn, tu, tv, a, l, static_cast<uint8_t*>(dst), h, w);
      else
        hipLaunchKernelGGL((warp_image_kernel<uint8_t, false>), g, b, 0, st, static_cast<const uint8_t*>(src), ih, iw,
                           cn, tu, tv, a, l, static_cast<uint8_t*>(dst), h, w);
      break;
    case VM_F32:
      hipLaunchKernelGGL((warp_image_kernel<float, false>), g, b, 0, st, static_cast<const float*>(src), ih, iw, cn,
                         tu, tv, a, l, static_cast<float*>(dst), h, w);
      break;
    case VM_F64:
      hipLaunchKernelGGL((warp_image_kernel<double, false>), g, b, 0, st, static_cast<const double*>(src), ih, iw, cn,
                         tu, tv, a, l, static_cast<double*>(dst), h, w);
      break;
    default: return fail(VM_EUNSUPPORTED, "warp_image: dtype %d", dtype);
  }
  return check_launch("warp_image");
}

extern "C" int vm_warp_affine(const void* src, int ih, int iw, int cn, int dtype, const double* m, void* dst, int h,
                              int w, void* stream) {
  if (!src || !dst || !m || ih <= 0 || iw <= 0 || cn <= 0 || h <= 0 || w <= 0)
    return fail(VM_EINVAL, "warp_affine: bad argument");
  if (dtype == VM_U8 && cn > 8) return fail(VM_EUNSUPPORTED, "warp_affine: uint8 images with more than 8 channels");
  if ((long)h * w >= (1L << 31)) return fail(VM_EUNSUPPORTED, "warp_affine: more than 2^31 pixels");
  const Affine a = invert_affine(m);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g(grid_for((long)h * w, 256)), b(256);
  switch (dtype) {
    case VM_U8:
      hipLaunchKernelGGL(warp_affine_kernel<uint8_t>, g, b, 0, st, static_cast<const uint8_t*>(src), ih, iw, cn, a,
                         static_cast<uint8_t*>(dst), h, w);
      break;
    case VM_F32:
      hipLaunchKernelGGL(warp_affine_kernel<float>, g, b, 0, st, static_cast<const float*>(src), ih, iw, cn, a,
                         static_cast<float*>(dst), h, w);
      break;
    case VM_F64:
      hipLaunchKernelGGL(warp_affine_kernel<double>, g, b, 0, st, static_cast<const double*>(src), ih, iw, cn, a,
                         static_cast<double*>(dst), h, w);
      break;
    default: return fail(VM_EUNSUPPORTED, "warp_affine: dtype %d", dtype);
  }
  return check_launch("warp_affine");
}

extern "C" int vm_change_illumination_u8(const uint8_t* bgr, long pixels, const uint8_t* lut, uint8_t* out,
                                         void* stream) {
  if (!bgr || !lut || !out || pixels <= 0) return fail(VM_EINVAL, "change_illumination: bad argument");
  Lut256 l;
  for (int i = 0; i < 256; ++i) l.t[i] = lut[i];
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(illumination_kernel, dim3(grid_for(pixels, 256)), dim3(256), 0, st, bgr, pixels, l, out);
  return check_launch("change_illumination");
}

extern "C" int vm_nonzero_stats(const void* alpha, int h, int w, int dtype, long long* stats, void* stream) {
  if (!alpha || !stats || h <= 0 || w <= 0) return fail(VM_EINVAL, "nonzero_stats: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(stats, 0, 3 * sizeof(long long), st) != hipSuccess) return fail(VM_EHIP, "nonzero_stats: memset");
  auto* s = reinterpret_cast<unsigned long long*>(stats);
  const dim3 g(h < 1024 ? h : 1024), b(256);
  switch (dtype) {
    case VM_F64:
      hipLaunchKernelGGL(nonzero_stats_kernel<double>, g, b, 0, st, static_cast<const double*>(alpha), h, w, s);
      break;
    case VM_F32:
      hipLaunchKernelGGL(nonzero_stats_kernel<float>, g, b, 0, st, static_cast<const float*>(alpha), h, w, s);
      break;
    case VM_U8:
      hipLaunchKernelGGL(nonzero_stats_kernel<uint8_t>, g, b, 0, st, static_cast<const uint8_t*>(alpha), h, w, s);
      break;
    default: return fail(VM_EUNSUPPORTED, "nonzero_stats: dtype %d", dtype);
  }
  return check_launch("nonzero_stats");
}


extern "C" int vm_bgra_u8(const uint8_t* fg, const void* alpha, int alpha_dtype, long pixels, uint8_t* out,
                          void* stream) {
  if (!fg || !alpha || !out || pixels <= 0 || reinterpret_cast<uintptr_t>(out) % 4)
    return fail(VM_EINVAL, "bgra: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g(grid_for(pixels, 256)), b(256);
  uint32_t* o = reinterpret_cast<uint32_t*>(out);
  switch (alpha_dtype) {
    case VM_F64: hipLaunchKernelGGL(bgra_kernel<double>, g, b, 0, st, fg, static_cast<const double*>(alpha), pixels, o);
      break;
    case VM_F32: hipLaunchKernelGGL(bgra_kernel<float>, g, b, 0, st, fg, static_cast<const float*>(alpha), pixels, o);
      break;
    default: return fail(VM_EUNSUPPORTED, "bgra: alpha dtype %d", alpha_dtype);
  }
  return check_launch("bgra");
}

extern "C" int vm_trimap_from_matte(const double* matte, int h, int w, int dilate, int crop, uint8_t* trimap,
                                    void* stream) {
  if (!matte || !trimap || h <= 0 || w <= 0 || dilate < 0 || crop < 0)
    return fail(VM_EINVAL, "trimap_from_matte: bad argument");
  if (dilate > kTriMaxSide || crop > kTriMaxSide)
    return fail(VM_EUNSUPPORTED, "trimap_from_matte: dilate/crop above %d", kTriMaxSide);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 g((w + kTriW - 1) / kTriW, (h + kTriH - 1) / kTriH), b(256);
  hipLaunchKernelGGL(trimap_kernel, g, b, 0, st, matte, h, w, dilate, crop, trimap);
  return check_launch("trimap_from_matte");
}

// ---------------------------------------------------------------------------------------------------- batches (C ABI)
// scratch of one sample: the TPS lattice [2][h/2][w/2] f64, the resampled fg [(h+1)(w+1)][3] u8 and alpha f64
static void aug_lattice(int h, int w, int& nx, int& ny, double& xstep, double& ystep, double& xsteps, double& ysteps) {
  // tps._make_inverse_warp with output_region (0, 0, h, w), approximate_grid 2 (augmentation.py:49-54): x_steps =
  // h / 2 (a float), np.mgrid[0:h:x_steps*1j] -> int(x_steps) points, step h / (count - 1) (tps.py:46-51, 55-63)
  xsteps = (double)h / 2.0;
  ysteps = (double)w / 2.0;
  nx = (int)xsteps;
  ny = (int)ysteps;
  xstep = nx > 1 ? (double)h / (double)(nx - 1) : 1.0;
  ystep = ny > 1 ? (double)w / (double)(ny - 1) : 1.0;
}

static size_t al16(size_t b) { return (b + 255) & ~(size_t)255; }

extern "C" size_t vm_augment_scratch_bytes(int h, int w) {
  if (h <= 0 || w <= 0) return 0;
  int nx, ny;
  double a, b, c, d;
  aug_lattice(h, w, nx, ny, a, b, c, d);
  const size_t px = (size_t)(h + 1) * (w + 1);
  return al16(2 * (size_t)nx * ny * 8) + al16(px * 3) + al16(px * 8) + al16((size_t)(h + w + 2) * sizeof(UpAxis));
}

extern "C" int vm_augment_batch(const vm_augment_job* jobs, int n, void* stream) {
  if (!jobs || n <= 0) return fail(VM_EINVAL, "augment_batch: bad argument");
  for (int i = 0; i < n; ++i) {
    const vm_augment_job& q = jobs[i];
    if (!q.fg || !q.bg || !q.alpha || !q.tps_points || !q.tps_coeffs || !q.scratch || !q.new_fg || !q.new_bg ||
        !q.new_alpha || q.h < 4 || q.w < 4 || q.bg_h <= 0 || q.bg_w <= 0 || q.npts <= 0 ||
        reinterpret_cast<uintptr_t>(q.new_bgra) % 4)
      return fail(VM_EINVAL, "augment_batch: job %d: bad argument", i);
    if ((long)(q.h + 1) * (q.w + 1) >= (1L << 31) || (long)q.bg_h * q.bg_w >= (1L << 31))
      return fail(VM_EUNSUPPORTED, "augment_batch: job %d: more than 2^31 pixels", i);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int b0 = 0; b0 < n; b0 += kAugJobs) {
    const int m = n - b0 < kAugJobs ? n - b0 : kAugJobs;
    AugGridJobs G{};
    AugSampleJobs S{};
    AugWarpU8Jobs U{};
    AugWarpObjJobs O{};
    long gmax = 1, pmax = 1, wmax = 1, bmax = 1;
    for (int k = 0; k < m; ++k) {
      const vm_augment_job& q = jobs[b0 + k];
      int nx, ny;
      double xstep, ystep, xsteps, ysteps;
      aug_lattice(q.h, q.w, nx, ny, xstep, ystep, xsteps, ysteps);
      char* sc = static_cast<char*>(q.scratch);
      double* grid = reinterpret_cast<double*>(sc);
      const size_t px = (size_t)(q.h + 1) * (q.w + 1);
      uint8_t* fg_t = reinterpret_cast<uint8_t*>(sc + al16(2 * (size_t)nx * ny * 8));
      double* al_t = reinterpret_cast<double*>(sc + al16(2 * (size_t)nx * ny * 8) + al16(px * 3));
      UpAxis* axes = reinterpret_cast<UpAxis*>(sc + al16(2 * (size_t)nx * ny * 8) + al16(px * 3) + al16(px * 8));
      G.pts[k] = q.tps_points;
      G.coef[k] = q.tps_coeffs;
      G.grid[k] = grid;
      G.npts[k] = q.npts;
      G.nx[k] = nx;
      G.ny[k] = ny;
      G.xstep[k] = xstep;
      G.ystep[k] = ystep;
      G.axes[k] = axes;
      G.h[k] = q.h;
      G.w[k] = q.w;
      G.xsteps[k] = xsteps;
      G.ysteps[k] = ysteps;
      S.axes[k] = axes;
      gmax = gmax > (long)nx * ny ? gmax : (long)nx * ny;
      S.grid[k] = grid;
      S.fg[k] = q.fg;
      S.al[k] = q.alpha;
      S.fg_t[k] = fg_t;
      S.al_t[k] = al_t;
      S.h[k] = q.h;
      S.w[k] = q.w;
      S.nx[k] = nx;
      S.ny[k] = ny;
      S.xsteps[k] = xsteps;
      S.ysteps[k] = ysteps;
      pmax = pmax > (long)px ? pmax : (long)px;
      // camera motion on the background (its own size); object motion on the resampled fg and alpha, one pass
      U.src[k] = q.bg;
      U.dst[k] = q.new_bg;
      U.ih[k] = U.h[k] = q.bg_h;
      U.iw[k] = U.w[k] = q.bg_w;
      U.tu[k] = q.tu_bg;
      U.tv[k] = q.tv_bg;
      U.a[k] = invert_affine(q.m_bg);
      for (int i = 0; i < 256; ++i) U.lut[k].t[i] = O.lut[k].t[i] = q.lut[i];
      bmax = bmax > (long)q.bg_h * q.bg_w ? bmax : (long)q.bg_h * q.bg_w;
      O.fg[k] = fg_t;
      O.al[k] = al_t;
      O.dfg[k] = q.new_fg;
      O.dal[k] = q.new_alpha;
      O.bgra[k] = reinterpret_cast<uint32_t*>(q.new_bgra);
      O.ih[k] = q.h + 1;
      O.iw[k] = q.w + 1;
      O.h[k] = q.h;
      O.w[k] = q.w;
      O.tu[k] = q.tu_fg;
      O.tv[k] = q.tv_fg;
      O.a[k] = invert_affine(q.m_fg);
      wmax = wmax > (long)q.h * q.w ? wmax : (long)q.h * q.w;
    }
    hipLaunchKernelGGL(tps_grid_batch_kernel, dim3(grid_for(gmax, 256, 1024), m), dim3(256), 0, st, G);
    hipLaunchKernelGGL(tps_sample_pair_kernel, dim3(grid_for(pmax, 256, 1024), m), dim3(256), 0, st, S);
    hipLaunchKernelGGL(warp_bg_batch_kernel, dim3(grid_for(bmax, 256, 1024), m), dim3(256), 0, st, U);
    hipLaunchKernelGGL(warp_object_batch_kernel, dim3(grid_for(wmax, 256, 1024), m), dim3(256), 0, st, O);
  }
  return check_launch("augment_batch");
}

extern "C" int vm_nonzero_stats_batch(const double* const* alphas, const int* h, const int* w, int n,
                                      long long* stats, void* stream) {
  if (!alphas || !h || !w || !stats || n <= 0) return fail(VM_EINVAL, "nonzero_stats_batch: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(stats, 0, 3 * sizeof(long long) * (size_t)n, st) != hipSuccess)
    return fail(VM_EHIP, "nonzero_stats_batch: memset");
  for (int b0 = 0; b0 < n; b0 += 2 * kAugJobs) {
    const int m = n - b0 < 2 * kAugJobs ? n - b0 : 2 * kAugJobs;
    AugStatsJobs J{};
    int hmax = 1;
    for (int k = 0; k < m; ++k) {
      if (!alphas[b0 + k] || h[b0 + k] <= 0 || w[b0 + k] <= 0) return fail(VM_EINVAL, "nonzero_stats_batch: job %d", b0 + k);
      J.a[k] = alphas[b0 + k];
      J.h[k] = h[b0 + k];
      J.w[k] = w[b0 + k];
      hmax = hmax > h[b0 + k] ? hmax : h[b0 + k];
    }
    hipLaunchKernelGGL(nonzero_stats_batch_kernel, dim3(hmax < 1024 ? hmax : 1024, m), dim3(256), 0, st, J,
                       reinterpret_cast<unsigned long long*>(stats + 3 * (long)b0));
  }
  return check_launch("nonzero_stats_batch");
}

extern "C" int vm_bgra_u8_batch(const uint8_t* const* fg, const double* const* alpha, const long* pixels,
                                uint8_t* const* out, int n, void* stream) {
  if (!fg || !alpha || !pixels || !out || n <= 0) return fail(VM_EINVAL, "bgra_batch: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int b0 = 0; b0 < n; b0 += 2 * kAugJobs) {
    const int m = n - b0 < 2 * kAugJobs ? n - b0 : 2 * kAugJobs;
    AugBgraJobs J{};
    long pmax = 1;
    for (int k = 0; k < m; ++k) {
      const int i = b0 + k;
      if (!fg[i] || !alpha[i] || !out[i] || pixels[i] <= 0 || reinterpret_cast<uintptr_t>(out[i]) % 4)
        return fail(VM_EINVAL, "bgra_batch: job %d", i);
      J.fg[k] = fg[i];
      J.al[k] = alpha[i];
      J.out[k] = reinterpret_cast<uint32_t*>(out[i]);
      J.px[k] = pixels[i];
      pmax = pmax > pixels[i] ? pmax : pixels[i];
    }
    hipLaunchKernelGGL(bgra_batch_kernel, dim3(grid_for(pmax, 256, 1024), m), dim3(256), 0, st, J);
  }
  return check_launch("bgra_batch");
}
