// Memory-bound NHWC kernels: max-pool, TF-1 bilinear resize, dtype/pad conversion,
// batch-norm statistics + apply, channel softmax.  All vectorised to 16-byte accesses
// when the view allows (gfx950 Guideline 13), element-wise otherwise.

#include "vm_common.h"

namespace vm {

struct View {
  char* p;
  int n, h, w, c, cs, coff, dt;
};

static View view(const vm_tensor* t) {
  View v;
  v.p = reinterpret_cast<char*>(t->ptr);
  v.n = t->n; v.h = t->h; v.w = t->w; v.c = t->c; v.cs = t->cstride; v.coff = t->coff; v.dt = t->dtype;
  return v;
}

__device__ __forceinline__ float ldv(const View& v, long pix, int c) {
  const long o = pix * v.cs + v.coff + c;
  return v.dt == VM_F32 ? reinterpret_cast<const float*>(v.p)[o] : bf2f(reinterpret_cast<const uint16_t*>(v.p)[o]);
}

__device__ __forceinline__ void stv(const View& v, long pix, int c, float x) {
  const long o = pix * v.cs + v.coff + c;
  if (v.dt == VM_F32) reinterpret_cast<float*>(v.p)[o] = x;
  else reinterpret_cast<uint16_t*>(v.p)[o] = f2bf(x);
}

// 16-byte chunk of CE channels starting at channel c (caller guarantees alignment)
template <typename T>
__device__ __forceinline__ void ldc(const View& v, long pix, int c, float* f) {
  const T* base = reinterpret_cast<const T*>(v.p) + pix * v.cs + v.coff + c;
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(base), f);
}
template <typename T>
__device__ __forceinline__ void stc(const View& v, long pix, int c, const float* f) {
  T* base = reinterpret_cast<T*>(v.p) + pix * v.cs + v.coff + c;
  *reinterpret_cast<uint4*>(base) = Chunk<T>::pack(f);
}

// ---------------------------------------------------------------- max pool 2x2 / 2, SAME
// tf.nn.max_pool SAME (unet.py:33): out = ceil(n/2), pad_before 0, padded taps never win.
template <typename T, bool VEC>
__global__ void maxpool2x2_kernel(View x, View y) {
  constexpr int CE = VEC ? 16 / sizeof(T) : 1;
  const int cpp = (y.c + CE - 1) / CE;
  const long total = (long)y.n * y.h * y.w * cpp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpp);
    const long op = i / cpp;
    const int ow = (int)(op % y.w);
    const long t = op / y.w;
    const int oh = (int)(t % y.h);
    const int n = (int)(t / y.h);
    const int ih = 2 * oh, iw = 2 * ow;
    const long p00 = ((long)n * x.h + ih) * x.w + iw;
    const bool hasr = iw + 1 < x.w, hasd = ih + 1 < x.h;
    const int c = cc * CE;
    if (VEC) {
      float m[CE], f[CE];
      ldc<T>(x, p00, c, m);
      if (hasr) { ldc<T>(x, p00 + 1, c, f); for (int j = 0; j < CE; ++j) m[j] = fmaxf(m[j], f[j]); }
      if (hasd) { ldc<T>(x, p00 + x.w, c, f); for (int j = 0; j < CE; ++j) m[j] = fmaxf(m[j], f[j]); }
      if (hasr && hasd) { ldc<T>(x, p00 + x.w + 1, c, f); for (int j = 0; j < CE; ++j) m[j] = fmaxf(m[j], f[j]); }
      stc<T>(y, op, c, m);
    } else {
      float m = ldv(x, p00, c);
      if (hasr) m = fmaxf(m, ldv(x, p00 + 1, c));
      if (hasd) m = fmaxf(m, ldv(x, p00 + x.w, c));
      if (hasr && hasd) m = fmaxf(m, ldv(x, p00 + x.w + 1, c));
      stv(y, op, c, m);
    }
  }
}

// Row-blocked vector variant: block b covers chunks [part*256, part*256+256) of output row b / bpr, so the
// (n, oh) decode is wave-uniform and each lane only splits its chunk index into (ow, channel chunk).
template <typename T>
__global__ __launch_bounds__(256) void maxpool2x2_rows(View x, View y, int bpr) {
  constexpr int CE = 16 / sizeof(T);
  const int row = blockIdx.x / bpr;
  const int part = blockIdx.x - row * bpr;
  const int n = row / y.h, oh = row - n * y.h;
  const int cpp = y.c / CE;
  const int i = part * 256 + threadIdx.x;
  if (i >= y.w * cpp) return;
  const int ow = i / cpp, c = (i - ow * cpp) * CE;
  const int ih = 2 * oh, iw = 2 * ow;
  const long p00 = ((long)n * x.h + ih) * x.w + iw;
  const bool hasr = iw + 1 < x.w, hasd = ih + 1 < x.h;
  const T* xb = reinterpret_cast<const T*>(x.p) + x.coff + c;
  const uint4 a = *reinterpret_cast<const uint4*>(xb + p00 * x.cs);
  const uint4 b = *reinterpret_cast<const uint4*>(xb + (p00 + (hasr ? 1 : 0)) * x.cs);
  const uint4 d = *reinterpret_cast<const uint4*>(xb + (p00 + (hasd ? x.w : 0)) * x.cs);
  const uint4 e = *reinterpret_cast<const uint4*>(xb + (p00 + (hasd ? x.w : 0) + (hasr ? 1 : 0)) * x.cs);
  float m[CE], f[CE];
  Chunk<T>::unpack(a, m);
  Chunk<T>::unpack(b, f);
#pragma unroll
  for (int j = 0; j < CE; ++j) m[j] = fmaxf(m[j], f[j]);
  Chunk<T>::unpack(d, f);
#pragma unroll
  for (int j = 0; j < CE; ++j) m[j] = fmaxf(m[j], f[j]);
  Chunk<T>::unpack(e, f);
#pragma unroll
  for (int j = 0; j < CE; ++j) m[j] = fmaxf(m[j], f[j]);
  T* yb = reinterpret_cast<T*>(y.p) + ((long)row * y.w + ow) * y.cs + y.coff + c;
  *reinterpret_cast<uint4*>(yb) = Chunk<T>::pack(m);
}

// ---------------------------------------------------------------- TF-1.x legacy bilinear resize
// tf.image.resize_images (unet.py:58): scale = (float)in/out, src = (float)dst * scale,
// lo = floor(src), hi = min(lo + 1, in - 1), lerp = src - floor(src);
// top = tl + (tr - tl) * xl; bot = bl + (br - bl) * xl; out = top + (bot - top) * yl.
// TF's scaler runs in plain float32; contraction would fuse (float)i*scale into src - floor(src)
// and produce a MORE precise lerp than TF's — kept off for the coordinate arithmetic.
__device__ __forceinline__ void tf1_coord(int i, float scale, int in, int& lo, int& hi, float& lerp) {
#pragma clang fp contract(off)
  const float src = (float)i * scale;
  const float fl = floorf(src);
  lo = (int)fl;
  hi = min(lo + 1, in - 1);
  lerp = src - fl;
}

template <typename T, bool VEC>
__global__ void resize_tf1_kernel(View x, View y, float sy, float sx) {
  constexpr int CE = VEC ? 16 / sizeof(T) : 1;
  const int cpp = (y.c + CE - 1) / CE;
  const long total = (long)y.n * y.h * y.w * cpp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpp);
    const long op = i / cpp;
    const int ow = (int)(op % y.w);
    const long t = op / y.w;
    const int oh = (int)(t % y.h);
    const int n = (int)(t / y.h);
    int y0, y1, x0, x1;
    float yl, xl;
    tf1_coord(oh, sy, x.h, y0, y1, yl);
    tf1_coord(ow, sx, x.w, x0, x1, xl);
    const long rb = (long)n * x.h;
    const long ptl = (rb + y0) * x.w + x0, ptr_ = (rb + y0) * x.w + x1;
    const long pbl = (rb + y1) * x.w + x0, pbr = (rb + y1) * x.w + x1;
    const int c = cc * CE;
    if (VEC) {
      float tl[CE], tr[CE], bl[CE], br[CE], o[CE];
      ldc<T>(x, ptl, c, tl); ldc<T>(x, ptr_, c, tr); ldc<T>(x, pbl, c, bl); ldc<T>(x, pbr, c, br);
#pragma unroll
      for (int j = 0; j < CE; ++j) {
#pragma clang fp contract(off)
        const float top = tl[j] + (tr[j] - tl[j]) * xl;
        const float bot = bl[j] + (br[j] - bl[j]) * xl;
        o[j] = top + (bot - top) * yl;
      }
      stc<T>(y, op, c, o);
    } else {
#pragma clang fp contract(off)
      const float vtl = ldv(x, ptl, c), vtr = ldv(x, ptr_, c), vbl = ldv(x, pbl, c), vbr = ldv(x, pbr, c);
      const float top = vtl + (vtr - vtl) * xl;
      const float bot = vbl + (vbr - vbl) * xl;
      stv(y, op, c, top + (bot - top) * yl);
    }
  }
}

// Row-blocked vector variant (see maxpool2x2_rows): the vertical taps and weight are wave-uniform.
template <typename T>
__global__ __launch_bounds__(256) void resize_tf1_rows(View x, View y, float sy, float sx, int bpr) {
  constexpr int CE = 16 / sizeof(T);
  const int row = blockIdx.x / bpr;
  const int part = blockIdx.x - row * bpr;
  const int n = row / y.h, oh = row - n * y.h;
  const int cpp = y.c / CE;
  const int i = part * 256 + threadIdx.x;
  if (i >= y.w * cpp) return;
  const int ow = i / cpp, c = (i - ow * cpp) * CE;
  int y0, y1, x0, x1;
  float yl, xl;
  tf1_coord(oh, sy, x.h, y0, y1, yl);
  tf1_coord(ow, sx, x.w, x0, x1, xl);
  const T* xb = reinterpret_cast<const T*>(x.p) + x.coff + c;
  const long r0 = ((long)n * x.h + y0) * x.w, r1 = ((long)n * x.h + y1) * x.w;
  const uint4 qtl = *reinterpret_cast<const uint4*>(xb + (r0 + x0) * x.cs);
  const uint4 qtr = *reinterpret_cast<const uint4*>(xb + (r0 + x1) * x.cs);
  const uint4 qbl = *reinterpret_cast<const uint4*>(xb + (r1 + x0) * x.cs);
  const uint4 qbr = *reinterpret_cast<const uint4*>(xb + (r1 + x1) * x.cs);
  float tl[CE], tr[CE], bl[CE], br[CE], o[CE];
  Chunk<T>::unpack(qtl, tl);
  Chunk<T>::unpack(qtr, tr);
  Chunk<T>::unpack(qbl, bl);
  Chunk<T>::unpack(qbr, br);
#pragma unroll
  for (int j = 0; j < CE; ++j) {
#pragma clang fp contract(off)
    const float top = tl[j] + (tr[j] - tl[j]) * xl;
    const float bot = bl[j] + (br[j] - bl[j]) * xl;
    o[j] = top + (bot - top) * yl;
  }
  T* yb = reinterpret_cast<T*>(y.p) + ((long)row * y.w + ow) * y.cs + y.coff + c;
  *reinterpret_cast<uint4*>(yb) = Chunk<T>::pack(o);
}

// Exact 2x upsampling (y = 2 * x in both dims, scale 0.5): every output pixel's taps are the low-res pixels
// (i|i+1, j|j+1) of its 2x2 quad, so one lane loads those 4 chunks once and writes the 4 outputs of the quad —
// the same float32 arithmetic as resize_tf1_kernel (lerp 0 or 0.5), bit-identical results.
template <typename T>
__global__ __launch_bounds__(256) void resize2x_tf1_rows(View x, View y, int bpr) {
  constexpr int CE = 16 / sizeof(T);
  const int row = blockIdx.x / bpr;  // low-res row n*x.h + i
  const int part = blockIdx.x - row * bpr;
  const int n = row / x.h, i = row - n * x.h;
  const int cpp = y.c / CE;
  const int t = part * 256 + threadIdx.x;
  if (t >= x.w * cpp) return;
  const int j = t / cpp, c = (t - j * cpp) * CE;
  const int i1 = min(i + 1, x.h - 1), j1 = min(j + 1, x.w - 1);
  const T* xb = reinterpret_cast<const T*>(x.p) + x.coff + c;
  const long r0 = ((long)n * x.h + i) * x.w, r1 = ((long)n * x.h + i1) * x.w;
  float a00[CE], a01[CE], a10[CE], a11[CE];
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(xb + (r0 + j) * x.cs), a00);
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(xb + (r0 + j1) * x.cs), a01);
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(xb + (r1 + j) * x.cs), a10);
  Chunk<T>::unpack(*reinterpret_cast<const uint4*>(xb + (r1 + j1) * x.cs), a11);
  T* yb = reinterpret_cast<T*>(y.p) + y.coff + c;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy) {
    const int oy = 2 * i + dy;
    if (oy >= y.h) break;
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int ox = 2 * j + dx;
      if (ox >= y.w) break;
      int ly0, ly1, lx0, lx1;
      float fy, fx;
      tf1_coord(oy, 0.5f, x.h, ly0, ly1, fy);
      tf1_coord(ox, 0.5f, x.w, lx0, lx1, fx);
      // taps: (ly0, lx0) = (i, j); ly1 / lx1 are i1 / j1 when the lerp is nonzero, else they equal i / j
      const float* tl = a00;
      const float* tr = (lx1 == lx0) ? a00 : a01;
      const float* bl = (ly1 == ly0) ? a00 : a10;
      const float* br = (ly1 == ly0) ? tr : ((lx1 == lx0) ? a10 : a11);
      float o[CE];
#pragma unroll
      for (int e = 0; e < CE; ++e) {
#pragma clang fp contract(off)
        const float top = tl[e] + (tr[e] - tl[e]) * fx;
        const float bot = bl[e] + (br[e] - bl[e]) * fx;
        o[e] = top + (bot - top) * fy;
      }
      *reinterpret_cast<uint4*>(yb + (((long)n * y.h + oy) * y.w + ox) * y.cs) = Chunk<T>::pack(o);
    }
  }
}

// ---------------------------------------------------------------- convert / pad / affine
__device__ __forceinline__ float convert_one(const View& x, long p, int c, const float* scale, const float* shift,
                                             int act) {
  float v = ldv(x, p, c);
  if (scale) v *= scale[c];
  if (shift) v += shift[c];
  return act == VM_ACT_RELU ? fmaxf(v, 0.f) : act == VM_ACT_SIGMOID ? sigmoid_precise(v) : v;
}

__global__ void convert_kernel(View x, View y, const float* scale, const float* shift, int act) {
  const long total = (long)y.n * y.h * y.w * y.c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % y.c);
    const long p = i / y.c;
    stv(y, p, c, c < x.c ? convert_one(x, p, c, scale, shift, act) : 0.f);
  }
}

// narrow outputs (y.c <= 16: the network inputs, pads and channel slices): one thread per pixel walks its channels,
// so no element index is divided (the 64-bit i / y.c above costs more than the copy)
__global__ void convert_px_kernel(View x, View y, const float* scale, const float* shift, int act) {
  const long M = (long)y.n * y.h * y.w;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < M; p += (long)gridDim.x * blockDim.x)
    for (int c = 0; c < y.c; ++c) stv(y, p, c, c < x.c ? convert_one(x, p, c, scale, shift, act) : 0.f);
}

// one 16-byte chunk of 8 bf16 channels per pixel (the training towers' 8-channel input frames, loader outputs): the
// per-channel 2-byte stores of convert_px_kernel ran these at ~0.7 TB/s
__global__ void convert_px8_bf16_kernel(View x, View y, const float* scale, const float* shift, int act) {
  const long M = (long)y.n * y.h * y.w;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < M; p += (long)gridDim.x * blockDim.x) {
    float f[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) f[c] = c < x.c ? convert_one(x, p, c, scale, shift, act) : 0.f;
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(y.p) + p * y.cs + y.coff) = Chunk<uint16_t>::pack(f);
  }
}

// f32 -> bf16 of whole 8-channel runs (the UNetImage backward's bf16 copies of its upconv gradients: the element-wise
// kernel above ran them at ~2.2 TB/s): two f32x4 loads and one 16-byte store per lane, the same f2bf rounding
__global__ void convert8_f32_bf16_kernel(const float* __restrict__ x, int xcs, uint16_t* __restrict__ y, int ycs,
                                         long M, int c8) {
  const long total = M * c8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / c8;
    const int c = (int)(i - p * c8) * 8;
    const float4 a = *reinterpret_cast<const float4*>(x + p * xcs + c);
    const float4 b = *reinterpret_cast<const float4*>(x + p * xcs + c + 4);
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    *reinterpret_cast<uint4*>(y + p * ycs + c) = Chunk<uint16_t>::pack(f);
  }
}

// ---------------------------------------------------------------- batch-norm statistics
// tf.contrib.layers.batch_norm(is_training=True) (unet_simple.py:25): per-channel mean and biased
// variance over N*H*W.  Pass 1: grid (ceil(C/64), nblk); lane = channel (64 consecutive channels of a
// pixel per wave -> coalesced), the 4 waves of a block stride over pixels, f64 partial sums,
// combined across waves in LDS.  Pass 2: one thread per channel folds the nblk partials.
long g_bn_target = 4096;  // vm_common.h bn_blocks

// CP = lanes per pixel: 64 for c > 32 (a block covers 64 channels of each pixel, blockIdx.x picks the group);
// for narrow tensors CP = next power of two >= c, so one wave reads 64 / CP pixels per step instead of idling lanes.
template <typename T, int CP>
__global__ __launch_bounds__(256) void bn_partial_kernel(View x, double* part, int nblk) {
  constexpr int PPW = 64 / CP;
  __shared__ double sh[2][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * CP + (lane % CP);
  const long M = (long)x.n * x.h * x.w;
  double s = 0.0, ss = 0.0;
  if (c < x.c) {
    const long stp = (long)nblk * 4 * PPW;
    long p = ((long)blockIdx.y * 4 + wave) * PPW + lane / CP;
    for (; p + 3 * stp < M; p += 4 * stp) {  // 4 loads in flight per lane (same summation order)
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = ldv(x, p + u * stp, c);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += v[u];
        ss += v[u] * v[u];
      }
    }
    for (; p < M; p += stp) {
      const double v = ldv(x, p, c);
      s += v;
      ss += v * v;
    }
  }
  sh[0][wave][lane] = s;
  sh[1][wave][lane] = ss;
  __syncthreads();
  if ((int)threadIdx.x < CP && c < x.c) {
    s = ss = 0.0;
    for (int w = 0; w < 4; ++w)
      for (int k = 0; k < PPW; ++k) {
        s += sh[0][w][k * CP + threadIdx.x];
        ss += sh[1][w][k * CP + threadIdx.x];
      }
    part[(long)c * nblk + blockIdx.y] = s;  // channel-major [k][C][nblk]: the fold reads each channel's run
    part[(long)nblk * x.c + (long)c * nblk + blockIdx.y] = ss;
  }
}

// one block per channel folds the nblk partials (vm_common.h fold_columns)
__global__ __launch_bounds__(256) void bn_final_kernel(const double* part, int nblk, int C, long M, float* mean,
                                                       float* var) {
  const int c = blockIdx.x;
  double r[3];
  fold_columns(part, nblk, C, c, 2, r);
  if (threadIdx.x == 0) {
    const double m = r[0] / (double)M;
    double v = r[1] / (double)M - m * m;
    if (v < 0.0) v = 0.0;
    mean[c] = (float)m;
    var[c] = (float)v;
  }
}

template <typename T>
static int launch_bn_partial(const View& xv, double* part, hipStream_t st) {
  const int C = xv.c;
  const int nb = bn_blocks((long)xv.n * xv.h * xv.w, C);
  const int cp = C > 32 ? 64 : C > 16 ? 32 : C > 8 ? 16 : C > 4 ? 8 : C > 2 ? 4 : C > 1 ? 2 : 1;
  dim3 grid(cp == 64 ? (C + 63) / 64 : 1, nb);
  switch (cp) {
    case 1: hipLaunchKernelGGL((bn_partial_kernel<T, 1>), grid, dim3(256), 0, st, xv, part, nb); break;
    case 2: hipLaunchKernelGGL((bn_partial_kernel<T, 2>), grid, dim3(256), 0, st, xv, part, nb); break;
    case 4: hipLaunchKernelGGL((bn_partial_kernel<T, 4>), grid, dim3(256), 0, st, xv, part, nb); break;
    case 8: hipLaunchKernelGGL((bn_partial_kernel<T, 8>), grid, dim3(256), 0, st, xv, part, nb); break;
    case 16: hipLaunchKernelGGL((bn_partial_kernel<T, 16>), grid, dim3(256), 0, st, xv, part, nb); break;
    case 32: hipLaunchKernelGGL((bn_partial_kernel<T, 32>), grid, dim3(256), 0, st, xv, part, nb); break;
    default: hipLaunchKernelGGL((bn_partial_kernel<T, 64>), grid, dim3(256), 0, st, xv, part, nb); break;
  }
  return nb;
}

// CP (power of two >= C, at most 64) lanes per pixel, channel block blockIdx.y: each lane keeps one channel's
// constants in registers and no element index is divided
template <int CP>
__global__ __launch_bounds__(256) void bn_apply_kernel(View x, View y, const float* mean, const float* var,
                                                       const float* gamma, const float* beta, float eps, int act) {
  const long M = (long)x.n * x.h * x.w;
  const int c = blockIdx.y * CP + (threadIdx.x & (CP - 1));
  if (c >= x.c) return;
  const float m = mean ? mean[c] : 0.f;
  const float v = var ? var[c] : 1.f;
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  const float r = 1.0f / sqrtf(v + eps);
  const long step = (long)gridDim.x * (blockDim.x / CP);
  long p = (long)blockIdx.x * (blockDim.x / CP) + threadIdx.x / CP;
  for (; p + 3 * step < M; p += 4 * step) {  // 4 loads in flight before the stores (y may alias x: in place)
    float t[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) t[u] = ldv(x, p + u * step, c);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v = (t[u] - m) * r * g + b;
      v = act == VM_ACT_RELU ? fmaxf(v, 0.f) : act == VM_ACT_SIGMOID ? sigmoid_precise(v) : v;
      stv(y, p + u * step, c, v);
    }
  }
  for (; p < M; p += step) {
    float t = (ldv(x, p, c) - m) * r * g + b;
    t = act == VM_ACT_RELU ? fmaxf(t, 0.f) : act == VM_ACT_SIGMOID ? sigmoid_precise(t) : t;
    stv(y, p, c, t);
  }
}

// Whole 8-channel runs (C % 8 == 0, C <= 512, 16-byte aligned views): a lane takes 8 channels of a pixel, one or two
// 16-byte accesses per side where the per-channel forms issue one 2- / 4-byte access per element.  bn_partial8: the
// same f64 sums per channel over another partition of the pixels ([2][C][nblk] tables, bn_final_kernel folds them);
// bn_apply8: the same expression per element (y may alias x).
template <typename T>
__device__ __forceinline__ void ld8v(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    Chunk<uint16_t>::unpack(*reinterpret_cast<const uint4*>(p), v);
  }
}
template <typename T>
__device__ __forceinline__ void st8v(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    *reinterpret_cast<uint4*>(p) = Chunk<uint16_t>::pack(v);
  }
}

template <typename T, int TPG>
__global__ __launch_bounds__(256) void bn_partial8_kernel(const T* x, int xcs, long M, int C, double* part, int nblk) {
  constexpr int PPB = 256 / TPG;
  __shared__ double sh[8][256];
  const int t = threadIdx.x, j = t % TPG, pl = t / TPG, c0 = 8 * j;
  double s[8], ss[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = ss[k] = 0.0;
  if (c0 < C) {
    for (long p = (long)blockIdx.x * PPB + pl; p < M; p += (long)nblk * PPB) {
      float v[8];
      ld8v(x + p * xcs + c0, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double d = v[k];
        s[k] += d;
        ss[k] += d * d;
      }
    }
  }
#pragma unroll
  for (int tab = 0; tab < 2; ++tab) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[k][t] = tab ? ss[k] : s[k];
    __syncthreads();
    for (int c = t; c < C; c += 256) {
      const int jj = c >> 3, k = c & 7;
      double r = 0.0;
      for (int q = 0; q < PPB; ++q) r += sh[k][q * TPG + jj];
      part[(long)tab * nblk * C + (long)c * nblk + blockIdx.x] = r;  // channel-major, as bn_partial_kernel
    }
    __syncthreads();
  }
}

template <typename TX, typename TY, int TPG>
__global__ __launch_bounds__(256) void bn_apply8_kernel(const TX* x, int xcs, TY* y, int ycs, long M, int C,
                                                        const float* mean, const float* var, const float* gamma,
                                                        const float* beta, float eps, int act) {
  constexpr int PPB = 256 / TPG;
  const int t = threadIdx.x, j = t % TPG, pl = t / TPG, c0 = 8 * j;
  if (c0 >= C) return;
  float m[8], r[8], g[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    m[k] = mean ? mean[c] : 0.f;
    const float v = var ? var[c] : 1.f;
    g[k] = gamma ? gamma[c] : 1.f;
    b[k] = beta ? beta[c] : 0.f;
    r[k] = 1.0f / sqrtf(v + eps);
  }
  for (long p = (long)blockIdx.x * PPB + pl; p < M; p += (long)gridDim.x * PPB) {
    float v[8];
    ld8v(x + p * xcs + c0, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float u = (v[k] - m[k]) * r[k] * g[k] + b[k];
      v[k] = act == VM_ACT_RELU ? fmaxf(u, 0.f) : act == VM_ACT_SIGMOID ? sigmoid_precise(u) : u;
    }
    st8v(y + p * ycs + c0, v);
  }
}

// vm_set_option "bn_vec_fwd" (A/B, off): the 8-channel forms measured no faster in the config-5 step (4.75-4.76 vs
// 4.77-4.79 ms, same box: these passes run beside the select chains, where their 16 KB reduction buffer costs
// occupancy), unlike the backward's (train.hip bn_bwd_partial8 / apply8: -2 %)
long g_bn_vec_fwd = 0;

static bool vec8_view(const vm_tensor* t) {
  return t->cstride % 8 == 0 && t->coff % 8 == 0 && reinterpret_cast<uintptr_t>(t->ptr) % 16 == 0 && t->c % 8 == 0 &&
         t->c <= 512;
}
static int tpg8(int C) {
  return C / 8 > 32 ? 64 : C / 8 > 16 ? 32 : C / 8 > 8 ? 16 : C / 8 > 4 ? 8 : C / 8 > 2 ? 4 : C / 8 > 1 ? 2 : 1;
}

// two f32 channels per pixel, one pixel per thread, one 8-byte load and store each (the 2-channel select convs of the
// training step: at a 32-byte pixel stride the 2-lanes-per-pixel form above spent a dtype branch and a 64-bit index
// product per 4-byte element, ~0.8 TB/s).  Per element the same expression, so the same values.
__global__ __launch_bounds__(256) void bn_apply2_f32_kernel(const float* x, int xcs, float* y, int ycs,
                                                            long M, const float* mean, const float* var,
                                                            const float* gamma, const float* beta, float eps, int act) {
  float m[2], r[2], g[2], b[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    m[c] = mean ? mean[c] : 0.f;
    const float v = var ? var[c] : 1.f;
    g[c] = gamma ? gamma[c] : 1.f;
    b[c] = beta ? beta[c] : 0.f;
    r[c] = 1.0f / sqrtf(v + eps);
  }
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < M; p += (long)gridDim.x * blockDim.x) {
    const float2 t2 = *reinterpret_cast<const float2*>(x + p * xcs);
    float t[2] = {t2.x, t2.y};
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v = (t[c] - m[c]) * r[c] * g[c] + b[c];
      v = act == VM_ACT_RELU ? fmaxf(v, 0.f) : act == VM_ACT_SIGMOID ? sigmoid_precise(v) : v;
      t[c] = v;
    }
    *reinterpret_cast<float2*>(y + p * ycs) = make_float2(t[0], t[1]);
  }
}

static bool f32_pair_view(const vm_tensor* t) {  // 2 f32 channels at an 8-byte aligned offset of every pixel
  return t->dtype == VM_F32 && t->c == 2 && t->cstride % 2 == 0 && t->coff % 2 == 0 &&
         reinterpret_cast<uintptr_t>(t->ptr) % 8 == 0;
}

// ---------------------------------------------------------------- channel softmax (refine.py:31)
__global__ void softmax_kernel(View x, View y) {
  const long M = (long)x.n * x.h * x.w;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < M; p += (long)gridDim.x * blockDim.x) {
    float mx = -INFINITY;
    for (int c = 0; c < x.c; ++c) mx = fmaxf(mx, ldv(x, p, c));
    float s = 0.f;
    for (int c = 0; c < x.c; ++c) s += expf(ldv(x, p, c) - mx);
    const float inv = 1.f / s;
    for (int c = 0; c < x.c; ++c) stv(y, p, c, expf(ldv(x, p, c) - mx) * inv);
  }
}

static bool same_dtype_vec(const vm_tensor* x, const vm_tensor* y) {
  return x->dtype == y->dtype && x->c == y->c && vec16_ok(x) && vec16_ok(y);
}

}  // namespace vm

using namespace vm;

extern "C" int vm_maxpool2x2_same_nhwc(const vm_tensor* x, vm_tensor* y, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y)) return fail(VM_EINVAL, "maxpool: invalid tensor");
  if (y->n != x->n || y->h != (x->h + 1) / 2 || y->w != (x->w + 1) / 2 || y->c != x->c)
    return fail(VM_EINVAL, "maxpool: output must be [%d,%d,%d,%d]", x->n, (x->h + 1) / 2, (x->w + 1) / 2, x->c);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool vec = same_dtype_vec(x, y);
  const int ce = vec ? 16 / elem_bytes(x->dtype) : 1;
  const long work = (long)y->n * y->h * y->w * ((y->c + ce - 1) / ce);
  const int grid = grid_for(work, 256);
  View xv = view(x), yv = view(y);
  if (vec) {
    const int bpr = (int)(((long)y->w * (y->c / ce) + 255) / 256);
    const long blocks = (long)y->n * y->h * bpr;
    if (blocks > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "maxpool: output too large");
    if (x->dtype == VM_BF16) hipLaunchKernelGGL((maxpool2x2_rows<uint16_t>), dim3(blocks), dim3(256), 0, st, xv, yv, bpr);
    else hipLaunchKernelGGL((maxpool2x2_rows<float>), dim3(blocks), dim3(256), 0, st, xv, yv, bpr);
  } else {
    hipLaunchKernelGGL((maxpool2x2_kernel<float, false>), dim3(grid), dim3(256), 0, st, xv, yv);
  }
  return check_launch("maxpool2x2");
}

extern "C" int vm_resize_bilinear_tf1_nhwc(const vm_tensor* x, vm_tensor* y, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y)) return fail(VM_EINVAL, "resize: invalid tensor");
  if (y->n != x->n || y->c != x->c) return fail(VM_EINVAL, "resize: batch/channel mismatch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const float sy = (float)x->h / (float)y->h;
  const float sx = (float)x->w / (float)y->w;
  const bool vec = same_dtype_vec(x, y);
  const int ce = vec ? 16 / elem_bytes(x->dtype) : 1;
  const long work = (long)y->n * y->h * y->w * ((y->c + ce - 1) / ce);
  const int grid = grid_for(work, 256);
  View xv = view(x), yv = view(y);
  // same size: TF-1 resize_images returns its input; the kernel degenerates to a copy (lerp 0)
  if (vec && y->h == 2 * x->h && y->w == 2 * x->w) {
    const int bpr = (int)(((long)x->w * (y->c / ce) + 255) / 256);
    const long blocks = (long)x->n * x->h * bpr;
    if (blocks > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "resize: output too large");
    if (x->dtype == VM_BF16) hipLaunchKernelGGL((resize2x_tf1_rows<uint16_t>), dim3(blocks), dim3(256), 0, st, xv, yv, bpr);
    else hipLaunchKernelGGL((resize2x_tf1_rows<float>), dim3(blocks), dim3(256), 0, st, xv, yv, bpr);
  } else if (vec) {
    const int bpr = (int)(((long)y->w * (y->c / ce) + 255) / 256);
    const long blocks = (long)y->n * y->h * bpr;
    if (blocks > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "resize: output too large");
    if (x->dtype == VM_BF16)
      hipLaunchKernelGGL((resize_tf1_rows<uint16_t>), dim3(blocks), dim3(256), 0, st, xv, yv, sy, sx, bpr);
    else hipLaunchKernelGGL((resize_tf1_rows<float>), dim3(blocks), dim3(256), 0, st, xv, yv, sy, sx, bpr);
  } else {
    hipLaunchKernelGGL((resize_tf1_kernel<float, false>), dim3(grid), dim3(256), 0, st, xv, yv, sy, sx);
  }
  return check_launch("resize_tf1");
}


// ---------------------------------------------------------------- split-bf16 x6 operands (unet.py forward at f32 accuracy)
// An f32 activation x is held as three bf16 parts x = h + m + l (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m):
// both differences are exact in f32, so the parts carry x's 24 significant bits).  A conv over such an input is a
// bf16 MFMA conv over 6 channel slabs with exact bf16 x bf16 products and f32 sums: the slabs [l, m, h, m, h, h] meet
// the filter parts [h, m, l, h, m, h] packed along K, i.e. l*Wh + m*Wm + h*Wl + m*Wh + h*Wm + h*Wh — every product
// down to 2^-16 of the leading one, smallest first (the MFMA K loop sums granules in order, so the 2^-16 terms are
// summed while the accumulator is still small).  Layout of the split buffer: slab p of channel c at p*S + coff + c,
// S = cstride / 6 (the channel count of the whole concat this view is a segment of).
// POOL: the tile's 2x2 SAME max-pool of x (f32, before the split) is split into a second view of the same layout.
__device__ __forceinline__ void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f2bf(x);
  const float r1 = x - bf2f(h);
  m = f2bf(r1);
  l = f2bf(r1 - bf2f(m));
}

__device__ __forceinline__ void store_split6(uint16_t* base, long S, const float* v) {
  uint32_t wh[4], wm[4], wl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint16_t h0, m0, l0, h1, m1, l1;
    split3(v[2 * i], h0, m0, l0);
    split3(v[2 * i + 1], h1, m1, l1);
    wh[i] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    wm[i] = (uint32_t)m0 | ((uint32_t)m1 << 16);
    wl[i] = (uint32_t)l0 | ((uint32_t)l1 << 16);
  }
  const uint4 H = make_uint4(wh[0], wh[1], wh[2], wh[3]), M = make_uint4(wm[0], wm[1], wm[2], wm[3]),
              L = make_uint4(wl[0], wl[1], wl[2], wl[3]);
  *reinterpret_cast<uint4*>(base) = L;
  *reinterpret_cast<uint4*>(base + S) = M;
  *reinterpret_cast<uint4*>(base + 2 * S) = H;
  *reinterpret_cast<uint4*>(base + 3 * S) = M;
  *reinterpret_cast<uint4*>(base + 4 * S) = H;
  *reinterpret_cast<uint4*>(base + 5 * S) = H;
}

// one thread = one 8-channel chunk of one output pixel (POOL: of one pooled pixel and the 2x2 window under it)
template <bool POOL>
__global__ __launch_bounds__(256) void split6_kernel(View x, View y, View yp) {
  const int cpp = (y.c + 7) / 8;
  const long S = y.cs / 6;
  const int on = POOL ? yp.n : y.n, oh = POOL ? yp.h : y.h, ow = POOL ? yp.w : y.w;
  const long total = (long)on * oh * ow * cpp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpp);
    const long op = i / cpp;
    const int c = cc * 8;
    auto load = [&](long pix, float* f) {
      const float* src = reinterpret_cast<const float*>(x.p) + pix * x.cs + x.coff + c;
      if (c + 8 <= x.c && ((x.cs | x.coff) & 3) == 0 && (reinterpret_cast<uintptr_t>(x.p) & 15) == 0) {
        const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
        f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = c + j < x.c ? src[j] : 0.f;  // channels past x.c: zero padding
      }
    };
    auto out = [&](const View& v, long pix) {
      return reinterpret_cast<uint16_t*>(v.p) + pix * v.cs + v.coff + c;
    };
    if constexpr (!POOL) {
      float f[8];
      load(op, f);
      store_split6(out(y, op), S, f);
    } else {
      const int pw = (int)(op % yp.w);
      const long t = op / yp.w;
      const int ph = (int)(t % yp.h), n = (int)(t / yp.h);
      const int iy = 2 * ph, ix = 2 * pw;
      const bool hasr = ix + 1 < x.w, hasd = iy + 1 < x.h;
      const long p00 = ((long)n * x.h + iy) * x.w + ix;
      float f[8], m[8];
      load(p00, f);
      store_split6(out(y, p00), S, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = f[j];
      auto tap = [&](long pix) {
        load(pix, f);
        store_split6(out(y, pix), S, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
      };
      if (hasr) tap(p00 + 1);
      if (hasd) tap(p00 + x.w);
      if (hasr && hasd) tap(p00 + x.w + 1);
      store_split6(out(yp, op), yp.cs / 6, m);
    }
  }
}


static bool split6_view_ok(const vm_tensor* y, const vm_tensor* x) {
  return y->dtype == VM_BF16 && y->cstride % 48 == 0 && y->coff % 8 == 0 && y->c % 8 == 0 && y->c >= x->c &&
         y->coff + y->c <= y->cstride / 6 && reinterpret_cast<uintptr_t>(y->ptr) % 16 == 0;
}

extern "C" int vm_split6_nhwc(const vm_tensor* x, vm_tensor* y, vm_tensor* y_pool, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y) || (y_pool && !valid_tensor(y_pool)) || x->dtype != VM_F32)
    return fail(VM_EINVAL, "split6: x must be an f32 view");
  if (y->n != x->n || y->h != x->h || y->w != x->w) return fail(VM_EINVAL, "split6: shape mismatch");
  if (!split6_view_ok(y, x) || (y_pool && !split6_view_ok(y_pool, x)))
    return fail(VM_EUNSUPPORTED, "split6: the split view must be bf16, 16-byte aligned, c and coff multiples of 8, "
                                 "cstride = 6 x a multiple of 8 channels");
  if (y_pool && (y_pool->n != x->n || y_pool->h != (x->h + 1) / 2 || y_pool->w != (x->w + 1) / 2 ||
                 y_pool->c != y->c))
    return fail(VM_EINVAL, "split6: pool view shape mismatch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const vm_tensor* o = y_pool ? y_pool : y;
  const long work = (long)o->n * o->h * o->w * ((y->c + 7) / 8);
  if (y_pool)
    hipLaunchKernelGGL(split6_kernel<true>, dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y),
                       view(y_pool));
  else
    hipLaunchKernelGGL(split6_kernel<false>, dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y), view(y));
  return check_launch("split6");
}

// ---------------------------------------------------------------- split-fp16 x3 operands (vmatting/split3.py)
// x = h + l with h = fp16(x), l = fp16(x - h) (the difference is exact in f32): 22 significant bits where the two
// bf16 parts of a bf16 x3 split hold 16, so three fp16 products l*Wh + h*Wl + h*Wh (the filter likewise cut in two
// fp16 parts, pre-scaled by a power of two into fp16's normal range) carry an f32-class conv.  Slabs [l, h, h] at
// p*S + coff + c meet the filter parts [Wh, Wl, Wh] packed along K: the two 2^-11 terms first, h*Wh last.
// |x| >= 65520 rounds h to inf: *overflow is set (the caller checks it and falls back for that frame).
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t f16x2_bits(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));  // RNE
}

__device__ __forceinline__ bool store_split3h(uint16_t* base, long S, const float* v, bool three) {
  uint32_t wh[4], wl[4];
  bool ovf = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    wh[i] = f16x2_bits(v[2 * i], v[2 * i + 1]);
    const f16x2_t h = __builtin_bit_cast(f16x2_t, wh[i]);
    wl[i] = f16x2_bits(v[2 * i] - (float)h[0], v[2 * i + 1] - (float)h[1]);
    ovf |= !(fabsf(v[2 * i]) < 65520.f) || !(fabsf(v[2 * i + 1]) < 65520.f);  // (NaN counts too)
  }
  const uint4 H = make_uint4(wh[0], wh[1], wh[2], wh[3]), L = make_uint4(wl[0], wl[1], wl[2], wl[3]);
  *reinterpret_cast<uint4*>(base) = L;
  *reinterpret_cast<uint4*>(base + S) = H;
  if (three) *reinterpret_cast<uint4*>(base + 2 * S) = H;
  return ovf;
}

// one thread = one 8-channel chunk of one output pixel (POOL: of one pooled pixel and the 2x2 window under it)
// I: the index type (int when the work fits: 32-bit divisions instead of 64-bit ones, which cost more than the
// element's loads and stores)
template <bool POOL, typename I>
__global__ __launch_bounds__(256) void split3h_kernel(View x, View y, View yp, long S, long Sp, int* overflow) {
  const int cpp = (y.c + 7) / 8;
  const int on = POOL ? yp.n : y.n, oh = POOL ? yp.h : y.h, ow = POOL ? yp.w : y.w;
  const I total = (I)on * oh * ow * cpp;
  bool ovf = false;
  const bool vec = ((x.cs | x.coff) & 3) == 0 && (reinterpret_cast<uintptr_t>(x.p) & 15) == 0;
  const bool y3 = 3 * S <= y.cs;  // the third slab [h again] where the pixel row holds it (else [l, h] only)
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpp);
    const long op = (long)(i / cpp);
    const int c = cc * 8;
    auto load = [&](long pix, float* f) {
      const float* src = reinterpret_cast<const float*>(x.p) + pix * x.cs + x.coff + c;
      if (c + 8 <= x.c && vec) {
        const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
        f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = c + j < x.c ? src[j] : 0.f;  // channels past x.c: zero padding
      }
    };
    auto out = [&](const View& v, long pix) { return reinterpret_cast<uint16_t*>(v.p) + pix * v.cs + v.coff + c; };
    if constexpr (!POOL) {
      float f[8];
      load(op, f);
      ovf |= store_split3h(out(y, op), S, f, y3);
    } else {
      const int pw = (int)(op % yp.w);
      const long t = op / yp.w;
      const int ph = (int)(t % yp.h), n = (int)(t / yp.h);
      const int iy = 2 * ph, ix = 2 * pw;
      const bool hasr = ix + 1 < x.w, hasd = iy + 1 < x.h;
      const long p00 = ((long)n * x.h + iy) * x.w + ix;
      float f[8], m[8];
      load(p00, f);
      ovf |= store_split3h(out(y, p00), S, f, y3);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = f[j];
      auto tap = [&](long pix) {
        load(pix, f);
        ovf |= store_split3h(out(y, pix), S, f, y3);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
      };
      if (hasr) tap(p00 + 1);
      if (hasd) tap(p00 + x.w);
      if (hasr && hasd) tap(p00 + x.w + 1);
      store_split3h(out(yp, op), Sp, m, 3 * Sp <= yp.cs);
    }
  }
  if (ovf && overflow) *overflow = 1;  // a plain vector store: any writer's 1 is the answer
}

// tf.image.resize_images (unet.py:58) of an f32 activation written straight as its split-fp16 x3 operand: the
// resize's float32 arithmetic of resize_tf1_kernel / resize2x_tf1_rows (bit-identical values), then the split of
// split3h_kernel — no f32 resized tensor.  One thread = 8 channels; TWO: the exact-2x quad form (one thread loads
// the 2x2 low-res taps of low-res pixel (i, j) once and writes the 4 output pixels of its quad).
__device__ __forceinline__ void ld8f(const View& x, long pix, int c, float* f) {
  const float* src = reinterpret_cast<const float*>(x.p) + pix * x.cs + x.coff + c;
  const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

template <bool TWO, typename I>
__global__ __launch_bounds__(256) void resize_split3h_kernel(View x, View y, long S, float sy, float sx,
                                                             int* overflow) {
  const int cpp = y.c / 8;
  const bool y3 = 3 * S <= y.cs;
  const int oh_n = TWO ? x.h : y.h, ow_n = TWO ? x.w : y.w;
  const I total = (I)y.n * oh_n * ow_n * cpp;
  bool ovf = false;
  for (I i = blockIdx.x * (I)blockDim.x + threadIdx.x; i < total; i += (I)gridDim.x * blockDim.x) {
    const int cc = (int)(i % cpp);
    const I op = i / cpp;
    const int ow = (int)(op % ow_n);
    const I t = op / ow_n;
    const int oh = (int)(t % oh_n), n = (int)(t / oh_n);
    const int c = cc * 8;
    const long rb = (long)n * x.h;
    if constexpr (TWO) {  // (oh, ow) = low-res pixel (i, j)
      const int i1 = min(oh + 1, x.h - 1), j1 = min(ow + 1, x.w - 1);
      float a00[8], a01[8], a10[8], a11[8];
      ld8f(x, (rb + oh) * x.w + ow, c, a00);
      ld8f(x, (rb + oh) * x.w + j1, c, a01);
      ld8f(x, (rb + i1) * x.w + ow, c, a10);
      ld8f(x, (rb + i1) * x.w + j1, c, a11);
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const int oy = 2 * oh + dy;
        if (oy >= y.h) break;
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          const int ox = 2 * ow + dx;
          if (ox >= y.w) break;
          int ly0, ly1, lx0, lx1;
          float fy, fx;
          tf1_coord(oy, 0.5f, x.h, ly0, ly1, fy);
          tf1_coord(ox, 0.5f, x.w, lx0, lx1, fx);
          const float* tl = a00;
          const float* tr = (lx1 == lx0) ? a00 : a01;
          const float* bl = (ly1 == ly0) ? a00 : a10;
          const float* br = (ly1 == ly0) ? tr : ((lx1 == lx0) ? a10 : a11);
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
#pragma clang fp contract(off)
            const float top = tl[e] + (tr[e] - tl[e]) * fx;
            const float bot = bl[e] + (br[e] - bl[e]) * fx;
            o[e] = top + (bot - top) * fy;
          }
          uint16_t* yo = reinterpret_cast<uint16_t*>(y.p) + (((long)n * y.h + oy) * y.w + ox) * y.cs + y.coff + c;
          ovf |= store_split3h(yo, S, o, y3);
        }
      }
    } else {
      int y0, y1, x0, x1;
      float yl, xl;
      tf1_coord(oh, sy, x.h, y0, y1, yl);
      tf1_coord(ow, sx, x.w, x0, x1, xl);
      float tl[8], tr[8], bl[8], br[8], o[8];
      ld8f(x, (rb + y0) * x.w + x0, c, tl);
      ld8f(x, (rb + y0) * x.w + x1, c, tr);
      ld8f(x, (rb + y1) * x.w + x0, c, bl);
      ld8f(x, (rb + y1) * x.w + x1, c, br);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma clang fp contract(off)
        const float top = tl[e] + (tr[e] - tl[e]) * xl;
        const float bot = bl[e] + (br[e] - bl[e]) * xl;
        o[e] = top + (bot - top) * yl;
      }
      uint16_t* yo = reinterpret_cast<uint16_t*>(y.p) + (long)op * y.cs + y.coff + c;
      ovf |= store_split3h(yo, S, o, y3);
    }
  }
  if (ovf && overflow) *overflow = 1;
}

static bool split3h_view_ok(const vm_tensor* y, const vm_tensor* x, long S) {
  return y->dtype == VM_F16 && S % 8 == 0 && 2 * S <= y->cstride && y->coff % 8 == 0 && y->c % 8 == 0 &&
         y->c >= x->c && y->coff + y->c <= S && y->cstride % 8 == 0 && reinterpret_cast<uintptr_t>(y->ptr) % 16 == 0;
}

extern "C" int vm_split3h_nhwc(const vm_tensor* x, vm_tensor* y, vm_tensor* y_pool, int slab, int* overflow,
                               void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y, true) || (y_pool && !valid_tensor(y_pool, true)) || x->dtype != VM_F32)
    return fail(VM_EINVAL, "split3h: x must be an f32 view");
  if (y->n != x->n || y->h != x->h || y->w != x->w) return fail(VM_EINVAL, "split3h: shape mismatch");
  const long S = slab > 0 ? slab : y->cstride / 2, Sp = y_pool ? (slab > 0 ? slab : y_pool->cstride / 2) : S;
  if (!split3h_view_ok(y, x, S) || (y_pool && !split3h_view_ok(y_pool, x, Sp)))
    return fail(VM_EUNSUPPORTED, "split3h: the split view must be fp16, 16-byte aligned, c and coff multiples of 8, "
                                 "three slabs of S (a multiple of 8) channels inside the pixel row");
  if (y_pool && (y_pool->n != x->n || y_pool->h != (x->h + 1) / 2 || y_pool->w != (x->w + 1) / 2 ||
                 y_pool->c != y->c))
    return fail(VM_EINVAL, "split3h: pool view shape mismatch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const vm_tensor* o = y_pool ? y_pool : y;
  const long work = (long)o->n * o->h * o->w * ((y->c + 7) / 8);
  const bool i32 = work + 256L * 4096 < 0x7fffffffL;  // (the grid-stride index stays below 2^31)
  if (y_pool && i32)
    hipLaunchKernelGGL((split3h_kernel<true, int>), dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y),
                       view(y_pool), S, Sp, overflow);
  else if (y_pool)
    hipLaunchKernelGGL((split3h_kernel<true, long>), dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y),
                       view(y_pool), S, Sp, overflow);
  else if (i32)
    hipLaunchKernelGGL((split3h_kernel<false, int>), dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y),
                       view(y), S, Sp, overflow);
  else
    hipLaunchKernelGGL((split3h_kernel<false, long>), dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y),
                       view(y), S, Sp, overflow);
  return check_launch("split3h");
}

extern "C" int vm_resize_split3h_nhwc(const vm_tensor* x, vm_tensor* y, int slab, int* overflow, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y, true) || x->dtype != VM_F32)
    return fail(VM_EINVAL, "resize_split3h: x must be an f32 view");
  if (y->n != x->n || y->c != x->c) return fail(VM_EINVAL, "resize_split3h: batch/channel mismatch");
  const long S = slab > 0 ? slab : y->cstride / 2;
  if (!split3h_view_ok(y, x, S) || x->c % 8 || x->cstride % 4 || x->coff % 4 ||
      reinterpret_cast<uintptr_t>(x->ptr) % 16)
    return fail(VM_EUNSUPPORTED, "resize_split3h: 16-byte aligned views of c %% 8 == 0 channels, the split layout of "
                                 "vm_split3h_nhwc");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool two = y->h == 2 * x->h && y->w == 2 * x->w;
  const long work = (long)y->n * (two ? (long)x->h * x->w : (long)y->h * y->w) * (y->c / 8);
  const float sy = (float)x->h / (float)y->h, sx = (float)x->w / (float)y->w;
  const bool i32 = work + 256L * 4096 < 0x7fffffffL;
  const dim3 grid(grid_for(work, 256));
  if (two && i32)
    hipLaunchKernelGGL((resize_split3h_kernel<true, int>), grid, dim3(256), 0, st, view(x), view(y), S, sy, sx, overflow);
  else if (two)
    hipLaunchKernelGGL((resize_split3h_kernel<true, long>), grid, dim3(256), 0, st, view(x), view(y), S, sy, sx,
                       overflow);
  else if (i32)
    hipLaunchKernelGGL((resize_split3h_kernel<false, int>), grid, dim3(256), 0, st, view(x), view(y), S, sy, sx,
                       overflow);
  else
    hipLaunchKernelGGL((resize_split3h_kernel<false, long>), grid, dim3(256), 0, st, view(x), view(y), S, sy, sx,
                       overflow);
  return check_launch("resize_split3h");
}

extern "C" int vm_convert_nhwc(const vm_tensor* x, vm_tensor* y, const float* scale, const float* shift, int act,
                               void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y)) return fail(VM_EINVAL, "convert: invalid tensor");
  if (y->n != x->n || y->h != x->h || y->w != x->w || y->c < x->c) return fail(VM_EINVAL, "convert: shape mismatch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long work = (long)y->n * y->h * y->w * y->c;
  if (x->dtype == VM_F32 && y->dtype == VM_BF16 && x->c == y->c && y->c % 8 == 0 && y->c > 8 && !scale && !shift &&
      act == VM_ACT_NONE && vec16_ok(x) && vec16_ok(y)) {
    const long M = (long)y->n * y->h * y->w;
    hipLaunchKernelGGL(convert8_f32_bf16_kernel, dim3(grid_for(work / 8, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float*>(x->ptr) + x->coff, x->cstride,
                       reinterpret_cast<uint16_t*>(y->ptr) + y->coff, y->cstride, M, y->c / 8);
  } else if (y->dtype == VM_BF16 && y->c == 8 && vec16_ok(y))
    hipLaunchKernelGGL(convert_px8_bf16_kernel, dim3(grid_for(work / 8, 256)), dim3(256), 0, st, view(x), view(y), scale,
                       shift, act);
  else if (y->c <= 16)
    hipLaunchKernelGGL(convert_px_kernel, dim3(grid_for(work / y->c, 256)), dim3(256), 0, st, view(x), view(y), scale,
                       shift, act);
  else
    hipLaunchKernelGGL(convert_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, view(x), view(y), scale, shift,
                       act);
  return check_launch("convert");
}

extern "C" size_t vm_bn_workspace_bytes(const vm_tensor* x) {
  if (!x) return 0;
  return (size_t)2 * bn_max_blocks(x->c) * x->c * sizeof(double);
}

extern "C" int vm_bn_stats_nhwc(const vm_tensor* x, float* mean, float* var, void* work, void* stream) {
  if (!valid_tensor(x) || !mean || !var || !work) return fail(VM_EINVAL, "bn_stats: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)x->n * x->h * x->w;
  double* part = reinterpret_cast<double*>(work);
  int nb;
  if (g_bn_vec_fwd && vec8_view(x)) {
    nb = bn_blocks(M, x->c);
    const int C = x->c, tp = tpg8(C);
#define VM_BP8(TPG)                                                                                                 \
  case TPG:                                                                                                         \
    if (x->dtype == VM_BF16)                                                                                        \
      hipLaunchKernelGGL((bn_partial8_kernel<uint16_t, TPG>), dim3(nb), dim3(256), 0, st,                           \
                         reinterpret_cast<const uint16_t*>(x->ptr) + x->coff, x->cstride, M, C, part, nb);          \
    else                                                                                                            \
      hipLaunchKernelGGL((bn_partial8_kernel<float, TPG>), dim3(nb), dim3(256), 0, st,                              \
                         reinterpret_cast<const float*>(x->ptr) + x->coff, x->cstride, M, C, part, nb);             \
    break;
    switch (tp) { VM_BP8(1) VM_BP8(2) VM_BP8(4) VM_BP8(8) VM_BP8(16) VM_BP8(32) VM_BP8(64) }
#undef VM_BP8
  } else {
    nb = x->dtype == VM_BF16 ? launch_bn_partial<uint16_t>(view(x), part, st)
                             : launch_bn_partial<float>(view(x), part, st);
  }
  int rc = check_launch("bn_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_final_kernel, dim3(x->c), dim3(256), 0, st, part, nb, x->c, M, mean, var);
  return check_launch("bn_final");
}

extern "C" int vm_bn_apply_nhwc(const vm_tensor* x, vm_tensor* y, const float* mean, const float* var,
                                const float* gamma, const float* beta, float eps, int act, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y)) return fail(VM_EINVAL, "bn_apply: invalid tensor");
  if (y->n != x->n || y->h != x->h || y->w != x->w || y->c != x->c) return fail(VM_EINVAL, "bn_apply: shape mismatch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)x->n * x->h * x->w;
  const int C = x->c;
  const int cp = C > 32 ? 64 : C > 16 ? 32 : C > 8 ? 16 : C > 4 ? 8 : C > 2 ? 4 : C > 1 ? 2 : 1;
  const long px = (M + 256 / cp - 1) / (256 / cp);
  const dim3 grid((unsigned)(px < 4096 ? px : 4096), (unsigned)((C + cp - 1) / cp));
  if (g_bn_vec_fwd && vec8_view(x) && vec8_view(y)) {
    const int tp = tpg8(C);
    const long px8 = (M + 256 / tp - 1) / (256 / tp);
    const dim3 g8((unsigned)(px8 < 4096 ? px8 : 4096));
    const bool xf = x->dtype == VM_F32, yf = y->dtype == VM_F32;
#define VM_BA8(TPG)                                                                                                 \
  case TPG:                                                                                                         \
    if (xf && yf)                                                                                                   \
      hipLaunchKernelGGL((bn_apply8_kernel<float, float, TPG>), g8, dim3(256), 0, st,                               \
                         reinterpret_cast<const float*>(x->ptr) + x->coff, x->cstride,                              \
                         reinterpret_cast<float*>(y->ptr) + y->coff, y->cstride, M, C, mean, var, gamma, beta, eps, act); \
    else if (xf)                                                                                                    \
      hipLaunchKernelGGL((bn_apply8_kernel<float, uint16_t, TPG>), g8, dim3(256), 0, st,                            \
                         reinterpret_cast<const float*>(x->ptr) + x->coff, x->cstride,                              \
                         reinterpret_cast<uint16_t*>(y->ptr) + y->coff, y->cstride, M, C, mean, var, gamma, beta, eps, \
                         act);                                                                                      \
    else if (yf)                                                                                                    \
      hipLaunchKernelGGL((bn_apply8_kernel<uint16_t, float, TPG>), g8, dim3(256), 0, st,                            \
                         reinterpret_cast<const uint16_t*>(x->ptr) + x->coff, x->cstride,                           \
                         reinterpret_cast<float*>(y->ptr) + y->coff, y->cstride, M, C, mean, var, gamma, beta, eps, act); \
    else                                                                                                            \
      hipLaunchKernelGGL((bn_apply8_kernel<uint16_t, uint16_t, TPG>), g8, dim3(256), 0, st,                         \
                         reinterpret_cast<const uint16_t*>(x->ptr) + x->coff, x->cstride,                           \
                         reinterpret_cast<uint16_t*>(y->ptr) + y->coff, y->cstride, M, C, mean, var, gamma, beta, eps, \
                         act);                                                                                      \
    break;
    switch (tp) { VM_BA8(1) VM_BA8(2) VM_BA8(4) VM_BA8(8) VM_BA8(16) VM_BA8(32) VM_BA8(64) }
#undef VM_BA8
    return check_launch("bn_apply");
  }
  if (f32_pair_view(x) && f32_pair_view(y)) {
    hipLaunchKernelGGL(bn_apply2_f32_kernel, dim3(grid_for(M, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float*>(x->ptr) + x->coff, x->cstride,
                       reinterpret_cast<float*>(y->ptr) + y->coff, y->cstride, M, mean, var, gamma, beta, eps, act);
    return check_launch("bn_apply");
  }
  const View xv = view(x), yv = view(y);
  switch (cp) {
#define VM_BA(CP) \
  case CP: hipLaunchKernelGGL((bn_apply_kernel<CP>), grid, dim3(256), 0, st, xv, yv, mean, var, gamma, beta, eps, act); break;
    VM_BA(1) VM_BA(2) VM_BA(4) VM_BA(8) VM_BA(16) VM_BA(32) VM_BA(64)
#undef VM_BA
  }
  return check_launch("bn_apply");
}

extern "C" int vm_softmax_lastdim_nhwc(const vm_tensor* x, vm_tensor* y, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y)) return fail(VM_EINVAL, "softmax: invalid tensor");
  if (y->n != x->n || y->h != x->h || y->w != x->w || y->c != x->c) return fail(VM_EINVAL, "softmax: shape mismatch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)x->n * x->h * x->w;
  hipLaunchKernelGGL(softmax_kernel, dim3(grid_for(M, 256)), dim3(256), 0, st, view(x), view(y));
  return check_launch("softmax");
}

// ---------------------------------------------------------------- compositing
// reader.create_composite_image (reader.py:72-79): tri_alpha = zeros_like(fg) with channels 0..2 set to alpha,
// composite = tri_alpha * fg + (1 - tri_alpha) * bg, in float64 like numpy (channels >= 3 get alpha 0, i.e. bg).
// Each element is computed in double, products and sum rounded separately (no fma), then rounded to the
// output dtype, so an f64 output is bit-identical to the numpy expression and an f32 output is its f32 rounding.
template <typename TI, typename TA, typename TO>
__global__ void __launch_bounds__(256) composite_kernel(const TI* __restrict__ fg, const TI* __restrict__ bg,
                                                        const TA* __restrict__ alpha, long elems, int cn,
                                                        TO* __restrict__ out) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < elems; i += stride) {
    const long p = i / cn;
    const int c = (int)(i - p * cn);
    const double a = c < 3 ? (double)alpha[p] : 0.0;
    double p0 = a * (double)fg[i], p1 = (1.0 - a) * (double)bg[i];
    asm volatile("" : "+v"(p0), "+v"(p1));  // opaque: the products stay rounded (hipcc would fuse them into v_fmac_f64)
    const double v = p0 + p1;
    out[i] = (TO)v;
  }
}

template <typename TI, typename TA>
static void launch_composite(const void* fg, const void* bg, const void* alpha, long elems, int cn, void* out,
                             int out_dtype, hipStream_t st) {
  const dim3 grid(grid_for(elems, 256, 256 * 32)), block(256);
  if (out_dtype == VM_F64)
    hipLaunchKernelGGL((composite_kernel<TI, TA, double>), grid, block, 0, st, (const TI*)fg, (const TI*)bg,
                       (const TA*)alpha, elems, cn, (double*)out);
  else
    hipLaunchKernelGGL((composite_kernel<TI, TA, float>), grid, block, 0, st, (const TI*)fg, (const TI*)bg,
                       (const TA*)alpha, elems, cn, (float*)out);
}

template <typename TI>
static void launch_composite_a(const void* fg, const void* bg, const void* alpha, int alpha_dtype, long elems, int cn,
                               void* out, int out_dtype, hipStream_t st) {
  if (alpha_dtype == VM_F64) launch_composite<TI, double>(fg, bg, alpha, elems, cn, out, out_dtype, st);
  else launch_composite<TI, float>(fg, bg, alpha, elems, cn, out, out_dtype, st);
}

extern "C" int vm_composite_image(const void* fg, const void* bg, int img_dtype, const void* alpha, int alpha_dtype,
                                  long pixels, int cn, void* out, int out_dtype, void* stream) {
  if (pixels < 0 || cn < 1) return fail(VM_EINVAL, "composite: bad size");
  if (img_dtype != VM_U8 && img_dtype != VM_F32 && img_dtype != VM_F64)
    return fail(VM_EUNSUPPORTED, "composite: image dtype must be u8, f32 or f64");
  if ((alpha_dtype != VM_F32 && alpha_dtype != VM_F64) || (out_dtype != VM_F32 && out_dtype != VM_F64))
    return fail(VM_EUNSUPPORTED, "composite: alpha / output dtype must be f32 or f64");
  if (pixels == 0) return VM_OK;
  if (!fg || !bg || !alpha || !out) return fail(VM_EINVAL, "composite: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long elems = pixels * cn;
  if (img_dtype == VM_U8) launch_composite_a<uint8_t>(fg, bg, alpha, alpha_dtype, elems, cn, out, out_dtype, st);
  else if (img_dtype == VM_F32) launch_composite_a<float>(fg, bg, alpha, alpha_dtype, elems, cn, out, out_dtype, st);
  else launch_composite_a<double>(fg, bg, alpha, alpha_dtype, elems, cn, out, out_dtype, st);
  return check_launch("composite");
}

// A stream created with a full CU mask (hipExtStreamCreateWithCUMask).  A plain hipStream shares one of the process's
// GPU_MAX_HW_QUEUES hardware queues, and which one it gets is not under the caller's control: kernel traces
// (profiles/r06o_imgtrace_queues.txt) caught UNetImage trainers whose side stream sat on the caller's queue, which
// serialises the filter gradients behind the data-gradient chain (backward 4.8 ms instead of 4.1).  A CU-masked
// stream gets a queue of its own, but measured slower still (8.3 ms per step): kept for A/B, the trainers probe a
// pooled stream instead (vm_spin below, ops.concurrent_stream).
extern "C" int vm_stream_create_masked(void** stream) {
  if (!stream) return vm::fail(VM_EINVAL, "stream_create_masked: NULL");
  int dev = 0, ncu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess || ncu <= 0) return vm::fail(VM_EHIP, "stream_create_masked: %s", hipGetErrorString(e));
  uint32_t mask[64];
  const int words = (ncu + 31) / 32;
  if (words > 64) return vm::fail(VM_EUNSUPPORTED, "stream_create_masked: %d CUs", ncu);
  for (int i = 0; i < words; ++i) mask[i] = 0xffffffffu;
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return vm::fail(VM_EHIP, "hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
  *stream = reinterpret_cast<void*>(s);
  return VM_OK;
}

extern "C" int vm_stream_destroy(void* stream) {
  if (!stream) return vm::fail(VM_EINVAL, "stream_destroy: NULL");
  const hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? VM_OK : vm::fail(VM_EHIP, "hipStreamDestroy: %s", hipGetErrorString(e));
}

// A kernel that holds one wave busy for `us` microseconds of the device's constant-rate wall clock: the probe that
// tells whether a second stream runs beside the caller's (ops.concurrent_stream) — a short kernel queued on that
// stream finishes while this one still spins only if the two streams sit on different hardware queues
__global__ void spin_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int vm_spin(int microseconds, void* stream) {
  if (microseconds < 0 || microseconds > 1000000) return vm::fail(VM_EINVAL, "spin: %d us", microseconds);
  int dev = 0, khz = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess || khz <= 0) return vm::fail(VM_EHIP, "spin: wall clock rate: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     (long long)microseconds * khz / 1000);
  return check_launch("spin");
}

