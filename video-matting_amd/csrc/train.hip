// Backward pass + optimizer of the config-5 training step (train.py:288-343, video_procedure; the same graph
// as simple_procedure, train.py:176-227): the gradient of
//   loss = mean(0.5*regular_l1(pred, gt) + 0.5*regular_l1(composite(raw_fg, bg, pred), cmp))   (train.py:294-298)
// through UNetSimple's trainable layers (unet_simple.py:116-142: conv + bias -> batch_norm(is_training) -> relu,
// upconv_concat's resize -> conv -> relu -> concat -> batch_norm), and tf.train.AdamOptimizer's update
// (train.py:302-304).  The frozen VGG towers (tf.constant weights, unet_simple.py:109-113) need no gradient.
//
//   loss_backward   dL/dlogits of sigmoid(logits) under the Charbonnier alpha + compositional loss
//   bn_backward     fused-BN gradient (batch statistics), optional relu mask from the BN+relu output:
//                   dx = gamma*rstd*(g - sum(g)/M - xhat*sum(g*xhat)/M), dgamma = sum(g*xhat), dbeta = sum(g)
//   conv_wgrad      dW[kh,kw,ci,co] = sum_p x[p + (kh-1, kw-1), ci] * dy[p, co]: per block an LDS patch of
//                   (4+2) x (32+2) pixels x CC channels and the 4 x 32 dy tile; each thread owns one (kh, ci,
//                   4-channel co group) and slides the three kw taps along a pixel row (1 new LDS x read and one
//                   float4 dy read per 12 FMAs); blocks walk tiles persistently and store one partial filter
//                   gradient each, summed in fixed order by a second pass (deterministic, no atomics)
//   conv dgrad      the forward conv kernels on flipped, transposed weights (flip_weights here)
//   resize_backward adjoint of the TF-1 legacy bilinear resize, gathered per input element (no atomics)
//   relu_backward   dy * (y > 0)
//   maxpool_bwd     tf.nn.max_pool 2x2/2 SAME adjoint: the window's gradient to its first maximum (small.py:40,42)
//   adam            TF ApplyAdam: m += (g-m)(1-b1); v += (g^2-v)(1-b2); var -= m*lr_t/(sqrt(v)+eps)

#include <algorithm>
#include <cstring>

#include "conv_common.h"
#include "vm_common.h"

namespace vm {
namespace trn {

struct V {
  char* p;
  int n, h, w, c, cs, coff, dt;
  int sc;     // > 0: channel c lives in source c / sc (tower-major features), sources ss elements apart
  long ss;
};

static V mk(const vm_tensor* t) {
  V v;
  v.p = reinterpret_cast<char*>(t->ptr);
  v.n = t->n; v.h = t->h; v.w = t->w; v.c = t->c; v.cs = t->cstride; v.coff = t->coff; v.dt = t->dtype;
  v.sc = 0; v.ss = 0;
  return v;
}

__device__ __forceinline__ long vchan(const V& v, int c) {
  if (v.sc <= 0) return c;
  const int s = c / v.sc;
  return (long)s * v.ss + (c - s * v.sc);
}

__device__ __forceinline__ float ld(const V& v, long pix, int c) {
  const long o = pix * v.cs + v.coff + vchan(v, c);
  return v.dt == VM_F32 ? reinterpret_cast<const float*>(v.p)[o] : bf2f(reinterpret_cast<const uint16_t*>(v.p)[o]);
}

__device__ __forceinline__ void st(const V& v, long pix, int c, float x) {
  const long o = pix * v.cs + v.coff + c;
  if (v.dt == VM_F32) reinterpret_cast<float*>(v.p)[o] = x;
  else reinterpret_cast<uint16_t*>(v.p)[o] = f2bf(x);
}

// ---------------------------------------------------------------- loss backward (train.py:21-28, 294-298)
// s_loss is [N,H,W,3] (the [N,H,W,1] alpha term broadcast), so with P pixels
//   dL/dpred = 0.5/(3P) * (3*(a-g)/La + sum_k e_k/Lc_k * (fg_k - bg_k)),   e_k = a*fg_k + (1-a)*bg_k - cmp_k
// and dL/dlogits = dL/dpred * a*(1-a) (tf.nn.sigmoid's gradient in terms of its output).
__global__ __launch_bounds__(256) void loss_backward_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                            const float* __restrict__ fg, const float* __restrict__ bg,
                                                            const float* __restrict__ cmp, long P, float* dlogit) {
  const float eps2 = 1e-6f * 1e-6f;
  const float k = 0.5f / (3.0f * (float)P);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < P; i += (long)gridDim.x * blockDim.x) {
    const float a = pred[i];
    const float d = a - gt[i];
    float s = 3.f * d / sqrtf(d * d + eps2);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float f = fg[i * 3 + j], b = bg[i * 3 + j];
      const float e = a * f + (1.f - a) * b - cmp[i * 3 + j];
      s += e / sqrtf(e * e + eps2) * (f - b);
    }
    dlogit[i] = k * s * a * (1.f - a);
  }
}

// ---------------------------------------------------------------- batch-norm backward (training statistics)

template <bool MASK>
__device__ __forceinline__ float grad_in(const V& dy, const V& y, long p, int c) {
  const float g = ld(dy, p, c);
  if (MASK) return ld(y, p, c) > 0.f ? g : 0.f;
  return g;
}

// per (channel group, pixel block): double partial sums of g and g*xhat (x == NULL: g only).  CP lanes per pixel as
// in elementwise.hip's bn_partial_kernel: narrow tensors put 64 / CP pixels in flight per wave.
template <bool MASK, int CP>
__global__ __launch_bounds__(256) void bn_bwd_partial(V x, V dy, V y, const float* mean, const float* var, float eps,
                                                      double* part, int nblk) {
  constexpr int PPW = 64 / CP;
  __shared__ double sh[3][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * CP + (lane % CP);
  const long M = (long)dy.n * dy.h * dy.w;
  double s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < dy.c) {
    const float m = x.p ? mean[c] : 0.f;
    const float r = x.p ? 1.0f / sqrtf(var[c] + eps) : 0.f;
    const long stp = (long)nblk * 4 * PPW;
    long p = ((long)blockIdx.y * 4 + wave) * PPW + lane / CP;
    // 4 pixels' loads in flight per lane before any is summed (same summation order as one at a time)
    for (; p + 3 * stp < M; p += 4 * stp) {
      float g[4], xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        g[u] = grad_in<MASK>(dy, y, p + u * stp, c);
        xv[u] = x.p ? ld(x, p + u * stp, c) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s1 += g[u];
        if (x.p) {
          const float xh = (xv[u] - m) * r;
          s2 += (double)g[u] * (double)xh;
          s3 += (double)xh;
        }
      }
    }
    for (; p < M; p += stp) {
      const float g = grad_in<MASK>(dy, y, p, c);
      s1 += g;
      if (x.p) {
        const float xh = (ld(x, p, c) - m) * r;
        s2 += (double)g * (double)xh;
        s3 += (double)xh;
      }
    }
  }
  sh[0][wave][lane] = s1;
  sh[1][wave][lane] = s2;
  sh[2][wave][lane] = s3;
  __syncthreads();
  if ((int)threadIdx.x < CP && c < dy.c) {
    s1 = s2 = s3 = 0.0;
    for (int w = 0; w < 4; ++w)
      for (int k = 0; k < PPW; ++k) {
        s1 += sh[0][w][k * CP + threadIdx.x];
        s2 += sh[1][w][k * CP + threadIdx.x];
        s3 += sh[2][w][k * CP + threadIdx.x];
      }
    part[(long)c * nblk + blockIdx.y] = s1;  // channel-major [k][C][nblk] (vm_common.h fold_columns)
    part[(long)nblk * dy.c + (long)c * nblk + blockIdx.y] = s2;
    part[2L * nblk * dy.c + (long)c * nblk + blockIdx.y] = s3;
  }
}

// folds the partials; with dbias also the gradient of a bias added before the BN (new_conv's conv bias,
// unet_simple.py:23-25): sum_p dx = gamma*rstd*(sum g - M*mean g - sum xhat * sum(g*xhat)/M), zero in exact
// arithmetic (BN removes the bias), evaluated from the same double sums instead of a pass over dx
__global__ __launch_bounds__(256) void bn_bwd_final(const double* part, int nblk, int C, float* sum_g, float* sum_gx,
                                                    float* dbias, const float* gamma, const float* var, float eps,
                                                    long M) {
  const int c = blockIdx.x;
  double r[3];
  fold_columns(part, nblk, C, c, dbias ? 3 : 2, r);
  if (threadIdx.x == 0) {
    const double s1 = r[0], s2 = r[1], s3 = r[2];
    if (sum_g) sum_g[c] = (float)s1;
    if (sum_gx) sum_gx[c] = (float)s2;
    if (dbias) {
      const double rs = 1.0 / sqrt((double)var[c] + (double)eps), g = gamma ? gamma[c] : 1.0;
      dbias[c] = (float)(g * rs * (s1 - (double)M * (s1 / (double)M) - s3 * s2 / (double)M));
    }
  }
}

template <bool MASK>
static void launch_bn_bwd_partial(const V& x, const V& dy, const V& y, const float* mean, const float* var, float eps,
                                  double* part, int nb, hipStream_t st) {
  const int C = dy.c;
  const int cp = C > 32 ? 64 : C > 16 ? 32 : C > 8 ? 16 : C > 4 ? 8 : C > 2 ? 4 : C > 1 ? 2 : 1;
  dim3 g(cp == 64 ? (C + 63) / 64 : 1, nb), b(256);
  switch (cp) {
    case 1: hipLaunchKernelGGL((bn_bwd_partial<MASK, 1>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
    case 2: hipLaunchKernelGGL((bn_bwd_partial<MASK, 2>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
    case 4: hipLaunchKernelGGL((bn_bwd_partial<MASK, 4>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
    case 8: hipLaunchKernelGGL((bn_bwd_partial<MASK, 8>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
    case 16: hipLaunchKernelGGL((bn_bwd_partial<MASK, 16>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
    case 32: hipLaunchKernelGGL((bn_bwd_partial<MASK, 32>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
    default: hipLaunchKernelGGL((bn_bwd_partial<MASK, 64>), g, b, 0, st, x, dy, y, mean, var, eps, part, nb); break;
  }
}

// Vectorised BN backward for whole 8-channel runs (f32 x / dy / dx, an optional bf16 relu mask y and bf16 copy dx2;
// every view 16-byte aligned, C % 8 == 0, C <= 512): a lane takes 8 channels of a pixel — two f32x4 of x and of dy,
// one 16-byte y chunk — where the per-channel forms above issue a 4-byte access per element (~3.5 TB/s on the 32-
// channel full-resolution layers of the config-5 step).  Per element the same expressions, summed in f64 per block
// into the same [3][C][nblk] tables (another partition of the pixels; bn_bwd_final folds them as before).
__device__ __forceinline__ void ld8f32(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void ld8bf(const uint16_t* p, float (&v)[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p);
  const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = bf2f((uint16_t)(w4[k] & 0xffffu));
    v[2 * k + 1] = bf2f((uint16_t)(w4[k] >> 16));
  }
}
struct Bn8 {
  const float* x;
  const float* dy;
  const uint16_t* y;  // bf16 relu output (mask) or nullptr
  float* dx;
  uint16_t* dx2;      // bf16 copy or nullptr
  int xcs, dycs, ycs, dxcs, dx2cs, C;
  long M;
};

template <bool MASK, int TPG>
__global__ __launch_bounds__(256) void bn_bwd_partial8(Bn8 a, const float* mean, const float* var, float eps,
                                                       double* part, int nblk) {
  constexpr int PPB = 256 / TPG;
  __shared__ double sh[8][256];
  const int t = threadIdx.x, j = t % TPG, pl = t / TPG, c0 = 8 * j;
  double s1[8], s2[8], s3[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = s3[k] = 0.0;
  if (c0 < a.C) {
    float m[8], r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m[k] = mean[c0 + k];
      r[k] = 1.0f / sqrtf(var[c0 + k] + eps);
    }
    for (long p = (long)blockIdx.x * PPB + pl; p < a.M; p += (long)nblk * PPB) {
      float g[8], xv[8];
      ld8f32(a.dy + p * a.dycs + c0, g);
      ld8f32(a.x + p * a.xcs + c0, xv);
      if constexpr (MASK) {
        float yv[8];
        ld8bf(a.y + p * a.ycs + c0, yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s1[k] += g[k];
        const float xh = (xv[k] - m[k]) * r[k];
        s2[k] += (double)g[k] * (double)xh;
        s3[k] += (double)xh;
      }
    }
  }
  // three tables through one 16 KB staging buffer
#pragma unroll
  for (int tab = 0; tab < 3; ++tab) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[k][t] = tab == 0 ? s1[k] : tab == 1 ? s2[k] : s3[k];
    __syncthreads();
    for (int c = t; c < a.C; c += 256) {
      const int jj = c >> 3, k = c & 7;
      double v = 0.0;
      for (int q = 0; q < PPB; ++q) v += sh[k][q * TPG + jj];
      part[(long)tab * nblk * a.C + (long)c * nblk + blockIdx.x] = v;
    }
    __syncthreads();
  }
}

template <bool MASK, bool DX2, int TPG>
__global__ __launch_bounds__(256) void bn_bwd_apply8(Bn8 a, const float* mean, const float* var, const float* gamma,
                                                     float eps, const float* sum_g, const float* sum_gx) {
  constexpr int PPB = 256 / TPG;
  const int t = threadIdx.x, j = t % TPG, pl = t / TPG, c0 = 8 * j;
  if (c0 >= a.C) return;
  const float invM = 1.0f / (float)a.M;
  float m[8], r[8], kk[8], sg[8], sgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c0 + k;
    r[k] = 1.0f / sqrtf(var[c] + eps);
    m[k] = mean[c];
    kk[k] = (gamma ? gamma[c] : 1.f) * r[k];
    sg[k] = sum_g[c] * invM;
    sgx[k] = sum_gx[c] * invM;
  }
  for (long p = (long)blockIdx.x * PPB + pl; p < a.M; p += (long)gridDim.x * PPB) {
    float g[8], xv[8], v[8];
    ld8f32(a.dy + p * a.dycs + c0, g);
    ld8f32(a.x + p * a.xcs + c0, xv);
    if constexpr (MASK) {
      float yv[8];
      ld8bf(a.y + p * a.ycs + c0, yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = kk[k] * (g[k] - sg[k] - (xv[k] - m[k]) * r[k] * sgx[k]);
    float* o = a.dx + p * a.dxcs + c0;
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
    if constexpr (DX2) *reinterpret_cast<uint4*>(a.dx2 + p * a.dx2cs + c0) = Chunk<uint16_t>::pack(v);
  }
}

// elementwise passes over [M pixels x C channels]: CP (power of two >= C, at most 64) lanes per pixel, channel
// block blockIdx.y, so a lane keeps one channel (its per-channel constants in registers) and no element index is
// ever divided
// count > 0: the sums are over `count` pixels (SyncBN: all replicas' pixels), else over this view's M
template <bool MASK, int CP>
__global__ __launch_bounds__(256) void bn_bwd_apply(V x, V dy, V y, const float* mean, const float* var,
                                                    const float* gamma, float eps, const float* sum_g,
                                                    const float* sum_gx, V dx, V dx2, long count = 0) {
  const long M = (long)dy.n * dy.h * dy.w;
  const int c = blockIdx.y * CP + (threadIdx.x & (CP - 1));
  if (c >= dy.c) return;
  const float invM = 1.0f / (float)(count > 0 ? count : M);
  const float r = 1.0f / sqrtf(var[c] + eps);
  const float m = mean[c];
  const float k = (gamma ? gamma[c] : 1.f) * r;
  const float sg = sum_g[c] * invM, sgx = sum_gx[c] * invM;
  const long step = (long)gridDim.x * (blockDim.x / CP);
  long p = (long)blockIdx.x * (blockDim.x / CP) + threadIdx.x / CP;
  for (; p + 3 * step < M; p += 4 * step) {  // 4 pixels' loads in flight before the stores
    float xv[4], g[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      xv[u] = ld(x, p + u * step, c);
      g[u] = grad_in<MASK>(dy, y, p + u * step, c);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v = k * (g[u] - sg - (xv[u] - m) * r * sgx);
      st(dx, p + u * step, c, v);
      if (dx2.p) st(dx2, p + u * step, c, v);
    }
  }
  for (; p < M; p += step) {
    const float xh = (ld(x, p, c) - m) * r;
    const float g = grad_in<MASK>(dy, y, p, c);
    const float v = k * (g - sg - xh * sgx);
    st(dx, p, c, v);
    if (dx2.p) st(dx2, p, c, v);  // the bf16 copy the data-gradient conv reads
  }
}

// the unmasked 2-channel f32 case (the training step's select1_* convs) one pixel per thread with 8-byte loads and
// stores: at their 32-byte pixel stride the 2-lanes-per-pixel form above ran at ~0.5 TB/s, its per-element dtype
// branches and 64-bit index products the bound.  Per element the same expression as bn_bwd_apply, so the same values.
__global__ __launch_bounds__(256) void bn_bwd_apply2_f32(const float* x, int xcs, const float* dy, int dycs, float* dx,
                                                         int dxcs, long M, const float* mean, const float* var,
                                                         const float* gamma, float eps, const float* sum_g,
                                                         const float* sum_gx) {
  const float invM = 1.0f / (float)M;
  float r[2], m[2], k[2], sg[2], sgx[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    r[c] = 1.0f / sqrtf(var[c] + eps);
    m[c] = mean[c];
    k[c] = (gamma ? gamma[c] : 1.f) * r[c];
    sg[c] = sum_g[c] * invM;
    sgx[c] = sum_gx[c] * invM;
  }
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < M; p += (long)gridDim.x * blockDim.x) {
    const float2 x2 = *reinterpret_cast<const float2*>(x + p * xcs);
    const float2 g2 = *reinterpret_cast<const float2*>(dy + p * dycs);
    const float xv[2] = {x2.x, x2.y}, g[2] = {g2.x, g2.y};
    float v[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) v[c] = k[c] * (g[c] - sg[c] - (xv[c] - m[c]) * r[c] * sgx[c]);
    *reinterpret_cast<float2*>(dx + p * dxcs) = make_float2(v[0], v[1]);
  }
}

static bool f32_pair(const vm_tensor* t) {  // 2 f32 channels at an 8-byte aligned offset of every pixel
  return t->dtype == VM_F32 && t->c == 2 && t->cstride % 2 == 0 && t->coff % 2 == 0 &&
         reinterpret_cast<uintptr_t>(t->ptr) % 8 == 0;
}

// channels [0, split) go to dxlo at c, [split, C) to dx / dx2 at c - split (split 0: all to dx / dx2)
template <int CP>
__global__ __launch_bounds__(256) void relu_bwd_kernel(V dy, V y, V dx, V dx2, V dxlo, int split) {
  const long M = (long)dy.n * dy.h * dy.w;
  const int c = blockIdx.y * CP + (threadIdx.x & (CP - 1));
  if (c >= dy.c) return;
  const bool lo = c < split;
  const V o = lo ? dxlo : dx;
  const int oc = lo ? c : c - split;
  const bool two = dx2.p && !lo;
  const long step = (long)gridDim.x * (blockDim.x / CP);
  long p = (long)blockIdx.x * (blockDim.x / CP) + threadIdx.x / CP;
  for (; p + 3 * step < M; p += 4 * step) {  // 4 pixels' loads in flight before the stores
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld(y, p + u * step, c) > 0.f ? ld(dy, p + u * step, c) : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      st(o, p + u * step, oc, v[u]);
      if (two) st(dx2, p + u * step, oc, v[u]);
    }
  }
  for (; p < M; p += step) {
    const float v = ld(y, p, c) > 0.f ? ld(dy, p, c) : 0.f;
    st(o, p, oc, v);
    if (two) st(dx2, p, oc, v);
  }
}

static int lanes_for(int C) { return C > 32 ? 64 : C > 16 ? 32 : C > 8 ? 16 : C > 4 ? 8 : C > 2 ? 4 : C > 1 ? 2 : 1; }

// grid of an [M x C] packed-lane pass: x = pixel blocks (256/CP pixels each, capped), y = channel blocks
static dim3 lanes_grid(long M, int C, int cp) {
  const long px = (M + 256 / cp - 1) / (256 / cp);
  return dim3((unsigned)(px < 4096 ? px : 4096), (unsigned)((C + cp - 1) / cp));
}

#define VM_CP_SWITCH(CP_, CALL) \
  switch (CP_) {                \
    case 1: CALL(1); break;     \
    case 2: CALL(2); break;     \
    case 4: CALL(4); break;     \
    case 8: CALL(8); break;     \
    case 16: CALL(16); break;   \
    case 32: CALL(32); break;   \
    default: CALL(64); break;   \
  }

// ---------------------------------------------------------------- max-pool backward (small.py:40,42)
// Adjoint of tf.nn.max_pool 2x2/2 SAME (vm_maxpool2x2_same_nhwc): an input element receives its window's gradient
// iff it is the window's FIRST maximum in row-major order — TF's MaxPoolGrad scans the window with a strict '>'
// (taps past an odd edge are not in the window).  dx = add + that share (add optional; it may alias dx: each lane
// reads its own element before writing it).  CP lanes per input pixel as the other elementwise passes; a lane
// re-reads its window's other three values (L1/L2 hits) instead of a stored argmax.
template <int CP>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(V x, V dy, V add, V dx) {
  const long HW = (long)x.h * x.w, M = (long)x.n * HW;
  const int c = blockIdx.y * CP + (threadIdx.x & (CP - 1));
  if (c >= x.c) return;
  const int oh = dy.h, ow = dy.w;
  const long step = (long)gridDim.x * (blockDim.x / CP);
  for (long p = (long)blockIdx.x * (blockDim.x / CP) + threadIdx.x / CP; p < M; p += step) {
    const int n = (int)(p / HW);
    const int r = (int)(p - (long)n * HW);
    const int iy = r / x.w, ix = r - iy * x.w;
    const int y0 = iy & ~1, x0 = ix & ~1;
    const long base = (long)n * HW;
    float best = 0.f;
    int win = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int yy = y0 + (k >> 1), xx = x0 + (k & 1);
      if (yy < x.h && xx < x.w) {
        const float v = ld(x, base + (long)yy * x.w + xx, c);
        if (win < 0 || v > best) { best = v; win = k; }
      }
    }
    float g = win == ((iy - y0) << 1) + (ix - x0) ? ld(dy, ((long)n * oh + (iy >> 1)) * ow + (ix >> 1), c) : 0.f;
    if (add.p) g += ld(add, p, c);
    st(dx, p, c, g);
  }
}

// ---------------------------------------------------------------- relu conv backward front end (UNetImage training)
// For y = relu(conv(x) + b) (unet.py:35-42,65-74), one pass from the incoming gradient to what the conv's filter /
// data gradients read: dz = (y > 0) * g, written ONLY as the bf16 copy those MFMA convs read (no f32 dz), with the
// bias gradient sum_p dz from the same pass (f64 partials per block, folded in fixed order: deterministic).
//   plain: g = dy (+ add)                                 dy, add, y, dz all [n,h,w,c]
//   POOL : g = add + the 2x2 SAME max-pool adjoint of dy   dy [n,ceil(h/2),ceil(w/2),c], y / add / dz [n,h,w,c]
//          (tf.nn.max_pool's gradient to the window's first maximum of y in row-major order, TF MaxPoolGrad; the
//          skip half of an [up, skip] concat carries `add`, unet.py:62, so pool adjoint + concat gradient + relu
//          mask + bias sum are one pass instead of three)
// One lane per channel (CP lanes per pixel / window), a block's 4 waves stride over pixels (windows).
template <bool POOL, int CP>
__global__ __launch_bounds__(256) void relu_bwd_bias_kernel(V dy, V y, V add, V dz, double* part, int nblk) {
  constexpr int PPW = 64 / CP;
  __shared__ double sh[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * CP + (lane % CP);
  double s = 0.0;
  if (c < y.c) {
    const long units = POOL ? (long)dy.n * dy.h * dy.w : (long)y.n * y.h * y.w;
    const long stp = (long)nblk * 4 * PPW;
    for (long u = ((long)blockIdx.y * 4 + wave) * PPW + lane / CP; u < units; u += stp) {
      if constexpr (!POOL) {
        float g = ld(dy, u, c);
        if (add.p) g += ld(add, u, c);
        const float z = ld(y, u, c) > 0.f ? g : 0.f;
        st(dz, u, c, z);
        s += (double)z;
      } else {
        const long hw = (long)dy.h * dy.w;
        const int n = (int)(u / hw);
        const int r = (int)(u - (long)n * hw);
        const int oy = r / dy.w, ox = r - oy * dy.w;
        const long base = (long)n * y.h * y.w;
        const float gp = ld(dy, u, c);
        float yv[4];
        long pix[4];
        bool in[4];
        float best = 0.f;
        int win = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int yy = 2 * oy + (k >> 1), xx = 2 * ox + (k & 1);
          in[k] = yy < y.h && xx < y.w;
          pix[k] = base + (long)yy * y.w + xx;
          yv[k] = in[k] ? ld(y, pix[k], c) : 0.f;
          if (in[k] && (win < 0 || yv[k] > best)) {
            best = yv[k];
            win = k;
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!in[k]) continue;
          float g = k == win ? gp : 0.f;
          if (add.p) g += ld(add, pix[k], c);
          const float z = yv[k] > 0.f ? g : 0.f;
          st(dz, pix[k], c, z);
          s += (double)z;
        }
      }
    }
  }
  sh[wave][lane] = s;
  __syncthreads();
  if ((int)threadIdx.x < CP && c < y.c) {
    s = 0.0;
    for (int w = 0; w < 4; ++w)
      for (int k = 0; k < PPW; ++k) s += sh[w][k * CP + threadIdx.x];
    part[(long)c * nblk + blockIdx.y] = s;  // channel-major [C][nblk] (vm_common.h fold_columns)
  }
}

// Vectorised form for the bf16 path (bf16 y and dz, f32 dy / add; C % 8 == 0, C <= 512): a lane takes 8 channels of
// a pixel — one 16-byte y chunk, two f32x4 of dy and of add, one 16-byte dz store — where the per-element form above
// issued a 2- to 4-byte access per channel (~2.5 TB/s).  Per element the same arithmetic (g = dy, g += add in f32;
// the first-maximum pool adjoint; z rounded to bf16 as st() does), so dz is bit-identical; the channel sums are f64
// partials per block in another partition of the pixels, folded in fixed order by fold_sum_kernel as before.
// TPG: lanes per pixel (a power of two >= C / 8).  TD / TA: f32 or bf16 dy / add (the bf16 training path hands its
// data gradients over as bf16; a bf16 chunk widens exactly to f32, so the arithmetic after the load is the same).
template <bool POOL, bool ADD, int TPG, typename TD = float, typename TA = float>
__global__ __launch_bounds__(256) void relu_bwd_bias8_kernel(const TD* __restrict__ dy, int dycs,
                                                             const uint16_t* __restrict__ y, int ycs,
                                                             const TA* __restrict__ add, int acs,
                                                             uint16_t* __restrict__ dz, int zcs, int N, int H, int W,
                                                             int DH, int DW, int C, double* part, int nblk) {
  constexpr int PPB = 256 / TPG;
  __shared__ double sh[8][256];
  const int t = threadIdx.x, j = t % TPG, pl = t / TPG;
  const int c0 = 8 * j;
  double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  auto ld8y = [&](const uint16_t* p, float (&v)[8]) __attribute__((always_inline)) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = bf2f((uint16_t)(w4[k] & 0xffffu));
      v[2 * k + 1] = bf2f((uint16_t)(w4[k] >> 16));
    }
  };
  auto ld8f = [&](const auto* p, float (&v)[8]) __attribute__((always_inline)) {
    if constexpr (sizeof(*p) == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      ld8y(reinterpret_cast<const uint16_t*>(p), v);
    }
  };
  auto st8 = [&](uint16_t* p, const float (&z)[8]) __attribute__((always_inline)) {
    uint32_t w4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w4[k] = (uint32_t)f2bf(z[2 * k]) | ((uint32_t)f2bf(z[2 * k + 1]) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  };
  if (c0 < C) {
    const long units = POOL ? (long)N * DH * DW : (long)N * H * W;
    for (long u = (long)blockIdx.x * PPB + pl; u < units; u += (long)gridDim.x * PPB) {
      if constexpr (!POOL) {
        float g[8], yv[8], z[8];
        ld8f(dy + u * dycs + c0, g);
        if constexpr (ADD) {
          float a8[8];
          ld8f(add + u * acs + c0, a8);
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] += a8[k];
        }
        ld8y(y + u * ycs + c0, yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          z[k] = yv[k] > 0.f ? g[k] : 0.f;
          s[k] += (double)z[k];
        }
        st8(dz + u * zcs + c0, z);
      } else {
        const long hw = (long)DH * DW;
        const int n = (int)(u / hw);
        const int r = (int)(u - (long)n * hw);
        const int oy = r / DW, ox = r - oy * DW;
        float gp[8], yv[4][8];
        ld8f(dy + u * dycs + c0, gp);
        long pix[4];
        bool in[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int yy = 2 * oy + (q >> 1), xx = 2 * ox + (q & 1);
          in[q] = yy < H && xx < W;
          pix[q] = ((long)n * H + yy) * W + xx;
          if (in[q]) ld8y(y + pix[q] * ycs + c0, yv[q]);
          else
#pragma unroll
            for (int k = 0; k < 8; ++k) yv[q][k] = 0.f;
        }
        int win[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // TF MaxPoolGrad: the window's first maximum
          float best = 0.f;
          win[k] = -1;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (in[q] && (win[k] < 0 || yv[q][k] > best)) {
              best = yv[q][k];
              win[k] = q;
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (!in[q]) continue;
          float a8[8], z[8];
          if constexpr (ADD) ld8f(add + pix[q] * acs + c0, a8);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float g = k < 8 && win[k] == q ? gp[k] : 0.f;
            if constexpr (ADD) g += a8[k];
            z[k] = yv[q][k] > 0.f ? g : 0.f;
            s[k] += (double)z[k];
          }
          st8(dz + pix[q] * zcs + c0, z);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) sh[k][t] = s[k];
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    const int jj = c >> 3, k = c & 7;
    double r = 0.0;
    for (int q = 0; q < PPB; ++q) r += sh[k][q * TPG + jj];
    part[(long)c * nblk + blockIdx.x] = r;  // channel-major [C][nblk], as relu_bwd_bias_kernel
  }
}

__global__ __launch_bounds__(256) void fold_sum_kernel(const double* part, int nblk, int C, float* out) {
  double r[3];
  fold_columns(part, nblk, C, blockIdx.x, 1, r);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)r[0];
}

// ---------------------------------------------------------------- resize backward (adjoint of resize_tf1)
__device__ __forceinline__ void tf1c(int i, float scale, int in, int& lo, int& hi, float& lerp) {
#pragma clang fp contract(off)
  const float src = (float)i * scale;
  const float fl = floorf(src);
  lo = (int)fl;
  hi = min(lo + 1, in - 1);
  lerp = src - fl;
}

// Gather form (deterministic, no atomics): input pixel (iy, ix) collects the output pixels whose taps hit it.  With
// scale = in/out <= ~1 those lie in rows [floor((iy-1)/sy)-1, ceil((iy+1)/sy)+1] (likewise columns); each candidate's
// taps are recomputed with the forward's exact f32 coordinate arithmetic, so the weights match it bit for bit.
__device__ __forceinline__ float tap_w(int o, float scale, int in, int i) {
  int lo, hi;
  float l;
  tf1c(o, scale, in, lo, hi, l);
  return (lo == i ? 1.f - l : 0.f) + (hi == i ? l : 0.f);
}

__global__ void resize_bwd_kernel(V dy, float* dx, int ih, int iw, float sy, float sx) {
  const long total = (long)dy.n * ih * iw * dy.c;
  const int C = dy.c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long ip = i / C;
    const int ix = (int)(ip % iw);
    const long t = ip / iw;
    const int iy = (int)(t % ih);
    const int n = (int)(t / ih);
    const int r0 = max(0, (int)floorf((iy - 1) / sy) - 1), r1 = min(dy.h - 1, (int)ceilf((iy + 1) / sy) + 1);
    const int q0 = max(0, (int)floorf((ix - 1) / sx) - 1), q1 = min(dy.w - 1, (int)ceilf((ix + 1) / sx) + 1);
    float acc = 0.f;
    for (int oh = r0; oh <= r1; ++oh) {
      const float wy = tap_w(oh, sy, ih, iy);
      if (wy == 0.f) continue;
      float row = 0.f;
      for (int ow = q0; ow <= q1; ++ow) {
        const float wx = tap_w(ow, sx, iw, ix);
        if (wx != 0.f) row += wx * ld(dy, ((long)n * dy.h + oh) * dy.w + ow, c);
      }
      acc += wy * row;
    }
    dx[i] = acc;
  }
}

// the same gather, 4 channels per thread with 16-byte loads / stores (c % 4 == 0, 16-byte aligned dy channel
// vectors): the taps and weights are computed once per 4 channels; per channel the arithmetic is resize_bwd_kernel's
// TD: dy f32 (16-byte loads) or bf16 (8-byte loads: the bf16 training path's data gradients); TX: dx f32, or bf16
// (each f32 sum rounded to nearest even once, as a bf16 store of the f32 result would)
template <typename TD, typename TX = float>
__global__ void resize_bwd_kernel4(V dy, TX* dx, int ih, int iw, float sy, float sx) {
  const int C4 = dy.c / 4;
  const long total = (long)dy.n * ih * iw * C4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const long ip = i / C4;
    const int ix = (int)(ip % iw);
    const long t = ip / iw;
    const int iy = (int)(t % ih);
    const int n = (int)(t / ih);
    const int r0 = max(0, (int)floorf((iy - 1) / sy) - 1), r1 = min(dy.h - 1, (int)ceilf((iy + 1) / sy) + 1);
    const int q0 = max(0, (int)floorf((ix - 1) / sx) - 1), q1 = min(dy.w - 1, (int)ceilf((ix + 1) / sx) + 1);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int oh = r0; oh <= r1; ++oh) {
      const float wy = tap_w(oh, sy, ih, iy);
      if (wy == 0.f) continue;
      float4 row = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int ow = q0; ow <= q1; ++ow) {
        const float wx = tap_w(ow, sx, iw, ix);
        if (wx != 0.f) {
          float4 v;
          if constexpr (sizeof(TD) == 4) {
            v = *reinterpret_cast<const float4*>(
                reinterpret_cast<const float*>(dy.p) + (((long)n * dy.h + oh) * dy.w + ow) * dy.cs + dy.coff + c);
          } else {
            const uint2 u = *reinterpret_cast<const uint2*>(
                reinterpret_cast<const uint16_t*>(dy.p) + (((long)n * dy.h + oh) * dy.w + ow) * dy.cs + dy.coff + c);
            v = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                            __uint_as_float(u.y & 0xffff0000u));
          }
          row.x += wx * v.x;
          row.y += wx * v.y;
          row.z += wx * v.z;
          row.w += wx * v.w;
        }
      }
      acc.x += wy * row.x;
      acc.y += wy * row.y;
      acc.z += wy * row.z;
      acc.w += wy * row.w;
    }
    if constexpr (sizeof(TX) == 4) {
      *reinterpret_cast<float4*>(dx + ip * dy.c + c) = acc;
    } else {
      const uint2 u = make_uint2((uint32_t)f2bf(acc.x) | ((uint32_t)f2bf(acc.y) << 16),
                                 (uint32_t)f2bf(acc.z) | ((uint32_t)f2bf(acc.w) << 16));
      *reinterpret_cast<uint2*>(dx + ip * dy.c + c) = u;
    }
  }
}

// ---------------------------------------------------------------- conv weight gradient
constexpr int WG_TH = 4, WG_TW = 32, WG_PH = WG_TH + 2, WG_PW = WG_TW + 2, WG_NT = 256;

// XV: x is T-typed with 16-byte aligned channel vectors (cin, coff, cstride multiples of the vector width), so a
// pixel's CC channels arrive as CC/VE 16-byte loads, all of a thread's loads issued before any LDS store.
// DV: likewise dy as float4 (cout % 4 == 0).  Otherwise element loads.
template <int CC, int CO4, typename T, bool XV, bool DV>
__global__ __launch_bounds__(WG_NT) void wgrad_kernel(V x, V dy, float* partials,
                                                      int tiles_h, int tiles_w, long ntiles) {
  constexpr int TASKS = 3 * CC * CO4;
  constexpr int TPT = (TASKS + WG_NT - 1) / WG_NT;
  constexpr int VE = 16 / sizeof(T), NVP = CC / VE, NV = WG_PH * WG_PW * NVP;
  constexpr int VPT = XV ? (NV + WG_NT - 1) / WG_NT : 1;
  constexpr int ND = WG_TH * WG_TW * CO4, DPT = DV ? (ND + WG_NT - 1) / WG_NT : 1;
  __shared__ float xs[WG_PH * WG_PW * CC];
  __shared__ float4 ds[WG_TH * WG_TW * CO4];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.y * CC;
  const int cin = x.c, cout = dy.c;
  // this block's partial filter gradient: row blockIdx.x of the [gridDim.x][3][3][cin][cout] workspace
  float* part = partials + (long)blockIdx.x * 9 * cin * cout;
  float acc[TPT][3][4];
#pragma unroll
  for (int k = 0; k < TPT; ++k)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[k][j][0] = acc[k][j][1] = acc[k][j][2] = acc[k][j][3] = 0.f;

  // vector paths: the next tile's 16-byte loads are issued into registers before the current tile's FMAs,
  // so their latency hides under the compute (register double buffer; LDS holds the current tile)
  uint4 xb[VPT];
  float4 db[DPT];
  auto coords = [&](long tile, int& n, int& y0, int& x0) {
    const int tx = (int)(tile % tiles_w);
    const long t2 = tile / tiles_w;
    y0 = (int)(t2 % tiles_h) * WG_TH;
    n = (int)(t2 / tiles_h);
    x0 = tx * WG_TW;
  };
  auto issue = [&](int tile) {
    int n, y0, x0;
    coords(tile, n, y0, x0);
    if constexpr (XV) {
#pragma unroll
      for (int k = 0; k < VPT; ++k) {
        const int e = tid + k * WG_NT;
        xb[k] = make_uint4(0, 0, 0, 0);
        if (NV % WG_NT == 0 || e < NV) {
          const int j = e % NVP, pc = e / NVP;
          const int gy = y0 + pc / WG_PW - 1, gx = x0 + pc % WG_PW - 1, c = c0 + j * VE;
          if (gy >= 0 && gy < x.h && gx >= 0 && gx < x.w && c < cin)
            xb[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(x.p) +
                                                    (((long)n * x.h + gy) * x.w + gx) * x.cs + x.coff + vchan(x, c));
        }
      }
    }
    if constexpr (DV) {
#pragma unroll
      for (int k = 0; k < DPT; ++k) {
        const int e = tid + k * WG_NT;
        db[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ND % WG_NT == 0 || e < ND) {
          const int cg = e % CO4, pp = e / CO4;
          const int gy = y0 + pp / WG_TW, gx = x0 + pp % WG_TW;
          if (gy < x.h && gx < x.w && cg * 4 < cout)
            db[k] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dy.p) +
                                                     (((long)n * x.h + gy) * x.w + gx) * dy.cs + dy.coff + cg * 4);
        }
      }
    }
  };
  auto commit = [&](long tile) {
    int n, y0, x0;
    coords(tile, n, y0, x0);
    if constexpr (XV) {
#pragma unroll
      for (int k = 0; k < VPT; ++k) {
        const int e = tid + k * WG_NT;
        if (NV % WG_NT == 0 || e < NV) {
          float f[VE];
          Chunk<T>::unpack(xb[k], f);
          const int c = c0 + (e % NVP) * VE;  // a vector straddling cin (padded views): zero the lanes past it
#pragma unroll
          for (int i = 0; i < VE; ++i)
            if (c + i >= cin) f[i] = 0.f;
          float4* d = reinterpret_cast<float4*>(xs + (e / NVP) * CC + (e % NVP) * VE);
#pragma unroll
          for (int i = 0; i < VE / 4; ++i) d[i] = make_float4(f[4 * i], f[4 * i + 1], f[4 * i + 2], f[4 * i + 3]);
        }
      }
    } else {
      for (int e = tid; e < WG_PH * WG_PW * CC; e += WG_NT) {
        const int ci = e % CC;
        const int pc = e / CC;
        const int gy = y0 + pc / WG_PW - 1, gx = x0 + pc % WG_PW - 1, c = c0 + ci;
        float v = 0.f;
        if (gy >= 0 && gy < x.h && gx >= 0 && gx < x.w && c < cin) v = ld(x, ((long)n * x.h + gy) * x.w + gx, c);
        xs[e] = v;
      }
    }
    if constexpr (DV) {
#pragma unroll
      for (int k = 0; k < DPT; ++k) {
        const int e = tid + k * WG_NT;
        if (ND % WG_NT == 0 || e < ND) ds[e] = db[k];
      }
    } else {
      float* dsf = reinterpret_cast<float*>(ds);
      for (int e = tid; e < WG_TH * WG_TW * CO4 * 4; e += WG_NT) {
        const int co = e % (CO4 * 4);
        const int pp = e / (CO4 * 4);
        const int gy = y0 + pp / WG_TW, gx = x0 + pp % WG_TW;
        float v = 0.f;
        if (gy < x.h && gx < x.w && co < cout) v = ld(dy, ((long)n * x.h + gy) * x.w + gx, co);
        dsf[e] = v;
      }
    }
  };

  if (blockIdx.x < ntiles) issue(blockIdx.x);
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    commit(tile);
    __syncthreads();
    if (tile + gridDim.x < ntiles) issue(tile + gridDim.x);
#pragma unroll
    for (int k = 0; k < TPT; ++k) {
      const int t = tid + k * WG_NT;
      if (TASKS % WG_NT == 0 || t < TASKS) {
        const int ci = t % CC;
        const int cg = (t / CC) % CO4;
        const int kh = t / (CC * CO4);
        for (int py = 0; py < WG_TH; ++py) {
          const float* row = xs + ((py + kh) * WG_PW) * CC + ci;
          const float4* drow = ds + py * WG_TW * CO4 + cg;
          float xa = row[0], xb = row[CC];
#pragma unroll 8
          for (int px = 0; px < WG_TW; ++px) {
            const float xc = row[(px + 2) * CC];
            const float4 d = drow[px * CO4];
            acc[k][0][0] += xa * d.x; acc[k][0][1] += xa * d.y; acc[k][0][2] += xa * d.z; acc[k][0][3] += xa * d.w;
            acc[k][1][0] += xb * d.x; acc[k][1][1] += xb * d.y; acc[k][1][2] += xb * d.z; acc[k][1][3] += xb * d.w;
            acc[k][2][0] += xc * d.x; acc[k][2][1] += xc * d.y; acc[k][2][2] += xc * d.z; acc[k][2][3] += xc * d.w;
            xa = xb;
            xb = xc;
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < TPT; ++k) {
    const int t = tid + k * WG_NT;
    if (TASKS % WG_NT == 0 || t < TASKS) {
      const int ci = t % CC;
      const int cg = (t / CC) % CO4;
      const int kh = t / (CC * CO4);
      const int c = c0 + ci;
      if (c < cin) {
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int co = cg * 4 + j;
            if (co < cout) part[(((long)(kh * 3 + kw) * cin + c) * cout + co)] = acc[k][kw][j];
          }
      }
    }
  }
}

// ---------------------------------------------------------------- conv weight gradient on MFMA (bf16 operands)
// dW_t[ci][co] = sum_p X[p + off_t][ci] * DY[p][co] (t = kh*3 + kw, off_t = (kh-1, kw-1)) as 9 GEMMs whose K axis is
// the pixels: v_mfma_f32_16x16x32_bf16 with A = X^T (16 input channels x 32 pixels), B = DY (32 pixels x 16 output
// channels), f32 accumulation.  Both operands sit in LDS in their natural NHWC order ([pixel][channel] rows) and are
// read k-major with ds_read_b64_tr_b16, so no transpose pass exists anywhere.  One of the two operands carries the
// 1-pixel halo and is read at the 9 tap offsets; the other is read once per K-step and reused by the 9 taps:
//   SX  (shift x):  X patch (TH+2) x (TW+2) x CIB, DY tile TH x TW x COP        — wide cout (upconv*, conv*)
//   !SX (shift dy): X tile TH x TW x CIB, DY patch (TH+2) x (TW+2) x COP       — narrow cout (select*, output):
//                   dW_t = sum_q X[q] * DY[q - off_t], with DY zero outside the frame
// Block = 4 waves on one TH(4) x TW(32) pixel tile, wave w owns tile row w (one 32-pixel K-step); blocks walk tiles
// (split-K over gridDim.x, one partial per block, the fixed-order wgrad_reduce_kernel sums them: deterministic).
// DY arrives f32 and is rounded to bf16 when staged (the bf16 training path's precision: bf16 operands, f32 sums).
// The LDS images are swizzled so every transposed read (two 16-lane groups 8 rows apart per 32-lane half) is
// conflict-free for any row base (tap shifts move it by 0..2 rows/pixels).
constexpr int WM_TW = 32, WM_PW = WM_TW + 2;
// patch pixels of a TH x 32 tile with its halo, and the image rows allocated for them (a multiple of 16, so the row
// swizzle stays in range)
template <int TH>
constexpr int wm_ppix() { return (TH + 2) * WM_PW; }
template <int TH>
constexpr int wm_prows() { return (wm_ppix<TH>() + 15) / 16 * 16; }

struct WgArgs {
  const uint16_t* x;  // bf16 input view base (pixel 0, channel coff applied)
  int n, h, w, cin, xcs, x_src_c;  // x_src_c > 0: channel c lives in source c / x_src_c at + x_src_stride elements
  long x_src_stride;
  const float* dy;  // f32 output-gradient view base (coff applied)
  int cout, dcs;
  float* part;      // [gridDim.x][9][cin][cout]
  int tiles_h, tiles_w;
  long ntiles;
};

// byte offset of 32-byte piece c (16 bf16 channels) of image row r, rows of RB bytes (32, 64 or 128)
template <int RB>
__device__ __forceinline__ int wm_off(int r, int c) {
  if constexpr (RB == 32) return 32 * (r ^ (((r >> 3) & 1) << 2));
  else if constexpr (RB == 64) return 64 * r + 32 * (c ^ ((r >> 3) & 1));
  else return 128 * r + 32 * (c ^ ((r >> 1) & 1) ^ (((r >> 3) & 1) << 1));
}

typedef short v4s __attribute__((ext_vector_type(4)));

// the 16x16x32 operand fragment whose k rows are image rows rk(0..7) (8 consecutive pixels of one image row band),
// columns = 16-channel piece c: two transposed 4-row reads
template <int RB>
__device__ __forceinline__ bf16x8 wm_frag(const char* img, int r0, int c, int lane) {
  const int q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) v4s* lp;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + wm_off<RB>(r0 + q, c) + 8 * p));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + wm_off<RB>(r0 + 4 + q, c) + 8 * p));
  v4s v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v);
}

// PIPE (r05): every fragment address is computed once per kernel (the LDS images keep their layout from tile to
// tile) and the next tap's fragments are read while the current tap's MFMAs run (the plain loop let hipcc recompute
// the swizzled addresses and wait lgkmcnt(0) in front of every tap's MFMAs).  Same MFMAs per accumulator in the same
// order: bit-identical.
template <int NCI, int NCO, bool SX, int TH, bool PIPE = true>
__global__ __launch_bounds__(256, 2) void wgrad_mfma_kernel(WgArgs a) {
  constexpr int WM_TH = TH, WM_PPIX = wm_ppix<TH>(), WM_PROWS = wm_prows<TH>();
  constexpr int CIB = NCI * 16, COP = NCO * 16;
  constexpr int RBX = NCI == 1 ? 32 : NCI == 2 ? 64 : 128;
  constexpr int RBD = NCO == 1 ? 32 : NCO == 2 ? 64 : 128;
  constexpr int XROWS = SX ? WM_PROWS : WM_TH * WM_TW, DROWS = SX ? WM_TH * WM_TW : WM_PROWS;
  constexpr int XBYTES = XROWS * RBX, DBYTES = DROWS * RBD;
  constexpr int XPIX = SX ? WM_PPIX : WM_TH * WM_TW, DPIX = SX ? WM_TH * WM_TW : WM_PPIX;
  constexpr int XCH = CIB / 8, DCH = COP / 8;                    // 16-byte chunks per pixel row
  constexpr int NXC = XPIX * XCH, NDC = DPIX * DCH;
  constexpr int XPT = (NXC + 255) / 256, DPT = (NDC + 255) / 256;
  constexpr int RED = 9 * NCI * NCO * 4 * 64 * 4;                // one wave's accumulators in bytes
  constexpr int MAIN = XBYTES + DBYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  (void)RED;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.y * CIB;
  char* ximg = smem;
  char* dimg = smem + XBYTES;

  f32x4 acc[9][NCI][NCO];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < NCI; ++i)
#pragma unroll
      for (int o = 0; o < NCO; ++o) acc[t][i][o] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 xb[XPT];
  float4 db[DPT][2];
  auto coords = [&](int tile, int& n, int& y0, int& x0) {
    const int tx = tile % a.tiles_w;
    const int t2 = tile / a.tiles_w;
    y0 = (t2 % a.tiles_h) * WM_TH;
    n = t2 / a.tiles_h;
    x0 = tx * WM_TW;
  };
  // image pixel e of the patch (halo: origin (y0-1, x0-1), 34 wide) or the tile (origin (y0, x0), 32 wide)
  auto pix = [&](int e, bool halo, int y0, int x0, int& gy, int& gx) {
    if (halo) {
      gy = y0 - 1 + e / WM_PW;
      gx = x0 - 1 + e % WM_PW;
    } else {
      gy = y0 + e / WM_TW;
      gx = x0 + e % WM_TW;
    }
  };
  auto issue = [&](int tile) {
    int n, y0, x0;
    coords(tile, n, y0, x0);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      xb[k] = make_uint4(0, 0, 0, 0);
      if (NXC % 256 == 0 || e < NXC) {
        const int pe = e / XCH, j = e % XCH;
        int gy, gx;
        pix(pe, SX, y0, x0, gy, gx);
        const int c = c0 + j * 8;
        if ((unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w && c < a.cin) {
          long off = (((long)n * a.h + gy) * a.w + gx) * a.xcs;
          if (a.x_src_c > 0) off += (long)(c / a.x_src_c) * a.x_src_stride + c % a.x_src_c;
          else off += c;
          xb[k] = *reinterpret_cast<const uint4*>(a.x + off);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = tid + k * 256;
      db[k][0] = db[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (NDC % 256 == 0 || e < NDC) {
        const int pe = e / DCH, j = e % DCH;
        int gy, gx;
        pix(pe, !SX, y0, x0, gy, gx);
        const int co = j * 8;
        if ((unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w && co < a.cout) {
          const float* src = a.dy + (((long)n * a.h + gy) * a.w + gx) * a.dcs + co;
          if (co + 8 <= a.cout && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            db[k][0] = *reinterpret_cast<const float4*>(src);
            db[k][1] = *reinterpret_cast<const float4*>(src + 4);
          } else {
            float f[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) f[i] = co + i < a.cout ? src[i] : 0.f;
            db[k][0] = make_float4(f[0], f[1], f[2], f[3]);
            db[k][1] = make_float4(f[4], f[5], f[6], f[7]);
          }
        }
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      if (NXC % 256 == 0 || e < NXC) {
        const int pe = e / XCH, j = e % XCH;
        uint4 v = xb[k];
        const int c = c0 + j * 8;
        if (c + 8 > a.cin) {  // a chunk straddling cin (padded views): zero the lanes past it
          uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (c + 2 * i >= a.cin) w4[i] = 0u;
            else if (c + 2 * i + 1 >= a.cin) w4[i] &= 0xffffu;
          }
          v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        *reinterpret_cast<uint4*>(ximg + wm_off<RBX>(pe, j >> 1) + (j & 1) * 16) = v;
      }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = tid + k * 256;
      if (NDC % 256 == 0 || e < NDC) {
        const int pe = e / DCH, j = e % DCH;
        const float f[8] = {db[k][0].x, db[k][0].y, db[k][0].z, db[k][0].w,
                            db[k][1].x, db[k][1].y, db[k][1].z, db[k][1].w};
        *reinterpret_cast<uint4*>(dimg + wm_off<RBD>(pe, j >> 1) + (j & 1) * 16) = Chunk<uint16_t>::pack(f);
      }
    }
  };

  const int g = lane >> 4;
  // a contiguous run of tiles per block: consecutive K-steps stay on neighbouring rows of the same pages (a
  // gridDim-strided walk jumps megabytes per step and pays TLB misses on every one)
  const int t_beg = (int)((long)blockIdx.x * a.ntiles / gridDim.x);
  const int t_end = (int)((long)(blockIdx.x + 1) * a.ntiles / gridDim.x);
  if constexpr (PIPE) {
    constexpr int RR = TH / 4, NTX = SX ? 9 : 1, NTD = SX ? 1 : 9;
    const int q = (lane >> 2) & 3, p = lane & 3;
    int xa[RR][NTX][NCI][2], da[RR][NTD][NCO][2];  // byte offsets of the lo / hi reads of every fragment
#pragma unroll
    for (int rr = 0; rr < RR; ++rr) {
      const int row = wave + 4 * rr;
#pragma unroll
      for (int tt = 0; tt < NTX; ++tt) {
        const int r0 = SX ? (row + tt / 3) * WM_PW + tt % 3 + 8 * g : row * WM_TW + 8 * g;
#pragma unroll
        for (int i = 0; i < NCI; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h) xa[rr][tt][i][h] = wm_off<RBX>(r0 + 4 * h + q, i) + 8 * p;
      }
#pragma unroll
      for (int tt = 0; tt < NTD; ++tt) {
        const int r0 = SX ? row * WM_TW + 8 * g : (row + 2 - tt / 3) * WM_PW + 2 - tt % 3 + 8 * g;
#pragma unroll
        for (int o = 0; o < NCO; ++o)
#pragma unroll
          for (int h = 0; h < 2; ++h) da[rr][tt][o][h] = wm_off<RBD>(r0 + 4 * h + q, o) + 8 * p;
      }
    }
    auto frag = [&](const char* img, const int (&ad)[2]) __attribute__((always_inline)) {
      typedef __attribute__((address_space(3))) v4s* lp;
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + ad[0]));
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + ad[1]));
      v4s v[2] = {lo, hi};
      return __builtin_bit_cast(bf16x8, v);
    };
    constexpr int NP = SX ? NCI : NCO;  // fragments read per tap (the shifted operand)
    if (t_beg < t_end) issue(t_beg);
    for (int tile = t_beg; tile < t_end; ++tile) {
      commit();
      __syncthreads();
      if (tile + 1 < t_end) issue(tile + 1);
      // (a row's 9 taps carry only 9 x NCI x NCO MFMAs, too few to hide a read one tap ahead: all of the row's
      // fragments are read up front and the MFMAs wait for them in order)
      static_for<0, RR>([&](auto rc) __attribute__((always_inline)) {
        constexpr int rr = decltype(rc)::value;
        bf16x8 fix[SX ? NCO : NCI], sh[9][NP];  // the per-row operand, the per-tap one
#pragma unroll
        for (int k = 0; k < (SX ? NCO : NCI); ++k) fix[k] = SX ? frag(dimg, da[rr][0][k]) : frag(ximg, xa[rr][0][k]);
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int k = 0; k < NP; ++k) sh[t][k] = SX ? frag(ximg, xa[rr][SX ? t : 0][k]) : frag(dimg, da[rr][SX ? 0 : t][k]);
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int i = 0; i < NCI; ++i)
#pragma unroll
            for (int o = 0; o < NCO; ++o)
              acc[t][i][o] = SX ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(sh[t][i], fix[o], acc[t][i][o], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fix[i], sh[t][o], acc[t][i][o], 0, 0, 0);
        // (pinned: left alone, hipcc sinks each tap's reads to just before its MFMAs to keep 3 waves per SIMD)
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * ((SX ? NCO : NCI) + 9 * NP), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 9 * NCI * NCO, 0);
      });
      __syncthreads();
    }
  } else {
  if (t_beg < t_end) issue(t_beg);
  for (int tile = t_beg; tile < t_end; ++tile) {
    commit();
    __syncthreads();
    if (tile + 1 < t_end) issue(tile + 1);
    // K-steps: the 32 pixels of tile rows wave, wave+4, ...; group g of a fragment holds pixels 8g..8g+7
#pragma unroll
    for (int rr = 0; rr < TH / 4; ++rr) {
      const int row = wave + 4 * rr;
      if constexpr (SX) {
        bf16x8 bd[NCO];
#pragma unroll
        for (int o = 0; o < NCO; ++o) bd[o] = wm_frag<RBD>(dimg, row * WM_TW + 8 * g, o, lane);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int r0 = (row + t / 3) * WM_PW + t % 3 + 8 * g;
#pragma unroll
          for (int i = 0; i < NCI; ++i) {
            const bf16x8 ax = wm_frag<RBX>(ximg, r0, i, lane);
#pragma unroll
            for (int o = 0; o < NCO; ++o)
              acc[t][i][o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax, bd[o], acc[t][i][o], 0, 0, 0);
          }
        }
      } else {
        bf16x8 ax[NCI];
#pragma unroll
        for (int i = 0; i < NCI; ++i) ax[i] = wm_frag<RBX>(ximg, row * WM_TW + 8 * g, i, lane);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          // DY[q - off_t]: patch coordinates (row + 2 - kh, col + 2 - kw)
          const int r0 = (row + 2 - t / 3) * WM_PW + 2 - t % 3 + 8 * g;
#pragma unroll
          for (int o = 0; o < NCO; ++o) {
            const bf16x8 bd = wm_frag<RBD>(dimg, r0, o, lane);
#pragma unroll
            for (int i = 0; i < NCI; ++i)
              acc[t][i][o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[i], bd, acc[t][i][o], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  }
  }

  // fold the 4 waves' accumulators (LDS, two rounds), wave 0 stores the block's partial
  float* red = reinterpret_cast<float*>(smem);
  constexpr int NA = 9 * NCI * NCO * 4;
  auto put = [&](int slot) {
    int k = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < NCI; ++i)
#pragma unroll
        for (int o = 0; o < NCO; ++o)
#pragma unroll
          for (int j = 0; j < 4; ++j, ++k) red[(slot * NA + k) * 64 + lane] = acc[t][i][o][j];
  };
  auto add = [&](int slot) {
    int k = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < NCI; ++i)
#pragma unroll
        for (int o = 0; o < NCO; ++o)
#pragma unroll
          for (int j = 0; j < 4; ++j, ++k) acc[t][i][o][j] += red[(slot * NA + k) * 64 + lane];
  };
  if (wave >= 2) put(wave - 2);
  __syncthreads();
  if (wave < 2) add(wave);
  __syncthreads();
  if (wave == 1) put(0);
  __syncthreads();
  if (wave == 0) {
    add(0);
    float* part = a.part + (long)blockIdx.x * 9 * a.cin * a.cout;
    const int co_l = lane & 15, ci_l = 4 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < NCI; ++i)
#pragma unroll
        for (int o = 0; o < NCO; ++o) {
          const int co = o * 16 + co_l;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ci = c0 + i * 16 + ci_l + j;
            if (ci < a.cin && co < a.cout) part[((long)t * a.cin + ci) * a.cout + co] = acc[t][i][o][j];
          }
        }
  }
  (void)MAIN;
}

template <int NCI, int NCO, bool SX, int TH>
constexpr int wgrad_mfma_lds() {
  constexpr int RBX = NCI == 1 ? 32 : NCI == 2 ? 64 : 128;
  constexpr int RBD = NCO == 1 ? 32 : NCO == 2 ? 64 : 128;
  constexpr int XROWS = SX ? wm_prows<TH>() : TH * WM_TW, DROWS = SX ? TH * WM_TW : wm_prows<TH>();
  constexpr int MAIN = XROWS * RBX + DROWS * RBD;
  constexpr int RED = 2 * 9 * NCI * NCO * 4 * 64 * 4;
  return MAIN > RED ? MAIN : RED;
}

// Narrow-cout weight gradient with the taps packed into N (select convs, cout <= 8): one GEMM
//   dW[ci][t*cout + co] = sum_q X[q][ci] * DY[q - off_t][co]
// whose N axis holds all 9 taps x cout columns (cout 2 -> 18 of 32, 4 -> 36 of 48, 8 -> 72 of 80), so a K-step of 32
// pixels costs NCI x NT MFMAs (2 x 4 = 8 for cout 2) where wgrad_mfma_kernel's !SX form spends 9 per 16 channels
// on one 16-wide column block holding cout of them.  The B fragments come from three bf16 planes of the DY patch,
// plane kw pre-shifted by its tap column (P_kw[r][j] = patch(r, j + 2 - kw)), so every lane's 8 pixels are one
// aligned 16-byte LDS read: lane (n, g) reads P_kw[row + 2 - kh][8g .. 8g + 7] of channel co, (kh, kw, co) = n's tap.
// With 32-80 accumulator registers a block holds 64 input channels (one tower source: 128-byte pixel rows) and
// 8 blocks fit a CU, so ~4x the bytes of X are in flight per CU than with the 160-register variants — the select
// wgrads read 40-315 MB of tower features each and are bound by that.
template <int TH>
constexpr int wt_drows() { return TH + 2; }

template <int NCI, int NT, int TH>
__global__ __launch_bounds__(256) void wgrad_taps_kernel(WgArgs a) {
  constexpr int CIB = NCI * 16;
  constexpr int RBX = NCI == 1 ? 32 : NCI == 2 ? 64 : 128;
  constexpr int XPIX = TH * WM_TW, XCH = CIB / 8, NXC = XPIX * XCH, XPT = (NXC + 255) / 256;
  constexpr int DR = wt_drows<TH>();
  constexpr int COMAX = NT * 16 / 9;                        // the widest cout this NT serves
  constexpr int NDE = DR * WM_PW * COMAX, DPT = (NDE + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.y * CIB;
  const int cout = a.cout, ndy = DR * WM_PW * cout;
  char* ximg = smem;
  uint16_t* dpl = reinterpret_cast<uint16_t*>(smem + XPIX * RBX);  // [3][cout][DR][32]

  f32x4 acc[NCI][NT];
#pragma unroll
  for (int i = 0; i < NCI; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this lane's B column: n = nt * 16 + (lane & 15) -> (tap, co); columns past 9 * cout read a zero slot
  const int g = lane >> 4;
  int boff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = t * 16 + (lane & 15);
    if (n < 9 * cout) {
      const int tap = n / cout, co = n - tap * cout, kh = tap / 3, kw = tap - kh * 3;
      boff[t] = ((kw * cout + co) * DR + 2 - kh) * WM_TW + 8 * g;  // + row * 32 per K-step
    } else {
      boff[t] = -1;
    }
  }

  uint4 xb[XPT];
  float db[DPT];
  auto coords = [&](int tile, int& n, int& y0, int& x0) {
    const int tx = tile % a.tiles_w;
    const int t2 = tile / a.tiles_w;
    y0 = (t2 % a.tiles_h) * TH;
    n = t2 / a.tiles_h;
    x0 = tx * WM_TW;
  };
  auto issue = [&](int tile) {
    int n, y0, x0;
    coords(tile, n, y0, x0);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      xb[k] = make_uint4(0, 0, 0, 0);
      if (NXC % 256 == 0 || e < NXC) {
        const int pe = e / XCH, j = e % XCH;
        const int gy = y0 + pe / WM_TW, gx = x0 + pe % WM_TW, c = c0 + j * 8;
        if (gy < a.h && gx < a.w && c < a.cin) {
          long off = (((long)n * a.h + gy) * a.w + gx) * a.xcs;
          if (a.x_src_c > 0) off += (long)(c / a.x_src_c) * a.x_src_stride + c % a.x_src_c;
          else off += c;
          xb[k] = *reinterpret_cast<const uint4*>(a.x + off);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {  // the halo patch, (pixel, co) elements in memory order
      const int e = tid + k * 256;
      db[k] = 0.f;
      if (e < ndy) {
        const int pe = e / cout, co = e - pe * cout;
        const int gy = y0 - 1 + pe / WM_PW, gx = x0 - 1 + pe % WM_PW;
        if ((unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w)
          db[k] = a.dy[(((long)n * a.h + gy) * a.w + gx) * a.dcs + co];
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      if (NXC % 256 == 0 || e < NXC) {
        const int pe = e / XCH, j = e % XCH;
        uint4 v = xb[k];
        const int c = c0 + j * 8;
        if (c + 8 > a.cin) {  // a chunk straddling cin (padded views): zero the lanes past it
          uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (c + 2 * i >= a.cin) w4[i] = 0u;
            else if (c + 2 * i + 1 >= a.cin) w4[i] &= 0xffffu;
          }
          v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        *reinterpret_cast<uint4*>(ximg + wm_off<RBX>(pe, j >> 1) + (j & 1) * 16) = v;
      }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = tid + k * 256;
      if (e < ndy) {
        const int pe = e / cout, co = e - pe * cout;
        const int r = pe / WM_PW, pc = pe % WM_PW;
        const uint16_t v = f2bf(db[k]);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int j = pc - 2 + kw;
          if (j >= 0 && j < WM_TW) dpl[((kw * cout + co) * DR + r) * WM_TW + j] = v;
        }
      }
    }
  };

  const int t_beg = (int)((long)blockIdx.x * a.ntiles / gridDim.x);
  const int t_end = (int)((long)(blockIdx.x + 1) * a.ntiles / gridDim.x);
  if (t_beg < t_end) issue(t_beg);
  for (int tile = t_beg; tile < t_end; ++tile) {
    commit();
    __syncthreads();
    if (tile + 1 < t_end) issue(tile + 1);
#pragma unroll
    for (int rr = 0; rr < TH / 4; ++rr) {
      const int row = wave + 4 * rr;
      bf16x8 ax[NCI];
#pragma unroll
      for (int i = 0; i < NCI; ++i) ax[i] = wm_frag<RBX>(ximg, row * WM_TW + 8 * g, i, lane);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        bf16x8 bd = {};
        if (boff[t] >= 0) bd = *reinterpret_cast<const bf16x8*>(dpl + boff[t] + row * WM_TW);
#pragma unroll
        for (int i = 0; i < NCI; ++i) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[i], bd, acc[i][t], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // fold the 4 waves' accumulators (LDS, two rounds), wave 0 stores the block's partial
  float* red = reinterpret_cast<float*>(smem);
  constexpr int NA = NCI * NT * 4;
  auto put = [&](int slot) {
#pragma unroll
    for (int i = 0; i < NCI; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(slot * NA + (i * NT + t) * 4 + j) * 64 + lane] = acc[i][t][j];
  };
  auto add = [&](int slot) {
#pragma unroll
    for (int i = 0; i < NCI; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][t][j] += red[(slot * NA + (i * NT + t) * 4 + j) * 64 + lane];
  };
  if (wave >= 2) put(wave - 2);
  __syncthreads();
  if (wave < 2) add(wave);
  __syncthreads();
  if (wave == 1) put(0);
  __syncthreads();
  if (wave == 0) {
    add(0);
    float* part = a.part + (long)blockIdx.x * 9 * a.cin * cout;
    const int ci_l = 4 * g;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = t * 16 + (lane & 15);
      if (n < 9 * cout) {
        const int tap = n / cout, co = n - tap * cout;
#pragma unroll
        for (int i = 0; i < NCI; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ci = c0 + i * 16 + ci_l + j;
            if (ci < a.cin) part[((long)tap * a.cin + ci) * cout + co] = acc[i][t][j];
          }
      }
    }
  }
  (void)COMAX;
}

template <int NCI, int NT, int TH>
constexpr int wgrad_taps_lds() {
  constexpr int RBX = NCI == 1 ? 32 : NCI == 2 ? 64 : 128;
  constexpr int COMAX = NT * 16 / 9;
  constexpr int MAIN = TH * WM_TW * RBX + 3 * COMAX * wt_drows<TH>() * WM_TW * 2;
  constexpr int RED = 2 * NCI * NT * 4 * 64 * 4;
  return MAIN > RED ? MAIN : RED;
}

// ---------------------------------------------------------------- narrow weight gradient, LDS-DMA stream (r05)
// The select convs' weight gradients (unet_simple.py:120-139 through train.py:288-304's minimize) read 39-315 MB of
// tower features each for a few GFLOP: a stream.  wgrad_taps_kernel stages one 4 x 32-pixel tile per block in
// registers and exposes its load latency every step (2.0 TB/s at 320^2, 0.4 TB/s at 40^2 on MI355X; 1.0 ms of the
// 4.9 ms step).  Here the X tiles and the f32 DY halo patches are DMA'd (buffer_load ... lds) into an S-slot LDS
// ring, S-1 tiles in flight per block and no staging registers, so two blocks per CU keep ~100 KB in flight.  Same
// GEMM as wgrad_taps_kernel (taps in N, B from the three pre-shifted bf16 DY planes, built from the landed f32 patch
// after the ring barrier), same tiles per block and the same MFMA order: the partials are bit-identical to it.
// The X image keeps wm_off's swizzle by permuting the SOURCE chunk of each LDS position (the DMA writes lane-linear).
// cout <= 16 (NT <= 9 column tiles); cin a multiple of 8, the block's 16 NCI channels inside one source.
template <int RB>
__device__ __forceinline__ void wm_src(int e, int& pe, int& j) {  // LDS chunk e of the X image -> (pixel, chunk)
  if constexpr (RB == 32) {
    const int r = e >> 1;
    pe = r ^ (((r >> 3) & 1) << 2);
    j = e & 1;
  } else if constexpr (RB == 64) {
    const int r = e >> 2, s = e & 3;
    pe = r;
    j = 2 * ((s >> 1) ^ ((r >> 3) & 1)) + (s & 1);
  } else {
    const int r = e >> 3, s = e & 7;
    pe = r;
    j = 2 * ((s >> 1) ^ ((r >> 1) & 1) ^ (((r >> 3) & 1) << 1)) + (s & 1);
  }
}

// one 4-byte-per-lane LDS-DMA (buffer_load_dword ... offen lds): lane l writes lds_dst + 4 l (see glds16)
__device__ __forceinline__ void glds4(__amdgpu_buffer_rsrc_t rsrc, uint32_t lds_dst, int voffset) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voffset), "s"(lds_dst), "s"(rsrc)
      : "memory");
}

template <int NCI, int NT, int TH_>
struct WtDma {
  static constexpr int TH = TH_, CIB = NCI * 16, RBX = NCI == 1 ? 32 : NCI == 2 ? 64 : 128;
  static constexpr int XPIX = TH * WM_TW, XCH = CIB / 8, NXC = XPIX * XCH, XPT = (NXC + 255) / 256;
  static constexpr int DR = TH + 2, COMAX = NT * 16 / 9, NDE = DR * WM_PW * COMAX, DPT = (NDE + 255) / 256;
  static constexpr int XS = XPT * 256 * 16, DS = DPT * 256 * 4, SLOT = XS + DS, NP = XPT + DPT;
  static constexpr int PLANES = 3 * COMAX * DR * WM_TW * 2;
  static constexpr int RED = 2 * NCI * NT * 4 * 64 * 4;
  template <int S>
  static constexpr int lds() { return S * SLOT + PLANES > RED ? S * SLOT + PLANES : RED; }
};

template <int NCI, int NT, int TH_, int S>
__global__ __launch_bounds__(256, 2) void wgrad_taps_dma_kernel(WgArgs a) {
  using C = WtDma<NCI, NT, TH_>;
  constexpr int TH = C::TH, RBX = C::RBX, XPT = C::XPT, DPT = C::DPT, DR = C::DR, NP = C::NP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c0 = blockIdx.y * C::CIB;
  const int cout = a.cout, ndy = DR * WM_PW * cout;
  uint16_t* dpl = reinterpret_cast<uint16_t*>(smem + S * C::SLOT);  // [3][cout][DR][32]
  const uint32_t lds0 = lds_addr(smem);

  f32x4 acc[NCI][NT];
#pragma unroll
  for (int i = 0; i < NCI; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4;
  int boff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = t * 16 + (lane & 15);
    if (n < 9 * cout) {
      const int tap = n / cout, co = n - tap * cout, kh = tap / 3, kw = tap - kh * 3;
      boff[t] = ((kw * cout + co) * DR + 2 - kh) * WM_TW + 8 * g;
    } else {
      boff[t] = -1;
    }
  }
  // this block's channel slice inside its source (the host checks it does not straddle two)
  const long xsrc = a.x_src_c > 0 ? (long)(c0 / a.x_src_c) * a.x_src_stride + c0 % a.x_src_c : (long)c0;
  const int t_beg = (int)((long)blockIdx.x * a.ntiles / gridDim.x);
  const int t_end = (int)((long)(blockIdx.x + 1) * a.ntiles / gridDim.x);
  const int nsteps = t_end - t_beg;
  // DMA of step j (tile t_beg + j) into slot j % S; steps past the end load out-of-range zeros, so every thread
  // issues exactly NP pieces per step and the counted waits stay uniform
  auto issue = [&](int j) __attribute__((always_inline)) {
    const bool real = j < nsteps;
    const int tile = t_beg + (real ? j : 0);
    const int tx = tile % a.tiles_w, t2 = tile / a.tiles_w;
    const int y0 = (t2 % a.tiles_h) * TH, n = t2 / a.tiles_h, x0 = tx * WM_TW;
    const uint16_t* Xn = a.x + (long)n * a.h * a.w * a.xcs + xsrc;
    const float* Dn = a.dy + (long)n * a.h * a.w * a.dcs;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(const_cast<uint16_t*>(Xn)), 0, 0x7ffffff0, 0x00020000);
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(const_cast<float*>(Dn)), 0, 0x7ffffff0, 0x00020000);
    const uint32_t slot = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((j % S) * C::SLOT));
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      int pe, jj;
      wm_src<RBX>(e, pe, jj);
      const int gy = y0 + pe / WM_TW, gx = x0 + pe % WM_TW, c = c0 + jj * 8;
      const bool ok = real & (e < C::NXC) & (gy < a.h) & (gx < a.w) & (c < a.cin);
      glds16(xrs, slot + (uint32_t)((k * 256 + wave * 64) * 16), ok ? ((gy * a.w + gx) * a.xcs + jj * 8) * 2 : OOB);
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {  // the halo patch, (pixel, co) elements in memory order
      const int e = tid + k * 256;
      const int pe = e / cout, co = e - pe * cout;
      const int gy = y0 - 1 + pe / WM_PW, gx = x0 - 1 + pe % WM_PW;
      const bool ok = real & (e < ndy) & ((unsigned)gy < (unsigned)a.h) & ((unsigned)gx < (unsigned)a.w);
      glds4(drs, slot + (uint32_t)(C::XS + (k * 256 + wave * 64) * 4), ok ? ((gy * a.w + gx) * a.dcs + co) * 4 : OOB);
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing older in the DMA counts
#pragma unroll
  for (int j = 0; j < S - 1; ++j) issue(j);
  for (int j = 0; j < nsteps; ++j) {
    // step j landed (this wave's own DMAs; the S-2 younger steps may fly), then everyone's, and every wave's reads
    // of step j-1 (slot (j-1) % S and the planes) retired
    wait_vm((S - 2) * NP);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(j + S - 1);  // into slot (j - 1) % S
    const char* ximg = smem + (j % S) * C::SLOT;
    const float* dys = reinterpret_cast<const float*>(ximg + C::XS);
    for (int e = tid; e < ndy; e += 256) {  // the three pre-shifted bf16 DY planes (wgrad_taps_kernel's commit)
      const int pe = e / cout, co = e - pe * cout;
      const int r = pe / WM_PW, pc = pe % WM_PW;
      const uint16_t v = f2bf(dys[e]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int jx = pc - 2 + kw;
        if (jx >= 0 && jx < WM_TW) dpl[((kw * cout + co) * DR + r) * WM_TW + jx] = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < TH / 4; ++rr) {  // K-steps: tile rows wave, wave + 4 (wgrad_taps_kernel's order)
      const int row = wave + 4 * rr;
      bf16x8 ax[NCI];
#pragma unroll
      for (int i = 0; i < NCI; ++i) ax[i] = wm_frag<RBX>(ximg, row * WM_TW + 8 * g, i, lane);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        bf16x8 bd = {};
        if (boff[t] >= 0) bd = *reinterpret_cast<const bf16x8*>(dpl + boff[t] + row * WM_TW);
#pragma unroll
        for (int i = 0; i < NCI; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[i], bd, acc[i][t], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // ring drained: LDS reused

  float* red = reinterpret_cast<float*>(smem);
  constexpr int NA = NCI * NT * 4;
  auto put = [&](int sl) {
#pragma unroll
    for (int i = 0; i < NCI; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[(sl * NA + (i * NT + t) * 4 + q) * 64 + lane] = acc[i][t][q];
  };
  auto add = [&](int sl) {
#pragma unroll
    for (int i = 0; i < NCI; ++i)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][t][q] += red[(sl * NA + (i * NT + t) * 4 + q) * 64 + lane];
  };
  if (wave >= 2) put(wave - 2);
  __syncthreads();
  if (wave < 2) add(wave);
  __syncthreads();
  if (wave == 1) put(0);
  __syncthreads();
  if (wave == 0) {
    add(0);
    float* part = a.part + (long)blockIdx.x * 9 * a.cin * cout;
    const int ci_l = 4 * g;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = t * 16 + (lane & 15);
      if (n < 9 * cout) {
        const int tap = n / cout, co = n - tap * cout;
#pragma unroll
        for (int i = 0; i < NCI; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ci = c0 + i * 16 + ci_l + q;
            if (ci < a.cin) part[((long)tap * a.cin + ci) * cout + co] = acc[i][t][q];
          }
      }
    }
  }
}

// ---------------------------------------------------------------- wide conv weight gradient (UNetImage training)
// train.py's training_procedure (train.py:37-109) back-propagates through every conv of unet.UNetImage
// (unet.py:86-148): cin 6 ... 1024, cout 64 ... 512.  dW_t[ci][co] = sum_p X[p + off_t][ci] * DY[p][co] as 9 GEMMs
// with K = the pixels, v_mfma_f32_16x16x32_bf16 (A = X^T: 16 input channels x 32 pixels, B = DY: 32 pixels x 16
// output channels, f32 accumulation), both operands read k-major from their natural NHWC LDS images with
// ds_read_b64_tr_b16 (wm_frag), like wgrad_mfma_kernel.  The narrow kernel above runs every output channel in one
// block and splits its K-steps over the waves (cout <= 48); here a block owns a 64 x 64 (ci x co) tile of all 9
// taps and the 4 waves split the OUTPUT: wave w holds ci 16w..16w+15 x all 64 co x 9 taps (144 f32 accumulators)
// and walks every pixel row of the tile, so no cross-wave reduction is needed.  Per 32-pixel row a wave reads 4 DY
// fragments (reused by the 9 taps) and 9 X fragments (each reused by the 4 co pieces): 13 fragment reads per 36
// MFMAs, i.e. ~370 B of LDS reads per MFMA — inside the CU's LDS bandwidth at the matrix pipes' rate (a 32 x 32
// split read 20 fragments per 36 MFMAs, ~570 B, above it).
// Grid: gx K-split blocks (contiguous tile ranges, one partial filter gradient each, summed in fixed order by
// wgrad_reduce_kernel: deterministic) x the 64-channel blocks of cin and cout, as ONE dimension whose order is
// XCD-aware: the blocks that share a pixel range (every channel block of it) are dispatched to the same XCD, so
// its X patch and DY tile are fetched from HBM once per XCD and re-read from that XCD's L2.
// DY is bf16 (the bf16 gradient copy the relu / BN backward writes for the data-gradient conv) or f32 (rounded
// to bf16 when staged); X is the bf16 conv input, channels past cin (UNetImage's 6-channel conv1_1) read as 0.
struct WwArgs {
  const uint16_t* x;  // bf16 input view base (pixel 0, coff applied)
  int n, h, w, cin, xcs;
  const void* dy;     // bf16 / f32 output-gradient view base (coff applied)
  int cout, dcs;
  float* part;        // [gx][9][cin][cout]
  int tiles_h, tiles_w;
  long ntiles;
  int gx, ncin, ncout;
  int dbuf;           // PIPE: two LDS image buffers, tile t in buffer t & 1 (one barrier per tile)
};

constexpr int WW_TH = 4;
constexpr int WW_TARGET_BLOCKS = 512;  // ~2 resident blocks per CU: one round; the partials stay <= 75 MB

// Pipelined fragment reads (PIPE, r05).  The plain loop below left hipcc a per-tap chain of ~12 VALU for the
// swizzled row address, two ds_read_b64_tr_b16 and an lgkmcnt(0) wait in front of every 4 MFMAs, so each tap paid
// the whole LDS latency.  The row loop is unrolled and every fragment address is a per-lane base register plus an
// immediate: wm_off<128>(C + u, c) = 128 C + [128 u + 32 (c ^ x((C + u) mod 16))] for the lane's u = 8g + q, so 16
// bases per X piece (C mod 16) and 2 per DY piece cover every (row, tap); the next tap's X fragment (and, over the
// last two taps of a row, the next row's DY fragments and first X fragment) is read while the current tap's MFMAs
// run.  Each accumulator sees the same MFMAs in the same order: bit-identical to the plain loop.
template <int RB>
__device__ __forceinline__ int wm_base(int u, int c, int p) {  // wm_off<RB>(u, c) + 8p, RB = 128
  static_assert(RB == 128, "the 128-byte image rows of wgrad_wide_kernel");
  return 128 * u + 32 * (c ^ ((u >> 1) & 1) ^ (((u >> 3) & 1) << 1)) + 8 * p;
}

template <int C>  // fragment whose k rows are image rows C + u (lo) and C + 4 + u (hi), bases per C mod 16
__device__ __forceinline__ bf16x8 wm_frag_b(const char* img, const int (&b)[16]) {
  typedef __attribute__((address_space(3))) v4s* lp;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + 128 * C + b[C & 15]));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(img + 128 * (C + 4) + b[(C + 4) & 15]));
  v4s v[2] = {lo, hi};
  return __builtin_bit_cast(bf16x8, v);
}

// PIPE: one block per CU (the unrolled rows, the bases and the next tile's staging registers need > 256 VGPRs)
// CS (cin <= 16, plain loop): the 4 waves split the OUTPUT channels instead — wave w takes ci 0..15 x co 16w..16w+15
// x 9 taps — so UNetImage's 6-channel conv1_1 does not leave 3 of 4 waves multiplying zero input channels.  Each
// accumulator (ci piece 0, co piece w) sees the same MFMAs on the same fragments in the same order as wave 0's
// accumulator o = w in the default split: bit-identical.
template <int TH, bool DYF32, bool PIPE = true, bool CS = false>
__global__ __launch_bounds__(256, PIPE ? 1 : 2) void wgrad_wide_kernel(WwArgs a) {  // A/B (scripts/build_variant.sh):
                                                                           // (256,2) 2.58 ms vs (256,1) 2.87 ms
  constexpr int XPIX = wm_ppix<TH>(), DPIX = TH * WM_TW;
  constexpr int XBYTES = wm_prows<TH>() * 128;
  constexpr int NXC = XPIX * 8, NDC = DPIX * 8;                 // 16-byte chunks (8 channels) of each image
  constexpr int XPT = (NXC + 255) / 256, DPT = (NDC + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ximg = smem;
  char* dimg = smem + XBYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = the 16-channel piece of ci this wave owns
  const int nb = gridDim.x, lin = blockIdx.x;
  // consecutive work ids on one XCD (workgroups are dealt to the 8 XCDs round-robin)
  const int wid = (nb % 8 == 0) ? (lin % 8) * (nb / 8) + lin / 8 : lin;
  const int nch = a.ncin * a.ncout;
  const int kx = wid / nch, cb = wid - kx * nch;
  const int c0 = (cb % a.ncin) * 64, o0 = (cb / a.ncin) * 64;

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int o = 0; o < 4; ++o) acc[t][o] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 xb[XPT];
  uint4 db[DPT];
  float4 df[DYF32 ? DPT : 1][2];
  auto issue = [&](int tile) {
    const int tx = tile % a.tiles_w;
    const int t2 = tile / a.tiles_w;
    const int y0 = (t2 % a.tiles_h) * TH, n = t2 / a.tiles_h, x0 = tx * WM_TW;
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      xb[k] = make_uint4(0, 0, 0, 0);
      if (NXC % 256 == 0 || e < NXC) {
        const int pe = e >> 3, j = e & 7;
        const int gy = y0 - 1 + pe / WM_PW, gx = x0 - 1 + pe % WM_PW;
        const int c = c0 + j * 8;
        if ((unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w && c < a.cin)
          xb[k] = *reinterpret_cast<const uint4*>(a.x + (((long)n * a.h + gy) * a.w + gx) * a.xcs + c);
      }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = tid + k * 256;
      const int pe = e >> 3, j = e & 7;
      const int gy = y0 + pe / WM_TW, gx = x0 + pe % WM_TW;
      const bool in = (NDC % 256 == 0 || e < NDC) && (unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w;
      const long off = (((long)n * a.h + gy) * a.w + gx) * a.dcs + o0 + j * 8;
      if constexpr (DYF32) {
        df[k][0] = df[k][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (in) {
          const float* src = reinterpret_cast<const float*>(a.dy) + off;
          df[k][0] = *reinterpret_cast<const float4*>(src);
          df[k][1] = *reinterpret_cast<const float4*>(src + 4);
        }
      } else {
        db[k] = make_uint4(0, 0, 0, 0);
        if (in) db[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(a.dy) + off);
      }
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int e = tid + k * 256;
      if (NXC % 256 == 0 || e < NXC) {
        const int pe = e >> 3, j = e & 7;
        uint4 v = xb[k];
        const int c = c0 + j * 8;
        if (c + 8 > a.cin) {  // a chunk straddling cin: zero the channels past it
          uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (c + 2 * i >= a.cin) w4[i] = 0u;
            else if (c + 2 * i + 1 >= a.cin) w4[i] &= 0xffffu;
          }
          v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        *reinterpret_cast<uint4*>(ximg + wm_off<128>(pe, j >> 1) + (j & 1) * 16) = v;
      }
    }
#pragma unroll
    for (int k = 0; k < DPT; ++k) {
      const int e = tid + k * 256;
      if (NDC % 256 == 0 || e < NDC) {
        const int pe = e >> 3, j = e & 7;
        uint4 v;
        if constexpr (DYF32) {
          const float f[8] = {df[k][0].x, df[k][0].y, df[k][0].z, df[k][0].w,
                              df[k][1].x, df[k][1].y, df[k][1].z, df[k][1].w};
          v = Chunk<uint16_t>::pack(f);
        } else {
          v = db[k];
        }
        *reinterpret_cast<uint4*>(dimg + wm_off<128>(pe, j >> 1) + (j & 1) * 16) = v;
      }
    }
  };

  const int g = lane >> 4;
  const int t_beg = (int)((long)kx * a.ntiles / a.gx);
  const int t_end = (int)((long)(kx + 1) * a.ntiles / a.gx);
  if constexpr (PIPE) {
    // per-lane fragment bases: X piece `wave` for every C mod 16, DY piece o for C mod 16 in {0, 4} (C = 32 row)
    const int u = 8 * g + ((lane >> 2) & 3), p = lane & 3;
    int bx[16], bdy[4][16];
#pragma unroll
    for (int k = 0; k < 16; ++k) bx[k] = wm_base<128>(k + u, wave, p) - 128 * k;
#pragma unroll
    for (int o = 0; o < 4; ++o)
#pragma unroll
      for (int k = 0; k < 16; ++k) bdy[o][k] = (k == 0 || k == 4) ? wm_base<128>(k + u, o, p) - 128 * k : 0;
    // dbuf: tile t's images go to buffer t & 1.  Buffer (t + 1) & 1 was last read by tile t - 1's MFMAs, which every
    // wave finished before the barrier after tile t's commit, so the trailing barrier is not needed: a wave that is
    // done with tile t commits tile t + 1 while the others still compute.
    const int bstride = a.dbuf ? XBYTES + DPIX * 128 : 0;
    if (t_beg < t_end) issue(t_beg);
    for (int tile = t_beg; tile < t_end; ++tile) {
      ximg = smem + ((tile - t_beg) & 1) * bstride;
      dimg = ximg + XBYTES;
      commit();
      __syncthreads();
      if (tile + 1 < t_end) issue(tile + 1);
      bf16x8 bd[2][4], ax[2];
#pragma unroll
      for (int o = 0; o < 4; ++o) bd[0][o] = wm_frag_b<0>(dimg, bdy[o]);
      ax[0] = wm_frag_b<0>(ximg, bx);
      static_for<0, TH>([&](auto rc) __attribute__((always_inline)) {
        constexpr int row = decltype(rc)::value, cb = row & 1;
        static_for<0, 9>([&](auto tc) __attribute__((always_inline)) {
          constexpr int t = decltype(tc)::value;
          constexpr int gi = row * 9 + t;  // X fragments alternate between two slots over the tile's rows x taps
          if constexpr (t + 1 < 9) {
            constexpr int C = (row + (t + 1) / 3) * WM_PW + (t + 1) % 3;
            ax[(gi + 1) & 1] = wm_frag_b<C>(ximg, bx);
          } else if constexpr (row + 1 < TH) {
            constexpr int C = (row + 1) * WM_PW;  // the next row's tap 0
            ax[(gi + 1) & 1] = wm_frag_b<C>(ximg, bx);
          }
          if constexpr (t == 7 && row + 1 < TH) {
#pragma unroll
            for (int o = 0; o < 4; ++o) bd[cb ^ 1][o] = wm_frag_b<(row + 1) * WM_TW>(dimg, bdy[o]);
          }
#pragma unroll
          for (int o = 0; o < 4; ++o)
            acc[t][o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[gi & 1], bd[cb][o], acc[t][o], 0, 0, 0);
          // the reads issued above go out ahead of this tap's MFMAs
          if constexpr (t == 7 && row + 1 < TH) __builtin_amdgcn_sched_group_barrier(0x100, 10, 0);
          else if constexpr (t + 1 < 9 || row + 1 < TH) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        });
      });
      if (!a.dbuf) __syncthreads();
    }
  } else {
  if (t_beg < t_end) issue(t_beg);
  for (int tile = t_beg; tile < t_end; ++tile) {
    commit();
    __syncthreads();
    if (tile + 1 < t_end) issue(tile + 1);
#pragma unroll 1
    for (int row = 0; row < TH; ++row) {
      if constexpr (CS) {
        const bf16x8 bdw = wm_frag<128>(dimg, row * WM_TW + 8 * g, wave, lane);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int r0 = (row + t / 3) * WM_PW + t % 3 + 8 * g;
          const bf16x8 ax = wm_frag<128>(ximg, r0, 0, lane);
          acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax, bdw, acc[t][0], 0, 0, 0);
        }
        continue;
      }
      bf16x8 bd[4];
#pragma unroll
      for (int o = 0; o < 4; ++o) bd[o] = wm_frag<128>(dimg, row * WM_TW + 8 * g, o, lane);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int r0 = (row + t / 3) * WM_PW + t % 3 + 8 * g;
        const bf16x8 ax = wm_frag<128>(ximg, r0, wave, lane);
#pragma unroll
        for (int o = 0; o < 4; ++o) acc[t][o] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax, bd[o], acc[t][o], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  }

  // this block's partial of its 64 x 64 x 9 tile (lanes: co = lane & 15, ci = 4 * (lane >> 4) + j)
  float* part = a.part + (long)kx * 9 * a.cin * a.cout;
  const int co_l = lane & 15, ci_l = 4 * g;
  if constexpr (CS) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int co = o0 + 16 * wave + co_l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ci = c0 + ci_l + j;
        if (ci < a.cin) part[((long)t * a.cin + ci) * a.cout + co] = acc[t][0][j];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int co = o0 + 16 * o + co_l;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ci = c0 + 16 * wave + ci_l + j;
        if (ci < a.cin) part[((long)t * a.cin + ci) * a.cout + co] = acc[t][o][j];
      }
    }
}

template <int TH>
constexpr int wgrad_wide_lds() { return wm_prows<TH>() * 128 + TH * WM_TW * 128; }

// The exact-f32 wide weight gradient of the fp32 (parity) training path: a plain FMA GEMM per tap.  Block = 256
// threads on one (tap, 32 input channels, 64 output channels) tile; per 32-pixel K chunk the shifted X rows and
// the DY rows are staged in LDS, each thread accumulates 2 ci x 4 co in f32 over its block's contiguous pixel
// range (fixed order), and wgrad_reduce_kernel sums the gx partials in fixed order: deterministic.
struct WfArgs {
  const float* x;
  int n, h, w, cin, xcs;
  const float* dy;
  int cout, dcs;
  float* part;  // [gx][9][cin][cout]
  long npix;
  int gx, ncin, ncout;
};

__global__ __launch_bounds__(256) void wgrad_wide_f32_kernel(WfArgs a) {
  __shared__ float xs[32][33];
  __shared__ float ds[32][65];
  const int tid = threadIdx.x;
  int b = blockIdx.y;
  const int t = b % 9;
  b /= 9;
  const int c0 = (b % a.ncin) * 32, o0 = (b / a.ncin) * 64;
  const int kh = t / 3 - 1, kw = t % 3 - 1;
  const int kx = blockIdx.x;
  const long p_beg = kx * a.npix / a.gx, p_end = (kx + 1) * a.npix / a.gx;
  const int tc = tid / 16, to = tid % 16;  // thread: ci 2tc, 2tc+1; co 4to .. 4to+3
  float acc[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (long p0 = p_beg; p0 < p_end; p0 += 32) {
    // stage X[p + off_t][c0 .. c0+31] and DY[p][o0 .. o0+63] for 32 pixels
    for (int e = tid; e < 32 * 32; e += 256) {
      const int pk = e / 32, c = e % 32;
      const long p = p0 + pk;
      float v = 0.f;
      if (p < p_end && c0 + c < a.cin) {
        const int xx = (int)(p % a.w);
        const long r = p / a.w;
        const int yy = (int)(r % a.h), nn = (int)(r / a.h);
        const int gy = yy + kh, gx = xx + kw;
        if ((unsigned)gy < (unsigned)a.h && (unsigned)gx < (unsigned)a.w)
          v = a.x[(((long)nn * a.h + gy) * a.w + gx) * a.xcs + c0 + c];
      }
      xs[pk][c] = v;
    }
    for (int e = tid; e < 32 * 64; e += 256) {
      const int pk = e / 64, c = e % 64;
      const long p = p0 + pk;
      ds[pk][c] = (p < p_end && o0 + c < a.cout) ? a.dy[p * a.dcs + o0 + c] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < 32; ++k) {
      const float x0 = xs[k][2 * tc], x1 = xs[k][2 * tc + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = ds[k][4 * to + j];
        acc[0][j] = fmaf(x0, d, acc[0][j]);
        acc[1][j] = fmaf(x1, d, acc[1][j]);
      }
    }
    __syncthreads();
  }
  float* part = a.part + (long)kx * 9 * a.cin * a.cout;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ci = c0 + 2 * tc + i;
    if (ci >= a.cin) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = o0 + 4 * to + j;
      if (co < a.cout) part[((long)t * a.cin + ci) * a.cout + co] = acc[i][j];
    }
  }
}

// HWIO [3][3][cin][cout] -> the dgrad filter [3][3][cout][cin], spatially flipped
__global__ void flip_weights_kernel(const float* w, int cin, int cout, float* wt) {
  const long total = 9L * cin * cout;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % cout);
    const long r = i / cout;
    const int ci = (int)(r % cin);
    const int tap = (int)(r / cin);
    wt[((long)(8 - tap) * cout + co) * cin + ci] = w[i];
  }
}

// ---------------------------------------------------------------- Adam (tf.train.AdamOptimizer, train.py:302-304)
__global__ void adam_kernel(float* var, float* m, float* v, const float* grad, long n, float lr_t, float beta1,
                            float beta2, float eps, float grad_scale) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
#pragma clang fp contract(off)
    const float g = grad[i] * grad_scale;
    const float mi = m[i] + (g - m[i]) * (1.f - beta1);
    const float vi = v[i] + (g * g - v[i]) * (1.f - beta2);
    m[i] = mi;
    v[i] = vi;
    var[i] = var[i] - (mi * lr_t) / (sqrtf(vi) + eps);
  }
}

// dw[i] += sum over the gx block rows of the partials (fixed order: deterministic).  A block owns COLS columns;
// its 256 / COLS row groups stride the rows (independent loads in flight), then fold through LDS.  64 columns for
// wide filters; 16 for narrow ones (S = 9 cin cout under 32k: 64-column blocks left a few hundred blocks each
// walking hundreds of rows).  256-thread blocks: a 1024-thread form waited for whole free CUs behind the
// side-stream weight gradients.
template <int COLS>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* part, int rows, long S, float* dw) {
  constexpr int RG = 256 / COLS;
  __shared__ float sh[RG][COLS];
  const int col = threadIdx.x % COLS, rg = threadIdx.x / COLS;
  const long i = (long)blockIdx.x * COLS + col;
  float s = 0.f;
  if (i < S) {
#pragma unroll 8
    for (int b = rg; b < rows; b += RG) s += part[(long)b * S + i];
  }
  sh[rg][col] = s;
  __syncthreads();
  if (rg == 0 && i < S) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < RG; ++g) t += sh[g][col];
    dw[i] += t;
  }
}

// The same fixed-order sum, 4 columns per lane (16-byte loads) and 16 row groups per block (r06): the 64-column form
// kept one 256-byte run per row group in flight and read the partials at ~0.8 TB/s (UNetImage step: 18 reductions,
// 45 us each, profiles/r05_train_image_kernel_stats.csv).  Each column's rows are summed in the order b = rg, rg + 16,
// ... per group, then the 16 groups in order: deterministic (another order than wgrad_reduce_kernel's).
__global__ __launch_bounds__(256) void wgrad_reduce4_kernel(const float* __restrict__ part, int rows, long S,
                                                            float* __restrict__ dw) {
  constexpr int RG = 16, CQ = 256 / RG;
  __shared__ float4 sh[RG][CQ];
  const int cq = threadIdx.x % CQ, rg = threadIdx.x / CQ;
  const long i = ((long)blockIdx.x * CQ + cq) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < S) {
#pragma unroll 4
    for (int b = rg; b < rows; b += RG) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long)b * S + i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  sh[rg][cq] = s;
  __syncthreads();
  if (rg == 0 && i < S) {
    float4 t = sh[0][cq];
#pragma unroll
    for (int g = 1; g < RG; ++g) {
      const float4 v = sh[g][cq];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    float4 d = *reinterpret_cast<float4*>(dw + i);
    d.x += t.x; d.y += t.y; d.z += t.z; d.w += t.w;
    *reinterpret_cast<float4*>(dw + i) = d;
  }
}

static long g_wgrad_reduce4 = 1;  // vm_set_option "wgrad_reduce4": 0 = the r05 scalar-column reduction (A/B)

static void launch_wgrad_reduce(const float* part, int rows, long S, float* dw, hipStream_t st) {
  if (g_wgrad_reduce4 && S % 4 == 0 && reinterpret_cast<uintptr_t>(dw) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(part) % 16 == 0 && rows > 1) {
    hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3((unsigned)((S / 4 + 15) / 16)), dim3(256), 0, st, part, rows, S, dw);
    return;
  }
  if (S >= 64L * 512)
    hipLaunchKernelGGL(wgrad_reduce_kernel<64>, dim3((unsigned)((S + 63) / 64)), dim3(256), 0, st, part, rows, S, dw);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<16>, dim3((unsigned)((S + 15) / 16)), dim3(256), 0, st, part, rows, S, dw);
}

constexpr size_t WG_WS_CAP = 64ull << 20;  // workspace bytes

// pixel-tile blocks per channel chunk: ~1024 blocks in all (4 per CU), fewer when the partial rows would pass
// WG_WS_CAP
static long wgrad_rows(int n, int h, int w, int cin, int cout, int cc) {
  const long ntiles = (long)n * ((h + WG_TH - 1) / WG_TH) * ((w + WG_TW - 1) / WG_TW);
  const int ncc = (cin + cc - 1) / cc;
  long gx = (1024 + ncc - 1) / ncc;
  const long cap = (long)(WG_WS_CAP / (9ull * cin * cout * sizeof(float)));
  if (gx > cap) gx = cap;
  if (gx > ntiles) gx = ntiles;
  return gx < 1 ? 1 : gx;
}

static int wgrad_cc(int cout) { return (cout + 3) / 4 <= 2 ? 64 : 32; }

template <int CC, int CO4, typename T, bool XV, bool DV>
static void launch_wgrad_t(const V& xv, const V& dy, float* dw, float* ws, hipStream_t st) {
  const int tiles_h = (xv.h + WG_TH - 1) / WG_TH, tiles_w = (xv.w + WG_TW - 1) / WG_TW;
  const long ntiles = (long)xv.n * tiles_h * tiles_w;
  const int ncc = (xv.c + CC - 1) / CC;
  const long gx = wgrad_rows(xv.n, xv.h, xv.w, xv.c, dy.c, CC);
  hipLaunchKernelGGL((wgrad_kernel<CC, CO4, T, XV, DV>), dim3((unsigned)gx, ncc), dim3(WG_NT), 0, st, xv, dy, ws,
                     tiles_h, tiles_w, ntiles);
  const long S = 9L * xv.c * dy.c;
  launch_wgrad_reduce(ws, (int)gx, S, dw, st);
}

static bool vec_ok(const V& v, int ve) {
  return reinterpret_cast<uintptr_t>(v.p) % 16 == 0 && v.c % ve == 0 && v.coff % ve == 0 && v.cs % ve == 0;
}

// x may also be read in 16-byte vectors past its last channel when the row stride holds them (the padded
// concat / input buffers: up1n[..., :30] of a 32-wide row, in9[..., :9] of a 16-wide row); the extra lanes are zeroed
static bool xvec_ok(const V& v, int ve) {
  if (v.sc > 0)  // split sources: a vector never straddles two sources
    return reinterpret_cast<uintptr_t>(v.p) % 16 == 0 && v.coff % ve == 0 && v.cs % ve == 0 && v.sc % ve == 0 &&
           v.ss % ve == 0 && v.coff + v.sc <= v.cs;
  return reinterpret_cast<uintptr_t>(v.p) % 16 == 0 && v.coff % ve == 0 && v.cs % ve == 0 &&
         v.coff + (v.c + ve - 1) / ve * ve <= v.cs;
}

template <int CC, int CO4>
static void launch_wgrad(const V& xv, const V& dy, float* dw, float* ws, hipStream_t st) {
  const bool dv = vec_ok(dy, 4);
  if (xv.dt == VM_BF16 && xvec_ok(xv, 8)) {
    if (dv) launch_wgrad_t<CC, CO4, uint16_t, true, true>(xv, dy, dw, ws, st);
    else launch_wgrad_t<CC, CO4, uint16_t, true, false>(xv, dy, dw, ws, st);
  } else if (xv.dt == VM_F32 && xvec_ok(xv, 4)) {
    if (dv) launch_wgrad_t<CC, CO4, float, true, true>(xv, dy, dw, ws, st);
    else launch_wgrad_t<CC, CO4, float, true, false>(xv, dy, dw, ws, st);
  } else {
    if (dv) launch_wgrad_t<CC, CO4, float, false, true>(xv, dy, dw, ws, st);
    else launch_wgrad_t<CC, CO4, float, false, false>(xv, dy, dw, ws, st);
  }
}

struct WmCfg {
  int nci, nco;
  bool sx;
  int nt;  // > 0: wgrad_taps_kernel with NT = nt column tiles (cout <= 8)
};

// operand tiling of the MFMA weight gradient: cout -> NCO 16-wide fragments, the input-channel fragments per block
// as wide as 144 accumulator registers allow; the operand with fewer fragments per K-step carries the tap shift
// blocks per channel chunk of the MFMA weight gradient: ~1024 in all, at most one per tile (tiles of the smallest
// variant, so the workspace query, which cannot know the variant, is an upper bound), capped by the workspace
static long wgrad_mfma_rows(const WgArgs& a, int cib) {
  return wgrad_rows(a.n, a.h, a.w, a.cin, a.cout, cib) < a.ntiles ? wgrad_rows(a.n, a.h, a.w, a.cin, a.cout, cib)
                                                                  : (a.ntiles < 1 ? 1 : a.ntiles);
}

// (at most 72-108 accumulator registers: the 144-register tilings spill next to the staging registers)
// cout <= 8: the taps-in-N kernel, 64 input channels per block (32 for NT 4-5: 80 accumulator registers at most)
static WmCfg wgrad_mfma_cfg(int cin, int cout) {
  WmCfg c;
  c.nco = cout <= 16 ? 1 : cout <= 32 ? 2 : 3;
  c.nci = (c.nco == 1 && cin > 16) ? 2 : 1;
  c.sx = c.nco >= c.nci;
  c.nt = cout <= 8 ? (9 * cout + 15) / 16 : 0;
  if (c.nt) c.nci = cin <= 16 ? 1 : cin <= 32 || c.nt > 3 ? 2 : 4;
  return c;
}

// one round of blocks: the ~1024-block target (the workspace bound) cut to what is resident at once (160-VGPR
// variants: 3 blocks per CU), so no block waits for a second round (measured 2 x 72 us per select wgrad)
static int launch_wgrad_grid(const void* kern, int lds, int th, int cib, int& attr_dev, int& resident, WgArgs& a,
                             float* dw, hipStream_t st, void (*launch)(dim3, int, hipStream_t, const WgArgs&)) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (attr_dev != dev) {
    hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    int per_cu = 0, n_cu = 0;
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return fail(VM_EHIP, "wgrad_mfma setup: %s", hipGetErrorString(e));
    resident = per_cu * n_cu;
    attr_dev = dev;
  }
  a.tiles_h = (a.h + th - 1) / th;
  a.tiles_w = (a.w + WM_TW - 1) / WM_TW;
  a.ntiles = (long)a.n * a.tiles_h * a.tiles_w;
  if (a.ntiles > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv_wgrad: too many pixel tiles");
  const int ncc = (a.cin + cib - 1) / cib;
  long gx = wgrad_mfma_rows(a, cib);
  if (resident >= ncc && gx * ncc > resident) gx = resident / ncc;
  launch(dim3((unsigned)gx, ncc), lds, st, a);
  const long S = 9L * a.cin * a.cout;
  launch_wgrad_reduce(a.part, (int)gx, S, dw, st);
  return VM_OK;
}

static long g_bn_vec = 1;  // vm_set_option "bn_vec": 0 = the per-channel BN backward forms (A/B)
static long g_resize_bwd_2x = 1;  // vm_set_option "resize_bwd_2x": 0 = the windowed-search kernels for 2x too (A/B)
static long g_relu_bias_vec = 1;  // vm_set_option "relu_bias_vec": 0 = the per-element relu / bias backward (A/B)
static long g_relu_bias_iters = 8;  // vm_set_option "relu_bias_iters": pixel iterations per thread of the 8-channel
                                    // form's grid (0 = bn_blocks' rule)
static long g_wgrad_mfma_pipe = 1;  // vm_set_option "wgrad_mfma_pipe": 0 = wgrad_mfma_kernel's plain loop (A/B)
template <int NCI, int NCO, bool SX, int TH, bool PIPE>
static int launch_wgrad_mfma_p(WgArgs& a, float* dw, hipStream_t st) {
  static int attr_dev = -1, resident = 0;  // blocks of this variant resident on the whole chip at once
  return launch_wgrad_grid(reinterpret_cast<const void*>(&wgrad_mfma_kernel<NCI, NCO, SX, TH, PIPE>),
                           wgrad_mfma_lds<NCI, NCO, SX, TH>(), TH, NCI * 16, attr_dev, resident, a, dw, st,
                           [](dim3 g, int lds, hipStream_t s, const WgArgs& x) {
                             hipLaunchKernelGGL((wgrad_mfma_kernel<NCI, NCO, SX, TH, PIPE>), g, dim3(256), lds, s, x);
                           });
}
template <int NCI, int NCO, bool SX, int TH>
static int launch_wgrad_mfma_t(WgArgs& a, float* dw, hipStream_t st) {
  return g_wgrad_mfma_pipe ? launch_wgrad_mfma_p<NCI, NCO, SX, TH, true>(a, dw, st)
                           : launch_wgrad_mfma_p<NCI, NCO, SX, TH, false>(a, dw, st);
}

template <int NCI, int NT, int TH>
static int launch_wgrad_taps_t(WgArgs& a, float* dw, hipStream_t st) {
  static int attr_dev = -1, resident = 0;
  return launch_wgrad_grid(reinterpret_cast<const void*>(&wgrad_taps_kernel<NCI, NT, TH>),
                           wgrad_taps_lds<NCI, NT, TH>(), TH, NCI * 16, attr_dev, resident, a, dw, st,
                           [](dim3 g, int lds, hipStream_t s, const WgArgs& x) {
                             hipLaunchKernelGGL((wgrad_taps_kernel<NCI, NT, TH>), g, dim3(256), lds, s, x);
                           });
}

static long g_wgrad_variant = 0;  // A/B knob (vm_set_option "wgrad_variant"): 0/1 4-row tiles, 2 8-row tiles
static long g_wgrad_taps = 1;     // vm_set_option "wgrad_taps": 0 sends cout <= 8 to wgrad_mfma_kernel (A/B)
// vm_set_option "wgrad_dma": 1 = the LDS-DMA narrow kernel.  Off: measured at the config-5 select shapes with L2 /
// MALL flushed between calls (tools/selectwgrad_bench.py, MI355X) it streams x no faster than the register-staged
// kernels (select1 136 vs 128 us, 2.3-2.5 TB/s; select4 150 vs 42 us: its f32 DY patch outweighs the 40^2 X tile)
static long g_wgrad_dma = 0;

// the LDS-DMA narrow weight gradient: cout <= 16, 8-channel chunks, the block's channels inside one source, 32-bit
// byte offsets inside one image
static bool wgrad_dma_ok(const WgArgs& a, int cib) {
  return g_wgrad_dma && a.cout >= 1 && a.cout <= 16 && a.cin % 8 == 0 && a.xcs % 8 == 0 &&
         reinterpret_cast<uintptr_t>(a.x) % 16 == 0 && (a.x_src_c <= 0 || (a.x_src_c % cib == 0 && a.x_src_stride % 8 == 0)) &&
         (long)a.h * a.w * a.xcs * 2 < 0x7ff00000L && (long)a.h * a.w * a.dcs * 4 < 0x7ff00000L;
}

static long g_wgrad_wide_pipe = 1;  // vm_set_option "wgrad_wide_pipe": 0 = the plain-loop kernel at 2 blocks per CU (A/B)
static long g_wgrad_wide_cs = 1;  // vm_set_option "wgrad_wide_cs": 0 = the input-channel wave split for cin <= 16 too
static long g_wgrad_wide_dbuf = 1;  // vm_set_option "wgrad_wide_dbuf": 0 = one LDS image buffer, two barriers per tile
static long g_wgrad_wide_target = 0;  // vm_set_option "wgrad_wide_target": > 0 overrides the K-split's block target

static long g_wgrad_dma_cfg = 0;  // vm_set_option "wgrad_dma_cfg" (A/B): 0 auto, 1 = 8-row tiles, 2 = 4 rows x 6 slots

template <int NCI, int NT, int TH, int S>
static int launch_wgrad_taps_dma_s(WgArgs& a, float* dw, hipStream_t st) {
  using C = WtDma<NCI, NT, TH>;
  static int attr_dev = -1, resident = 0;
  return launch_wgrad_grid(reinterpret_cast<const void*>(&wgrad_taps_dma_kernel<NCI, NT, TH, S>),
                           C::template lds<S>(), TH, C::CIB, attr_dev, resident, a, dw, st,
                           [](dim3 g, int lds, hipStream_t s, const WgArgs& x) {
                             hipLaunchKernelGGL((wgrad_taps_dma_kernel<NCI, NT, TH, S>), g, dim3(256), lds, s, x);
                           });
}

template <int NCI, int NT>
static int launch_wgrad_taps_dma_t(WgArgs& a, float* dw, hipStream_t st) {
  // 4 ring slots where two blocks still fit a CU's 160 KB, else 3
  constexpr int S4 = WtDma<NCI, NT, 4>::template lds<4>() <= 80 * 1024 ? 4 : 3;
  if (g_wgrad_dma_cfg == 1) return launch_wgrad_taps_dma_s<NCI, NT, 8, 3>(a, dw, st);
  if (g_wgrad_dma_cfg == 2) return launch_wgrad_taps_dma_s<NCI, NT, 4, 6>(a, dw, st);
  return launch_wgrad_taps_dma_s<NCI, NT, 4, S4>(a, dw, st);
}

static int launch_wgrad_taps_dma(WgArgs& a, float* dw, hipStream_t st) {
  const int nt = (9 * a.cout + 15) / 16;
  if (nt <= 5 && a.cin > 32) {
    switch (nt) {
      case 1: return launch_wgrad_taps_dma_t<4, 1>(a, dw, st);
      case 2: return launch_wgrad_taps_dma_t<4, 2>(a, dw, st);
      case 3: return launch_wgrad_taps_dma_t<4, 3>(a, dw, st);
      case 4: return launch_wgrad_taps_dma_t<4, 4>(a, dw, st);
      default: return launch_wgrad_taps_dma_t<4, 5>(a, dw, st);
    }
  }
  switch (nt) {
    case 1: return launch_wgrad_taps_dma_t<2, 1>(a, dw, st);
    case 2: return launch_wgrad_taps_dma_t<2, 2>(a, dw, st);
    case 3: return launch_wgrad_taps_dma_t<2, 3>(a, dw, st);
    case 4: return launch_wgrad_taps_dma_t<2, 4>(a, dw, st);
    case 5: return launch_wgrad_taps_dma_t<2, 5>(a, dw, st);
    case 6: return launch_wgrad_taps_dma_t<2, 6>(a, dw, st);
    case 7: return launch_wgrad_taps_dma_t<2, 7>(a, dw, st);
    case 8: return launch_wgrad_taps_dma_t<2, 8>(a, dw, st);
    default: return launch_wgrad_taps_dma_t<2, 9>(a, dw, st);
  }
}
}  // namespace trn

int train_set_option(const char* key, long value) {
  if (!strcmp(key, "wgrad_reduce4")) {
    trn::g_wgrad_reduce4 = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_variant")) {
    trn::g_wgrad_variant = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_taps")) {
    trn::g_wgrad_taps = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_dma")) {
    trn::g_wgrad_dma = value;
    return 1;
  }
  if (!strcmp(key, "bn_vec")) {
    trn::g_bn_vec = value;
    return 1;
  }
  if (!strcmp(key, "relu_bias_vec")) {
    trn::g_relu_bias_vec = value;
    return 1;
  }
  if (!strcmp(key, "resize_bwd_2x")) {
    trn::g_resize_bwd_2x = value;
    return 1;
  }
  if (!strcmp(key, "relu_bias_iters")) {
    trn::g_relu_bias_iters = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_mfma_pipe")) {
    trn::g_wgrad_mfma_pipe = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_wide_pipe")) {
    trn::g_wgrad_wide_pipe = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_wide_target")) {  // (<= WW_TARGET_BLOCKS: the workspace query's bound)
    trn::g_wgrad_wide_target = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_wide_cs")) {
    trn::g_wgrad_wide_cs = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_wide_dbuf")) {
    trn::g_wgrad_wide_dbuf = value;
    return 1;
  }
  if (!strcmp(key, "wgrad_dma_cfg")) {
    trn::g_wgrad_dma_cfg = value;
    return 1;
  }
  return 0;
}

namespace trn {

static int launch_wgrad_mfma(WgArgs& a, float* dw, hipStream_t st) {
  WmCfg c = wgrad_mfma_cfg(a.cin, a.cout);
  const bool th8 = g_wgrad_variant == 2;
  if (wgrad_dma_ok(a, (9 * a.cout + 15) / 16 <= 5 && a.cin > 32 ? 64 : 32)) return launch_wgrad_taps_dma(a, dw, st);
  if (c.nt && g_wgrad_taps) {
#define VM_WT(NCI, NT) \
  return th8 ? launch_wgrad_taps_t<NCI, NT, 8>(a, dw, st) : launch_wgrad_taps_t<NCI, NT, 4>(a, dw, st)
    if (c.nci == 1) {
      switch (c.nt) { case 1: VM_WT(1, 1); case 2: VM_WT(1, 2); case 3: VM_WT(1, 3); case 4: VM_WT(1, 4); default: VM_WT(1, 5); }
    } else if (c.nci == 2) {
      switch (c.nt) { case 1: VM_WT(2, 1); case 2: VM_WT(2, 2); case 3: VM_WT(2, 3); case 4: VM_WT(2, 4); default: VM_WT(2, 5); }
    } else {
      switch (c.nt) { case 1: VM_WT(4, 1); case 2: VM_WT(4, 2); default: VM_WT(4, 3); }
    }
#undef VM_WT
  }
  if (c.nt) {  // the legacy tiling of this shape
    c.nt = 0;
    c.nci = a.cin > 16 ? 2 : 1;
  }
  if (c.nco == 1 && c.nci >= 2)
    return th8 ? launch_wgrad_mfma_t<2, 1, false, 8>(a, dw, st) : launch_wgrad_mfma_t<2, 1, false, 4>(a, dw, st);
  if (c.nci == 1 && c.nco == 1)
    return th8 ? launch_wgrad_mfma_t<1, 1, true, 8>(a, dw, st) : launch_wgrad_mfma_t<1, 1, true, 4>(a, dw, st);
  if (c.nci == 2 && c.nco == 2)
    return th8 ? launch_wgrad_mfma_t<2, 2, true, 8>(a, dw, st) : launch_wgrad_mfma_t<2, 2, true, 4>(a, dw, st);
  if (c.nci == 1 && c.nco == 2)
    return th8 ? launch_wgrad_mfma_t<1, 2, true, 8>(a, dw, st) : launch_wgrad_mfma_t<1, 2, true, 4>(a, dw, st);
  return th8 ? launch_wgrad_mfma_t<1, 3, true, 8>(a, dw, st) : launch_wgrad_mfma_t<1, 3, true, 4>(a, dw, st);
}

// K-split of the wide weight gradients: WW_TARGET_BLOCKS blocks in all (one resident round), at most one per pixel
// tile (bf16) / 32-pixel chunk (f32), and partials of at most WW_WS_CAP bytes
constexpr size_t WW_WS_CAP = 128ull << 20;

static long wgrad_wide_gx(int n, int h, int w, int cin, int cout, bool f32, long target = WW_TARGET_BLOCKS) {
  long units, nch;
  if (f32) {
    units = ((long)n * h * w + 31) / 32;
    nch = 9L * ((cin + 31) / 32) * ((cout + 63) / 64);
  } else {
    units = (long)n * ((h + WW_TH - 1) / WW_TH) * ((w + WM_TW - 1) / WM_TW);
    nch = (long)((cin + 63) / 64) * (cout / 64);
  }
  long gx = (target + nch - 1) / nch;
  const long cap = (long)(WW_WS_CAP / (9ull * cin * cout * sizeof(float)));
  if (gx > cap) gx = cap;
  if (gx > units) gx = units;
  return gx < 1 ? 1 : gx;
}

static int launch_wgrad_wide(const vm_tensor* x, const vm_tensor* dy, float* dw, void* work, hipStream_t st) {
  WwArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x->ptr) + x->coff;
  a.n = x->n; a.h = x->h; a.w = x->w; a.cin = x->c; a.xcs = x->cstride;
  const bool f32 = dy->dtype == VM_F32;
  a.dy = f32 ? static_cast<const void*>(reinterpret_cast<const float*>(dy->ptr) + dy->coff)
             : static_cast<const void*>(reinterpret_cast<const uint16_t*>(dy->ptr) + dy->coff);
  a.cout = dy->c; a.dcs = dy->cstride;
  a.part = reinterpret_cast<float*>(work);
  a.tiles_h = (a.h + WW_TH - 1) / WW_TH;
  a.tiles_w = (a.w + WM_TW - 1) / WM_TW;
  a.ntiles = (long)a.n * a.tiles_h * a.tiles_w;
  if (a.ntiles > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv_wgrad: too many pixel tiles");
  a.ncin = (a.cin + 63) / 64;
  a.ncout = a.cout / 64;
  // the pipelined kernel runs one block per CU: one resident round of WW_TARGET_BLOCKS / 2 blocks (half the partials)
  const bool pipe = g_wgrad_wide_pipe != 0;
  long target = pipe ? WW_TARGET_BLOCKS / 2 : WW_TARGET_BLOCKS;
  if (g_wgrad_wide_target > 0 && g_wgrad_wide_target <= WW_TARGET_BLOCKS) target = g_wgrad_wide_target;
  a.gx = (int)wgrad_wide_gx(a.n, a.h, a.w, a.cin, a.cout, false, target);
  const long nb = (long)a.gx * a.ncin * a.ncout;
  if (nb > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv_wgrad: grid too large");
  a.dbuf = pipe && g_wgrad_wide_dbuf ? 1 : 0;
  const int lds = wgrad_wide_lds<WW_TH>() * (a.dbuf ? 2 : 1);
  constexpr int lds_max = 2 * wgrad_wide_lds<WW_TH>();
  if (f32) {
    static int attr = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (attr != dev) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_wide_kernel<WW_TH, true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
      if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_wide_kernel<WW_TH, true, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
      if (e != hipSuccess) return fail(VM_EHIP, "wgrad_wide setup: %s", hipGetErrorString(e));
      attr = dev;
    }
    if (pipe) hipLaunchKernelGGL((wgrad_wide_kernel<WW_TH, true>), dim3((unsigned)nb), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((wgrad_wide_kernel<WW_TH, true, false>), dim3((unsigned)nb), dim3(256), lds, st, a);
  } else if (a.cin <= 16 && g_wgrad_wide_cs) {  // (the 6-channel conv1_1: output-channel wave split)
    static int attr = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    constexpr int lds1 = wgrad_wide_lds<WW_TH>();
    if (attr != dev) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_wide_kernel<WW_TH, false, false, true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds1);
      if (e != hipSuccess) return fail(VM_EHIP, "wgrad_wide setup: %s", hipGetErrorString(e));
      attr = dev;
    }
    hipLaunchKernelGGL((wgrad_wide_kernel<WW_TH, false, false, true>), dim3((unsigned)nb), dim3(256), lds1, st, a);
  } else {
    static int attr = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (attr != dev) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_wide_kernel<WW_TH, false>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
      if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_wide_kernel<WW_TH, false, false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
      if (e != hipSuccess) return fail(VM_EHIP, "wgrad_wide setup: %s", hipGetErrorString(e));
      attr = dev;
    }
    if (pipe) hipLaunchKernelGGL((wgrad_wide_kernel<WW_TH, false>), dim3((unsigned)nb), dim3(256), lds, st, a);
    else hipLaunchKernelGGL((wgrad_wide_kernel<WW_TH, false, false>), dim3((unsigned)nb), dim3(256), lds, st, a);
  }
  launch_wgrad_reduce(a.part, a.gx, 9L * a.cin * a.cout, dw, st);
  return VM_OK;
}

static int launch_wgrad_wide_f32(const vm_tensor* x, const vm_tensor* dy, float* dw, void* work, hipStream_t st) {
  WfArgs a{};
  a.x = reinterpret_cast<const float*>(x->ptr) + x->coff;
  a.n = x->n; a.h = x->h; a.w = x->w; a.cin = x->c; a.xcs = x->cstride;
  a.dy = reinterpret_cast<const float*>(dy->ptr) + dy->coff;
  a.cout = dy->c; a.dcs = dy->cstride;
  a.part = reinterpret_cast<float*>(work);
  a.npix = (long)a.n * a.h * a.w;
  a.ncin = (a.cin + 31) / 32;
  a.ncout = (a.cout + 63) / 64;
  a.gx = (int)wgrad_wide_gx(a.n, a.h, a.w, a.cin, a.cout, true);
  const long ny = 9L * a.ncin * a.ncout;
  if (ny > 65535) return fail(VM_EUNSUPPORTED, "conv_wgrad: too many channel blocks");
  hipLaunchKernelGGL(wgrad_wide_f32_kernel, dim3((unsigned)a.gx, (unsigned)ny), dim3(256), 0, st, a);
  launch_wgrad_reduce(a.part, a.gx, 9L * a.cin * a.cout, dw, st);
  return VM_OK;
}

static bool ok_view(const vm_tensor* t) { return valid_tensor(t); }

static bool same_shape(const vm_tensor* a, const vm_tensor* b) {
  return a->n == b->n && a->h == b->h && a->w == b->w && a->c == b->c;
}

}  // namespace trn
}  // namespace vm

using namespace vm;
using namespace vm::trn;

extern "C" int vm_bn_backward_ex_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                                      const float* var, const float* gamma, float eps, vm_tensor* dx, vm_tensor* dx2,
                                      float* dgamma, float* dbeta, float* dbias, void* work, void* stream);
extern "C" int vm_relu_backward_ex_nhwc(const vm_tensor* dy, const vm_tensor* y, vm_tensor* dx, vm_tensor* dx2,
                                        void* stream);
extern "C" int vm_relu_backward_split_nhwc(const vm_tensor* dy, const vm_tensor* y, int split, vm_tensor* dx_lo,
                                           vm_tensor* dx, vm_tensor* dx2, void* stream);

extern "C" int vm_matting_loss_backward(const float* pred, const float* gt, const float* raw_fg, const float* bg,
                                        const float* cmp, long pixels, float* dlogits, void* stream) {
  if (!pred || !gt || !raw_fg || !bg || !cmp || !dlogits || pixels <= 0)
    return fail(VM_EINVAL, "matting_loss_backward: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(loss_backward_kernel, dim3(grid_for(pixels, 256)), dim3(256), 0, st, pred, gt, raw_fg, bg, cmp,
                     pixels, dlogits);
  return check_launch("matting_loss_backward");
}

extern "C" size_t vm_bn_backward_workspace_bytes(int channels) {
  return channels <= 0 ? 0 : (size_t)3 * bn_max_blocks(channels) * channels * sizeof(double) + (size_t)2 * channels * sizeof(float);
}

extern "C" int vm_bn_backward_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                                   const float* var, const float* gamma, float eps, vm_tensor* dx, float* dgamma,
                                   float* dbeta, void* work, void* stream) {
  return vm_bn_backward_ex_nhwc(x, dy, y, mean, var, gamma, eps, dx, nullptr, dgamma, dbeta, nullptr, work, stream);
}

extern "C" int vm_bn_backward_ex_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                                      const float* var, const float* gamma, float eps, vm_tensor* dx, vm_tensor* dx2,
                                      float* dgamma, float* dbeta, float* dbias, void* work, void* stream) {
  if (dx2 && (!dx || !ok_view(dx2) || !same_shape(dx2, dy)))
    return fail(VM_EINVAL, "bn_backward: dx2 needs dx and an [n,h,w,c] view");
  if (dbias && !x) return fail(VM_EINVAL, "bn_backward: dbias needs x");
  if (!ok_view(dy) || dy->dtype != VM_F32 || !work) return fail(VM_EINVAL, "bn_backward: bad dy / workspace");
  if (x && (!ok_view(x) || !same_shape(x, dy) || !mean || !var)) return fail(VM_EINVAL, "bn_backward: bad x");
  if (y && (!ok_view(y) || !same_shape(y, dy))) return fail(VM_EINVAL, "bn_backward: bad relu mask y");
  if (dx && (!x || !ok_view(dx) || !same_shape(dx, dy) || dx->dtype != VM_F32))
    return fail(VM_EINVAL, "bn_backward: dx needs x and an f32 [n,h,w,c] view");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  V xv{}, yv{}, dyv = mk(dy);
  if (x) xv = mk(x);
  if (y) yv = mk(y);
  const int C = dy->c;
  double* part = reinterpret_cast<double*>(work);
  // the two channel sums land in dbeta / dgamma when given, else in the float tail of the workspace
  float* tail = reinterpret_cast<float*>(part + 3L * bn_max_blocks(C) * C);
  float* sg = dbeta ? dbeta : tail;
  float* sgx = dgamma ? dgamma : tail + C;
  const long M = (long)dy->n * dy->h * dy->w;
  const int nb = bn_blocks(M, C);
  auto v16 = [](const vm_tensor* t) {
    return t->cstride % 8 == 0 && t->coff % 8 == 0 && reinterpret_cast<uintptr_t>(t->ptr) % 16 == 0;
  };
  const bool vec = g_bn_vec && x && x->dtype == VM_F32 && C % 8 == 0 && C <= 512 && v16(x) && v16(dy) &&
                   (!y || (y->dtype == VM_BF16 && v16(y))) && (!dx || v16(dx)) &&
                   (!dx2 || (dx2->dtype == VM_BF16 && v16(dx2)));
  Bn8 b8{};
  int tpg = 1;
  if (vec) {
    b8.x = reinterpret_cast<const float*>(x->ptr) + x->coff;
    b8.dy = reinterpret_cast<const float*>(dy->ptr) + dy->coff;
    b8.y = y ? reinterpret_cast<const uint16_t*>(y->ptr) + y->coff : nullptr;
    b8.dx = dx ? reinterpret_cast<float*>(dx->ptr) + dx->coff : nullptr;
    b8.dx2 = dx2 ? reinterpret_cast<uint16_t*>(dx2->ptr) + dx2->coff : nullptr;
    b8.xcs = x->cstride; b8.dycs = dy->cstride; b8.ycs = y ? y->cstride : 0;
    b8.dxcs = dx ? dx->cstride : 0; b8.dx2cs = dx2 ? dx2->cstride : 0;
    b8.C = C; b8.M = M;
    tpg = C / 8 > 32 ? 64 : C / 8 > 16 ? 32 : C / 8 > 8 ? 16 : C / 8 > 4 ? 8 : C / 8 > 2 ? 4 : C / 8 > 1 ? 2 : 1;
#define VM_BP8(TPG)                                                                                                   \
  case TPG:                                                                                                           \
    if (y) hipLaunchKernelGGL((bn_bwd_partial8<true, TPG>), dim3(nb), dim3(256), 0, st, b8, mean, var, eps, part, nb); \
    else hipLaunchKernelGGL((bn_bwd_partial8<false, TPG>), dim3(nb), dim3(256), 0, st, b8, mean, var, eps, part, nb); \
    break;
    switch (tpg) { VM_BP8(1) VM_BP8(2) VM_BP8(4) VM_BP8(8) VM_BP8(16) VM_BP8(32) VM_BP8(64) }
#undef VM_BP8
  } else if (y) {
    launch_bn_bwd_partial<true>(xv, dyv, yv, mean, var, eps, part, nb, st);
  } else {
    launch_bn_bwd_partial<false>(xv, dyv, yv, mean, var, eps, part, nb, st);
  }
  int rc = check_launch("bn_backward_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_bwd_final, dim3(C), dim3(256), 0, st, part, nb, C, sg, x ? sgx : nullptr, dbias, gamma, var,
                     eps, M);
  rc = check_launch("bn_backward_final");
  if (rc || !dx) return rc;
  if (vec) {
    const long px = (M + 256 / tpg - 1) / (256 / tpg);
    const dim3 g8((unsigned)(px < 4096 ? px : 4096));
#define VM_BA8(TPG)                                                                                                  \
  case TPG:                                                                                                          \
    if (y && dx2) hipLaunchKernelGGL((bn_bwd_apply8<true, true, TPG>), g8, dim3(256), 0, st, b8, mean, var, gamma,   \
                                     eps, sg, sgx);                                                                  \
    else if (y) hipLaunchKernelGGL((bn_bwd_apply8<true, false, TPG>), g8, dim3(256), 0, st, b8, mean, var, gamma,    \
                                   eps, sg, sgx);                                                                    \
    else if (dx2) hipLaunchKernelGGL((bn_bwd_apply8<false, true, TPG>), g8, dim3(256), 0, st, b8, mean, var, gamma,  \
                                     eps, sg, sgx);                                                                  \
    else hipLaunchKernelGGL((bn_bwd_apply8<false, false, TPG>), g8, dim3(256), 0, st, b8, mean, var, gamma, eps, sg, \
                            sgx);                                                                                    \
    break;
    switch (tpg) { VM_BA8(1) VM_BA8(2) VM_BA8(4) VM_BA8(8) VM_BA8(16) VM_BA8(32) VM_BA8(64) }
#undef VM_BA8
    return check_launch("bn_backward_apply");
  }
  if (!y && !dx2 && f32_pair(x) && f32_pair(dy) && f32_pair(dx) && x->cstride > 0) {
    hipLaunchKernelGGL(bn_bwd_apply2_f32, dim3(grid_for(M, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float*>(x->ptr) + x->coff, x->cstride,
                       reinterpret_cast<const float*>(dy->ptr) + dy->coff, dy->cstride,
                       reinterpret_cast<float*>(dx->ptr) + dx->coff, dx->cstride, M, mean, var, gamma, eps, sg, sgx);
    return check_launch("bn_backward_apply");
  }
  const int cp = lanes_for(C);
  const dim3 grid = lanes_grid(M, C, cp);
  const V dxv = mk(dx), dx2v = dx2 ? mk(dx2) : V{};
#define VM_BNA(CP)                                                                                                    \
  if (y) hipLaunchKernelGGL((bn_bwd_apply<true, CP>), grid, dim3(256), 0, st, xv, dyv, yv, mean, var, gamma, eps, sg, \
                            sgx, dxv, dx2v);                                                                          \
  else hipLaunchKernelGGL((bn_bwd_apply<false, CP>), grid, dim3(256), 0, st, xv, dyv, yv, mean, var, gamma, eps, sg,  \
                          sgx, dxv, dx2v)
  VM_CP_SWITCH(cp, VM_BNA)
#undef VM_BNA
  return check_launch("bn_backward_apply");
}

extern "C" int vm_bn_backward_apply_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y,
                                         const float* mean, const float* var, const float* gamma, float eps,
                                         const float* sum_g, const float* sum_gx, long count, vm_tensor* dx,
                                         vm_tensor* dx2, void* stream) {
  if (!ok_view(x) || !ok_view(dy) || dy->dtype != VM_F32 || !same_shape(x, dy) || !mean || !var || !sum_g ||
      !sum_gx || count <= 0 || !dx || !ok_view(dx) || !same_shape(dx, dy) || dx->dtype != VM_F32 ||
      (y && (!ok_view(y) || !same_shape(y, dy))) || (dx2 && (!ok_view(dx2) || !same_shape(dx2, dy))))
    return fail(VM_EINVAL, "bn_backward_apply: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)dy->n * dy->h * dy->w;
  const V xv = mk(x), dyv = mk(dy), yv = y ? mk(y) : V{}, dxv = mk(dx), dx2v = dx2 ? mk(dx2) : V{};
  const int cp = lanes_for(dy->c);
  const dim3 grid = lanes_grid(M, dy->c, cp);
#define VM_BNA(CP)                                                                                                    \
  if (y) hipLaunchKernelGGL((bn_bwd_apply<true, CP>), grid, dim3(256), 0, st, xv, dyv, yv, mean, var, gamma, eps,     \
                            sum_g, sum_gx, dxv, dx2v, count);                                                         \
  else hipLaunchKernelGGL((bn_bwd_apply<false, CP>), grid, dim3(256), 0, st, xv, dyv, yv, mean, var, gamma, eps,      \
                          sum_g, sum_gx, dxv, dx2v, count)
  VM_CP_SWITCH(cp, VM_BNA)
#undef VM_BNA
  return check_launch("bn_backward_apply");
}

extern "C" int vm_relu_backward_nhwc(const vm_tensor* dy, const vm_tensor* y, vm_tensor* dx, void* stream) {
  return vm_relu_backward_ex_nhwc(dy, y, dx, nullptr, stream);
}

extern "C" int vm_relu_backward_ex_nhwc(const vm_tensor* dy, const vm_tensor* y, vm_tensor* dx, vm_tensor* dx2,
                                        void* stream) {
  return vm_relu_backward_split_nhwc(dy, y, 0, nullptr, dx, dx2, stream);
}

extern "C" int vm_relu_backward_split_nhwc(const vm_tensor* dy, const vm_tensor* y, int split, vm_tensor* dx_lo,
                                           vm_tensor* dx, vm_tensor* dx2, void* stream) {
  if (!ok_view(dy) || !ok_view(y) || !same_shape(dy, y) || split < 0 || split >= dy->c)
    return fail(VM_EINVAL, "relu_backward: bad tensors");
  auto part_ok = [&](const vm_tensor* t, int c) {
    return ok_view(t) && t->n == dy->n && t->h == dy->h && t->w == dy->w && t->c == c;
  };
  if (!part_ok(dx, dy->c - split) || (dx2 && !part_ok(dx2, dy->c - split)) || (split > 0 && !(dx_lo && part_ok(dx_lo, split))))
    return fail(VM_EINVAL, "relu_backward: outputs must be [n,h,w,%d] (dx, dx2) and [n,h,w,%d] (dx_lo)",
                dy->c - split, split);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)dy->n * dy->h * dy->w;
  const int cp = lanes_for(dy->c);
  const dim3 grid = lanes_grid(M, dy->c, cp);
  const V a = mk(dy), b = mk(y), c = mk(dx), d = dx2 ? mk(dx2) : V{}, e = split > 0 ? mk(dx_lo) : V{};
#define VM_RB(CP) hipLaunchKernelGGL((relu_bwd_kernel<CP>), grid, dim3(256), 0, st, a, b, c, d, e, split)
  VM_CP_SWITCH(cp, VM_RB)
#undef VM_RB
  return check_launch("relu_backward");
}

extern "C" int vm_maxpool2x2_backward_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* add, vm_tensor* dx,
                                           void* stream) {
  if (!ok_view(x) || !ok_view(dy) || !ok_view(dx) || !same_shape(x, dx) || (add && (!ok_view(add) || !same_shape(add, x))))
    return fail(VM_EINVAL, "maxpool_backward: bad tensors");
  if (dy->n != x->n || dy->h != (x->h + 1) / 2 || dy->w != (x->w + 1) / 2 || dy->c != x->c)
    return fail(VM_EINVAL, "maxpool_backward: dy must be [%d,%d,%d,%d]", x->n, (x->h + 1) / 2, (x->w + 1) / 2, x->c);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)x->n * x->h * x->w;
  const int cp = lanes_for(x->c);
  const dim3 grid = lanes_grid(M, x->c, cp);
  const V a = mk(x), b = mk(dy), c = add ? mk(add) : V{}, d = mk(dx);
#define VM_MPB(CP) hipLaunchKernelGGL((maxpool_bwd_kernel<CP>), grid, dim3(256), 0, st, a, b, c, d)
  VM_CP_SWITCH(cp, VM_MPB)
#undef VM_MPB
  return check_launch("maxpool_backward");
}


extern "C" size_t vm_relu_backward_bias_workspace_bytes(int channels) {
  return channels <= 0 ? 0 : (size_t)bn_max_blocks(channels) * channels * sizeof(double);
}

extern "C" int vm_relu_backward_bias_nhwc(const vm_tensor* dy, const vm_tensor* y, const vm_tensor* add,
                                          vm_tensor* dz, float* dbias, void* work, void* stream) {
  if (!ok_view(dy) || !ok_view(y) || !ok_view(dz) || (add && !ok_view(add)) || !dbias || !work)
    return fail(VM_EINVAL, "relu_backward_bias: bad argument");
  if (!same_shape(dz, y) || (add && !same_shape(add, y)) || dy->n != y->n || dy->c != y->c)
    return fail(VM_EINVAL, "relu_backward_bias: dz and add shaped like y");
  const bool pool = !(dy->h == y->h && dy->w == y->w);
  if (pool && (dy->h != (y->h + 1) / 2 || dy->w != (y->w + 1) / 2))
    return fail(VM_EINVAL, "relu_backward_bias: dy must be y's shape or its 2x2 SAME pool's");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int C = y->c;
  const long units = pool ? (long)dy->n * dy->h * dy->w : (long)y->n * y->h * y->w;
  auto al16 = [](const vm_tensor* t, int es) {  // every 8-channel run of the view 16-byte aligned
    return t->cstride % 8 == 0 && t->coff % 8 == 0 && reinterpret_cast<uintptr_t>(t->ptr) % 16 == 0 && es > 0;
  };
  if (g_relu_bias_vec && y->dtype == VM_BF16 && dz->dtype == VM_BF16 && C % 8 == 0 && C <= 512 && al16(y, 2) &&
      al16(dz, 2) && al16(dy, 4) && (!add || al16(add, 4))) {
    const int tpg = C / 8 > 32 ? 64 : C / 8 > 16 ? 32 : C / 8 > 8 ? 16 : C / 8 > 4 ? 8 : C / 8 > 2 ? 4 : C / 8 > 1 ? 2 : 1;
    // every block covers all C channels of 256 / tpg pixels per iteration: size the grid for ~g_relu_bias_iters
    // iterations per thread (bn_blocks' per-channel-group rule left the 512-channel levels at 12-50 blocks)
    int nb = bn_blocks(pool ? 4 * units : units, C);
    if (g_relu_bias_iters > 0) {
      const long want = (pool ? 4 * units : units) / ((256 / tpg) * g_relu_bias_iters);
      nb = (int)std::max(1L, std::min<long>(want, bn_max_blocks(C)));
    }
    const uint16_t* yp = reinterpret_cast<const uint16_t*>(y->ptr) + y->coff;
    uint16_t* zp = reinterpret_cast<uint16_t*>(dz->ptr) + dz->coff;
    double* part = reinterpret_cast<double*>(work);
    auto go = [&](auto dyt, auto at) {  // dy / add element types
      using TD = decltype(dyt);
      using TA = decltype(at);
      const TD* dyp = reinterpret_cast<const TD*>(dy->ptr) + dy->coff;
      const TA* ap = add ? reinterpret_cast<const TA*>(add->ptr) + add->coff : nullptr;
      const int acs = add ? add->cstride : 0;
#define VM_RB8(TPG)                                                                                                  \
  case TPG:                                                                                                          \
    if (pool && add)                                                                                                 \
      hipLaunchKernelGGL((relu_bwd_bias8_kernel<true, true, TPG, TD, TA>), dim3(nb), dim3(256), 0, st, dyp,          \
                         dy->cstride, yp, y->cstride, ap, acs, zp, dz->cstride, y->n, y->h, y->w, dy->h, dy->w, C,   \
                         part, nb);                                                                                  \
    else if (pool)                                                                                                   \
      hipLaunchKernelGGL((relu_bwd_bias8_kernel<true, false, TPG, TD, TA>), dim3(nb), dim3(256), 0, st, dyp,         \
                         dy->cstride, yp, y->cstride, ap, acs, zp, dz->cstride, y->n, y->h, y->w, dy->h, dy->w, C,   \
                         part, nb);                                                                                  \
    else if (add)                                                                                                    \
      hipLaunchKernelGGL((relu_bwd_bias8_kernel<false, true, TPG, TD, TA>), dim3(nb), dim3(256), 0, st, dyp,         \
                         dy->cstride, yp, y->cstride, ap, acs, zp, dz->cstride, y->n, y->h, y->w, dy->h, dy->w, C,   \
                         part, nb);                                                                                  \
    else                                                                                                             \
      hipLaunchKernelGGL((relu_bwd_bias8_kernel<false, false, TPG, TD, TA>), dim3(nb), dim3(256), 0, st, dyp,        \
                         dy->cstride, yp, y->cstride, ap, acs, zp, dz->cstride, y->n, y->h, y->w, dy->h, dy->w, C,   \
                         part, nb);                                                                                  \
    break;
      switch (tpg) { VM_RB8(1) VM_RB8(2) VM_RB8(4) VM_RB8(8) VM_RB8(16) VM_RB8(32) VM_RB8(64) }
#undef VM_RB8
    };
    const bool dyb = dy->dtype == VM_BF16, ab = add && add->dtype == VM_BF16;
    if (dyb && ab) go(uint16_t{}, uint16_t{});
    else if (dyb) go(uint16_t{}, float{});
    else if (ab) go(float{}, uint16_t{});
    else go(float{}, float{});
    int rc = check_launch("relu_backward_bias");
    if (rc) return rc;
    hipLaunchKernelGGL(fold_sum_kernel, dim3(C), dim3(256), 0, st, part, nb, C, dbias);
    return check_launch("relu_backward_bias fold");
  }
  const int nb = bn_blocks(pool ? 4 * units : units, C);
  const int cp = C > 32 ? 64 : C > 16 ? 32 : C > 8 ? 16 : C > 4 ? 8 : C > 2 ? 4 : C > 1 ? 2 : 1;
  const dim3 grid(cp == 64 ? (C + 63) / 64 : 1, nb);
  V a = mk(dy), b = mk(y), c = add ? mk(add) : V{}, d = mk(dz);
  double* part = reinterpret_cast<double*>(work);
#define VM_RBB(CP)                                                                                           \
  if (pool) hipLaunchKernelGGL((relu_bwd_bias_kernel<true, CP>), grid, dim3(256), 0, st, a, b, c, d, part, nb); \
  else hipLaunchKernelGGL((relu_bwd_bias_kernel<false, CP>), grid, dim3(256), 0, st, a, b, c, d, part, nb)
  VM_CP_SWITCH(cp, VM_RBB)
#undef VM_RBB
  int rc = check_launch("relu_backward_bias");
  if (rc) return rc;
  hipLaunchKernelGGL(fold_sum_kernel, dim3(C), dim3(256), 0, st, part, nb, C, dbias);
  return check_launch("relu_backward_bias fold");
}

// Exact 2x upsampling (oh = 2 ih, ow = 2 iw: scale 0.5, the UNet decoders' every resize): the TF-1 taps are known in
// closed form — output o takes input o/2 with weight 1 when o is even; lo = (o-1)/2 and hi = min(lo + 1, in - 1) with
// 0.5 each when odd (1.0 on the last input, where hi = lo) — so input i collects output rows 2i-1, 2i, 2i+1 (weights
// 0.5, 1, 0.5 or 1 on the last) and the same columns.  Only resize_bwd_kernel's nonzero terms, in its order (rows
// ascending, columns ascending within a row, row = sum of wx * v from 0, acc = sum of wy * row from 0), and every
// product is exact (weights 0.5 / 1), so the sums are bit-identical to the windowed search's.  A lane takes 8 channels
// of one input pixel: 9 16-byte (bf16) or 2x16-byte (f32) loads, one 16-byte / 2x16-byte store.
template <typename TD, typename TX>
__global__ __launch_bounds__(256) void resize2x_bwd_kernel8(V dy, TX* __restrict__ dx, int ih, int iw) {
  const int C8 = dy.c / 8;
  const long total = (long)dy.n * ih * iw * C8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C8) * 8;
    const long ip = i / C8;
    const int ix = (int)(ip % iw);
    const long t = ip / iw;
    const int iy = (int)(t % ih);
    const int n = (int)(t / ih);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int oh = 2 * iy - 1 + r;
      if (oh < 0) continue;
      const float wy = r == 1 ? 1.f : (r == 2 && iy == ih - 1) ? 1.f : 0.5f;
      float row[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int ow = 2 * ix - 1 + q;
        if (ow < 0) continue;
        const float wx = q == 1 ? 1.f : (q == 2 && ix == iw - 1) ? 1.f : 0.5f;
        const long off = (((long)n * dy.h + oh) * dy.w + ow) * dy.cs + dy.coff + c;
        float v[8];
        if constexpr (sizeof(TD) == 4) {
          const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dy.p) + off);
          const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dy.p) + off + 4);
          v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        } else {
          const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(dy.p) + off);
          const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[2 * k] = __uint_as_float(w4[k] << 16);
            v[2 * k + 1] = __uint_as_float(w4[k] & 0xffff0000u);
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) row[k] += wx * v[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += wy * row[k];
    }
    TX* o = dx + ip * dy.c + c;
    if constexpr (sizeof(TX) == 4) {
      *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      *reinterpret_cast<float4*>(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    } else {
      uint32_t w4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w4[k] = (uint32_t)f2bf(acc[2 * k]) | ((uint32_t)f2bf(acc[2 * k + 1]) << 16);
      *reinterpret_cast<uint4*>(o) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
}

// the exact-2x form when it applies (dy 2x dx, c % 8 == 0, 16-byte aligned); false = not launched
static bool resize2x_bwd(const vm_tensor* dy, void* dx, bool dx_bf16, int ih, int iw, hipStream_t st) {
  if (!g_resize_bwd_2x || dy->h != 2 * ih || dy->w != 2 * iw || dy->c % 8 || dy->cstride % 8 || dy->coff % 8 ||
      reinterpret_cast<uintptr_t>(dy->ptr) % 16 || reinterpret_cast<uintptr_t>(dx) % 16)
    return false;
  const long n8 = (long)dy->n * ih * iw * (dy->c / 8);
  const dim3 g(grid_for(n8, 256, 256 * 64)), b(256);
  if (dy->dtype == VM_F32 && !dx_bf16)
    hipLaunchKernelGGL((resize2x_bwd_kernel8<float, float>), g, b, 0, st, mk(dy), (float*)dx, ih, iw);
  else if (dy->dtype == VM_F32)
    hipLaunchKernelGGL((resize2x_bwd_kernel8<float, uint16_t>), g, b, 0, st, mk(dy), (uint16_t*)dx, ih, iw);
  else if (!dx_bf16)
    hipLaunchKernelGGL((resize2x_bwd_kernel8<uint16_t, float>), g, b, 0, st, mk(dy), (float*)dx, ih, iw);
  else
    hipLaunchKernelGGL((resize2x_bwd_kernel8<uint16_t, uint16_t>), g, b, 0, st, mk(dy), (uint16_t*)dx, ih, iw);
  return true;
}

extern "C" int vm_resize_bilinear_tf1_backward(const vm_tensor* dy, float* dx, int ih, int iw, void* stream) {
  if (!ok_view(dy) || !dx || ih <= 0 || iw <= 0) return fail(VM_EINVAL, "resize_backward: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dy->h > 4 * ih || dy->w > 4 * iw || ih > 2 * dy->h || iw > 2 * dy->w)
    return fail(VM_EUNSUPPORTED, "resize_backward: scale %dx%d -> %dx%d outside the upsampling range", ih, iw, dy->h,
                dy->w);
  const float sy = (float)ih / (float)dy->h, sx = (float)iw / (float)dy->w;
  if (resize2x_bwd(dy, dx, false, ih, iw, st)) return check_launch("resize_backward");
  if (dy->c % 4 == 0 && dy->cstride % 4 == 0 && dy->coff % 4 == 0 && reinterpret_cast<uintptr_t>(dy->ptr) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(dx) % 16 == 0) {
    const long n4 = (long)dy->n * ih * iw * (dy->c / 4);
    if (dy->dtype == VM_F32)
      hipLaunchKernelGGL(resize_bwd_kernel4<float>, dim3(grid_for(n4, 256)), dim3(256), 0, st, mk(dy), dx, ih, iw, sy,
                         sx);
    else
      hipLaunchKernelGGL(resize_bwd_kernel4<uint16_t>, dim3(grid_for(n4, 256)), dim3(256), 0, st, mk(dy), dx, ih, iw,
                         sy, sx);
    return check_launch("resize_backward");
  }
  const long n = (long)dy->n * ih * iw * dy->c;
  hipLaunchKernelGGL(resize_bwd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, mk(dy), dx, ih, iw, sy, sx);
  return check_launch("resize_backward");
}

// dx as a view: f32 as above, or dense bf16 with c % 4 == 0 and 8-byte aligned (the bf16 training path's relu
// gradients: the relu backward rounds dz to bf16 anyway, so a bf16 dx changes no dz where no `add` joins it)
extern "C" int vm_resize_bilinear_tf1_backward_nhwc(const vm_tensor* dy, vm_tensor* dx, void* stream) {
  if (!ok_view(dy) || !ok_view(dx) || dx->n != dy->n || dx->c != dy->c)
    return fail(VM_EINVAL, "resize_backward: dx [n,ih,iw,c] with dy's n and c");
  if (dx->cstride != dx->c || dx->coff != 0) return fail(VM_EUNSUPPORTED, "resize_backward: dx must be dense");
  if (dx->dtype == VM_F32) return vm_resize_bilinear_tf1_backward(dy, reinterpret_cast<float*>(dx->ptr), dx->h, dx->w,
                                                                  stream);
  const int ih = dx->h, iw = dx->w;
  if (dy->h > 4 * ih || dy->w > 4 * iw || ih > 2 * dy->h || iw > 2 * dy->w)
    return fail(VM_EUNSUPPORTED, "resize_backward: scale %dx%d -> %dx%d outside the upsampling range", ih, iw, dy->h,
                dy->w);
  if (dy->c % 4 || dy->cstride % 4 || dy->coff % 4 || reinterpret_cast<uintptr_t>(dy->ptr) % 16 ||
      reinterpret_cast<uintptr_t>(dx->ptr) % 8)
    return fail(VM_EUNSUPPORTED, "resize_backward: bf16 dx needs c %% 4 == 0 and aligned views");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (resize2x_bwd(dy, dx->ptr, true, ih, iw, st)) return check_launch("resize_backward");
  const float sy = (float)ih / (float)dy->h, sx = (float)iw / (float)dy->w;
  const long n4 = (long)dy->n * ih * iw * (dy->c / 4);
  uint16_t* d = reinterpret_cast<uint16_t*>(dx->ptr);
  if (dy->dtype == VM_F32)
    hipLaunchKernelGGL((resize_bwd_kernel4<float, uint16_t>), dim3(grid_for(n4, 256)), dim3(256), 0, st, mk(dy), d, ih,
                       iw, sy, sx);
  else
    hipLaunchKernelGGL((resize_bwd_kernel4<uint16_t, uint16_t>), dim3(grid_for(n4, 256)), dim3(256), 0, st, mk(dy), d,
                       ih, iw, sy, sx);
  return check_launch("resize_backward");
}

extern "C" size_t vm_conv3x3_wgrad_workspace_bytes(int n, int h, int w, int cin, int cout) {
  if (n <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return 0;
  return (size_t)wgrad_rows(n, h, w, cin, cout, wgrad_cc(cout)) * 9 * cin * cout * sizeof(float);
}

extern "C" int vm_conv3x3_wgrad_nhwc(const vm_tensor* x, const vm_tensor* dy, float* dw, void* work, void* stream) {
  if (!ok_view(x) || !ok_view(dy) || !dw || !work || dy->dtype != VM_F32 || dy->n != x->n || dy->h != x->h ||
      dy->w != x->w)
    return fail(VM_EINVAL, "conv3x3_wgrad: bad argument");
  const int cout = dy->c;
  if (cout > 48) return fail(VM_EUNSUPPORTED, "conv3x3_wgrad: cout %d > 48", cout);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  V xv = mk(x), dv = mk(dy);
  float* ws = reinterpret_cast<float*>(work);
  const int co4 = (cout + 3) / 4;
  switch (co4) {
    case 1: launch_wgrad<64, 1>(xv, dv, dw, ws, st); break;
    case 2: launch_wgrad<64, 2>(xv, dv, dw, ws, st); break;
    case 3:
    case 4: launch_wgrad<32, 4>(xv, dv, dw, ws, st); break;
    case 5:
    case 6: launch_wgrad<32, 6>(xv, dv, dw, ws, st); break;
    case 7:
    case 8: launch_wgrad<32, 8>(xv, dv, dw, ws, st); break;
    default: launch_wgrad<32, 12>(xv, dv, dw, ws, st); break;
  }
  return check_launch("conv3x3_wgrad");
}

extern "C" size_t vm_conv3x3_wgrad_ex_workspace_bytes(int n, int h, int w, int cin, int cout, int mode) {
  if (n <= 0 || h <= 0 || w <= 0 || cin <= 0 || cout <= 0) return 0;
  if (cout > 48)  // the wide kernels (UNetImage training)
    return (size_t)wgrad_wide_gx(n, h, w, cin, cout, mode != 1) * 9 * cin * cout * sizeof(float);
  if (mode != 1) return (size_t)wgrad_rows(n, h, w, cin, cout, wgrad_cc(cout)) * 9 * cin * cout * sizeof(float);
  const WmCfg c = wgrad_mfma_cfg(cin, cout);
  long rows = wgrad_rows(n, h, w, cin, cout, c.nci * 16);
  if (cout <= 16) {  // the LDS-DMA narrow kernel may take 64-channel blocks (fewer of them, more rows each)
    const long r64 = wgrad_rows(n, h, w, cin, cout, 64);
    if (r64 > rows) rows = r64;
  }
  return (size_t)rows * 9 * cin * cout * sizeof(float);
}

extern "C" int vm_conv3x3_wgrad_ex_nhwc(const vm_tensor* x, int x_src_c, long x_src_stride, const vm_tensor* dy,
                                        float* dw, void* work, int mode, void* stream) {
  vm_tensor xs = x ? *x : vm_tensor{};
  if (x_src_c > 0) xs.c = x_src_c;  // the view of source 0 must be valid; the others follow at x_src_stride
  if (!x || !ok_view(&xs) || !ok_view(dy) || !dw || !work || (dy->dtype != VM_F32 && !(dy->dtype == VM_BF16 && dy->c > 48)) || dy->n != x->n || dy->h != x->h ||
      dy->w != x->w || x_src_c < 0 || (x_src_c > 0 && (x_src_stride <= 0 || x->c % x_src_c)) ||
      (mode != 0 && mode != 1))
    return fail(VM_EINVAL, "conv3x3_wgrad_ex: bad argument");
  if (dy->c > 48) {  // the wide weight gradients of UNetImage's convs (train.py:37-109)
    if (x_src_c > 0) return fail(VM_EUNSUPPORTED, "conv3x3_wgrad_ex: split sources need cout <= 48");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (mode == 0) {
      if (x->dtype != VM_F32 || dy->dtype != VM_F32)
        return fail(VM_EUNSUPPORTED, "conv3x3_wgrad_ex: the exact mode with cout > 48 needs f32 x and dy");
      int rc = launch_wgrad_wide_f32(x, dy, dw, work, st);
      return rc ? rc : check_launch("conv3x3_wgrad_ex");
    }
    const int dch = dy->dtype == VM_F32 ? 4 : 8;  // elements per 16 bytes
    if (x->dtype != VM_BF16 || reinterpret_cast<uintptr_t>(x->ptr) % 16 || x->coff % 8 || x->cstride % 8 ||
        x->coff + (x->c + 7) / 8 * 8 > x->cstride || dy->c % 64 || (dy->dtype != VM_F32 && dy->dtype != VM_BF16) ||
        reinterpret_cast<uintptr_t>(dy->ptr) % 16 || dy->coff % dch || dy->cstride % dch)
      return fail(VM_EUNSUPPORTED, "conv3x3_wgrad_ex: the wide MFMA mode needs a bf16 x of 16-byte channel chunks "
                                   "and a 16-byte aligned dy of a multiple of 64 channels");
    int rc = launch_wgrad_wide(x, dy, dw, work, st);
    return rc ? rc : check_launch("conv3x3_wgrad_ex");
  }
  if (mode == 0) {  // exact f32 FMA kernel, optionally over split sources
    V xv = mk(x), dv = mk(dy);
    xv.sc = x_src_c;
    xv.ss = x_src_stride;
    float* ws = reinterpret_cast<float*>(work);
    switch ((dy->c + 3) / 4) {
      case 1: launch_wgrad<64, 1>(xv, dv, dw, ws, reinterpret_cast<hipStream_t>(stream)); break;
      case 2: launch_wgrad<64, 2>(xv, dv, dw, ws, reinterpret_cast<hipStream_t>(stream)); break;
      case 3:
      case 4: launch_wgrad<32, 4>(xv, dv, dw, ws, reinterpret_cast<hipStream_t>(stream)); break;
      case 5:
      case 6: launch_wgrad<32, 6>(xv, dv, dw, ws, reinterpret_cast<hipStream_t>(stream)); break;
      case 7:
      case 8: launch_wgrad<32, 8>(xv, dv, dw, ws, reinterpret_cast<hipStream_t>(stream)); break;
      default: launch_wgrad<32, 12>(xv, dv, dw, ws, reinterpret_cast<hipStream_t>(stream)); break;
    }
    return check_launch("conv3x3_wgrad_ex");
  }
  if (x->dtype != VM_BF16 || reinterpret_cast<uintptr_t>(x->ptr) % 16 || x->coff % 8 || x->cstride % 8 ||
      (x_src_c > 0 ? (x_src_c % 8 || x->c % x_src_c || x->coff + x_src_c > x->cstride || x_src_stride % 8)
                   : x->coff + (x->c + 7) / 8 * 8 > x->cstride))
    return fail(VM_EUNSUPPORTED, "conv3x3_wgrad_ex: the MFMA mode needs a bf16 x of 16-byte channel chunks");
  WgArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x->ptr) + x->coff;
  a.n = x->n; a.h = x->h; a.w = x->w; a.cin = x->c; a.xcs = x->cstride;
  a.x_src_c = x_src_c; a.x_src_stride = x_src_stride;
  a.dy = reinterpret_cast<const float*>(dy->ptr) + dy->coff;
  a.cout = dy->c; a.dcs = dy->cstride;
  a.part = reinterpret_cast<float*>(work);
  int rc = launch_wgrad_mfma(a, dw, reinterpret_cast<hipStream_t>(stream));
  if (rc) return rc;
  return check_launch("conv3x3_wgrad_ex");
}

extern "C" int vm_conv3x3_flip_weights(const float* w_hwio, int cin, int cout, float* w_flipped, void* stream) {
  if (!w_hwio || !w_flipped || cin <= 0 || cout <= 0) return fail(VM_EINVAL, "flip_weights: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(flip_weights_kernel, dim3(grid_for(9L * cin * cout, 256)), dim3(256), 0, st, w_hwio, cin, cout,
                     w_flipped);
  return check_launch("flip_weights");
}

extern "C" int vm_adam_tf(float* var, float* m, float* v, const float* grad, long n, float lr_t, float beta1,
                          float beta2, float eps, float grad_scale, void* stream) {
  if (!var || !m || !v || !grad || n <= 0) return fail(VM_EINVAL, "adam: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, var, m, v, grad, n, lr_t, beta1, beta2,
                     eps, grad_scale);
  return check_launch("adam");
}
