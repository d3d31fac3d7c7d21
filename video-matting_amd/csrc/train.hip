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
//   adam            TF ApplyAdam: m += (g-m)(1-b1); v += (g^2-v)(1-b2); var -= m*lr_t/(sqrt(v)+eps)

#include "vm_common.h"

namespace vm {
namespace trn {

struct V {
  char* p;
  int n, h, w, c, cs, coff, dt;
};

static V mk(const vm_tensor* t) {
  V v;
  v.p = reinterpret_cast<char*>(t->ptr);
  v.n = t->n; v.h = t->h; v.w = t->w; v.c = t->c; v.cs = t->cstride; v.coff = t->coff; v.dt = t->dtype;
  return v;
}

__device__ __forceinline__ float ld(const V& v, long pix, int c) {
  const long o = pix * v.cs + v.coff + c;
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
constexpr int BN_NBLK = 1024;  // pixel blocks (max); launches use min(BN_NBLK, M / 256)

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
  __shared__ double sh[2][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * CP + (lane % CP);
  const long M = (long)dy.n * dy.h * dy.w;
  double s1 = 0.0, s2 = 0.0;
  if (c < dy.c) {
    const float m = x.p ? mean[c] : 0.f;
    const float r = x.p ? 1.0f / sqrtf(var[c] + eps) : 0.f;
    for (long p = ((long)blockIdx.y * 4 + wave) * PPW + lane / CP; p < M; p += (long)nblk * 4 * PPW) {
      const float g = grad_in<MASK>(dy, y, p, c);
      s1 += g;
      if (x.p) s2 += (double)g * (double)((ld(x, p, c) - m) * r);
    }
  }
  sh[0][wave][lane] = s1;
  sh[1][wave][lane] = s2;
  __syncthreads();
  if ((int)threadIdx.x < CP && c < dy.c) {
    s1 = s2 = 0.0;
    for (int w = 0; w < 4; ++w)
      for (int k = 0; k < PPW; ++k) {
        s1 += sh[0][w][k * CP + threadIdx.x];
        s2 += sh[1][w][k * CP + threadIdx.x];
      }
    part[(long)blockIdx.y * dy.c + c] = s1;
    part[(long)nblk * dy.c + (long)blockIdx.y * dy.c + c] = s2;
  }
}

__global__ __launch_bounds__(64) void bn_bwd_final(const double* part, int nblk, int C, float* sum_g, float* sum_gx) {
  const int c = blockIdx.x, lane = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  for (int b = lane; b < nblk; b += 64) {
    s1 += part[(long)b * C + c];
    s2 += part[(long)nblk * C + (long)b * C + c];
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_down(s1, o);
    s2 += __shfl_down(s2, o);
  }
  if (lane == 0) {
    if (sum_g) sum_g[c] = (float)s1;
    if (sum_gx) sum_gx[c] = (float)s2;
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

template <bool MASK>
__global__ void bn_bwd_apply(V x, V dy, V y, const float* mean, const float* var, const float* gamma, float eps,
                             const float* sum_g, const float* sum_gx, V dx) {
  const long M = (long)dy.n * dy.h * dy.w;
  const long total = M * dy.c;
  const float invM = 1.0f / (float)M;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % dy.c);
    const long p = i / dy.c;
    const float r = 1.0f / sqrtf(var[c] + eps);
    const float xh = (ld(x, p, c) - mean[c]) * r;
    const float g = grad_in<MASK>(dy, y, p, c);
    const float gm = gamma ? gamma[c] : 1.f;
    st(dx, p, c, gm * r * (g - sum_g[c] * invM - xh * sum_gx[c] * invM));
  }
}

__global__ void relu_bwd_kernel(V dy, V y, V dx) {
  const long total = (long)dy.n * dy.h * dy.w * dy.c;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % dy.c);
    const long p = i / dy.c;
    st(dx, p, c, ld(y, p, c) > 0.f ? ld(dy, p, c) : 0.f);
  }
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
  auto issue = [&](long tile) {
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
                                                    (((long)n * x.h + gy) * x.w + gx) * x.cs + x.coff + c);
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

// dw[i] += sum over the gx block rows of the partials (fixed order: deterministic).  A block owns 64 columns; its
// 16 waves stride the rows (independent loads in flight), then fold through LDS.
__global__ __launch_bounds__(1024) void wgrad_reduce_kernel(const float* part, int rows, long S, float* dw) {
  __shared__ float sh[16][64];
  const int col = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + col;
  float s = 0.f;
  if (i < S) {
#pragma unroll 8
    for (int b = rg; b < rows; b += 16) s += part[(long)b * S + i];
  }
  sh[rg][col] = s;
  __syncthreads();
  if (rg == 0 && i < S) {
    float t = 0.f;
    for (int g = 0; g < 16; ++g) t += sh[g][col];
    dw[i] += t;
  }
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
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((S + 63) / 64)), dim3(1024), 0, st, ws, (int)gx, S, dw);
}

static bool vec_ok(const V& v, int ve) {
  return reinterpret_cast<uintptr_t>(v.p) % 16 == 0 && v.c % ve == 0 && v.coff % ve == 0 && v.cs % ve == 0;
}

// x may also be read in 16-byte vectors past its last channel when the row stride holds them (the padded
// concat / input buffers: up1n[..., :30] of a 32-wide row, in9[..., :9] of a 16-wide row); the extra lanes are zeroed
static bool xvec_ok(const V& v, int ve) {
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

static bool ok_view(const vm_tensor* t) { return valid_tensor(t); }

static bool same_shape(const vm_tensor* a, const vm_tensor* b) {
  return a->n == b->n && a->h == b->h && a->w == b->w && a->c == b->c;
}

}  // namespace trn
}  // namespace vm

using namespace vm;
using namespace vm::trn;

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
  return channels <= 0 ? 0 : (size_t)2 * BN_NBLK * channels * sizeof(double) + (size_t)2 * channels * sizeof(float);
}

extern "C" int vm_bn_backward_nhwc(const vm_tensor* x, const vm_tensor* dy, const vm_tensor* y, const float* mean,
                                   const float* var, const float* gamma, float eps, vm_tensor* dx, float* dgamma,
                                   float* dbeta, void* work, void* stream) {
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
  float* tail = reinterpret_cast<float*>(part + 2L * BN_NBLK * C);
  float* sg = dbeta ? dbeta : tail;
  float* sgx = dgamma ? dgamma : tail + C;
  const long M = (long)dy->n * dy->h * dy->w;
  const int nb = (int)(M / 256 < 1 ? 1 : M / 256 > BN_NBLK ? BN_NBLK : M / 256);
  if (y) launch_bn_bwd_partial<true>(xv, dyv, yv, mean, var, eps, part, nb, st);
  else launch_bn_bwd_partial<false>(xv, dyv, yv, mean, var, eps, part, nb, st);
  int rc = check_launch("bn_backward_partial");
  if (rc) return rc;
  hipLaunchKernelGGL(bn_bwd_final, dim3(C), dim3(64), 0, st, part, nb, C, sg, x ? sgx : nullptr);
  rc = check_launch("bn_backward_final");
  if (rc || !dx) return rc;
  const long work_n = (long)dy->n * dy->h * dy->w * C;
  if (y)
    hipLaunchKernelGGL(bn_bwd_apply<true>, dim3(grid_for(work_n, 256)), dim3(256), 0, st, xv, dyv, yv, mean, var,
                       gamma, eps, sg, sgx, mk(dx));
  else
    hipLaunchKernelGGL(bn_bwd_apply<false>, dim3(grid_for(work_n, 256)), dim3(256), 0, st, xv, dyv, yv, mean, var,
                       gamma, eps, sg, sgx, mk(dx));
  return check_launch("bn_backward_apply");
}

extern "C" int vm_relu_backward_nhwc(const vm_tensor* dy, const vm_tensor* y, vm_tensor* dx, void* stream) {
  if (!ok_view(dy) || !ok_view(y) || !ok_view(dx) || !same_shape(dy, y) || !same_shape(dy, dx))
    return fail(VM_EINVAL, "relu_backward: bad tensors");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long n = (long)dy->n * dy->h * dy->w * dy->c;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, mk(dy), mk(y), mk(dx));
  return check_launch("relu_backward");
}

extern "C" int vm_resize_bilinear_tf1_backward(const vm_tensor* dy, float* dx, int ih, int iw, void* stream) {
  if (!ok_view(dy) || !dx || ih <= 0 || iw <= 0) return fail(VM_EINVAL, "resize_backward: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dy->h > 4 * ih || dy->w > 4 * iw || ih > 2 * dy->h || iw > 2 * dy->w)
    return fail(VM_EUNSUPPORTED, "resize_backward: scale %dx%d -> %dx%d outside the upsampling range", ih, iw, dy->h,
                dy->w);
  const float sy = (float)ih / (float)dy->h, sx = (float)iw / (float)dy->w;
  const long n = (long)dy->n * ih * iw * dy->c;
  hipLaunchKernelGGL(resize_bwd_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, mk(dy), dx, ih, iw, sy, sx);
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
