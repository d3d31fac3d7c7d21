// 3x3 SAME stride-1 convolution as an implicit GEMM on gfx950 MFMA.
//
// Replaces tf.nn.conv2d + tf.nn.bias_add (+ relu / sigmoid / inference BN / softmax) at
// unet.py:35-42, 44-63, 65-74; unet_simple.py:19-42, 98-107; small.py:13-34; refine.py:18-31.
//
// GEMM view: D[cout][pixel] = sum_k Wp[cout][k] * X[pixel][k], k = tap*cin_pad + c,
// tap = kh*3 + kw, X[pixel][k] = x[n, h+kh-1, w+kw-1, c] (zero outside the frame).
//   A operand = packed weights (rows = output channels), B operand = activations
//   (rows = pixels); both K-contiguous, so every MFMA operand fragment is ONE 16-byte
//   LDS read per lane.  Output of a 16x16 MFMA tile: lane holds 4 consecutive output
//   channels of one pixel -> 16-byte LDS staging writes, then coalesced 16-byte stores.
// Tiles: 256 threads = 4 waves, each wave 64 pixels x 64 channels (4x4 MFMA 16x16 tiles);
//   block tile (BM pixels x BN channels) = (128 x 128) or (256 x 64).
// K-step: one 128-byte row per operand row (64 bf16 / 32 f32), double-buffered in LDS,
//   register-staged global loads issued before the MFMAs of the previous step.
// LDS image: [row][8 x 16-byte chunks], chunk XOR-swizzled by (row>>1)&7 — conflict-free for
//   the ds_read_b128 lane groups of a 16-row fragment read.
// bf16: v_mfma_f32_16x16x32_bf16; f32: v_mfma_f32_16x16x4_f32 (exact f32 products, f32 sums).

#include "vm_common.h"

namespace vm {

struct ConvArgs {
  const void* x;
  int x_cstride, x_coff, H, W;
  long M;  // N*H*W pixels
  int cin_pad, K9, nk;
  const void* w;
  int K_pad, cout, cout_pad;
  const float* bias;
  const float* scale;
  const float* shift;
  int act;
  void* y;
  int y_cstride, y_coff, y_dtype, y_vec;
  int tiles_n, tiles_total;
};

constexpr int ROWB = 128;  // bytes of one operand row per K-step

__device__ __forceinline__ int swz(int row, int chunk) { return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4); }

template <typename T>
__device__ __forceinline__ void mma16(const uint4& a, const uint4& b, f32x4& c);

template <>
__device__ __forceinline__ void mma16<uint16_t>(const uint4& a, const uint4& b, f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                               0);
}

template <>
__device__ __forceinline__ void mma16<float>(const uint4& a, const uint4& b, f32x4& c) {
  // lane k-slot s = lane>>4 holds k = 4s..4s+3 of the 16-wide k-block; MFMA t consumes element t.
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
}

template <int BM, int BN>
constexpr int conv_lds_bytes() {
  return (2 * (BM + BN) * ROWB) > (BM * (BN + 4) * 4) ? (2 * (BM + BN) * ROWB) : (BM * (BN + 4) * 4);
}

template <typename T, int BM, int BN, bool FAST>
__global__ __launch_bounds__(256, 2) void conv3x3_mfma(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CE = 16 / sizeof(T);      // elements per 16-byte chunk
  constexpr int BKE = ROWB / sizeof(T);   // K elements per step
  constexpr int XR = BM / 32;             // X chunks per thread per step
  constexpr int WR = BN / 32;             // W chunks per thread per step
  constexpr int WM = BM / 64;
  constexpr int WN = BN / 64;
  static_assert(WM * WN == 4, "4 waves of 64x64");
  constexpr int STAGE = (BM + BN) * ROWB;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;

  // XCD-aware bijective remap: blocks b and b+8 share an XCD -> give each XCD a contiguous tile range
  const int nwg = a.tiles_total;
  const int b = blockIdx.x;
  const int q = nwg >> 3, r8 = nwg & 7, xcd = b & 7;
  const int t = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (b >> 3);
  const int mt = t / a.tiles_n;
  const int nt = t - mt * a.tiles_n;
  const long m0 = (long)mt * BM;
  const int n0 = nt * BN;

  const int H = a.H, W = a.W;
  const long HW = (long)H * W;
  const int chunk = tid & 7;
  const int rbase = tid >> 3;

  long pix[XR];
  int ph[XR], pw[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    long p = m0 + rbase + 32 * i;
    pix[i] = p;
    if (p < a.M) {
      long rem = p % HW;
      ph[i] = (int)(rem / W);
      pw[i] = (int)(rem - (long)ph[i] * W);
    } else {
      ph[i] = -0x40000000;
      pw[i] = 0;
    }
  }

  // Bounds-checked buffer descriptors (wave-uniform, rebased per block so 32-bit offsets suffice for any
  // batch): a lane whose tap falls outside the frame gets an out-of-range offset and the hardware returns
  // 0 — the SAME-padding zero fill without a branch or a select on addresses.
  const long xbase = m0 - W - 1;  // lowest pixel any tap of this tile can touch
  const T* Xb = reinterpret_cast<const T*>(a.x) + a.x_coff + xbase * (long)a.x_cstride;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Xb), 0, 0x7ffffff0, 0x00020000);
  const T* Wb = reinterpret_cast<const T*>(a.w) + (long)n0 * a.K_pad;
  const uint32_t wbytes = (uint32_t)((long)(a.cout_pad - n0) * a.K_pad * (long)sizeof(T));
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(Wb), 0, wbytes, 0x00020000);
  const int xcs = a.x_cstride;
  int prow[XR];  // pixel index relative to xbase
#pragma unroll
  for (int i = 0; i < XR; ++i) prow[i] = (int)(pix[i] - xbase);

  uint4 xr[XR], wr[WR];

  auto load = [&](int kt) {
    int tap, c;
    if (FAST) {
      const int k0 = kt * BKE;
      tap = k0 / a.cin_pad;
      c = k0 - tap * a.cin_pad + chunk * CE;
    } else {
      const int k = kt * BKE + chunk * CE;
      tap = k < a.K9 ? k / a.cin_pad : 9;
      c = k - tap * a.cin_pad;
    }
    const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int hh = ph[i] + dh, ww = pw[i] + dw;
      const bool ok = tap < 9 && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      const int off = ok ? ((prow[i] + dh * W + dw) * xcs + c) * (int)sizeof(T) : (int)0x80000000;
      xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int off = ((rbase + 32 * i) * a.K_pad + kt * BKE + chunk * CE) * (int)sizeof(T);
      wr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
    }
  };

  auto store = [&](int buf) {
    char* s = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < XR; ++i) *reinterpret_cast<uint4*>(s + swz(rbase + 32 * i, chunk)) = xr[i];
#pragma unroll
    for (int i = 0; i < WR; ++i) *reinterpret_cast<uint4*>(s + BM * ROWB + swz(rbase + 32 * i, chunk)) = wr[i];
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // f32 path: the 32 products of one K-step chain into a fresh partial that is then added to the
  // running sum (two-level summation: error ~ (32 + K/32) ulp instead of K ulp for K up to 9216);
  // bf16 path: one chain (the bf16 operand rounding dominates).
  constexpr bool SPLIT = sizeof(T) == 4;
  auto compute = [&](int buf) {
    const char* s = smem + buf * STAGE;
    f32x4 part[4][4];
    if (SPLIT) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int ck = kb * 4 + (lane >> 4);
      uint4 av[4], bv[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) av[f] = *reinterpret_cast<const uint4*>(s + BM * ROWB + swz(wn * 64 + f * 16 + (lane & 15), ck));
#pragma unroll
      for (int f = 0; f < 4; ++f) bv[f] = *reinterpret_cast<const uint4*>(s + swz(wm * 64 + f * 16 + (lane & 15), ck));
#pragma unroll
      for (int fc = 0; fc < 4; ++fc)
#pragma unroll
        for (int fp = 0; fp < 4; ++fp) mma16<T>(av[fc], bv[fp], SPLIT ? part[fc][fp] : acc[fc][fp]);
    }
    if (SPLIT) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += part[i][j];
    }
  };

  const int nk = a.nk;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load(kt + 1);
    compute(kt & 1);
    if (kt + 1 < nk) store((kt + 1) & 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  constexpr int SROW = BN + 4;
  float* stg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int fc = 0; fc < 4; ++fc) {
    const int col = wn * 64 + fc * 16 + 4 * (lane >> 4);
    float bsv[4] = {0.f, 0.f, 0.f, 0.f}, scv[4] = {1.f, 1.f, 1.f, 1.f}, shv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = min(n0 + col + j, a.cout - 1);  // clamped: always a valid address, value unused if padded
      if (a.bias) bsv[j] = a.bias[co];
      if (a.scale) scv[j] = a.scale[co];
      if (a.shift) shv[j] = a.shift[co];
    }
#pragma unroll
    for (int fp = 0; fp < 4; ++fp) {
      const int row = wm * 64 + fp * 16 + (lane & 15);
      float4 v;
      float* vv = reinterpret_cast<float*>(&v);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float tv = (acc[fc][fp][j] + bsv[j]) * scv[j] + shv[j];
        if (a.act == VM_ACT_RELU) tv = tv > 0.f ? tv : 0.f;
        else if (a.act == VM_ACT_SIGMOID) tv = sigmoid_precise(tv);
        vv[j] = tv;
      }
      *reinterpret_cast<float4*>(stg + row * SROW + col) = v;
    }
  }
  __syncthreads();

  if (a.act == VM_ACT_SOFTMAX) {  // host guarantees a single channel tile (n0 == 0, cout <= BN)
    for (int rr = tid; rr < BM; rr += 256) {
      float* rowp = stg + rr * SROW;
      float mx = -INFINITY;
      for (int c = 0; c < a.cout; ++c) mx = fmaxf(mx, rowp[c]);
      float sum = 0.f;
      for (int c = 0; c < a.cout; ++c) {
        const float e = expf(rowp[c] - mx);
        rowp[c] = e;
        sum += e;
      }
      const float inv = 1.f / sum;
      for (int c = 0; c < a.cout; ++c) rowp[c] *= inv;
    }
    __syncthreads();
  }

  if (a.y_dtype == VM_BF16) {
    constexpr int CPR = BN / 8;
    uint16_t* Y = reinterpret_cast<uint16_t*>(a.y) + a.y_coff;
    for (int idx = tid; idx < BM * CPR; idx += 256) {
      const int rr = idx / CPR, cc = idx - rr * CPR;
      const long p = m0 + rr;
      const int co = n0 + cc * 8;
      if (p >= a.M || co >= a.cout) continue;
      const float* src = stg + rr * SROW + cc * 8;
      uint16_t* dst = Y + p * (long)a.y_cstride + co;
      if (a.y_vec && co + 8 <= a.cout) {
        *reinterpret_cast<uint4*>(dst) = Chunk<uint16_t>::pack(src);
      } else {
        for (int j = 0; j < 8 && co + j < a.cout; ++j) dst[j] = f2bf(src[j]);
      }
    }
  } else {
    constexpr int CPR = BN / 4;
    float* Y = reinterpret_cast<float*>(a.y) + a.y_coff;
    for (int idx = tid; idx < BM * CPR; idx += 256) {
      const int rr = idx / CPR, cc = idx - rr * CPR;
      const long p = m0 + rr;
      const int co = n0 + cc * 4;
      if (p >= a.M || co >= a.cout) continue;
      const float* src = stg + rr * SROW + cc * 4;
      float* dst = Y + p * (long)a.y_cstride + co;
      if (a.y_vec && co + 4 <= a.cout) {
        *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
      } else {
        for (int j = 0; j < 4 && co + j < a.cout; ++j) dst[j] = src[j];
      }
    }
  }
}

// ---------------------------------------------------------------- Cout == 1 head (conv1_5 + sigmoid)
// unet.py:203-205 / unet_simple.py:142 / small.py:49-50: a 1-channel 3x3 conv over 128 (or fewer)
// channels at full resolution is a memory-bound dot product: 16 lanes per pixel, each lane one
// 16-byte channel chunk per tap (a wave reads 4 pixels x 256 contiguous bytes), a 4-step
// xor-shuffle reduction inside each 16-lane group, weights staged once per block in LDS.
struct HeadArgs {
  const void* x;
  int x_cstride, x_coff, H, W;
  long M;
  int cin_pad;
  const void* w;
  const float* bias;
  const float* scale;
  const float* shift;
  int act;
  void* y;
  int y_cstride, y_coff, y_dtype;
};

template <typename T>
__global__ __launch_bounds__(256) void conv3x3_head(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CE = 16 / sizeof(T);
  float* sw = reinterpret_cast<float*>(smem);
  const int K9 = 9 * a.cin_pad;
  const T* Wt = reinterpret_cast<const T*>(a.w);
  for (int k = threadIdx.x; k < K9; k += 256) sw[k] = ld_elem<T>(Wt + k);
  __syncthreads();

  const int sub = threadIdx.x & 15;
  const int slot = threadIdx.x >> 4;
  const T* X = reinterpret_cast<const T*>(a.x) + a.x_coff;
  const long HW = (long)a.H * a.W;
  const float bias = a.bias ? a.bias[0] : 0.f;
  const float sc = a.scale ? a.scale[0] : 1.f;
  const float sh = a.shift ? a.shift[0] : 0.f;
  for (long p = (long)blockIdx.x * 16 + slot; p < a.M; p += (long)gridDim.x * 16) {
    const long rem = p % HW;
    const int h = (int)(rem / a.W);
    const int w = (int)(rem - (long)h * a.W);
    float acc = 0.f;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int dh = tap / 3 - 1, dw = tap % 3 - 1;
      const int hh = h + dh, ww = w + dw;
      if ((unsigned)hh >= (unsigned)a.H || (unsigned)ww >= (unsigned)a.W) continue;
      const T* px = X + (p + (long)dh * a.W + dw) * a.x_cstride;
      const float* wt = sw + tap * a.cin_pad;
      for (int c = sub * CE; c < a.cin_pad; c += 16 * CE) {
        float f[CE];
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(px + c), f);
#pragma unroll
        for (int j = 0; j < CE; ++j) acc = fmaf(f[j], wt[c + j], acc);
      }
    }
    acc += __shfl_xor(acc, 8, 16);
    acc += __shfl_xor(acc, 4, 16);
    acc += __shfl_xor(acc, 2, 16);
    acc += __shfl_xor(acc, 1, 16);
    if (sub == 0) {
      float v = (acc + bias) * sc + sh;
      if (a.act == VM_ACT_RELU) v = v > 0.f ? v : 0.f;
      else if (a.act == VM_ACT_SIGMOID) v = sigmoid_precise(v);
      else if (a.act == VM_ACT_SOFTMAX) v = 1.f;  // softmax over a single channel
      const long o = p * (long)a.y_cstride + a.y_coff;
      if (a.y_dtype == VM_BF16) reinterpret_cast<uint16_t*>(a.y)[o] = f2bf(v);
      else reinterpret_cast<float*>(a.y)[o] = v;
    }
  }
}

// ---------------------------------------------------------------- weight packing
// HWIO f32 [3][3][cin][cout] (unet.py:15 / the VGG npy layout) -> [cout_pad][K_pad] in the compute dtype.
template <typename T>
__global__ void pack_weights(const float* w, int cin, int cout, int cin_pad, int K_pad, int cout_pad, T* out) {
  const long total = (long)cout_pad * K_pad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i / K_pad);
    const int k = (int)(i - (long)co * K_pad);
    const int tap = k / cin_pad;
    const int c = k - tap * cin_pad;
    float v = 0.f;
    if (co < cout && tap < 9 && c < cin) v = w[((long)tap * cin + c) * cout + co];
    st_elem<T>(out + i, v);
  }
}

struct PackGeom {
  int cin_pad, bke, K9, K_pad, cout_pad, nk;
};

static PackGeom geom(int cin, int cout, int dtype) {
  PackGeom g;
  const int eb = elem_bytes(dtype);
  g.cin_pad = (cin + 7) / 8 * 8;
  g.bke = ROWB / eb;
  g.K9 = 9 * g.cin_pad;
  g.nk = (g.K9 + g.bke - 1) / g.bke;
  g.K_pad = g.nk * g.bke;
  g.cout_pad = (cout + 63) / 64 * 64;
  return g;
}

template <typename T, int BM, int BN, bool FAST>
static int launch_mfma(const ConvArgs& a, hipStream_t st) {
  constexpr int lds = conv_lds_bytes<BM, BN>();
  static bool attr_set = false;  // idempotent; benign race
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_mfma<T, BM, BN, FAST>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return fail(VM_EHIP, "hipFuncSetAttribute: %s", hipGetErrorString(e));
    attr_set = true;
  }
  hipLaunchKernelGGL((conv3x3_mfma<T, BM, BN, FAST>), dim3(a.tiles_total), dim3(256), lds, st, a);
  return check_launch("conv3x3_mfma");
}

template <typename T>
static int dispatch_mfma(ConvArgs& a, bool fast, hipStream_t st) {
  if (a.cout <= 64) {
    a.tiles_n = (a.cout + 63) / 64;
    a.tiles_total = (int)((a.M + 255) / 256) * a.tiles_n;
    return fast ? launch_mfma<T, 256, 64, true>(a, st) : launch_mfma<T, 256, 64, false>(a, st);
  }
  a.tiles_n = (a.cout + 127) / 128;
  a.tiles_total = (int)((a.M + 127) / 128) * a.tiles_n;
  return fast ? launch_mfma<T, 128, 128, true>(a, st) : launch_mfma<T, 128, 128, false>(a, st);
}

}  // namespace vm

using namespace vm;

extern "C" size_t vm_conv3x3_packed_bytes(int cin, int cout, int dtype) {
  if (cin <= 0 || cout <= 0 || (dtype != VM_F32 && dtype != VM_BF16)) return 0;
  PackGeom g = geom(cin, cout, dtype);
  return (size_t)g.cout_pad * g.K_pad * elem_bytes(dtype);
}

extern "C" int vm_conv3x3_pack_weights(const float* w_hwio, int cin, int cout, int dtype, void* packed, void* stream) {
  if (!w_hwio || !packed || cin <= 0 || cout <= 0) return fail(VM_EINVAL, "pack_weights: bad argument");
  if (dtype != VM_F32 && dtype != VM_BF16) return fail(VM_EINVAL, "pack_weights: dtype %d", dtype);
  PackGeom g = geom(cin, cout, dtype);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long total = (long)g.cout_pad * g.K_pad;
  const int grid = grid_for(total, 256);
  if (dtype == VM_BF16)
    hipLaunchKernelGGL(pack_weights<uint16_t>, dim3(grid), dim3(256), 0, st, w_hwio, cin, cout, g.cin_pad, g.K_pad,
                       g.cout_pad, reinterpret_cast<uint16_t*>(packed));
  else
    hipLaunchKernelGGL(pack_weights<float>, dim3(grid), dim3(256), 0, st, w_hwio, cin, cout, g.cin_pad, g.K_pad,
                       g.cout_pad, reinterpret_cast<float*>(packed));
  return check_launch("pack_weights");
}

extern "C" int vm_conv3x3_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                               const float* scale, const float* shift, int act, vm_tensor* y, void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y) || !packed) return fail(VM_EINVAL, "conv3x3: invalid tensor/weights");
  if (cin <= 0 || cout <= 0 || x->c != cin || y->c != cout)
    return fail(VM_EINVAL, "conv3x3: channel mismatch x.c=%d cin=%d y.c=%d cout=%d", x->c, cin, y->c, cout);
  if (x->n != y->n || x->h != y->h || x->w != y->w)
    return fail(VM_EINVAL, "conv3x3: spatial mismatch [%d,%d,%d] vs [%d,%d,%d]", x->n, x->h, x->w, y->n, y->h, y->w);
  if (act < VM_ACT_NONE || act > VM_ACT_SOFTMAX) return fail(VM_EINVAL, "conv3x3: act %d", act);
  const int dt = x->dtype;
  PackGeom g = geom(cin, cout, dt);
  const int ce = 16 / elem_bytes(dt);
  if (reinterpret_cast<uintptr_t>(x->ptr) % 16 || x->cstride % ce || x->coff % ce || x->coff + g.cin_pad > x->cstride)
    return fail(VM_EUNSUPPORTED,
                "conv3x3: input view must be 16-byte aligned with channel padding to %d (coff=%d cstride=%d)",
                g.cin_pad, x->coff, x->cstride);
  if (act == VM_ACT_SOFTMAX && cout > 128) return fail(VM_EUNSUPPORTED, "conv3x3: fused softmax needs cout <= 128");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)x->n * x->h * x->w;

  if (cout == 1) {
    HeadArgs h{};
    h.x = x->ptr; h.x_cstride = x->cstride; h.x_coff = x->coff; h.H = x->h; h.W = x->w; h.M = M;
    h.cin_pad = g.cin_pad; h.w = packed; h.bias = bias; h.scale = scale; h.shift = shift; h.act = act;
    h.y = y->ptr; h.y_cstride = y->cstride; h.y_coff = y->coff; h.y_dtype = y->dtype;
    const int grid = grid_for((M + 15) / 16, 1, 256 * 8);
    const size_t lds = (size_t)9 * g.cin_pad * 4;
    if (dt == VM_BF16) hipLaunchKernelGGL(conv3x3_head<uint16_t>, dim3(grid), dim3(256), lds, st, h);
    else hipLaunchKernelGGL(conv3x3_head<float>, dim3(grid), dim3(256), lds, st, h);
    return check_launch("conv3x3_head");
  }

  ConvArgs a{};
  a.x = x->ptr; a.x_cstride = x->cstride; a.x_coff = x->coff; a.H = x->h; a.W = x->w; a.M = M;
  a.cin_pad = g.cin_pad; a.K9 = g.K9; a.nk = g.nk;
  a.w = packed; a.K_pad = g.K_pad; a.cout = cout; a.cout_pad = g.cout_pad;
  a.bias = bias; a.scale = scale; a.shift = shift; a.act = act;
  a.y = y->ptr; a.y_cstride = y->cstride; a.y_coff = y->coff; a.y_dtype = y->dtype;
  const int yve = 16 / elem_bytes(y->dtype);
  a.y_vec = (reinterpret_cast<uintptr_t>(y->ptr) % 16 == 0) && (y->cstride % yve == 0) && (y->coff % yve == 0);
  const bool fast = (g.cin_pad % g.bke) == 0;
  if (dt == VM_BF16) return dispatch_mfma<uint16_t>(a, fast, st);
  return dispatch_mfma<float>(a, fast, st);
}
