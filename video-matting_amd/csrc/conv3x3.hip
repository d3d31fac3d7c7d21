// 3x3 SAME stride-1 convolution as an implicit GEMM on gfx950 MFMA.
//
// Replaces tf.nn.conv2d + tf.nn.bias_add (+ relu / sigmoid / inference BN / softmax) at
// unet.py:35-42, 44-63, 65-74; unet_simple.py:19-42, 98-107; small.py:13-34; refine.py:18-31.
//
// GEMM view: D[cout][pixel] = sum_k Wp[cout][k] * X[pixel][k], k <-> (tap, c), tap = kh*3 + kw,
// X[pixel][k] = x[n, h+kh-1, w+kw-1, c] (zero outside the frame).
//   A operand = packed weights (rows = output channels), B operand = activations (rows = pixels);
//   both K-contiguous, so every MFMA operand fragment is ONE 16-byte LDS read per lane, and a 16x16
//   MFMA tile leaves 4 consecutive output channels of one pixel in each lane.
// K layout ("granules" of 64 bytes = GE elements): when cin_pad % GE == 0 the K axis is
//   channel-chunk-major — granule g covers channels (g/9)*GE .. +GE of tap g%9 — so the 9 taps that
//   re-read the same input rows are consecutive K-steps and hit L2; otherwise tap-major k = tap*cin_pad+c.
//
// Two kernels:
//   conv3x3_mfma  register-staged, 256 threads, tiles 128x128 / 256x64, 128-byte K-steps, 2-slot LDS.
//                 Used for small grids, the fused softmax and as the reference implementation.
//   conv3x3_glds  LDS-DMA pipelined (buffer_load ... lds), 512 threads, tiles 256x256 / 256x128 / 512x64,
//                 64-byte K-steps in a 4-6 slot ring with counted vmcnt (3-5 stages in flight).
// bf16: v_mfma_f32_16x16x32_bf16; f32: v_mfma_f32_16x16x4_f32 (exact f32 products; a 2-level sum).

#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <cstdio>

#include "conv_common.h"

namespace vm {

// ConvArgs, swizzles, MFMA wrappers, LDS-DMA helpers: conv_common.h
// (K element index k) -> (tap, channel); tap 9 = padding (contributes zero)
template <int GE>
__device__ __forceinline__ void k_to_tap(const ConvArgs& a, int k, int& tap, int& c) {
  if (a.chunk_major) {
    const int g = k / GE;
    if (g < a.ng) {
      const int cc = g / 9;
      tap = g - cc * 9;
      c = cc * GE + (k - g * GE);
    } else {
      tap = 9;
      c = 0;
    }
  } else if (k < a.K9) {
    tap = k / a.cin_pad;
    c = k - tap * a.cin_pad;
  } else {
    tap = 9;
    c = 0;
  }
}

// Decode (h, w) of the pixels m0 + r of a tile without per-lane 64-bit division: the tile origin is decoded
// once (wave-uniform), a row offset r < BM + W is split by a float reciprocal (exact after one fix-up for
// values < 2^24).  Pixels at or past M get h = -2^30 so every tap is out of range.
struct TileOrigin {
  int h0, w0;
  float rcp_w, rcp_h;
};

__device__ __forceinline__ TileOrigin tile_origin(long m0, int H, int W) {
  TileOrigin o;
  const long q = m0 / W;
  o.w0 = (int)(m0 - q * W);
  o.h0 = (int)(q % H);
  o.rcp_w = __builtin_amdgcn_rcpf((float)W);  // approximate: fast_div corrects the quotient
  o.rcp_h = __builtin_amdgcn_rcpf((float)H);
  return o;
}

__device__ __forceinline__ int fast_div(int t, int d, float rcp) {
  int q = (int)((float)t * rcp);
  q -= (q * d > t) ? 1 : 0;
  q += ((q + 1) * d <= t) ? 1 : 0;
  return q;
}

__device__ __forceinline__ void pixel_hw(const TileOrigin& o, int r, int H, int W, bool valid, int& h, int& w) {
  const int t = o.w0 + r;
  const int dq = fast_div(t, W, o.rcp_w);
  w = t - dq * W;
  h = o.h0 + dq;
  if (h >= H) h -= fast_div(h, H, o.rcp_h) * H;  // the tile runs into the next frame
  if (!valid) h = -0x40000000;
}

// ================================================================ register-staged kernel
template <int BM, int BN>
constexpr int mfma_lds_bytes() {
  return (2 * (BM + BN) * 128) > (BM * (BN + 4) * 4) ? (2 * (BM + BN) * 128) : (BM * (BN + 4) * 4);
}

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv3x3_mfma(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int RB = 128;
  constexpr int CE = 16 / sizeof(T);  // elements per 16-byte chunk
  constexpr int GE = 64 / sizeof(T);  // elements per 64-byte granule
  constexpr int BKE = RB / sizeof(T);  // K elements per step
  constexpr int XR = BM / 32, WR = BN / 32;
  constexpr int WM = BM / 64, WN = BN / 64;
  static_assert(WM * WN == 4, "4 waves of 64x64");
  constexpr int STAGE = (BM + BN) * RB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int t = xcd_tile(blockIdx.x, a.tiles_total);
  const int mt = t / a.tiles_n, nt = t - mt * a.tiles_n;
  const long m0 = (long)mt * BM;
  const int n0 = nt * BN;
  const int H = a.H, W = a.W;
  const int chunk = tid & 7, rbase = tid >> 3;

  const long xbase = m0 - W - 1;  // lowest pixel any tap of this tile touches
  const __amdgpu_buffer_rsrc_t xrs = x_rsrc<T>(a, xbase);
  const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, n0);
  const TileOrigin org = tile_origin(m0, H, W);
  const int xcs = a.x_cstride;
  // per row: byte offset of the pixel relative to xbase, and a 9-bit mask of the taps that stay inside the
  // frame (bit 9, the K padding "tap", is never set) -> a K-step costs one bit test + add + select per load
  int pofs[XR], tmask[XR];
  int ph0, pw0;
  pixel_hw(org, rbase, H, W, true, ph0, pw0);
  const int pofs0 = (rbase + W + 1) * xcs * (int)sizeof(T);
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int r = rbase + 32 * i;
    int ph, pw;
    if (W >= 32) {  // rows of a lane are 32 pixels apart: at most one row wrap per step
      ph = ph0;
      pw = pw0;
      pw0 += 32;
      if (pw0 >= W) {
        pw0 -= W;
        ph0 = ph0 + 1 == H ? 0 : ph0 + 1;
      }
    } else {
      pixel_hw(org, r, H, W, true, ph, pw);
    }
    if (m0 + r >= a.M) ph = -0x40000000;
    pofs[i] = pofs0 + i * 32 * xcs * (int)sizeof(T);
    const int vr = (ph >= 1 && ph <= H) | ((ph >= 0 && ph < H) << 1) | ((ph >= -1 && ph < H - 1) << 2);
    const int vc = (pw >= 1) | (((unsigned)pw < (unsigned)W) << 1) | ((pw < W - 1) << 2);
    const int vcc = ((unsigned)pw < (unsigned)W) ? vc : 0;
    int m = 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) m |= (((vr >> (t / 3)) & (vcc >> (t % 3))) & 1) << t;
    tmask[i] = m;
  }
  uint4 xr[XR], wr[WR];
  const int wofs = (rbase * a.K_pad + chunk * CE) * (int)sizeof(T);
  const int wstride = 32 * a.K_pad * (int)sizeof(T);

  auto load = [&](int kt) {
    int tap, delta;
    if (a.chunk_major) {  // the step's two granules (chunks 0-3 and 4-7) decoded on the scalar unit
      const int g0 = 2 * kt, g1 = g0 + 1;
      const int cc0 = g0 / 9, cc1 = g1 / 9;
      const int tap0 = g0 < a.ng ? g0 - cc0 * 9 : 9, tap1 = g1 < a.ng ? g1 - cc1 * 9 : 9;
      const int d0 = (int)(((tap0 / 3 - 1) * W + tap0 % 3 - 1) * xcs + src_chan(a, cc0 * GE)) * (int)sizeof(T);
      const int d1 = (int)(((tap1 / 3 - 1) * W + tap1 % 3 - 1) * xcs + src_chan(a, cc1 * GE)) * (int)sizeof(T);
      const bool hi = chunk >= 4;
      tap = hi ? tap1 : tap0;
      delta = (hi ? d1 : d0) + (chunk & 3) * 16;
    } else {
      int c;
      k_to_tap<GE>(a, kt * BKE + chunk * CE, tap, c);
      delta = (int)(((tap / 3 - 1) * W + tap % 3 - 1) * xcs + src_chan(a, c)) * (int)sizeof(T);
    }
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int off = ((tmask[i] >> tap) & 1) ? pofs[i] + delta : OOB;
      xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int off = wofs + i * wstride + kt * RB;
      wr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 0));
    }
  };
  auto store = [&](int buf) {
    char* s = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < XR; ++i) *reinterpret_cast<uint4*>(s + swz<RB>(rbase + 32 * i, chunk)) = xr[i];
#pragma unroll
    for (int i = 0; i < WR; ++i) *reinterpret_cast<uint4*>(s + BM * RB + swz<RB>(rbase + 32 * i, chunk)) = wr[i];
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // f32: the products of one K-step chain into a fresh partial added to the running sum (two-level
  // summation, error ~(32 + K/32) ulp instead of K ulp for K up to 9216); bf16: one chain.
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
      for (int f = 0; f < 4; ++f)
        av[f] = *reinterpret_cast<const uint4*>(s + BM * RB + swz<RB>(wn * 64 + f * 16 + (lane & 15), ck));
#pragma unroll
      for (int f = 0; f < 4; ++f) bv[f] = *reinterpret_cast<const uint4*>(s + swz<RB>(wm * 64 + f * 16 + (lane & 15), ck));
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

  // fast epilogue (bf16 output, no softmax): y = act(acc * scale' + shift') in registers, bf16 rows staged
  // in LDS (4 channels = one ds_write_b64 per fragment), then 16-byte buffer stores whose descriptor ends at
  // the last pixel, so rows past M drop in hardware.
  if (sizeof(T) == 2 && a.y_dtype == VM_BF16 && a.act != VM_ACT_SOFTMAX && a.y_vec && (a.cout & 7) == 0) {
    constexpr int SR16 = BN * 2 + 16;  // staging row stride in bytes
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) {
      const int col = wn * 64 + fc * 16 + 4 * (lane >> 4);
      float mul[4], add[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = min(n0 + col + j, a.cout - 1);
        const float sc = a.scale ? a.scale[co] : 1.f;
        mul[j] = sc;
        add[j] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
      }
#pragma unroll
      for (int fp = 0; fp < 4; ++fp) {
        const int row = wm * 64 + fp * 16 + (lane & 15);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = fmaf(acc[fc][fp][j], mul[j], add[j]);
          if (a.act == VM_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
          else if (a.act == VM_ACT_SIGMOID) v[j] = sigmoid_precise(v[j]);
        }
        uint2 pk;
        pk.x = bf16x2_bits(v[0], v[1]);
        pk.y = bf16x2_bits(v[2], v[3]);
        *reinterpret_cast<uint2*>(smem + row * SR16 + col * 2) = pk;
      }
    }
    __syncthreads();
    constexpr int CPR = BN / 8;
    const int ycs2 = a.y_cstride * 2;
    const long rows_left = a.M - m0;
    const long rec = rows_left * (long)ycs2;
    uint16_t* Yb = reinterpret_cast<uint16_t*>(a.y) + a.y_coff + m0 * (long)a.y_cstride + n0;
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc(Yb, 0, rec > 0x7ffffff0L ? 0x7ffffff0 : (int)rec, 0x00020000);
#pragma unroll
    for (int it = 0; it < BM * CPR / 256; ++it) {
      const int idx = it * 256 + tid;
      const int rr = idx / CPR, cc = idx % CPR;
      const uint4 d = *reinterpret_cast<const uint4*>(smem + rr * SR16 + cc * 16);
      const int off = (n0 + cc * 8 < a.cout) ? rr * ycs2 + cc * 16 : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), yrs,
                                             off, 0, 0);
    }
    return;
  }

  // general epilogue: f32 staging in LDS, then coalesced 16-byte stores
  constexpr int SROW = BN + 4;
  float* stg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int fc = 0; fc < 4; ++fc) {
    const int col = wn * 64 + fc * 16 + 4 * (lane >> 4);
    float bsv[4] = {0.f, 0.f, 0.f, 0.f}, scv[4] = {1.f, 1.f, 1.f, 1.f}, shv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = min(n0 + col + j, a.cout - 1);  // clamped: always a valid address
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
      if (a.y_vec && co + 8 <= a.cout) *reinterpret_cast<uint4*>(dst) = Chunk<uint16_t>::pack(src);
      else
        for (int j = 0; j < 8 && co + j < a.cout; ++j) dst[j] = f2bf(src[j]);
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
      if (a.y_vec && co + 4 <= a.cout) *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
      else
        for (int j = 0; j < 4 && co + j < a.cout; ++j) dst[j] = src[j];
    }
  }
}

// ================================================================ LDS-DMA pipelined kernel
// Tiles are filled by buffer_load_dwordx4 ... lds (global -> LDS, no VGPRs, 1 KiB = 1024/RB operand rows
// per wave-instruction, called a "piece"):
//   * the LDS image is lane-linear, so the XOR swizzle moves to the SOURCE: the lane that fills physical
//     chunk p of row r fetches logical chunk p ^ f(r) (an involution; the MFMA reads use swz<RB>()).
//   * SAME padding / pixels past the end get an out-of-range buffer offset -> the DMA writes zeros.
//   * S-slot ring with 64-byte K-steps: slot kt%S is waited with a COUNTED vmcnt (up to S-2 younger
//     stages stay in flight), then one raw s_barrier per K-step publishes slot kt and frees slot (kt-1)%S,
//     which the pieces of K-step kt+S-1 refill while the MFMAs of K-step kt run.
// 8 waves of (BM/WM) pixels x 64 output channels each.
template <typename T, int RB, int BM, int BN, int WM, int WN, int S>
struct GldsCfg {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int TPM = BM / WM, TPN = BN / WN;
  static constexpr int FP = TPM / 16, FC = TPN / 16;
  static constexpr int RPP = 1024 / RB;           // operand rows per DMA piece
  static constexpr int XP = BM / RPP, WP = BN / RPP;  // pieces per stage
  static constexpr int XPW = XP / NW;              // X pieces per wave
  static constexpr int WPW = (WP + NW - 1) / NW;   // max W pieces per wave
  static constexpr int STAGE = (BM + BN) * RB;
  static constexpr int EPI = BM * (64 + 4) * 4;    // one 64-channel f32 slab
  static constexpr int LDS = (S * STAGE > EPI ? S * STAGE : EPI);
  static_assert(NW == 8, "8-wave blocks");
  static_assert(TPN == 64, "epilogue slabs are one wave-column (64 channels) wide");
  static_assert(XP % NW == 0, "whole X pieces per wave");
  static_assert(S >= 2 && S <= 8, "ring depth");
};

template <typename T, int RB, int BM, int BN, int WM, int WN, int S, bool FAST>
__global__ __launch_bounds__(512, 1) void conv3x3_glds(ConvArgs a) {
  using C = GldsCfg<T, RB, BM, BN, WM, WN, S>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CE = 16 / sizeof(T);
  constexpr int GE = 64 / sizeof(T);
  constexpr int BKE = RB / sizeof(T);
  constexpr int CPR = RB / 16;  // chunks per row
  constexpr int FP = C::FP, FC = C::FC, XPW = C::XPW, WPW = C::WPW, NT = C::NT, NW = C::NW;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int t = xcd_tile(blockIdx.x, a.tiles_total);
  const int mt = t / a.tiles_n, nt = t - mt * a.tiles_n;
  const long m0 = (long)mt * BM;
  const int n0 = nt * BN;
  const int H = a.H, W = a.W;

  const long xbase = m0 - W - 1;
  const __amdgpu_buffer_rsrc_t xrs = x_rsrc<T>(a, xbase);
  const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, n0);

  // this lane's DMA rows: X piece i of this wave fills rows (wave + i*NW)*RPP + lane/CPR, physical chunk lane%CPR
  const int lrow = lane / CPR, lpos = lane % CPR;
  const TileOrigin org = tile_origin(m0, H, W);
  int prow[XPW], ph[XPW], pw[XPW], xq[XPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int row = (wave + i * NW) * C::RPP + lrow;
    xq[i] = (swz<RB>(row, lpos) - row * RB) >> 4;  // logical chunk that belongs in physical chunk lpos
    prow[i] = row + W + 1;
    pixel_hw(org, row, H, W, m0 + row < a.M, ph[i], pw[i]);
  }
  int woff[WPW];
  int nwp = 0;  // W pieces of this wave (wave-uniform)
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int piece = wave + i * NW;
    const int row = piece * C::RPP + lrow;
    woff[i] = (row * a.K_pad + ((swz<RB>(row, lpos) - row * RB) >> 4) * CE) * (int)sizeof(T);
    if (piece < C::WP) ++nwp;
  }
  const int lps = XPW + nwp;  // DMA pieces this wave issues per stage
  const int xcs = a.x_cstride;

  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  auto issue = [&](int kt, int slot) {
    const uint32_t sbase = lds0 + slot * C::STAGE;
    int tapu = 0, c0 = 0;
    if (FAST && RB == 64) {  // one granule per K-step: tap and channel base are wave-uniform
      const int cc = kt / 9;
      tapu = kt - cc * 9;
      c0 = cc * GE;
    }
#pragma unroll
    for (int i = 0; i < XPW; ++i) {
      int tap, c;
      if (FAST && RB == 64) {
        tap = tapu;
        c = c0 + xq[i] * CE;
      } else {
        k_to_tap<GE>(a, kt * BKE + xq[i] * CE, tap, c);
      }
      const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
      const int hh = ph[i] + dh, ww = pw[i] + dw;
      const bool ok = tap < 9 && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      const int off = ok ? ((prow[i] + dh * W + dw) * xcs + c) * (int)sizeof(T) : OOB;
      glds16(xrs, sbase + (wave + i * NW) * 1024, off);
    }
    const int kb = kt * RB;
#pragma unroll
    for (int i = 0; i < WPW; ++i)
      if (wave + i * NW < C::WP) glds16(wrs, sbase + BM * RB + (wave + i * NW) * 1024, woff[i] + kb);
  };

  f32x4 acc[FC][FP];
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool SPLIT = sizeof(T) == 4;
  auto compute = [&](int slot) {
    const char* sp = smem + slot * C::STAGE;
    f32x4 part[SPLIT ? FC : 1][SPLIT ? FP : 1];
    if constexpr (SPLIT) {
#pragma unroll
      for (int i = 0; i < FC; ++i)
#pragma unroll
        for (int j = 0; j < FP; ++j) part[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kb = 0; kb < RB / 64; ++kb) {
      const int ck = kb * 4 + (lane >> 4);
      uint4 av[FC], bv[FP];
#pragma unroll
      for (int f = 0; f < FC; ++f)
        av[f] = *reinterpret_cast<const uint4*>(sp + BM * RB + swz<RB>(wn * 64 + f * 16 + (lane & 15), ck));
#pragma unroll
      for (int f = 0; f < FP; ++f)
        bv[f] = *reinterpret_cast<const uint4*>(sp + swz<RB>(wm * C::TPM + f * 16 + (lane & 15), ck));
#pragma unroll
      for (int fc = 0; fc < FC; ++fc)
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          if constexpr (SPLIT) mma16<T>(av[fc], bv[fp], part[fc][fp]);
          else mma16<T>(av[fc], bv[fp], acc[fc][fp]);
        }
    }
    if constexpr (SPLIT) {
#pragma unroll
      for (int i = 0; i < FC; ++i)
#pragma unroll
        for (int j = 0; j < FP; ++j) acc[i][j] += part[i][j];
    }
  };

  const int nk = a.nk;
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once only the min(S-2, nk-1-kt) younger stages are still in flight
    wait_vm(min(S - 2, nk - 1 - kt) * lps);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (fragment reads of the slot refilled below: see conv3x3_patch)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + S - 1 < nk) {
      int ns = slot + S - 1;
      ns -= ns >= S ? S : 0;
      issue(kt + S - 1, ns);
    }
    compute(slot);
    slot = slot + 1 == S ? 0 : slot + 1;
  }

  // ---------------------------------------------------------------- epilogue, one 64-channel slab at a time
  constexpr int SROW = 64 + 4;
  float* stg = reinterpret_cast<float*>(smem);
  for (int sl = 0; sl < WN; ++sl) {
    asm volatile("" ::: "memory");
    __syncthreads();
    if (wn == sl) {
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        const int col = fc * 16 + 4 * (lane >> 4);
        float bsv[4] = {0.f, 0.f, 0.f, 0.f}, scv[4] = {1.f, 1.f, 1.f, 1.f}, shv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = min(n0 + wn * 64 + col + j, a.cout - 1);
          if (a.bias) bsv[j] = a.bias[co];
          if (a.scale) scv[j] = a.scale[co];
          if (a.shift) shv[j] = a.shift[co];
        }
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          const int row = wm * C::TPM + fp * 16 + (lane & 15);
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
    }
    __syncthreads();
    const int nb = n0 + sl * 64;
    if (a.y_dtype == VM_BF16) {
      uint16_t* Y = reinterpret_cast<uint16_t*>(a.y) + a.y_coff;
      for (int idx = tid; idx < BM * 8; idx += NT) {
        const int rr = idx >> 3, cc = idx & 7;
        const long p = m0 + rr;
        const int co = nb + cc * 8;
        if (p >= a.M || co >= a.cout) continue;
        const float* src = stg + rr * SROW + cc * 8;
        uint16_t* dst = Y + p * (long)a.y_cstride + co;
        if (a.y_vec && co + 8 <= a.cout) *reinterpret_cast<uint4*>(dst) = Chunk<uint16_t>::pack(src);
        else
          for (int j = 0; j < 8 && co + j < a.cout; ++j) dst[j] = f2bf(src[j]);
      }
    } else {
      float* Y = reinterpret_cast<float*>(a.y) + a.y_coff;
      for (int idx = tid; idx < BM * 16; idx += NT) {
        const int rr = idx >> 4, cc = idx & 15;
        const long p = m0 + rr;
        const int co = nb + cc * 4;
        if (p >= a.M || co >= a.cout) continue;
        const float* src = stg + rr * SROW + cc * 4;
        float* dst = Y + p * (long)a.y_cstride + co;
        if (a.y_vec && co + 4 <= a.cout) *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
        else
          for (int j = 0; j < 4 && co + j < a.cout; ++j) dst[j] = src[j];
      }
    }
  }
}

// ================================================================ patch kernel (bf16, chunk-major K)
// 2-D output tile of 8 x 32 pixels.  Per 64-byte channel granule the (8+2) x (32+2) input patch is DMA'd to
// LDS ONCE and serves all 9 taps: the MFMA pixel fragments of tap (dh, dw) are the patch rows shifted by
// (dh+1)*34 + dw+1, so the input costs 1.33x its bytes per granule instead of 9x.  Weights stream per tap
// (granule order cc*9+tap is exactly the chunk-major packing) through an S-slot ring.  LDS-DMA with the
// 64-byte-row XOR swizzle applied at the source (conflict-free fragment reads for any start row); counted
// vmcnt per wave + one barrier per step; dummy (out-of-range) pieces past the end keep the counts uniform.
template <int BN, int WM, int WN, int S, int TH_ = 8, int G_ = 1>
struct PatchCfg {
  static constexpr int G = G_;                               // taps per weight-ring slot (one barrier per slot)
  static constexpr int TH = TH_, TW = 32, BM = TH * TW;
  static constexpr int PW = TW + 2, PPIX = (TH + 2) * PW;  // 340 patch pixels
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int XP = (PPIX + 15) / 16;                // 22 DMA pieces per patch
  static constexpr int XPW = (XP + NW - 1) / NW;             // max X pieces per wave
  static constexpr int PB = XP * 1024;
  static constexpr int WP = BN / 16;                         // DMA pieces per weight slot
  static constexpr int WPW = (WP + NW - 1) / NW;
  static constexpr int WSLOT = BN * 64;
  static constexpr int TPM = BM / WM, TPN = BN / WN;
  static constexpr int FP = TPM / 16, FC = TPN / 16;
  static constexpr int SR = 64 * 2 + 16;                    // epilogue staging row (one 64-channel slab, bf16)
  static constexpr int SR32 = 64 * 4 + 16;                  // the same slab in f32 (f32 output views)
  static constexpr int EPI = BM * SR32;
  static constexpr int MAIN = 2 * PB + S * G * WSLOT;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static constexpr int IW = TW + 4, IPIX = (TH + 4) * IW;   // FIRST: 8-channel input patch (16 B per pixel)
  static constexpr int LDS_FIRST = MAIN + IPIX * 16 > EPI ? MAIN + IPIX * 16 : EPI;
  // register epilogue (vm_set_option "patch_repi"): a wave's pixel fragments must cover 2 whole rows so the fused
  // 2x2 pool pairs rows inside the wave; 32-pixel waves of 8 x 32 / 4 x 32 tiles (TH == WM) are remapped to 2 rows x
  // 16 pixels (wave pair 2k, 2k+1 = rows 2k, 2k+1), 64-pixel waves already hold 2 rows x 32 pixels.  Either way every
  // output pixel keeps its MFMA sequence, so results do not depend on the mapping.
  static constexpr bool REMAP = TPM == 32 && TW == 32 && WM % 2 == 0 && TH == WM;
  static constexpr bool REPI_OK = G == 3 && (REMAP || TPM == 64);
  static constexpr int PSTEP = REMAP ? 1 : 2;  // pixel fragment of the row below fragment fp (pool partner)
  __device__ static int prow(int wm, int fp) { return REMAP ? 2 * (wm >> 1) + fp : (wm * TPM + fp * 16) / TW; }
  __device__ static int pcol(int wm, int fp) { return REMAP ? 16 * (wm & 1) : (wm * TPM + fp * 16) % TW; }
  __device__ static int tpix(int wm, int fp) { return prow(wm, fp) * TW + pcol(wm, fp); }  // first tile pixel
  static_assert(TPN % 64 == 0, "whole 64-channel epilogue slabs per wave column");
  static_assert(TPM % 32 == 0 || TPM == 16, "pixel fragments stay inside one patch row");
  static_assert(G == 1 || G == 3, "a slot holds one tap or one kernel row");
  static_assert(G == 1 ? (S >= 3 && S <= 9) : (S >= 2 && S <= 4), "ring depth (the X group is counted in at most one window)");
};

// First conv (cin <= 8 -> 64 channels, + bias + relu) of the patch pixels, for the FIRST patch kernel.  The 8-channel
// input patch (TH+4) x (TW+4) is staged at ip; 16-pixel fragments of the (TH+2) x (TW+2) patch are spread over the
// waves; a 32-deep K-step covers 4 taps x 8 channels (tap-major packing k = tap*8 + c, like conv3x3_first).
template <class C>
__device__ __forceinline__ void first_layer_patch(const ConvArgs& a, char* smem, int pb, char* ip, int n, int r0, int c0,
                                                  int wave, int lane, int tid) {
  using T = uint16_t;
  const int H = a.H, W = a.W;
  const T* x8 = reinterpret_cast<const T*>(a.x) + a.x_coff;
  const float* xf = reinterpret_cast<const float*>(a.x) + a.x_coff;
  for (int i = tid; i < C::IPIX; i += C::NT) {
    const int ir = i / C::IW, ic = i - ir * C::IW;
    const int h = r0 - 2 + ir, w = c0 - 2 + ic;
    uint4 v = make_uint4(0, 0, 0, 0);
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
      const long pix = (((long)n * H + h) * W + w) * (long)a.x_cstride;
      if (a.x_f32) {  // the caller's f32 frame (loader.py:76-78 layout), rounded to bf16 like vm_convert_nhwc
        // (measured: one pixel per lane beats a coalesced channel-pair sweep, whose extra LDS stores cost more)
        float f[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) f[c] = c < a.x_c ? xf[pix + c] : 0.f;
        v = Chunk<T>::pack(f);
      } else {
        v = *reinterpret_cast<const uint4*>(x8 + pix);
      }
    }
    *reinterpret_cast<uint4*>(ip + i * 16) = v;
  }
  const int col = lane & 15, q = lane >> 4;
  const T* w1 = reinterpret_cast<const T*>(a.w1);
  uint4 wf[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) wf[j][fc] = *reinterpret_cast<const uint4*>(w1 + (fc * 16 + col) * 128 + j * 32 + q * 8);
  float b1[4][4];
#pragma unroll
  for (int fc = 0; fc < 4; ++fc)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) b1[fc][jj] = a.bias1 ? a.bias1[fc * 16 + 4 * q + jj] : 0.f;
  __syncthreads();
  constexpr int NF = (C::PPIX + 15) / 16;
  for (int f = wave; f < NF; f += C::NW) {
    const int p = f * 16 + col;
    const int pr = p / C::PW, pc = p - pr * C::PW;
    f32x4 acc[4];
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) acc[fc] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int tap = 4 * j + q;
      uint4 bv = make_uint4(0, 0, 0, 0);
      if (tap < 9 && p < C::PPIX) bv = *reinterpret_cast<const uint4*>(ip + ((pr + tap / 3) * C::IW + pc + tap % 3) * 16);
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) mma16<T>(wf[j][fc], bv, acc[fc]);
    }
    const int h = r0 - 1 + pr, w = c0 - 1 + pc;
    const bool inside = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    if (p < C::PPIX) {
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        float v[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[jj] = inside ? fmaxf(acc[fc][jj] + b1[fc][jj], 0.f) : 0.f;
        uint2 pk;
        pk.x = bf16x2_bits(v[0], v[1]);
        pk.y = bf16x2_bits(v[2], v[3]);
        // channel fc*16 + 4q: granule fc/2, 16-byte chunk (fc&1)*2 + q/2, half q&1
        *reinterpret_cast<uint2*>(smem + (fc >> 1) * pb + swz<64>(p, (fc & 1) * 2 + (q >> 1)) + (q & 1) * 8) = pk;
      }
    }
  }
  __syncthreads();
}

// FIRST: the conv's 64-channel input is itself conv3x3(x8) + bias + relu of an 8-channel frame (unet.py:170-171,
// conv1_1 -> conv1_2): the prologue evaluates that first conv on the (TH+2) x (TW+2) patch straight into the two
// granule buffers (zero outside the frame = the second conv's SAME padding), so the 64-channel activation never
// touches HBM; the main loop then streams only weights.
// UPSKIP: the folded-upconv instantiation (vm_conv3x3_up2x_nhwc), which skips its phase filters' zero taps
// MT: the MFMA operand type (uint16_t = bf16; f16_t = the split-fp16 forward's fp16 parts, same data path)
template <int BN, int WM, int WN, int S, int TH, int MINB, int UNR, bool PF, int ABL, bool FIRST, int G = 1,
          bool UPSKIP = false, typename MT = uint16_t>
__global__ __launch_bounds__(64 * WM * WN)
__attribute__((amdgpu_waves_per_eu((UPSKIP || G > 1) && MINB * WM * WN < 16 ? 4 : MINB * WM * WN / 4)))  // <= 128 VGPRs
void conv3x3_patch(ConvArgs a) {
  using C = PatchCfg<BN, WM, WN, S, TH, G>;
  using T = uint16_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NW = C::NW, NT = C::NT, FP = C::FP, FC = C::FC, XPW = C::XPW, WPW = C::WPW;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.prio && NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int wm = wave % WM, wn = wave / WM;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int VW = a.vstride ? a.vW : W;  // packed frames: one virtual image (n = 0), ConvArgs::vstride
  const int th = (H + C::TH - 1) / C::TH, tw = (VW + C::TW - 1) / C::TW;
  int st, nt;
  if (a.cband) {  // channel-banded: XCD b % 8 owns output tiles [xcd * cband, +cband) over every pixel tile
    const int i = blockIdx.x >> 3;
    st = i / a.cband;
    nt = (blockIdx.x & 7) * a.cband + (i - st * a.cband);
  } else if (a.ngroup) {  // grouped: ngroup output tiles x every pixel tile, group after group (XCD ranges within)
    const int t = xcd_tile(blockIdx.x, a.tiles_total);
    const int per = (a.tiles_total / a.tiles_n) * a.ngroup, gi = t / per, r = t - gi * per;
    st = r / a.ngroup;
    nt = gi * a.ngroup + (r - st * a.ngroup);
  } else {
    const int t = xcd_tile(blockIdx.x, a.tiles_total);
    st = t / a.tiles_n;
    nt = t - st * a.tiles_n;
  }
  const int n = st / (th * tw), srem = st - n * th * tw;
  const int r0 = (srem / tw) * C::TH, c0 = (srem - (srem / tw) * tw) * C::TW;
  const int n0 = nt * BN;
  // pixel offset (in pixels, from row r0 of the tile's frame / of frame 0 when packed) of tile pixel (pr, pc) of
  // the output; ok says whether it is a real output pixel
  auto out_pix = [&](int pr, int pc, bool& ok) {
    const int v = c0 + pc;
    if (a.vstride) {
      const int f = v / a.vstride, x = v - f * a.vstride;
      ok = r0 + pr < H && x < W && v < VW;
      return (f * H + pr) * W + x;
    }
    ok = r0 + pr < H && v < W;
    return pr * W + pc;
  };

  const T* xb = reinterpret_cast<const T*>(a.x) + a.x_coff + ((long)n * H + r0 - 1) * (long)W * cs;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(xb), 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, n0);

  // DMA geometry: piece k fills 16 LDS rows (4 lanes x 16 B per row); the lane filling physical chunk lpos of
  // row r fetches logical chunk swz(r, lpos)
  const int lrow = lane >> 2, lpos = lane & 3;
  int xoff[XPW];
  int x_n = 0;
#pragma unroll
  for (int i = 0; i < XPW && !FIRST; ++i) {
    const int piece = wave + i * NW;
    const int row = piece * 16 + lrow;
    const int lq = (swz<64>(row, lpos) - row * 64) >> 4;
    const int pr = row / C::PW, pc = row - pr * C::PW;
    int h = r0 - 1 + pr, w = c0 - 1 + pc;
    if (a.up) {  // folded 2x resize: past the bottom/right edge the low-res frame is replicated (TF1 clamp)
      h = min(h, H - 1);
      w = min(w, W - 1);
    }
    bool ok = row < C::PPIX && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)VW;
    int pix = (h - r0 + 1) * W + w;
    if (a.vstride && ok) {  // virtual column -> (frame, column); the two columns past a frame read as zero
      const int f = w / a.vstride, x = w - f * a.vstride;
      ok = x < W;
      pix = (f * H + h - r0 + 1) * W + x;
    }
    xoff[i] = ok ? (pix * cs + lq * 8) * 2 : OOB;
    if (piece < C::XP) ++x_n;
  }
  int woff[WPW];
  int w_n = 0;
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int piece = wave + i * NW;
    const int row = piece * 16 + lrow;
    const int lq = (swz<64>(row, lpos) - row * 64) >> 4;
    woff[i] = (row * a.K_pad + lq * 8) * 2;
    if (piece < C::WP) ++w_n;
  }
  const int nch_all = a.cin_pad / 32;
  const int ksp = a.ksplit > 1 ? a.ksplit : 1;
  const int per_split = (nch_all + ksp - 1) / ksp;  // host: every split non-empty
  const int cc_beg = (int)blockIdx.y * per_split;
  const int nch = min(nch_all, cc_beg + per_split), nsteps = nch * 9;  // end granule / step of this split
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const uint32_t wring = lds0 + 2 * C::PB;

  auto issue_x = [&](int cc, int buf) {
    if constexpr (FIRST) return;
    const bool real = cc < nch;
#pragma unroll
    for (int i = 0; i < XPW; ++i)
      if (wave + i * NW < C::XP)
        glds16(xrs, lds0 + buf * C::PB + (wave + i * NW) * 1024, real ? xoff[i] + (int)src_chan(a, cc * 32) * 2 : OOB);
  };
  auto issue_w = [&](int s, int slot) {  // ring step s = taps s*G .. s*G+G-1 (chunk-major K: consecutive 64 B)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool real = s * G + g < nsteps;
#pragma unroll
      for (int i = 0; i < WPW; ++i)
        if (wave + i * NW < C::WP)
          glds16(wrs, wring + (slot * G + g) * C::WSLOT + (wave + i * NW) * 1024, real ? woff[i] + (s * G + g) * 64 : OOB);
    }
  };

  int boff[FC], abase[FP];
#pragma unroll
  for (int f = 0; f < FC; ++f) boff[f] = 2 * C::PB + swz<64>(wn * C::TPN + f * 16 + (lane & 15), lane >> 4);
#pragma unroll
  for (int f = 0; f < FP; ++f) {
    abase[f] = C::prow(wm, f) * C::PW + C::pcol(wm, f) + (lane & 15);
  }
  const int ck = lane >> 4;

  f32x4 acc[FC][FP];
#pragma unroll
  for (int i = 0; i < FC; ++i)
#pragma unroll
    for (int j = 0; j < FP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto frags = [&](uint4 (&av)[FC], uint4 (&bv)[FP], int slot, int buf, int tap) {
    const char* wp = smem + (slot * G + (G == 1 ? 0 : tap % G)) * C::WSLOT;
    const char* xp = smem + buf * C::PB;
#pragma unroll
    for (int f = 0; f < FC; ++f) av[f] = *reinterpret_cast<const uint4*>(wp + boff[f]);
    const int toff = (tap / 3) * C::PW + tap % 3;
#pragma unroll
    for (int f = 0; f < FP; ++f) {
      int row = abase[f] + toff;
      if constexpr (FC * FP >= 16) asm volatile("" : "+v"(row));  // recompute per step: no 9-tap address table
      bv[f] = *reinterpret_cast<const uint4*>(xp + swz<64>(row, ck));
    }
  };
  // counted DMA wait, then lgkmcnt(0): this wave's fragment reads of the ring slot / patch buffer that the DMAs
  // issued right after the barrier refill must have returned before the barrier — the MFMAs consuming them may be
  // scheduled past it (seen in the 4 x 32 folded-upconv instantiation: under a second process on the GPU the refill
  // overtook a queued ds_read about once per 100 frames)
  auto sync = [&](int n) {
    wait_vm(n);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // folded 2x resize: the TF1 legacy upsampling makes an odd output row (phase a = 1) a blend of low-res rows i and
  // i+1 only, so its phase filter's kernel row 0 (offset -1) is exactly zero; likewise kernel column 0 for odd
  // output columns (b = 1).  A block whose channels are one phase skips those taps' fragment reads and MFMAs:
  // phases (0,0) / (0,1) / (1,0) / (1,1) run 9 / 6 / 6 / 4 of the 9 taps (25 of 36, bit-identical: the skipped
  // products are exact zeros).  The weight DMA and the barriers keep their schedule: the folded convs are
  // latency-bound on that ring, and a variant that also dropped the zero rows from the ring (shorter prefetch cover)
  // measured 1.3 % slower on the whole forward, this one 0.3 % faster (same-box A/B, tools/ab_unet.py).
  const int up_phase = UPSKIP && a.up && n0 / a.up_cout == (n0 + BN - 1) / a.up_cout ? n0 / a.up_cout : 0;
  const bool skip_r0 = (up_phase >> 1) != 0 && (a.upmask & 1), skip_c0 = (up_phase & 1) != 0 && (a.upmask & 2);

  if constexpr (G > 1) {
    // one ring slot = one kernel row (G = 3 taps): one barrier per row; inside the row the fragments of tap g+1 are
    // read while tap g's MFMAs run (same slot and patch, no synchronisation needed)
    static_assert(!PF && !FIRST, "row-slot pipeline: plain configuration only");
    constexpr int R = 9 / G;
    issue_x(cc_beg, cc_beg & 1);
#pragma unroll
    for (int j = 0; j < S - 1; ++j) issue_w(cc_beg * R + j, j);
    int slot = 0;
    for (int cc = cc_beg; cc < nch; ++cc) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = cc * R + r;
        // in flight after W(k): S-2 younger row slots, plus the next patch when it was issued inside that window
        // timing ablations (results are garbage): ABL&4 no synchronisation, ABL&8 barrier without the DMA wait,
        // ABL&2 no DMA, ABL&1 no MFMA
        if constexpr (ABL & 8) {
          asm volatile("" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        } else if constexpr (!(ABL & 4)) {
          sync((S - 2) * G * w_n + ((r >= 1 && r <= S - 2) ? x_n : 0));
        }
        if constexpr (!(ABL & 2)) {
          if (r == 0) issue_x(cc + 1, (cc + 1) & 1);
          int ns = slot + S - 1;
          ns -= ns >= S ? S : 0;
          issue_w(k + S - 1, ns);
        }
        if (!(UPSKIP && skip_r0 && r == 0)) {  // (a folded upconv's zero kernel row: no reads, no MFMAs)
          uint4 av[2][FC], bv[2][FP];
          frags(av[0], bv[0], slot, cc & 1, r * G);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (g + 1 < G) frags(av[(g + 1) & 1], bv[(g + 1) & 1], slot, cc & 1, r * G + g + 1);
            if constexpr (ABL & 1) {
#pragma unroll
              for (int fc = 0; fc < FC; ++fc) asm volatile("" ::"v"(av[g & 1][fc].x), "v"(av[g & 1][fc].w));
#pragma unroll
              for (int fp = 0; fp < FP; ++fp) asm volatile("" ::"v"(bv[g & 1][fp].x), "v"(bv[g & 1][fp].w));
            } else if (!(UPSKIP && skip_c0 && g == 0)) {  // (its zero kernel column: no MFMAs)
#pragma unroll
              for (int fc = 0; fc < FC; ++fc)
#pragma unroll
                for (int fp = 0; fp < FP; ++fp) mma16<MT>(av[g & 1][fc], bv[g & 1][fp], acc[fc][fp]);
            }
          }
        }
        // schedule experiments (ABL 16 / 32): pin the order of the row's fragment reads and MFMAs
        if constexpr (ABL & 16) {  // all reads of tap g+1 issued ahead of tap g's MFMAs
          __builtin_amdgcn_sched_group_barrier(0x100, FC + FP, 0);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (g + 1 < G) __builtin_amdgcn_sched_group_barrier(0x100, FC + FP, 0);
            __builtin_amdgcn_sched_group_barrier(0x8, FC * FP, 0);
          }
        } else if constexpr (ABL & 32) {  // tap g+1's reads spread one per MFMA of tap g
          __builtin_amdgcn_sched_group_barrier(0x100, FC + FP, 0);
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < FC * FP; ++i) {
              __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
              if (g + 1 < G && i < FC + FP) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        }
        slot = slot + 1 == S ? 0 : slot + 1;
      }
    }
  } else if constexpr (PF) {
    // fragments of step s+1 are read right after the barrier of step s, while step s's MFMAs run; the ring
    // holds S steps (slot s%S is refilled with step s+S once every wave has its step-s fragments in registers)
    issue_x(0, 0);
    issue_x(1, 1);
#pragma unroll
    for (int j = 0; j < S; ++j) issue_w(j, j);
    sync((S - 1) * w_n);
    uint4 av[FC], bv[FP];
    frags(av, bv, 0, 0, 0);
    int slot = 0;
    for (int cc = 0; cc < nch; ++cc) {
#pragma unroll UNR
      for (int tap = 0; tap < 9; ++tap) {
        const int s = cc * 9 + tap;
#pragma unroll
        for (int fc = 0; fc < FC; ++fc)
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mma16<MT>(av[fc], bv[fp], acc[fc][fp]);
        if (s + 1 < nsteps) {
          // in flight after W(s+1): S-2 younger weight steps, plus the patch issued at the end of the last chunk
          sync((S - 2) * w_n + ((tap <= S - 2 && cc >= 1) ? x_n : 0));
          issue_w(s + S, slot);
          if (tap == 8) issue_x(cc + 2, cc & 1);
          slot = slot + 1 == S ? 0 : slot + 1;
          frags(av, bv, slot, tap == 8 ? (cc + 1) & 1 : cc & 1, tap == 8 ? 0 : tap + 1);
        }
      }
    }
  } else {
    issue_x(0, 0);
#pragma unroll
    for (int j = 0; j < S - 1; ++j) issue_w(j, j);
    if constexpr (FIRST) first_layer_patch<C>(a, smem, C::PB, smem + C::MAIN, n, r0, c0, wave, lane, tid);
    int slot = 0;
    for (int cc = 0; cc < nch; ++cc) {
#pragma unroll UNR
      for (int tap = 0; tap < 9; ++tap) {
        const int s = cc * 9 + tap;
        // in flight after W(s): S-2 younger weight slots, plus the next patch when it was issued inside the window
        if constexpr (!(ABL & 4)) sync((S - 2) * w_n + ((tap >= 1 && tap <= S - 2) ? x_n : 0));
        if constexpr (!(ABL & 2)) {
          if (tap == 0) issue_x(cc + 1, (cc + 1) & 1);
          int ns = slot + S - 1;
          ns -= ns >= S ? S : 0;
          issue_w(s + S - 1, ns);
        }
        uint4 av[FC], bv[FP];
        frags(av, bv, slot, cc & 1, tap);
        if constexpr (!(ABL & 1)) {  // (no zero-tap skipping here: it made this pipeline spill)
#pragma unroll
          for (int fc = 0; fc < FC; ++fc)
#pragma unroll
            for (int fp = 0; fp < FP; ++fp) mma16<MT>(av[fc], bv[fp], acc[fc][fp]);
        } else {  // keep the fragment reads alive without the MFMAs
#pragma unroll
          for (int fc = 0; fc < FC; ++fc) asm volatile("" ::"v"(av[fc].x), "v"(av[fc].w));
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) asm volatile("" ::"v"(bv[fp].x), "v"(bv[fp].w));
        }
        if constexpr (FC * FP >= 32) __builtin_amdgcn_sched_barrier(0);  // no cross-tap hoisting: registers
        slot = slot + 1 == S ? 0 : slot + 1;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: one 64-channel slab per wave column, bf16 staged, 16-byte buffer stores (masked by OOB offsets)
  // a.up (folded 2x resize, vm_conv3x3_up2x_nhwc): output channel n0+sl*64+c is phase p = (a,b) of channel
  // c' = (n0+sl*64) - p*up_cout + c, stored at full-res pixel (2*h+a, 2*w+b) of the [N,2H,2W,up_cout] view
  const int ycs2 = a.y_cstride * 2;
  const int YW = a.up ? 2 * W : W;
  T* yb = reinterpret_cast<T*>(a.y) + a.y_coff +
          (a.up ? (((long)n * 2 * H + 2 * r0) * YW + 2 * c0) : (((long)n * H + r0) * W + (a.vstride ? 0 : c0))) *
              (long)a.y_cstride;
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yb, 0, 0x7ffffff0, 0x00020000);
  constexpr int SPW = C::TPN / 64;  // 64-channel slabs per wave column
  const bool splitk = a.ksplit > 1;
  if (a.y_dtype == VM_F32 || splitk) {
    // f32 output (the training step's pre-BN buffers, unet_simple.py:19-27) or a split-K partial: f32 slab staging,
    // 4 channels per 16-byte store; no fused pool / folded resize on this path (host-checked)
    const int ycs = splitk ? a.cout : a.y_cstride;
    const long pix0 = ((long)n * H + r0) * W + (a.vstride ? 0 : c0);
    float* yf = splitk ? a.part + (long)blockIdx.y * a.M * a.cout + pix0 * ycs
                       : reinterpret_cast<float*>(a.y) + a.y_coff + pix0 * ycs;
    const __amdgpu_buffer_rsrc_t yfr = __builtin_amdgcn_make_buffer_rsrc(yf, 0, 0x7ffffff0, 0x00020000);
    const int ycs4 = ycs * 4;
    // split-fp16 x3 output (ConvArgs::ysplit): the same f32 staging, then 8 channels per thread split into [l, h, h]
    const bool ysp = a.ysplit > 0 && !splitk;
    // (a folded upconv's split output: [N, 2H, 2W] pixels from (2 r0, 2 c0), as the bf16 epilogues' yb)
    uint16_t* ys = reinterpret_cast<uint16_t*>(a.y) + a.y_coff +
                   (a.up ? ((long)n * 2 * H + 2 * r0) * YW + 2 * c0 : pix0) * (long)a.y_cstride;
    const __amdgpu_buffer_rsrc_t ysr = __builtin_amdgcn_make_buffer_rsrc(ys, 0, 0x7ffffff0, 0x00020000);
    bool ovf = false;
    for (int sl = 0; sl < BN / 64; ++sl) {
      const int cb = n0 + sl * 64;
      __syncthreads();
      if (wn == sl / SPW) {
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          if (fc / 4 != sl % SPW) continue;
          const int col = (fc % 4) * 16 + 4 * (lane >> 4);
          // (a folded upconv, split output only: the slab is one phase of up_cout channels, ConvArgs::up)
          const int uph = a.up ? cb / a.up_cout : 0;
          const int cbp = cb - uph * a.up_cout, ccap = a.up ? a.up_cout : a.cout;
          float mul[4], add[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int co = min(cbp + col + j, ccap - 1);
            const float sc = (a.scale && !splitk) ? a.scale[co] : 1.f;
            mul[j] = sc;
            add[j] = splitk ? 0.f : (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
          }
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) {
            const int row = C::tpix(wm, fp) + (lane & 15);
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              v[j] = fmaf(acc[fc][fp][j], mul[j], add[j]);
              if (!splitk && a.act == VM_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
              else if (!splitk && a.act == VM_ACT_SIGMOID) v[j] = sigmoid_precise(v[j]);
            }
            *reinterpret_cast<float4*>(smem + row * C::SR32 + col * 4) = make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
      __syncthreads();
      if (ysp) {
        const int S2 = a.ysplit * 2;
        const bool y3 = 3 * a.ysplit <= a.y_cstride;  // the third slab [h again] where the pixel row holds it
#pragma unroll
        for (int it = 0; it < C::BM * 8 / NT; ++it) {
          const int idx = it * NT + tid;
          const int rr = idx >> 3, cq = idx & 7;
          const float4 d0 = *reinterpret_cast<const float4*>(smem + rr * C::SR32 + cq * 32);
          const float4 d1 = *reinterpret_cast<const float4*>(smem + rr * C::SR32 + cq * 32 + 16);
          const float v[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
          const int pr = rr / C::TW, pc = rr % C::TW;
          bool ok;
          int pix = out_pix(pr, pc, ok);
          const int uph = a.up ? cb / a.up_cout : 0;
          const int cbp = cb - uph * a.up_cout;  // (the phase's own channel, a.up)
          ok = ok && cbp + cq * 8 < (a.up ? a.up_cout : a.cout);
          if (a.up) pix = (2 * pr + (uph >> 1)) * YW + 2 * pc + (uph & 1);
          uint4 hv, lv;
          const bool o = split3h_chunk(v, hv, lv);
          ovf |= ok && o;
          const int off = ok ? pix * ycs2 + (cbp + cq * 8) * 2 : OOB;
          const int off1 = ok ? off + S2 : OOB, off2 = ok ? off + 2 * S2 : OOB;
          typedef __attribute__((ext_vector_type(4))) unsigned u4_t;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, lv), ysr, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, hv), ysr, off1, 0, 0);
          if (y3) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, hv), ysr, off2, 0, 0);
        }
        if (a.py) {
          // the split of the fused 2x2 SAME max-pool (unet.py:32-33) of the staged f32 slab, as the bf16 path's
          // pool: tiles start on even rows / columns, taps past the frame edge never win
          const int PH = (H + 1) >> 1, PW = (W + 1) >> 1;
          const int pr0 = r0 >> 1, pc0 = c0 >> 1;
          uint16_t* pbs = reinterpret_cast<uint16_t*>(a.py) + a.py_coff +
                          (((long)n * PH + pr0) * PW + (a.vstride ? 0 : pc0)) * (long)a.py_cstride + n0;
          const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pbs, 0, 0x7ffffff0, 0x00020000);
          const int P2 = a.psplit * 2;
          constexpr int PTW = C::TW / 2, PITEMS = C::BM / 4 * 8;
#pragma unroll
          for (int it = 0; it < (PITEMS + NT - 1) / NT; ++it) {
            const int idx = it * NT + tid;
            if (idx >= PITEMS) break;
            const int pp = idx >> 3, cq = idx & 7;
            const int pr = pp / PTW, pc = pp % PTW;
            const int rr = 2 * pr * C::TW + 2 * pc;
            bool in;
            const int fpix = out_pix(2 * pr, 2 * pc, in);
            const int fx = fpix % W;
            const bool vh = r0 + 2 * pr + 1 < H, vw = a.vstride ? fx + 1 < W : c0 + 2 * pc + 1 < W;
            auto ld8 = [&](int r, float* f) {
              const float4 q0 = *reinterpret_cast<const float4*>(smem + r * C::SR32 + cq * 32);
              const float4 q1 = *reinterpret_cast<const float4*>(smem + r * C::SR32 + cq * 32 + 16);
              f[0] = q0.x; f[1] = q0.y; f[2] = q0.z; f[3] = q0.w; f[4] = q1.x; f[5] = q1.y; f[6] = q1.z; f[7] = q1.w;
            };
            float m[8], f[8];
            ld8(rr, m);
            if (vw) {
              ld8(rr + 1, f);
#pragma unroll
              for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
            }
            if (vh) {
              ld8(rr + C::TW, f);
#pragma unroll
              for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
            }
            if (vh && vw) {
              ld8(rr + C::TW + 1, f);
#pragma unroll
              for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
            }
            int ppix = pr * PW + pc;
            bool ok = pr0 + pr < PH && pc0 + pc < PW;
            if (a.vstride) {
              ok = in;
              ppix = ((fpix / W - 2 * pr) / H * PH + pr) * PW + fx / 2;
            }
            ok = ok && n0 + sl * 64 + cq * 8 < a.cout;
            uint4 hv, lv;
            split3h_chunk(m, hv, lv);
            const int off = ok ? (ppix * a.py_cstride + sl * 64 + cq * 8) * 2 : OOB;
            typedef __attribute__((ext_vector_type(4))) unsigned u4_t;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, lv), prs, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, hv), prs, ok ? off + P2 : OOB, 0, 0);
            if (3 * a.psplit <= a.py_cstride)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4_t, hv), prs, ok ? off + 2 * P2 : OOB, 0, 0);
          }
        }
        continue;
      }
#pragma unroll
      for (int it = 0; it < C::BM * 16 / NT; ++it) {
        const int idx = it * NT + tid;
        const int rr = idx >> 4, cq = idx & 15;
        const uint4 d = *reinterpret_cast<const uint4*>(smem + rr * C::SR32 + cq * 16);
        const int pr = rr / C::TW, pc = rr % C::TW;
        bool ok;
        const int pix = out_pix(pr, pc, ok);
        ok = ok && cb + cq * 4 < a.cout;
        const int off = ok ? pix * ycs4 + (cb + cq * 4) * 4 : OOB;
        if (splitk || a.y_vec) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                 yfr, off, 0, 0);
        } else {  // a view whose channel offset / stride is not a multiple of 4 (up1[..., 6:30]): dword stores
          __builtin_amdgcn_raw_buffer_store_b32(d.x, yfr, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(d.y, yfr, off + 4, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(d.z, yfr, off + 8, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(d.w, yfr, off + 12, 0, 0);
        }
      }
    }
    if (ovf && a.ovf) *a.ovf = 1;  // a plain vector store: any writer's 1 is the answer
    return;
  }
  if constexpr (C::REPI_OK) {
    if (a.repi && !a.vstride) {
      // register epilogue: bias / affine / act in registers, chunk_pair turns each pair of 16-channel fragments' lane
      // quads into whole 16-byte chunks stored straight from the lane (no staging, no block barrier); the fused pool
      // takes the row below from the wave's partner fragment and the column partner through DPP quad_perm [1,0,3,2]
      const int col = lane & 15, ckq = lane >> 4;
      const int c16 = (ckq & 1) ? 2 + (ckq >> 1) : ckq >> 1;
      const int PH = (H + 1) >> 1, PWo = (W + 1) >> 1;
      T* pb = a.py ? reinterpret_cast<T*>(a.py) + a.py_coff +
                         (((long)n * PH + (r0 >> 1)) * PWo + (c0 >> 1)) * (long)a.py_cstride + n0
                   : nullptr;
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pb, 0, 0x7ffffff0, 0x00020000);
      // head split (a.hd, vm_conv3x3_up2x_head_nhwc): the wave holds all 64 channels of its pixels (one phase of the
      // folded upconv), so conv1_5's per-tap shares of them are 2 MFMAs on the bf16 outputs, as in the pair kernels:
      // A rows = the 9 taps, k ordered like the lane's output channels (2kk + j/4)*16 + 4q + j%4
      constexpr bool HEADOK = FC == 4 && BN == 64;
      // every global load of the epilogue (per-channel constants of all FC fragments, the head filter) is issued
      // here, before any is used, so the block waits for one round trip instead of one per channel group
      const int ccap = a.up ? a.up_cout : a.cout;
      float mul[FC][4], add[FC][4];
#pragma unroll
      for (int f = 0; f < FC; ++f) {
        const int chb = n0 + wn * C::TPN + (f & ~1) * 16;
        const int cb = chb - (a.up ? chb / a.up_cout : 0) * a.up_cout;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = min(cb + (f & 1) * 16 + 4 * ckq + j, ccap - 1);
          const float sc = a.scale ? a.scale[co] : 1.f;
          mul[f][j] = sc;
          add[f][j] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);  // (as the staged epilogue)
        }
      }
      float hwv[2][8];
      if (HEADOK && a.hd) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int hc = (2 * kk + j / 4) * 16 + 4 * ckq + j % 4;
            hwv[kk][j] = col < 9 ? a.hw[col * a.hw_cin + a.hw_coff + hc] : 0.f;
          }
      }
      uint4 hb[FP][2];  // head split: the B operands (bf16 outputs) of each fragment's 2 head MFMAs, used at the end
#pragma unroll
      for (int g2 = 0; g2 < FC / 2; ++g2) {
        const int chb = n0 + wn * C::TPN + g2 * 32;  // first block channel of this 32-channel group
        const int phase = a.up ? chb / a.up_cout : 0;
        const int cb = chb - phase * a.up_cout;
        float v[FP][2][4];
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          uint2 pk[2];
#pragma unroll
          for (int f = 0; f < 2; ++f) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float t = fmaf(acc[2 * g2 + f][fp][j], mul[2 * g2 + f][j], add[2 * g2 + f][j]);
              if (a.act == VM_ACT_RELU) t = fmaxf(t, 0.f);
              else if (a.act == VM_ACT_SIGMOID) t = sigmoid_precise(t);
              v[fp][f][j] = t;
            }
            pk[f].x = bf16x2_bits(v[fp][f][0], v[fp][f][1]);
            pk[f].y = bf16x2_bits(v[fp][f][2], v[fp][f][3]);
          }
          hb[fp][g2] = make_uint4(pk[0].x, pk[0].y, pk[1].x, pk[1].y);
          const uint4 d = chunk_pair(pk[0], pk[1]);
          const int tr = C::prow(wm, fp), tc = C::pcol(wm, fp) + col;
          const bool ok = r0 + tr < H && c0 + tc < W && cb + c16 * 8 < ccap && !a.y_skip;
          const int pix = a.up ? (2 * tr + (phase >> 1)) * YW + 2 * tc + (phase & 1) : tr * W + tc;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                 yrs, ok ? pix * ycs2 + (cb + c16 * 8) * 2 : OOB, 0, 0);
        }
        if (a.py) {  // tiles start on even rows/columns: every 2x2 window lies inside the tile (host: no a.up)
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) {
            if (C::prow(wm, fp) & 1) continue;  // (compile-time per fp: the top row of each window)
            const int tr = C::prow(wm, fp), tc = C::pcol(wm, fp) + col;
            const bool v0 = r0 + tr < H && c0 + tc < W, v1 = r0 + tr + 1 < H && c0 + tc < W;
            float m[2][4];
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                float t = v0 ? v[fp][f][j] : -INFINITY;
                if (v1) t = fmaxf(t, v[fp + C::PSTEP][f][j]);
                const float u = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0xB1, 0xF, 0xF, false));
                m[f][j] = fmaxf(t, u);
              }
            uint2 q2[2];
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              q2[f].x = bf16x2_bits(m[f][0], m[f][1]);
              q2[f].y = bf16x2_bits(m[f][2], m[f][3]);
            }
            const uint4 d = chunk_pair(q2[0], q2[1]);
            const int pr = tr >> 1, pc = tc >> 1;
            const int chl = wn * C::TPN + g2 * 32 + c16 * 8;  // channel relative to n0
            const bool pok = (col & 1) == 0 && v0 && (r0 >> 1) + pr < PH && (c0 >> 1) + pc < PWo && n0 + chl < a.cout;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                   prs, pok ? ((pr * PWo + pc) * a.py_cstride + chl) * 2 : OOB, 0, 0);
          }
        }
      }
      if constexpr (HEADOK) {
        if (a.hd) {
          // the head's shares, last: the filter loads issued at the top of the epilogue had the whole epilogue to land.
          // A fragments: rows = taps (9 of 16), k = 8q + j <-> channel (2kk + j/4)*16 + 4q + j%4
          uint4 hwf[2];
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            hwf[kk] = make_uint4(bf16x2_bits(hwv[kk][0], hwv[kk][1]),
                                 bf16x2_bits(hwv[kk][2], hwv[kk][3]),
                                 bf16x2_bits(hwv[kk][4], hwv[kk][5]),
                                 bf16x2_bits(hwv[kk][6], hwv[kk][7]));
          const int phase = a.up ? (n0 + wn * C::TPN) / a.up_cout : 0;
          const int YH = a.up ? 2 * H : H;
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) {
            f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
            mma16<T>(hwf[0], hb[fp][0], d);
            mma16<T>(hwf[1], hb[fp][1], d);
            const int tr = C::prow(wm, fp), tc = C::pcol(wm, fp) + col;
            if (ckq < 3 && r0 + tr < H && c0 + tc < W) {
              const int yy = a.up ? 2 * (r0 + tr) + (phase >> 1) : r0 + tr;
              const int xx = a.up ? 2 * (c0 + tc) + (phase & 1) : c0 + tc;
              *reinterpret_cast<f32x4*>(a.hd + (((long)n * YH + yy) * YW + xx) * 12 + 4 * ckq) = d;
            }
          }
        }
      }
      return;
    }
  }
  for (int sl = 0; sl < BN / 64; ++sl) {
    const int phase = a.up ? (n0 + sl * 64) / a.up_cout : 0;
    const int cb = n0 + sl * 64 - phase * a.up_cout;  // first (per-phase) output channel of the slab
    const int ccap = a.up ? a.up_cout : a.cout;
    __syncthreads();
    if (wn == sl / SPW) {
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        if (fc / 4 != sl % SPW) continue;
        const int col = (fc % 4) * 16 + 4 * (lane >> 4);
        float mul[4], add[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = min(cb + col + j, ccap - 1);
          const float sc = a.scale ? a.scale[co] : 1.f;
          mul[j] = sc;
          add[j] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
        }
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          const int row = C::tpix(wm, fp) + (lane & 15);
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = fmaf(acc[fc][fp][j], mul[j], add[j]);
            if (a.act == VM_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
            else if (a.act == VM_ACT_SIGMOID) v[j] = sigmoid_precise(v[j]);
          }
          uint2 pk;
          pk.x = bf16x2_bits(v[0], v[1]);
          pk.y = bf16x2_bits(v[2], v[3]);
          *reinterpret_cast<uint2*>(smem + row * C::SR + col * 2) = pk;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < C::BM * 8 / NT; ++it) {
      const int idx = it * NT + tid;
      const int rr = idx >> 3, cq = idx & 7;
      const uint4 d = *reinterpret_cast<const uint4*>(smem + rr * C::SR + cq * 16);
      const int pr = rr / C::TW, pc = rr % C::TW;
      bool ok;
      int pix = out_pix(pr, pc, ok);
      ok = ok && cb + cq * 8 < ccap;
      if (a.up) pix = (2 * pr + (phase >> 1)) * YW + 2 * pc + (phase & 1);
      const int off = ok ? pix * ycs2 + (cb + cq * 8) * 2 : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), yrs,
                                             off, 0, 0);
    }
    if (a.py) {
      // fused tf.nn.max_pool 2x2/2 SAME (unet.py:32-33) of the staged slab: tiles start on even rows/columns,
      // so every window lies inside the tile; taps past the frame edge are skipped (never win)
      // (packed frames: W even, so frames start on even virtual columns and every window is inside one frame)
      const int PH = (H + 1) >> 1, PW = (W + 1) >> 1;
      const int pr0 = r0 >> 1, pc0 = c0 >> 1;
      T* pb = reinterpret_cast<T*>(a.py) + a.py_coff +
              (((long)n * PH + pr0) * PW + (a.vstride ? 0 : pc0)) * (long)a.py_cstride + n0;
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pb, 0, 0x7ffffff0, 0x00020000);
      constexpr int PTW = C::TW / 2, PITEMS = C::BM / 4 * 8;
#pragma unroll
      for (int it = 0; it < (PITEMS + NT - 1) / NT; ++it) {
        const int idx = it * NT + tid;
        if (idx >= PITEMS) break;
        const int pp = idx >> 3, cq = idx & 7;
        const int pr = pp / PTW, pc = pp % PTW;
        const int rr = 2 * pr * C::TW + 2 * pc;
        bool in;
        const int fpix = out_pix(2 * pr, 2 * pc, in);  // the window's top-left output pixel
        const int fx = fpix % W;                        // its frame column (even)
        const bool vh = r0 + 2 * pr + 1 < H, vw = a.vstride ? fx + 1 < W : c0 + 2 * pc + 1 < W;
        float m[8], f[8];
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + rr * C::SR + cq * 16), m);
        if (vw) {
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + (rr + 1) * C::SR + cq * 16), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
        }
        if (vh) {
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + (rr + C::TW) * C::SR + cq * 16), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
        }
        if (vh && vw) {
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + (rr + C::TW + 1) * C::SR + cq * 16), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
        }
        int ppix = pr * PW + pc;
        bool ok = pr0 + pr < PH && pc0 + pc < PW;
        if (a.vstride) {  // pooled pixel (frame, pr0 + pr, fx / 2)
          ok = in;
          ppix = ((fpix / W - 2 * pr) / H * PH + pr) * PW + fx / 2;
        }
        ok = ok && n0 + sl * 64 + cq * 8 < a.cout;
        const int off = ok ? (ppix * a.py_cstride + sl * 64 + cq * 8) * 2 : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, Chunk<T>::pack(m)), prs, off, 0, 0);
      }
    }
  }
}

// ================================================================ persistent row-slot patch kernel
// The G = 3 patch pipeline above with the tile loop inside the kernel (vm_set_option "patch_persist"): a resident
// grid of 8 x J blocks; block b lives on XCD b % 8 and walks the (pixel tile, 64-channel output tile) items of its
// XCD's band of pixel tiles [lo, hi): round `it` hands walker j the item it*J + j, so the walkers of a round cover
// all output tiles of adjacent pixel tiles (the input patch is fetched from HBM about once per XCD) and, J being a
// multiple of the output tile count, each walker keeps one output tile.  A folded upconv's phases run 9 / 6 / 6 / 4
// taps, so there (ConvArgs::prot) walker j takes item it*J + (j + it) % J instead and cycles through the phases:
// a fixed phase per walker leaves the 9-tap walkers as the tail.  The DMA stream (input granules, weight row slots) runs on
// across tile boundaries: the next item's first granule and weight rows are issued during the current one's last
// steps and land while it finishes its MFMAs and its register epilogue, so an item pays no prologue latency.  The
// per-channel affine of every output channel and the head filter fragments are staged in LDS once per block (the
// epilogue then has no global load, whose vmcnt wait would drain the prefetch).  Every output pixel keeps the
// non-persistent kernel's MFMA sequence and epilogue arithmetic: results are bit-identical.
template <int BN, int WM, int WN, int S, int TH, int MINB, bool UPSKIP>
__global__ __launch_bounds__(64 * WM * WN)
__attribute__((amdgpu_waves_per_eu(MINB * WM * WN < 16 ? 4 : MINB * WM * WN / 4)))  // <= 128 VGPRs
void conv3x3_patch_persist(ConvArgs a) {
  using C = PatchCfg<BN, WM, WN, S, TH, 3>;
  using T = uint16_t;
  static_assert(BN == 64 && WN == 1 && C::REPI_OK && C::FC == 4, "64-channel output tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NW = C::NW, NT = C::NT, FP = C::FP, FC = C::FC, XPW = C::XPW, WPW = C::WPW, R = 3, G = 3;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a.prio && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int wm = wave;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + C::TH - 1) / C::TH, tw = (W + C::TW - 1) / C::TW;
  const int tn = a.tiles_n, sp = a.tiles_total / tn, CT = tn * BN;
  const int xcd = blockIdx.x & 7, jw = blockIdx.x >> 3, J = (int)(gridDim.x >> 3);
  const int lo = (int)((long)xcd * sp / 8), hi = (int)((long)(xcd + 1) * sp / 8);
  const int nitem = (hi - lo) * tn;
  int it = 0, q = jw;
  if (q >= nitem) return;  // (before any barrier: the block has no work)
  // band-local pixel tile i -> pixel tile; with halfskip the band's last-column tiles (s % tw == tw - 1; [0, s) holds
  // s / tw of them) come after its other tiles, in order
  const int nhalf = a.halfskip ? hi / tw - lo / tw : 0, nfull = hi - lo - nhalf;
  auto band_tile = [&](int i) __attribute__((always_inline)) {
    if (!a.halfskip) return lo + i;
    if (i < nfull) {
      const int g = lo - lo / tw + i;  // the g-th tile off the last column
      return g + g / (tw - 1);
    }
    return (lo / tw + i - nfull) * tw + tw - 1;
  };
  // round r's item of walker jw: prot 1 rotates the walkers over the output tiles, prot 2 reverses the order of the
  // walker groups (tn walkers, one per output tile) in odd rounds, so the walkers that end a round late start the
  // next one early (each walker keeps its output tile)
  auto item_of = [&](int r) __attribute__((always_inline)) {
    if (a.prot == 1) return r * J + (jw + r) % J;
    if (a.prot == 2 && (r & 1)) return r * J + J - tn - jw + 2 * (jw % tn);
    return r * J + jw;
  };

  // per-block constants in LDS: mul[CT], add[CT] (f32, output channel order), then the head A fragments [lane][2]
  char* kc = smem + C::MAIN;
  const int ccap = a.up ? a.up_cout : a.cout;
  for (int c = tid; c < CT; c += NT) {
    const int chb = c & ~31;  // (the register epilogue's 32-channel group base and phase)
    const int cb = chb - (a.up ? chb / a.up_cout : 0) * a.up_cout;
    const int co = min(cb + (c & 31), ccap - 1);
    const float sc = a.scale ? a.scale[co] : 1.f;
    reinterpret_cast<float*>(kc)[c] = sc;
    reinterpret_cast<float*>(kc)[CT + c] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
  }
  char* kh = kc + CT * 8;
  const int col = lane & 15, ckq = lane >> 4;
  if (a.hd && tid < 64) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      float hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int hc = (2 * kk + j / 4) * 16 + 4 * ckq + j % 4;
        hv[j] = col < 9 ? a.hw[col * a.hw_cin + a.hw_coff + hc] : 0.f;
      }
      *reinterpret_cast<uint4*>(kh + (lane * 2 + kk) * 16) =
          make_uint4(bf16x2_bits(hv[0], hv[1]),
                     bf16x2_bits(hv[2], hv[3]),
                     bf16x2_bits(hv[4], hv[5]),
                     bf16x2_bits(hv[6], hv[7]));
    }
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, 0);  // (item weights at n0 * K_pad * 2 bytes: host-checked)
  const int lrow = lane >> 2, lpos = lane & 3;
  int woff[WPW];
  int w_n = 0;
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int piece = wave + i * NW;
    const int row = piece * 16 + lrow;
    const int lq = (swz<64>(row, lpos) - row * 64) >> 4;
    woff[i] = (row * a.K_pad + lq * 8) * 2;
    if (piece < C::WP) ++w_n;
  }
  int x_n = 0;
#pragma unroll
  for (int i = 0; i < XPW; ++i)
    if (wave + i * NW < C::XP) ++x_n;

  // input DMA state of the tile whose granules are being fetched (switches to the next tile at the last granule)
  __amdgpu_buffer_rsrc_t xrs;
  int xoff[XPW];
  auto set_xtile = [&](int s) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int lrow = ln >> 2, lpos = ln & 3;
    const int n = s / (th * tw), srem = s - n * th * tw;
    const int r0 = (srem / tw) * C::TH, c0 = (srem - (srem / tw) * tw) * C::TW;
    const T* xb = reinterpret_cast<const T*>(a.x) + a.x_coff + ((long)n * H + r0 - 1) * (long)W * cs;
    xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(xb), 0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int i = 0; i < XPW; ++i) {
      const int row = (wave + i * NW) * 16 + lrow;
      const int lq = (swz<64>(row, lpos) - row * 64) >> 4;
      const int pr = row / C::PW, pc = row - pr * C::PW;
      int h = r0 - 1 + pr, w = c0 - 1 + pc;
      if (a.up) {  // folded 2x resize: the low-res frame's edge is replicated (as conv3x3_patch)
        h = min(h, H - 1);
        w = min(w, W - 1);
      }
      const bool ok = row < C::PPIX && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      xoff[i] = ok ? (((h - r0 + 1) * W + w) * cs + lq * 8) * 2 : OOB;
    }
  };
  const int nch = a.cin_pad / 32, nsr = nch * R;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const uint32_t wring = lds0 + 2 * C::PB;
  auto issue_x = [&](int cc, int buf, bool real) {
#pragma unroll
    for (int i = 0; i < XPW; ++i)
      if (wave + i * NW < C::XP)
        glds16(xrs, lds0 + buf * C::PB + (wave + i * NW) * 1024, real ? xoff[i] + (int)src_chan(a, cc * 32) * 2 : OOB);
  };
  auto issue_w = [&](int s, int slot, bool real, int wb) {  // wb: the item's weight byte offset
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < WPW; ++i)
        if (wave + i * NW < C::WP)
          glds16(wrs, wring + (slot * G + g) * C::WSLOT + (wave + i * NW) * 1024,
                 real ? woff[i] + wb + (s * G + g) * 64 : OOB);
  };

  int boff[FC], abase[FP];
#pragma unroll
  for (int f = 0; f < FC; ++f) boff[f] = 2 * C::PB + swz<64>(f * 16 + (lane & 15), lane >> 4);
#pragma unroll
  for (int f = 0; f < FP; ++f) abase[f] = C::prow(wm, f) * C::PW + C::pcol(wm, f) + (lane & 15);
  const int ck = lane >> 4;
  auto frags = [&](uint4 (&av)[FC], uint4 (&bv)[FP], int slot, int buf, int tap) {
    const char* wp = smem + (slot * G + tap % G) * C::WSLOT;
    const char* xp = smem + buf * C::PB;
#pragma unroll
    for (int f = 0; f < FC; ++f) av[f] = *reinterpret_cast<const uint4*>(wp + boff[f]);
    const int toff = (tap / 3) * C::PW + tap % 3;
#pragma unroll
    for (int f = 0; f < FP; ++f) bv[f] = *reinterpret_cast<const uint4*>(xp + swz<64>(abase[f] + toff, ck));
  };
  // counted DMA wait, then lgkmcnt(0): this wave's fragment reads of the ring slot / patch buffer that the DMAs
  // issued right after the barrier refill must have returned before the barrier — the MFMAs consuming them may be
  // scheduled past it (seen in the 4 x 32 folded-upconv instantiation: under a second process on the GPU the refill
  // overtook a queued ds_read about once per 100 frames)
  auto sync = [&](int n) {
    wait_vm(n);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // stores of one epilogue (counted into the first waits of the next tile: they are younger than the weight rows
  // issued before it); the head's conditional stores are not counted (waiting longer is safe)
  int e_st = 2 * FP;
  if (a.py) {
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) e_st += (C::prow(wm, fp) & 1) ? 0 : 2;
  }

  const int ycs2 = a.y_cstride * 2;
  const int YW = a.up ? 2 * W : W;
  const int PH = (H + 1) >> 1, PWo = (W + 1) >> 1;
  auto epilogue = [&](const f32x4 (&acc)[FC][FP], int s, int n0) {
    // lane-derived values from an opaque copy of the lane id: recomputed per tile instead of held across the loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int col = ln & 15, ckq = ln >> 4;
    const int n = s / (th * tw), srem = s - n * th * tw;
    const int r0 = (srem / tw) * C::TH, c0 = (srem - (srem / tw) * tw) * C::TW;
    T* yb = reinterpret_cast<T*>(a.y) + a.y_coff +
            (a.up ? (((long)n * 2 * H + 2 * r0) * YW + 2 * c0) : (((long)n * H + r0) * W + c0)) * (long)a.y_cstride;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yb, 0, 0x7ffffff0, 0x00020000);
    const int c16 = (ckq & 1) ? 2 + (ckq >> 1) : ckq >> 1;
    T* pb = a.py ? reinterpret_cast<T*>(a.py) + a.py_coff +
                       (((long)n * PH + (r0 >> 1)) * PWo + (c0 >> 1)) * (long)a.py_cstride + n0
                 : nullptr;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pb, 0, 0x7ffffff0, 0x00020000);
    f32x4 dh[FP];  // head split: conv1_5's per-tap partials, accumulated over the two 32-channel groups
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) dh[fp] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g2 = 0; g2 < FC / 2; ++g2) {
      const int chb = n0 + g2 * 32;
      const int phase = a.up ? chb / a.up_cout : 0;
      const int cb = chb - phase * a.up_cout;
      float v[FP][2][4];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const float4 m4 = *reinterpret_cast<const float4*>(kc + (n0 + (2 * g2 + f) * 16 + 4 * ckq) * 4);
        const float4 a4 = *reinterpret_cast<const float4*>(kc + (CT + n0 + (2 * g2 + f) * 16 + 4 * ckq) * 4);
        const float mul[4] = {m4.x, m4.y, m4.z, m4.w}, add[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int fp = 0; fp < FP; ++fp)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float t = fmaf(acc[2 * g2 + f][fp][j], mul[j], add[j]);
            if (a.act == VM_ACT_RELU) t = fmaxf(t, 0.f);
            else if (a.act == VM_ACT_SIGMOID) t = sigmoid_precise(t);
            v[fp][f][j] = t;
          }
      }
#pragma unroll
      for (int fp = 0; fp < FP; ++fp) {
        uint2 pk[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          pk[f].x = bf16x2_bits(v[fp][f][0], v[fp][f][1]);
          pk[f].y = bf16x2_bits(v[fp][f][2], v[fp][f][3]);
        }
        if (a.hd)  // (the same two MFMAs, in the same order, as the register epilogue's head split)
          mma16<T>(*reinterpret_cast<const uint4*>(kh + (ln * 2 + g2) * 16),
                   make_uint4(pk[0].x, pk[0].y, pk[1].x, pk[1].y), dh[fp]);
        const uint4 d = chunk_pair(pk[0], pk[1]);
        const int tr = C::prow(wm, fp), tc = C::pcol(wm, fp) + col;
        const bool ok = r0 + tr < H && c0 + tc < W && cb + c16 * 8 < ccap && !a.y_skip;
        const int pix = a.up ? (2 * tr + (phase >> 1)) * YW + 2 * tc + (phase & 1) : tr * W + tc;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), yrs,
                                               ok ? pix * ycs2 + (cb + c16 * 8) * 2 : OOB, 0, 0);
      }
      if (a.py) {
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          if (C::prow(wm, fp) & 1) continue;
          const int tr = C::prow(wm, fp), tc = C::pcol(wm, fp) + col;
          const bool v0 = r0 + tr < H && c0 + tc < W, v1 = r0 + tr + 1 < H && c0 + tc < W;
          float m[2][4];
#pragma unroll
          for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float t = v0 ? v[fp][f][j] : -INFINITY;
              if (v1) t = fmaxf(t, v[fp + C::PSTEP][f][j]);
              const float u = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(t), 0xB1, 0xF, 0xF, false));
              m[f][j] = fmaxf(t, u);
            }
          uint2 q2[2];
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            q2[f].x = bf16x2_bits(m[f][0], m[f][1]);
            q2[f].y = bf16x2_bits(m[f][2], m[f][3]);
          }
          const uint4 d = chunk_pair(q2[0], q2[1]);
          const int pr = tr >> 1, pc = tc >> 1;
          const int chl = g2 * 32 + c16 * 8;
          const bool pok = (col & 1) == 0 && v0 && (r0 >> 1) + pr < PH && (c0 >> 1) + pc < PWo && n0 + chl < a.cout;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d),
                                                 prs, pok ? ((pr * PWo + pc) * a.py_cstride + chl) * 2 : OOB, 0, 0);
        }
      }
    }
    if (a.hd) {
      const int phase = a.up ? n0 / a.up_cout : 0;
      const int YH = a.up ? 2 * H : H;
#pragma unroll
      for (int fp = 0; fp < FP; ++fp) {
        const f32x4 d = dh[fp];
        const int tr = C::prow(wm, fp), tc = C::pcol(wm, fp) + col;
        if (ckq < 3 && r0 + tr < H && c0 + tc < W) {
          const int yy = a.up ? 2 * (r0 + tr) + (phase >> 1) : r0 + tr;
          const int xx = a.up ? 2 * (c0 + tc) + (phase & 1) : c0 + tc;
          *reinterpret_cast<f32x4*>(a.hd + (((long)n * YH + yy) * YW + xx) * 12 + 4 * ckq) = d;
        }
      }
    }
  };

  const int wstep = a.K_pad * 2 * BN;  // weight bytes of one output tile
  int st = band_tile(q / tn), n0 = (q % tn) * BN;
  set_xtile(st);
  int gcnt = 0;  // granules issued so far (input buffer parity)
  issue_x(0, 0, true);
#pragma unroll
  for (int j = 0; j < S - 1; ++j) issue_w(j, j, j < nsr, (q % tn) * wstep);
  int slot = 0;
  bool first = true;
  for (;;) {
    const int qn = item_of(it + 1);
    const bool more = qn < nitem;
    const int stn = more ? band_tile(qn / tn) : st, wbn = more ? (qn % tn) * wstep : 0, wb = (n0 / BN) * wstep;
    // a last-column tile of a halfskip frame: the right-half waves' pixels are all outside it (stores masked as ever)
    const bool idle = a.halfskip && (wm & 1) && st % tw == tw - 1;
    const int up_phase = UPSKIP && a.up && n0 / a.up_cout == (n0 + BN - 1) / a.up_cout ? n0 / a.up_cout : 0;
    const bool skip_r0 = (up_phase >> 1) != 0 && (a.upmask & 1), skip_c0 = (up_phase & 1) != 0 && (a.upmask & 2);
    f32x4 acc[FC][FP];
#pragma unroll
    for (int i = 0; i < FC; ++i)
#pragma unroll
      for (int j = 0; j < FP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int cc = 0; cc < nch; ++cc) {
      const int buf = gcnt & 1;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = cc * R + r;
        int nw = (S - 2) * G * w_n + ((r >= 1 && r <= S - 2) ? x_n : 0);
        if (!first && k < S - 1) nw += e_st;
        sync(nw);
        if (r == 0) {
          if (cc + 1 < nch) {
            issue_x(cc + 1, buf ^ 1, true);
          } else {  // the next item's first granule (a dummy past the walk's end)
            if (more && stn != st) set_xtile(stn);
            issue_x(0, buf ^ 1, more);
          }
        }
        int ws = k + S - 1;
        if (ws < nsr) {
          issue_w(ws, slot + S - 1 - (slot + S - 1 >= S ? S : 0), true, wb);
        } else {
          issue_w(ws - nsr, slot + S - 1 - (slot + S - 1 >= S ? S : 0), more, wbn);
        }
        if (!(UPSKIP && skip_r0 && r == 0) && !idle) {
          uint4 av[2][FC], bv[2][FP];
          frags(av[0], bv[0], slot, buf, r * G);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            if (g + 1 < G) frags(av[(g + 1) & 1], bv[(g + 1) & 1], slot, buf, r * G + g + 1);
            if (!(UPSKIP && skip_c0 && g == 0)) {
#pragma unroll
              for (int fc = 0; fc < FC; ++fc)
#pragma unroll
                for (int fp = 0; fp < FP; ++fp) mma16<T>(av[g & 1][fc], bv[g & 1][fp], acc[fc][fp]);
            }
          }
        }
        slot = slot + 1 == S ? 0 : slot + 1;
      }
      ++gcnt;
    }
    epilogue(acc, st, n0);
    if (!more) break;
    ++it;
    q = qn;
    st = stn;
    n0 = (qn % tn) * BN;
    first = false;
  }
}

// ================================================================ persistent first pair (conv1_1 -> conv1_2 [-> pool1])
// unet.py:170-172 at full resolution.  conv1_2 has only 2 channel granules (18 K-steps), so in the streaming patch
// kernel the per-tile fixed costs (input latency, the first conv, the epilogue) dominate.  Here ONE 512-thread block
// per CU keeps all of conv1_2's weights in LDS (18 K-step slots x 64 couts x 64 B = 72 KB, loaded once) and walks
// the 8 x 32 tiles t = blockIdx.x, +gridDim.x, ...: the main loop has no barrier and no DMA, and the next tile's
// input pixels are loaded into registers while the current tile's MFMAs run.
// The pair kernel's own patch images use a 2-bit chunk swizzle: like swz<64>, conflict-free for the ds_read_b128
// fragment reads from any start row, and also for ds_write_b128 of 8 consecutive rows (swz<64> is 2-way there)
// (swz2: conv_common.h)

struct PairCfg {
  static constexpr int TH = 8, TW = 32, BM = TH * TW, PW = TW + 2, PPIX = (TH + 2) * PW;
  static constexpr int IW = TW + 4, IPIX = (TH + 4) * IW;  // 8-channel input patch, origin (r0-2, c0-2)
  static constexpr int NW = 8, NT = 512, NSTEP = 18;
  static constexpr int PB = ((PPIX + 15) / 16) * 1024;     // one 32-channel granule of the patch (64-B rows)
  static constexpr int WSLOT = 64 * 64;
  static constexpr int PBU = PPIX * 64;                   // bytes of a granule buffer actually addressed
  static constexpr int SR = 64 * 2 + 16;                   // epilogue staging row
  static constexpr int P_OFF = NSTEP * WSLOT, I_OFF = P_OFF + 2 * PBU, S_OFF = I_OFF + IPIX * 16;
  static constexpr int R_OFF = S_OFF + BM * SR;             // per-channel epilogue constants: mul[64], add[64], b1[64]
  static constexpr int LDS = R_OFF + 3 * 64 * 4;
};
static_assert(PairCfg::LDS <= 163840, "weights + patch + input + staging in one CU's LDS");
static_assert(PairCfg::IPIX <= PairCfg::NT, "one input pixel per thread");

// PABL: timing ablations (results are garbage): 1 no first-conv MFMAs, 2 no conv1_2 MFMAs, 4 no output stores,
// 8 no input loads
// XIN: the input dtype/load form — a compile-time choice, so the input loads carry no runtime branch (a branch join
// made hipcc wait for the loads right after issuing them, before conv1_2).  0: bf16 8-channel chunks; 1: f32 frame,
// one dword load per channel; 2: f32 frame with 4 <= x_c <= 8 channels (the UNetVideo path), two 16-byte loads per
// pixel (channels 0..3 and x_c-4..x_c-1, dword-aligned) instead of 8 dword loads
// a workgroup barrier that orders LDS only (no vmcnt(0) as __syncthreads emits): global stores and loads stay in
// flight across it
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int PABL = 0, int XIN = 2>
__global__ __launch_bounds__(512) void conv3x3_pair_persist(ConvArgs a) {
  using C = PairCfg;
  using T = uint16_t;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, W = a.W;
  const int th = (H + C::TH - 1) / C::TH, tw = (W + C::TW - 1) / C::TW;
  const int ntiles = (int)(a.M / ((long)H * W)) * th * tw;
  const int col = lane & 15, q = lane >> 4;

  // conv1_2 weights: slot s = K-step s of the chunk-major packing (granule cc*9 + tap), swizzled 64-B rows
  const T* wg = reinterpret_cast<const T*>(a.w);
  for (int i = tid; i < C::NSTEP * 64 * 4; i += C::NT) {
    const int st = i >> 8, row = (i >> 2) & 63, ch = i & 3;
    *reinterpret_cast<uint4*>(smem + st * C::WSLOT + swz<64>(row, ch)) =
        *reinterpret_cast<const uint4*>(wg + (long)row * a.K_pad + st * 32 + ch * 8);
  }
  // conv1_1 (tap-major, K_pad 128) weight fragments and bias stay in registers
  const T* w1 = reinterpret_cast<const T*>(a.w1);
  uint4 wf[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) wf[j][fc] = *reinterpret_cast<const uint4*>(w1 + (fc * 16 + col) * 128 + j * 32 + q * 8);
  // consume the fragments here: otherwise hipcc's wait for these loads sits inside the tile loop (it cannot tell the
  // first iteration from the rest), where every tile then waits vmcnt(3..0) for the PREVIOUS tile's output stores
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0) (expcnt / lgkmcnt at max): a real S_WAITCNT the wait pass accounts for
  // per-channel constants live in LDS (registers go to the conv1_2 fragment prefetch)
  float* rmul = reinterpret_cast<float*>(smem + C::R_OFF);
  if (tid < 64) {
    const int co = min(tid, a.cout - 1);
    const float sc = a.scale ? a.scale[co] : 1.f;
    rmul[tid] = sc;
    rmul[64 + tid] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
    rmul[128 + tid] = a.bias1 ? a.bias1[tid] : 0.f;
  }
  // head split: A fragments of the skip half's head filter, rows = taps (9 of 16), k = 8q + j <-> conv1_2 channel
  // (2kk + j/4)*16 + 4q + j%4 — the channel order in which the epilogue's lane holds its bf16 outputs (B operand)
  uint4 hwf[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  if (a.hd) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint32_t u[4];
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const int j0 = 2 * jp, j1 = 2 * jp + 1;
        const int c0 = (2 * kk + j0 / 4) * 16 + 4 * q + j0 % 4, c1 = (2 * kk + j1 / 4) * 16 + 4 * q + j1 % 4;
        const float w0 = col < 9 ? a.hw[col * a.hw_cin + a.hw_coff + c0] : 0.f;
        const float w1 = col < 9 ? a.hw[col * a.hw_cin + a.hw_coff + c1] : 0.f;
        u[jp] = bf16x2_bits(w0, w1);
      }
      hwf[kk] = make_uint4(u[0], u[1], u[2], u[3]);
    }
  }

  // input pixel of this thread (one per thread): raw registers while in flight, bf16 chunk in LDS
  const T* x8 = reinterpret_cast<const T*>(a.x) + a.x_coff;
  const float* xf = reinterpret_cast<const float*>(a.x) + a.x_coff;
  uint4 xq = make_uint4(0, 0, 0, 0);
  float xr[8];
  f32x4 xlo = f32x4{0.f, 0.f, 0.f, 0.f}, xhi = xlo;
  bool xin = false;
  auto load_in = [&](int t) {
    const int n = t / (th * tw), rem = t - n * th * tw;
    const int ir = tid / C::IW, ic = tid - ir * C::IW;
    const int h = (rem / tw) * C::TH - 2 + ir, w = (rem % tw) * C::TW - 2 + ic;
    xin = tid < C::IPIX && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    if (PABL & 8) return;
    // branch-free: out-of-frame lanes read pixel (0,0) and channels past x_c re-read the last one, so all loads
    // issue back to back and are waited for once, at store_in (a per-element conditional load makes hipcc wait
    // for each load in turn)
    const long pix = xin ? (((long)n * H + h) * W + w) * (long)a.x_cstride : 0;
    if constexpr (XIN == 2) {  // unaligned 16-byte loads (4-byte aligned): memcpy keeps hipcc from assuming 16
      __builtin_memcpy(&xlo, xf + pix, 16);
      __builtin_memcpy(&xhi, xf + pix + (a.x_c - 4), 16);
    } else if constexpr (XIN == 1) {
#pragma unroll
      for (int c = 0; c < 8; ++c) xr[c] = xf[pix + min(c, a.x_c - 1)];
    } else {
      xq = *reinterpret_cast<const uint4*>(x8 + pix);
    }
  };
  auto store_in = [&]() {
    if (tid < C::IPIX) {
      uint4 v = xq;
      if constexpr (XIN == 2) {
        float xz[8];
        const int sh = a.x_c - 4;  // xhi[k] = channel sh + k
#pragma unroll
        for (int c = 0; c < 4; ++c) xz[c] = xlo[c];
#pragma unroll
        for (int c = 4; c < 8; ++c) {
          const int k = c - sh;
          const float h = k == 0 ? xhi[0] : k == 1 ? xhi[1] : k == 2 ? xhi[2] : xhi[3];
          xz[c] = c < a.x_c ? h : 0.f;
        }
        v = Chunk<T>::pack(xz);
      } else if constexpr (XIN == 1) {
        float xz[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) xz[c] = c < a.x_c ? xr[c] : 0.f;
        v = Chunk<T>::pack(xz);
      }
      *reinterpret_cast<uint4*>(smem + C::I_OFF + tid * 16) = xin ? v : make_uint4(0, 0, 0, 0);
    }
  };

  int t = blockIdx.x;
  if (t < ntiles) {
    load_in(t);
    store_in();
    // the input of the block's second tile is in flight from here on (a whole tile ahead of its store_in)
    if (t + (int)gridDim.x < ntiles) load_in(t + gridDim.x);
  }
  __syncthreads();
  const int ycs2 = a.y_cstride * 2;
  for (; t < ntiles; t += gridDim.x) {
    const int n = t / (th * tw), rem = t - n * th * tw;
    const int r0 = (rem / tw) * C::TH, c0 = (rem % tw) * C::TW;
    // (1) conv1_1 + bias + relu of the (TH+2) x (TW+2) patch into both granule buffers (zero outside the frame)
    for (int f = wave; f < (C::PPIX + 15) / 16; f += C::NW) {
      const int p = f * 16 + col;
      const int pr = p / C::PW, pc = p - pr * C::PW;
      f32x4 acc1[4];
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) acc1[fc] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int tap = 4 * j + q;
        uint4 bv = make_uint4(0, 0, 0, 0);
        if (tap < 9 && p < C::PPIX)
          bv = *reinterpret_cast<const uint4*>(smem + C::I_OFF + ((pr + tap / 3) * C::IW + pc + tap % 3) * 16);
        if constexpr (PABL & 1) {
          asm volatile("" ::"v"(bv.x), "v"(bv.w));
        } else {
#pragma unroll
          for (int fc = 0; fc < 4; ++fc) mma16<T>(wf[j][fc], bv, acc1[fc]);
        }
      }
      const int h = r0 - 1 + pr, w = c0 - 1 + pc;
      const bool inside = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      uint2 pk[4];
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        const float4 bb = *reinterpret_cast<const float4*>(rmul + 128 + fc * 16 + 4 * q);
        const float b1[4] = {bb.x, bb.y, bb.z, bb.w};
        float v[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[jj] = inside ? fmaxf(acc1[fc][jj] + b1[jj], 0.f) : 0.f;
        pk[fc].x = bf16x2_bits(v[0], v[1]);
        pk[fc].y = bf16x2_bits(v[2], v[3]);
      }
      // whole 16-byte chunks per lane (conflict-free ds_write_b128 under swz2) instead of 8-byte halves
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const uint4 ck = chunk_pair(pk[2 * g], pk[2 * g + 1]);
        if (p < C::PPIX)
          *reinterpret_cast<uint4*>(smem + C::P_OFF + g * C::PBU + swz2(p, (q & 1) ? 2 + (q >> 1) : q >> 1)) = ck;
      }
    }
    lds_barrier();  // LDS only: the previous tile's output stores stay in flight across it
    const int tn = t + gridDim.x;
    // (3) conv1_2: 2 granules x 9 taps, operands straight from LDS, no barrier
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
    int abase[2];
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) {
      const int p = wave * 32 + fp * 16;
      abase[fp] = (p / C::TW) * C::PW + (p % C::TW) + col;
    }
    // K-step s = (granule s / 9, tap s % 9); the fragments of step s + 1 are read while step s's MFMAs run
    auto frags = [&](uint4 (&av)[4], uint4 (&bv)[2], int s) {
      const int cc = s / 9, tap = s - cc * 9;
      const char* wp = smem + s * C::WSLOT;
      const char* xp = smem + C::P_OFF + cc * C::PBU;
      const int toff = (tap / 3) * C::PW + tap % 3;
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) av[fc] = *reinterpret_cast<const uint4*>(wp + swz<64>(fc * 16 + col, q));
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) bv[fp] = *reinterpret_cast<const uint4*>(xp + swz2(abase[fp] + toff, q));
    };
    uint4 av[2][4], bv[2][2];
    frags(av[0], bv[0], 0);
#pragma unroll
    for (int s = 0; s < C::NSTEP; ++s) {
      if (s + 1 < C::NSTEP) frags(av[(s + 1) & 1], bv[(s + 1) & 1], s + 1);
      if constexpr (PABL & 2) {
#pragma unroll
        for (int fc = 0; fc < 4; ++fc) asm volatile("" ::"v"(av[s & 1][fc].x), "v"(av[s & 1][fc].w));
#pragma unroll
        for (int fp = 0; fp < 2; ++fp) asm volatile("" ::"v"(bv[s & 1][fp].x), "v"(bv[s & 1][fp].w));
      } else {
#pragma unroll
        for (int fc = 0; fc < 4; ++fc)
#pragma unroll
          for (int fp = 0; fp < 2; ++fp) mma16<T>(av[s & 1][fc], bv[s & 1][fp], acc[fc][fp]);
      }
    }
    if constexpr (!(PABL & 2)) {  // pin the order: step s+1's 6 reads ahead of step s's 8 MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
      for (int s = 0; s < C::NSTEP; ++s) {
        if (s + 1 < C::NSTEP) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 8, 0);
      }
    }
    if (tn < ntiles) store_in();  // ip was last read by this tile's first conv, before the barrier above
    // (2') the input of the tile after next goes in flight now, in the registers store_in just freed: one whole tile
    // of work (its epilogue, first conv and conv1_2) covers the HBM latency of the f32 frame reads
    if (tn + (int)gridDim.x < ntiles) load_in(tn + gridDim.x);
    // (4) epilogue: bias/affine/act -> bf16 staging -> 16-byte stores (+ fused 2x2 SAME max-pool)
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) {
      const int row = wave * 32 + fp * 16 + col;
      uint2 pk[4];
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        const int cl = fc * 16 + 4 * q;
        const float4 m4 = *reinterpret_cast<const float4*>(rmul + cl);
        const float4 a4 = *reinterpret_cast<const float4*>(rmul + 64 + cl);
        const float mul[4] = {m4.x, m4.y, m4.z, m4.w}, add[4] = {a4.x, a4.y, a4.z, a4.w};
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = fmaf(acc[fc][fp][j], mul[j], add[j]);
          if (a.act == VM_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
          else if (a.act == VM_ACT_SIGMOID) v[j] = sigmoid_precise(v[j]);
        }
        pk[fc].x = bf16x2_bits(v[0], v[1]);
        pk[fc].y = bf16x2_bits(v[2], v[3]);
      }
      if (a.hd) {  // the skip half's head partials of this lane's pixel: 2 MFMAs on the bf16 outputs just made
        f32x4 dacc = f32x4{0.f, 0.f, 0.f, 0.f};
        mma16<T>(hwf[0], make_uint4(pk[0].x, pk[0].y, pk[1].x, pk[1].y), dacc);
        mma16<T>(hwf[1], make_uint4(pk[2].x, pk[2].y, pk[3].x, pk[3].y), dacc);
        const int pc = fp * 16 + col;
        if (q < 3 && r0 + wave < H && c0 + pc < W)
          *reinterpret_cast<f32x4*>(a.hd + (((long)n * H + r0 + wave) * W + c0 + pc) * 12 + 4 * q) = dacc;
      }
      // 16-byte chunks: rows of 144 B make 8 consecutive rows hit 8 distinct 4-bank groups (conflict-free b128)
#pragma unroll
      for (int g = 0; g < 2; ++g)
        *reinterpret_cast<uint4*>(smem + C::S_OFF + row * C::SR + 64 * g +
                                  16 * ((q & 1) ? 2 + (q >> 1) : q >> 1)) = chunk_pair(pk[2 * g], pk[2 * g + 1]);
    }
    // one barrier publishes the staging, the next tile's input and (for the next first conv) the end of this
    // tile's patch reads; the stores below then overlap the next tile's first conv (staging is rewritten only
    // after the next tile's first barrier)
    lds_barrier();  // LDS only: the previous tile's output stores stay in flight across it
    T* yb = reinterpret_cast<T*>(a.y) + a.y_coff + (((long)n * H + r0) * W + c0) * (long)a.y_cstride;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yb, 0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int it = 0; it < C::BM * 8 / C::NT; ++it) {
      if (a.y_skip) break;
      const int idx = it * C::NT + tid;
      const int rr = idx >> 3, cq = idx & 7;
      const uint4 d = *reinterpret_cast<const uint4*>(smem + C::S_OFF + rr * C::SR + cq * 16);
      const int pr = rr / C::TW, pc = rr % C::TW;
      const bool ok = r0 + pr < H && c0 + pc < W && cq * 8 < a.cout && !(PABL & 4);
      const int off = ok ? (pr * W + pc) * ycs2 + cq * 16 : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), yrs,
                                             off, 0, 0);
    }
    if (a.py) {
      const int PH = (H + 1) >> 1, PWd = (W + 1) >> 1;
      const int pr0 = r0 >> 1, pc0 = c0 >> 1;
      T* pb = reinterpret_cast<T*>(a.py) + a.py_coff + (((long)n * PH + pr0) * PWd + pc0) * (long)a.py_cstride;
      const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pb, 0, 0x7ffffff0, 0x00020000);
      constexpr int PTW = C::TW / 2, PITEMS = C::BM / 4 * 8;
#pragma unroll
      for (int it = 0; it < (PITEMS + C::NT - 1) / C::NT; ++it) {
        const int idx = it * C::NT + tid;
        if (idx >= PITEMS) break;
        const int pp = idx >> 3, cq = idx & 7;
        const int pr = pp / PTW, pc = pp % PTW;
        const int rr = 2 * pr * C::TW + 2 * pc;
        const bool vh = r0 + 2 * pr + 1 < H, vw = c0 + 2 * pc + 1 < W;
        float m[8], f[8];
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + C::S_OFF + rr * C::SR + cq * 16), m);
        if (vw) {
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + C::S_OFF + (rr + 1) * C::SR + cq * 16), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
        }
        if (vh) {
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + C::S_OFF + (rr + C::TW) * C::SR + cq * 16), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
        }
        if (vh && vw) {
          Chunk<T>::unpack(*reinterpret_cast<const uint4*>(smem + C::S_OFF + (rr + C::TW + 1) * C::SR + cq * 16), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], f[j]);
        }
        const bool ok = pr0 + pr < PH && pc0 + pc < PWd && cq * 8 < a.cout && !(PABL & 4);
        const int off = ok ? ((pr * PWd + pc) * a.py_cstride + cq * 8) * 2 : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, Chunk<T>::pack(m)), prs, off, 0, 0);
      }
    }
  }
}

// ================================================================ first layer: cin <= 8 (conv1_1, unet.py:65-74)
// One 16-byte chunk per pixel, so a 32-deep MFMA K-step covers 4 taps x 8 channels: lane group q of the pixel
// fragment reads the patch row shifted by tap 4j+q (taps >= 9 read as zero), matching the tap-major packing
// k = tap*8 + c.  The 10 x 34 patch (5.4 KB) is loaded once per tile; the 64 x 96 weight slice sits in LDS (12 KB,
// one uint4 per MFMA operand lane: in registers it took 48 VGPRs and the persistent loop spilled).
// 8 waves of 32 px x 64 channels; same bf16 slab epilogue as the patch kernel.  Persistent: a block walks tiles
// b, b + G, ... (G a multiple of 8, so xcd_tile keeps each block on its XCD's tile range) with the next tile's
// patch chunk in flight in a register while the current one computes and stores, and reloads its weight slice
// only when the output-channel block changes.  (One tile per block spent ~10 us of serial load latency per tile
// at 2 resident blocks per CU: 185 us for the training towers' 2.5 M pixels, 1.7 TB/s of stores.)
__global__ __launch_bounds__(512, 4) void conv3x3_first(ConvArgs a) {
  using T = uint16_t;
  constexpr int TH = 8, TW = 32, PW = TW + 2, PPIX = (TH + 2) * PW, BM = TH * TW, SR = 64 * 2 + 16;
  __shared__ __attribute__((aligned(16))) uint4 patch[PPIX];
  __shared__ __attribute__((aligned(16))) char stg[BM * SR];
  __shared__ __attribute__((aligned(16))) uint4 wl[3][4][64];  // the weight slice, one uint4 per (step, fc, lane)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int col = lane & 15, q = lane >> 4;
  auto coords = [&](int l, int& n, int& r0, int& c0, int& n0) {
    const int t = xcd_tile(l, a.tiles_total);
    const int st = t / a.tiles_n, nt = t - st * a.tiles_n;
    n = st / (th * tw);
    const int srem = st - n * th * tw;
    r0 = (srem / tw) * TH;
    c0 = (srem - (srem / tw) * tw) * TW;
    n0 = nt * 64;
  };
  auto load_patch = [&](int n, int r0, int c0) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (tid < PPIX) {
      const T* xb = reinterpret_cast<const T*>(a.x) + a.x_coff + ((long)n * H + r0 - 1) * (long)W * cs;
      const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(xb), 0, 0x7ffffff0, 0x00020000);
      const int pr = tid / PW, pc = tid - pr * PW;
      const int h = r0 - 1 + pr, w = c0 - 1 + pc;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const int off = ok ? (pr * W + w) * cs * 2 : OOB;
      v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
    return v;
  };
  const int G = gridDim.x;
  int l = blockIdx.x;
  if (l >= a.tiles_total) return;
  int n, r0, c0, n0, wn0 = -1;
  coords(l, n, r0, c0, n0);
  uint4 pv = load_patch(n, r0, c0);
  for (; l < a.tiles_total; l += G) {
    if (n0 != wn0) {  // block-uniform; the previous tile's MFMAs are behind its two barriers
      const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, n0);
      for (int e = tid; e < 3 * 4 * 64; e += 512) {
        const int j = e >> 8, fc = (e >> 6) & 3, ln = e & 63;
        wl[j][fc][ln] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      wrs, ((fc * 16 + (ln & 15)) * a.K_pad + j * 32 + (ln >> 4) * 8) * 2,
                                                      0, 0));
      }
      wn0 = n0;
    }
    if (tid < PPIX) patch[tid] = pv;
    __syncthreads();
    // the next tile's patch chunk: in flight through this tile's MFMAs, epilogue and stores
    const int cn = n, cr0 = r0, cc0 = c0, cn0 = n0;
    if (l + G < a.tiles_total) {
      coords(l + G, n, r0, c0, n0);
      pv = load_patch(n, r0, c0);
    }

    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k < 2; ++k) acc[i][k] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int tap = 4 * j + q;
      const int toff = (tap / 3) * PW + tap % 3;
      uint4 bv[2];
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) {
        const int p = wave * 32 + fp * 16;  // tile pixel of the fragment's first row: one patch row per wave
        const uint4 v = patch[(p / TW) * PW + (p % TW) + col + (tap < 9 ? toff : 0)];
        bv[fp] = tap < 9 ? v : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        const uint4 wv = wl[j][fc][lane];
#pragma unroll
        for (int fp = 0; fp < 2; ++fp) mma16<T>(wv, bv[fp], acc[fc][fp]);
      }
    }

#pragma unroll
    for (int fc = 0; fc < 4; ++fc) {
      const int cc = fc * 16 + 4 * q;
      float mul[4], add[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int co = min(cn0 + cc + jj, a.cout - 1);
        const float sc = a.scale ? a.scale[co] : 1.f;
        mul[jj] = sc;
        add[jj] = (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
      }
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) {
        const int row = wave * 32 + fp * 16 + col;
        float v[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          v[jj] = fmaf(acc[fc][fp][jj], mul[jj], add[jj]);
          if (a.act == VM_ACT_RELU) v[jj] = fmaxf(v[jj], 0.f);
          else if (a.act == VM_ACT_SIGMOID) v[jj] = sigmoid_precise(v[jj]);
        }
        uint2 pk;
        pk.x = bf16x2_bits(v[0], v[1]);
        pk.y = bf16x2_bits(v[2], v[3]);
        *reinterpret_cast<uint2*>(stg + row * SR + cc * 2) = pk;
      }
    }
    __syncthreads();
    const int ycs2 = a.y_cstride * 2;
    T* yb = reinterpret_cast<T*>(a.y) + a.y_coff + (((long)cn * H + cr0) * W + cc0) * (long)a.y_cstride + cn0;
    const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yb, 0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int it = 0; it < BM * 8 / 512; ++it) {
      const int idx = it * 512 + tid;
      const int rr = idx >> 3, cq = idx & 7;
      const uint4 d = *reinterpret_cast<const uint4*>(stg + rr * SR + cq * 16);
      const int pr = rr / TW, pc = rr % TW;
      const bool ok = cr0 + pr < H && cc0 + pc < W && cn0 + cq * 8 < a.cout;
      const int off = ok ? (pr * W + pc) * ycs2 + cq * 16 : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, d), yrs,
                                             off, 0, 0);
    }
  }
}

// {x[l], x[l ^ 16]} and {x[l], x[l ^ 32]} in VALU (v_permlane16/32_swap of x with itself) instead of ds_bpermute:
// max and + of the pair are commutative, so the results equal fmaxf / + with __shfl_xor bit for bit
__device__ __forceinline__ float max_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float add_xor16(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add_xor32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ================================================================ refine conv4 + softmax (refine.py:27-32)
// RefineNet's only live layer: a cin <= 8 -> 64 3x3 conv whose 64 logits per pixel go straight into
// tf.nn.softmax and out as f32.  The conv is conv3x3_first's (one 16-byte chunk per pixel, 4 taps x 8 channels
// per K-step, the 64 x 96 weight slice in registers); the softmax never leaves registers: a pixel's 64 logits
// sit in the 4 lanes col, col+16, col+32, col+48 (16 each), so two xor-shuffles give the row max and the row
// sum.  Every lane then stores its four 16-byte channel quads (a wave store covers 16 pixels x 64 contiguous
// bytes).  The kernel writes 256 B per pixel and reads 16: HBM-write-bound.  NT: nontemporal stores (the
// 531 MB 1080p output is never re-read by this pass).
// STG: each wave transposes its 16 pixels x 64 channels through a private LDS slab so that every store instruction
// writes 4 whole pixels (1 KB contiguous when the output is dense) instead of 16 pixels x 64 bytes.
// WL: the weight fragments staged once per block in LDS instead of 48 registers (4 waves per SIMD without spills)
template <bool NT, bool STG = false, bool WL = false>
__global__ __launch_bounds__(512, WL ? 4 : 2) void conv3x3_first_softmax(ConvArgs a) {
  using T = uint16_t;
  constexpr int TH = 8, TW = 32, PW = TW + 2, PPIX = (TH + 2) * PW;
  constexpr int SRF = 68;  // staging row: 64 floats + 4 (rows 272 B apart)
  __shared__ __attribute__((aligned(16))) uint4 patch[PPIX];
  __shared__ __attribute__((aligned(16))) float stg[STG ? 8 * 16 * SRF : 4];
  __shared__ __attribute__((aligned(16))) float rmul[2 * 64];  // per-channel scale, bias*scale + shift
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int ntiles = a.tiles_total;
  // persistent: the block walks tiles blockIdx.x, +gridDim.x, ... (bands of consecutive tiles per XCD); the next
  // tile's patch pixel is loaded into a register while the current tile computes and stores
  auto tile_of = [&](int i) {  // a partial last round keeps block order (the band remap is a bijection of a full one)
    const int base = (i / a.tiles_n) * a.tiles_n;
    return base + a.tiles_n <= ntiles ? base + xcd_tile(i - base, a.tiles_n) : i;
  };
  auto load_patch = [&](int t) {
    const int n = t / (th * tw), srem = t - n * th * tw;
    const int r0 = (srem / tw) * TH, c0 = (srem - (srem / tw) * tw) * TW;
    const int pr = tid / PW, pc = tid - pr * PW;
    const int h = r0 - 1 + pr, w = c0 - 1 + pc;
    const bool ok = tid < PPIX && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    const T* xb = reinterpret_cast<const T*>(a.x) + a.x_coff + ((long)n * H + (ok ? h : 0)) * (long)W * cs;
    return ok ? *reinterpret_cast<const uint4*>(xb + (long)w * cs) : make_uint4(0, 0, 0, 0);
  };
  const int col = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, 0);
  __shared__ __attribute__((aligned(16))) uint4 wlds[WL ? 3 * 4 * 64 : 1];
  uint4 wf[WL ? 1 : 3][4];
  if constexpr (WL) {
    for (int e = tid; e < 3 * 4 * 64; e += 512) {  // [j][fc][lane]
      const int j = e >> 8, fc = (e >> 6) & 3, l = e & 63;
      wlds[e] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                              wrs, ((fc * 16 + (l & 15)) * a.K_pad + j * 32 + (l >> 4) * 8) * 2, 0, 0));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int fc = 0; fc < 4; ++fc)
        wf[j][fc] = __builtin_bit_cast(
            uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, ((fc * 16 + col) * a.K_pad + j * 32 + q * 8) * 2, 0, 0));
  }
  if (tid < 64) {  // constants in LDS (read per tile): 2 blocks per CU fit the register file
    const float sc = a.scale ? a.scale[tid] : 1.f;
    rmul[tid] = sc;
    rmul[64 + tid] = (a.bias ? a.bias[tid] : 0.f) * sc + (a.shift ? a.shift[tid] : 0.f);
  }
  int i = blockIdx.x;
  uint4 nxt = i < ntiles ? load_patch(tile_of(i)) : make_uint4(0, 0, 0, 0);
  for (; i < ntiles; i += gridDim.x) {
    const int t = tile_of(i);
    const int n = t / (th * tw), srem = t - n * th * tw;
    const int r0 = (srem / tw) * TH, c0 = (srem - (srem / tw) * tw) * TW;
    __syncthreads();  // the previous tile's patch reads are done
    if (tid < PPIX) patch[tid] = nxt;
    __syncthreads();
    if (i + (int)gridDim.x < ntiles) nxt = load_patch(tile_of(i + gridDim.x));

    f32x4 acc[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) acc[k][fp] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int tap = 4 * j + q;
      const int toff = (tap / 3) * PW + tap % 3;
      uint4 bv[2];
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) {
        const uint4 v = patch[wave * PW + fp * 16 + col + (tap < 9 ? toff : 0)];  // patch row `wave` + kernel row
        bv[fp] = tap < 9 ? v : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        const uint4 wv = WL ? wlds[(j * 4 + fc) * 64 + lane] : wf[WL ? 0 : j][fc];
#pragma unroll
        for (int fp = 0; fp < 2; ++fp) mma16<T>(wv, bv[fp], acc[fc][fp]);
      }
    }

    const int ycs = a.y_cstride;
    float* yb = reinterpret_cast<float*>(a.y) + a.y_coff + (((long)n * H + r0 + wave) * W + c0) * (long)ycs;
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) {
      float v[4][4];
      float mx = -INFINITY;
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        const float4 m4 = *reinterpret_cast<const float4*>(rmul + fc * 16 + 4 * q);
        const float4 a4 = *reinterpret_cast<const float4*>(rmul + 64 + fc * 16 + 4 * q);
        const float mul[4] = {m4.x, m4.y, m4.z, m4.w}, add[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          v[fc][jj] = fmaf(acc[fc][fp][jj], mul[jj], add[jj]);
          mx = fmaxf(mx, v[fc][jj]);
        }
      }
      mx = max_xor32(max_xor16(mx));
      float sum = 0.f;
#pragma unroll
      for (int fc = 0; fc < 4; ++fc)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          v[fc][jj] = expf(v[fc][jj] - mx);
          sum += v[fc][jj];
        }
      sum = add_xor32(add_xor16(sum));
      const float inv = 1.f / sum;
      if constexpr (STG) {
        float* ws = stg + wave * 16 * SRF;
#pragma unroll
        for (int fc = 0; fc < 4; ++fc)
          *reinterpret_cast<f32x4*>(ws + col * SRF + fc * 16 + 4 * q) =
              f32x4{v[fc][0] * inv, v[fc][1] * inv, v[fc][2] * inv, v[fc][3] * inv};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int it = 0; it < 4; ++it) {  // lane l: pixel 4*it + l/16, channels 4*(l%16) .. +3
          const int px = 4 * it + (lane >> 4), ch = 4 * (lane & 15);
          const f32x4 o = *reinterpret_cast<const f32x4*>(ws + px * SRF + ch);
          const int pc = fp * 16 + px;
          if (r0 + wave < H && c0 + pc < W) {
            float* yp = yb + (long)pc * ycs + ch;
            if constexpr (NT) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(yp));
            else *reinterpret_cast<f32x4*>(yp) = o;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads done before the next fragment's writes
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
        const int pc = fp * 16 + col;
        if (r0 + wave < H && c0 + pc < W) {
          float* yp = yb + (long)pc * ycs + 4 * q;
#pragma unroll
          for (int fc = 0; fc < 4; ++fc) {
            const f32x4 o = f32x4{v[fc][0] * inv, v[fc][1] * inv, v[fc][2] * inv, v[fc][3] * inv};
            if constexpr (NT) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(yp + fc * 16));
            else *reinterpret_cast<f32x4*>(yp + fc * 16) = o;
          }
        }
      }
    }
  }
}

// The refine softmax of one wave's 32-pixel x 64-channel accumulator strip (acc[fc][fp]: MFMA 16x16 layout, pixel
// fp*16 + col, channels fc*16 + 4q .. +3), its per-channel affine from rmul ([scale | bias*scale + shift]), and the
// whole-pixel nontemporal stores through the wave's private 16 x 68-float LDS slab `ws`: every store instruction
// writes 4 whole pixels.  `valid` = pixels of the strip inside the frame.
// strip accumulators: zero (the epilogue applies the affine), or the bias (no scale / shift: rmul[64..] = bias)
__device__ __forceinline__ void init_strip_acc(f32x4 (&acc)[4][2], const float* rmul, bool aff, int q) {
#pragma unroll
  for (int fc = 0; fc < 4; ++fc) {
    const f32x4 b = aff ? f32x4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f32x4*>(rmul + 64 + fc * 16 + 4 * q);
    acc[fc][0] = b;
    acc[fc][1] = b;
  }
}

// AFF: apply rmul's per-channel affine; without it the accumulators already hold the logits (the kernel started
// them at the bias: the refine conv has no BN, scale/shift are absent).  The exponential is v_exp_f32 on x*log2(e)
// (__expf): for the softmax of logits bounded by max-subtraction its relative error (~1e-6 near 0, below 1e-5
// absolute on every probability) is far inside the 1e-4 bound, at a third of expf's instructions — this epilogue is
// the VALU-bound half of the kernel.
template <bool AFF>
__device__ __forceinline__ void softmax_store_strip(const f32x4 (&acc)[4][2], const float* rmul, float* ws, float* yb,
                                                    int ycs, int valid, int lane) {
  constexpr int SRF = 68;
  const int col = lane & 15, q = lane >> 4;
#pragma unroll
  for (int fp = 0; fp < 2; ++fp) {
    float v[4][4];
    float mx = -INFINITY;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) {
      if constexpr (AFF) {
        const float4 m4 = *reinterpret_cast<const float4*>(rmul + fc * 16 + 4 * q);
        const float4 a4 = *reinterpret_cast<const float4*>(rmul + 64 + fc * 16 + 4 * q);
        const float mul[4] = {m4.x, m4.y, m4.z, m4.w}, add[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[fc][jj] = fmaf(acc[fc][fp][jj], mul[jj], add[jj]);
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) v[fc][jj] = acc[fc][fp][jj];
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) mx = fmaxf(mx, v[fc][jj]);
    }
    mx = max_xor32(max_xor16(mx));
    float sum = 0.f;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v[fc][jj] = __expf(v[fc][jj] - mx);
        sum += v[fc][jj];
      }
    sum = add_xor32(add_xor16(sum));
    const float inv = 1.f / sum;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc)
      *reinterpret_cast<f32x4*>(ws + col * SRF + fc * 16 + 4 * q) =
          f32x4{v[fc][0] * inv, v[fc][1] * inv, v[fc][2] * inv, v[fc][3] * inv};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < 4; ++it) {  // lane l: pixel 4*it + l/16, channels 4*(l%16) .. +3
      const int px = 4 * it + (lane >> 4), ch = 4 * (lane & 15);
      const f32x4 o = *reinterpret_cast<const f32x4*>(ws + px * SRF + ch);
      const int pc = fp * 16 + px;
      if (pc < valid) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(yb + (long)pc * ycs + ch));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// bf16 refine conv4 + softmax on wave-private strips (see conv3x3_first_softmax_f32 below for the strip scheme): the
// conv is conv3x3_first's (one 16-byte pixel chunk per lane, 4 taps x 8 channels per 32-deep K-step, 3 steps); each
// wave stages its 3 x 34-pixel patch, the weight fragments live in LDS ([step][fc][lane]), no block barrier per tile.
__global__ __launch_bounds__(512, 4) void conv3x3_first_softmax_strip(ConvArgs a) {
  using T = uint16_t;
  constexpr int TH = 8, TW = 32, PW = TW + 2, SP = 3 * PW;
  constexpr int SRF = 68;
  __shared__ __attribute__((aligned(16))) uint4 wlds[3 * 4 * 64];
  __shared__ __attribute__((aligned(16))) float rmul[2 * 64];
  __shared__ __attribute__((aligned(16))) uint4 pat[8 * SP];
  __shared__ __attribute__((aligned(16))) float stg[8 * 16 * SRF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int ntiles = a.tiles_total;
  auto tile_of = [&](int i) {
    const int base = (i / a.tiles_n) * a.tiles_n;
    return base + a.tiles_n <= ntiles ? base + xcd_tile(i - base, a.tiles_n) : i;
  };
  auto load_strip = [&](int t, uint4 (&v)[2]) {
    const int n = t / (th * tw), srem = t - n * th * tw;
    const int r = (srem / tw) * TH + wave, c0 = (srem - (srem / tw) * tw) * TW;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const int pr = e / PW, pc = e - pr * PW;
      const int h = r - 1 + pr, w = c0 - 1 + pc;
      const bool ok = e < SP && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const T* xp = reinterpret_cast<const T*>(a.x) + a.x_coff + ((long)n * H + (ok ? h : 0)) * (long)W * cs +
                    (long)(ok ? w : 0) * cs;
      v[k] = ok ? *reinterpret_cast<const uint4*>(xp) : make_uint4(0, 0, 0, 0);
    }
  };
  const int col = lane & 15, q = lane >> 4;
  const __amdgpu_buffer_rsrc_t wrs = w_rsrc<T>(a, 0);
  for (int e = tid; e < 3 * 4 * 64; e += 512) {  // [j][fc][lane]
    const int j = e >> 8, fc = (e >> 6) & 3, l = e & 63;
    wlds[e] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            wrs, ((fc * 16 + (l & 15)) * a.K_pad + j * 32 + (l >> 4) * 8) * 2, 0, 0));
  }
  if (tid < 64) {
    const float sc = a.scale ? a.scale[tid] : 1.f;
    rmul[tid] = sc;
    rmul[64 + tid] = (a.bias ? a.bias[tid] : 0.f) * sc + (a.shift ? a.shift[tid] : 0.f);
  }
  uint4* P = pat + wave * SP;
  const bool aff = a.scale || a.shift;  // else the accumulators start at the bias and hold the logits
  __syncthreads();  // the only block-wide barrier: the staged tables
  int i = blockIdx.x;
  uint4 nv[2];
  if (i < ntiles) load_strip(tile_of(i), nv);
  for (; i < ntiles; i += gridDim.x) {
    const int t = tile_of(i);
    const int n = t / (th * tw), srem = t - n * th * tw;
    const int r = (srem / tw) * TH + wave, c0 = (srem - (srem / tw) * tw) * TW;
    P[lane] = nv[0];
    if (lane + 64 < SP) P[lane + 64] = nv[1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (i + (int)gridDim.x < ntiles) load_strip(tile_of(i + gridDim.x), nv);
    if (r >= H) continue;
    f32x4 acc[4][2];
    init_strip_acc(acc, rmul, aff, q);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int tap = 4 * j + q;
      const int toff = (tap / 3) * PW + tap % 3;
      uint4 bv[2];
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) {
        const uint4 v = P[fp * 16 + col + (tap < 9 ? toff : 0)];
        bv[fp] = tap < 9 ? v : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        const uint4 wv = wlds[(j * 4 + fc) * 64 + lane];
#pragma unroll
        for (int fp = 0; fp < 2; ++fp) mma16<T>(wv, bv[fp], acc[fc][fp]);
      }
    }
    float* yb = reinterpret_cast<float*>(a.y) + a.y_coff + (((long)n * H + r) * W + c0) * (long)a.y_cstride;
    if (aff) softmax_store_strip<true>(acc, rmul, stg + wave * 16 * SRF, yb, a.y_cstride, W - c0, lane);
    else softmax_store_strip<false>(acc, rmul, stg + wave * 16 * SRF, yb, a.y_cstride, W - c0, lane);
  }
}

// ================================================================ refine conv4 + softmax in f32 (refine.py:27-32)
// The reference's precision for config 3: f32 input row [cmp, alpha, warped] (CIN <= 8 of an 8-channel pixel), exact
// f32 products on v_mfma_f32_16x16x4_f32, f32 sums, f32 softmax.  K is COMPACT: k = tap * CIN + c over the 9 * CIN
// real taps (45 for the refine's CIN 5 -> 12 four-deep MFMA steps instead of the 18 of the padded 72); the lane in
// k-slot q of step s reads tap (4s+q) / CIN, channel (4s+q) % CIN.
// Work unit = one wave's STRIP (1 output row x 32 px x 64 channels): the wave stages its own 3 x 34 px patch in LDS as
// channel planes (the 16 lanes of a k-slot read 16 consecutive pixels: conflict-free) and never waits for the other
// waves, so one wave's MFMA phase (12 steps x 8 MFMAs of 32 cycles) runs under another's softmax + store phase; a
// block-wide barrier per tile had serialised the two (0.225 ms at 1080p).  The 8 waves of a block take the 8 rows of
// one 8 x 32 tile (their halo rows meet in L1/L2), tiles walk persistently in XCD bands.  Weights and per-lane patch
// offsets are staged once per block ([step][lane] records: one ds_read_b128 for the 4 cout fragments + one offset);
// the next strip's pixels are prefetched into registers.  Softmax + per-wave LDS transpose + whole-pixel nontemporal
// stores as in conv3x3_first_softmax.
template <int CIN, int ABL = 0>  // ABL (study builds only, results are garbage): 1 = no softmax / store, 2 = no MFMA
__global__ __launch_bounds__(512, 4) void conv3x3_first_softmax_f32(ConvArgs a) {
  constexpr int NS = (9 * CIN + 3) / 4;
  constexpr int TH = 8, TW = 32, PW = TW + 2, SP = 3 * PW;  // strip patch: 3 rows x 34 px
  constexpr int WPF = (CIN * SP + 32 + 3) / 4 * 4;            // per-wave patch floats (+ 32 zeros)
  constexpr int ZERO = CIN * SP;
  constexpr int SRF = 68;  // staging row: 64 floats + 4
  __shared__ __attribute__((aligned(16))) f32x4 wl[NS * 64];
  __shared__ int pl[NS * 4];
  __shared__ __attribute__((aligned(16))) float rmul[2 * 64];
  __shared__ __attribute__((aligned(16))) float pat[8 * WPF];
  __shared__ __attribute__((aligned(16))) float stg[8 * 16 * SRF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int ntiles = a.tiles_total;
  auto tile_of = [&](int i) {
    const int base = (i / a.tiles_n) * a.tiles_n;
    return base + a.tiles_n <= ntiles ? base + xcd_tile(i - base, a.tiles_n) : i;
  };
  // this wave's strip of tile t: rows r - 1 .. r + 1 (r = tile row 0 + wave), pixels c0 - 1 .. c0 + 32; lane e (and
  // e + 64) fetch patch pixel e
  auto load_strip = [&](int t, float4 (&v)[2][2]) {
    const int n = t / (th * tw), srem = t - n * th * tw;
    const int r = (srem / tw) * TH + wave, c0 = (srem - (srem / tw) * tw) * TW;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const int pr = e / PW, pc = e - pr * PW;
      const int h = r - 1 + pr, w = c0 - 1 + pc;
      const bool ok = e < SP && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const float* xp = reinterpret_cast<const float*>(a.x) + a.x_coff + ((long)n * H + (ok ? h : 0)) * (long)W * cs +
                        (long)(ok ? w : 0) * cs;
      v[k][0] = ok ? *reinterpret_cast<const float4*>(xp) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[k][1] = ok && CIN > 4 ? *reinterpret_cast<const float4*>(xp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const int col = lane & 15, q = lane >> 4;
  const float* Wt = reinterpret_cast<const float*>(a.w);
  for (int e = tid; e < NS * 64; e += 512) {  // wl[s][l] = the 4 cout fragments of lane l's (tap, c) at step s
    const int st = e >> 6, l = e & 63;
    const int kk = 4 * st + (l >> 4), co = l & 15;
    const int tap = kk / CIN, c = kk - tap * CIN;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kk < 9 * CIN)
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) v[fc] = Wt[(long)(fc * 16 + co) * a.K_pad + tap * 8 + c];
    wl[e] = v;
  }
  if (tid < NS * 4) {
    const int kk = tid;  // step tid / 4, k-slot tid % 4
    const int tap = kk / CIN, c = kk - tap * CIN;
    pl[tid] = kk < 9 * CIN ? c * SP + (tap / 3) * PW + tap % 3 : ZERO;  // k past 9 * CIN: 32 zeros
  }
  float* P = pat + wave * WPF;
  if (lane < 32) P[ZERO + lane] = 0.f;
  if (tid < 64) {
    const float sc = a.scale ? a.scale[tid] : 1.f;
    rmul[tid] = sc;
    rmul[64 + tid] = (a.bias ? a.bias[tid] : 0.f) * sc + (a.shift ? a.shift[tid] : 0.f);
  }
  const bool aff = a.scale || a.shift;  // else the accumulators start at the bias and hold the logits
  __syncthreads();  // the only block-wide barrier: the staged tables
  int poff[NS];  // this lane's patch offset of every K step in registers (no dependent LDS load per step)
#pragma unroll
  for (int s = 0; s < NS; ++s) poff[s] = pl[s * 4 + q] + col;
  int i = blockIdx.x;
  float4 nv[2][2];
  if (i < ntiles) load_strip(tile_of(i), nv);
  for (; i < ntiles; i += gridDim.x) {
    const int t = tile_of(i);
    const int n = t / (th * tw), srem = t - n * th * tw;
    const int r = (srem / tw) * TH + wave, c0 = (srem - (srem / tw) * tw) * TW;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const float v[8] = {nv[k][0].x, nv[k][0].y, nv[k][0].z, nv[k][0].w, nv[k][1].x, nv[k][1].y, nv[k][1].z, nv[k][1].w};
      if (e < SP)
#pragma unroll
        for (int c = 0; c < CIN; ++c) P[c * SP + e] = v[c];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (i + (int)gridDim.x < ntiles) load_strip(tile_of(i + gridDim.x), nv);
    if (r >= H) continue;  // a strip below the frame (wave-uniform): nothing to compute or store

    f32x4 acc[4][2];
    init_strip_acc(acc, rmul, aff, q);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const f32x4 w4 = wl[s * 64 + lane];
      const float b0 = P[poff[s]], b1 = P[poff[s] + 16];
      if constexpr (ABL & 2) {
        asm volatile("" ::"v"(w4[0]), "v"(w4[3]), "v"(b0), "v"(b1));
        continue;
      }
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        acc[fc][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[fc], b0, acc[fc][0], 0, 0, 0);
        acc[fc][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[fc], b1, acc[fc][1], 0, 0, 0);
      }
    }

    if constexpr (ABL & 1) {
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) asm volatile("" ::"v"(acc[fc][0][0]), "v"(acc[fc][1][3]));
      continue;
    }
    float* yb = reinterpret_cast<float*>(a.y) + a.y_coff + (((long)n * H + r) * W + c0) * (long)a.y_cstride;
    if (aff) softmax_store_strip<true>(acc, rmul, stg + wave * 16 * SRF, yb, a.y_cstride, W - c0, lane);
    else softmax_store_strip<false>(acc, rmul, stg + wave * 16 * SRF, yb, a.y_cstride, W - c0, lane);
  }
}

// Pipelined form of conv3x3_first_softmax_f32 (r04): a wave computes strip i+1's MFMAs (accumulator set N) in the same
// basic block as strip i's softmax + stores (set C), so the matrix pipe runs under the VALU-bound softmax instead of
// beside it only when another wave happens to be in the other phase (ablations: the two phases of the non-pipelined
// kernel overlapped by ~0.02 ms).  What makes one basic block possible: the per-wave patch is double-buffered, the
// output is written straight from the accumulator lanes (per (16-pixel fragment, 16-channel group) one store of 16
// pixels x 64 contiguous bytes: the four stores of a fragment fill its 16 whole pixels) through a buffer descriptor
// whose out-of-range offsets drop the pixels past the frame — no LDS transpose, no wave barrier, no branch; the next
// strip's global loads are clamped the same way.  Arithmetic per output is the non-pipelined kernel's (same K order,
// same softmax expression), so results are bit-identical to it.

// The strip softmax of softmax_store_strip cut into 10 chunks, one per K step of the next strip's MFMAs, computed in
// place in the accumulators C (acc[fc][fp]: pixel fp*16 + col, channels fc*16 + 4q .. +3); same operations in the same
// order as softmax_store_strip (max over fc, jj; exp and the sum fc-major), so the probabilities are bit-identical.
// Chunks: 0, 1 affine + row max of fragment 0 / 1; 2 the max across the 4 lane groups; 3..6 exp + partial sums (half a
// fragment each); 7 the sums across lanes and their reciprocals; 8, 9 the scaled stores of fragment 0 / 1, straight
// from the lanes (per 16-channel group one store of 16 pixels x 64 contiguous bytes; pixels past `valid` dropped by
// the buffer descriptor's range check).
// AUX: the stores' cache policy (0: through L2, where the four 64-byte pieces of a pixel's 256-byte row meet before
// write-back; 2: non-temporal, each piece its own partial-line write)
// AUX & 16: the scaled fragment goes through a wave-private LDS slab (16 pixels x 68 floats) and leaves as 4 stores
// of 4 whole pixels (1 KB contiguous for a dense 64-channel output), with cache policy AUX & 15.
template <bool AFF, int S, int ABL = 0, int AUX = 0>  // ABL (study build, timing only): 1 no stores, 4 no softmax math
__device__ __forceinline__ void softmax_chunk(f32x4 (&C)[4][2], float (&mx)[2], float (&sm)[2], const float* rmul,
                                              __amdgpu_buffer_rsrc_t yrs, int ycs, int valid, int lane,
                                              float* slab = nullptr) {
  const int col = lane & 15, q = lane >> 4;
  if constexpr ((ABL & 4) && S < 8) {
    return;
  } else if constexpr (S == 0 || S == 1) {
    constexpr int fp = S;
    float m = -INFINITY;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) {
      if constexpr (AFF) {
        const float4 m4 = *reinterpret_cast<const float4*>(rmul + fc * 16 + 4 * q);
        const float4 a4 = *reinterpret_cast<const float4*>(rmul + 64 + fc * 16 + 4 * q);
        const float mul[4] = {m4.x, m4.y, m4.z, m4.w}, add[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) C[fc][fp][jj] = fmaf(C[fc][fp][jj], mul[jj], add[jj]);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) m = fmaxf(m, C[fc][fp][jj]);
    }
    mx[fp] = m;
  } else if constexpr (S == 2) {
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) mx[fp] = max_xor32(max_xor16(mx[fp]));
  } else if constexpr (S >= 3 && S <= 6) {
    constexpr int fp = (S - 3) / 2, h = (S - 3) % 2;
    float t = h ? sm[fp] : 0.f;
#pragma unroll
    for (int fc = 2 * h; fc < 2 * h + 2; ++fc)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        C[fc][fp][jj] = __expf(C[fc][fp][jj] - mx[fp]);
        t += C[fc][fp][jj];
      }
    sm[fp] = t;
  } else if constexpr (S == 7) {
#pragma unroll
    for (int fp = 0; fp < 2; ++fp) sm[fp] = 1.f / add_xor32(add_xor16(sm[fp]));
  } else if constexpr ((S == 8 || S == 9) && (AUX & 16)) {
    constexpr int fp = S - 8, SRF = 68;
    const float inv = sm[fp];
#pragma unroll
    for (int fc = 0; fc < 4; ++fc)
      *reinterpret_cast<f32x4*>(slab + col * SRF + fc * 16 + 4 * q) =
          f32x4{C[fc][fp][0] * inv, C[fc][fp][1] * inv, C[fc][fp][2] * inv, C[fc][fp][3] * inv};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int it = 0; it < 4; ++it) {  // lane l: pixel 4 it + l / 16, channels 4 (l % 16) .. +3
      const int px = 4 * it + (lane >> 4), ch = 4 * (lane & 15);
      const f32x4 o = *reinterpret_cast<const f32x4*>(slab + px * SRF + ch);
      const int pc = fp * 16 + px;
      if constexpr (ABL & 1) {
        asm volatile("" ::"v"(o[0]), "v"(o[3]));
        continue;
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, o), yrs,
                                             pc < valid ? (pc * ycs + ch) * 4 : OOB, 0, AUX & 15);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the slab's reads retire before fragment 1 rewrites it
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else if constexpr (S == 8 || S == 9) {
    constexpr int fp = S - 8;
    const float inv = sm[fp];
    const int pc = fp * 16 + col;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) {
      const f32x4 o = f32x4{C[fc][fp][0] * inv, C[fc][fp][1] * inv, C[fc][fp][2] * inv, C[fc][fp][3] * inv};
      if constexpr (ABL & 1) {
        asm volatile("" ::"v"(o[0]), "v"(o[3]));
        continue;
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, o), yrs,
                                             pc < valid ? (pc * ycs + fc * 16 + 4 * q) * 4 : OOB, 0, AUX);
    }
  }
}

// X6 (CIN <= 5): the same conv at f32 accuracy on the bf16 MFMA (v_mfma_f32_16x16x32_bf16, 16x the f32 rate).  Each
// f32 input x and filter tap w is split exactly into three bf16 parts (h + m + l, as split6_kernel in elementwise.hip),
// and one 32-deep K step per tap carries the six products l*Wh + m*Wm + h*Wl + m*Wh + h*Wm + h*Wh of every channel
// (the parts' 24 significant bits; the dropped m*Wl, l*Wm, l*Wl terms are below 2^-24 of h*Wh): the per-wave patch
// holds a 64-byte record [l, m, h, m, h, h] (CIN channels each, zero padded) per pixel in 4 chunk planes, the weight
// table the matching [Wh, Wm, Wl, Wh, Wm, Wh] fragments.  9 steps of 8 bf16 MFMAs replace 12 of 8 f32 ones at a
// quarter of the cycles each, which leaves the kernel bound by its softmax and its 256-byte-per-pixel output stores.
// Single-buffered patch (the LDS budget: 36 KB of weight fragments + 8 x 6.5 KB of records + the store slabs; a wave's
// LDS reads and writes stay in program order, so restaging over the previous strip's records is safe).
__device__ __forceinline__ void split3_bf16(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = f2bf(x);
  const float r1 = x - bf2f((uint16_t)h);
  m = f2bf(r1);
  l = f2bf(r1 - bf2f((uint16_t)m));
}

template <int CIN, int MINW = 2, bool AFF = false, int ABL = 0, int AUX = 0, bool X6 = false>  // MINW: min waves per
                                                                      // SIMD; AFF: a scale / shift epilogue; AUX: stores
__global__ __launch_bounds__(512, MINW) void conv3x3_first_softmax_f32p(ConvArgs a) {  // epilogue; ABL: study only
  static_assert(!X6 || CIN * 6 <= 32, "x6: six parts of every channel in one 32-deep K step");
  constexpr int NS = X6 ? 9 : (9 * CIN + 3) / 4;
  constexpr int TH = 8, TW = 32, PW = TW + 2, SP = 3 * PW;
  constexpr int WPF = X6 ? 4 * SP * 4 : (CIN * SP + 32 + 3) / 4 * 4;  // per-wave patch floats (x6: 4 chunk planes)
  constexpr int NBUF = X6 ? 1 : 2;
  constexpr int ZERO = CIN * SP;
  __shared__ __attribute__((aligned(16))) f32x4 wl[X6 ? 1 : NS * 64];
  __shared__ __attribute__((aligned(16))) uint4 wx[X6 ? 9 * 4 * 64 : 1];  // x6: [tap][fc][lane] A fragments
  __shared__ int pl[X6 ? 1 : NS * 4];
  __shared__ __attribute__((aligned(16))) float rmul[2 * 64];
  __shared__ __attribute__((aligned(16))) float pat[8 * NBUF * WPF];
  __shared__ __attribute__((aligned(16))) float stg[(AUX & 16) ? 8 * 16 * 68 : 4];  // AUX & 16: the store slabs
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* const slab = stg + ((AUX & 16) ? wave * 16 * 68 : 0);
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int th = (H + TH - 1) / TH, tw = (W + TW - 1) / TW;
  const int ntiles = a.tiles_total;
  const int G = (int)gridDim.x;
  auto tile_of = [&](int i) {
    const int base = (i / a.tiles_n) * a.tiles_n;
    return base + a.tiles_n <= ntiles ? base + xcd_tile(i - base, a.tiles_n) : i;
  };
  // strip i of this wave: frame n, row r, first column c0 (i past the end: a zero strip below every frame)
  auto strip = [&](int i, int& n, int& r, int& c0) __attribute__((always_inline)) {
    const bool real = i < ntiles;
    const int t = tile_of(real ? i : 0);
    n = t / (th * tw);
    const int srem = t - n * th * tw;
    r = real ? (srem / tw) * TH + wave : H;
    c0 = (srem - (srem / tw) * tw) * TW;
  };
  // strip coordinates are decoded outside the interleaved region (the decode's integer divisions expand with
  // branches, which would split the basic block the schedule below needs)
  struct SC {
    int n, r, c0;
  };
  auto coords = [&](int i) __attribute__((always_inline)) {
    SC c;
    strip(i, c.n, c.r, c.c0);
    return c;
  };
  auto load_strip = [&](const SC& sc, float4 (&v)[2][2]) __attribute__((always_inline)) {
    const int n = sc.n, r = sc.r, c0 = sc.c0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const int pr = e / PW, pc = e - pr * PW;
      const int h = r - 1 + pr, w = c0 - 1 + pc;
      const bool ok = e < SP && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const float* xp = reinterpret_cast<const float*>(a.x) + a.x_coff + ((long)n * H + (ok ? h : 0)) * (long)W * cs +
                        (long)(ok ? w : 0) * cs;
      v[k][0] = ok ? *reinterpret_cast<const float4*>(xp) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[k][1] = ok && CIN > 4 ? *reinterpret_cast<const float4*>(xp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const int col = lane & 15, q = lane >> 4;
  const float* Wt = reinterpret_cast<const float*>(a.w);
  if constexpr (X6) {
    // k slot kk of a tap: part group g = kk / CIN (record [l, m, h, m, h, h] against filter parts [h, m, l, h, m, h]),
    // channel kk % CIN; slots past 6 * CIN are zero
    for (int e = tid; e < 9 * 4 * 64; e += 512) {
      const int tap = e >> 8, fc = (e >> 6) & 3, l = e & 63;
      const int co = fc * 16 + (l & 15);
      uint32_t v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = 8 * (l >> 4) + j, g = kk / CIN, c = kk - g * CIN;
        uint32_t h = 0, m = 0, lo = 0;
        if (kk < 6 * CIN) split3_bf16(Wt[(long)co * a.K_pad + tap * 8 + c], h, m, lo);
        v[j] = g == 0 || g == 3 || g == 5 ? h : g == 1 || g == 4 ? m : g == 2 ? lo : 0u;
      }
      wx[e] = make_uint4(v[0] | v[1] << 16, v[2] | v[3] << 16, v[4] | v[5] << 16, v[6] | v[7] << 16);
    }
  } else {
    for (int e = tid; e < NS * 64; e += 512) {
      const int st = e >> 6, l = e & 63;
      const int kk = 4 * st + (l >> 4), co = l & 15;
      const int tap = kk / CIN, c = kk - tap * CIN;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (kk < 9 * CIN)
#pragma unroll
        for (int fc = 0; fc < 4; ++fc) v[fc] = Wt[(long)(fc * 16 + co) * a.K_pad + tap * 8 + c];
      wl[e] = v;
    }
    if (tid < NS * 4) {
      const int kk = tid;
      const int tap = kk / CIN, c = kk - tap * CIN;
      pl[tid] = kk < 9 * CIN ? c * SP + (tap / 3) * PW + tap % 3 : ZERO;
    }
  }
  float* P0 = pat + wave * NBUF * WPF;
  float* P1 = P0 + (NBUF - 1) * WPF;
  if (!X6 && lane < 32) {
    P0[ZERO + lane] = 0.f;
    P1[ZERO + lane] = 0.f;
  }
  if (tid < 64) {
    const float sc = a.scale ? a.scale[tid] : 1.f;
    rmul[tid] = sc;
    rmul[64 + tid] = (a.bias ? a.bias[tid] : 0.f) * sc + (a.shift ? a.shift[tid] : 0.f);
  }
  constexpr bool aff = AFF;
  __syncthreads();  // the only block-wide barrier: the staged tables
  auto stage = [&](float* P, const float4 (&v)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const float vv[8] = {v[k][0].x, v[k][0].y, v[k][0].z, v[k][0].w, v[k][1].x, v[k][1].y, v[k][1].z, v[k][1].w};
      if constexpr (X6) {  // the pixel's 32-slot record [l, m, h, m, h, h] as 4 chunk planes of SP x 16 bytes
        uint32_t h[CIN], m[CIN], lo[CIN], r[32];
#pragma unroll
        for (int c = 0; c < CIN; ++c) split3_bf16(vv[c], h[c], m[c], lo[c]);
#pragma unroll
        for (int kk = 0; kk < 32; ++kk) {
          const int g = kk / CIN, c = kk % CIN;
          r[kk] = kk >= 6 * CIN ? 0u : g == 0 ? lo[c] : (g == 1 || g == 3) ? m[c] : h[c];
        }
        if (e < SP)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            reinterpret_cast<uint4*>(P)[j * SP + e] =
                make_uint4(r[8 * j] | r[8 * j + 1] << 16, r[8 * j + 2] | r[8 * j + 3] << 16,
                           r[8 * j + 4] | r[8 * j + 5] << 16, r[8 * j + 6] | r[8 * j + 7] << 16);
      } else if (e < SP) {
#pragma unroll
        for (int c = 0; c < CIN; ++c) P[c * SP + e] = vv[c];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // the MFMAs of strip P into N; with C, the 10 softmax chunks of the previous strip, one per K step: each step is its
  // own scheduling region (sched_barrier), so the chunk's VALU work issues between that step's MFMAs, and the next
  // step's fragments are read under them
  // this lane's patch offsets of every K step (the pl table's entry for its k-slot q, plus its pixel column), held
  // in registers: read from LDS inside the step they made each step's fragment reads wait on a dependent LDS load
  int poff[X6 ? 1 : NS];
  if constexpr (!X6) {
#pragma unroll
    for (int s = 0; s < NS; ++s) poff[s] = pl[s * 4 + q] + col;
  }
  // x6: step s = tap s; A = the 4 cout fragments of the tap, B = chunk q of the records of pixels col, col + 16
  auto mma_x6 = [&](const float* P, f32x4 (&N)[4][2], f32x4* Cp, const __amdgpu_buffer_rsrc_t& yrs, int valid)
      __attribute__((always_inline)) {
    init_strip_acc(N, rmul, aff, q);
    float mx[2] = {0.f, 0.f}, sm[2] = {0.f, 0.f};
    const uint4* R = reinterpret_cast<const uint4*>(P) + q * SP + col;
    uint4 av[4], bv[2];
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) av[fc] = wx[fc * 64 + lane];
    bv[0] = R[0];
    bv[1] = R[16];
    static_for<0, 9>([&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      uint4 an[4], bn[2];
      if constexpr (s + 1 < 9) {
        constexpr int toff = ((s + 1) / 3) * PW + (s + 1) % 3;
#pragma unroll
        for (int fc = 0; fc < 4; ++fc) an[fc] = wx[((s + 1) * 4 + fc) * 64 + lane];
        bn[0] = R[toff];
        bn[1] = R[toff + 16];
      }
      if constexpr (!(ABL & 2)) {
#pragma unroll
        for (int fc = 0; fc < 4; ++fc) {
          mma16<uint16_t>(av[fc], bv[0], N[fc][0]);
          mma16<uint16_t>(av[fc], bv[1], N[fc][1]);
        }
      }
      if (Cp) {
        softmax_chunk<AFF, s, ABL, AUX>(*reinterpret_cast<f32x4(*)[4][2]>(Cp), mx, sm, rmul, yrs, a.y_cstride, valid,
                                        lane, slab);
      }
      if constexpr (s + 1 < 9) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (s + 1 < 9) {
#pragma unroll
        for (int fc = 0; fc < 4; ++fc) av[fc] = an[fc];
        bv[0] = bn[0];
        bv[1] = bn[1];
      }
    });
    if (Cp) {  // the 10th chunk
      softmax_chunk<AFF, 9, ABL, AUX>(*reinterpret_cast<f32x4(*)[4][2]>(Cp), mx, sm, rmul, yrs, a.y_cstride, valid,
                                      lane, slab);
    }
  };
  auto mma = [&](const float* P, f32x4 (&N)[4][2], f32x4* Cp, const __amdgpu_buffer_rsrc_t& yrs, int valid)
      __attribute__((always_inline)) {
    if constexpr (X6) {
      mma_x6(P, N, Cp, yrs, valid);
    } else {
      init_strip_acc(N, rmul, aff, q);
      float mx[2] = {0.f, 0.f}, sm[2] = {0.f, 0.f};
      f32x4 w4 = wl[lane];
      float b0 = P[poff[0]], b1 = P[poff[0] + 16];
      static_for<0, NS>([&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        f32x4 w4n = w4;
        float b0n = b0, b1n = b1;
        if constexpr (s + 1 < NS) {
          w4n = wl[(s + 1) * 64 + lane];
          b0n = P[poff[s + 1]];
          b1n = P[poff[s + 1] + 16];
        }
        if constexpr (ABL & 2) {
          asm volatile("" ::"v"(w4[0]), "v"(w4[3]), "v"(b0), "v"(b1));
        } else {
  #pragma unroll
          for (int fc = 0; fc < 4; ++fc) {
            N[fc][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[fc], b0, N[fc][0], 0, 0, 0);
            N[fc][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[fc], b1, N[fc][1], 0, 0, 0);
          }
        }
        if (Cp) {
          if constexpr (s < 10)
            softmax_chunk<AFF, s, ABL, AUX>(*reinterpret_cast<f32x4(*)[4][2]>(Cp), mx, sm, rmul, yrs, a.y_cstride, valid,
                                            lane, slab);
        }
        // the next step's fragment reads first (else hipcc sinks them to the step's end and the next step's first
        // MFMA waits a whole LDS latency), then one MFMA per 3 VALU of the softmax chunk
        if constexpr (s + 1 < NS) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        if constexpr (s + 1 >= NS) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
        w4 = w4n;
        b0 = b0n;
        b1 = b1n;
      });
      if (Cp) {  // a short K loop (CIN < 4): the chunks left over
        static_for<NS, 10>([&](auto sc) __attribute__((always_inline)) {
          softmax_chunk<AFF, decltype(sc)::value, ABL, AUX>(*reinterpret_cast<f32x4(*)[4][2]>(Cp), mx, sm, rmul, yrs,
                                                             a.y_cstride, valid, lane, slab);
        });
      }
    }
  };
  auto yrs_of = [&](const SC& sc, int& valid) __attribute__((always_inline)) {
    float* yb = reinterpret_cast<float*>(a.y) + a.y_coff +
                (((long)sc.n * H + (sc.r < H ? sc.r : 0)) * W + sc.c0) * (long)a.y_cstride;
    valid = sc.r < H ? W - sc.c0 : 0;
    return __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(yb), 0, 0x7ffffff0, 0x00020000);
  };
  // the last strip's softmax alone (no MFMAs left to hide it under)
  auto store = [&](const SC& sc, f32x4 (&C)[4][2]) __attribute__((always_inline)) {
    int valid;
    const __amdgpu_buffer_rsrc_t yrs = yrs_of(sc, valid);
    float mx[2] = {0.f, 0.f}, sm[2] = {0.f, 0.f};
    static_for<0, 10>([&](auto sc2) __attribute__((always_inline)) {
      softmax_chunk<AFF, decltype(sc2)::value, ABL, AUX>(C, mx, sm, rmul, yrs, a.y_cstride, valid, lane, slab);
    });
  };
  int cur = blockIdx.x;
  if (cur >= ntiles) return;
  float4 nv[2][2];
  SC s0 = coords(cur), s1 = coords(cur + G), s2;  // strips cur (accumulators C), cur + G (patch in flight)
  load_strip(s0, nv);
  stage(P0, nv);
  load_strip(s1, nv);
  f32x4 acc0[4][2], acc1[4][2];
  {
    int v0;
    mma(P0, acc0, nullptr, yrs_of(s0, v0), 0);
  }
  // one step: strip cur's accumulators are in C; stage strip cur+G into buffer B and compute it into N while C's
  // softmax and stores go out between its MFMAs
  auto step = [&](auto bconst, f32x4 (&C)[4][2], f32x4 (&N)[4][2]) __attribute__((always_inline)) {
    constexpr int b = decltype(bconst)::value;
    float* Pn = b ? P1 : P0;
    stage(Pn, nv);
    s2 = coords(cur + 2 * G);
    int valid;
    const __amdgpu_buffer_rsrc_t yrs = yrs_of(s0, valid);
    load_strip(s2, nv);
    mma(Pn, N, &C[0][0], yrs, valid);
    s0 = s1;
    s1 = s2;
    cur += G;
  };
  while (true) {
    if (cur + G >= ntiles) {
      store(s0, acc0);
      break;
    }
    step(std::integral_constant<int, 1>{}, acc0, acc1);
    if (cur + G >= ntiles) {
      store(s0, acc1);
      break;
    }
    step(std::integral_constant<int, 0>{}, acc1, acc0);
  }
}

// Row-ring form of conv3x3_first_softmax_f32p (r04): a wave walks a column band of 32 pixels down a segment of
// a.seg rows instead of taking one row of an 8-row tile, so each strip stages ONE new input row (its window's bottom
// row) instead of three: the per-wave patch is a ring of 4 row slots, and the rows in slots 0 and 1 are written
// twice (slots 4 and 5 too), so the 3-row window of every strip is contiguous at slot base (strip - first) % 4 and
// the per-step patch offsets stay fixed registers (the window base moves the pointer, not the offsets).  Staging
// alone was 0.048 of the pipelined kernel's 0.167 ms (smxabl abl 7): 3 input rows read per output row.  The MFMA
// order, softmax chunks and stores are the pipelined kernel's, so results are bit-identical to it.
template <int CIN, int AUX = 18>
__global__ __launch_bounds__(512, 2) void conv3x3_first_softmax_f32r(ConvArgs a) {
  constexpr int NS = (9 * CIN + 3) / 4;
  constexpr int TW = 32, PW = TW + 2, SP = 6 * PW;  // 6 row slots: ring of 4 + copies of slots 0 and 1
  constexpr int ZERO = CIN * SP;                     // 32 + 3 * PW zeros: the padded k-slots read at any base
  constexpr int WPF = (ZERO + 32 + 3 * PW + 3) / 4 * 4;
  constexpr bool AFF = false;
  __shared__ __attribute__((aligned(16))) f32x4 wl[NS * 64];
  __shared__ int pl[NS * 4];
  __shared__ __attribute__((aligned(16))) float rmul[2 * 64];
  __shared__ __attribute__((aligned(16))) float pat[8 * WPF];
  __shared__ __attribute__((aligned(16))) float stg[(AUX & 16) ? 8 * 16 * 68 : 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* const slab = stg + ((AUX & 16) ? wave * 16 * 68 : 0);
  const int H = a.H, W = a.W, cs = a.x_cstride;
  const int tw = (W + TW - 1) / TW, RS = a.seg, nseg = (H + RS - 1) / RS;
  const int nitems = a.tiles_total;  // frames x segments x bands
  const int gw = blockIdx.x * 8 + wave, GW = (int)gridDim.x * 8;
  // strip = (item, row); the walk: rows r0 .. rend-1 of item gw, then of gw + GW, ...
  struct SC {
    int n, r, c0, rend, item;
  };
  auto item_start = [&](int item) __attribute__((always_inline)) {
    SC c;
    c.item = item;
    if (item >= nitems) {
      c.n = 0; c.r = H; c.c0 = 0; c.rend = H;
      return c;
    }
    const int band = item % tw, t = item / tw;
    const int seg = t % nseg;
    c.n = t / nseg;
    c.c0 = band * TW;
    c.r = seg * RS;
    c.rend = min(H, c.r + RS);
    return c;
  };
  auto next_strip = [&](const SC& c) __attribute__((always_inline)) {
    if (c.item < nitems && c.r + 1 < c.rend) {
      SC d = c;
      d.r += 1;
      return d;
    }
    return item_start(c.item + GW);
  };
  const int col = lane & 15, q = lane >> 4;
  const float* Wt = reinterpret_cast<const float*>(a.w);
  for (int e = tid; e < NS * 64; e += 512) {
    const int st = e >> 6, l = e & 63;
    const int kk = 4 * st + (l >> 4), co = l & 15;
    const int tap = kk / CIN, c = kk - tap * CIN;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (kk < 9 * CIN)
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) v[fc] = Wt[(long)(fc * 16 + co) * a.K_pad + tap * 8 + c];
    wl[e] = v;
  }
  if (tid < NS * 4) {
    const int kk = tid;
    const int tap = kk / CIN, c = kk - tap * CIN;
    pl[tid] = kk < 9 * CIN ? c * SP + (tap / 3) * PW + tap % 3 : ZERO;
  }
  float* const P = pat + wave * WPF;
  for (int e = lane; e < 32 + 3 * PW; e += 64) P[ZERO + e] = 0.f;
  if (tid < 64) {
    rmul[tid] = 1.f;
    rmul[64 + tid] = a.bias ? a.bias[tid] : 0.f;
  }
  __syncthreads();  // the only block-wide barrier: the staged tables
  int poff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) poff[s] = pl[s * 4 + q] + col;
  // input rows of a strip: its whole 3-row window when it starts an item (first), else the window's bottom row
  auto load_rows = [&](const SC& sc, bool first, float4 (&v)[2][2]) __attribute__((always_inline)) {
    const int n = sc.n, c0 = sc.c0;
    const int rlo = first ? sc.r - 1 : sc.r + 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const int pr = e / PW, pc = e - pr * PW;
      const int h = rlo + pr, w = c0 - 1 + pc;
      const bool ok = e < (first ? 3 * PW : PW) && sc.r < H && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const float* xp = reinterpret_cast<const float*>(a.x) + a.x_coff + ((long)n * H + (ok ? h : 0)) * (long)W * cs +
                        (long)(ok ? w : 0) * cs;
      v[k][0] = ok ? *reinterpret_cast<const float4*>(xp) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[k][1] = ok && CIN > 4 ? *reinterpret_cast<const float4*>(xp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // ring slot of the window's first row for strip row r of an item starting at r0
  auto base_of = [&](const SC& sc) __attribute__((always_inline)) {
    return (sc.r - (sc.r / RS) * RS) & 3;
  };
  auto stage = [&](const SC& sc, bool first, const float4 (&v)[2][2]) __attribute__((always_inline)) {
    const int j = base_of(sc);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = lane + 64 * k;
      const float vv[8] = {v[k][0].x, v[k][0].y, v[k][0].z, v[k][0].w, v[k][1].x, v[k][1].y, v[k][1].z, v[k][1].w};
      const int pr = e / PW, pc = e - pr * PW;
      const int slot = first ? pr : (j + 2) & 3;  // first: window base 0
      if (e < (first ? 3 * PW : PW)) {
#pragma unroll
        for (int c = 0; c < CIN; ++c) {
          P[c * SP + slot * PW + pc] = vv[c];
          if (slot < 2) P[c * SP + (slot + 4) * PW + pc] = vv[c];
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto mma = [&](const float* Pw, f32x4 (&N)[4][2], f32x4* Cp, const __amdgpu_buffer_rsrc_t& yrs, int valid)
      __attribute__((always_inline)) {
    init_strip_acc(N, rmul, false, q);
    float mx[2] = {0.f, 0.f}, sm[2] = {0.f, 0.f};
    f32x4 w4 = wl[lane];
    float b0 = Pw[poff[0]], b1 = Pw[poff[0] + 16];
    static_for<0, NS>([&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      f32x4 w4n = w4;
      float b0n = b0, b1n = b1;
      if constexpr (s + 1 < NS) {
        w4n = wl[(s + 1) * 64 + lane];
        b0n = Pw[poff[s + 1]];
        b1n = Pw[poff[s + 1] + 16];
      }
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) {
        N[fc][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[fc], b0, N[fc][0], 0, 0, 0);
        N[fc][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w4[fc], b1, N[fc][1], 0, 0, 0);
      }
      if (Cp) {
        if constexpr (s < 10)
          softmax_chunk<AFF, s, 0, AUX>(*reinterpret_cast<f32x4(*)[4][2]>(Cp), mx, sm, rmul, yrs, a.y_cstride, valid,
                                        lane, slab);
      }
      if constexpr (s + 1 < NS) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
      if constexpr (s + 1 >= NS) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_barrier(0);
      w4 = w4n;
      b0 = b0n;
      b1 = b1n;
    });
    if (Cp) {
      static_for<NS, 10>([&](auto sc) __attribute__((always_inline)) {
        softmax_chunk<AFF, decltype(sc)::value, 0, AUX>(*reinterpret_cast<f32x4(*)[4][2]>(Cp), mx, sm, rmul, yrs,
                                                         a.y_cstride, valid, lane, slab);
      });
    }
  };
  auto yrs_of = [&](const SC& sc, int& valid) __attribute__((always_inline)) {
    float* yb = reinterpret_cast<float*>(a.y) + a.y_coff +
                (((long)sc.n * H + (sc.r < H ? sc.r : 0)) * W + sc.c0) * (long)a.y_cstride;
    valid = sc.r < H ? W - sc.c0 : 0;
    return __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(yb), 0, 0x7ffffff0, 0x00020000);
  };
  auto store = [&](const SC& sc, f32x4 (&C)[4][2]) __attribute__((always_inline)) {
    int valid;
    const __amdgpu_buffer_rsrc_t yrs = yrs_of(sc, valid);
    float mx[2] = {0.f, 0.f}, sm[2] = {0.f, 0.f};
    static_for<0, 10>([&](auto sc2) __attribute__((always_inline)) {
      softmax_chunk<AFF, decltype(sc2)::value, 0, AUX>(C, mx, sm, rmul, yrs, a.y_cstride, valid, lane, slab);
    });
  };
  SC s0 = item_start(gw);
  if (s0.item >= nitems) return;  // (wave-uniform; the block barrier above is behind every wave)
  float4 nv[2][2];
  load_rows(s0, true, nv);
  stage(s0, true, nv);
  SC s1 = next_strip(s0);
  bool f1 = s1.item != s0.item;
  load_rows(s1, f1, nv);
  f32x4 acc0[4][2], acc1[4][2];
  {
    int v0;
    mma(P + base_of(s0) * PW, acc0, nullptr, yrs_of(s0, v0), 0);
  }
  // one step: strip s0's accumulators are in C; stage strip s1 and compute it into N while C's softmax and stores go
  // out between its MFMAs
  auto step = [&](f32x4 (&C)[4][2], f32x4 (&N)[4][2]) __attribute__((always_inline)) {
    stage(s1, f1, nv);
    const SC s2 = next_strip(s1);
    const bool f2 = s2.item != s1.item;
    int valid;
    const __amdgpu_buffer_rsrc_t yrs = yrs_of(s0, valid);
    load_rows(s2, f2, nv);
    mma(P + base_of(s1) * PW, N, &C[0][0], yrs, valid);
    s0 = s1;
    s1 = s2;
    f1 = f2;
  };
  while (true) {
    if (s1.item >= nitems) {
      store(s0, acc0);
      break;
    }
    step(acc0, acc1);
    if (s1.item >= nitems) {
      store(s0, acc1);
      break;
    }
    step(acc1, acc0);
  }
}

// ================================================================ Cout == 1 head (conv1_5 + sigmoid)
// unet.py:203-205 / unet_simple.py:142 / small.py:49-50: a 1-channel 3x3 conv over <=128 channels at full
// resolution is a memory-bound dot product: 16 lanes per pixel, each lane one 16-byte channel chunk per
// tap (a wave reads 4 pixels x 256 contiguous bytes), a 4-step xor-shuffle reduction inside each 16-lane
// group, weights un-permuted once per block into tap-major order in LDS.
struct HeadArgs {
  const void* x;
  int x_cstride, x_coff, H, W;
  long M;
  int cin_pad, K9, K_pad, chunk_major, ng;
  const void* w;
  const float* bias;
  const float* scale;
  const float* shift;
  int act;
  void* y;
  int y_cstride, y_coff, y_dtype;
  float* y2;  // optional: sigmoid of the pre-activation value, f32 [M] (unet.py:204-205 output beside conv1_3)
  const float* part;  // optional: per-tap partials [M][12] of the channels x does not carry (the pair kernel's hd)
  const float* yacc;  // optional: f32 [M] added to the pre-activation (a head over channel chunks, split-bf16 x6)
};

template <typename T>
__global__ __launch_bounds__(256) void conv3x3_head(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CE = 16 / sizeof(T);
  constexpr int GE = 64 / sizeof(T);
  float* sw = reinterpret_cast<float*>(smem);
  const T* Wt = reinterpret_cast<const T*>(a.w);
  for (int k = threadIdx.x; k < a.K_pad; k += 256) {
    int tap, c;
    if (a.chunk_major) {
      const int g = k / GE;
      if (g >= a.ng) continue;
      const int cc = g / 9;
      tap = g - cc * 9;
      c = cc * GE + (k - g * GE);
    } else {
      if (k >= a.K9) continue;
      tap = k / a.cin_pad;
      c = k - tap * a.cin_pad;
    }
    sw[tap * a.cin_pad + c] = ld_elem<T>(Wt + k);
  }
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
      if (a.y2) a.y2[p] = sigmoid_precise(v);
      if (a.act == VM_ACT_RELU) v = v > 0.f ? v : 0.f;
      else if (a.act == VM_ACT_SIGMOID) v = sigmoid_precise(v);
      else if (a.act == VM_ACT_SOFTMAX) v = 1.f;  // softmax over a single channel
      const long o = p * (long)a.y_cstride + a.y_coff;
      if (a.y_dtype == VM_BF16) reinterpret_cast<uint16_t*>(a.y)[o] = f2bf(v);
      else reinterpret_cast<float*>(a.y)[o] = v;
    }
  }
}

// Strip variant for cin_pad == 16 * CE * NCH (conv1_5: 128 channels).  A 16-lane group owns NCH 16-byte channel
// chunks of P consecutive output pixels of one row: it loads the 3 x (P+2) input pixels once (all loads of a
// row in flight together), keeps its 9-tap weight slice in registers and reduces the P sums across the group.
// bf16 uses v_dot2_f32_bf16 on the packed pairs (f32 accumulation, no unpack); f32 uses fma.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

template <typename T, int NCH>
__device__ __forceinline__ float chunk_dot(const uint4 (&x)[NCH], const uint4 (&w)[NCH], float acc) {
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const uint32_t xs[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
    const uint32_t ws[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (sizeof(T) == 2)
        acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, xs[j]), __builtin_bit_cast(bf16x2_t, ws[j]),
                                              acc, false);
      else
        acc = fmaf(__uint_as_float(xs[j]), __uint_as_float(ws[j]), acc);
    }
  }
  return acc;
}

template <typename T, int NCH, int P>
__global__ __launch_bounds__(256) void conv3x3_head_strip(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CE = 16 / sizeof(T);
  constexpr int GE = 64 / sizeof(T);
  T* sw = reinterpret_cast<T*>(smem);  // [9][cin_pad] tap-major, compute dtype
  const T* Wt = reinterpret_cast<const T*>(a.w);
  for (int k = threadIdx.x; k < a.K_pad; k += 256) {
    int tap, c;
    if (a.chunk_major) {
      const int g = k / GE;
      if (g >= a.ng) continue;
      const int cc = g / 9;
      tap = g - cc * 9;
      c = cc * GE + (k - g * GE);
    } else {
      if (k >= a.K9) continue;
      tap = k / a.cin_pad;
      c = k - tap * a.cin_pad;
    }
    sw[tap * a.cin_pad + c] = Wt[k];
  }
  __syncthreads();

  const int sub = threadIdx.x & 15;
  const int grp = threadIdx.x >> 4;
  const int H = a.H, W = a.W, cs = a.x_cstride;
  uint4 wr[9][NCH];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int q = 0; q < NCH; ++q)
      wr[t][q] = *reinterpret_cast<const uint4*>(sw + t * a.cin_pad + (q * 16 + sub) * CE);

  const T* X = reinterpret_cast<const T*>(a.x) + a.x_coff;
  const float bias = a.bias ? a.bias[0] : 0.f;
  const float sc = a.scale ? a.scale[0] : 1.f;
  const float sh = a.shift ? a.shift[0] : 0.f;
  const int spr = (W + P - 1) / P;
  const long rows = a.M / W;
  const long nstrips = rows * spr;
  const int rowb = W * cs * (int)sizeof(T);
  for (long s0 = (long)blockIdx.x * 16; s0 < nstrips; s0 += (long)gridDim.x * 16) {
    // buffer descriptor rebased on the row above the block's first strip (wave-uniform); halo and
    // out-of-image taps get an out-of-range offset and read as zero (SAME padding)
    const long row0 = s0 / spr - 1;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(X + row0 * (long)W * cs), 0, 0x7ffffff0, 0x00020000);
    const long s = s0 + grp;
    if (s >= nstrips) break;
    const long row = s / spr;
    const int w0 = (int)(s - row * spr) * P;
    const int h = (int)(row % H);
    const int rel = (int)(row - row0);
    float acc[P];
#pragma unroll
    for (int o = 0; o < P; ++o) acc[o] = 0.f;
#pragma unroll
    for (int dh = -1; dh <= 1; ++dh) {
      const bool rok = (unsigned)(h + dh) < (unsigned)H;
      const int rbase = (rel + dh) * rowb + sub * CE * (int)sizeof(T);
      uint4 v[P + 2][NCH];
#pragma unroll
      for (int i = 0; i < P + 2; ++i) {
        const int ww = w0 - 1 + i;
        const bool ok = rok && (unsigned)ww < (unsigned)W;
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
          const int off = ok ? rbase + ww * cs * (int)sizeof(T) + q * 16 * CE * (int)sizeof(T) : OOB;
          v[i][q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the row's loads in flight together (the scheduler serialises them)
#pragma unroll
      for (int i = 0; i < P + 2; ++i)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const int o = i - dw;
          if (o >= 0 && o < P) acc[o] = chunk_dot<T, NCH>(v[i], wr[(dh + 1) * 3 + dw], acc[o]);
        }
    }
    float mine = 0.f;
#pragma unroll
    for (int o = 0; o < P; ++o) {
      float r = acc[o];
      r += __shfl_xor(r, 8, 16);
      r += __shfl_xor(r, 4, 16);
      r += __shfl_xor(r, 2, 16);
      r += __shfl_xor(r, 1, 16);
      if (sub == o) mine = r;
    }
    if (sub < P && w0 + sub < W) {
      float v = (mine + bias) * sc + sh;
      if (a.y2) a.y2[row * W + w0 + sub] = sigmoid_precise(v);
      if (a.act == VM_ACT_RELU) v = v > 0.f ? v : 0.f;
      else if (a.act == VM_ACT_SIGMOID) v = sigmoid_precise(v);
      else if (a.act == VM_ACT_SOFTMAX) v = 1.f;
      const long o = (row * W + w0 + sub) * (long)a.y_cstride + a.y_coff;
      if (a.y_dtype == VM_BF16) reinterpret_cast<uint16_t*>(a.y)[o] = f2bf(v);
      else reinterpret_cast<float*>(a.y)[o] = v;
    }
  }
}

// MFMA head: cout == 1 recast as a 1x1 GEMM over the 9 taps.  For a TH x TW output tile the block computes
// Y[p][t] = sum_c X[p][c] * W[t][c] for every pixel p of the (TH+2) x (TW+2) input window (MFMA: 16 pixels x
// 16 tap-columns, 9 used), parks Y in LDS, then out(r,c) = sum_t Y[(r+dh_t, c+dw_t)][t].  Every input pixel is
// read once per tile (plus the halo) straight into MFMA A-fragments; no 3x3 re-reads, no VALU dot products.
// ALIAS (split-fp16 x3, vmatting/split3.py): x holds two slabs [l, h] of S = cin / 3 channels and the filter runs over
// [l, h, h] (cin = 3S): the k-steps of the third range reuse the second range's fragments (no extra loads), so one
// call does conv1_5's three products, the small ones first in each tap's chain
template <typename T, int TH, int TW, int NKS, bool ALIAS = false>
__global__ __launch_bounds__(256) void conv3x3_head_mfma(HeadArgs a) {
  constexpr int CE = 16 / sizeof(T);
  constexpr int KS = 4 * CE;  // channels per MFMA k-step
  constexpr int GE = 64 / sizeof(T);
  constexpr int IW = TW + 2, NPIX = (TH + 2) * IW, NG = (NPIX + 15) / 16;
  // pixel groups whose loads are in flight together (ALIAS: 8 of the 12 k-steps' fragments are loaded, so the
  // registers hold 4 groups)
  constexpr int GB = ALIAS ? 4 : 3;
  constexpr int NL = ALIAS ? 2 * (NKS / 3) : NKS;  // fragments loaded per pixel group
  __shared__ float ys[NG * 16 * 9];
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* sw = reinterpret_cast<T*>(smem);  // [9][cin_pad] tap-major
  const T* Wt = reinterpret_cast<const T*>(a.w);
  if (sizeof(T) == 2 && a.chunk_major) {
    // 16-byte pieces: 8 consecutive k of a granule are 8 consecutive channels of one tap (the element loop below
    // issued 14 dependent 2-byte loads per thread for a 384-channel head before any pixel load)
    const int nvec = a.ng * GE / 8;
    for (int v = threadIdx.x; v < nvec; v += 256) {
      const int k = v * 8, g = k / GE, cc = g / 9, tap = g - cc * 9;
      *reinterpret_cast<uint4*>(sw + tap * a.cin_pad + cc * GE + (k - g * GE)) =
          *reinterpret_cast<const uint4*>(Wt + k);
    }
  } else {
    for (int k = threadIdx.x; k < a.K_pad; k += 256) {
      int tap, c;
      if (a.chunk_major) {
        const int g = k / GE;
        if (g >= a.ng) continue;
        const int cc = g / 9;
        tap = g - cc * 9;
        c = cc * GE + (k - g * GE);
      } else {
        if (k >= a.K9) continue;
        tap = k / a.cin_pad;
        c = k - tap * a.cin_pad;
      }
      sw[tap * a.cin_pad + c] = Wt[k];
    }
  }
  __syncthreads();

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, ks = lane >> 4;
  const int H = a.H, W = a.W, cs = a.x_cstride, cin = a.cin_pad;
  uint4 wf[NKS];
#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const int c = s * KS + ks * CE;
    wf[s] = (col < 9 && c < cin) ? *reinterpret_cast<const uint4*>(sw + col * cin + c) : make_uint4(0, 0, 0, 0);
  }

  const int tw = (W + TW - 1) / TW, th = (H + TH - 1) / TH;
  const int b = blockIdx.x;
  const int n = b / (tw * th), rem = b - n * tw * th;
  const int r0 = (rem / tw) * TH, c0 = (rem % tw) * TW;
  const T* base = reinterpret_cast<const T*>(a.x) + a.x_coff + ((long)n * H + r0 - 1) * (long)W * cs;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(base), 0, 0x7ffffff0, 0x00020000);

  for (int g0 = wave * GB; g0 < NG; g0 += 4 * GB) {
    uint4 xa[GB][NL];
    float pv[GB][4];  // head split: the partials this lane adds (issued with the input loads, used after the MFMAs)
#pragma unroll
    for (int u = 0; u < GB; ++u) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = (g0 + u) * 16 + 4 * ks + i, lr = j / IW, lc = j - lr * IW;
        const int hh = r0 - 1 + lr, ww = c0 - 1 + lc;
        const bool ok = a.part && col < 9 && g0 + u < NG && j < NPIX && (unsigned)hh < (unsigned)H &&
                        (unsigned)ww < (unsigned)W;
        pv[u][i] = ok ? a.part[(((long)n * H + hh) * W + ww) * 12 + col] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < GB; ++u) {
      const int j = (g0 + u) * 16 + col;  // input-window pixel of this lane's A row
      const int lr = j / IW, lc = j - lr * IW;
      const int hh = r0 - 1 + lr, ww = c0 - 1 + lc;
      const bool ok = g0 + u < NG && j < NPIX && (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
      const int pix = (lr * W + ww) * cs;
#pragma unroll
      for (int s = 0; s < NL; ++s) {  // (ALIAS: the third range reuses the second's fragments)
        const int c = s * KS + ks * CE;
        const int off = (ok && c < cin) ? (pix + c) * (int)sizeof(T) : OOB;
        xa[u][s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < GB; ++u) {
      if (g0 + u >= NG) break;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NKS; ++s) mma16<T>(xa[u][s < NL ? s : s - NKS / 3], wf[s], acc);
      if (col < 9) {
        const int p = (g0 + u) * 16 + 4 * ks;
#pragma unroll
        for (int i = 0; i < 4; ++i) ys[(p + i) * 9 + col] = acc[i] + pv[u][i];  // + the other channels' share
      }
    }
  }
  __syncthreads();

  const float bias = a.bias ? a.bias[0] : 0.f;
  const float sc = a.scale ? a.scale[0] : 1.f;
  const float sh = a.shift ? a.shift[0] : 0.f;
  for (int o = tid; o < TH * TW; o += 256) {
    const int orow = o / TW, ocol = o - orow * TW;
    const int h = r0 + orow, w = c0 + ocol;
    if (h >= H || w >= W) continue;
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) sum += ys[((orow + t / 3) * IW + ocol + t % 3) * 9 + t];
    if (a.yacc) sum += a.yacc[((long)n * H + h) * W + w];
    float v = (sum + bias) * sc + sh;
    if (a.y2) a.y2[((long)n * H + h) * W + w] = sigmoid_precise(v);
    if (a.act == VM_ACT_RELU) v = v > 0.f ? v : 0.f;
    else if (a.act == VM_ACT_SIGMOID) v = sigmoid_precise(v);
    else if (a.act == VM_ACT_SOFTMAX) v = 1.f;
    const long oi = (((long)n * H + h) * W + w) * a.y_cstride + a.y_coff;
    if (a.y_dtype == VM_BF16) reinterpret_cast<uint16_t*>(a.y)[oi] = f2bf(v);
    else reinterpret_cast<float*>(a.y)[oi] = v;
  }
}

// ================================================================ weight packing
// HWIO f32 [3][3][cin][cout] (unet.py:15 / the VGG npy layout) -> [cout_pad][K_pad] in the compute dtype,
// K in granule order (see the header comment).
template <typename T>
__global__ void pack_weights(const float* w, int cin, int cout, ConvArgs g) {
  constexpr int GE = 64 / sizeof(T);
  T* out = reinterpret_cast<T*>(const_cast<void*>(g.w));
  const long total = (long)g.cout_pad * g.K_pad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i / g.K_pad);
    const int k = (int)(i - (long)co * g.K_pad);
    int tap, c;
    k_to_tap<GE>(g, k, tap, c);
    float v = 0.f;
    if (co < cout && tap < 9 && c < cin) v = w[((long)tap * cin + c) * cout + co];
    st_elem<T>(out + i, v);
  }
}

constexpr int PACK_MAX_JOBS = 48;
struct PackBatch {
  int n;
  vm_pack_job j[PACK_MAX_JOBS];
  int K_pad[PACK_MAX_JOBS], cout_pad[PACK_MAX_JOBS], cin_pad[PACK_MAX_JOBS];
};

// job blockIdx.y: k_to_tap's decode of the conv geometry (as pack_weights), value from the (flipped) source filter
__global__ void pack_weights_batch(PackBatch b) {
  const vm_pack_job& j = b.j[blockIdx.y];
  const bool bf = j.dtype == VM_BF16;
  const int GE = bf ? 32 : 16;
  ConvArgs g{};
  g.cin_pad = b.cin_pad[blockIdx.y];
  g.K9 = 9 * g.cin_pad;
  g.chunk_major = g.cin_pad % GE == 0;
  g.ng = g.chunk_major ? g.K9 / GE : 0;
  const int K_pad = b.K_pad[blockIdx.y];
  const long total = (long)b.cout_pad[blockIdx.y] * K_pad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i / K_pad);
    const int k = (int)(i - (long)co * K_pad);
    int tap, c;
    if (bf) k_to_tap<32>(g, k, tap, c);
    else k_to_tap<16>(g, k, tap, c);
    float v = 0.f;
    if (tap < 9 && co < j.cout && c < j.cin) {
      if (!j.flip) {
        if (co < j.w_cout && c < j.w_cin) v = j.w[((long)tap * j.w_cin + c) * j.w_cout + co];
      } else if (c < j.w_cout && co < j.w_cin) {
        v = j.w[((long)(8 - tap) * j.w_cin + co) * j.w_cout + c];
      }
    }
    if (bf) reinterpret_cast<uint16_t*>(j.packed)[i] = f2bf(v);
    else reinterpret_cast<float*>(j.packed)[i] = v;
  }
}

// the forward packs of chunk-major bf16 filters (every conv of the UNetImage / UNetVideo training re-pack): a block
// transposes one (granule, 64-output-channel) tile through LDS, so the source filter is read along cout (256-byte
// runs; pack_weights_batch's one element per thread read it with a w_cout stride) and each packed row receives 64
// contiguous bytes; zero padding (cin / cout past the filter, the K_pad tail granule) as pack_weights_batch, and the
// same RNE rounding: bit-identical
__global__ __launch_bounds__(256) void pack_weights_tiled(PackBatch b) {
  const int jb = blockIdx.y;
  const vm_pack_job& j = b.j[jb];
  const int K_pad = b.K_pad[jb], ngr = K_pad / 32, ng = 9 * b.cin_pad[jb] / 32, ncot = b.cout_pad[jb] / 64;
  const int t = blockIdx.x;
  if (t >= ngr * ncot) return;
  const int gr = t % ngr, co0 = (t / ngr) * 64;
  __shared__ float tile[32][65];
  const int tid = threadIdx.x;
  if (gr < ng) {
    const int cc = gr / 9, tap = gr - cc * 9;
    for (int e = tid; e < 32 * 64; e += 256) {
      const int ci = e >> 6, coj = e & 63;
      const int c = cc * 32 + ci, co = co0 + coj;
      float v = 0.f;
      if (co < j.cout && c < j.cin && co < j.w_cout && c < j.w_cin) v = j.w[((long)tap * j.w_cin + c) * j.w_cout + co];
      tile[ci][coj] = v;
    }
  }
  __syncthreads();
  const int coj = tid >> 2, ch = tid & 3;
  float f[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = gr < ng ? tile[ch * 8 + k][coj] : 0.f;
  *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(j.packed) + (long)(co0 + coj) * K_pad + gr * 32 + ch * 8) =
      Chunk<uint16_t>::pack(f);
}

// the flipped (data-gradient) packs of chunk-major bf16 filters: a lane fills one 16-byte run of 8 packed channels,
// whose sources w[8 - tap][co][c .. c + 7] are 8 consecutive floats (the filter's contiguous cout axis), where
// pack_weights_batch decoded and stored one element per thread; same zero padding, same RNE rounding: bit-identical
__global__ __launch_bounds__(256) void pack_weights_flip8(PackBatch b) {
  const int jb = blockIdx.y;
  const vm_pack_job& j = b.j[jb];
  const int K_pad = b.K_pad[jb], ng = 9 * b.cin_pad[jb] / 32, kq8 = K_pad / 8;
  const long total = (long)b.cout_pad[jb] * kq8;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < total; q += (long)gridDim.x * 256) {
    const int co = (int)(q / kq8), kq = (int)(q - (long)co * kq8);
    const int gr = kq >> 2, c0 = (kq & 3) * 8;
    float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (gr < ng && co < j.cout && co < j.w_cin) {
      const int cc = gr / 9, tap = gr - cc * 9;
      const float* src = j.w + ((long)(8 - tap) * j.w_cin + co) * j.w_cout;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = cc * 32 + c0 + k;
        if (c < j.cin && c < j.w_cout) f[k] = src[c];
      }
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(j.packed) + (long)co * K_pad + kq * 8) =
        Chunk<uint16_t>::pack(f);
  }
}

struct PackGeom {
  int cin_pad, ge, K9, K_pad, cout_pad, chunk_major, ng;
};

static PackGeom geom(int cin, int cout, int dtype) {
  PackGeom g;
  g.ge = 64 / elem_bytes(dtype);
  g.cin_pad = (cin + 7) / 8 * 8;
  g.K9 = 9 * g.cin_pad;
  g.chunk_major = g.cin_pad % g.ge == 0;
  g.ng = g.chunk_major ? g.K9 / g.ge : 0;
  g.K_pad = (g.K9 + 2 * g.ge - 1) / (2 * g.ge) * (2 * g.ge);  // whole 128-byte steps
  g.cout_pad = (cout + 63) / 64 * 64;
  return g;
}

static void fill_geom(ConvArgs& a, const PackGeom& g) {
  a.cin_pad = g.cin_pad;
  a.K9 = g.K9;
  a.chunk_major = g.chunk_major;
  a.ng = g.ng;
  a.K_pad = g.K_pad;
  a.cout_pad = g.cout_pad;
}

// ================================================================ folded 2x resize (unet.py:44-63 upconv_concat)
// conv3x3(resize2x(x)) with TF1 legacy bilinear (scale 0.5) is linear in x: resized row 2i = x[i], row 2i+1 =
// (x[i] + x[i+1]) / 2.  So output pixel (2i+a, 2j+b) is a 3x3 conv of the LOW-RES frame at (i, j) with a phase
// filter W'_ab[u][v] = sum_{kh,kw} R_a[u][kh] R_b[v][kw] W[kh][kw], u,v in {-1,0,+1}:
//   R_0 = [[.5,0,0],[.5,1,.5],[0,0,.5]]  (rows u, columns kh)      R_1 = [[0,0,0],[1,.5,0],[0,.5,1]]
// Output channel p*cout + co of the folded conv is phase p = 2a+b of channel co.  Exact in the interior and, with
// the low-res frame replicated past its bottom/right edge, at output rows/columns 2H-2; output row/column 0 and
// 2H-1 / 2W-1 see the resized image's zero padding instead and are recomputed by conv3x3_up2x_border.
__global__ void fold_up2x_weights(const float* w, int cin, int cout, float* wu) {
  const long total = 9L * cin * cout;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % cout);
    const long r = i / cout;
    const int ci = (int)(r % cin);
    const int tap = (int)(r / cin), u = tap / 3, v = tap % 3;  // low-res tap (u, v) = offset (u-1, v-1)
    constexpr float R[2][3][3] = {{{.5f, 0.f, 0.f}, {.5f, 1.f, .5f}, {0.f, 0.f, .5f}},
                                  {{0.f, 0.f, 0.f}, {1.f, .5f, 0.f}, {0.f, .5f, 1.f}}};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int pa = p >> 1, pb = p & 1;
      double s = 0.0;
      for (int kh = 0; kh < 3; ++kh)
        for (int kw = 0; kw < 3; ++kw) {
          const float c = R[pa][u][kh] * R[pb][v][kw];
          if (c != 0.f) s += (double)c * (double)w[((long)(kh * 3 + kw) * cin + ci) * cout + co];
        }
      wu[((long)tap * cin + ci) * (4L * cout) + (long)p * cout + co] = (float)s;
    }
  }
}

struct BorderArgs {
  const void* x;  // low-res [N,H,W,cin] bf16 view
  int x_cstride, x_coff, H, W, nframes;
  const void* w;  // plain packed filter (chunk-major bf16)
  int K_pad, cout, nch;
  const float* bias;
  const float* scale;
  const float* shift;
  int act;
  void* y;  // [N,2H,2W,cout] bf16 view
  int y_cstride, y_coff;
  int nb;  // border pixels per frame
  float* hd;        // head split (cout == 64): per-tap head shares of the border pixels, as the conv's epilogue
  const float* hw;  // conv1_5 HWIO f32 [3,3,hw_cin,1]
  int hw_cin, hw_coff, y_skip;
  // SPL (split-fp16 x3, vm_conv3x3_up2x_split3_nhwc): x is the low-res split input [l, h] (xs channels per slab; the
  // K granules run over [l, h, h], nch = 3 xs / 32); y the split output (slab ysplit); ovf as ConvArgs::ovf
  int xs, ysplit;
  int* ovf;
};

// 8 fp16 values of a 16-byte chunk -> f32
__device__ __forceinline__ void unpack_f16x8(uint4 u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[i] & 0xffffu));
    f[2 * i + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[i] >> 16));
  }
}

// Border pixels of the folded upconv, computed the unfused way: the 9 resized taps (TF1 legacy bilinear in f32,
// rounded to bf16 as vm_resize_bilinear_tf1_nhwc stores them; zero outside the 2H x 2W frame) of 16 pixels are
// staged per 32-channel granule and consumed by MFMAs.  The pass is latency-bound (a few hundred blocks; each granule
// costs a round trip for its gathers), so a 1024-thread block splits the granules 4 ways (wave w: output channels
// 16 (w & 3) .. +15, granules (w >> 2), (w >> 2) + 4, ...: each 4-wave group stages and consumes its own granules,
// double-buffered, with one LDS-only barrier per step) and adds the 4 partial sums in a fixed order at the end.
__device__ __forceinline__ uint4 sel3(int i, uint4 a, uint4 b, uint4 c) { return i == 0 ? a : (i == 1 ? b : c); }

// SPL: the split-fp16 x3 form (the folded upconvs of vmatting/split3.py): each staged value is the resize of the f32
// activation x = h + l (exact in f32), split again into fp16 (h', l'); K granule cc stages l' (slab 0) or h' (slabs 1,
// 2) for the fp16 filter parts [Wh, Wl, Wh]; the output is written split (ConvArgs::ysplit's layout)
template <int BD_KS, bool SPL = false>  // granule split of the border pass (waves = 4 x BD_KS)
__global__ __launch_bounds__(256 * BD_KS) void conv3x3_up2x_border(BorderArgs a) {
  using T = uint16_t;
  using MT = std::conditional_t<SPL, f16_t, uint16_t>;
  __shared__ __attribute__((aligned(16))) char stg[BD_KS][2][9 * 16 * 64];  // [split][buffer][tap][pixel][32 ch]
  __shared__ __attribute__((aligned(16))) float red[BD_KS * 16 * 64];       // [split][pixel][channel] partial sums
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = wave & 3, ks = wave >> 2, gt = tid & 255;  // channel group, granule split, thread in the split group
  const int OH = 2 * a.H, OW = 2 * a.W;
  const long total = (long)a.nframes * a.nb, b0 = (long)blockIdx.x * 16;
  const int cob = blockIdx.y * 64;
  auto decode = [&](long b, int& n, int& oy, int& ox) {
    n = (int)(b / a.nb);
    const int r = (int)(b - (long)n * a.nb);
    if (r < OW) { oy = 0; ox = r; }
    else if (r < 2 * OW) { oy = OH - 1; ox = r - OW; }
    else if (r < 2 * OW + OH - 2) { oy = r - 2 * OW + 1; ox = 0; }
    else { oy = r - 2 * OW - (OH - 2) + 1; ox = OW - 1; }
  };
  const T* xb = reinterpret_cast<const T*>(a.x) + a.x_coff;
  const T* wb = reinterpret_cast<const T*>(a.w);
  // staging role inside the split group: thread (px, q, dh) builds taps (dh, 0..2) of pixel px for channels 8q..8q+7
  // of the granule; its resized row oy + dh - 1 blends low-res rows y0, y1, whose columns x0c .. x0c+2 cover the taps
  const int spx = gt & 15, sq = (gt >> 4) & 3, sdh = gt >> 6;  // sdh == 3: no staging work
  int pn = 0, oy = 0, ox = 0;
  const bool live = b0 + spx < total && sdh < 3;
  if (b0 + spx < total) decode(b0 + spx, pn, oy, ox);
  const int ry = oy + sdh - 1;
  const bool rok = live && (unsigned)ry < (unsigned)OH;
  const float sy = (float)max(ry, 0) * 0.5f;
  const float fy0 = floorf(sy);
  const int y0 = (int)fy0, y1 = min(y0 + 1, a.H - 1);
  const float ly = sy - fy0;
  const int cx0 = max(ox - 1, 0) >> 1;
  const T* xr = xb + ((long)pn * a.H) * a.W * (long)a.x_cstride + sq * 8;
  // SPL: granule cc of [l, h, h] reads input channels (cc mod xs/32) * 32 of both stored slabs (l at 0, h at xs)
  const int sg = SPL ? a.xs / 32 : 1;
  auto gather = [&](int cc, uint4 (&g)[SPL ? 12 : 6]) __attribute__((always_inline)) {
    const int cin0 = SPL ? (cc % sg) * 32 : cc * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int yy = i ? y1 : y0, xx = min(cx0 + j, a.W - 1);
        const T* p = xr + ((long)yy * a.W + xx) * a.x_cstride + cin0;
        const bool ok = rok && cc < a.nch;
        g[i * 3 + j] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
        if constexpr (SPL) g[6 + i * 3 + j] = ok ? *reinterpret_cast<const uint4*>(p + a.xs) : make_uint4(0, 0, 0, 0);
      }
  };
  auto stage = [&](const uint4 (&g)[SPL ? 12 : 6], char* dst, int cc) __attribute__((always_inline)) {
    if (sdh >= 3) return;
    // SPL: the tap's f32 value x = h + l (exact), unpacked from both slabs
    auto unp = [&](int k, float* f) __attribute__((always_inline)) {
      if constexpr (SPL) {
        float fl[8];
        unpack_f16x8(k < 3 ? sel3(k, g[6], g[7], g[8]) : sel3(k - 3, g[9], g[10], g[11]), f);
        unpack_f16x8(k < 3 ? sel3(k, g[0], g[1], g[2]) : sel3(k - 3, g[3], g[4], g[5]), fl);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += fl[e];
      } else {
        Chunk<T>::unpack(k < 3 ? sel3(k, g[0], g[1], g[2]) : sel3(k - 3, g[3], g[4], g[5]), f);
      }
    };
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int rx = ox + dw - 1;
      if (rok && (unsigned)rx < (unsigned)OW) {
#pragma clang fp contract(off)
        const float sx = (float)rx * 0.5f;
        const float fx0 = floorf(sx);
        const int x0 = (int)fx0, x1 = min(x0 + 1, a.W - 1);
        const float lx = sx - fx0;
        // (top row, then bottom row: fewer values live at once, the same arithmetic)
        float l8[8], r8[8], top[8];
        unp(x0 - cx0, l8);
        unp(x1 - cx0, r8);
#pragma unroll
        for (int e = 0; e < 8; ++e) top[e] = l8[e] + (r8[e] - l8[e]) * lx;
        unp(3 + x0 - cx0, l8);
        unp(3 + x1 - cx0, r8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float bot = l8[e] + (r8[e] - l8[e]) * lx;
          o[e] = top[e] + (bot - top[e]) * ly;
        }
      }
      uint4 q;
      if constexpr (SPL) {
        uint4 hq, lq;
        split3h_chunk(o, hq, lq);
        q = cc / sg == 0 ? lq : hq;
      } else {
        q = Chunk<T>::pack(o);
      }
      *reinterpret_cast<uint4*>(dst + ((sdh * 3 + dw) * 16 + spx) * 64 + sq * 16) = q;
    }
  };
  // filter fragments of this wave's 16 output channels: A rows = channels cob + 16 cg + (lane & 15)
  const T* wrow = wb + (long)(cob + cg * 16 + (lane & 15)) * a.K_pad + (lane >> 4) * 8;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  const int steps = (a.nch + BD_KS - 1) / BD_KS;  // every group runs the same number of steps (uniform barriers)
  uint4 g[SPL ? 12 : 6];
  gather(ks, g);
  for (int i = 0; i < steps; ++i) {
    const int cc = ks + i * BD_KS;
    char* buf = stg[ks][i & 1];
    stage(g, buf, cc);
    gather(cc + BD_KS, g);  // the group's next granule goes in flight under this one's barrier and MFMAs
    uint4 w[9];
    if (cc < a.nch) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) w[tap] = *reinterpret_cast<const uint4*>(wrow + (cc * 9 + tap) * 32);
    }
    // LDS-only barrier: __syncthreads would also wait (vmcnt(0)) for the gathers in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (cc < a.nch) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
        mma16<MT>(w[tap], *reinterpret_cast<const uint4*>(buf + (tap * 16 + (lane & 15)) * 64 + (lane >> 4) * 16), acc);
    }
  }
  // partial sums: lane holds channels 16 cg + 4 (lane >> 4) + j of pixel lane & 15
#pragma unroll
  for (int j = 0; j < 4; ++j) red[(ks * 16 + (lane & 15)) * 64 + cg * 16 + 4 * (lane >> 4) + j] = acc[j];
  __syncthreads();
  // one thread per (pixel, 4 channels): the splits added in order, then bias / affine / act
  const bool ew = tid < 256;
  const int ep = tid >> 4, cq = (tid & 15) * 4;
  const long b = b0 + ep;
  const bool bok = ew && b < total;
  int n = 0, ey = 0, ex = 0;
  if (bok) decode(b, n, ey, ex);
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  uint2 pk = make_uint2(0, 0);
  if (ew) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sum = red[(0 * 16 + ep) * 64 + cq + j];
#pragma unroll
      for (int k = 1; k < BD_KS; ++k) sum += red[(k * 16 + ep) * 64 + cq + j];
      const int co = cob + cq + j;
      const float sc = a.scale ? a.scale[co] : 1.f;
      v[j] = fmaf(sum, sc, (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f));
      if (a.act == VM_ACT_RELU) v[j] = fmaxf(v[j], 0.f);
      else if (a.act == VM_ACT_SIGMOID) v[j] = sigmoid_precise(v[j]);
    }
    if constexpr (SPL) {  // [l, h(, h)] of the 4 channels
      typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
      uint32_t hw2[2], lw2[2];
      bool o = false;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const h2_t hh = {(_Float16)v[2 * k], (_Float16)v[2 * k + 1]};
        const h2_t ll = {(_Float16)(v[2 * k] - (float)hh[0]), (_Float16)(v[2 * k + 1] - (float)hh[1])};
        hw2[k] = __builtin_bit_cast(uint32_t, hh);
        lw2[k] = __builtin_bit_cast(uint32_t, ll);
        o |= !(fabsf(v[2 * k]) < 65520.f) || !(fabsf(v[2 * k + 1]) < 65520.f);
      }
      if (bok) {
        T* yo = reinterpret_cast<T*>(a.y) + (((long)n * OH + ey) * OW + ex) * (long)a.y_cstride + a.y_coff + cob + cq;
        *reinterpret_cast<uint2*>(yo) = make_uint2(lw2[0], lw2[1]);
        *reinterpret_cast<uint2*>(yo + a.ysplit) = make_uint2(hw2[0], hw2[1]);
        if (3 * a.ysplit <= a.y_cstride) *reinterpret_cast<uint2*>(yo + 2 * a.ysplit) = make_uint2(hw2[0], hw2[1]);
        if (o && a.ovf) *a.ovf = 1;
      }
    } else {
      pk.x = bf16x2_bits(v[0], v[1]);
      pk.y = bf16x2_bits(v[2], v[3]);
      if (!a.y_skip && bok)
        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(a.y) + (((long)n * OH + ey) * OW + ex) * (long)a.y_cstride +
                                  a.y_coff + cob + cq) = pk;
    }
  }
  if (!SPL && a.hd) {  // (uniform: a.hd is a kernel argument; every thread reaches the barriers below)
    // the border pixel's 64 bf16 outputs -> 9 per-tap shares sum_c bf16(hw[tap][coff + c]) * y[c] (f32, in channel
    // order); taps 9..11 zero like the MFMA epilogues'
    float* vals = reinterpret_cast<float*>(&stg[0][0][0]);  // [16 pixels][64]
    float* hwl = vals + 16 * 64;                              // the head filter's 9 x 64 taps, bf16-rounded
    __syncthreads();
    if (ew) {
#pragma unroll
      for (int j = 0; j < 4; ++j) vals[ep * 64 + cq + j] = bf2f(f2bf(v[j]));
    }
    for (int i = tid; i < 9 * 64; i += 256 * BD_KS) hwl[i] = bf2f(f2bf(a.hw[(i >> 6) * a.hw_cin + a.hw_coff + (i & 63)]));
    __syncthreads();
    if (tid < 16 * 12) {
      const int pe = tid / 12, tap = tid - pe * 12;
      const long bb = b0 + pe;
      if (bb < total) {
        int pn2, py, px2;
        decode(bb, pn2, py, px2);
        float hacc = 0.f;
        if (tap < 9)
#pragma unroll 16
          for (int c = 0; c < 64; ++c) hacc = fmaf(hwl[tap * 64 + c], vals[pe * 64 + c], hacc);
        a.hd[(((long)pn2 * OH + py) * OW + px2) * 12 + tap] = hacc;
      }
    }
  }
}

// ================================================================ head from per-tap partials (unet.py:203-205)
// conv1_5 over cat1 = [upconv_4, conv1_2] with both halves' shares taken where they were made (the folded upconv's
// and the pair kernel's epilogues): logits[p] = bias + sum_tap (pa + pb)[p + off(tap)][tap] (zero outside the
// frame), alpha = sigmoid(logits).  A block owns 8 x 64 output pixels: the (8+2) x 66 partial rows it needs are
// contiguous runs of 66 x 48 bytes, staged with 16-byte loads (taps summed over the two halves on the way, taps
// 9..11 dropped), and each thread then adds its pixels' 9 taps from LDS.
constexpr int HS_TH = 8, HS_TW = 64, HS_PW = HS_TW + 2, HS_PR = HS_TH + 2;
__global__ __launch_bounds__(256) void head_from_partials(const float* __restrict__ pa, const float* __restrict__ pb,
                                                          int N, int H, int W, const float* __restrict__ bias,
                                                          float* __restrict__ logits, int l_cstride,
                                                          float* __restrict__ alpha) {
  __shared__ float sp[HS_PR * HS_PW * 9];
  const int tw = (W + HS_TW - 1) / HS_TW, th = (H + HS_TH - 1) / HS_TH;
  const int b = blockIdx.x, n = b / (th * tw), rem = b - n * th * tw;
  const int y0 = (rem / tw) * HS_TH, x0 = (rem % tw) * HS_TW;
  const long img = (long)n * H * W;
  // stage: item i = (row, pixel, float4 group g < 3)
  for (int i = threadIdx.x; i < HS_PR * HS_PW * 3; i += 256) {
    const int g = i % 3, px = (i / 3) % HS_PW, row = i / (3 * HS_PW);
    const int yy = y0 - 1 + row, xx = x0 - 1 + px;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
      const long q = (img + (long)yy * W + xx) * 12 + 4 * g;
      const float4 u = *reinterpret_cast<const float4*>(pa + q), w = *reinterpret_cast<const float4*>(pb + q);
      v = make_float4(u.x + w.x, u.y + w.y, u.z + w.z, u.w + w.w);
    }
    float* d = sp + (row * HS_PW + px) * 9 + 4 * g;
    d[0] = v.x;
    if (g < 2) { d[1] = v.y; d[2] = v.z; d[3] = v.w; }  // (group 2 holds tap 8 and the three zero taps)
  }
  __syncthreads();
  const float b0 = bias ? bias[0] : 0.f;
  for (int o = threadIdx.x; o < HS_TH * HS_TW; o += 256) {
    const int ty = o / HS_TW, tx = o % HS_TW;
    const int y = y0 + ty, x = x0 + tx;
    if (y >= H || x >= W) continue;
    float s = b0;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) s += sp[((ty + tap / 3) * HS_PW + tx + tap % 3) * 9 + tap];
    const long p = img + (long)y * W + x;
    if (logits) logits[p * l_cstride] = s;
    if (alpha) alpha[p] = sigmoid_precise(s);
  }
}

// ================================================================ split-K reduction
// out[p][c] = act((sum_s part[s][p][c]) * scale + bias*scale + shift), the splits summed in order (deterministic);
// one thread per 4 output channels of a pixel
// ---------------------------------------------------------------- narrow convs (2 <= cout <= 16)
// The select convs of unet_simple.py:153-168 map 192..1536 channels onto 2..16: a 64-wide output tile would spend
// 4-32x the MFMA work on zero weights, and the conv is really a stream over its input.  One 16-column MFMA tile
// (A = the packed weights' first 16 output channels, B = 16 patch pixels), the (TH+2) x 34 input patch of one
// 32-channel chunk staged in LDS (swizzled 64-byte pixel rows), the next chunk's patch and filter held in registers
// while this one is consumed.  Output lane l: pixel l % 16, channels 4 (l / 16) .. +3.  ksplit > 1 splits the
// chunks over gridDim.y into raw f32 partials (splitk_reduce_kernel, fixed order).
// One chunk of the narrow conv for a wave's RPW output rows: the chunk's 9 filter fragments are read once, and each
// patch row's 6 pixel fragments (3 column shifts x 2 halves) once, each feeding the MFMAs of every output row it
// reaches (kernel row kh = patch row - output row).  Per accumulator the MFMAs still run taps 0..8 in order (patch
// rows ascend with kh), so the sums are those of the tap-major loop bit for bit, with (RPW + 2) * 6 fragment reads
// per chunk instead of RPW * 18.
template <int RPW, int PW>
__device__ __forceinline__ void thin_chunk(const uint4* xs, const uint4* ws, int wv, int lane, f32x4 (&acc)[2 * RPW]) {
  uint4 w[9];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp) w[tp] = ws[tp * 64 + lane];  // A operand: co lane % 16, k = 8 (lane / 16) .. +7
#pragma unroll
  for (int pr = 0; pr < RPW + 2; ++pr) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pp = (wv * RPW + pr) * PW + h * 16 + (lane & 15) + kw;
        const uint4 b = xs[pp * 4 + ((lane >> 4) ^ (((pp >> 2) & 1) << 1))];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
          const int kh = pr - r;
          if (kh >= 0 && kh < 3) mma16<uint16_t>(w[kh * 3 + kw], b, acc[2 * r + h]);
        }
      }
    }
  }
}

template <int TH, bool RR = true>  // RR: thin_chunk's row reuse (false: the r03 tap-major loop, for A/B)
__global__ __launch_bounds__(256, TH <= 4 ? 4 : TH <= 8 ? 3 : 2) void conv3x3_thin(ConvArgs a) {
  constexpr int TW = 32, PW = TW + 2, PPIX = (TH + 2) * PW, PIECES = PPIX * 4, PPT = (PIECES + 255) / 256;
  constexpr int RPW = TH / 4;    // patch rows per wave
  constexpr int WPIECES = 9 * 16 * 4, WPT = (WPIECES + 255) / 256;  // the chunk's filter: [tap][k/8][co 16]
  __shared__ uint4 xs[PPIX * 4];
  __shared__ uint4 ws[WPT * 256];  // tail slots hold clamped duplicates (unconditional stores)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tw = (a.W + TW - 1) / TW, th = (a.H + TH - 1) / TH;
  const int ntiles = a.tiles_total;
  const int nch = a.cin_pad / 32;
  int cb = 0, ce = nch;
  if (a.ksplit > 1) {
    const int per = (nch + a.ksplit - 1) / a.ksplit;
    cb = blockIdx.y * per;
    ce = min(nch, cb + per);
  }
  // persistent: the block walks tiles blockIdx.x, +gridDim.x, ...; with a.twalk (r04) XCD x = blockIdx.x % 8 takes
  // the contiguous eighth [lo, hi) of the tile list and its gridDim.x / 8 blocks every (gridDim.x / 8)-th tile of it,
  // so the tiles resident at once on one XCD are neighbours whose patches share halo rows and 128-byte lines in that
  // XCD's L2 (round-robin placement put horizontally adjacent tiles on different XCDs: FETCH_SIZE 1.8x the input)
  int tile = blockIdx.x, tstep = (int)gridDim.x, tend = ntiles;
  if (a.twalk && (gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    tile = (int)((long)xcd * ntiles / 8) + (int)(blockIdx.x >> 3);
    tstep = (int)(gridDim.x >> 3);
    tend = (int)((long)(xcd + 1) * ntiles / 8);
  }
  if (cb >= ce || tile >= tend) return;
  // the block streams (tile, chunk) steps; the next step's
  // patch and filter pieces (the next tile's first chunk at a tile's end) are in registers while this one computes
  auto geo = [&](int t, int& n, int& r0, int& c0, int (&xo)[PPT]) {
    const int tx = t % tw;
    t /= tw;
    const int ty = t % th;
    n = t / th;
    r0 = ty * TH;
    c0 = tx * TW;
    // byte offsets of this thread's patch pieces inside image n (out of the frame: out of range -> the hardware
    // returns 0, SAME padding); the host guarantees H*W*cstride*2 < 2^31
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int id = tid + i * 256;
      const int p = id >> 2, q = id & 3;
      const int pr = p / PW, pc = p - pr * PW;
      const int yy = r0 - 1 + pr, xx = c0 - 1 + pc;
      const bool ok = id < PIECES && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      xo[i] = ok ? ((yy * a.W + xx) * a.x_cstride + q * 8) * 2 : OOB;
    }
  };
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7ffffff0, 0x00020000);  // 16 x K_pad bf16 used
  uint4 xr[PPT], wr[WPT];
  // a chunk's patch pieces and filter pieces (tap, k/8, co: the A operand's lane order) into registers
  auto fetch = [&](int n, const int (&xo)[PPT], int cc) {
    const uint16_t* Xn = reinterpret_cast<const uint16_t*>(a.x) + a.x_coff + (long)n * a.H * a.W * a.x_cstride;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Xn + src_chan(a, cc * 32)), 0, 0x7ffffff0, 0x00020000);
#pragma unroll
    for (int i = 0; i < PPT; ++i)
      xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo[i], 0, 0));
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int id = min(tid + i * 256, WPIECES - 1);
      wr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            wrs, ((id & 15) * a.K_pad + (cc * 9 + (id >> 6)) * 32 + ((id >> 4) & 3) * 8) * 2,
                                            0, 0));
    }
  };
  const int co0 = 4 * (lane >> 4);
  const bool splitk = a.ksplit > 1;
  float mul[4], add[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = min(co0 + j, a.cout - 1);
    const float sc = (a.scale && !splitk) ? a.scale[co] : 1.f;
    mul[j] = sc;
    add[j] = splitk ? 0.f : (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
  }

  int n, r0, c0, xo[PPT];
  geo(tile, n, r0, c0, xo);
  fetch(n, xo, cb);
  int cc = cb;
  f32x4 acc[2 * RPW];
#pragma unroll
  for (int f = 0; f < 2 * RPW; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (;;) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int id = tid + i * 256;
      const int p = id >> 2, q = id & 3;
      if (id < PIECES) xs[p * 4 + (q ^ (((p >> 2) & 1) << 1))] = xr[i];
    }
#pragma unroll
    for (int i = 0; i < WPT; ++i) ws[tid + i * 256] = wr[i];
    __syncthreads();
    // the next step: the next chunk of this tile, or the first chunk of the block's next tile
    const bool last = cc + 1 == ce;
    const int ntile = last ? tile + tstep : tile;
    const bool more = ntile < tend;
    int nn = n, nr0 = r0, nc0 = c0, nxo[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) nxo[i] = xo[i];
    if (more) {
      if (last) geo(ntile, nn, nr0, nc0, nxo);
      fetch(nn, nxo, last ? cb : cc + 1);
    }
    if constexpr (RR) {
      thin_chunk<RPW, PW>(xs, ws, wv, lane, acc);
    } else {
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const uint4 w = ws[tp * 64 + lane];  // A operand: output channel lane % 16, k = 8 (lane / 16) .. +7
#pragma unroll
        for (int f = 0; f < 2 * RPW; ++f) {
          const int rr = wv * RPW + (f >> 1), c = (f & 1) * 16 + (lane & 15);
          const int pp = (rr + tp / 3) * PW + c + tp % 3;
          const uint4 b = xs[pp * 4 + ((lane >> 4) ^ (((pp >> 2) & 1) << 1))];
          mma16<uint16_t>(w, b, acc[f]);
        }
        __builtin_amdgcn_sched_barrier(0);  // one tap's fragments live at a time (registers: the prefetch in flight)
      }
    }
    if (last) {  // the tile's epilogue, straight from registers (no LDS: the next step's commit may follow)
      if (co0 < a.cout) {
#pragma unroll
        for (int f = 0; f < 2 * RPW; ++f) {
          const int row = r0 + wv * RPW + (f >> 1), col = c0 + (f & 1) * 16 + (lane & 15);
          if (row >= a.H || col >= a.W) continue;
          const long m = ((long)n * a.H + row) * a.W + col;
          if (splitk) {
            float* d = a.part + ((long)blockIdx.y * a.M + m) * a.cout + co0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (co0 + j < a.cout) d[j] = acc[f][j];
            continue;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (co0 + j >= a.cout) break;
            float v = fmaf(acc[f][j], mul[j], add[j]);
            if (a.act == VM_ACT_RELU) v = fmaxf(v, 0.f);
            else if (a.act == VM_ACT_SIGMOID) v = sigmoid_precise(v);
            const long o = m * a.y_cstride + a.y_coff + co0 + j;
            if (a.y_dtype == VM_BF16) reinterpret_cast<uint16_t*>(a.y)[o] = f2bf(v);
            else reinterpret_cast<float*>(a.y)[o] = v;
          }
        }
      }
#pragma unroll
      for (int f = 0; f < 2 * RPW; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (!more) break;
    tile = ntile;
    cc = last ? cb : cc + 1;
    n = nn;
    r0 = nr0;
    c0 = nc0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) xo[i] = nxo[i];
  }
}

// ---------------------------------------------------------------- narrow-input convs (cin <= 16, cout <= 32)
// UNetSmall's encoder and decoder convs (small.py:39-48: 6 -> 8, 8 -> 16, 16 -> 32, 16 -> 8) hold 8 or 16 channels per
// pixel, so there is no 32-channel granule: K runs tap-major (k = tap * cin_pad + c, the generic packing) and one
// MFMA K-step of 32 takes 4 (tap, 8-channel group) pieces, each a 16-byte LDS read of one patch pixel.  One 8 x 32
// tile per block: its 10 x 34 patch in LDS (G pieces per pixel), the filter (NS K-steps x NT 16-channel tiles) in
// registers.  Output lane l: pixel l % 16, channels 4 (l / 16) .. +3 of the tile.  The MFMAs chain k in ascending
// 32-blocks and the epilogue is conv3x3_mfma's (fmaf form for bf16 outputs, (acc + b) * s + t for f32), so the
// results are bit-identical to the generic kernel's (which spent a 256 x 64 tile and 64-K steps on these).
template <int G, int NT>
__global__ __launch_bounds__(256) void conv3x3_narrowin(ConvArgs a) {
  constexpr int TH = 8, TW = 32, PW = TW + 2, PPIX = (TH + 2) * PW, PIECES = PPIX * G, PPT = (PIECES + 255) / 256;
  constexpr int NQ = 9 * G, NS = (NQ + 3) / 4, RPW = TH / 4;
  __shared__ uint4 xs[PIECES];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int tw = (a.W + TW - 1) / TW, th = (a.H + TH - 1) / TH;
  int t = blockIdx.x;
  const int tx = t % tw;
  t /= tw;
  const int ty = t % th, n = t / th;
  const int r0 = ty * TH, c0 = tx * TW;
  const uint16_t* Xn = reinterpret_cast<const uint16_t*>(a.x) + a.x_coff + (long)n * a.H * a.W * a.x_cstride;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Xn), 0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7ffffff0, 0x00020000);
  uint4 xr[PPT], w[NT][NS];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {  // patch pieces: pixel id / G, channel group id % G (out of frame: zeros)
    const int id = tid + i * 256;
    const int p = id / G, q = id - p * G;
    const int pr = p / PW, pc = p - pr * PW;
    const int yy = r0 - 1 + pr, xx = c0 - 1 + pc;
    const bool ok = id < PIECES && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
    xr[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                          xrs, ok ? ((yy * a.W + xx) * a.x_cstride + q * 8) * 2 : OOB, 0, 0));
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)  // A operand: output channel nt * 16 + lane % 16, k = 32 s + 8 (lane / 16) .. +7
#pragma unroll
    for (int s = 0; s < NS; ++s)
      w[nt][s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                               wrs, ((nt * 16 + (lane & 15)) * a.K_pad + 32 * s + 8 * (lane >> 4)) * 2,
                                               0, 0));
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int id = tid + i * 256;
    if (id < PIECES) xs[id] = xr[i];
  }
  __syncthreads();
  f32x4 acc[NT][2 * RPW];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int f = 0; f < 2 * RPW; ++f) acc[nt][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int q = 4 * s + (lane >> 4);
    const bool kv = q < NQ;  // K padding past tap 8: zero pieces (the packed filter is zero there too)
    const int tap = kv ? q / G : 0, g = q - (q / G) * G;
    const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
    for (int f = 0; f < 2 * RPW; ++f) {
      const int pp = (wv * RPW + (f >> 1) + kh) * PW + (f & 1) * 16 + (lane & 15) + kw;
      uint4 b = xs[pp * G + (kv ? g : 0)];
      if (!kv) b = uint4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) mma16<uint16_t>(w[nt][s], b, acc[nt][f]);
    }
  }
  const bool f32o = a.y_dtype == VM_F32;
  const bool fma_form = !f32o && a.y_vec && (a.cout & 7) == 0;  // conv3x3_mfma's fast bf16 epilogue, else its general one
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int co0 = nt * 16 + 4 * (lane >> 4);
    if (co0 >= a.cout) continue;
    float bs[4], sc[4], sh[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = min(co0 + j, a.cout - 1);
      bs[j] = a.bias ? a.bias[co] : 0.f;
      sc[j] = a.scale ? a.scale[co] : 1.f;
      sh[j] = a.shift ? a.shift[co] : 0.f;
    }
    const bool full = co0 + 4 <= a.cout && a.y_vec;
#pragma unroll
    for (int f = 0; f < 2 * RPW; ++f) {
      const int row = r0 + wv * RPW + (f >> 1), col = c0 + (f & 1) * 16 + (lane & 15);
      if (row >= a.H || col >= a.W) continue;
      const long o = (((long)n * a.H + row) * a.W + col) * a.y_cstride + a.y_coff + co0;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float tv = fma_form ? fmaf(acc[nt][f][j], sc[j], bs[j] * sc[j] + sh[j]) : (acc[nt][f][j] + bs[j]) * sc[j] + sh[j];
        if (a.act == VM_ACT_RELU) tv = fma_form ? fmaxf(tv, 0.f) : (tv > 0.f ? tv : 0.f);
        else if (a.act == VM_ACT_SIGMOID) tv = sigmoid_precise(tv);
        v[j] = tv;
      }
      if (f32o) {
        float* Y = reinterpret_cast<float*>(a.y) + o;
        if (full) {
          *reinterpret_cast<float4*>(Y) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) Y[j] = v[j];
        }
      } else {
        uint16_t* Y = reinterpret_cast<uint16_t*>(a.y) + o;
        if (full) {
          *reinterpret_cast<uint2*>(Y) = uint2{bf16x2_bits(v[0], v[1]), bf16x2_bits(v[2], v[3])};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (co0 + j < a.cout) Y[j] = f2bf(v[j]);
        }
      }
    }
  }
}

// LDS-DMA form of conv3x3_thin (r04).  The select convs are a stream over 192..1536-channel tower features (1.3 GB
// per training step) and conv3x3_thin ran them at 1.1-2.8 TB/s: one chunk in flight per block, its patch and filter
// held in registers from the end of one chunk's compute to the start of the next, so every chunk exposed most of
// the load latency.  Here chunk t+S-1's patch and filter are DMA'd (buffer_load ... lds) into an S-slot LDS ring
// while chunk t computes: S-1 chunks in flight per block, no registers held.  One raw barrier per chunk, after the
// wave's own DMAs of chunk t have landed (counted vmcnt: every thread issues exactly PPT + WPT pieces per step;
// steps past the end load out-of-range zeros) and its fragment reads of chunk t-1 have retired (lgkmcnt(0): the
// slot the next DMA overwrites).  The patch swizzle is applied on the source side (LDS position p*4 + q holds
// piece (p, q ^ swz(p))); MFMA order and epilogue are conv3x3_thin's, so results are bit-identical to it.
template <int TH, int S>
__global__ __launch_bounds__(256, 1) void conv3x3_thin_dma(ConvArgs a) {
  constexpr int TW = 32, PW = TW + 2, PPIX = (TH + 2) * PW, PIECES = PPIX * 4, PPT = (PIECES + 255) / 256;
  constexpr int RPW = TH / 4;
  constexpr int WPIECES = 9 * 16 * 4, WPT = (WPIECES + 255) / 256;
  constexpr int XS = PPT * 256 * 16, WS = WPT * 256 * 16, SLOT = XS + WS, NP = PPT + WPT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tw = (a.W + TW - 1) / TW, th = (a.H + TH - 1) / TH;
  const int ntiles = a.tiles_total;
  const int nch = a.cin_pad / 32;
  int cb = 0, ce = nch;
  if (a.ksplit > 1) {
    const int per = (nch + a.ksplit - 1) / a.ksplit;
    cb = blockIdx.y * per;
    ce = min(nch, cb + per);
  }
  if (cb >= ce || (int)blockIdx.x >= ntiles) return;
  const int nsteps_per_tile = ce - cb;
  // step j of this block: tile blockIdx.x + (j / nsteps) * gridDim.x, chunk cb + j % nsteps
  const int ntile_blk = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int nsteps = ntile_blk * nsteps_per_tile;
  const __amdgpu_buffer_rsrc_t wrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7ffffff0, 0x00020000);
  const uint32_t lds0 = lds_addr(smem);
  // DMA of step j into slot j % S (j >= nsteps: out-of-range zeros, so every step issues NP pieces)
  auto issue = [&](int j) __attribute__((always_inline)) {
    const bool real = j < nsteps;
    const int jj = real ? j : 0;
    const int t = (int)blockIdx.x + (jj / nsteps_per_tile) * (int)gridDim.x;
    const int cc = cb + jj % nsteps_per_tile;
    int tt = t;
    const int tx = tt % tw;
    tt /= tw;
    const int ty = tt % th;
    const int n = tt / th;
    const int r0 = ty * TH, c0 = tx * TW;
    const uint16_t* Xn = reinterpret_cast<const uint16_t*>(a.x) + a.x_coff + (long)n * a.H * a.W * a.x_cstride +
                         src_chan(a, cc * 32);
    const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(const_cast<uint16_t*>(Xn)), 0,
                                                                         0x7ffffff0, 0x00020000);
    const uint32_t slot = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)((j % S) * SLOT));
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int id = tid + i * 256;
      const int p = id >> 2, qq = id & 3;
      const int q = qq ^ (((p >> 2) & 1) << 1);  // the piece whose swizzled home is LDS position id
      const int pr = p / PW, pc = p - pr * PW;
      const int yy = r0 - 1 + pr, xx = c0 - 1 + pc;
      const bool ok = real & (id < PIECES) & ((unsigned)yy < (unsigned)a.H) & ((unsigned)xx < (unsigned)a.W);
      const int off = ((yy * a.W + xx) * a.x_cstride + q * 8) * 2;  // (32-bit: checked by the host)
      glds16(xrs, slot + (uint32_t)((i * 256 + wv * 64) * 16), ok ? off : OOB);
    }
#pragma unroll
    for (int i = 0; i < WPT; ++i) {
      const int id = tid + i * 256;
      const bool ok = real & (id < WPIECES);
      const int off = ((id & 15) * a.K_pad + (cc * 9 + (id >> 6)) * 32 + ((id >> 4) & 3) * 8) * 2;
      glds16(wrs, slot + (uint32_t)(XS + (i * 256 + wv * 64) * 16), ok ? off : OOB);
    }
  };
  const int co0 = 4 * (lane >> 4);
  const bool splitk = a.ksplit > 1;
  float mul[4], add[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int co = min(co0 + j, a.cout - 1);
    const float sc = (a.scale && !splitk) ? a.scale[co] : 1.f;
    mul[j] = sc;
    add[j] = splitk ? 0.f : (a.bias ? a.bias[co] : 0.f) * sc + (a.shift ? a.shift[co] : 0.f);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the epilogue constants: nothing older in the DMA counts
#pragma unroll
  for (int j = 0; j < S - 1; ++j) issue(j);
  f32x4 acc[2 * RPW];
#pragma unroll
  for (int f = 0; f < 2 * RPW; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
  int tile = blockIdx.x;
  for (int j = 0; j < nsteps; ++j) {
    // chunk j landed (the S-2 younger steps may stay in flight); this wave's reads of slot (j-1) % S retired
    if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else wait_vm((S - 2) * NP);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(j + S - 1);  // into slot (j - 1) % S, free since the barrier
    const uint4* xs = reinterpret_cast<const uint4*>(smem + (j % S) * SLOT);
    const uint4* ws = reinterpret_cast<const uint4*>(smem + (j % S) * SLOT + XS);
    thin_chunk<RPW, PW>(xs, ws, wv, lane, acc);
    if ((j + 1) % nsteps_per_tile == 0) {  // the tile's epilogue (conv3x3_thin's), straight from registers
      int t = tile;
      const int tx = t % tw;
      t /= tw;
      const int ty = t % th;
      const int n = t / th;
      const int r0 = ty * TH, c0 = tx * TW;
      if (co0 < a.cout) {
#pragma unroll
        for (int f = 0; f < 2 * RPW; ++f) {
          const int row = r0 + wv * RPW + (f >> 1), col = c0 + (f & 1) * 16 + (lane & 15);
          if (row >= a.H || col >= a.W) continue;
          const long m = ((long)n * a.H + row) * a.W + col;
          if (splitk) {
            float* d = a.part + ((long)blockIdx.y * a.M + m) * a.cout + co0;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              if (co0 + jj < a.cout) d[jj] = acc[f][jj];
            continue;
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            if (co0 + jj >= a.cout) break;
            float v = fmaf(acc[f][jj], mul[jj], add[jj]);
            if (a.act == VM_ACT_RELU) v = fmaxf(v, 0.f);
            else if (a.act == VM_ACT_SIGMOID) v = sigmoid_precise(v);
            const long o = m * a.y_cstride + a.y_coff + co0 + jj;
            if (a.y_dtype == VM_BF16) reinterpret_cast<uint16_t*>(a.y)[o] = f2bf(v);
            else reinterpret_cast<float*>(a.y)[o] = v;
          }
        }
      }
#pragma unroll
      for (int f = 0; f < 2 * RPW; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
      tile += gridDim.x;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing zero-fill DMAs land before the block exits
}
template <int TH, int S>
constexpr int thin_dma_lds() {
  constexpr int PPT = ((TH + 2) * 34 * 4 + 255) / 256, WPT = (9 * 16 * 4 + 255) / 256;
  return S * (PPT + WPT) * 256 * 16;
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int ks, long M, int cout,
                                                            const float* bias, const float* scale, const float* shift,
                                                            int act, void* y, int y_dtype, int ycs, int ycoff,
                                                            int ysplit = 0, int* ovf = nullptr) {
  const int c4 = (cout + 3) / 4;
  const long total = M * c4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / c4;
    const int c = (int)(i - p * c4) * 4;
    float4 s = *reinterpret_cast<const float4*>(part + p * cout + c);
    for (int k = 1; k < ks; ++k) {
      const float4 t = *reinterpret_cast<const float4*>(part + (long)k * M * cout + p * cout + c);
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float v[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (c + j >= cout) break;
      const float sc = scale ? scale[c + j] : 1.f;
      float t = fmaf(v[j], sc, (bias ? bias[c + j] : 0.f) * sc + (shift ? shift[c + j] : 0.f));
      if (act == VM_ACT_RELU) t = fmaxf(t, 0.f);
      else if (act == VM_ACT_SIGMOID) t = sigmoid_precise(t);
      const long o = p * ycs + ycoff + c + j;
      if (ysplit > 0) {  // split-fp16 x3 output (ConvArgs::ysplit): [l, h, h] at 0, ysplit, 2 * ysplit
        const _Float16 h = (_Float16)t;
        const _Float16 l = (_Float16)(t - (float)h);
        uint16_t* yo = reinterpret_cast<uint16_t*>(y) + o;
        yo[0] = __builtin_bit_cast(uint16_t, l);
        yo[ysplit] = __builtin_bit_cast(uint16_t, h);
        if (3 * ysplit <= ycs) yo[2 * ysplit] = __builtin_bit_cast(uint16_t, h);
        if (!(fabsf(t) < 65520.f) && ovf) *ovf = 1;
      } else if (y_dtype == VM_F32) {
        reinterpret_cast<float*>(y)[o] = t;
      } else {
        reinterpret_cast<uint16_t*>(y)[o] = f2bf(t);
      }
    }
  }
}

// ================================================================ dispatch
// name of the kernel the last conv call on this thread launched, spelled as rocprofv3 reports it
// (bench.py matches its per-launch PMC traffic by this name)
thread_local char g_last_kernel[128];
template <typename T>
static const char* tname() { return sizeof(T) == 2 ? "unsigned short" : "float"; }

template <typename T, int BM, int BN>
static int launch_mfma(ConvArgs& a, hipStream_t st) {
  constexpr int lds = mfma_lds_bytes<BM, BN>();
  static bool attr_set = false;  // idempotent; benign race
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_mfma<T, BM, BN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return fail(VM_EHIP, "hipFuncSetAttribute: %s", hipGetErrorString(e));
    attr_set = true;
  }
  a.nk = a.K_pad / (128 / (int)sizeof(T));
  a.tiles_n = (a.cout + BN - 1) / BN;
  a.tiles_total = (int)((a.M + BM - 1) / BM) * a.tiles_n;
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_mfma<%s, %d, %d>", tname<T>(), BM, BN);
  hipLaunchKernelGGL((conv3x3_mfma<T, BM, BN>), dim3(a.tiles_total), dim3(256), lds, st, a);
  return check_launch("conv3x3_mfma");
}

template <typename T, int RB, int BM, int BN, int WM, int WN, int S, bool FAST>
static int launch_glds(ConvArgs& a, hipStream_t st) {
  using C = GldsCfg<T, RB, BM, BN, WM, WN, S>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_glds<T, RB, BM, BN, WM, WN, S, FAST>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return fail(VM_EHIP, "hipFuncSetAttribute(glds): %s", hipGetErrorString(e));
    attr_set = true;
  }
  const int bke = RB / (int)sizeof(T);
  a.nk = (FAST && RB == 64) ? a.ng : a.K_pad / bke;
  a.tiles_n = (a.cout + BN - 1) / BN;
  a.tiles_total = (int)((a.M + BM - 1) / BM) * a.tiles_n;
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_glds<%s, %d, %d, %d, %d, %d, %d, %s>", tname<T>(), RB,
           BM, BN, WM, WN, S, FAST ? "true" : "false");
  hipLaunchKernelGGL((conv3x3_glds<T, RB, BM, BN, WM, WN, S, FAST>), dim3(a.tiles_total), dim3(C::NT), C::LDS, st,
                     a);
  return check_launch("conv3x3_glds");
}

static long g_border_ks = 1;  // folded-upconv border pass: granule split (1, 2 or 4 wave groups per block)
static long g_up_skip_mask = 3;  // folded upconvs: which zero taps are skipped (1 = kernel row, 2 = column, 3 = both)
static long g_patch_repi = 1;  // patch kernel: register epilogue (bf16 outputs, no packed frames) where the tiling allows
// channel-banded patch tiles (ConvArgs::cband): 0 off, 1 folded upconvs, 2 all.  Off: measured on upconv_2 (9.4 MB
// folded filter) 0.261 -> 0.312 ms and on the L5 convs 0.053 -> 0.057 ms (same box, bench.py --option cband=0|1|2):
// every XCD then reads the whole input from the Infinity Cache, which costs more than the weight stream it saves
static long g_cband = 0;
static long g_cband_bytes = 4L << 20;   // ... for filters of at least this many bytes (an XCD's L2)
// grouped tile order (ConvArgs::ngroup): this many output tiles per group for filters of >= cband_bytes (0: off) —
// the XCD working set is ngroup filter slices instead of the whole filter; the input is read tiles_n / ngroup times.
// Off: same-box A/B (gpurun_out/r6g_ab.log, profiles/r06g_ngroup_ab.log) bf16 forward 2.967 -> 2.993..3.010 ms for
// ngroup 2..8, f16x3 10.04 -> 10.01..10.04 ms: the re-streamed filter slices come from the Infinity Cache
static long g_ngroup = 0;

template <int BN, int WM, int WN, int S, int TH = 8, int MINB = 1, int UNR = 9, bool PF = false, int ABL = 0,
          bool FIRST = false, int G = 1, bool UPSKIP = false>
static int launch_patch(ConvArgs& a, hipStream_t st) {
  using C = PatchCfg<BN, WM, WN, S, TH, G>;
  static_assert(!(FIRST && PF), "FIRST uses the plain pipeline");
  constexpr int lds = FIRST ? C::LDS_FIRST : C::LDS;
  // fp16 operands (ConvArgs::f16, the split-fp16 forward): the same tiling on v_mfma_f32_16x16x32_f16
  constexpr bool F16_OK = !FIRST && ABL == 0;
  const bool f16 = F16_OK && a.f16;
  if (a.f16 && !F16_OK) return fail(VM_EUNSUPPORTED, "conv3x3_patch: no fp16 instantiation of this tiling");
  static bool attr_set = false, attr16_set = false;
  if (!(f16 ? attr16_set : attr_set)) {
    const void* fn = f16 ? reinterpret_cast<const void*>(
                               &conv3x3_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G, UPSKIP, f16_t>)
                         : reinterpret_cast<const void*>(
                               &conv3x3_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G, UPSKIP>);
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return fail(VM_EHIP, "hipFuncSetAttribute(patch): %s", hipGetErrorString(e));
    (f16 ? attr16_set : attr_set) = true;
  }
  const long N = a.M / ((long)a.H * a.W);
  const long sp = a.vstride ? ((a.H + C::TH - 1) / C::TH) * (long)((a.vW + C::TW - 1) / C::TW)
                            : N * ((a.H + C::TH - 1) / C::TH) * ((a.W + C::TW - 1) / C::TW);
  a.tiles_n = (a.cout + BN - 1) / BN;
  a.repi = (int)g_patch_repi;
  a.upmask = (int)g_up_skip_mask;
  a.prio = (int)g_conv_prio;
  if (sp * a.tiles_n > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3: too many tiles");
  a.tiles_total = (int)(sp * a.tiles_n);
  // channel-banded tile order (ConvArgs::cband) for weight-heavy layers: the whole filter exceeds an XCD's 4 MB L2
  // and its output tiles split evenly over the 8 XCDs.  cband option: 0 off, 1 folded upconvs, 2 any such layer
  const long wbytes = (long)a.cout_pad * a.K_pad * 2;
  a.cband = (g_cband >= (a.up ? 1 : 2)) && !FIRST && BN == 64 && a.tiles_n % 8 == 0 && wbytes >= g_cband_bytes
                ? a.tiles_n / 8 : 0;
  a.ngroup = !a.cband && g_ngroup > 0 && a.tiles_n > g_ngroup && a.tiles_n % g_ngroup == 0 && wbytes >= g_cband_bytes
                 ? (int)g_ngroup : 0;
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_patch<%d, %d, %d, %d, %d, %d, %d, %s, %d, %s, %d, %s%s>",
           BN, WM, WN, S, TH, MINB, UNR, PF ? "true" : "false", ABL, FIRST ? "true" : "false", G,
           UPSKIP ? "true" : "false", f16 ? ", vm::f16_t" : "");
  const dim3 grid(a.tiles_total, a.ksplit > 1 ? a.ksplit : 1);
  if constexpr (F16_OK) {
    if (f16) {
      hipLaunchKernelGGL((conv3x3_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G, UPSKIP, f16_t>), grid,
                         dim3(C::NT), lds, st, a);
      return check_launch("conv3x3_patch");
    }
  }
  hipLaunchKernelGGL((conv3x3_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G, UPSKIP>), grid, dim3(C::NT), lds,
                     st, a);
  return check_launch("conv3x3_patch");
}

static long g_pack_tiled = 1;  // vm_set_option "pack_tiled": 0 = every job on the element-wise pack_weights_batch (A/B)
static long g_up_skip = 1;  // vm_set_option "up_skip": 0 runs the folded upconvs without the zero-tap skipping (A/B)

// persistent row-slot patch kernel (conv3x3_patch_persist): a resident grid of 8 XCD bands x J walkers, on grids of
// >= g_persist_rounds full rounds of items (a shorter walk gains no prologue overlap and its last round is ragged);
// the callers check persist_ok, then persist_launch returns 1 when the grid is too small (the caller falls back)
static long g_patch_persist = 1;
static long g_persist_rounds = 2;
static long g_persist_up_rounds = 6;
static long g_persist_all = 0;  // (A/B) every plain grid of >= persist_rounds rounds
static long g_persist_rot = 0;  // (A/B) walker rotation: 0 = folded upconvs only, 1 = all, 2 = none
static long g_persist_half = 1;  // (A/B) halfskip walk for frames whose last tile column is <= 16 px (ConvArgs::halfskip)
static bool persist_ok(const ConvArgs& a) {
  return g_patch_persist && g_patch_repi && a.ksplit <= 1 && !a.vstride && a.y_dtype == VM_BF16 &&
         (!a.up || a.up_cout % 32 == 0) && (long)a.cout_pad * a.K_pad * 2 < 0x7fff0000L;
}
template <int BN, int WM, int WN, int S, int TH, int MINB, bool UPSKIP>
static int launch_patch_persist(ConvArgs& a, hipStream_t st) {
  using C = PatchCfg<BN, WM, WN, S, TH, 3>;
  const int tn = (a.cout + BN - 1) / BN;
  const int lds = C::MAIN + tn * BN * 8 + 2048;  // + per-channel affine of every output tile + head fragments
  constexpr int lds_max = 160 * 1024 / (160 * 1024 / C::MAIN);  // as many blocks per CU as the streaming kernel
  if (lds > lds_max) return 1;
  const void* fn = reinterpret_cast<const void*>(&conv3x3_patch_persist<BN, WM, WN, S, TH, MINB, UPSKIP>);
  static int dev_seen = -1, per_cu = 0, n_cu = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != dev_seen) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, C::NT, lds_max);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return fail(VM_EHIP, "conv3x3_patch_persist: %s", hipGetErrorString(e));
    dev_seen = dev;
  }
  const long N = a.M / ((long)a.H * a.W);
  const long sp = N * ((a.H + C::TH - 1) / C::TH) * ((a.W + C::TW - 1) / C::TW);
  const long resident = (long)per_cu * n_cu;
  // where it pays (same-box A/B per layer of the 1080p forward, 2 blocks per CU = 512 resident): a folded upconv
  // (phases of 9 / 6 / 6 / 4 taps, rotated over the walkers) needs >= g_persist_up_rounds rounds of items to even
  // out (upconv_3 / upconv_4, 8 / 16 rounds: -3 % / -18 %; upconv_2, 4 rounds: +13 %); a plain conv gains on grids of
  // 2..3 rounds (conv4_x, conv5 of 1024 / 512 channels: -2..-3 %) and on the 2-granule K loop (conv2_1: -9 %), and
  // loses a little on 4..8 rounds of 4..8 granules (conv2_2, conv3_2, conv3_3: +2..+3 %)
  const long items = sp * tn;
  bool use;
  if (a.up) use = items >= g_persist_up_rounds * resident;
  else use = items >= g_persist_rounds * resident && (items < 3 * resident || a.cin_pad <= 64 || g_persist_rounds == 0 ||
                                                        g_persist_all);
  if (sp < 8 || resident < 8 || !use || items > 0x7fffffffL) return 1;
  a.tiles_n = tn;
  a.prot = g_persist_rot == 0 ? (a.up ? 1 : 0) : g_persist_rot == 1 ? 1 : 0;
  // a last tile column of <= 16 frame columns (135 x 240: 7.5 tiles) costs half a tile: walk those tiles last and
  // serpentine the rounds, so the 2.125 rounds of items of the conv4 level end after ~2.2 tile times instead of 3
  const long J_ = resident / 8;
  a.halfskip = g_persist_half && C::REMAP && a.W % C::TW != 0 && a.W % C::TW <= 16 && a.W > C::TW;
  if (a.halfskip && !a.prot && J_ % tn == 0) a.prot = 2;
  a.repi = 1;
  a.prio = (int)g_conv_prio;
  a.upmask = (int)g_up_skip_mask;
  a.tiles_total = (int)(sp * tn);
  const long J = resident / 8;  // walkers per XCD band (every band has >= 2 rounds of items)
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_patch_persist<%d, %d, %d, %d, %d, %d, %s>", BN, WM, WN, S,
           TH, MINB, UPSKIP ? "true" : "false");
  hipLaunchKernelGGL((conv3x3_patch_persist<BN, WM, WN, S, TH, MINB, UPSKIP>), dim3((unsigned)(8 * J)), dim3(C::NT), lds,
                     st, a);
  return check_launch("conv3x3_patch_persist");
}

// a shipped tiling: the folded-upconv instantiation (zero phase taps skipped, row-slot pipeline G = 3) for a.up,
// else the plain one
template <int BN, int WM, int WN, int S, int TH = 8, int MINB = 1, int UNR = 9, bool PF = false, int ABL = 0,
          bool FIRST = false, int G = 1>
static int launch_patch_up(ConvArgs& a, hipStream_t st) {
  if (G > 1 && a.up && g_up_skip) return launch_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G, (G > 1)>(a, st);
  return launch_patch<BN, WM, WN, S, TH, MINB, UNR, PF, ABL, FIRST, G, false>(a, st);
}

// split-K plan of a patch-kernel conv: small grids (under g_splitk_tiles 4 x 32 pixel x 64 channel tiles) with a
// long K loop split the channel granules so that ~1024 blocks run; 1 = no split.  Deterministic in the geometry,
// so vm_conv3x3_workspace_bytes and the launch agree.
static long g_splitk_tiles = 512;
static int splitk_plan(long n, int h, int w, int cin_pad, int cout) {
  const long tiles = n * ((h + 3) / 4) * ((w + 31) / 32) * ((cout + 63) / 64);
  const int nch = cin_pad / 32;
  if (tiles >= g_splitk_tiles || nch < 4 || tiles <= 0) return 1;
  int ks = (int)((1024 + tiles - 1) / tiles);
  if (ks > nch / 2) ks = nch / 2;
  if (ks < 2) return 1;
  const int per = (nch + ks - 1) / ks;
  return (nch + per - 1) / per;  // every split non-empty
}

// narrow-cout convs (conv3x3_thin): bf16, chunk-major 32-channel granules, 2..16 output channels, no pool / resize
static long g_thin_kernel = 1;
static bool thin_ok(int dt, const PackGeom& g, int cout, int x_src_c, int act, const vm_tensor* x) {
  return g_thin_kernel && dt == VM_BF16 && cout >= 2 && cout <= 16 && g.chunk_major && g.cin_pad % 32 == 0 &&
         (x_src_c <= 0 || x_src_c % 32 == 0) && act != VM_ACT_SOFTMAX &&
         (long)x->h * x->w * x->cstride * 2 < 0x7ffffff0L;  // 32-bit byte offsets inside one image
}
// narrow-input convs (conv3x3_narrowin): bf16, 8 or 16 tap-major input channels, <= 32 outputs, one source
static long g_narrowin = 1;
static bool narrowin_ok(const ConvArgs& a, const PackGeom& g, int cout, int act, const vm_tensor* x, const vm_tensor* y) {
  return g_narrowin && !g.chunk_major && (g.cin_pad == 8 || g.cin_pad == 16) && cout <= 32 && a.x_src_c <= 0 &&
         act != VM_ACT_SOFTMAX && (y->dtype == VM_F32 || y->dtype == VM_BF16) && g.K_pad >= 32 * ((9 * g.cin_pad / 8 + 3) / 4) &&
         (long)x->h * x->w * x->cstride * 2 < 0x7ffffff0L;
}
static int launch_narrowin(ConvArgs& a, long n, const PackGeom& g, hipStream_t st) {
  const long tiles = n * ((a.H + 7) / 8) * (long)((a.W + 31) / 32);
  if (tiles > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_narrowin: too many tiles");
  const int G = g.cin_pad / 8, NT = a.cout > 16 ? 2 : 1;
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_narrowin<%d, %d>", G, NT);
  const dim3 grid((unsigned)tiles);
  if (G == 1 && NT == 1) hipLaunchKernelGGL((conv3x3_narrowin<1, 1>), grid, dim3(256), 0, st, a);
  else if (G == 1) hipLaunchKernelGGL((conv3x3_narrowin<1, 2>), grid, dim3(256), 0, st, a);
  else if (NT == 1) hipLaunchKernelGGL((conv3x3_narrowin<2, 1>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((conv3x3_narrowin<2, 2>), grid, dim3(256), 0, st, a);
  return check_launch("conv3x3_narrowin");
}
// split-K plan: below 1024 blocks of 8 x 32 pixels, split the 32-channel chunks over ~thin_blocks (512) blocks
static long g_thin_th = 8, g_thin_blocks = 512;
static int thin_splitk_plan(long n, int h, int w, int cin_pad) {
  const long tiles = n * ((h + 7) / 8) * ((w + 31) / 32);  // in 8-row units whatever the tile height
  const int nch = cin_pad / 32;
  if (tiles <= 0 || tiles >= 1024 || nch < 4) return 1;
  int ks = (int)((g_thin_blocks + tiles - 1) / tiles);
  if (ks > nch / 2) ks = nch / 2;
  if (ks < 2) return 1;
  const int per = (nch + ks - 1) / ks;
  return (nch + per - 1) / per;
}
// persistent grid: at most g_thin_rounds resident rounds of blocks (0: one block per tile, the r02 launch)
static long g_thin_rounds = 1;
template <int TH>
static int thin_resident() {
  static int dev_seen = -1, resident = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != dev_seen) {
    int per_cu = 0, n_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&conv3x3_thin<TH, true>), 256, 0);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return -1;
    resident = per_cu * n_cu;
    dev_seen = dev;
  }
  return resident;
}
// the LDS-DMA thin kernel (conv3x3_thin_dma): 0 off; 1 = 8-row tiles, 3-slot ring; 2 = 4-row tiles, 4 slots;
// 3 = 4-row tiles, 3 slots; 4 = 8-row tiles, 2 slots.  A resident grid of thin_dma_rounds x blocks per CU x CUs
static long g_thin_dma = 0, g_thin_dma_rounds = 1;
long g_conv_prio = 0;  // ConvArgs::prio (conv_common.h)
static long g_thin_rowreuse = 1;  // conv3x3_thin: thin_chunk's row reuse (0: the r03 tap-major loop)
static long g_thin_twalk = 1;     // conv3x3_thin: XCD-banded tile walk (ConvArgs::twalk; 0: round-robin)
template <int TH, int S>
static int launch_thin_dma_cfg(ConvArgs& a, long n, int ks, hipStream_t st) {
  constexpr int lds = thin_dma_lds<TH, S>();
  static int dev_seen = -1, resident = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != dev_seen) {
    const void* fn = reinterpret_cast<const void*>(&conv3x3_thin_dma<TH, S>);
    int per_cu = 0, n_cu = 0;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return fail(VM_EHIP, "conv3x3_thin_dma: %s", hipGetErrorString(e));
    resident = per_cu * n_cu;
    dev_seen = dev;
  }
  long gx = n * ((a.H + TH - 1) / TH) * (long)((a.W + 31) / 32);
  if (gx > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_thin_dma: too many tiles");
  a.tiles_total = (int)gx;
  const long cap = g_thin_dma_rounds * (long)resident / ks;
  if (gx > cap) gx = cap < 1 ? 1 : cap;
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_thin_dma<%d, %d>", TH, S);
  hipLaunchKernelGGL((conv3x3_thin_dma<TH, S>), dim3((unsigned)gx, ks), dim3(256), lds, st, a);
  return check_launch("conv3x3_thin_dma");
}
static int launch_thin_dma(ConvArgs& a, long n, int ks, hipStream_t st) {
  switch (g_thin_dma) {
    case 2: return launch_thin_dma_cfg<4, 4>(a, n, ks, st);
    case 3: return launch_thin_dma_cfg<4, 3>(a, n, ks, st);
    case 4: return launch_thin_dma_cfg<8, 2>(a, n, ks, st);
    default: return launch_thin_dma_cfg<8, 3>(a, n, ks, st);
  }
}
static int dispatch_thin(ConvArgs& a, long n, hipStream_t st) {
  const int th = (int)g_thin_th;
  const long tiles = n * ((a.H + th - 1) / th) * ((a.W + 31) / 32);
  if (tiles > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_thin: too many tiles");
  a.tiles_total = (int)tiles;
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  const int res = th == 16 ? thin_resident<16>() : th == 4 ? thin_resident<4>() : thin_resident<8>();
  if (res < 0) return fail(VM_EHIP, "conv3x3_thin: occupancy query failed");
  long gx = tiles;
  if (g_thin_rounds > 0 && res > 0) {
    const long cap = g_thin_rounds * (long)res / ks;
    if (gx > cap) gx = cap < 1 ? 1 : cap;
  }
  if (g_thin_dma) {
    const int rc = launch_thin_dma(a, n, ks, st);
    if (rc) return rc;
    if (a.ksplit <= 1) return VM_OK;
    const long work = a.M * ((a.cout + 3) / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, a.part, a.ksplit, a.M,
                       a.cout, a.bias, a.scale, a.shift, a.act, a.y, a.y_dtype, a.y_cstride, a.y_coff);
    return check_launch("splitk_reduce");
  }
  const dim3 grid((unsigned)gx, ks);
  a.twalk = (int)g_thin_twalk;
  if (!g_thin_rowreuse) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_thin<%d, false>", th);
    if (th == 16) hipLaunchKernelGGL((conv3x3_thin<16, false>), grid, dim3(256), 0, st, a);
    else if (th == 4) hipLaunchKernelGGL((conv3x3_thin<4, false>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_thin<8, false>), grid, dim3(256), 0, st, a);
  } else {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_thin<%d, true>", th);
    if (th == 16) hipLaunchKernelGGL((conv3x3_thin<16, true>), grid, dim3(256), 0, st, a);
    else if (th == 4) hipLaunchKernelGGL((conv3x3_thin<4, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_thin<8, true>), grid, dim3(256), 0, st, a);
  }
  int rc = check_launch("conv3x3_thin");
  if (rc || a.ksplit <= 1) return rc;
  const long work = a.M * ((a.cout + 3) / 4);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, a.part, a.ksplit, a.M, a.cout,
                     a.bias, a.scale, a.shift, a.act, a.y, a.y_dtype, a.y_cstride, a.y_coff);
  return check_launch("splitk_reduce");
}

// tuning knobs (vm_set_option): conv_kernel 0 = auto, 1 = register-staged only, 2 = LDS-DMA whenever legal;
// conv_min_tiles = smallest grid (in 256-wide output tiles) for which auto picks the LDS-DMA kernel;
// glds_rb = K-step bytes of the 256x256 LDS-DMA tile (64: 4-slot ring, 128: 2-slot).
static long g_conv_kernel = 0;
static long g_conv_min_tiles = 128;
static long g_glds_rb = 128;
static long g_head_kernel = 0;
static long g_head_th = 16;  // conv3x3_head_mfma tile height for the bf16 128-channel head (8 or 16)
static long g_patch_cfg = 0;
#ifdef VM_STUDY
static long g_softmax_abl = 0;  // conv3x3_first_softmax_f32 timing ablations
static long g_patch_rowslot = 1;  // 0 = the per-tap-barrier dispatch of r01 (A/B runs)
static long g_patch_ablate = 0;
#endif
static long g_rows_kernel = 1;        // conv_rows.hip: 0 = off, 1 = auto (grid size), 8 / 16 = forced tile height
static long g_rows_min_blocks = 400;
static long g_rows_up = 0;            // 1: the folded upconvs too
static long g_rows_min_cin = 64;       // r04 A/B: conv2_1 (cin 64, 2040 blocks) +0.3 % on rows<16>; below 64 the
                                       // 2-blocks-per-CU patch kernel hides prologue/epilogue better
static long g_src_span_limit = 0x7ffffff0L;  // split-source byte span the 32-bit offset kernels take (option
                                              // "src_span_limit" lowers it for the fallback tests)
static long g_pair_strip = 1;  // vm_conv3x3_pair_first*: 1 = the strip-walking kernel (conv_pair.hip) where it applies
static long g_pair_kernel = 0;  // vm_conv3x3_pair_first_nhwc: 0 = persistent weights-resident kernel when cout == 64,
                                // 1 = streaming patch kernel

static bool patch_ok(const ConvArgs& a, size_t tsize) {
  // bf16 output (16-byte aligned view), or f32 output without the fused pool / folded resize (cout multiple of 4;
  // dword stores when the view is not 16-byte aligned)
  const bool yok = a.y_dtype == VM_BF16 ? (a.cout & 7) == 0 && a.y_vec
                                        : (a.y_dtype == VM_F32 && (!a.py || a.ysplit) && (!a.up || a.ysplit) &&
                                           (a.cout & 3) == 0);
  return tsize == 2 && a.chunk_major && a.cin_pad % 32 == 0 && yok && a.act != VM_ACT_SOFTMAX &&
         (a.x_src_c <= 0 || a.x_src_c % 32 == 0);
}

// packed frames (ConvArgs::vstride): a batch of narrow frames tiled as one virtual image when that saves >= 10 % of
// the column tiles (8 x 320^2 training crops: the 80 / 40 / 20-wide tower levels, 3 / 2 / 1 tiles per frame -> 2.6
// / 1.3 / 0.7).  Results are bit-identical (every output keeps its K loop); only which pixels share a block changes.
// Off for the folded upconvs, odd widths under a fused pool, and where the batch's 32-bit byte offsets would wrap.
static long g_pack_frames = 1;
static void plan_packed_frames(ConvArgs& a) {
  a.vstride = a.vW = 0;
  const long N = a.M / ((long)a.H * a.W);
  if (!g_pack_frames || a.up || N < 2 || (a.py && (a.W & 1))) return;
  const long plain = N * ((a.W + 31) / 32), packed = (N * (a.W + 2) + 31) / 32;
  if (packed * 10 > plain * 9 || N * (a.W + 2) > 0x7fffffffL) return;
  const long lim = 0x7ffffff0L;
  long xspan = a.M * a.x_cstride * 2;
  if (a.x_src_c > 0) xspan += (long)(a.cin_pad / a.x_src_c - 1) * a.x_src_stride * 2;
  const long yspan = a.ksplit > 1 ? a.M * a.cout * 4 : a.M * a.y_cstride * (a.y_dtype == VM_F32 ? 4 : 2);
  const long pspan = a.py ? N * ((a.H + 1) / 2) * ((a.W + 1) / 2) * a.py_cstride * 2 : 0;
  if (xspan >= lim || yspan >= lim || pspan >= lim) return;
  a.vstride = a.W + 2;
  a.vW = (int)(N * (a.W + 2));
}

static int dispatch_patch(ConvArgs& a, hipStream_t st) {
  plan_packed_frames(a);
  if (a.ksplit > 1) {  // split-K: the 4 x 32-pixel row-slot config, then the fixed-order reduction
    int rc = launch_patch<64, 4, 1, 2, 4, 2, 9, false, 0, false, 3>(a, st);
    if (rc) return rc;
    const long work = a.M * ((a.cout + 3) / 4);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid_for(work, 256)), dim3(256), 0, st, a.part, a.ksplit, a.M,
                       a.cout, a.bias, a.scale, a.shift, a.act, a.y, a.y_dtype, a.y_cstride, a.y_coff, a.ysplit, a.ovf);
    return check_launch("splitk_reduce");
  }
#ifdef VM_STUDY
  switch (g_patch_ablate) {  // timing experiments on the default tiling (results are garbage)
    case 1: return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 1>(a, st);
    case 2: return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 2>(a, st);
    case 3: return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 3>(a, st);
    case 4: return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 4>(a, st);
    case 6: return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 6>(a, st);
    case 7: return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 7>(a, st);
    // the same ablations on the row-slot default (64 x 8 waves, 2-slot ring of kernel rows)
    case 11: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 1, false, 3>(a, st);
    case 12: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 2, false, 3>(a, st);
    case 14: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 4, false, 3>(a, st);
    case 16: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 6, false, 3>(a, st);
    case 18: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 8, false, 3>(a, st);
    case 19: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 5, false, 3>(a, st);
    case 20: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 16, false, 3>(a, st);
    case 21: return launch_patch<64, 8, 1, 2, 8, 1, 9, false, 32, false, 3>(a, st);
    case 22: return launch_patch<64, 8, 1, 2, 8, 2, 9, false, 16, false, 3>(a, st);
    default: break;
  }
#endif
  switch (g_patch_cfg) {
    // the tilings the dispatcher below picks (the only ones in the shipped library)
    case 19: return launch_patch_up<64, 8, 1, 3, 8, 1, 9, false, 0, false, 3>(a, st);
    case 22: return launch_patch_up<64, 8, 1, 2, 8, 1, 9, false, 0, false, 3>(a, st);
    case 25: return launch_patch_up<64, 4, 1, 2, 4, 2, 9, false, 0, false, 3>(a, st);
    case 30: return launch_patch_up<128, 4, 2, 3, 8, 2>(a, st);
#ifdef VM_STUDY
    // study build only (make study): every tiling of the r01/r02 sweeps (scripts/sweep.sh, scripts/conv_study.sh)
    case 1: return launch_patch<64, 4, 1, 6>(a, st);
    case 2: return launch_patch<128, 2, 2, 6>(a, st);
    case 3: return launch_patch<128, 4, 2, 4>(a, st);
    case 4: return launch_patch<128, 4, 2, 6>(a, st);
    case 5: return launch_patch<64, 8, 1, 6>(a, st);
    case 6: return launch_patch<64, 8, 1, 6, 8, 1, 9, true>(a, st);
    case 7: return launch_patch<64, 8, 1, 4, 8, 1, 9, true>(a, st);
    case 8: return launch_patch<128, 4, 1, 4, 8, 2>(a, st);
    case 9: return launch_patch<128, 2, 2, 4, 8, 2>(a, st);
    case 10: return launch_patch<256, 4, 2, 3, 8, 1>(a, st);
    case 11: return launch_patch<64, 8, 1, 6, 4>(a, st);
    case 12: return launch_patch<64, 4, 1, 6, 4>(a, st);
    case 13: return launch_patch<128, 4, 1, 4, 8, 2, 9, true>(a, st);
    case 14: return launch_patch<128, 4, 1, 5, 8, 2, 9, true>(a, st);
    case 15: return launch_patch<128, 4, 1, 6, 8, 2, 9, false>(a, st);
    // 16 x 32 px tiles: half the weight-stream DMA per pixel of the 8 x 32 tiles
    case 16: return launch_patch<64, 8, 1, 6, 16>(a, st);
    case 17: return launch_patch<128, 8, 1, 4, 16>(a, st);
    case 18: return launch_patch<128, 4, 2, 4, 16>(a, st);
    // one barrier per kernel row (3 taps per ring slot), tap g+1's fragments read under tap g's MFMAs
    case 20: return launch_patch<64, 4, 1, 3, 8, 2, 9, false, 0, false, 3>(a, st);
    case 21: return launch_patch<128, 4, 1, 2, 4, 2, 9, false, 0, false, 3>(a, st);
    case 23: return launch_patch<128, 8, 1, 2, 8, 1, 9, false, 0, false, 3>(a, st);
    case 24: return launch_patch<128, 4, 2, 2, 8, 1, 9, false, 0, false, 3>(a, st);
    // one 8 x 32 px patch shared by 256 output channels (8 waves of 64 px x 128 channels, one block per CU)
    case 26: return launch_patch<256, 4, 2, 2, 8, 1, 9, false, 0, false, 3>(a, st);
    // 64 px x 64 channel wave tiles, 4 waves (two 256 px x 64 channel blocks per CU)
    case 27: return launch_patch<64, 4, 1, 2, 8, 2, 9, false, 0, false, 3>(a, st);
    // 16 x 32 px tiles on 16 waves of 32 px x 64 channels (1024 threads, one block per CU): half the weight DMA per MFMA
    case 28: return launch_patch<64, 16, 1, 2, 16, 1, 9, false, 0, false, 3>(a, st);
    case 29: return launch_patch<64, 16, 1, 3, 16, 1, 9, false, 0, false, 3>(a, st);
    // 64 px x 64 channel wave tiles at 4 waves per SIMD, 4-slot ring
    case 31: return launch_patch<128, 4, 2, 4, 8, 2>(a, st);
#endif
    default: break;
  }
  // row-stationary kernel (conv_rows.hip) on grids of >= g_rows_min_blocks 16 x 32 px x 64 channel blocks (one block
  // per CU: ~4 full rounds); rows_kernel 8 / 16 forces that tile height wherever it is legal
  if (g_rows_kernel && rows_ok(a)) {
    if (g_rows_kernel == 8 || g_rows_kernel == 16) {  // forced: per-frame tiles (the rows kernel does not pack)
      a.vstride = a.vW = 0;
      return launch_rows(a, st, (int)g_rows_kernel);
    }
    const long N16 = a.M / ((long)a.H * a.W);
    const long blocks16 = N16 * ((a.H + 15) / 16) * ((a.W + 31) / 32) * ((a.cout + 63) / 64);
    // measured in the 1080p forward (scripts/opt_ab.sh, bench.py --layers --option rows_min_*): a win for cin >= 256
    // on >= 400 blocks (conv3_4, conv2_3, conv3_2, conv3_3: -3..-4 %) and for cin 128 on >= 800 blocks (conv2_2,
    // conv3_1: -2..-3 %; r03: whole forward +1.0 % same-box); a loss for the folded upconvs (8-byte phase-scattered
    // stores), cin 64 (conv2_1: the persistent patch kernel is faster)
    // ... and only where its 16-row tiles waste no more rows than the patch kernel's 8-row ones (the training
    // towers' 40 x 40 level: 48 of 40 rows vs 40, measured 612 vs ~800 TFLOP/s)
    const bool rows_fit = ((a.H + 15) / 16) * 16 <= ((a.H + 7) / 8) * 8 + a.H / 32;
    if ((!a.up || g_rows_up) && !a.vstride && rows_fit && blocks16 >= g_rows_min_blocks && a.cin_pad >= g_rows_min_cin &&
        (a.cin_pad >= 2 * g_rows_min_cin || blocks16 >= 2 * g_rows_min_blocks))
      return launch_rows(a, st, 16);
  }
  // measured per layer inside the UNetVideo 1080p forward (scripts/sweep.sh, profiles/r01_patch_cfg_sweep.txt):
  // 8 waves of 32 px x 64 channels with one barrier per kernel row (3 taps per ring slot) everywhere, except
  // 4 waves of 64 px x 128 channels (2 blocks per CU, one barrier per tap) for cin >= 512, cout >= 128 on grids
  // of >= ~2 full rounds of blocks, a 3-slot ring for the largest grids, 4 x 32 px tiles for grids under 2 rounds.
  // Same-box A/B of the whole forward (bench.py --option patch_rowslot=0|1): 292.4 -> 306.8 frames/s
  const long N = a.M / ((long)a.H * a.W);
  const long sp = a.vstride ? ((a.H + 7) / 8) * (long)((a.vW + 31) / 32) : N * ((a.H + 7) / 8) * ((a.W + 31) / 32);
  const long blocks64 = sp * ((a.cout + 63) / 64);
#ifdef VM_STUDY
  if (!g_patch_rowslot) {
    if (a.cout >= 128 && a.cin_pad >= 256 && sp * ((a.cout + 127) / 128) >= 1000)
      return launch_patch<128, 4, 1, 4, 8, 2>(a, st);
    if (blocks64 < 512) return launch_patch<64, 4, 1, 6, 4>(a, st);
    return launch_patch<64, 8, 1, 6>(a, st);
  }
#endif
  // (a folded upconv takes the row-slot configs below, whose instantiation skips its phases' zero taps)
  if (!(a.up && g_up_skip) && a.cout >= 128 && a.cin_pad >= 512 && sp * ((a.cout + 127) / 128) >= 1000) {
    // fp16 operands (the split x3 forward's upconv_2 / _3, K = 3 x cin): the 3-slot 64-channel ring measured faster
    // (same box, patch_cfg 19 vs auto: 0.759 / 0.803 -> 0.732 / 0.754 ms, profiles/r06k_f16x3_patch_cfg_ab.log)
    if (a.f16) return launch_patch_up<64, 8, 1, 3, 8, 1, 9, false, 0, false, 3>(a, st);
    return launch_patch_up<128, 4, 2, 3, 8, 2>(a, st);  // 64 px x 64 channel waves, 4 per SIMD (r02: -5% vs 4x1)
  }
  if (persist_ok(a)) {  // the same tilings, persistent (2-slot ring: the LDS also holds the block's constants)
    const bool sk = a.up && g_up_skip;
    int rc = 1;
    if (blocks64 >= 512)
      rc = sk ? launch_patch_persist<64, 8, 1, 2, 8, 1, true>(a, st) : launch_patch_persist<64, 8, 1, 2, 8, 1, false>(a, st);
    else
      rc = sk ? launch_patch_persist<64, 4, 1, 2, 4, 2, true>(a, st) : launch_patch_persist<64, 4, 1, 2, 4, 2, false>(a, st);
    if (rc != 1) return rc;
  }
  // the 3-slot ring for the largest grids and for the folded upconvs the persistent kernel leaves (upconv_2: its
  // zero-tap phases are latency-bound on the ring, a deeper prefetch measured -2 %)
  if (blocks64 >= 8000 || (a.up && g_up_skip && blocks64 >= 512))
    return launch_patch_up<64, 8, 1, 3, 8, 1, 9, false, 0, false, 3>(a, st);
  if (blocks64 < 512) return launch_patch_up<64, 4, 1, 2, 4, 2, 9, false, 0, false, 3>(a, st);  // L5: 4 x 32 px tiles
  return launch_patch_up<64, 8, 1, 2, 8, 1, 9, false, 0, false, 3>(a, st);
}

template <typename T, bool FAST>
static int dispatch_glds(ConvArgs& a, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    if (a.cout > 128) {
      if (g_glds_rb == 64) return launch_glds<T, 64, 256, 256, 2, 4, 4, FAST>(a, st);
      return launch_glds<T, 128, 256, 256, 2, 4, 2, FAST>(a, st);
    }
  }
  if (a.cout > 64) return launch_glds<T, 64, 256, 128, 4, 2, 6, FAST>(a, st);
  return launch_glds<T, 64, 512, 64, 8, 1, 4, FAST>(a, st);
}

static int launch_first(ConvArgs& a, hipStream_t st) {
  const long N = a.M / ((long)a.H * a.W);
  const long sp = N * ((a.H + 7) / 8) * ((a.W + 31) / 32);
  a.tiles_n = (a.cout + 63) / 64;
  if (sp * a.tiles_n > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3: too many tiles");
  a.tiles_total = (int)(sp * a.tiles_n);
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first");
  static int attr_dev = -1, resident = 0;  // blocks resident on the whole chip (2 per CU at 98 VGPRs, 41 KB LDS)
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (attr_dev != dev) {
    int per_cu = 0, n_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&conv3x3_first),
                                                                512, 0);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return fail(VM_EHIP, "conv3x3_first setup: %s", hipGetErrorString(e));
    resident = per_cu * n_cu / 8 * 8;
    attr_dev = dev;
  }
  // a multiple of 8 blocks (xcd_tile's XCD ranges stay per block), at most one resident round
  int grid = resident > 0 && resident < a.tiles_total ? resident : a.tiles_total;
  if (grid > 8) grid = grid / 8 * 8;
  hipLaunchKernelGGL(conv3x3_first, dim3(grid), dim3(512), 0, st, a);
  return check_launch("conv3x3_first");
}

static int g_softmax_kernel = 6;  // 0: the generic kernels' softmax epilogue, 1: conv3x3_first_softmax, 2: its NT form,
                                  // 3 / 4: plain / NT with the per-wave LDS transpose (whole-pixel stores), 5: 4 with
                                  // LDS weights, 6: wave-private strips (conv3x3_first_softmax_strip, default)
static long g_softmax_blocks = 2048;  // persistent grid of conv3x3_first_softmax*
static long g_pair_xin_wide = 1;  // pair kernel, f32 frames with >= 4 channels: two 16-byte loads per pixel (XIN 2)

static int launch_first_softmax(ConvArgs& a, hipStream_t st) {
  const long N = a.M / ((long)a.H * a.W);
  const long sp = N * ((a.H + 7) / 8) * ((a.W + 31) / 32);
  if (sp > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3: too many tiles");
  a.tiles_total = (int)sp;
  // persistent grid of g_softmax_blocks; tile_of() maps block-order indices in rounds of tiles_n = grid onto
  // contiguous per-XCD bands (xcd_tile within a round)
  const int grid = (int)std::min<long>(sp, g_softmax_blocks);
  a.tiles_n = grid;
  if (g_softmax_kernel == 3) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax<false, true>");
    hipLaunchKernelGGL((conv3x3_first_softmax<false, true>), dim3(grid), dim3(512), 0, st, a);
  } else if (g_softmax_kernel == 4) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax<true, true>");
    hipLaunchKernelGGL((conv3x3_first_softmax<true, true>), dim3(grid), dim3(512), 0, st, a);
  } else if (g_softmax_kernel == 6) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_strip");
    hipLaunchKernelGGL(conv3x3_first_softmax_strip, dim3(grid), dim3(512), 0, st, a);
  } else if (g_softmax_kernel == 5) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax<true, true, true>");
    hipLaunchKernelGGL((conv3x3_first_softmax<true, true, true>), dim3(grid), dim3(512), 0, st, a);
  } else if (g_softmax_kernel == 2) {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax<true>");
    hipLaunchKernelGGL(conv3x3_first_softmax<true>, dim3(grid), dim3(512), 0, st, a);
  } else {
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax<false>");
    hipLaunchKernelGGL(conv3x3_first_softmax<false>, dim3(grid), dim3(512), 0, st, a);
  }
  return check_launch("conv3x3_first_softmax");
}

static long g_softmax_f32p = 4;  // the pipelined f32 refine kernel's variant (softmax_f32p option); 0: the r03 one

static int launch_first_softmax_f32(ConvArgs& a, int cin, hipStream_t st) {
  const long N = a.M / ((long)a.H * a.W);
  const long sp = N * ((a.H + 7) / 8) * ((a.W + 31) / 32);
  if (sp > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3: too many tiles");
  a.tiles_total = (int)sp;
  const int grid = (int)std::min<long>(sp, g_softmax_blocks);
  a.tiles_n = grid;
  if (g_softmax_f32p && !a.scale && !a.shift) {  // (a scale / shift epilogue: the r03 kernel below)
    // one resident round (2 waves per SIMD: one 512-thread block per CU); softmax_blocks caps it for tests
    static int n_cu = 0;
    if (!n_cu) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
        return fail(VM_EHIP, "conv3x3_first_softmax_f32p: CU count query failed");
    }
    const int gp = (int)std::min<long>(std::min<long>(sp, n_cu), g_softmax_blocks);
    a.tiles_n = gp;
#define VM_SMP(C)                                                                             \
  case C:                                                                                    \
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<%d, 2, false, 0, 18>", C); \
    hipLaunchKernelGGL((conv3x3_first_softmax_f32p<C, 2, false, 0, 18>), dim3(gp), dim3(512), 0, st, a);     \
    break;
    if (g_softmax_f32p == 6) {  // the row-ring form: segments of a.seg rows x 32-pixel bands, one per wave
      const long nimg = N, bands = (a.W + 31) / 32;
      const long waves = (long)gp * 8;
      long seg = (nimg * bands * a.H + waves - 1) / waves;  // rows per segment for about one item per wave
      if (seg < 4) seg = 4;
      const long items = nimg * bands * ((a.H + seg - 1) / seg);
      if (items > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_first_softmax_f32r: too many items");
      a.seg = (int)seg;
      a.tiles_total = (int)items;
      switch (cin) {
#define VM_SMR(C)                                                                                              \
  case C:                                                                                                      \
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32r<%d>", C);                   \
    hipLaunchKernelGGL((conv3x3_first_softmax_f32r<C>), dim3((unsigned)std::min<long>(gp, (items + 7) / 8)),  \
                       dim3(512), 0, st, a);                                                                   \
    break;
        VM_SMR(1) VM_SMR(2) VM_SMR(3) VM_SMR(4) VM_SMR(5) VM_SMR(6) VM_SMR(7) VM_SMR(8)
#undef VM_SMR
        default: return fail(VM_EINVAL, "conv3x3_first_softmax_f32r: cin %d", cin);
      }
      return check_launch("conv3x3_first_softmax_f32r");
    }
#ifdef VM_STUDY
    if (cin == 5 && g_softmax_abl) {  // timing ablations (garbage results): 1 no stores, 2 no MFMA, 4 no softmax
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<5, 2, false, %ld, 18>", g_softmax_abl);
      switch (g_softmax_abl) {
        case 1: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 1, 18>), dim3(gp), dim3(512), 0, st, a); break;
        case 2: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 2, 18>), dim3(gp), dim3(512), 0, st, a); break;
        case 3: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 3, 18>), dim3(gp), dim3(512), 0, st, a); break;
        case 4: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 4, 18>), dim3(gp), dim3(512), 0, st, a); break;
        case 5: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 5, 18>), dim3(gp), dim3(512), 0, st, a); break;
        case 6: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 6, 18>), dim3(gp), dim3(512), 0, st, a); break;
        default: hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 7, 18>), dim3(gp), dim3(512), 0, st, a); break;
      }
      return check_launch("conv3x3_first_softmax_f32p");
    }
#endif
    if (cin <= 5 && g_softmax_f32p == 7) {  // split-bf16 x6 on the bf16 MFMA (f32 accuracy; X6 above)
      switch (cin) {
#define VM_SMX(C)                                                                                        \
  case C:                                                                                                \
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<%d, 2, false, 0, 18, true>", C); \
    hipLaunchKernelGGL((conv3x3_first_softmax_f32p<C, 2, false, 0, 18, true>), dim3(gp), dim3(512), 0, st, a);     \
    break;
        VM_SMX(1) VM_SMX(2) VM_SMX(3) VM_SMX(4) VM_SMX(5)
#undef VM_SMX
        default: break;
      }
      return check_launch("conv3x3_first_softmax_f32p");
    }
    if (cin == 5 && g_softmax_f32p == 2) {
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<5, 4>");
      hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 4>), dim3(gp), dim3(512), 0, st, a);
      return check_launch("conv3x3_first_softmax_f32p");
    }
    if (cin == 5 && g_softmax_f32p >= 4) {  // LDS-transposed whole-pixel stores: 4 non-temporal, 5 through L2
      if (g_softmax_f32p == 4) {
        snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<5, 2, false, 0, 18>");
        hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 0, 18>), dim3(gp), dim3(512), 0, st, a);
      } else {
        snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<5, 2, false, 0, 16>");
        hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 0, 16>), dim3(gp), dim3(512), 0, st, a);
      }
      return check_launch("conv3x3_first_softmax_f32p");
    }
    if (cin == 5 && g_softmax_f32p == 1) {  // stores straight from the accumulator lanes through L2 (A/B)
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<5>");
      hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5>), dim3(gp), dim3(512), 0, st, a);
      return check_launch("conv3x3_first_softmax_f32p");
    }
    if (cin == 5 && g_softmax_f32p == 3) {  // non-temporal stores (A/B)
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32p<5, 2, false, 0, 2>");
      hipLaunchKernelGGL((conv3x3_first_softmax_f32p<5, 2, false, 0, 2>), dim3(gp), dim3(512), 0, st, a);
      return check_launch("conv3x3_first_softmax_f32p");
    }
    switch (cin) {
      VM_SMP(1) VM_SMP(2) VM_SMP(3) VM_SMP(4) VM_SMP(5) VM_SMP(6) VM_SMP(7) VM_SMP(8)
      default: return fail(VM_EINVAL, "conv3x3_first_softmax_f32p: cin %d", cin);
    }
#undef VM_SMP
    return check_launch("conv3x3_first_softmax_f32p");
  }
#define VM_SMF(C)                                                                            \
  case C:                                                                                   \
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32<%d>", C); \
    hipLaunchKernelGGL(conv3x3_first_softmax_f32<C>, dim3(grid), dim3(512), 0, st, a);      \
    break;
#ifdef VM_STUDY
  if (cin == 5 && g_softmax_abl) {  // timing ablations of the f32 refine kernel (results are garbage)
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_first_softmax_f32<5, %ld>", g_softmax_abl);
    if (g_softmax_abl == 1) hipLaunchKernelGGL((conv3x3_first_softmax_f32<5, 1>), dim3(grid), dim3(512), 0, st, a);
    else if (g_softmax_abl == 2) hipLaunchKernelGGL((conv3x3_first_softmax_f32<5, 2>), dim3(grid), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_first_softmax_f32<5, 3>), dim3(grid), dim3(512), 0, st, a);
    return check_launch("conv3x3_first_softmax_f32");
  }
#endif
  switch (cin) {
    VM_SMF(1) VM_SMF(2) VM_SMF(3) VM_SMF(4) VM_SMF(5) VM_SMF(6) VM_SMF(7) VM_SMF(8)
    default: return fail(VM_EINVAL, "conv3x3_first_softmax_f32: cin %d", cin);
  }
#undef VM_SMF
  return check_launch("conv3x3_first_softmax_f32");
}

template <typename T>
static int dispatch_mfma(ConvArgs& a, hipStream_t st, int cin = 0) {
  // f32 refine conv + softmax (cin <= 8 of a 16-byte-aligned 8-float pixel, 64 outputs, f32 out)
  if (sizeof(T) == 4 && g_softmax_kernel != 0 && g_conv_kernel != 1 && g_conv_kernel != 2 && cin > 0 && cin <= 8 &&
      a.cin_pad == 8 && !a.chunk_major && a.x_src_c <= 0 && a.y_dtype == VM_F32 && a.y_vec && a.act == VM_ACT_SOFTMAX &&
      a.cout == 64 && a.K_pad == 96 && a.x_cstride % 4 == 0 && a.x_coff % 4 == 0 &&
      reinterpret_cast<uintptr_t>(a.x) % 16 == 0)
    return launch_first_softmax_f32(a, cin, st);
  if (sizeof(T) == 2 && g_softmax_kernel != 0 && g_conv_kernel != 1 && g_conv_kernel != 2 && a.cin_pad == 8 &&
      !a.chunk_major && a.x_src_c <= 0 && a.y_dtype == VM_F32 && a.y_vec && a.act == VM_ACT_SOFTMAX && a.cout == 64 &&
      a.K_pad == 128)
    return launch_first_softmax(a, st);
  if (sizeof(T) == 2 && g_conv_kernel != 1 && g_conv_kernel != 2 && a.cin_pad == 8 && !a.chunk_major && a.x_src_c <= 0 &&
      a.y_dtype == VM_BF16 && a.y_vec && a.act != VM_ACT_SOFTMAX && (a.cout & 7) == 0 && a.K_pad == 128)
    return launch_first(a, st);
  if ((g_conv_kernel == 0 || g_conv_kernel == 3) && patch_ok(a, sizeof(T))) return dispatch_patch(a, st);
  if (g_conv_kernel != 1 && a.act != VM_ACT_SOFTMAX && a.x_src_c <= 0) {
    // measured (tools/convbench.py): the LDS-DMA kernel wins for cout >= 256 (256x256 tiles); for
    // cout <= 128 its 64-channel-wide waves are DMA-issue-bound and the register-staged kernel is faster
    const int bm = a.cout > 64 ? 256 : 512;
    const long tiles = ((a.M + bm - 1) / bm) * ((a.cout + 255) / 256);
    const bool wide = sizeof(T) == 2 && a.cout > 128;
    if (g_conv_kernel == 2 || (wide && tiles >= g_conv_min_tiles))
      return a.chunk_major ? dispatch_glds<T, true>(a, st) : dispatch_glds<T, false>(a, st);
  }
  if (a.cout <= 64) return launch_mfma<T, 256, 64>(a, st);
  return launch_mfma<T, 128, 128>(a, st);
}

}  // namespace vm

using namespace vm;

extern "C" int vm_set_option(const char* key, long value) {
  if (!key) return fail(VM_EINVAL, "set_option: NULL key");
  if (!strcmp(key, "conv_kernel")) {
    if (value < 0 || value > 3) return fail(VM_EINVAL, "conv_kernel must be 0..3");
    g_conv_kernel = value;
    return VM_OK;
  }
  if (!strcmp(key, "softmax_kernel")) {
    if (value < 0 || value > 6) return fail(VM_EINVAL, "softmax_kernel must be 0..6");
    g_softmax_kernel = value;
    return VM_OK;
  }
  if (!strcmp(key, "softmax_blocks")) {
    if (value < 1 || value > (1 << 20)) return fail(VM_EINVAL, "softmax_blocks must be 1..2^20");
    g_softmax_blocks = value;
    return VM_OK;
  }
  if (!strcmp(key, "head_th")) {
    if (value != 8 && value != 16) return fail(VM_EINVAL, "head_th must be 8 or 16");
    g_head_th = value;
    return VM_OK;
  }
  if (!strcmp(key, "softmax_f32p")) {  // 0 the r03 kernel; 1 pipelined; 2 its 4-waves-per-SIMD build; 3 NT stores;
                                       // 4 / 5 LDS-transposed whole-pixel stores, NT / through L2;
                                       // 6 the row-ring form (conv3x3_first_softmax_f32r); 7 split-bf16 x6
    if (value < 0 || value > 7) return fail(VM_EINVAL, "softmax_f32p must be 0..7");
    g_softmax_f32p = value;
    return VM_OK;
  }
  if (!strcmp(key, "cband")) {
    if (value < 0 || value > 2) return fail(VM_EINVAL, "cband must be 0, 1 or 2");
    g_cband = value;
    return VM_OK;
  }
  if (!strcmp(key, "ngroup")) {
    if (value < 0 || value > 64) return fail(VM_EINVAL, "ngroup must be 0..64");
    g_ngroup = value;
    return VM_OK;
  }
  if (!strcmp(key, "cband_bytes")) {
    g_cband_bytes = value;
    return VM_OK;
  }
  if (!strcmp(key, "rows_kernel")) {
    if (value != 0 && value != 1 && value != 8 && value != 16) return fail(VM_EINVAL, "rows_kernel must be 0, 1, 8 or 16");
    g_rows_kernel = value;
    return VM_OK;
  }
  if (!strcmp(key, "pack_tiled")) {
    g_pack_tiled = value;
    return VM_OK;
  }
  if (!strcmp(key, "persist_half")) {
    g_persist_half = value;
    return VM_OK;
  }
  if (!strcmp(key, "rows_up")) {
    g_rows_up = value;
    return VM_OK;
  }
  if (!strcmp(key, "rows_min_cin")) {
    g_rows_min_cin = value;
    return VM_OK;
  }
  if (!strcmp(key, "rows_min_blocks")) {
    g_rows_min_blocks = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_rounds")) {
    if (value < 0 || value > 64) return fail(VM_EINVAL, "thin_rounds must be 0..64");
    g_thin_rounds = value;
    return VM_OK;
  }
  if (!strcmp(key, "pack_frames")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "pack_frames must be 0 or 1");
    g_pack_frames = value;
    return VM_OK;
  }
  if (!strcmp(key, "up_skip")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "up_skip must be 0 or 1");
    g_up_skip = value;
    return VM_OK;
  }
  if (!strcmp(key, "src_span_limit")) {
    if (value < 1 || value > 0x7ffffff0L) return fail(VM_EINVAL, "src_span_limit must be 1..0x7ffffff0");
    g_src_span_limit = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_blocks")) {
    g_thin_blocks = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_th")) {
    if (value != 4 && value != 8 && value != 16) return fail(VM_EINVAL, "thin_th must be 4, 8 or 16");
    g_thin_th = value;
    return VM_OK;
  }
  if (!strcmp(key, "conv_prio")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "conv_prio must be 0 or 1");
    g_conv_prio = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_twalk")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "thin_twalk must be 0 or 1");
    g_thin_twalk = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_rowreuse")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "thin_rowreuse must be 0 or 1");
    g_thin_rowreuse = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_dma")) {  // 0: conv3x3_thin; 1..4: conv3x3_thin_dma configs (launch_thin_dma)
    if (value < 0 || value > 4) return fail(VM_EINVAL, "thin_dma must be 0..4");
    g_thin_dma = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_dma_rounds")) {
    if (value < 1 || value > 64) return fail(VM_EINVAL, "thin_dma_rounds must be 1..64");
    g_thin_dma_rounds = value;
    return VM_OK;
  }
  if (!strcmp(key, "narrowin_kernel")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "narrowin_kernel must be 0 or 1");
    g_narrowin = value;
    return VM_OK;
  }
  if (!strcmp(key, "thin_kernel")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "thin_kernel must be 0 or 1");
    g_thin_kernel = value;
    return VM_OK;
  }
  if (!strcmp(key, "conv_min_tiles")) {
    g_conv_min_tiles = value;
    return VM_OK;
  }
  if (!strcmp(key, "patch_cfg")) {
#ifdef VM_STUDY
    if (value < 0 || value > 31) return fail(VM_EINVAL, "patch_cfg must be 0..31");
#else
    if (value != 0 && value != 19 && value != 22 && value != 25 && value != 30)
      return fail(VM_EINVAL, "patch_cfg must be 0, 19, 22, 25 or 30 (other tilings: the study build, make study)");
#endif
    g_patch_cfg = value;
    return VM_OK;
  }
#ifdef VM_STUDY
  if (!strcmp(key, "patch_ablate")) {  // timing-only ablations: garbage results
    g_patch_ablate = value;
    return VM_OK;
  }
  if (!strcmp(key, "softmax_abl")) {  // timing-only ablations of the f32 refine kernel: garbage results
    g_softmax_abl = value;
    return VM_OK;
  }
  if (!strcmp(key, "patch_rowslot")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "patch_rowslot must be 0 or 1");
    g_patch_rowslot = value;
    return VM_OK;
  }
#endif
  if (!strcmp(key, "pair_xin_wide")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "pair_xin_wide must be 0 or 1");
    g_pair_xin_wide = value;
    return VM_OK;
  }
#ifdef VM_STUDY
  if (!strcmp(key, "pair_strip_abl")) {  // timing-only ablations of the strip pair kernel (garbage results)
    vm::g_pair_strip_abl = value;
    return VM_OK;
  }
#endif
  if (!strcmp(key, "border_ks")) {
    if (value != 1 && value != 2 && value != 4) return fail(VM_EINVAL, "border_ks must be 1, 2 or 4");
    g_border_ks = value;
    return VM_OK;
  }
  if (!strcmp(key, "patch_repi")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "patch_repi must be 0 or 1");
    g_patch_repi = value;
    return VM_OK;
  }
  if (!strcmp(key, "persist_rounds") || !strcmp(key, "persist_up_rounds")) {
    if (value < 0 || value > 64) return fail(VM_EINVAL, "%s must be in 0..64 (0: any grid)", key);
    (key[8] == 'u' ? g_persist_up_rounds : g_persist_rounds) = value;
    return VM_OK;
  }
  if (!strcmp(key, "persist_all") || !strcmp(key, "persist_rot")) {
    if (value < 0 || value > 2) return fail(VM_EINVAL, "%s must be 0, 1 or 2", key);
    (key[8] == 'a' ? g_persist_all : g_persist_rot) = value;
    return VM_OK;
  }
  if (!strcmp(key, "up_skip_mask")) {
    if (value < 0 || value > 3) return fail(VM_EINVAL, "up_skip_mask must be 0..3");
    g_up_skip_mask = value;
    return VM_OK;
  }
  if (!strcmp(key, "patch_persist")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "patch_persist must be 0 or 1");
    g_patch_persist = value;
    return VM_OK;
  }
  if (!strcmp(key, "pair_strip_pin")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "pair_strip_pin must be 0 or 1");
    vm::g_pair_strip_pin = value;
    return VM_OK;
  }
  if (!strcmp(key, "pair_strip")) {
    if (value < 0 || value > 1) return fail(VM_EINVAL, "pair_strip must be 0 or 1");
    g_pair_strip = value;
    return VM_OK;
  }
  if (!strcmp(key, "pair_kernel")) {
#ifdef VM_STUDY
    if (value < 0 || (value > 1 && value < 10) || value > 18) return fail(VM_EINVAL, "pair_kernel must be 0, 1 or 10..18");
#else
    if (value < 0 || value > 1) return fail(VM_EINVAL, "pair_kernel must be 0 or 1 (ablations: the study build)");
#endif
    g_pair_kernel = value;
    return VM_OK;
  }
  if (!strcmp(key, "head_kernel")) {
    if (value < 0 || value > 2) return fail(VM_EINVAL, "head_kernel must be 0, 1 or 2");
    g_head_kernel = value;
    return VM_OK;
  }
  if (!strcmp(key, "splitk_tiles")) {
    g_splitk_tiles = value;
    return VM_OK;
  }
  if (!strcmp(key, "glds_rb")) {
    if (value != 64 && value != 128) return fail(VM_EINVAL, "glds_rb must be 64 or 128");
    g_glds_rb = value;
    return VM_OK;
  }
  if (!strcmp(key, "bn_vec_fwd")) {
    g_bn_vec_fwd = value;
    return VM_OK;
  }
  if (!strcmp(key, "bn_blocks")) {
    if (value < 1 || value > BN_TARGET_MAX) return fail(VM_EINVAL, "set_option: bn_blocks must be 1..%d", BN_TARGET_MAX);
    g_bn_target = value;
    return VM_OK;
  }
  if (train_set_option(key, value)) return VM_OK;
  return fail(VM_EINVAL, "set_option: unknown key '%s'", key);
}

extern "C" const char* vm_conv3x3_last_kernel(void) { return g_last_kernel; }

extern "C" size_t vm_conv3x3_packed_bytes(int cin, int cout, int dtype) {
  if (cin <= 0 || cout <= 0 || (dtype != VM_F32 && dtype != VM_BF16 && dtype != VM_F16)) return 0;
  PackGeom g = geom(cin, cout, dtype);
  return (size_t)g.cout_pad * g.K_pad * elem_bytes(dtype);
}

extern "C" int vm_conv3x3_pack_weights(const float* w_hwio, int cin, int cout, int dtype, void* packed, void* stream) {
  if (!w_hwio || !packed || cin <= 0 || cout <= 0) return fail(VM_EINVAL, "pack_weights: bad argument");
  if (dtype != VM_F32 && dtype != VM_BF16 && dtype != VM_F16) return fail(VM_EINVAL, "pack_weights: dtype %d", dtype);
  PackGeom g = geom(cin, cout, dtype);
  ConvArgs a{};
  fill_geom(a, g);
  a.w = packed;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int grid = grid_for((long)g.cout_pad * g.K_pad, 256);
  if (dtype == VM_BF16) hipLaunchKernelGGL(pack_weights<uint16_t>, dim3(grid), dim3(256), 0, st, w_hwio, cin, cout, a);
  else if (dtype == VM_F16) hipLaunchKernelGGL(pack_weights<f16_t>, dim3(grid), dim3(256), 0, st, w_hwio, cin, cout, a);
  else hipLaunchKernelGGL(pack_weights<float>, dim3(grid), dim3(256), 0, st, w_hwio, cin, cout, a);
  return check_launch("pack_weights");
}

extern "C" int vm_conv3x3_pack_weights_batch(int njobs, const vm_pack_job* jobs, void* stream) {
  if (njobs < 0 || (njobs > 0 && !jobs)) return fail(VM_EINVAL, "pack_weights_batch: bad argument");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int i = 0; i < njobs; ++i) {
    const vm_pack_job& j = jobs[i];
    if (!j.w || !j.packed || j.cin <= 0 || j.cout <= 0 || j.w_cin <= 0 || j.w_cout <= 0 ||
        (j.dtype != VM_F32 && j.dtype != VM_BF16))
      return fail(VM_EINVAL, "pack_weights_batch: bad job %d", i);
  }
  // chunk-major bf16 packs: forward ones to the tiled transpose (pack_weights_tiled), flipped ones 8 channels per
  // lane (pack_weights_flip8); the rest element-wise.  kind 0 element-wise, 1 tiled, 2 flip8
  for (int tiled = 0; tiled < 3; ++tiled) {
    PackBatch b{};
    long mx = 1;
    auto flush = [&]() -> int {
      if (!b.n) return VM_OK;
      if (tiled == 1)
        hipLaunchKernelGGL(pack_weights_tiled, dim3((unsigned)mx, b.n), dim3(256), 0, st, b);
      else if (tiled == 2)
        hipLaunchKernelGGL(pack_weights_flip8, dim3(grid_for(mx, 256, 1024), b.n), dim3(256), 0, st, b);
      else
        hipLaunchKernelGGL(pack_weights_batch, dim3(grid_for(mx, 256, 256), b.n), dim3(256), 0, st, b);
      const int rc = check_launch("pack_weights_batch");
      b.n = 0;
      mx = 1;
      return rc;
    };
    for (int i = 0; i < njobs; ++i) {
      const vm_pack_job& j = jobs[i];
      const PackGeom g = geom(j.cin, j.cout, j.dtype);
      const bool vec = g_pack_tiled && j.dtype == VM_BF16 && g.chunk_major &&
                       reinterpret_cast<uintptr_t>(j.packed) % 16 == 0;
      const int kind = !vec ? 0 : j.flip ? 2 : 1;
      if (kind != tiled) continue;
      b.j[b.n] = j;
      b.K_pad[b.n] = g.K_pad;
      b.cout_pad[b.n] = g.cout_pad;
      b.cin_pad[b.n] = g.cin_pad;
      const long t = tiled == 1 ? (long)(g.K_pad / 32) * (g.cout_pad / 64)
                     : tiled == 2 ? (long)g.cout_pad * (g.K_pad / 8) : (long)g.cout_pad * g.K_pad;
      if (t > mx) mx = t;
      if (++b.n == PACK_MAX_JOBS) {
        const int rc = flush();
        if (rc) return rc;
      }
    }
    const int rc = flush();
    if (rc) return rc;
  }
  return VM_OK;
}

// split-fp16 x3 output of vm_conv3x3_split3_nhwc (ConvArgs::ysplit / psplit / ovf)
struct SplitOut {
  int yslab, pslab;
  int* ovf;
};

static int conv_impl(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias, const float* scale,
                     const float* shift, int act, vm_tensor* y, const vm_tensor* yp, void* stream,
                     float* y2 = nullptr, int nsrc = 0, long src_stride = 0, void* work = nullptr,
                     size_t work_bytes = 0, const float* head_part = nullptr, const float* y_acc = nullptr,
                     const SplitOut* so = nullptr);

extern "C" int vm_conv3x3_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                               const float* scale, const float* shift, int act, vm_tensor* y, void* stream) {
  return conv_impl(x, packed, cin, cout, bias, scale, shift, act, y, nullptr, stream);
}

extern "C" int vm_conv3x3_sources_nhwc(const vm_tensor* x, int nsrc, long src_stride, const void* packed, int cin,
                                       int cout, const float* bias, const float* scale, const float* shift, int act,
                                       vm_tensor* y, void* stream) {
  if (nsrc < 1 || (nsrc > 1 && src_stride <= 0)) return fail(VM_EINVAL, "conv3x3_sources: nsrc %d stride %ld", nsrc,
                                                            src_stride);
  return conv_impl(x, packed, cin, cout, bias, scale, shift, act, y, nullptr, stream, nullptr, nsrc, src_stride);
}

extern "C" int vm_conv3x3_pool_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                                    const float* scale, const float* shift, int act, vm_tensor* y, vm_tensor* ypool,
                                    void* stream) {
  if (!valid_tensor(ypool) || !y) return fail(VM_EINVAL, "conv3x3_pool: invalid pool tensor");
  if (ypool->n != y->n || ypool->h != (y->h + 1) / 2 || ypool->w != (y->w + 1) / 2 || ypool->c != cout ||
      ypool->dtype != y->dtype)
    return fail(VM_EINVAL, "conv3x3_pool: pool output must be [n, ceil(h/2), ceil(w/2), cout] in the output dtype");
  return conv_impl(x, packed, cin, cout, bias, scale, shift, act, y, ypool, stream);
}

extern "C" int vm_conv3x3_fold_up2x_weights(const float* w_hwio, int cin, int cout, float* w_up_hwio, void* stream) {
  if (!w_hwio || !w_up_hwio || cin <= 0 || cout <= 0) return fail(VM_EINVAL, "fold_up2x: bad argument");
  hipLaunchKernelGGL(fold_up2x_weights, dim3(grid_for(9L * cin * cout, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), w_hwio, cin, cout, w_up_hwio);
  return check_launch("fold_up2x_weights");
}

// head split of the folded upconv (vm_conv3x3_up2x_head_nhwc -> vm_conv3x3_up2x_nhwc): per-thread, set only for the
// duration of that call
struct UpHead {
  const float* hw;
  int hw_cin, hw_coff;
  float* hd;
  int y_skip;
};
static thread_local UpHead g_up_head = {};

extern "C" int vm_conv3x3_up2x_nhwc(const vm_tensor* x, const void* packed_up, const void* packed, int cin, int cout,
                                    const float* bias, const float* scale, const float* shift, int act, vm_tensor* y,
                                    void* stream) {
  if (!valid_tensor(x) || !valid_tensor(y) || !packed_up || !packed)
    return fail(VM_EINVAL, "conv3x3_up2x: invalid tensor/weights");
  if (cin <= 0 || cout <= 0 || x->c != cin || y->c != cout)
    return fail(VM_EINVAL, "conv3x3_up2x: channel mismatch x.c=%d cin=%d y.c=%d cout=%d", x->c, cin, y->c, cout);
  if (y->n != x->n || y->h != 2 * x->h || y->w != 2 * x->w)
    return fail(VM_EINVAL, "conv3x3_up2x: output must be [%d,%d,%d,%d]", x->n, 2 * x->h, 2 * x->w, cout);
  if (act < VM_ACT_NONE || act > VM_ACT_SOFTMAX) return fail(VM_EINVAL, "conv3x3_up2x: act %d", act);
  const PackGeom g = geom(cin, 4 * cout, x->dtype), g1 = geom(cin, cout, x->dtype);
  const bool xvec = reinterpret_cast<uintptr_t>(x->ptr) % 16 == 0 && x->cstride % 8 == 0 && x->coff % 8 == 0 &&
                    x->coff + g.cin_pad <= x->cstride;
  const bool yvec = reinterpret_cast<uintptr_t>(y->ptr) % 16 == 0 && y->cstride % 8 == 0 && y->coff % 8 == 0;
  if (x->dtype != VM_BF16 || y->dtype != VM_BF16 || cout % 64 || !xvec || !yvec || act == VM_ACT_SOFTMAX ||
      g_conv_kernel == 1 || g_conv_kernel == 2)
    return fail(VM_EUNSUPPORTED, "conv3x3_up2x: folded resize needs the bf16 patch kernel (cout %% 64 == 0, "
                                 "16-byte channel views)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ConvArgs a{};
  a.x = x->ptr; a.x_cstride = x->cstride; a.x_coff = x->coff; a.H = x->h; a.W = x->w;
  a.M = (long)x->n * x->h * x->w;
  fill_geom(a, g);
  a.w = packed_up; a.cout = 4 * cout;
  a.bias = bias; a.scale = scale; a.shift = shift; a.act = act;
  a.y = y->ptr; a.y_cstride = y->cstride; a.y_coff = y->coff; a.y_dtype = y->dtype; a.y_vec = 1;
  a.up = 1; a.up_cout = cout;
  a.hd = g_up_head.hd; a.hw = g_up_head.hw; a.hw_cin = g_up_head.hw_cin; a.hw_coff = g_up_head.hw_coff;
  a.y_skip = g_up_head.y_skip;
  if (!patch_ok(a, 2)) return fail(VM_EUNSUPPORTED, "conv3x3_up2x: shape not supported by the patch kernel");
  int rc = dispatch_patch(a, st);
  if (rc != VM_OK) return rc;
  BorderArgs b{};
  b.x = x->ptr; b.x_cstride = x->cstride; b.x_coff = x->coff; b.H = x->h; b.W = x->w; b.nframes = x->n;
  b.w = packed; b.K_pad = g1.K_pad; b.cout = cout; b.nch = g1.cin_pad / 32;
  b.bias = bias; b.scale = scale; b.shift = shift; b.act = act;
  b.y = y->ptr; b.y_cstride = y->cstride; b.y_coff = y->coff;
  b.hd = g_up_head.hd; b.hw = g_up_head.hw; b.hw_cin = g_up_head.hw_cin; b.hw_coff = g_up_head.hw_coff;
  b.y_skip = g_up_head.y_skip;
  const int OH = 2 * x->h, OW = 2 * x->w;
  b.nb = 2 * OW + 2 * (OH - 2);
  const long nblk = ((long)x->n * b.nb + 15) / 16;
  if (nblk > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_up2x: too many border pixels");
  if (g_border_ks == 4)
    hipLaunchKernelGGL(conv3x3_up2x_border<4>, dim3((unsigned)nblk, cout / 64), dim3(1024), 0, st, b);
  else if (g_border_ks == 2)
    hipLaunchKernelGGL(conv3x3_up2x_border<2>, dim3((unsigned)nblk, cout / 64), dim3(512), 0, st, b);
  else
    hipLaunchKernelGGL(conv3x3_up2x_border<1>, dim3((unsigned)nblk, cout / 64), dim3(256), 0, st, b);
  return check_launch("conv3x3_up2x_border");
}

static bool split3_view_ok(const vm_tensor* t, int slab, int c) {
  return t->dtype == VM_F16 && slab > 0 && slab % 8 == 0 && t->coff % 8 == 0 && t->cstride % 8 == 0 &&
         t->coff + c <= slab && 2 * slab <= t->cstride && reinterpret_cast<uintptr_t>(t->ptr) % 16 == 0;
}

extern "C" int vm_conv3x3_up2x_split3_nhwc(const vm_tensor* x, const void* packed_up, const void* packed, int cin,
                                           int cout, const float* bias, const float* scale, const float* shift, int act,
                                           vm_tensor* y, int y_slab, int* overflow, void* stream) {
  if (!valid_tensor(x, true) || !valid_tensor(y, true) || !packed_up || !packed)
    return fail(VM_EINVAL, "conv3x3_up2x_split3: invalid tensor/weights");
  const int S = x->c / 2;
  if (x->dtype != VM_F16 || y->dtype != VM_F16 || x->c % 64 || cin != 3 * S || y->c != cout)
    return fail(VM_EINVAL, "conv3x3_up2x_split3: fp16 views, x = [l, h] slabs of S %% 32 == 0 channels, cin = 3 S "
                           "(x.c=%d cin=%d y.c=%d cout=%d)", x->c, cin, y->c, cout);
  if (y->n != x->n || y->h != 2 * x->h || y->w != 2 * x->w)
    return fail(VM_EINVAL, "conv3x3_up2x_split3: output must be [%d,%d,%d,%d]", x->n, 2 * x->h, 2 * x->w, cout);
  if (act < VM_ACT_NONE || act >= VM_ACT_SOFTMAX) return fail(VM_EINVAL, "conv3x3_up2x_split3: act %d", act);
  const int ys = y_slab > 0 ? y_slab : y->cstride / 2;
  const PackGeom g = geom(cin, 4 * cout, VM_F16), g1 = geom(cin, cout, VM_F16);
  const bool xvec = reinterpret_cast<uintptr_t>(x->ptr) % 16 == 0 && x->cstride % 8 == 0 && x->coff % 8 == 0 &&
                    x->coff + x->c <= x->cstride;
  if (cout % 64 || !xvec || !split3_view_ok(y, ys, cout) || !g_up_skip || g_conv_kernel == 1 || g_conv_kernel == 2)
    return fail(VM_EUNSUPPORTED, "conv3x3_up2x_split3: cout %% 64 == 0, 16-byte channel views, the split layout");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ConvArgs a{};
  a.x = x->ptr; a.x_cstride = x->cstride; a.x_coff = x->coff; a.H = x->h; a.W = x->w;
  a.M = (long)x->n * x->h * x->w;
  fill_geom(a, g);
  a.w = packed_up; a.cout = 4 * cout;
  a.bias = bias; a.scale = scale; a.shift = shift; a.act = act;
  a.y = y->ptr; a.y_cstride = y->cstride; a.y_coff = y->coff;
  a.y_dtype = VM_F32;  // f32 staging, split stores (ConvArgs::ysplit)
  a.y_vec = 1;
  a.ysplit = ys;
  a.ovf = overflow;
  a.f16 = 1;
  a.xalias = S;
  a.up = 1; a.up_cout = cout;
  a.ksplit = 1;
  if (!patch_ok(a, 2)) return fail(VM_EUNSUPPORTED, "conv3x3_up2x_split3: shape not supported by the patch kernel");
  int rc = dispatch_patch(a, st);
  if (rc != VM_OK) return rc;
  BorderArgs b{};
  b.x = x->ptr; b.x_cstride = x->cstride; b.x_coff = x->coff; b.H = x->h; b.W = x->w; b.nframes = x->n;
  b.w = packed; b.K_pad = g1.K_pad; b.cout = cout; b.nch = g1.cin_pad / 32;
  b.bias = bias; b.scale = scale; b.shift = shift; b.act = act;
  b.y = y->ptr; b.y_cstride = y->cstride; b.y_coff = y->coff;
  b.xs = S; b.ysplit = ys; b.ovf = overflow;
  const int OH = 2 * x->h, OW = 2 * x->w;
  b.nb = 2 * OW + 2 * (OH - 2);
  const long nblk = ((long)x->n * b.nb + 15) / 16;
  if (nblk > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3_up2x_split3: too many border pixels");
  hipLaunchKernelGGL((conv3x3_up2x_border<4, true>), dim3((unsigned)nblk, cout / 64), dim3(1024), 0, st, b);
  return check_launch("conv3x3_up2x_border(split)");
}

extern "C" int vm_conv3x3_up2x_head_nhwc(const vm_tensor* x, const void* packed_up, const void* packed, int cin,
                                         int cout, const float* bias, const float* scale, const float* shift, int act,
                                         vm_tensor* y, const float* head_w, int head_cin, int head_coff, float* partial,
                                         int store_y, void* stream) {
  if (!head_w || !partial || cout != 64 || head_cin <= 0 || head_coff < 0 || head_coff + cout > head_cin)
    return fail(VM_EINVAL, "conv3x3_up2x_head: head filter [3,3,%d,1] with the conv's %d channels at %d", head_cin, cout,
                head_coff);
  // the partials come from the patch kernel's register epilogue (64-channel row-slot tilings)
  if (!g_patch_repi || g_patch_cfg || g_rows_up || !g_up_skip)
    return fail(VM_EUNSUPPORTED, "conv3x3_up2x_head: needs the patch kernel's register epilogue");
  g_up_head = {head_w, head_cin, head_coff, partial, store_y ? 0 : 1};
  const int rc = vm_conv3x3_up2x_nhwc(x, packed_up, packed, cin, cout, bias, scale, shift, act, y, stream);
  g_up_head = {};
  return rc;
}

extern "C" int vm_conv3x3_head_from_partials(const float* pa, const float* pb, int n, int h, int w, const float* bias,
                                             vm_tensor* logits, float* alpha, void* stream) {
  if (!pa || !pb || n <= 0 || h <= 0 || w <= 0) return fail(VM_EINVAL, "head_from_partials: bad argument");
  if (logits && (!valid_tensor(logits) || logits->dtype != VM_F32 || logits->n != n || logits->h != h ||
                 logits->w != w || logits->c != 1))
    return fail(VM_EINVAL, "head_from_partials: logits must be an f32 [n,h,w,1] view");
  const long tiles = (long)n * ((h + HS_TH - 1) / HS_TH) * ((w + HS_TW - 1) / HS_TW);
  if (tiles > 0x7fffffffL || (long)n * h * w * 12 > 0x7fffffffffffL) return fail(VM_EUNSUPPORTED, "head_from_partials");
  float* lp = logits ? reinterpret_cast<float*>(logits->ptr) + logits->coff : nullptr;
  hipLaunchKernelGGL(head_from_partials, dim3((unsigned)tiles), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), pa, pb, n, h, w, bias, lp, logits ? logits->cstride : 1,
                     alpha);
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::head_from_partials");
  return check_launch("head_from_partials");
}

template <int PABL, int XIN = 2>
static int launch_pair_persist(ConvArgs& a, long sp, hipStream_t st) {
  if constexpr (XIN == 2) {
    if (!a.x_f32) return launch_pair_persist<PABL, 0>(a, sp, st);
    if (a.x_c < 4 || !g_pair_xin_wide) return launch_pair_persist<PABL, 1>(a, sp, st);
  }
  static int attr_dev = -1, n_cu = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (attr_dev != dev) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_pair_persist<PABL, XIN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, PairCfg::LDS);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return fail(VM_EHIP, "conv3x3_pair_persist setup: %s", hipGetErrorString(e));
    attr_dev = dev;
  }
  const int grid = (int)(sp < n_cu ? sp : n_cu);
  snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_pair_persist");
  hipLaunchKernelGGL((conv3x3_pair_persist<PABL, XIN>), dim3(grid), dim3(PairCfg::NT), PairCfg::LDS, st, a);
  return check_launch("conv3x3_pair_persist");
}

static int pair_first_impl(const vm_tensor* x, const void* packed1, int cin1, const float* bias1, const void* packed2,
                           int cout2, const float* bias2, const float* scale2, const float* shift2, int act2,
                           vm_tensor* y, vm_tensor* ypool, const float* head_w, int head_cin, int head_coff,
                           float* partial, int store_y, void* stream, vm_tensor* mid = nullptr);

extern "C" int vm_conv3x3_pair_first_mid_nhwc(const vm_tensor* x, const void* packed1, int cin1, const float* bias1,
                                              const void* packed2, int cout2, const float* bias2, const float* scale2,
                                              const float* shift2, int act2, vm_tensor* y, vm_tensor* ypool,
                                              vm_tensor* mid, void* stream) {
  if (!valid_tensor(mid) || mid->dtype != VM_BF16 || mid->c != 64 || !x || mid->n != x->n || mid->h != x->h ||
      mid->w != x->w || reinterpret_cast<uintptr_t>(mid->ptr) % 16 || mid->cstride % 8 || mid->coff % 8)
    return fail(VM_EINVAL, "conv3x3_pair_first_mid: mid must be a 16-byte aligned bf16 [n,h,w,64] view");
  return pair_first_impl(x, packed1, cin1, bias1, packed2, cout2, bias2, scale2, shift2, act2, y, ypool, nullptr, 0, 0,
                         nullptr, 1, stream, mid);
}

extern "C" int vm_conv3x3_pair_first_nhwc(const vm_tensor* x, const void* packed1, int cin1, const float* bias1,
                                          const void* packed2, int cout2, const float* bias2, const float* scale2,
                                          const float* shift2, int act2, vm_tensor* y, vm_tensor* ypool, void* stream) {
  return pair_first_impl(x, packed1, cin1, bias1, packed2, cout2, bias2, scale2, shift2, act2, y, ypool, nullptr, 0, 0,
                         nullptr, 1, stream);
}

extern "C" int vm_conv3x3_pair_first_head_nhwc(const vm_tensor* x, const void* packed1, int cin1, const float* bias1,
                                               const void* packed2, int cout2, const float* bias2,
                                               const float* scale2, const float* shift2, int act2, vm_tensor* y,
                                               vm_tensor* ypool, const float* head_w, int head_cin, int head_coff,
                                               float* partial, int store_y, void* stream) {
  if (!head_w || !partial || head_cin <= 0 || head_coff < 0 || head_coff + cout2 > head_cin)
    return fail(VM_EINVAL, "conv3x3_pair_first_head: head filter [3,3,%d,1] with the pair's %d channels at %d",
                head_cin, cout2, head_coff);
  return pair_first_impl(x, packed1, cin1, bias1, packed2, cout2, bias2, scale2, shift2, act2, y, ypool, head_w,
                         head_cin, head_coff, partial, store_y, stream);
}

extern "C" int vm_conv3x3_head_acc_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias,
                                        const float* y_acc, vm_tensor* y, float* alpha, void* stream) {
  if (!y_acc) return fail(VM_EINVAL, "conv3x3_head_acc: y_acc is NULL");
  return conv_impl(x, packed, cin, 1, bias, nullptr, nullptr, VM_ACT_NONE, y, nullptr, stream, alpha, 0, 0, nullptr, 0,
                   nullptr, y_acc);
}

extern "C" int vm_conv3x3_head_acc_ex_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias,
                                           const float* scale, const float* shift, const float* y_acc, vm_tensor* y,
                                           float* alpha, void* stream) {
  return conv_impl(x, packed, cin, 1, bias, scale, shift, VM_ACT_NONE, y, nullptr, stream, alpha, 0, 0, nullptr, 0,
                   nullptr, y_acc);
}


extern "C" int vm_conv3x3_split3_nhwc(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias,
                                      const float* scale, const float* shift, int act, vm_tensor* y, int y_slab,
                                      vm_tensor* ypool, int pool_slab, int* overflow, void* work, size_t work_bytes,
                                      void* stream) {
  if (!x || !y || !valid_tensor(y, true) || (ypool && !valid_tensor(ypool, true)))
    return fail(VM_EINVAL, "conv3x3_split3: invalid tensor");
  SplitOut so{y_slab > 0 ? y_slab : y->cstride / 2, 0, overflow};
  if (cout % 8 || !split3_view_ok(y, so.yslab, cout))
    return fail(VM_EUNSUPPORTED, "conv3x3_split3: y must be an fp16 view of cout %% 8 == 0 channels inside the first "
                                 "of two (or three) slabs of S %% 8 == 0 channels, 16-byte aligned");
  if (ypool) {
    so.pslab = pool_slab > 0 ? pool_slab : ypool->cstride / 2;
    if (!split3_view_ok(ypool, so.pslab, cout) || ypool->n != y->n || ypool->h != (y->h + 1) / 2 ||
        ypool->w != (y->w + 1) / 2 || ypool->c != cout)
      return fail(VM_EINVAL, "conv3x3_split3: pool view must be [n, ceil(h/2), ceil(w/2), cout] in the split layout");
  }
  return conv_impl(x, packed, cin, cout, bias, scale, shift, act, y, ypool, stream, nullptr, 0, 0, work, work_bytes,
                   nullptr, nullptr, &so);
}

extern "C" int vm_conv3x3_head_partial_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias,
                                            const float* scale, const float* shift, int act, vm_tensor* y,
                                            float* alpha, const float* partial, void* stream) {
  if (!partial) return fail(VM_EINVAL, "conv3x3_head_partial: partial is NULL");
  return conv_impl(x, packed, cin, 1, bias, scale, shift, act, y, nullptr, stream, alpha, 0, 0, nullptr, 0, partial);
}

static int pair_first_impl(const vm_tensor* x, const void* packed1, int cin1, const float* bias1, const void* packed2,
                           int cout2, const float* bias2, const float* scale2, const float* shift2, int act2,
                           vm_tensor* y, vm_tensor* ypool, const float* head_w, int head_cin, int head_coff,
                           float* partial, int store_y, void* stream, vm_tensor* mid) {
  if (!valid_tensor(x) || !valid_tensor(y) || !packed1 || !packed2)
    return fail(VM_EINVAL, "conv3x3_pair_first: invalid tensor/weights");
  if (cin1 <= 0 || cin1 > 8 || x->c != cin1 || cout2 <= 0 || y->c != cout2)
    return fail(VM_EINVAL, "conv3x3_pair_first: x.c=%d cin1=%d (<= 8) y.c=%d cout2=%d", x->c, cin1, y->c, cout2);
  if (x->n != y->n || x->h != y->h || x->w != y->w) return fail(VM_EINVAL, "conv3x3_pair_first: spatial mismatch");
  if (act2 < VM_ACT_NONE || act2 > VM_ACT_SOFTMAX) return fail(VM_EINVAL, "conv3x3_pair_first: act %d", act2);
  if (ypool && (!valid_tensor(ypool) || ypool->n != y->n || ypool->h != (y->h + 1) / 2 || ypool->w != (y->w + 1) / 2 ||
                ypool->c != cout2 || ypool->dtype != y->dtype))
    return fail(VM_EINVAL, "conv3x3_pair_first: pool output must be [n, ceil(h/2), ceil(w/2), cout2]");
  const bool xf32 = x->dtype == VM_F32;
  const bool xvec = xf32 || (reinterpret_cast<uintptr_t>(x->ptr) % 16 == 0 && x->cstride % 8 == 0 &&
                             x->coff % 8 == 0 && x->coff + 8 <= x->cstride);
  const bool yvec = reinterpret_cast<uintptr_t>(y->ptr) % 16 == 0 && y->cstride % 8 == 0 && y->coff % 8 == 0;
  const bool pvec = !ypool || (reinterpret_cast<uintptr_t>(ypool->ptr) % 16 == 0 && ypool->cstride % 8 == 0 &&
                               ypool->coff % 8 == 0);
  if (y->dtype != VM_BF16 || !xvec || !yvec || !pvec || cout2 % 8 || act2 == VM_ACT_SOFTMAX || g_conv_kernel == 1 ||
      g_conv_kernel == 2)
    return fail(VM_EUNSUPPORTED, "conv3x3_pair_first: needs a bf16 output and 16-byte channel views (bf16 x: "
                                 "8-channel pixels)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  ConvArgs a{};
  a.x = x->ptr; a.x_cstride = x->cstride; a.x_coff = x->coff; a.H = x->h; a.W = x->w;
  a.M = (long)x->n * x->h * x->w;
  fill_geom(a, geom(64, cout2, VM_BF16));
  a.w = packed2; a.cout = cout2;
  a.bias = bias2; a.scale = scale2; a.shift = shift2; a.act = act2;
  a.y = y->ptr; a.y_cstride = y->cstride; a.y_coff = y->coff; a.y_dtype = y->dtype; a.y_vec = 1;
  a.w1 = packed1; a.bias1 = bias1; a.x_f32 = xf32; a.x_c = cin1;
  if (ypool) { a.py = ypool->ptr; a.py_cstride = ypool->cstride; a.py_coff = ypool->coff; }
  const long sp = (long)x->n * ((x->h + 7) / 8) * ((x->w + 31) / 32);
  if (partial) {
    a.hd = partial; a.hw = head_w; a.hw_cin = head_cin; a.hw_coff = head_coff; a.y_skip = store_y ? 0 : 1;
  }
  // the strip kernel addresses one image's output / pool with 32-bit byte offsets
  const bool strip_fits = (long)x->h * x->w * y->cstride * 2 < 0x7ffffff0L &&
                          (!ypool || (long)ypool->h * ypool->w * ypool->cstride * 2 < 0x7ffffff0L);
  if (mid) {  // conv1_1's output too: the strip kernel only (the caller otherwise runs the two convs)
    if (!(g_pair_strip && g_pair_kernel == 0 && strip_fits && pair_strip_ok(a) &&
          (long)mid->h * mid->w * mid->cstride * 2 < 0x7ffffff0L))
      return fail(VM_EUNSUPPORTED, "conv3x3_pair_first_mid: needs the strip pair kernel");
    a.y1 = mid->ptr; a.y1_cstride = mid->cstride; a.y1_coff = mid->coff;
  }
  if (g_pair_strip && g_pair_kernel == 0 && strip_fits && pair_strip_ok(a)) return launch_pair_strip(a, x->n, st);
  if (partial) {  // the head split lives in the persistent pair kernel only
    if (cout2 != 64 || g_pair_kernel != 0 || sp > 0x7fffffffL)
      return fail(VM_EUNSUPPORTED, "conv3x3_pair_first_head: needs the persistent pair kernel (cout2 64)");
    a.hd = partial; a.hw = head_w; a.hw_cin = head_cin; a.hw_coff = head_coff; a.y_skip = store_y ? 0 : 1;
    return launch_pair_persist<0>(a, sp, st);
  }
  if (cout2 == 64 && (g_pair_kernel == 0 || g_pair_kernel >= 10) && sp <= 0x7fffffffL) {
#ifdef VM_STUDY
    switch (g_pair_kernel) {  // >= 10: timing ablations (garbage results), study build only
      case 11: return launch_pair_persist<1>(a, sp, st);
      case 12: return launch_pair_persist<2>(a, sp, st);
      case 14: return launch_pair_persist<4>(a, sp, st);
      case 18: return launch_pair_persist<8>(a, sp, st);
      case 13: return launch_pair_persist<3>(a, sp, st);
      default: break;
    }
#endif
    return launch_pair_persist<0>(a, sp, st);
  }
  if (sp * ((cout2 + 63) / 64) < 512) return launch_patch<64, 4, 1, 6, 4, 1, 9, false, 0, true>(a, st);
  return launch_patch<64, 8, 1, 6, 8, 1, 9, false, 0, true>(a, st);
}

extern "C" int vm_conv3x3_head_nhwc(const vm_tensor* x, const void* packed, int cin, const float* bias,
                                    const float* scale, const float* shift, int act, vm_tensor* y, float* alpha,
                                    void* stream) {
  return conv_impl(x, packed, cin, 1, bias, scale, shift, act, y, nullptr, stream, alpha);
}

static int conv_impl(const vm_tensor* x, const void* packed, int cin, int cout, const float* bias, const float* scale,
                     const float* shift, int act, vm_tensor* y, const vm_tensor* yp, void* stream, float* y2, int nsrc,
                     long src_stride, void* work, size_t work_bytes, const float* head_part, const float* y_acc,
                     const SplitOut* so) {
  if (!valid_tensor(x, true) || !valid_tensor(y, so != nullptr) || !packed)
    return fail(VM_EINVAL, "conv3x3: invalid tensor/weights");
  // fp16 operands (the split-fp16 forward, vmatting/split3.py): f32 outputs of the patch kernel (any cout % 4 == 0)
  // or the MFMA head (cout == 1, <= 256 channels per call), or (so) the split-fp16 output with its fused pool; no
  // split sources or softmax
  const bool f16 = x->dtype == VM_F16;
  if (so && (!f16 || y->dtype != VM_F16 || cout == 1))
    return fail(VM_EINVAL, "conv3x3_split3: fp16 input and fp16 split output views, cout > 1");
  if (f16 && ((!so && (y->dtype != VM_F32 || yp)) || nsrc > 1 || act == VM_ACT_SOFTMAX || head_part))
    return fail(VM_EUNSUPPORTED, "conv3x3: fp16 operands need an f32 (or split) output without sources / softmax");
  if (y_acc && cout != 1) return fail(VM_EINVAL, "conv3x3: an accumulated pre-activation needs cout == 1");
  if (head_part && cout != 1) return fail(VM_EINVAL, "conv3x3: head partials need cout == 1");
  int xc = nsrc > 1 ? nsrc * x->c : x->c;  // sources: x is the view of source 0
  // split-fp16 input stored as two slabs [l, h] (x->c = 2S) for a filter over [l, h, h] (cin = 3S): the third slab is
  // read from the second (ConvArgs::xalias)
  int xalias = 0;
  if (x->dtype == VM_F16 && nsrc <= 1 && 2 * cin == 3 * x->c && x->c % 64 == 0) {
    xalias = x->c / 2;
    xc = cin;
  }
  if (cin <= 0 || cout <= 0 || xc != cin || y->c != cout)
    return fail(VM_EINVAL, "conv3x3: channel mismatch x.c=%d cin=%d y.c=%d cout=%d", xc, cin, y->c, cout);
  if (nsrc > 1 && (cout == 1 || yp || x->c % (x->dtype == VM_BF16 ? 32 : 16) || src_stride % 8))
    return fail(VM_EUNSUPPORTED, "conv3x3: split sources need whole 64-byte granules per source (x.c=%d)", x->c);
  if (x->n != y->n || x->h != y->h || x->w != y->w)
    return fail(VM_EINVAL, "conv3x3: spatial mismatch [%d,%d,%d] vs [%d,%d,%d]", x->n, x->h, x->w, y->n, y->h, y->w);
  if (act < VM_ACT_NONE || act > VM_ACT_SOFTMAX) return fail(VM_EINVAL, "conv3x3: act %d", act);
  const int dt = x->dtype;
  PackGeom g = geom(cin, cout, dt);
  const int ce = 16 / elem_bytes(dt);
  if (reinterpret_cast<uintptr_t>(x->ptr) % 16 || x->cstride % ce || x->coff % ce ||
      x->coff + (nsrc > 1 || xalias ? x->c : g.cin_pad) > x->cstride)
    return fail(VM_EUNSUPPORTED,
                "conv3x3: input view must be 16-byte aligned with channel padding to %d (coff=%d cstride=%d)",
                g.cin_pad, x->coff, x->cstride);
  if (act == VM_ACT_SOFTMAX && cout > 128) return fail(VM_EUNSUPPORTED, "conv3x3: fused softmax needs cout <= 128");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long M = (long)x->n * x->h * x->w;
  if (yp && cout == 1) return fail(VM_EUNSUPPORTED, "conv3x3_pool: no fused pooling for cout == 1");

  if (cout == 1) {
    HeadArgs h{};
    h.x = x->ptr; h.x_cstride = x->cstride; h.x_coff = x->coff; h.H = x->h; h.W = x->w; h.M = M;
    h.cin_pad = g.cin_pad; h.K9 = g.K9; h.K_pad = g.K_pad; h.chunk_major = g.chunk_major; h.ng = g.ng;
    h.w = packed; h.bias = bias; h.scale = scale; h.shift = shift; h.act = act;
    h.y = y->ptr; h.y_cstride = y->cstride; h.y_coff = y->coff; h.y_dtype = y->dtype; h.y2 = y2;
    h.part = head_part;
    h.yacc = y_acc;
    const int nks = (g.cin_pad + 4 * ce - 1) / (4 * ce);
    // the split-fp16 x3 head over a two-slab [l, h] view of 128-channel slabs (cin 384 as [l, h, h]): one call
    if (f16 && xalias == 128 && nks == 12 && g_head_kernel == 0) {
      // 16-row tiles: an 18 x 66 input window per 16 x 64 outputs (1.16x the tile's pixels, 1.29x for 8 rows); the
      // per-pixel tap sums and the 9-tap epilogue are the same arithmetic whatever the tile: bit-identical
      constexpr int TW = 64;
      const int th16 = g_head_th == 16 ? 16 : 8;
      const long tiles = (long)x->n * ((x->h + th16 - 1) / th16) * ((x->w + TW - 1) / TW);
      if (tiles > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3 head: too many tiles");
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_head_mfma<vm::f16_t, %d, %d, 12, true>", th16, TW);
      if (th16 == 16)
        hipLaunchKernelGGL((conv3x3_head_mfma<f16_t, 16, TW, 12, true>), dim3(tiles), dim3(256),
                           (size_t)9 * g.cin_pad * 2, st, h);
      else
        hipLaunchKernelGGL((conv3x3_head_mfma<f16_t, 8, TW, 12, true>), dim3(tiles), dim3(256),
                           (size_t)9 * g.cin_pad * 2, st, h);
      return check_launch("conv3x3_head_mfma");
    }
    if ((head_part || y_acc || f16) && (g_head_kernel != 0 || nks > 8))
      return fail(VM_EUNSUPPORTED, "conv3x3 head: partials / accumulation / fp16 need the MFMA head kernel (cin <= 256, "
                                   "or 384 as a two-slab split-fp16 view)");
    if (g_head_kernel == 0 && nks <= 8) {
      constexpr int TW = 64;
      // 16-row tiles for the bf16 128-channel head (cat1 of UNetVideo): input window 18 x 66 per 16 x 64 outputs
      // (1.16x the tile's bytes instead of 1.29x for 8 rows)
      const int TH = (dt == VM_BF16 && (nks == 4 || (nks == 2 && head_part)) && g_head_th == 16) ? 16 : 8;
      const long tiles = (long)x->n * ((x->h + TH - 1) / TH) * ((x->w + TW - 1) / TW);
      if (tiles > 0x7fffffffL) return fail(VM_EUNSUPPORTED, "conv3x3 head: too many tiles");
      const size_t lds = (size_t)9 * g.cin_pad * elem_bytes(dt);
      const int nk = nks <= 1 ? 1 : nks <= 2 ? 2 : nks <= 4 ? 4 : 8;
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_head_mfma<%s, %d, %d, %d>",
               dt == VM_BF16 ? "unsigned short" : "float", TH, TW, nk);
#define VM_HEAD_MFMA(TT, NK) \
  hipLaunchKernelGGL((conv3x3_head_mfma<TT, 8, TW, NK>), dim3(tiles), dim3(256), lds, st, h)
      if (f16) {
        snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_head_mfma<vm::f16_t, 8, %d, %d>", TW, nk);
        if (nk == 1) VM_HEAD_MFMA(f16_t, 1); else if (nk == 2) VM_HEAD_MFMA(f16_t, 2);
        else if (nk == 4) VM_HEAD_MFMA(f16_t, 4); else VM_HEAD_MFMA(f16_t, 8);
      } else if (TH == 16 && nk == 2) {  // the split head's 64-channel half
        hipLaunchKernelGGL((conv3x3_head_mfma<uint16_t, 16, TW, 2>), dim3(tiles), dim3(256), lds, st, h);
      } else if (TH == 16) {
        hipLaunchKernelGGL((conv3x3_head_mfma<uint16_t, 16, TW, 4>), dim3(tiles), dim3(256), lds, st, h);
      } else if (dt == VM_BF16) {
        if (nk == 1) VM_HEAD_MFMA(uint16_t, 1); else if (nk == 2) VM_HEAD_MFMA(uint16_t, 2);
        else if (nk == 4) VM_HEAD_MFMA(uint16_t, 4); else VM_HEAD_MFMA(uint16_t, 8);
      } else {
        if (nk == 1) VM_HEAD_MFMA(float, 1); else if (nk == 2) VM_HEAD_MFMA(float, 2);
        else if (nk == 4) VM_HEAD_MFMA(float, 4); else VM_HEAD_MFMA(float, 8);
      }
#undef VM_HEAD_MFMA
      return check_launch("conv3x3_head_mfma");
    }
    constexpr int P = 8;
    const int nch = g.cin_pad / (16 * ce);
    if ((nch == 1 || nch == 2) && g.cin_pad % (16 * ce) == 0 && g_head_kernel != 1) {
      const long strips = (M / x->w) * ((x->w + P - 1) / P);
      const int grid = grid_for((strips + 15) / 16, 1, 256 * 8);
      const size_t lds = (size_t)9 * g.cin_pad * elem_bytes(dt);
      snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_head_strip<%s, %d, %d>",
               dt == VM_BF16 ? "unsigned short" : "float", nch, P);
      if (dt == VM_BF16) {
        if (nch == 1) hipLaunchKernelGGL((conv3x3_head_strip<uint16_t, 1, P>), dim3(grid), dim3(256), lds, st, h);
        else hipLaunchKernelGGL((conv3x3_head_strip<uint16_t, 2, P>), dim3(grid), dim3(256), lds, st, h);
      } else {
        if (nch == 1) hipLaunchKernelGGL((conv3x3_head_strip<float, 1, P>), dim3(grid), dim3(256), lds, st, h);
        else hipLaunchKernelGGL((conv3x3_head_strip<float, 2, P>), dim3(grid), dim3(256), lds, st, h);
      }
      return check_launch("conv3x3_head_strip");
    }
    const int grid = grid_for((M + 15) / 16, 1, 256 * 8);
    const size_t lds = (size_t)9 * g.cin_pad * 4;
    snprintf(g_last_kernel, sizeof g_last_kernel, "vm::conv3x3_head<%s>", dt == VM_BF16 ? "unsigned short" : "float");
    if (dt == VM_BF16) hipLaunchKernelGGL(conv3x3_head<uint16_t>, dim3(grid), dim3(256), lds, st, h);
    else hipLaunchKernelGGL(conv3x3_head<float>, dim3(grid), dim3(256), lds, st, h);
    return check_launch("conv3x3_head");
  }

  ConvArgs a{};
  a.x = x->ptr; a.x_cstride = x->cstride; a.x_coff = x->coff; a.H = x->h; a.W = x->w; a.M = M;
  fill_geom(a, g);
  if (nsrc > 1) {
    a.x_src_c = x->c;
    a.x_src_stride = src_stride;
  }
  a.ksplit = 1;
  a.w = packed; a.cout = cout;
  a.bias = bias; a.scale = scale; a.shift = shift; a.act = act;
  a.y = y->ptr; a.y_cstride = y->cstride; a.y_coff = y->coff; a.y_dtype = y->dtype;
  const int yve = 16 / elem_bytes(y->dtype);
  a.y_vec = (reinterpret_cast<uintptr_t>(y->ptr) % 16 == 0) && (y->cstride % yve == 0) && (y->coff % yve == 0);
  if (yp && !f16) {
    const bool pvec = reinterpret_cast<uintptr_t>(yp->ptr) % 16 == 0 && yp->cstride % 8 == 0 && yp->coff % 8 == 0;
    if (cout == 1 || dt != VM_BF16 || !pvec || !patch_ok(a, 2) || g_conv_kernel == 1 || g_conv_kernel == 2)
      return fail(VM_EUNSUPPORTED, "conv3x3_pool: fused pooling needs the bf16 patch kernel");
    a.py = yp->ptr;
    a.py_cstride = yp->cstride;
    a.py_coff = yp->coff;
    return dispatch_patch(a, st);
  }
  if (f16) {  // the patch kernel's fp16 form (+ split-K on small grids with a workspace)
    a.f16 = 1;
    a.xalias = xalias;
    a.py = nullptr;
    a.up = 0;
    if (so) {  // split output: staged like an f32 output, stored as fp16 slabs (y_cstride stays in fp16 elements)
      a.y_dtype = VM_F32;
      a.y_vec = 1;
      a.ysplit = so->yslab;
      a.ovf = so->ovf;
      if (yp) {
        a.py = yp->ptr;
        a.py_cstride = yp->cstride;
        a.py_coff = yp->coff;
        a.psplit = so->pslab;
      }
    }
    if (!patch_ok(a, 2)) return fail(VM_EUNSUPPORTED, "conv3x3: fp16 operands need the patch kernel (cin %% 32 == 0)");
    if (work && (cout & 3) == 0 && !yp) {
      const int ks = splitk_plan(x->n, x->h, x->w, a.cin_pad, cout);
      if (ks > 1 && work_bytes >= (size_t)ks * M * cout * sizeof(float)) {
        a.ksplit = ks;
        a.part = reinterpret_cast<float*>(work);
      }
    }
    return dispatch_patch(a, st);
  }
  if (g_conv_kernel == 0 && thin_ok(dt, g, cout, a.x_src_c, act, x)) {
    const int ks = work ? thin_splitk_plan(x->n, x->h, x->w, a.cin_pad) : 1;
    if (ks > 1 && work_bytes >= (size_t)ks * M * cout * sizeof(float)) {
      a.ksplit = ks;
      a.part = reinterpret_cast<float*>(work);
    }
    return dispatch_thin(a, x->n, st);
  }
  if (nsrc > 1) {
    // the patch / row-stationary / generic kernels add source s's offset (s * src_stride elements) into 32-bit
    // byte offsets inside one image's buffer resource: the whole span must stay below it (the thin kernel above
    // forms 64-bit source pointers).  Callers materialise the concat instead (ops.conv3x3)
    const long span = ((long)(nsrc - 1) * src_stride + (long)x->h * x->w * x->cstride) * elem_bytes(dt);
    if (span >= g_src_span_limit)
      return fail(VM_EUNSUPPORTED, "conv3x3: split sources span %ld bytes (limit %ld): materialise the concat", span,
                  g_src_span_limit);
  }
  if (dt == VM_BF16 && work && g_conv_kernel == 0 && patch_ok(a, 2) && (cout & 3) == 0) {
    const int ks = splitk_plan(x->n, x->h, x->w, a.cin_pad, cout);
    if (ks > 1 && work_bytes >= (size_t)ks * M * cout * sizeof(float)) {
      a.ksplit = ks;
      a.part = reinterpret_cast<float*>(work);
      return dispatch_patch(a, st);
    }
  }
  if (dt == VM_BF16 && g_conv_kernel == 0 && narrowin_ok(a, g, cout, act, x, y)) return launch_narrowin(a, x->n, g, st);
  if (dt == VM_BF16) return dispatch_mfma<uint16_t>(a, st);
  return dispatch_mfma<float>(a, st, cin);
}

// workspace of vm_conv3x3_ex_nhwc: the split-K partial sums of a small-grid bf16 conv, else 0
extern "C" size_t vm_conv3x3_workspace_bytes(const vm_tensor* x, int cin, int cout) {
  if (!x || (x->dtype != VM_BF16 && x->dtype != VM_F16) || cin <= 0 || cout <= 0) return 0;
  const PackGeom g = geom(cin, cout, VM_BF16);
  if (x->dtype == VM_BF16 && g_conv_kernel == 0 && thin_ok(VM_BF16, g, cout, cin == x->c ? 0 : x->c, VM_ACT_NONE, x)) {
    const int ks = thin_splitk_plan(x->n, x->h, x->w, g.cin_pad);
    return ks > 1 ? (size_t)ks * x->n * x->h * x->w * cout * sizeof(float) : 0;
  }
  if (cout & 3) return 0;
  if (!g.chunk_major || g.cin_pad % 32) return 0;
  const int ks = splitk_plan(x->n, x->h, x->w, g.cin_pad, cout);
  return ks > 1 ? (size_t)ks * x->n * x->h * x->w * cout * sizeof(float) : 0;
}

extern "C" int vm_conv3x3_ex_nhwc(const vm_tensor* x, int nsrc, long src_stride, const void* packed, int cin, int cout,
                                  const float* bias, const float* scale, const float* shift, int act, vm_tensor* y,
                                  void* work, size_t work_bytes, void* stream) {
  if (nsrc < 0 || (nsrc > 1 && src_stride <= 0)) return fail(VM_EINVAL, "conv3x3_ex: nsrc %d stride %ld", nsrc,
                                                            src_stride);
  return conv_impl(x, packed, cin, cout, bias, scale, shift, act, y, nullptr, stream, nullptr, nsrc, src_stride, work,
                   work_bytes);
}
